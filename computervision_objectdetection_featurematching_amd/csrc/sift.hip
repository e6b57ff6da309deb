// sift.hip — SIFT::detectAndCompute (OpenCV 4.5.4 defaults) and resize(INTER_LINEAR, 8U) on gfx950.
//
// Replaces the feature extraction around the matcher: the model views (/root/reference/src/
// ModelsDetector.cpp:75, with mask) and every scene scale (TestsDetector.cpp:102 resize, :106
// detectAndCompute), SIFT::create() defaults (main.cpp:17): 3 octave layers, contrast 0.04, edge 10,
// sigma 1.6, first octave -1 (the image doubled), CV_32F descriptors of 0..255 integers.
//
// One launch per stage, every pixel / candidate / keypoint its own thread; the stages after the
// extrema run on fixed grids over device-side counts, so a call synchronises twice (the counts, then
// the copies of keypoints and descriptors):
//   up2       u8 -> float, x2 INTER_LINEAR (createInitialImage)
//   blur_row  Gaussian row pass, taps in order          } GaussianBlur(CV_32F, BORDER_REFLECT_101):
//   blur_col  Gaussian column pass, symmetric pairs     } OpenCV's RowFilter / SymmColumnFilter sums
//   down2     next octave's first layer (INTER_NEAREST, every 2nd pixel)
//   dog       difference of adjacent layers, all 5 of an octave in one launch
//   extrema   26-neighbour test + threshold over layers 1..3, candidates appended
//   refine    adjustLocalExtrema (<= 5 Newton steps, Cramer 3x3 solve), contrast + edge tests,
//             calcOrientationHist (36 bins, smoothed), one keypoint per peak >= 80 % of the maximum
//   kp_post   KeyPointsFilter::removeDuplicatedSorted (bitonic sort by KeypointGreater in LDS, one
//             1024-thread block), the 1/2 rescale of octave -1, the mask filter (runByPixelsMask)
//   descr     calcSIFTDescriptor: 4x4x8 trilinear histogram in LDS (per thread, pixel order),
//             wrap, clamp at 0.2 of the norm, x 512 / norm, saturate to 0..255
// The histograms accumulate in the reference's pixel order (one thread per keypoint), so the results
// are the CPU restatement's (oracle/sift_oracle.c) bit for bit up to the rare last-bit difference of
// a double-precision exp/sin/cos/pow rounded to float (both sides use those, see sift_oracle.h).
#include "mim_internal.h"

#include <float.h>
#include <limits.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace mim {

namespace {

constexpr int kNOL = 3;
constexpr int kBorder = 5;
constexpr int kOriBins = 36;
constexpr int kDW = 4, kDB = 8;
constexpr int kHistLen = (kDW + 2) * (kDW + 2) * (kDB + 2);  // 360

// BORDER_REFLECT_101 (borderInterpolate): the reflection is periodic with period 2 len - 2 and even, so
// a closed form instead of OpenCV's reflect loop (no loop between a kernel's independent loads)
__device__ __forceinline__ int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    const int period = 2 * len - 2, q = abs(p) % period;
    return q < len ? q : period - q;
}

__device__ __forceinline__ int cv_round(float v) { return __float2int_rn(v); }  // ties to even
__device__ __forceinline__ int cv_round_d(double v) { return __double2int_rn(v); }

struct LinCoef {
    int s;
    float a0, a1;
};

// resize(INTER_LINEAR) source offset and weights of destination index d (resize.cpp)
__device__ __forceinline__ LinCoef lin_coef(int d, int ssize, double scale, bool clamp) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)floor(f);
    f -= s;
    if (clamp) {
        if (s < 0) f = 0, s = 0;
        if (s >= ssize - 1) f = 0, s = ssize - 1;
    }
    return LinCoef{s, 1.f - f, f};
}

// Batched launches: every stage of a SIFT call runs ONE launch for all its images (the five scene
// scales of TestsDetector.cpp:99-106, or one model view).  Image j of a flattened launch owns blocks
// off[j] .. off[j + 1] - 1, laid out as rows of gx[j] blocks; per-image operands are kernel-argument
// arrays indexed by the block-uniform j (scalar loads from the kernarg segment).
constexpr int kMaxImg = 8;
struct Flat {
    int n;
    int off[kMaxImg + 1];
    int gx[kMaxImg];
};

__device__ __forceinline__ int flat_job(const Flat& f, int b, int& bx, int& by) {
    int j = 0;
#pragma unroll
    for (int k = 1; k < kMaxImg; ++k) j += (k < f.n && b >= f.off[k]);
    j = __builtin_amdgcn_readfirstlane(j);
    const int lb = b - f.off[j];
    by = lb / f.gx[j];
    bx = lb - by * f.gx[j];
    return j;
}

struct Up2B {
    Flat f;
    const uint8_t* src[kMaxImg];
    int rows[kMaxImg], cols[kMaxImg];
    float* dst[kMaxImg];
};

__global__ void up2_kernel(Up2B A) {
    int bx, y;
    const int j = flat_job(A.f, blockIdx.x, bx, y);
    const uint8_t* __restrict__ src = A.src[j];
    float* __restrict__ dst = A.dst[j];
    const int rows = A.rows[j], cols = A.cols[j];
    const int x = bx * blockDim.x + threadIdx.x;
    const int dr = rows * 2, dc = cols * 2;
    if (x >= dc) return;
    const LinCoef cx = lin_coef(x, cols, (double)cols / dc, true), cy = lin_coef(y, rows, (double)rows / dr, false);
    float h[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        int sy = cy.s + k;
        sy = sy < 0 ? 0 : (sy >= rows ? rows - 1 : sy);
        const uint8_t* S = src + (size_t)sy * cols;
        h[k] = cx.s + 1 < cols ? (float)S[cx.s] * cx.a0 + (float)S[cx.s + 1] * cx.a1 : (float)S[cx.s];
    }
    dst[(size_t)y * dc + x] = h[0] * cy.a0 + h[1] * cy.a1;
}

// resize(INTER_LINEAR) of CV_8UC1: fixed-point weights (x 2048); the vertical pass as OpenCV's
// 128-bit vector path for columns < (dcols / 16) * 16, the exact rounding shift for the rest
struct ResizeB {
    Flat f;
    const uint8_t* src;
    int rows, cols;
    uint8_t* dst[kMaxImg];
    int drows[kMaxImg], dcols[kMaxImg];
    double sx[kMaxImg], sy[kMaxImg];
};

__global__ void resize_u8_kernel(ResizeB A) {
    int bx, y;
    const int j = flat_job(A.f, blockIdx.x, bx, y);
    const uint8_t* __restrict__ src = A.src;
    uint8_t* __restrict__ dst = A.dst[j];
    const int rows = A.rows, cols = A.cols, dcols = A.dcols[j];
    const double sx = A.sx[j], sy = A.sy[j];
    const int x = bx * blockDim.x + threadIdx.x;
    if (x >= dcols) return;
    const LinCoef cx = lin_coef(x, cols, sx, true), cy = lin_coef(y, rows, sy, false);
    const int a0 = cv_round(cx.a0 * 2048.f), a1 = cv_round(cx.a1 * 2048.f);
    const int b0 = (short)cv_round(cy.a0 * 2048.f), b1 = (short)cv_round(cy.a1 * 2048.f);
    int h[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        int sy = cy.s + k;
        sy = sy < 0 ? 0 : (sy >= rows ? rows - 1 : sy);
        const uint8_t* S = src + (size_t)sy * cols;
        h[k] = cx.s + 1 < cols ? S[cx.s] * a0 + S[cx.s + 1] * a1 : S[cx.s] * 2048;
    }
    int v;
    if (x < dcols / 16 * 16) {
        const int p0 = (int)(short)(h[0] >> 4), p1 = (int)(short)(h[1] >> 4);
        v = (((p0 * b0) >> 16) + ((p1 * b1) >> 16) + 2) >> 2;
    } else {
        v = (h[0] * b0 + h[1] * b1 + (1 << 21)) >> 22;
    }
    dst[(size_t)y * dcols + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

struct Taps {
    float k[64];
    int n;
};

// GaussianBlur (sepFilter2D, BORDER_REFLECT_101) of one 64 x 16 output tile: the source rows the
// column pass needs (reflected) are staged in LDS with their reflected column margins, the row pass
// writes its 16 + 2a rows x 64 columns to LDS, the column pass reads them.  Each output is computed
// with the same float operations in the same order as the separate row / column passes of OpenCV's
// filter engine (row: k0 s0 + k1 s1 + ...; column, symmetric kernel: k_a m + sum of k_{a+i} (m_+i + m_-i)).
constexpr int kBlurTW = 64, kBlurTH = 16;

struct BlurB {
    Flat f;
    const float* src[kMaxImg];
    float* dst[kMaxImg];
    float* dog[kMaxImg];       // dst - src (the DoG plane of layers src, dst), or null: fused so the
                               // large octaves need no separate DoG pass over two Gaussian planes
    int rows[kMaxImg], cols[kMaxImg];
};

__global__ __launch_bounds__(256) void blur_kernel(BlurB A, Taps t) {
    extern __shared__ float lds[];
    __shared__ float tk[64];     // the taps, read per tap from LDS rather than the kernel arguments
    int bx, by;
    const int j = flat_job(A.f, blockIdx.x, bx, by);
    const float* __restrict__ src = A.src[j];
    float* __restrict__ dst = A.dst[j];
    float* __restrict__ dog = A.dog[j];
    const int rows = A.rows[j], cols = A.cols[j];
    const int a = t.n / 2, W = kBlurTW + 2 * a, H = kBlurTH + 2 * a;
    float* in = lds;             // H x W
    float* mid = lds + H * W;    // H x kBlurTW
    const int x0 = bx * kBlurTW, y0 = by * kBlurTH, tid = threadIdx.x;
    if (tid < 64) tk[tid] = t.k[tid];
    // 8 loads in flight per thread: a launch is one or two rounds of this loop on the small octaves,
    // where one dependent global load per iteration made every blur ~11 us whatever its size
    // (profiles/r03e_kernel_stats_c1img.csv: 1-block launches 13.9 us)
    for (int e0 = tid; e0 < H * W; e0 += 256 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + 256 * u;
            if (e < H * W) {
                const int r = e / W, c = e - r * W;
                v[u] = src[(size_t)reflect101(y0 - a + r, rows) * cols + reflect101(x0 - a + c, cols)];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (e0 + 256 * u < H * W) in[e0 + 256 * u] = v[u];
    }
    __syncthreads();
    for (int e = tid; e < H * kBlurTW; e += 256) {
        const int r = e / kBlurTW, c = e - r * kBlurTW;
        const float* S = in + r * W + c;
        float acc = tk[0] * S[0];
        for (int i = 1; i < t.n; ++i) acc += tk[i] * S[i];
        mid[e] = acc;
    }
    __syncthreads();
    for (int e = tid; e < kBlurTH * kBlurTW; e += 256) {
        const int r = e / kBlurTW, c = e - r * kBlurTW, y = y0 + r, x = x0 + c;
        if (y >= rows || x >= cols) continue;
        const float* M = mid + (r + a) * kBlurTW + c;
        float acc = tk[a] * M[0] + 0.f;
        for (int i = 1; i <= a; ++i) acc += tk[a + i] * (M[i * kBlurTW] + M[-i * kBlurTW]);
        dst[(size_t)y * cols + x] = acc;
        if (dog) dog[(size_t)y * cols + x] = acc - in[(r + a) * W + c + a];
    }
}

// blur_kernel with the half-width A a compile-time constant (the SIFT taps are fixed: A = 5, 5, 6, 8, 10,
// 13), register-blocked.  The taps are kernel-argument SGPRs (the unrolled loops index them by
// constants), the row pass computes 4 adjacent outputs per work item from one window read as float4s
// (4 + 2A LDS values for 4 outputs instead of 2 (2A + 1) per output: source and tap), and the column pass
// one column strip of kColR outputs per thread from kColR + 2A values held in registers.  The float
// operations and their order per output are blur_kernel's (row: k0 s0 + k1 s1 + ...; column: k_A m +
// sum of k_{A+i} (m_+i + m_-i)), so the planes are identical.  Tile kBlurTW x TH.
#ifndef MIM_BLUR_TH
#define MIM_BLUR_TH 32
#endif
#ifndef MIM_BLUR_TH_BIG
#define MIM_BLUR_TH_BIG 32  // tile rows for A >= 10 (fewer halo rows per output row in the row pass)
#endif
template <int A, int TH>
__global__ __launch_bounds__(256) void blur_reg_kernel(BlurB B, Taps t) {
    constexpr int N = 2 * A + 1, H = TH + 2 * A;
    constexpr int WS = (kBlurTW + 2 * A + 3) / 4 * 4 + 4;  // in row stride: float4-aligned, 4 floats of slack
    constexpr int kColR = TH / 4;                           // output rows per thread in the column pass
    constexpr int kWin = (4 + 2 * A + 3) / 4;               // float4s of a row-pass window
    __shared__ __attribute__((aligned(16))) float in[H * WS];
    __shared__ __attribute__((aligned(16))) float mid[H * kBlurTW];
    int bx, by;
    const int j = flat_job(B.f, blockIdx.x, bx, by);
    const float* __restrict__ src = B.src[j];
    float* __restrict__ dst = B.dst[j];
    float* __restrict__ dog = B.dog[j];
    const int rows = B.rows[j], cols = B.cols[j];
    const int x0 = bx * kBlurTW, y0 = by * TH, tid = threadIdx.x;
    constexpr int W = kBlurTW + 2 * A, NE = H * W;
    for (int e0 = tid; e0 < NE; e0 += 256 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + 256 * u;
            if (e < NE) {
                const int r = e / W, c = e - r * W;
                v[u] = src[(size_t)reflect101(y0 - A + r, rows) * cols + reflect101(x0 - A + c, cols)];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = e0 + 256 * u;
            if (e < NE) {
                const int r = e / W, c = e - r * W;
                in[r * WS + c] = v[u];
            }
        }
    }
    __syncthreads();
    // row pass: item = (row r of H, group g of 4 output columns)
    for (int item = tid; item < H * (kBlurTW / 4); item += 256) {
        const int r = item >> 4, g = item & 15;
        float w[4 * kWin];
        const float4* S = (const float4*)(in + r * WS + 4 * g);
#pragma unroll
        for (int q = 0; q < kWin; ++q) {
            const float4 f = S[q];
            w[4 * q] = f.x;
            w[4 * q + 1] = f.y;
            w[4 * q + 2] = f.z;
            w[4 * q + 3] = f.w;
        }
        float o[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float acc = t.k[0] * w[c];
#pragma unroll
            for (int i = 1; i < N; ++i) acc += t.k[i] * w[c + i];
            o[c] = acc;
        }
        *(float4*)(mid + r * kBlurTW + 4 * g) = make_float4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
    // column pass: column c, rows r0 .. r0 + kColR - 1 of the tile
    const int c = tid & 63, r0 = (tid >> 6) * kColR, x = x0 + c;
    float m[kColR + 2 * A];
#pragma unroll
    for (int i = 0; i < kColR + 2 * A; ++i) m[i] = mid[(r0 + i) * kBlurTW + c];
#pragma unroll
    for (int q = 0; q < kColR; ++q) {
        const int y = y0 + r0 + q;
        float acc = t.k[A] * m[q + A] + 0.f;
#pragma unroll
        for (int i = 1; i <= A; ++i) acc += t.k[A + i] * (m[q + A + i] + m[q + A - i]);
        if (y < rows && x < cols) {
            dst[(size_t)y * cols + x] = acc;
            if (dog) dog[(size_t)y * cols + x] = acc - in[(r0 + q + A) * WS + c + A];
        }
    }
}

// The small octaves (plane <= kSmallPlane) of one image in ONE launch of one 1024-thread block: per
// octave the down-sample of the previous octave's layer kNOL, the five blurs (row pass into LDS, column
// pass with reflected rows, the same float operations in the same order as blur_kernel) and the five
// DoG planes, the layers ping-ponging in LDS and written out for the later kernels.  Replaces ~7
// launches per small octave (each ~4-14 us whatever its size) by one for all of them.
#ifndef MIM_SMALL_PLANE
#define MIM_SMALL_PLANE 512  // measured: 8192 1.81 ms per 640x480 image, 2048 1.54, 512 1.49-1.52 (profiles/r03s_sift_small_plane.txt)
#endif
constexpr int kSmallPlane = MIM_SMALL_PLANE;  // largest octave plane (pixels) fused
struct Layer {
    const float* p;
    int rows, cols;
};

struct Pyr {
    Layer gauss[16][kNOL + 3];
    Layer dog[16][kNOL + 2];
};

// one block per image: octaves o0[j] .. n_oct[j] - 1 (o0 >= 1), geometry and planes from its Pyr table
struct SmallB {
    int n;
    const Pyr* pyr[kMaxImg];
    int o0[kMaxImg], n_oct[kMaxImg];
    Taps t[kNOL + 2];          // blur taps of layers 1 .. kNOL + 2 (the same for every image)
};

__global__ __launch_bounds__(1024) void small_octaves_kernel(SmallB so) {
    const int jb = blockIdx.x;
    const Pyr* __restrict__ py = so.pyr[jb];
    const int o_begin = so.o0[jb], o_end = so.n_oct[jb];
    __shared__ float sm[4 * kSmallPlane];  // 128 KiB
    __shared__ float taps[kNOL + 2][64];   // the kernel-argument taps, read per tap from LDS
    float* bufA = sm;                     // current layer
    float* bufB = sm + kSmallPlane;       // next layer
    float* tmp = sm + 2 * kSmallPlane;    // row pass
    float* nxt = sm + 3 * kSmallPlane;    // layer kNOL down-sampled: the next octave's layer 0
    const int tid = threadIdx.x;
    if (tid < (kNOL + 2) * 64) taps[tid >> 6][tid & 63] = so.t[tid >> 6].k[tid & 63];
    for (int o = o_begin; o < o_end; ++o) {
        const int rows = py->gauss[o][0].rows, cols = py->gauss[o][0].cols, plane = rows * cols;
        float* G = const_cast<float*>(py->gauss[o][0].p);  // layers i at G + i * plane
        float* D = const_cast<float*>(py->dog[o][0].p);
        // layer 0 = every second pixel of the previous octave's layer kNOL (down2_kernel)
        if (o == o_begin) {
            const int pc = py->gauss[o - 1][0].cols;
            const float* src = py->gauss[o - 1][kNOL].p;
            for (int e = tid; e < plane; e += 1024) {
                const int y = e / cols, x = e - y * cols;
                bufA[e] = src[(long long)(2 * y) * pc + 2 * x];
            }
        } else {
            for (int e = tid; e < plane; e += 1024) bufA[e] = nxt[e];
        }
        __syncthreads();
        for (int e = tid; e < plane; e += 1024) G[e] = bufA[e];
        for (int i = 1; i < kNOL + 3; ++i) {
            const float* tk = taps[i - 1];
            const int tn = so.t[i - 1].n, a = tn / 2;
            for (int e = tid; e < plane; e += 1024) {  // row pass (reflected columns)
                const int y = e / cols, x = e - y * cols;
                const float* S = bufA + y * cols;
                float acc = tk[0] * S[reflect101(x - a, cols)];
                for (int j = 1; j < tn; ++j) acc += tk[j] * S[reflect101(x - a + j, cols)];
                tmp[e] = acc;
            }
            __syncthreads();
            for (int e = tid; e < plane; e += 1024) {  // column pass (reflected rows), DoG
                const int y = e / cols, x = e - y * cols;
                float acc = tk[a] * tmp[e] + 0.f;
                for (int j = 1; j <= a; ++j)
                    acc += tk[a + j] * (tmp[reflect101(y + j, rows) * cols + x] + tmp[reflect101(y - j, rows) * cols + x]);
                bufB[e] = acc;
                G[(long long)i * plane + e] = acc;
                D[(long long)(i - 1) * plane + e] = acc - bufA[e];
            }
            __syncthreads();
            if (i == kNOL && o + 1 < o_end) {
                const int nc = py->gauss[o + 1][0].cols, np = py->gauss[o + 1][0].rows * nc;
                for (int e = tid; e < np; e += 1024) {
                    const int y = e / nc, x = e - y * nc;
                    nxt[e] = bufB[(2 * y) * cols + 2 * x];
                }
            }
            float* sw = bufA;
            bufA = bufB;
            bufB = sw;
            __syncthreads();
        }
    }
}

struct DownB {
    Flat f;
    const float* src[kMaxImg];
    int scols[kMaxImg];
    float* dst[kMaxImg];
    int cols[kMaxImg];
};

__global__ void down2_kernel(DownB A) {
    int bx, y;
    const int j = flat_job(A.f, blockIdx.x, bx, y);
    const int x = bx * blockDim.x + threadIdx.x, cols = A.cols[j];
    if (x >= cols) return;
    A.dst[j][(size_t)y * cols + x] = A.src[j][(size_t)(2 * y) * A.scols[j] + 2 * x];
}

// the 5 DoG layers of one octave (blockIdx.y = layer): dog[i] = gauss[i + 1] - gauss[i]
struct Cand {
    int o, layer, r, c;
};

// findScaleSpaceExtrema's pixel test over layers 1..3 of one octave (blockIdx.z = layer - 1), every image
// of the batch with that octave
struct ExtB {
    Flat f;
    const float* dog[kMaxImg];
    int rows[kMaxImg], cols[kMaxImg];
    Cand* cand[kMaxImg];
    int* n_cand[kMaxImg];
    int octave, threshold, cap;
};

// One block per kExtTW x kExtTH tile of one layer: the tile of the three DoG planes (one-pixel halo) staged
// in LDS with coalesced loads, the 26-neighbour test per pixel from LDS, the block's extrema gathered in an
// LDS list and appended with ONE global atomic per block.  Round 5's one-thread-per-pixel form (26 global
// loads per pixel over the threshold, one returning atomic per wave with an extremum on the single
// counter) took 259 us on octave 0 of a 640x480 scene (profiles/r06d_c1img_timeline_rank.txt).
constexpr int kExtTW = 64, kExtTH = 16, kExtW = kExtTW + 2, kExtH = kExtTH + 2;

__global__ __launch_bounds__(256) void extrema_kernel(ExtB A) {
    static_assert(kExtTW == 64 && kExtW - 64 <= 64, "one tile row per wave, lane = column");
    __shared__ float t[3][kExtH][kExtW];
    __shared__ Cand list[kExtTW * kExtTH];
    __shared__ int n_list, base;
    int bx, by;
    const int j = flat_job(A.f, blockIdx.x, bx, by);
    const float* __restrict__ dog = A.dog[j];
    const int rows = A.rows[j], cols = A.cols[j], octave = A.octave, threshold = A.threshold, cap = A.cap;
    const int layer = blockIdx.z + 1, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r0 = kBorder + by * kExtTH, c0 = kBorder + bx * kExtTW;  // first pixel of the tile
    const size_t plane = (size_t)rows * cols;
    if (tid == 0) n_list = 0;
    // staging: wave w loads tile rows w, w + 4, ... of the three planes (lane = column; the two halo
    // columns past 64 by lanes 0, 1), every load in flight before the LDS writes.  Rows/columns past
    // the last tested pixel are clamped into the image: only pixels outside the tested range
    // [kBorder, rows|cols - kBorder) ever read them.
    constexpr int kRows = 3 * kExtH, kRPW = (kRows + 3) / 4;
    const int xa = min(c0 - 1 + lane, cols - 1), xb = min(c0 + 63 + lane, cols - 1);
    float va[kRPW], vb[kRPW];
#pragma unroll
    for (int i = 0; i < kRPW; ++i) {
        const int row = wv + 4 * i;
        if (row < kRows) {
            const int z = row / kExtH, r = row - z * kExtH;
            const float* bp = dog + (layer - 1 + z) * plane + (size_t)min(r0 - 1 + r, rows - 1) * cols;
            va[i] = bp[xa];
            if (lane < kExtW - 64) vb[i] = bp[xb];
        }
    }
#pragma unroll
    for (int i = 0; i < kRPW; ++i) {
        const int row = wv + 4 * i;
        if (row < kRows) {
            float* tr = &t[0][0][0] + row * kExtW;
            tr[lane] = va[i];
            if (lane < kExtW - 64) tr[64 + lane] = vb[i];
        }
    }
    __syncthreads();
    // wave w tests tile rows w, w + 4, w + 8, w + 12 (lane = column).  OpenCV's predicate (val >= every
    // neighbour for val > 0, val <= every neighbour otherwise) as one comparison against the max / min
    // of the 26 neighbours (finite values: the same outcome)
#pragma unroll
    for (int u = 0; u < kExtTH / 4; ++u) {
        const int lr = wv + 4 * u, lc = lane, r = r0 + lr, c = c0 + lc;
        if (r >= rows - kBorder || c >= cols - kBorder) continue;
        const float val = t[1][lr + 1][lc + 1];
        if (!(fabsf(val) > (float)threshold)) continue;
        float mx = t[0][lr][lc], mn = mx;
#pragma unroll
        for (int dz = 0; dz < 3; ++dz)
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    if ((dz == 1 && dy == 1 && dx == 1) || (dz == 0 && dy == 0 && dx == 0)) continue;
                    const float nb = t[dz][lr + dy][lc + dx];
                    mx = fmaxf(mx, nb);
                    mn = fminf(mn, nb);
                }
        if (val > 0 ? val >= mx : val <= mn) list[atomicAdd(&n_list, 1)] = Cand{octave, layer, r, c};
    }
    __syncthreads();
    const int n = n_list;
    if (n == 0) return;
    if (tid == 0) base = atomicAdd(A.n_cand[j], n);
    __syncthreads();
    Cand* __restrict__ cand = A.cand[j];
    for (int i = tid; i < n; i += 256)
        if (base + i < cap) cand[base + i] = list[i];
}

#define AT(L, r, c) ((L).p[(size_t)(r) * (L).cols + (c)])

// OpenCV fastAtan2 (degrees)
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI), p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI), p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// Matx33f::solve(DECOMP_LU) for 3x3: Cramer with the float determinant
__device__ __forceinline__ bool solve3(const float* H, const float* b, float* x) {
    float d = H[0] * (H[4] * H[8] - H[7] * H[5]) - H[1] * (H[3] * H[8] - H[6] * H[5]) + H[2] * (H[3] * H[7] - H[6] * H[4]);
    if (d == 0) return false;
    d = 1 / d;
    x[0] = d * (b[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (b[1] * H[8] - H[5] * b[2]) + H[2] * (b[1] * H[7] - H[4] * b[2]));
    x[1] = d * (H[0] * (b[1] * H[8] - H[5] * b[2]) - b[0] * (H[3] * H[8] - H[5] * H[6]) + H[2] * (H[3] * b[2] - b[1] * H[6]));
    x[2] = d * (H[0] * (H[4] * b[2] - b[1] * H[7]) - H[1] * (H[3] * b[2] - b[1] * H[6]) + b[0] * (H[3] * H[7] - H[4] * H[6]));
    return true;
}

struct Surv {  // an extremum that passed adjustLocalExtrema: its keypoint (angle 0) and DoG position
    mim_keypoint k;
    int r, c, layer;
};

// adjustLocalExtrema (<= 5 Newton steps, contrast and edge tests), one thread per candidate; the
// survivors go to orient_kernel (octave field packed as OpenCV's)
struct RefB {
    const Pyr* pyr[kMaxImg];
    const Cand* cand[kMaxImg];
    const int* n_cand[kMaxImg];
    Surv* surv[kMaxImg];
    int* n_surv[kMaxImg];
    int cap, surv_cap;
};

__global__ void refine_kernel(RefB A) {  // blockIdx.y = image
  const int j = blockIdx.y;
  const Pyr* __restrict__ pyr = A.pyr[j];
  const Cand* __restrict__ cand = A.cand[j];
  Surv* __restrict__ surv = A.surv[j];
  int* __restrict__ n_surv = A.n_surv[j];
  const int surv_cap = A.surv_cap;
  const int n_c = min(*A.n_cand[j], A.cap);
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n_c; t += gridDim.x * blockDim.x) {  // fixed grid
    const float kSigma = 1.6f, kContrast = 0.04f, kEdge = 10.f;
    const float img_scale = 1.f / 255, deriv_scale = img_scale * 0.5f, second_deriv_scale = img_scale;
    const float cross_deriv_scale = img_scale * 0.25f;
    const Cand cd = cand[t];
    const int octv = cd.o;
    int layer = cd.layer, r = cd.r, c = cd.c;
    float xi = 0, xr = 0, xc = 0, contr = 0;
    int i = 0;
    for (; i < 5; i++) {
        const Layer im = pyr->dog[octv][layer], pv = pyr->dog[octv][layer - 1], nx = pyr->dog[octv][layer + 1];
        const float dD[3] = {(AT(im, r, c + 1) - AT(im, r, c - 1)) * deriv_scale,
                             (AT(im, r + 1, c) - AT(im, r - 1, c)) * deriv_scale,
                             (AT(nx, r, c) - AT(pv, r, c)) * deriv_scale};
        const float v2 = AT(im, r, c) * 2;
        const float dxx = (AT(im, r, c + 1) + AT(im, r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (AT(im, r + 1, c) + AT(im, r - 1, c) - v2) * second_deriv_scale;
        const float dss = (AT(nx, r, c) + AT(pv, r, c) - v2) * second_deriv_scale;
        const float dxy = (AT(im, r + 1, c + 1) - AT(im, r + 1, c - 1) - AT(im, r - 1, c + 1) + AT(im, r - 1, c - 1)) * cross_deriv_scale;
        const float dxs = (AT(nx, r, c + 1) - AT(nx, r, c - 1) - AT(pv, r, c + 1) + AT(pv, r, c - 1)) * cross_deriv_scale;
        const float dys = (AT(nx, r + 1, c) - AT(nx, r - 1, c) - AT(pv, r + 1, c) + AT(pv, r - 1, c)) * cross_deriv_scale;
        const float H[9] = {dxx, dxy, dxs, dxy, dyy, dys, dxs, dys, dss};
        float X[3] = {0, 0, 0};
        if (!solve3(H, dD, X)) X[0] = X[1] = X[2] = 0;
        xi = -X[2];
        xr = -X[1];
        xc = -X[0];
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        if (fabsf(xi) > (float)(INT_MAX / 3) || fabsf(xr) > (float)(INT_MAX / 3) || fabsf(xc) > (float)(INT_MAX / 3)) {
            i = 6;  // diverged: rejected
            break;
        }
        c += cv_round(xc);
        r += cv_round(xr);
        layer += cv_round(xi);
        if (layer < 1 || layer > kNOL || c < kBorder || c >= im.cols - kBorder || r < kBorder || r >= im.rows - kBorder) {
            i = 6;  // left the scale space: rejected
            break;
        }
    }
    if (i >= 5) continue;  // no convergence in 5 steps (or rejected above)
    {
        const Layer im = pyr->dog[octv][layer], pv = pyr->dog[octv][layer - 1], nx = pyr->dog[octv][layer + 1];
        const float dD[3] = {(AT(im, r, c + 1) - AT(im, r, c - 1)) * deriv_scale,
                             (AT(im, r + 1, c) - AT(im, r - 1, c)) * deriv_scale,
                             (AT(nx, r, c) - AT(pv, r, c)) * deriv_scale};
        const float tt = dD[0] * xc + dD[1] * xr + dD[2] * xi;
        contr = AT(im, r, c) * img_scale + tt * 0.5f;
        if (fabsf(contr) * kNOL < kContrast) continue;
        const float v2 = AT(im, r, c) * 2.f;
        const float dxx = (AT(im, r, c + 1) + AT(im, r, c - 1) - v2) * second_deriv_scale;
        const float dyy = (AT(im, r + 1, c) + AT(im, r - 1, c) - v2) * second_deriv_scale;
        const float dxy = (AT(im, r + 1, c + 1) - AT(im, r + 1, c - 1) - AT(im, r - 1, c + 1) + AT(im, r - 1, c - 1)) * cross_deriv_scale;
        const float tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
        if (det <= 0 || tr * tr * kEdge >= (kEdge + 1) * (kEdge + 1) * det) continue;
    }
    mim_keypoint k;
    k.x = (c + xc) * (1 << octv);
    k.y = (r + xr) * (1 << octv);
    k.octave = octv + (layer << 8) + (cv_round_d((xi + 0.5) * 255) << 16);
    k.size = kSigma * (float)pow(2.0, (double)((layer + xi) / kNOL)) * (1 << octv) * 2;
    k.response = fabsf(contr);
    k.angle = 0;

    const int slot = atomicAdd(n_surv, 1);
    if (slot < surv_cap) surv[slot] = Surv{k, r, c, layer};
  }
}

// calcOrientationHist + the peak loop of findScaleSpaceExtrema, one wave per surviving extremum.  The
// 36 bins accumulate in the reference's pixel order: per batch of 64 patch pixels each lane computes
// one pixel's (bin, weight * magnitude), then the lanes walk the batch in order and lane b adds the
// values of bin b (one bin per pixel: no reordering).  Keypoints in the doubled image's coordinates.
struct OriB {
    const Pyr* pyr[kMaxImg];
    const Surv* surv[kMaxImg];
    const int* n_surv[kMaxImg];
    mim_keypoint* kp[kMaxImg];
    int* n_kp[kMaxImg];
    int surv_cap, kp_cap;
};

// Four survivors per 256-thread block, one per wave: the waves synchronise among their own lanes only
// (their patches differ in size), and the block appends all its keypoints with ONE counter atomic.
// Round 5's one-survivor blocks did one returning atomic per keypoint on the image's single counter:
// 11.4 ns each serialised (profiles/r06e_atomic_probe.txt), ~60 us of a 5-scale scene's 234 us
// (r06h: the kernel without the counter, profiles/r06h_sift_ab.txt).
constexpr int kOriWaves = 4;
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ __launch_bounds__(64 * kOriWaves) void orient_kernel(OriB A) {  // blockIdx.y = image
    __shared__ int rb_[kOriWaves][64];
    __shared__ float rv_[kOriWaves][64];
    __shared__ float th_[kOriWaves][kOriBins + 4];
    __shared__ float pang[kOriWaves][kOriBins];  // the angles of each wave's keypoints, in peak order
    __shared__ int npk[kOriWaves], base;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, j = blockIdx.y;
    int* rb = rb_[wv];
    float* rv = rv_[wv];
    float* th = th_[wv];
    const Pyr* __restrict__ pyr = A.pyr[j];
    const Surv* __restrict__ surv = A.surv[j];
    mim_keypoint* __restrict__ kp = A.kp[j];
    int* __restrict__ n_kp = A.n_kp[j];
    const int kp_cap = A.kp_cap;
  const int n_s = min(*A.n_surv[j], A.surv_cap);
  for (int t0 = blockIdx.x * kOriWaves; t0 < n_s; t0 += gridDim.x * kOriWaves) {  // block-uniform loop
    const int t = t0 + wv;
    mim_keypoint k{};
    if (lane == 0) npk[wv] = 0;
    if (t < n_s) {
    const Surv sv = surv[t];
    k = sv.k;
    const int octv = k.octave & 255;
    const Layer g = pyr->gauss[octv][sv.layer];
    const float scl_octv = k.size * 0.5f / (1 << octv);
    const int radius = cv_round(4.5f * scl_octv);
    const float sigma = 1.5f * scl_octv;
    const float expf_scale = -1.f / (2.f * sigma * sigma);
    const int W = 2 * radius + 1, P = W * W;
    float acc = 0.f;  // th[lane + 2] for lane < 36
    // the four gradient reads of a batch's pixel are issued one batch ahead (software pipelined): a
    // batch's loads are in flight while the previous batch's sums run
    auto fetch = [&](int b, float& xr, float& xl, float& yu, float& yd) {
        const int q = b + lane;
        if (q < P) {
            const int ii = q / W - radius, j = q % W - radius;
            const int y = sv.r + ii, x = sv.c + j;
            if (y > 0 && y < g.rows - 1 && x > 0 && x < g.cols - 1) {
                xr = AT(g, y, x + 1);
                xl = AT(g, y, x - 1);
                yu = AT(g, y - 1, x);
                yd = AT(g, y + 1, x);
            }
        }
    };
    float nxr = 0.f, nxl = 0.f, nyu = 0.f, nyd = 0.f;
    fetch(0, nxr, nxl, nyu, nyd);
    for (int base = 0; base < P; base += 64) {
        const float cxr = nxr, cxl = nxl, cyu = nyu, cyd = nyd;
        if (base + 64 < P) fetch(base + 64, nxr, nxl, nyu, nyd);
        const int q = base + lane;
        int bin = -1;
        float val = 0.f;
        if (q < P) {
            const int ii = q / W - radius, j = q % W - radius;
            const int y = sv.r + ii, x = sv.c + j;
            if (y > 0 && y < g.rows - 1 && x > 0 && x < g.cols - 1) {
                const float dx = cxr - cxl;
                const float dy = cyu - cyd;
                const float w = (float)exp((double)((float)(ii * ii + j * j) * expf_scale));
                const float ori = fast_atan2(dy, dx);
                const float mag = sqrtf(dx * dx + dy * dy);
                bin = cv_round((kOriBins / 360.f) * ori);
                if (bin >= kOriBins) bin -= kOriBins;
                if (bin < 0) bin += kOriBins;
                val = w * mag;
            }
        }
        rb[lane] = bin;
        rv[lane] = val;
        wave_sync();
        const int m = min(64, P - base);
        // unrolled: the batch's (bin, value) reads are broadcast LDS loads independent of the sums, so
        // 16 issue back to back instead of one dependent round trip per pixel (the adds stay in order)
#pragma unroll 16
        for (int i = 0; i < m; ++i) {
            const int bi = rb[i];
            const float vi = rv[i], sum = acc + vi;
            acc = bi == lane ? sum : acc;
        }
        wave_sync();
    }
    if (lane < kOriBins) th[lane + 2] = acc;
    wave_sync();
    if (lane == 0) {
    th[1] = th[kOriBins + 1];
    th[0] = th[kOriBins];
    th[kOriBins + 2] = th[2];
    th[kOriBins + 3] = th[3];
    float hist[kOriBins];
    float mx = 0;
    for (int b = 0; b < kOriBins; b++) {
        hist[b] = (th[b] + th[b + 4]) * (1.f / 16.f) + (th[b + 1] + th[b + 3]) * (4.f / 16.f) + th[b + 2] * (6.f / 16.f);
        mx = b == 0 ? hist[0] : fmaxf(mx, hist[b]);
    }
    const float mag_thr = mx * 0.8f;
    int np = 0;
    for (int j = 0; j < kOriBins; j++) {
        const int l = j > 0 ? j - 1 : kOriBins - 1, r2 = j < kOriBins - 1 ? j + 1 : 0;
        if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
            float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
            bin = bin < 0 ? kOriBins + bin : (bin >= kOriBins ? bin - kOriBins : bin);
            float angle = 360.f - (float)((360.f / kOriBins) * bin);
            if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
            pang[wv][np++] = angle;
        }
    }
    npk[wv] = np;
    }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
#pragma unroll
        for (int w = 0; w < kOriWaves; ++w) tot += npk[w];
        base = tot ? atomicAdd(n_kp, tot) : 0;
    }
    __syncthreads();
    int off = base;
    for (int w = 0; w < wv; ++w) off += npk[w];
    if (lane < npk[wv]) {
        const int slot = off + lane;
        k.angle = pang[wv][lane];
        if (slot < kp_cap) kp[slot] = k;
    }
    __syncthreads();  // rb, rv, th, pang, npk, base reused by the block's next survivors
  }
}

__device__ __forceinline__ int ctz64(unsigned long long m) { return __builtin_ctzll(m); }

// calcSIFTDescriptor, one 256-thread block per keypoint (keypoints in input coordinates, octave field
// packed as OpenCV's).  Every bin must receive its contributions in the reference's pixel order
// (row-major over the patch), so the work splits in two per batch of 256 consecutive patch pixels:
//   A  each thread computes one pixel's contribution (gradient, fastAtan2, the double-rounded exp
//      weight) and its 8 trilinear values with the reference's own operations (v_r1 = mag rbin,
//      v_r0 = mag - v_r1, v_rc11 = v_r1 cbin, ...) in registers, and sets its bit in the 256-bit
//      pixel masks of its 8 target bins idx + {0, 1, 10, 11, 60, 61, 70, 71} (LDS ORs, order-free);
//   B  a stable counting sort of the batch's contributions by bin: per bin the masks give its total
//      and each pixel's rank among the pixels hitting it (popcounts), a block scan the segments, and
//      every value is written to its bin's segment at its rank; thread b then adds the segments of
//      bins b and b + 256 in order, so every bin's sum runs in pixel order: the oracle's float sums,
//      bit for bit, with independent LDS reads instead of a dependent round trip per contribution.
// The wrap, the 0.2 clamp and the x 512 normalisation then run on wave 0 in the reference's order.
// Round 5: only about half the (2 radius + 1)^2 patch can pass the window test (the rotated 5 x 5-cell
// square inside its circumscribed square), so the batches run over a compacted patch: per row a
// conservative column range from the window's two linear constraints (in double, widened by a value
// margin and one pixel, intersected with the image), rows concatenated in order.  The exact float test
// still decides every pixel, and the excluded pixels are ones it rejects, so the contributions and
// their pixel order are unchanged.  Patches of more than kDescrRowsMax rows take the full square.
// (Round 3 history: one wave walking the pixels one at a time, 0.76 ms per call; one wave with 64-bit
// masks walked by the owners, 0.64 ms; 256 threads with the mask walk, 0.37 ms: each contribution a
// dependent chain of two LDS reads.)
#ifndef MIM_PROBE_DESCR
#define MIM_PROBE_DESCR 0
#endif
#ifndef MIM_DESCR_SPLIT
#define MIM_DESCR_SPLIT 0  // batched SIFT: one descriptor launch per image instead of one for all
#endif
#ifndef MIM_DESCR_GRID
#define MIM_DESCR_GRID 4096  // descriptor blocks of a batch launch (at least 1024 per image)
#endif
constexpr int kDescrT = 256;        // threads of a descriptor block: pixels per batch of a patch
[[maybe_unused]] constexpr int kDescrTBig = 1024;    // MIM_DESCR_BIG_SPLIT: the large patches by 1024-thread blocks
constexpr int kDescrRowsMax = 512;
// MIM_DESCR_BIG_SPLIT (off; measured slower, r06c): patches wider than MIM_DESCR_BIG_W described by
// kDescrTBig blocks in a launch of their own (4x fewer batches in their chains).  The launch is bound by
// the blocks resident per CU (4 at 108 VGPRs) times each block's chain of batches, so the split only
// lengthened it; a software prefetch of the next batch's gradient loads and a 5-block register cap were
// even (r06d)
#ifndef MIM_DESCR_BIG_W
#define MIM_DESCR_BIG_W 64
#endif
#ifndef MIM_DESCR_BIG_SPLIT
#define MIM_DESCR_BIG_SPLIT 0
#endif

// columns j of one patch row with a j + b in (-2.5, 2.5) (c_rot or r_rot of the window test, rbin /
// cbin in (-1, kDW)), intersected into [lo, hi]: conservative (value margin 1e-3, one pixel each side)
__device__ __forceinline__ void window_cols(double a, double b, int& lo, int& hi) {
    constexpr double kM = 2.5 + 1e-3;
    if (fabs(a) < 1e-30) {
        if (fabs(b) >= kM) hi = lo - 1;
        return;
    }
    double j0 = (-kM - b) / a, j1 = (kM - b) / a;
    if (j0 > j1) { const double t = j0; j0 = j1; j1 = t; }
    j0 = fmax(j0, -1e9);
    j1 = fmin(j1, 1e9);
    lo = max(lo, (int)floor(j0));
    hi = min(hi, (int)ceil(j1));
}
struct DescB {
    const Pyr* pyr[kMaxImg];
    const mim_keypoint* kp[kMaxImg];
    const int* n[kMaxImg];
    int n_cap[kMaxImg];
    float* desc[kMaxImg];
};

// T threads per block (kDescrT or kDescrTBig); cls: which keypoints the launch describes by patch width W
// (0: W <= MIM_DESCR_BIG_W, 1: W > MIM_DESCR_BIG_W, -1: all).  The result does not depend on T: a bin's
// values are summed in pixel order across the batches whatever their size.
template <int T>
__global__ __launch_bounds__(T) void descr_kernel(DescB A, int cls) {  // blockIdx.y = image
    constexpr int kWords = T / 64;                          // mask words per bin (one per wave)
    constexpr int kBinsPer = (kHistLen + T - 1) / T;        // bins owned per thread
    constexpr int kRowsPer = (kDescrRowsMax + T - 1) / T;   // compacted patch rows per thread
    const Pyr* __restrict__ pyr = A.pyr[blockIdx.y];
    const mim_keypoint* __restrict__ kp = A.kp[blockIdx.y];
    float* __restrict__ desc = A.desc[blockIdx.y];
    __shared__ float hist[kHistLen];
    __shared__ unsigned long long bm[kHistLen][kWords];  // per bin: the batch's pixels that hit it
    __shared__ unsigned short pre[kHistLen][kWords];      // per bin and word: pixels in earlier words
    __shared__ int seg[kHistLen];                         // per bin: its segment of `sorted`
    __shared__ int wsum[kWords];
    __shared__ float sorted[T * 8];                       // the batch's values grouped by bin
    __shared__ int row_off[kDescrRowsMax + 1], row_lo[kDescrRowsMax];  // the compacted patch's rows
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int e = tid; e < kHistLen * kWords; e += T) (&bm[0][0])[e] = 0ull;
    __syncthreads();
  const int n = min(*A.n[blockIdx.y], A.n_cap[blockIdx.y]);
  for (int t = blockIdx.x; t < n; t += gridDim.x) {  // fixed grid, block-uniform loop
    const mim_keypoint p = kp[t];
    int octave = p.octave & 255;
    const int layer = (p.octave >> 8) & 255;
    octave = octave < 128 ? octave : (-128 | octave);
    const float scale = octave >= 0 ? 1.f / (1 << octave) : (float)(1 << -octave);
    const float size = p.size * scale;
    const Layer im = pyr->gauss[octave + 1][layer];
    float ori = 360.f - p.angle;
    if (fabsf(ori - 360.f) < FLT_EPSILON) ori = 0.f;
    const float scl = size * 0.5f;
    const int px = cv_round(p.x * scale), py = cv_round(p.y * scale);
    float cos_t = (float)cos((double)(ori * (float)(M_PI / 180))), sin_t = (float)sin((double)(ori * (float)(M_PI / 180)));
    const float bins_per_rad = kDB / 360.f, exp_scale = -1.f / (kDW * kDW * 0.5f);
    const float hist_width = 3.f * scl;
    int radius = cv_round(hist_width * 1.4142135623730951f * (kDW + 1) * 0.5f);
    const int rmax = (int)sqrt((double)im.cols * im.cols + (double)im.rows * im.rows);
    if (radius > rmax) radius = rmax;
    cos_t /= hist_width;
    sin_t /= hist_width;
    const int W = 2 * radius + 1;
    if (cls >= 0 && (W > MIM_DESCR_BIG_W) != (cls == 1)) continue;  // the other launch's keypoint (block-uniform)
    const bool compact = W <= kDescrRowsMax;
    int P = W * W;
    if (compact) {  // per row: the first column and the count of the conservative range, then offsets
        int len[kRowsPer];
#pragma unroll
        for (int k = 0; k < kRowsPer; ++k) {
            len[k] = 0;
            const int rr = kRowsPer * tid + k;
            if (rr < W) {
                const int i = rr - radius, r = py + i;
                int lo = max(-radius, 1 - px), hi = min(radius, im.cols - 2 - px);
                if (r <= 0 || r >= im.rows - 1) hi = lo - 1;
                window_cols((double)sin_t, (double)i * (double)cos_t, lo, hi);  // r_rot = j sin_t + i cos_t
                window_cols((double)cos_t, -(double)i * (double)sin_t, lo, hi);  // c_rot = j cos_t - i sin_t
                len[k] = max(0, hi - lo + 1);
                row_lo[rr] = lo;
            }
        }
        int mine = 0;
#pragma unroll
        for (int k = 0; k < kRowsPer; ++k) mine += len[k];
        int incl = mine;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int excl = incl - mine;
#pragma unroll
        for (int w = 0; w < kWords; ++w) excl += w < wv ? wsum[w] : 0;
#pragma unroll
        for (int k = 0, o = excl; k < kRowsPer; o += len[k], ++k)
            if (kRowsPer * tid + k < W) row_off[kRowsPer * tid + k] = o;
        if (tid == T - 1) row_off[W] = excl + mine;  // the last thread's inclusive sum: the total
        __syncthreads();
        P = row_off[W];
        __syncthreads();  // wsum reused by the batches' scans
    }
    float hb[kBinsPer];  // bins tid + T s2
#pragma unroll
    for (int s2 = 0; s2 < kBinsPer; ++s2) hb[s2] = 0.f;
    for (int base = 0; base < P; base += T) {
        // ---- A: pixel base + tid ----
        int idx = -1;
        float vals[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        {
            const int q = base + tid;
            if (q < P) {
                int i, j;
                if (compact) {  // the row holding compacted pixel q: last rr with row_off[rr] <= q
                    int lo = 0, hi = W - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (row_off[mid] <= q) lo = mid; else hi = mid - 1;
                    }
                    i = lo - radius;
                    j = row_lo[lo] + (q - row_off[lo]);
                } else {
                    i = q / W - radius;
                    j = q % W - radius;
                }
                const float c_rot = j * cos_t - i * sin_t, r_rot = j * sin_t + i * cos_t;
                float rbin = r_rot + kDW / 2 - 0.5f, cbin = c_rot + kDW / 2 - 0.5f;
                const int r = py + i, c = px + j;
                if (rbin > -1 && rbin < kDW && cbin > -1 && cbin < kDW && r > 0 && r < im.rows - 1 && c > 0 &&
                    c < im.cols - 1) {
                    const float dx = AT(im, r, c + 1) - AT(im, r, c - 1), dy = AT(im, r - 1, c) - AT(im, r + 1, c);
#if MIM_PROBE_DESCR == 1  // timing probe only (not the reference's weights)
                    const float w = __expf((c_rot * c_rot + r_rot * r_rot) * exp_scale);
#else
                    const float w = (float)exp((double)((c_rot * c_rot + r_rot * r_rot) * exp_scale));
#endif
                    const float o = fast_atan2(dy, dx), m = sqrtf(dx * dx + dy * dy);
                    float obin = (o - ori) * bins_per_rad;
                    const float mag = m * w;
                    const int r0 = (int)floorf(rbin), c0 = (int)floorf(cbin);
                    int o0 = (int)floorf(obin);
                    const float rb = rbin - r0, cb = cbin - c0, ob = obin - o0;
                    if (o0 < 0) o0 += kDB;
                    if (o0 >= kDB) o0 -= kDB;
                    idx = ((r0 + 1) * (kDW + 2) + c0 + 1) * (kDB + 2) + o0;
                    // calcSIFTDescriptor's trilinear split, same operations
                    const float v_r1 = mag * rb, v_r0 = mag - v_r1;
                    const float v_rc11 = v_r1 * cb, v_rc10 = v_r1 - v_rc11;
                    const float v_rc01 = v_r0 * cb, v_rc00 = v_r0 - v_rc01;
                    vals[7] = v_rc11 * ob; vals[6] = v_rc11 - vals[7];
                    vals[5] = v_rc10 * ob; vals[4] = v_rc10 - vals[5];
                    vals[3] = v_rc01 * ob; vals[2] = v_rc01 - vals[3];
                    vals[1] = v_rc00 * ob; vals[0] = v_rc00 - vals[1];
                }
            }
        }
#if MIM_PROBE_DESCR == 2  // timing probe only: phase A alone
        hb[0] += vals[0] + vals[1] + vals[2] + vals[3] + vals[4] + vals[5] + vals[6] + vals[7] + (float)idx;
        continue;
#endif
        // ---- B: stable counting sort of the batch's contributions by bin, then sequential sums ----
        constexpr int kOff[8] = {0, 1, kDB + 2, kDB + 3, (kDW + 2) * (kDB + 2), (kDW + 2) * (kDB + 2) + 1,
                                 (kDW + 3) * (kDB + 2), (kDW + 3) * (kDB + 2) + 1};
        if (idx >= 0) {
            const unsigned long long bit = 1ull << lane;
#pragma unroll
            for (int k = 0; k < 8; ++k) atomicOr(&bm[idx + kOff[k]][wv], bit);
        }
        __syncthreads();
        // owned bins: per mask word the count of earlier pixels, and the bin's total
        int tot[kBinsPer];
#pragma unroll
        for (int s2 = 0; s2 < kBinsPer; ++s2) {
            tot[s2] = 0;
            const int bin = tid + T * s2;
            if (bin < kHistLen) {
                int run = 0;
#pragma unroll
                for (int w = 0; w < kWords; ++w) {
                    pre[bin][w] = (unsigned short)run;
                    run += __popcll(bm[bin][w]);
                }
                tot[s2] = run;
            }
        }
        // segment starts: exclusive scan of the owners' totals over the block
        int mine = 0;
#pragma unroll
        for (int s2 = 0; s2 < kBinsPer; ++s2) mine += tot[s2];
        int incl = mine;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int excl = incl - mine;
#pragma unroll
        for (int w = 0; w < kWords; ++w) excl += w < wv ? wsum[w] : 0;
        int st0[kBinsPer];  // the owned bins' segment starts (bins tid + T s2 are consecutive in `sorted`)
#pragma unroll
        for (int s2 = 0, o = excl; s2 < kBinsPer; o += tot[s2], ++s2) {
            st0[s2] = o;
            if (tid + T * s2 < kHistLen) seg[tid + T * s2] = o;
        }
        __syncthreads();
        // scatter: the pixel's value for bin b goes to b's segment at its rank among the batch's pixels
        // hitting b (the earlier pixels of its own mask word and the words before)
        if (idx >= 0) {
            const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int b = idx + kOff[k];
                sorted[seg[b] + pre[b][wv] + __popcll(bm[b][wv] & below)] = vals[k];
            }
        }
        __syncthreads();
        // owners: the bin's values in pixel order (independent LDS reads, one add chain)
#pragma unroll
        for (int s2 = 0; s2 < kBinsPer; ++s2) {
            const int bin = tid + T * s2;
            if (bin < kHistLen) {
                float acc = hb[s2];
#if MIM_PROBE_DESCR == 3  // timing probe only: no ordered sums
                acc += tot[s2] ? sorted[st0[s2]] : 0.f;
#else
#pragma unroll 4
                for (int i = 0; i < tot[s2]; ++i) acc += sorted[st0[s2] + i];
#endif
                hb[s2] = acc;
#pragma unroll
                for (int w = 0; w < kWords; ++w) bm[bin][w] = 0ull;  // cleared for the next batch
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int s2 = 0; s2 < kBinsPer; ++s2)
        if (tid + T * s2 < kHistLen) hist[tid + T * s2] = hb[s2];
    __syncthreads();
    // the orientation wrap (cells independent: one thread each)
    if (tid < kDW * kDW) {
        const int idx = ((tid / kDW + 1) * (kDW + 2) + (tid % kDW + 1)) * (kDB + 2);
        hist[idx] += hist[idx + kDB];
        hist[idx + 1] += hist[idx + kDB + 1];
    }
    __syncthreads();
    // wave 0: the two norms summed in the reference's order (descriptor index order) over values held
    // two per lane, the clamp and the x 512 rounding per lane
    if (wv == 0) {
    float v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int k = lane + 64 * u, cell = k / kDB;  // k = (i kDW + j) kDB + o
        v[u] = hist[((cell / kDW + 1) * (kDW + 2) + (cell % kDW + 1)) * (kDB + 2) + k % kDB];
    }
    auto ordered_sumsq = [&]() {
        const float q0 = v[0] * v[0], q1 = v[1] * v[1];
        float acc = 0;
        for (int k = 0; k < 64; ++k) acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q0), k));
        for (int k = 0; k < 64; ++k) acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(q1), k));
        return acc;
    };
    float nrm2 = ordered_sumsq();
    const float thr = sqrtf(nrm2) * 0.2f;
    v[0] = fminf(v[0], thr);
    v[1] = fminf(v[1], thr);
    nrm2 = ordered_sumsq();
    nrm2 = 512.f / fmaxf(sqrtf(nrm2), FLT_EPSILON);
    float* out = desc + (size_t)t * 128;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int r = cv_round(v[u] * nrm2);
        out[lane + 64 * u] = (float)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
    }
    __syncthreads();  // hist reused by the block's next keypoint
  }
}

// KeyPointsFilter::removeDuplicatedSorted (sort by KeypointGreater, drop consecutive keypoints equal in
// x, y, size and angle), the 1/2 rescale of the doubled image's octave -1 and runByPixelsMask, in that
// order (sift.dispatch.cpp detectAndCompute), on one 1024-thread block: a bitonic sort of the keypoint
// indices in LDS (the keys compared from the L2-resident list), then two ordered compactions.  More
// than kSortCap keypoints: *n_out = -n and the host finishes (sift_describe_host).
constexpr int kSortCap = 16384;
constexpr int kKeySortCap = 8192;  // keypoints sorted by LDS keys (more: comparisons on the keypoints)

// float -> uint32 with the same order (negative values reversed below the positive ones)
__device__ __forceinline__ unsigned f32_order_key(float f) {
    const unsigned u = __float_as_uint(f + 0.f);  // -0 -> +0: the comparison sees them equal
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ bool kp_greater_d(const mim_keypoint& a, const mim_keypoint& b) {  // KeypointGreater
    if (a.x != b.x) return a.x > b.x;
    if (a.y != b.y) return a.y > b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle > b.angle;
    if (a.response != b.response) return a.response > b.response;
    return a.octave > b.octave;
}

struct KpB {
    const mim_keypoint* kp[kMaxImg];
    const int* n_kp[kMaxImg];
    const uint8_t* mask[kMaxImg];
    long long mstep[kMaxImg];
    mim_keypoint* out[kMaxImg];
    int* n_out[kMaxImg];
    int kp_cap, sort_cap;
};

__global__ __launch_bounds__(1024) void kp_post_kernel(KpB A) {  // blockIdx.y = image
    const mim_keypoint* __restrict__ kp = A.kp[blockIdx.y];
    const int* __restrict__ n_kp = A.n_kp[blockIdx.y];
    const uint8_t* __restrict__ mask = A.mask[blockIdx.y];
    const long long mstep = A.mstep[blockIdx.y];
    mim_keypoint* __restrict__ out = A.out[blockIdx.y];
    int* __restrict__ n_out = A.n_out[blockIdx.y];
    const int kp_cap = A.kp_cap, sort_cap = A.sort_cap;
    __shared__ int idx[kSortCap];
    __shared__ unsigned long long skey[kKeySortCap];
    __shared__ int wsum[16];
    __shared__ int carry;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = min(*n_kp, kp_cap);
    if (n > sort_cap) {  // sort_cap <= kSortCap
        if (tid == 0) *n_out = -n;
        return;
    }
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = tid; i < P; i += 1024) idx[i] = i < n ? i : -1;  // -1: padding, sorts last
    if (P <= kKeySortCap)  // (x, y) as one order-preserving 64-bit key per keypoint, in LDS
        for (int i = tid; i < P; i += 1024) {
            unsigned long long key = 0;
            if (i < n) {
                const mim_keypoint q = kp[i];
                key = ((unsigned long long)f32_order_key(q.x) << 32) | f32_order_key(q.y);
            }
            skey[i] = key;
        }
    __syncthreads();
    // before(a, b): a precedes b in KeypointGreater order (padding never precedes)
    auto before = [&](int a, int b) { return a >= 0 && (b < 0 || kp_greater_d(kp[a], kp[b])); };
    if (P <= kKeySortCap) {
        // bitonic sort of (key, index) pairs in LDS by the key alone, then the runs of equal keys
        // (duplicate positions: a keypoint's extra orientations) put in KeypointGreater order by the full
        // comparison.  KeypointGreater compares x, then y first, so the key decides every pair with
        // different (x, y).  Was (to round 6): the full comparison inside the network on equal keys, a
        // dependent L2 read in most of its ~90 barrier-separated stages (~300 us per 5-scale scene).
        // One compare-exchange per thread and pair, the pairs enumerated directly (no idle half).
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int q = tid; q < P / 2; q += 1024) {
                    const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), l = i | j;
                    const unsigned long long ka = skey[i], kb = skey[l];
                    if ((i & k) == 0 ? kb > ka : ka > kb) {
                        const int a = idx[i], b = idx[l];
                        idx[i] = b;
                        idx[l] = a;
                        skey[i] = kb;
                        skey[l] = ka;
                    }
                }
                __syncthreads();
            }
        // runs of equal keys (padding, key 0, is never part of one: it sorts after every keypoint)
        for (int i = tid; i < n; i += 1024) {
            const unsigned long long ki = skey[i];
            if ((i > 0 && skey[i - 1] == ki) || i + 1 >= n || skey[i + 1] != ki) continue;
            int e = i + 2;
            while (e < n && skey[e] == ki) ++e;
            for (int u = i + 1; u < e; ++u) {  // insertion sort of idx[i, e) (a stable order for ties)
                const int v = idx[u];
                const mim_keypoint kv = kp[v];
                int w = u;
                while (w > i && kp_greater_d(kv, kp[idx[w - 1]])) {
                    idx[w] = idx[w - 1];
                    --w;
                }
                idx[w] = v;
            }
        }
        __syncthreads();
    } else {
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = tid; i < P; i += 1024) {
                    const int l = i ^ j;
                    if (l > i) {
                        const int a = idx[i], b = idx[l];
                        if ((i & k) == 0 ? before(b, a) : before(a, b)) {
                            idx[i] = b;
                            idx[l] = a;
                        }
                    }
                }
                __syncthreads();
            }
    }
    // dedupe (keep the first of equal x, y, size, angle), rescale, mask; ordered compaction in chunks
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int i = base + tid;
        bool keep = false;
        mim_keypoint k{};
        if (i < n) {
            k = kp[idx[i]];
            keep = true;
            if (i > 0) {
                const mim_keypoint& q = kp[idx[i - 1]];
                keep = !(q.x == k.x && q.y == k.y && q.size == k.size && q.angle == k.angle);
            }
            if (keep) {
                k.octave = (k.octave & ~255) | ((k.octave - 1) & 255);
                k.x *= 0.5f;
                k.y *= 0.5f;
                k.size *= 0.5f;
                if (mask) keep = mask[(long long)(int)(k.y + 0.5f) * mstep + (int)(k.x + 0.5f)] != 0;
            }
        }
        const unsigned long long bal = __ballot(keep);
        const int within = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        if (lane == 0) wsum[wave] = __popcll(bal);
        __syncthreads();
        int before_w = 0, all = 0;
        for (int w = 0; w < 16; ++w) {
            before_w += w < wave ? wsum[w] : 0;
            all += wsum[w];
        }
        if (keep) out[carry + before_w + within] = k;
        __syncthreads();
        if (tid == 0) carry += all;
        __syncthreads();
    }
    if (tid == 0) *n_out = carry;
}

// ---- host ---------------------------------------------------------------------------------------

int gauss_taps(double sigma, Taps& t) {
    const int n = (int)lrint(sigma * 4 * 2 + 1) | 1;
    if (n > 64) return -1;
    const double scale2X = -0.5 / (sigma * sigma);
    double sum = 0;
    for (int i = 0; i < n; ++i) {
        const double x = i - (n - 1) * 0.5;
        t.k[i] = (float)exp(scale2X * x * x);
        sum += t.k[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < n; ++i) t.k[i] = (float)(t.k[i] * sum);
    t.n = n;
    return n;
}

bool kp_greater(const mim_keypoint& a, const mim_keypoint& b) {  // KeypointGreater
    if (a.x != b.x) return a.x > b.x;
    if (a.y != b.y) return a.y > b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle > b.angle;
    if (a.response != b.response) return a.response > b.response;
    return a.octave > b.octave;
}

}  // namespace

struct SiftWs {
    void* img = nullptr;   size_t img_cap = 0;
    void* pyr = nullptr;   size_t pyr_cap = 0;
    void* tmp = nullptr;   size_t tmp_cap = 0;
    void* aux = nullptr;   size_t aux_cap = 0;  // candidates, keypoints, counters, Pyr table
    void* desc = nullptr;  size_t desc_cap = 0;
    void* batch = nullptr; size_t batch_cap = 0;  // a call's Pyr tables and counters (batch owner only)
    Pyr* h_pyr = nullptr;  // pinned staging of the Pyr tables
    int* h_cnt = nullptr;  // pinned copy of the counters
    // pinned staging of the caller's 8-bit planes (0: image, 1: mask), see stage_h2d
    struct Stage {
        uint8_t* p = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;  // recorded after the copy out of p
    } stage[2];
};

static hipError_t grow(void*& p, size_t& cap, size_t need) {
    if (need <= cap) return hipSuccess;
    if (p) {
        hipError_t e = hipFree(p);
        if (e != hipSuccess) return e;
        p = nullptr;
        cap = 0;
    }
    const size_t want = need + need / 4;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
}

SiftWs* sift_ws_create() { return new SiftWs(); }

void sift_ws_destroy(SiftWs* w) {
    if (!w) return;
    for (void* p : {w->img, w->pyr, w->tmp, w->aux, w->desc, w->batch})
        if (p) (void)hipFree(p);
    if (w->h_pyr) (void)hipHostFree(w->h_pyr);
    if (w->h_cnt) (void)hipHostFree(w->h_cnt);
    for (auto& S : w->stage) {
        if (S.ev) (void)hipEventSynchronize(S.ev), (void)hipEventDestroy(S.ev);
        if (S.p) (void)hipHostFree(S.p);
    }
    delete w;
}

#define SCHK(x)                                              \
    do {                                                     \
        hipError_t e_ = (x);                                 \
        if (e_ != hipSuccess) {                              \
            err = std::string(#x) + ": " + hipGetErrorString(e_); \
            return -1;                                       \
        }                                                    \
    } while (0)

// rows x cols bytes of a caller's plane (row step `step`) to the device: copied on the host into the
// workspace's pinned stage, then one asynchronous copy.  hipMemcpy2DAsync straight from the caller's
// pageable rows took 11-27 ms per 640x480 image in some processes against ~25 us in others
// (profiles/r06g_sift_phases.txt).  The stage is reused only after its previous copy has completed.
static int stage_h2d(SiftWs* w, int slot, void* dst, const uint8_t* src, long long step, int cols, int rows,
                     hipStream_t st, std::string& err) {
    SiftWs::Stage& S = w->stage[slot];
    const size_t bytes = (size_t)rows * cols;
    if (bytes == 0) return 0;
    if (S.ev) SCHK(hipEventSynchronize(S.ev));
    else SCHK(hipEventCreateWithFlags(&S.ev, hipEventDisableTiming));
    if (bytes > S.cap) {
        if (S.p) SCHK(hipHostFree(S.p));
        S.p = nullptr;
        S.cap = 0;
        SCHK(hipHostMalloc((void**)&S.p, bytes + bytes / 4, hipHostMallocDefault));
        S.cap = bytes + bytes / 4;
    }
    if (step == cols) memcpy(S.p, src, bytes);
    else
        for (int r = 0; r < rows; ++r) memcpy(S.p + (size_t)r * cols, src + (size_t)r * step, cols);
    SCHK(hipMemcpyAsync(dst, S.p, bytes, hipMemcpyHostToDevice, st));
    SCHK(hipEventRecord(S.ev, st));
    return 0;
}

// One image of a SIFT call: its workspace (the 8-bit image already in w->img, rows x cols packed),
// its mask (host, optional), where its keypoints / descriptors go and their capacity.
struct SiftJob {
    SiftWs* w;
    int rows, cols;
    const uint8_t* mask;
    long long mstep;
    int cap;
    mim_keypoint* kps;
    float* desc;
    int n = 0;  // keypoints found (may exceed cap: then only cap are written)
    // internal
    int n_oct = 0, o_small = 0;
    int orows[16], ocols[16];
    size_t goff[16], doff[16];
    float* P = nullptr;   // pyramid: per octave kNOL + 3 Gaussian planes, then kNOL + 2 DoG planes
    float* T0 = nullptr;  // the doubled image
    Pyr h_pyr{};
    Pyr* d_pyr = nullptr;  // in the call's batch buffer
    int* d_cnt = nullptr;  // [0] candidates, [1] keypoints, [2] survivors, [3] final keypoints (batch buffer)
    int h_cnt[4] = {0, 0, 0, 0};
    Cand* d_cand = nullptr;
    mim_keypoint* d_kp = nullptr;
    Surv* d_surv = nullptr;
    mim_keypoint* d_kp2 = nullptr;  // the post-processed keypoints (kp_post_kernel)
    uint8_t* d_mask = nullptr;
    const mim_keypoint* out_kp = nullptr;  // the final keypoints on the device (d_kp2, or d_kp after the host path)
    std::vector<mim_keypoint> k;
};

constexpr int kCandCap = 1 << 20, kKpCap = 1 << 19;

// Test knobs (environment, read once): MIM_SIFT_CAND_CAP / MIM_SIFT_SORT_CAP lower the candidate
// capacity (past it: MIM_ELIMIT) and the device post-processing limit (past it: the host path of
// sift_describe_host), so that small images reach both paths (tests/test_sift_limits_gpu.py)
static int env_limit(const char* name, int dflt) {
    const char* e = getenv(name);
    const int v = e ? atoi(e) : 0;
    return v > 0 && v < dflt ? v : dflt;
}
static int cand_limit() {
    static const int v = env_limit("MIM_SIFT_CAND_CAP", kCandCap);
    return v;
}
static int sort_limit() {
    static const int v = env_limit("MIM_SIFT_SORT_CAP", kSortCap);
    return v;
}

// Flattened grid of one batched launch: image j gets gx[j] x gy[j] blocks
template <class F>
static int flatten(Flat& f, const std::vector<int>& imgs, F&& dims) {
    f.n = (int)imgs.size();
    int tot = 0;
    for (int k = 0; k < f.n; ++k) {
        int gx = 0, gy = 0;
        dims(imgs[k], gx, gy);
        f.off[k] = tot;
        f.gx[k] = std::max(gx, 1);
        tot += std::max(gx, 1) * std::max(gy, 0);
    }
    for (int k = f.n; k <= kMaxImg; ++k) f.off[k] = tot;
    return tot;
}

// Octave geometry, workspace buffers and the Pyr table of one image (host only)
static int sift_geometry(SiftJob& J, std::string& err) {
    SiftWs* w = J.w;
    const int R = J.rows * 2, C = J.cols * 2;
    J.n_oct = (int)lrint(log((double)std::min(R, C)) / log(2.) - 2) + 1;
    if (J.n_oct < 1) {  // no octave (sides < 2 px after doubling): no keypoints, as OpenCV
        J.n_oct = 0;
        return 0;
    }
    if (J.n_oct > 16) {
        err = "image too large for SIFT (more than 16 octaves)";
        return -4;
    }
    size_t total = 0;
    for (int o = 0; o < J.n_oct; ++o) {
        J.orows[o] = o == 0 ? R : J.orows[o - 1] / 2;
        J.ocols[o] = o == 0 ? C : J.ocols[o - 1] / 2;
        const size_t plane = (size_t)J.orows[o] * J.ocols[o];
        J.goff[o] = total;
        total += plane * (kNOL + 3);
        J.doff[o] = total;
        total += plane * (kNOL + 2);
    }
    // the small octaves (all after the first whose plane fits kSmallPlane) run in one block
    J.o_small = J.n_oct;
    for (int o = 1; o < J.n_oct; ++o)
        if ((size_t)J.orows[o] * J.ocols[o] <= (size_t)kSmallPlane) { J.o_small = o; break; }
    SCHK(grow(w->pyr, w->pyr_cap, total * sizeof(float)));
    SCHK(grow(w->tmp, w->tmp_cap, (size_t)R * C * sizeof(float)));
    J.P = (float*)w->pyr;
    J.T0 = (float*)w->tmp;
    for (int o = 0; o < J.n_oct; ++o) {
        const size_t plane = (size_t)J.orows[o] * J.ocols[o];
        for (int i = 0; i < kNOL + 3; ++i) J.h_pyr.gauss[o][i] = Layer{J.P + J.goff[o] + i * plane, J.orows[o], J.ocols[o]};
        for (int i = 0; i < kNOL + 2; ++i) J.h_pyr.dog[o][i] = Layer{J.P + J.doff[o] + i * plane, J.orows[o], J.ocols[o]};
    }
    const size_t mask_bytes = J.mask ? ((size_t)J.rows * J.cols + 255) / 256 * 256 : 0;
    const size_t aux_bytes = sizeof(Cand) * kCandCap + sizeof(mim_keypoint) * kKpCap + sizeof(Surv) * kCandCap +
                             sizeof(mim_keypoint) * kSortCap + mask_bytes;
    SCHK(grow(w->aux, w->aux_cap, aux_bytes));
    char* A = (char*)w->aux;
    J.d_cand = (Cand*)A;
    J.d_kp = (mim_keypoint*)(J.d_cand + kCandCap);
    J.d_surv = (Surv*)(J.d_kp + kKpCap);
    J.d_kp2 = (mim_keypoint*)(J.d_surv + kCandCap);
    J.d_mask = J.mask ? (uint8_t*)(J.d_kp2 + kSortCap) : nullptr;
    SCHK(grow(w->desc, w->desc_cap, sizeof(float) * 128 * (size_t)kSortCap));
    return 0;
}

// KeyPointsFilter::removeDuplicatedSorted, the octave -1 rescale, runByPixelsMask on the host, then the
// descriptors: only for an image with more than kSortCap keypoints (kp_post_kernel's limit).  The
// first min(n, cap) keypoints end in J.d_kp (and J.k), their descriptors in w->desc.
static int sift_describe_host(SiftJob& J, hipStream_t st, std::string& err) {
    if (J.h_cnt[1] > kKpCap) { err = "more than 2^19 SIFT keypoints"; return -4; }
    std::vector<mim_keypoint>& k = J.k;
    k.resize(J.h_cnt[1]);
    if (!k.empty()) SCHK(hipMemcpyAsync(k.data(), J.d_kp, sizeof(mim_keypoint) * k.size(), hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    std::sort(k.begin(), k.end(), kp_greater);
    size_t m = 0;
    for (size_t j = 0; j < k.size(); ++j) {
        if (m > 0 && k[m - 1].x == k[j].x && k[m - 1].y == k[j].y && k[m - 1].size == k[j].size && k[m - 1].angle == k[j].angle)
            continue;
        k[m++] = k[j];
    }
    k.resize(m);
    for (auto& p : k) {
        p.octave = (p.octave & ~255) | ((p.octave - 1) & 255);
        p.x *= 0.5f;
        p.y *= 0.5f;
        p.size *= 0.5f;
    }
    if (J.mask) {
        m = 0;
        for (size_t j = 0; j < k.size(); ++j) {
            const int yy = (int)(k[j].y + 0.5f), xx = (int)(k[j].x + 0.5f);
            if (J.mask[(size_t)yy * J.mstep + xx] != 0) k[m++] = k[j];
        }
        k.resize(m);
    }
    J.n = (int)k.size();
    J.out_kp = J.d_kp;
    const int n = std::min(J.n, J.cap);
    if (n <= 0) return 0;
    SCHK(hipMemcpyAsync(J.d_kp, k.data(), sizeof(mim_keypoint) * n, hipMemcpyHostToDevice, st));
    SCHK(grow(J.w->desc, J.w->desc_cap, sizeof(float) * 128 * (size_t)n));
    SCHK(hipMemcpyAsync(J.d_cnt + 3, &n, sizeof(int), hipMemcpyHostToDevice, st));
    DescB D{};
    D.pyr[0] = J.d_pyr;
    D.kp[0] = J.d_kp;
    D.n[0] = J.d_cnt + 3;
    D.n_cap[0] = n;
    D.desc[0] = (float*)J.w->desc;
    descr_kernel<kDescrT><<<dim3(4096, 1), kDescrT, 0, st>>>(D, -1);
    SCHK(hipGetLastError());
    SCHK(hipStreamSynchronize(st));  // `n` and `k` are host locals of this call
    return 0;
}

// Every stage of every image of `jobs` enqueued as one batched launch per stage, then ONE host
// synchronisation for the counts.  `bw` holds the batch buffer (the Pyr tables and counters of the
// images, one upload and one download).  Afterwards J.n / J.out_kp / J.w->desc hold each image's
// final keypoints and descriptors on the device (the host path already ran for an image past
// kp_post_kernel's limit).
static int sift_batch(std::vector<SiftJob>& jobs, SiftWs* bw, hipStream_t st, std::string& err) {
    const int nj = (int)jobs.size();
    if (nj > kMaxImg) {
        err = "sift: more than 8 images in one call";
        return -3;
    }
    for (auto& J : jobs)
        if (int r = sift_geometry(J, err)) return r;
    // taps (the same for every image): the initial blur, then layers 1 .. kNOL + 2
    Taps t0;
    const float sig_diff = sqrtf(std::max(1.6f * 1.6f - 0.5f * 0.5f * 4, 0.01f));
    if (gauss_taps(sig_diff, t0) < 0) { err = "kernel size"; return -4; }
    double sig[kNOL + 3];
    sig[0] = 1.6;
    const double kk = pow(2., 1. / kNOL);
    for (int i = 1; i < kNOL + 3; i++) {
        const double sp = pow(kk, (double)(i - 1)) * 1.6, stt = sp * kk;
        sig[i] = sqrt(stt * stt - sp * sp);
    }
    Taps tl[kNOL + 2];
    for (int i = 1; i < kNOL + 3; ++i)
        if (gauss_taps(sig[i], tl[i - 1]) < 0) { err = "kernel size"; return -4; }
    // batch buffer: Pyr tables, then 4 counters per image
    const size_t pyr_bytes = sizeof(Pyr) * nj;
    SCHK(grow(bw->batch, bw->batch_cap, pyr_bytes + 256));
    if (!bw->h_pyr) SCHK(hipHostMalloc((void**)&bw->h_pyr, sizeof(Pyr) * kMaxImg, hipHostMallocDefault));
    if (!bw->h_cnt) SCHK(hipHostMalloc((void**)&bw->h_cnt, sizeof(int) * 4 * kMaxImg, hipHostMallocDefault));
    Pyr* d_pyr = (Pyr*)bw->batch;
    int* d_cnt = (int*)((char*)bw->batch + pyr_bytes);
    std::vector<int> live;  // images with at least one octave
    for (int j = 0; j < nj; ++j) {
        SiftJob& J = jobs[j];
        J.d_pyr = d_pyr + j;
        J.d_cnt = d_cnt + 4 * j;
        bw->h_pyr[j] = J.h_pyr;
        if (J.n_oct > 0) live.push_back(j);
        if (J.d_mask)
            if (int r = stage_h2d(J.w, 1, J.d_mask, J.mask, J.mstep, J.cols, J.rows, st, err)) return r;
    }
    SCHK(hipMemcpyAsync(d_pyr, bw->h_pyr, pyr_bytes, hipMemcpyHostToDevice, st));
    SCHK(hipMemsetAsync(d_cnt, 0, sizeof(int) * 4 * nj, st));
    if (!live.empty()) {
        // createInitialImage: x2 INTER_LINEAR, then the initial blur into octave 0 layer 0
        {
            Up2B A{};
            const int nb = flatten(A.f, live, [&](int j, int& gx, int& gy) {
                gx = (jobs[j].cols * 2 + 255) / 256;
                gy = jobs[j].rows * 2;
            });
            for (int k = 0; k < A.f.n; ++k) {
                const SiftJob& J = jobs[live[k]];
                A.src[k] = (const uint8_t*)J.w->img;
                A.rows[k] = J.rows;
                A.cols[k] = J.cols;
                A.dst[k] = J.T0;
            }
            up2_kernel<<<nb, 256, 0, st>>>(A);
        }
        auto blur = [&](const std::vector<int>& imgs, int o, int layer, bool init, const Taps& t) -> bool {
            BlurB A{};
            const int nb = flatten(A.f, imgs, [&](int j, int& gx, int& gy) {
                gx = (jobs[j].ocols[o] + kBlurTW - 1) / kBlurTW;
                gy = (jobs[j].orows[o] + kBlurTH - 1) / kBlurTH;
            });
            for (int k = 0; k < A.f.n; ++k) {
                const SiftJob& J = jobs[imgs[k]];
                const size_t plane = (size_t)J.orows[o] * J.ocols[o];
                A.src[k] = init ? J.T0 : J.P + J.goff[o] + (layer - 1) * plane;
                A.dst[k] = J.P + J.goff[o] + layer * plane;
                A.dog[k] = init ? nullptr : J.P + J.doff[o] + (layer - 1) * plane;
                A.rows[k] = J.orows[o];
                A.cols[k] = J.ocols[o];
            }
            const int a = t.n / 2;
            auto reg = [&](auto kern, int th) {
                // the register-blocked kernel's tiles are th rows: its own grid
                const int nb2 = flatten(A.f, imgs, [&](int j, int& gx, int& gy) {
                    gx = (jobs[j].ocols[o] + kBlurTW - 1) / kBlurTW;
                    gy = (jobs[j].orows[o] + th - 1) / th;
                });
                kern<<<nb2, 256, 0, st>>>(A, t);
                return true;
            };
            switch (a) {
            case 5: return reg(blur_reg_kernel<5, MIM_BLUR_TH>, MIM_BLUR_TH);
            case 6: return reg(blur_reg_kernel<6, MIM_BLUR_TH>, MIM_BLUR_TH);
            case 8: return reg(blur_reg_kernel<8, MIM_BLUR_TH>, MIM_BLUR_TH);
            case 10: return reg(blur_reg_kernel<10, MIM_BLUR_TH_BIG>, MIM_BLUR_TH_BIG);
            case 13: return reg(blur_reg_kernel<13, MIM_BLUR_TH_BIG>, MIM_BLUR_TH_BIG);
            default: break;
            }
            const size_t lds = sizeof(float) * (size_t)(kBlurTH + 2 * a) * (kBlurTW + 2 * a + kBlurTW);
            if (lds > 64 * 1024) return false;
            blur_kernel<<<nb, 256, lds, st>>>(A, t);
            return true;
        };
        if (!blur(live, 0, 0, true, t0)) { err = "kernel size"; return -4; }
        // buildGaussianPyramid + DoG of the large octaves, all images with octave o at once (each blur
        // after the first writes the DoG plane of its source and destination layers too)
        int o_max = 0;
        for (int j : live) o_max = std::max(o_max, jobs[j].o_small);
        for (int o = 0; o < o_max; ++o) {
            std::vector<int> imgs;
            for (int j : live)
                if (o < jobs[j].o_small) imgs.push_back(j);
            if (o > 0) {
                DownB A{};
                const int nb = flatten(A.f, imgs, [&](int j, int& gx, int& gy) {
                    gx = (jobs[j].ocols[o] + 255) / 256;
                    gy = jobs[j].orows[o];
                });
                for (int k = 0; k < A.f.n; ++k) {
                    const SiftJob& J = jobs[imgs[k]];
                    A.src[k] = J.P + J.goff[o - 1] + kNOL * (size_t)J.orows[o - 1] * J.ocols[o - 1];
                    A.scols[k] = J.ocols[o - 1];
                    A.dst[k] = J.P + J.goff[o];
                    A.cols[k] = J.ocols[o];
                }
                down2_kernel<<<nb, 256, 0, st>>>(A);
            }
            for (int i = 1; i < kNOL + 3; ++i)
                if (!blur(imgs, o, i, false, tl[i - 1])) { err = "kernel size"; return -4; }
        }
        {  // the small octaves: one block per image
            SmallB A{};
            for (int j : live)
                if (jobs[j].o_small < jobs[j].n_oct) {
                    A.pyr[A.n] = jobs[j].d_pyr;
                    A.o0[A.n] = jobs[j].o_small;
                    A.n_oct[A.n] = jobs[j].n_oct;
                    ++A.n;
                }
            for (int i = 0; i < kNOL + 2; ++i) A.t[i] = tl[i];
            if (A.n > 0) small_octaves_kernel<<<A.n, 1024, 0, st>>>(A);
        }
        // findScaleSpaceExtrema's pixel test, per octave all images at once
        const int threshold = (int)floor(0.5 * 0.04 / kNOL * 255);
        int oct_max = 0;
        for (int j : live) oct_max = std::max(oct_max, jobs[j].n_oct);
        for (int o = 0; o < oct_max; ++o) {
            std::vector<int> imgs;
            for (int j : live)
                if (o < jobs[j].n_oct && jobs[j].orows[o] > 2 * kBorder && jobs[j].ocols[o] > 2 * kBorder) imgs.push_back(j);
            if (imgs.empty()) continue;
            ExtB A{};
            const int nb = flatten(A.f, imgs, [&](int j, int& gx, int& gy) {
                gx = (jobs[j].ocols[o] - 2 * kBorder + kExtTW - 1) / kExtTW;
                gy = (jobs[j].orows[o] - 2 * kBorder + kExtTH - 1) / kExtTH;
            });
            for (int k = 0; k < A.f.n; ++k) {
                const SiftJob& J = jobs[imgs[k]];
                A.dog[k] = J.P + J.doff[o];
                A.rows[k] = J.orows[o];
                A.cols[k] = J.ocols[o];
                A.cand[k] = J.d_cand;
                A.n_cand[k] = J.d_cnt;
            }
            A.octave = o;
            A.threshold = threshold;
            A.cap = cand_limit();
            extrema_kernel<<<dim3(nb, 1, kNOL), 256, 0, st>>>(A);
        }
        // adjustLocalExtrema, orientations, keypoint post-processing, descriptors: grids of (X, images)
        RefB Rf{};
        OriB Or{};
        KpB Kp{};
        DescB Ds{};
        const int nl = (int)live.size();
        for (int k = 0; k < nl; ++k) {
            SiftJob& J = jobs[live[k]];
            Rf.pyr[k] = J.d_pyr;
            Rf.cand[k] = J.d_cand;
            Rf.n_cand[k] = J.d_cnt;
            Rf.surv[k] = J.d_surv;
            Rf.n_surv[k] = J.d_cnt + 2;
            Or.pyr[k] = J.d_pyr;
            Or.surv[k] = J.d_surv;
            Or.n_surv[k] = J.d_cnt + 2;
            Or.kp[k] = J.d_kp;
            Or.n_kp[k] = J.d_cnt + 1;
            Kp.kp[k] = J.d_kp;
            Kp.n_kp[k] = J.d_cnt + 1;
            Kp.mask[k] = J.d_mask;
            Kp.mstep[k] = J.cols;
            Kp.out[k] = J.d_kp2;
            Kp.n_out[k] = J.d_cnt + 3;
            Ds.pyr[k] = J.d_pyr;
            Ds.kp[k] = J.d_kp2;
            Ds.n[k] = J.d_cnt + 3;
            Ds.n_cap[k] = kSortCap;
            Ds.desc[k] = (float*)J.w->desc;
        }
        Rf.cap = cand_limit();
        Rf.surv_cap = kCandCap;
        Or.surv_cap = kCandCap;
        Or.kp_cap = kKpCap;
        Kp.kp_cap = kKpCap;
        Kp.sort_cap = sort_limit();
        refine_kernel<<<dim3(std::max(1024 / nl, 128), nl), 128, 0, st>>>(Rf);
        orient_kernel<<<dim3(std::max(1024 / nl, 128), nl), 64 * kOriWaves, 0, st>>>(Or);
        kp_post_kernel<<<dim3(1, nl), 1024, 0, st>>>(Kp);
#if MIM_DESCR_SPLIT
        for (int k = 0; k < nl; ++k) {  // one launch per image, in order
            DescB D1{};
            D1.pyr[0] = Ds.pyr[k];
            D1.kp[0] = Ds.kp[k];
            D1.n[0] = Ds.n[k];
            D1.n_cap[0] = Ds.n_cap[k];
            D1.desc[0] = Ds.desc[k];
            descr_kernel<kDescrT><<<dim3(MIM_DESCR_GRID, 1), kDescrT, 0, st>>>(D1, -1);
        }
#else
#if MIM_DESCR_BIG_SPLIT  // measured slower (r06c: 1.42 + 0.76 ms against 0.99 ms for one launch per scene)
        descr_kernel<kDescrTBig><<<dim3(64, nl), kDescrTBig, 0, st>>>(Ds, 1);
        descr_kernel<kDescrT><<<dim3(std::max(MIM_DESCR_GRID / nl, 1024), nl), kDescrT, 0, st>>>(Ds, 0);
#else
        descr_kernel<kDescrT><<<dim3(std::max(MIM_DESCR_GRID / nl, 1024), nl), kDescrT, 0, st>>>(Ds, -1);
#endif
#endif
        SCHK(hipGetLastError());
    }
    SCHK(hipMemcpyAsync(bw->h_cnt, d_cnt, sizeof(int) * 4 * nj, hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    for (int j = 0; j < nj; ++j) {
        SiftJob& J = jobs[j];
        for (int q = 0; q < 4; ++q) J.h_cnt[q] = bw->h_cnt[4 * j + q];
        J.n = 0;
        J.out_kp = J.d_kp2;
        if (J.n_oct < 1) continue;
        // extrema_kernel counts every candidate but stores only the first cand_limit(): more would
        // silently drop keypoints OpenCV (no cap) keeps
        if (J.h_cnt[0] > cand_limit()) {
            err = "more than " + std::to_string(cand_limit()) + " SIFT candidates";
            return -4;
        }
        if (J.h_cnt[3] < 0) {
            if (int r = sift_describe_host(J, st, err)) return r;
        } else {
            J.n = J.h_cnt[3];
        }
    }
    return 0;
}

// copies of the first J.cap keypoints / descriptors of every image, one synchronisation
static int sift_fetch(std::vector<SiftJob>& jobs, hipStream_t st, std::string& err) {
    for (auto& J : jobs) {
        const int n = std::min(J.n, J.cap);
        if (n <= 0) continue;
        SCHK(hipMemcpyAsync(J.kps, J.out_kp, sizeof(mim_keypoint) * n, hipMemcpyDeviceToHost, st));
        SCHK(hipMemcpyAsync(J.desc, J.w->desc, sizeof(float) * 128 * (size_t)n, hipMemcpyDeviceToHost, st));
    }
    SCHK(hipStreamSynchronize(st));
    return 0;
}

int sift_detect_compute(SiftWs* w, hipStream_t st, const uint8_t* img, int rows, int cols, long long step,
                        const uint8_t* mask, long long mstep, int max_kp, mim_keypoint* kps, float* desc, int* n_out,
                        std::string& err) {
    *n_out = 0;
    // MIM_SIFT_TRACE=1: host times of the call's phases on stderr (diagnostic)
    static const bool trace = getenv("MIM_SIFT_TRACE") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t0 = now();
    SCHK(grow(w->img, w->img_cap, (size_t)rows * cols));
    if (int r = stage_h2d(w, 0, w->img, img, step, cols, rows, st, err)) return r;
    const auto t1 = now();
    std::vector<SiftJob> jobs(1);
    SiftJob& J = jobs[0];
    J.w = w;
    J.rows = rows;
    J.cols = cols;
    J.mask = mask;
    J.mstep = mstep;
    J.cap = max_kp;
    J.kps = kps;
    J.desc = desc;
    int r = sift_batch(jobs, w, st, err);
    const auto t2 = now();
    if (!r) r = sift_fetch(jobs, st, err);
    if (trace) {
        const auto t3 = now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[mim] sift %dx%d: image copy %.0f us, batch %.0f us, fetch %.0f us\n", rows, cols, us(t0, t1),
                us(t1, t2), us(t2, t3));
    }
    *n_out = J.n;
    return r;
}

// resize(scene, scaled, Size(), s, s, INTER_LINEAR) of every scale into its workspace, one launch
static int sift_scale_images(std::vector<SiftWs*>& ws, hipStream_t st, const uint8_t* img, int rows, int cols,
                             long long step, int n_scales, const float* scales, std::vector<SiftJob>& jobs,
                             std::string& err) {
    if (n_scales > kMaxImg) {
        err = "sift scales: more than 8 scales";
        return -3;
    }
    while ((int)ws.size() < n_scales + 1) ws.push_back(sift_ws_create());
    SiftWs* src = ws[n_scales];  // the scene itself, and the batch buffer
    SCHK(grow(src->img, src->img_cap, (size_t)rows * cols));
    if (int r = stage_h2d(src, 0, src->img, img, step, cols, rows, st, err)) return r;
    jobs.assign(n_scales, SiftJob{});
    ResizeB A{};
    A.src = (const uint8_t*)src->img;
    A.rows = rows;
    A.cols = cols;
    std::vector<int> all(n_scales);
    for (int i = 0; i < n_scales; ++i) {
        all[i] = i;
        const double f = (double)scales[i];
        const int dc = (int)lrint(cols * f), dr = (int)lrint(rows * f);  // Size() + fx: saturate_cast<int>
        if (dc <= 0 || dr <= 0) { err = "sift scales: a scale leaves no pixels"; return -3; }
        SiftJob& J = jobs[i];
        J.w = ws[i];
        J.rows = dr;
        J.cols = dc;
        J.mask = nullptr;
        J.mstep = 0;
        J.cap = 0;
        SCHK(grow(J.w->img, J.w->img_cap, (size_t)dr * dc));
        A.dst[i] = (uint8_t*)J.w->img;
        A.drows[i] = dr;
        A.dcols[i] = dc;
        A.sx[i] = A.sy[i] = 1. / f;
    }
    const int nb = flatten(A.f, all, [&](int i, int& gx, int& gy) {
        gx = (jobs[i].cols + 255) / 256;
        gy = jobs[i].rows;
    });
    resize_u8_kernel<<<nb, 256, 0, st>>>(A);
    SCHK(hipGetLastError());
    return 0;
}

// TestsDetector.cpp:99-107 for one scene: resize(scene, scaled, Size(), s, s, INTER_LINEAR) and
// detectAndCompute(scaled) at every scale, all in one call (the scene uploaded once, one launch per
// stage for all scales, 2 synchronisations in all).  Keypoints / descriptors of the scales are
// concatenated in scale order into kps / desc (capacity max_kp in all); n_out[s] = the keypoints of
// scale s.
int sift_detect_compute_scales(std::vector<SiftWs*>& ws, hipStream_t st, const uint8_t* img, int rows, int cols,
                               long long step, int n_scales, const float* scales, int max_kp, mim_keypoint* kps,
                               float* desc, int* n_out, std::string& err) {
    std::vector<SiftJob> jobs;
    if (int r = sift_scale_images(ws, st, img, rows, cols, step, n_scales, scales, jobs, err)) return r;
    for (auto& J : jobs) J.cap = INT_MAX;  // the host path describes every keypoint: copies come below
    if (int r = sift_batch(jobs, ws[n_scales], st, err)) return r;
    int used = 0;
    for (int i = 0; i < n_scales; ++i) {
        SiftJob& J = jobs[i];
        J.cap = std::max(0, max_kp - used);
        J.kps = kps + used;
        J.desc = desc + (size_t)128 * used;
        n_out[i] = J.n;
        used += std::min(J.n, J.cap);
    }
    if (int r = sift_fetch(jobs, st, err)) return r;
    int total = 0;
    for (int i = 0; i < n_scales; ++i) total += n_out[i];
    if (total > max_kp) {
        err = "sift scales: more keypoints than max_kp";
        return -2;
    }
    return 0;
}

// The same on the device only: out[i] = scale i's keypoints / descriptors in the workspaces (valid until
// the next SIFT call on them), one synchronisation (the counts)
int sift_scales_device(std::vector<SiftWs*>& ws, hipStream_t st, const uint8_t* img, int rows, int cols,
                       long long step, int n_scales, const float* scales, SiftDevOut* out, std::string& err) {
    std::vector<SiftJob> jobs;
    if (int r = sift_scale_images(ws, st, img, rows, cols, step, n_scales, scales, jobs, err)) return r;
    for (auto& J : jobs) J.cap = INT_MAX;
    if (int r = sift_batch(jobs, ws[n_scales], st, err)) return r;
    for (int i = 0; i < n_scales; ++i) out[i] = SiftDevOut{jobs[i].out_kp, (const float*)jobs[i].w->desc, jobs[i].n};
    return 0;
}

// The scales' rows and keypoint positions copied into their sets' storage in one launch (was two copies
// per scale, each a blit launch and ~30 us of host enqueue): thread e copies float4 e % 32 of row e / 32
// of the scale holding it, and the row's KeyPoint::pt with its first float4
struct SetCopyB {
    const float* desc[kMaxImg];
    const mim_keypoint* kp[kMaxImg];
    float* ddesc[kMaxImg];
    float2* dkp[kMaxImg];
    long long off[kMaxImg + 1];  // first float4 of each scale
    int m;
};

__global__ __launch_bounds__(256) void set_copy_kernel(SetCopyB A) {
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < A.off[A.m]; e += (long long)gridDim.x * 256) {
        int j = 0;
        while (j + 1 < A.m && A.off[j + 1] <= e) ++j;
        const long long v = e - A.off[j], row = v >> 5;
        reinterpret_cast<float4*>(A.ddesc[j])[v] = reinterpret_cast<const float4*>(A.desc[j])[v];
        if ((v & 31) == 0) A.dkp[j][row] = make_float2(A.kp[j][row].x, A.kp[j][row].y);
    }
}

int sift_copy_sets(const SiftDevOut* out, int n, float* const* ddesc, float2* const* dkp, hipStream_t st) {
    if (n <= 0 || n > kMaxImg) return n == 0 ? 0 : -3;
    SetCopyB A{};
    A.m = n;
    for (int j = 0; j < n; ++j) {
        A.desc[j] = out[j].desc;
        A.kp[j] = out[j].kp;
        A.ddesc[j] = ddesc[j];
        A.dkp[j] = dkp[j];
        A.off[j + 1] = A.off[j] + (long long)out[j].n * (kDim / 4);
    }
    if (A.off[n] == 0) return 0;
    const long long nb = std::min<long long>((A.off[n] + 255) / 256, 4096);
    set_copy_kernel<<<(int)nb, 256, 0, st>>>(A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sift_resize_u8(SiftWs* w, hipStream_t st, const uint8_t* src, int rows, int cols, long long step, uint8_t* dst,
                   int drows, int dcols, double fx, double fy, std::string& err) {
    const size_t sb = (size_t)rows * cols, db = (size_t)drows * dcols;
    SCHK(grow(w->img, w->img_cap, sb + db));
    uint8_t* ds = (uint8_t*)w->img;
    uint8_t* dd = ds + sb;
    if (int r = stage_h2d(w, 0, ds, src, step, cols, rows, st, err)) return r;
    ResizeB A{};
    A.src = ds;
    A.rows = rows;
    A.cols = cols;
    A.dst[0] = dd;
    A.drows[0] = drows;
    A.dcols[0] = dcols;
    A.sx[0] = 1. / (fx > 0 ? fx : (double)dcols / cols);
    A.sy[0] = 1. / (fy > 0 ? fy : (double)drows / rows);
    const int nb = flatten(A.f, std::vector<int>{0}, [&](int, int& gx, int& gy) {
        gx = (dcols + 255) / 256;
        gy = drows;
    });
    resize_u8_kernel<<<nb, 256, 0, st>>>(A);
    SCHK(hipGetLastError());
    SCHK(hipMemcpyAsync(dst, dd, db, hipMemcpyDeviceToHost, st));
    SCHK(hipStreamSynchronize(st));
    return 0;
}

}  // namespace mim
