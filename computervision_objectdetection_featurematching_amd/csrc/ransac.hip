// ransac.hip — cv::findHomography(obj, scene, RANSAC, 5.0, mask) on gfx950, batched over problems.
//
// Replaces /root/reference/src/TestsDetector.cpp:78 (+ the gates :74,:79-84) — OpenCV
// calib3d/src/fundam.cpp (findHomography, HomographyEstimatorCallback, HomographyRefineCallback),
// calib3d/src/ptsetreg.cpp (RANSACPointSetRegistrator::run/getSubset/findInliers,
// RANSACUpdateNumIters), calib3d/src/levmarq.cpp (LMSolverImpl), core/src/lapack.cpp (Jacobi).
//
// The sequential RANSAC loop is re-cut into data-parallel stages with identical results:
//   sample  one wave per problem replays cv::RNG((uint64)-1) + getSubset + checkSubset with 64
//           speculative subset attempts per round (attempt j assumed to start 4j draws ahead; the
//           first attempt with a repeated index is resolved serially and later lanes re-issued);
//   hypo    one lane per iteration: normalized DLT + OpenCV's Jacobi eigensolver in fp64, bit-exact
//           (matrix state lives in LDS, [element][lane] interleaved: conflict-free dynamic indexing);
//   score   one lane per iteration, points streamed through scalar loads: fp32 computeError,
//           no FMA contraction, IEEE division — the reference's float arithmetic bit for bit;
//   select  one wave per problem replays "goodCount > max(best,3)" + RANSACUpdateNumIters in
//           iteration order (ballot over 64 iterations at a time);
//   refine  one block per problem: best mask, inlier compaction, refit DLT and 10-iteration
//           Levenberg-Marquardt in fp64 (block reductions), determinant and gates.
// Chunks of iterations grow geometrically so adaptive termination (niters) stops the work early.
#include <float.h>

#include <algorithm>

#include "../../include/mim.h"
#include "mim_internal.h"

namespace mim {

// ------------------------------------------------------------------------------------------------
// shared fp64 helpers (core/src/lapack.cpp)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double d_hypot(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    if (a > b) {
        b /= a;
        return a * sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * sqrt(1 + a * a);
    }
    return 0;
}

// packed upper-triangle index of (i, j), i < j, for an n x n symmetric matrix
template <int n> __device__ __forceinline__ int pk(int i, int j) { return (i * (2 * n - i - 1)) / 2 + (j - i - 1); }

// JacobiImpl_<double> (core/src/lapack.cpp) on strided storage: element e of an array lives at
// base[e * S] (S = 64 in the per-lane hypothesis kernel, 1 for single-thread use).
//   A: packed strict upper triangle; W: diagonal on entry, eigenvalues (descending) on exit;
//   V: n x n, eigenvectors in rows; ind: indR[0..n) then indC[0..n).
template <int n, int S>
__device__ void jacobi_strided(double* __restrict__ A, double* __restrict__ W, double* __restrict__ V,
                               int* __restrict__ ind) {
#define AU(i, j) A[pk<n>((i), (j)) * S]
#define WW(k) W[(k) * S]
#define VV(r, c) V[((r) * n + (c)) * S]
#define IR(k) ind[(k) * S]
#define IC(k) ind[(n + (k)) * S]
    const double eps = DBL_EPSILON;
    int i, j, k, m;
    double mv;
    for (i = 0; i < n; i++)
        for (j = 0; j < n; j++) VV(i, j) = i == j ? 1.0 : 0.0;
    for (k = 0; k < n; k++) {
        if (k < n - 1) {
            for (m = k + 1, mv = fabs(AU(k, m)), i = k + 2; i < n; i++) {
                const double val = fabs(AU(k, i));
                if (mv < val) mv = val, m = i;
            }
            IR(k) = m;
        }
        if (k > 0) {
            for (m = 0, mv = fabs(AU(0, k)), i = 1; i < k; i++) {
                const double val = fabs(AU(i, k));
                if (mv < val) mv = val, m = i;
            }
            IC(k) = m;
        }
    }
    for (int iters = 0; iters < n * n * 30; iters++) {
        for (k = 0, mv = fabs(AU(0, IR(0))), i = 1; i < n - 1; i++) {
            const double val = fabs(AU(i, IR(i)));
            if (mv < val) mv = val, k = i;
        }
        int l = IR(k);
        for (i = 1; i < n; i++) {
            const int ci = IC(i);
            const double val = fabs(AU(ci, i));
            if (mv < val) mv = val, k = ci, l = i;
        }
        const double p = AU(k, l);
        if (fabs(p) <= eps) break;
        double y = (WW(l) - WW(k)) * 0.5;
        double t = fabs(y) + d_hypot(p, y);
        double s = d_hypot(p, t);
        const double c = t / s;
        s = p / s;
        t = (p / t) * p;
        if (y < 0) s = -s, t = -t;
        AU(k, l) = 0;
        WW(k) -= t;
        WW(l) += t;
        double a0, b0;
#define ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
        for (i = 0; i < k; i++) ROT(AU(i, k), AU(i, l));
        for (i = k + 1; i < l; i++) ROT(AU(k, i), AU(i, l));
        for (i = l + 1; i < n; i++) ROT(AU(k, i), AU(l, i));
        for (i = 0; i < n; i++) ROT(VV(k, i), VV(l, i));
#undef ROT
        for (j = 0; j < 2; j++) {
            const int idx = j == 0 ? k : l;
            if (idx < n - 1) {
                for (m = idx + 1, mv = fabs(AU(idx, m)), i = idx + 2; i < n; i++) {
                    const double val = fabs(AU(idx, i));
                    if (mv < val) mv = val, m = i;
                }
                IR(idx) = m;
            }
            if (idx > 0) {
                for (m = 0, mv = fabs(AU(0, idx)), i = 1; i < idx; i++) {
                    const double val = fabs(AU(i, idx));
                    if (mv < val) mv = val, m = i;
                }
                IC(idx) = m;
            }
        }
    }
    for (k = 0; k < n - 1; k++) {
        m = k;
        for (i = k + 1; i < n; i++)
            if (WW(m) < WW(i)) m = i;
        if (k != m) {
            double tmp = WW(m);
            WW(m) = WW(k);
            WW(k) = tmp;
            for (i = 0; i < n; i++) {
                tmp = VV(m, i);
                VV(m, i) = VV(k, i);
                VV(k, i) = tmp;
            }
        }
    }
#undef AU
#undef WW
#undef VV
#undef IR
#undef IC
}

// storage footprint of jacobi_strided<9>: 36 + 9 + 81 doubles, 18 ints
constexpr int kJ9D = 36 + 9 + 81;
constexpr int kJ9I = 18;
constexpr int kJ8D = 28 + 8 + 64;
constexpr int kJ8I = 16;

__device__ __forceinline__ void mat3_mul(const double* a, const double* b, double* c) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            c[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}

// Eigen-decompose LtL (upper incl. diagonal in lt[45], row-major (j,k>=j) order) and build H from
// the smallest eigenvector: HomographyEstimatorCallback::runKernel after completeSymm.
template <int S>
__device__ void dlt_finish(const double* lt, double* D, int* I, const double* invHnorm, const double* Hnorm2,
                           double* H) {
    double* A = D;
    double* W = D + 36 * S;
    double* V = D + 45 * S;
    int e = 0;
    for (int j = 0; j < 9; ++j)
        for (int k = j; k < 9; ++k, ++e) {
            if (k == j) W[j * S] = lt[e];
            else A[pk<9>(j, k) * S] = lt[e];
        }
    jacobi_strided<9, S>(A, W, V, I);
    double H0[9], Ht[9];
    for (int i = 0; i < 9; ++i) H0[i] = V[(8 * 9 + i) * S];
    mat3_mul(invHnorm, H0, Ht);
    mat3_mul(Ht, Hnorm2, H0);
    const double sc = 1. / H0[8];  // _H0.convertTo(_model, type, 1./H0(2,2))
    for (int i = 0; i < 9; ++i) H[i] = H0[i] * sc;
}

// runKernel on the 4 points of a minimal sample (M = object, m = scene), one lane.
template <int S>
__device__ int run_kernel4(const float* M, const float* m, double* D, int* I, double* H) {
    const int count = 4;
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
#pragma unroll
    for (int i = 0; i < count; i++) {
        cmx += m[2 * i]; cmy += m[2 * i + 1];
        cMx += M[2 * i]; cMy += M[2 * i + 1];
    }
    cmx /= count; cmy /= count; cMx /= count; cMy /= count;
#pragma unroll
    for (int i = 0; i < count; i++) {
        smx += fabs(m[2 * i] - cmx);
        smy += fabs(m[2 * i + 1] - cmy);
        sMx += fabs(M[2 * i] - cMx);
        sMy += fabs(M[2 * i + 1] - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return 0;
    smx = count / smx; smy = count / smy; sMx = count / sMx; sMy = count / sMy;
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double lt[45];
#pragma unroll
    for (int e = 0; e < 45; ++e) lt[e] = 0;
#pragma unroll
    for (int i = 0; i < count; i++) {
        const double x = (m[2 * i] - cmx) * smx, y = (m[2 * i + 1] - cmy) * smy;
        const double X = (M[2 * i] - cMx) * sMx, Y = (M[2 * i + 1] - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        int e = 0;
#pragma unroll
        for (int j = 0; j < 9; j++)
#pragma unroll
            for (int k = j; k < 9; k++, ++e) lt[e] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    dlt_finish<S>(lt, D, I, invHnorm, Hnorm2, H);
    return 1;
}

// ------------------------------------------------------------------------------------------------
// checkSubset (fundam.cpp haveCollinearPoints + the Marquez-Neila orientation test), fp64
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool collinear4(const float* xy) {
    const int i = 3;
#pragma unroll
    for (int j = 0; j < i; ++j) {
        const double dx1 = (double)(xy[2 * j] - xy[2 * i]);
        const double dy1 = (double)(xy[2 * j + 1] - xy[2 * i + 1]);
#pragma unroll
        for (int k = 0; k < j; ++k) {
            const double dx2 = (double)(xy[2 * k] - xy[2 * i]);
            const double dy2 = (double)(xy[2 * k + 1] - xy[2 * i + 1]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return true;
        }
    }
    return false;
}

__device__ __forceinline__ double det3xy(double x0, double y0, double x1, double y1, double x2, double y2) {
    // Matx_DetOp<double,3> of [x0 y0 1; x1 y1 1; x2 y2 1]
    return x0 * (y1 * 1. - y2 * 1.) - y0 * (x1 * 1. - x2 * 1.) + 1. * (x1 * y2 - x2 * y1);
}

__device__ __forceinline__ bool check_subset(const float* s, const float* d) {
    if (collinear4(s) || collinear4(d)) return false;
    const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    int negative = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a = tt[i][0], b = tt[i][1], c = tt[i][2];
        const double dA = det3xy(s[2 * a], s[2 * a + 1], s[2 * b], s[2 * b + 1], s[2 * c], s[2 * c + 1]);
        const double dB = det3xy(d[2 * a], d[2 * a + 1], d[2 * b], d[2 * b + 1], d[2 * c], d[2 * c + 1]);
        negative += dA * dB < 0;
    }
    return !(negative != 0 && negative != 4);
}

// ------------------------------------------------------------------------------------------------
// RANSACUpdateNumIters (ptsetreg.cpp)
// ------------------------------------------------------------------------------------------------
__device__ int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p;
    if (num < DBL_MIN) num = DBL_MIN;
    double denom = 1. - pow(1. - ep, (double)model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    if (denom >= 0 || -num >= max_iters * (-denom)) return max_iters;
    return (int)rint(num / denom);  // cvRound
}

// ------------------------------------------------------------------------------------------------
// init: per-problem RANSAC state from the ratio-test survivors
// ------------------------------------------------------------------------------------------------
__global__ void ransac_init_kernel(RansacState* __restrict__ st, const int* __restrict__ n_good, int n_probs,
                                   int max_iters, int min_good) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_probs) return;
    RansacState S{};
    S.n = n_good[p];
    S.active = (S.n >= min_good && S.n > 4) ? 1 : 0;  // n == 4: direct runKernel, no RANSAC
    S.niters = max(max_iters, 1);
    S.fail_iter = -1;
    S.best_iter = -1;
    st[p] = S;
}

// ------------------------------------------------------------------------------------------------
// sample: getSubset replay, one wave per problem
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ransac_sample_kernel(RansacState* __restrict__ st,
                                                           const ProbDev* __restrict__ probs,
                                                           const float4* __restrict__ pts,
                                                           const uint32_t* __restrict__ stream, long long slen,
                                                           int4* __restrict__ samples, int c1,
                                                           int* __restrict__ err) {
    const int p = blockIdx.x, lane = threadIdx.x;
    RansacState S = st[p];
    if (!S.active || S.done || S.fail_iter != -1) return;
    const int target = min(c1, S.niters);
    if (S.produced >= target) return;
    const unsigned N = (unsigned)S.n;
    const float4* P = pts + probs[p].good_off;
    int4* out = samples + probs[p].it_off;
    long long pos = S.stream_pos;
    int produced = S.produced, fail_run = S.fail_run;
    bool stopped = false;
    while (produced < target && !stopped) {
        const long long p0 = pos + 4LL * lane;
        int i0 = 0, i1 = 0, i2 = 0, i3 = 0;
        bool coll = true;
        if (p0 + 4 <= slen) {
            i0 = (int)(stream[p0] % N);
            i1 = (int)(stream[p0 + 1] % N);
            i2 = (int)(stream[p0 + 2] % N);
            i3 = (int)(stream[p0 + 3] % N);
            coll = i1 == i0 || i2 == i0 || i2 == i1 || i3 == i0 || i3 == i1 || i3 == i2;
        }
        const unsigned long long cm = __ballot(coll);
        const int fc = cm ? __ffsll((long long)cm) - 1 : 64;  // first attempt with a repeated draw
        long long end = p0 + 4;
        bool oob = false;
        if (lane == fc) {  // resolve serially: redraw while the index repeats (getSubset inner loop)
            long long q = p0;
            int idx[4];
            for (int i = 0; i < 4 && !oob; ++i) {
                for (;;) {
                    if (q >= slen) { oob = true; break; }
                    const int v = (int)(stream[q++] % N);
                    bool dup = false;
                    for (int j = 0; j < i; ++j) dup |= idx[j] == v;
                    if (!dup) { idx[i] = v; break; }
                }
            }
            i0 = idx[0]; i1 = idx[1]; i2 = idx[2]; i3 = idx[3];
            end = q;
        }
        if (__any(oob)) {  // RNG stream exhausted: report, never guess
            if (lane == 0) atomicOr(err, 1);
            S.fail_iter = -2;
            stopped = true;
            break;
        }
        const bool valid = lane <= fc;
        bool pass = false;
        if (valid) {
            const float4 a = P[i0], b = P[i1], c = P[i2], d = P[i3];
            const float s[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
            const float t[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
            pass = check_subset(s, t);
        }
        const unsigned long long pm = __ballot(pass);
        const int last_valid = fc < 64 ? fc : 63;
        const unsigned long long vmask = last_valid == 63 ? ~0ull : ((1ull << (last_valid + 1)) - 1);
        // lane at which the target-th sample is produced
        const int need = target - produced;
        const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        const int rank = __popcll(pm & below);  // passes before this lane
        const bool is_target = pass && rank == need - 1;
        const unsigned long long tm = __ballot(is_target);
        // consecutive failures reaching getSubset's maxAttempts = 10000
        const unsigned long long pb = pm & below;
        const int run = pb ? (lane - (63 - __clzll((long long)pb))) : (fail_run + lane + 1);
        const bool is_fail = valid && !pass && run >= 10000;
        const unsigned long long fm = __ballot(is_fail);
        int stop_lane = last_valid;
        bool hit_target = false, hit_fail = false;
        const int tl = tm ? __ffsll((long long)tm) - 1 : 64;
        const int fl = fm ? __ffsll((long long)fm) - 1 : 64;
        if (tl < 64 && tl <= fl) { stop_lane = tl; hit_target = true; }
        else if (fl < 64) { stop_lane = fl; hit_fail = true; }
        // emit samples of passing lanes up to the stop lane
        if (pass && lane <= stop_lane) out[produced + rank] = make_int4(i0, i1, i2, i3);
        const unsigned long long upto = stop_lane == 63 ? ~0ull : ((1ull << (stop_lane + 1)) - 1);
        const unsigned long long pu = pm & upto & vmask;
        produced += __popcll(pu);
        if (pu) fail_run = stop_lane - (63 - __clzll((long long)pu));
        else fail_run += stop_lane + 1;
        pos = __shfl(end, stop_lane);
        if (hit_fail) {
            S.fail_iter = produced;  // getSubset returned false in this iteration
            stopped = true;
        }
        if (hit_target) break;
    }
    if (lane == 0) {
        S.stream_pos = pos;
        S.produced = produced;
        S.fail_run = fail_run;
        st[p] = S;
    }
}

// ------------------------------------------------------------------------------------------------
// hypo: runKernel on each minimal sample, one lane per iteration (bit-exact fp64)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ransac_hypo_kernel(const RansacState* __restrict__ st,
                                                         const ProbDev* __restrict__ probs,
                                                         const float4* __restrict__ pts,
                                                         const int4* __restrict__ samples,
                                                         float* __restrict__ hyp, int* __restrict__ counts, int c0,
                                                         int c1, int bpp) {
    __shared__ double sd[kJ9D * 64];
    __shared__ int si[kJ9I * 64];
    const int p = blockIdx.x / bpp, lane = threadIdx.x;
    const int it = c0 + (blockIdx.x % bpp) * 64 + lane;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    if (it >= c1 || it >= S.produced) return;
    const long long o = probs[p].it_off + it;
    const float4* P = pts + probs[p].good_off;
    const int4 s4 = samples[o];
    const float4 a = P[s4.x], b = P[s4.y], c = P[s4.z], d = P[s4.w];
    const float M[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
    const float m[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
    double H[9];
    const int ok = run_kernel4<64>(M, m, sd + lane, si + lane, H);
    counts[o] = ok ? 0 : -1;
    if (ok) {
        float4* h = reinterpret_cast<float4*>(hyp + o * 8);
        h[0] = make_float4((float)H[0], (float)H[1], (float)H[2], (float)H[3]);
        h[1] = make_float4((float)H[4], (float)H[5], (float)H[6], (float)H[7]);
    }
}

// ------------------------------------------------------------------------------------------------
// score: findInliers, one lane per hypothesis, points uniform across the wave (scalar loads)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float reproj_err(const float* Hf, float x, float y, float u, float v) {
    // HomographyEstimatorCallback::computeError (fp32; no contraction: -ffp-contract=off)
    const float ww = 1.f / (Hf[6] * x + Hf[7] * y + 1.f);
    const float dx = (Hf[0] * x + Hf[1] * y + Hf[2]) * ww - u;
    const float dy = (Hf[3] * x + Hf[4] * y + Hf[5]) * ww - v;
    return dx * dx + dy * dy;
}

__global__ __launch_bounds__(256) void ransac_score_kernel(const RansacState* __restrict__ st,
                                                           const ProbDev* __restrict__ probs,
                                                           const float4* __restrict__ pts,
                                                           const float* __restrict__ hyp,
                                                           int* __restrict__ counts, int c0, int c1, int bpp,
                                                           float thr2) {
    const int p = blockIdx.x / bpp;
    const int it = c0 + (blockIdx.x % bpp) * 256 + threadIdx.x;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    const long long o = probs[p].it_off + it;
    bool act = it < c1 && it < S.produced;
    if (act) act = counts[o] == 0;
    if (!act) return;
    float Hf[8];
    const float4* h = reinterpret_cast<const float4*>(hyp + o * 8);
    const float4 h0 = h[0], h1 = h[1];
    Hf[0] = h0.x; Hf[1] = h0.y; Hf[2] = h0.z; Hf[3] = h0.w;
    Hf[4] = h1.x; Hf[5] = h1.y; Hf[6] = h1.z; Hf[7] = h1.w;
    const float4* __restrict__ P = pts + probs[p].good_off;
    const int n = S.n;
    int cnt = 0;
#pragma unroll 4
    for (int i = 0; i < n; ++i) {
        const float4 q = P[i];
        cnt += reproj_err(Hf, q.x, q.y, q.z, q.w) <= thr2;
    }
    counts[o] = cnt;
}

// ------------------------------------------------------------------------------------------------
// select: replay best-model updates and adaptive termination in iteration order
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ransac_select_kernel(RansacState* __restrict__ st,
                                                           const ProbDev* __restrict__ probs,
                                                           const int* __restrict__ counts, int c1, double conf) {
    const int p = blockIdx.x, lane = threadIdx.x;
    RansacState S = st[p];
    if (!S.active || S.done) return;
    const int* C = counts + probs[p].it_off;
    int end = min(c1, S.produced);
    const int N = S.n;
    for (int base = S.next_iter; base < end && base < S.niters; base += 64) {
        const int t = base + lane;
        const int c = t < end ? C[t] : -1;
        for (;;) {
            const int thr = max(S.max_good, 3);  // goodCount > MAX(maxGoodCount, modelPoints-1)
            const unsigned long long m = __ballot(t < end && t < S.niters && c > thr);
            if (!m) break;
            const int f = __ffsll((long long)m) - 1;
            const int cf = __shfl(c, f);
            S.max_good = cf;
            S.best_iter = base + f;
            S.niters = update_num_iters(conf, (double)(N - cf) / N, 4, S.niters);
        }
    }
    S.next_iter = end;
    const bool failed = S.fail_iter != -1 && S.produced <= end;  // getSubset failure reached
    if (S.niters <= end || failed) {
        S.done = 1;
    }
    if (lane == 0) st[p] = S;
}

// ------------------------------------------------------------------------------------------------
// refine: best mask, refit DLT + LM on the inliers, gates (TestsDetector.cpp:74-84)
// ------------------------------------------------------------------------------------------------
constexpr int kRT = 256;  // refine block

// deterministic block sum of K doubles (wave shuffles, then the 4 wave partials in order)
template <int K>
__device__ void block_sum(double (&v)[K], double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double x = v[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
        v[k] = x;
    }
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[wave * K + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = ((red[k] + red[K + k]) + red[2 * K + k]) + red[3 * K + k];
    __syncthreads();
}

__device__ double block_max(double x, double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x = fmax(x, __shfl_xor(x, off));
    __syncthreads();
    if (lane == 0) red[wave] = x;
    __syncthreads();
    x = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    return x;
}

// HomographyRefineCallback::compute for one point: residuals and (optionally) the Jacobian rows
__device__ __forceinline__ void refine_point(const double* h, double Mx, double My, double mx, double my,
                                             double& ex, double& ey, double* Jx, double* Jy) {
    double ww = h[6] * Mx + h[7] * My + 1.;
    ww = fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
    const double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
    const double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
    ex = xi - mx;
    ey = yi - my;
    if (Jx) {
        Jx[0] = Mx * ww; Jx[1] = My * ww; Jx[2] = ww; Jx[3] = Jx[4] = Jx[5] = 0.;
        Jx[6] = -Mx * ww * xi; Jx[7] = -My * ww * xi;
        Jy[0] = Jy[1] = Jy[2] = 0.; Jy[3] = Mx * ww; Jy[4] = My * ww; Jy[5] = ww;
        Jy[6] = -Mx * ww * yi; Jy[7] = -My * ww * yi;
    }
}

// A = J^T J (upper, 36), v = J^T r (8), S = |r|^2, rinf = |r|_inf over the inliers
__device__ void lm_normal(const float4* __restrict__ X, int n, const double* h, double* red, double* A, double* v,
                          double& S, double& rinf) {
    double acc[45];
#pragma unroll
    for (int k = 0; k < 45; ++k) acc[k] = 0;
    double mx = 0;
    for (int i = threadIdx.x; i < n; i += kRT) {
        const float4 q = X[i];
        double ex, ey, Jx[8], Jy[8];
        refine_point(h, q.x, q.y, q.z, q.w, ex, ey, Jx, Jy);
        int e = 0;
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int b = a; b < 8; ++b, ++e) acc[e] += Jx[a] * Jx[b] + Jy[a] * Jy[b];
#pragma unroll
        for (int a = 0; a < 8; ++a) acc[36 + a] += Jx[a] * ex + Jy[a] * ey;
        acc[44] += ex * ex + ey * ey;
        mx = fmax(mx, fmax(fabs(ex), fabs(ey)));
    }
    block_sum<45>(acc, red);
    rinf = block_max(mx, red);
    int e = 0;
    for (int a = 0; a < 8; ++a)
        for (int b = a; b < 8; ++b, ++e) A[a * 8 + b] = A[b * 8 + a] = acc[e];
    for (int a = 0; a < 8; ++a) v[a] = acc[36 + a];
    S = acc[44];
}

__device__ double lm_cost(const float4* __restrict__ X, int n, const double* h, double* red) {
    double acc[1] = {0};
    for (int i = threadIdx.x; i < n; i += kRT) {
        const float4 q = X[i];
        double ex, ey;
        refine_point(h, q.x, q.y, q.z, q.w, ex, ey, nullptr, nullptr);
        acc[0] += ex * ex + ey * ey;
    }
    block_sum<1>(acc, red);
    return acc[0];
}

// Jacobi of an 8x8 symmetric matrix (single thread, stride-1 scratch)
__device__ void eig8(const double* Ain, double* J, int* JI, double* w, double* V) {
    double* A = J;
    double* W = J + 28;
    double* VV = J + 36;
    for (int i = 0; i < 8; ++i) {
        W[i] = Ain[9 * i];
        for (int j = i + 1; j < 8; ++j) A[pk<8>(i, j)] = Ain[8 * i + j];
    }
    jacobi_strided<8, 1>(A, W, VV, JI);
    for (int i = 0; i < 8; ++i) w[i] = W[i];
    for (int i = 0; i < 64; ++i) V[i] = VV[i];
}

// solve(Ap, v, d, DECOMP_EIG) = Jacobi + SVBkSb(eps = 2 DBL_EPSILON)
__device__ void solve_eig8(const double* Ap, const double* b, double* x, double* J, int* JI) {
    double w[8], V[64];
    eig8(Ap, J, JI, w, V);
    double threshold = 0;
    for (int i = 0; i < 8; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int j = 0; j < 8; j++) x[j] = 0;
    for (int i = 0; i < 8; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < 8; j++) s += V[8 * i + j] * b[j];
        s *= wi;
        for (int j = 0; j < 8; j++) x[j] = x[j] + s * V[8 * i + j];
    }
}

__device__ double inv_diag_max8(const double* A, double* J, int* JI) {
    double w[8], V[64];
    eig8(A, J, JI, w, V);
    double threshold = 0;
    for (int i = 0; i < 8; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    double maxval = DBL_EPSILON;
    for (int c = 0; c < 8; ++c) {
        double diag = 0;
        for (int i = 0; i < 8; i++) {
            if (fabs(w[i]) <= threshold) continue;
            diag += V[8 * i + c] * V[8 * i + c] / w[i];
        }
        maxval = fmax(maxval, fabs(diag));
    }
    return maxval;
}

struct RefineShared {
    double red[4 * 45];
    double lt[45];
    double norm[8];       // cm, cM, sm, sM (x,y each)
    double H[9], Hb[9];
    double A[64], v[8], D[8], x[8], xd[8], d[8];
    double S, Sd, rinf, dinf, lambda, lc;
    double J9[kJ9D];
    int J9I[kJ9I];
    int flag, n_inl, proceed, accept;
    int wcnt[4];
};

__global__ __launch_bounds__(kRT) void ransac_refine_kernel(const RansacState* __restrict__ st,
                                                            const ProbDev* __restrict__ probs,
                                                            const float4* __restrict__ pts,
                                                            const int* __restrict__ n_good_arr,
                                                            const int4* __restrict__ samples,
                                                            float4* __restrict__ inl, uint8_t* __restrict__ masks,
                                                            mim_result* __restrict__ results, RansacParams prm,
                                                            int raw) {
    __shared__ RefineShared sh;
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const RansacState S = st[p];
    const int ng = n_good_arr[p];
    const long long go = probs[p].good_off;
    const float4* P = pts + go;
    uint8_t* mask = masks + go;
    float4* X = inl + go;
    mim_result res{};
    res.n_good = ng;
    // ---- gate :74 ----
    if (ng < prm.min_good || ng < 4) {
        res.status = MIM_FEW_GOOD;
        if (tid == 0) results[p] = res;
        return;
    }
    int ok = 0;
    if (!S.active) {  // n == 4: findHomography calls runKernel directly, mask = ones, no refine
        if (tid == 0) {
            float M[8], m[8];
            for (int i = 0; i < 4; ++i) {
                const float4 q = P[i];
                M[2 * i] = q.x; M[2 * i + 1] = q.y; m[2 * i] = q.z; m[2 * i + 1] = q.w;
            }
            sh.flag = run_kernel4<1>(M, m, sh.J9, sh.J9I, sh.H);
        }
        __syncthreads();
        ok = sh.flag;
        if (tid < 4) mask[tid] = ok ? 1 : 0;
        sh.n_inl = ok ? 4 : 0;
        res.iters = 0;
    } else {
        ok = S.max_good > 0 && S.fail_iter != -2;
        res.iters = (S.fail_iter >= 0 && S.fail_iter < S.niters) ? S.fail_iter : S.niters;
        if (ok) {
            // bestModel = runKernel(sample[best_iter]) (bit-identical to the hypo kernel's)
            if (tid == 0) {
                const int4 s4 = samples[probs[p].it_off + S.best_iter];
                const float4 a = P[s4.x], b = P[s4.y], c = P[s4.z], d = P[s4.w];
                const float M[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
                const float m[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
                run_kernel4<1>(M, m, sh.J9, sh.J9I, sh.Hb);
            }
            __syncthreads();
            float Hf[8];
            for (int i = 0; i < 8; ++i) Hf[i] = (float)sh.Hb[i];
            const float thr2 = (float)(prm.thresh * prm.thresh);
            // best mask + ordered compaction of the inliers (compressElems)
            int base = 0;
            for (int b0 = 0; b0 < ng; b0 += kRT) {
                const int i = b0 + tid;
                bool in = false;
                float4 q = make_float4(0, 0, 0, 0);
                if (i < ng) {
                    q = P[i];
                    in = reproj_err(Hf, q.x, q.y, q.z, q.w) <= thr2;
                    mask[i] = in ? 1 : 0;
                }
                const unsigned long long bal = __ballot(in);
                const int within = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
                if (lane == 0) sh.wcnt[wave] = __popcll(bal);
                __syncthreads();
                int wb = 0;
                for (int w = 0; w < wave; ++w) wb += sh.wcnt[w];
                const int tot = sh.wcnt[0] + sh.wcnt[1] + sh.wcnt[2] + sh.wcnt[3];
                if (in) X[base + wb + within] = q;
                base += tot;
                __syncthreads();
            }
            if (tid == 0) sh.n_inl = base;
            __syncthreads();
            const int k = sh.n_inl;
            if (k > 0) {
                // ---- refit: runKernel over all inliers (parallel sums; contract is |dH| <= 1e-4) ----
                double c4[4] = {0, 0, 0, 0};
                for (int i = tid; i < k; i += kRT) {
                    const float4 q = X[i];
                    c4[0] += q.z; c4[1] += q.w; c4[2] += q.x; c4[3] += q.y;  // cm (scene), cM (object)
                }
                block_sum<4>(c4, sh.red);
                const double cmx = c4[0] / k, cmy = c4[1] / k, cMx = c4[2] / k, cMy = c4[3] / k;
                double s4[4] = {0, 0, 0, 0};
                for (int i = tid; i < k; i += kRT) {
                    const float4 q = X[i];
                    s4[0] += fabs(q.z - cmx); s4[1] += fabs(q.w - cmy);
                    s4[2] += fabs(q.x - cMx); s4[3] += fabs(q.y - cMy);
                }
                block_sum<4>(s4, sh.red);
                const bool degenerate = fabs(s4[0]) < DBL_EPSILON || fabs(s4[1]) < DBL_EPSILON ||
                                        fabs(s4[2]) < DBL_EPSILON || fabs(s4[3]) < DBL_EPSILON;
                if (!degenerate) {
                    const double smx = k / s4[0], smy = k / s4[1], sMx = k / s4[2], sMy = k / s4[3];
                    double lt[45];
                    for (int e = 0; e < 45; ++e) lt[e] = 0;
                    for (int i = tid; i < k; i += kRT) {
                        const float4 q = X[i];
                        const double x = (q.z - cmx) * smx, y = (q.w - cmy) * smy;
                        const double Xx = (q.x - cMx) * sMx, Yy = (q.y - cMy) * sMy;
                        const double Lx[9] = {Xx, Yy, 1, 0, 0, 0, -x * Xx, -x * Yy, -x};
                        const double Ly[9] = {0, 0, 0, Xx, Yy, 1, -y * Xx, -y * Yy, -y};
                        int e = 0;
#pragma unroll
                        for (int j = 0; j < 9; j++)
#pragma unroll
                            for (int kk = j; kk < 9; kk++, ++e) lt[e] += Lx[j] * Lx[kk] + Ly[j] * Ly[kk];
                    }
                    block_sum<45>(lt, sh.red);
                    if (tid == 0) {
                        const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
                        const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
                        dlt_finish<1>(lt, sh.J9, sh.J9I, invHnorm, Hnorm2, sh.H);
                    }
                } else if (tid == 0) {
                    for (int i = 0; i < 9; ++i) sh.H[i] = sh.Hb[i];  // runKernel returned 0: H kept
                }
                __syncthreads();
                // ---- LMSolverImpl (levmarq.cpp) on H8 = H[0..7], maxIters 10, eps FLT_EPSILON ----
                if (tid < 8) sh.x[tid] = sh.H[tid];
                __syncthreads();
                double x[8];
                for (int i = 0; i < 8; ++i) x[i] = sh.x[i];
                double A[64], v[8], Sv, rinf;
                lm_normal(X, k, x, sh.red, A, v, Sv, rinf);
                if (tid == 0) {
                    for (int i = 0; i < 64; ++i) sh.A[i] = A[i];
                    for (int i = 0; i < 8; ++i) { sh.v[i] = v[i]; sh.D[i] = A[9 * i]; }
                    sh.S = Sv; sh.rinf = rinf; sh.lambda = 1; sh.lc = 0.75;
                }
                __syncthreads();
                int iter = 0;
                for (;;) {
                    if (tid == 0) {
                        double Ap[64];
                        for (int i = 0; i < 64; ++i) Ap[i] = sh.A[i];
                        for (int i = 0; i < 8; ++i) Ap[9 * i] += sh.lambda * sh.D[i];
                        solve_eig8(Ap, sh.v, sh.d, sh.J9, sh.J9I);
                        double dinf = 0;
                        for (int i = 0; i < 8; ++i) {
                            sh.xd[i] = sh.x[i] - sh.d[i];
                            dinf = fmax(dinf, fabs(sh.d[i]));
                        }
                        sh.dinf = dinf;
                    }
                    __syncthreads();
                    double xd[8];
                    for (int i = 0; i < 8; ++i) xd[i] = sh.xd[i];
                    const double Sd = lm_cost(X, k, xd, sh.red);
                    if (tid == 0) {
                        const double Rlo = 0.25, Rhi = 0.75;
                        double temp_d[8];
                        for (int i = 0; i < 8; ++i) {
                            double s = 0;
                            for (int j = 0; j < 8; ++j) s += sh.A[8 * i + j] * sh.d[j];
                            temp_d[i] = -s + 2 * sh.v[i];
                        }
                        double dS = 0;
                        for (int i = 0; i < 8; ++i) dS += sh.d[i] * temp_d[i];
                        const double R = (sh.S - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1);
                        if (R > Rhi) {
                            sh.lambda *= 0.5;
                            if (sh.lambda < sh.lc) sh.lambda = 0;
                        } else if (R < Rlo) {
                            double t = 0;
                            for (int i = 0; i < 8; ++i) t += sh.d[i] * sh.v[i];
                            double nu = (Sd - sh.S) / (fabs(t) > DBL_EPSILON ? t : 1) + 2;
                            nu = fmin(fmax(nu, 2.), 10.);
                            if (sh.lambda == 0) {
                                const double maxval = inv_diag_max8(sh.A, sh.J9, sh.J9I);
                                sh.lambda = sh.lc = 1. / maxval;
                                nu *= 0.5;
                            }
                            sh.lambda *= nu;
                        }
                        sh.accept = Sd < sh.S;
                        if (sh.accept) {
                            sh.S = Sd;
                            for (int i = 0; i < 8; ++i) sh.x[i] = sh.xd[i];
                        }
                    }
                    __syncthreads();
                    if (sh.accept) {
                        for (int i = 0; i < 8; ++i) x[i] = sh.x[i];
                        double S2;
                        lm_normal(X, k, x, sh.red, A, v, S2, rinf);
                        if (tid == 0) {
                            for (int i = 0; i < 64; ++i) sh.A[i] = A[i];
                            for (int i = 0; i < 8; ++i) sh.v[i] = v[i];
                            sh.rinf = rinf;
                        }
                    }
                    ++iter;
                    if (tid == 0) sh.proceed = iter < 10 && sh.dinf >= FLT_EPSILON && sh.rinf >= FLT_EPSILON;
                    __syncthreads();
                    const bool proceed = sh.proceed;
                    __syncthreads();
                    if (!proceed) break;
                }
                if (tid < 8) sh.H[tid] = sh.x[tid];
                __syncthreads();
            } else if (tid == 0) {
                for (int i = 0; i < 9; ++i) sh.H[i] = sh.Hb[i];
            }
            __syncthreads();
        } else {
            for (int i = tid; i < ng; i += kRT) mask[i] = 0;
            if (tid == 0) sh.n_inl = 0;
        }
    }
    __syncthreads();
    if (tid != 0) return;
    res.n_inl = ok ? sh.n_inl : 0;
    if (!ok) {
        res.status = MIM_EMPTY_H;
    } else {
        for (int i = 0; i < 9; ++i) res.H[i] = sh.H[i];
        const double* H = sh.H;
        double t = H[0] * (H[4] * H[8] - H[5] * H[7]);  // cv::determinant (3x3 CV_64F)
        t -= H[1] * (H[3] * H[8] - H[5] * H[6]);
        t += H[2] * (H[3] * H[7] - H[4] * H[6]);
        res.det = t;
        if (raw) res.status = MIM_ACCEPTED;
        else if (res.n_inl < prm.min_inliers) res.status = MIM_FEW_INLIERS;
        else {
            const double ad = fabs(t);
            res.status = (ad < prm.det_lo || ad > prm.det_hi) ? MIM_BAD_DET : MIM_ACCEPTED;
        }
    }
    results[p] = res;
}

// ------------------------------------------------------------------------------------------------
// host orchestration (called by api.cpp with the ctx mutex held)
// ------------------------------------------------------------------------------------------------
void ransac_enqueue(const RansacParams& prm, int n_probs, const ProbDev* probs, const float4* pts,
                    const int* n_good, const RansacBufs& b, uint8_t* masks, mim_result* results, int raw,
                    hipStream_t s, void (*mark)(void*, const char*), void* mark_ctx) {
    if (n_probs <= 0) return;
    ransac_init_kernel<<<(n_probs + 255) / 256, 256, 0, s>>>(b.state, n_good, n_probs, prm.max_iters, prm.min_good);
    const int max_iters = prm.max_iters > 1 ? prm.max_iters : 1;
    int c0 = 0, chunk = 512;
    const float thr2 = (float)(prm.thresh * prm.thresh);
    while (c0 < max_iters) {
        const int c1 = (int)std::min<long long>((long long)c0 + chunk, max_iters);
        ransac_sample_kernel<<<n_probs, 64, 0, s>>>(b.state, probs, pts, b.stream, b.stream_len, b.samples, c1, b.err);
        mark(mark_ctx, "sample");
        const int bpp64 = (c1 - c0 + 63) / 64;
        ransac_hypo_kernel<<<n_probs * bpp64, 64, 0, s>>>(b.state, probs, pts, b.samples, b.hyp, b.counts, c0, c1,
                                                         bpp64);
        mark(mark_ctx, "hypo");
        const int bpp256 = (c1 - c0 + 255) / 256;
        ransac_score_kernel<<<n_probs * bpp256, 256, 0, s>>>(b.state, probs, pts, b.hyp, b.counts, c0, c1, bpp256,
                                                            thr2);
        mark(mark_ctx, "score");
        ransac_select_kernel<<<n_probs, 64, 0, s>>>(b.state, probs, b.counts, c1, prm.conf);
        mark(mark_ctx, "select");
        c0 = c1;
        chunk = chunk < (1 << 16) ? chunk * 4 : chunk;
    }
    ransac_refine_kernel<<<n_probs, kRT, 0, s>>>(b.state, probs, pts, n_good, b.samples, b.inl, masks, results, prm,
                                                 raw);
    mark(mark_ctx, "refine");
}

}  // namespace mim
