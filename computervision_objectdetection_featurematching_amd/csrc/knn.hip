// knn.hip — brute-force NORM_L2 k=2 matching + Lowe ratio test on gfx950.
//
// Replaces BFMatcher(NORM_L2).knnMatch(view, scene, m, 2) and the ratio-test loop of
// /root/reference/src/TestsDetector.cpp:36,60,66-72 (OpenCV: matchers.cpp knnMatchImpl ->
// batch_distance.cpp batchDistance(K=2) -> normL2Sqr_).
//
// Exact path (SIFT rows: integers in [0,255]): D[i][j] = |t_i|^2 - 2 q_j.t_i on the bf16 MFMA
// (v_mfma_f32_32x32x16_bf16, fp32 accumulate).  Every operand (0..255, -2q in -510..0) is exact in
// bf16 and every partial sum is an integer of magnitude < 2^24, so D is exact in any order and
// d = sqrtf(D + |q_j|^2) is bit-identical to OpenCV's sqrt(normL2Sqr_).
// Top-2 selection: OpenCV orders by the float distance sqrtf(d^2) (ties -> lower train index).  The
// sweep keeps, branch-free, the two smallest (d^2, index) per query.  sqrtf is monotone and, below
// 2^22, injective on integers, so that pair is OpenCV's top-2 whenever the 2nd d^2 < 4e6 (equal d^2
// keep the lower index); other queries are rescanned exactly by knn2_rescan_kernel.
//
// Generic path (any other float rows): per-pair fp32 arithmetic in OpenCV's SSE normL2Sqr_ order
// (4 accumulators x 4 lanes, no FMA), bit-identical to oracle/mim_oracle.c l2sqr_sse_order.
#include "mim_internal.h"
#include <float.h>
#include <limits.h>

namespace mim {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// ------------------------------------------------------------------------------------------------
// prep: fp32 rows -> bf16 fragment-major tiles + squared norms + integrality flag.
// Fragment-major: a tile of 64 rows is [u 0..1][kstep s 0..7][lane 0..63][j 0..7] with
// row = 32u + (lane & 31), col = 16s + 8(lane >> 5) + j — exactly the per-lane operand of
// v_mfma_f32_32x32x16_bf16, so one 1 KiB wave load = one fragment, fully coalesced.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void prep_tile(const float* __restrict__ src, int n, uint16_t* __restrict__ frag,
                                          float* __restrict__ norm, int* __restrict__ flags, int tile) {
    const int tid = threadIdx.x;
    int bad = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ci = k * 256 + tid;  // output chunk (16 B) within the tile
        const int u = ci >> 9, s = (ci >> 6) & 7, lane = ci & 63;
        const int row = tile * 64 + 32 * u + (lane & 31);
        const int col = 16 * s + 8 * (lane >> 5);
        uint16_t o[8];
        if (row < n) {
            const float4* p = reinterpret_cast<const float4*>(src + (size_t)row * kDim + col);
            float4 a = p[0], b = p[1];
            float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bad |= !(v[j] >= 0.f && v[j] <= 255.f && v[j] == rintf(v[j]));
                __bf16 hb = (__bf16)v[j];
                o[j] = __builtin_bit_cast(uint16_t, hb);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0;
        }
        uint4 w;
        w.x = o[0] | (uint32_t(o[1]) << 16);
        w.y = o[2] | (uint32_t(o[3]) << 16);
        w.z = o[4] | (uint32_t(o[5]) << 16);
        w.w = o[6] | (uint32_t(o[7]) << 16);
        reinterpret_cast<uint4*>(frag)[(size_t)tile * 1024 + ci] = w;
    }
    if (tid < 64) {
        const int row = tile * 64 + tid;
        float s = 0.f;
        if (row < n) {
            const float* p = src + (size_t)row * kDim;
            for (int c = 0; c < kDim; ++c) s += p[c] * p[c];
        }
        norm[row] = row < n ? s : FLT_MAX;  // padded rows never win (copied as is by the DMA)
    }
    if (__any(bad) && (tid & 63) == 0) atomicOr(flags, 1);
}

// Every set created since the last batch in one launch: block b preps tile b - tile0 of the last
// job with tile0 <= b (jobs ascending in tile0; sets without rows own no tile).
__global__ __launch_bounds__(256) void prep_batch_kernel(const PrepJob* __restrict__ jobs, int njobs) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].tile0 <= (int)blockIdx.x) lo = mid;
        else hi = mid - 1;
    }
    const PrepJob J = jobs[lo];
    prep_tile(J.src, J.n, J.frag, J.norm, J.flags, (int)blockIdx.x - J.tile0);
}

// ------------------------------------------------------------------------------------------------
// Running top-2 of one query in the exact integer domain D = d^2 - |q|^2.  Candidates of one
// selection arrive in increasing train index: strict `<` keeps the earlier of equal D.
// ------------------------------------------------------------------------------------------------
struct LaneSel {
    float m1, m2;  // two smallest D
    int i1, i2;    // their train indices (INT_MAX = absent)
};

__device__ __forceinline__ void sel_init(LaneSel& s) {
    s.m1 = s.m2 = FLT_MAX;
    s.i1 = s.i2 = INT_MAX;
}

// min without IEEE-mode operand canonicalisation (fminf emits v_max x,x per operand): D values are
// finite integers or FLT_MAX, never NaN, and >= -FLT_MAX
__device__ __forceinline__ float dmin(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, -FLT_MAX); }

// branch-free insertion of (v, idx): 7 VALU
__device__ __forceinline__ void sel_push(LaneSel& s, float v, int idx) {
    const bool c1 = v < s.m1, c2 = v < s.m2;
    s.m2 = __builtin_amdgcn_fmed3f(s.m1, s.m2, v);
    s.i2 = c2 ? (c1 ? s.i1 : idx) : s.i2;
    s.m1 = dmin(s.m1, v);
    s.i1 = c1 ? idx : s.i1;
}

__device__ __forceinline__ bool dlt(float da, int ia, float db, int ib) { return da < db || (da == db && ia < ib); }

// union of two selections over disjoint rows: two smallest (D, index)
__device__ __forceinline__ LaneSel sel_merge(LaneSel a, const LaneSel& b) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float w = k ? b.m2 : b.m1;
        const int iw = k ? b.i2 : b.i1;
        const bool l1 = dlt(w, iw, a.m1, a.i1), l2 = dlt(w, iw, a.m2, a.i2);
        a.m2 = l1 ? a.m1 : (l2 ? w : a.m2);
        a.i2 = l1 ? a.i1 : (l2 ? iw : a.i2);
        a.m1 = l1 ? w : a.m1;
        a.i1 = l1 ? iw : a.i1;
    }
    return a;
}

__device__ __forceinline__ bool key_less(float ka, int ia, float kb, int ib) {
    return ka < kb || (ka == kb && ia < ib);
}

struct T2 {
    float k1; int i1; float k2; int i2;
};

__device__ __forceinline__ T2 top2_merge(T2 a, float k, int i) {
    const bool l1 = key_less(k, i, a.k1, a.i1);
    const bool l2 = key_less(k, i, a.k2, a.i2);
    T2 r;
    r.k1 = l1 ? k : a.k1;
    r.i1 = l1 ? i : a.i1;
    r.k2 = l1 ? a.k1 : (l2 ? k : a.k2);
    r.i2 = l1 ? a.i1 : (l2 ? i : a.i2);
    return r;
}

constexpr int kRescan = -2;  // Top2::i2 marker: the split's top-2 needs the exact rescan

// D value g of a 32x32 MFMA tile is train row (g&3) + 8(g>>2) + 4h of its 32-row block.  Indices
// are stored without the lane's 4h (uniform, scalar) and corrected at the end.
//   early tiles (the top-2 still changes often): every value is inserted branch-free (kPartials
//     independent selections per query: 1 measured best, it keeps the kernel at 128 VGPRs = 4
//     waves/SIMD);
//   later tiles (the partials merged into one selection): 4 consecutive rows are tested at once
//     against the 2nd best, the insertion runs only when some lane of the wave has a candidate.
#ifndef MIM_KNN_EARLY
#define MIM_KNN_EARLY 12
#endif
#ifndef MIM_KNN_GROUP
#define MIM_KNN_GROUP 4
#endif
#ifndef MIM_KNN_PREFETCH
#define MIM_KNN_PREFETCH 0
#endif
#ifndef MIM_KNN_PARTIALS
#define MIM_KNN_PARTIALS 1
#endif
constexpr int kPartials = MIM_KNN_PARTIALS;  // independent early-tile selections per query (1 or 2)
constexpr int kEarlyTiles = MIM_KNN_EARLY;
constexpr int kGroup = MIM_KNN_GROUP;  // values tested together in the late tiles (4 or 8)

// late tiles: the hit test of values g = kGroup*j .. kGroup*j + kGroup-1 (branch-free, scheduled
// between the MFMAs); T = the lane's filter
__device__ __forceinline__ bool sel_test(const f32x16& p, int j, float T) {
    float m = dmin(dmin(p[kGroup * j], p[kGroup * j + 1]), dmin(p[kGroup * j + 2], p[kGroup * j + 3]));
#pragma unroll
    for (int k = 4; k < kGroup; k += 2) m = dmin(m, dmin(p[kGroup * j + k], p[kGroup * j + k + 1]));
    return m < T;
}

// ... and the insertion of that group for the lanes that hit (rows in increasing order)
__device__ __forceinline__ void sel_group(const f32x16& p, int j, LaneSel& s, int base) {
#pragma unroll
    for (int k = 0; k < kGroup; ++k) {
        const int g = kGroup * j + k;
        sel_push(s, p[g], base + (g & 3) + 8 * (g >> 2));
    }
}

// Filter of a lane in the late tiles: below its own 2nd best, and not above the other row half's
// 2nd best (lanes l, l ^ 32 hold the same query; an equal D may still win on the lower index).
__device__ __forceinline__ float sel_filter(const LaneSel& s) {
    const int v = __float_as_int(s.m2);
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    const float other = __int_as_float((threadIdx.x & 32) ? r[0] : r[1]);
    return dmin(s.m2, other + 1.f);  // D are integers: other + 1 keeps D == other
}

// ------------------------------------------------------------------------------------------------
// Exact distance kernel.  Block = 4 waves = 256 queries (each wave: two 32-query MFMA column
// tiles, their -2q fragments held in VGPRs for the whole sweep).  Train tiles of 64 rows stream
// HBM -> registers -> LDS (double buffer, one barrier per tile); each wave reads the 16 KiB tile
// as 16 conflict-free ds_read_b128 and issues 32 MFMAs per tile.
// ------------------------------------------------------------------------------------------------
constexpr int kLdsTile = kTileBytes + 256;  // fragments + 64 norms

#ifndef MIM_KNN_OCC
#define MIM_KNN_OCC 4
#endif
__global__ __launch_bounds__(256, MIM_KNN_OCC) void knn2_bf16_kernel(const ProbDev* __restrict__ probs,
                                                          const KnnWork* __restrict__ works,
                                                          Top2* __restrict__ parts) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * kLdsTile];
    const KnnWork w = works[blockIdx.x];
    const ProbDev* P = probs + w.problem;
    if (*P->q.flags | *P->t.flags) return;  // not integer-valued: generic kernel handles it
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, r = lane & 31;
    const int nq = P->q.n;
    const uint4* __restrict__ tsrc = reinterpret_cast<const uint4*>(P->t.frag);
    const float* __restrict__ tnorm = P->t.norm;

    // ---- query fragments: B[k][j] = -2 q_j[k] (exact in bf16) ----
    const int qtile = (w.q0 >> 6) + wave;
    const bool qvalid = qtile < P->q.n_tiles;
    bf16x8 B[2][8];
    float qn[2] = {0.f, 0.f};
    {
        const uint4* qsrc = reinterpret_cast<const uint4*>(P->q.frag) + (size_t)(qvalid ? qtile : 0) * 1024;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                uint4 v = qvalid ? qsrc[(u * 8 + s) * 64 + lane] : make_uint4(0, 0, 0, 0);
                bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
                for (int j = 0; j < 8; ++j) b[j] = (__bf16)(-2.f * (float)b[j]);
                B[u][s] = b;
            }
            qn[u] = qvalid ? P->q.norm[qtile * 64 + 32 * u + r] : 0.f;
        }
    }
    LaneSel st[2][2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        sel_init(st[0][k]);
        sel_init(st[1][k]);
    }

    // ---- train tile staging: HBM -> LDS by DMA (global_load_lds, no VGPR staging), double
    // buffered; the barrier ending an iteration retires the DMA of the next tile ----
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define GLDS(tile, buf)                                                                          \
    do {                                                                                         \
        const u32x4* g_ = reinterpret_cast<const u32x4*>(tsrc) + (size_t)(tile) * 1024 + tid;     \
        u32x4* d_ = reinterpret_cast<u32x4*>(smem + (buf) * kLdsTile) + tid;                     \
        __builtin_amdgcn_global_load_lds(g_, d_, 16, 0, 0);                                      \
        __builtin_amdgcn_global_load_lds(g_ + 256, d_ + 256, 16, 0, 0);                          \
        __builtin_amdgcn_global_load_lds(g_ + 512, d_ + 512, 16, 0, 0);                          \
        __builtin_amdgcn_global_load_lds(g_ + 768, d_ + 768, 16, 0, 0);                          \
        if (tid < 64)                                                                            \
            __builtin_amdgcn_global_load_lds(tnorm + (size_t)(tile) * 64 + tid,                  \
                                             reinterpret_cast<float*>(smem + (buf) * kLdsTile + kTileBytes) + tid, \
                                             4, 0, 0);                                           \
    } while (0)

    if (w.tile0 < w.tile1) GLDS(w.tile0, 0);
    __syncthreads();
    float T0 = FLT_MAX, T1 = FLT_MAX;  // late-tile filters
    for (int tile = w.tile0; tile < w.tile1; ++tile) {
        const int buf = (tile - w.tile0) & 1;
        const bool more = tile + 1 < w.tile1;
        if (more) GLDS(tile + 1, buf ^ 1);
        const bf16x8* A = reinterpret_cast<const bf16x8*>(smem + buf * kLdsTile);
        const float* tn = reinterpret_cast<const float*>(smem + buf * kLdsTile + kTileBytes);
        const bool early = tile - w.tile0 < kEarlyTiles;
        if (tile - w.tile0 == kEarlyTiles) {  // switch: fold the partials into selection 0
            st[0][0] = sel_merge(st[0][0], st[0][1]);
            st[1][0] = sel_merge(st[1][0], st[1][1]);
            sel_init(st[0][1]);
            sel_init(st[1][1]);
            T0 = sel_filter(st[0][0]);
            T1 = sel_filter(st[1][0]);
        }
#pragma unroll
        for (int u2 = 0; u2 < 2; ++u2) {
            f32x16 acc0;
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                float4 v = *reinterpret_cast<const float4*>(tn + 32 * u2 + 8 * gg + 4 * h);
                acc0[4 * gg + 0] = v.x; acc0[4 * gg + 1] = v.y; acc0[4 * gg + 2] = v.z; acc0[4 * gg + 3] = v.w;
            }
            f32x16 acc1 = acc0;
#if MIM_KNN_PREFETCH
            bf16x8 af[8];  // all 8 A fragments of the half-tile issued before the first MFMA
#pragma unroll
            for (int s = 0; s < 8; ++s) af[s] = A[(u2 * 8 + s) * 64 + lane];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], B[0][s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], B[1][s], acc1, 0, 0, 0);
            }
#else
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const bf16x8 a = A[(u2 * 8 + s) * 64 + lane];
                acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, B[0][s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, B[1][s], acc1, 0, 0, 0);
            }
#endif
            const int row0 = tile * 64 + 32 * u2;
#ifdef MIM_KNN_NOSEL  // timing probe only: MFMA loop without the selection (results invalid)
            st[0][0].m1 = fminf(st[0][0].m1, fminf(acc0[0], acc0[15]));
            st[1][0].m1 = fminf(st[1][0].m1, fminf(acc1[0], acc1[15]));
            continue;
#endif
            if (early) {
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int idx = row0 + (g & 3) + 8 * (g >> 2);
                    sel_push(st[0][g % kPartials], acc0[g], idx);
                    sel_push(st[1][g % kPartials], acc1[g], idx);
                }
            } else {
                constexpr int NG = 16 / kGroup;
                bool h0[NG], h1[NG];
                bool any = false;
#pragma unroll
                for (int j = 0; j < NG; ++j) {
                    h0[j] = sel_test(acc0, j, T0);
                    h1[j] = sel_test(acc1, j, T1);
                    any |= h0[j] | h1[j];
                }
                if (__builtin_expect(__any(any), 0)) {  // rare past the early tiles
#pragma unroll
                    for (int j = 0; j < NG; ++j) {
                        if (__any(h0[j])) {
                            if (h0[j]) sel_group(acc0, j, st[0][0], row0);
                        }
                        if (__any(h1[j])) {
                            if (h1[j]) sel_group(acc1, j, st[1][0], row0);
                        }
                    }
                    T0 = sel_filter(st[0][0]);
                    T1 = sel_filter(st[1][0]);
                }
            }
        }
        __syncthreads();
    }
#undef GLDS

    // ---- merge partials and the two lane halves (disjoint train rows of the same query), keys ----
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        LaneSel m = sel_merge(st[u][0], st[u][1]);
        if (m.i1 != INT_MAX) m.i1 += 4 * h;
        if (m.i2 != INT_MAX) m.i2 += 4 * h;
        LaneSel o;
        o.m1 = __shfl_xor(m.m1, 32); o.m2 = __shfl_xor(m.m2, 32);
        o.i1 = __shfl_xor(m.i1, 32); o.i2 = __shfl_xor(m.i2, 32);
        m = sel_merge(m, o);
        const int q = qtile * 64 + 32 * u + r;
        if (h == 0 && qvalid && q < nq) {
            const float qq = qn[u];
            Top2 t;
            t.k1 = m.i1 == INT_MAX ? FLT_MAX : sqrtf(m.m1 + qq);
            t.k2 = m.i2 == INT_MAX ? FLT_MAX : sqrtf(m.m2 + qq);
            t.i1 = m.i1;
            t.i2 = m.i2;
            // d^2 >= 4e6: distinct integers may share a key (sqrt class), where the lower index
            // wins: rescan exactly.  Below, equal keys mean equal d^2, already in index order.
            if (t.i2 != INT_MAX && m.m2 + qq >= 4.0e6f) t.i2 = kRescan;
            parts[P->part_off + (long long)w.split * P->q_pad + q] = t;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Exact rescan of the queries the distance kernel marked (kRescan): one wave per query over the
// work item's train rows, fp32 distances of integer rows (exact in any order), keys sqrtf(d^2),
// (key, index) order.  Rare: the marked queries have a 3rd row in the 2nd key's sqrt class.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void knn2_rescan_kernel(const ProbDev* __restrict__ probs,
                                                          const KnnWork* __restrict__ works,
                                                          Top2* __restrict__ parts) {
    const KnnWork w = works[blockIdx.x];
    const ProbDev* P = probs + w.problem;
    if (*P->q.flags | *P->t.flags) return;  // generic kernel's parts are exact already
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nq = P->q.n, nt = P->t.n;
    Top2* out = parts + P->part_off + (long long)w.split * P->q_pad;
    const int r0 = w.tile0 * 64, r1 = min(w.tile1 * 64, nt);
    for (int k = 0; k < 256; k += 64) {
        const int q = w.q0 + k + lane;
        const bool marked = q < nq && out[q].i2 == kRescan;
        unsigned long long m = __ballot(marked);
        // waves take the marked queries round-robin
        int pick = 0;
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            if ((pick++ & 3) != wave) continue;
            const int qq = w.q0 + k + b;
            const float* qv = P->q.f32 + (size_t)qq * kDim;
            T2 t{FLT_MAX, INT_MAX, FLT_MAX, INT_MAX};
            for (int row = r0 + lane; row < r1; row += 64) {
                const float* tv = P->t.f32 + (size_t)row * kDim;
                float d2 = 0.f;
                for (int c = 0; c < kDim; ++c) {
                    const float d = qv[c] - tv[c];
                    d2 = fmaf(d, d, d2);  // integer terms, partial sums < 2^24: exact
                }
                t = top2_merge(t, sqrtf(d2), row);
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const float ok1 = __shfl_xor(t.k1, off), ok2 = __shfl_xor(t.k2, off);
                const int oi1 = __shfl_xor(t.i1, off), oi2 = __shfl_xor(t.i2, off);
                t = top2_merge(t, ok1, oi1);
                t = top2_merge(t, ok2, oi2);
            }
            if (lane == 0) out[qq] = Top2{t.k1, t.i1, t.k2, t.i2};
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Generic fp32 path: one thread per query, train rows broadcast from LDS, OpenCV SSE summation
// order (core/src/norm.cpp normL2Sqr_: 4 accumulators x 4 lanes, v_reduce_sum (a0+a2)+(a1+a3)).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float l2sqr_sse_order(const float* q, const float* t) {
    float acc[4][4];
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int l = 0; l < 4; ++l) acc[v][l] = 0.f;
#pragma unroll
    for (int j = 0; j < kDim; j += 16) {
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                const float d = q[j + 4 * v + l] - t[j + 4 * v + l];
                acc[v][l] = __fadd_rn(__fmul_rn(d, d), acc[v][l]);
            }
    }
    float s[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) s[l] = ((acc[0][l] + acc[1][l]) + acc[2][l]) + acc[3][l];
    return (s[0] + s[2]) + (s[1] + s[3]);
}

__global__ __launch_bounds__(256) void knn2_f32_kernel(const ProbDev* __restrict__ probs,
                                                       const KnnWork* __restrict__ works,
                                                       Top2* __restrict__ parts) {
    __shared__ __attribute__((aligned(16))) float tl[kTileRows * kDim];
    const KnnWork w = works[blockIdx.x];
    const ProbDev* P = probs + w.problem;
    if (!(*P->q.flags | *P->t.flags)) return;  // integer-valued: exact MFMA kernel handles it
    const int tid = threadIdx.x;
    const int nq = P->q.n, nt = P->t.n;
    const int q = w.q0 + tid;
    float qv[kDim];
    const bool qvalid = q < nq;
#pragma unroll
    for (int c = 0; c < kDim; c += 4) {
        float4 v = qvalid ? *reinterpret_cast<const float4*>(P->q.f32 + (size_t)q * kDim + c)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        qv[c] = v.x; qv[c + 1] = v.y; qv[c + 2] = v.z; qv[c + 3] = v.w;
    }
    float k1 = FLT_MAX, k2 = FLT_MAX;
    int i1 = INT_MAX, i2 = INT_MAX;
    for (int tile = w.tile0; tile < w.tile1; ++tile) {
        __syncthreads();
        for (int e = tid; e < kTileRows * kDim / 4; e += 256) {
            const int row = tile * 64 + e / (kDim / 4);
            float4 v = row < nt ? reinterpret_cast<const float4*>(P->t.f32)[(size_t)tile * 64 * (kDim / 4) + e]
                                : make_float4(0.f, 0.f, 0.f, 0.f);
            reinterpret_cast<float4*>(tl)[e] = v;
        }
        __syncthreads();
        const int rows = min(64, nt - tile * 64);
        for (int rr = 0; rr < rows; ++rr) {
            const float d = sqrtf(l2sqr_sse_order(qv, tl + rr * kDim));
            // OpenCV compares the bit patterns as int: for non-negative floats that is float order;
            // NaN (> FLT_MAX bits) and values >= FLT_MAX are never inserted.
            if (d < k2) {
                const int j = tile * 64 + rr;
                if (d < k1) { k2 = k1; i2 = i1; k1 = d; i1 = j; }
                else { k2 = d; i2 = j; }
            }
        }
    }
    if (qvalid) parts[P->part_off + (long long)w.split * P->q_pad + q] = Top2{k1, i1, k2, i2};
}

// ------------------------------------------------------------------------------------------------
// Merge train splits, emit knnMatch rows, Lowe ratio test and ordered compaction
// (TestsDetector.cpp:62-72): survivors keep ascending query order — the order findHomography's
// point lists and inlier mask are indexed by.  One 1024-thread block per problem.
// Output pts[k] = (objPt.x, objPt.y, scenePt.x, scenePt.y) of the k-th good match.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void ratio_compact_kernel(const ProbDev* __restrict__ probs,
                                                            const Top2* __restrict__ parts, float ratio,
                                                            int32_t* __restrict__ good_q,
                                                            int32_t* __restrict__ good_t,
                                                            float4* __restrict__ pts,
                                                            int* __restrict__ n_good,
                                                            int32_t* __restrict__ knn_idx,
                                                            float* __restrict__ knn_dist) {
    __shared__ int wsum[16];
    __shared__ int wbase[17];
    const ProbDev* P = probs + blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nq = P->q.n;
    int running = 0;
    for (int base = 0; base < nq; base += 1024) {
        const int q = base + tid;
        T2 m{FLT_MAX, INT_MAX, FLT_MAX, INT_MAX};
        if (q < nq) {
            for (int sp = 0; sp < P->nsplit; ++sp) {
                const Top2 t = parts[P->part_off + (long long)sp * P->q_pad + q];
                m = top2_merge(m, t.k1, t.i1);
                m = top2_merge(m, t.k2, t.i2);
            }
        }
        const float k1 = m.k1, k2 = m.k2;
        const int i1 = m.i1, i2 = m.i2;
        if (q < nq) {
            if (knn_idx) {
                knn_idx[2 * q] = i1 == INT_MAX ? -1 : i1;
                knn_idx[2 * q + 1] = i2 == INT_MAX ? -1 : i2;
                knn_dist[2 * q] = k1;
                knn_dist[2 * q + 1] = k2;
            }
        }
        const bool good = q < nq && i1 != INT_MAX && i2 != INT_MAX && k1 < ratio * k2;
        const unsigned long long bal = __ballot(good);
        const int within = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        if (lane == 0) wsum[wave] = __popcll(bal);
        __syncthreads();
        if (tid == 0) {
            int acc = 0;
            for (int i = 0; i < 16; ++i) { wbase[i] = acc; acc += wsum[i]; }
            wbase[16] = acc;
        }
        __syncthreads();
        if (good) {
            const long long o = P->good_off + running + wbase[wave] + within;
            good_q[o] = q;
            good_t[o] = i1;
            const float2 a = P->q.kp[q], b = P->t.kp[i1];
            pts[o] = make_float4(a.x, a.y, b.x, b.y);
        }
        running += wbase[16];
        __syncthreads();
    }
    if (tid == 0) n_good[blockIdx.x] = running;
}

// ------------------------------------------------------------------------------------------------
// host-side launchers (called from api.cpp)
// ------------------------------------------------------------------------------------------------
void launch_prep_batch(const PrepJob* jobs, int njobs, int total_tiles, hipStream_t st) {
    if (njobs > 0 && total_tiles > 0) prep_batch_kernel<<<total_tiles, 256, 0, st>>>(jobs, njobs);
}

// Both kernels are enqueued; each block reads its problem's integrality flags (set by prep on the
// device) and only the matching kernel does the work, so no host round trip is needed.
void launch_knn(const ProbDev* probs, const KnnWork* works, int n_works, Top2* parts, hipStream_t st) {
    if (n_works <= 0) return;
    knn2_bf16_kernel<<<n_works, 256, 0, st>>>(probs, works, parts);
    knn2_rescan_kernel<<<n_works, 256, 0, st>>>(probs, works, parts);
    knn2_f32_kernel<<<n_works, 256, 0, st>>>(probs, works, parts);
}

void launch_ratio(const ProbDev* probs, int n_probs, const Top2* parts, float ratio, int32_t* good_q,
                  int32_t* good_t, float4* pts, int* n_good, int32_t* knn_idx, float* knn_dist,
                  hipStream_t st) {
    if (n_probs > 0)
        ratio_compact_kernel<<<n_probs, 1024, 0, st>>>(probs, parts, ratio, good_q, good_t, pts, n_good,
                                                       knn_idx, knn_dist);
}

}  // namespace mim
