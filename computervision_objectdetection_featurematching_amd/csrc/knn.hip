// knn.hip — brute-force NORM_L2 k=2 matching + Lowe ratio test on gfx950.
//
// Replaces BFMatcher(NORM_L2).knnMatch(view, scene, m, 2) and the ratio-test loop of
// /root/reference/src/TestsDetector.cpp:36,60,66-72 (OpenCV: matchers.cpp knnMatchImpl ->
// batch_distance.cpp batchDistance(K=2) -> normL2Sqr_).
//
// Exact path (SIFT rows: integers in [0,255]): a set is stored once as t'' = 127 - t in [-128,127]
// (exact in i8); as a query the same bytes give q' = q - 128 = ~t''.  Then q - t = q' + t'' + 1 and
//   |q - t|^2 = n2(t) + 2 q'.t'' + c(q),   n2(t) = |t - 128|^2,  c(q) = |q - 128|^2 + 2 sum(q - 128),
// with q'.t'' on the i8 MFMA (v_mfma_i32_32x32x32_i8, i32 accumulate: 2x the bf16 rate).  Every
// distance is an exact integer, so d = sqrtf(d^2) is bit-identical to OpenCV's sqrt(normL2Sqr_)
// (SURVEY.md Appendix B).  The accumulator starts at floor(n2/2), so the MFMA yields
// R = q'.t'' + floor(n2/2) and D = d^2 - c(q) = 2R + (n2 & 1) (one v_lshl_add_u32).
// Top-2 selection: OpenCV orders by the float distance sqrtf(d^2) (ties -> lower train index).  The
// sweep keeps, branch-free, the two smallest (D, index) per query.  sqrtf is monotone and, below
// 2^22, injective on integers, so that pair is OpenCV's top-2 whenever the 2nd d^2 < 4e6 (equal d^2
// keep the lower index); other queries are rescanned exactly by knn2_rescan_kernel.
//
// Generic path (any other float rows): per-pair fp32 arithmetic in OpenCV's SSE normL2Sqr_ order
// (4 accumulators x 4 lanes, no FMA), bit-identical to oracle/mim_oracle.c l2sqr_sse_order.
#include "mim_internal.h"
#include <float.h>
#include <limits.h>

namespace mim {

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(16))) int i32x16;
typedef const __attribute__((address_space(1))) i32x4 gi32x4;  // global (not flat) loads
typedef const __attribute__((address_space(1))) int gint;

// ------------------------------------------------------------------------------------------------
// prep: fp32 rows -> i8 fragment-major tiles of 127 - d + norms + integrality flag.
// Fragment-major: a tile of 64 rows is [u 0..1][kstep s 0..3][lane 0..63][j 0..15] with
// row = 32u + (lane & 31), col = 32s + 16(lane >> 5) + j — the per-lane operand of
// v_mfma_i32_32x32x32_i8 (query and train use the same k order, so the product is k-order free);
// one 1 KiB wave load = one fragment, fully coalesced.
// Norm block per tile (kNormWords): [64] floor(n2/2), [2] the 64 values n2 & 1 as a bit mask + [62]
// zero (the train side, staged to LDS as is), [64] c (the query side), [64] the early-phase key
// addends K = 2^28 + 128 (n2 & 1) + row (train side, staged for the early tiles only); padded rows
// floor(n2/2) = 2^30 - 1, n2 & 1 = 1, so D = INT_MAX, and K = 255, so their early key is UINT_MAX.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void prep_tile(const float* __restrict__ src, int n, int8_t* __restrict__ frag,
                                          int* __restrict__ norm, int* __restrict__ flags, int tile) {
    // per row: n2 and sum(t - 128) in 4 partials (one per 32-column block = one per wave), summed by
    // the first wave; every row is read once, by the fragment pass (integer sums: exact in any order)
    __shared__ int2 part[4][64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int bad = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int ci = k * 256 + tid;  // output chunk (16 B) within the tile: u = k, s = w
        const int row = tile * 64 + 32 * k + (lane & 31);
        const int col = 32 * w + 16 * (lane >> 5);
        uint32_t o[4] = {0, 0, 0, 0};
        int n2 = 0, sum = 0;
        if (row < n) {
            const float4* p = reinterpret_cast<const float4*>(src + (size_t)row * kDim + col);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 a = p[c];
                const float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    bad |= !(v[j] >= 0.f && v[j] <= 255.f && v[j] == rintf(v[j]));
                    const int d = (int)v[j] - 128;  // garbage for non-integer rows (flagged, unused)
                    n2 += d * d;
                    sum += d;
                    o[c] |= (uint32_t)((127 - (int)v[j]) & 0xff) << (8 * j);
                }
            }
        }
        reinterpret_cast<uint4*>(frag)[(size_t)tile * 512 + ci] = make_uint4(o[0], o[1], o[2], o[3]);
        n2 += __shfl_xor(n2, 32);  // the other 16 columns of the row's 32-column block
        sum += __shfl_xor(sum, 32);
        if (lane < 32) part[w][32 * k + lane] = make_int2(n2, sum);
    }
    __syncthreads();
    if (tid < 64) {
        const int row = tile * 64 + tid;
        int n2 = 0, sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            n2 += part[q][tid].x;
            sum += part[q][tid].y;
        }
        int* nb = norm + (size_t)tile * kNormWords;
        nb[tid] = row < n ? n2 >> 1 : (1 << 30) - 1;
        // the 64 parities as one bit mask (row i = bit i) in words 64, 65; words 66..127 zero
        const unsigned long long pm = __ballot(row < n ? n2 & 1 : 1);  // tid < 64: wave 0, all lanes
        nb[64 + tid] = tid < 2 ? (int)(uint32_t)(pm >> (32 * tid)) : 0;
        nb[128 + tid] = n2 + 2 * sum;
        nb[192 + tid] = row < n ? (1 << 28) + ((n2 & 1) << 7) + tid : 255;
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
// Running top-2 of one query in the exact integer domain D = d^2 - c(q).  Candidates of one
// selection arrive in increasing train index: strict `<` keeps the earlier of equal D.
// ------------------------------------------------------------------------------------------------
struct LaneSel {
    int m1, m2;  // two smallest D (INT_MAX = absent)
    int i1, i2;  // their train indices (INT_MAX = absent)
};

__device__ __forceinline__ void sel_init(LaneSel& s) {
    s.m1 = s.m2 = INT_MAX;
    s.i1 = s.i2 = INT_MAX;
}

// branch-free insertion of (v, idx): 7 VALU
__device__ __forceinline__ void sel_push(LaneSel& s, int v, int idx) {
    const bool c1 = v < s.m1, c2 = v < s.m2;
    s.m2 = max(min(s.m1, s.m2), min(max(s.m1, s.m2), v));  // med3 (one v_med3_i32)
    s.i2 = c2 ? (c1 ? s.i1 : idx) : s.i2;
    s.m1 = min(s.m1, v);
    s.i1 = c1 ? idx : s.i1;
}

__device__ __forceinline__ bool dlt(int da, int ia, int db, int ib) { return da < db || (da == db && ia < ib); }

// union of two selections over disjoint rows: two smallest (D, index)
__device__ __forceinline__ LaneSel sel_merge(LaneSel a, const LaneSel& b) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int w = k ? b.m2 : b.m1;
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

// Accumulator value g of a 32x32 MFMA tile is train row (g&3) + 8(g>>2) + 4h of its 32-row block.
// Indices are stored without the lane's 4h (uniform, scalar) and corrected at the end.
//   early tiles (the top-2 still changes often): every D = 2R + p inserted branch-free;
//   later tiles: the min of a lane's 16 R is tested against the lane's threshold on R (a superset of
//     the rows that can enter the top-2); the exact insertion runs only for the 4-row groups in
//     which some lane of the wave has a candidate.
#ifndef MIM_KNN_EARLY
#define MIM_KNN_EARLY 4
#endif
constexpr int kEarlyTiles = MIM_KNN_EARLY;
#ifndef MIM_KNN_LATE_UNROLL
#define MIM_KNN_LATE_UNROLL 1
#endif
// timing probes (diagnostic builds only, results wrong): 1 late tiles without the insertion events,
// 2 without the min filter too, 3 and with zero accumulator seeds (no seed LDS reads)
#ifndef MIM_KNN_PROBE
#define MIM_KNN_PROBE 0
#endif
// parity word of a late half tile waited for with the seeds, before the MFMAs (1) or after them (0)
#ifndef MIM_KNN_PW_EARLY
#define MIM_KNN_PW_EARLY 0
#endif
// s_setprio 1 for waves 4-7 (the younger half of each SIMD's pair)
#ifndef MIM_KNN_PRIO
#define MIM_KNN_PRIO 0
#endif


// Threshold on R of a lane in the late tiles.  Lanes l, l ^ 32 hold the same query over disjoint
// row halves; the union of their two top-2 lists always contains the query's top-2 so far.  A new
// row can enter that top-2 only if D <= Dc, the 2nd smallest of the pair's four D (an equal D may
// still win on the lower index), and a row that does enters its own lane's list, so the filter
// keeps the invariant.  D = 2R + p with p in {0,1} gives R <= floor(Dc/2).
// o1 <= o2: the partner lane's m1, m2 (exchanged by permlane32_swap once per stage; the partner's
// values only decrease, so a stale copy gives a threshold >= the exact one: still a superset).
__device__ __forceinline__ int late_threshold(const LaneSel& s, int o1, int o2) {
    return min(max(s.m1, o1), min(s.m2, o2)) >> 1;  // 2nd smallest of {m1 <= m2, o1 <= o2}, halved
}
__device__ __forceinline__ int dval(int R, int p) { return (R << 1) | p; }  // v_lshl_or_b32

// v_med3_u32 (the compiler rewrites the max/min form of a top-2 update into a max and two mins)
__device__ __forceinline__ unsigned med3_u32(unsigned a, unsigned b, unsigned c) {
    unsigned r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ int med3_i32(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// insertion events of the late tiles: 0 a ballot per row of a hit row group and an out-of-line push per
// hit row; 1 the group's two smallest (R, row) keys branch-free, the first pushed in every lane, the
// second only when some lane can still take it, the rest of the group by rows after that (rare)
#ifndef MIM_KNN_EVENT
#define MIM_KNN_EVENT 0
#endif
// waves 4-7 (the second wave of each SIMD's pair in a block) defer the filter and events of each
// stage's last half tile past the stage barrier, so a SIMD's two waves of one block do not filter at
// the same time (MI355X_MICROARCH.md, "try a stagger")
#ifndef MIM_KNN_STAGGER
#define MIM_KNN_STAGGER 0
#endif

// ------------------------------------------------------------------------------------------------
// Exact distance kernel.  Block = kKnnWaves waves = kKnnBlockQ queries (each wave: kKnnQT 32-query
// MFMA column tiles, their q' fragments held in VGPRs for the whole sweep).  Train rows stream
// HBM -> LDS by LDS-DMA in stages of kKnnStage 64-row tiles (double buffer, one barrier per stage);
// per tile a wave reads the 8 KiB of fragments as 8 conflict-free ds_read_b128 and issues 8 kKnnQT
// i8 MFMAs.
// ------------------------------------------------------------------------------------------------
constexpr int kLdsTile = kTileBytes + 768;  // fragments + the train half of the norm block + the key addends
constexpr int kStage = kKnnStage;
constexpr int kThreads = 64 * kKnnWaves;
constexpr int kStageChunks = kStage * kTileBytes / 16 / kThreads;  // 16-B fragment chunks per thread
static_assert(kStageChunks * 16 * kThreads == kStage * kTileBytes, "stage split");

#ifndef MIM_KNN_OCC
#define MIM_KNN_OCC 4
#endif
__global__ __launch_bounds__(kThreads, MIM_KNN_OCC) void knn2_i8_kernel(  // OCC = waves per SIMD
    const ProbDev* __restrict__ probs, const KnnWork* __restrict__ works, const int* __restrict__ seg_start,
    Top2* __restrict__ parts, int* __restrict__ dyn_ctr) {
    constexpr int QT = kKnnQT;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * kStage * kLdsTile];
    __shared__ int s_item;
    // static: block b runs works[seg_start[b] .. seg_start[b + 1]); dynamic (dyn_ctr != null): the works
    // are 8 lists (seg_start[0..8]), block b pulls items from list b mod 8 (its XCD's) with an atomic
    // counter, then from the other lists, so a block that starts late (its CU held by another batch's
    // kernel) takes less
    int si = dyn_ctr ? 0 : seg_start[blockIdx.x];
    const int si_end = dyn_ctr ? 0 : seg_start[blockIdx.x + 1];
    int list = blockIdx.x & 7, lists_done = 0;
  for (;;) {
    if (dyn_ctr) {
        int idx = -1;
        while (lists_done < 8) {
            if (threadIdx.x == 0) s_item = atomicAdd(dyn_ctr + list, 1);
            __syncthreads();
            const int k = s_item;
            __syncthreads();
            if (k < seg_start[list + 1] - seg_start[list]) {
                idx = seg_start[list] + k;
                break;
            }
            list = (list + 1) & 7;
            ++lists_done;
        }
        if (idx < 0) break;
        si = idx;
    } else if (si >= si_end) {
        break;
    }
    const KnnWork w = works[si];
    ++si;
    const ProbDev* P = probs + w.problem;
    if (*P->q.flags | *P->t.flags) continue;  // not integer-valued: generic kernel handles it
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, r = lane & 31;
    const int nq = P->q.n;
    const uint4* __restrict__ tsrc = reinterpret_cast<const uint4*>(P->t.frag);
    const int* __restrict__ tnorm = P->t.norm;

    // ---- query fragments q': column tile u = query rows qbase + 32u .. + 31 ----
    const int qbase = w.q0 + wave * 32 * QT;
    i32x4 B[QT][4];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
        const int qr = qbase + 32 * u, qt = qr >> 6, qh = (qr >> 5) & 1;
        const bool ok = qt < P->q.n_tiles;
        const int qtc = ok ? qt : 0;  // rows past the set: loaded from tile 0, never written out
        const gi32x4* qsrc = (const gi32x4*)(P->q.frag) + (size_t)qtc * 512;
#pragma unroll
        for (int s = 0; s < 4; ++s) B[u][s] = ~qsrc[(qh * 4 + s) * 64 + lane];  // q' = ~t''
    }
    LaneSel st[QT];
    int T[QT];  // late-tile thresholds on R
    // the partner lane's (l ^ 32) m1, m2 as of the last refresh (every stage): between refreshes an
    // insertion recomputes the threshold from its own fresh pair and these (the partner's values only
    // decrease, so a stale copy gives a threshold >= the exact one: a superset, no exchange per event)
    int o1c[QT], o2c[QT];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
        sel_init(st[u]);
        T[u] = INT_MAX;
    }

    // ---- staging: LDS-DMA (global_load_lds_dwordx4 / _dword), double buffered, one barrier per
    // stage of kStage 64-row tiles.  One wave-instruction writes 64 lanes x size contiguous bytes at a
    // wave-uniform LDS base, which the fragment-major tile already is; the norm half of the tile's
    // norm block (floor(n2/2), parity mask) is two 256-B pieces.  No staging VGPRs, no ds_write pass.
    // LDS stage layout: kStage x [8 KiB fragments | 512 B norms]; tiles past the work item's range
    // are not loaded.  (Every LDS read is an ext-vector or int access of the one smem array: with the
    // seeds read as a struct type the waitcnt pass could not tell them from the DMA's target and
    // waited for the next stage's DMA before each tile.)
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    if (MIM_KNN_PRIO && wv >= 4) __builtin_amdgcn_s_setprio(1);
    auto stage_dma = [&](int t0, int buf, bool keys) {
        unsigned char* base = smem + buf * kStage * kLdsTile;
#pragma unroll
        for (int c = 0; c < kStageChunks; ++c) {
            const int cw = c * kThreads + wv * 64, tt = cw >> 9;  // the wave's first chunk: uniform
            if (kStage == 1 || t0 + tt < w.tile1)
                __builtin_amdgcn_global_load_lds((const void*)(tsrc + (size_t)t0 * 512 + cw + lane),
                                                 (__attribute__((address_space(3))) void*)(base + tt * kLdsTile + (cw & 511) * 16),
                                                 16, 0, 0);
        }
#pragma unroll
        for (int p = wv; p < 2 * kStage; p += kKnnWaves) {  // piece p: tile p >> 1, norm words 64 (p & 1) ..
            const int tt = p >> 1;
            if (kStage == 1 || t0 + tt < w.tile1)
                __builtin_amdgcn_global_load_lds((const void*)(tnorm + (size_t)(t0 + tt) * kNormWords + 64 * (p & 1) + lane),
                                                 (__attribute__((address_space(3))) void*)(base + tt * kLdsTile + kTileBytes + 256 * (p & 1)),
                                                 4, 0, 0);
        }
        if (keys) {  // early stages: the key addends (norm words 192..255) of each tile
#pragma unroll
            for (int tt = wv; tt < kStage; tt += kKnnWaves)
                if (kStage == 1 || t0 + tt < w.tile1)
                    __builtin_amdgcn_global_load_lds((const void*)(tnorm + (size_t)(t0 + tt) * kNormWords + 192 + lane),
                                                     (__attribute__((address_space(3))) void*)(base + tt * kLdsTile + kTileBytes + 512),
                                                     4, 0, 0);
        }
    };

    const int tile_e = min(w.tile1, w.tile0 + (kEarlyTiles + kStage - 1) / kStage * kStage);
    if (w.tile0 < w.tile1) stage_dma(w.tile0, 0, w.tile0 < tile_e);
    // retire every prologue load (q' fragments included) here: with one still pending at the loop
    // entry the waitcnt pass keeps a vmcnt(0) in the loop
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

    // the 32x32 block u2 of a tile: accumulators start at floor(n2/2) (LDS), R = q'.t'' + floor(n2/2)
    auto block_mfma = [&](const unsigned char* tb, int u2, i32x16 (&acc)[QT]) {
        const i32x4* A = reinterpret_cast<const i32x4*>(tb);
        const int* tnu = reinterpret_cast<const int*>(tb + kTileBytes) + 32 * u2 + 4 * h;
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            const i32x4 n = MIM_KNN_PROBE >= 3 ? i32x4{0, 0, 0, 0} : *reinterpret_cast<const i32x4*>(tnu + 8 * gg);
            acc[0][4 * gg + 0] = n.x; acc[0][4 * gg + 1] = n.y; acc[0][4 * gg + 2] = n.z; acc[0][4 * gg + 3] = n.w;
        }
#pragma unroll
        for (int u = 1; u < QT; ++u) acc[u] = acc[0];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const i32x4 a = A[(u2 * 4 + s) * 64 + lane];
#pragma unroll
            for (int u = 0; u < QT; ++u) acc[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, B[u][s], acc[u], 0, 0, 0);
        }
    };
    // early tiles: every value enters a branch-free top-2 of 32-bit keys
    //   key = (R << 8) + K = 128 D + row + 2^28  (K = 2^28 + 128 (n2 & 1) + row from the tile's norm block)
    // ordered as (D, row): R in [-2^20.1, 2^22] keeps real keys in (0, 2^31); a padded row (R = 2^30 - 1,
    // K = 255) wraps to exactly UINT_MAX and never enters.  Three VALU per value (v_lshl_add_u32,
    // v_med3_u32, v_min_u32); the tile's two keys per lane and column tile are decoded and merged into the
    // (D, index) lists at the tile's end.
    auto tile_early = [&](const unsigned char* tb, int tile) {
        const int* tk = reinterpret_cast<const int*>(tb + kTileBytes + 512) + 4 * h;
        unsigned k1[QT], k2[QT];
#pragma unroll
        for (int u = 0; u < QT; ++u) k1[u] = k2[u] = 0xFFFFFFFFu;
#pragma unroll
        for (int u2 = 0; u2 < 2; ++u2) {
            i32x16 acc[QT];
            block_mfma(tb, u2, acc);
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const i32x4 kv = *reinterpret_cast<const i32x4*>(tk + 32 * u2 + 8 * gg);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
#pragma unroll
                    for (int u = 0; u < QT; ++u) {
                        const unsigned key = ((unsigned)acc[u][4 * gg + k] << 8) + (unsigned)kv[k];
                        k2[u] = med3_u32(k1[u], k2[u], key);  // = max(k1, min(k2, key)) as k1 <= k2
                        k1[u] = min(k1[u], key);
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < QT; ++u) {
            LaneSel t;
            // D = (key - 2^28) >> 7, row = key & 127 (with the lane's 4h, which the lists store without)
            t.m1 = k1[u] == 0xFFFFFFFFu ? INT_MAX : (int)(k1[u] - (1u << 28)) >> 7;
            t.i1 = k1[u] == 0xFFFFFFFFu ? INT_MAX : tile * 64 + (int)(k1[u] & 127) - 4 * h;
            t.m2 = k2[u] == 0xFFFFFFFFu ? INT_MAX : (int)(k2[u] - (1u << 28)) >> 7;
            t.i2 = k2[u] == 0xFFFFFFFFu ? INT_MAX : tile * 64 + (int)(k2[u] & 127) - 4 * h;
            st[u] = sel_merge(st[u], t);
        }
    };
    // late tiles: one min over a lane's 16 R per column tile against its threshold, the exact
    // insertion only in groups some lane hits.  half_filter: the 32-row half tile starting at row0
    // (accumulators acc, parity word pw); keyed: keys (R << 3 | g) cannot overflow (no padded row)
    auto half_filter = [&](const i32x16 (&acc)[QT], unsigned pw, int row0, bool keyed) {
        // a lane's 16 R as two row groups (g 0-7, 8-15): the group minima cost one v_min more
        // than a single min chain and let an event compare the rows of the hit groups only
        int mn[QT], gmn[QT][2];
        unsigned long long bm[QT], any = 0;  // wave masks of the lanes with a candidate (SGPR pairs)
#pragma unroll
        for (int u = 0; u < QT; ++u) {
            const i32x16& p = acc[u];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                int a = min(min(p[8 * i], p[8 * i + 1]), p[8 * i + 2]);
                a = min(min(a, p[8 * i + 3]), p[8 * i + 4]);
                a = min(min(a, p[8 * i + 5]), p[8 * i + 6]);
                gmn[u][i] = min(a, p[8 * i + 7]);
            }
            mn[u] = min(gmn[u][0], gmn[u][1]);
            bm[u] = __ballot(mn[u] <= T[u]);
            any |= bm[u];
        }
        // the masks are tested on the scalar unit (re-evaluating the compare as a ballot made the
        // compiler rebuild each one with a v_cndmask + v_cmp pair per event)
        if (MIM_KNN_PROBE == 1) asm volatile("" ::"s"(any));
        if (MIM_KNN_PROBE != 1 && __builtin_expect(any != 0, 0)) {  // ~1 insertion per wave and half tile
#pragma unroll
            for (int u = 0; u < QT; ++u) {
                if (bm[u] != 0) {
                    // per row of a hit group: one compare (the ballot) and, if some lane has the row
                    // under its threshold, an unconditional insertion in every lane (the lane lists
                    // stay the exact top-2 of the rows pushed, a superset of the filtered ones); the
                    // row ballots of a group first (independent compares into SGPR pairs), then a
                    // not-taken scalar test per row: the insertion code sits out of line
                    unsigned long long gb[2];
#pragma unroll
                    for (int i = 0; i < 2; ++i) gb[i] = __ballot(gmn[u][i] <= T[u]);
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (gb[i] != 0) {
                            // rows of group i in this lane: pos = (g & 3) + 8 (g >> 2) + 16 i (without 4h),
                            // ascending with g; the parity of the row is bit pos of pw
                            int k2 = INT_MAX;
                            if (MIM_KNN_EVENT == 1 && keyed) {
                                // the group's two smallest (R, row) keys: every lane pushes its own
                                // smallest row (pushing rows beyond the filter keeps a lane list the
                                // exact top-2 of the rows pushed into it); the second only if some lane
                                // can still take it once the first is in; further rows by row ballots
                                int k1 = INT_MAX;
#pragma unroll
                                for (int g = 0; g < 8; ++g) {
                                    const int key = (acc[u][8 * i + g] << 3) | g;
                                    k2 = med3_i32(k1, k2, key);
                                    k1 = min(k1, key);
                                }
                                const int pos1 = (k1 & 3) + 8 * ((k1 >> 2) & 1) + 16 * i;
                                sel_push(st[u], dval(k1 >> 3, (pw >> pos1) & 1), row0 + pos1);
                                T[u] = late_threshold(st[u], o1c[u], o2c[u]);
                                if (__builtin_expect(__ballot((k2 >> 3) <= T[u]) == 0, 1)) continue;
                                const int pos2 = (k2 & 3) + 8 * ((k2 >> 2) & 1) + 16 * i;
                                sel_push(st[u], dval(k2 >> 3, (pw >> pos2) & 1), row0 + pos2);
                                T[u] = late_threshold(st[u], o1c[u], o2c[u]);
                            }
                            // rows in index order (keyed: only those after the second key, all of which
                            // have a larger D than the two pushed rows' or an equal D and a larger row)
                            unsigned long long hm[8];
#pragma unroll
                            for (int g = 0; g < 8; ++g)
                                hm[g] = __ballot(acc[u][8 * i + g] <= T[u] &&
                                                 (MIM_KNN_EVENT != 1 || !keyed || ((acc[u][8 * i + g] << 3) | g) > k2));
#pragma unroll
                            for (int g = 8 * i; g < 8 * i + 8; ++g) {
                                if (__builtin_expect(hm[g - 8 * i] != 0, 0))
                                    sel_push(st[u], dval(acc[u][g], (pw >> ((g & 3) + 8 * (g >> 2))) & 1),
                                             row0 + (g & 3) + 8 * (g >> 2));
                            }
                        }
                    }
                    T[u] = late_threshold(st[u], o1c[u], o2c[u]);
                }
            }
        }
    };
    // deferred half tile (MIM_KNN_STAGGER, waves 4-7): its accumulators, parity word and first row
    i32x16 dacc[QT];
    unsigned dpw = 0;
    int drow0 = -1;
    bool dkeyed = false;
    const bool stagger = MIM_KNN_STAGGER && wv >= 4;
    // the last set tile holds padded rows (R ~ 2^30): no keyed events there
    const int pad_tile = (P->t.n & 63) ? P->t.n_tiles - 1 : INT_MAX;
    auto tile_late = [&](const unsigned char* tb, int tile, bool defer) {
        const int* tn = reinterpret_cast<const int*>(tb + kTileBytes);
#pragma unroll
        for (int u2 = 0; u2 < 2; ++u2) {
            const int row0 = tile * 64 + 32 * u2;
            const unsigned pw = (unsigned)tn[64 + u2] >> (4 * h);  // bit 8j + k: n2 & 1 of the lane's row
            i32x16 acc[QT];
            if (MIM_KNN_PW_EARLY) asm volatile("" ::"v"(pw));
            block_mfma(tb, u2, acc);
            // the parity word is read with the seeds (its LDS latency hidden behind the MFMAs), not
            // inside the rare insertion path where the compiler would sink it: one LDS round trip per event
            if (!MIM_KNN_PW_EARLY) asm volatile("" ::"v"(pw));
            if (MIM_KNN_PROBE >= 2) {
#pragma unroll
                for (int u = 0; u < QT; ++u) asm volatile("" ::"v"(acc[u]));
                continue;
            }
            if (defer && u2 == 1) {
#pragma unroll
                for (int u = 0; u < QT; ++u) dacc[u] = acc[u];
                dpw = pw;
                drow0 = row0;
                dkeyed = tile != pad_tile;
                continue;
            }
            half_filter(acc, pw, row0, tile != pad_tile);
        }
    };
    auto flush_deferred = [&]() {
        if (stagger && drow0 >= 0) {
            half_filter(dacc, dpw, drow0, dkeyed);
            drow0 = -1;
        }
    };

    int stage = w.tile0;
    for (; stage < tile_e; stage += kStage) {
        const int buf = ((stage - w.tile0) / kStage) & 1;
        const bool more = stage + kStage < w.tile1;
        if (more) stage_dma(stage + kStage, buf ^ 1, stage + kStage < tile_e);
        const unsigned char* sb = smem + buf * kStage * kLdsTile;
#pragma unroll
        for (int ts = 0; ts < kStage; ++ts)
            if (kStage == 1 || stage + ts < w.tile1) tile_early(sb + ts * kLdsTile, stage + ts);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA into the next buffer landed
        __syncthreads();
    }
    for (; stage < w.tile1; stage += kStage) {
        const int buf = ((stage - w.tile0) / kStage) & 1;
        const bool more = stage + kStage < w.tile1;
        if (more) stage_dma(stage + kStage, buf ^ 1, false);
        const unsigned char* sb = smem + buf * kStage * kLdsTile;
        flush_deferred();  // the previous stage's last half tile (waves 4-7 with MIM_KNN_STAGGER)
        auto refresh = [&]() {  // thresholds from the partner lane's current m1, m2 (every tile: slower, r03bd)
#pragma unroll
            for (int u = 0; u < QT; ++u) {
                const auto a = __builtin_amdgcn_permlane32_swap(st[u].m1, st[u].m1, false, false);
                const auto b = __builtin_amdgcn_permlane32_swap(st[u].m2, st[u].m2, false, false);
                o1c[u] = (tid & 32) ? (int)a[0] : (int)a[1];
                o2c[u] = (tid & 32) ? (int)b[0] : (int)b[1];
                T[u] = late_threshold(st[u], o1c[u], o2c[u]);
            }
        };
        refresh();
        // rolled by default (unrolling measured no faster; the late tile is ~3 KiB of code)
#pragma unroll MIM_KNN_LATE_UNROLL
        for (int ts = 0; ts < kStage; ++ts)
            if (kStage == 1 || stage + ts < w.tile1)
                tile_late(sb + ts * kLdsTile, stage + ts, stagger && (ts == kStage - 1 || stage + ts + 1 == w.tile1));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA into the next buffer landed
        __syncthreads();
    }
    flush_deferred();

    // ---- merge the two lane halves (disjoint train rows of the same query), keys ----
#pragma unroll
    for (int u = 0; u < QT; ++u) {
        LaneSel m = st[u];
        if (m.i1 != INT_MAX) m.i1 += 4 * h;
        if (m.i2 != INT_MAX) m.i2 += 4 * h;
        LaneSel o;
        o.m1 = __shfl_xor(m.m1, 32); o.m2 = __shfl_xor(m.m2, 32);
        o.i1 = __shfl_xor(m.i1, 32); o.i2 = __shfl_xor(m.i2, 32);
        m = sel_merge(m, o);
        const int q = qbase + 32 * u + r;
        if (h == 0 && q < nq) {
            // c(q), read here rather than held in a register for the whole sweep
            const int qq = ((const gint*)P->q.norm)[(size_t)(q >> 6) * kNormWords + 128 + (q & 63)];
            Top2 t;
            const int d1 = m.m1 + qq, d2 = m.m2 + qq;  // exact d^2 = D + c(q) (< 2^23)
            t.k1 = m.i1 == INT_MAX ? FLT_MAX : sqrtf((float)d1);
            t.k2 = m.i2 == INT_MAX ? FLT_MAX : sqrtf((float)d2);
            t.i1 = m.i1;
            t.i2 = m.i2;
            // d^2 >= 4e6: distinct integers may share a key (sqrt class), where the lower index
            // wins: rescan exactly.  Below, equal keys mean equal d^2, already in index order.
            if (t.i2 != INT_MAX && d2 >= 4000000) t.i2 = kRescan;
            parts[P->part_off + (long long)w.split * P->q_pad + q] = t;
        }
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
    for (int k = 0; k < kKnnBlockQ; k += 64) {
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
                                                       Top2* __restrict__ parts, int n_works) {
    __shared__ __attribute__((aligned(16))) float tl[kTileRows * kDim];
    // grid-stride over the work items: the grid is capped (knn_launch), since nearly every item is
    // integer-valued and exits at the flag test; one early-exit block per item (32 KiB of LDS, 128
    // query VGPRs) cost ~0.12 ms of dispatch per C3 batch
  for (int wi = blockIdx.x; wi < n_works; wi += gridDim.x) {
    const KnnWork w = works[wi];
    const ProbDev* P = probs + w.problem;
    if (!(*P->q.flags | *P->t.flags)) continue;  // integer-valued: exact MFMA kernel handles it (block-uniform)
    const int tid = threadIdx.x;
    const int nq = P->q.n, nt = P->t.n;
  for (int qo = 0; qo < kKnnBlockQ; qo += 256) {  // the work item's queries, 256 per pass
    const int q = w.q0 + qo + tid;
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
    __syncthreads();  // the next work item's first tile load overwrites tl
  }
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
// knnMatch rows alone (mim_knn2_l2 / mim_knn2_sets_dev): merge the train splits of every query of
// one problem, one thread per query over the whole grid (no ratio test, no compaction).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void knn_emit_kernel(const ProbDev* __restrict__ probs,
                                                      const Top2* __restrict__ parts,
                                                      int32_t* __restrict__ knn_idx, float* __restrict__ knn_dist) {
    const ProbDev* P = probs;
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= P->q.n) return;
    T2 m{FLT_MAX, INT_MAX, FLT_MAX, INT_MAX};
    for (int sp = 0; sp < P->nsplit; ++sp) {
        const Top2 t = parts[P->part_off + (long long)sp * P->q_pad + q];
        m = top2_merge(m, t.k1, t.i1);
        m = top2_merge(m, t.k2, t.i2);
    }
    reinterpret_cast<int2*>(knn_idx)[q] = make_int2(m.i1 == INT_MAX ? -1 : m.i1, m.i2 == INT_MAX ? -1 : m.i2);
    reinterpret_cast<float2*>(knn_dist)[q] = make_float2(m.k1, m.k2);
}

// ------------------------------------------------------------------------------------------------
// allUnfilteredScenePts of a batch (TestsDetector.cpp:87-94): for every accepted problem, the scene
// keypoints of its RANSAC inliers in mask order, divided by the problem's scale in float when it is
// not 1 (scalePoints, :48-55), at offs[i] (the host's prefix sum of the accepted problems' n_inl).
// One 256-thread block per problem; ordered compaction by wave ballots.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void inlier_gather_kernel(const ProbDev* __restrict__ probs,
                                                          const mim_result* __restrict__ res,
                                                          const int32_t* __restrict__ good_t,
                                                          const uint8_t* __restrict__ masks,
                                                          const long long* __restrict__ offs,
                                                          const float* __restrict__ scales,
                                                          float2* __restrict__ out) {
    __shared__ int wsum[4];
    const int i = blockIdx.x;
    if (res[i].status != MIM_ACCEPTED) return;  // block-uniform
    const ProbDev* P = probs + i;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int ng = res[i].n_good;
    const float s = scales ? scales[i] : 1.0f;
    long long o = offs[i];
    for (int base = 0; base < ng; base += 256) {
        const int k = base + tid;
        const bool in = k < ng && masks[P->good_off + k] != 0;
        const unsigned long long bal = __ballot(in);
        const int within = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        if (lane == 0) wsum[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, all = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            before += w < wave ? wsum[w] : 0;
            all += wsum[w];
        }
        if (in) {
            float2 p = P->t.kp[good_t[P->good_off + k]];
            if (s != 1.0f) {  // pt.x /= scale; pt.y /= scale (IEEE float division)
                p.x = __fdiv_rn(p.x, s);
                p.y = __fdiv_rn(p.y, s);
            }
            out[o + before + within] = p;
        }
        o += all;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// host-side launchers (called from api.cpp)
// ------------------------------------------------------------------------------------------------
void launch_prep_batch(const PrepJob* jobs, int njobs, int total_tiles, hipStream_t st) {
    if (njobs > 0 && total_tiles > 0) prep_batch_kernel<<<total_tiles, 256, 0, st>>>(jobs, njobs);
}

// Both kernels are enqueued; each block reads its problem's integrality flags (set by prep on the
// device) and only the matching kernel does the work, so no host round trip is needed.
int knn_blocks_per_cu() {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, knn2_i8_kernel, kThreads, 0) != hipSuccess) nb = 1;
    return nb;
}

void launch_knn(const ProbDev* probs, const KnnWork* works, int n_works, const int* seg_start, int n_blocks,
                Top2* parts, int* dyn_ctr, hipStream_t st) {
    if (n_works <= 0) return;
    if (dyn_ctr) (void)hipMemsetAsync(dyn_ctr, 0, 8 * sizeof(int), st);
    knn2_i8_kernel<<<n_blocks, kThreads, 0, st>>>(probs, works, seg_start, parts, dyn_ctr);
    knn2_rescan_kernel<<<n_works, 256, 0, st>>>(probs, works, parts);
    knn2_f32_kernel<<<std::min(n_works, 2048), 256, 0, st>>>(probs, works, parts, n_works);
}

void launch_inlier_gather(const ProbDev* probs, int n, const mim_result* res, const int32_t* good_t,
                          const uint8_t* masks, const long long* offs, const float* scales, float2* out, hipStream_t st) {
    if (n > 0) inlier_gather_kernel<<<n, 256, 0, st>>>(probs, res, good_t, masks, offs, scales, out);
}

void launch_knn_emit(const ProbDev* probs, int nq, const Top2* parts, int32_t* knn_idx, float* knn_dist,
                     hipStream_t st) {
    if (nq > 0) knn_emit_kernel<<<(nq + 255) / 256, 256, 0, st>>>(probs, parts, knn_idx, knn_dist);
}

void launch_ratio(const ProbDev* probs, int n_probs, const Top2* parts, float ratio, int32_t* good_q,
                  int32_t* good_t, float4* pts, int* n_good, int32_t* knn_idx, float* knn_dist,
                  hipStream_t st) {
    if (n_probs > 0)
        ratio_compact_kernel<<<n_probs, 1024, 0, st>>>(probs, parts, ratio, good_q, good_t, pts, n_good,
                                                       knn_idx, knn_dist);
}

}  // namespace mim
