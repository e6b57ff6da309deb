// ransac.hip — cv::findHomography(obj, scene, RANSAC, 5.0, mask) on gfx950, batched over problems.
//
// Replaces /root/reference/src/TestsDetector.cpp:78 (+ the gates :74,:79-84) — OpenCV
// calib3d/src/fundam.cpp (findHomography, HomographyEstimatorCallback, HomographyRefineCallback),
// calib3d/src/ptsetreg.cpp (RANSACPointSetRegistrator::run/getSubset/findInliers,
// RANSACUpdateNumIters), calib3d/src/levmarq.cpp (LMSolverImpl), core/src/lapack.cpp (Jacobi).
//
// The sequential RANSAC loop is re-cut into data-parallel stages with identical results
// (DESIGN.md section 4):
//   attempt  every getSubset attempt outcome of a window of stream positions, GPU-wide;
//   irr/chain  the chain of attempt start positions walked over its repeated-index redraws only,
//           passing attempts ranked and written in parallel (sample: exact attempt-by-attempt walker
//           for whatever the chain kernel leaves);
//   bound    closed-form homography per iteration + lower/upper bounds of its inlier count;
//   cand/exact/replay  only iterations that can be a new best are solved with OpenCV's exact
//           arithmetic (normalized DLT + JacobiImpl_ on a 16-lane group, bit-identical), counted,
//           and replayed in iteration order with RANSACUpdateNumIters;
//   refine   one block per problem: best mask, inlier compaction, refit DLT and 10-iteration
//           Levenberg-Marquardt in fp64 (block reductions), determinant and gates.
// Reference mode (MIM_RANSAC_EXACT=1): hypo/score/select evaluate every iteration exactly.
#include <float.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/mim.h"
#include "mim_debug.h"
#include "mim_internal.h"

namespace mim {

// ------------------------------------------------------------------------------------------------
// shared fp64 helpers (core/src/lapack.cpp)
// ------------------------------------------------------------------------------------------------
// hypot<double> of core/src/lapack.cpp in select form (same operations, no divergent branches):
//   a > b ? a*sqrt(1+(b/a)^2) : (b > 0 ? b*sqrt(1+(a/b)^2) : 0)
__device__ __forceinline__ double d_hypot(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    const bool ab = a > b;
    const double big = ab ? a : b, sm = ab ? b : a;
    const double r = sm / big;
    const double res = big * sqrt(1 + r * r);
    return (ab || b > 0) ? res : 0.0;
}

// packed upper-triangle index of (i, j), i < j, for an n x n symmetric matrix
// (the masks are exact for 0 <= i < n <= 16 and let the product select the full-rate 24-bit multiply;
// __umul24 compiled to the quarter-rate v_mul_lo_u32 in the Jacobi rotation)
template <int n> __device__ __forceinline__ int pk(int i, int j) {
    static_assert(n <= 16, "packed index masks");
    return (int)(((unsigned)(i & 15) * (unsigned)((2 * n - 1 - i) & 31)) >> 1) + (j - i - 1);
}

template <int n> __device__ __forceinline__ int pk_any(int a, int b) {  // (min, max) of two distinct indices
    const int i = min(a, b), j = max(a, b);
    return pk<n>(i, j);
}

// JacobiImpl_<double> (core/src/lapack.cpp), bit-identical arithmetic, restructured for a GPU lane:
// the matrix lives in LDS with element e at base[e * S] (S = 64: one lane's private column in an
// [element][lane] interleave, conflict-free for any per-lane index; S = 1 for single-thread use),
// indR/indC live in registers, and every loop has static bounds so all loads of a phase issue
// back to back (two LDS round trips per rotation instead of one per element).  OpenCV's cached
// row/column maxima are refreshed only for rows k and l, exactly like the reference.
//   A: packed strict upper triangle; W: diagonal on entry (unsorted eigenvalues on exit);
//   V: n x n rows = eigenvectors (unsorted).  Outputs Ws = eigenvalues in OpenCV's descending
//   selection-sort order and perm[i] = row of V holding the i-th sorted eigenvector.
template <int n, int S>
__device__ void jacobi_fast(double* __restrict__ A, double* __restrict__ W, double* __restrict__ V,
                            double (&Ws)[n], int (&perm)[n]) {
#define AU(i, j) A[pk<n>((i), (j)) * S]
    // spare slot after the matrix state (A | W | V | trash) absorbing predicated-off stores
    const int trash = n * (n - 1) / 2 + n + n * n;
    const double eps = DBL_EPSILON;
#pragma unroll
    for (int i = 0; i < n; i++)
#pragma unroll
        for (int j = 0; j < n; j++) V[(i * n + j) * S] = i == j ? 1.0 : 0.0;
    int indR[n], indC[n];
#pragma unroll
    for (int k = 0; k < n; k++) {
        indR[k] = 0;
        indC[k] = 0;
        if (k < n - 1) {
            int m = k + 1;
            double mv = fabs(AU(k, k + 1));
#pragma unroll
            for (int i = k + 2; i < n; i++) {
                const double val = fabs(AU(k, i));
                if (mv < val) mv = val, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            int m = 0;
            double mv = fabs(AU(0, k));
#pragma unroll
            for (int i = 1; i < k; i++) {
                const double val = fabs(AU(i, k));
                if (mv < val) mv = val, m = i;
            }
            indC[k] = m;
        }
    }
    for (int iters = 0; iters < n * n * 30; iters++) {
        double vr[n], vc[n];
#pragma unroll
        for (int i = 0; i < n - 1; i++) vr[i] = A[(pk<n>(i, i + 1) + indR[i] - i - 1) * S];
#pragma unroll
        for (int i = 1; i < n; i++) vc[i] = A[pk_any<n>(indC[i], i) * S];
        int k = 0, l = indR[0];
        double mv = fabs(vr[0]), p = vr[0];
#pragma unroll
        for (int i = 1; i < n - 1; i++) {  // select form of `if (mv < val) mv = val, k = i`
            const double val = fabs(vr[i]);
            const bool u = mv < val;
            mv = u ? val : mv;
            k = u ? i : k;
            l = u ? indR[i] : l;
            p = u ? vr[i] : p;
        }
#pragma unroll
        for (int i = 1; i < n; i++) {
            const double val = fabs(vc[i]);
            const bool u = mv < val;
            mv = u ? val : mv;
            k = u ? indC[i] : k;
            l = u ? i : l;
            p = u ? vc[i] : p;
        }
        if (fabs(p) <= eps) break;
        // issue every load of this rotation before the dependent arithmetic
        const double wk = W[k * S], wl = W[l * S];
        double a0[n], b0[n], vk[n], vl[n];
#pragma unroll
        for (int i = 0; i < n; i++) {
            const bool vi = i != k && i != l;
            a0[i] = A[(vi ? pk_any<n>(i, k) : 0) * S];
            b0[i] = A[(vi ? pk_any<n>(i, l) : 0) * S];
            vk[i] = V[(k * n + i) * S];
            vl[i] = V[(l * n + i) * S];
        }
        const double y = (wl - wk) * 0.5;
        double t = fabs(y) + d_hypot(p, y);
        const double q = fabs(p) / t;  // hypot(p, t) = t sqrt(1 + q^2) and p / t = ±q (jacobi_group)
        double s = t * sqrt(1 + q * q);
        const double c = t / s;
        s = p / s;
        t = copysign(q, p) * p;
        s = y < 0 ? -s : s;
        t = y < 0 ? -t : t;
        AU(k, l) = 0;
        W[k * S] = wk - t;
        W[l * S] = wl + t;
        double rk[n], rl[n];  // rows k and l after the rotation (column entries by symmetry)
#pragma unroll
        for (int i = 0; i < n; i++) {
            const bool vi = i != k && i != l;
            const double na = a0[i] * c - b0[i] * s;
            const double nb = a0[i] * s + b0[i] * c;
            // unconditional stores (a dropped pair goes to the spare slot `trash`): no branches
            A[(vi ? pk_any<n>(i, k) : trash) * S] = na;
            A[(vi ? pk_any<n>(i, l) : trash) * S] = nb;
            rk[i] = vi ? na : 0.0;
            rl[i] = vi ? nb : 0.0;
            V[(k * n + i) * S] = vk[i] * c - vl[i] * s;
            V[(l * n + i) * S] = vk[i] * s + vl[i] * c;
        }
        // refresh the cached maxima of rows/columns k and l (the only ones OpenCV refreshes)
        int rkR = -1, rkC = -1, rlR = -1, rlC = -1;
        double bkR = 0, bkC = 0, blR = 0, blC = 0;
#pragma unroll
        for (int m = 0; m < n; m++) {
            const double ak = fabs(rk[m]), al = fabs(rl[m]);
            const bool u1 = m > k && (rkR < 0 || bkR < ak);
            const bool u2 = m < k && (rkC < 0 || bkC < ak);
            const bool u3 = m > l && (rlR < 0 || blR < al);
            const bool u4 = m < l && (rlC < 0 || blC < al);
            bkR = u1 ? ak : bkR; rkR = u1 ? m : rkR;
            bkC = u2 ? ak : bkC; rkC = u2 ? m : rkC;
            blR = u3 ? al : blR; rlR = u3 ? m : rlR;
            blC = u4 ? al : blC; rlC = u4 ? m : rlC;
        }
#pragma unroll
        for (int i = 0; i < n; i++) {
            indR[i] = (i == k && i < n - 1) ? rkR : ((i == l && i < n - 1) ? rlR : indR[i]);
            indC[i] = (i == k && i > 0) ? rkC : ((i == l && i > 0) ? rlC : indC[i]);
        }
    }
    // selection sort to descending order (OpenCV swaps V rows; here the permutation is tracked)
#pragma unroll
    for (int i = 0; i < n; i++) {
        Ws[i] = W[i * S];
        perm[i] = i;
    }
#pragma unroll
    for (int k = 0; k < n - 1; k++) {
        int m = k;
        double wm = Ws[k];
#pragma unroll
        for (int i = k + 1; i < n; i++)
            if (wm < Ws[i]) wm = Ws[i], m = i;
        const double wk = Ws[k];
        const int pkk = perm[k];
        int pm = perm[k];
#pragma unroll
        for (int i = k + 1; i < n; i++) pm = i == m ? perm[i] : pm;
#pragma unroll
        for (int i = k + 1; i < n; i++) {
            if (i == m) {
                Ws[i] = wk;
                perm[i] = pkk;
            }
        }
        Ws[k] = wm;
        perm[k] = pm;
    }
#undef AU
}

// storage footprint of jacobi_fast<9>: 36 + 9 + 81 doubles
constexpr int kJ9D = 36 + 9 + 81 + 1;  // + the trash slot

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
__device__ void dlt_finish(const double* lt, double* D, const double* invHnorm, const double* Hnorm2, double* H) {
    double* A = D;
    double* W = D + 36 * S;
    double* V = D + 45 * S;
    int e = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
        for (int k = j; k < 9; ++k, ++e) {
            if (k == j) W[j * S] = lt[e];
            else A[pk<9>(j, k) * S] = lt[e];
        }
    double Ws[9];
    int perm[9];
    jacobi_fast<9, S>(A, W, V, Ws, perm);
    double H0[9], Ht[9];
    const int r = perm[8];  // eigenvector of the smallest eigenvalue (V[8] after OpenCV's sort)
#pragma unroll
    for (int i = 0; i < 9; ++i) H0[i] = V[(r * 9 + i) * S];
    mat3_mul(invHnorm, H0, Ht);
    mat3_mul(Ht, Hnorm2, H0);
    const double sc = 1. / H0[8];  // _H0.convertTo(_model, type, 1./H0(2,2))
#pragma unroll
    for (int i = 0; i < 9; ++i) H[i] = H0[i] * sc;
}

// runKernel on the 4 points of a minimal sample (M = object, m = scene), one lane.
template <int S>
__device__ int run_kernel4(const float* M, const float* m, double* D, double* H) {
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
    dlt_finish<S>(lt, D, invHnorm, Hnorm2, H);
    return 1;
}

// ------------------------------------------------------------------------------------------------
// JacobiImpl_<double> for one 9x9 matrix on a group of 16 lanes (bit-identical to jacobi_fast).
// One rotation touches 16 disjoint pairs — rows k, l of V (9 pairs) and the 7 (A(i,k), A(i,l)),
// i != k, l — so slot j of the group rotates pair j.  The pivot search (OpenCV's first maximum over
// the 16 cached row/column candidates) and the refresh of the caches of rows/columns k and l are
// group reductions over DPP row permutations: no serial 16-step scans, no barriers.  State lives
// in LDS (per group: A packed upper | W | V); lane j < 9 keeps indR[j], indC[j] in registers.
// ------------------------------------------------------------------------------------------------
constexpr int kJ9G = 36 + 9 + 81;  // doubles of LDS state per group

__device__ __forceinline__ int dpp_row(int v, int ctrl) {
    // every lane of the row is written (full masks, in-row permutations), so no "old" value is needed:
    // mov_dpp with bound_ctrl avoids materialising one per DPP move
    switch (ctrl) {  // constant after inlining
        case 0: return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);   // quad_perm 1,0,3,2
        case 1: return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);   // quad_perm 2,3,0,1
        case 2: return __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true);  // row_half_mirror
        default: return __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true); // row_mirror
    }
}

__device__ __forceinline__ double dpp_row_d(double v, int ctrl) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_row((int)(unsigned)b, ctrl), hi = dpp_row((int)(b >> 32), ctrl);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// lanes of this lane's 16-lane group in a wave ballot, as bits 0..15
__device__ __forceinline__ unsigned group_bits(unsigned long long m) {
    return (unsigned)(m >> (threadIdx.x & 48)) & 0xFFFFu;
}

// Max over the 16 lanes of a DPP row of R values that are each >= +0 or -1.0 (every lane receives
// the R maxima), in two 32-bit passes: the signed max of the high words (doubles >= +0 order as their
// high words, -1.0's is negative), then the unsigned max of the low words over the lanes holding
// that high word.  The result is the bits of the maximal element, as fmax gives; the 32-bit maxes
// take the DPP operand directly (v_max_i32_dpp: no 64-bit moves, no fmax canonicalisation) and the
// R reductions are interleaved step by step, so one's DPP read hazard is covered by the others.
template <int R>
__device__ __forceinline__ void row_max_nn(double (&v)[R]) {
    int hi[R];
    unsigned lo[R];
#pragma unroll
    for (int j = 0; j < R; ++j) hi[j] = (int)(__double_as_longlong(v[j]) >> 32);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < R; ++j) hi[j] = max(hi[j], dpp_row(hi[j], c));
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const long long b = __double_as_longlong(v[j]);
        lo[j] = (int)(b >> 32) == hi[j] ? (unsigned)b : 0u;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < R; ++j) lo[j] = max(lo[j], (unsigned)dpp_row((int)lo[j], c));
#pragma unroll
    for (int j = 0; j < R; ++j)
        v[j] = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi[j] << 32) | lo[j]));
}

// First maximum of |A(idx, i)| over the slots' candidate indices (slots 9..15 carry the rotated
// values, in increasing index order) plus, optionally, a zero entry at index `zi` (-1: none), for the
// four caches of rows/columns k and l at once.  The first maximal slot's index is the smallest index
// among the slots holding the maximum: each slot's own index (the (slot-9)-th index outside {k, l},
// increasing with the slot) min-reduced over the row, the four reductions interleaved step by step
// (round 5: a ballot and find-first-set per cache, four dependent chains one after another).
template <int n>
__device__ __forceinline__ void refresh_argmax4(const double (&val)[4], const bool (&cand)[4], int k, int l,
                                                const int (&zi)[4], int (&first)[4]) {
    double mx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) mx[j] = cand[j] ? val[j] : -1.0;
    row_max_nn<4>(mx);
    int im = (int)(threadIdx.x & 15) - n;
    im += im >= k;
    im += im >= l;
    int f[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) f[j] = (cand[j] && val[j] == mx[j]) ? im : INT_MAX;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = min(f[j], dpp_row(f[j], c));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int fj = f[j];
        if (zi[j] >= 0 && !(mx[j] > 0.0)) fj = min(fj, zi[j]);
        first[j] = fj;
    }
}

// A/W/V: this group's LDS state (A packed strict upper, W diagonal) written by the caller.
// n = 9 (runKernel's LtL) uses all 16 slots (9 V pairs + 7 A pairs), n = 8 (LMSolverImpl's normal
// matrix) 14 of them.  Outputs, in every slot, Ws = the eigenvalues in OpenCV's descending
// selection-sort order and perm[i] = the row of V holding the i-th of them.
template <int n>
__device__ __forceinline__ void jacobi_group(double* __restrict__ A, double* __restrict__ W, double* __restrict__ V,
                                             double (&Ws)[n], int (&perm)[n]) {
    static_assert(2 * n - 2 <= 16, "one rotation's pairs must fit the 16 slots");
    const int slot = threadIdx.x & 15;
    const double eps = DBL_EPSILON;
    for (int e = slot; e < n * n; e += 16) V[e] = (e % (n + 1) == 0) ? 1.0 : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int indR = 0, indC = 0;
    if (slot < n - 1) {
        int m = slot + 1;
        double mv = fabs(A[pk<n>(slot, slot + 1)]);
        for (int i = slot + 2; i < n; i++) {
            const double val = fabs(A[pk<n>(slot, i)]);
            if (mv < val) mv = val, m = i;
        }
        indR = m;
    }
    if (slot > 0 && slot < n) {
        int m = 0;
        double mv = fabs(A[pk<n>(0, slot)]);
        for (int i = 1; i < slot; i++) {
            const double val = fabs(A[pk<n>(i, slot)]);
            if (mv < val) mv = val, m = i;
        }
        indC = m;
    }
    for (int iters = 0; iters < n * n * 30; iters++) {
        // ---- pivot: OpenCV scans rows 0..7 (A(i, indR[i])) then columns 1..8 (A(indC[i], i)) and
        // keeps the first strict maximum; slot i holds both of its candidates (row first) ----
        // key = pos << 20 | sign(p) << 16 | l << 8 | k: positions are distinct over the valid slots, so
        // comparing keys compares positions.  The first maximum of |p| in position order as three 32-bit
        // DPP passes (row_max_nn's two for |p|, then the smallest key among the lanes holding it); the
        // winner's p is its |p| bits with the sign bit from the key.
        // branch-free: every slot reads two entries (slots without that candidate read entry 0)
        const bool hr = slot < n - 1, hc = slot > 0 && slot < n;
        const double ar = A[hr ? pk<n>(slot, indR) : 0], ac = A[hc ? pk<n>(indC, slot) : 0];
        const double vr = hr ? ar : 0.0, vc = hc ? ac : 0.0;
        const bool row = hr && (slot == 0 || fabs(vr) >= fabs(vc));
        const double p0 = row ? vr : vc;
        const int key0 = row ? (slot << 20 | indR << 8 | slot) : ((slot + n - 2) << 20 | slot << 8 | indC);
        const double pv = slot < n ? p0 : 0.0;
        const unsigned long long pb = (unsigned long long)__double_as_longlong(pv);
        const int key = (slot < n ? key0 : 99 << 20) | (int)(pb >> 63) << 16;
        double pm[1] = {fabs(pv)};
        row_max_nn<1>(pm);
        int kc = fabs(pv) == pm[0] ? key : INT_MAX;
#pragma unroll
        for (int c = 0; c < 4; ++c) kc = min(kc, dpp_row(kc, c));
        const double p = (kc >> 16) & 1 ? -pm[0] : pm[0];
        if (fabs(p) <= eps) break;
        const int k = kc & 255, l = (kc >> 8) & 255;  // k < l
        // ---- the pair of this slot ----
        int im = slot - n;  // slots 9..15: the (slot-9)-th index outside {k, l}
        im += im >= k;
        im += im >= l;
        const bool vslot = slot < n;
        const bool idle = slot >= 2 * n - 2;  // n = 8: slots 14, 15
        // both forms computed and selected (no divergent branch around the packed indices); im < k <
        // l is the common case of the min/max
        const int pak = pk<n>(min(im, k), max(im, k)), pal = pk<n>(min(im, l), max(im, l));
        const int ia = vslot ? k * n + slot : (idle ? 0 : pak);
        const int ib = vslot ? l * n + slot : (idle ? 0 : pal);
        double* base = vslot ? V : A;
        const double a0 = base[ia], b0 = base[ib];
        const double wk = W[k], wl = W[l];
        const double y = (wl - wk) * 0.5;
        double t = fabs(y) + d_hypot(p, y);
        // hypot(p, t) with t >= hypot(p, y) >= |p| > 0: its larger operand is t and its quotient |p| / t
        // is p / t up to the sign (IEEE division is sign-symmetric), which OpenCV's update of W divides
        // again: the same bits with one fp64 division less per rotation
        const double q = fabs(p) / t;
        double s = t * sqrt(1 + q * q);
        const double c = t / s;
        s = p / s;
        t = copysign(q, p) * p;
        s = y < 0 ? -s : s;
        t = y < 0 ? -t : t;
        const double na = a0 * c - b0 * s;
        const double nb = a0 * s + b0 * c;
        if (!idle) {
            base[ia] = na;
            base[ib] = nb;
        }
        if (slot == 0) {
            A[pk<n>(k, l)] = 0;
            W[k] = wk - t;
            W[l] = wl + t;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- refresh the cached maxima of rows/columns k and l (row k: A(k,i) = na of the A
        // slots, plus A(k,l) = 0; row l: nb, plus A(l,k) = 0) ----
        const bool aslot = !vslot && !idle;
        const double va = fabs(na), vb = fabs(nb);
        const double rv[4] = {va, va, vb, vb};
        const bool rc[4] = {aslot && im > k, aslot && im < k, aslot && im > l, aslot && im < l};
        const int rz[4] = {l, -1, -1, k};
        int rf[4];
        refresh_argmax4<n>(rv, rc, k, l, rz, rf);
        const int rk = rf[0], ck = rf[1], rl = rf[2], cl = rf[3];
        if (slot == k) {
            if (k < n - 1) indR = rk;
            if (k > 0) indC = ck;
        }
        if (slot == l) {
            if (l < n - 1) indR = rl;
            if (l > 0) indC = cl;
        }
    }
    // ---- OpenCV's selection sort (descending), tracked as a permutation ----
#pragma unroll
    for (int i = 0; i < n; i++) {
        Ws[i] = W[i];
        perm[i] = i;
    }
#pragma unroll
    for (int k = 0; k < n - 1; k++) {
        int m = k;
        double wm = Ws[k];
#pragma unroll
        for (int i = k + 1; i < n; i++)
            if (wm < Ws[i]) wm = Ws[i], m = i;
        const double wk = Ws[k];
        const int pkk = perm[k];
        int pm = perm[k];
#pragma unroll
        for (int i = k + 1; i < n; i++) pm = i == m ? perm[i] : pm;
#pragma unroll
        for (int i = k + 1; i < n; i++) {
            if (i == m) {
                Ws[i] = wk;
                perm[i] = pkk;
            }
        }
        Ws[k] = wm;
        perm[k] = pm;
    }
}

// runKernel's 9x9: the row of V holding the eigenvector of the smallest eigenvalue
__device__ __forceinline__ int jacobi9_group(double* __restrict__ A, double* __restrict__ W, double* __restrict__ V) {
    double Ws[9];
    int perm[9];
    jacobi_group<9>(A, W, V, Ws, perm);
    return perm[8];
}

// normalized-DLT accumulation of runKernel for `count` points, entry e of LtL (upper incl. the
// diagonal, row-major) computed by slot e % 16: every entry is the same sum in the same order as
// run_kernel4 / the oracle (points in order, Lx then Ly).
__device__ __forceinline__ void dlt_entries_group(const float* M, const float* m, int count, double cmx, double cmy,
                                                  double cMx, double cMy, double smx, double smy, double sMx,
                                                  double sMy, double* __restrict__ A, double* __restrict__ W) {
    const int slot = threadIdx.x & 15;
    for (int e = slot; e < 45; e += 16) {
        int j = 0, r = e;
        while (r >= 9 - j) { r -= 9 - j; ++j; }
        const int kk = j + r;
        double acc = 0;
        for (int i = 0; i < count; i++) {
            const double x = (m[2 * i] - cmx) * smx, y = (m[2 * i + 1] - cmy) * smy;
            const double X = (M[2 * i] - cMx) * sMx, Y = (M[2 * i + 1] - cMy) * sMy;
            const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
            const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
            acc += Lx[j] * Lx[kk] + Ly[j] * Ly[kk];
        }
        if (kk == j) W[j] = acc;
        else A[pk<9>(j, kk)] = acc;
    }
}

// runKernel on the 4 points of a minimal sample, by a 16-lane group (bit-identical to run_kernel4).
// D: the group's kJ9G doubles of LDS.  Every slot returns the result and H.
__device__ int run_kernel4_group(const float* M, const float* m, double* D, double* H) {
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
    double* A = D;
    double* W = D + 36;
    double* V = D + 45;
    dlt_entries_group(M, m, count, cmx, cmy, cMx, cMy, smx, smy, sMx, sMy, A, W);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int r = jacobi9_group(A, W, V);
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double H0[9], Ht[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) H0[i] = V[r * 9 + i];
    mat3_mul(invHnorm, H0, Ht);
    mat3_mul(Ht, Hnorm2, H0);
    const double sc = 1. / H0[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) H[i] = H0[i] * sc;
    return 1;
}

// dlt_finish by a 16-lane group: lt (upper incl. diagonal, every slot holds it) -> H
__device__ void dlt_finish_group(const double* lt, double* D, const double* invHnorm, const double* Hnorm2,
                                 double* H) {
    const int slot = threadIdx.x & 15;
    double* A = D;
    double* W = D + 36;
    double* V = D + 45;
    for (int e = slot; e < 45; e += 16) {
        int j = 0, r = e;
        while (r >= 9 - j) { r -= 9 - j; ++j; }
        const int kk = j + r;
        double v = 0;
#pragma unroll
        for (int q = 0; q < 45; ++q) v = q == e ? lt[q] : v;
        if (kk == j) W[j] = v;
        else A[pk<9>(j, kk)] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int r = jacobi9_group(A, W, V);
    double H0[9], Ht[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) H0[i] = V[r * 9 + i];
    mat3_mul(invHnorm, H0, Ht);
    mat3_mul(Ht, Hnorm2, H0);
    const double sc = 1. / H0[8];
#pragma unroll
    for (int i = 0; i < 9; ++i) H[i] = H0[i] * sc;
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

// checkSubset decided in fp32 where fp32 cannot disagree with the fp64 reference, else fp64 (round 6
// form: the orientation determinants reuse the collinearity test's cross products).
// Per point set, with the deltas d_j = p_j - p_3 in float (as haveCollinearPoints subtracts) and
// m >= every |delta| component:
// Collinearity: c_kj = fma(dx_k, dy_j, -rn(dy_k dx_j)) is the fp64 test's cross product X' = dx_k dy_j -
//   dy_k dx_j within 2^-24 (|c| + m^2); the fp64 right side is at most 2^-23 S (1 + 2^-51), S <= 4 m; so
//   |c| > 2^-21 m (m + 4) (the round-5 bound, proof there) gives "clearly not collinear".
// Orientation: the same c_kj is orient(p_k, p_j, p_3) of the exact points within 5 2^-24 m^2 + 2^-24 |c|
//   (the deltas' roundings, 2 2^-24 relative on each product, plus the two roundings above), and
//   orient(p_0, p_1, p_2) = c_21 - c_20 + c_10 (the 4-point identity [012] = [123] - [023] + [013], two
//   float additions) within 25 2^-24 m^2 + 2^-24 |c_012|.  The fp64 reference det3xy (float inputs,
//   no FMA) is within ~60 2^-53 A^2 < 2^-44 A^2 of the exact value, A = max(|x_3|, |y_3|) + m >= every
//   coordinate.  So |c| > 2^-20 m (m + 4) + 2^-44 A^2 (the three triples with p_3) and |c_012| > 2^-18 m^2
//   + 2^-44 A^2 give the fp64 signs (each bound above the error with a factor >= 2.5 for the roundings
//   of the bounds themselves); a floor of 2^-100 keeps products out of the subnormal range, where the
//   relative error model fails.  "Not clear" (near-collinear or tiny sets, duplicated points) runs the
//   fp64 check_subset: same result as check_subset always.
__device__ __forceinline__ bool set_orient_fp32(const float* xy, float (&o)[4]) {
    float dx[3], dy[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        dx[j] = xy[2 * j] - xy[6];
        dy[j] = xy[2 * j + 1] - xy[7];
    }
    const float m = fmaxf(fmaxf(fmaxf(fabsf(dx[0]), fabsf(dx[1])), fabsf(dx[2])),
                          fmaxf(fmaxf(fabsf(dy[0]), fabsf(dy[1])), fabsf(dy[2])));
    const float A = fmaxf(fabsf(xy[6]), fabsf(xy[7])) + m;
    const float a2 = (A * A) * 0x1p-44f;
    const float c10 = fmaf(dx[0], dy[1], -(dy[0] * dx[1]));  // orient(p0, p1, p3): triple 3
    const float c20 = fmaf(dx[0], dy[2], -(dy[0] * dx[2]));  // orient(p0, p2, p3): triple 2
    const float c21 = fmaf(dx[1], dy[2], -(dy[1] * dx[2]));  // orient(p1, p2, p3): triple 1
    const float c012 = (c21 - c20) + c10;                     // orient(p0, p1, p2): triple 0
    const float thr = fmaxf(fmaf(m * (m + 4.f), 0x1p-20f, a2), 0x1p-100f);
    const float thr0 = fmaxf(fmaf(m * m, 0x1p-18f, a2), 0x1p-100f);
    o[0] = c012; o[1] = c21; o[2] = c20; o[3] = c10;
    return fminf(fminf(fabsf(c10), fabsf(c20)), fabsf(c21)) > thr && fabsf(c012) > thr0;
}

// the fp32 decision and whether it is the fp64 one (clear); !clear: check_subset decides
__device__ __forceinline__ bool check_subset_fp32(const float* s, const float* d, bool& clear_out) {
    float os[4], od[4];
    const bool cs = set_orient_fp32(s, os), cd = set_orient_fp32(d, od);
    clear_out = cs && cd;
    // checkSubset's count of triples whose orientations differ, 0 or 4 to pass: the four sign bits of
    // os ^ od all equal
    const unsigned x0 = __float_as_uint(os[0]) ^ __float_as_uint(od[0]);
    const unsigned x1 = __float_as_uint(os[1]) ^ __float_as_uint(od[1]);
    const unsigned x2 = __float_as_uint(os[2]) ^ __float_as_uint(od[2]);
    const unsigned x3 = __float_as_uint(os[3]) ^ __float_as_uint(od[3]);
    return (int)((x0 ^ x1) | (x0 ^ x2) | (x0 ^ x3)) >= 0;
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
// RNG::uniform(0, n) = next() % n by Barrett reduction with m = M >> 32 = floor(2^32 / n), where
// M = floor((2^64 - 1) / n) + 1 is the per-problem constant (RansacState::modM), 2 <= n < 2^32:
// m <= 2^32/n and m >= 2^32/n - 1, so q = mulhi(a, m) is the quotient or one less and a - q n lies
// in [0, 2n); one unsigned min folds it (two quarter-rate multiplies instead of Lemire's six).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned fastmod(unsigned a, unsigned long long M, unsigned d) {
    const unsigned q = __umulhi(a, (unsigned)(M >> 32));
    const unsigned r = a - q * d;
    return min(r, r - d);
}


// getSubset's draw loop for one attempt starting at stream position q: redraw while an index
// repeats.  Returns the number of draws consumed (0 if the stream ends first).
__device__ __forceinline__ int resolve_at(long long q, const uint32_t* __restrict__ stream, long long slen,
                                          unsigned N, unsigned long long M, int (&idx)[4]) {
    unsigned buf[8];
    long long bq = q, r = q;
#pragma unroll
    for (int k = 0; k < 8; ++k) buf[k] = stream[min(q + k, slen - 1)];  // unconditional: one latency
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // unrolled: idx stays in registers
        for (;;) {
            if (r >= slen) return 0;
            if (r >= bq + 8) {
#pragma unroll
                for (int k = 0; k < 8; ++k) buf[k] = stream[min(r + k, slen - 1)];
                bq = r;
            }
            unsigned raw = buf[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) raw = (r - bq) == k ? buf[k] : raw;
            ++r;
            const int v = (int)fastmod(raw, M, N);
            bool dup = false;
#pragma unroll
            for (int j = 0; j < i; ++j) dup |= idx[j] == v;
            if (!dup) {
                idx[i] = v;
                break;
            }
        }
    }
    return (int)(r - q);
}

// A sample is stored as (q, -1, 0, 0) when its 4 draws are stream[q..q+3] (no repeat), as
// (q, -2, 0, 0) when getSubset redrew repeated indices starting at q, or as the 4 indices.
__device__ __forceinline__ int4 decode_sample(int4 s, const uint32_t* __restrict__ stream, unsigned N,
                                              unsigned long long M) {
    if (s.y >= 0) return s;
    const long long q = s.x;
    if (s.y == -1)
        return make_int4((int)fastmod(stream[q], M, N), (int)fastmod(stream[q + 1], M, N),
                         (int)fastmod(stream[q + 2], M, N), (int)fastmod(stream[q + 3], M, N));
    int idx[4] = {0, 0, 0, 0};
    resolve_at(q, stream, 1LL << 62, N, M, idx);  // the walker already checked the stream bound
    return make_int4(idx[0], idx[1], idx[2], idx[3]);
}

// The sampler kernels (count, sample) and the selection kernels (replay) may run concurrently on
// two streams (the next chunk's getSubset replay beside this chunk's selection): each stores only
// the fields it owns.  Reads of the other group's fields may see either value; see DESIGN.md
// "Sampler stream" for why every outcome is the same.
__device__ __forceinline__ void store_sampler_state(RansacState* d, const RansacState& S) {
    d->stream_pos = S.stream_pos;
    d->produced = S.produced;
    d->fail_iter = S.fail_iter;
    d->fail_run = S.fail_run;
    d->win_base = S.win_base;
    d->win_len = S.win_len;
}
__device__ __forceinline__ void store_select_state(RansacState* d, const RansacState& S) {
    d->max_good = S.max_good;
    d->best_iter = S.best_iter;
    d->niters = S.niters;
    d->next_iter = S.next_iter;
    d->done = S.done;
}

// ------------------------------------------------------------------------------------------------
// init: per-problem RANSAC state from the ratio-test survivors
// ------------------------------------------------------------------------------------------------
__global__ void ransac_init_kernel(RansacState* __restrict__ st, const int* __restrict__ n_good, int n_probs,
                                   int max_iters, int min_good, double* __restrict__ best_h) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_probs) return;
    RansacState S{};
    S.n = n_good[p];
    S.modM = S.n > 0 ? (~0ull / (unsigned long long)S.n + 1) : 0;
    S.active = (S.n >= min_good && S.n > 4) ? 1 : 0;  // n == 4: direct runKernel, no RANSAC
    S.niters = max(max_iters, 1);
    S.fail_iter = -1;
    S.best_iter = -1;
    st[p] = S;
    best_h[(long long)p * 9 + 8] = 0.0;  // "not computed" until an exact pass stores bestModel
}

// ------------------------------------------------------------------------------------------------
// attempt: the draws a getSubset attempt that starts at stream position q consumes, for every q of a
// window ahead of each problem's current position — fully parallel over the GPU (one flag byte per
// position: kPassUnknown | (draws - 4) << 1, or kAttemptSerial).  The chain kernels then walk the
// attempt start positions and ransac_check_kernel evaluates checkSubset for the chain's attempts.
// attempts precomputed ahead of the walker: the expected draws of the remaining iterations of the
// chunk (draws per iteration measured so far, 28 before any) + 6 % (25 % unmeasured) + 4096, capped by the buffer
// problems with fewer points are replayed by ransac_small_kernel from the stream alone (no window)
constexpr int kSmallMaxN = 128;

__device__ __forceinline__ int window_len(const RansacState& S, int c1, int wcap) {
    const int need = min(c1, S.niters) - S.produced;
    const double rate = S.produced > 0 ? (double)S.stream_pos / S.produced : 28.0;
    // measured rate: the draws of ~46k iterations vary by < 0.5 % (1 sigma), 6 % + 4096 covers them
    const long long w = (long long)((double)need * rate * (S.produced > 0 ? 1.06 : 1.25)) + 4096;
    return (int)min((long long)wcap, w) & ~63;  // whole 16-byte flag vectors and 32-bit pass words
}

// Outcome of the getSubset attempt whose draws start at q, as one byte: bit 0 = checkSubset
// passes, bits 1..6 = draws consumed - 4 (repeated indices redrawn); 0xFF = the walker must resolve
// it itself (RNG stream end, or > 67 draws).
constexpr int kAttemptSerial = 0xFF;
__device__ __forceinline__ int attempt_flag(long long q, const uint32_t* __restrict__ stream, long long slen,
                                            unsigned N, unsigned long long M, const float4* __restrict__ P) {
    if (q + 4 > slen) return kAttemptSerial;
    int idx[4] = {(int)fastmod(stream[q], M, N), (int)fastmod(stream[q + 1], M, N),
                  (int)fastmod(stream[q + 2], M, N), (int)fastmod(stream[q + 3], M, N)};
    int len = 4;
    if (idx[1] == idx[0] || idx[2] == idx[0] || idx[2] == idx[1] || idx[3] == idx[0] || idx[3] == idx[1] ||
        idx[3] == idx[2]) {
        len = resolve_at(q, stream, slen, N, M, idx);
        if (len == 0 || len > 67) return kAttemptSerial;
    }
    const float4 a = P[idx[0]], b = P[idx[1]], c = P[idx[2]], d = P[idx[3]];
    const float s4[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
    const float t4[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
    return ((len - 4) << 1) | (check_subset(s4, t4) ? 1 : 0);
}

// The redraw length of the attempt at q as a flag with the pass bit unknown (what the attempt kernel
// records), for positions past the precomputed window
__device__ __forceinline__ int length_flag(long long q, const uint32_t* __restrict__ stream, long long slen,
                                           unsigned N, unsigned long long M);

// The chain only visits ~1/4 of the window's positions (attempts start 4 draws apart), so the
// attempt kernel records the draws an attempt would consume (its repeated-index redraws) for every
// position, and checkSubset runs later for the chain's attempts only (ransac_check_kernel).
// kPassUnknown marks such a flag: bits 1..6 valid, bit 0 not evaluated.
constexpr int kPassUnknown = 0x80;

__device__ __forceinline__ int length_flag(long long q, const uint32_t* __restrict__ stream, long long slen,
                                           unsigned N, unsigned long long M) {
    if (q + 4 > slen) return kAttemptSerial;
    int idx[4] = {(int)fastmod(stream[q], M, N), (int)fastmod(stream[q + 1], M, N),
                  (int)fastmod(stream[q + 2], M, N), (int)fastmod(stream[q + 3], M, N)};
    if (!(idx[1] == idx[0] || idx[2] == idx[0] || idx[2] == idx[1] || idx[3] == idx[0] || idx[3] == idx[1] ||
          idx[3] == idx[2]))
        return kPassUnknown;
    const int len = resolve_at(q, stream, slen, N, M, idx);
    return (len == 0 || len > 67) ? kAttemptSerial : (((len - 4) << 1) | kPassUnknown);
}

// RNG::uniform(0, n) = next() % n by Barrett reduction: m = floor((2^32 - 1) / n) >= 2^32/n - 1, so
// q = mulhi(a, m) is the quotient or one less and a - q*n lies in [0, 2n); one unsigned min folds it
// into [0, n).  For n > 256 the quotient fits 24 bits and q*n is the full-rate v_mul_u32_u24 (the
// 64-bit Lemire product of fastmod is six quarter-rate multiplies).
template <bool kNgt256>
__device__ __forceinline__ unsigned mod_barrett(unsigned a, unsigned m, unsigned n) {
    const unsigned q = __umulhi(a, m);
    // the 24-bit product as the full-rate v_mul_u32_u24 (written out: __umul24 and masked operands both
    // compiled to a mask and the quarter-rate v_mul_lo_u32 here, the range of n coming from a branch)
    unsigned qn;
    if (kNgt256)
        asm("v_mul_u32_u24 %0, %1, %2" : "=v"(qn) : "v"(q), "v"(n));
    else
        qn = q * n;
    const unsigned r = a - qn;
    return min(r, r - n);
}

constexpr int kAttemptPerThread = 8;  // window positions per thread (11 draws reduced for 8 attempts)
#ifndef MIM_ATTEMPT_PREFETCH
#define MIM_ATTEMPT_PREFETCH 0
#endif

// The block's 2048 + 3 draws are staged through LDS with coalesced 16-byte loads (a lane's own 11
// draws at a 32-byte lane stride would touch 12 cache lines per load instruction, 11 times over).
constexpr int kAttemptSpan = 256 * kAttemptPerThread;  // window positions per block
// draws per wanted iteration the sampler grids are sized for.  Measured windows (profiles/
// r04_sampler_probe.txt): ~21 draws per iteration on C4 (checkSubset passes ~1 attempt in 5 on 92 %
// outliers), 29 with the window's margin; the flag capacity allows 28.  The grid is sized for 6: a C4
// chunk launches ~35 k attempt blocks (and ~18 k check blocks), each looping over ~4 rounds.
constexpr int kAttemptRateEst = 6;
// the sampler grids' floor (blocks in all, ~16 per CU) for batches too small to fill the GPU otherwise
constexpr int kSamplerMinBlocks = 4096;

// Positions whose first 4 draws repeat an index (~0.3 % at n = 2000, ~5 % at n = 128) are listed in LDS
// over all of the block's rounds and their redraw lengths resolved once at the block's end, one per
// thread (resolved in place, every wave holding one of them, ~80 % of the waves, ran the redraw loop).
constexpr int kAttemptRepCap = 2048;

// Placement (speed only; blocks b and b + 8 share an XCD under round-robin dispatch): the problems share
// one RNG stream and their windows start near the same position, so block b runs window slice kb of
// problem p with kb = b mod 8 (mod 8) and the problems in dispatch order: an XCD streams only its
// slices (1/8 of the window), and consecutive blocks on it read the same slice for different
// problems from its L2.  bpp is a multiple of 8; the grid is n_probs x bpp.
__device__ __forceinline__ void sampler_slice_block(int n_probs, int bpp, int& p, int& kb) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    p = j % n_probs;
    kb = 8 * (j / n_probs) + x;
    (void)bpp;
}

__global__ __launch_bounds__(256) void ransac_attempt_kernel(const RansacState* __restrict__ st,
                                                             const uint32_t* __restrict__ stream, long long slen,
                                                             uint8_t* __restrict__ flags, uint8_t* __restrict__ ibits,
                                                             int wcap, int bpp, int c1, int rep_cap, int n_probs) {
    constexpr int D = kAttemptPerThread + 3;  // the first 4 draws of the thread's 8 attempts
    constexpr int kStageVecs = kAttemptSpan / 4 + 4;  // 16-byte vectors: the span, its 3 extra draws, alignment
    __shared__ __attribute__((aligned(16))) unsigned sdraw[4 * kStageVecs];
    __shared__ int rep_pos[kAttemptRepCap];
    __shared__ int n_rep;
    int p, kb;
    sampler_slice_block(n_probs, bpp, p, kb);
    const RansacState S = st[p];
    if (!S.active || S.done || S.fail_iter != -1 || S.n < kSmallMaxN || S.produced >= min(c1, S.niters)) return;
    const int wlen = window_len(S, c1, wcap);  // a multiple of 64
    MIM_DEBUG_PRINT(threadIdx.x == 0 && kb == 0 && (p == 0 || p == 100),
                    "[attempt] p=%d c1=%d wlen=%d bpp=%d produced=%d stream_pos=%lld n=%d\n", p, c1, wlen, bpp, S.produced,
                    (long long)S.stream_pos, S.n);
    uint8_t* __restrict__ F = flags + (long long)p * wcap;
    uint8_t* __restrict__ IB = ibits + (long long)p * (wcap >> 3);
    const unsigned N = (unsigned)S.n, mB = 0xFFFFFFFFu / N;
    const bool big = N > 256 && N < (1u << 24);  // q and n both fit 24 bits
    if (threadIdx.x == 0) n_rep = 0;
    // stream positions fit 32 bits (the stream is capped at 2^28 draws; 64 zero draws pad its end);
    // the stage starts at the 16-byte vector holding qb: draw qb + e is sdraw[shift + e]
    const int nvec = ((int)slen + 64) >> 2;  // 16-byte vectors in the padded stream buffer
    const uint4* __restrict__ sv = reinterpret_cast<const uint4*>(stream);
    uint4* sd4 = reinterpret_cast<uint4*>(sdraw);
    constexpr int NV = (kStageVecs + 255) / 256;
    // every load of a stage in flight before the first LDS write (unconditional, clamped loads; three
    // named registers: an array carried across the loop went to scratch)
    static_assert(NV == 3, "stage vectors per thread");
#define MIM_ATTEMPT_LOAD_STAGE(bo)                                                   \
    {                                                                                \
        const int qv = ((int)S.stream_pos + (bo)) >> 2;                              \
        v0 = sv[min(qv + min((int)threadIdx.x, kStageVecs - 1), nvec - 1)];          \
        v1 = sv[min(qv + min((int)threadIdx.x + 256, kStageVecs - 1), nvec - 1)];    \
        v2 = sv[min(qv + min((int)threadIdx.x + 512, kStageVecs - 1), nvec - 1)];    \
    }
    uint4 v0, v1, v2;
    if (MIM_ATTEMPT_PREFETCH) MIM_ATTEMPT_LOAD_STAGE(kb * kAttemptSpan);
    // the grid covers the window a typical draw rate implies (kAttemptRateEst), not its capacity; a
    // longer window (low checkSubset pass rate) is covered by the same blocks looping
    for (int boff = kb * kAttemptSpan; boff < wlen; boff += bpp * kAttemptSpan) {
    __syncthreads();  // the previous round's reads of sdraw are done (and n_rep's reset seen)
    const int qb = (int)S.stream_pos + boff;
    const int shift = qb & 3;
    if (!MIM_ATTEMPT_PREFETCH) MIM_ATTEMPT_LOAD_STAGE(boff);
    sd4[threadIdx.x] = v0;
    sd4[threadIdx.x + 256] = v1;
    if (threadIdx.x + 512 < kStageVecs) sd4[threadIdx.x + 512] = v2;
    __syncthreads();
    if (MIM_ATTEMPT_PREFETCH && boff + bpp * kAttemptSpan < wlen) MIM_ATTEMPT_LOAD_STAGE(boff + bpp * kAttemptSpan);
    const int off = boff + threadIdx.x * kAttemptPerThread;
    if (off < wlen) {
    const int q0 = qb + threadIdx.x * kAttemptPerThread;
    unsigned u[D];
#pragma unroll
    for (int k = 0; k < D; ++k) u[k] = sdraw[shift + threadIdx.x * kAttemptPerThread + k];
    if (big) {
#pragma unroll
        for (int k = 0; k < D; ++k) u[k] = mod_barrett<true>(u[k], mB, N);
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) u[k] = mod_barrett<false>(u[k], mB, N);
    }
    // repeated index among the 4 draws of position j: pairs at distance 1, 2, 3, each tested once
    bool d1[D - 1], d2[D - 2], d3[D - 3];
#pragma unroll
    for (int k = 0; k < D - 1; ++k) d1[k] = u[k] == u[k + 1];
#pragma unroll
    for (int k = 0; k < D - 2; ++k) d2[k] = u[k] == u[k + 2];
#pragma unroll
    for (int k = 0; k < D - 3; ++k) d3[k] = u[k] == u[k + 3];
    // one irregular bit per position (a byte per thread's 8 positions); flag bytes only for the irregular
    // positions (~0.3 % at n = 2000): a regular position's outcome is kPassUnknown, implied by its clear bit
    unsigned repm = 0, tailm = 0;
#pragma unroll
    for (int j = 0; j < kAttemptPerThread; ++j) {
        const bool rep = d1[j] | d1[j + 1] | d1[j + 2] | d2[j] | d2[j + 1] | d3[j];
        const bool tail = q0 + j + 4 > (int)slen;
        repm |= (unsigned)(rep && !tail) << j;
        tailm |= (unsigned)tail << j;
    }
    IB[off >> 3] = (uint8_t)(repm | tailm);
    if (tailm) {  // the stream's end: resolved by the walker
        for (unsigned m = tailm; m; m &= m - 1) F[off + __builtin_ctz(m)] = (uint8_t)kAttemptSerial;
    }
    if (repm) {  // rare: list them (a full list: resolved here, from the stream)
        const int sl = atomicAdd(&n_rep, __popc(repm));
        int k = 0;
        for (unsigned m = repm; m; m &= m - 1, ++k) {
            const int j = __builtin_ctz(m);
            if (sl + k < rep_cap) {
                rep_pos[sl + k] = off + j;
            } else {
                int idx[4];
                const int len = resolve_at(q0 + j, stream, slen, N, S.modM, idx);
                F[off + j] = (uint8_t)((len == 0 || len > 67) ? kAttemptSerial : (((len - 4) << 1) | kPassUnknown));
            }
        }
    }
    }
    }
    // the listed positions' redraw lengths, one per thread, over the flag bytes just written (same block)
    __syncthreads();
    const int nr = min(n_rep, rep_cap);
    for (int e = threadIdx.x; e < nr; e += 256) {
        const int pos = rep_pos[e];
        int idx[4];
        const int len = resolve_at(S.stream_pos + pos, stream, slen, N, S.modM, idx);
        F[pos] = (uint8_t)((len == 0 || len > 67) ? kAttemptSerial : (((len - 4) << 1) | kPassUnknown));
    }
}

__device__ __forceinline__ int wave_excl_prefix_sum(int v) {
    const int lane = threadIdx.x & 63;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    return incl - v;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off));
    return v;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off));
    return v;
}

constexpr int kFlagWin = 16384;       // LDS window of attempt flags (bytes)
constexpr int kFlagUnknown = 0xFE;    // past the precomputed window: evaluate inline

__device__ __forceinline__ int ctz64(unsigned long long m) { return __builtin_ctzll(m); }
// wave-uniform values: keep them in SGPRs so the walk's control flow stays scalar
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ long long uni64(long long v) {
    const int lo = __builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int clz64(unsigned long long m) { return __builtin_clzll(m); }
__device__ __forceinline__ int mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// ------------------------------------------------------------------------------------------------
// chain sampler.  getSubset attempts start 4 draws apart until one redraws a repeated index (an
// "irregular" attempt, ~0.3 % of them at n = 2000), so the chain of attempt start positions is a
// few arithmetic runs joined at irregular attempts.  ransac_irr_kernel lists the irregular
// positions of the window (parallel), ransac_chain_kernel walks only those (one wave, LDS) and
// then counts, ranks and writes the passing attempts of the runs in parallel from a pass bitmask.
// Whatever it cannot settle (list overflow, RNG stream end, window end) it leaves to the
// attempt-by-attempt walker (ransac_sample_kernel), which resumes from the state it stores.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ransac_irr_kernel(const RansacState* __restrict__ st,
                                                         const uint8_t* __restrict__ ibits, int wcap, int bpp,
                                                         int c1, int* __restrict__ irr, int* __restrict__ irr_cnt,
                                                         int irr_blocks) {
    __shared__ int wsum[4];
    const int p = blockIdx.x / bpp, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const RansacState S = st[p];
    if (!S.active || S.done || S.fail_iter != -1 || S.n < kSmallMaxN || S.produced >= min(c1, S.niters)) return;
    const int wlen = window_len(S, c1, wcap);
    for (int b = blockIdx.x % bpp; b * kIrrBlock < wlen; b += bpp) {
    __syncthreads();  // wsum of the previous round read
    const int b0 = b * kIrrBlock;
    const int r0 = b0 + tid * 64;  // 64 positions per thread: one 8-byte word of irregular bits
    // positions past wlen read as regular (wlen is a multiple of 64: a thread's word is all in or all
    // out); the chain kernels never walk past wlen
    uint64_t irrm = r0 + 64 <= wlen ? *reinterpret_cast<const uint64_t*>(ibits + (long long)p * (wcap >> 3) + (r0 >> 3)) : 0ull;
    const int c = __popcll(irrm);
    int incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int base = incl - c, total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        base += w < wave ? wsum[w] : 0;
        total += wsum[w];
    }
    const long long slot = (long long)p * irr_blocks + b;
    if (tid == 0) irr_cnt[slot] = total <= kIrrCap ? total : -1;
    if (total > kIrrCap) continue;
    int* L = irr + slot * kIrrCap;
    while (irrm) {
        const int bit = __builtin_ctzll(irrm);
        irrm &= irrm - 1;
        L[base++] = r0 + bit;
    }
    }
}

constexpr int kChainThreads = 1024;
#ifndef MIM_WALK_THREADS
#define MIM_WALK_THREADS 1024
#endif
#ifndef MIM_WALK_ENTRIES
#define MIM_WALK_ENTRIES 8192
#endif
constexpr int kWalkThreads = MIM_WALK_THREADS;     // walk kernel block (>= kIrrBlocksMax)
constexpr int kChainEntries = MIM_WALK_ENTRIES;    // irregular attempts staged in LDS per piece
constexpr int kIrrBlocksMax = 512;                  // list blocks per window (7.3M positions max)
constexpr int kChainSegs = 4 * kChainThreads - 2;   // runs (segments) walked per chunk
constexpr int kNoEvent = INT_MAX;

// The walked chain of one problem and chunk (global, between the walk, check and count kernels).
// Segment j: the regular attempts seg_s[j], seg_s[j] + 4, ... closed by the irregular attempt
// seg_q[j]; segment nseg is the open tail run from seg_s[nseg] (tail attempts).  A[j] = chain index
// of the segment's first attempt, A[nseg + 1] = T attempts in all.
constexpr int kCheckBlock = 256;
constexpr int kChainBlk = 8192;  // check blocks per chunk: >= max window / 4 / kCheckBlock

struct ChainSegs {
    int nseg, tail, s_end, T;
    long long wbase;
    int wlen, pad;
    int blk_seg[kChainBlk];  // segment holding attempt b * kCheckBlock
    int A[kChainSegs + 2];
    int seg_s[kChainSegs + 1];
    int seg_q[kChainSegs];
    uint8_t seg_f[kChainSegs];
};

struct ChainWalkShared {
    int q[kChainEntries];
    uint8_t f[kChainEntries];
    int boff[kIrrBlocksMax + 1];
    int wred[kWalkThreads / 64];
    int wred2[kWalkThreads / 64];
    int n_entries, limit, nseg, tail, cut, stop;
};
static_assert(kWalkThreads >= kIrrBlocksMax, "one thread per irregular-list block");
static_assert((kChainSegs + 2) % kWalkThreads == 0, "walk: segments per thread");
constexpr int kWalkSegsPer = (kChainSegs + 2) / kWalkThreads;

__device__ __forceinline__ int block_excl_sum(int v, int* wred, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    __syncthreads();
    if (lane == 63) wred[wave] = incl;
    __syncthreads();
    int base = incl - v;
    total = 0;
    for (int w = 0; w < nw; ++w) {
        base += w < wave ? wred[w] : 0;
        total += wred[w];
    }
    return base;
}

__device__ __forceinline__ int block_excl_max(int v, int init, int* wred, int& all) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl = max(incl, o);
    }
    int ex = __shfl_up(incl, 1);
    if (lane == 0) ex = INT_MIN;
    __syncthreads();
    if (lane == 63) wred[wave] = incl;
    __syncthreads();
    int r = max(init, ex);
    all = init;
    for (int w = 0; w < nw; ++w) {
        if (w < wave) r = max(r, wred[w]);
        all = max(all, wred[w]);
    }
    return r;
}

__device__ __forceinline__ int block_min(int v, int* wred) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_min(v);
    __syncthreads();
    if (lane == 0) wred[wave] = v;
    __syncthreads();
    int r = INT_MAX;
    for (int w = 0; w < nw; ++w) r = min(r, wred[w]);
    return r;
}

// ---- walk: stage the irregular list in LDS, follow the chain over it (one wave) ----
__global__ __launch_bounds__(kWalkThreads) void ransac_walk_kernel(const RansacState* __restrict__ st,
                                                                    const uint8_t* __restrict__ flags, int wcap,
                                                                    int c1, const int* __restrict__ irr,
                                                                    const int* __restrict__ irr_cnt, int irr_blocks,
                                                                    ChainSegs* __restrict__ chains) {
    __shared__ ChainWalkShared sh;
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const RansacState S = st[p];
    ChainSegs* G = chains + p;
    if (!S.active || S.done || S.fail_iter != -1 || S.n < kSmallMaxN || S.produced >= min(c1, S.niters)) {
        if (tid == 0) G->T = -1;  // nothing to do this chunk (small problems: ransac_small_kernel)
        return;
    }
    const int wlen = window_len(S, c1, wcap);
    const uint8_t* F = flags + (long long)p * wcap;
    const int nb = min((wlen + kIrrBlock - 1) / kIrrBlock, kIrrBlocksMax);
    // the listed blocks up to the first overflowing one (more than kIrrCap irregular positions)
    {
        const int cnt = tid < nb ? irr_cnt[(long long)p * irr_blocks + tid] : 0;
        const int bad = tid < nb && cnt < 0 ? tid : INT_MAX;
        int total;
        const int off = block_excl_sum(max(cnt, 0), sh.wred, total);
        const int cut = min(block_min(bad, sh.wred2), nb);
        if (tid <= nb) sh.boff[tid] = tid < nb ? off : 0;
        __syncthreads();
        if (tid == 0) {
            sh.cut = cut;
            sh.n_entries = cut > 0 ? sh.boff[cut - 1] + irr_cnt[(long long)p * irr_blocks + cut - 1] : 0;
            sh.limit = min(wlen, cut * kIrrBlock);
            sh.stop = 0;
        }
        __syncthreads();
    }
    // the entries stream through LDS in pieces of kChainEntries; wave 0 walks each piece, keeping its
    // chain position across pieces (entries are in ascending position order)
    int s = 0, nwalk = 0, limit = sh.limit;
    const int E = sh.n_entries, cut = sh.cut;
    for (int eb = 0; eb < E; eb += kChainEntries) {
        const int ee = min(E, eb + kChainEntries);
        for (int e = eb + tid; e < ee; e += kWalkThreads) {
            int lo = 0, hi = cut - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (sh.boff[mid] <= e) lo = mid; else hi = mid - 1;
            }
            const int q = irr[((long long)p * irr_blocks + lo) * kIrrCap + (e - sh.boff[lo])];
            sh.q[e - eb] = q;
            sh.f[e - eb] = F[q];
        }
        __syncthreads();
        if (tid < 64) {
            bool stop = false;
            for (int e0 = eb; e0 < ee && !stop; e0 += 64) {
                const int e = e0 + lane;
                const int q = e < ee ? sh.q[e - eb] : INT_MAX;
                const int f = e < ee ? (int)sh.f[e - eb] : 0;
                for (;;) {
                    const unsigned long long m = __ballot(q >= s && q < limit && ((q - s) & 3) == 0);
                    if (!m) break;
                    // wave-uniform lane index: v_readlane (no LDS round trip per walked event)
                    const int k = uni(__builtin_ctzll(m));
                    const int qq = __builtin_amdgcn_readlane(q, k), ff = __builtin_amdgcn_readlane(f, k);
                    if (ff == kAttemptSerial || nwalk == kChainSegs) {  // resolved by the walker
                        limit = qq;
                        stop = true;
                        break;
                    }
                    if (lane == 0) {
                        G->seg_s[nwalk] = s;
                        G->seg_q[nwalk] = qq;
                        G->seg_f[nwalk] = (uint8_t)ff;
                    }
                    ++nwalk;
                    s = uni(qq + 4 + ((ff & 0x7F) >> 1));
                }
            }
            if (lane == 0 && stop) sh.stop = 1;
        }
        __syncthreads();
        if (sh.stop) break;
    }
    if (tid < 64) {
        if (lane == 0) {
            const int tail = s < limit ? (limit - s + 3) >> 2 : 0;
            G->seg_s[nwalk] = s;
            sh.nseg = nwalk;
            sh.tail = tail;
            G->nseg = nwalk;
            G->tail = tail;
            G->s_end = s + 4 * tail;
            G->wbase = S.stream_pos;
            G->wlen = wlen;
        }
    }
    __syncthreads();
    const int nseg = sh.nseg;
    // chain index of every segment start
    int v[kWalkSegsPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kWalkSegsPer; ++k) {
        const int j = kWalkSegsPer * tid + k;
        v[k] = j < nseg ? ((G->seg_q[j] - G->seg_s[j]) >> 2) + 1 : (j == nseg ? sh.tail : 0);
        sum += v[k];
    }
    int total;
    int base = block_excl_sum(sum, sh.wred, total);
#pragma unroll
    for (int k = 0; k < kWalkSegsPer; ++k) {
        const int j = kWalkSegsPer * tid + k;
        if (j <= nseg + 1) G->A[j] = base;
        if (j <= nseg)  // the check blocks whose first attempt falls in segment j
            for (int b = (base + kCheckBlock - 1) / kCheckBlock; b * kCheckBlock < base + v[k] && b < kChainBlk; ++b)
                G->blk_seg[b] = j;
        base += v[k];
    }
    if (tid == 0) G->T = total;
}

// position of chain attempt t in segment j (A[j] <= t < A[j+1]); irregular: the closing attempt
__device__ __forceinline__ int chain_pos(const ChainSegs* G, int j, int t, bool& irregular) {
    irregular = j < G->nseg && t == G->A[j + 1] - 1;
    return irregular ? G->seg_q[j] : G->seg_s[j] + 4 * (t - G->A[j]);
}

__device__ __forceinline__ int chain_seg(const ChainSegs* G, int t) {
    int lo = 0, hi = G->nseg;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (G->A[mid] <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// ---- check: checkSubset of every attempt on the walked chain (one thread per attempt) ----

// Each thread checks kCheckPer attempts (block-strided, so every round is one ballot word pair per
// wave): their stream draws and point gathers are all in flight at once.
constexpr int kCheckPer = MIM_CHECK_PER;
constexpr int kCheckSegs = 8;  // segments preloaded per block (a block spans ~4 on average)
#ifndef MIM_PROBE_CHECK
#define MIM_PROBE_CHECK 0  // timing probe only (wrong samples): 1 = no deferred pass, 2 = and no fp32 checks,
                           // 3 = no deferred pass, every point gathered, a 16-add stand-in for the fp32 check
#endif
// Deferred attempts listed per check round (ransac_check_defer_kernel); a round with more decides the
// rest in place.  C4: ~4 per round of 1,024 attempts.
constexpr int kDefSlots = kRansacDefSlots;
#ifndef MIM_CHECK_LDS
#define MIM_CHECK_LDS 0  // 1: the check blocks gather the points of problems with n <= 2,048 from LDS
#endif
constexpr int kCheckLdsPts = MIM_CHECK_LDS ? 2048 : 1;
static_assert(kCheckBlock * kCheckPer == kRansacDefRoundAttempts, "check round size shared with api.cpp");

// checkSubset (fp64) of a deferred attempt: qe = its first draw's stream position, or -position - 1 for
// a redraw attempt.  Out of line: inlined, its fp64 sample and redraw buffer raised the check kernel's
// register count (102 against 71 without it, i.e. 5 instead of 7 waves per SIMD to hide the gathers).
__device__ __attribute__((noinline)) bool check_deferred(int qe, const uint32_t* __restrict__ stream, long long slen,
                                                         unsigned N, unsigned long long modM,
                                                         const float4* __restrict__ P) {
    const long long qq = qe < 0 ? -(long long)qe - 1 : qe;
    int ix[4];
    if (qe < 0) {
        resolve_at(qq, stream, slen, N, modM, ix);  // the walk only listed resolvable ones
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) ix[k] = (int)fastmod(stream[qq + k], modM, N);
    }
    const float4 a = P[ix[0]], bp = P[ix[1]], c = P[ix[2]], d = P[ix[3]];
    const float s4[8] = {a.x, a.y, bp.x, bp.y, c.x, c.y, d.x, d.y};
    const float t4[8] = {a.z, a.w, bp.z, bp.w, c.z, c.w, d.z, d.w};
    return check_subset(s4, t4);
}

#ifndef MIM_CHECK_OCC
#define MIM_CHECK_OCC 1  // minimum waves per SIMD the check kernel's register budget is fitted to (build knob)
#endif
__global__ __launch_bounds__(kCheckBlock, MIM_CHECK_OCC) void ransac_check_kernel(const ChainSegs* __restrict__ chains,
                                                                   const ProbDev* __restrict__ probs,
                                                                   const float4* __restrict__ pts,
                                                                   const RansacState* __restrict__ st,
                                                                   const uint32_t* __restrict__ stream, long long slen,
                                                                   uint32_t* __restrict__ pass_bits, int wcap, int bpp,
                                                                   int2* __restrict__ defer, int* __restrict__ defer_n,
                                                                   int def_rounds, int n_probs) {
    __shared__ uint32_t words[kCheckBlock * kCheckPer / 32];  // the round's pass bits
    __shared__ int def_t[kCheckBlock * kCheckPer], def_q[kCheckBlock * kCheckPer];  // the round's deferred attempts
    __shared__ int4 seg_tab[kCheckSegs];
    __shared__ int n_def;
    __shared__ float4 spts[kCheckLdsPts];  // the problem's points (MIM_CHECK_LDS, n <= kCheckLdsPts)
    // placement (speed only): problem p on XCD p mod 8 (its points stay in one L2), and an XCD's
    // problems in dispatch order for each chain slice kb (the slice's stream draws read from that L2 by
    // all of them); grid 8 ceil(n_probs / 8) bpp, blocks past n_probs idle
    const int x = blockIdx.x & 7, jx = blockIdx.x >> 3, np8 = (n_probs + 7) >> 3;
    const int p = x + 8 * (jx % np8), kb0 = jx / np8, lane = threadIdx.x & 63;
    if (p >= n_probs) return;
    const ChainSegs* G = chains + p;
    const int T = G->T;
    if (T <= 0) return;  // nothing this chunk
    const RansacState S = st[p];
    const float4* P = pts + probs[p].good_off;
    const bool lds = MIM_CHECK_LDS && S.n <= kCheckLdsPts;  // uniform over the block
    if (lds) {
        for (int i = threadIdx.x; i < S.n; i += kCheckBlock) spts[i] = P[i];
        // (the first round's barriers order these stores before the gathers)
    }
    for (int b = kb0; b * kCheckBlock * kCheckPer < T; b += bpp) {
    const int base = b * kCheckBlock * kCheckPer;
    // segment data of the block's first kCheckSegs segments in one round of (uniform, scalar) loads
    const int nseg = G->nseg;
    const int bb = base / kCheckBlock;
    const int j0 = bb < kChainBlk ? G->blk_seg[bb] : chain_seg(G, base);
    // {A[j], A[j + 1], seg_s[j], seg_q[j]} of segments j0 .. j0 + kCheckSegs - 1 in LDS (one 16-byte read
    // per attempt once its segment is known); the segment starts for the count in scalar registers
    if (threadIdx.x < kCheckSegs) {
        const int j = j0 + threadIdx.x;
        seg_tab[threadIdx.x] = make_int4(G->A[min(j, nseg + 1)], G->A[min(j + 1, nseg + 1)], G->seg_s[min(j, nseg)],
                                         G->seg_q[min(j, max(nseg - 1, 0))]);
    }
    int segA[kCheckSegs];
#pragma unroll
    for (int k = 1; k < kCheckSegs; ++k) segA[k] = j0 + k <= nseg ? G->A[j0 + k] : INT_MAX;
    const unsigned N = (unsigned)S.n;
    if (threadIdx.x == 0) n_def = 0;
    __syncthreads();  // seg_tab
    int q[kCheckPer];
    bool irr[kCheckPer], valid[kCheckPer];
#pragma unroll
    for (int r = 0; r < kCheckPer; ++r) {
        const int t = base + r * kCheckBlock + threadIdx.x;
        valid[r] = t < T;
        int k = 0;
#pragma unroll
        for (int i = 1; i < kCheckSegs; ++i) k += t >= segA[i];
        const int4 e = seg_tab[k];
        int j = j0 + k, pos;
        bool irregular;
        if (j < nseg && t >= e.y) {  // past the preloaded segments (rare)
            while (j < nseg && t >= G->A[j + 1]) ++j;
            pos = chain_pos(G, j, t, irregular);
        } else {
            irregular = j < nseg && t == e.y - 1;
            pos = irregular ? e.w : e.z + 4 * (t - e.x);
        }
        q[r] = valid[r] ? (int)(G->wbase + pos) : 0;
        irr[r] = valid[r] && irregular;
    }
    // all regular draws first (one 16-byte load per attempt: consecutive chain attempts are 4 draws
    // apart, so a wave reads 1 KiB contiguously; dword-aligned vector loads), then the reductions
    typedef unsigned uint4a4 __attribute__((ext_vector_type(4), aligned(4)));
    unsigned raw[kCheckPer][4];
#pragma unroll
    for (int r = 0; r < kCheckPer; ++r) {
        const uint4a4 v = *reinterpret_cast<const uint4a4*>(stream + q[r]);  // 4-B aligned 16-B load
        raw[r][0] = v.x; raw[r][1] = v.y; raw[r][2] = v.z; raw[r][3] = v.w;
    }
    int idx[kCheckPer][4];
#pragma unroll
    for (int r = 0; r < kCheckPer; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) idx[r][k] = valid[r] ? (int)fastmod(raw[r][k], S.modM, N) : 0;
    float4 g[kCheckPer][4];
    __syncthreads();  // n_def reset (and the staged points)
    if (lds) {
#pragma unroll
        for (int r = 0; r < kCheckPer; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k) g[r][k] = spts[idx[r][k]];
    } else {
#pragma unroll
        for (int r = 0; r < kCheckPer; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k) g[r][k] = P[idx[r][k]];
    }
    const bool listed = b < def_rounds;
#pragma unroll
    for (int r = 0; r < kCheckPer; ++r) {
        const float s4[8] = {g[r][0].x, g[r][0].y, g[r][1].x, g[r][1].y, g[r][2].x, g[r][2].y, g[r][3].x, g[r][3].y};
        const float t4[8] = {g[r][0].z, g[r][0].w, g[r][1].z, g[r][1].w, g[r][2].z, g[r][2].w, g[r][3].z, g[r][3].w};
        bool clear = true;
        const bool pass32 = MIM_PROBE_CHECK == 3 ? (s4[0] + s4[1] + s4[2] + s4[3] + s4[4] + s4[5] + s4[6] + s4[7] +
                                                    t4[0] + t4[1] + t4[2] + t4[3] + t4[4] + t4[5] + t4[6] + t4[7]) > 4000.f
                          : MIM_PROBE_CHECK == 2 ? s4[0] != t4[1] : check_subset_fp32(s4, t4, clear);
        MIM_DEBUG_CHECK(!valid[r] || !clear || pass32 == check_subset(s4, t4),
                        "[check] fp32 checkSubset %d differs from fp64 (p=%d t=%d)\n", (int)pass32, p,
                        base + r * kCheckBlock + (int)threadIdx.x);
        // deferred: the redraw attempts (their indices need the walk over the stream) and the samples
        // fp32 cannot decide, decided by ransac_check_defer_kernel (in place they made most waves run
        // both slow paths)
        const bool defer = MIM_PROBE_CHECK == 0 && valid[r] && (irr[r] || !clear);
        const unsigned long long m = __ballot(valid[r] && !defer && pass32);
        const int wl = (r * kCheckBlock + (threadIdx.x & ~63)) >> 5;  // the wave's 2 words of the block's
        if (lane == 0) words[wl] = (uint32_t)m;
        if (lane == 32) words[wl + 1] = (uint32_t)(m >> 32);
        if (defer) {
            const int slot = atomicAdd(&n_def, 1);
            def_t[slot] = r * kCheckBlock + threadIdx.x;
            def_q[slot] = irr[r] ? -q[r] - 1 : q[r];
        }
    }
    __syncthreads();
    MIM_DEBUG_PRINT(threadIdx.x == 0 && (p == 0 || p == 100), "[check] p=%d b=%d bpp=%d T=%d nseg=%d n_def=%d wlen=%d\n",
                    p, b, bpp, T, nseg, n_def, G->wlen);
    // the round's first kDefSlots deferred attempts go to ransac_check_defer_kernel's list (their pass
    // bits are set there, after this kernel), so the block does not wait on their draws and gathers;
    // any further ones (rare) are decided here
    const int nl = listed ? min(n_def, kDefSlots) : 0;
    if (listed && threadIdx.x == 0) defer_n[(long long)p * def_rounds + b] = nl;
    if (threadIdx.x < nl)
        defer[((long long)p * def_rounds + b) * kDefSlots + threadIdx.x] =
            make_int2(base + def_t[threadIdx.x], def_q[threadIdx.x]);
    if (n_def > nl) {
        for (int e = nl + threadIdx.x; e < n_def; e += kCheckBlock) {  // one deferred attempt per thread
            const int tl = def_t[e];
            if (check_deferred(def_q[e], stream, slen, N, S.modM, P)) atomicOr(&words[tl >> 5], 1u << (tl & 31));
        }
        __syncthreads();
    }
    uint32_t* PB = pass_bits + (long long)p * (wcap / 32);
    if (threadIdx.x < kCheckBlock * kCheckPer / 32 && (base + 32 * (int)threadIdx.x) < T)
        PB[(base >> 5) + threadIdx.x] = words[threadIdx.x];
    __syncthreads();  // words / n_def reused by the next round
    }
}

// The check rounds' listed deferred attempts (redraw attempts, samples fp32 could not decide): one
// thread each, fp64 checkSubset as in the check kernel's second pass, the pass bit OR-ed into the
// round's word the check kernel stored.  Grid n_probs x nblk, thread j of problem p: round j / kDefSlots,
// slot j % kDefSlots; rounds past the chain's attempts hold stale counts and are skipped.
__global__ __launch_bounds__(256) void ransac_check_defer_kernel(const ChainSegs* __restrict__ chains,
                                                                 const ProbDev* __restrict__ probs,
                                                                 const float4* __restrict__ pts,
                                                                 const RansacState* __restrict__ st,
                                                                 const uint32_t* __restrict__ stream, long long slen,
                                                                 uint32_t* __restrict__ pass_bits, int wcap,
                                                                 const int2* __restrict__ defer,
                                                                 const int* __restrict__ defer_n, int def_rounds,
                                                                 int nblk, int n_probs) {
    const int p = blockIdx.x / nblk;
    const int j = (blockIdx.x % nblk) * 256 + threadIdx.x, round = j / kDefSlots, e = j % kDefSlots;
    if (p >= n_probs || round >= def_rounds) return;
    const int T = chains[p].T;
    if (round * (kCheckBlock * kCheckPer) >= T) return;
    const long long rr = (long long)p * def_rounds + round;
    if (e >= defer_n[rr]) return;
    const int2 en = defer[rr * kDefSlots + e];
    const int t = en.x, qe = en.y;
    if (check_deferred(qe, stream, slen, (unsigned)st[p].n, st[p].modM, pts + probs[p].good_off))
        atomicOr(pass_bits + (long long)p * (wcap / 32) + (t >> 5), 1u << (t & 31));
}

// ---- count: ranks of the passing attempts, getSubset's failure rule, samples, state ----
// Visit the passing attempts with chain index in [t0, t1), in order: fn(t).
// (words fetched 8 at a time with unconditional loads: one memory latency per 8 words)
template <class Fn>
__device__ __forceinline__ void pass_visit(const uint32_t* __restrict__ PB, int t0, int t1, Fn&& fn) {
    if (t0 >= t1) return;
    const int wl = (t1 - 1) >> 5;
    for (int w0 = t0 >> 5; w0 <= wl; w0 += 8) {
        uint32_t wd[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) wd[k] = PB[min(w0 + k, wl)];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int w = w0 + k;
            if (w > wl) break;
            const int lo_b = max(t0 - 32 * w, 0), hi_b = min(t1 - 32 * w, 32);
            const uint32_t rm = (hi_b == 32 ? 0xFFFFFFFFu : ((1u << hi_b) - 1)) & ~((1u << lo_b) - 1);
            uint32_t bits = wd[k] & rm;
            while (bits) {
                const int bit = __builtin_ctz(bits);
                bits &= bits - 1;
                fn(32 * w + bit);
            }
        }
    }
}

struct ChainCountShared {
    int wred[kChainThreads / 64];
    int wred2[kChainThreads / 64];
    int t_need;
};

__global__ __launch_bounds__(kChainThreads) void ransac_count_kernel(RansacState* __restrict__ st,
                                                                     const ProbDev* __restrict__ probs,
                                                                     const ChainSegs* __restrict__ chains,
                                                                     const uint32_t* __restrict__ pass_bits,
                                                                     const uint8_t* __restrict__ flags, int wcap,
                                                                     int4* __restrict__ samples, int c1) {
    __shared__ ChainCountShared sh;
    const int p = blockIdx.x, tid = threadIdx.x;
    const ChainSegs* G = chains + p;
    const int T = G->T;
    if (T < 0) return;
    RansacState S = st[p];
    const int target = min(c1, S.niters);
    // with the sampler stream the previous chunk's replay may lower niters after the walk kernel
    // read it: nothing is left to produce then (never write past the target: the samples of a
    // problem hold at most maxIters rows, the next problem's follow)
    if (S.produced >= target) return;
    const long long wbase = G->wbase;
    const uint32_t* PB = pass_bits + (long long)p * (wcap / 32);
    // contiguous ranges of attempts, whole 32-bit words per thread
    const int words = (T + 31) >> 5;
    const int wpt = (words + kChainThreads - 1) / kChainThreads;
    const int t0 = min(T, tid * wpt * 32), t1 = min(T, t0 + wpt * 32);
    int cnt = 0, first = -1, last = -1;
    pass_visit(PB, t0, t1, [&](int t) {
        if (first < 0) first = t;
        last = t;
        ++cnt;
    });
    // failure rule of getSubset: 10000 consecutive rejected attempts (ranges here are < 10000 long,
    // so a failure can only end a gap that starts at an earlier thread's last pass)
    int total;
    const int base = block_excl_sum(cnt, sh.wred, total);
    const int v0 = -1 - S.fail_run;  // virtual pass before the chunk
    int last_all;
    const int prev = block_excl_max(cnt ? last : INT_MIN, v0, sh.wred2, last_all);
    int ev = (cnt && first - prev - 1 >= 10000) ? prev + 10000 : kNoEvent;
    if (tid == 0 && T - 1 - last_all >= 10000) ev = min(ev, last_all + 10000);
    const int t_fail = block_min(ev, sh.wred);
    const int need = target - S.produced;
    if (tid == 0) sh.t_need = kNoEvent;
    __syncthreads();
    if (base < need && need <= base + cnt) {  // the attempt completing the chunk's last iteration
        int k = need - base;
        pass_visit(PB, t0, t1, [&](int t) {
            if (--k == 0) sh.t_need = t;
        });
    }
    __syncthreads();
    const int t_need = sh.t_need;
    int keep;  // passes written (ranks [0, keep))
    if (t_fail < t_need) {
        int before = 0;
        if (cnt && last < t_fail) before = cnt;
        else if (cnt && first < t_fail) pass_visit(PB, t0, t1, [&](int t) { before += t < t_fail; });
        int tot_before;
        block_excl_sum(before, sh.wred, tot_before);
        keep = tot_before;
    } else {
        keep = t_need != kNoEvent ? need : total;
    }
    if (base < keep) {
        int4* out = samples + probs[p].it_off + S.produced;
        int r = base, j = -1, a_next = 0, a_j = 0, s_j = 0, q_j = 0;
        pass_visit(PB, t0, t1, [&](int t) {
            if (r < keep) {
                if (j < 0 || t >= a_next) {  // passes come in increasing t: segment data cached
                    j = j < 0 ? chain_seg(G, t) : j + 1;
                    while (j < G->nseg && t >= G->A[j + 1]) ++j;
                    a_j = G->A[j];
                    a_next = G->A[j + 1];
                    s_j = G->seg_s[j];
                    q_j = j < G->nseg ? G->seg_q[j] : 0;
                }
                const bool irregular = j < G->nseg && t == a_next - 1;
                const int pos = irregular ? q_j : s_j + 4 * (t - a_j);
                out[r] = make_int4((int)(wbase + pos), irregular ? -2 : -1, 0, 0);
            }
            ++r;
        });
    }
    if (tid == 0) {
        S.win_base = wbase;
        S.win_len = G->wlen;
        if (t_fail < t_need) {
            S.produced += keep;
            S.fail_iter = S.produced;  // getSubset returned false in this iteration
            S.fail_run = 10000;
        } else if (t_need != kNoEvent) {
            const int j = chain_seg(G, t_need);
            bool irregular;
            const int pos = chain_pos(G, j, t_need, irregular);
            const int len = irregular ? 4 + ((flags[(long long)p * wcap + pos] & 0x7F) >> 1) : 4;
            S.produced = target;
            S.stream_pos = wbase + pos + len;
            S.fail_run = 0;
        } else {
            S.produced += total;
            S.fail_run = total > 0 ? T - 1 - last_all : S.fail_run + T;
            S.stream_pos = wbase + G->s_end;
        }
        store_sampler_state(st + p, S);
    }
}


// ------------------------------------------------------------------------------------------------
// small: the getSubset replay of problems with fewer than kSmallMaxN points, one block each.
// Repeated indices make most attempts' lengths irregular there (n = 8: 59 % redraw) and degenerate
// real-data problems (duplicated keypoints) pass checkSubset ~1/30 attempts, so the first chunk's
// 512 iterations can take ~20k attempts; walked one by one that is ~580 cycles per attempt.  A
// round of this kernel covers 16k stream positions from the chain's current position:
//   0. the round's draws, reduced mod n, are staged in LDS as bytes (n < 256), with the draws
//      consumed by the attempt starting at each position (getSubset's redraw-on-repeat);
//   1. every thread walks its own 64-position segment from the segment's first position
//      (speculative: the visited positions as a 64-bit mask, and the exit position);
//   2. wave 0 joins the segments in order: the true chain enters segment i at e; a speculative walk
//      through e is the chain from there on, otherwise the chain is walked from e until it meets
//      the speculative one (chains of random lengths merge within a few attempts) or leaves;
//   3. checkSubset of every chain attempt (indices from LDS, points staged in LDS);
//   4. ranks of the passes, the wanted iteration and the 10000-rejection failure by block scans.
// An attempt that needs more draws than staged (> 67, or the RNG stream end) closes the round
// before it and is then resolved alone.  These problems never use the attempt window.
// ------------------------------------------------------------------------------------------------
constexpr int kSmallThreads = 256;
constexpr int kSmallRound = kSmallThreads * 64;  // positions per round (one 64-bit mask per thread)
constexpr int kSmallExtra = 128;                 // draws staged past the round's last position
constexpr uint8_t kSmallAlone = 0xFF;            // attempt resolved alone

struct SmallShared {
    uint8_t idx[kSmallRound + kSmallExtra];  // draw k of the round, mod n
    uint8_t len[kSmallRound];                // draws - 4 of the attempt starting at each position
    float4 P[kSmallMaxN];
    unsigned long long V[kSmallThreads];     // per segment: exits of the walks from its first 16 positions
    int X[kSmallThreads];                    // per segment: the chain's entry (-1: jumped over)
    unsigned long long Wt[kSmallThreads / 64];  // exit tables composed over each wave's segments
    int wred[kSmallThreads / 64];
    int wred2[kSmallThreads / 64];
    int bad, e_end, q_sel;
};

// exit tables: nibble r = where the walk entering a segment at offset r leaves it (offset into the
// next segment; 15: 15 or more, the table cannot continue).  compose_exits(A, B) = B after A.
__device__ __forceinline__ unsigned long long compose_exits(unsigned long long A, unsigned long long B) {
    unsigned long long R = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int x = (int)(A >> (4 * r)) & 15;
        const int y = x == 15 ? 15 : (int)(B >> (4 * x)) & 15;
        R |= (unsigned long long)y << (4 * r);
    }
    return R;
}

__device__ __forceinline__ unsigned long long shfl_up64(unsigned long long v, int off) {
    const int lo = __shfl_up((int)(unsigned)v, off), hi = __shfl_up((int)(v >> 32), off);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// getSubset's sample from 16 consecutive draws: the first 4 distinct; c < 4 if they do not suffice
__device__ __forceinline__ int first4_distinct(const unsigned (&u)[16], int (&a)[4]) {
    a[0] = (int)u[0];
    a[1] = a[2] = a[3] = 0;
    int c = 1, len = 0;
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        const int v = (int)u[k];
        const bool take = c < 4 && v != a[0] && (c < 2 || v != a[1]) && (c < 3 || v != a[2]);
        a[1] = take && c == 1 ? v : a[1];
        a[2] = take && c == 2 ? v : a[2];
        a[3] = take && c == 3 ? v : a[3];
        len = take && c == 3 ? k + 1 : len;
        c += take ? 1 : 0;
    }
    return len;  // 0: more than 16 draws
}

__global__ __launch_bounds__(kSmallThreads) void ransac_small_kernel(RansacState* __restrict__ st,
                                                                     const ProbDev* __restrict__ probs,
                                                                     const float4* __restrict__ pts,
                                                                     const uint32_t* __restrict__ stream, long long slen,
                                                                     int4* __restrict__ samples, int c1,
                                                                     int* __restrict__ err) {
    __shared__ __attribute__((aligned(16))) SmallShared sh;
    constexpr int BIG = 1 << 30;
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    RansacState S = st[p];
    if (!S.active || S.done || S.fail_iter != -1 || S.n >= kSmallMaxN) return;
    const int target = min(c1, S.niters);
    if (S.produced >= target) return;
    const unsigned N = (unsigned)S.n;
    const unsigned long long M = S.modM;
    const float4* Pg = pts + probs[p].good_off;
    if (tid < (int)N) sh.P[tid] = Pg[tid];
    int4* out = samples + probs[p].it_off;
    long long pos = S.stream_pos;  // the chain's next attempt (absolute stream position)
    int produced = S.produced, fail_run = S.fail_run;
    bool stop_all = false;
    while (!stop_all && produced < target) {
        // 0. stage the draws of [pos, pos + kSmallRound + kSmallExtra), then the attempt lengths
        const long long avail = slen - pos;  // draws left in the RNG stream (past it: 64 zero draws)
        {
            // 16-byte loads from the aligned vector holding pos, all in flight at once
            constexpr int kVec = (kSmallRound + kSmallExtra + 3) / 4 + 1, kVecPer = (kVec + kSmallThreads - 1) / kSmallThreads;
            const long long v0 = pos >> 2, nvec = (slen + 64) >> 2;
            const int shift = (int)(pos & 3);
            const uint4* __restrict__ sv = reinterpret_cast<const uint4*>(stream);
            uint4 v[kVecPer];
#pragma unroll
            for (int j = 0; j < kVecPer; ++j) v[j] = sv[min(v0 + tid + kSmallThreads * j, nvec - 1)];
#pragma unroll
            for (int j = 0; j < kVecPer; ++j) {
                const unsigned vv[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int e = 4 * (tid + kSmallThreads * j) + c - shift;
                    if (e >= 0 && e < kSmallRound + kSmallExtra) sh.idx[e] = (uint8_t)fastmod(vv[c], M, N);
                }
            }
        }
        if (tid == 0) sh.bad = kSmallRound;
        __syncthreads();
        // the draws consumed by the attempt at each of the thread's 64 positions, by two pointers:
        // the attempt at j ends at k4(j), the first r with 4 distinct draws in [j, r), and k4 never
        // decreases with j.  The window's distinct draws are 4 (value, last occurrence) slots.
        int bad_mine = BIG;
        {
            const int jend = 64 * tid + 64;
            int j = 64 * tid, r = j, cnt = 0;
            int val[4] = {0, 0, 0, 0}, last[4] = {-1, -1, -1, -1};  // last < 0: free slot
            while (j < jend) {
                const int v = sh.idx[min(r, kSmallRound + kSmallExtra - 1)], u = sh.idx[j];
                if (cnt < 4 && r < kSmallRound + kSmallExtra) {  // extend the window by draw r
                    int hit = -1, fr = -1;
#pragma unroll
                    for (int k = 3; k >= 0; --k) {
                        hit = last[k] >= 0 && val[k] == v ? k : hit;
                        fr = last[k] < 0 ? k : fr;
                    }
                    const int sl = hit >= 0 ? hit : fr;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        val[k] = k == sl ? v : val[k];
                        last[k] = k == sl ? r : last[k];
                    }
                    cnt += hit < 0 ? 1 : 0;
                    ++r;
                } else {  // the attempt at j: r - j draws (more than staged: resolved alone)
                    const int len = cnt == 4 ? r - j : 0;
                    const bool alone = len == 0 || len > 67 || j + len > avail;
                    sh.len[j] = alone ? kSmallAlone : (uint8_t)(len - 4);
                    if (alone) bad_mine = min(bad_mine, j);
#pragma unroll
                    for (int k = 0; k < 4; ++k)  // draw j leaves the window: its slot if it was the last
                        if (last[k] == j && val[k] == u) {
                            last[k] = -1;
                            --cnt;
                        }
                    ++j;
                }
            }
        }
        if (bad_mine < BIG) atomicMin(&sh.bad, bad_mine);
        __syncthreads();
        const int Rz = sh.bad;  // the round: positions [0, Rz), the chain's attempts starting there
        if (Rz == 0) {
            // the chain's next attempt is resolved alone (uniform)
            int idx[4] = {0, 0, 0, 0};
            const int len = resolve_at(pos, stream, slen, N, M, idx);
            if (len == 0) {  // RNG stream exhausted: report, never guess
                if (tid == 0) atomicOr(err, 1);
                S.fail_iter = -2;
                break;
            }
            const float4 a = sh.P[idx[0]], b = sh.P[idx[1]], c = sh.P[idx[2]], d = sh.P[idx[3]];
            const float s4[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
            const float t4[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
            if (uni(check_subset(s4, t4) ? 1 : 0)) {
                if (tid == 0) out[produced] = make_int4((int)pos, len != 4 ? -2 : -1, 0, 0);
                ++produced;
                fail_run = 0;
            } else if (++fail_run >= 10000) {
                S.fail_iter = produced;  // getSubset returned false in this iteration
                stop_all = true;
            }
            pos += len;
            __syncthreads();  // sh.idx / sh.len are restaged
            continue;
        }
        const int nseg = (Rz + 63) >> 6;
        // 1. the segment's walks from its first 16 positions: where each leaves the segment, as a
        //    nibble (exit - segment end; 15: 15 or more, then walked again in step 2)
        if (tid < nseg) {
            const int s0 = 64 * tid, se = min(s0 + 64, Rz);
            int q[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) q[r] = s0 + r;
#pragma unroll
            for (int step = 0; step < 16; ++step)  // >= 4 draws an attempt: <= 16 attempts a walk
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (q[r] < se) q[r] += 4 + sh.len[q[r]];
            unsigned long long nib = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) nib |= (unsigned long long)min(max(q[r] - se, 0), 15) << (4 * r);
            sh.V[tid] = nib;
        }
        __syncthreads();
        // 2. the chain's entry into every segment: a block scan of the exit tables under
        //    composition (segment 0 is entered at 0; segment i at T_{i-1}(...T_0(0))).  An exit of
        //    15 or more breaks the tables: from that segment on wave 0 joins in order, walking on LDS.
        {
            constexpr unsigned long long kId = 0xFEDCBA9876543210ull;  // identity table
            const unsigned long long T = tid < nseg ? sh.V[tid] : kId;
            unsigned long long incl = T;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned long long o = shfl_up64(incl, off);
                if (lane >= off) incl = compose_exits(o, incl);
            }
            if (lane == 63) sh.Wt[tid >> 6] = incl;
            __syncthreads();
            unsigned long long pw = kId;  // the waves before this one
            for (int w = 0; w < (tid >> 6); ++w) pw = compose_exits(pw, sh.Wt[w]);
            unsigned long long excl = shfl_up64(incl, 1);
            if (lane == 0) excl = kId;
            excl = compose_exits(pw, excl);
            incl = compose_exits(pw, incl);
            const int ent = (int)(excl & 15);
            if (tid < nseg) sh.X[tid] = ent;
            if (tid == nseg - 1) sh.e_end = (int)(incl & 15) == 15 ? -1 : Rz + (int)(incl & 15);
            const int esc = block_min(tid < nseg && ent == 15 ? tid : BIG, sh.wred2);
            const bool esc_end = sh.e_end < 0;  // (written before block_min's barriers)
            if ((esc < BIG || esc_end) && tid < 64) {  // wave 0, uniform: join in order from the break
                int i = esc < BIG ? esc - 1 : nseg - 1;
                int e = 64 * i + sh.X[i];
                for (; i < nseg; ++i) {
                    const int s0 = 64 * i, se = min(s0 + 64, Rz);
                    int ent_i = -1;
                    if (e < se) {  // else the chain jumps over the segment
                        const int off = e - s0;
                        ent_i = off;
                        const int x = off < 16 ? (int)(uni64((long long)sh.V[i]) >> (4 * off)) & 15 : 15;
                        if (x < 15) {
                            e = se + x;
                        } else {
                            int qq = e;
                            while (qq < se) qq += 4 + uni((int)sh.len[qq]);
                            e = qq;
                        }
                    }
                    if (lane == 0) sh.X[i] = ent_i;
                }
                if (lane == 0) sh.e_end = e;
            }
            __syncthreads();
        }
        // the chain's attempts in the segment, from its entry
        unsigned long long C = 0;
        if (tid < nseg && sh.X[tid] >= 0) {
            const int s0 = 64 * tid, se = min(s0 + 64, Rz);
            for (int q = s0 + sh.X[tid]; q < se; q += 4 + sh.len[q]) C |= 1ull << (q - s0);
        }
        const int e_end = sh.e_end;
        // 3. checkSubset of the segment's chain attempts
        unsigned long long PM = 0;
        for (unsigned long long m = C; m; m &= m - 1) {
            const int bit = ctz64(m), q = 64 * tid + bit;
            unsigned u[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) u[k] = sh.idx[q + k];
            int a[4];
            if (first4_distinct(u, a) == 0) {  // more than 16 draws (staged: the length was <= 67)
                int c = 1, k = q + 16;
                while (c < 4) {
                    const int v = sh.idx[k++];
                    if (v == a[0] || (c > 1 && v == a[1]) || (c > 2 && v == a[2])) continue;
                    a[c++] = v;
                }
            }
            const float4 A0 = sh.P[a[0]], A1 = sh.P[a[1]], A2 = sh.P[a[2]], A3 = sh.P[a[3]];
            const float s4[8] = {A0.x, A0.y, A1.x, A1.y, A2.x, A2.y, A3.x, A3.y};
            const float t4[8] = {A0.z, A0.w, A1.z, A1.w, A2.z, A2.w, A3.z, A3.w};
            PM |= (unsigned long long)(check_subset(s4, t4) ? 1 : 0) << bit;
        }
        __syncthreads();
        // 4. ranks: attempts A (chain order) and passes B before this segment
        int Tr, Pt;
        const int A = block_excl_sum(__popcll(C), sh.wred, Tr);
        const int B = block_excl_sum(__popcll(PM), sh.wred, Pt);
        const int first_ord = PM ? A + __popcll(C & ((PM & -PM) - 1)) : BIG;
        const int last_ord = PM ? A + __popcll(C & (~0ull >> clz64(PM))) - 1 : -1;
        const int a_p = min(block_min(first_ord, sh.wred2), Tr);
        int last_all;
        block_excl_max(last_ord, -1, sh.wred2, last_all);
        const int need = target - produced;
        const int af = fail_run + a_p >= 10000 ? 10000 - fail_run - 1 : BIG;  // the 10000th rejection
        int keep;
        bool hit_t = false, hit_f = false;
        if (af < BIG) {
            keep = 0;
            hit_f = true;
        } else if (Pt >= need) {
            keep = need;
            hit_t = true;
        } else {
            keep = Pt;
        }
        // samples of the kept passes, and the position of the attempt the round stops at
        if (tid == 0) sh.q_sel = -1;
        __syncthreads();
        {
            int r = B;
            for (unsigned long long m = PM; m && r < keep; m &= m - 1, ++r) {
                const int q = 64 * tid + ctz64(m);
                out[produced + r] = make_int4((int)(pos + q), sh.len[q] ? -2 : -1, 0, 0);
                if (hit_t && r == need - 1) sh.q_sel = q;
            }
            if (hit_f && A <= af && af < A + __popcll(C)) {
                unsigned long long m = C;
                for (int k = af - A; k > 0; --k) m &= m - 1;
                sh.q_sel = 64 * tid + ctz64(m);
            }
        }
        __syncthreads();
        if (hit_t || hit_f) {
            const int q = sh.q_sel;
            pos += q + 4 + sh.len[q];
            produced += keep;
            fail_run = hit_t ? 0 : 10000;
            if (hit_f) S.fail_iter = produced;  // getSubset returned false in this iteration
            stop_all = true;
        } else {
            produced += Pt;
            fail_run = Pt > 0 ? Tr - 1 - last_all : fail_run + Tr;
            pos += e_end;
        }
        __syncthreads();  // sh.idx / sh.len / sh.V are restaged by the next round
    }
    if (tid == 0) {
        S.stream_pos = pos;
        S.produced = produced;
        S.fail_run = fail_run;
        store_sampler_state(st + p, S);
    }
}

// ------------------------------------------------------------------------------------------------
// sample: walk the chain of getSubset attempts with the outcomes precomputed by
// ransac_attempt_kernel; reproduces getSubset's redraw-on-repeat, the checkSubset rejections and
// the 10000-attempt failure exactly (ptsetreg.cpp).
//
// The attempt flags stream through a 16 KiB LDS window.  A round reads 1 KiB of it (16 bytes per
// lane: stream positions wb+16l .. wb+16l+15) and walks every attempt of the chain inside that
// span: attempts start 4 draws apart (residue rho mod 4) until one redraws repeated indices, after
// which the walk continues in the residue it lands on (a sub-round).  All bookkeeping is done on
// ballot masks in scalar registers: attempt a = 4*lane + i of a sub-round is bit `lane` of mask i.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ransac_sample_kernel(RansacState* __restrict__ st,
                                                           const ProbDev* __restrict__ probs,
                                                           const float4* __restrict__ pts,
                                                           const uint32_t* __restrict__ stream, long long slen,
                                                           int4* __restrict__ samples, int c1,
                                                           int* __restrict__ err, const uint8_t* __restrict__ flags,
                                                           const uint8_t* __restrict__ ibits, int wcap, int after_chain) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kFlagWin];
    constexpr int BIG = 1 << 30;
    const int p = blockIdx.x, lane = threadIdx.x;
    RansacState S = st[p];
    if (!S.active || S.done || S.fail_iter != -1 || S.n < kSmallMaxN) return;  // small: ransac_small_kernel
    const int target = min(c1, S.niters);
    if (S.produced >= target) return;
    // resume where ransac_chain_kernel stopped; flags[rel] is the attempt starting at wbase + rel
    const long long wbase = after_chain ? S.win_base : S.stream_pos;
    const int wlen = after_chain ? S.win_len : window_len(S, c1, wcap);
    const uint8_t* F = flags + (long long)p * wcap;
    const uint8_t* IB = ibits + (long long)p * (wcap >> 3);
    const unsigned N = (unsigned)S.n;
    const unsigned long long M = S.modM;
    const float4* P = pts + probs[p].good_off;
    int4* out = samples + probs[p].it_off;
    long long rel = S.stream_pos - wbase;  // next attempt, relative to wbase
    long long lb = -(1LL << 40);
    int produced = S.produced, fail_run = S.fail_run;
    bool stop_all = false;
    // (re)load the LDS window of flags at relative position `at` (16-byte aligned), every lane
    auto refill = [&](long long at) {
        lb = at;
        __syncthreads();
#pragma unroll 4
        for (int j = 0; j < kFlagWin / 1024; ++j) {
            const long long r0 = lb + 16LL * (lane + 64 * j);
            uint4 v;
            if (r0 + 16 <= wlen) {
                // the flag bytes of the irregular positions, kPassUnknown for the others (their bytes
                // are not written: ransac_attempt_kernel)
                const unsigned ib = *reinterpret_cast<const uint16_t*>(IB + (r0 >> 3));
                if (ib == 0) {
                    v = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
                } else {
                    uint32_t w4[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        uint32_t w = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            w |= (uint32_t)((ib >> (4 * k + b)) & 1 ? F[r0 + 4 * k + b] : kPassUnknown) << (8 * b);
                        w4[k] = w;
                    }
                    v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                }
            } else {
                // past the precomputed window: the redraw lengths computed here (pass bits unknown)
                uint32_t w4[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    uint32_t w = 0;
                    for (int b = 0; b < 4; ++b) {
                        const long long r = r0 + 4 * k + b;
                        const int fr = r < wlen ? (((IB[r >> 3] >> (r & 7)) & 1) ? F[r] : kPassUnknown)
                                                : length_flag(wbase + r, stream, slen, N, M);
                        w |= (uint32_t)fr << (8 * b);
                    }
                    w4[k] = w;
                }
                v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            }
            *reinterpret_cast<uint4*>(win + 16 * (lane + 64 * j)) = v;
        }
        __syncthreads();
    };
    while (!stop_all && produced < target) {
        const long long wb = rel & ~15LL;
        if (wb < lb || wb + 1024 > lb + kFlagWin) refill(wb);  // refill the LDS window at wb
        const uint4 w = *reinterpret_cast<const uint4*>(win + (wb - lb) + 16 * lane);
        const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
        long long s = rel;  // chain position inside [wb, wb + 1024)
        while (s < wb + 1024) {
            const int rho = (int)(s - wb) & 3;
            const int a0 = (int)(s - wb) >> 2;  // first attempt of this sub-round (a = 4 lane + i)
            int f[4];
            unsigned long long I[4], Pm[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int a = 4 * lane + i;
                int fi = (int)((wd[i] >> (8 * rho)) & 0xFF);
                                // outside the window, or checkSubset not evaluated yet (kPassUnknown): evaluate here
                if (a >= a0 && (fi == kFlagUnknown || (fi != kAttemptSerial && (fi & kPassUnknown))))
                    fi = attempt_flag(wbase + wb + 4LL * a + rho, stream, slen, N, M, P);
                f[i] = fi;
                const bool irr = fi == kAttemptSerial || (fi >> 1) != 0;
                I[i] = __ballot(a >= a0 && irr);
                Pm[i] = __ballot(a >= a0 && !irr && (fi & 1));
            }
            // first attempt whose length is not 4 draws (or must be resolved here)
            int afc = 256;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (I[i]) afc = min(afc, 4 * ctz64(I[i]) + i);
            long long endfc = 0;  // chain position after the afc attempt
            int fcpass = 0, fcres = 0;
            if (afc < 256) {
                const int fsel = uni(__shfl(f[afc & 3], afc >> 2));
                const long long qfc = wb + 4LL * afc + rho;
                if (fsel != kAttemptSerial) {
                    endfc = qfc + 4 + (fsel >> 1);
                    fcpass = fsel & 1;
                    fcres = 1;
                } else {  // resolve here (stream end or a very long redraw run)
                    int idx[4] = {0, 0, 0, 0};
                    const int len = resolve_at(wbase + qfc, stream, slen, N, M, idx);
                    if (len == 0) {  // RNG stream exhausted: report, never guess
                        if (lane == 0) atomicOr(err, 1);
                        S.fail_iter = -2;
                        stop_all = true;
                        break;
                    }
                    const float4 a = P[idx[0]], b = P[idx[1]], c = P[idx[2]], d = P[idx[3]];
                    const float s4[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
                    const float t4[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
                    fcpass = uni(check_subset(s4, t4) ? 1 : 0);
                    fcres = uni(len != 4);
                    endfc = uni64(qfc + len);
                }
                // keep only passes before afc, then add afc itself
                const int L = afc >> 2, e = afc & 3;
                const unsigned long long below = L ? (~0ull >> (64 - L)) : 0ull;  // lanes < L
#pragma unroll
                for (int i = 0; i < 4; ++i) Pm[i] &= (i < e) ? (below | (1ull << L)) : below;
                if (fcpass) Pm[e] |= 1ull << L;
            }
            const int end = afc < 256 ? afc + 1 : 256;  // attempts a0 .. end-1 are walked
            int tot = 0, a_p = BIG, a_lp = -1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                tot += __popcll(Pm[i]);
                if (Pm[i]) {
                    a_p = min(a_p, 4 * ctz64(Pm[i]) + i);
                    a_lp = max(a_lp, 4 * (63 - clz64(Pm[i])) + i);
                }
            }
            unsigned bits = 0;
            int E = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                bits |= (unsigned)((Pm[i] >> lane) & 1ull) << i;
                E += mbcnt64(Pm[i]);
            }
            const int need = target - produced;
            int at = BIG;  // attempt completing the chunk's last wanted iteration
            if (tot >= need) {
                const unsigned long long hm = __ballot(E < need && need <= E + __popc(bits));
                const int Lh = ctz64(hm);
                const unsigned hb = (unsigned)uni(__shfl((int)bits, Lh));
                int k = need - uni(__shfl(E, Lh));
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (((hb >> i) & 1) && --k == 0) at = 4 * Lh + i;
            }
            const int fails_before = (a_p < BIG ? a_p : end) - a0;
            const int af = fail_run + fails_before >= 10000 ? a0 + (10000 - fail_run - 1) : BIG;  // 10000th failure
            int stop = end - 1, got = tot;
            bool hit_t = false, hit_f = false;
            if (at < BIG && at < af) { stop = at; hit_t = true; got = need; }
            else if (af < BIG) { stop = af; hit_f = true; got = 0; }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int a = 4 * lane + i;
                if (((bits >> i) & 1) && a <= stop) {
                    const int rank = E + __popc(bits & ((1u << i) - 1));
                    out[produced + rank] = make_int4((int)(wbase + wb + 4LL * a + rho), (a == afc && fcres) ? -2 : -1, 0, 0);
                }
            }
            produced += got;
            fail_run = hit_t ? 0 : (hit_f ? 10000 : (tot > 0 ? stop - a_lp : fail_run + (end - a0)));
            s = uni64(stop == afc ? endfc : wb + 4LL * (stop + 1) + rho);
            if (hit_f) {
                S.fail_iter = produced;  // getSubset returned false in this iteration
                stop_all = true;
                break;
            }
            if (hit_t) { stop_all = true; break; }
        }
        rel = uni64(s);
    }
    if (lane == 0) {
        S.stream_pos = wbase + rel;
        S.produced = produced;
        S.fail_run = fail_run;
        store_sampler_state(st + p, S);
    }
}

// ------------------------------------------------------------------------------------------------
// hypo: runKernel on each minimal sample, one lane per iteration (bit-exact fp64)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ransac_hypo_kernel(const RansacState* __restrict__ st,
                                                         const ProbDev* __restrict__ probs,
                                                         const float4* __restrict__ pts,
                                                         const int4* __restrict__ samples,
                                                         const uint32_t* __restrict__ stream,
                                                         float* __restrict__ hyp, int* __restrict__ counts, int c0,
                                                         int c1, int bpp) {
    __shared__ double sd[kJ9D * 64];
    const int p = blockIdx.x / bpp, lane = threadIdx.x;
    const int it = c0 + (blockIdx.x % bpp) * 64 + lane;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    if (it >= c1 || it >= S.produced) return;
    const long long o = probs[p].it_off + it;
    const float4* P = pts + probs[p].good_off;
    const int4 s4 = decode_sample(samples[o], stream, (unsigned)S.n, S.modM);
    const float4 a = P[s4.x], b = P[s4.y], c = P[s4.z], d = P[s4.w];
    const float M[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
    const float m[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
    double H[9];
    const int ok = run_kernel4<64>(M, m, sd + lane, H);
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
// Filtered path (default).  Deciding the RANSAC trajectory only needs, per iteration, whether the
// exact inlier count beats max(best, 3).  `bound` brackets every count from a closed-form fp64
// homography through the same 4 correspondences (Heckbert's square->quad maps), with a per-point
// margin on the reprojection error that is orders of magnitude above the disagreement between that
// solution and OpenCV's normalized-DLT/Jacobi one for any sample that passes the conditioning
// screen; samples that fail the screen get [0, N].  `select_filtered` then evaluates exactly —
// OpenCV's runKernel + computeError, bit for bit — only the iterations whose upper bound can
// exceed the running best, and replays them in order.  tests/test_ransac_gpu.py checks the
// filtered and the all-exact paths produce identical results.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void square_to_quad(const double* x, const double* y, double* Q) {
    const double sx = x[0] - x[1] + x[2] - x[3], sy = y[0] - y[1] + y[2] - y[3];
    const double dx1 = x[1] - x[2], dx2 = x[3] - x[2], dy1 = y[1] - y[2], dy2 = y[3] - y[2];
    const double iden = 1.0 / (dx1 * dy2 - dx2 * dy1);  // one division: g, h within an ulp of the quotients
    const double g = (sx * dy2 - sy * dx2) * iden, h = (dx1 * sy - dy1 * sx) * iden;
    Q[0] = x[1] - x[0] + g * x[1]; Q[1] = x[3] - x[0] + h * x[3]; Q[2] = x[0];
    Q[3] = y[1] - y[0] + g * y[1]; Q[4] = y[3] - y[0] + h * y[3]; Q[5] = y[0];
    Q[6] = g; Q[7] = h; Q[8] = 1.0;
}

// min over the 4 triangles of |2*area| / bbox_diag^2 (conditioning of a 4-point configuration)
__device__ __forceinline__ double min_rel_area(const double* x, const double* y) {
    const double mnx = fmin(fmin(x[0], x[1]), fmin(x[2], x[3])), mxx = fmax(fmax(x[0], x[1]), fmax(x[2], x[3]));
    const double mny = fmin(fmin(y[0], y[1]), fmin(y[2], y[3])), mxy = fmax(fmax(y[0], y[1]), fmax(y[2], y[3]));
    const double d2 = (mxx - mnx) * (mxx - mnx) + (mxy - mny) * (mxy - mny);
    const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    double m = 1e300;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a = tt[i][0], b = tt[i][1], c = tt[i][2];
        m = fmin(m, fabs((x[b] - x[a]) * (y[c] - y[a]) - (x[c] - x[a]) * (y[b] - y[a])));
    }
    return d2 > 0 ? m / d2 : 0.0;
}

// Conditioning screen of the closed-form bound (rho = min relative triangle area of the sample).
// Model of the disagreement between the closed form and OpenCV's normalized-DLT eigenvector:
// eta ~ eps * kappa^2 with kappa ~ 1/rho (normal equations), taken ~100x larger: eta = 1e-14/rho^2.
// A relative model error eta moves a reprojection error e <= 25.5 px^2 by <= 10.2*eta*s + (eta*s)^2
// (s = |x|+|y|+|u|+|v| of the point).  The base margin 0.5 + 1e-7 s^2 (which also absorbs the fp32
// rounding of both error evaluations) dominates 10.2*eta*s for every s once eta <= 4.4e-5, i.e.
//   rho >= 2e-5        base margin only
//   1e-7 <= rho < 2e-5 margin widened by 10.2*eta*s + (eta*s)^2 (rare: ~6e-4 of random samples)
//   rho < 1e-7         no bound: [0, N] (the iteration is evaluated exactly)
constexpr double kScreenArea = 1e-7;
constexpr double kScreenTight = 2e-5;

// Closed-form hypothesis of the bound kernels for the sample s4: Hd = H / H[8] (fp64); invalid =
// runKernel's degeneracy test; uncertain = no usable bound (conditioning screen, H[8] ~ 0, non-finite);
// eta > 0 widens the margin (poorly conditioned samples).
__device__ __forceinline__ void bound_hypothesis(const float4* __restrict__ P, int4 s4, double (&Hd)[8],
                                                 bool& invalid, bool& uncertain, float& eta, double& eta_model) {
    const float4 q0 = P[s4.x], q1 = P[s4.y], q2 = P[s4.z], q3 = P[s4.w];
    // runKernel's own degeneracy test (exact, cheap): spread < DBL_EPSILON -> no model
    const float M[8] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
    const float m[8] = {q0.z, q0.w, q1.z, q1.w, q2.z, q2.w, q3.z, q3.w};
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        cmx += m[2 * i]; cmy += m[2 * i + 1];
        cMx += M[2 * i]; cMy += M[2 * i + 1];
    }
    cmx /= 4; cmy /= 4; cMx /= 4; cMy /= 4;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        smx += fabs(m[2 * i] - cmx); smy += fabs(m[2 * i + 1] - cmy);
        sMx += fabs(M[2 * i] - cMx); sMy += fabs(M[2 * i + 1] - cMy);
    }
    invalid = fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON ||
              fabs(sMy) < DBL_EPSILON;
    const double sx[4] = {q0.x, q1.x, q2.x, q3.x}, sy[4] = {q0.y, q1.y, q2.y, q3.y};
    const double dx[4] = {q0.z, q1.z, q2.z, q3.z}, dy[4] = {q0.w, q1.w, q2.w, q3.w};
    const double rho = fmin(min_rel_area(sx, sy), min_rel_area(dx, dy));
    uncertain = !(rho >= kScreenArea);
    eta_model = 1e-14 / (rho * rho);  // the disagreement model at this sample's conditioning
    if (rho < kScreenTight) eta = (float)eta_model;
    double Qs[9], Qd[9], Ai[9], H[9];
    square_to_quad(sx, sy, Qs);
    square_to_quad(dx, dy, Qd);
    // adjugate of Qs (inverse up to scale)
    Ai[0] = Qs[4] * Qs[8] - Qs[5] * Qs[7]; Ai[1] = Qs[2] * Qs[7] - Qs[1] * Qs[8]; Ai[2] = Qs[1] * Qs[5] - Qs[2] * Qs[4];
    Ai[3] = Qs[5] * Qs[6] - Qs[3] * Qs[8]; Ai[4] = Qs[0] * Qs[8] - Qs[2] * Qs[6]; Ai[5] = Qs[2] * Qs[3] - Qs[0] * Qs[5];
    Ai[6] = Qs[3] * Qs[7] - Qs[4] * Qs[6]; Ai[7] = Qs[1] * Qs[6] - Qs[0] * Qs[7]; Ai[8] = Qs[0] * Qs[4] - Qs[1] * Qs[3];
    mat3_mul(Qd, Ai, H);
    double hmax = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) hmax = fmax(hmax, fabs(H[i]));
    uncertain |= !(fabs(H[8]) > 1e-9 * hmax);  // also catches NaN
    const double inv = 1.0 / H[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) Hd[i] = H[i] * inv;
#pragma unroll
    for (int i = 0; i < 8; ++i) uncertain |= !isfinite((float)Hd[i]);
}

// ------------------------------------------------------------------------------------------------
// Upper bounds on the matrix cores (chunks after the first).  Per (hypothesis, point) the box test
// needs ex = X - uW, ey = Y - vW and W: three dot products of length 6 between the hypothesis and
// the point, i.e. three small GEMMs [points x 16] x [16 x hypotheses] on v_mfma_f32_32x32x16_f16.
// Coordinates are scaled by powers of two into [-1, 1] (x' = sa x, u' = sb u, exact), the
// hypothesis H' = diag(sb, sb, 1) H diag(1/sa, 1/sa, 1) by a power of two into [-1, 1] (h8 = 2^-e
// exact in f16 for e <= 24), and every factor is split into f16 hi + lo: a*b ~ ah*bh + ah*bl +
// al*bh, so each of the six products takes 3 K-slots (2 for the factors that are exact: 1 and h8):
//   point   ax = [xh xl xh  yh yl yh  1 1 | uxh uxl uxh  uyh uyl uyh  uh ul]
//   hyp     bx = [h0h h0h h0l  h1h h1h h1l  h2h h2l | -h6h -h6h -h6l  -h7h -h7h -h7l  -h8 -h8]
//   (ay, by: v and h3 h4 h5; W = ax . [h6h h6h h6l h7h h7h h7l h8 0 | 0 ...]).
// Error of each computed quantity (|factors| <= 1, f16 split 2^-22 per factor and 2^-22 per dropped
// al*bl, fp32 products u'x' 2^-24, fp32 accumulation of <= 16 terms of total magnitude <= 6):
// < 1e-5 in these units; kMfmaErr = 2^-15 = 3.05e-5.  A point is outside only if
//   |ex| + |ey| > C |W| + (2 + C) kMfmaErr,  C = sqrt 2 sb sqrt(thr2 + d_max (+ widening)) (1 + 1e-6)
// with d_max the largest per-point margin of the problem, so the count of the rest bounds the
// exact inlier count from above ("Exactness of the filtered RANSAC").
// MI355X MFMA keeps f16 subnormal operands (tools/probe/f16_probe.hip).
// ------------------------------------------------------------------------------------------------
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16acc __attribute__((ext_vector_type(16)));
constexpr float kMfmaErr = 0x1p-15f;
// the bound kernel's fragments: points (ransac_tiles_kernel) and hypotheses each times 2^15, so its
// MFMA outputs are K = 2^30 times the quantities above
constexpr float kPointScale = 0x1p15f;
constexpr double kHypScale = 0x1p15;
constexpr double kOutScale = 0x1p30;
#ifndef MIM_BOUND_CHUNK
#define MIM_BOUND_CHUNK 8
#endif
#ifndef MIM_BOUND_WAVES
#define MIM_BOUND_WAVES 4
#endif
constexpr int kBoundThreads = 64 * MIM_BOUND_WAVES;  // iterations per MFMA bound block (64 per wave)
constexpr int kTileChunk = MIM_BOUND_CHUNK;  // 32-point tiles per LDS stage of the MFMA bound kernel (2 x 16 KiB)

// clamp to [0, 1]: folds into the producing instruction's clamp bit (no NaN reaches it here)
__device__ __forceinline__ float clamp01(float x) { return __builtin_amdgcn_fmed3f(x, 0.f, 1.f); }

// hi + lo = a to 2^-22 relative, with hi = (f16)a and lo = (f16)(a - hi) taken from the SAME value a.
// `a` is pinned in a register first: given split_f16(u * x), the compiler otherwise forms
// hi = v_fma_mixlo_f16(u, x, 0) (the exact product rounded once to f16) next to a - hi from the fp32
// product; where the fp32 product is an f16 rounding tie the two hi differ by one f16 ulp and hi + lo
// is off by 2^-11 relative (found by tests/test_bounds_corpus_gpu.py: a missed upper bound).
__device__ __forceinline__ void split_f16(float a, _Float16& hi, _Float16& lo) {
    asm volatile("" : "+v"(a));
    hi = (_Float16)a;
    lo = (_Float16)(a - (float)hi);  // a - hi is exact in fp32
}
__device__ __forceinline__ void split_f16(double a, _Float16& hi, _Float16& lo) {
    float af = (float)a;
    asm volatile("" : "+v"(af));
    hi = (_Float16)af;
    lo = (_Float16)(float)(a - (double)(float)hi);
}

// Point tiles of every active problem, once per batch: scales, then per 32-point tile the A-operand
// fragments of lane l (row l & 31, k = 8 (l >> 5) .. + 7) for ax and ay.  Rows past n are zero.
__global__ __launch_bounds__(256) void ransac_tiles_kernel(RansacState* __restrict__ st,
                                                           const ProbDev* __restrict__ probs,
                                                           const float4* __restrict__ pts,
                                                           uint4* __restrict__ tiles) {
    __shared__ float red[3][4];
    const int p = blockIdx.x, tid = threadIdx.x;
    RansacState* Sp = st + p;
    if (!Sp->active || Sp->done) return;
    const int n = Sp->n;
    const long long go = probs[p].good_off;  // multiple of 32 (build_tables)
    const float4* __restrict__ P = pts + go;
    float mxy = 0.f, muv = 0.f, ms = 0.f;
    for (int i = tid; i < n; i += 256) {
        const float4 q = P[i];
        mxy = fmaxf(mxy, fmaxf(fabsf(q.x), fabsf(q.y)));
        muv = fmaxf(muv, fmaxf(fabsf(q.z), fabsf(q.w)));
        ms = fmaxf(ms, fabsf(q.x) + fabsf(q.y) + fabsf(q.z) + fabsf(q.w));
    }
    for (int off = 32; off >= 1; off >>= 1) {
        mxy = fmaxf(mxy, __shfl_xor(mxy, off));
        muv = fmaxf(muv, __shfl_xor(muv, off));
        ms = fmaxf(ms, __shfl_xor(ms, off));
    }
    if ((tid & 63) == 0) {
        red[0][tid >> 6] = mxy;
        red[1][tid >> 6] = muv;
        red[2][tid >> 6] = ms;
    }
    __syncthreads();
    mxy = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    muv = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
    ms = fmaxf(fmaxf(red[2][0], red[2][1]), fmaxf(red[2][2], red[2][3]));
    int ea = 0, eb = 0;
    (void)frexpf(mxy, &ea);  // mxy < 2^ea
    (void)frexpf(muv, &eb);
    const float sa = ldexpf(1.f, -ea), sb = ldexpf(1.f, -eb);
    if (tid == 0) {
        Sp->sa = sa;
        Sp->sb = sb;
        Sp->smax = ms;
    }
    uint4* __restrict__ T = tiles + (go >> 5) * 128;
    const int nt = (n + 31) >> 5;
    // the fragments carry kPointScale = 2^15 (|x'| < 1, so every entry stays below 2^15 in f16)
    const _Float16 one = (_Float16)kPointScale;
    for (int i = tid; i < nt * 32; i += 256) {
        h8v lo = {}, axh = {}, ayh = {};
        if (i < n) {
            const float4 q = P[i];
            const float x = q.x * sa, y = q.y * sa, u = q.z * sb, v = q.w * sb;
            const float xk = x * kPointScale, yk = y * kPointScale, uk = u * kPointScale, vk = v * kPointScale;
            _Float16 a, b;
            split_f16(xk, a, b); lo[0] = a; lo[1] = b; lo[2] = a;
            split_f16(yk, a, b); lo[3] = a; lo[4] = b; lo[5] = a;
            lo[6] = one; lo[7] = one;
            split_f16(u * xk, a, b); axh[0] = a; axh[1] = b; axh[2] = a;
            split_f16(u * yk, a, b); axh[3] = a; axh[4] = b; axh[5] = a;
            split_f16(uk, a, b); axh[6] = a; axh[7] = b;
            split_f16(v * xk, a, b); ayh[0] = a; ayh[1] = b; ayh[2] = a;
            split_f16(v * yk, a, b); ayh[3] = a; ayh[4] = b; ayh[5] = a;
            split_f16(vk, a, b); ayh[6] = a; ayh[7] = b;
        }
        uint4* t = T + (i >> 5) * 128;
        const int r = i & 31;
        t[r] = __builtin_bit_cast(uint4, lo);        // ax, lanes 0-31
        t[32 + r] = __builtin_bit_cast(uint4, axh);  // ax, lanes 32-63
        t[64 + r] = __builtin_bit_cast(uint4, lo);   // ay, lanes 0-31
        t[96 + r] = __builtin_bit_cast(uint4, ayh);  // ay, lanes 32-63
    }
}

// Upper bounds of the inlier counts of 256 consecutive iterations per block (64 per wave: two
// column blocks of 32 hypotheses), the point tiles staged through LDS and shared by the 4 waves.
// Both bounds test the L1 norm |ex| + |ey| (a diamond: the same area as the box max(|ex|, |ey|) of
// rounds 2-4 around the same disc, so as tight, and v_add/v_sub with |.| operands issue at the
// fp32 rate where the max / med3 issues ~1.5x slower, tools/issue_probe.hip).
// Upper bound: a point can be an inlier only if
//   |ex| + |ey| <= C |W| + (C + 2) kMfmaErr + 2 A,  C = sqrt 2 sb sqrt(thr2 + d_max (+ widening)),
// since (|ex| - A, |ey| - A) lies in the disc of radius C |W| / sqrt 2 and each MFMA output is
// within kMfmaErr.  kLo (first chunk) also a lower bound from the diamond inscribed in the inner
// disc, |ex| + |ey| < C_lo |W| - (C_lo + 2) kMfmaErr - 2 A, C_lo = sb sqrt(thr2 - d_max (- widening)),
// which implies ex^2 + ey^2 < (thr2 - d) W^2 for every point's margin d <= d_max.
// A (both bounds): absolute slack on |X - uW|, |Y - vW| for OpenCV's own fp32 evaluation of
// computeError and the closed-form/eigenvector disagreement, which the relative margin d cannot
// cover near the hypothesis' horizon (|W| -> 0): X and W each carry an absolute error of
// gamma * (sum of |terms|), gamma = 4 ulp(1/2) (float cast of H, product, two sums) + eta, so
// |X_c/W_c - u| moves by <= (err_X + (|u| + 6) err_W) / |W|, i.e. |ex| by <= A.
// Counting (round 5): the point and the hypothesis fragments each carry a factor 2^15, so every MFMA
// output is K = kOutScale = 2^30 times the quantity above (X' = K ex, ...; exact: powers of two,
// every fragment stays below 2^15 in f16, and the split's error only shrinks relative to the
// outputs), and each (point, hypothesis) pair adds u = clamp(C |W'| + (K E + 1) - |X'| - |Y'|) to a
// float count: exactly 1 for every point the test keeps (C and E carry 1e-6 relative slack, above the
// three roundings' 2^-22 of C |W'| + K E + 1 >= 3, so the value cannot fall below 1), 0 past the
// diamond widened by 1/K (2^-30 in the scaled units: no wider in practice), a fraction only there.
// That is four fast-rate VALU per pair (fma, sub, sub with clamp, add) where the sign bit took a
// v_alignbit and a v_bcnt at the slow rate; hi = floor(sum + slack) - padded rows, slack bounding
// the float sum's rounding.  The lower bound adds clamp(C_lo |W'| - K E_lo - (|X'| + |Y'|)), positive
// only where the point is surely in, so lo = ceil(sum - slack) never exceeds the exact count.
template <bool kLo>
__global__ __launch_bounds__(kBoundThreads) void ransac_bound_mfma_kernel(const RansacState* __restrict__ st,
                                                                const ProbDev* __restrict__ probs,
                                                                const float4* __restrict__ pts,
                                                                const int4* __restrict__ samples,
                                                                const uint32_t* __restrict__ stream,
                                                                const uint4* __restrict__ tiles,
                                                                int2* __restrict__ bounds, int c0, int c1, int bpp,
                                                                float thr2, int n_probs) {
    __shared__ uint4 lt[2][kTileChunk * 128];
    // XCD-aware order: blocks b and b + 8 share an XCD under round-robin dispatch (speed only), so
    // problem p's blocks are the ones with b % 8 == p % 8 and its point tiles are fetched into one
    // XCD's L2 instead of eight (grid: 8 x ceil(n_probs / 8) x bpp, blocks past n_probs idle)
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int p = xcd + 8 * (j / bpp), kb = j % bpp;
    if (p >= n_probs) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int it = c0 + kb * kBoundThreads + tid;
    const RansacState S = st[p];
    if (!S.active || S.done) return;  // uniform over the block
    if (c0 + kb * kBoundThreads >= min(c1, S.produced)) return;  // whole block idle
    const bool act = it < c1 && it < S.produced;
    const long long o = probs[p].it_off + it;
    const long long go = probs[p].good_off;
    const float4* __restrict__ P = pts + go;
    const int n = S.n;
    bool uncertain = false, invalid = false;
    float eta = 0.f;
    double Hd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double eta_model = 0;
    if (act) {
        const int4 s4 = decode_sample(samples[o], stream, (unsigned)n, S.modM);
        bound_hypothesis(P, s4, Hd, invalid, uncertain, eta, eta_model);
    }
    // H' in scaled coordinates, then scaled by 2^-e into [-1, 1] (sa, sb are powers of two, so their
    // reciprocals and quotient are exact and the divisions become multiplications, bit for bit)
    const double isa = ldexp(1.0, -ilogb((double)S.sa)), rs = (double)S.sb * isa;
    double h[9] = {Hd[0] * rs, Hd[1] * rs, Hd[2] * S.sb, Hd[3] * rs, Hd[4] * rs, Hd[5] * S.sb,
                   Hd[6] * isa, Hd[7] * isa, 1.0};
    double hm = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) hm = fmax(hm, fabs(h[i]));
    int e = 0;
    (void)frexp(hm, &e);  // hm < 2^e, e >= 1 (h8 = 1)
    uncertain |= e > 24;  // h8 = 2^-e would not be an f16
    const bool count = act && !invalid && !uncertain;
    const double sc = ldexp(1.0, -e);
#pragma unroll
    for (int i = 0; i < 9; ++i) h[i] *= sc;
    // the fragments carry 2^15 on top (|h 2^15| < 2^15: f16 range), h[8] 2^15 = 2^(15 - e) exact
    double hk[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) hk[i] = h[i] * kHypScale;
    // per-hypothesis box constants (d_max and, for poorly conditioned samples, the widening at smax)
    float tt = thr2 + fmaf(1e-7f * S.smax, S.smax, 0.5f);
    if (eta > 0.f) tt += S.smax * fmaf(eta * eta, S.smax, 10.2f * eta);
    const float C = S.sb * sqrtf(tt) * 1.41421366f * (1.f + 1e-6f);  // sqrt 2 rounded up
    // near-horizon slack A (pixel units, |x|, |y| < 1/sa and |u|, |v| < 1/sb), in the scaled units of
    // the MFMA outputs, with the sample's modelled closed-form/eigenvector disagreement eta_model
    const double mx = isa, mu = ldexp(1.0, -ilogb((double)S.sb));
    const double gam = 4.0 * 0x1p-24 + fmin(eta_model, 1.0);
    const double ax = fmax((fabs(Hd[0]) + fabs(Hd[1])) * mx + fabs(Hd[2]), (fabs(Hd[3]) + fabs(Hd[4])) * mx + fabs(Hd[5]));
    const double aw = (fabs(Hd[6]) + fabs(Hd[7])) * mx + 1.0;
    const float A = (float)(gam * (ax + (mu + 6.0) * aw) * S.sb * sc * (1.0 + 1e-6));
    const float E = ((2.f + C) * kMfmaErr + 2.f * A) * (1.f + 1e-6f);
    float CL = 0.f, EL = 0.f;
    if (kLo) {
        float tl = thr2 - fmaf(1e-7f * S.smax, S.smax, 0.5f);
        if (eta > 0.f) tl -= S.smax * fmaf(eta * eta, S.smax, 10.2f * eta);
        // diamond inscribed in the disc of radius sqrt(tl): |ex| + |ey| <= sqrt(tl) |W| (two
        // coordinates' errors 2 (kMfmaErr + A) beside C_lo kMfmaErr from |W|), sharing the upper
        // bound's |ex| + |ey|
        CL = S.sb * sqrtf(fmaxf(tl, 0.f)) * (1.f - 1e-6f);
        EL = ((CL + 2.f) * kMfmaErr + 2.f * A) * (1.f + 1e-6f);
    }
    // B-operand fragments of the own hypothesis: k 0-7 (bx, by, bw) and k 8-15 (shared by bx, by)
    h8v fx = {}, fy = {}, fw = {}, fn = {};
    if (count) {
        _Float16 a, b;
        split_f16(hk[0], a, b); fx[0] = a; fx[1] = a; fx[2] = b;
        split_f16(hk[1], a, b); fx[3] = a; fx[4] = a; fx[5] = b;
        split_f16(hk[2], a, b); fx[6] = a; fx[7] = b;
        split_f16(hk[3], a, b); fy[0] = a; fy[1] = a; fy[2] = b;
        split_f16(hk[4], a, b); fy[3] = a; fy[4] = a; fy[5] = b;
        split_f16(hk[5], a, b); fy[6] = a; fy[7] = b;
        split_f16(hk[6], a, b); fw[0] = a; fw[1] = a; fw[2] = b;
        split_f16(hk[7], a, b); fw[3] = a; fw[4] = a; fw[5] = b;
        fw[6] = (_Float16)(float)hk[8];  // 2^(15 - e): exact
        fn = -fw;
        fn[7] = fn[6];
    }
    // column block 0 = hypotheses (lanes) 0-31, block 1 = 32-63; lane l holds column l & 31 at
    // k = 8 (l >> 5) .. + 7, so half the fragments come from the partner lane l ^ 32:
    // low lanes need the partner's fx, fy, fw (block 1), high lanes the partner's fn (block 0)
    const bool lowh = lane < 32;
    const uint4 ux = __builtin_bit_cast(uint4, fx), uy = __builtin_bit_cast(uint4, fy);
    const uint4 uw = __builtin_bit_cast(uint4, fw), un = __builtin_bit_cast(uint4, fn);
    const uint4 s1 = lowh ? un : ux;
    uint4 r1, r2, r3;
    r1.x = __shfl_xor(s1.x, 32); r1.y = __shfl_xor(s1.y, 32); r1.z = __shfl_xor(s1.z, 32); r1.w = __shfl_xor(s1.w, 32);
    r2.x = __shfl_xor(uy.x, 32); r2.y = __shfl_xor(uy.y, 32); r2.z = __shfl_xor(uy.z, 32); r2.w = __shfl_xor(uy.w, 32);
    r3.x = __shfl_xor(uw.x, 32); r3.y = __shfl_xor(uw.y, 32); r3.z = __shfl_xor(uw.z, 32); r3.w = __shfl_xor(uw.w, 32);
    const uint4 zero4 = make_uint4(0, 0, 0, 0);
    const h8v b0x = __builtin_bit_cast(h8v, lowh ? ux : r1);
    const h8v b0y = __builtin_bit_cast(h8v, lowh ? uy : r1);
    const h8v b0w = __builtin_bit_cast(h8v, lowh ? uw : zero4);
    const h8v b1x = __builtin_bit_cast(h8v, lowh ? r1 : un);
    const h8v b1y = __builtin_bit_cast(h8v, lowh ? r2 : un);
    const h8v b1w = __builtin_bit_cast(h8v, lowh ? r3 : zero4);
    // in output units: K E + 1 (the band outside the upper test) and -K E_lo
    const float EK = fmaf(E, (float)kOutScale, 1.f), ELK = -EL * (float)kOutScale;
    const float Cp = __shfl_xor(C, 32), Ep = __shfl_xor(EK, 32);
    const float C0 = lowh ? C : Cp, E0 = lowh ? EK : Ep, C1 = lowh ? Cp : C, E1 = lowh ? Ep : EK;
    float CL0 = 0.f, EL0 = 0.f, CL1 = 0.f, EL1 = 0.f;
    if (kLo) {
        const float CLp = __shfl_xor(CL, 32), ELp = __shfl_xor(ELK, 32);
        CL0 = lowh ? CL : CLp; EL0 = lowh ? ELK : ELp; CL1 = lowh ? CLp : CL; EL1 = lowh ? ELp : ELK;
    }
    const bool wave_counts = __any(count);
    const uint4* __restrict__ T = tiles + (go >> 5) * 128;
    const int nt = (n + 31) >> 5;
    float keep0 = 0.f, keep1 = 0.f, in0 = 0.f, in1 = 0.f;  // float counts (see above)
    // point tiles through LDS by LDS-DMA in chunks of kTileChunk, double buffered: the next chunk's
    // pieces are in flight while this chunk is scored; one barrier per chunk
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto stage = [&](int t0, int buf) {
        const int tc = min(kTileChunk, nt - t0);
        for (int i0 = wv * 64; i0 < tc * 128; i0 += kBoundThreads)
            __builtin_amdgcn_global_load_lds((const void*)(T + (long long)t0 * 128 + i0 + lane),
                                             (__attribute__((address_space(3))) void*)(lt[buf] + i0), 16, 0, 0);
    };
#ifndef MIM_PROBE_BOUND
#define MIM_PROBE_BOUND 0  // timing probe only (wrong bounds): 1 = no tile arithmetic, 2 = no tile loop
#endif
    if (nt > 0) stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t0 = 0, buf = 0; t0 < (MIM_PROBE_BOUND == 2 ? 0 : nt); t0 += kTileChunk, buf ^= 1) {
        const int tc = min(kTileChunk, nt - t0);
        if (t0 + kTileChunk < nt) stage(t0 + kTileChunk, buf ^ 1);
        if (wave_counts && MIM_PROBE_BOUND == 0) {
          for (int t = 0; t < tc; ++t) {
            const h8v ax = __builtin_bit_cast(h8v, lt[buf][t * 128 + lane]);
            const h8v ay = __builtin_bit_cast(h8v, lt[buf][t * 128 + 64 + lane]);
            const f16acc zc = {};
            const f16acc ex0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax, b0x, zc, 0, 0, 0);
            const f16acc ey0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ay, b0y, zc, 0, 0, 0);
            const f16acc w0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax, b0w, zc, 0, 0, 0);
            const f16acc ex1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax, b1x, zc, 0, 0, 0);
            const f16acc ey1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ay, b1y, zc, 0, 0, 0);
            const f16acc w1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax, b1w, zc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (kLo) {  // the lower bound shares s = |X'| + |Y'|
                    const float s0 = fabsf(ex0[r]) + fabsf(ey0[r]);
                    const float s1 = fabsf(ex1[r]) + fabsf(ey1[r]);
                    keep0 += clamp01(fmaf(C0, fabsf(w0[r]), E0) - s0);
                    keep1 += clamp01(fmaf(C1, fabsf(w1[r]), E1) - s1);
                    in0 += clamp01(fmaf(CL0, fabsf(w0[r]), EL0) - s0);
                    in1 += clamp01(fmaf(CL1, fabsf(w1[r]), EL1) - s1);
                } else {
                    keep0 += clamp01((fmaf(C0, fabsf(w0[r]), E0) - fabsf(ex0[r])) - fabsf(ey0[r]));
                    keep1 += clamp01((fmaf(C1, fabsf(w1[r]), E1) - fabsf(ex1[r])) - fabsf(ey1[r]));
                }
            }
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of the next chunk landed
        __syncthreads();
    }
    // rows (points) of a column are split over lanes l and l ^ 32.  Rounding of the float counts: a
    // lane adds m = 16 nt values in [0, 1] in order, then the two lanes' sums are added: m additions
    // on the longest chain, so the computed sum s' is within gamma_m s of the exact sum s of the values
    // (recursive summation of nonnegative terms, gamma_m = m 2^-24 / (1 - m 2^-24)), and s <= s' + that,
    // so |error| <= 1.25 m 2^-24 (s' + 1) for m 2^-24 < 0.1 (slack: 0.0007 for a random hypothesis at
    // 2,000 points; it grows with the count, not with n^2: tight brackets at any n); an exact integer
    // count (no value in the band) is unchanged by floor(+ slack) while slack < 1.
    // Zero-padded rows (ex = ey = W = 0) add exactly 1 to the upper count (K E + 1 >= 1) and 0 to the
    // lower one (-K E_lo < 0).
    const float k0 = keep0 + __shfl_xor(keep0, 32), k1 = keep1 + __shfl_xor(keep1, 32);
    const double m2 = 0x1p-24 * 1.25 * (double)(16 * nt + 2);
    const double kk = (double)(lowh ? k0 : k1);
    const int hi = min(n, max(0, (int)floor(kk + m2 * (kk + 1.0)) - (32 * nt - n)));
    int lo = 0;
    if (kLo) {
        const float i0 = in0 + __shfl_xor(in0, 32), i1 = in1 + __shfl_xor(in1, 32);
        const double ii = (double)(lowh ? i0 : i1);
        lo = min(hi, max(0, (int)ceil(ii - m2 * (ii + 1.0))));
    }
    if (act) bounds[o] = invalid ? make_int2(-1, -1) : (uncertain ? make_int2(0, n) : make_int2(lo, hi));
}

// exact count of one hypothesis (runKernel + computeError + findInliers, bit-exact)
__device__ int exact_count(const float4* __restrict__ P, int n, int4 s4, double* D, float thr2, double (&H)[9]) {
    const float4 a = P[s4.x], b = P[s4.y], c = P[s4.z], d = P[s4.w];
    const float M[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
    const float m[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
    if (!run_kernel4<64>(M, m, D, H)) return -1;
    float Hf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) Hf[i] = (float)H[i];
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        const float4 q = P[i];
        cnt += reproj_err(Hf, q.x, q.y, q.z, q.w) <= thr2;
    }
    return cnt;
}

// Debug check of the bound kernels (MIM_CHECK_BOUNDS=1): the exact count of every iteration of
// the chunk (runKernel + computeError, bit-exact, one lane each) against its [lo, hi] bracket.
// stats: [0] iterations checked, [1] lo > exact, [2] hi < exact, [3] validity disagreements,
// [4] sum of hi - lo, [5] iterations with lo == hi.
__global__ __launch_bounds__(64) void ransac_bound_check_kernel(const RansacState* __restrict__ st,
                                                                const ProbDev* __restrict__ probs,
                                                                const float4* __restrict__ pts,
                                                                const int4* __restrict__ samples,
                                                                const uint32_t* __restrict__ stream,
                                                                const int2* __restrict__ bounds, int c0, int c1,
                                                                int bpp, float thr2, unsigned long long* stats) {
    __shared__ double sd[kJ9D * 64];
    const int p = blockIdx.x / bpp, lane = threadIdx.x;
    const int it = c0 + (blockIdx.x % bpp) * 64 + lane;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    if (!(it < c1 && it < S.produced)) return;
    const long long o = probs[p].it_off + it;
    double H[9];
    const int ex = exact_count(pts + probs[p].good_off, S.n, decode_sample(samples[o], stream, (unsigned)S.n, S.modM),
                               sd + lane, thr2, H);
    const int2 b = bounds[o];
    atomicAdd(stats + 0, 1ull);
    if ((b.x == -1) != (ex == -1)) atomicAdd(stats + 3, 1ull);
    if (ex >= 0 && b.x >= 0) {
        if (b.x > ex) atomicAdd(stats + 1, 1ull);
        if (b.y < ex) atomicAdd(stats + 2, 1ull);
        if (b.x > ex || b.y < ex) {  // details of a violation (debug path only)
            double Hd[8];
            bool inv = false, unc = false;
            float eta = 0.f;
            double eta_m = 0;
            bound_hypothesis(pts + probs[p].good_off, decode_sample(samples[o], stream, (unsigned)S.n, S.modM), Hd,
                             inv, unc, eta, eta_m);
            double dmax = 0;
            for (int i = 0; i < 8; ++i) dmax = fmax(dmax, fabs(Hd[i] - H[i]) / (fabs(H[i]) + 1e-12));
            const int4 s4v = decode_sample(samples[o], stream, (unsigned)S.n, S.modM);
            printf("[mim] bound violation p=%d it=%d exact=%d lo=%d hi=%d eta=%g uncertain=%d max_rel_dH=%g sample %d %d %d %d\n",
                   p, it, ex, b.x, b.y, (double)eta, (int)unc, dmax, s4v.x, s4v.y, s4v.z, s4v.w);
            float Hf[8], Hb[8];
            for (int i = 0; i < 8; ++i) { Hf[i] = (float)H[i]; Hb[i] = (float)Hd[i]; }
            const float4* P = pts + probs[p].good_off;
            for (int i = 0; i < S.n; ++i) {
                const float4 q = P[i];
                const float err = reproj_err(Hf, q.x, q.y, q.z, q.w);
                const float W = fmaf(Hb[6], q.x, fmaf(Hb[7], q.y, 1.f));
                const float exx = fmaf(-q.z, W, fmaf(Hb[0], q.x, fmaf(Hb[1], q.y, Hb[2])));
                const float eyy = fmaf(-q.w, W, fmaf(Hb[3], q.x, fmaf(Hb[4], q.y, Hb[5])));
                const float eb = fmaf(exx, exx, eyy * eyy) / (W * W);
                if (err <= thr2 || (err <= thr2) != (eb <= thr2))
                    printf("[mim]   pt %d (%g %g -> %g %g) exact err %.6g bound-form err %.6g W %g sa %g sb %g smax %g\n", i,
                           q.x, q.y, q.z, q.w, (double)err, (double)eb, (double)W, (double)S.sa, (double)S.sb,
                           (double)S.smax);
            }
        }
        atomicAdd(stats + 4, (unsigned long long)(b.y - b.x));
        if (b.x == b.y) atomicAdd(stats + 5, 1ull);
    }
}

// Split form of the filtered select (default): candidates of every problem are listed first,
// evaluated exactly by a GPU-wide grid (one lane each), then replayed in order per problem.
constexpr int kCandWaves = 16;                 // exact-evaluation waves per problem and chunk
constexpr int kCandCap = kCandWaves * 64;      // listed candidates per problem and chunk
static_assert(kCandCap == kCandPerProblem, "candidate list layout shared with api.cpp");

constexpr int kCandThreads = 1024;  // the cand kernel's block

// Candidate prescreen (round 5): before the exact pass, every listed candidate whose count the
// closed-form hypothesis already decides gets it here, without the eigensolve; the exact kernel's waves
// take only the rest (flagged undecided in `decided`, in list order).  Decided: a bracket with lo == hi (chunk 1), or no point in
// the uncertain band of the disc test the bound kernel's diamonds relax, evaluated in fp64 in pixel
// units: with (X, Y, W) = Hd (x, y, 1), ex = |X - u W|, ey = |Y - v W| and the bound kernel's per-point
// margins (tt / tl = thr2 -/+ the margin d_max (+ the widening of a poorly conditioned sample), the
// near-horizon slack A per coordinate),
//   surely in:  (ex + A)^2 + (ey + A)^2 < tl W^2      surely out:  (ex - A)+^2 + (ey - A)+^2 > tt W^2
// — the conditions the bound kernel's diamond tests are derived from ("Exactness of the
// filtered RANSAC"), so the count of surely-in points is the exact count when no point is in between.
// Samples the conditioning screen rejects (uncertain) are left to the exact kernel.  One wave per
// candidate (points over the lanes), kPreWaves one-wave blocks per problem.
__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

constexpr int kPreWaves = 16;  // prescreen blocks (one wave each) per problem

__global__ __launch_bounds__(64) void ransac_prescreen_kernel(const RansacState* __restrict__ st,
                                                              const ProbDev* __restrict__ probs,
                                                              const int2* __restrict__ bounds,
                                                              const float4* __restrict__ pts,
                                                              const int4* __restrict__ samples,
                                                              const uint32_t* __restrict__ stream,
                                                              const int* __restrict__ cand,
                                                              const int* __restrict__ ncand, int* __restrict__ cex,
                                                              double* __restrict__ cH, int* __restrict__ decided,
                                                              float thr2, int L, int cap) {
    const int p = blockIdx.x / kPreWaves, j = blockIdx.x % kPreWaves, lane = threadIdx.x;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    const ProbDev PD = probs[p];
    const int2* Bd = bounds + PD.it_off;
    const long long lb = (long long)(2 * p + L) * kCandCap;
    const int nl = min(ncand[2 * p + L], cap);
    const float4* __restrict__ P = pts + PD.good_off;
    const int n = S.n;
    for (int k = j; k < nl; k += kPreWaves) {
        const int t = cand[lb + k];
        const int2 bd = Bd[t];
        int res = 0, cnt = 0;
        if (bd.x == bd.y) {
            res = 1;
            cnt = bd.x;
        } else {
            const int4 s4 = decode_sample(samples[PD.it_off + t], stream, (unsigned)n, S.modM);
            double Hd[8];
            bool invalid = false, uncertain = false;
            float eta = 0.f;
            double eta_model = 0;
            bound_hypothesis(P, s4, Hd, invalid, uncertain, eta, eta_model);
            if (!invalid && !uncertain) {
                float tt = thr2 + fmaf(1e-7f * S.smax, S.smax, 0.5f);
                float tl = thr2 - fmaf(1e-7f * S.smax, S.smax, 0.5f);
                if (eta > 0.f) {
                    const float wd = S.smax * fmaf(eta * eta, S.smax, 10.2f * eta);
                    tt += wd;
                    tl -= wd;
                }
                // |x|, |y| <= mx and |u|, |v| <= mu (powers of two from the tiles kernel's scales)
                const double mx = ldexp(1.0, -ilogb((double)S.sa)), mu = ldexp(1.0, -ilogb((double)S.sb));
                const double gam = 4.0 * 0x1p-24 + fmin(eta_model, 1.0);
                const double ax = fmax((fabs(Hd[0]) + fabs(Hd[1])) * mx + fabs(Hd[2]),
                                       (fabs(Hd[3]) + fabs(Hd[4])) * mx + fabs(Hd[5]));
                const double aw = (fabs(Hd[6]) + fabs(Hd[7])) * mx + 1.0;
                const double A = gam * (ax + (mu + 6.0) * aw) * (1.0 + 1e-6);
                const double TT = (double)tt * (1.0 + 1e-9), TL = (double)fmaxf(tl, 0.f) * (1.0 - 1e-9);
                int in = 0, unc = 0;
                for (int i = lane; i < n; i += 64) {
                    const float4 q = P[i];
                    const double x = q.x, y = q.y;
                    const double W = fma(Hd[6], x, fma(Hd[7], y, 1.0));
                    const double X = fma(Hd[0], x, fma(Hd[1], y, Hd[2]));
                    const double Y = fma(Hd[3], x, fma(Hd[4], y, Hd[5]));
                    const double ex = fabs(X - (double)q.z * W), ey = fabs(Y - (double)q.w * W);
                    const double ux = fmax(ex - A, 0.0), uy = fmax(ey - A, 0.0);
                    const double W2 = W * W;
                    const bool maybe = ux * ux + uy * uy <= TT * W2;
                    const bool surely = (ex + A) * (ex + A) + (ey + A) * (ey + A) < TL * W2;
                    in += surely ? 1 : 0;
                    unc += (maybe && !surely) ? 1 : 0;
                }
                in = wave_isum(in);
                unc = wave_isum(unc);
                if (unc == 0) {
                    res = 1;
                    cnt = in;
                }
            }
        }
        if (lane == 0) {
            decided[lb + k] = res;
            if (res) {
                cex[lb + k] = cnt;
                cH[(lb + k) * 9 + 8] = 0.0;  // H not computed (refine recomputes the best sample's)
            }
        }
    }
}

// After the prescreen, in list order (one wave per problem): an undecided candidate whose upper bound
// does not exceed max(3, maxGoodCount before the chunk, the decided counts listed before it) cannot be
// a new best wherever the running best stands (it is at least that bar), so it is settled as
// irrelevant (decided = 2, count 0: the replay's `count > best` test skips it) without the eigensolve.
// Earlier candidates past the final niters only precede later ones that are past it as well.
constexpr int kWinnerHMaxN = 256;
constexpr int kDecidedForceH = 3;  // decided flag: for the exact pass, with runKernel even when lo == hi

__global__ __launch_bounds__(64) void ransac_settle_kernel(const RansacState* __restrict__ st,
                                                           const ProbDev* __restrict__ probs,
                                                           const int2* __restrict__ bounds,
                                                           const int* __restrict__ cand, const int* __restrict__ ncand,
                                                           int* __restrict__ cex, double* __restrict__ cH,
                                                           int* __restrict__ decided, int L, int cap,
                                                           int winner_h) {
    const int p = blockIdx.x, lane = threadIdx.x;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    const long long lb = (long long)(2 * p + L) * kCandCap;
    const int nl = min(ncand[2 * p + L], cap);
    const int2* Bd = bounds + probs[p].it_off;
    int bar = max(S.max_good, 3);
    for (int base = 0; base < nl; base += 64) {
        const int k = base + lane;
        const bool in = k < nl;
        const int dec = in ? decided[lb + k] : 1;
        int incl = (in && dec == 1) ? cex[lb + k] : INT_MIN;  // decided counts (exact)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(incl, off);
            if (lane >= off) incl = max(incl, o);
        }
        int excl = __shfl_up(incl, 1);
        if (lane == 0) excl = INT_MIN;
        const int before = max(bar, excl);
        if (in && dec == 0 && Bd[cand[lb + k]].y <= before) {
            decided[lb + k] = 2;
            cex[lb + k] = 0;
            cH[(lb + k) * 9 + 8] = 0.0;
        }
        bar = max(bar, __shfl(incl, 63));
    }
    // winner_h: 1 every problem, 2 problems of fewer than kWinnerHMaxN good matches (where the refine's
    // own runKernel is a large share of its chain: real SIFT views), 0 none
    if ((winner_h == 1 || (winner_h == 2 && S.n < kWinnerHMaxN)) && bar > max(S.max_good, 3)) {
        // the first listed decided candidate holding the largest decided count is the chunk's likely
        // bestModel: send it through the exact pass too (same count), so its fp64 H reaches best_h and
        // the refine needs no runKernel of its own (MIM_WINNER_H=1; the count and the outcome are unchanged).
        // decided = 3: undecided with its H forced, so a candidate the bound kernel pinned (lo == hi) runs
        // runKernel in the exact pass instead of taking the tight shortcut (which stores no H)
        for (int base = 0; base < nl; base += 64) {
            const int k = base + lane;
            const bool hit = k < nl && decided[lb + k] == 1 && cex[lb + k] == bar;
            const unsigned long long m = __ballot(hit);
            if (m) {
                if (lane == __builtin_ctzll(m)) decided[lb + k] = kDecidedForceH;
                break;
            }
        }
    }
}

// position of the r-th undecided listed candidate (list order), -1 past them: one wave scans the flags
__device__ __forceinline__ int undecided_position(const int* __restrict__ decided, long long lb, int nl, int r) {
    const int lane = threadIdx.x & 63;
    int seen = 0;
    for (int base = 0; base < nl; base += 64) {
        const int dv = base + lane < nl ? decided[lb + base + lane] : 1;
        const bool u = dv == 0 || dv == kDecidedForceH;
        const unsigned long long m = __ballot(u);
        const int c = __popcll(m);
        if (r < seen + c) {  // the (r - seen)-th set bit of m
            const int before = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            const unsigned long long hit = __ballot(u && before == r - seen);
            return base + __builtin_ctzll(hit);
        }
        seen += c;
    }
    return -1;
}

// Debug check of the prescreen (MIM_CHECK_PRESCREEN=1): every listed candidate the prescreen decided
// (flagged in `decided`) recounted exactly (runKernel + computeError, one lane each) against its cex.
__global__ __launch_bounds__(64) void ransac_prescreen_check_kernel(const RansacState* __restrict__ st,
                                                                    const ProbDev* __restrict__ probs,
                                                                    const float4* __restrict__ pts,
                                                                    const int4* __restrict__ samples,
                                                                    const uint32_t* __restrict__ stream,
                                                                    const int* __restrict__ cand,
                                                                    const int* __restrict__ ncand,
                                                                    const int* __restrict__ cex,
                                                                    const int* __restrict__ decided,
                                                                    const int2* __restrict__ bounds, float thr2,
                                                                    int L, int cap, unsigned long long* stats) {
    __shared__ double sd[kJ9D * 64];
    const int p = blockIdx.x / (kCandCap / 64), k = (blockIdx.x % (kCandCap / 64)) * 64 + threadIdx.x;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    const int nl = min(ncand[2 * p + L], cap);
    if (k >= nl) return;
    const long long lb = (long long)(2 * p + L) * kCandCap;
    if (decided[lb + k] != 1) return;  // undecided (the exact kernel's) or settled as irrelevant
    const int t = cand[lb + k];
    double H[9];
    const int ex = exact_count(pts + probs[p].good_off, S.n, decode_sample(samples[probs[p].it_off + t], stream,
                                                                           (unsigned)S.n, S.modM),
                               sd + threadIdx.x, thr2, H);
    atomicAdd(stats + 0, 1ull);
    if (ex != cex[lb + k]) {
        atomicAdd(stats + 1, 1ull);
        const int2 bd = bounds[probs[p].it_off + t];
        printf("[mim] prescreen mismatch p=%d it=%d exact=%d prescreen=%d lo=%d hi=%d n=%d\n", p, t, ex, cex[lb + k],
               bd.x, bd.y, S.n);
    }
}

// Candidates of one chunk: iteration t is listed iff hi_t > max(3, maxGoodCount, earlier lower
// bounds) — a prefix maximum over the chunk, computed by a 1024-thread block (contiguous ranges
// per thread, block max-scan, ordered compaction).

__global__ __launch_bounds__(kCandThreads) void ransac_cand_kernel(RansacState* __restrict__ st,
                                                                   const ProbDev* __restrict__ probs,
                                                                   const int2* __restrict__ bounds, int c1,
                                                                   int* __restrict__ cand, int* __restrict__ ncand,
                                                                   int L, int cap) {
    __shared__ int wred[kCandThreads / 64], wred2[kCandThreads / 64];
    const int p = blockIdx.x, tid = threadIdx.x;
    const RansacState S = st[p];
    if (!S.active || S.done) {
        if (tid == 0) ncand[2 * p + L] = 0;
        return;
    }
    const int2* Bd = bounds + probs[p].it_off;
    const int t0 = S.next_iter, t1 = max(t0, min(min(c1, S.produced), S.niters));
    const int ch = (t1 - t0 + kCandThreads - 1) / kCandThreads;
    const int a = min(t1, t0 + tid * ch), e = min(t1, a + ch);
    // batches of 16 unconditional (clamped) loads: one memory latency per batch, not per iteration
    constexpr int kB = 16;
    int lmax = INT_MIN;
    for (int t = a; t < e; t += kB) {
        int2 v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) v[k] = Bd[min(t + k, e - 1)];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            lmax = t + k < e ? max(lmax, v[k].x) : lmax;
        }
    }
    const int init = max(3, max(S.max_good, S.lo_max));
    int all;
    const int run0 = block_excl_max(lmax, init, wred, all);  // bound before this thread's first iteration
    int cnt = 0, run = run0;
    for (int t = a; t < e; t += kB) {
        int2 v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) v[k] = Bd[min(t + k, e - 1)];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            if (t + k < e) {
                cnt += v[k].y > run;
                run = max(run, v[k].x);
            }
        }
    }
    int total;
    int o = block_excl_sum(cnt, wred2, total);
    if (cnt && o < cap) {  // ordered list (beyond the capacity the replay kernel rescans)
        int* C = cand + (long long)(2 * p + L) * kCandCap;
        run = run0;
        for (int t = a; t < e && o < cap; ++t) {
            const int2 b = Bd[t];
            if (b.y > run) C[o++] = t;
            run = max(run, b.x);
        }
    }
    if (tid == 0) {
        ncand[2 * p + L] = total;
        st[p].lo_max = max(S.lo_max, all);
        // chunk 1's exact pass is never deferred into chunk 2's (measured -3 % on C3: the combined
        // pass has a longer Jacobi tail); the replay/exact kernels still accept a deferred list
        if (L == 0) st[p].defer = 0;
    }
}

// Exact evaluation of the listed candidates: 4 per wave, each solved by a 16-lane group
// (cooperative Jacobi), then counted by the whole wave.
constexpr int kExactGroups = 4;
constexpr int kExactWaves = kCandCap / kExactGroups;

#ifndef MIM_EXACT_OCC
#define MIM_EXACT_OCC 1  // waves per SIMD the exact kernel's register budget is sized for (1: no cap)
#endif
__global__ __launch_bounds__(64, MIM_EXACT_OCC) void ransac_exact_kernel(const RansacState* __restrict__ st,
                                                          const ProbDev* __restrict__ probs,
                                                          const float4* __restrict__ pts,
                                                          const int4* __restrict__ samples,
                                                          const uint32_t* __restrict__ stream,
                                                          const int* __restrict__ cand, const int* __restrict__ ncand,
                                                          const int2* __restrict__ bounds,
                                                          int* __restrict__ cex, double* __restrict__ cH, float thr2,
                                                          int L, int cap, const int* __restrict__ decided,
                                                          int prescreen) {
    __shared__ double sd[kExactGroups * kJ9G];
    // blocks: [list pass][wave][problem]; chunk 1 (L = 0): list 0 of the problems not deferred;
    // chunk 2 (L = 1): list 1 of every problem, then list 0 of the deferred ones.  Problem-minor
    // order: the first (and usually only) busy wave of every problem comes first and lands on all 8
    // XCDs (blocks b and b+8 share an XCD under round-robin dispatch)
    const int np = gridDim.x / (kExactWaves * (L + 1));
    const int pass = blockIdx.x / (np * kExactWaves), rem = blockIdx.x % (np * kExactWaves);
    const int list = L - pass;
    const int p = rem % np, w = rem / np, lane = threadIdx.x, grp = lane >> 4, slot = lane & 15;
    const RansacState S = st[p];
    if (!S.active || S.done) return;
    if (list == 0 && (L == 0) == (S.defer != 0)) return;  // uniform over the block
    const long long lb = (long long)(2 * p + list) * kCandCap;
    const int nc = min(ncand[2 * p + list], cap);
    // with the prescreen, wave w takes the undecided candidates 4w .. 4w + 3 in list order
    int kg[kExactGroups];
#pragma unroll
    for (int g = 0; g < kExactGroups; ++g) {
        const int r = w * kExactGroups + g;
        kg[g] = prescreen ? undecided_position(decided, lb, nc, r) : (r < nc ? r : -1);
    }
    if (kg[0] < 0) return;  // uniform over the wave
    const bool valid = kg[grp] >= 0;  // groups past the list only join the counting
    const int k = valid ? kg[grp] : kg[0];
    const int t = cand[lb + k];
    const long long o = lb + k;
    const int2 bd = bounds[probs[p].it_off + t];
    // lo == hi pins the exact count: no eigensolve needed, unless the settle pass wants the H
    const bool tight = bd.x == bd.y && !(prescreen && decided[o] == kDecidedForceH);
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int ok = 0;
    const float4* __restrict__ P = pts + probs[p].good_off;
    if (valid && !tight) {  // uniform over the group
        const int4 s4 = decode_sample(samples[probs[p].it_off + t], stream, (unsigned)S.n, S.modM);
        const float4 a = P[s4.x], b = P[s4.y], c = P[s4.z], d = P[s4.w];
        const float M[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
        const float m[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
        ok = run_kernel4_group(M, m, sd + grp * kJ9G, H);
    }
    // findInliers of every solved candidate by the whole wave (computeError is per point: the count
    // does not depend on the order)
    float Hf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) Hf[i] = (float)H[i];
    int ex = tight ? bd.x : -1;
    unsigned long long todo = __ballot(ok != 0 && slot == 0);
    const int n = S.n;
    while (todo) {
        const int c = __builtin_ctzll(todo);
        todo &= todo - 1;
        float hc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) hc[i] = __shfl(Hf[i], c);
        int cnt = 0;
        for (int i = lane; i < n; i += 64) {
            const float4 q = P[i];
            cnt += reproj_err(hc, q.x, q.y, q.z, q.w) <= thr2;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
        if (lane == c) ex = cnt;
    }
    if (!valid || slot != 0) return;
    cex[o] = ex;
    if (tight) {
        cH[o * 9 + 8] = 0.0;  // H not computed (H22 of a computed model is never 0)
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) cH[o * 9 + i] = H[i];
    }
}

__global__ __launch_bounds__(64) void ransac_replay_kernel(RansacState* __restrict__ st,
                                                           const ProbDev* __restrict__ probs,
                                                           const float4* __restrict__ pts,
                                                           const int4* __restrict__ samples,
                                                           const uint32_t* __restrict__ stream,
                                                           const int2* __restrict__ bounds, const int* __restrict__ cand,
                                                           const int* __restrict__ ncand, const int* __restrict__ cex,
                                                           const double* __restrict__ cH, int c1, double conf,
                                                           float thr2, double* __restrict__ best_h, int L,
                                                           int c1_prev, int cap) {
    __shared__ double sd[kJ9D * 64];
    const int p = blockIdx.x, lane = threadIdx.x;
    RansacState S = st[p];
    if (!S.active || S.done) return;
    if (L == 0 && S.defer) {  // chunk 1's list is replayed with chunk 2's (ransac_cand_kernel)
        if (lane == 0) st[p].next_iter = min(c1, S.produced);
        return;
    }
    const int N = S.n;
    int end = 0;
    // lists in iteration order: a deferred chunk 1 (iterations < c1_prev), then this chunk
    for (int li = (L == 1 && S.defer) ? 0 : L; li <= L; ++li) {
    end = min(li == L ? c1 : c1_prev, S.produced);
    const int nc = ncand[2 * p + li];
    const int* C = cand + (long long)(2 * p + li) * kCandCap;
    const int* E = cex + (long long)(2 * p + li) * kCandCap;
    const double* HH = cH + (long long)(2 * p + li) * kCandCap * 9;
    int best_k = -1;  // candidate index whose H becomes bestModel (listed part)
    for (int k0 = 0; k0 < min(nc, cap); k0 += 64) {
        const int k = k0 + lane;
        const bool in = k < min(nc, cap);
        const int t = in ? C[k] : INT_MAX;
        const int ex = in ? E[k] : -1;
        for (;;) {
            const int thr = max(S.max_good, 3);
            const unsigned long long m = __ballot(t < S.niters && ex > thr);
            if (!m) break;
            const int f = __ffsll((long long)m) - 1;
            S.max_good = __shfl(ex, f);
            S.best_iter = __shfl(t, f);
            S.niters = update_num_iters(conf, (double)(N - S.max_good) / N, 4, S.niters);
            best_k = k0 + f;
        }
    }
    if (best_k >= 0 && lane < 9) best_h[(long long)p * 9 + lane] = HH[(long long)best_k * 9 + lane];
    if (nc > cap) {
        // overflow (very many candidates): rescan the iterations after the last listed one and
        // evaluate their candidates here, 64 at a time, with the running exact best
        const int2* Bd = bounds + probs[p].it_off;
        const float4* __restrict__ P = pts + probs[p].good_off;
        const int4* Sm = samples + probs[p].it_off;
        const int start = C[cap - 1] + 1;
        for (int base = start; base < end && base < S.niters; base += 64) {
            const int t = base + lane;
            const bool valid = t < end;
            const int2 b = valid ? Bd[t] : make_int2(-1, -1);
            const bool c = valid && t < S.niters && b.y > max(S.max_good, 3);
            int ex = -1;
            double H[9];
            if (__any(c)) {
                if (c) ex = exact_count(P, N, decode_sample(Sm[t], stream, (unsigned)N, S.modM), sd + lane, thr2, H);
            }
            int fbest = -1;
            for (;;) {
                const int thr = max(S.max_good, 3);
                const unsigned long long m = __ballot(c && t < S.niters && ex > thr);
                if (!m) break;
                const int f = __ffsll((long long)m) - 1;
                S.max_good = __shfl(ex, f);
                S.best_iter = __shfl(t, f);
                S.niters = update_num_iters(conf, (double)(N - S.max_good) / N, 4, S.niters);
                fbest = f;
            }
            if (fbest >= 0 && lane == fbest)
                for (int i = 0; i < 9; ++i) best_h[(long long)p * 9 + i] = H[i];
        }
    }
    }  // lists
    S.next_iter = end;
    // getSubset failed at iteration fail_iter (or the stream ran out: -2) within this chunk's range;
    // a failure the concurrent sampler finds in the next chunk has fail_iter >= end or is not yet
    // visible, and only stops the loop where OpenCV stops it too
    const bool failed = S.fail_iter != -1 && S.fail_iter <= end;
    if (S.niters <= end || failed) S.done = 1;
    if (lane == 0) store_select_state(st + p, S);
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
#ifndef MIM_LM_MERGE
#define MIM_LM_MERGE 1  // the trial step's cost S(x - d) from the normal-equation pass at x - d (see below)
#endif
#ifndef MIM_LTL_STAGE
#define MIM_LTL_STAGE 1  // the refit's LtL sums read the inliers' L rows from LDS (0: select them in registers)
#endif
#ifndef MIM_REFINE_TIMING
#define MIM_REFINE_TIMING 0  // diagnostic: print the refine phases (wall clock) of the slow problems
#endif
#ifndef MIM_REFINE_RW
#define MIM_REFINE_RW 4
#endif
constexpr int kRW = MIM_REFINE_RW;  // refine: problems (waves) per block
constexpr int kRT = 64 * kRW;  // refine block

// LDS visibility between the lanes of one wave (the refine runs one problem per wave)
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double wave_max_d(double x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x = fmax(x, __shfl_xor(x, off));
    return x;
}

// ---- LM sums in OpenCV's order ------------------------------------------------------------------
// HomographyRefineCallback::compute fills r (2k rows) and J (2k x 8) row by row; LMSolverImpl forms
// A = J^T J and v = J^T r (mulTransposed / gemm: each entry one sequential sum over the rows) and
// S = |r|^2 (norm(r, NORM_L2SQR): sequential).  The per-point quantities (ww, xi, yi, residuals) are
// computed by all threads into an LDS chunk; each of 45 lanes then owns one sum (36 A entries, 8 v
// entries, S) and adds the chunk's rows in order: the same operations in the same order as the oracle
// (lm_refine / normal_eq in oracle/mim_oracle.c), so the refined H is bit-identical, also for the
// near-degenerate inlier sets of real data (duplicated keypoints) where a reordered sum moves the
// LM path far (tests/test_pipeline_gpu.py).
constexpr int kLmChunk = 64;
constexpr int kLmRow = 9;  // J row (8 entries) + the residual, per x / y row of a point
struct LmStage {
    double rx[kLmChunk * kLmRow], ry[kLmChunk * kLmRow];  // [point][Jx(0..7), r_x] and [point][Jy, r_y]
};

// stage points [c0, c0 + n) of X under model h into L (J rows only when `jac`); returns this
// thread's max |residual|
__device__ double lm_stage(const float4* __restrict__ X, int c0, int n, const double* h, LmStage& L, bool jac) {
    double mx = 0;
    for (int i = threadIdx.x & 63; i < n; i += 64) {
        const float4 q = X[c0 + i];
        const double Mx = q.x, My = q.y;
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
        const double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
        const double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
        const double ex = xi - (double)q.z, ey = yi - (double)q.w;
        double* x = L.rx + i * kLmRow;
        double* y = L.ry + i * kLmRow;
        if (jac) {  // HomographyRefineCallback::compute's J rows
            x[0] = Mx * ww; x[1] = My * ww; x[2] = ww; x[3] = x[4] = x[5] = 0.;
            x[6] = -Mx * ww * xi; x[7] = -My * ww * xi;
            y[0] = y[1] = y[2] = 0.; y[3] = Mx * ww; y[4] = My * ww; y[5] = ww;
            y[6] = -Mx * ww * yi; y[7] = -My * ww * yi;
        }
        x[8] = ex;
        y[8] = ey;
        mx = fmax(mx, fmax(fabs(ex), fabs(ey)));
    }
    return mx;
}

// A = J^T J, v = J^T r, S = |r|^2 as the 45 entries (a, b), a <= b <= 8, of [J r]^T [J r] (column 8
// = r): out[e] in the packing order A upper (36), v (8), S; each entry one lane's sequential sum over
// the rows (x row, then y row, point by point).  rinf = |r|_inf.
__device__ void lm_normal(const float4* __restrict__ X, int n, const double* h, LmStage& L,
                          double* out, double& rinf) {
    const int e = threadIdx.x & 63;
    int a = 8, b = 8;  // e == 44: S
    if (e < 36) {      // (a, b), b >= a, row-major upper triangle of A
        a = 0;
        int r = e;
        while (r >= 8 - a) { r -= 8 - a; ++a; }
        b = a + r;
    } else if (e < 44) {
        a = e - 36;
    }
    double acc = 0, mx = 0;
    for (int c0 = 0; c0 < n; c0 += kLmChunk) {
        const int m = min(kLmChunk, n - c0);
        wsync();
        mx = fmax(mx, lm_stage(X, c0, m, h, L, true));
        wsync();
        if (e < 45) {
#pragma unroll 4
            for (int i = 0; i < m; ++i) {
                const double* x = L.rx + i * kLmRow;
                const double* y = L.ry + i * kLmRow;
                acc += x[a] * x[b];
                acc += y[a] * y[b];
            }
        }
    }
    if (e < 45) out[e] = acc;
    rinf = wave_max_d(mx);  // max is order-free
    wsync();
}

// S(h) = |r(h)|^2, sequential over the rows
__device__ double lm_cost(const float4* __restrict__ X, int n, const double* h, LmStage& L, double* red) {
    double acc = 0;
    for (int c0 = 0; c0 < n; c0 += kLmChunk) {
        const int m = min(kLmChunk, n - c0);
        wsync();
        lm_stage(X, c0, m, h, L, false);
        wsync();
        if ((threadIdx.x & 63) == 0)
#pragma unroll 8
            for (int i = 0; i < m; ++i) {
                const double ex = L.rx[i * kLmRow + 8], ey = L.ry[i * kLmRow + 8];
                acc += ex * ex;
                acc += ey * ey;
            }
    }
    if ((threadIdx.x & 63) == 0) red[0] = acc;
    wsync();
    const double r = red[0];
    wsync();
    return r;
}

// eig8 by a 16-lane group (jacobi_group<8>, bit-identical to OpenCV's JacobiImpl_): the state lives in
// J (A packed upper | W | V); every slot gets the sorted eigenvalues Ws and perm (row of V of each)
__device__ __forceinline__ void eig8_group(const double* Ain, double* J, double (&Ws)[8], int (&perm)[8]) {
    const int slot = threadIdx.x & 15;
    double* A = J;
    double* W = J + 28;
    double* VV = J + 36;
    for (int e = slot; e < 64; e += 16) {
        const int i = e >> 3, j = e & 7;
        if (i == j) W[i] = Ain[e];
        else if (j > i) A[pk<8>(i, j)] = Ain[e];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    jacobi_group<8>(A, W, VV, Ws, perm);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// solve(Ap, v, d, DECOMP_EIG) = Jacobi + SVBkSb(eps = 2 DBL_EPSILON) (Ap, b in LDS); called by a
// 16-lane group, every slot gets x and the decomposition (w sorted, perm; V stays in J + 36)
__device__ void solve_eig8(const double* Ap, const double* b, double (&x)[8], double* J, double (&w)[8],
                           int (&perm)[8]) {
    eig8_group(Ap, J, w, perm);
    const double* V = J + 36;
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        const double* Vi = V + perm[i] * 8;
        double s = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) s += Vi[j] * b[j];
        s *= wi;
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = x[j] + s * Vi[j];
    }
}

// invert(A, Ai, DECOMP_EIG), max |Ai(i,i)| (LMSolverImpl's lambda restart) from an eigendecomposition
// of A.  LMSolverImpl restarts lambda only when it is 0, and then this iteration's step matrix
// Ap = A + 0 * diag(A) is A bit for bit (the diagonal of JᵀJ is never −0): the step solve's
// decomposition is invert's, so no second Jacobi
__device__ double inv_diag_max8(const double (&w)[8], const int (&perm)[8], const double* V) {
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    double maxval = DBL_EPSILON;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        double diag = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (fabs(w[i]) <= threshold) continue;
            const double v = V[perm[i] * 8 + c];
            diag += v * v / w[i];
        }
        maxval = fmax(maxval, fabs(diag));
    }
    return maxval;
}

#if MIM_REFINE_TIMING
#define MIM_RT_MARK(acc)                          \
    do {                                          \
        const unsigned long long t_ = wall_clock64(); \
        acc += t_ - rt_last;                      \
        rt_last = t_;                             \
    } while (0)
#else
#define MIM_RT_MARK(acc) do {} while (0)
#endif

struct RefineShared {  // one per wave (problem)
    double red[2];
    double lt[45];
    double nrm[45];       // LM sums: A upper (36), v (8), S
    LmStage lm;
    double norm[8];       // cm, cM, sm, sM (x,y each)
    double H[9], Hb[9];
    double A[64], Ap[64], v[8], D[8], x[8], xd[8], d[8];
    double S, Sd, rinf, dinf, lambda, lc;
    double J9[kJ9D];
    int flag, n_inl, proceed, accept;
};

__global__ __launch_bounds__(kRT) void ransac_refine_kernel(const RansacState* __restrict__ st,
                                                            const ProbDev* __restrict__ probs,
                                                            const float4* __restrict__ pts,
                                                            const int* __restrict__ n_good_arr,
                                                            const int4* __restrict__ samples,
                                                            const uint32_t* __restrict__ stream,
                                                            float4* __restrict__ inl, uint8_t* __restrict__ masks,
                                                            mim_result* __restrict__ results, RansacParams prm,
                                                            int raw, const double* __restrict__ best_h, int exact_all,
                                                            int n_probs) {
    // one problem per wave: kRW problems per block, so the latency-bound refine holds few CUs'
    // registers and LDS while the next batches' distance and bound kernels fill the GPU
    __shared__ RefineShared shs[kRW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = lane;
    const int p = blockIdx.x * kRW + wave;
    if (p >= n_probs) return;
    RefineShared& sh = shs[wave];
    const RansacState S = st[p];
    const int ng = n_good_arr[p];
    const long long go = probs[p].good_off;
    const float4* P = pts + go;
    uint8_t* mask = masks + go;
    float4* X = inl + go;
    mim_result res{};
    res.n_good = ng;
#if MIM_REFINE_TIMING
    unsigned long long rt_last = wall_clock64(), t_mask = 0, t_refit = 0, t_norm0 = 0, t_solve = 0, t_cost = 0,
                       t_norm = 0;
    const unsigned long long rt_start = rt_last;
    int rt_iters = 0;
#endif
    // ---- gate :74 ----
    if (ng < prm.min_good || ng < 4) {
        res.status = MIM_FEW_GOOD;
        if (tid == 0) results[p] = res;
        return;
    }
    int ok = 0;
    if (!S.active) {  // n == 4: findHomography calls runKernel directly, mask = ones, no refine
        if (tid < 16) {  // one 16-lane group
            float M[8], m[8];
            for (int i = 0; i < 4; ++i) {
                const float4 q = P[i];
                M[2 * i] = q.x; M[2 * i + 1] = q.y; m[2 * i] = q.z; m[2 * i + 1] = q.w;
            }
            double Hl[9];
            const int f = run_kernel4_group(M, m, sh.J9, Hl);
            if (tid == 0) {
                sh.flag = f;
                for (int i = 0; i < 9; ++i) sh.H[i] = Hl[i];
            }
        }
        wsync();
        ok = sh.flag;
        if (tid < 4) mask[tid] = ok ? 1 : 0;
        sh.n_inl = ok ? 4 : 0;
        res.iters = 0;
    } else {
        ok = S.max_good > 0 && S.fail_iter != -2;
        // the loop counter at exit: niters, or best_iter + 1 when the last update dropped niters to or
        // below the iteration that found the best model (RANSACPointSetRegistrator::run's `for`)
        const int stop = max(S.niters, S.best_iter + 1);
        res.iters = (S.fail_iter >= 0 && S.fail_iter < stop) ? S.fail_iter : stop;
        if (ok) {
            // bestModel = runKernel(sample[best_iter]) (bit-identical to the hypo kernel's)
            if (tid == 0 && !exact_all && best_h[(long long)p * 9 + 8] != 0.0) {
                for (int i = 0; i < 9; ++i) sh.Hb[i] = best_h[(long long)p * 9 + i];  // from the exact pass
            } else if (tid < 16 && (exact_all || best_h[(long long)p * 9 + 8] == 0.0)) {
                // bestModel = runKernel(sample[best_iter]), bit-identical, by one 16-lane group
                const int4 s4 = decode_sample(samples[probs[p].it_off + S.best_iter], stream, (unsigned)S.n, S.modM);
                const float4 a = P[s4.x], b = P[s4.y], c = P[s4.z], d = P[s4.w];
                const float M[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
                const float m[8] = {a.z, a.w, b.z, b.w, c.z, c.w, d.z, d.w};
                double Hl[9];
                run_kernel4_group(M, m, sh.J9, Hl);
                if (tid == 0)
                    for (int i = 0; i < 9; ++i) sh.Hb[i] = Hl[i];
            }
            wsync();
            float Hf[8];
            for (int i = 0; i < 8; ++i) Hf[i] = (float)sh.Hb[i];
            const float thr2 = (float)(prm.thresh * prm.thresh);
            // best mask + ordered compaction of the inliers (compressElems)
            int base = 0;
            for (int b0 = 0; b0 < ng; b0 += 64) {
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
                if (in) X[base + within] = q;
                base += __popcll(bal);
            }
            MIM_RT_MARK(t_mask);
            if (tid == 0) sh.n_inl = base;
            if (tid == 0)  // the best model's mask holds maxGoodCount inliers
                MIM_DEBUG_CHECK(base == S.max_good, "[refine] p=%d n=%d max_good=%d mask=%d best_iter=%d niters=%d\n",
                                p, S.n, S.max_good, base, S.best_iter, S.niters);
            wsync();
            const int k = sh.n_inl;
            if (k > 0) {
                // ---- refit: runKernel over all inliers, OpenCV's sequential sums (fundam.cpp) ----
                if (tid < 4) {  // centroids cm (scene), cM (object): one sequential sum each
                    double c = 0;
#pragma unroll 8
                    for (int i = 0; i < k; ++i) {
                        const float4 q = X[i];
                        c += tid == 0 ? q.z : tid == 1 ? q.w : tid == 2 ? q.x : q.y;
                    }
                    sh.norm[tid] = c / k;
                }
                wsync();
                if (tid < 4) {  // mean absolute deviations
                    const double c = sh.norm[tid];
                    double sd = 0;
#pragma unroll 8
                    for (int i = 0; i < k; ++i) {
                        const float4 q = X[i];
                        sd += fabs((tid == 0 ? q.z : tid == 1 ? q.w : tid == 2 ? q.x : q.y) - c);
                    }
                    sh.norm[4 + tid] = sd;
                }
                wsync();
                const double cmx = sh.norm[0], cmy = sh.norm[1], cMx = sh.norm[2], cMy = sh.norm[3];
                const bool degenerate = fabs(sh.norm[4]) < DBL_EPSILON || fabs(sh.norm[5]) < DBL_EPSILON ||
                                        fabs(sh.norm[6]) < DBL_EPSILON || fabs(sh.norm[7]) < DBL_EPSILON;
                if (!degenerate) {
                    const double smx = k / sh.norm[4], smy = k / sh.norm[5], sMx = k / sh.norm[6], sMy = k / sh.norm[7];
#if MIM_LTL_STAGE
                    {  // LtL entry (j, kk), kk >= j: one sequential sum over the inliers per lane, the
                       // inliers' L rows staged in LDS 64 at a time (one point per lane) so each lane
                       // reads its four entries instead of selecting them from the 18 (same values,
                       // same expression, same order)
                        int j = 8, kk = 8;
                        if (tid < 45) {
                            int r = tid;
                            j = 0;
                            while (r >= 9 - j) { r -= 9 - j; ++j; }
                            kk = j + r;
                        }
                        double acc = 0;
                        for (int c0 = 0; c0 < k; c0 += kLmChunk) {
                            const int m = min(kLmChunk, k - c0);
                            wsync();
                            if (tid < m) {
                                const float4 q = X[c0 + tid];
                                const double x = (q.z - cmx) * smx, y = (q.w - cmy) * smy;
                                const double Xx = (q.x - cMx) * sMx, Yy = (q.y - cMy) * sMy;
                                double* lx = sh.lm.rx + tid * kLmRow;
                                double* ly = sh.lm.ry + tid * kLmRow;
                                lx[0] = Xx; lx[1] = Yy; lx[2] = 1; lx[3] = 0; lx[4] = 0; lx[5] = 0;
                                lx[6] = -x * Xx; lx[7] = -x * Yy; lx[8] = -x;
                                ly[0] = 0; ly[1] = 0; ly[2] = 0; ly[3] = Xx; ly[4] = Yy; ly[5] = 1;
                                ly[6] = -y * Xx; ly[7] = -y * Yy; ly[8] = -y;
                            }
                            wsync();
                            if (tid < 45) {
#pragma unroll 4
                                for (int i = 0; i < m; ++i) {
                                    const double* lx = sh.lm.rx + i * kLmRow;
                                    const double* ly = sh.lm.ry + i * kLmRow;
                                    const double lxj = lx[j], lxk = lx[kk], lyj = ly[j], lyk = ly[kk];
                                    acc += lxj * lxk + lyj * lyk;
                                }
                            }
                        }
                        if (tid < 45) sh.lt[tid] = acc;
                    }
#else
                    if (tid < 45) {  // LtL entry (j, kk), kk >= j: one sequential sum over the inliers
                        int j = 0, r = tid;
                        while (r >= 9 - j) { r -= 9 - j; ++j; }
                        const int kk = j + r;
                        double acc = 0;
#pragma unroll 4
                        for (int i = 0; i < k; ++i) {
                            const float4 q = X[i];
                            const double x = (q.z - cmx) * smx, y = (q.w - cmy) * smy;
                            const double Xx = (q.x - cMx) * sMx, Yy = (q.y - cMy) * sMy;
                            const double Lx[9] = {Xx, Yy, 1, 0, 0, 0, -x * Xx, -x * Yy, -x};
                            const double Ly[9] = {0, 0, 0, Xx, Yy, 1, -y * Xx, -y * Yy, -y};
                            double lxj = 0, lxk = 0, lyj = 0, lyk = 0;
#pragma unroll
                            for (int t = 0; t < 9; ++t) {
                                lxj = t == j ? Lx[t] : lxj; lxk = t == kk ? Lx[t] : lxk;
                                lyj = t == j ? Ly[t] : lyj; lyk = t == kk ? Ly[t] : lyk;
                            }
                            acc += lxj * lxk + lyj * lyk;
                        }
                        sh.lt[tid] = acc;
                    }
#endif
                    wsync();
                    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
                    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
                    if (tid < 16) {  // the Jacobi of runKernel, one 16-lane group (bit-identical)
                        double Hl[9];
                        dlt_finish_group(sh.lt, sh.J9, invHnorm, Hnorm2, Hl);
                        if (tid == 0)
                            for (int i = 0; i < 9; ++i) sh.H[i] = Hl[i];
                    }
                } else if (tid == 0) {
                    for (int i = 0; i < 9; ++i) sh.H[i] = sh.Hb[i];  // runKernel returned 0: H kept
                }
                wsync();
                MIM_RT_MARK(t_refit);
                // ---- LMSolverImpl (levmarq.cpp) on H8 = H[0..7], maxIters 10, eps FLT_EPSILON ----
                if (tid < 8) sh.x[tid] = sh.H[tid];
                wsync();
                double x[8];
                for (int i = 0; i < 8; ++i) x[i] = sh.x[i];
                double rinf;
                lm_normal(X, k, x, sh.lm, sh.nrm, rinf);
                if (tid == 0) {
                    int e = 0;
                    for (int a = 0; a < 8; ++a)
                        for (int b = a; b < 8; ++b, ++e) sh.A[a * 8 + b] = sh.A[b * 8 + a] = sh.nrm[e];
                    for (int i = 0; i < 8; ++i) { sh.v[i] = sh.nrm[36 + i]; sh.D[i] = sh.A[9 * i]; }
                    sh.S = sh.nrm[44]; sh.rinf = rinf; sh.lambda = 1; sh.lc = 0.75;
                }
                wsync();
                MIM_RT_MARK(t_norm0);
                int iter = 0;
                double ew[8];  // the step solve's eigendecomposition (group lanes), for the lambda restart
                int eperm[8];
                for (;;) {
                    if (tid < 16) {  // the step solve on one 16-lane group (group Jacobi)
                        for (int i = tid; i < 64; i += 16) sh.Ap[i] = (i % 9) == 0 ? sh.A[i] + sh.lambda * sh.D[i / 9] : sh.A[i];
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        double dl[8];
                        solve_eig8(sh.Ap, sh.v, dl, sh.J9, ew, eperm);
                        if (tid == 0) {
                            double dinf = 0;
                            for (int i = 0; i < 8; ++i) {
                                sh.d[i] = dl[i];
                                sh.xd[i] = sh.x[i] - dl[i];
                                dinf = fmax(dinf, fabs(dl[i]));
                            }
                            sh.dinf = dinf;
                        }
                    }
                    wsync();
                    MIM_RT_MARK(t_solve);
                    double xd[8];
                    for (int i = 0; i < 8; ++i) xd[i] = sh.xd[i];
#if MIM_LM_MERGE
                    // S(x - d) is the normal pass's S entry at x - d (the same rows, summed in the same
                    // order as lm_cost), and an accepted step needs that pass's A, v and |r|_inf next:
                    // one pass over the inliers per iteration instead of two
                    double rinf_d;
                    lm_normal(X, k, xd, sh.lm, sh.nrm, rinf_d);
                    const double Sd = sh.nrm[44];
#else
                    const double Sd = lm_cost(X, k, xd, sh.lm, sh.red);
#endif
                    MIM_RT_MARK(t_cost);
                    if (tid < 16) {  // every slot evaluates the same update; slot 0 stores it
                        const double Rlo = 0.25, Rhi = 0.75;
                        double lambda = sh.lambda, lc = sh.lc;
                        const double Scur = sh.S;
                        double temp_d[8];
                        for (int i = 0; i < 8; ++i) {
                            double s = 0;
                            for (int j = 0; j < 8; ++j) s += sh.A[8 * i + j] * sh.d[j];
                            temp_d[i] = -s + 2 * sh.v[i];
                        }
                        double dS = 0;
                        for (int i = 0; i < 8; ++i) dS += sh.d[i] * temp_d[i];
                        const double R = (Scur - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1);
                        if (R > Rhi) {
                            lambda *= 0.5;
                            if (lambda < lc) lambda = 0;
                        } else if (R < Rlo) {
                            double t = 0;
                            for (int i = 0; i < 8; ++i) t += sh.d[i] * sh.v[i];
                            double nu = (Sd - Scur) / (fabs(t) > DBL_EPSILON ? t : 1) + 2;
                            nu = fmin(fmax(nu, 2.), 10.);
                            if (lambda == 0) {
                                const double maxval = inv_diag_max8(ew, eperm, sh.J9 + 36);
                                lambda = lc = 1. / maxval;
                                nu *= 0.5;
                            }
                            lambda *= nu;
                        }
                        if (tid == 0) {
                            sh.lambda = lambda;
                            sh.lc = lc;
                            sh.accept = Sd < Scur;
                            if (sh.accept) {
                                sh.S = Sd;
                                for (int i = 0; i < 8; ++i) sh.x[i] = sh.xd[i];
                            }
                        }
                    }
                    wsync();
                    if (sh.accept) {
#if MIM_LM_MERGE
                        rinf = rinf_d;
#else
                        for (int i = 0; i < 8; ++i) x[i] = sh.x[i];
                        lm_normal(X, k, x, sh.lm, sh.nrm, rinf);
#endif
                        if (tid == 0) {
                            int e = 0;
                            for (int a = 0; a < 8; ++a)
                                for (int b = a; b < 8; ++b, ++e) sh.A[a * 8 + b] = sh.A[b * 8 + a] = sh.nrm[e];
                            for (int i = 0; i < 8; ++i) sh.v[i] = sh.nrm[36 + i];
                            sh.rinf = rinf;
                        }
                    }
                    MIM_RT_MARK(t_norm);
                    ++iter;
                    if (tid == 0) sh.proceed = iter < 10 && sh.dinf >= FLT_EPSILON && sh.rinf >= FLT_EPSILON;
                    wsync();
                    const bool proceed = sh.proceed;
                    wsync();
                    if (!proceed) break;
                }
#if MIM_REFINE_TIMING
                rt_iters = iter;
#endif
                if (tid < 8) sh.H[tid] = sh.x[tid];
                wsync();
            } else if (tid == 0) {
                for (int i = 0; i < 9; ++i) sh.H[i] = sh.Hb[i];
            }
            wsync();
        } else {
            for (int i = tid; i < ng; i += 64) mask[i] = 0;
            if (tid == 0) sh.n_inl = 0;
        }
    }
    wsync();
    if (tid != 0) return;
#if MIM_REFINE_TIMING
    {  // wall clock at 100 MHz: 10 ns ticks
        const unsigned long long tot = wall_clock64() - rt_start;
        if (tot > 20000)
            printf("[refine-timing] p=%d ng=%d inl=%d iters=%d total=%llu mask=%llu refit=%llu norm0=%llu "
                   "solve=%llu cost=%llu norm=%llu (us x100) niters=%d produced=%d done=%d small=%d\n", p, ng,
                   sh.n_inl, rt_iters, tot, t_mask, t_refit, t_norm0, t_solve, t_cost, t_norm, S.niters, S.produced,
                   S.done, (int)(S.n < kSmallMaxN));
    }
#endif
    res.n_inl = ok ? sh.n_inl : 0;
    if (!ok) {
        // the RNG stream ran out before the loop ended: the host grows it and re-runs the batch
        res.status = (S.active && S.fail_iter == -2) ? MIM_STREAM_SHORT : MIM_EMPTY_H;
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
size_t ransac_chain_bytes() { return sizeof(ChainSegs); }

// cv::RNG((uint64)-1).next() stream (core/include/opencv2/core/operations.hpp): thread i expands
// segment i from its start state (computed on the host by jump-ahead) with the MWC recurrence
// state = (u32)state * 4164903690 + (state >> 32), emitting the low 32 bits.
__global__ __launch_bounds__(256) void rng_stream_kernel(const unsigned long long* __restrict__ seg_state,
                                                         uint32_t* __restrict__ out, long long len, int seg,
                                                         int n_seg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_seg) return;
    unsigned long long st = seg_state[i];
    const long long p0 = (long long)i * seg;
    const int m = (int)min((long long)seg, len - p0);
    for (int k = 0; k < m; ++k) {
        out[p0 + k] = (uint32_t)st;
        st = (unsigned long long)(uint32_t)st * 4164903690ull + (st >> 32);
    }
}

void launch_rng_stream(const unsigned long long* seg_state, uint32_t* out, long long len, int seg, int n_seg,
                       hipStream_t s) {
    rng_stream_kernel<<<(n_seg + 255) / 256, 256, 0, s>>>(seg_state, out, len, seg, n_seg);
}

void ransac_enqueue(const RansacParams& prm, int n_probs, const ProbDev* probs, const float4* pts,
                    const int* n_good, const RansacBufs& b, uint8_t* masks, mim_result* results, int raw,
                    hipStream_t s, void (*mark)(void*, const char*, hipStream_t), void* mark_ctx, int exact_all) {
    if (n_probs <= 0) return;
    ransac_init_kernel<<<(n_probs + 255) / 256, 256, 0, s>>>(b.state, n_good, n_probs, prm.max_iters, prm.min_good,
                                                             b.best_h);
    const int max_iters = prm.max_iters > 1 ? prm.max_iters : 1;
    // MIM_SAMPLER_WALK=1: attempt-by-attempt walker only (reference mode for cross-checks)
    const char* sw = getenv("MIM_SAMPLER_WALK");
    const int use_chain = !(sw && sw[0] == '1');
    // first chunk: 4,096 iterations, 512 when maxIters <= 4,096 (findHomography's default 2,000): a
    // problem that terminates early (niters falls after a good model) then never samples the rest —
    // with few, duplicated points getSubset can need ~100 draws per iteration (MIM_FIRST_CHUNK: knob)
    int first = max_iters <= 4096 ? 512 : 4096;
    if (const char* fc = getenv("MIM_FIRST_CHUNK")) first = std::max(1, atoi(fc));
    int c0 = 0, chunk = first;
    const float thr2 = (float)(prm.thresh * prm.thresh);
    if (!exact_all) ransac_tiles_kernel<<<n_probs, 256, 0, s>>>(b.state, probs, pts, b.tiles);
    // the getSubset replay on the sampler stream when there is one (not in the reference mode)
    const bool split = b.s2 && !exact_all;
    hipStream_t ss = split ? b.s2 : s;
    if (split) {
        (void)hipEventRecord(b.ev_fork, s);
        (void)hipStreamWaitEvent(ss, b.ev_fork, 0);
        mark(mark_ctx, "fork", ss);
    }
    int ci = 0, c1_first = 0;
    // listed candidates per problem and chunk (MIM_CAND_CAP < 1024: test knob forcing the replay's
    // overflow rescan)
    const int cap = prm.cand_cap > 0 ? std::min(prm.cand_cap, kCandCap) : kCandCap;
    // candidate prescreen in the cand kernel (MIM_PRESCREEN=0: every listed candidate through the exact kernel)
    const char* pe = getenv("MIM_PRESCREEN");
    const int prescreen = (pe && pe[0] == '0') ? 0 : 1;
    // settling irrelevant candidates after the prescreen (MIM_SETTLE=0: off)
    const char* se = getenv("MIM_SETTLE");
    const int settle = (se && se[0] == '0') ? 0 : 1;
    // the chunk's largest decided candidate through the exact pass as well: by default for problems of
    // fewer than kWinnerHMaxN good matches (MIM_WINNER_H=1: every problem, 0: none)
    const char* we = getenv("MIM_WINNER_H");
    const int winner_h = !we ? 2 : we[0] == '1' ? 1 : we[0] == '0' ? 0 : 2;
    // the sampler grids' floor (MIM_SAMPLER_MIN_BLOCKS: blocks in all; 0 = only what the window needs)
    int min_blocks = kSamplerMinBlocks;
    if (const char* mb = getenv("MIM_SAMPLER_MIN_BLOCKS")) min_blocks = std::max(0, atoi(mb));
    while (c0 < max_iters) {
        const int c1 = (int)std::min<long long>((long long)c0 + chunk, max_iters);
        // attempt outcomes for a window of ~28 draws per wanted iteration (pass rate ~1/5), the walk
        // falls back to inline evaluation past the window
        // (a multiple of 64: flags are read as 16-byte vectors, pass bits as 32-bit words)
        const int wcap = (int)(std::min<long long>((long long)(c1 - c0) * 28 + 4096, b.flag_cap / std::max(n_probs, 1)) & ~63LL);
        // grids for the window a typical draw rate implies (the kernels loop over a longer one)
        const int west = (int)std::min<long long>(wcap, (long long)(c1 - c0) * kAttemptRateEst + 4096);
        // at least kSamplerMinBlocks blocks in all while the window holds that many slices (a small batch's
        // first chunk would otherwise leave most of the GPU idle), a multiple of 8 per problem (placement)
        const int bppw_cap = std::max(1, wcap / kAttemptSpan);
        const int bppw = (std::max((west + kAttemptSpan - 1) / kAttemptSpan,
                                   std::min(bppw_cap, (min_blocks + n_probs - 1) / n_probs)) + 7) / 8 * 8;
        // (MIM_ATTEMPT_REP_CAP < kAttemptRepCap: test knob forcing the in-place redraw resolution)
        const int rep_cap = prm.rep_cap > 0 ? std::min(prm.rep_cap, kAttemptRepCap) : kAttemptRepCap;
        ransac_attempt_kernel<<<n_probs * bppw, 256, 0, ss>>>(b.state, b.stream, b.stream_len, b.flags, b.irr_bits, wcap,
                                                             bppw, c1, rep_cap, n_probs);
        mark(mark_ctx, "attempt", ss);
        if (use_chain) {
            ChainSegs* chains = reinterpret_cast<ChainSegs*>(b.chains);
            const int bpp_irr = (west + kIrrBlock - 1) / kIrrBlock;
            ransac_irr_kernel<<<n_probs * bpp_irr, 256, 0, ss>>>(b.state, b.irr_bits, wcap, bpp_irr, c1, b.irr,
                                                               b.irr_cnt, b.irr_blocks);
            ransac_walk_kernel<<<n_probs, kWalkThreads, 0, ss>>>(b.state, b.flags, wcap, c1, b.irr, b.irr_cnt,
                                                                 b.irr_blocks, chains);
            mark(mark_ctx, "chain", ss);
            constexpr int kChkSpan = kCheckBlock * kCheckPer;
            const int bpp_chk = std::max((west / 4 + kChkSpan) / kChkSpan,  // T ~ wlen / 4
                                         std::min(std::max(1, wcap / 4 / kChkSpan), (min_blocks + n_probs - 1) / n_probs));
            ransac_check_kernel<<<8 * ((n_probs + 7) / 8) * bpp_chk, kCheckBlock, 0, ss>>>(
                chains, probs, pts, b.state, b.stream, b.stream_len, b.pass_bits, wcap, bpp_chk, b.defer, b.defer_n,
                b.def_rounds, n_probs);
            if (b.def_rounds > 0) {
                const int nblk = (b.def_rounds * kDefSlots + 255) / 256;
                ransac_check_defer_kernel<<<n_probs * nblk, 256, 0, ss>>>(chains, probs, pts, b.state, b.stream,
                                                                        b.stream_len, b.pass_bits, wcap, b.defer,
                                                                        b.defer_n, b.def_rounds, nblk, n_probs);
            }
            mark(mark_ctx, "check", ss);
            ransac_count_kernel<<<n_probs, kChainThreads, 0, ss>>>(b.state, probs, chains, b.pass_bits, b.flags, wcap,
                                                                  b.samples, c1);
            mark(mark_ctx, "chain", ss);
        }
        ransac_small_kernel<<<n_probs, kSmallThreads, 0, ss>>>(b.state, probs, pts, b.stream, b.stream_len, b.samples,
                                                              c1, b.err);
        ransac_sample_kernel<<<n_probs, 64, 0, ss>>>(b.state, probs, pts, b.stream, b.stream_len, b.samples, c1, b.err,
                                                    b.flags, b.irr_bits, wcap, use_chain);
        mark(mark_ctx, "sample", ss);
        if (split) {  // this chunk's selection waits for its samples; the next chunk's sampler does not
            (void)hipEventRecord(b.ev_samp[ci & 1], ss);
            (void)hipStreamWaitEvent(s, b.ev_samp[ci & 1], 0);
            mark(mark_ctx, "join", s);  // span origin of the selection kernels after the wait
        }
        ++ci;
        const int bpp256 = (c1 - c0 + 255) / 256;
        const int bppb = (c1 - c0 + kBoundThreads - 1) / kBoundThreads;
        if (exact_all) {  // reference mode: every hypothesis through runKernel + computeError
            const int bpp64 = (c1 - c0 + 63) / 64;
            ransac_hypo_kernel<<<n_probs * bpp64, 64, 0, s>>>(b.state, probs, pts, b.samples, b.stream, b.hyp, b.counts, c0, c1,
                                                             bpp64);
            mark(mark_ctx, "hypo", s);
            ransac_score_kernel<<<n_probs * bpp256, 256, 0, s>>>(b.state, probs, pts, b.hyp, b.counts, c0, c1,
                                                                bpp256, thr2);
            mark(mark_ctx, "score", s);
            ransac_select_kernel<<<n_probs, 64, 0, s>>>(b.state, probs, b.counts, c1, prm.conf);
            mark(mark_ctx, "select", s);
            if (getenv("MIM_DEBUG_TRACE") && n_probs == 1) {  // debug: problem 0's samples and exact counts
                std::vector<int> hc(c1 - c0);
                std::vector<int4> hs(c1 - c0);
                (void)hipMemcpyAsync(hc.data(), b.counts + c0, sizeof(int) * (c1 - c0), hipMemcpyDeviceToHost, s);
                (void)hipMemcpyAsync(hs.data(), b.samples + c0, sizeof(int4) * (c1 - c0), hipMemcpyDeviceToHost, s);
                (void)hipStreamSynchronize(s);
                for (int i = 0; i < c1 - c0; ++i)
                    fprintf(stderr, "[trace] %d %d %d %d %d %d\n", c0 + i, hc[i], hs[i].x, hs[i].y, hs[i].z, hs[i].w);
            }
        } else {
            if (c0 == 0)
                ransac_bound_mfma_kernel<true><<<8 * ((n_probs + 7) / 8) * bppb, kBoundThreads, 0, s>>>(
                    b.state, probs, pts, b.samples, b.stream, b.tiles, b.bounds, c0, c1, bppb, thr2, n_probs);
            else
                ransac_bound_mfma_kernel<false><<<8 * ((n_probs + 7) / 8) * bppb, kBoundThreads, 0, s>>>(
                    b.state, probs, pts, b.samples, b.stream, b.tiles, b.bounds, c0, c1, bppb, thr2, n_probs);
            mark(mark_ctx, "score", s);
            if (getenv("MIM_CHECK_BOUNDS")) {  // debug: every bracket against the exact count
                unsigned long long* dst = nullptr;
                unsigned long long h[6] = {0, 0, 0, 0, 0, 0};
                if (hipMalloc(&dst, sizeof h) == hipSuccess) {
                    (void)hipMemsetAsync(dst, 0, sizeof h, s);
                    const int bpp64 = (c1 - c0 + 63) / 64;
                    ransac_bound_check_kernel<<<n_probs * bpp64, 64, 0, s>>>(b.state, probs, pts, b.samples, b.stream,
                                                                             b.bounds, c0, c1, bpp64, thr2, dst);
                    (void)hipMemcpyAsync(h, dst, sizeof h, hipMemcpyDeviceToHost, s);
                    (void)hipStreamSynchronize(s);
                    (void)hipFree(dst);
                }
                fprintf(stderr, "[mim] bound check chunk [%d,%d): checked %llu lo_viol %llu hi_viol %llu valid_mismatch %llu "
                        "mean_width %.2f tight %llu\n", c0, c1, h[0], h[1], h[2], h[3], h[0] ? (double)h[4] / h[0] : 0.0, h[5]);
            }
            const int L = c0 == 0 ? 0 : 1;  // candidate list of this chunk (at most two chunks)
            ransac_cand_kernel<<<n_probs, kCandThreads, 0, s>>>(b.state, probs, b.bounds, c1, b.cand, b.ncand, L,
                                                                cap);
            if (prescreen) {
                ransac_prescreen_kernel<<<n_probs * kPreWaves, 64, 0, s>>>(b.state, probs, b.bounds, pts, b.samples,
                                                                          b.stream, b.cand, b.ncand, b.cex, b.cH,
                                                                          b.decided, thr2, L, cap);
                if (settle)
                    ransac_settle_kernel<<<n_probs, 64, 0, s>>>(b.state, probs, b.bounds, b.cand, b.ncand, b.cex, b.cH,
                                                                b.decided, L, cap, winner_h);
            }
            mark(mark_ctx, "cand", s);
            if (prescreen && getenv("MIM_CHECK_PRESCREEN")) {  // debug: decided candidates recounted exactly
                unsigned long long* dst = nullptr;
                unsigned long long h[2] = {0, 0};
                if (hipMalloc(&dst, sizeof h) == hipSuccess) {
                    (void)hipMemsetAsync(dst, 0, sizeof h, s);
                    ransac_prescreen_check_kernel<<<n_probs * (kCandCap / 64), 64, 0, s>>>(
                        b.state, probs, pts, b.samples, b.stream, b.cand, b.ncand, b.cex, b.decided, b.bounds,
                        thr2, L, cap, dst);
                    (void)hipMemcpyAsync(h, dst, sizeof h, hipMemcpyDeviceToHost, s);
                    (void)hipStreamSynchronize(s);
                    (void)hipFree(dst);
                }
                fprintf(stderr, "[mim] prescreen check chunk [%d,%d): decided %llu mismatch %llu\n", c0, c1, h[0], h[1]);
            }
            if (getenv("MIM_DEBUG_NCAND")) {
                std::vector<int> h(2 * n_probs), dec((size_t)2 * n_probs * kCandCap);
                (void)hipMemcpyAsync(h.data(), b.ncand, sizeof(int) * 2 * n_probs, hipMemcpyDeviceToHost, s);
                if (prescreen)
                    (void)hipMemcpyAsync(dec.data(), b.decided, sizeof(int) * dec.size(), hipMemcpyDeviceToHost, s);
                (void)hipStreamSynchronize(s);
                long long sum = 0, sum2 = 0; int mx = 0;
                for (int i = 0; i < n_probs; ++i) {
                    const int nl = std::min(h[2 * i + L], cap);
                    sum += h[2 * i + L];
                    mx = std::max(mx, h[2 * i + L]);
                    for (int k = 0; k < nl; ++k) sum2 += prescreen ? dec[(size_t)(2 * i + L) * kCandCap + k] == 0 : 1;
                }
                fprintf(stderr, "[mim] chunk [%d,%d): candidates mean %.1f max %d undecided mean %.1f\n", c0, c1,
                        (double)sum / n_probs, mx, (double)sum2 / n_probs);
            }
            // chunk 2 also evaluates the list of every problem whose chunk-1 pass was deferred
            ransac_exact_kernel<<<n_probs * kExactWaves * (L + 1), 64, 0, s>>>(b.state, probs, pts, b.samples, b.stream,
                                                                             b.cand, b.ncand, b.bounds, b.cex, b.cH,
                                                                             thr2, L, cap, b.decided, prescreen);
            mark(mark_ctx, "exact", s);
            ransac_replay_kernel<<<n_probs, 64, 0, s>>>(b.state, probs, pts, b.samples, b.stream, b.bounds, b.cand,
                                                        b.ncand, b.cex, b.cH, c1, prm.conf, thr2, b.best_h, L,
                                                        c1_first, cap);
            mark(mark_ctx, "select", s);
        }
        if (c0 == 0) c1_first = c1;
        c0 = c1;
        chunk = 1 << 30;  // one chunk after the first: every chunk costs a latency-bound exact pass
    }
    if (getenv("MIM_CHECK_BESTH")) {  // debug: problems whose bestModel the refine must recompute itself
        std::vector<double> bh((size_t)n_probs * 9);
        std::vector<RansacState> hs(n_probs);
        (void)hipMemcpyAsync(bh.data(), b.best_h, sizeof(double) * bh.size(), hipMemcpyDeviceToHost, s);
        (void)hipMemcpyAsync(hs.data(), b.state, sizeof(RansacState) * n_probs, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        int with = 0, without = 0;
        for (int i = 0; i < n_probs; ++i)
            if (hs[i].active && hs[i].best_iter >= 0 && hs[i].n >= kSmallMaxN) (bh[9 * i + 8] != 0.0 ? with : without)++;
        fprintf(stderr, "[mim] best_h: %d problems with the exact pass's fp64 bestModel, %d without\n", with, without);
    }
    ransac_refine_kernel<<<(n_probs + kRW - 1) / kRW, kRT, 0, s>>>(b.state, probs, pts, n_good, b.samples, b.stream, b.inl,
                                                                  masks, results, prm, raw, b.best_h, exact_all, n_probs);
    mark(mark_ctx, "refine", s);
}

}  // namespace mim
