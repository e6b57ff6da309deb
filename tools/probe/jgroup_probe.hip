// Latency probe: cooperative 16-lane Jacobi (run_kernel4_group) vs lane-per-matrix run_kernel4 on
// gfx950, with clock64 calibrated against the 100 MHz realtime counter.
#include "../../computervision_objectdetection_featurematching_amd/csrc/ransac.hip"
#include <cstdio>
#include <cstdlib>

using namespace mim;

__device__ __forceinline__ int jacobi9_group_prof(double* __restrict__ A, double* __restrict__ W, double* __restrict__ V, long long* tp) {
    long long tc = clock64(); int nrot = 0;
#define TP(k) { long long t_ = clock64(); tp[k] += t_ - tc; tc = t_; }
    constexpr int n = 9;
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
        double p = 0.0;
        int pos = 99, kl = 0;
        if (slot < n) {
            const double vr = slot < n - 1 ? A[pk<n>(slot, indR)] : 0.0;
            const double vc = slot > 0 ? A[pk<n>(indC, slot)] : 0.0;
            const bool row = slot < n - 1 && (slot == 0 || fabs(vr) >= fabs(vc));
            p = row ? vr : vc;
            pos = row ? slot : slot + n - 2;
            kl = row ? (slot | (indR << 8)) : (indC | (slot << 8));
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double po = dpp_row_d(p, c);
            const int poso = dpp_row(pos, c), klo = dpp_row(kl, c);
            // bitwise: no short-circuit branches
            const bool take = (fabs(po) > fabs(p)) | ((fabs(po) == fabs(p)) & (poso < pos));
            p = take ? po : p;
            pos = take ? poso : pos;
            kl = take ? klo : kl;
        }
        TP(0);
        if (fabs(p) <= eps) break;
        ++nrot;
        const int k = kl & 255, l = kl >> 8;  // k < l
        // ---- the pair of this slot ----
        int im = slot - n;  // slots 9..15: the (slot-9)-th index outside {k, l}
        if (im >= k) ++im;
        if (im >= l) ++im;
        const bool vslot = slot < n;
        const int ia = vslot ? k * n + slot : pk_any<n>(im, k);
        const int ib = vslot ? l * n + slot : pk_any<n>(im, l);
        double* base = vslot ? V : A;
        const double a0 = base[ia], b0 = base[ib];
        const double wk = W[k], wl = W[l];
        const double y = (wl - wk) * 0.5;
        double t = fabs(y) + d_hypot(p, y);
        double s = d_hypot(p, t);
        const double c = t / s;
        s = p / s;
        t = (p / t) * p;
        s = y < 0 ? -s : s;
        t = y < 0 ? -t : t;
        TP(1);
        const double na = a0 * c - b0 * s;
        const double nb = a0 * s + b0 * c;
        base[ia] = na;
        base[ib] = nb;
        if (slot == 0) {
            A[pk<n>(k, l)] = 0;
            W[k] = wk - t;
            W[l] = wl + t;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        TP(2);
        // ---- refresh the cached maxima of rows/columns k and l (row k: A(k,i) = na of the A
        // slots, plus A(k,l) = 0; row l: nb, plus A(l,k) = 0) ----
        const bool aslot = !vslot;
        const double va = fabs(na), vb = fabs(nb);
        const int rk = refresh_argmax(va, aslot & (im > k), k, l, l);
        const int ck = refresh_argmax(va, aslot & (im < k), k, l, -1);
        const int rl = refresh_argmax(vb, aslot & (im > l), k, l, -1);
        const int cl = refresh_argmax(vb, aslot & (im < l), k, l, k);
        if (slot == k) {
            if (k < n - 1) indR = rk;
            if (k > 0) indC = ck;
        }
        if (slot == l) {
            if (l < n - 1) indR = rl;
            if (l > 0) indC = cl;
        }
        TP(3);
    }
    tp[4] = nrot;
    // ---- OpenCV's selection sort (descending), tracked as a permutation ----
    double Ws[n];
    int perm[n];
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
    return perm[n - 1];
}


__global__ __launch_bounds__(64) void prof_kernel(const float* pts, long long* tp) {
    __shared__ double sd[4 * kJ9G];
    const int lane = threadIdx.x, grp = lane >> 4;
    const float* q = pts + grp * 16;
    float M[8], m[8];
    for (int i = 0; i < 8; ++i) { M[i] = q[i]; m[i] = q[8 + i]; }
    // the DLT of run_kernel4_group, then the timed Jacobi
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    for (int i = 0; i < 4; i++) { cmx += m[2 * i]; cmy += m[2 * i + 1]; cMx += M[2 * i]; cMy += M[2 * i + 1]; }
    cmx /= 4; cmy /= 4; cMx /= 4; cMy /= 4;
    for (int i = 0; i < 4; i++) { smx += fabs(m[2 * i] - cmx); smy += fabs(m[2 * i + 1] - cmy); sMx += fabs(M[2 * i] - cMx); sMy += fabs(M[2 * i + 1] - cMy); }
    smx = 4 / smx; smy = 4 / smy; sMx = 4 / sMx; sMy = 4 / sMy;
    double* D = sd + grp * kJ9G;
    dlt_entries_group(M, m, 4, cmx, cmy, cMx, cMy, smx, smy, sMx, sMy, D, D + 36);
    __builtin_amdgcn_wave_barrier();
    long long t[5] = {0, 0, 0, 0, 0};
    int r = jacobi9_group_prof(D, D + 36, D + 45, t);
    if (lane == 0) for (int i = 0; i < 5; ++i) tp[i] = t[i];
    if (lane == 0) tp[5] = r;
}
__global__ __launch_bounds__(64) void grp_kernel(const float* pts, double* out, long long* cyc) {
    __shared__ double sd[4 * kJ9G];
    const int lane = threadIdx.x, grp = lane >> 4;
    const float* q = pts + grp * 16;
    float M[8], m[8];
    for (int i = 0; i < 8; ++i) { M[i] = q[i]; m[i] = q[8 + i]; }
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = clock64();
    double H[9];
    int ok = run_kernel4_group(M, m, sd + grp * kJ9G, H);
    const long long t1 = clock64();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((lane & 15) == 0) for (int i = 0; i < 9; ++i) out[grp * 9 + i] = ok ? H[i] : -1;
    if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

__global__ __launch_bounds__(64) void lane_kernel(const float* pts, double* out, long long* cyc) {
    __shared__ double sd[kJ9D * 64];
    const int lane = threadIdx.x;
    if (lane >= 4) return;
    const float* q = pts + lane * 16;
    float M[8], m[8];
    for (int i = 0; i < 8; ++i) { M[i] = q[i]; m[i] = q[8 + i]; }
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = clock64();
    double H[9];
    int ok = run_kernel4<64>(M, m, sd + lane, H);
    const long long t1 = clock64();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < 9; ++i) out[36 + lane * 9 + i] = ok ? H[i] : -1;
    if (lane == 0) { cyc[2] = t1 - t0; cyc[3] = r1 - r0; }
}

int main() {
    float h[64];
    srand(3);
    for (int i = 0; i < 64; ++i) h[i] = (float)(rand() % 64000) / 100.f;
    float* d; double* o; long long* c;
    hipMalloc(&d, sizeof h); hipMalloc(&o, 72 * 8); hipMalloc(&c, 8 * 4);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    {
        long long* tp; hipMalloc(&tp, 64);
        for (int rep = 0; rep < 2; ++rep) {
            prof_kernel<<<1, 64>>>(d, tp);
            long long h5[6]; hipMemcpy(h5, tp, 48, hipMemcpyDeviceToHost);
            printf("jacobi phases (cycles): pivot %lld rotate-prep %lld rotate %lld refresh %lld | rotations %lld r %lld\n", h5[0], h5[1], h5[2], h5[3], h5[4], h5[5]);
        }
    }
    for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1, e2; hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
        hipEventRecord(e0);
        grp_kernel<<<1, 64>>>(d, o, c);
        hipEventRecord(e1);
        lane_kernel<<<1, 64>>>(d, o, c);
        hipEventRecord(e2); hipEventSynchronize(e2);
        float ms1, ms2; hipEventElapsedTime(&ms1, e0, e1); hipEventElapsedTime(&ms2, e1, e2);
        long long cy[4]; hipMemcpy(cy, c, 32, hipMemcpyDeviceToHost);
        double ho[72]; hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
        int same = 1;
        for (int i = 0; i < 36; ++i) same &= ho[i] == ho[36 + i];
        printf("group: %.3f ms, clock64 %lld, realtime %lld (%.1f us) | lane: %.3f ms, clock64 %lld, realtime %lld (%.1f us) | same %d\n",
               ms1, cy[0], cy[1], cy[1] / 100.0, ms2, cy[2], cy[3], cy[3] / 100.0, same);
    }
    return 0;
}
