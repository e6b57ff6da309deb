// Probe: accuracy of v_mfma_f32_32x32x16_f16 on a cancelling dot product of mixed magnitudes (normal
// hi parts + subnormal lo parts of f16-split factors), the situation of the RANSAC bound kernel's
// X - uW for a sample point (mfma_cancel_vec.h: point 89 of tests/test_bounds_corpus_gpu.py
// big_persp:22 against its violating hypothesis).  Prints the MFMA result against the exact sum,
// then the same with every subnormal operand flushed, and a per-slot scan.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "mfma_cancel_vec.h"
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
__global__ void k(const _Float16* A, const _Float16* B, float* C) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    h8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = A[r * 16 + 8 * h + j]; b[j] = B[(8 * h + j) * 32 + r]; }
    f16v c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}
static double run(const float* av, const float* bv, double* exact) {
    _Float16 hA[32 * 16] = {}, hB[16 * 32] = {};
    for (int kk = 0; kk < 16; ++kk) { hA[kk] = (_Float16)av[kk]; hB[kk * 32] = (_Float16)bv[kk]; }
    double s = 0;
    for (int kk = 0; kk < 16; ++kk) s += (double)(float)hA[kk] * (double)(float)hB[kk * 32];
    *exact = s;
    _Float16 *dA, *dB; float* dC; float out[1024];
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof out);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dB, dC);
    hipMemcpy(out, dC, sizeof out, hipMemcpyDeviceToHost);
    hipFree(dA); hipFree(dB); hipFree(dC);
    return out[0];
}
int main() {
    double ex;
    double m = run(AX, BX, &ex);
    printf("mfma %.9g exact %.9g err %.3g\n", m, ex, m - ex);
    float af[16], bf[16];
    for (int i = 0; i < 16; ++i) { af[i] = fabsf(AX[i]) < 6.103515625e-05f ? 0.f : AX[i]; bf[i] = fabsf(BX[i]) < 6.103515625e-05f ? 0.f : BX[i]; }
    double e2; double m2 = run(af, bf, &e2);
    printf("flushed-subnormal inputs: mfma %.9g exact(flushed) %.9g | vs unflushed exact err %.3g\n", m2, e2, m2 - ex);
    // single subnormal product vs one large term: 0.5 * 1 + 2^-16 * 1 (normal) / 2^-20 * 1 (subnormal)
    for (int sh = 14; sh <= 24; sh += 2) {
        float a2[16] = {0.5f, ldexpf(1.f, -sh)}, b2[16] = {1.f, 1.f};
        double e3; double m3 = run(a2, b2, &e3);
        printf("0.5 + 2^-%d: mfma %.12g exact %.12g err %.3g\n", sh, m3, e3, m3 - e3);
    }
    return 0;
}
