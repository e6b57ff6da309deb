// Probe: does v_mfma_f32_32x32x16_f16 keep f16 subnormal inputs, and the operand/result lane maps.
#include <hip/hip_runtime.h>
#include <cstdio>
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
int run(float scale) {
    _Float16 hA[32 * 16], hB[16 * 32];
    float ref[32 * 32], out[32 * 32];
    for (int i = 0; i < 32; ++i)
        for (int kk = 0; kk < 16; ++kk) hA[i * 16 + kk] = (_Float16)((float)((i * 7 + kk * 3) % 11 - 5) * scale);
    for (int kk = 0; kk < 16; ++kk)
        for (int j = 0; j < 32; ++j) hB[kk * 32 + j] = (_Float16)((float)((kk * 5 + j) % 7 - 3));
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            double s = 0;
            for (int kk = 0; kk < 16; ++kk) s += (double)(float)hA[i * 16 + kk] * (double)(float)hB[kk * 32 + j];
            ref[i * 32 + j] = (float)s;
        }
    _Float16 *dA, *dB; float* dC;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof out);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dB, dC);
    hipMemcpy(out, dC, sizeof out, hipMemcpyDeviceToHost);
    int bad = 0; double maxrel = 0;
    for (int i = 0; i < 1024; ++i) {
        if (out[i] != ref[i]) ++bad;
        if (ref[i] != 0) maxrel = fmax(maxrel, fabs(out[i] - ref[i]) / fabs(ref[i]));
    }
    printf("A scale %g: mismatches %d / 1024, max rel %.3g, sample out %.6g ref %.6g\n", scale, bad, maxrel,
           out[5], ref[5]);
    return bad;
}
int main() { run(1.f); run(0x1p-20f); run(0x1p-24f); return 0; }
