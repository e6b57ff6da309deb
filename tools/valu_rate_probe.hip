// VALU issue-rate probe: wave64 v_fma_f32 throughput per SIMD at 1, 2, 4, 8 waves per SIMD.
// Each wave runs ITER x 64 independent fmas (8 chains); one block of 64*W*4 threads per CU (W waves per
// SIMD), grid = CUs.  Reports cycles per wave-instruction per SIMD from wall time and the clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
constexpr int ITER = 4096;
__global__ void fma_loop(float* out, float a, float b) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    if (s == 12345.f) out[0] = s;
}
// dependent chain variant: one chain per wave (latency-bound alone)
__global__ void fma_dep(float* out, float a, float b) {
    float x = threadIdx.x * 0.001f;
    for (int it = 0; it < ITER * 64; ++it) x = __builtin_fmaf(x, a, b);
    if (x == 12345.f) out[0] = x;
}
int main() {
    int dev = 0, cus = 0, clk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    float* out;
    hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("CUs %d, clock attr %.0f MHz\n", cus, clk / 1e3);
    for (int dep = 0; dep < 2; ++dep)
        for (int W : {1, 2, 4, 8}) {
            const int threads = 64 * 4 * W;  // W waves per SIMD (4 SIMDs)
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (dep) fma_dep<<<cus, threads>>>(out, 0.999f, 0.001f);
                else fma_loop<<<cus, threads>>>(out, 0.999f, 0.001f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                const double instr_per_simd = (double)W * ITER * 64;  // wave-instructions per SIMD
                if (rep == 2)
                    printf("%s W=%d: %.3f ms, %.2f ns per wave-instr per SIMD (= %.2f cycles at 2.4 GHz, %.2f at 2.0)\n",
                           dep ? "dep " : "indep", W, ms, ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4,
                           ms * 1e6 / instr_per_simd * 2.0);
            }
        }
    return 0;
}
