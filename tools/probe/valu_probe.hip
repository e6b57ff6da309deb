// VALU issue-rate probe: scalar fma vs packed fma (v_pk_fma_f32), 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void k_fma(float* out, int iters, unsigned long long* cyc) {
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
    const float b = 1.0001f, c = 0.5f;
    const unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_fmaf(a[i], b, c);
    }
    const unsigned long long t1 = clock64();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_pkfma(float* out, int iters, unsigned long long* cyc) {
    f2 a[8];
    for (int i = 0; i < 8; ++i) a[i] = f2{threadIdx.x * 0.001f + i, i * 0.5f};
    const f2 b = {1.0001f, 1.0002f}, c = {0.5f, 0.25f};
    const unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_elementwise_fma(a[i], b, c);
    }
    const unsigned long long t1 = clock64();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_cmpadd(const float* in, int iters, int* out, unsigned long long* cyc) {
    float v[8];
    for (int i = 0; i < 8; ++i) v[i] = in[threadIdx.x + i];
    int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { cnt[i] += v[i] < (float)it; }
    }
    const unsigned long long t1 = clock64();
    int s = 0;
    for (int i = 0; i < 8; ++i) s += cnt[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out; int* iout; float* in; unsigned long long* cyc;
    hipMalloc(&out, 1 << 24); hipMalloc(&iout, 1 << 24); hipMalloc(&in, 1 << 20); hipMalloc(&cyc, 1 << 16);
    hipMemset(in, 0, 1 << 20);
    const int iters = 4096;
    for (int waves_per_simd : {1, 2, 4, 8}) {
        const int blocks = 256 * 4 * waves_per_simd;  // 1 wave per block
        unsigned long long h[8];
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        for (int kind = 0; kind < 3; ++kind) {
            hipEventRecord(e0);
            if (kind == 0) k_fma<<<blocks, 64>>>(out, iters, cyc);
            else if (kind == 1) k_pkfma<<<blocks, 64>>>(out, iters, cyc);
            else k_cmpadd<<<blocks, 64>>>(in, iters, iout, cyc);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
            const double instr = (double)iters * 8 * (kind == 2 ? 2 : 1);  // cmp+add per element
            const double total_wave_instr = instr * blocks;
            // chip-wide rate: wave-instructions per SIMD per cycle (2.1 GHz nominal), per-wave cycles/instr
            printf("waves/SIMD %d %-8s %.3f ms  per-wave cyc/instr %.2f  chip wave-instr/SIMD/ns %.3f\n", waves_per_simd,
                   kind == 0 ? "fma" : (kind == 1 ? "pk_fma" : "cmp+add"), ms, (double)h[0] / instr,
                   total_wave_instr / 1024 / (ms * 1e6));
        }
    }
    return 0;
}
