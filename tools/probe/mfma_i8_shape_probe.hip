// Probe: sustained i8 MFMA throughput and in-kernel clock of the two gfx950 i8 shapes in an
// LDS-fed loop shaped like the distance kernel (4 waves per SIMD, A fragments read from LDS per
// k-step, B in registers, two accumulators per wave).  Random operands (DVFS depends on data).
//   hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_i8_shape_probe.hip -o tools/probe/mfma_i8_shape_probe
// Prints TOPS, the in-kernel clock (s_memtime / s_memrealtime x 100 MHz) and the MFMA-bound floor.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kIters = 4096;

template <bool k16>
__global__ __launch_bounds__(512, 4) void probe(const i32x4* __restrict__ src, int* __restrict__ out,
                                                unsigned long long* __restrict__ stamps) {
    __shared__ i32x4 lds[8 * 512];  // 64 KiB of fragments
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 8 * 512; i += 512) lds[i] = src[(blockIdx.x * 8 * 512 + i) & ((1 << 20) - 1)];
    __syncthreads();
    i32x4 b0 = src[(tid * 7 + 3) & 1023], b1 = src[(tid * 11 + 5) & 1023];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    int x = 0;
    if (k16) {
        // 16x16x64: 16384 MACs per MFMA, 2 per k-step pair to match a 32x32x32's work
        i32x4 c[4] = {};
        for (int it = 0; it < kIters; ++it) {
            const i32x4 a = lds[((it & 7) * 512 + tid) & 4095];
#pragma unroll
            for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, j & 1 ? b1 : b0, c[j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) x ^= c[j][0] ^ c[j][1] ^ c[j][2] ^ c[j][3];
    } else {
        i32x16 c[2] = {};
        for (int it = 0; it < kIters; ++it) {
            const i32x4 a = lds[((it & 7) * 512 + tid) & 4095];
            c[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b0, c[0], 0, 0, 0);
            c[1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b1, c[1], 0, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < 16; ++g) x ^= c[0][g] ^ c[1][g];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 512 + tid] = x;
    if (tid == 0) {
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    const int blocks = 256 * 2 * 8;  // 8 rounds of 2 blocks (16 waves) per CU
    std::vector<int> h(1 << 22);
    srand(1);
    for (auto& v : h) v = rand();
    i32x4* src;
    int* out;
    unsigned long long* st;
    hipMalloc(&src, sizeof(int) << 22);
    hipMalloc(&out, sizeof(int) * blocks * 512);
    hipMalloc(&st, 16 * blocks);
    hipMemcpy(src, h.data(), sizeof(int) << 22, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int shape = 0; shape < 2; ++shape) {
        for (int rep = 0; rep < 6; ++rep) {
            hipEventRecord(e0);
            if (shape) probe<true><<<blocks, 512>>>(src, out, st);
            else probe<false><<<blocks, 512>>>(src, out, st);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            std::vector<unsigned long long> s(2 * blocks);
            hipMemcpy(s.data(), st, 16 * blocks, hipMemcpyDeviceToHost);
            double ct = 0, rt = 0;
            for (int b = 0; b < blocks; ++b) { ct += s[2 * b]; rt += s[2 * b + 1]; }
            const double ghz = ct / rt * 0.1;  // s_memrealtime ticks at 100 MHz
            const double ops = 2.0 * blocks * 8.0 * kIters * 2 * 32768;  // 8 waves, 2 x 32x32x32 per k-step
            const double floor_ms = blocks * 8.0 * kIters * 2 * 32 / 1024.0 / (ghz * 1e9) * 1e3;
            if (rep >= 2)
                printf("%s  %.3f ms  %.0f TOPS  clock %.2f GHz  MFMA floor at that clock %.3f ms (%.0f %%)\n",
                       shape ? "16x16x64" : "32x32x32", ms, ops / ms / 1e9, ghz, floor_ms, 100.0 * floor_ms / ms);
        }
    }
    return 0;
}
