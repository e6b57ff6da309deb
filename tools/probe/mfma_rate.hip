// Probe: chip-wide throughput of back-to-back MFMAs (bf16 32x32x16 vs i8 32x32x32 vs i8 16x16x64),
// 4 independent accumulators per wave, operands in registers.  Prints TFLOP/s (TOPS for i8).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(16))) int i32x16;
typedef __attribute__((ext_vector_type(4))) int i32x16_4;
typedef __attribute__((ext_vector_type(4))) int i32x4;
constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void bf16_rate(float* out, int seed) {
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(float)((threadIdx.x + j + seed) & 7); b[j] = (__bf16)(float)((threadIdx.x * 3 + j) & 7); }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < kIters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0; for (int g = 0; g < 16; ++g) s += c0[g] + c1[g] + c2[g] + c3[g];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void i8_rate(int* out, int seed) {
  i32x4 a, b;
  for (int j = 0; j < 4; ++j) { a[j] = 0x01010101 * ((threadIdx.x + j + seed) & 7); b[j] = 0x01020304 + j; }
  i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < kIters; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
  }
  int s = 0; for (int g = 0; g < 16; ++g) s += c0[g] ^ c1[g] ^ c2[g] ^ c3[g];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void i8_16_rate(int* out, int seed) {
  i32x4 a, b;
  for (int j = 0; j < 4; ++j) { a[j] = 0x01010101 * ((threadIdx.x + j + seed) & 7); b[j] = 0x01020304 + j; }
  i32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < kIters; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
  }
  int s = 0; for (int g = 0; g < 4; ++g) s += c0[g] ^ c1[g] ^ c2[g] ^ c3[g];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD over the grid
  void* d; hipMalloc(&d, blocks * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int k = 0; k < 3; ++k) {
    float ms;
    const double waves = blocks * 4.0;
    hipEventRecord(e0); bf16_rate<<<blocks, 256>>>((float*)d, k); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("bf16 32x32x16: %.1f TFLOP/s\n", waves * kIters * 4 * 32768.0 / (ms * 1e-3) / 1e12);
    hipEventRecord(e0); i8_rate<<<blocks, 256>>>((int*)d, k); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("i8 32x32x32:   %.1f TOPS\n", waves * kIters * 4 * 65536.0 / (ms * 1e-3) / 1e12);
    hipEventRecord(e0); i8_16_rate<<<blocks, 256>>>((int*)d, k); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("i8 16x16x64:   %.1f TOPS\n", waves * kIters * 4 * 32768.0 / (ms * 1e-3) / 1e12);
  }
  return 0;
}
