// Probe: verify MFMA operand/accumulator lane maps on gfx950 with exact integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(16))) int i32x16;
typedef __attribute__((ext_vector_type(4))) int i32x4;

// A: 32x16 (row-major), B: 16x32 (row-major), C = A*B 32x32
__global__ void bf16_probe(const float* A, const float* B, float* C) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)A[r*16 + 8*h + j]; b[j] = (__bf16)B[(8*h + j)*32 + r]; }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int g = 0; g < 16; ++g) { int row = (g&3) + 8*(g>>2) + 4*h; C[row*32 + r] = acc[g]; }
}
// A: 32x32 i8, B: 32x32 i8 ; guess k = 16h + j
__global__ void i8_probe(const int* A, const int* B, int* C) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  int8_t av[16], bv[16];
  for (int j = 0; j < 16; ++j) { av[j] = (int8_t)A[r*32 + 16*h + j]; bv[j] = (int8_t)B[(16*h + j)*32 + r]; }
  i32x4 a, b;
  __builtin_memcpy(&a, av, 16); __builtin_memcpy(&b, bv, 16);
  i32x16 acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
  for (int g = 0; g < 16; ++g) { int row = (g&3) + 8*(g>>2) + 4*h; C[row*32 + r] = acc[g]; }
}
__global__ void div_probe(const float* x, float* y, int n) {
  int i = blockIdx.x*blockDim.x + threadIdx.x;
  if (i < n) y[i] = 1.f / x[i];
}
__global__ void sqrt_probe(const float* x, float* y, int n) {
  int i = blockIdx.x*blockDim.x + threadIdx.x;
  if (i < n) y[i] = sqrtf(x[i]);
}
int main() {
  float hA[32*16], hB[16*32], hC[32*32];
  srand(1);
  for (int i = 0; i < 32*16; ++i) hA[i] = (float)(rand() % 256);
  for (int i = 0; i < 16*32; ++i) hB[i] = (float)(rand() % 256) * -2.f;
  float *dA, *dB, *dC;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  bf16_probe<<<1, 64>>>(dA, dB, dC);
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
    double s = 0; for (int k = 0; k < 16; ++k) s += (double)hA[i*16+k] * hB[k*32+j];
    if (s != hC[i*32+j]) ++bad;
  }
  printf("bf16 32x32x16 map mismatches: %d\n", bad);
  int iA[32*32], iB[32*32], iC[32*32];
  for (int i = 0; i < 32*32; ++i) { iA[i] = rand() % 256 - 128; iB[i] = rand() % 256 - 128; }
  int *diA, *diB, *diC;
  hipMalloc(&diA, sizeof iA); hipMalloc(&diB, sizeof iB); hipMalloc(&diC, sizeof iC);
  hipMemcpy(diA, iA, sizeof iA, hipMemcpyHostToDevice); hipMemcpy(diB, iB, sizeof iB, hipMemcpyHostToDevice);
  i8_probe<<<1, 64>>>(diA, diB, diC);
  hipMemcpy(iC, diC, sizeof iC, hipMemcpyDeviceToHost);
  bad = 0;
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
    long s = 0; for (int k = 0; k < 32; ++k) s += (long)iA[i*32+k] * iB[k*32+j];
    if (s != iC[i*32+j]) ++bad;
  }
  printf("i8 32x32x32 map (k=16h+j) mismatches: %d\n", bad);
  // correctly rounded division / sqrt check on random floats
  const int n = 1 << 22;
  float* hx = (float*)malloc(n*4); float* hy = (float*)malloc(n*4);
  for (int i = 0; i < n; ++i) { unsigned u = (unsigned)rand() * 2654435761u; u = (u & 0x007fffff) | (((u >> 23) % 60 + 97) << 23); hx[i] = *(float*)&u; }
  float *dx, *dy; hipMalloc(&dx, n*4); hipMalloc(&dy, n*4);
  hipMemcpy(dx, hx, n*4, hipMemcpyHostToDevice);
  div_probe<<<n/256, 256>>>(dx, dy, n);
  hipMemcpy(hy, dy, n*4, hipMemcpyDeviceToHost);
  bad = 0; for (int i = 0; i < n; ++i) if (hy[i] != 1.f / hx[i]) ++bad;
  printf("fp32 div mismatches vs host: %d / %d\n", bad, n);
  sqrt_probe<<<n/256, 256>>>(dx, dy, n);
  hipMemcpy(hy, dy, n*4, hipMemcpyDeviceToHost);
  bad = 0; for (int i = 0; i < n; ++i) if (hy[i] != sqrtf(hx[i])) ++bad;
  printf("fp32 sqrt mismatches vs host: %d / %d\n", bad, n);
  return 0;
}
