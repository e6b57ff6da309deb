// Probe: issue throughput of single VALU instructions on gfx950 (the bound kernel's per-pair test
// ops and candidate replacements).  Each kernel runs 16 independent chains of one instruction per
// lane; 8 or 1 waves per SIMD; reports ns per wave-instruction per SIMD and the ratio to v_fma_f32.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate_probe tools/probe/valu_rate_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define R16(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7) OP(8) OP(9) OP(10) OP(11) OP(12) OP(13) OP(14) OP(15)
#define OUTS                                                                                          \
    "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), \
        "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])

#define KERNEL(NAME, OP)                                                                  \
    __global__ __launch_bounds__(256) void k_##NAME(float* out, int iters) {             \
        float r[16];                                                                      \
        for (int j = 0; j < 16; ++j) r[j] = 1.f + 1e-3f * (threadIdx.x + j);              \
        float c = 1.0001f, d = 0.25f;                                                     \
        asm volatile("" : "+v"(c), "+v"(d));                                              \
        for (int i = 0; i < iters; ++i) asm volatile(R16(OP) : OUTS : "v"(c), "v"(d) : "vcc"); \
        float s = 0.f;                                                                    \
        for (int j = 0; j < 16; ++j) s += r[j];                                           \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                          \
    }

#define FMA(n) "v_fma_f32 %" #n ", %" #n ", %16, %17\n"
#define FMA_ABS(n) "v_fma_f32 %" #n ", %16, |%" #n "|, %17\n"
#define FMAC(n) "v_fmac_f32_e32 %" #n ", %16, %17\n"
#define MED3_ABS(n) "v_med3_f32 %" #n ", |%" #n "|, |%16|, %17\n"
#define MED3(n) "v_med3_f32 %" #n ", %" #n ", %16, %17\n"
#define MAX_ABS(n) "v_max_f32_e64 %" #n ", |%" #n "|, |%16|\n"
#define MAX_E32(n) "v_max_f32_e32 %" #n ", %" #n ", %16\n"
#define MAX3_ABS(n) "v_max3_f32 %" #n ", |%" #n "|, |%16|, %17\n"
#define SUB(n) "v_sub_f32_e32 %" #n ", %16, %" #n "\n"
#define SUB_ABS(n) "v_sub_f32_e64 %" #n ", %16, |%" #n "|\n"
#define ADD(n) "v_add_f32_e32 %" #n ", %" #n ", %16\n"
#define MUL(n) "v_mul_f32_e32 %" #n ", %" #n ", %16\n"
#define ALIGNBIT(n) "v_alignbit_b32 %" #n ", %" #n ", %16, 31\n"
#define LSHR(n) "v_lshrrev_b32_e32 %" #n ", 31, %" #n "\n"
#define ADDU(n) "v_add_u32_e32 %" #n ", %" #n ", %16\n"
#define BCNT(n) "v_bcnt_u32_b32 %" #n ", %" #n ", %16\n"
#define LSHL_OR(n) "v_lshl_or_b32 %" #n ", %" #n ", 1, %16\n"
#define AND_OR(n) "v_and_or_b32 %" #n ", %" #n ", %16, %17\n"
#define CVT_PKRTZ(n) "v_cvt_pkrtz_f16_f32 %" #n ", %" #n ", %16\n"
#define CNDMASK(n) "v_cndmask_b32_e32 %" #n ", %" #n ", %16, vcc\n"
#define MED3_I32(n) "v_med3_i32 %" #n ", %" #n ", %16, %17\n"
#define LSHL_ADD(n) "v_lshl_add_u32 %" #n ", %" #n ", 1, %16\n"

KERNEL(fma, FMA)
KERNEL(fma_abs, FMA_ABS)
KERNEL(fmac, FMAC)
KERNEL(med3_abs, MED3_ABS)
KERNEL(med3, MED3)
KERNEL(max_abs, MAX_ABS)
KERNEL(max_e32, MAX_E32)
KERNEL(max3_abs, MAX3_ABS)
KERNEL(sub, SUB)
KERNEL(sub_abs, SUB_ABS)
KERNEL(add, ADD)
KERNEL(mul, MUL)
KERNEL(alignbit, ALIGNBIT)
KERNEL(lshr, LSHR)
KERNEL(addu, ADDU)
KERNEL(bcnt, BCNT)
KERNEL(lshl_or, LSHL_OR)
KERNEL(and_or, AND_OR)
KERNEL(cvt_pkrtz, CVT_PKRTZ)
KERNEL(cndmask, CNDMASK)
KERNEL(med3_i32, MED3_I32)
KERNEL(lshl_add, LSHL_ADD)

typedef void (*kfn)(float*, int);
struct Entry { const char* name; kfn f; };

int main() {
    const Entry ks[] = {{"v_fma_f32", k_fma},           {"v_fma_f32 |b|", k_fma_abs},     {"v_fmac_f32_e32", k_fmac},
                        {"v_med3_f32 |a| |b|", k_med3_abs}, {"v_med3_f32", k_med3},        {"v_max_f32_e64 |a| |b|", k_max_abs},
                        {"v_max_f32_e32", k_max_e32},   {"v_max3_f32 |a| |b|", k_max3_abs}, {"v_sub_f32_e32", k_sub},
                        {"v_sub_f32_e64 |b|", k_sub_abs}, {"v_add_f32_e32", k_add},       {"v_mul_f32_e32", k_mul},
                        {"v_alignbit_b32", k_alignbit}, {"v_lshrrev_b32_e32", k_lshr},    {"v_add_u32_e32", k_addu},
                        {"v_bcnt_u32_b32", k_bcnt},     {"v_lshl_or_b32", k_lshl_or},     {"v_and_or_b32", k_and_or},
                        {"v_cvt_pkrtz_f16_f32", k_cvt_pkrtz}, {"v_cndmask_b32_e32", k_cndmask}, {"v_med3_i32", k_med3_i32},
                        {"v_lshl_add_u32", k_lshl_add}};
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int iters = 4096;
    float* out;
    hipMalloc(&out, (size_t)ncu * 8 * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    double ref[2] = {0, 0};
    printf("%d CUs, %d iterations x 16 instructions per wave\n", ncu, iters);
    printf("%-24s %14s %10s %14s %10s\n", "instruction", "8 waves/SIMD", "vs fma", "1 wave/SIMD", "vs fma");
    for (const Entry& k : ks) {
        double ns[2];
        for (int w = 0; w < 2; ++w) {
            const int blocks = ncu * (w == 0 ? 8 : 1);  // 256 threads = 1 wave per SIMD per block
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                hipEventRecord(e0);
                k.f<<<blocks, 256>>>(out, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep > 0 && ms < best) best = ms;
            }
            const double winst_per_simd = (double)(w == 0 ? 8 : 1) * iters * 16;
            ns[w] = best * 1e6 / winst_per_simd;
        }
        if (k.f == k_fma) { ref[0] = ns[0]; ref[1] = ns[1]; }
        printf("%-24s %11.3f ns %10.2f %11.3f ns %10.2f\n", k.name, ns[0], ns[0] / ref[0], ns[1], ns[1] / ref[1]);
    }
    hipFree(out);
    return 0;
}
