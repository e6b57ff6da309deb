// Issue-rate probe for gfx950 (replaces the two round-4 VALU probes).
//   A. single VALU instructions: ns per wave-instruction per SIMD at 8 waves per SIMD (16 independent
//      chains per lane), relative to v_fma_f32 -- the bound kernel's per-pair candidates;
//   B. MFMA + VALU co-execution on one SIMD: a loop of one v_mfma_f32_32x32x16_f16 (independent of
//      the VALU) plus N fast VALU per wave, at 1, 2 and 4 waves per SIMD, against MFMA alone and
//      VALU alone: do the VALU slots between MFMAs fill, and from which waves.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/issue_probe tools/issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define R16(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7) OP(8) OP(9) OP(10) OP(11) OP(12) OP(13) OP(14) OP(15)
#define OUTS                                                                                          \
    "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), \
        "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])

#define KERNEL(NAME, OP)                                                                       \
    __global__ __launch_bounds__(256) void k_##NAME(float* out, int iters) {                  \
        float r[16];                                                                           \
        for (int j = 0; j < 16; ++j) r[j] = 1.f + 1e-3f * (threadIdx.x + j);                   \
        float c = 1.0001f, d = 0.25f;                                                          \
        asm volatile("" : "+v"(c), "+v"(d));                                                   \
        for (int i = 0; i < iters; ++i) asm volatile(R16(OP) : OUTS : "v"(c), "v"(d) : "vcc", "s40", "s41"); \
        float s = 0.f;                                                                         \
        for (int j = 0; j < 16; ++j) s += r[j];                                                \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                               \
    }

#define FMA(n) "v_fma_f32 %" #n ", %16, |%" #n "|, %17\n"
#define SUB_ABS(n) "v_sub_f32_e64 %" #n ", %16, |%" #n "|\n"
#define SUB_ABS_CLAMP(n) "v_sub_f32_e64 %" #n ", %16, |%" #n "| clamp\n"
#define ADD(n) "v_add_f32_e32 %" #n ", %" #n ", %16\n"
#define ALIGNBIT(n) "v_alignbit_b32 %" #n ", %" #n ", %16, 31\n"
#define LSHR(n) "v_lshrrev_b32_e32 %" #n ", 31, %" #n "\n"
#define ASHR(n) "v_ashrrev_i32_e32 %" #n ", 31, %" #n "\n"
#define ADDU(n) "v_add_u32_e32 %" #n ", %" #n ", %16\n"
#define SUBU(n) "v_sub_u32_e32 %" #n ", %" #n ", %16\n"
#define ORB(n) "v_or_b32_e32 %" #n ", %" #n ", %16\n"
#define ANDB(n) "v_and_b32_e32 %" #n ", %" #n ", %16\n"
#define MINF(n) "v_min_f32_e32 %" #n ", %" #n ", %16\n"
#define CMP_E32(n) "v_cmp_lt_f32_e32 vcc, %" #n ", %16\n"
#define CMP_E64(n) "v_cmp_lt_f32_e64 s[40:41], %" #n ", |%16|\n"
#define ADDC(n) "v_addc_co_u32_e32 %" #n ", vcc, 0, %" #n ", vcc\n"
#define SUBREV_CO(n) "v_subrev_co_u32_e32 %" #n ", vcc, %16, %" #n "\n"
#define CVT_F32_U32(n) "v_cvt_f32_u32_e32 %" #n ", %" #n "\n"
#define PK_ADD(n) "v_pk_add_f32 %" #n ", %" #n ", %16\n"
#define MUL_LEGACY(n) "v_mul_legacy_f32 %" #n ", %" #n ", %16\n"
#define FMA_CLAMP(n) "v_fma_f32 %" #n ", %16, |%" #n "|, %17 clamp\n"
#define SUB_I32_E64(n) "v_sub_i32 %" #n ", %" #n ", %16\n"
#define BFE(n) "v_bfe_u32 %" #n ", %" #n ", 31, 1\n"
#define CND_E32(n) "v_cndmask_b32_e32 %" #n ", %" #n ", %16, vcc\n"
#define CND_E64(n) "v_cndmask_b32_e64 %" #n ", %" #n ", %16, s[40:41]\n"
#define MED3I(n) "v_med3_i32 %" #n ", %" #n ", %16, %17\n"
#define MINI(n) "v_min_i32_e32 %" #n ", %" #n ", %16\n"
#define MIN3I(n) "v_min3_i32 %" #n ", %" #n ", %16, %17\n"

KERNEL(fma, FMA)
KERNEL(sub_abs, SUB_ABS)
KERNEL(sub_abs_clamp, SUB_ABS_CLAMP)
KERNEL(add, ADD)
KERNEL(alignbit, ALIGNBIT)
KERNEL(lshr, LSHR)
KERNEL(ashr, ASHR)
KERNEL(addu, ADDU)
KERNEL(subu, SUBU)
KERNEL(orb, ORB)
KERNEL(andb, ANDB)
KERNEL(minf, MINF)
KERNEL(cmp_e32, CMP_E32)
KERNEL(cmp_e64, CMP_E64)
KERNEL(addc, ADDC)
KERNEL(subrev_co, SUBREV_CO)
KERNEL(cvt_f32_u32, CVT_F32_U32)
KERNEL(mul_legacy, MUL_LEGACY)
KERNEL(fma_clamp, FMA_CLAMP)
KERNEL(sub_i32, SUB_I32_E64)
KERNEL(bfe, BFE)
KERNEL(med3i, MED3I)
KERNEL(mini, MINI)
KERNEL(min3i, MIN3I)
// round 6: mixed-precision forms for the bound kernel's count (f32 test, f16 clamp result, f32 dot2 sum)
#define MIXLO(n) "v_fma_mixlo_f16 %" #n ", -|%" #n "|, %16, %17 op_sel_hi:[0,0,0] clamp\n"
#define MIXHI(n) "v_fma_mixhi_f16 %" #n ", -|%" #n "|, %16, %17 op_sel_hi:[0,0,0] clamp\n"
#define MIXF32(n) "v_fma_mix_f32 %" #n ", -|%" #n "|, %16, %17 op_sel_hi:[0,0,0]\n"
#define DOT2(n) "v_dot2_f32_f16 %" #n ", %16, %17, %" #n "\n"
#define DOT2C(n) "v_dot2c_f32_f16_e32 %" #n ", %16, %17\n"
#define PKADDH(n) "v_pk_add_f16 %" #n ", %" #n ", %16\n"
#define PKFMAH(n) "v_pk_fma_f16 %" #n ", %" #n ", %16, %17\n"
#define CVTPK(n) "v_cvt_pkrtz_f16_f32 %" #n ", %" #n ", %16\n"
#define ADDH(n) "v_add_f16_e32 %" #n ", %" #n ", %16\n"
#define SUBCL_FMA(n) "v_fma_f32 %" #n ", %16, |%" #n "|, -|%17|\n"
KERNEL(mixlo, MIXLO)
KERNEL(mixhi, MIXHI)
KERNEL(mixf32, MIXF32)
KERNEL(dot2, DOT2)
KERNEL(dot2c, DOT2C)
KERNEL(pkaddh, PKADDH)
KERNEL(pkfmah, PKFMAH)
KERNEL(cvtpk, CVTPK)
KERNEL(addh, ADDH)
KERNEL(fma_negabs, SUBCL_FMA)
// v_cndmask with the mask set once before the loop (VCC or an SGPR pair): does the form matter
#define KERNEL_CND(NAME, OP, SETUP)                                                            \
    __global__ __launch_bounds__(256) void k_##NAME(float* out, int iters) {                  \
        float r[16];                                                                           \
        for (int j = 0; j < 16; ++j) r[j] = 1.f + 1e-3f * (threadIdx.x + j);                   \
        float c = 1.0001f, d = 0.25f;                                                          \
        asm volatile("" : "+v"(c), "+v"(d));                                                   \
        asm volatile(SETUP ::: "vcc", "s40", "s41");                                           \
        for (int i = 0; i < iters; ++i) asm volatile(R16(OP) : OUTS : "v"(c), "v"(d) : "vcc", "s40", "s41"); \
        float s = 0.f;                                                                         \
        for (int j = 0; j < 16; ++j) s += r[j];                                                \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                               \
    }
KERNEL_CND(cnd_e32, CND_E32, "s_mov_b64 vcc, 0x5555\n")
// compare + select pairs as the compiler emits them: VOPC into VCC + v_cndmask_e32, or VOP3 compare into
// an SGPR pair (or VCC) + v_cndmask_e64 (reported per pair)
#define CS_E32(n) "v_cmp_gt_f32_e32 vcc, %" #n ", %16\nv_cndmask_b32_e32 %" #n ", %" #n ", %17, vcc\n"
#define CS_E64(n) "v_cmp_gt_f32_e64 s[40:41], %" #n ", %16\nv_cndmask_b32_e64 %" #n ", %" #n ", %17, s[40:41]\n"
#define CS_E64V(n) "v_cmp_gt_f32_e64 vcc, %" #n ", %16\nv_cndmask_b32_e64 %" #n ", %" #n ", %17, vcc\n"
KERNEL(cs_e32, CS_E32)
KERNEL(cs_e64, CS_E64)
KERNEL(cs_e64v, CS_E64V)
KERNEL_CND(cnd_e64, CND_E64, "s_mov_b64 s[40:41], 0x5555\n")


// packed f32: 8 independent 64-bit chains per lane (16 floats), one v_pk_* per pair
typedef float f2v __attribute__((ext_vector_type(2)));
#define PK8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)
#define PKADD(n) "v_pk_add_f32 %" #n ", %" #n ", %8\n"
#define PKFMA(n) "v_pk_fma_f32 %" #n ", %" #n ", %8, %9\n"
#define PKMUL(n) "v_pk_mul_f32 %" #n ", %" #n ", %8\n"
#define PKMOV(n) "v_pk_mov_b32 %" #n ", %8, %" #n " op_sel:[0,1]\n"
#define PKOUTS "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
#define PKKERNEL(NAME, OP)                                                                     \
    __global__ __launch_bounds__(256) void k_##NAME(float* out, int iters) {                  \
        f2v r[8];                                                                              \
        for (int j = 0; j < 8; ++j) r[j] = f2v{1.f + 1e-3f * (threadIdx.x + j), 2.f - j};      \
        f2v c = {1.0001f, 0.9999f}, d = {0.25f, 0.5f};                                         \
        asm volatile("" : "+v"(c), "+v"(d));                                                   \
        for (int i = 0; i < iters; ++i) asm volatile(PK8(OP) : PKOUTS : "v"(c), "v"(d));       \
        float s = 0.f;                                                                         \
        for (int j = 0; j < 8; ++j) s += r[j][0] + r[j][1];                                    \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                               \
    }
PKKERNEL(pk_add, PKADD)
PKKERNEL(pk_fma, PKFMA)
PKKERNEL(pk_mul, PKMUL)
PKKERNEL(pk_mov, PKMOV)

typedef void (*kfn)(float*, int);
struct Entry {
    const char* name;
    kfn f;
};

// ---- B: MFMA beside independent VALU -------------------------------------------------------------
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16acc __attribute__((ext_vector_type(16)));
#define F8(n) "v_fma_f32 %" #n ", %16, |%" #n "|, %17\n"
template <int NV, bool kMfma>
__global__ void k_coexec(float* out, int iters) {
    float r[16];
    for (int j = 0; j < 16; ++j) r[j] = 1.f + 1e-3f * (threadIdx.x + j);
    float c = 0.9999f, d = 0.25f;
    asm volatile("" : "+v"(c), "+v"(d));
    h8v a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)(0.01f * (threadIdx.x & 7) + j);
        b[j] = (_Float16)(0.02f * j);
    }
    f16acc acc0 = {}, acc1 = {};
    for (int i = 0; i < iters; ++i) {
        if (kMfma) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc0, 0, 0, 0);
        }
        if (NV >= 16) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
        if (NV >= 32) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
        if (kMfma) {
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc1, 0, 0, 0);
        }
        if (NV >= 8 && NV < 16) asm volatile(F8(0) F8(1) F8(2) F8(3) F8(4) F8(5) F8(6) F8(7) : OUTS : "v"(c), "v"(d));
        if (NV >= 48) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
        if (NV >= 64) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
    }
    float s = 0.f;
    for (int j = 0; j < 16; ++j) s += r[j] + acc0[j] + acc1[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


// ---- C: what an MFMA costs the VALU stream, by MFMA form, and with roles split over waves ------------
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef long i64x1;
// MODE 0: f16 32x32x16, srcC = 0 (results overwritten each time, like the bound kernel), VGPR dst
// MODE 1: f16 32x32x16 accumulating into AGPRs (asm, "a" constraint)
// MODE 2: i8 32x32x32 accumulating in VGPRs
// MODE 3: f16 16x16x32 accumulating in VGPRs (4 per iteration = the same pipe time)
template <int MODE, int NV>
__global__ void k_form(float* out, int iters) {
    float r[16];
    for (int j = 0; j < 16; ++j) r[j] = 1.f + 1e-3f * (threadIdx.x + j);
    float c = 0.9999f, d = 0.25f;
    asm volatile("" : "+v"(c), "+v"(d));
    h8v a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)(0.01f * (threadIdx.x & 7) + j);
        b[j] = (_Float16)(0.02f * j);
    }
    h8v b2 = b * (_Float16)0.5f;
    asm volatile("" : "+v"(b2));
    f16acc acc0 = {}, acc1 = {};
    typedef float f4acc __attribute__((ext_vector_type(4)));
    f4acc q0 = {}, q1 = {}, q2 = {}, q3 = {};
    i32x16 i0 = {}, i1 = {};
    const long ia = (long)threadIdx.x * 0x0102030405060708L, ib = 0x0101010101010101L;
    typedef int i4v __attribute__((ext_vector_type(4)));
    const i4v ia4 = {(int)ia, (int)(ia >> 32), (int)ia ^ 5, (int)ib};
    const i4v ib4 = {(int)ib, (int)ib, 3, 7};
    float sink = 0.f;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            const f16acc z = {};
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, z, 0, 0, 0);
            asm volatile("" : "+v"(acc0));
        } else if (MODE == 1) {
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc0) : "v"(a), "v"(b));
        } else if (MODE == 2) {
            i0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ia4, ib4, i0, 0, 0, 0);
        } else {
            q0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, q0, 0, 0, 0);
            q1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, q1, 0, 0, 0);
        }
        if (NV >= 16) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
        if (MODE == 0) {
            const f16acc z = {};
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b2, z, 0, 0, 0);
            asm volatile("" : "+v"(acc1));
            sink += acc0[3] + acc1[5];
        } else if (MODE == 1) {
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc1) : "v"(a), "v"(b));
        } else if (MODE == 2) {
            i1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ia4, ib4, i1, 0, 0, 0);
        } else {
            q2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, q2, 0, 0, 0);
            q3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, q3, 0, 0, 0);
        }
        if (NV >= 32) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
        if (NV >= 48) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
        if (NV >= 64) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
    }
    float s = sink;
    for (int j = 0; j < 16; ++j) s += r[j] + acc0[j] + acc1[j] + (float)i0[j] + (float)i1[j];
    for (int j = 0; j < 4; ++j) s += q0[j] + q1[j] + q2[j] + q3[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// roles split: in a 512-thread block (2 waves per SIMD) waves 0-3 run NM MFMAs per iteration only
// and waves 4-7 run NV fmas only (or the reverse placement), PRIO: s_setprio 1 for the VALU waves
template <int NM, int NV, int PRIO>
__global__ __launch_bounds__(512) void k_split(float* out, int iters) {
    float r[16];
    for (int j = 0; j < 16; ++j) r[j] = 1.f + 1e-3f * (threadIdx.x + j);
    float c = 0.9999f, d = 0.25f;
    asm volatile("" : "+v"(c), "+v"(d));
    h8v a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)(0.01f * (threadIdx.x & 7) + j);
        b[j] = (_Float16)(0.02f * j);
    }
    f16acc acc0 = {}, acc1 = {};
    const bool valu = threadIdx.x >= 256;
    if (valu) {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
        for (int i = 0; i < iters; ++i) {
            if (NV >= 16) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
            if (NV >= 32) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
            if (NV >= 48) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
            if (NV >= 64) asm volatile(R16(F8) : OUTS : "v"(c), "v"(d));
        }
    } else {
        for (int i = 0; i < iters; ++i) {
            if (NM >= 1) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc0, 0, 0, 0);
            if (NM >= 2) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc1, 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int j = 0; j < 16; ++j) s += r[j] + acc0[j] + acc1[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static hipEvent_t e0, e1;
static float time_ms(void (*f)(float*, int), int blocks, int threads, float* out, int iters) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(e0);
        f<<<blocks, threads>>>(out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
    }
    return best;
}

int main() {
    const Entry ks[] = {
        {"v_fma_f32 |b|", k_fma},          {"v_sub_f32_e64 |b|", k_sub_abs}, {"v_sub_f32 |b| clamp", k_sub_abs_clamp},
        {"v_add_f32_e32", k_add},          {"v_alignbit_b32", k_alignbit},   {"v_lshrrev_b32_e32", k_lshr},
        {"v_ashrrev_i32_e32", k_ashr},     {"v_add_u32_e32", k_addu},        {"v_sub_u32_e32", k_subu},
        {"v_or_b32_e32", k_orb},           {"v_and_b32_e32", k_andb},        {"v_min_f32_e32", k_minf},
        {"v_cmp_lt_f32_e32 vcc", k_cmp_e32}, {"v_cmp_lt_f32_e64 sgpr", k_cmp_e64}, {"v_addc_co_u32 vcc", k_addc},
        {"v_subrev_co_u32 vcc", k_subrev_co}, {"v_cvt_f32_u32", k_cvt_f32_u32}, {"v_mul_legacy_f32", k_mul_legacy},
        {"v_fma_f32 clamp", k_fma_clamp},  {"v_sub_i32 (vop3)", k_sub_i32},  {"v_bfe_u32", k_bfe},
        {"v_med3_i32", k_med3i},           {"v_min_i32_e32", k_mini},        {"v_min3_i32", k_min3i},
        {"v_cndmask_b32_e32 (vcc set)", k_cnd_e32}, {"v_cndmask_b32_e64 (sgpr)", k_cnd_e64},
        {"cmp_e32 vcc + cndmask_e32 (pair)", k_cs_e32}, {"cmp_e64 sgpr + cndmask_e64 (pair)", k_cs_e64},
        {"cmp_e64 vcc + cndmask_e64 (pair)", k_cs_e64v},
        {"v_fma_mixlo_f16 clamp", k_mixlo}, {"v_fma_mixhi_f16 clamp", k_mixhi}, {"v_fma_mix_f32", k_mixf32},
        {"v_dot2_f32_f16", k_dot2}, {"v_dot2c_f32_f16", k_dot2c}, {"v_pk_add_f16", k_pkaddh},
        {"v_pk_fma_f16", k_pkfmah}, {"v_cvt_pkrtz_f16_f32", k_cvtpk}, {"v_add_f16", k_addh},
        {"v_fma_f32 c,|a|,-|b|", k_fma_negabs}};
    // packed forms: 8 instructions per asm block, each doing 2 lanes' worth (reported per instruction)
    const Entry pk[] = {{"v_pk_add_f32", k_pk_add}, {"v_pk_fma_f32", k_pk_fma}, {"v_pk_mul_f32", k_pk_mul},
                        {"v_pk_mov_b32", k_pk_mov}};
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int iters = 4096;
    float* out;
    hipMalloc(&out, (size_t)ncu * 16 * 256 * sizeof(float));
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const bool only_a = getenv("PROBE_ONLY_A") != nullptr;
    printf("A. %d CUs, %d iterations x 16 instructions per wave, 8 waves per SIMD\n", ncu, iters);
    double ref = 0;
    for (const Entry& k : ks) {
        const float ms = time_ms(k.f, ncu * 8, 256, out, iters);
        const double ns = ms * 1e6 / ((double)8 * iters * 16);
        if (k.f == k_fma) ref = ns;
        printf("  %-26s %8.3f ns  %5.2f x fma\n", k.name, ns, ns / ref);
    }
    for (const Entry& k : pk) {
        const float ms = time_ms(k.f, ncu * 8, 256, out, iters);
        const double ns = ms * 1e6 / ((double)8 * iters * 8);
        printf("  %-26s %8.3f ns  %5.2f x fma (per instruction = 2 fp32 results)\n", k.name, ns, ns / ref);
    }
    if (only_a) return 0;
    printf("B. per loop iteration and SIMD: 2 v_mfma_f32_32x32x16_f16 (2 accumulators) + NV v_fma_f32 per wave\n");
    printf("  %-22s %10s %10s %10s\n", "variant", "1 w/SIMD", "2 w/SIMD", "4 w/SIMD");
    struct CE {
        const char* name;
        void (*f)(float*, int);
    } ce[] = {{"mfma only", k_coexec<0, true>},   {"valu 16 only", k_coexec<16, false>}, {"mfma + 8 valu", k_coexec<8, true>},
              {"mfma + 16 valu", k_coexec<16, true>}, {"valu 32 only", k_coexec<32, false>}, {"mfma + 32 valu", k_coexec<32, true>},
              {"valu 64 only", k_coexec<64, false>}, {"mfma + 64 valu", k_coexec<64, true>}};
    for (const CE& k : ce) {
        printf("  %-22s", k.name);
        for (int w : {1, 2, 4}) {
            const float ms = time_ms(k.f, ncu, 256 * w, out, 2048);
            // ns per loop iteration per SIMD: w waves per SIMD each run 2048 iterations
            printf(" %8.2f ns", ms * 1e6 / (2048.0 * w));
        }
        printf("\n");
    }

    printf("C. MFMA forms (2 32x32 MFMAs or 4 16x16 per iteration) + NV v_fma_f32, ns per wave-iteration per SIMD\n");
    printf("  %-34s %10s %10s %10s\n", "variant", "1 w/SIMD", "2 w/SIMD", "4 w/SIMD");
    struct CE2 {
        const char* name;
        void (*f)(float*, int);
    } cf[] = {{"f16 srcC=0 VGPR", k_form<0, 0>},       {"f16 srcC=0 VGPR + 32 valu", k_form<0, 32>},
              {"f16 srcC=0 VGPR + 64 valu", k_form<0, 64>}, {"f16 acc AGPR", k_form<1, 0>},
              {"f16 acc AGPR + 32 valu", k_form<1, 32>},   {"f16 acc AGPR + 64 valu", k_form<1, 64>},
              {"i8 32x32x32 VGPR", k_form<2, 0>},         {"i8 32x32x32 VGPR + 32 valu", k_form<2, 32>},
              {"i8 32x32x32 VGPR + 64 valu", k_form<2, 64>}, {"f16 16x16x32 x4", k_form<3, 0>},
              {"f16 16x16x32 x4 + 32 valu", k_form<3, 32>}, {"f16 16x16x32 x4 + 64 valu", k_form<3, 64>}};
    for (const CE2& k : cf) {
        printf("  %-34s", k.name);
        for (int w : {1, 2, 4}) {
            const float ms = time_ms(k.f, ncu, 256 * w, out, 2048);
            printf(" %8.2f ns", ms * 1e6 / (2048.0 * w));
        }
        printf("\n");
    }
    printf("D. roles split over the 2 waves of a SIMD (512-thread blocks): ns per iteration per SIMD\n");
    struct CE3 {
        const char* name;
        void (*f)(float*, int);
    } cs[] = {{"2 mfma | idle", k_split<2, 0, 0>},      {"idle | 64 valu", k_split<0, 64, 0>},
              {"2 mfma | 64 valu", k_split<2, 64, 0>},  {"2 mfma | 64 valu, valu prio 1", k_split<2, 64, 1>},
              {"2 mfma | 32 valu", k_split<2, 32, 0>},  {"2 mfma | 32 valu, valu prio 1", k_split<2, 32, 1>},
              {"1 mfma | 32 valu", k_split<1, 32, 0>}};
    for (const CE3& k : cs) {
        for (int bpc : {1, 2}) {
            const float ms = time_ms(k.f, ncu * bpc, 512, out, 2048);
            printf("  %-34s %d block/CU %8.2f ns\n", k.name, bpc, ms * 1e6 / (2048.0 * bpc));
        }
    }
    hipFree(out);
    return 0;
}
