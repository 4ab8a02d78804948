/*
 * valu_rate2.cpp -- the issue cost of a wider set of vector instruction forms
 * than valu_rate.cpp, same method (8 waves per SIMD, 8 independent chains per
 * lane): which forms issue at the full rate (about 2 cycles per wave64
 * instruction: v_add_u32, v_xor_b32 in valu_rate) and which at half (about 4).
 * k_dyn_row is bound by its vector instruction issue, so a half-rate form
 * that has a full-rate equivalent is worth replacing.
 *
 * Build: hipcc -x hip --offload-arch=gfx950 -O3 valu_rate2.cpp -o valu_rate2
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int ITER = 256;      /* loop trips */
constexpr int UNR = 16;        /* instructions per chain per trip */

#define OUTS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
/* f: the form with %0..%7 the chain registers (operand A), %8 the vector
 * constant, %9 the scalar constant */
#define FORM8(f0, f1, f2, f3, f4, f5, f6, f7)                                                          \
    asm volatile(f0 "\n\t" f1 "\n\t" f2 "\n\t" f3 "\n\t" f4 "\n\t" f5 "\n\t" f6 "\n\t" f7 : OUTS        \
                 : "v"(k), "s"(ks)                                                                    \
                 : "vcc")
#define V2(op) FORM8(op " %0, %0, %8", op " %1, %1, %8", op " %2, %2, %8", op " %3, %3, %8", op " %4, %4, %8", \
                     op " %5, %5, %8", op " %6, %6, %8", op " %7, %7, %8")
#define S2(op) FORM8(op " %0, %9, %0", op " %1, %9, %1", op " %2, %9, %2", op " %3, %9, %3", op " %4, %9, %4", \
                     op " %5, %9, %5", op " %6, %9, %6", op " %7, %9, %7")
#define V3(op) FORM8(op " %0, %0, %8, %0", op " %1, %1, %8, %1", op " %2, %2, %8, %2", op " %3, %3, %8, %3", \
                     op " %4, %4, %8, %4", op " %5, %5, %8, %5", op " %6, %6, %8, %6", op " %7, %7, %8, %7")
#define V3S(op) FORM8(op " %0, %0, %9, %0", op " %1, %1, %9, %1", op " %2, %2, %9, %2", op " %3, %3, %9, %3", \
                      op " %4, %4, %9, %4", op " %5, %5, %9, %5", op " %6, %6, %9, %6", op " %7, %7, %9, %7")
#define V1(op) FORM8(op " %0, %0", op " %1, %1", op " %2, %2", op " %3, %3", op " %4, %4", op " %5, %5", \
                     op " %6, %6", op " %7, %7")
#define V2X(op, sfx) FORM8(op " %0, %0, %8 " sfx, op " %1, %1, %8 " sfx, op " %2, %2, %8 " sfx, op " %3, %3, %8 " sfx, \
                           op " %4, %4, %8 " sfx, op " %5, %5, %8 " sfx, op " %6, %6, %8 " sfx, op " %7, %7, %8 " sfx)
#define V3X(op, sfx) FORM8(op " %0, %0, %8, %0 " sfx, op " %1, %1, %8, %1 " sfx, op " %2, %2, %8, %2 " sfx, \
                           op " %3, %3, %8, %3 " sfx, op " %4, %4, %8, %4 " sfx, op " %5, %5, %8, %5 " sfx, \
                           op " %6, %6, %8, %6 " sfx, op " %7, %7, %8, %7 " sfx)
#define CO(op) FORM8(op " %0, vcc, %0, %8", op " %1, vcc, %1, %8", op " %2, vcc, %2, %8", op " %3, vcc, %3, %8", \
                     op " %4, vcc, %4, %8", op " %5, vcc, %5, %8", op " %6, vcc, %6, %8", op " %7, vcc, %7, %8")
#define CND FORM8("v_cndmask_b32 %0, %0, %8, vcc", "v_cndmask_b32 %1, %1, %8, vcc", "v_cndmask_b32 %2, %2, %8, vcc", \
                  "v_cndmask_b32 %3, %3, %8, vcc", "v_cndmask_b32 %4, %4, %8, vcc", "v_cndmask_b32 %5, %5, %8, vcc", \
                  "v_cndmask_b32 %6, %6, %8, vcc", "v_cndmask_b32 %7, %7, %8, vcc")
#define LIT(op) FORM8(op " %0, 0x12345, %0", op " %1, 0x12345, %1", op " %2, 0x12345, %2", op " %3, 0x12345, %3", \
                      op " %4, 0x12345, %4", op " %5, 0x12345, %5", op " %6, 0x12345, %6", op " %7, 0x12345, %7")
#define DPP(op, ctl) FORM8(op " %0, %0, %8 " ctl, op " %1, %1, %8 " ctl, op " %2, %2, %8 " ctl, op " %3, %3, %8 " ctl, \
                           op " %4, %4, %8 " ctl, op " %5, %5, %8 " ctl, op " %6, %6, %8 " ctl, op " %7, %7, %8 " ctl)

#define FORMS(X)                                                                     \
    X(0, "v_add_u32", V2("v_add_u32"))                                               \
    X(1, "v_xor_b32", V2("v_xor_b32"))                                               \
    X(2, "v_and_b32", V2("v_and_b32"))                                               \
    X(3, "v_or_b32", V2("v_or_b32"))                                                 \
    X(4, "v_sub_u32", V2("v_sub_u32"))                                               \
    X(5, "v_subrev_u32", V2("v_subrev_u32"))                                         \
    X(6, "v_lshlrev_b32", V2("v_lshlrev_b32"))                                       \
    X(7, "v_lshrrev_b32", V2("v_lshrrev_b32"))                                       \
    X(8, "v_ashrrev_i32", V2("v_ashrrev_i32"))                                       \
    X(9, "v_max_u32", V2("v_max_u32"))                                               \
    X(10, "v_min_i32", V2("v_min_i32"))                                              \
    X(11, "v_mul_u32_u24", V2("v_mul_u32_u24"))                                      \
    X(12, "v_mul_hi_u32", V2("v_mul_hi_u32"))                                        \
    X(13, "v_add_f32", V2("v_add_f32"))                                              \
    X(14, "v_mul_f32", V2("v_mul_f32"))                                              \
    X(15, "v_fma_f32", V3("v_fma_f32"))                                              \
    X(16, "v_add_u16", V2("v_add_u16"))                                              \
    X(17, "v_pk_add_u16", V2("v_pk_add_u16"))                                        \
    X(18, "v_pk_sub_i16", V2("v_pk_sub_i16"))                                        \
    X(19, "v_pk_max_i16", V2("v_pk_max_i16"))                                        \
    X(20, "v_pk_lshlrev_b16", V2("v_pk_lshlrev_b16"))                                \
    X(21, "v_pk_mul_lo_u16", V2("v_pk_mul_lo_u16"))                                  \
    X(22, "v_pk_mad_i16", V3("v_pk_mad_i16"))                                        \
    X(23, "v_add3_u32", V3("v_add3_u32"))                                            \
    X(24, "v_or3_b32", V3("v_or3_b32"))                                              \
    X(25, "v_and_or_b32", V3("v_and_or_b32"))                                        \
    X(26, "v_lshl_add_u32", V3("v_lshl_add_u32"))                                    \
    X(27, "v_add_lshl_u32", V3("v_add_lshl_u32"))                                    \
    X(28, "v_lshl_or_b32", V3("v_lshl_or_b32"))                                      \
    X(29, "v_xad_u32", V3("v_xad_u32"))                                              \
    X(30, "v_bfe_u32", V3("v_bfe_u32"))                                              \
    X(31, "v_bfi_b32", V3("v_bfi_b32"))                                              \
    X(32, "v_perm_b32", V3("v_perm_b32"))                                            \
    X(33, "v_alignbit_b32", V3("v_alignbit_b32"))                                    \
    X(34, "v_alignbyte_b32", V3("v_alignbyte_b32"))                                  \
    X(35, "v_bitop3_b32", V3X("v_bitop3_b32", "bitop3:0xc8"))                        \
    X(36, "v_mad_u32_u24", V3("v_mad_u32_u24"))                                      \
    X(37, "v_mad_u32_u16", V3("v_mad_u32_u16"))                                      \
    X(38, "v_mad_i32_i16", V3("v_mad_i32_i16"))                                      \
    X(39, "v_max3_u32", V3("v_max3_u32"))                                            \
    X(40, "v_med3_i32", V3("v_med3_i32"))                                            \
    X(41, "v_sad_u8", V3("v_sad_u8"))                                                \
    X(42, "v_lerp_u8", V3("v_lerp_u8"))                                              \
    X(43, "v_dot2_i32_i16", V3("v_dot2_i32_i16"))                                    \
    X(44, "v_dot4_i32_i8", V3("v_dot4_i32_i8"))                                      \
    X(45, "v_bcnt_u32_b32", V2("v_bcnt_u32_b32"))                                    \
    X(46, "v_mov_b32", V1("v_mov_b32"))                                              \
    X(47, "v_not_b32", V1("v_not_b32"))                                              \
    X(48, "v_ffbh_u32", V1("v_ffbh_u32"))                                            \
    X(49, "v_bfrev_b32", V1("v_bfrev_b32"))                                          \
    X(50, "v_cvt_f32_u32", V1("v_cvt_f32_u32"))                                      \
    X(51, "v_cvt_u32_f32", V1("v_cvt_u32_f32"))                                      \
    X(52, "v_cndmask_b32", CND)                                                      \
    X(53, "v_add_co_u32", CO("v_add_co_u32"))                                        \
    X(54, "v_add_u32_e64", V2("v_add_u32_e64"))                                      \
    X(55, "v_xor_b32_e64", V2("v_xor_b32_e64"))                                      \
    X(56, "v_and_b32_e64", V2("v_and_b32_e64"))                                      \
    X(57, "v_add_u32 (sgpr)", S2("v_add_u32"))                                       \
    X(58, "v_and_b32 (sgpr)", S2("v_and_b32"))                                       \
    X(59, "v_add_u32 (literal)", LIT("v_add_u32"))                                   \
    X(60, "v_and_b32 (literal)", LIT("v_and_b32"))                                   \
    X(61, "v_add_u32_dpp row_shr:1", DPP("v_add_u32_dpp", "row_shr:1 row_mask:0xf bank_mask:0xf")) \
    X(62, "v_and_b32_sdwa", V2X("v_and_b32_sdwa", "dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")) \
    X(63, "v_add_u32_sdwa", V2X("v_add_u32_sdwa", "dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD")) \
    X(64, "v_bfi_b32 (sgpr)", V3S("v_bfi_b32"))                                      \
    X(65, "v_mad_u32_u24 (sgpr)", V3S("v_mad_u32_u24"))                              \
    X(66, "v_lshlrev_b32_e64", V2("v_lshlrev_b32_e64"))                              \
    X(67, "v_sub_u32_e64", V2("v_sub_u32_e64"))                                      \
    X(68, "v_or_b32_e64", V2("v_or_b32_e64"))                                        \
    X(69, "v_min_u32", V2("v_min_u32"))                                              \
    X(70, "v_cvt_f32_i32", V1("v_cvt_f32_i32"))                                      \
    X(71, "v_pk_add_i16", V2("v_pk_add_i16"))                                        \
    X(72, "v_sub_u16", V2("v_sub_u16"))                                              \
    X(73, "v_lshlrev_b16", V2("v_lshlrev_b16"))

#define NFORMS 74

template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t *out, uint32_t seed)
{
    uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 9u, a5 = a0 * 11u,
             a6 = a0 * 13u, a7 = a0 * 15u;
    const uint32_t k = seed | 1u, ks = __builtin_amdgcn_readfirstlane(seed * 3u);
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
#define CASE(n, name, body) \
    if constexpr (K == n) { body; }
            FORMS(CASE)
#undef CASE
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*KFn)(uint32_t *, uint32_t);

static float run(KFn fn, uint32_t *out, int grid)
{
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, out, 7u);   /* warm */
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, out, 7u + r);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    return ms / 5;
}

template <int... I>
struct Table {
    static constexpr KFn fns[] = {k_rate<I>...};
};
template <int... I>
constexpr Table<I...> make_table(std::integer_sequence<int, I...>)
{
    return {};
}

int main()
{
    int dev = 0, ncu = 0, clk = 0;
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CHK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));   /* kHz */
    const int grid = ncu * 8;               /* 8 workgroups of 4 waves per CU: 8 waves per SIMD */
    uint32_t *out;
    CHK(hipMalloc(&out, (size_t)grid * 256 * 4));
    using T = decltype(make_table(std::make_integer_sequence<int, NFORMS>{}));
    const char *names[NFORMS];
#define NAME(n, name, body) names[n] = name;
    FORMS(NAME)
#undef NAME
    /* the reference form first and last: a drift in the clock shows */
    const float ref0 = run(T::fns[0], out, grid);
    const double per_simd = 8.0 * ITER * UNR * 8;   /* waves per SIMD x trips x per chain x chains */
    printf("{\"cus\": %d, \"clock_khz\": %d, \"waves_per_simd\": 8, \"instr_per_simd\": %.0f, \"rates\": {", ncu, clk,
           per_simd);
    for (int i = 0; i < NFORMS; ++i) {
        const float ms = run(T::fns[i], out, grid);
        const double cyc = ms * 1e-3 * clk * 1e3 / per_simd;
        printf("%s\"%s\": {\"ms\": %.4f, \"cycles_per_wave64_instr\": %.2f, \"vs_v_add_u32\": %.2f}", i ? ", " : "",
               names[i], ms, cyc, ms / ref0);
    }
    const float ref1 = run(T::fns[0], out, grid);
    printf("}, \"v_add_u32_first_ms\": %.4f, \"v_add_u32_last_ms\": %.4f}\n", ref0, ref1);
    CHK(hipFree(out));
    return 0;
}
