/*
 * valu_rate.cpp -- issue cost of the vector instructions k_dyn_row is made
 * of, at full occupancy (8 waves per SIMD, 8 independent chains per lane so
 * no instruction waits for the one before it): cycles per wave64
 * instruction per SIMD for each form.  The kernel is bound by its vector
 * instruction issue, so which forms cost more than
 * one slot decides where instructions are worth removing.
 *
 * Build: hipcc -x hip --offload-arch=gfx950 -O3 valu_rate.cpp -o valu_rate
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
constexpr int UNR = 16;        /* instructions per chain per trip (asm block of 8 chains x 2) */

#define OP8(op)                                                                                             \
    asm volatile(op " %0, %0, %8\n\t" op " %1, %1, %8\n\t" op " %2, %2, %8\n\t" op " %3, %3, %8\n\t"       \
                 op " %4, %4, %8\n\t" op " %5, %5, %8\n\t" op " %6, %6, %8\n\t" op " %7, %7, %8"           \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)        \
                 : "v"(k))
#define OP8_3(op)                                                                                           \
    asm volatile(op " %0, %0, %8, %0\n\t" op " %1, %1, %8, %1\n\t" op " %2, %2, %8, %2\n\t"                 \
                 op " %3, %3, %8, %3\n\t" op " %4, %4, %8, %4\n\t" op " %5, %5, %8, %5\n\t"                 \
                 op " %6, %6, %8, %6\n\t" op " %7, %7, %8, %7"                                              \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)        \
                 : "v"(k))

template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t *out, uint32_t seed)
{
    uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3u, a2 = a0 * 5u, a3 = a0 * 7u, a4 = a0 * 9u, a5 = a0 * 11u,
             a6 = a0 * 13u, a7 = a0 * 15u;
    const uint32_t k = seed | 1u;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int u = 0; u < UNR / 2; ++u) {
            if constexpr (K == 0) { OP8("v_add_u32"); OP8("v_add_u32"); }
            if constexpr (K == 1) { OP8("v_mul_lo_u32"); OP8("v_mul_lo_u32"); }
            if constexpr (K == 2) { OP8("v_mul_u32_u24"); OP8("v_mul_u32_u24"); }
            if constexpr (K == 3) { OP8("v_pk_add_u16"); OP8("v_pk_add_u16"); }
            if constexpr (K == 4) { OP8_3("v_alignbit_b32"); OP8_3("v_alignbit_b32"); }
            if constexpr (K == 5) { OP8_3("v_bfi_b32"); OP8_3("v_bfi_b32"); }
            if constexpr (K == 6) { OP8_3("v_mad_i32_i16"); OP8_3("v_mad_i32_i16"); }
            if constexpr (K == 7) { OP8_3("v_pk_mad_u16"); OP8_3("v_pk_mad_u16"); }
            if constexpr (K == 8) { OP8("v_lshlrev_b32"); OP8("v_lshlrev_b32"); }
            if constexpr (K == 9) { OP8("v_bcnt_u32_b32"); OP8("v_bcnt_u32_b32"); }
            if constexpr (K == 10) {
                asm volatile("v_sub_u16_sdwa %0, %0, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
                             "v_sub_u16_sdwa %1, %1, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
                             "v_sub_u16_sdwa %2, %2, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
                             "v_sub_u16_sdwa %3, %3, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
                             "v_sub_u16_sdwa %4, %4, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
                             "v_sub_u16_sdwa %5, %5, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
                             "v_sub_u16_sdwa %6, %6, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
                             "v_sub_u16_sdwa %7, %7, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(k));
                asm volatile("v_sub_u16_sdwa %0, %0, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                             "v_sub_u16_sdwa %1, %1, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                             "v_sub_u16_sdwa %2, %2, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                             "v_sub_u16_sdwa %3, %3, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                             "v_sub_u16_sdwa %4, %4, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                             "v_sub_u16_sdwa %5, %5, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                             "v_sub_u16_sdwa %6, %6, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
                             "v_sub_u16_sdwa %7, %7, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:BYTE_0"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(k));
            }
            if constexpr (K == 11) {
                asm volatile("v_ashrrev_i32_sdwa %0, %8, %0 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
                             "v_ashrrev_i32_sdwa %1, %8, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
                             "v_ashrrev_i32_sdwa %2, %8, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
                             "v_ashrrev_i32_sdwa %3, %8, %3 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
                             "v_ashrrev_i32_sdwa %4, %8, %4 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
                             "v_ashrrev_i32_sdwa %5, %8, %5 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
                             "v_ashrrev_i32_sdwa %6, %8, %6 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
                             "v_ashrrev_i32_sdwa %7, %8, %7 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(k));
                OP8("v_add_u32");
            }
            if constexpr (K == 12) { OP8_3("v_lshl_or_b32"); OP8_3("v_lshl_or_b32"); }
            if constexpr (K == 13) { OP8("v_xor_b32"); OP8("v_xor_b32"); }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int K>
float run(uint32_t *out, int grid)
{
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_rate<K>, dim3(grid), dim3(256), 0, 0, out, 7u);   /* warm */
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_rate<K>, dim3(grid), dim3(256), 0, 0, out, 7u + r);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 5;
}

int main()
{
    int dev = 0, ncu = 0, clk = 0;
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CHK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));   /* kHz */
    const int grid = ncu * 8;               /* 8 workgroups of 4 waves per CU: 8 waves per SIMD */
    uint32_t *out;
    CHK(hipMalloc(&out, (size_t)grid * 256 * 4));
    const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_u32_u24", "v_pk_add_u16", "v_alignbit_b32",
                           "v_bfi_b32", "v_mad_i32_i16", "v_pk_mad_u16", "v_lshlrev_b32", "v_bcnt_u32_b32",
                           "v_sub_u16_sdwa", "v_ashrrev_i32_sdwa+v_add (pairs)", "v_lshl_or_b32", "v_xor_b32"};
    float ms[14];
    ms[0] = run<0>(out, grid); ms[1] = run<1>(out, grid); ms[2] = run<2>(out, grid); ms[3] = run<3>(out, grid);
    ms[4] = run<4>(out, grid); ms[5] = run<5>(out, grid); ms[6] = run<6>(out, grid); ms[7] = run<7>(out, grid);
    ms[8] = run<8>(out, grid); ms[9] = run<9>(out, grid); ms[10] = run<10>(out, grid); ms[11] = run<11>(out, grid);
    ms[12] = run<12>(out, grid); ms[13] = run<13>(out, grid);
    /* instructions per SIMD: waves per SIMD (8) x trips x 16 per chain x 8 chains */
    const double per_simd = 8.0 * ITER * UNR * 8;
    printf("{\"cus\": %d, \"clock_khz\": %d, \"waves_per_simd\": 8, \"instr_per_simd\": %.0f, \"rates\": {", ncu, clk,
           per_simd);
    for (int i = 0; i < 14; ++i) {
        const double cyc = ms[i] * 1e-3 * clk * 1e3 / per_simd;
        printf("%s\"%s\": {\"ms\": %.4f, \"cycles_per_wave64_instr\": %.2f}", i ? ", " : "", names[i], ms[i], cyc);
    }
    printf("}}\n");
    CHK(hipFree(out));
    return 0;
}
