/*
 * row_mfma.h -- k_dyn_row's levels on the matrix cores (round 6): an
 * opt-in build (-DSCROLL_ROW_MFMA) kept as a measured experiment; the
 * product path is the vector form (levels_pk), as the north star
 * prescribes no MFMA for this integer path (DESIGN.md §5 round 6 has the
 * numbers: 2.5 % on k_dyn_row).
 *
 * The residual transform of a 4x4 block is linear in its pixels: with X the
 * source rows and P the prediction rows, W = C (X - P) C^T, i.e. one 16 x 32
 * integer matrix times the block's 32 pixel bytes (16 source, 16 prediction).
 * Its entries are products of the core transform's {1, 2, -1, -2}: int8.  The
 * pixel bytes become int8 by subtracting 128 (xor 0x80); the 128s cancel
 * between X and P.  So one v_mfma_i32_16x16x32_i8 computes the 16
 * coefficients of 16 blocks exactly (int32 accumulators), where the vector
 * form took 56 half-rate instructions per block (16 byte-residual
 * subtractions, 40 packed butterflies: profiles/r06_valu_rate*.json has the
 * issue costs) -- k_dyn_row is bound by its vector instruction issue.
 *
 * Operand maps (16x16x32 i8, lane l, g = l >> 4, n = l & 15):
 *   B: lane (g, n) holds B[k = 8 g + e][block n], e = 0..7: the source row g
 *      of block n (bytes e = 0..3) and its prediction row g (e = 4..7);
 *   A: lane (g, n) holds A[coefficient n][k = 8 g + e] (g_kmat);
 *   D: lane (g, n) holds coefficients 4 g .. 4 g + 3 of block n.
 * The coefficient rows are in scan order (luma: scan m; chroma AC: scan
 * m + 1, row 15 the DC coefficient), so the quant writes lane (g, n)'s 4
 * levels straight into word g of the block's packed levels (levels_pk's
 * layout); a 4 x 4 transpose over (lane group, tile) with two
 * v_permlane32_swap and two v_permlane16_swap then gives each lane the four
 * words of one block.
 *
 * A wave's pass covers 64 blocks as 4 tiles: lane (g, n) loads 16 bytes of
 * one source row and 16 of the prediction row (tile j = the j-th 4-pixel
 * column of the 16: luma block x, chroma MB parity and block x), so a pass is
 * two 16-byte loads per lane (three for chroma: the lower bilinear row).
 *
 * Bit-exact to levels_pk (tools/mfma_levels_check.hip compares them on the
 * GPU over every QP; the k_dyn_row parity tests cover the rest).
 */
#ifndef SCROLL_ROW_MFMA_H
#define SCROLL_ROW_MFMA_H

#include "dyn_device.h"

namespace scroll {
namespace dyn {

typedef int mfma_v4i __attribute__((ext_vector_type(4)));

/* A[m][k]: coefficient row m (luma: scan m; chroma: scan m + 1, row 15 DC),
 * k = 8 g + e: source (e < 4) or prediction (e >= 4, negated) pixel (row g,
 * column e & 3) */
constexpr int kmat_elem(bool luma, int m, int k)
{
    constexpr int C[4][4] = {{1, 1, 1, 1}, {2, 1, -1, -2}, {1, -1, -1, 1}, {1, -2, 2, -1}};
    const int sc = luma ? m : (m < 15 ? m + 1 : 0);
    const int pos = ZZ[sc], u = pos >> 2, v = pos & 3;
    const int y = k >> 3, e = k & 7, x = e & 3;
    return (e < 4 ? 1 : -1) * C[u][y] * C[v][x];
}
struct KMat {
    uint64_t a[2][64];        /* [luma, chroma][lane]: the lane's 8 A bytes */
};
constexpr KMat make_kmat()
{
    KMat K{};
    for (int c = 0; c < 2; ++c)
        for (int l = 0; l < 64; ++l) {
            uint64_t v = 0;
            for (int e = 0; e < 8; ++e)
                v |= (uint64_t)(uint8_t)(int8_t)kmat_elem(c == 0, l & 15, 8 * (l >> 4) + e) << (8 * e);
            K.a[c][l] = v;
        }
    return K;
}

/* MF class (0: row and column even, 1: both odd, 2: else) of each
 * coefficient row, 2 bits per row: luma rows = scan 0..15; chroma rows = scan
 * 1..15 and the DC coefficient (3: mf 0).  From ZZ by tools/ (python: the
 * class of ZZ[s]); mquant_class_check below restates them */
constexpr uint32_t MQ_CLS_LUMA = 0x691aa128u, MQ_CLS_CHROMA = 0xda46a84au;
constexpr int mf_class_of_scan(int s)
{
    const int p = ZZ[s], r = p >> 2, c = p & 3;
    return ((r | c) & 1) == 0 ? 0 : (((r & c) & 1) ? 1 : 2);
}
constexpr bool mquant_class_check()
{
    for (int m = 0; m < 16; ++m) {
        if ((int)((MQ_CLS_LUMA >> (2 * m)) & 3u) != mf_class_of_scan(m)) return false;
        if ((int)((MQ_CLS_CHROMA >> (2 * m)) & 3u) != (m < 15 ? mf_class_of_scan(m + 1) : 3)) return false;
    }
    return true;
}
static_assert(mquant_class_check(), "the MF class codes follow ZZ");

/* The quant constants of lane group g: mf of its 4 coefficient rows packed
 * two per word (v_mad_i32_i16 reads a half by op_sel), the bias pair and the
 * shift.  Chroma's row 15 (the DC coefficient) gets mf 0: its level byte is 0
 * (both biases are below 2^qbits) */
struct MQuant {
    uint32_t m01, m23, k1, k0, sh;
};
__device__ __host__ inline MQuant mquant_of(int g, bool luma, const QParams &q)
{
    const uint32_t codes = (luma ? MQ_CLS_LUMA : MQ_CLS_CHROMA) >> (8 * g);
    /* mf by class (3: 0) as four 16-bit fields: one shift per row, no selects */
    const uint64_t lut = (uint64_t)(uint32_t)q.mf0 | (uint64_t)(uint32_t)q.mf1 << 16 | (uint64_t)(uint32_t)q.mf2 << 32;
    uint32_t mf[4];
    for (int i = 0; i < 4; ++i) mf[i] = (uint32_t)(lut >> (16u * ((codes >> (2 * i)) & 3u))) & 0xffffu;
    MQuant Q{mf[0] | mf[1] << 16, mf[2] | mf[3] << 16, (uint32_t)((1 << q.qbits) - 1 - q.qf), (uint32_t)q.qf,
             (uint32_t)q.qbits};
#ifdef __HIP_DEVICE_COMPILE__
    /* the bias pair in VGPRs: v_bitop3 reading an SGPR issues at half rate
     * (profiles/r06_valu_rate2.json) */
    asm("" : "+v"(Q.k1), "+v"(Q.k0));
#endif
    return Q;
}

/* two tiles' coefficients -> 4 int8 levels each in a word (byte i = row
 * 4 g + i): the bias by the sign (v_bitop3 select: full rate with the
 * constants in VGPRs), one v_mad_i32_i16 on the coefficient's low half
 * (|W| <= 9180; the odd rows' mf is the high half of its word, read as src0
 * with op_sel), the arithmetic shift into its byte (SDWA).
 *   - The first reads of the MFMA results are compiler-visible (the sign
 *     shifts): the hazard recognizer pads the MFMA -> VALU read there, which
 *     it does not do for an asm block's operands (read too early, they held
 *     stale values).
 *   - The two words' byte writes alternate: an SDWA byte write straight
 *     after one to the same register (UNUSED_PRESERVE reading it) measured
 *     wrong bytes on gfx950. */
__device__ inline void mquant2(const mfma_v4i &d, const mfma_v4i &e, const MQuant &Q, uint32_t &qd, uint32_t &qe)
{
    uint32_t s0 = __builtin_amdgcn_bitop3_b32((uint32_t)(d[0] >> 31), Q.k1, Q.k0, 0xca);
    uint32_t s1 = __builtin_amdgcn_bitop3_b32((uint32_t)(d[1] >> 31), Q.k1, Q.k0, 0xca);
    uint32_t s2 = __builtin_amdgcn_bitop3_b32((uint32_t)(d[2] >> 31), Q.k1, Q.k0, 0xca);
    uint32_t s3 = __builtin_amdgcn_bitop3_b32((uint32_t)(d[3] >> 31), Q.k1, Q.k0, 0xca);
    uint32_t t0 = __builtin_amdgcn_bitop3_b32((uint32_t)(e[0] >> 31), Q.k1, Q.k0, 0xca);
    uint32_t t1 = __builtin_amdgcn_bitop3_b32((uint32_t)(e[1] >> 31), Q.k1, Q.k0, 0xca);
    uint32_t t2 = __builtin_amdgcn_bitop3_b32((uint32_t)(e[2] >> 31), Q.k1, Q.k0, 0xca);
    uint32_t t3 = __builtin_amdgcn_bitop3_b32((uint32_t)(e[3] >> 31), Q.k1, Q.k0, 0xca);
    asm("v_mad_i32_i16 %[s0], %[d0], %[m01], %[s0]\n\t"
        "v_mad_i32_i16 %[s1], %[m01], %[d1], %[s1] op_sel:[1,0,0,0]\n\t"
        "v_mad_i32_i16 %[s2], %[d2], %[m23], %[s2]\n\t"
        "v_mad_i32_i16 %[s3], %[m23], %[d3], %[s3] op_sel:[1,0,0,0]\n\t"
        "v_mad_i32_i16 %[t0], %[e0], %[m01], %[t0]\n\t"
        "v_mad_i32_i16 %[t1], %[m01], %[e1], %[t1] op_sel:[1,0,0,0]\n\t"
        "v_mad_i32_i16 %[t2], %[e2], %[m23], %[t2]\n\t"
        "v_mad_i32_i16 %[t3], %[m23], %[e3], %[t3] op_sel:[1,0,0,0]\n\t"
        "v_ashrrev_i32_sdwa %[qd], %[sh], %[s0] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_ashrrev_i32_sdwa %[qe], %[sh], %[t0] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_ashrrev_i32_sdwa %[qd], %[sh], %[s1] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_ashrrev_i32_sdwa %[qe], %[sh], %[t1] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_ashrrev_i32_sdwa %[qd], %[sh], %[s2] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_ashrrev_i32_sdwa %[qe], %[sh], %[t2] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_ashrrev_i32_sdwa %[qd], %[sh], %[s3] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
        "v_ashrrev_i32_sdwa %[qe], %[sh], %[t3] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
        : [qd] "=&v"(qd), [qe] "=&v"(qe), [s0] "+v"(s0), [s1] "+v"(s1), [s2] "+v"(s2), [s3] "+v"(s3),
          [t0] "+v"(t0), [t1] "+v"(t1), [t2] "+v"(t2), [t3] "+v"(t3)
        : [d0] "v"(d[0]), [d1] "v"(d[1]), [d2] "v"(d[2]), [d3] "v"(d[3]), [e0] "v"(e[0]), [e1] "v"(e[1]),
          [e2] "v"(e[2]), [e3] "v"(e[3]), [m01] "v"(Q.m01), [m23] "v"(Q.m23), [sh] "s"(Q.sh));
}

/* the tile's coefficients: A (the lane's kmat bytes) times the block pixels
 * (x: source row word, p: prediction row word, both as bytes) */
__device__ inline mfma_v4i mtile(uint64_t a, uint32_t x, uint32_t p)
{
    const uint64_t b = (uint64_t)(x ^ 0x80808080u) | (uint64_t)(p ^ 0x80808080u) << 32;
    const mfma_v4i z = {0, 0, 0, 0};
    return __builtin_amdgcn_mfma_i32_16x16x32_i8((long)a, (long)b, z, 0, 0, 0);
}

/* w[j] in lane group g (word g of tile j's block) -> lane group g holds the
 * four words of tile g's block: X[g][j] -> X[j][g] */
__device__ inline void mtranspose(uint32_t w[4])
{
    const auto a = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
    const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
    const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
    w[0] = c[0];
    w[1] = c[1];
    w[2] = d[0];
    w[3] = d[1];
}

}  // namespace dyn
}  // namespace scroll

#endif
