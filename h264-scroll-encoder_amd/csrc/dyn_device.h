/*
 * dyn_device.h -- device functions of the dynamic-rect residual coder
 * (BASELINE configs 3-5, SURVEY §8a "dynamic-MB splice"; no reference
 * implementation exists, the bits are defined by oracle/dyn_oracle.h).
 *
 * Pure integer functions, no LDS / wave intrinsics: the kernels in
 * dyn_kernels.hip use them per lane, and tests/hostsim compiles this header
 * for the CPU to check each function against the oracle.
 *
 *  - prediction: full-pel luma, 1/8-pel bilinear chroma from the reference
 *    pictures A / B, a waypoint (long-term ref 2+k) resolved through its own
 *    row-uniform (ref, mv) (src/h264_writer.c:689-729), coordinates clamped;
 *  - 4x4 forward core transform, flat quantiser at the rect's QP (26 by
 *    default; chroma at QPc), chroma DC 2x2
 *    Hadamard (dyn_oracle.c or_fwd4x4 / or_quant);
 *  - CAVLC residual blocks (H.264 9.2) into any bit sink;
 *  - the emulation-prevention rule in closed form (nal.c:33-38).
 */
#ifndef SCROLL_DYN_DEVICE_H
#define SCROLL_DYN_DEVICE_H

#include "qparams.h"
#include "scroll_device.h"

namespace scroll {
namespace dyn {

/* the rect's QP: 26 by default (pic_init_qp 26, slice_qp_delta 0,
 * h264_writer.c:118-120); scroll_batch_set_dyn_qp[_stream / _at] picks
 * another, 0..51, written as the dynamic NAL's slice_qp_delta (under hints:
 * the rect MBs' mb_qp_delta chain).  QP_MIN: the lowest whose levels fit the
 * packed int8 form of k_dyn_row (|W| <= 9180: max level 127 at QP 22, 145 at
 * 21); below it a NAL takes the general path with 16-bit levels.
 * LEVEL_MAX: levels are clamped to the largest |level| every CAVLC context
 * codes with level_prefix <= 15 (only chroma DC below QPc 6 reaches it) */
constexpr int QP_DEFAULT = 26, QP_MIN = 22, QP_MAX = 51, LEVEL_MAX = 2063;
/* MF by QP % 6 and position class (Table 8-x inverse, the forward scale) */
__host__ __device__ constexpr int mf_of(int r, int cls)
{
    constexpr int T[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                             {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};
    return T[r][cls];
}
__host__ __device__ constexpr QParams qparams(int qp)
{
    return QParams{mf_of(qp % 6, 0), mf_of(qp % 6, 1), mf_of(qp % 6, 2), 15 + qp / 6, (1 << (15 + qp / 6)) / 6};
}
/* qparams for a QP known only at run time (wave-uniform: the selects stay
 * scalar; no table in private memory) */
__device__ __host__ inline QParams qparams_rt(int qp)
{
    const int r = qp % 6, b = 15 + qp / 6;
    const int m0 = r == 0 ? 13107 : r == 1 ? 11916 : r == 2 ? 10082 : r == 3 ? 9362 : r == 4 ? 8192 : 7282;
    const int m1 = r == 0 ? 5243 : r == 1 ? 4660 : r == 2 ? 4194 : r == 3 ? 3647 : r == 4 ? 3355 : 2893;
    const int m2 = r == 0 ? 8066 : r == 1 ? 7490 : r == 2 ? 6554 : r == 3 ? 5825 : r == 4 ? 5243 : 4559;
    return QParams{m0, m1, m2, b, (1 << b) / 6};
}
/* QPc of QP (Table 8-15, chroma_qp_index_offset 0 as the composer's PPS) */
__host__ __device__ constexpr int qp_chroma(int qp)
{
    constexpr int T[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
    return qp < 30 ? qp : T[qp - 30];
}
/* provable bound on the bits of one dynamic MB (codeword + residual):
 * 16 x 640 luma + 8 x 602 chroma AC + 2 x 130 chroma DC + cbp/qp + 64 < 16384 */
constexpr int MB_BITS_MAX = 16384;

/* coded_block_pattern -> codeNum, inter column of Table 9-4 */
struct Tabs {
    uint8_t ct_len[3][68], ct_bits[3][68];
    uint8_t ctdc_len[20], ctdc_bits[20];
    uint8_t tz_len[15][16], tz_bits[15][16];
    uint8_t tzdc_len[3][4], tzdc_bits[3][4];
    uint8_t rb_len[7][15], rb_bits[7][15];
    uint8_t cbp_code[48];
    uint8_t zz[16];
};

/* Tables 9-5 (coeff_token, 0 <= nC < 8 in three columns), 9-5 nC = -1,
 * 9-7/9-8 (total_zeros), 9-9a (chroma DC total_zeros), 9-10 (run_before). */
#define SCROLL_DYN_TABS                                                                        \
    {{{1, 0, 0, 0, 6, 2, 0, 0, 8, 6, 3, 0, 9, 8, 7, 5, 10, 9, 8, 6, 11, 10, 9, 7, 13, 11, 10, 8, \
       13, 13, 11, 9, 13, 13, 13, 10, 14, 14, 13, 11, 14, 14, 14, 13, 15, 15, 14, 14, 15, 15,    \
       15, 14, 16, 15, 15, 15, 16, 16, 16, 15, 16, 16, 16, 16, 16, 16, 16, 16},                  \
      {2, 0, 0, 0, 6, 2, 0, 0, 6, 5, 3, 0, 7, 6, 6, 4, 8, 6, 6, 4, 8, 7, 7, 5, 9, 8, 8, 6,       \
       11, 9, 9, 6, 11, 11, 11, 7, 12, 11, 11, 9, 12, 12, 12, 11, 12, 12, 12, 11, 13, 13, 13,    \
       12, 13, 13, 13, 13, 13, 14, 13, 13, 14, 14, 14, 13, 14, 14, 14, 14},                      \
      {4, 0, 0, 0, 6, 4, 0, 0, 6, 5, 4, 0, 6, 5, 5, 4, 7, 5, 5, 4, 7, 5, 5, 4, 7, 6, 6, 4,       \
       7, 6, 6, 4, 8, 7, 7, 5, 8, 8, 7, 6, 9, 8, 8, 7, 9, 9, 8, 8, 9, 9, 9, 8,                   \
       10, 9, 9, 9, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10}},                            \
     {{1, 0, 0, 0, 5, 1, 0, 0, 7, 4, 1, 0, 7, 6, 5, 3, 7, 6, 5, 3, 7, 6, 5, 4, 15, 6, 5, 4,      \
       11, 14, 5, 4, 8, 10, 13, 4, 15, 14, 9, 4, 11, 10, 13, 12, 15, 14, 9, 12, 11, 10, 13, 8,   \
       15, 1, 9, 12, 11, 14, 13, 8, 7, 10, 9, 12, 4, 6, 5, 8},                                   \
      {3, 0, 0, 0, 11, 2, 0, 0, 7, 7, 3, 0, 7, 10, 9, 5, 7, 6, 5, 4, 4, 6, 5, 6, 7, 6, 5, 8,     \
       15, 6, 5, 4, 11, 14, 13, 4, 15, 10, 9, 4, 11, 14, 13, 12, 8, 10, 9, 8, 15, 14, 13, 12,    \
       11, 10, 9, 12, 7, 11, 6, 8, 9, 8, 10, 1, 7, 6, 5, 4},                                     \
      {15, 0, 0, 0, 15, 14, 0, 0, 11, 15, 13, 0, 8, 12, 14, 12, 15, 10, 11, 11, 11, 8, 9, 10,    \
       9, 14, 13, 9, 8, 10, 9, 8, 15, 14, 13, 13, 11, 14, 10, 12, 15, 10, 13, 12, 11, 14, 9,     \
       12, 8, 10, 13, 8, 13, 7, 9, 12, 9, 12, 11, 10, 5, 8, 7, 6, 1, 4, 3, 2}},                  \
     {2, 0, 0, 0, 6, 1, 0, 0, 6, 6, 3, 0, 6, 7, 7, 6, 6, 8, 8, 7},                               \
     {1, 0, 0, 0, 7, 1, 0, 0, 4, 6, 1, 0, 3, 3, 2, 5, 2, 3, 2, 0},                               \
     {{1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6}, \
      {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6}, {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},      \
      {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5}, {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},                   \
      {6, 5, 3, 3, 3, 2, 3, 4, 3, 6}, {6, 4, 5, 3, 2, 2, 3, 3, 6}, {6, 6, 4, 2, 2, 3, 2, 5},     \
      {5, 5, 3, 2, 2, 2, 4}, {4, 4, 3, 3, 1, 3}, {4, 4, 2, 1, 3}, {3, 3, 1, 2}, {2, 2, 1},       \
      {1, 1}},                                                                                   \
     {{1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0}, \
      {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0}, {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},      \
      {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0}, {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},                   \
      {1, 1, 5, 4, 3, 3, 2, 1, 1, 0}, {1, 1, 1, 3, 3, 2, 2, 1, 0}, {1, 0, 1, 3, 2, 1, 1, 1},     \
      {1, 0, 1, 3, 2, 1, 1}, {0, 1, 1, 2, 1, 3}, {0, 1, 1, 1, 1}, {0, 1, 1, 1}, {0, 1, 1},       \
      {0, 1}},                                                                                   \
     {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}},                                                 \
     {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}},                                                 \
     {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3},                      \
      {2, 3, 3, 3, 3, 3, 3}, {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}},                   \
     {{1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0},                      \
      {3, 0, 1, 3, 2, 5, 4}, {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}},                     \
     {0, 2, 3, 7, 4, 8, 17, 13, 5, 18, 9, 14, 10, 15, 16, 11,                                    \
      1, 32, 33, 36, 34, 37, 44, 40, 35, 45, 38, 41, 39, 42, 43, 19,                             \
      6, 24, 25, 20, 26, 21, 46, 28, 27, 47, 22, 29, 23, 30, 31, 12},                            \
     {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15}}

/* ---------------------------------------------------------------------- */
/* bit sinks                                                               */
/* ---------------------------------------------------------------------- */
struct CountSink {
    uint32_t n;
    __device__ __host__ inline void put(uint32_t, int k) { n += (uint32_t)k; }
};

/* Captures up to 128 bits in registers (a 128-bit shift register, bits
 * right-aligned): a block is CAVLC-coded once, measured, and its bits kept
 * across the barrier until their position is known.  over = longer than
 * 128 bits (re-encode into the buffer then). */
struct CapSink {
    uint64_t hi, lo;
    uint32_t n;
    __device__ __host__ inline void put(uint32_t v, int k)      /* 0 <= k <= 32, branch-free */
    {
        v &= low_mask(k);
        hi = (hi << k) | ((lo >> 1) >> (63 - k));
        lo = (lo << k) | v;
        n += (uint32_t)k;
    }
    __device__ __host__ inline bool over() const { return n > 128; }
};

/* ORs bits into a zero-initialised word buffer starting at any bit
 * position; OR is the caller's atomic (LDS atomicOr) or plain |= on the
 * CPU.  Words are written once each except the two boundary words. */
template <class OR>
struct OrSink {
    OR orw;
    uint32_t wi;                  /* word of the pending bits                  */
    int fill;                     /* bits of word wi already used             */
    uint64_t acc;                 /* pending bits, left-aligned in 64         */
    __device__ __host__ inline void start(uint32_t pos)
    {
        wi = pos >> 5;
        fill = (int)(pos & 31);
        acc = 0;
    }
    __device__ __host__ inline void put(uint32_t v, int n)       /* n <= 32 */
    {
        if (n <= 0) return;
        v &= low_mask(n);
        acc |= ((uint64_t)v << (64 - n)) >> fill;
        fill += n;
        if (fill >= 32) {
            orw(wi, (uint32_t)(acc >> 32));
            acc <<= 32;
            fill -= 32;
            wi++;
        }
    }
    __device__ __host__ inline void finish()
    {
        if (fill > 0 && acc) orw(wi, (uint32_t)(acc >> 32));
    }
    /* the n <= 128 bits captured by c, first chunk n mod 32, then words */
    __device__ __host__ inline void put_cap(const CapSink &c)
    {
        int rem = (int)c.n;
        while (rem > 0) {
            const int k = ((rem - 1) & 31) + 1, pos = rem - k;
            uint64_t x;
            if (pos >= 64) x = c.hi >> (pos - 64);
            else if (pos == 0) x = c.lo;
            else x = (c.lo >> pos) | (c.hi << (64 - pos));
            put((uint32_t)x, k);
            rem -= k;
        }
    }
};

/* MB head without the trailing coded_block_pattern: mb_skip_run ue(0),
 * mb_type ue(0), ref_idx te(v), mvd_x se, mvd_y se (h264_writer.c:434-453) */
template <class S>
__device__ __host__ inline void put_mb_head(S &s, int ref, int dx, int dy, int nrefs)
{
    s.put(1, 1);
    s.put(1, 1);
    if (nrefs == 2) s.put((uint32_t)(1 - (ref & 1)), 1);
    else if (nrefs > 2) put_ue(s, (uint32_t)ref);
    put_se(s, dx);
    put_se(s, dy);
}

/* ---------------------------------------------------------------------- */
/* prediction                                                              */
/* ---------------------------------------------------------------------- */
/* waypoint table of the frame being coded (entries only ever appended) */
struct WpTab {
    const int32_t *wo, *wv;
    int h;                        /* picture height (luma)                    */
};

__device__ __host__ inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* (ref, mv_px) of MB row `row` of waypoint frame k: src/h264_writer.c:689-729
 * with the table as it stood when k was created (entries < k) */
__device__ __host__ inline void wp_row(const WpTab &T, int k, int row, int &ref, int &mv)
{
    const int wo = T.wo[k];
    const int a_end = (T.h - wo) / 16;                 /* C truncation (:690) */
    if (row < a_end) {
        int wa = -1, woa = 0;
        if (wo > MVL && k > 0)
            for (int i = 0; i < k; ++i) {
                if (!T.wv[i]) continue;
                const int w2 = T.wo[i];
                if (w2 <= wo && w2 > woa && wo - w2 <= MVL) {
                    wa = i;
                    woa = w2;
                }
            }
        ref = wa >= 0 ? 2 + wa : 0;
        mv = wa >= 0 ? wo - woa : wo;
    } else {
        ref = 1;
        mv = wo - T.h;
    }
}

/* luma: row y of reference ri -> (picture A / B, clamped row).  A waypoint
 * k only references pictures < k, so the chain ends within 9 steps. */
__device__ __host__ inline int luma_row(const WpTab &T, int ri, int y, int &yo)
{
    y = clampi(y, 0, T.h - 1);
    while (ri >= 2) {
        int ref, mv;
        wp_row(T, ri - 2, y / 16, ref, mv);
        y = clampi(y + mv, 0, T.h - 1);
        ri = ref;
    }
    yo = y;
    return ri;
}

/* chroma: the same chain for a row while every waypoint step is full-pel
 * (even mv, always so for waypoints created by the composer: offsets are
 * multiples of 496 and h of 16).  Returns -1 at a half-pel step. */
__device__ __host__ inline int chroma_row(const WpTab &T, int ri, int y, int &yo)
{
    const int hc = T.h / 2;
    y = clampi(y, 0, hc - 1);
    while (ri >= 2) {
        int ref, mv;
        wp_row(T, ri - 2, (2 * y) / 16, ref, mv);
        if ((4 * mv) & 7) return -1;
        y = clampi(y + ((4 * mv) >> 3), 0, hc - 1);
        ri = ref;
    }
    yo = y;
    return ri;
}

/* reference pictures of one stream: plane p of picture i */
struct RefPics {
    const uint8_t *pl[2][3];
    int w, h;
};

/* general chroma sample (or_ref_sample): any depth, bilinear at half-pel
 * waypoint steps.  D bounds the recursion (9 levels suffice). */
template <int D>
__device__ __host__ __attribute__((noinline)) int chroma_px_any(const WpTab &T, const RefPics &R,
                                                                int ri, int p, int x, int y)
{
    const int hc = T.h / 2;
    y = clampi(y, 0, hc - 1);
    if (ri < 2) return R.pl[ri][p][(size_t)y * (R.w / 2) + x];
    if constexpr (D == 0) {
        return 0;
    } else {
        int ref, mv;
        wp_row(T, ri - 2, (2 * y) / 16, ref, mv);
        const int q = 4 * mv, o = q >> 3, f = q & 7;
        const int a = chroma_px_any<D - 1>(T, R, ref, p, x, y + o);
        if (!f) return a;
        const int b = chroma_px_any<D - 1>(T, R, ref, p, x, y + o + 1);
        return ((8 - f) * a + f * b + 4) >> 3;
    }
}

/* ---------------------------------------------------------------------- */
/* transform / quantisation                                                */
/* ---------------------------------------------------------------------- */
__device__ __host__ inline void fwd4x4(const int x[16], int W[16])
{
    int t[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int s0 = x[4 * i] + x[4 * i + 3], s1 = x[4 * i + 1] + x[4 * i + 2];
        const int d0 = x[4 * i] - x[4 * i + 3], d1 = x[4 * i + 1] - x[4 * i + 2];
        t[4 * i + 0] = s0 + s1;
        t[4 * i + 1] = 2 * d0 + d1;
        t[4 * i + 2] = s0 - s1;
        t[4 * i + 3] = d0 - 2 * d1;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int s0 = t[j] + t[12 + j], s1 = t[4 + j] + t[8 + j];
        const int d0 = t[j] - t[12 + j], d1 = t[4 + j] - t[8 + j];
        W[j] = s0 + s1;
        W[4 + j] = 2 * d0 + d1;
        W[8 + j] = s0 - s1;
        W[12 + j] = d0 - 2 * d1;
    }
}

/* zig-zag scan (Table 8-13, frame): scan index -> raster position */
constexpr int ZZ[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};

/* a * b + c with a, b taken as signed 24-bit: one v_mad_i32_i24 (left to
 * itself the compiler picks a quarter-rate v_mad_u64_u32 here) */
__device__ __host__ inline int mad_i24(int a, int b, int c)
{
#ifdef __HIP_DEVICE_COMPILE__
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
#else
    return __mul24(a, b) + c;
#endif
}

/* raster position pos of a 4x4 block.  sign(w) ((|w| mf + f) >> qbits) as
 * one signed 24-bit multiply-add and an arithmetic shift: for w < 0 the
 * bias 2^qbits - 1 - f turns the floor into -((|w| mf + f) >> qbits)
 * (|w| <= 9180, mf < 2^14: the product fits 31 bits) */
__device__ __host__ inline int quant(int w, int pos, const QParams &q)
{
    const int i = pos >> 2, j = pos & 3;
    const int mf = ((i | j) & 1) == 0 ? q.mf0 : (((i & j) & 1) ? q.mf1 : q.mf2);
    /* bias by the sign mask as a bit select (v_bfi): no compare, no VCC */
    const uint32_t m = (uint32_t)(w >> 31);
    const int bias = (int)((m & (uint32_t)((1 << q.qbits) - 1 - q.qf)) | (~m & (uint32_t)q.qf));
    return clampi(mad_i24(w, mf, bias) >> q.qbits, -LEVEL_MAX, LEVEL_MAX);
}

/* ---------------------------------------------------------------------- */
/* residual -> transform -> quant on packed 16-bit pairs (k_dyn_row)        */
/* ---------------------------------------------------------------------- */
/* The same levels as fwd4x4 + quant, in about half the vector instructions:
 *   - residuals as 16-bit pairs straight from the pixel bytes (SDWA byte
 *     selects, one asm block for the 16): row i -> P = (r0, r1), Q = (r3, r2);
 *   - the horizontal butterflies on pairs: S = P + Q = (s03, s12), D = P - Q
 *     = (d03, d12); (t0, t2) = one v_pk_mad_i16 of S's halves, (t1, t3) two;
 *   - the vertical butterflies elementwise on the pairs (cols 0/2, cols 1/3);
 *     every value stays within int16 (|W| <= 9180);
 *   - quant per coefficient: the bias from the half's sign (v_bfi), one
 *     v_mad_i32_i16 reading the half (op_sel), the arithmetic shift written
 *     straight into its byte of the packed levels (SDWA dst_sel) -- in asm
 *     blocks of two words (8 coefficients interleaved, so no instruction
 *     reads the one before it).
 * The transform is plain vector code, so the compiler schedules it around
 * the packed-math forwarding wait state.  Both halves of a pair share their
 * MF class (cols 0/2 or 1/3 of one row).  On the host the same dataflow is
 * emulated (tests/hostsim checks it against fwd4x4 + quant). */
namespace pk {
__device__ __host__ inline uint32_t pack2(int lo, int hi) { return (uint32_t)(uint16_t)lo | (uint32_t)(uint16_t)hi << 16; }
__device__ __host__ inline int half(uint32_t x, int h) { return (int)(int16_t)(uint16_t)(x >> (16 * h)); }
}  // namespace pk

/* the quant blocks (generated: scan index k2 -> raster ZZ[k2] = 4 r + c ->
 * Ye[r] / Yo[r] (c even / odd), half c >> 1, MF by (r, c) parity; luma byte
 * k2, chroma AC byte k2 - 1) */
#define SCROLL_QLUMA0 \
    "v_bfe_i32 %[t0], %[ye0], 15, 1\n\t" \
    "v_bfe_i32 %[t1], %[yo0], 15, 1\n\t" \
    "v_bfe_i32 %[t2], %[ye1], 15, 1\n\t" \
    "v_bfe_i32 %[t3], %[ye2], 15, 1\n\t" \
    "v_bfe_i32 %[t4], %[yo1], 15, 1\n\t" \
    "v_ashrrev_i32 %[t5], 31, %[ye0]\n\t" \
    "v_ashrrev_i32 %[t6], 31, %[yo0]\n\t" \
    "v_ashrrev_i32 %[t7], 31, %[ye1]\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t2], %[t2], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t4], %[t4], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t5], %[t5], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t6], %[t6], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t7], %[t7], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_mad_i32_i16 %[t0], %[ye0], %[mf0], %[t0]\n\t" \
    "v_mad_i32_i16 %[t1], %[yo0], %[mf2], %[t1]\n\t" \
    "v_mad_i32_i16 %[t2], %[ye1], %[mf2], %[t2]\n\t" \
    "v_mad_i32_i16 %[t3], %[ye2], %[mf0], %[t3]\n\t" \
    "v_mad_i32_i16 %[t4], %[yo1], %[mf1], %[t4]\n\t" \
    "v_mad_i32_i16 %[t5], %[ye0], %[mf0], %[t5] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t6], %[yo0], %[mf2], %[t6] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t7], %[ye1], %[mf2], %[t7] op_sel:[1,0,0,0]\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t0] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t4] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t1] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t5] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t2] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t6] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t3] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t7] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
/* 8 coefficients */
#define SCROLL_QLUMA1 \
    "v_bfe_i32 %[t0], %[yo2], 15, 1\n\t" \
    "v_bfe_i32 %[t1], %[ye3], 15, 1\n\t" \
    "v_bfe_i32 %[t2], %[yo3], 15, 1\n\t" \
    "v_ashrrev_i32 %[t3], 31, %[ye2]\n\t" \
    "v_ashrrev_i32 %[t4], 31, %[yo1]\n\t" \
    "v_ashrrev_i32 %[t5], 31, %[yo2]\n\t" \
    "v_ashrrev_i32 %[t6], 31, %[ye3]\n\t" \
    "v_ashrrev_i32 %[t7], 31, %[yo3]\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t2], %[t2], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t4], %[t4], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t5], %[t5], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t6], %[t6], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t7], %[t7], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_mad_i32_i16 %[t0], %[yo2], %[mf2], %[t0]\n\t" \
    "v_mad_i32_i16 %[t1], %[ye3], %[mf2], %[t1]\n\t" \
    "v_mad_i32_i16 %[t2], %[yo3], %[mf1], %[t2]\n\t" \
    "v_mad_i32_i16 %[t3], %[ye2], %[mf0], %[t3] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t4], %[yo1], %[mf1], %[t4] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t5], %[yo2], %[mf2], %[t5] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t6], %[ye3], %[mf2], %[t6] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t7], %[yo3], %[mf1], %[t7] op_sel:[1,0,0,0]\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t0] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t4] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t1] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t5] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t2] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t6] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t3] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t7] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
/* 8 coefficients */
#define SCROLL_QCHROMA0 \
    "v_bfe_i32 %[t0], %[yo0], 15, 1\n\t" \
    "v_bfe_i32 %[t1], %[ye1], 15, 1\n\t" \
    "v_bfe_i32 %[t2], %[ye2], 15, 1\n\t" \
    "v_bfe_i32 %[t3], %[yo1], 15, 1\n\t" \
    "v_ashrrev_i32 %[t4], 31, %[ye0]\n\t" \
    "v_ashrrev_i32 %[t5], 31, %[yo0]\n\t" \
    "v_ashrrev_i32 %[t6], 31, %[ye1]\n\t" \
    "v_bfe_i32 %[t7], %[yo2], 15, 1\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t2], %[t2], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t4], %[t4], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t5], %[t5], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t6], %[t6], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t7], %[t7], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_mad_i32_i16 %[t0], %[yo0], %[mf2], %[t0]\n\t" \
    "v_mad_i32_i16 %[t1], %[ye1], %[mf2], %[t1]\n\t" \
    "v_mad_i32_i16 %[t2], %[ye2], %[mf0], %[t2]\n\t" \
    "v_mad_i32_i16 %[t3], %[yo1], %[mf1], %[t3]\n\t" \
    "v_mad_i32_i16 %[t4], %[ye0], %[mf0], %[t4] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t5], %[yo0], %[mf2], %[t5] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t6], %[ye1], %[mf2], %[t6] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t7], %[yo2], %[mf2], %[t7]\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t0] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t4] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t1] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t5] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t2] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t6] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t3] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t7] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
/* 8 coefficients */
#define SCROLL_QCHROMA1 \
    "v_bfe_i32 %[t0], %[ye3], 15, 1\n\t" \
    "v_bfe_i32 %[t1], %[yo3], 15, 1\n\t" \
    "v_ashrrev_i32 %[t2], 31, %[ye2]\n\t" \
    "v_ashrrev_i32 %[t3], 31, %[yo1]\n\t" \
    "v_ashrrev_i32 %[t4], 31, %[yo2]\n\t" \
    "v_ashrrev_i32 %[t5], 31, %[ye3]\n\t" \
    "v_ashrrev_i32 %[t6], 31, %[yo3]\n\t" \
    "v_bitop3_b32 %[t0], %[t0], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t2], %[t2], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t3], %[t3], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t4], %[t4], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t5], %[t5], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_bitop3_b32 %[t6], %[t6], %[k1], %[k0] bitop3:0xca\n\t" \
    "v_mad_i32_i16 %[t0], %[ye3], %[mf2], %[t0]\n\t" \
    "v_mad_i32_i16 %[t1], %[yo3], %[mf1], %[t1]\n\t" \
    "v_mad_i32_i16 %[t2], %[ye2], %[mf0], %[t2] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t3], %[yo1], %[mf1], %[t3] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t4], %[yo2], %[mf2], %[t4] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t5], %[ye3], %[mf2], %[t5] op_sel:[1,0,0,0]\n\t" \
    "v_mad_i32_i16 %[t6], %[yo3], %[mf1], %[t6] op_sel:[1,0,0,0]\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t0] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t4] dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t1] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t5] dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t2] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d1], %[sh], %[t6] dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t" \
    "v_ashrrev_i32_sdwa %[d0], %[sh], %[t3] dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n\t"
/* 7 coefficients */

/* a = source rows, pr = prediction rows (packed bytes): pk = 16 int8 levels
 * in scan order (chroma AC: the 15 from scan index 1, byte 15 zero), w0 =
 * W[0] (chroma DC, unquantised); the same values as fwd4x4 + quant of a - pr */
template <bool LUMA>
__device__ __host__ inline void levels_pk(const uint32_t a[4], const uint32_t pr[4], uint32_t pk4[4], int &w0,
                                          const QParams &q, uint32_t k1v, uint32_t k0v)
{
#ifdef __HIP_DEVICE_COMPILE__
    typedef short s2 __attribute__((ext_vector_type(2)));
    uint32_t P[4], Q[4];
    asm("v_sub_u16_sdwa %[p0], %[a0], %[b0] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_sub_u16_sdwa %[p1], %[a1], %[b1] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_sub_u16_sdwa %[p2], %[a2], %[b2] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_sub_u16_sdwa %[p3], %[a3], %[b3] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:BYTE_0\n\t"
        "v_sub_u16_sdwa %[q0], %[a0], %[b0] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "v_sub_u16_sdwa %[q1], %[a1], %[b1] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "v_sub_u16_sdwa %[q2], %[a2], %[b2] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "v_sub_u16_sdwa %[q3], %[a3], %[b3] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
        "v_sub_u16_sdwa %[p0], %[a0], %[b0] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_sub_u16_sdwa %[p1], %[a1], %[b1] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_sub_u16_sdwa %[p2], %[a2], %[b2] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_sub_u16_sdwa %[p3], %[a3], %[b3] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 src1_sel:BYTE_1\n\t"
        "v_sub_u16_sdwa %[q0], %[a0], %[b0] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_sub_u16_sdwa %[q1], %[a1], %[b1] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_sub_u16_sdwa %[q2], %[a2], %[b2] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 src1_sel:BYTE_2\n\t"
        "v_sub_u16_sdwa %[q3], %[a3], %[b3] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 src1_sel:BYTE_2"
        : [p0] "=&v"(P[0]), [p1] "=&v"(P[1]), [p2] "=&v"(P[2]), [p3] "=&v"(P[3]), [q0] "=&v"(Q[0]),
          [q1] "=&v"(Q[1]), [q2] "=&v"(Q[2]), [q3] "=&v"(Q[3])
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [b0] "v"(pr[0]), [b1] "v"(pr[1]),
          [b2] "v"(pr[2]), [b3] "v"(pr[3]));
    s2 E[4], O[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const s2 p = __builtin_bit_cast(s2, P[i]), q = __builtin_bit_cast(s2, Q[i]);
        const s2 S = p + q, D = p - q;
        E[i] = S.yy * (s2){1, -1} + S.xx;                   /* (t0, t2) */
        O[i] = D.yy * (s2){1, -2} + D.xx * (s2){2, 1};      /* (t1, t3) */
    }
    uint32_t ye[4], yo[4];                                  /* row k: (W[4k], W[4k+2]), (W[4k+1], W[4k+3]) */
    {
        const s2 s0 = E[0] + E[3], s1 = E[1] + E[2], d0 = E[0] - E[3], d1 = E[1] - E[2];
        ye[0] = __builtin_bit_cast(uint32_t, s0 + s1);
        ye[2] = __builtin_bit_cast(uint32_t, s0 - s1);
        ye[1] = __builtin_bit_cast(uint32_t, d0 * (s2){2, 2} + d1);
        ye[3] = __builtin_bit_cast(uint32_t, d0 - d1 * (s2){2, 2});
    }
    {
        const s2 s0 = O[0] + O[3], s1 = O[1] + O[2], d0 = O[0] - O[3], d1 = O[1] - O[2];
        yo[0] = __builtin_bit_cast(uint32_t, s0 + s1);
        yo[2] = __builtin_bit_cast(uint32_t, s0 - s1);
        yo[1] = __builtin_bit_cast(uint32_t, d0 * (s2){2, 2} + d1);
        yo[3] = __builtin_bit_cast(uint32_t, d0 - d1 * (s2){2, 2});
    }
    w0 = (int)(int16_t)(uint16_t)ye[0];
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
#define SCROLL_QOPS(D0, D1)                                                                            \
    : [d0] "=&v"(D0), [d1] "=&v"(D1), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),   \
      [t4] "=&v"(t4), [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7)                                     \
    : [ye0] "v"(ye[0]), [ye1] "v"(ye[1]), [ye2] "v"(ye[2]), [ye3] "v"(ye[3]), [yo0] "v"(yo[0]),          \
      [yo1] "v"(yo[1]), [yo2] "v"(yo[2]), [yo3] "v"(yo[3]),                                              \
      [k1] "v"(k1v), [k0] "v"(k0v), [sh] "v"(q.qbits), [mf0] "s"(q.mf0), \
      [mf1] "s"(q.mf1), [mf2] "s"(q.mf2)
    if constexpr (LUMA) {
        asm(SCROLL_QLUMA0 SCROLL_QOPS(pk4[0], pk4[1]));
        asm(SCROLL_QLUMA1 SCROLL_QOPS(pk4[2], pk4[3]));
    } else {
        asm(SCROLL_QCHROMA0 SCROLL_QOPS(pk4[0], pk4[1]));
        asm(SCROLL_QCHROMA1 SCROLL_QOPS(pk4[2], pk4[3]));
    }
#undef SCROLL_QOPS
#else
    (void)k1v;
    (void)k0v;
    using pk::half;
    using pk::pack2;
    uint32_t E[4], O[4];
    for (int i = 0; i < 4; ++i) {
        int r[4];
        for (int c = 0; c < 4; ++c) r[c] = (int)((a[i] >> (8 * c)) & 255u) - (int)((pr[i] >> (8 * c)) & 255u);
        const uint32_t P = pack2(r[0], r[1]), Q = pack2(r[3], r[2]);
        const uint32_t S = pack2(half(P, 0) + half(Q, 0), half(P, 1) + half(Q, 1));
        const uint32_t D = pack2(half(P, 0) - half(Q, 0), half(P, 1) - half(Q, 1));
        E[i] = pack2(half(S, 0) + half(S, 1), half(S, 0) - half(S, 1));
        O[i] = pack2(2 * half(D, 0) + half(D, 1), half(D, 0) - 2 * half(D, 1));
    }
    uint32_t ye[4], yo[4];
    for (int g = 0; g < 2; ++g) {
        const uint32_t *X = g ? O : E;
        uint32_t *Y = g ? yo : ye;
        for (int h = 0; h < 2; ++h) {
            const int s0 = half(X[0], h) + half(X[3], h), s1 = half(X[1], h) + half(X[2], h);
            const int d0 = half(X[0], h) - half(X[3], h), d1 = half(X[1], h) - half(X[2], h);
            const int v[4] = {s0 + s1, 2 * d0 + d1, s0 - s1, d0 - 2 * d1};
            for (int k = 0; k < 4; ++k) Y[k] = (h ? Y[k] & 0xffffu : 0u) | (uint32_t)(uint16_t)v[k] << (16 * h);
        }
    }
    w0 = half(ye[0], 0);
    pk4[0] = pk4[1] = pk4[2] = pk4[3] = 0;
    for (int k2 = LUMA ? 0 : 1; k2 < 16; ++k2) {
        const int p = ZZ[k2], r = p >> 2, c = p & 3, o = LUMA ? k2 : k2 - 1;
        const int mf = ((r | c) & 1) == 0 ? q.mf0 : (((r & c) & 1) ? q.mf1 : q.mf2);
        const uint32_t y = (c & 1) ? yo[r] : ye[r];
        const int w = half(y, c >> 1);
        const uint32_t sg = (uint32_t)(w >> 31);
        const uint32_t bias = (sg & (uint32_t)((1 << q.qbits) - 1 - q.qf)) | (~sg & (uint32_t)q.qf);
        const int v = w * mf + (int)bias;
        pk4[o >> 2] |= ((uint32_t)(v >> q.qbits) & 255u) << (8 * (o & 3));
    }
#endif
}

/* the same with the bias pair (k1 = 2^qbits - 1 - qf, k0 = qf) from the
 * QParams; callers in a loop pass them pinned in VGPRs (levels_bias), so
 * the bias select is a full-rate v_bitop3 (with an SGPR operand it issues
 * at half rate: profiles/r06_valu_rate2.json) */
template <bool LUMA>
__device__ __host__ inline void levels_pk(const uint32_t a[4], const uint32_t pr[4], uint32_t pk4[4], int &w0,
                                          const QParams &q)
{
    levels_pk<LUMA>(a, pr, pk4, w0, q, (uint32_t)((1 << q.qbits) - 1 - q.qf), (uint32_t)q.qf);
}
struct LevelsBias {
    uint32_t k1, k0;
};
__device__ __host__ inline LevelsBias levels_bias(const QParams &q)
{
    LevelsBias b{(uint32_t)((1 << q.qbits) - 1 - q.qf), (uint32_t)q.qf};
#ifdef __HIP_DEVICE_COMPILE__
    asm("" : "+v"(b.k1), "+v"(b.k0));
#endif
    return b;
}

/* non-zero bytes of a word (levels packed as int8) */
__device__ __host__ inline int nz_bytes(uint32_t x)
{
    return __builtin_popcount((((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u);
}

/* bit i = level i != 0 for 16 packed int8 levels (byte i & 3 of word
 * i >> 2): per word the bytes' "non-zero" flags at bits 7/15/23/31, gathered
 * to a nibble by one multiply (the partial products do not overlap) */
__device__ __host__ inline uint32_t nz_nibble(uint32_t x)
{
    const uint32_t hb = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
    return (hb * 0x00204081u) >> 28;
}
__device__ __host__ inline uint32_t nz_mask16(uint4 pk)
{
    return nz_nibble(pk.x) | nz_nibble(pk.y) << 4 | nz_nibble(pk.z) << 8 | nz_nibble(pk.w) << 12;
}
/* the same with the two byte masks passed in (k_dyn_row pins them in VGPRs:
 * the add and the v_bitop3 then issue at full rate, not half as with SGPR
 * operands) */
struct NzConst {
    uint32_t c7f, c80;
};
__device__ __host__ inline NzConst nz_const()
{
    NzConst c{0x7f7f7f7fu, 0x80808080u};
#ifdef __HIP_DEVICE_COMPILE__
    asm("" : "+v"(c.c7f), "+v"(c.c80));
#endif
    return c;
}
__device__ __host__ inline uint32_t nz_nibble_c(uint32_t x, const NzConst &c)
{
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t hb = __builtin_amdgcn_bitop3_b32((x & c.c7f) + c.c7f, c.c80, x, 0xc8);   /* ((x & 7f) + 7f | x) & 80 */
#else
    const uint32_t hb = (((x & c.c7f) + c.c7f) | x) & c.c80;
#endif
    return (hb * 0x00204081u) >> 28;
}
__device__ __host__ inline uint32_t nz_mask16_c(uint4 pk, const NzConst &c)
{
    return nz_nibble_c(pk.x, c) | nz_nibble_c(pk.y, c) << 4 | nz_nibble_c(pk.z, c) << 8 | nz_nibble_c(pk.w, c) << 12;
}

/* chroma DC (2x2): qbits + 1, f doubled (|w| <= 16320; q: the chroma QP's) */
__device__ __host__ inline int quant_dc(int w, const QParams &q)
{
    const int bias = w < 0 ? (1 << (q.qbits + 1)) - 1 - 2 * q.qf : 2 * q.qf;
    return clampi(mad_i24(w, q.mf0, bias) >> (q.qbits + 1), -LEVEL_MAX, LEVEL_MAX);
}

/* ---------------------------------------------------------------------- */
/* CAVLC (9.2)                                                             */
/* ---------------------------------------------------------------------- */
__device__ __host__ inline int nc_of(int nA, int nB)
{
    if (nA >= 0 && nB >= 0) return (nA + nB + 1) >> 1;
    if (nA >= 0) return nA;
    if (nB >= 0) return nB;
    return 0;
}

/* level_prefix / level_suffix as ONE field: prefix zeros, '1', suffix
 * (<= 16 + 12 bits) */
__device__ __host__ inline void level_field(int code, int sl, uint32_t &v, int &len)
{
    int prefix, ssize = sl, suffix = 0;
    if (sl == 0) {
        if (code < 14) {
            prefix = code;
            ssize = 0;
        } else if (code < 30) {
            prefix = 14;
            ssize = 4;
            suffix = code - 14;
        } else {
            prefix = 15;
            ssize = 12;
            suffix = code - 30;
        }
    } else if (code < (15 << sl)) {
        prefix = code >> sl;
        suffix = code & ((1 << sl) - 1);
    } else {
        prefix = 15;
        ssize = 12;
        suffix = code - (15 << sl);
    }
    v = (1u << ssize) | (uint32_t)suffix;
    len = prefix + 1 + ssize;
}

template <class S>
__device__ __host__ inline void put_level(S &s, int code, int sl)
{
    int prefix, ssize = sl, suffix = 0;
    if (sl == 0) {
        if (code < 14) {
            prefix = code;
            ssize = 0;
        } else if (code < 30) {
            prefix = 14;
            ssize = 4;
            suffix = code - 14;
        } else {
            prefix = 15;
            ssize = 12;
            suffix = code - 30;
        }
    } else if (code < (15 << sl)) {
        prefix = code >> sl;
        suffix = code & ((1 << sl) - 1);
    } else {
        prefix = 15;
        ssize = 12;
        suffix = code - (15 << sl);
    }
    s.put(1, prefix + 1);                              /* prefix zeros, then '1' */
    if (ssize) s.put((uint32_t)suffix, ssize);
}

/* coef: `max` levels in scan order (16 luma, 15 AC, 4 chroma DC with
 * nC = -1); returns TotalCoeff.  Works on a non-zero mask and reads the
 * levels in place (no per-lane arrays: nothing spills to scratch). */
__device__ __host__ inline int top_bit(uint32_t m) { return 31 - __clz((int)m); }

template <class S, class C>
__device__ __host__ inline int cavlc_block(S &s, const Tabs &T, const C *coef, int max, int nC)
{
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i < max && coef[i]) nz |= 1u << i;
    const int tc = __builtin_popcount(nz);
    int t1 = 0;
    {
        uint32_t m = nz;
        while (m && t1 < 3) {
            const int p = top_bit(m);
            const int v = coef[p];
            if (v != 1 && v != -1) break;
            t1++;
            m &= ~(1u << p);
        }
    }
    if (nC == -1) {
        s.put(T.ctdc_bits[4 * tc + t1], T.ctdc_len[4 * tc + t1]);
    } else if (nC >= 8) {
        s.put(tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u, 6);
    } else {
        const int tb = nC < 2 ? 0 : (nC < 4 ? 1 : 2);
        s.put(T.ct_bits[tb][4 * tc + t1], T.ct_len[tb][4 * tc + t1]);
    }
    if (tc == 0) return 0;
    const int hi = top_bit(nz);
    uint32_t m = nz;
    for (int k = 0; k < t1; ++k) {
        const int p = top_bit(m);
        s.put(coef[p] < 0 ? 1u : 0u, 1);
        m &= ~(1u << p);
    }
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int k = t1; k < tc; ++k) {
        const int p = top_bit(m);
        m &= ~(1u << p);
        const int L = coef[p];
        int code = L > 0 ? 2 * L - 2 : -2 * L - 1;
        if (k == t1 && t1 < 3) code -= 2;
        put_level(s, code, sl);
        if (sl == 0) sl = 1;
        if ((L < 0 ? -L : L) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    const int tz = hi + 1 - tc;
    if (tc < max) {
        if (max == 4) s.put(T.tzdc_bits[tc - 1][tz], T.tzdc_len[tc - 1][tz]);
        else s.put(T.tz_bits[tc - 1][tz], T.tz_len[tc - 1][tz]);
    }
    int zl = tz;
    m = nz;
    int p = hi;
    for (int k = 0; k < tc - 1 && zl > 0; ++k) {
        m &= ~(1u << p);
        const int q = top_bit(m);
        const int run = p - q - 1;
        const int zi = (zl < 7 ? zl : 7) - 1;
        s.put(T.rb_bits[zi][run], T.rb_len[zi][run]);
        zl -= run;
        p = q;
    }
    return tc;
}

/* drops the first `skip` bits (a coeff_token) of what is put: a block's
 * CAVLC body from cavlc_block */
template <class S>
struct SkipSink {
    S &in;
    uint32_t skip;
    __device__ __host__ inline void put(uint32_t v, int n)
    {
        if (n <= 0) return;
        if (skip >= (uint32_t)n) {
            skip -= (uint32_t)n;
            return;
        }
        if (skip) {
            n -= (int)skip;
            v &= low_mask(n);
            skip = 0;
        }
        in.put(v, n);
    }
};

/* TotalCoeff and TrailingOnes (9.2.1) of a block in scan order */
template <class C>
__device__ __host__ inline int tc_t1_of(const C *c, int max, int &t1)
{
    int tc = 0;
    t1 = 0;
    bool stop = false;
    for (int i = max - 1; i >= 0; --i) {
        if (!c[i]) continue;
        ++tc;
        if (stop || t1 >= 3) continue;
        if (c[i] == 1 || c[i] == -1) t1++;
        else stop = true;
    }
    return tc;
}

/* coeff_token (9.2.1) of (TotalCoeff, TrailingOnes) for nC: (bits, len) */
__device__ __host__ inline void coeff_token(const Tabs &T, int tc, int t1, int nC, uint32_t &v, int &len)
{
    if (nC == -1) {
        v = T.ctdc_bits[4 * tc + t1];
        len = T.ctdc_len[4 * tc + t1];
    } else if (nC >= 8) {
        v = tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u;
        len = 6;
    } else {
        const int tb = nC < 2 ? 0 : (nC < 4 ? 1 : 2);
        v = T.ct_bits[tb][4 * tc + t1];
        len = T.ct_len[tb][4 * tc + t1];
    }
}

/* CAVLC tables packed (len << 8 | bits) for one LDS read per field */
struct alignas(16) PTabs {
    uint16_t ct[4][68];           /* [0..2]: nC tables, [3]: chroma DC (nC = -1) */
    uint16_t tz[15][16];
    uint16_t tzdc[3][4];
    uint16_t rb[7][16];
};
/* the subset k_dyn_row keeps in LDS: its bodies take total_zeros / run_before
 * from one global table entry per block, so only coeff_token and the chroma
 * DC block's fields stay (480 bytes less per workgroup; config 5's 47-MB rows
 * still need 33.5 KB, four resident workgroups per CU -- five would need
 * 32 KB) */
struct alignas(16) RowTabs {
    uint16_t ct[4][68];
    uint16_t tzdc[3][4];
    uint16_t rb[7][16];
};

__device__ __host__ inline void build_ptabs(const Tabs &T, PTabs &P, int tid, int nthr)
{
    for (int i = tid; i < 3 * 68; i += nthr)
        P.ct[i / 68][i % 68] = (uint16_t)(T.ct_len[i / 68][i % 68] << 8 | T.ct_bits[i / 68][i % 68]);
    for (int i = tid; i < 68; i += nthr)
        P.ct[3][i] = i < 20 ? (uint16_t)(T.ctdc_len[i] << 8 | T.ctdc_bits[i]) : (uint16_t)0;
    for (int i = tid; i < 15 * 16; i += nthr)
        P.tz[i / 16][i % 16] = (uint16_t)(T.tz_len[i / 16][i % 16] << 8 | T.tz_bits[i / 16][i % 16]);
    for (int i = tid; i < 12; i += nthr)
        P.tzdc[i / 4][i % 4] = (uint16_t)(T.tzdc_len[i / 4][i % 4] << 8 | T.tzdc_bits[i / 4][i % 4]);
    for (int i = tid; i < 7 * 16; i += nthr)
        P.rb[i / 16][i % 16] = i % 16 < 15 ? (uint16_t)(T.rb_len[i / 16][i % 16] << 8 | T.rb_bits[i / 16][i % 16])
                                           : (uint16_t)0;
}

/* the same at compile time (kernels copy it into LDS with 16-byte loads) */
constexpr PTabs make_ptabs(const Tabs &T)
{
    PTabs P{};
    for (int i = 0; i < 3 * 68; ++i)
        P.ct[i / 68][i % 68] = (uint16_t)(T.ct_len[i / 68][i % 68] << 8 | T.ct_bits[i / 68][i % 68]);
    for (int i = 0; i < 68; ++i)
        P.ct[3][i] = i < 20 ? (uint16_t)(T.ctdc_len[i] << 8 | T.ctdc_bits[i]) : (uint16_t)0;
    for (int i = 0; i < 15 * 16; ++i)
        P.tz[i / 16][i % 16] = (uint16_t)(T.tz_len[i / 16][i % 16] << 8 | T.tz_bits[i / 16][i % 16]);
    for (int i = 0; i < 12; ++i)
        P.tzdc[i / 4][i % 4] = (uint16_t)(T.tzdc_len[i / 4][i % 4] << 8 | T.tzdc_bits[i / 4][i % 4]);
    for (int i = 0; i < 7 * 16; ++i)
        P.rb[i / 16][i % 16] = i % 16 < 15 ? (uint16_t)(T.rb_len[i / 16][i % 16] << 8 | T.rb_bits[i / 16][i % 16])
                                           : (uint16_t)0;
    return P;
}

/* level_prefix / level_suffix as one field, branch-free (9.2.2.1): the
 * common case (level_prefix = code >> sl, sl suffix bits) and the two
 * escapes (sl = 0: prefix 14 with a 4-bit suffix for codes 14..29; prefix 15
 * with a 12-bit suffix past the range) merged by bit masks -- written with
 * selects, the compiler made exec-mask branches of them */
__device__ __host__ inline void level_field_bf(int code, int sl, uint32_t &v, int &len)
{
    const int lim = sl ? (15 << sl) : 30;                  /* first escaped code */
    const uint32_t me = 0u - (uint32_t)(code >= lim);      /* prefix 15, 12-bit suffix */
    const uint32_t mm = 0u - (uint32_t)(sl == 0 && code >= 14 && code < 30);   /* prefix 14, 4-bit */
    const uint32_t mc = ~(me | mm);
    const uint32_t prefix = ((uint32_t)(code >> sl) & mc) | (14u & mm) | (15u & me);
    const uint32_t ssize = ((uint32_t)sl & mc) | (4u & mm) | (12u & me);
    const uint32_t suffix = ((uint32_t)(code & ((1 << sl) - 1)) & mc) | ((uint32_t)(code - 14) & mm) |
                            ((uint32_t)(code - lim) & me);
    v = (1u << ssize) | suffix;
    len = (int)(prefix + 1u + ssize);
}

/* The nC-independent part of a CAVLC block (everything after coeff_token:
 * trailing-ones signs, levels, total_zeros, run_before) of up to 16 packed
 * int8 levels (scan order, level i in byte i & 3 of word i >> 2), maxc =
 * maxNumCoeff (16 luma, 15 chroma AC; the level bytes past maxc are zero):
 * the trailing-one signs as one field, a loop over the other NON-ZERO
 * levels (branch-free inside: the wave iterates the max over its lanes;
 * callers group blocks by TotalCoeff), then a light loop for run_before
 * while zeros are left, its codes gathered in a 64-bit side register.
 * The levels come by value: an array indexed by a variable would be kept
 * in scratch memory.  Returns TotalCoeff, TrailingOnes in t1o; ok = false
 * when cap or the run register overflowed (cap.n is still exact). */
template <class CAP, bool LB = false>
__device__ __host__ inline int cavlc_body(CAP &cap, const PTabs &P, uint4 pk, int maxc, int &t1o, bool &ok,
                                          const int8_t *lb = nullptr)
{
    /* LB: lb holds the same 16 levels as bytes in LDS (k_dyn_row): one byte
     * read per level instead of a half select + 64-bit shift + sign extension */
    const uint32_t nz = nz_mask16(pk);
    const int tc = __builtin_popcount(nz);
    const uint64_t lo64 = (uint64_t)pk.x | (uint64_t)pk.y << 32, hi64 = (uint64_t)pk.z | (uint64_t)pk.w << 32;
    auto lev = [](uint64_t lo, uint64_t hi, int p) -> int {   /* captures nothing: no lambda object */
        const uint64_t v = (p & 8) ? hi : lo;
        return (int)(int8_t)(uint8_t)(v >> (8 * (p & 7)));
    };
    /* trailing ones (at most 3 +-1 levels from the top): their signs go out
     * as one field; the level loop starts below them */
    int t1 = 0;
    uint32_t sg = 0, m = nz;
    {
        bool run = true;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int p = m ? top_bit(m) : 0;
            const int v = m ? (LB ? (int)lb[p] : lev(lo64, hi64, p)) : 0;
            run = run && m && (v == 1 || v == -1);
            t1 += run ? 1 : 0;
            sg = run ? (sg << 1) | (v < 0 ? 1u : 0u) : sg;
            m &= run ? ~(1u << p) : ~0u;
        }
    }
    t1o = t1;
    ok = true;
    if (tc == 0) return 0;
    /* the fields gather in a 64-bit register (right-aligned, an bits) and
     * go to cap only when it would overflow and at the end */
    uint64_t acc = sg;
    uint32_t an = (uint32_t)t1;
    auto push = [](uint64_t &ac, uint32_t &n, uint32_t v, uint32_t len, CAP &c) {
        if (n + len > 64u) {                               /* rare: spill */
            if (n > 32u) c.put((uint32_t)(ac >> 32), (int)(n - 32u));
            c.put((uint32_t)ac, n > 32u ? 32 : (int)n);
            ac = 0;
            n = 0;
        }
        ac = (ac << len) | v;
        n += len;
    };
    const int hi = top_bit(nz);
    const int tz = hi + 1 - tc;
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    int adj = t1 < 3 ? 2 : 0;                              /* the first level after < 3 trailing ones */
    for (int k = t1; k < tc; ++k) {                        /* levels below the trailing ones */
        const int p = top_bit(m);
        m &= ~(1u << p);
        const int v = LB ? (int)lb[p] : lev(lo64, hi64, p);
        const int a = v < 0 ? -v : v;
        const int code = 2 * a - 2 + (v < 0 ? 1 : 0) - adj;
        adj = 0;
        /* level_prefix / level_suffix (9.2.2.1): code >> sl zeros and sl
         * suffix bits; escapes: prefix 14 + 4-bit suffix (sl 0, codes
         * 14..29), prefix 15 + 12-bit suffix past the range */
        const int lim = sl ? (15 << sl) : 30;
        const uint32_t mk = (1u << sl) - 1u;
        uint32_t fv = ((uint32_t)code & mk) | (mk + 1u);
        uint32_t fl = (uint32_t)((code >> sl) + 1 + sl);
        const bool e15 = code >= lim, e14 = sl == 0 && code >= 14;
        fv = e15 ? (uint32_t)(4096 + code - lim) : (e14 ? (uint32_t)(code + 2) : fv);
        fl = e15 ? 28u : (e14 ? 19u : fl);
        push(acc, an, fv, fl, cap);
        const int s1 = sl == 0 ? 1 : sl;
        sl = s1 + ((a > (3 << (s1 - 1)) && s1 < 6) ? 1 : 0);
    }
    if (tc < maxc) {
        const uint32_t e = P.tz[tc - 1][tz];
        push(acc, an, e & 255u, e >> 8, cap);
    }
    /* run_before: between consecutive non-zero levels from the top, while
     * zeros are left */
    int zl = tz, pprev = hi;
    uint32_t mm = nz & ~(1u << hi);
    for (int k = 1; k < tc && zl > 0; ++k) {
        const int p = top_bit(mm);
        mm &= ~(1u << p);
        const int run = pprev - p - 1;
        const uint32_t e = P.rb[(zl < 7 ? zl : 7) - 1][run];
        push(acc, an, e & 255u, e >> 8, cap);
        zl -= run;
        pprev = p;
    }
    if constexpr (LB) {                                    /* CapSink: nothing spilled -> acc is the body */
        if (cap.n == 0) {
            cap.lo = acc;
            cap.n = an;
            ok = true;
            return tc;
        }
    }
    if (an > 32u) cap.put((uint32_t)(acc >> 32), (int)(an - 32u));
    cap.put((uint32_t)acc, an > 32u ? 32 : (int)an);
    ok = cap.n <= 128;
    return tc;
}

/* total_zeros + run_before of a block depend only on its non-zero mask
 * (9.2.3, 9.2.4): k_dyn_row looks them up as ONE table entry instead of a
 * loop per block.  Entry = the bits MSB-first and left-aligned, then a '1'
 * sentinel, so len = 31 - ctz(entry) (at most 30 bits for 16 coefficients,
 * 25 for 15).  Table: [0, 65536) luma masks, [65536, 98304) chroma AC
 * (15 coefficients, bit i = scan index i + 1). */
constexpr int TZRB_N = 65536 + 32768;
__device__ __host__ inline uint32_t tzrb_entry(const Tabs &T, uint32_t nz, int maxc)
{
    const int tc = __builtin_popcount(nz);
    if (tc == 0) return 1u << 31;
    uint32_t acc = 0;
    int n = 0;
    const int hi = 31 - __builtin_clz(nz), tz = hi + 1 - tc;
    if (tc < maxc) {
        acc = T.tz_bits[tc - 1][tz];
        n = T.tz_len[tc - 1][tz];
    }
    int zl = tz, p = hi;
    uint32_t m = nz & ~(1u << hi);
    for (int k = 1; k < tc && zl > 0; ++k) {
        const int q = 31 - __builtin_clz(m);
        m &= ~(1u << q);
        const int run = p - q - 1, zi = (zl < 7 ? zl : 7) - 1;
        acc = (acc << T.rb_len[zi][run]) | T.rb_bits[zi][run];
        n += T.rb_len[zi][run];
        zl -= run;
        p = q;
    }
    return (n ? acc << (32 - n) : 0u) | (1u << (31 - n));
}

/* Level codewords of k_dyn_row's CAVLC body as ONE table entry per level
 * (9.2.2.1): class c = suffixLength 0..6, or 7 + suffixLength (0 / 1) for
 * the first level after fewer than three trailing ones (levelCode - 2), x
 * level v in [-LVT_V, LVT_V] at index v + LVT_V + 1.  Entry = codeword value
 * (the bits after level_prefix's zeros: at most 13) | its length << 13 | the
 * next level's class (suffixLength after this level) << 18.  Levels past
 * LVT_V take the arithmetic form. */
constexpr int LVT_V = 47, LVT_W = 96, LVT_C = 9, LVT_N = LVT_C * LVT_W;
__device__ __host__ constexpr uint32_t lvt_entry(int c, int v)
{
    if (v == 0 || v > LVT_V || v < -LVT_V) return 0u;
    const int sl = c >= 7 ? c - 7 : c, adj = c >= 7 ? 2 : 0;
    const int a = v < 0 ? -v : v;
    const int code = 2 * a - 2 + (v < 0 ? 1 : 0) - adj;
    if (code < 0) return 0u;                               /* |v| = 1 after < 3 trailing ones: never */
    const int lim = sl ? (15 << sl) : 30;
    const uint32_t mk = (1u << sl) - 1u;
    uint32_t fv = ((uint32_t)code & mk) | (mk + 1u), fl = (uint32_t)((code >> sl) + 1 + sl);
    if (code >= lim) {
        fv = (uint32_t)(4096 + code - lim);
        fl = 28u;
    } else if (sl == 0 && code >= 14) {
        fv = (uint32_t)(code + 2);
        fl = 19u;
    }
    const int s1 = sl == 0 ? 1 : sl;
    const int nx = s1 + ((a > (3 << (s1 - 1)) && s1 < 6) ? 1 : 0);
    return fv | fl << 13 | (uint32_t)nx << 18;
}
struct LvTab {
    uint32_t e[LVT_N];
};
constexpr LvTab make_lvt()
{
    LvTab T{};
    for (int c = 0; c < LVT_C; ++c)
        for (int i = 0; i < LVT_W; ++i) T.e[c * LVT_W + i] = lvt_entry(c, i - LVT_V - 1);
    return T;
}

/* cavlc_body for k_dyn_row (levels as LDS bytes lb, bit i = level i non-zero
 * in nz, tzrb = the block's tzrb_entry, loaded by the caller before the call
 * so its latency hides behind the level loop):
 *   - the top three non-zero levels read at once (positions from nz with a
 *     guard bit, so no zero test per find), TrailingOnes and their signs
 *     from them;
 *   - the level loop as in cavlc_body;
 *   - total_zeros + run_before as one field from the entry.
 * Same bits, TotalCoeff, TrailingOnes and ok as cavlc_body<CAP, true>.
 * bx: level i is byte i ^ bx of lb (k_dyn_row's records with their dwords
 * swizzled per slot, so lanes on consecutive slots read different banks) */
template <class CAP>
__device__ __host__ inline int cavlc_body_t(CAP &cap, const int8_t *lb, uint32_t nz, uint32_t tzrb, int &t1o,
                                            bool &ok, const uint32_t *lvt, uint32_t bx = 0)
{
    const int tc = __builtin_popcount(nz);
    /* g: the mask shifted up one with a guard bit 0 -- clz(g) <= 31, and
     * g's position q + 1 is level q; the guard reads lb[-1] (ignored) */
    const uint32_t g0 = (nz << 1) | 1u;
    const int c0 = __builtin_clz(g0);
    const uint32_t g1 = g0 & ~((0x80000000u >> c0) & ~1u);
    const int c1 = __builtin_clz(g1);
    const uint32_t g2 = g1 & ~((0x80000000u >> c1) & ~1u);
    const int c2 = __builtin_clz(g2);
    const uint32_t g3 = g2 & ~((0x80000000u >> c2) & ~1u);
    const int v0 = lb[(30 - c0) ^ (int)bx], v1 = lb[(30 - c1) ^ (int)bx], v2 = lb[(30 - c2) ^ (int)bx];
    /* a level is a trailing one iff it exists (not the guard) and is +-1 */
    const bool o0 = c0 < 31 && v0 * v0 == 1, o1 = o0 && c1 < 31 && v1 * v1 == 1;
    const bool o2 = o1 && c2 < 31 && v2 * v2 == 1;
    const int t1 = (int)o0 + (int)o1 + (int)o2;
    t1o = t1;
    ok = true;
    if (tc == 0) return 0;
    const uint32_t s3 = ((uint32_t)v0 >> 31) << 2 | ((uint32_t)v1 >> 31) << 1 | ((uint32_t)v2 >> 31);
    uint64_t acc = s3 >> (3 - t1);                         /* the trailing-one signs, first one first */
    uint32_t an = (uint32_t)t1;
    uint32_t m = (t1 == 0 ? g0 : (t1 == 1 ? g1 : (t1 == 2 ? g2 : g3))) >> 1;
    auto push = [](uint64_t &ac, uint32_t &n, uint32_t v, uint32_t len, CAP &c) {
        if (n + len > 64u) {                               /* rare: spill */
            if (n > 32u) c.put((uint32_t)(ac >> 32), (int)(n - 32u));
            c.put((uint32_t)ac, n > 32u ? 32 : (int)n);
            ac = 0;
            n = 0;
        }
        ac = (ac << len) | v;
        n += len;
    };
    /* the level class (lvt_entry): suffixLength, +7 for the first level
     * after fewer than three trailing ones */
    int cls = ((tc > 10 && t1 < 3) ? 1 : 0) + (t1 < 3 ? 7 : 0);
    /* the level codeword from the table, or (|v| > LVT_V) the arithmetic form */
    auto level_code = [&](int v, int cl) -> uint32_t {
        if (v >= -LVT_V && v <= LVT_V) return lvt[cl * LVT_W + v + LVT_V + 1];
        const int sl = cl >= 7 ? cl - 7 : cl, adj = cl >= 7 ? 2 : 0;
        const int a = v < 0 ? -v : v;
        const int code = 2 * a - 2 + (v < 0 ? 1 : 0) - adj;
        const int lim = sl ? (15 << sl) : 30;
        const uint32_t mk = (1u << sl) - 1u;
        uint32_t fv = ((uint32_t)code & mk) | (mk + 1u);
        uint32_t fl = (uint32_t)((code >> sl) + 1 + sl);
        const bool e15 = code >= lim, e14 = sl == 0 && code >= 14;
        fv = e15 ? (uint32_t)(4096 + code - lim) : (e14 ? (uint32_t)(code + 2) : fv);
        fl = e15 ? 28u : (e14 ? 19u : fl);
        const int s1 = sl == 0 ? 1 : sl;
        return fv | fl << 13 | (uint32_t)(s1 + ((a > (3 << (s1 - 1)) && s1 < 6) ? 1 : 0)) << 18;
    };
#ifndef SCROLL_CAVLC_NOPF
    /* round 6: the loop holds the table path only (levels clamped into the
     * table, a lane whose block has a level past LVT_V flagged), so the rare
     * arithmetic form costs no exec-mask branch per level; a flagged lane
     * codes its block again below with it.  The next level's byte is read
     * one iteration ahead, so each level waits for one LDS round trip (its
     * codeword) instead of two; past the last level m is 0 and the read is
     * the guard byte lb[-1] (unused) */
    const uint32_t m0 = m, an0 = an;
    const uint64_t acc0 = acc;
    const int cls0 = cls;
    const CAP cap0 = cap;
    bool big = false;
    int pn = top_bit(m);
    int vn = (int)lb[pn ^ (int)bx];
    for (int k = t1; k < tc; ++k) {                        /* levels below the trailing ones */
        const int v = vn;
        m &= ~(1u << pn);
        pn = top_bit(m);
        vn = (int)lb[pn ^ (int)bx];
        const int vc = v < -LVT_V ? -LVT_V : (v > LVT_V ? LVT_V : v);
        big |= vc != v;
        const uint32_t e = lvt[cls * LVT_W + vc + LVT_V + 1];
        push(acc, an, e & 0x1fffu, (e >> 13) & 31u, cap);
        cls = (int)(e >> 18);
    }
    if (big) {                                             /* rare: the block again, exact */
        m = m0;
        an = an0;
        acc = acc0;
        cls = cls0;
        cap = cap0;
        for (int k = t1; k < tc; ++k) {
            const int p = top_bit(m);
            m &= ~(1u << p);
            const uint32_t e = level_code((int)lb[p ^ (int)bx], cls);
            push(acc, an, e & 0x1fffu, (e >> 13) & 31u, cap);
            cls = (int)(e >> 18);
        }
    }
#else
    for (int k = t1; k < tc; ++k) {
        const int p = top_bit(m);
        m &= ~(1u << p);
        const uint32_t e = level_code((int)lb[p ^ (int)bx], cls);
        push(acc, an, e & 0x1fffu, (e >> 13) & 31u, cap);
        cls = (int)(e >> 18);
    }
#endif
    /* total_zeros + run_before: the entry's code, len = 31 - ctz */
    const uint32_t tzl = 31u - (uint32_t)__builtin_ctz(tzrb);
    push(acc, an, (tzrb >> 1) >> (31u - tzl), tzl, cap);
    if (cap.n == 0) {                                      /* nothing spilled: acc is the body */
        cap.lo = acc;
        cap.n = an;
        return tc;
    }
    if (an > 32u) cap.put((uint32_t)(acc >> 32), (int)(an - 32u));
    cap.put((uint32_t)acc, an > 32u ? 32 : (int)an);
    ok = cap.n <= 128;
    return tc;
}

/* chroma DC (2x2, nC = -1): the whole block from 4 levels in registers,
 * unrolled, packed LDS tables (P.ct[3], P.tzdc, P.rb) */
template <class CAP, class PT>
__device__ __host__ inline int cavlc_dc4(CAP &cap, const PT &P, const int c[4])
{
    const uint32_t nz = (c[0] != 0 ? 1u : 0u) | (c[1] != 0 ? 2u : 0u) | (c[2] != 0 ? 4u : 0u) |
                        (c[3] != 0 ? 8u : 0u);
    const int tc = __builtin_popcount(nz);
    int t1 = 0;
    bool trail = true;
#pragma unroll
    for (int i = 3; i >= 0; --i) {
        const bool one = c[i] == 1 || c[i] == -1;
        if (c[i] != 0) {
            trail = trail && one && t1 < 3;
            t1 += trail ? 1 : 0;
        }
    }
    {
        const uint32_t e = P.ct[3][4 * tc + t1];
        cap.put(e & 255u, (int)(e >> 8));
    }
    if (tc == 0) return 0;
    int k = 0, sl = 0, zl = 0, pprev = -1;
    uint64_t runs = 0;
    int rn = 0;
    const int hi = top_bit(nz);
    const int tz = hi + 1 - tc;
    zl = tz;
#pragma unroll
    for (int i = 3; i >= 0; --i) {
        const int v = c[i];
        if (v != 0) {
            const int a = v < 0 ? -v : v;
            if (k < t1) {
                cap.put(v < 0 ? 1u : 0u, 1);
            } else {
                int code = 2 * a - 2 + (v < 0 ? 1 : 0);
                if (k == t1 && t1 < 3) code -= 2;
                uint32_t fv;
                int fl;
                level_field_bf(code, sl, fv, fl);
                cap.put(fv, fl);
                if (sl == 0) sl = 1;
                if (a > (3 << (sl - 1)) && sl < 6) sl++;
            }
            if (k > 0 && zl > 0) {
                const int run = pprev - i - 1;
                const uint32_t e = P.rb[(zl < 7 ? zl : 7) - 1][run];
                runs = (runs << (e >> 8)) | (e & 255u);
                rn += (int)(e >> 8);
                zl -= run;
            }
            pprev = i;
            k++;
        }
    }
    if (tc < 4) {
        const uint32_t e = P.tzdc[tc - 1][tz];
        cap.put(e & 255u, (int)(e >> 8));
    }
    cap.put((uint32_t)runs, rn);                        /* <= 3 runs x 2 bits */
    return tc;
}

/* ---------------------------------------------------------------------- */
/* emulation prevention in closed form                                     */
/* ---------------------------------------------------------------------- */
/* nal.c:33-38 inserts 0x03 before RBSP byte i iff b_i <= 3 and the automaton
 * has seen two zero bytes since its last reset.  With k = the number of
 * zero bytes immediately before i in the ORIGINAL RBSP, that state is
 * exactly "k >= 2 and k even" (runs of zeros insert at k = 2, 4, 6, ...),
 * so every byte decides independently once k is known. */
__device__ __host__ inline bool ep_insert(uint32_t b, int k) { return b <= 3 && k >= 2 && !(k & 1); }

/* raster index of luma4x4BlkIdx blk (6.4.3) */
__device__ __host__ inline int blk_raster(int blk)
{
    const int q8 = blk >> 2, q4 = blk & 3;
    return 4 * ((q8 >> 1) * 2 + (q4 >> 1)) + (q8 & 1) * 2 + (q4 & 1);
}

/* ---------------------------------------------------------------------- */
/* MB order inside a NAL with the rect                                     */
/* ---------------------------------------------------------------------- */
struct Rect {
    int x0, y0, w, h;
};

/* x / d by multiply: m = magic(d) = ceil(2^32 / d) (0 for d = 1); exact for
 * x, d < 2^16 */
__device__ __host__ inline uint32_t magic32(uint32_t d) { return d <= 1 ? 0u : 0xffffffffu / d + 1u; }
__device__ __host__ inline uint32_t div_m(uint32_t x, uint32_t m) { return m ? __umulhi(x, m) : x; }
/* x / d for x * d < 2^16 (window task indices): m16 = ceil(2^16 / d) */
__device__ __host__ inline uint32_t magic16(uint32_t d) { return (65536u + d - 1u) / d; }
__device__ __host__ inline uint32_t div16(uint32_t x, uint32_t m16) { return __umul24(x, m16) >> 16; }

/* number of dynamic MBs before MB m (coding order) */
__device__ __host__ inline int dyn_rank(const Rect &r, int mbw, int m)
{
    const int y = m / mbw, x = m - y * mbw;
    if (y < r.y0) return 0;
    if (y >= r.y0 + r.h) return r.w * r.h;
    return (y - r.y0) * r.w + clampi(x - r.x0, 0, r.w);
}

/* dyn_rank / dyn_mb with the divisions by mbw / r.w as multiplies */
__device__ __host__ inline int dyn_rank_m(const Rect &r, int mbw, uint32_t m_mbw, int m)
{
    const int y = (int)div_m((uint32_t)m, m_mbw), x = m - y * mbw;
    if (y < r.y0) return 0;
    if (y >= r.y0 + r.h) return r.w * r.h;
    return (y - r.y0) * r.w + clampi(x - r.x0, 0, r.w);
}

__device__ __host__ inline int dyn_mb_m(const Rect &r, int mbw, uint32_t m_rw, int q)
{
    const int ry = (int)div_m((uint32_t)q, m_rw);
    return (r.y0 + ry) * mbw + r.x0 + (q - ry * r.w);
}

/* MB index of dynamic MB number q */
__device__ __host__ inline int dyn_mb(const Rect &r, int mbw, int q)
{
    const int ry = q / r.w;
    return (r.y0 + ry) * mbw + r.x0 + (q - ry * r.w);
}

}  // namespace dyn
}  // namespace scroll
#endif
