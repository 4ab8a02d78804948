/*
 * dyn_oracle.c -- CPU ORACLE (test infrastructure only): dynamic-rect
 * residual coder.  Specification and provenance: dyn_oracle.h.  Clause
 * numbers refer to ITU-T H.264; the CAVLC tables are transcribed from the
 * standard's Tables 9-5, 9-7, 9-8, 9-9, 9-10 and 9-4 and checked against
 * the reference's parser (trans_resizer.c:275-548) by tests.
 */
#include "dyn_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* synthetic pixels                                                          */
/* ------------------------------------------------------------------------ */
uint32_t or_mix32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

uint32_t or_dyn_seed(int s, int t)
{
    return (0x9E3779B9u * (uint32_t)s) ^ (0x85EBCA6Bu * (uint32_t)t);
}

static int or_clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

void or_dyn_source(uint8_t *dst, int s, int t, const or_dyn_rect *r)
{
    const uint32_t seed = or_dyn_seed(s, t);
    const int lw = 16 * r->w, lh = 16 * r->h, cw = 8 * r->w, ch = 8 * r->h;
    uint32_t i = 0;
    for (int y = 0; y < lh; ++y)
        for (int x = 0; x < lw; ++x, ++i) {
            const uint32_t h = or_mix32(seed + i * 0x9E3779B9u);
            const int X = 16 * r->x0 + x, Y = 16 * r->y0 + y;
            dst[i] = (uint8_t)or_clamp255(128 + ((X + 2 * Y + 3 * t) & 63) - 32 + (int)(h >> 28) - 8);
        }
    for (int p = 0; p < 2; ++p)
        for (int y = 0; y < ch; ++y)
            for (int x = 0; x < cw; ++x, ++i) {
                const uint32_t h = or_mix32(seed + i * 0x9E3779B9u);
                const int X = 8 * r->x0 + x, Y = 8 * r->y0 + y;
                dst[i] = (uint8_t)or_clamp255(128 + ((X + Y + t) & 15) - 8 + (int)(h >> 30));
            }
}

/* experiments/scroll-encoder/src/main.c:234-243 colours, bands of
 * h264_encoder.c:816-829 (or_ipcm_striped) */
void or_striped_planes(uint8_t *y, uint8_t *u, uint8_t *v, int w, int h, int which)
{
    static const uint8_t A[9] = {81, 90, 240, 145, 54, 34, 41, 240, 110};
    static const uint8_t B[9] = {210, 16, 146, 170, 166, 16, 106, 202, 222};
    const uint8_t *c = which == 0 ? A : B;
    const int mbh = h / 16, third = mbh / 3;
    for (int r = 0; r < h; ++r) {
        const int my = r / 16, s = my < third ? 0 : (my < 2 * third ? 1 : 2);
        memset(y + (size_t)r * w, c[3 * s], (size_t)w);
        if ((r & 1) == 0) {
            memset(u + (size_t)(r / 2) * (w / 2), c[3 * s + 1], (size_t)(w / 2));
            memset(v + (size_t)(r / 2) * (w / 2), c[3 * s + 2], (size_t)(w / 2));
        }
    }
}

/* ------------------------------------------------------------------------ */
/* reference samples (8.4.2.2): full-pel luma, 1/8-pel chroma, clamped       */
/* ------------------------------------------------------------------------ */
static int or_clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* (ref, mv_px) of MB row `row` in waypoint frame k: src/h264_writer.c:689-729
 * with the waypoint table as it stood when k was created (entries < k) */
static void or_wp_row(const or_cfg *c, int k, int row, int *ref, int *mv)
{
    const int wo = c->wp_off[k];
    const int a_end = (c->h - wo) / 16;
    if (row < a_end) {
        int wa = -1, woa = 0;
        if (wo > OR_MV_LIMIT && k > 0)
            for (int i = 0; i < k; ++i) {
                if (!c->wp_valid[i]) continue;
                const int w2 = c->wp_off[i];
                if (w2 <= wo && w2 > woa && wo - w2 <= OR_MV_LIMIT) { wa = i; woa = w2; }
            }
        *ref = wa >= 0 ? 2 + wa : 0;
        *mv = wa >= 0 ? wo - woa : wo;
    } else {
        *ref = 1;
        *mv = wo - c->h;
    }
}

int or_ref_sample(const or_cfg *c, const or_refs *R, int ri, int plane, int x, int y)
{
    const int pw = plane ? c->w / 2 : c->w, ph = plane ? c->h / 2 : c->h;
    x = or_clampi(x, 0, pw - 1);
    y = or_clampi(y, 0, ph - 1);
    if (ri < 2) {
        const or_pic *P = R->ab[ri];
        const uint8_t *pl = plane == 0 ? P->y : (plane == 1 ? P->u : P->v);
        return pl[(size_t)y * pw + x];
    }
    int ref, mv;
    or_wp_row(c, ri - 2, plane ? (2 * y) / 16 : y / 16, &ref, &mv);
    if (plane == 0) return or_ref_sample(c, R, ref, 0, x, y + mv);
    const int q = 4 * mv, o = q >> 3, f = q & 7;          /* 1/8 chroma pel */
    const int a = or_ref_sample(c, R, ref, plane, x, y + o);
    const int b = or_ref_sample(c, R, ref, plane, x, y + o + 1);
    return ((8 - f) * a + f * b + 4) >> 3;
}

/* ------------------------------------------------------------------------ */
/* transform / quantisation (8.5.12 inverse; JM-style forward)               */
/* ------------------------------------------------------------------------ */
static const int OR_MF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                                {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};
static const int OR_ZZ[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
#define OR_QP 26

void or_fwd4x4(const int x[16], int W[16])
{
    int t[16];
    for (int i = 0; i < 4; ++i) {
        const int *r = x + 4 * i;
        const int s0 = r[0] + r[3], s1 = r[1] + r[2], d0 = r[0] - r[3], d1 = r[1] - r[2];
        t[4 * i + 0] = s0 + s1;
        t[4 * i + 1] = 2 * d0 + d1;
        t[4 * i + 2] = s0 - s1;
        t[4 * i + 3] = d0 - 2 * d1;
    }
    for (int j = 0; j < 4; ++j) {
        const int s0 = t[j] + t[12 + j], s1 = t[4 + j] + t[8 + j];
        const int d0 = t[j] - t[12 + j], d1 = t[4 + j] - t[8 + j];
        W[j] = s0 + s1;
        W[4 + j] = 2 * d0 + d1;
        W[8 + j] = s0 - s1;
        W[12 + j] = d0 - 2 * d1;
    }
}

int or_qp_chroma(int qp)
{
    static const int T[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
    return qp < 30 ? qp : T[qp - 30];
}

int or_dyn_qp(const or_dyn_rect *r)
{
    return r->qp == OR_DYN_QP0 ? 0 : (r->qp ? r->qp : OR_QP);
}

/* pos = raster position in the 4x4 block; dc_chroma: 2x2 chroma DC; the
 * level clamped to +-OR_LEVEL_MAX (a bound only QP < 6 reaches) */
int or_quant(int w, int qp, int pos, int dc_chroma)
{
    const int i = pos / 4, j = pos % 4;
    const int cls = (i % 2 == 0 && j % 2 == 0) ? 0 : ((i % 2 == 1 && j % 2 == 1) ? 1 : 2);
    const int qbits = 15 + qp / 6, f = (1 << qbits) / 6;
    const int mf = OR_MF[qp % 6][dc_chroma ? 0 : cls];
    const int a = w < 0 ? -w : w;
    int z = dc_chroma ? (int)(((int64_t)a * mf + 2 * f) >> (qbits + 1))
                      : (int)(((int64_t)a * mf + f) >> qbits);
    if (z > OR_LEVEL_MAX) z = OR_LEVEL_MAX;
    return w < 0 ? -z : z;
}

/* ------------------------------------------------------------------------ */
/* CAVLC (9.2)                                                               */
/* ------------------------------------------------------------------------ */
/* coeff_token (Table 9-5): [table][TotalCoeff * 4 + TrailingOnes] */
static const uint8_t OR_CT_LEN[3][68] = {
    {1, 0, 0, 0, 6, 2, 0, 0, 8, 6, 3, 0, 9, 8, 7, 5, 10, 9, 8, 6, 11, 10, 9, 7, 13, 11, 10, 8,
     13, 13, 11, 9, 13, 13, 13, 10, 14, 14, 13, 11, 14, 14, 14, 13, 15, 15, 14, 14, 15, 15, 15, 14,
     16, 15, 15, 15, 16, 16, 16, 15, 16, 16, 16, 16, 16, 16, 16, 16},
    {2, 0, 0, 0, 6, 2, 0, 0, 6, 5, 3, 0, 7, 6, 6, 4, 8, 6, 6, 4, 8, 7, 7, 5, 9, 8, 8, 6,
     11, 9, 9, 6, 11, 11, 11, 7, 12, 11, 11, 9, 12, 12, 12, 11, 12, 12, 12, 11, 13, 13, 13, 12,
     13, 13, 13, 13, 13, 14, 13, 13, 14, 14, 14, 13, 14, 14, 14, 14},
    {4, 0, 0, 0, 6, 4, 0, 0, 6, 5, 4, 0, 6, 5, 5, 4, 7, 5, 5, 4, 7, 5, 5, 4, 7, 6, 6, 4,
     7, 6, 6, 4, 8, 7, 7, 5, 8, 8, 7, 6, 9, 8, 8, 7, 9, 9, 8, 8, 9, 9, 9, 8,
     10, 9, 9, 9, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10}};
static const uint8_t OR_CT_BITS[3][68] = {
    {1, 0, 0, 0, 5, 1, 0, 0, 7, 4, 1, 0, 7, 6, 5, 3, 7, 6, 5, 3, 7, 6, 5, 4, 15, 6, 5, 4,
     11, 14, 5, 4, 8, 10, 13, 4, 15, 14, 9, 4, 11, 10, 13, 12, 15, 14, 9, 12, 11, 10, 13, 8,
     15, 1, 9, 12, 11, 14, 13, 8, 7, 10, 9, 12, 4, 6, 5, 8},
    {3, 0, 0, 0, 11, 2, 0, 0, 7, 7, 3, 0, 7, 10, 9, 5, 7, 6, 5, 4, 4, 6, 5, 6, 7, 6, 5, 8,
     15, 6, 5, 4, 11, 14, 13, 4, 15, 10, 9, 4, 11, 14, 13, 12, 8, 10, 9, 8, 15, 14, 13, 12,
     11, 10, 9, 12, 7, 11, 6, 8, 9, 8, 10, 1, 7, 6, 5, 4},
    {15, 0, 0, 0, 15, 14, 0, 0, 11, 15, 13, 0, 8, 12, 14, 12, 15, 10, 11, 11, 11, 8, 9, 10,
     9, 14, 13, 9, 8, 10, 9, 8, 15, 14, 13, 13, 11, 14, 10, 12, 15, 10, 13, 12, 11, 14, 9, 12,
     8, 10, 13, 8, 13, 7, 9, 12, 9, 12, 11, 10, 5, 8, 7, 6, 1, 4, 3, 2}};
/* chroma DC (nC = -1) */
static const uint8_t OR_CTDC_LEN[20] = {2, 0, 0, 0, 6, 1, 0, 0, 6, 6, 3, 0, 6, 7, 7, 6, 6, 8, 8, 7};
static const uint8_t OR_CTDC_BITS[20] = {1, 0, 0, 0, 7, 1, 0, 0, 4, 6, 1, 0, 3, 3, 2, 5, 2, 3, 2, 0};
/* total_zeros (Tables 9-7, 9-8): [TotalCoeff - 1][total_zeros] */
static const uint8_t OR_TZ_LEN[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},       {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},             {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},                   {6, 4, 5, 3, 2, 2, 3, 3, 6},
    {6, 6, 4, 2, 2, 3, 2, 5},                         {5, 5, 3, 2, 2, 2, 4},
    {4, 4, 3, 3, 1, 3},                               {4, 4, 2, 1, 3},
    {3, 3, 1, 2},                                     {2, 2, 1},
    {1, 1}};
static const uint8_t OR_TZ_BITS[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},       {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},             {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},                   {1, 1, 1, 3, 3, 2, 2, 1, 0},
    {1, 0, 1, 3, 2, 1, 1, 1},                         {1, 0, 1, 3, 2, 1, 1},
    {0, 1, 1, 2, 1, 3},                               {0, 1, 1, 1, 1},
    {0, 1, 1, 1},                                     {0, 1, 1},
    {0, 1}};
/* chroma DC total_zeros (Table 9-9a): [TotalCoeff - 1][total_zeros] */
static const uint8_t OR_TZDC_LEN[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
static const uint8_t OR_TZDC_BITS[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};
/* run_before (Table 9-10): [min(zerosLeft, 7) - 1][run_before] */
static const uint8_t OR_RB_LEN[7][15] = {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3},
                                         {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},
                                         {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
static const uint8_t OR_RB_BITS[7][15] = {{1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0},
                                          {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},
                                          {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}};

static void or_put_level(or_bits *b, int code, int sl)
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
    if (suffix >= 4096) abort();             /* beyond Baseline/Main levels */
    or_put(b, 1, prefix + 1);                /* prefix zeros + '1' */
    if (ssize) or_put(b, (uint32_t)suffix, ssize);
}

int or_cavlc_block(or_bits *b, const int *coef, int max, int nC)
{
    int lv[16], pos[16], tc = 0;
    for (int i = max - 1; i >= 0; --i)
        if (coef[i]) {
            lv[tc] = coef[i];
            pos[tc] = i;
            tc++;
        }
    int t1 = 0;
    while (t1 < tc && t1 < 3 && (lv[t1] == 1 || lv[t1] == -1)) t1++;
    if (nC == -1) {
        or_put(b, OR_CTDC_BITS[4 * tc + t1], OR_CTDC_LEN[4 * tc + t1]);
    } else if (nC >= 8) {
        or_put(b, tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u, 6);
    } else {
        const int tb = nC < 2 ? 0 : (nC < 4 ? 1 : 2);
        or_put(b, OR_CT_BITS[tb][4 * tc + t1], OR_CT_LEN[tb][4 * tc + t1]);
    }
    if (tc == 0) return 0;
    for (int k = 0; k < t1; ++k) or_put(b, lv[k] < 0 ? 1u : 0u, 1);
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int k = t1; k < tc; ++k) {
        const int L = lv[k];
        int code = L > 0 ? 2 * L - 2 : -2 * L - 1;
        if (k == t1 && t1 < 3) code -= 2;
        or_put_level(b, code, sl);
        if (sl == 0) sl = 1;
        if ((L < 0 ? -L : L) > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int tz = pos[0] + 1 - tc;
    if (tc < max) {
        if (max == 4)
            or_put(b, OR_TZDC_BITS[tc - 1][tz], OR_TZDC_LEN[tc - 1][tz]);
        else
            or_put(b, OR_TZ_BITS[tc - 1][tz], OR_TZ_LEN[tc - 1][tz]);
    }
    int zl = tz;
    for (int k = 0; k < tc - 1 && zl > 0; ++k) {
        const int run = pos[k] - pos[k + 1] - 1;
        const int zi = (zl < 7 ? zl : 7) - 1;
        or_put(b, OR_RB_BITS[zi][run], OR_RB_LEN[zi][run]);
        zl -= run;
    }
    return tc;
}

/* code tables for decoders (splice_oracle.c): (bits, length), length 0 =
 * no such code */
int or_ct_code(int tc, int t1, int nC, uint32_t *bits)
{
    if (tc < 0 || tc > 16 || t1 < 0 || t1 > 3 || t1 > tc) return 0;
    if (nC == -1) {
        if (tc > 4) return 0;
        *bits = OR_CTDC_BITS[4 * tc + t1];
        return OR_CTDC_LEN[4 * tc + t1];
    }
    if (nC >= 8) {
        *bits = tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u;
        return 6;
    }
    const int tb = nC < 2 ? 0 : (nC < 4 ? 1 : 2);
    *bits = OR_CT_BITS[tb][4 * tc + t1];
    return OR_CT_LEN[tb][4 * tc + t1];
}
int or_tz_code(int tc, int tz, int maxc, uint32_t *bits)
{
    if (tc < 1 || tc >= maxc || tz < 0 || tz > maxc - tc) return 0;
    if (maxc == 4) {
        *bits = OR_TZDC_BITS[tc - 1][tz];
        return OR_TZDC_LEN[tc - 1][tz];
    }
    *bits = OR_TZ_BITS[tc - 1][tz];
    return OR_TZ_LEN[tc - 1][tz];
}
int or_rb_code(int zl, int run, uint32_t *bits)
{
    if (zl < 1 || run < 0 || run > zl || run > 14) return 0;
    const int zi = (zl < 7 ? zl : 7) - 1;
    *bits = OR_RB_BITS[zi][run];
    return OR_RB_LEN[zi][run];
}

/* coded_block_pattern me(v), Inter column of Table 9-4: cbp -> codeNum */
int or_cbp_code(int cbp)
{
    static const uint8_t golomb_to_inter[48] = {
        0,  16, 1,  2,  4,  8,  32, 3,  5,  10, 12, 15, 47, 7,  11, 13,
        14, 6,  9,  31, 35, 37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46,
        17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41};
    for (int k = 0; k < 48; ++k)
        if (golomb_to_inter[k] == cbp) return k;
    abort();
}

/* ------------------------------------------------------------------------ */
/* one dynamic MB: cbp, qp_delta, residual (7.3.5, 7.3.5.3)                  */
/* ------------------------------------------------------------------------ */
typedef struct {
    int tc[24];        /* TotalCoeff: 16 luma (raster) + Cb AC 4 + Cr AC 4 */
} or_tcctx;

static int or_nc(int nA, int nB)
{
    if (nA >= 0 && nB >= 0) return (nA + nB + 1) >> 1;
    if (nA >= 0) return nA;
    if (nB >= 0) return nB;
    return 0;
}

/* levels: luma per raster block in scan order; cdc[plane][4]; cac[plane][blk][15] */
static void or_mb_residual(or_bits *b, const int luma[16][16], const int cdc[2][4],
                           const int cac[2][4][15], const or_tcctx *left, const or_tcctx *top,
                           or_tcctx *cur)
{
    int cbp_l = 0, any_dc = 0, any_ac = 0;
    for (int r = 0; r < 16; ++r) {
        int nz = 0;
        for (int k = 0; k < 16; ++k) nz |= luma[r][k] != 0;
        const int y = r / 4, x = r % 4, q8 = (y / 2) * 2 + x / 2;
        if (nz) cbp_l |= 1 << q8;
    }
    for (int p = 0; p < 2; ++p) {
        for (int k = 0; k < 4; ++k) any_dc |= cdc[p][k] != 0;
        for (int k = 0; k < 4; ++k)
            for (int i = 0; i < 15; ++i) any_ac |= cac[p][k][i] != 0;
    }
    const int cbp_c = any_ac ? 2 : (any_dc ? 1 : 0);
    const int cbp = cbp_l | (cbp_c << 4);
    or_ue(b, (uint32_t)or_cbp_code(cbp));
    memset(cur, 0, sizeof(*cur));
    if (cbp == 0) return;
    or_se(b, 0);                                          /* mb_qp_delta */
    for (int blk = 0; blk < 16; ++blk) {                  /* luma4x4BlkIdx order */
        const int q8 = blk / 4, q4 = blk % 4;
        const int x = (q8 % 2) * 2 + q4 % 2, y = (q8 / 2) * 2 + q4 / 2, r = 4 * y + x;
        if (!(cbp_l & (1 << q8))) continue;
        const int nA = x > 0 ? cur->tc[r - 1] : (left ? left->tc[r + 3] : -1);
        const int nB = y > 0 ? cur->tc[r - 4] : (top ? top->tc[r + 12] : -1);
        cur->tc[r] = or_cavlc_block(b, luma[r], 16, or_nc(nA, nB));
    }
    if (cbp_c) {
        for (int p = 0; p < 2; ++p) or_cavlc_block(b, cdc[p], 4, -1);
        if (cbp_c == 2)
            for (int p = 0; p < 2; ++p)
                for (int k = 0; k < 4; ++k) {
                    const int x = k % 2, y = k / 2, i = 16 + 4 * p + k;
                    const int nA = x > 0 ? cur->tc[i - 1] : (left ? left->tc[i + 1] : -1);
                    const int nB = y > 0 ? cur->tc[i - 2] : (top ? top->tc[i + 2] : -1);
                    cur->tc[i] = or_cavlc_block(b, cac[p][k], 15, or_nc(nA, nB));
                }
    }
}

size_t or_dyn_mb_levels_bits(uint8_t *dst, size_t cap, const int luma[16][16],
                             const int cdc[2][4], const int cac[2][4][15],
                             const int nc_left[16 + 8], const int nc_top[16 + 8], int avail_l,
                             int avail_t, int *cbp_out, int tc_out[24], size_t *nbits)
{
    or_bits b;
    or_bits_init(&b, dst, cap);
    or_tcctx L, T, C;
    memcpy(L.tc, nc_left, sizeof(L.tc));
    memcpy(T.tc, nc_top, sizeof(T.tc));
    or_mb_residual(&b, luma, cdc, cac, avail_l ? &L : NULL, avail_t ? &T : NULL, &C);
    (void)cbp_out;
    memcpy(tc_out, C.tc, sizeof(C.tc));
    *nbits = b.nbits;
    return or_bytes(&b);
}

/* levels of dynamic MB (mbx, mby) of frame with row (ref, mv); src = rect planes */
static void or_mb_levels(const or_cfg *c, const or_refs *R, const or_dyn_rect *rc,
                         const uint8_t *src, int mbx, int mby, int ref, int mv, int luma[16][16],
                         int cdc[2][4], int cac[2][4][15])
{
    const int lw = 16 * rc->w, cw = 8 * rc->w;
    const uint8_t *sy = src, *su = src + (size_t)lw * 16 * rc->h, *sv = su + (size_t)cw * 8 * rc->h;
    const int lx0 = 16 * (mbx - rc->x0), ly0 = 16 * (mby - rc->y0);
    const int qp = or_dyn_qp(rc), qpc = or_qp_chroma(qp);
    for (int r = 0; r < 16; ++r) {
        const int bx = 4 * (r % 4), by = 4 * (r / 4);
        int res[16], W[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                const int X = 16 * mbx + bx + j, Y = 16 * mby + by + i;
                const int pred = or_ref_sample(c, R, ref, 0, X, Y + mv);
                res[4 * i + j] = sy[(size_t)(ly0 + by + i) * lw + lx0 + bx + j] - pred;
            }
        or_fwd4x4(res, W);
        for (int k = 0; k < 16; ++k) luma[r][k] = or_quant(W[OR_ZZ[k]], qp, OR_ZZ[k], 0);
    }
    const int cx0 = 8 * (mbx - rc->x0), cy0 = 8 * (mby - rc->y0);
    for (int p = 0; p < 2; ++p) {
        const uint8_t *sp = p ? sv : su;
        int dc[4];
        for (int k = 0; k < 4; ++k) {
            const int bx = 4 * (k % 2), by = 4 * (k / 2);
            int res[16], W[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) {
                    const int X = 8 * mbx + bx + j, Y = 8 * mby + by + i;
                    const int q = 4 * mv, o = q >> 3, f = q & 7;
                    const int a = or_ref_sample(c, R, ref, 1 + p, X, Y + o);
                    const int bb = or_ref_sample(c, R, ref, 1 + p, X, Y + o + 1);
                    const int pred = ((8 - f) * a + f * bb + 4) >> 3;
                    res[4 * i + j] = sp[(size_t)(cy0 + by + i) * cw + cx0 + bx + j] - pred;
                }
            or_fwd4x4(res, W);
            dc[k] = W[0];
            for (int i = 1; i < 16; ++i) cac[p][k][i - 1] = or_quant(W[OR_ZZ[i]], qpc, OR_ZZ[i], 0);
        }
        const int f00 = dc[0] + dc[1] + dc[2] + dc[3], f01 = dc[0] - dc[1] + dc[2] - dc[3];
        const int f10 = dc[0] + dc[1] - dc[2] - dc[3], f11 = dc[0] - dc[1] - dc[2] + dc[3];
        cdc[p][0] = or_quant(f00, qpc, 0, 1);
        cdc[p][1] = or_quant(f01, qpc, 0, 1);
        cdc[p][2] = or_quant(f10, qpc, 0, 1);
        cdc[p][3] = or_quant(f11, qpc, 0, 1);
    }
}

/* ------------------------------------------------------------------------ */
/* NAL: the reference's scroll frame (src/h264_writer.c:541-664) with the     */
/* dynamic MBs' residual after their mvd fields                              */
/* ------------------------------------------------------------------------ */
typedef struct {
    int mx, my, ref, avail;
} or_mvi2;

static int or_median3b(int a, int b, int c)   /* src/h264_writer.c:362-367 */
{
    if (a > b) { int t = a; a = b; b = t; }
    if (b > c) b = c;
    if (a > b) a = b;
    return b > a ? b : a;
}

static void or_predict2(int x, int y, int mbw, const or_mvi2 *above, const or_mvi2 *left,
                        int ref, int *px, int *py)         /* :369-432 */
{
    or_mvi2 n[3];
    int avail[3] = {0, 0, 0}, match[3] = {0, 0, 0};
    memset(n, 0, sizeof(n));
    if (x > 0 && left->avail) { n[0] = *left; avail[0] = 1; }
    if (y > 0 && above[x].avail) { n[1] = above[x]; avail[1] = 1; }
    if (y > 0 && x + 1 < mbw && above[x + 1].avail) { n[2] = above[x + 1]; avail[2] = 1; }
    else if (y > 0 && x > 0 && above[x - 1].avail) { n[2] = above[x - 1]; avail[2] = 1; }
    int na = 0, nm = 0;
    for (int k = 0; k < 3; ++k) {
        match[k] = avail[k] && n[k].ref == ref;
        na += avail[k];
        nm += match[k];
    }
    if (na == 0) { *px = 0; *py = 0; }
    else if (na == 1) {
        const int k = avail[0] ? 0 : (avail[1] ? 1 : 2);
        *px = match[k] ? n[k].mx : 0;
        *py = match[k] ? n[k].my : 0;
    } else if (nm == 1) {
        const int k = match[0] ? 0 : (match[1] ? 1 : 2);
        *px = n[k].mx;
        *py = n[k].my;
    } else {
        *px = or_median3b(avail[0] ? n[0].mx : 0, avail[1] ? n[1].mx : 0, avail[2] ? n[2].mx : 0);
        *py = or_median3b(avail[0] ? n[0].my : 0, avail[1] ? n[1].my : 0, avail[2] ? n[2].my : 0);
    }
}

/* test hook (tests/test_dyn_oracle.py): each dynamic MB's residual start
 * bit in the RBSP, its levels and its neighbours' TotalCoeffs, as coded */
static or_dyn_trace_fn or_trace_cb;
void or_dyn_set_trace(or_dyn_trace_fn fn) { or_trace_cb = fn; }

size_t or_scroll_nal_dyn(uint8_t *dst, size_t cap, or_cfg *c, int off, const or_dyn_rect *rc,
                         const uint8_t *src, const or_refs *R)
{
    if (!rc || rc->w <= 0 || rc->h <= 0) return or_scroll_nal(dst, cap, c, off);
    const int mbw = c->w / 16, mbh = c->h / 16;
    size_t rcap = 64 + (size_t)mbw * mbh * 24 + (size_t)rc->w * rc->h * 2048;
    /* per-thread scratch reused across calls (a fresh 1+ MB malloc per frame
     * is an mmap/munmap pair that serialises threads on the mm lock) */
    static __thread uint8_t *tl_rbsp;
    static __thread size_t tl_cap;
    if (tl_cap < rcap) {
        free(tl_rbsp);
        tl_rbsp = (uint8_t *)malloc(rcap);
        tl_cap = rcap;
    }
    uint8_t *rbsp = tl_rbsp;
    or_bits b;
    or_bits_init(&b, rbsp, rcap);
    or_scroll_header_qpd(&b, c, or_dyn_qp(rc) - OR_QP);   /* :549-553; the rect's QP */

    /* regions (:555-588) */
    int a_end = (c->h - off) / 16, wa = -1, woa = 0, wb = -1, wob = 0;
    if (off > OR_MV_LIMIT && c->nwp > 0)
        for (int i = 0; i < c->nwp; ++i) {
            if (!c->wp_valid[i]) continue;
            const int wo = c->wp_off[i];
            if (wo <= off && wo > woa && off - wo <= OR_MV_LIMIT) { wa = i; woa = wo; }
        }
    if (off - c->h < -OR_MV_LIMIT && c->nwp > 0)
        for (int i = 0; i < c->nwp; ++i) {
            if (!c->wp_valid[i]) continue;
            const int wo = c->wp_off[i];
            if (wo > off && off - wo >= -OR_MV_LIMIT) { wb = i; wob = wo; break; }
        }
    const int ra = wa >= 0 ? 2 + wa : 0, mva = wa >= 0 ? off - woa : off;
    const int rb = wb >= 0 ? 2 + wb : 1, mvb = wb >= 0 ? off - wob : off - c->h;
    const int nrefs = 2 + c->nwp;

    or_mvi2 *above = (or_mvi2 *)calloc((size_t)mbw, sizeof(or_mvi2));
    or_mvi2 *cur = (or_mvi2 *)calloc((size_t)mbw, sizeof(or_mvi2));
    or_tcctx *tc_above = (or_tcctx *)calloc((size_t)mbw, sizeof(or_tcctx));
    or_tcctx *tc_cur = (or_tcctx *)calloc((size_t)mbw, sizeof(or_tcctx));
    int luma[16][16], cdc[2][4], cac[2][4][15];           /* per call: thread-safe */
    for (int y = 0; y < mbh; ++y) {
        or_mvi2 left;
        memset(&left, 0, sizeof(left));
        for (int x = 0; x < mbw; ++x) {
            const int ref = y < a_end ? ra : rb;
            const int mvp = y < a_end ? mva : mvb;
            const int my = mvp * 4;
            int px, py;
            or_predict2(x, y, mbw, above, &left, ref, &px, &py);
            const int dyn = x >= rc->x0 && x < rc->x0 + rc->w && y >= rc->y0 && y < rc->y0 + rc->h;
            or_ue(&b, 0);                                  /* mb_skip_run */
            or_ue(&b, 0);                                  /* P_L0_16x16 */
            if (nrefs == 2) or_put(&b, (uint32_t)(1 - (ref & 1)), 1);
            else if (nrefs > 2) or_ue(&b, (uint32_t)ref);
            or_se(&b, 0 - px);
            or_se(&b, my - py);
            if (!dyn) {
                or_ue(&b, 0);                              /* cbp 0 */
                memset(&tc_cur[x], 0, sizeof(or_tcctx));
            } else {
                or_mb_levels(c, R, rc, src, x, y, ref, mvp, luma, cdc, cac);
                if (or_trace_cb)
                    or_trace_cb(x, y, (long long)b.nbits, &luma[0][0], &cdc[0][0], &cac[0][0][0],
                                x > 0 ? tc_cur[x - 1].tc : NULL, y > 0 ? tc_above[x].tc : NULL);
                or_mb_residual(&b, (const int(*)[16])luma, (const int(*)[4])cdc,
                               (const int(*)[4][15])cac, x > 0 ? &tc_cur[x - 1] : NULL,
                               y > 0 ? &tc_above[x] : NULL, &tc_cur[x]);
            }
            cur[x].mx = 0;
            cur[x].my = my;
            cur[x].ref = ref;
            cur[x].avail = 1;
            left = cur[x];
        }
        or_mvi2 *t = above; above = cur; cur = t;
        or_tcctx *u = tc_above; tc_above = tc_cur; tc_cur = u;
    }
    free(above);
    free(cur);
    free(tc_above);
    free(tc_cur);
    or_trailing(&b);
    const size_t n = or_nal(dst, cap, 0, 1, rbsp, or_bytes(&b));
    c->frame_num++;
    return n;
}

/* src/composer.c:255-264 with the dynamic rect in the scroll NAL */
size_t or_compose_dyn(uint8_t *dst, size_t cap, or_cfg *c, int off, int mode,
                      const or_dyn_rect *r, const uint8_t *src, const or_refs *R, int *n_wp_out)
{
    size_t n = 0;
    int nwp = 0;
    if (or_needs_waypoint(c, off)) {
        n += or_waypoint_nal(dst, cap, c, off);
        nwp = 1;
        if (mode == 1) {                      /* experiment: waypoint instead */
            if (n_wp_out) *n_wp_out = nwp;
            return n;
        }
    }
    n += or_scroll_nal_dyn(dst + n, cap - n, c, off, r, src, R);
    if (n_wp_out) *n_wp_out = nwp;
    return n;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline driver (bench.py cpu_baseline leg): BASELINE config 3 on     */
/* nthreads pthreads, streams split evenly; each stream cycles 4 source     */
/* frames of the synthetic generator (generated inside the timed region).   */
/* ------------------------------------------------------------------------ */
#include <pthread.h>
#include <time.h>

typedef struct {
    int s0, s1, nframes, w, h;
    or_dyn_rect r;
    const or_refs *R;
    unsigned long long bytes;
    long long frames;
} or_dyn_job;

static void *or_dyn_worker(void *arg)
{
    or_dyn_job *j = (or_dyn_job *)arg;
    const size_t sb = (size_t)384 * j->r.w * j->r.h;
    const size_t cap = (size_t)(j->w / 16) * (j->h / 16) * 24 + (size_t)j->r.w * j->r.h * 2048 + 4096;
    uint8_t *buf = (uint8_t *)malloc(cap), *src = (uint8_t *)malloc(4 * sb);
    for (int s = j->s0; s < j->s1; ++s) {
        or_cfg c;
        or_cfg_init(&c, j->w, j->h);
        c.frame_num = 2;
        for (int t = 0; t < 4; ++t) or_dyn_source(src + t * sb, s, t, &j->r);
        for (int i = 0; i < j->nframes; ++i) {
            const size_t n = or_compose_dyn(buf, cap, &c, or_synthetic_offset(s, i, j->h), 0, &j->r,
                                            src + (i & 3) * sb, j->R, NULL);
            j->bytes += n;
            j->frames++;
        }
    }
    free(buf);
    free(src);
    return NULL;
}

double or_bench_compose_dyn(int nstreams, int nframes, int w, int h, int rx0, int ry0, int rw,
                            int rh, int nthreads, unsigned long long *bytes_out)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nstreams) nthreads = nstreams;
    const size_t ys = (size_t)w * h, cs = ys / 4;
    uint8_t *pl = (uint8_t *)malloc(2 * (ys + 2 * cs));
    or_pic P[2];
    for (int k = 0; k < 2; ++k) {
        uint8_t *y = pl + k * (ys + 2 * cs);
        or_striped_planes(y, y + ys, y + ys + cs, w, h, k);
        P[k].w = w;
        P[k].h = h;
        P[k].y = y;
        P[k].u = y + ys;
        P[k].v = y + ys + cs;
    }
    or_refs R = {{&P[0], &P[1]}};
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    or_dyn_job *jobs = (or_dyn_job *)calloc((size_t)nthreads, sizeof(or_dyn_job));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].s0 = (int)((long long)nstreams * t / nthreads);
        jobs[t].s1 = (int)((long long)nstreams * (t + 1) / nthreads);
        jobs[t].nframes = nframes;
        jobs[t].w = w;
        jobs[t].h = h;
        jobs[t].r.x0 = rx0;
        jobs[t].r.y0 = ry0;
        jobs[t].r.w = rw;
        jobs[t].r.h = rh;
        jobs[t].R = &R;
    }
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, or_dyn_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    const double dt = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    unsigned long long bytes = 0;
    long long frames = 0;
    for (int t = 0; t < nthreads; ++t) {
        bytes += jobs[t].bytes;
        frames += jobs[t].frames;
    }
    if (bytes_out) *bytes_out = bytes;
    free(th);
    free(jobs);
    free(pl);
    return dt > 0 ? (double)frames / dt : 0.0;
}
