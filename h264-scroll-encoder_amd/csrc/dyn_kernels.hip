/*
 * dyn_kernels.hip -- MI355X (gfx950) kernels of the dynamic-rect residual
 * coder (BASELINE configs 3-5).  A scroll NAL with the rect is no longer a
 * handful of periodic runs: every dynamic MB carries a CAVLC residual, and
 * 60 % of such NALs need emulation prevention.  So these NALs take their own
 * kernels around the plan's sizing pass:
 *
 *   k_plan (state pass)   waypoint state machine, NalDesc per NAL
 *   k_dyn_rows            per NAL: prediction row offsets (waypoint chains)
 *   k_dyn_code[_general]  per 4x4 block: transform, quant, CAVLC body -> records
 *   k_dyn_group           one wave per MB-row group: tokens, cbp, offsets,
 *                         start bit by look-back, bits -> staging slot
 *   k_dyn_ep              emulation-prevention positions + count
 *   k_plan (size pass)    NAL sizes (dynamic: 5 + RBSP + EP), arena offsets
 *   k_emit                every other NAL (dynamic NALs are "external")
 *   k_dyn_emit_gather     staged RBSP -> arena: start code, NAL header, EP
 *                         bytes, 16-byte chunks (k_dyn_emit: > 2048 EP bytes)
 *
 * The bits are those of oracle/dyn_oracle.c (or_scroll_nal_dyn); parity is
 * checked bit-exact by tests/test_gpu_dyn.py.  Roofline: HBM (source pixels
 * + reference pixels in, NAL bytes out), DESIGN.md §5.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "dyn_device.h"
#include "dyn_engine.h"
#include "stage_util.h"

using namespace scroll;
using namespace scroll::dyn;
using namespace scroll::stage;

namespace {

__constant__ Tabs g_tabs = SCROLL_DYN_TABS;
constexpr Tabs k_tabs = SCROLL_DYN_TABS;
__constant__ PTabs g_ptabs = make_ptabs(k_tabs);

/* packed CAVLC tables -> LDS, one 16-byte load per thread */
__device__ inline void load_ptabs(PTabs &dst, int t, int nthr)
{
    constexpr int N = (int)(sizeof(PTabs) / 16);
    static_assert(sizeof(PTabs) % 16 == 0, "PTabs copies as uint4");
    for (int i = t; i < N; i += nthr) reinterpret_cast<uint4 *>(&dst)[i] = reinterpret_cast<const uint4 *>(&g_ptabs)[i];
}


constexpr int HEAD_MAX = 160;           /* bits of one MB head (huge mvd: 2 x 63 + ref) */
constexpr int HDR_MAX = 1024;           /* slice header bits (8 waypoints + MMCO ~ 250) */
constexpr int OBUF = 6400;              /* k_dyn_emit: 127 carry + 5 + 4096 x 1.5 */

constexpr uint32_t DF_OVER = 1u, DF_GENERAL = 2u;   /* DynFrame.err bits */

__device__ inline uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }

/* NalCtx of scroll NAL d of stream S with the waypoint table (wo, wl, wv) */
__device__ inline NalCtx nal_ctx(const DevStream *S, const NalDesc &d, const int32_t *wo, const int32_t *wl,
                                 const int32_t *wv)
{
    NalCtx c;
    c.w = S->w;
    c.h = S->h;
    c.log2_mfn = S->log2_mfn;
    c.poc_type = S->poc_type;
    c.log2_poc = S->log2_poc;
    c.deblock = S->deblock;
    c.kind = d.kind;
    c.off = d.off;
    c.frame_num = d.frame_num;
    c.nwp = d.nwp;
    c.wp_off = wo;
    c.wp_lt = wl;
    c.wp_valid = wv;
    return c;
}

/* ====================================================================== */
/* The dynamic-rect coder is four kernels:                 */
/*                                                                         */
/*   k_dyn_rows   per NAL: the waypoint chain of every prediction row of   */
/*                the rect, resolved once to byte offsets in picture A / B */
/*   k_dyn_code   per 4x4 block, all blocks of all NALs at once: residual, */
/*                transform, quant and the nC-independent CAVLC body      */
/*                (signs, levels, total_zeros, run_before) -> records;     */
/*                chroma DC whole (nC = -1)                                */
/*   k_dyn_group  per MB-row group of a NAL: coeff_token from the          */
/*                neighbours' TotalCoeff, cbp, MB heads, offsets; start    */
/*                bit by a look-back over the groups before; bits -> LDS   */
/*                -> staging words                                         */
/*   k_dyn_ep     per NAL: shared boundary words merged, emulation-        */
/*                prevention positions and count                           */
/*                                                                         */
/* Records of dynamic MB q (rect raster order) of NAL n, piece pc, at       */
/*   rec_of(q, pc): k_dyn_code's task order -- luma 16 q + pc, chroma AC    */
/*   16 nd + 8 q + pc - 18, chroma DC 24 nd + 2 q + pc - 16 (nd = w h):     */
/*   0..15 luma 4x4 (raster), 16 / 17 Cb / Cr DC, 18 + 4p + b chroma AC    */
/*   (plane p, raster b): meta[n][q][pc] (u16) = body bits | TotalCoeff << 8 | */
/*   TrailingOnes << 13 | ovf << 15, body[n][q][pc] = the body right-      */
/*   aligned in 128 bits (x = bits 0..31 .. w = bits 96..127); DC pieces   */
/*   hold the whole block.  ovf: more than 128 bits -- body holds the      */
/*   levels instead (int8 scan order; DC: int16) and k_dyn_group re-codes. */
/* ====================================================================== */
constexpr int NPC = DYN_PIECES;         /* pieces per dynamic MB */

/* a record body is two planes of 8 bytes: bits 0..63 (always) and 64..127
 * (only for bodies over 64 bits and for level records) */
__device__ inline void put_body(uint2 *BL, uint2 *BH, size_t i, uint4 v, bool hi)
{
    BL[i] = make_uint2(v.x, v.y);
    if (hi) BH[i] = make_uint2(v.z, v.w);
}

__device__ inline uint4 get_body(const uint2 *BL, const uint2 *BH, size_t i, bool hi)
{
    const uint2 a = BL[i], b = hi ? BH[i] : make_uint2(0u, 0u);
    return make_uint4(a.x, a.y, b.x, b.y);
}

__device__ inline int rec_of(int q, int pc, int ndt)
{
    return pc < 16 ? 16 * q + pc : (pc < 18 ? 24 * ndt + 2 * q + (pc - 16) : 16 * ndt + 8 * q + (pc - 18));
}
constexpr uint32_t M_OVF = 1u << 15;
constexpr uint32_t ROW_GEN = 1u << 31, ROW_OFF = 0x0fffffffu;

/* ---------------------------------------------------------------------- */
/* k_dyn_rows                                                              */
/* ---------------------------------------------------------------------- */
/* rows[n][i], i < 32 h (h = rect MB rows):
 *   i < 16 h        luma row 16 y0 + i: byte offset of its prediction row in
 *                   the stream's reference pair (picture * pic + row * w)
 *   16 h .. 24 h    chroma row 8 y0 + i': the upper bilinear row
 *                   (picture * pic + ysz + row * w / 2), the 1/8-pel
 *                   fraction in bits 28..30, ROW_GEN if the waypoint chain
 *                   has a half-pel step (the general path)
 *   24 h .. 32 h    the lower bilinear row (used when the fraction != 0)
 * Sets DynFrame.err = DF_GENERAL when some row of the NAL needs the general
 * path (never for waypoints the composer creates), else 0. */
__global__ __launch_bounds__(256) void k_dyn_rows(const DevStream *__restrict__ st,
                                                  const NalDesc *__restrict__ nal, int ld_nal,
                                                  const PlanPending *__restrict__ pend,
                                                  DynFrame *__restrict__ dfr, int ld_fr, DynGeom g,
                                                  uint32_t *__restrict__ rows)
{
    __shared__ int32_t wo[8], wl[8], wv[8];
    __shared__ int32_t gen;
    const int s = blockIdx.y, f = blockIdx.x, t = threadIdx.x;
    DynFrame *DF = dfr + (size_t)s * ld_fr + f;
    const int j = DF->nal;
    if (j < 0) return;
    if (t < 8) {
        wo[t] = pend[s].wo[t];
        wl[t] = pend[s].wl[t];
        wv[t] = pend[s].wv[t];
    }
    if (t == 0) gen = 0;
    __syncthreads();
    const DevStream *S = st + s;
    const NalDesc d = nal[(size_t)s * ld_nal + j];
    const NalCtx c = nal_ctx(S, d, wo, wl, wv);
    const Regions rg = regions(c);
    const int w = c.w, h = c.h, a_end = (h - c.off) / 16;
    const uint32_t ysz = (uint32_t)w * (uint32_t)h, pic = ysz + ysz / 2;
    const WpTab T{wo, wv, h};
    uint32_t *rw = rows + ((size_t)s * ld_fr + f) * (size_t)(32 * g.h);
    bool my_gen = false;
    for (int i = t; i < 32 * g.h; i += 256) {
        uint32_t e;
        if (i < 16 * g.h) {
            const int Y = 16 * g.y0 + i, row = Y >> 4;
            const bool cA = row < a_end;
            int yo;
            const int b = luma_row(T, cA ? rg.ra : rg.rb, Y + (cA ? rg.mva : rg.mvb), yo);
            e = (uint32_t)b * pic + (uint32_t)yo * (uint32_t)w;
        } else {
            const int i2 = i - 16 * g.h, bot = i2 >= 8 * g.h;
            const int Y = 8 * g.y0 + (bot ? i2 - 8 * g.h : i2), row = Y >> 3;
            const bool cA = row < a_end;
            const int q = 4 * (cA ? rg.mva : rg.mvb), o = q >> 3, fr = q & 7;
            int yo;
            const int b = chroma_row(T, cA ? rg.ra : rg.rb, Y + o + bot, yo);
            if (b < 0) {
                e = ROW_GEN;
                if (!bot || fr) my_gen = true;
            } else {
                e = ((uint32_t)b * pic + ysz + (uint32_t)yo * (uint32_t)(w / 2)) | (uint32_t)fr << 28;
            }
        }
        rw[i] = e;
    }
    if (my_gen) gen = 1;
    __syncthreads();
    if (t == 0) DF->err = gen ? DF_GENERAL : 0u;
}

/* ---------------------------------------------------------------------- */
/* k_dyn_code                                                              */
/* ---------------------------------------------------------------------- */
/* grid (ceil(24 nd / 256), frames, streams); task = one 4x4 block of a NAL:
 * [0, 16 nd) luma, MB-major (16 lanes = one MB: 4 MBs per wave read 64
 * contiguous source bytes per row), then [16 nd, 24 nd) chroma AC, MB-major,
 * Cb quad then Cr quad (a quad's lanes exchange their DC coefficients).
 * Phase 1: residual -> transform -> quant -> levels (LDS); phase 2, after
 * one barrier: blocks with <= 3 non-zero levels are coded first, so the
 * CAVLC loop of most waves iterates <= 3 times. */
#ifndef SCROLL_CODE_T
#define SCROLL_CODE_T 256
#endif
constexpr int CODE_T = SCROLL_CODE_T, CODE_NW = CODE_T / 64;
/* sort classes: TotalCoeff 0 .. SORT_KEYS - 2 each, the rest together (the
 * tail is rare; fewer classes, fewer ballots) */
#ifndef SCROLL_SORT_KEYS
#define SCROLL_SORT_KEYS 9
#endif
constexpr int SORT_KEYS = SCROLL_SORT_KEYS;
static_assert(SORT_KEYS >= 2 && SORT_KEYS <= 17, "TotalCoeff classes");

template <bool GENERAL>
__device__ inline void code_frame(const DevStream *__restrict__ st,
                                                     const DynFrame *__restrict__ dfr, int ld_fr,
                                                     const PlanPending *__restrict__ pend,
                                                     const NalDesc *__restrict__ nal, int ld_nal,
                                                     DynGeom g, const uint32_t *__restrict__ rows,
                                                     const uint8_t *__restrict__ src,
                                                     const uint8_t *__restrict__ refs,
                                                     uint16_t *__restrict__ meta, uint2 *__restrict__ blo,
                                                     uint2 *__restrict__ bhi, int s, int f, int bx)
{
    __shared__ uint4 lv[CODE_T];
    __shared__ uint16_t wc[CODE_NW][SORT_KEYS];    /* per wave: blocks per TotalCoeff class */
    __shared__ uint16_t order[CODE_T];
    __shared__ PTabs ptabs;
    __shared__ int32_t wo[8], wv[8];
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const DynFrame df = dfr[(size_t)s * ld_fr + f];
    if (df.nal < 0) return;
    if (GENERAL != ((df.err & DF_GENERAL) != 0)) return;
    load_ptabs(ptabs, t, CODE_T);
    if (GENERAL && t < 8) {
        wo[t] = pend[s].wo[t];
        wv[t] = pend[s].wv[t];
    }
    /* the general chroma path reads wo / wv before the sort; otherwise the
     * sort's first barrier publishes ptabs, and the pixel loads need not
     * wait for the table copy */
    if (GENERAL) __syncthreads();

    const int ndt = g.w * g.h, ntask = 24 * ndt;
    const int task = bx * CODE_T + t;
    const size_t nb = (size_t)s * ld_fr + f;
    const uint32_t *rw = rows + nb * (size_t)(32 * g.h);
    const int w = st[s].w, h = st[s].h;
    const uint32_t ysz = (uint32_t)w * (uint32_t)h, csz = ysz / 4;
    const uint8_t *rb = refs + (size_t)s * g.ref_ld;
    const uint8_t *fs = src + (size_t)s * g.src_ld + (size_t)f * g.src_fr;
    const int lstride = 16 * g.w, cstride = 8 * g.w;
    const uint8_t *fcb = fs + (size_t)256 * ndt, *fcr = fcb + (size_t)64 * ndt;
    const uint32_t m_rw = magic32((uint32_t)g.w);
    uint16_t *M = meta + nb * (size_t)(NPC * ndt);
    uint2 *BL = blo + nb * (size_t)(NPC * ndt), *BH = bhi + nb * (size_t)(NPC * ndt);

    const bool luma = task < 16 * ndt;
    const bool act = task < ntask;
    int k, r, p = 0;                    /* MB, raster block, chroma plane */
    if (luma) {
        k = task >> 4;
        r = task & 15;
    } else {
        const int jj = task - 16 * ndt;
        k = jj >> 3;
        p = (jj >> 2) & 1;
        r = jj & 3;
    }
    const int ry = (int)div_m((uint32_t)k, m_rw), cx = k - ry * g.w;
    const int col = g.x0 + cx;
    uint32_t pk[4] = {0, 0, 0, 0};
    int n = 0, w0 = 0;
    if (act && luma) {
        const int bx = r & 3, by = r >> 2;
        const uint8_t *sp = fs + (size_t)(16 * ry + 4 * by) * lstride + 16 * cx + 4 * bx;
        const uint8_t *pp = rb + 16 * col + 4 * bx;
        const uint32_t *re = rw + 16 * ry + 4 * by;
        uint32_t sv[4], pv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#ifdef SCROLL_ABL_NOLOAD
            sv[i] = 0x80808080u + (uint32_t)(task * 7 + i * 3) * 0x01010101u;
            pv[i] = 0x80808080u;
#else
            sv[i] = ld32(sp + (size_t)i * lstride);
            pv[i] = ld32(pp + re[i]);
#endif
        }
        int res[16], W[16];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int x = 0; x < 4; ++x)
                res[4 * i + x] = (int)((sv[i] >> (8 * x)) & 255u) - (int)((pv[i] >> (8 * x)) & 255u);
        fwd4x4(res, W);
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) {
            const int v = quant(W[ZZ[k2]], ZZ[k2]);          /* |v| <= 78: int8 */
            pk[k2 >> 2] |= ((uint32_t)v & 255u) << (8 * (k2 & 3));
            n += v != 0;
        }
    } else if (act) {
        const int bx = r & 1, by = r >> 1;
        const uint8_t *sp = (p ? fcr : fcb) + (size_t)(8 * ry + 4 * by) * cstride + 8 * cx + 4 * bx;
        const int X = 8 * col + 4 * bx;
        const uint8_t *cp = rb + (size_t)p * csz + X;
        const uint32_t *re = rw + 16 * g.h + 8 * ry + 4 * by;
        int res[16], W[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#ifdef SCROLL_ABL_NOLOAD
            const uint32_t sv = 0x80808080u + (uint32_t)(task * 5 + i) * 0x01010101u;
            const uint32_t ea = 0;
#else
            const uint32_t sv = ld32(sp + (size_t)i * cstride);
            const uint32_t ea = re[i];
#endif
            int pred[4];
            if (!GENERAL || !(ea & ROW_GEN)) {
                const uint32_t fr = (ea >> 28) & 7u;
#ifdef SCROLL_ABL_NOLOAD
                const uint32_t av = 0x80808080u, bv = 0u;
#else
                const uint32_t av = ld32(cp + (ea & ROW_OFF));
                const uint32_t bv = fr ? ld32(cp + (re[8 * g.h + i] & ROW_OFF)) : 0u;
#endif
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    const int a = (int)((av >> (8 * x)) & 255u), b = (int)((bv >> (8 * x)) & 255u);
                    pred[x] = ((8 - (int)fr) * a + (int)fr * b + 4) >> 3;
                }
            } else {
                if constexpr (GENERAL) {        /* half-pel waypoint step: any depth */
                    const NalDesc d = nal[(size_t)s * ld_nal + df.nal];
                    const int off = d.off, a_end = (h - off) / 16;
                    const int row = g.y0 + ry;
                    int32_t wl0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    const NalCtx c = nal_ctx(st + s, d, wo, wl0, wv);
                    const Regions rg = regions(c);
                    const bool cA = row < a_end;
                    const int ref = cA ? rg.ra : rg.rb, q = 4 * (cA ? rg.mva : rg.mvb);
                    const int o = q >> 3, fr = q & 7;
                    const WpTab T{wo, wv, h};
                    RefPics P;
                    P.w = w;
                    P.h = h;
                    const size_t pic = (size_t)ysz + 2 * csz;
                    for (int i2 = 0; i2 < 2; ++i2) {
                        P.pl[i2][0] = rb + i2 * pic;
                        P.pl[i2][1] = P.pl[i2][0] + ysz;
                        P.pl[i2][2] = P.pl[i2][1] + csz;
                    }
                    const int ya = 8 * row + 4 * by + i + o;
                    for (int x = 0; x < 4; ++x) {
                        const int a = chroma_px_any<9>(T, P, ref, 1 + p, X + x, ya);
                        const int b = fr ? chroma_px_any<9>(T, P, ref, 1 + p, X + x, ya + 1) : 0;
                        pred[x] = ((8 - fr) * a + fr * b + 4) >> 3;
                    }
                }
            }
#pragma unroll
            for (int x = 0; x < 4; ++x) res[4 * i + x] = (int)((sv >> (8 * x)) & 255u) - pred[x];
        }
        fwd4x4(res, W);
        w0 = W[0];
#pragma unroll
        for (int k2 = 1; k2 < 16; ++k2) {
            const int v = quant(W[ZZ[k2]], ZZ[k2]);
            pk[(k2 - 1) >> 2] |= ((uint32_t)v & 255u) << (8 * ((k2 - 1) & 3));
            n += v != 0;
        }
    }
    /* chroma DC: the quad's four DC coefficients -> 2x2 Hadamard, quant; the
     * whole CAVLC block (nC = -1) is coded by the quad's first lane after the
     * sort's first barrier, which publishes the LDS tables (ptabs) */
    int dq[4] = {0, 0, 0, 0};
    const bool dc_lane = act && !luma && r == 0;
    {
        const int qb = lane & ~3;
        const int d0 = __shfl(w0, qb, 64), d1 = __shfl(w0, qb + 1, 64);
        const int d2 = __shfl(w0, qb + 2, 64), d3 = __shfl(w0, qb + 3, 64);
        if (dc_lane) {
            dq[0] = quant_dc(d0 + d1 + d2 + d3);
            dq[1] = quant_dc(d0 - d1 + d2 - d3);
            dq[2] = quant_dc(d0 + d1 - d2 - d3);
            dq[3] = quant_dc(d0 - d1 - d2 + d3);
        }
    }
    /* encode order: by TotalCoeff, largest first (a counting sort over the
     * workgroup), so each wave's CAVLC loop runs about its own blocks' count */
    lv[t] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    {
        const int key = SORT_KEYS - 1 - min(n, SORT_KEYS - 1);   /* inactive tasks: n = 0 */
        uint32_t below = 0;
#pragma unroll
        for (int k = 0; k < SORT_KEYS; ++k) {
            const uint64_t m = __ballot(key == k);
            if (lane == 0) wc[wave][k] = (uint16_t)__popcll(m);
            if (key == k)
                below = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        }
        __syncthreads();                                /* also publishes ptabs */
        if (dc_lane) {
            CapSink cap{0, 0, 0};
            const int tc = cavlc_dc4(cap, ptabs, dq);
            const size_t idx = (size_t)24 * ndt + 2 * k + p;    /* rec_of(k, 16 + p) */
            if (cap.n <= 128) {
                M[idx] = (uint16_t)(cap.n | (uint32_t)tc << 8);
                if (cap.n)
                    put_body(BL, BH, idx, make_uint4((uint32_t)cap.lo, (uint32_t)(cap.lo >> 32), (uint32_t)cap.hi,
                                                     (uint32_t)(cap.hi >> 32)), cap.n > 64);
            } else {
                M[idx] = (uint16_t)((uint32_t)tc << 8 | M_OVF);
                put_body(BL, BH, idx, make_uint4(((uint32_t)dq[0] & 0xffffu) | (uint32_t)dq[1] << 16,
                                                 ((uint32_t)dq[2] & 0xffffu) | (uint32_t)dq[3] << 16, 0u, 0u), false);
            }
        }
        if (t < SORT_KEYS) {                            /* key k = t: wave prefixes, key offsets */
            uint32_t tot = 0;
#pragma unroll
            for (int w2 = 0; w2 < CODE_NW; ++w2) tot += wc[w2][t];
            uint32_t kb = tot;
#pragma unroll
            for (int d = 1; d < 32; d <<= 1) {
                const uint32_t o = __shfl_up(kb, d, 64);
                if (lane >= d) kb += o;
            }
            uint32_t run = kb - tot;
#pragma unroll
            for (int w2 = 0; w2 < CODE_NW; ++w2) {
                const uint32_t c = wc[w2][t];
                wc[w2][t] = (uint16_t)run;
                run += c;
            }
        }
        __syncthreads();
        order[wc[wave][key] + below] = (uint16_t)t;
    }
    __syncthreads();
    const int u = order[t];
    const int tk = bx * CODE_T + u;
    const uint4 v4 = lv[u];
    const uint32_t q[4] = {v4.x, v4.y, v4.z, v4.w};
    const bool ul = tk < 16 * ndt;
    CapSink cap{0, 0, 0};
    int t1 = 0;
    bool ok = true;
    int tc = 0;
    if (tk < ntask) {
#ifdef SCROLL_ABL_NOCAVLC
        tc = __builtin_popcount(q[0] | q[1] | q[2] | q[3]) & 15;
#else
        tc = cavlc_body(cap, ptabs, q, ul ? 16 : 15, t1, ok);
#endif
    }
    /* each lane stores its own block's record (task order, so a workgroup's
     * records are one contiguous range; un-sorting through LDS first was
     * measured 3 % slower: light waves waited at its barrier for the heavy one) */
    if (tk < ntask) {
        const uint16_t mm = ok ? (uint16_t)(cap.n | (uint32_t)tc << 8 | (uint32_t)t1 << 13)
                               : (uint16_t)((uint32_t)tc << 8 | (uint32_t)t1 << 13 | M_OVF);
        M[tk] = mm;
        if ((mm & 255u) || (mm & M_OVF))
            put_body(BL, BH, tk,
                     ok ? make_uint4((uint32_t)cap.lo, (uint32_t)(cap.lo >> 32), (uint32_t)cap.hi,
                                     (uint32_t)(cap.hi >> 32))
                        : v4,
                     (mm & 255u) > 64u || (mm & M_OVF));
    }
}

/* the frames without a half-pel waypoint chain: grid (chunks, frames, streams) */
__global__ __launch_bounds__(CODE_T) void k_dyn_code(const DevStream *__restrict__ st,
                                                     const DynFrame *__restrict__ dfr, int ld_fr,
                                                     const PlanPending *__restrict__ pend,
                                                     const NalDesc *__restrict__ nal, int ld_nal,
                                                     DynGeom g, const uint32_t *__restrict__ rows,
                                                     const uint8_t *__restrict__ src,
                                                     const uint8_t *__restrict__ refs,
                                                     uint16_t *__restrict__ meta, uint2 *__restrict__ blo,
                                                     uint2 *__restrict__ bhi)
{
    code_frame<false>(st, dfr, ld_fr, pend, nal, ld_nal, g, rows, src, refs, meta, blo, bhi, blockIdx.z,
                      blockIdx.y, blockIdx.x);
}

/* the others (general chroma path, never for the composer's own waypoints):
 * grid (chunks, CODE_GEN_Y), each workgroup finds flagged (stream, frame)
 * pairs 64 at a time -- a launch over every frame would cost more in empty
 * workgroups than the frames it serves */
constexpr int CODE_GEN_Y = 64;
__global__ __launch_bounds__(CODE_T) void k_dyn_code_general(const DevStream *__restrict__ st,
                                                             const DynFrame *__restrict__ dfr, int ld_fr,
                                                             const PlanPending *__restrict__ pend,
                                                             const NalDesc *__restrict__ nal, int ld_nal,
                                                             DynGeom g, const uint32_t *__restrict__ rows,
                                                             const uint8_t *__restrict__ src,
                                                             const uint8_t *__restrict__ refs,
                                                             uint16_t *__restrict__ meta,
                                                             uint2 *__restrict__ blo, uint2 *__restrict__ bhi, int nframes,
                                                             int nstreams)
{
    const int lane = threadIdx.x & 63, np = nstreams * nframes;
    for (int p0 = (int)blockIdx.y * 64; p0 < np; p0 += (int)gridDim.y * 64) {
        bool gen = false;
        const int p = p0 + lane;
        if (p < np) {
            const int s = p / nframes, f = p - s * nframes;
            const DynFrame df = dfr[(size_t)s * ld_fr + f];
            gen = df.nal >= 0 && (df.err & DF_GENERAL);
        }
        uint64_t m = __ballot(gen);                     /* the same in every wave */
        while (m) {
            const int q = p0 + __builtin_ctzll(m);
            m &= m - 1;
            const int s = q / nframes, f = q - s * nframes;
            code_frame<true>(st, dfr, ld_fr, pend, nal, ld_nal, g, rows, src, refs, meta, blo, bhi, s, f,
                             blockIdx.x);
            __syncthreads();
        }
    }
}

struct LdsOrWin {
    uint32_t *b;
    uint32_t lo, n;
    __device__ inline void operator()(uint32_t i, uint32_t v) const
    {
        const uint32_t k = i - lo;
        if (k < n) atomicOr(&b[k], v);
    }
};
typedef OrSink<LdsOrWin> WSink;

/* ---------------------------------------------------------------------- */
/* k_dyn_group / k_dyn_ep: records -> staged RBSP                         */
/* ---------------------------------------------------------------------- */
/* A NAL's bits are: slice header, then per MB row the MB heads (one of 12
 * codeword classes) and, for dynamic MBs, coded_block_pattern,
 * mb_qp_delta and the present pieces (coeff_token from the neighbours'
 * TotalCoeff + the body k_dyn_code left in the records), then the stop bit. */

__device__ inline int tc_of(uint32_t m) { return (int)((m >> 8) & 31u); }

/* the head codeword classes of a NAL (3 row types x first / middle / last) */
struct HeadCtx {
    Regions rg;
    int a_end, mbw, nrefs;
    __device__ inline int sel(int row, int col) const
    {
        const bool curA = row < a_end, abvA = (row - 1) < a_end;
        return 3 * (row == 0 ? 0 : (curA ? 1 : (abvA ? 2 : 3))) + (col == 0 ? 0 : (col == mbw - 1 ? 2 : 1));
    }
    /* head of class cls (h264_writer.c:434-453 after the row-uniform predictor) */
    template <class S>
    __device__ inline void put_class(S &sk, int cls) const
    {
        const int ty = cls / 3, pos = cls - 3 * ty;
        const int x = pos == 0 ? 0 : (pos == 1 ? min(1, mbw - 1) : mbw - 1);
        const bool cur = ty == 0 ? 0 < a_end : ty == 1;
        const bool abv = ty == 1 || ty == 2;
        const int ref = cur ? rg.ra : rg.rb, mv4 = 4 * (cur ? rg.mva : rg.mvb);
        const int aref = abv ? rg.ra : rg.rb, amv4 = 4 * (abv ? rg.mva : rg.mvb);
        int px, py;
        predict(x, ty == 0 ? 0 : 1, mbw, ref, mv4, aref, amv4, px, py);
        put_mb_head(sk, ref, 0 - px, mv4 - py, nrefs);
    }
    /* the same for MB (row, col) directly (heads over 128 bits) */
    template <class S>
    __device__ inline void put_slow(S &sk, int row, int col) const
    {
        const bool curA = row < a_end, abvA = (row - 1) < a_end;
        const int ref = curA ? rg.ra : rg.rb, mv4 = 4 * (curA ? rg.mva : rg.mvb);
        const int aref = abvA ? rg.ra : rg.rb, amv4 = 4 * (abvA ? rg.mva : rg.mvb);
        int px, py;
        predict(col, row, mbw, ref, mv4, aref, amv4, px, py);
        put_mb_head(sk, ref, 0 - px, mv4 - py, nrefs);
    }
};

__device__ inline HeadCtx head_ctx(const NalCtx &c)
{
    HeadCtx H;
    H.rg = regions(c);
    H.a_end = (c.h - c.off) / 16;
    H.mbw = c.w / 16;
    H.nrefs = 2 + c.nwp;
    return H;
}

/* bits of the non-dynamic MBs of one row: (head + coded_block_pattern ue(0))
 * per MB, by class counts (first / middle / last column) */
__device__ inline uint32_t row_static_bits(const HeadCtx &H, const uint32_t *hlen, int row, const Rect &R)
{
    const int mbw = H.mbw;
    const bool in = row >= R.y0 && row < R.y0 + R.h;
    auto isdyn = [&](int col) { return in && col >= R.x0 && col < R.x0 + R.w; };
    const int base = H.sel(row, 0) - 0;                     /* class of column 0 */
    uint32_t bits = isdyn(0) ? 0u : hlen[base] + 1u;
    if (mbw >= 2) {
        if (!isdyn(mbw - 1)) bits += hlen[base + 2] + 1u;
        int nmid = mbw - 2;
        if (in) nmid -= max(0, min(R.x0 + R.w, mbw - 1) - max(R.x0, 1));
        bits += (uint32_t)nmid * (hlen[base + 1] + 1u);
    }
    return bits;
}

/* Row groups of a NAL: g = 0 the rows above the rect (with the slice
 * header), g = 1 .. h the rect rows, g = h + 1 the rows below (with the stop
 * bit).  One workgroup per group measures its bits, takes its start bit from
 * the groups before it by a decoupled look-back over per-group status words,
 * and writes the staging words of its bits; a word shared with the group
 * before / after is completed through the tail hand-off below. */

/* status word: epoch (24) | flag (2: 1 aggregate, 2 inclusive prefix) | bits (38) */
__device__ inline uint64_t lb_pack(uint32_t epoch, uint32_t flag, uint64_t v)
{
    return (uint64_t)(epoch & 0xffffffu) << 40 | (uint64_t)flag << 38 | v;
}

__device__ inline void lb_store(unsigned long long *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* exclusive prefix of group g, by the 64 lanes of one wave: publishes the
 * aggregate, then reads the status of the 64 groups before at once, sums
 * back to the nearest inclusive prefix (retrying while a group in that span
 * has not published), publishes its own inclusive prefix */
__device__ inline uint64_t lb_lookback(unsigned long long *sa, int g, uint32_t epoch, uint64_t bits, int lane)
{
    if (g == 0) {
        if (lane == 0) lb_store(sa, lb_pack(epoch, 2, bits));
        return 0;
    }
    if (lane == 0) lb_store(sa + g, lb_pack(epoch, 1, bits));
    uint64_t pre = 0;
    for (int j = g - 1;;) {
        const int jj = j - lane;
        uint64_t v = 0;
        uint32_t fl = 2;                                    /* before group 0: empty, inclusive */
        if (jj >= 0) {
            v = __hip_atomic_load(sa + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fl = (uint32_t)(v >> 40) == (epoch & 0xffffffu) ? (uint32_t)(v >> 38) & 3u : 0u;
            v &= (1ull << 38) - 1;
        }
        const uint64_t incl = __ballot(fl == 2), none = __ballot(fl == 0);
        const int fi = incl ? __builtin_ctzll(incl) : 63;   /* nearest inclusive in the window */
        const uint64_t span = fi == 63 ? ~0ull : (2ull << fi) - 1;
        if (none & span) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        const uint64_t c = lane <= fi ? v : 0;
        uint32_t lo = (uint32_t)(c & 0xffffffu), hi = (uint32_t)(c >> 24);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            lo += __shfl_xor(lo, d, 64);
            hi += __shfl_xor(hi, d, 64);
        }
        pre += ((uint64_t)hi << 24) + lo;
        if (incl) break;
        j -= 64;
    }
    if (lane == 0) lb_store(sa + g, lb_pack(epoch, 2, pre + bits));
    return pre;
}

/* a > 128-bit block from its levels (rare): measure / write */
__device__ __attribute__((noinline)) uint32_t ovf_bits(const PTabs &PT, const Tabs &TB, uint4 bd, int pc, int nC)
{
    CountSink cn{0};
    if (nC == -1) {
        const int dq[4] = {(int)(int16_t)(bd.x & 0xffffu), (int)(int16_t)(bd.x >> 16),
                           (int)(int16_t)(bd.y & 0xffffu), (int)(int16_t)(bd.y >> 16)};
        cavlc_dc4(cn, PT, dq);
    } else {
        const int8_t *lvp = reinterpret_cast<const int8_t *>(&bd);
        cavlc_block(cn, TB, lvp, pc < 16 ? 16 : 15, nC);
    }
    return cn.n;
}

/* the sink lives in the callee: a sink passed by reference would be kept in
 * scratch memory by the caller on its every put */
__device__ __attribute__((noinline)) void ovf_put(uint32_t *buf, uint32_t lo, uint32_t n, uint32_t pos,
                                                  const PTabs &PT, const Tabs &TB, uint4 bd, int pc, int nC)
{
    WSink sk{LdsOrWin{buf, lo, n}, 0, 0, 0};
    sk.start(pos);
    if (nC == -1) {
        const int dq[4] = {(int)(int16_t)(bd.x & 0xffffu), (int)(int16_t)(bd.x >> 16),
                           (int)(int16_t)(bd.y & 0xffffu), (int)(int16_t)(bd.y >> 16)};
        cavlc_dc4(sk, PT, dq);
    } else {
        const int8_t *lvp = reinterpret_cast<const int8_t *>(&bd);
        cavlc_block(sk, TB, lvp, pc < 16 ? 16 : 15, nC);
    }
    sk.finish();
}

/* k_dyn_group is ONE wave per row group: the group's work is a chain of
 * short dependent phases (records -> tokens -> MB layout -> scans ->
 * look-back -> bits -> words), so throughput comes from many groups in
 * flight per CU rather than from wide workgroups; LDS is sized to the rect
 * (dynamic shared memory, group_lds_bytes) */
constexpr int GW = 64;
#ifndef SCROLL_GBUF_WORDS
#define SCROLL_GBUF_WORDS 256
#endif
constexpr int GBUF_WORDS = SCROLL_GBUF_WORDS;          /* 8 Kbit per pass (a config-3 row: ~18 Kbit in 3 passes);
                                           each pass walks only the MBs / rows it covers */

struct GroupFixed {
    uint32_t buf[GBUF_WORDS];
    uint64_t hhi[12], hlo[12];
    uint32_t hlen[12];
    int32_t head_over;
    int32_t wo[8], wl[8], wv[8];
    uint16_t ct[3][68];                 /* coeff_token tables (nC 0-1, 2-3, 4-7), PTabs layout */
};

/* dynamic LDS: moff [lines + 1] u32, mbits [w] u32, mt, lo, off16 [NPC w]
 * u16, ma [8 w] u16, cbp / code [w] u8 */
__host__ __device__ inline size_t group_lds_bytes(int w, int lines)
{
    return (size_t)4 * (lines + 1 + w) + (size_t)2 * (3 * NPC * w + 8 * w) + (size_t)2 * w + 16;
}

/* lo[i]: piece length (11) | nC + 1 (5) << 11 */
constexpr uint32_t LO_LEN = 0x7ffu;

/* coeff_token of a piece with meta mv at context nC >= 0 (Table 9-5) */
__device__ inline void piece_token(const uint16_t (*ct)[68], uint32_t mv, int nC, uint32_t &tv, uint32_t &tl)
{
    const int tc = tc_of(mv), t1 = (int)((mv >> 13) & 3u);
    if (nC >= 8) {
        tv = tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u;
        tl = 6;
    } else {
        const uint32_t e = ct[nC < 2 ? 0 : (nC < 4 ? 1 : 2)][4 * tc + t1];
        tv = e & 255u;
        tl = e >> 8;
    }
}

/* k_dyn_group's workgroup is ONE wave: its LDS handoffs need ordering, not a
 * workgroup barrier (whose release fence would also wait for every global
 * store of the wave to complete) */
__device__ inline void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* grid (g.ngroups, frames, streams), GW threads.  The kernel is latency-bound
 * (one wave per group, look-back waits): SCROLL_GROUP_WAVES caps the VGPRs so
 * that many waves fit per SIMD */
#ifndef SCROLL_GROUP_WAVES
#define SCROLL_GROUP_WAVES 6
#endif
__global__ __launch_bounds__(GW) __attribute__((amdgpu_waves_per_eu(SCROLL_GROUP_WAVES)))
void k_dyn_group(DevStream *__restrict__ st,
                                                  const NalDesc *__restrict__ nal, int ld_nal,
                                                  const PlanPending *__restrict__ pend,
                                                  DynFrame *__restrict__ dfr, int ld_fr, DynGeom g,
                                                  const uint16_t *__restrict__ meta,
                                                  const uint2 *__restrict__ blo, const uint2 *__restrict__ bhi,
                                                  unsigned long long *__restrict__ status,
                                                  unsigned long long *__restrict__ tails, uint32_t epoch, int lines,
                                                  uint8_t *__restrict__ stage, uint64_t *__restrict__ stamps)
{
    __shared__ GroupFixed L;
    extern __shared__ uint32_t gdyn[];
    uint64_t stv[6] = {0, 0, 0, 0, 0, 0};
    if (stamps) stv[0] = __builtin_amdgcn_s_memrealtime();
    const int gi = blockIdx.x, ng = (int)gridDim.x, f = blockIdx.y, s = blockIdx.z, t = threadIdx.x;
    DynFrame *DF = dfr + (size_t)s * ld_fr + f;
    const Rect R{g.x0, g.y0, g.w, g.h};
    const size_t nb = (size_t)s * ld_fr + f;
    const int ndt = R.w * R.h;
    const uint16_t *M = meta + nb * (size_t)(NPC * ndt);
    const uint2 *BL = blo + nb * (size_t)(NPC * ndt), *BH = bhi + nb * (size_t)(NPC * ndt);
    /* groups: nA static groups above the rect (the first one holds the slice
     * header, and exists even with no rows), one per rect row, the static
     * groups below (the last one holds the stop bit); DYN_STATIC_ROWS rows
     * per static group */
    constexpr int SR = DYN_STATIC_ROWS;
    const int nA = max(1, (R.y0 + SR - 1) / SR);
    const bool first = gi == 0, last = gi == ng - 1, rect = gi >= nA && gi < nA + R.h;
    const int row = rect ? R.y0 + gi - nA : 0;
    const int nd = rect ? R.w : 0, npc = NPC * nd;
    const int q0 = rect ? (row - R.y0) * R.w : 0;
    uint32_t *moff = gdyn, *mbits = moff + lines + 1;
    uint16_t *mt = reinterpret_cast<uint16_t *>(mbits + R.w), *lo = mt + NPC * R.w, *off16 = lo + NPC * R.w;
    uint16_t *ma = off16 + NPC * R.w;
    uint8_t *cbpa = reinterpret_cast<uint8_t *>(ma + 8 * R.w), *codea = cbpa + R.w;
    /* piece j of the row in record order (three contiguous runs: luma, chroma
     * AC, chroma DC) -> its record and its slot k NPC + pc in mt / lo / off16 */
    auto rec_run = [&](int jr, int &slot) -> int {
        if (jr < 16 * nd) {
            slot = (jr >> 4) * NPC + (jr & 15);
            return 16 * q0 + jr;
        }
        if (jr < 24 * nd) {
            const int a = jr - 16 * nd;
            slot = (a >> 3) * NPC + 18 + (a & 7);
            return 16 * ndt + 8 * q0 + a;
        }
        const int a = jr - 24 * nd;
        slot = (a >> 1) * NPC + 16 + (a & 1);
        return 24 * ndt + 2 * q0 + a;
    };

    /* rect row: the records first */
    for (int i0 = 0; i0 < npc; i0 += 4 * GW) {
        uint16_t v[4];
        int sl[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int jr = i0 + t + GW * u;
            sl[u] = -1;
            v[u] = jr < npc ? M[rec_run(jr, sl[u])] : (uint16_t)0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (sl[u] >= 0) mt[sl[u]] = v[u];
    }
    for (int i0 = 0; i0 < 8 * nd; i0 += 4 * GW) {
        uint16_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + t + GW * u, k = i >> 3, e = i & 7;
            const int pcA = e < 4 ? 12 + e : (e < 6 ? 16 + e : 18 + e);
            v[u] = i < 8 * nd && row > R.y0 ? M[rec_of(q0 + k - R.w, pcA, ndt)] : (uint16_t)0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + t + GW * u;
            if (i < 8 * nd) ma[i] = v[u];
        }
    }
    const int j = DF->nal;
    if (j < 0) return;
    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    if (t == 0) L.head_over = 0;
    static_assert(sizeof(L.ct) % 8 == 0, "ct copies as uint2");
    for (int i = t; i < (int)(sizeof(L.ct) / 8); i += GW)      /* only coeff_token lives in LDS here */
        reinterpret_cast<uint2 *>(&L.ct[0][0])[i] = reinterpret_cast<const uint2 *>(&g_ptabs.ct[0][0])[i];
    DevStream *S = st + s;
    const NalDesc d = nal[(size_t)s * ld_nal + j];
    wave_sync();                                        /* waypoint table, ptabs, records */
    const NalCtx c = nal_ctx(S, d, L.wo, L.wl, L.wv);
    const HeadCtx H = head_ctx(c);
    const int mbw = H.mbw, mbh = c.h / 16;
    const Tabs &TB = g_tabs;
    const PTabs &PT = *reinterpret_cast<const PTabs *>(&g_ptabs);   /* the rare overflow paths */
    int ra, rb;
    if (gi < nA) {
        ra = gi * SR;
        rb = min(ra + SR, R.y0);
    } else if (rect) {
        ra = row;
        rb = row + 1;
    } else {
        ra = R.y0 + R.h + (gi - nA - R.h) * SR;
        rb = min(ra + SR, mbh);
    }
    uint32_t F = 0;
    if (first) {
        CountSink hc{0};
        emit_slice_header(hc, c);
        F = hc.n;
    }
    if (t < 12) {
        CapSink hc{0, 0, 0};
        H.put_class(hc, t);
        L.hhi[t] = hc.hi;
        L.hlo[t] = hc.lo;
        L.hlen[t] = hc.n;
        if (hc.over()) L.head_over = 1;
    }
    wave_sync();
    const bool head_over = L.head_over;
    auto head_bits = [&](int r, int col) -> uint32_t {
        if (!head_over) return L.hlen[H.sel(r, col)];
        CountSink cn{0};
        H.put_slow(cn, r, col);
        return cn.n;
    };

    uint64_t bits = 0;                   /* the group's bits */
    if (rect) {
        /* pieces: coeff_token from the neighbours' TotalCoeff, length */
        const uint32_t m26 = magic32(NPC);
        for (int i = t; i < npc; i += GW) {
            const int k = (int)div_m((uint32_t)i, m26), pc = i - k * NPC;
            const int col = R.x0 + k;
            const uint32_t mv = mt[i];
            const uint16_t *mk = mt + k * NPC;
            uint32_t tv = 0, tl = 0;
            int nC = -1;
            if (pc != 16 && pc != 17) {
                const int nAe = col > 0 ? 0 : -1, nBe = row > 0 ? 0 : -1;
                int nA, nB;
                if (pc < 16) {
                    const int bx = pc & 3, by = pc >> 2;
                    nA = bx > 0 ? tc_of(mk[pc - 1]) : (k > 0 ? tc_of(mk[pc + 3 - NPC]) : nAe);
                    nB = by > 0 ? tc_of(mk[pc - 4]) : (row > R.y0 ? tc_of(ma[8 * k + pc]) : nBe);
                } else {
                    const int b = (pc - 18) & 3, bx = b & 1, by = b >> 1;
                    nA = bx > 0 ? tc_of(mk[pc - 1]) : (k > 0 ? tc_of(mk[pc + 1 - NPC]) : nAe);
                    nB = by > 0 ? tc_of(mk[pc - 2])
                                : (row > R.y0 ? tc_of(ma[8 * k + (pc < 22 ? pc - 14 : pc - 16)]) : nBe);
                }
                nC = nc_of(nA, nB);
                piece_token(L.ct, mv, nC, tv, tl);
            }
            uint32_t len = tl + (mv & 255u);
            if (mv & M_OVF) len = ovf_bits(PT, TB, get_body(BL, BH, rec_of(q0 + k, pc, ndt), true), pc, nC);   /* rare */
            lo[i] = (uint16_t)(len | (uint32_t)(nC + 1) << 11);
        }
        wave_sync();
        if (stamps) stv[1] = __builtin_amdgcn_s_memrealtime();
        /* per dynamic MB: cbp, its code, piece offsets, bits */
        for (int k = t; k < nd; k += GW) {
            const uint16_t *mk = mt + k * NPC;
            int cbp_l = 0;
#pragma unroll
            for (int pc = 0; pc < 16; ++pc)
                if (tc_of(mk[pc])) cbp_l |= 1 << (2 * (pc >> 3) + ((pc & 3) >> 1));
            bool ac = false;
#pragma unroll
            for (int pc = 18; pc < NPC; ++pc) ac |= tc_of(mk[pc]) != 0;
            const bool dc = (tc_of(mk[16]) | tc_of(mk[17])) != 0;
            const int cbp_c = ac ? 2 : (dc ? 1 : 0);
            const int cbp = cbp_l | cbp_c << 4;
            const int code = TB.cbp_code[cbp];
            CountSink hs{head_bits(row, R.x0 + k)};
            put_ue(hs, (uint32_t)code);
            if (cbp) put_se(hs, 0);                         /* mb_qp_delta */
            uint32_t off = hs.n;
            const uint16_t *lk = lo + k * NPC;
            uint16_t *ok = off16 + k * NPC;
#pragma unroll
            for (int blk = 0; blk < 16; ++blk) {            /* luma4x4BlkIdx order */
                const int r = blk_raster(blk);
                const bool pres = (cbp_l >> (blk >> 2)) & 1;
                ok[r] = pres ? (uint16_t)off : (uint16_t)0xffffu;
                off += pres ? (lk[r] & LO_LEN) : 0u;
            }
#pragma unroll
            for (int k2 = 16; k2 < NPC; ++k2) {             /* Cb DC, Cr DC, Cb AC 0-3, Cr AC 0-3 */
                const bool pres = k2 < 18 ? cbp_c >= 1 : cbp_c == 2;
                ok[k2] = pres ? (uint16_t)off : (uint16_t)0xffffu;
                off += pres ? (lk[k2] & LO_LEN) : 0u;
            }
            mbits[k] = off;
            cbpa[k] = (uint8_t)cbp;
            codea[k] = (uint8_t)code;
        }
        wave_sync();
        if (stamps) stv[2] = __builtin_amdgcn_s_memrealtime();
        uint32_t carry = 0;
        for (int c0 = 0; c0 < mbw; c0 += GW) {
            const int col = c0 + t;
            uint32_t len = 0;
            if (col < mbw) {
                const int k = col - R.x0;
                len = (k >= 0 && k < R.w) ? mbits[k] : head_bits(row, col) + 1u;
            }
            const uint32_t incl = wave_incl_sum(len, t);
            if (col < mbw) moff[col] = carry + incl - len;
            carry += __shfl(incl, GW - 1, GW);
        }
        if (t == 0) moff[mbw] = carry;
        bits = carry;
    } else {
        /* rows without dynamic MBs: row offsets */
        uint32_t carry = F;
        for (int r0 = ra; r0 < rb; r0 += GW) {
            const int r = r0 + t;
            uint32_t len = 0;
            if (r < rb) {
                if (!head_over) {
                    len = row_static_bits(H, L.hlen, r, R);
                } else {
                    for (int col = 0; col < mbw; ++col) len += head_bits(r, col) + 1u;
                }
            }
            const uint32_t incl = wave_incl_sum(len, t);
            if (r < rb) moff[r - ra] = carry + incl - len;
            carry += __shfl(incl, GW - 1, GW);
        }
        if (t == 0) moff[rb - ra] = carry;
        bits = carry + (last ? 1u : 0u);
    }

    /* start bit from the groups before */
    if (stamps) stv[3] = __builtin_amdgcn_s_memrealtime();
    const uint64_t start = lb_lookback(status + nb * (size_t)ng, gi, epoch, bits, t);
    if (stamps) stv[4] = __builtin_amdgcn_s_memrealtime();
    const uint64_t end = start + bits;
    uint32_t *out = reinterpret_cast<uint32_t *>(stage + nb * g.slot_bytes);
    const uint64_t cap_words = (g.slot_bytes - DYN_OVF_BYTES) / 4 - 4;
    const bool over = bits && ((end - 1) >> 5) + 2 > cap_words;
    if (last && t == 0) {
        DF->ep = 0;
        DF->err = over ? DF_OVER : 0u;
        DF->rbsp_bytes = over ? 0u : (uint32_t)((end + 7) >> 3);   /* bitwriter.c:103-111 */
        if (over) atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_DYN);
    }
    const uint32_t rel0 = (uint32_t)(start & 31u);
    const uint64_t w0 = start >> 5, wl = bits ? (end - 1) >> 5 : 0;
    const uint32_t nw = (over || !bits) ? 0u : (uint32_t)(wl - w0 + 1);
    /* The word at the start (when rel0 != 0) also holds the groups before;
     * the word at the end (when end is not word-aligned) the groups after.
     * Each group publishes its TAIL -- the pending end word, OR of every
     * group's bits in it so far -- in an epoch-tagged word, and ORs its
     * predecessor's tail into its own first word.  The last window is
     * written first, so the tail is out early and successors hardly wait. */
    unsigned long long *ts = tails + nb * (size_t)ng;
    const uint32_t ep24 = epoch & 0xffffffu;
    const bool in_sh = rel0 != 0, out_sh = (end & 31u) != 0 && !last;   /* the last group writes its end word */
    auto tail_pub = [&](uint32_t v) { lb_store(ts + gi, (uint64_t)ep24 << 40 | 1ull << 32 | v); };
    auto tail_wait = [&]() -> uint32_t {
        for (;;) {
            const uint64_t v = __hip_atomic_load(ts + gi - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(v >> 40) == ep24 && ((v >> 32) & 1u)) return (uint32_t)v;
            __builtin_amdgcn_s_sleep(1);
        }
    };
    if (t == 0) {
        if (nw == 0) tail_pub(over || !in_sh ? 0u : tail_wait());  /* empty group: passes the tail on */
        else if (!out_sh) tail_pub(0u);
    }
    const int npass = (int)((nw + GBUF_WORDS - 1) / GBUF_WORDS);
    for (int pi = npass - 1; pi >= 0; --pi) {
        const uint32_t p0 = (uint32_t)pi * GBUF_WORDS;
        const uint32_t n = min((uint32_t)GBUF_WORDS, nw - p0);
        for (uint32_t i = (uint32_t)t; i < n; i += GW) L.buf[i] = 0u;
        wave_sync();
        const LdsOrWin win{L.buf, p0, n};
        /* the entries (rect: MB columns, static: rows) whose bits meet the
         * window [32 p0, 32 (p0 + n)): [ea, eb), by binary search on moff */
        const int ne = rect ? mbw : rb - ra;
        auto cnt_le = [&](uint32_t x) -> int {          /* # e in [0, ne] with rel0 + moff[e] <= x */
            int lo = 0, hi = ne + 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (rel0 + moff[mid] <= x) lo = mid + 1;
                else hi = mid;
            }
            return lo;
        };
        const int ea = max(cnt_le(32u * p0) - 1, 0), eb = min(cnt_le(32u * (p0 + n) - 1u), ne);
        if (rect) {
            for (int col = ea + t; col < eb; col += GW) {
                WSink sk{win, 0, 0, 0};
                sk.start(rel0 + moff[col]);
                if (!head_over) {
                    const int cls = H.sel(row, col);
                    sk.put_cap(CapSink{L.hhi[cls], L.hlo[cls], L.hlen[cls]});
                } else {
                    H.put_slow(sk, row, col);
                }
                const int k = col - R.x0;
                if (!(k >= 0 && k < R.w)) {
                    sk.put(1, 1);                           /* coded_block_pattern ue(0) */
                } else {
                    put_ue(sk, (uint32_t)codea[k]);
                    if (cbpa[k]) put_se(sk, 0);
                }
                sk.finish();
            }
            const uint32_t m26 = magic32(NPC);
            const int pa = NPC * max(ea - R.x0, 0), pb = NPC * min(eb - R.x0, nd);
            for (int i0 = pa; i0 < pb; i0 += 4 * GW) {
                uint4 bd[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {               /* four body loads in flight */
                    const int i = i0 + t + GW * u;
                    bd[u] = make_uint4(0, 0, 0, 0);
                    if (i < pb && off16[i] != 0xffffu && (mt[i] & (255u | M_OVF))) {
                        const int k = (int)div_m((uint32_t)i, m26);
                        bd[u] = get_body(BL, BH, rec_of(q0 + k, i - k * NPC, ndt), (mt[i] & 255u) > 64u || (mt[i] & M_OVF));
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = i0 + t + GW * u;
                    if (i >= pb) continue;
                    const uint32_t o = off16[i];
                    if (o == 0xffffu) continue;
                    const int k = (int)div_m((uint32_t)i, m26), pc = i - k * NPC;
                    const uint32_t e = lo[i], mv = mt[i];
                    const int nC = (int)(e >> 11) - 1;
                    const uint32_t pos = rel0 + moff[R.x0 + k] + o;
                    if (!(mv & M_OVF)) {
                        WSink sk{win, 0, 0, 0};
                        sk.start(pos);
                        if (nC != -1) {
                            uint32_t tv, tl;
                            piece_token(L.ct, mv, nC, tv, tl);
                            sk.put(tv, (int)tl);
                        }
                        sk.put_cap(CapSink{(uint64_t)bd[u].z | (uint64_t)bd[u].w << 32,
                                           (uint64_t)bd[u].x | (uint64_t)bd[u].y << 32, mv & 255u});
                        sk.finish();
                    } else {
                        ovf_put(L.buf, p0, n, pos, PT, TB, bd[u], pc, nC);
                    }
                }
            }
        } else {
            if (first && t == 0 && p0 * 32u < F) {          /* slice header, h264_writer.c:549-553 */
                WSink hs{win, 0, 0, 0};
                hs.start(0);
                emit_slice_header(hs, c);
                hs.finish();
            }
            const int nm = eb * mbw;
            const uint32_t m_mbw = magic32((uint32_t)mbw);
            for (int m = ea * mbw + t; m < nm; m += GW) {
                const int rr = (int)div_m((uint32_t)m, m_mbw), col = m - rr * mbw, r = ra + rr;
                uint32_t off = moff[rr];
                WSink sk{win, 0, 0, 0};
                if (!head_over) {
                    const int b3 = H.sel(r, 0);
                    off += col == 0 ? 0u : L.hlen[b3] + 1u + (uint32_t)(col - 1) * (L.hlen[b3 + 1] + 1u);
                    const int cls = b3 + (col == 0 ? 0 : (col == mbw - 1 ? 2 : 1));
                    sk.start(rel0 + off);
                    sk.put_cap(CapSink{L.hhi[cls], L.hlo[cls], L.hlen[cls]});
                } else {
                    for (int c2 = 0; c2 < col; ++c2) off += head_bits(r, c2) + 1u;
                    sk.start(rel0 + off);
                    H.put_slow(sk, r, col);
                }
                sk.put(1, 1);                               /* coded_block_pattern ue(0) */
                sk.finish();
            }
            if (last && t == 0) {                           /* rbsp_stop_one_bit */
                WSink sk{win, 0, 0, 0};
                sk.start(rel0 + (uint32_t)bits - 1u);
                sk.put(1, 1);
                sk.finish();
            }
        }
        wave_sync();
        /* every word but a shared first one first -- the out-shared tail is
         * published before this wave waits for its predecessor's, so small
         * one-pass groups do not chain their successors behind that wait */
        for (uint32_t i = (uint32_t)t; i < n; i += GW) {
            const uint32_t q = p0 + i, v = L.buf[i];
            if (q == 0 && in_sh) continue;
            if (q == nw - 1 && out_sh) tail_pub(v);
            else out[w0 + q] = __builtin_bswap32(v);
        }
        if (p0 == 0 && in_sh && t == 0) {
            const uint32_t v2 = L.buf[0] | tail_wait();
            if (nw == 1 && out_sh) tail_pub(v2);
            else out[w0] = __builtin_bswap32(v2);
        }
        wave_sync();
    }
    if (stamps && t == 0) {
        stv[5] = __builtin_amdgcn_s_memrealtime();
        uint64_t *o = stamps + (((size_t)s * gridDim.y + f) * ng + gi) * 8;
        for (int k2 = 0; k2 < 6; ++k2) o[k2] = stv[k2];
        o[6] = bits;
        o[7] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);     /* HW_ID */
    }
}

/* grid (EP_G, frames, streams): workgroup x scans chunks x, x + EP_G, .. of
 * EP_CHUNK bytes of its NAL's staged RBSP; a chunk's carry-in (the last
 * non-zero byte before it) is looked up backwards in the staged bytes, so
 * chunks are independent.  EP positions (slot tail, unsorted) and count. */
constexpr int EP_G = 8, EP_T = 256, EP_NW = EP_T / 64, EP_CHUNK = EP_T * 32;

__global__ __launch_bounds__(EP_T) void k_dyn_ep(DynFrame *__restrict__ dfr, int ld_fr, DynGeom g,
                                                 const uint8_t *__restrict__ stage)
{
    __shared__ int32_t wmax[EP_NW];
    __shared__ int32_t back;
    const int s = blockIdx.z, f = blockIdx.y, t = threadIdx.x, lane = t & 63;
    DynFrame *DF = dfr + (size_t)s * ld_fr + f;
    const DynFrame df = *DF;
    if (df.nal < 0 || df.err) return;
    const size_t nb = (size_t)s * ld_fr + f;
    const uint8_t *in = stage + nb * g.slot_bytes;
    uint32_t *eplist = reinterpret_cast<uint32_t *>(const_cast<uint8_t *>(in) + g.slot_bytes - DYN_OVF_BYTES);
    const uint32_t nin = df.rbsp_bytes;
    for (uint32_t c0 = (uint32_t)blockIdx.x * EP_CHUNK; c0 < nin; c0 += EP_G * EP_CHUNK) {
        /* carry-in: wave 0 reads the 256 bytes before the chunk, further back
         * only while they are all zero */
        if (t < 64) {
            int pv = -1;
            for (int64_t b0 = (int64_t)c0 - 256; b0 > -256; b0 -= 256) {
                const int64_t o = b0 + 4 * lane;
                const uint32_t m = o >= 0 ? *reinterpret_cast<const uint32_t *>(in + o) : 0u;
                const uint64_t nz = __ballot(m != 0);
                if (nz) {
                    const int hl = 63 - __builtin_clzll(nz);
                    const uint32_t mh = __shfl(m, hl, 64);
                    pv = (int)(b0 + 4 * hl) + 3 - (__builtin_clz(mh) >> 3);
                    break;
                }
            }
            if (t == 0) back = pv;
        }
        const uint32_t ib = c0 + 32u * (uint32_t)t;
        uint32_t wv[8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint32_t o = ib + 16u * u;
            const uint4 v = o < nin ? *reinterpret_cast<const uint4 *>(in + o) : make_uint4(0, 0, 0, 0);
            wv[4 * u] = v.x;
            wv[4 * u + 1] = v.y;
            wv[4 * u + 2] = v.z;
            wv[4 * u + 3] = v.w;
        }
        int lnz = -1;                                   /* bytes >= nin: not scanned */
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const uint32_t m = ib + 4u * w < nin ? wv[w] : 0u;
            if (m) lnz = (int)(ib + 4u * w) + 3 - (__builtin_clz(m) >> 3);
        }
        int ex, tot;
        block_excl_max<EP_NW>(lnz, wmax, ex, tot);     /* its barriers also publish `back` */
        int prev = max(back, ex);
        uint32_t ins = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const uint32_t gi = ib + (uint32_t)i;
            const uint32_t b = gi < nin ? (wv[i >> 2] >> (8 * (i & 3))) & 255u : 256u;   /* past the end: never inserts */
            ins |= (ep_insert(b, (int)gi - 1 - prev) ? 1u : 0u) << i;
            prev = b ? (int)gi : prev;
        }
        const uint32_t cnt = (uint32_t)__builtin_popcount(ins);
        const uint32_t incl = wave_incl_sum(cnt, lane);
        const uint32_t wtot = __shfl(incl, 63, 64);
        uint32_t base = 0;
        if (wtot) {
            if (lane == 0) base = atomicAdd(&DF->ep, wtot);
            base = __shfl(base, 0, 64);
        }
        uint32_t k = base + incl - cnt;
        while (ins) {
            const int i = __builtin_ctz(ins);
            ins &= ins - 1u;
            if (k < (uint32_t)EPLIST_MAX) eplist[k] = ib + (uint32_t)i;   /* RBSP index the 03 precedes */
            k++;
        }
        __syncthreads();                                /* `back` is rewritten by the next chunk */
    }
}


/* ---------------------------------------------------------------------- */
/* k_dyn_emit: staged RBSP -> arena with start code, header, EP bytes       */
/* ---------------------------------------------------------------------- */
__device__ inline void store16(uint8_t *A, uint64_t p, const uint8_t *src, uint64_t lo, uint64_t hi)
{
    if (p >= lo && p + 16 <= hi) {
        *reinterpret_cast<uint4 *>(A + p) = *reinterpret_cast<const uint4 *>(src);
        return;
    }
    for (int i = 0; i < 16; ++i)
        if (p + i >= lo && p + i < hi) A[p + i] = src[i];
}

__global__ __launch_bounds__(DT) void k_dyn_emit(const DevStream *__restrict__ st,
                                                 const NalDesc *__restrict__ nal, int ld_nal,
                                                 const DynFrame *__restrict__ dfr, int ld_fr,
                                                 DynGeom g, const uint8_t *__restrict__ stage,
                                                 uint8_t *__restrict__ arena, uint64_t ld_arena)
{
    __shared__ alignas(16) uint8_t ob[OBUF];
    __shared__ int32_t wmax[NW];
    __shared__ uint32_t wsum[NW];
    const int f = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
    const DynFrame df = dfr[(size_t)s * ld_fr + f];
    const int j = df.nal;
    if (j < 0 || j >= st[s].nnal || df.err) return;          /* nnal = 0: nothing committed */
    if (df.ep <= ep_cap(g)) return;                          /* k_dyn_emit_gather's NAL */
    const NalDesc d = nal[(size_t)s * ld_nal + j];
    if (d.slow != 2) return;
    uint8_t *A = arena + (size_t)s * ld_arena;
    const uint64_t o0 = d.out_off, o1 = o0 + d.size;
    const uint8_t *in = stage + ((size_t)s * ld_fr + f) * g.slot_bytes;
    const uint32_t nin = df.rbsp_bytes;

    uint64_t lb = o0 & ~127ull;                  /* arena byte of ob[0] (line aligned) */
    uint32_t fill = (uint32_t)(o0 - lb);
    if (t < 5) ob[fill + t] = t < 3 ? 0 : (t == 3 ? 1 : nal_header_byte(0));   /* nal.c:59-64 */
    fill += 5;
    int carry = -1;
    for (uint32_t i0 = 0; i0 < nin; i0 += DT * 16) {
        const uint32_t ib = i0 + 16u * (uint32_t)t;
        const uint32_t n = ib < nin ? min(16u, nin - ib) : 0u;
        uint8_t b[16];
        {
            const uint4 v = n ? *reinterpret_cast<const uint4 *>(in + ib) : make_uint4(0, 0, 0, 0);
            const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int i = 0; i < 16; ++i) b[i] = (uint8_t)(wv[i >> 2] >> (8 * (i & 3)));
        }
        int lnz = -1;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((uint32_t)i < n && b[i]) lnz = (int)(ib + i);
        int ex, tot;
        block_excl_max(lnz, wmax, ex, tot);
        int prev = max(carry, ex);
        uint32_t ins = 0, cnt = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if ((uint32_t)i >= n) break;
            if (ep_insert(b[i], (int)(ib + i) - 1 - prev)) {
                ins |= 1u << i;
                cnt++;
            }
            if (b[i]) prev = (int)(ib + i);
        }
        uint32_t opos, otot;
        block_excl_sum(n + cnt, wsum, opos, otot);
        uint32_t p = fill + opos;
        for (int i = 0; i < 16; ++i) {
            if ((uint32_t)i >= n) break;
            if ((ins >> i) & 1u) ob[p++] = 3;
            ob[p++] = b[i];
        }
        __syncthreads();
        const uint32_t nf = fill + otot, nlines = nf >> 7;
        for (uint32_t c = (uint32_t)t; c < nlines * 8; c += DT)
            store16(A, lb + 16u * c, ob + 16u * c, o0, o1);
        const uint32_t rem = nf - (nlines << 7);
        const uint8_t keep = (uint32_t)t < rem ? ob[(nlines << 7) + t] : 0;
        __syncthreads();
        if ((uint32_t)t < rem) ob[t] = keep;
        lb += (uint64_t)nlines << 7;
        fill = rem;
        carry = max(carry, tot);
        __syncthreads();
    }
    for (uint32_t c = (uint32_t)t; 16u * c < fill; c += DT) store16(A, lb + 16u * c, ob + 16u * c, o0, o1);
}

/* ---------------------------------------------------------------------- */
/* k_dyn_emit_gather: the same output for NALs with <= EPLIST_MAX EP bytes  */
/* (all in practice: 82 per config-3 frame).  k_dyn_ep recorded where       */
/* the 03 bytes go; after sorting those positions once, every thread builds */
/* whole 16-byte arena chunks independently -- no barriers, no LDS byte     */
/* buffer: a chunk without an EP byte is a funnel shift of the staged RBSP. */
/* ---------------------------------------------------------------------- */
__device__ inline uint32_t pick4(const uint32_t w[8], int i)     /* w[i], i in 0..7, no indexing */
{
    const uint32_t a = (i & 1) ? w[1] : w[0], b = (i & 1) ? w[3] : w[2];
    const uint32_t c = (i & 1) ? w[5] : w[4], e = (i & 1) ? w[7] : w[6];
    const uint32_t ab = (i & 2) ? b : a, ce = (i & 2) ? e : c;
    return (i & 4) ? ce : ab;
}

constexpr int GATHER_Z = 1;             /* workgroups per NAL (2 and 4 measured slower) */

__global__ __launch_bounds__(DT) void k_dyn_emit_gather(const DevStream *__restrict__ st,
                                                        const NalDesc *__restrict__ nal, int ld_nal,
                                                        const DynFrame *__restrict__ dfr, int ld_fr,
                                                        DynGeom g, const uint8_t *__restrict__ stage,
                                                        uint8_t *__restrict__ arena, uint64_t ld_arena,
                                                        uint64_t *__restrict__ stamps)
{
    __shared__ uint32_t raw[EPLIST_MAX], sp[EPLIST_MAX];
    const int s = blockIdx.y, f = dyn_frame_of(blockIdx.x, s), t = threadIdx.x;
    /* debug: realtime at entry / after the sort / at exit, EP count, HW_ID */
    uint64_t *stp = stamps && t == 0 && blockIdx.z == 0 ? stamps + ((size_t)s * gridDim.x + f) * 8 : nullptr;
    if (stp) stp[0] = __builtin_amdgcn_s_memrealtime();
    const DynFrame df = dfr[(size_t)s * ld_fr + f];
    const int j = df.nal;
    if (j < 0 || j >= st[s].nnal || df.err) return;          /* nnal = 0: nothing committed */
    const uint32_t n = df.ep;
    if (n > ep_cap(g)) return;                               /* k_dyn_emit's NAL */
    const NalDesc d = nal[(size_t)s * ld_nal + j];
    if (d.slow != 2) return;
    const uint8_t *in = stage + ((size_t)s * ld_fr + f) * g.slot_bytes;
    const uint32_t *el = reinterpret_cast<const uint32_t *>(in + g.slot_bytes - DYN_OVF_BYTES);
    for (uint32_t i = t; i < n; i += DT) raw[i] = el[i];
    __syncthreads();
    /* sort by rank (positions are distinct): sp[j] = j-th smallest */
    for (uint32_t i = t; i < n; i += DT) {
        const uint32_t v = raw[i];
        uint32_t r = 0;
        for (uint32_t k = 0; k < n; ++k) r += raw[k] < v ? 1u : 0u;
        sp[r] = v;
    }
    __syncthreads();
    if (stp) {
        stp[1] = __builtin_amdgcn_s_memrealtime();
        stp[3] = n;
        stp[4] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);    /* HW_ID */
    }

    uint8_t *A = arena + (size_t)s * ld_arena;
    const uint64_t o0 = d.out_off, o1 = o0 + d.size;
    const uint32_t nin = df.rbsp_bytes;
    const uint8_t hdr[5] = {0, 0, 0, 1, nal_header_byte(0)};           /* nal.c:59-64 */
    /* U chunks per thread and iteration: all their loads are in flight
     * before the first is used (the loop is load-latency bound otherwise) */
    constexpr int U = 4;
    /* the NAL's 16-byte chunks are split over gridDim.z workgroups */
    const uint64_t cfirst = o0 >> 4, cnal = ((o1 + 15) >> 4) - cfirst;
    const uint64_t per = (cnal + gridDim.z - 1) / gridDim.z;
    const uint64_t cbeg = cfirst + per * blockIdx.z, cend = min(cfirst + cnal, cbeg + per);
    /* coarse index (in raw, free after the sort): raw[b] = EP bytes before
     * EBSP index b << cs, by one binary search per block; a chunk then
     * starts from its block's count and steps over the few EP bytes between */
    int lg = 0;                   /* binary-search steps: 2^lg > n */
    while ((1u << lg) <= n) lg++;
    int cs = 10;
    while ((d.size >> cs) >= 1024) cs++;
    const int nblk = (int)(d.size >> cs) + 1;
    for (int bi = t; bi < nblk; bi += DT) {
        const int64_t e0 = (int64_t)bi << cs;
        uint32_t K = 0;
        for (int b = lg - 1; b >= 0; --b) {
            const uint32_t k2 = K + (1u << b);
            K = k2 <= n && (int64_t)(sp[k2 - 1] + (k2 - 1)) < e0 ? k2 : K;
        }
        raw[bi] = K;
    }
    __syncthreads();
    for (uint64_t cb = cbeg + (uint64_t)t; cb < cend; cb += (uint64_t)U * DT) {
        uint32_t Ku[U], epm[U], shv[U];
        bool inner[U];
        uint4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t q0 = (cb + (uint64_t)u * DT) << 4;
            const int64_t u0 = (int64_t)q0 - (int64_t)o0 - 5;        /* EBSP index of byte 0 */
            /* K = EP bytes before the chunk; the j-th sits at EBSP index
             * sp[j] + j (strictly increasing) */
            uint32_t K = u0 > 0 ? raw[min((int)(u0 >> cs), nblk - 1)] : 0u;
            while (K < n && (int64_t)(sp[K] + K) < u0) K++;
            Ku[u] = K;
            inner[u] = u0 >= 0 && q0 + 16 <= o1;
            epm[u] = 0;
            shv[u] = 0;
            x[u] = y[u] = make_uint4(0, 0, 0, 0);
            if (inner[u]) {
                /* interior chunk: EP bytes of the chunk as a mask; output byte
                 * b takes RBSP byte i0 + b - (EP bytes before b), or is 03 */
                uint32_t em = 0;
                for (uint32_t m = K; m < n; ++m) {
                    const int64_t e = (int64_t)(sp[m] + m) - u0;
                    if (e >= 16) break;
                    em |= 1u << e;
                }
                epm[u] = em;
                const uint32_t i0 = (uint32_t)u0 - K, a0 = i0 & ~15u;
                shv[u] = i0 & 15u;
                x[u] = *reinterpret_cast<const uint4 *>(in + a0);
                if (a0 + 16 < nin) y[u] = *reinterpret_cast<const uint4 *>(in + a0 + 16);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c = cb + (uint64_t)u * DT;
            if (c >= cend) break;
            const uint64_t q0 = c << 4;
            if (inner[u]) {
                const uint32_t w[8] = {x[u].x, x[u].y, x[u].z, x[u].w, y[u].x, y[u].y, y[u].z, y[u].w};
                const uint32_t sh = shv[u], em = epm[u];
                uint32_t o[4];
                if (em == 0) {                               /* funnel shift */
                    const int wi = (int)(sh >> 2), bs = (int)(sh & 3u);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t lo = pick4(w, wi + k), hi = pick4(w, wi + k + 1);
                        o[k] = bs ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)bs) : lo;
                    }
                } else {               /* a word's bytes span <= 2 RBSP words: v_perm */
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t b0 = 4u * (uint32_t)k;
                        const uint32_t r0 = sh + b0 - (uint32_t)__builtin_popcount(em & ((1u << b0) - 1u));
                        const uint32_t base = r0 >> 2;
                        const uint32_t lo = pick4(w, (int)base), hi = pick4(w, (int)base + 1);
                        uint32_t sel = 0, three = 0;
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t bb = b0 + (uint32_t)i;
                            uint32_t v;
                            if ((em >> bb) & 1u) {
                                v = 0x0cu;                           /* perm: byte 00 */
                                three |= 3u << (8 * i);
                            } else {
                                v = sh + bb - (uint32_t)__builtin_popcount(em & ((1u << bb) - 1u)) - 4u * base;
                            }
                            sel |= v << (8 * i);
                        }
                        o[k] = __builtin_amdgcn_perm(hi, lo, sel) | three;
                    }
                }
                *reinterpret_cast<uint4 *>(A + q0) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {                                     /* NAL edges, start code */
                uint32_t kk = Ku[u];
                for (int b = 0; b < 16; ++b) {
                    const uint64_t q = q0 + (uint64_t)b;
                    if (q < o0 || q >= o1) continue;
                    const int64_t uu = (int64_t)q - (int64_t)o0 - 5;
                    uint8_t v;
                    if (uu < 0) {
                        v = hdr[q - o0];
                    } else if (kk < n && (int64_t)(sp[kk] + kk) == uu) {
                        v = 3;
                        kk++;
                    } else {
                        v = in[(uint32_t)uu - kk];
                    }
                    A[q] = v;
                }
            }
        }
    }
    if (stp) stp[2] = __builtin_amdgcn_s_memrealtime();
}

/* ---------------------------------------------------------------------- */
/* k_dyn_synth: the synthetic dynamic-rect source of SURVEY §8d            */
/* (dyn_oracle.h), one thread per pixel                                    */
/* ---------------------------------------------------------------------- */
__device__ inline uint32_t mix32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void k_dyn_synth(uint8_t *__restrict__ src, DynGeom g,
                                                   int stream_base, int t0)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const int f = blockIdx.y, s = blockIdx.z;
    const uint32_t npx = 384u * (uint32_t)g.w * (uint32_t)g.h;
    if (i >= npx) return;
    const uint32_t tt = (uint32_t)(t0 + f);
    const uint32_t seed = (0x9E3779B9u * (uint32_t)(stream_base + s)) ^ (0x85EBCA6Bu * tt);
    const uint32_t hv = mix32(seed + i * 0x9E3779B9u);
    const uint32_t ly = 256u * (uint32_t)g.w * (uint32_t)g.h;
    int v;
    if (i < ly) {
        const int lw = 16 * g.w;
        const int y = (int)(i / (uint32_t)lw), x = (int)(i - (uint32_t)(y * lw));
        const int X = 16 * g.x0 + x, Y = 16 * g.y0 + y;
        v = 128 + ((X + 2 * Y + 3 * (int)tt) & 63) - 32 + (int)(hv >> 28) - 8;
    } else {
        const uint32_t r = (i - ly) % (64u * (uint32_t)g.w * (uint32_t)g.h);
        const int cw = 8 * g.w;
        const int y = (int)(r / (uint32_t)cw), x = (int)(r - (uint32_t)(y * cw));
        const int X = 8 * g.x0 + x, Y = 8 * g.y0 + y;
        v = 128 + ((X + Y + (int)tt) & 15) - 8 + (int)(hv >> 30);
    }
    src[(size_t)s * g.src_ld + (size_t)f * g.src_fr + i] = (uint8_t)clampi(v, 0, 255);
}

}  // namespace

/* ---------------------------------------------------------------------- */
/* launchers (engine-internal, engine.h)                                   */
/* ---------------------------------------------------------------------- */
int dyn_launch_code(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal,
                    int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                    const DynGeom *g, const uint8_t *src, const uint8_t *refs, const DynScratch *x)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_dyn_rows, dim3(nframes, S), dim3(256), 0, hs, st, nal, ld_nal, pend, dfr, ld_fr,
                       *g, x->rows);
    if (hipGetLastError() != hipSuccess) return -1;
    const int nchunk = (24 * g->w * g->h + CODE_T - 1) / CODE_T;
    hipLaunchKernelGGL(k_dyn_code, dim3(nchunk, nframes, S), dim3(CODE_T), 0, hs, st, dfr, ld_fr,
                       pend, nal, ld_nal, *g, x->rows, src, refs, x->meta, x->body_lo, x->body_hi);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(k_dyn_code_general, dim3(nchunk, CODE_GEN_Y), dim3(CODE_T), 0, hs, st, dfr, ld_fr,
                       pend, nal, ld_nal, *g, x->rows, src, refs, x->meta, x->body_lo, x->body_hi, nframes, S);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int dyn_launch_pack(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                    int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                    const DynGeom *g, const DynScratch *x, uint8_t *stage, uint32_t epoch,
                    uint64_t *stamps, int mbw, int mbh)
{
    if (nframes <= 0 || S <= 0) return 0;
    const int ng = g->ngroups;
    const int lines = mbw > mbh ? mbw : mbh;
    hipLaunchKernelGGL(k_dyn_group, dim3(ng, nframes, S), dim3(GW), group_lds_bytes(g->w, lines), hs, st, nal,
                       ld_nal, pend, dfr, ld_fr, *g, x->meta, x->body_lo, x->body_hi, x->status, x->tails, epoch, lines,
                       stage, stamps);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(k_dyn_ep, dim3(EP_G, nframes, S), dim3(EP_T), 0, hs, dfr, ld_fr, *g, stage);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int dyn_launch_emit(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal,
                    int ld_nal, const DynFrame *dfr, int ld_fr, const DynGeom *g,
                    const uint8_t *stage, uint8_t *arena, uint64_t ld_arena, uint64_t *stamps)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_dyn_emit_gather, dim3(nframes, S, GATHER_Z), dim3(DT), 0, hs, st, nal, ld_nal, dfr,
                       ld_fr, *g, stage, arena, ld_arena, stamps);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(k_dyn_emit, dim3(nframes, S), dim3(DT), 0, hs, st, nal, ld_nal, dfr, ld_fr,
                       *g, stage, arena, ld_arena);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int dyn_launch_synth(hipStream_t hs, int nframes, int S, uint8_t *src, const DynGeom *g,
                     int stream_base, int t0)
{
    if (nframes <= 0 || S <= 0) return 0;
    const uint32_t npx = 384u * (uint32_t)g->w * (uint32_t)g->h;
    hipLaunchKernelGGL(k_dyn_synth, dim3((npx + 255) / 256, nframes, S), dim3(256), 0, hs, src, *g,
                       stream_base, t0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t dyn_slot_bound(int mbw, int mbh, int rw, int rh)
{
    /* header + every MB head (+ cbp) + every dynamic MB at its provable
     * maximum + the stop word + a 16-byte read margin (k_dyn_ep) */
    const size_t bits = (size_t)HDR_MAX + (size_t)mbw * mbh * (HEAD_MAX + 1) +
                        (size_t)rw * rh * MB_BITS_MAX + 64;
    return ((bits / 8 + 32 + DYN_OVF_BYTES) + 255) & ~(size_t)255;
}
