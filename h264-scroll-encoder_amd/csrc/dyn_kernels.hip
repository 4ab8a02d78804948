/*
 * dyn_kernels.hip -- MI355X (gfx950) kernels of the dynamic-rect residual
 * coder (BASELINE configs 3-5).  A scroll NAL with the rect is no longer a
 * handful of periodic runs: every dynamic MB carries a CAVLC residual, and
 * 60 % of such NALs need emulation prevention.  So these NALs take their own
 * kernels around the plan's sizing pass:
 *
 *   k_plan (state pass)   waypoint state machine, NalDesc per NAL
 *   k_dyn_rows            per NAL: prediction row offsets (waypoint chains)
 *   k_dyn_code_general    the rare half-pel-chroma NALs: block records
 *   k_dyn_row             one workgroup per rect MB row: transform, quant,
 *                         CAVLC, coeff_token, cbp, MB offsets, bits -> the
 *                         row's own row-stage words (records stay in LDS)
 *   k_dyn_static          one wave per static row group (slice header, rows
 *                         above / below the rect, stop bit) -> row-stage words
 *   k_dyn_epfix           per NAL: row-group offsets, emulation-prevention
 *                         positions from the groups' EP-candidate words
 *                         (or, past what those settle, a scan of the NAL)
 *   k_plan (size pass)    NAL sizes (dynamic: 5 + RBSP + EP), arena offsets
 *   k_emit                every other NAL (dynamic NALs are "external")
 *   k_dyn_gather          row-stage groups -> arena: start code, NAL header,
 *                         EP bytes, 16-byte chunks (emit_serial in the same
 *                         workgroup past 2048 EP bytes); the RBSP is never
 *                         staged
 *
 * The bits are those of oracle/dyn_oracle.c (or_scroll_nal_dyn); parity is
 * checked bit-exact by tests/test_gpu_dyn.py.  Roofline: HBM (source pixels
 * + reference pixels in, NAL bytes out), DESIGN.md §5.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <mutex>

#include "dyn_device.h"
#include "dyn_engine.h"
#include "row_mfma.h"
#include "stage_util.h"

using namespace scroll;
using namespace scroll::dyn;
using namespace scroll::stage;

namespace {

__constant__ Tabs g_tabs = SCROLL_DYN_TABS;
constexpr Tabs k_tabs = SCROLL_DYN_TABS;
__constant__ PTabs g_ptabs = make_ptabs(k_tabs);
/* total_zeros + run_before per non-zero mask (tzrb_entry), k_dyn_row's
 * table: 384 KB, filled once per device by k_tzrb_init; mostly L2-resident
 * (the masks of real blocks are few) */
__device__ uint32_t g_tzrb[TZRB_N];
/* level codewords (lvt_entry), copied into k_dyn_row's bit window for its
 * CAVLC phase */
__constant__ LvTab g_lvt = make_lvt();

/* the quantiser at every rect QP, luma and chroma (QPc, Table 8-15): one
 * uniform index -> scalar loads (qparams_rt's six-way selects compiled to a
 * branch maze per workgroup) */
struct QpPair {
    QParams l, c;
};
struct QpTab {
    QpPair q[QP_MAX + 1];
};
constexpr QpTab make_qptab()
{
    QpTab T{};
    for (int i = 0; i <= QP_MAX; ++i) T.q[i] = QpPair{qparams(i), qparams(qp_chroma(i))};
    return T;
}
__constant__ QpTab g_qptab = make_qptab();

__global__ __launch_bounds__(256) void k_tzrb_init()
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < TZRB_N) g_tzrb[i] = i < 65536 ? tzrb_entry(g_tabs, (uint32_t)i, 16) : tzrb_entry(g_tabs, (uint32_t)(i - 65536), 15);
}

/* packed CAVLC tables -> LDS, one 16-byte load per thread */
__device__ inline void load_ptabs(PTabs &dst, int t, int nthr)
{
    constexpr int N = (int)(sizeof(PTabs) / 16);
    static_assert(sizeof(PTabs) % 16 == 0, "PTabs copies as uint4");
    for (int i = t; i < N; i += nthr) reinterpret_cast<uint4 *>(&dst)[i] = reinterpret_cast<const uint4 *>(&g_ptabs)[i];
}

/* RowTabs from g_ptabs, one 32-bit word per thread and step */
__device__ inline void load_rowtabs(RowTabs &dst, int t, int nthr)
{
    constexpr int NC = (int)(sizeof(dst.ct) / 4), NZ = (int)(sizeof(dst.tzdc) / 4), NR = (int)(sizeof(dst.rb) / 4);
    static_assert(sizeof(dst.ct) % 4 == 0 && sizeof(dst.tzdc) % 4 == 0 && sizeof(dst.rb) % 4 == 0, "word copies");
    const uint32_t *ct = reinterpret_cast<const uint32_t *>(g_ptabs.ct);
    const uint32_t *tz = reinterpret_cast<const uint32_t *>(g_ptabs.tzdc);
    const uint32_t *rb = reinterpret_cast<const uint32_t *>(g_ptabs.rb);
    uint32_t *dc = reinterpret_cast<uint32_t *>(dst.ct), *dz = reinterpret_cast<uint32_t *>(dst.tzdc);
    uint32_t *dr = reinterpret_cast<uint32_t *>(dst.rb);
    for (int i = t; i < NC + NZ + NR; i += nthr) {
        if (i < NC) dc[i] = ct[i];
        else if (i < NC + NZ) dz[i - NC] = tz[i - NC];
        else dr[i - NC - NZ] = rb[i - NC - NZ];
    }
}


constexpr int HEAD_MAX = 160;           /* bits of one MB head (huge mvd: 2 x 63 + ref) */
constexpr int HDR_MAX = 1024;           /* slice header bits (8 waypoints + MMCO ~ 250) */
constexpr int OBUF = 6400;              /* emit_serial: 127 carry + 5 + 4096 x 1.5 */

/* DynFrame.err bits: a pool ran out (the batch grows it, the compose is
 * repeated); the general chroma path; k_dyn_row's wait for the row above
 * expired (the stream fails, SCROLL_ERR_DEVICE) */
constexpr uint32_t DF_OVER = 1u, DF_GENERAL = 2u, DF_HANDOFF = 4u;
/* the bound on that wait: 50 ms of s_memrealtime (100 MHz).  A row above is
 * dispatched first and publishes within microseconds; the bound only turns a
 * broken hand-off into a failed stream instead of a GPU hang */
constexpr uint64_t HANDOFF_TICKS = 5000000ull;
constexpr uint64_t HANDOFF_GAP = 100000ull;     /* 1 ms: a longer gap between two polls is a preemption */
/* k_dyn_epfix could not settle the NAL's EP positions from the candidates
 * (too many): it scanned the NAL whole (ep_scan, list unsorted); not an
 * error for the emit */
constexpr uint32_t DF_EPSLOW = 0x100u;
/* the NAL's size and EP list are final (ep_fix ran; the list is sorted
 * unless DF_EPSLOW) */
constexpr uint32_t DF_FIXED = 0x200u;

/* ---------------------------------------------------------------------- */
/* emulation-prevention runs                                                */
/* ---------------------------------------------------------------------- */
/* A 03 goes before RBSP byte i only if b_i <= 3 after two zero bytes: 22
 * consecutive zero bits.  Every row group records, while it flushes its
 * bits, the words in which such a run may start (ep_quick: a cheap
 * superset); k_dyn_epfix finds the exact runs there (start a after a one
 * bit, end e = the first one bit after it; group-local, bits past the
 * group's count taken as ones) and, once the group's NAL bit offset O is
 * known, the run's EP bytes by arithmetic: with A = O + a rounded up to a
 * byte, the bytes starting at A + 8m for m = 2, 4, 6, ... while A + 8m + 6
 * <= O + e (each is <= 3 after m zero bytes; the byte holding bit a - 1 is
 * non-zero).  Runs starting at the group's first bit, and the bytes reaching
 * past the group's end, are the group seam's (k_dyn_epfix reads those
 * bytes).  At most EPC_ROW - 1 / EPC_STATIC - 1 words per group (more: the
 * NAL takes the whole scan, ep_scan). */
/* record words per group (count, then word indices): rect rows, static
 * groups (64 MB rows of scroll heads: large-mv codewords can repeat a run
 * in every MB) */
constexpr int EPC_ROW = 256, EPC_STATIC = 4096;

/* word gi of a group with `bits` data bits, data bits past the end as ones */
__device__ inline uint32_t ep_data(uint32_t w, uint32_t gi, uint32_t bits)
{
    const uint32_t b0 = 32u * gi;
    if (__builtin_expect(b0 + 32u <= bits, 1)) return w;
    return w | (bits > b0 ? 0xffffffffu >> (bits - b0) : 0xffffffffu);
}

/* positions (bit 31 - j = position j from the top) in word w (group word
 * gi) where a run of >= 22 zero data bits starts after a one; pw, nx: the
 * words before / after (pw = 0 for the group's first word: a run there is
 * the seam's) */
__device__ inline uint32_t ep_run_starts(uint32_t pw, uint32_t w, uint32_t nx, uint32_t gi, uint32_t bits)
{
    uint64_t X = (uint64_t)ep_data(w, gi, bits) << 32 | ep_data(nx, gi + 1u, bits);
    X |= X << 1;
    X |= X << 2;
    X |= X << 4;
    X |= X << 8;                                 /* bit j (from the top): OR of bits j .. j + 15 */
    X |= X << 6;                                 /* .. j + 21 */
    const uint32_t z22 = ~(uint32_t)(X >> 32);
    return z22 & ((ep_data(w, gi, bits) >> 1) | (pw << 31));   /* bit j - 1 is a one */
}

/* a superset of the words where a run of >= 22 zero bits starts: 22 zero
 * bits inside w, or w's trailing + nx's leading zeros (padding past the
 * data counts as zeros here: a few extra words, settled by k_dyn_epfix) */
__device__ inline bool ep_quick(uint32_t w, uint32_t nx)
{
    uint32_t y = w | w << 1;
    y |= y << 2;
    y |= y << 4;
    y |= y << 8;
    y |= y << 6;                                 /* bit 31 - j: OR of bits j .. j + 21 (j <= 10) */
    const uint32_t tz = w ? (uint32_t)__builtin_ctz(w) : 32u, lz = nx ? (uint32_t)__builtin_clz(nx) : 32u;
    return (~y & 0xffe00000u) != 0u || tz + lz >= 22u;
}

/* the flush of an LDS window buf[0, n) = group words [p0, p0 + n) by a
 * block of nthr threads (a multiple of 64): the words to the group's
 * row-stage slot, and the words passing ep_quick to the group's record cg
 * (count in *ncand, LDS) -- one LDS atomic per wave that has any */
__device__ inline void flush_window(const uint32_t *buf, uint32_t n, uint32_t p0, bool last, uint32_t *out,
                                    uint32_t *ncand, uint32_t *cg, uint32_t cmax, int t, int nthr)
{
    const int lane = t & 63;
    for (uint32_t i0 = 0; i0 < n; i0 += (uint32_t)nthr) {
        const uint32_t i = i0 + (uint32_t)t;
        bool q = false;
        if (i < n) {
            const uint32_t w = buf[i];
            out[p0 + i] = w;                            /* MSB-first words */
            q = ep_quick(w, i + 1 < n ? buf[i + 1] : (last ? 0xffffffffu : 0u));
        }
        const uint64_t m = __builtin_amdgcn_ballot_w64(q);
        if (m) {
            uint32_t base = 0;
            if (lane == (int)__builtin_ctzll(m)) base = atomicAdd(ncand, (uint32_t)__builtin_popcountll(m));
            base = (uint32_t)__shfl((int)base, (int)__builtin_ctzll(m), 64);
            const uint32_t k = base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
            if (q && k < cmax) cg[1 + k] = p0 + i;
        }
    }
}

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
/* Pieces of dynamic MB q (rect raster order): pc 0..15 luma 4x4 (raster),  */
/* 16 / 17 Cb / Cr DC, 18 + 4p + b chroma AC (plane p, raster b).  A piece's */
/* meta (u16) = body bits | TotalCoeff << 8 | TrailingOnes << 13 | ovf << 15;*/
/* its body = the CAVLC bits after coeff_token right-aligned in 128 bits    */
/* (x = bits 0..31 .. w = bits 96..127; DC pieces hold the whole block).    */
/* ovf: more than 128 bits -- the body holds the levels instead (int8 scan  */
/* order; DC: int16) and the packer re-codes them.  k_dyn_row keeps them in */
/* LDS by slot q NPC + pc of its row; k_dyn_code_general's records live in  */
/* global memory at rec_of(q, pc) -- its task order: luma 16 q + pc, chroma */
/* AC 16 nd + 8 q + pc - 18, chroma DC 24 nd + 2 q + pc - 16 (nd = w h).    */
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
/* k_dyn_code_general: block records of the general-path NALs              */
/* ---------------------------------------------------------------------- */
/* NALs whose waypoint chain has a half-pel chroma step (k_dyn_rows flags
 * them; never for the waypoints the composer creates) predict chroma
 * through chroma_px_any, a bilinear tree too register-hungry for k_dyn_row.
 * Their blocks are coded here into records in global memory, which
 * k_dyn_row then packs.  Workgroup = 256 block tasks of one NAL: [0, 16 nd)
 * luma MB-major, [16 nd, 24 nd) chroma AC (MB, plane, raster 2x2; a quad's
 * lanes exchange their DC coefficients); levels, a counting sort on
 * TotalCoeff, then the CAVLC bodies largest first. */
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

__device__ inline void code_frame(const DevStream *__restrict__ st,
                                                     const DynFrame *__restrict__ dfr, int ld_fr,
                                                     const PlanPending *__restrict__ pend,
                                                     const NalDesc *__restrict__ nal, int ld_nal,
                                                     DynGeom g, const uint32_t *__restrict__ rows,
                                                     const uint8_t *__restrict__ src,
                                                     const uint8_t *__restrict__ refs,
                                                     uint16_t *__restrict__ meta, uint2 *__restrict__ blo,
                                                     uint2 *__restrict__ bhi, uint4 *__restrict__ bwd, int s,
                                                     int f, int bx)
{
    __shared__ uint4 lv[CODE_T];
    __shared__ int16_t lw[CODE_T][16];              /* below QP_MIN: the levels as int16 */
    __shared__ uint16_t wc[CODE_NW][SORT_KEYS];    /* per wave: blocks per TotalCoeff class */
    __shared__ uint16_t order[CODE_T];
    __shared__ PTabs ptabs;
    __shared__ int32_t wo[8], wv[8];
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const DynFrame df = dfr[(size_t)s * ld_fr + f];
    if (df.nal < 0 || !(df.err & DF_GENERAL)) return;
    load_ptabs(ptabs, t, CODE_T);
    if (t < 8) {
        wo[t] = pend[s].wo[t];
        wv[t] = pend[s].wv[t];
    }
    __syncthreads();

    const int ndt = g.w * g.h, ntask = 24 * ndt;
    const int task = bx * CODE_T + t;
    /* the stream's rect QP; below QP_MIN the levels need 16 bits (wide) */
    const int qpy = __builtin_amdgcn_readfirstlane(st[s].dyn_qp);
    const QParams ql = qparams_rt(qpy), qc = qparams_rt(qp_chroma(qpy));
    const bool wide = qpy < QP_MIN;
    const size_t nb = (size_t)s * ld_fr + f;
    const uint32_t *rw = rows + nb * (size_t)(32 * g.h);
    const int w = st[s].w, h = st[s].h;
    const uint32_t ysz = (uint32_t)w * (uint32_t)h, csz = ysz / 4;
    const uint8_t *rb = refs + (size_t)s * g.ref_ld;
    const uint8_t *fs = src + (size_t)s * g.src_ld + (size_t)f * g.src_fr;
    const int lstride = 16 * g.w, cstride = 8 * g.w;
    const uint8_t *fcb = fs + (size_t)256 * ndt, *fcr = fcb + (size_t)64 * ndt;
    const uint32_t m_rw = magic32((uint32_t)g.w);
    const size_t gs = df.rbsp_bytes;                    /* its record slot (k_dyn_rows) */
    uint16_t *M = meta + gs * (size_t)(NPC * ndt);
    uint2 *BL = blo + gs * (size_t)(NPC * ndt), *BH = bhi + gs * (size_t)(NPC * ndt);
    uint4 *BW = bwd + gs * (size_t)(NPC * ndt);

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
            sv[i] = ld32(sp + (size_t)i * lstride);
            pv[i] = ld32(pp + re[i]);
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
            const int v = quant(W[ZZ[k2]], ZZ[k2], ql);      /* |v| <= 127 at QP >= 22: int8 */
            pk[k2 >> 2] |= ((uint32_t)v & 255u) << (8 * (k2 & 3));
            if (wide) lw[t][k2] = (int16_t)v;
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
            const uint32_t sv = ld32(sp + (size_t)i * cstride);
            const uint32_t ea = re[i];
            int pred[4];
            if (!(ea & ROW_GEN)) {
                const uint32_t fr = (ea >> 28) & 7u;
                const uint32_t av = ld32(cp + (ea & ROW_OFF));
                const uint32_t bv = fr ? ld32(cp + (re[8 * g.h + i] & ROW_OFF)) : 0u;
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    const int a = (int)((av >> (8 * x)) & 255u), b = (int)((bv >> (8 * x)) & 255u);
                    pred[x] = ((8 - (int)fr) * a + (int)fr * b + 4) >> 3;
                }
            } else {
                {                               /* half-pel waypoint step: any depth */
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
            const int v = quant(W[ZZ[k2]], ZZ[k2], qc);
            pk[(k2 - 1) >> 2] |= ((uint32_t)v & 255u) << (8 * ((k2 - 1) & 3));
            if (wide) lw[t][k2 - 1] = (int16_t)v;
            n += v != 0;
        }
        if (wide) lw[t][15] = 0;
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
            dq[0] = quant_dc(d0 + d1 + d2 + d3, qc);
            dq[1] = quant_dc(d0 - d1 + d2 - d3, qc);
            dq[2] = quant_dc(d0 + d1 - d2 - d3, qc);
            dq[3] = quant_dc(d0 - d1 - d2 + d3, qc);
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
    const bool ul = tk < 16 * ndt;
    CapSink cap{0, 0, 0};
    int t1 = 0;
    bool ok = true;
    int tc = 0;
    if (tk < ntask && !wide) {
        tc = cavlc_body(cap, ptabs, v4, ul ? 16 : 15, t1, ok);
    } else if (tk < ntask) {
        /* 16-bit levels: the whole block through the coder's tables, its
         * coeff_token (at nC 0) skipped; over 128 bits the record keeps the
         * levels (32 bytes: BL, BH, BW) */
        const int max = ul ? 16 : 15;
        tc = tc_t1_of(lw[u], max, t1);
        uint32_t tv;
        int tl;
        coeff_token(g_tabs, tc, t1, 0, tv, tl);
        SkipSink<CapSink> sk{cap, (uint32_t)tl};
        cavlc_block(sk, g_tabs, lw[u], max, 0);
        ok = cap.n <= 128;
    }
    /* each lane stores its own block's record (task order, so a workgroup's
     * records are one contiguous range; un-sorting through LDS first was
     * measured 3 % slower: light waves waited at its barrier for the heavy one) */
    if (tk < ntask) {
        const uint16_t mm = ok ? (uint16_t)(cap.n | (uint32_t)tc << 8 | (uint32_t)t1 << 13)
                               : (uint16_t)((uint32_t)tc << 8 | (uint32_t)t1 << 13 | M_OVF);
        M[tk] = mm;
        uint4 ov = v4;                                  /* the levels of a > 128-bit body */
        if (wide && !ok) {
            const uint4 *l2 = reinterpret_cast<const uint4 *>(lw[u]);
            ov = l2[0];
            BW[tk] = l2[1];
        }
        if ((mm & 255u) || (mm & M_OVF))
            put_body(BL, BH, tk,
                     ok ? make_uint4((uint32_t)cap.lo, (uint32_t)(cap.lo >> 32), (uint32_t)cap.hi,
                                     (uint32_t)(cap.hi >> 32))
                        : ov,
                     (mm & 255u) > 64u || (mm & M_OVF));
    }
}

/* grid (chunks, CODE_GEN_Y): workgroup (c, y) codes chunk c of the flagged
 * NALs y, y + CODE_GEN_Y, ... of k_dyn_rows' list (ctr[1] of them, as
 * k_dyn_row<true> reads it): with none flagged a launch reads one word */
#ifndef SCROLL_CODE_GEN_Y
#define SCROLL_CODE_GEN_Y 64        /* 16 measured: the no-op launch 4.3 us, the step the same */
#endif
constexpr int CODE_GEN_Y = SCROLL_CODE_GEN_Y;
__global__ __launch_bounds__(CODE_T) void k_dyn_code_general(const DevStream *__restrict__ st,
                                                             const DynFrame *__restrict__ dfr, int ld_fr,
                                                             const PlanPending *__restrict__ pend,
                                                             const NalDesc *__restrict__ nal, int ld_nal,
                                                             DynGeom g, const uint32_t *__restrict__ rows,
                                                             const uint8_t *__restrict__ src,
                                                             const uint8_t *__restrict__ refs,
                                                             uint16_t *__restrict__ meta,
                                                             uint2 *__restrict__ blo, uint2 *__restrict__ bhi,
                                                             uint4 *__restrict__ bwd, const uint32_t *__restrict__ ctr)
{
    const uint32_t n = min(__builtin_amdgcn_readfirstlane(ctr[1]), g.gen_cap);
    for (uint32_t j = blockIdx.y; j < n; j += gridDim.y) {
        const uint32_t q = __builtin_amdgcn_readfirstlane(ctr[DYN_CTR_LIST + j]);
        const int s = (int)(q / (uint32_t)ld_fr), f = (int)(q - (uint32_t)s * (uint32_t)ld_fr);
        code_frame(st, dfr, ld_fr, pend, nal, ld_nal, g, rows, src, refs, meta, blo, bhi, bwd, s, f, blockIdx.x);
        __syncthreads();
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
/* MB heads and coeff_tokens of the dynamic NAL's row groups              */
/* ---------------------------------------------------------------------- */
/* A NAL's bits are: slice header, then per MB row the MB heads (one of 12
 * codeword classes) and, for dynamic MBs, coded_block_pattern,
 * mb_qp_delta and the present pieces (coeff_token from the neighbours'
 * TotalCoeff + the body k_dyn_row coded), then the stop bit. */

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

/* a tagged 8-byte granule, written through to the fabric (k_dyn_row's
 * TotalCoeff hand-off: epoch in the top 24 bits, read with sc1 polls) */
__device__ inline void lb_store(unsigned long long *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* first row-stage word of row group gi in its frame's region: the static
 * groups above (rs_static_words each), the rect rows (rs_row_words), the
 * static groups below */
__host__ __device__ inline uint64_t rs_group_words(const DynGeom &g, int nA, int gi)
{
    if (gi < nA) return (uint64_t)gi * g.rs_static_words;
    if (gi < nA + g.h) return (uint64_t)nA * g.rs_static_words + (uint64_t)(gi - nA) * g.rs_row_words;
    return (uint64_t)(gi - g.h) * g.rs_static_words + (uint64_t)g.h * g.rs_row_words;
}

/* the EP-candidate record of row group gi (EPC_ROW / EPC_STATIC words at the end of its
 * row-stage slot, after the group's provable bits) */
__host__ __device__ inline uint64_t rs_runs_words(const DynGeom &g, int nA, int gi)
{
    const bool row = gi >= nA && gi < nA + g.h;
    return rs_group_words(g, nA, gi) + (row ? g.rs_row_words - EPC_ROW : g.rs_static_words - EPC_STATIC);
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

/* one-wave workgroups: LDS hand-offs need ordering, not a workgroup barrier
 * (whose release fence would also wait for every global store of the wave) */
__device__ inline void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* a > 128-bit block from its levels (rare): measure / write.  bd: 16 int8
 * levels (chroma DC: 4 int16); bw != nullptr: the 16-bit form of the
 * general path below QP_MIN -- bd levels 0-7, *bw levels 8-15, int16 */
template <class S>
__device__ inline void ovf_code(S &sk, const PTabs &PT, const Tabs &TB, uint4 bd, const uint4 *bw, int pc, int nC)
{
    if (nC == -1) {
        const int dq[4] = {(int)(int16_t)(bd.x & 0xffffu), (int)(int16_t)(bd.x >> 16),
                           (int)(int16_t)(bd.y & 0xffffu), (int)(int16_t)(bd.y >> 16)};
        cavlc_dc4(sk, PT, dq);
    } else if (bw) {
        const uint4 hi = *bw;
        const uint32_t w8[8] = {bd.x, bd.y, bd.z, bd.w, hi.x, hi.y, hi.z, hi.w};
        int16_t l16[16];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            l16[2 * i] = (int16_t)(w8[i] & 0xffffu);
            l16[2 * i + 1] = (int16_t)(w8[i] >> 16);
        }
        cavlc_block(sk, TB, l16, pc < 16 ? 16 : 15, nC);
    } else {
        const int8_t *lvp = reinterpret_cast<const int8_t *>(&bd);
        cavlc_block(sk, TB, lvp, pc < 16 ? 16 : 15, nC);
    }
}

__device__ __attribute__((noinline)) uint32_t ovf_bits(const PTabs &PT, const Tabs &TB, uint4 bd, const uint4 *bw,
                                                       int pc, int nC)
{
    CountSink cn{0};
    ovf_code(cn, PT, TB, bd, bw, pc, nC);
    return cn.n;
}

/* the sink lives in the callee: a sink passed by reference would be kept in
 * scratch memory by the caller on its every put */
__device__ __attribute__((noinline)) void ovf_put(uint32_t *buf, uint32_t lo, uint32_t n, uint32_t pos,
                                                  const PTabs &PT, const Tabs &TB, uint4 bd, const uint4 *bw, int pc,
                                                  int nC)
{
    WSink sk{LdsOrWin{buf, lo, n}, 0, 0, 0};
    sk.start(pos);
    ovf_code(sk, PT, TB, bd, bw, pc, nC);
    sk.finish();
}

/* a block body of n <= 128 bits held right-aligned in hi:lo -> four words,
 * MSB first, left-aligned (k_dyn_row's LDS form: the piece writer then
 * needs only funnel shifts by the token length and the bit position) */
__device__ inline uint4 body_msb(uint64_t hi, uint64_t lo, uint32_t n)
{
    const uint32_t k = 128u - n;
    uint64_t H, Lw;
    if (k >= 64u) {
        H = k >= 128u ? 0ull : lo << (k - 64u);
        Lw = 0ull;
    } else {
        H = k ? (hi << k) | (lo >> (64u - k)) : hi;
        Lw = lo << k;
    }
    return make_uint4((uint32_t)(H >> 32), (uint32_t)H, (uint32_t)(Lw >> 32), (uint32_t)Lw);
}

/* ---------------------------------------------------------------------- */
/* k_dyn_static: the static row groups of a dynamic NAL                    */
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
                                                  uint32_t *__restrict__ rows, uint32_t *__restrict__ ctr,
                                                  uint4 *__restrict__ heads)
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
    if (t < 12) {
        /* the NAL's 12 MB-head classes, MSB first, for every
         * rect row of k_dyn_row (which computed them once per row before):
         * vectors 0-11 the bits, 12-14 the lengths (bit 31: over 128 bits,
         * the row then writes its heads through the bit sink) */
        const HeadCtx H = head_ctx(c);
        CapSink hc{0, 0, 0};
        H.put_class(hc, t);
        uint4 *hv = heads + ((size_t)s * ld_fr + f) * DYN_HEAD_VECS;
        hv[t] = body_msb(hc.hi, hc.lo, min(hc.n, 128u));
        reinterpret_cast<uint32_t *>(hv + 12)[t] = hc.n | (hc.over() ? 0x80000000u : 0u);
    }
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
    if (my_gen || S->dyn_qp < QP_MIN) gen = 1;            /* half-pel chroma chains; 16-bit levels */
    __syncthreads();
    if (t == 0) {
        /* a general-path NAL takes a record slot (index in rbsp_bytes until
         * k_dyn_epfix); none left: the frame fails (DF_OVER, the batch
         * grows the pool for the next compose) */
        uint32_t e = 0u;
        if (gen) {
            const uint32_t k = atomicAdd(&ctr[1], 1u);
            if (k < g.gen_cap) {
                DF->rbsp_bytes = k;
                ctr[DYN_CTR_LIST + k] = (uint32_t)((size_t)s * ld_fr + f);   /* k_dyn_row<true>'s list */
                e = DF_GENERAL;
            } else {
                e = DF_OVER;
            }
        }
        DF->err = e;
        DF->ep = 0u;                                    /* k_dyn_epfix sets it */
    }
}

/* ---------------------------------------------------------------------- */
/* A NAL's bits are: slice header, then per MB row the MB heads (one of 12
 * codeword classes) and, for dynamic MBs, coded_block_pattern,
 * mb_qp_delta and the present pieces, then the stop bit.  Its MB rows are
 * row groups: g < nA the rows above the rect, DYN_STATIC_ROWS per group (the
 * first one holds the slice header and exists even with no rows), then one
 * per rect row (k_dyn_row), then the static groups below (the last one
 * holds rbsp_stop_one_bit).  Every group writes its own bits from bit 0 of
 * its row-stage slot and its bit count; k_dyn_epfix places them. */
constexpr int GW = 64;
#ifndef SCROLL_GBUF_WORDS
#define SCROLL_GBUF_WORDS 256
#endif
constexpr int GBUF_WORDS = SCROLL_GBUF_WORDS;   /* 8 Kbit per pass */

#ifndef SCROLL_STATIC_WORDS
#define SCROLL_STATIC_WORDS 1       /* static rows word by word from the head patterns (0: MB by MB) */
#endif

struct StaticFixed {
    uint32_t ncand;
    uint32_t buf[GBUF_WORDS];
    uint64_t hhi[12], hlo[12];
    uint4 pat[12];                  /* head class + coded_block_pattern '1', MSB first (hlen + 1 <= 128) */
    uint32_t hlen[12];
    int32_t head_over;
    int32_t wo[8], wl[8], wv[8];
    uint32_t moff[DYN_STATIC_ROWS + 1];
};

/* grid (nA + nB, frames, streams), one wave each */
__global__ __launch_bounds__(GW) void k_dyn_static(const DevStream *__restrict__ st,
                                                   const NalDesc *__restrict__ nal, int ld_nal,
                                                   const PlanPending *__restrict__ pend,
                                                   const DynFrame *__restrict__ dfr, int ld_fr, DynGeom g,
                                                   uint32_t *__restrict__ rowstage, uint32_t *__restrict__ gbits)
{
    __shared__ StaticFixed L;
    constexpr int SR = DYN_STATIC_ROWS;
    const Rect R{g.x0, g.y0, g.w, g.h};
    const int nA = max(1, (R.y0 + SR - 1) / SR);
    const int gi = (int)blockIdx.x >= nA ? (int)blockIdx.x + R.h : (int)blockIdx.x;
    const int ng = g.ngroups, f = blockIdx.y, s = blockIdx.z, t = threadIdx.x;
    const size_t nb = (size_t)s * ld_fr + f;
    const int j = dfr[nb].nal;
    if (j < 0) return;
    const bool first = gi == 0, last = gi == ng - 1;
    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    if (t == 0) {
        L.head_over = 0;
        L.ncand = 0;
    }
    const DevStream *S = st + s;
    const NalDesc d = nal[(size_t)s * ld_nal + j];
    wave_sync();
    NalCtx c = nal_ctx(S, d, L.wo, L.wl, L.wv);
    c.qpd = S->dyn_qp - QP_DEFAULT;                     /* the stream's rect QP: slice_qp_delta */
    const HeadCtx H = head_ctx(c);
    const int mbw = H.mbw, mbh = c.h / 16;
    int ra, rb;
    if (gi < nA) {
        ra = gi * SR;
        rb = min(ra + SR, R.y0);
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
        if (hc.n < 128u) {                              /* the class's bits and the cbp '1' */
            const uint64_t hi = (hc.hi << 1) | (hc.lo >> 63), lo = (hc.lo << 1) | 1u;
            L.pat[t] = body_msb(hi, lo, hc.n + 1u);
        } else {
            L.head_over = 1;                            /* (the word path needs patterns of <= 128 bits) */
        }
    }
    wave_sync();
    const bool head_over = L.head_over;
    auto head_bits = [&](int r, int col) -> uint32_t {
        if (!head_over) return L.hlen[H.sel(r, col)];
        CountSink cn{0};
        H.put_slow(cn, r, col);
        return cn.n;
    };
    /* row offsets (rows <= SR: one wave scan) */
    uint32_t len = 0;
    const int r = ra + t;
    if (r < rb) {
        if (!head_over) {
            len = row_static_bits(H, L.hlen, r, R);
        } else {
            for (int col = 0; col < mbw; ++col) len += head_bits(r, col) + 1u;
        }
    }
    const uint32_t incl = wave_incl_sum(len, t);
    if (r < rb) L.moff[r - ra] = F + incl - len;
    const uint32_t rows_end = F + __shfl(incl, GW - 1, GW);
    if (t == 0) L.moff[rb - ra] = rows_end;
    const uint32_t bits = rows_end + (last ? 1u : 0u);
    if (t == 0) gbits[nb * (size_t)ng + gi] = bits;
    wave_sync();

    uint32_t *out = rowstage + nb * g.rs_frame_words + rs_group_words(g, nA, gi);
    const uint32_t nw = min((bits + 31u) >> 5, g.rs_static_words - EPC_STATIC);   /* provable bound: never clipped */
    const int ne = rb - ra;
    auto cnt_le = [&](uint32_t x) -> int {              /* # e in [0, ne] with moff[e] <= x */
        int lo = 0, hi = ne + 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (L.moff[mid] <= x) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const uint32_t m_mbw = magic32((uint32_t)mbw);
    for (uint32_t p0 = 0; p0 < nw; p0 += GBUF_WORDS) {
        const uint32_t n = min((uint32_t)GBUF_WORDS, nw - p0);
        for (uint32_t i = (uint32_t)t; i < n; i += GW) L.buf[i] = 0u;
        wave_sync();
        const LdsOrWin win{L.buf, p0, n};
        if (!(SCROLL_STATIC_WORDS && !head_over) && first && t == 0 && p0 * 32u < F) {   /* slice header, h264_writer.c:549-553 */
            WSink hs{win, 0, 0, 0};
            hs.start(0);
            emit_slice_header(hs, c);
            hs.finish();
        }
        if (SCROLL_STATIC_WORDS && !head_over) {
            /* word by word: a static row is its first column's head, mbw - 2
             * copies of the middle class's, the last column's (each with the
             * cbp '1': the patterns); a lane builds whole words of the window
             * from the patterns the word's bits fall in (plain stores; the
             * slice header and the stop bit are ORed in after) */
            const uint32_t rbeg = L.moff[0], rend = L.moff[ne];
            for (uint32_t i = (uint32_t)t; i < n; i += GW) {
                const uint32_t W0 = 32u * (p0 + i), W1 = W0 + 32u;
                uint32_t acc = 0, b = max(W0, rbeg), R0 = 0, R1 = 0, L0 = 0, Lm = 1;
                int b3 = 0;
                float inv = 1.0f;
                while (b < W1 && b < rend) {
                    if (b >= R1 || b < R0) {                    /* the row holding bit b */
                        const int e = cnt_le(b) - 1;
                        R0 = L.moff[e];
                        R1 = L.moff[e + 1];
                        b3 = H.sel(ra + e, 0);
                        L0 = L.hlen[b3] + 1u;
                        Lm = L.hlen[b3 + 1] + 1u;
                        inv = 1.0f / (float)Lm;
                    }
                    const uint32_t o = b - R0;
                    uint32_t cl = (uint32_t)b3, off = o;
                    if (o >= L0) {
                        const uint32_t o2 = o - L0;
                        uint32_t q = (uint32_t)((float)o2 * inv);   /* o2 < 2^24: off by at most one */
                        if (q * Lm > o2) --q;
                        else if ((q + 1u) * Lm <= o2) ++q;
                        if (q < (uint32_t)(mbw - 2)) {
                            cl = (uint32_t)b3 + 1u;
                            off = o2 - q * Lm;
                        } else {
                            cl = (uint32_t)b3 + 2u;
                            off = o2 - (uint32_t)(mbw - 2) * Lm;
                        }
                    }
                    const uint32_t k = min(L.hlen[cl] + 1u - off, W1 - b);
                    const uint4 P = L.pat[cl];
                    const uint32_t wi = off >> 5, sh = off & 31u;
                    const uint32_t w0 = wi == 0 ? P.x : (wi == 1 ? P.y : (wi == 2 ? P.z : P.w));
                    const uint32_t w1 = wi == 0 ? P.y : (wi == 1 ? P.z : (wi == 2 ? P.w : 0u));
                    uint32_t v = sh ? __builtin_amdgcn_alignbit(w0, w1, 32u - sh) : w0;
                    v &= k >= 32u ? 0xffffffffu : ~(0xffffffffu >> k);
                    acc |= v >> (b - W0);
                    b += k;
                }
                L.buf[i] = acc;
            }
            wave_sync();
            if (first && t == 0 && p0 * 32u < F) {      /* slice header, h264_writer.c:549-553 */
                WSink hs{win, 0, 0, 0};
                hs.start(0);
                emit_slice_header(hs, c);
                hs.finish();
            }
            if (last && t == 0) {                       /* rbsp_stop_one_bit */
                WSink sk{win, 0, 0, 0};
                sk.start(bits - 1u);
                sk.put(1, 1);
                sk.finish();
            }
            wave_sync();
            flush_window(L.buf, n, p0, p0 + n >= nw, out, &L.ncand,
                         rowstage + nb * g.rs_frame_words + rs_runs_words(g, nA, gi), EPC_STATIC - 1, t, GW);
            wave_sync();
            continue;
        }
        /* the rows whose bits meet the window: [ea, eb) */
        const int ea = max(cnt_le(32u * p0) - 1, 0), eb = min(cnt_le(32u * (p0 + n) - 1u), ne);
        const int nm = eb * mbw;
        for (int m = ea * mbw + t; m < nm; m += GW) {
            const int rr = (int)div_m((uint32_t)m, m_mbw), col = m - rr * mbw, rw = ra + rr;
            uint32_t off = L.moff[rr];
            WSink sk{win, 0, 0, 0};
            if (!head_over) {
                const int b3 = H.sel(rw, 0);
                off += col == 0 ? 0u : L.hlen[b3] + 1u + (uint32_t)(col - 1) * (L.hlen[b3 + 1] + 1u);
                if (off >= 32u * (p0 + n)) continue;
                const int cls = b3 + (col == 0 ? 0 : (col == mbw - 1 ? 2 : 1));
                if (off + L.hlen[cls] + 1u <= 32u * p0) continue;
                sk.start(off);
                sk.put_cap(CapSink{L.hhi[cls], L.hlo[cls], L.hlen[cls]});
            } else {
                for (int c2 = 0; c2 < col; ++c2) off += head_bits(rw, c2) + 1u;
                sk.start(off);
                H.put_slow(sk, rw, col);
            }
            sk.put(1, 1);                               /* coded_block_pattern ue(0) */
            sk.finish();
        }
        if (last && t == 0) {                           /* rbsp_stop_one_bit */
            WSink sk{win, 0, 0, 0};
            sk.start(bits - 1u);
            sk.put(1, 1);
            sk.finish();
        }
        wave_sync();
        flush_window(L.buf, n, p0, p0 + n >= nw, out, &L.ncand,
                     rowstage + nb * g.rs_frame_words + rs_runs_words(g, nA, gi), EPC_STATIC - 1, t, GW);
        wave_sync();
    }
    if (t == 0) rowstage[nb * g.rs_frame_words + rs_runs_words(g, nA, gi)] = L.ncand;
}


/* body_msb's inverse for the MB-head classes k_dyn_row keeps MSB first
 * (a = words 0-1, b = words 2-3): the n bits right-aligned (CapSink) */
__device__ inline CapSink cap_of_msb(uint64_t a, uint64_t b, uint32_t n)
{
    if (n == 0u) return CapSink{0, 0, 0};
    const uint32_t sh = 128u - n;
    if (sh >= 64u) return CapSink{0, a >> (sh - 64u), n};
    if (sh == 0u) return CapSink{a, b, n};
    return CapSink{a >> sh, (b >> sh) | (a << (64u - sh)), n};
}

/* token (tl <= 16 bits) + MSB-first body b (bl <= 128 bits) ORed into the
 * LDS window buf = words [p0, p0 + n) at bit pos: the <= 144 bits as five
 * words shifted by tl, then six words shifted by pos mod 32 (v_alignbit);
 * words outside the window are dropped (the next pass writes them) */
__device__ inline void put_piece(uint32_t *buf, uint32_t p0, uint32_t n, uint32_t pos, uint32_t tv, uint32_t tl,
                                 uint4 b, uint32_t bl)
{
    const uint32_t tw = tv & low_mask((int)tl);
    const uint32_t c0 = __builtin_amdgcn_alignbit(tw, b.x, tl), c1 = __builtin_amdgcn_alignbit(b.x, b.y, tl);
    const uint32_t c2 = __builtin_amdgcn_alignbit(b.y, b.z, tl), c3 = __builtin_amdgcn_alignbit(b.z, b.w, tl);
    const uint32_t c4 = __builtin_amdgcn_alignbit(b.w, 0u, tl);
    const uint32_t sh = pos & 31u;
    const uint32_t o[6] = {c0 >> sh, __builtin_amdgcn_alignbit(c0, c1, sh), __builtin_amdgcn_alignbit(c1, c2, sh),
                           __builtin_amdgcn_alignbit(c2, c3, sh), __builtin_amdgcn_alignbit(c3, c4, sh),
                           __builtin_amdgcn_alignbit(c4, 0u, sh)};
    const uint32_t nw = (sh + tl + bl + 31u) >> 5, w0 = (pos >> 5) - p0;
#pragma unroll
    for (uint32_t j = 0; j < 6; ++j)
        if (j < nw && w0 + j < n && o[j]) atomicOr(&buf[w0 + j], o[j]);
}

/* put_piece for a row written in one pass (the window is the row's words
 * from 0, with ROW_PAD spare words after it): the first SCROLL_PUT_FIRST
 * words ORed whatever the piece's length (zero words past its end change
 * nothing), the rest only for pieces that reach them -- no window tests.
 * Round 6: 1 instead of 3 -- a zero OR into the word the next lane's piece
 * starts in is a same-address LDS conflict (k_dyn_row's conflicts 112 ->
 * 91 M per config-3 launch, its time equal within noise) */
constexpr uint32_t ROW_PAD = 4;

/* SCROLL_LV_SWZ=1 (measured, not kept): k_dyn_row's level records between
 * the sort and the CAVLC bodies with dword d of the record in slot s at
 * d ^ lv_key(s) (an involution), swizzled in the sort's pass -- LDS bank
 * conflicts 91 -> 68 M per config-3 launch, but k_dyn_row 1.206 -> 1.232 ms
 * (the extra record read / permute / write per block costs more than the
 * conflicts did; profiles/r06j_lds_swizzle_p720dyn.txt) */
#ifndef SCROLL_LV_SWZ
#define SCROLL_LV_SWZ 0
#endif
__device__ inline uint32_t lv_key(int slot) { return ((uint32_t)slot >> 4) & 3u; }
__device__ inline uint4 lv_swz(uint4 v, uint32_t key)
{
    if (key & 1u) v = make_uint4(v.y, v.x, v.w, v.z);
    if (key & 2u) v = make_uint4(v.z, v.w, v.x, v.y);
    return v;
}
__device__ inline void put_piece1(uint32_t *buf, uint32_t pos, uint32_t tv, uint32_t tl, uint4 b, uint32_t bl)
{
    const uint32_t tw = tv & low_mask((int)tl);
    const uint32_t c0 = __builtin_amdgcn_alignbit(tw, b.x, tl), c1 = __builtin_amdgcn_alignbit(b.x, b.y, tl);
    const uint32_t c2 = __builtin_amdgcn_alignbit(b.y, b.z, tl), c3 = __builtin_amdgcn_alignbit(b.z, b.w, tl);
    const uint32_t c4 = __builtin_amdgcn_alignbit(b.w, 0u, tl);
    const uint32_t sh = pos & 31u, nw = (sh + tl + bl + 31u) >> 5;
    uint32_t *d = buf + (pos >> 5);
#ifndef SCROLL_PUT_FIRST
#define SCROLL_PUT_FIRST 1       /* words ORed whatever the length (round 6: 3 -> 1, fewer same-address ORs) */
#endif
    atomicOr(d, c0 >> sh);
    if (SCROLL_PUT_FIRST >= 2 || nw > 1u) atomicOr(d + 1, __builtin_amdgcn_alignbit(c0, c1, sh));
    if (SCROLL_PUT_FIRST >= 3 || nw > 2u) atomicOr(d + 2, __builtin_amdgcn_alignbit(c1, c2, sh));
    if (nw > 3u) {
        atomicOr(d + 3, __builtin_amdgcn_alignbit(c2, c3, sh));
        if (nw > 4u) {
            atomicOr(d + 4, __builtin_amdgcn_alignbit(c3, c4, sh));
            if (nw > 5u) atomicOr(d + 5, __builtin_amdgcn_alignbit(c4, 0u, sh));
        }
    }
}

/* ---------------------------------------------------------------------- */
/* k_dyn_row: one workgroup per rect MB row of a NAL                       */
/* ---------------------------------------------------------------------- */
/* Block coding and row packing in one workgroup: the row's 24 w block
 * tasks are one thread each (two for rects over 42 MBs wide), their
 * records never leave LDS.
 *   1. residual -> transform -> quant -> levels (LDS), chroma DC 2x2;
 *      the row's bottom TotalCoeffs go out as one tagged 8-byte granule
 *      per MB (the row below waits for them: its top neighbours, the only
 *      hand-off between workgroups);
 *   2. counting sort on TotalCoeff, CAVLC bodies in that order (each
 *      wave's loop runs about its own blocks' count);
 *   3. coeff_token per piece from the left / top TotalCoeffs (nC);
 *   4. per MB cbp, its code and the piece offsets; the row's MB offsets;
 *   5. the row's bits -> LDS window -> its own row-stage words, from bit 0
 *      (no position known yet: k_dyn_epfix places every row group), with
 *      the words that may hold an EP site recorded for k_dyn_epfix.
 * The static row groups (slice header, rows above / below the rect, stop
 * bit) are k_dyn_static's.  NALs whose chroma prediction needs the general
 * path (k_dyn_rows flags them) take their records from k_dyn_code_general
 * in global memory instead of steps 1-2. */
constexpr int ROW_MAXT = 1024;
/* waves per SIMD the register allocation targets: 8 (eight row workgroups
 * per CU; the SGPR budget then spills some uniform values to VGPR lanes).
 * With the general path in its own instantiation the normal one needs 53
 * VGPRs and 8 beat 7 (1.43 against 1.50 ms); with both paths in one kernel
 * (63 VGPRs) the spills ate the gain */
#ifndef SCROLL_ROW_WAVES
#define SCROLL_ROW_WAVES 8
#endif
/* block tasks per thread (about: threads = 24 w / NP rounded up to waves):
 * 3 for rows up to SCROLL_ROW_WIDE MBs, SCROLL_ROW_NP_WIDE past it.  Config
 * 3's 25-MB rows: 1.29 ms at 3 against 1.41 at 4 or 5; config 5's 47-MB
 * rows: 2.72 ms at 4 against 2.86 at 3 and 2.81 at 5 (round 5) */
#ifndef SCROLL_ROW_NP
#define SCROLL_ROW_NP 3
#endif
#ifndef SCROLL_ROW_NP_WIDE
#define SCROLL_ROW_NP_WIDE 4
#endif
#ifndef SCROLL_ROW_WIDE
#define SCROLL_ROW_WIDE 40
#endif
constexpr int ROW_NPMAX = 8;                    /* tasks per thread at most (1536 tasks / 192) */
#ifndef SCROLL_ROW_GB
#define SCROLL_ROW_GB 896
#endif
constexpr int ROW_GB = SCROLL_ROW_GB;           /* bit window: 28 Kbit (a config-3 row ~18 Kbit, one pass) */

struct RowFixed {
    RowTabs ptabs;
    union {                                      /* the sort's counts and the level table are dead before the bit window */
        uint32_t buf[ROW_GB + 4];                /* + ROW_PAD: put_piece1's spare words */
        struct {
            uint32_t kc[2][SORT_KEYS];           /* the sort: blocks per TotalCoeff class, then its base */
            uint32_t kc_pad[32 - 2 * SORT_KEYS];
            uint32_t lvt[LVT_N];                 /* level codewords (CAVLC phase) */
        };
    };
    uint64_t hhi[12], hlo[12];
    uint32_t hlen[12];
    int32_t wo[8], wl[8], wv[8];
    int32_t head_over;
    uint32_t rt[32];                             /* the row's prediction-row table (k_dyn_rows) */
    uint32_t ncand;                              /* EP candidate words of the row */
    uint32_t spill;                              /* its spill slot (a row over its slot) */
    uint32_t pcd[NPC];                           /* per piece class: its nC neighbours (pc_desc) */
};

static_assert(2 * SORT_KEYS <= 32 && 32 + LVT_N <= ROW_GB, "the sort counts and the level table share the bit window");
static_assert(ROW_PAD == 4, "RowFixed::buf holds ROW_PAD spare words");
static_assert(offsetof(RowFixed, lvt) % 8 == 0, "the level table is copied in 8-byte words");

/* dynamic LDS of k_dyn_row: lv [NPC w] uint4 (levels, then bodies), moff
 * [w + 1] u32 (the rect columns' bit offsets in the row; the static
 * columns' are closed forms of their three head classes), mt / lo / off16
 * [NPC w] u16 (the sort's order [24 w] u16 lives in off16 until phase 4), ta
 * [8 w] u8 (top TotalCoeffs; from phase 4 on the MBs' bit counts, u32 [w]),
 * cbp / code [w] u8.  (Round 4 kept moff for every column of the picture:
 * 964 bytes more at 4K, config 5's row workgroups needed 33.5 KB) */
__host__ __device__ inline size_t row_lds_base(int w)
{
    return (size_t)16 * NPC * w + (size_t)4 * (w + 1) + (size_t)2 * (3 * NPC * w) + (size_t)10 * w + 16;
}
/* rows over SCROLL_ROW_WIDE MBs write through a wider bit window of
 * ROW_GB_WIDE words at the end of the dynamic LDS (when the workgroup still
 * fits the CU's 160 KB): config 5's 47-MB rows (about 37 Kbit) in one pass
 * instead of two, 2.70 -> 2.49 ms per launch; config 3 keeps the static
 * window (its 8 workgroups per CU have no LDS to spare) */
#ifndef SCROLL_ROW_GB_WIDE
#define SCROLL_ROW_GB_WIDE 1248
#endif
constexpr int ROW_GB_WIDE = SCROLL_ROW_GB_WIDE;
__host__ __device__ inline size_t row_wide_off(int w) { return (row_lds_base(w) + 15) & ~(size_t)15; }
__host__ __device__ inline bool row_wide_win(int w)
{
    return w > SCROLL_ROW_WIDE && row_wide_off(w) + 4 * (size_t)(ROW_GB_WIDE + ROW_PAD) + sizeof(RowFixed) <= 163840;
}
__host__ __device__ inline size_t row_lds_bytes(int w)
{
    return row_wide_win(w) ? row_wide_off(w) + 4 * (size_t)(ROW_GB_WIDE + ROW_PAD) : row_lds_base(w);
}

/* The nC neighbours of piece class pc (0-15 luma raster, 16 / 17 chroma DC,
 * 18 + 4 p + b chroma AC), relative to the piece's slot i = k NPC + pc:
 * bits 0-5 the left neighbour's slot - i + 32 (same MB, or the left MB's
 * right column), bit 6 it is in the left MB, bits 7-12 the top neighbour's
 * slot - i + 32 (same MB), bit 13 it is in the row above (then bits 14-16
 * its index in the row's top TotalCoeffs ta[8 k + e]), bit 17 chroma DC
 * (nC = -1). */
__host__ __device__ constexpr uint32_t pc_desc(int pc)
{
    if (pc == 16 || pc == 17) return 1u << 17;
    int da = 0, db = 0, e = 0;
    bool al = false, bt = false;
    if (pc < 16) {
        const int bx = pc & 3, by = pc >> 2;
        al = bx == 0;
        da = al ? 3 - NPC : -1;
        bt = by == 0;
        db = bt ? 0 : -4;
        e = bt ? pc : 0;
    } else {
        const int b = (pc - 18) & 3, bx = b & 1, by = b >> 1;
        al = bx == 0;
        da = al ? 1 - NPC : -1;
        bt = by == 0;
        db = bt ? 0 : -2;
        e = bt ? (pc < 22 ? pc - 14 : pc - 16) : 0;
    }
    return (uint32_t)(da + 32) | (al ? 1u : 0u) << 6 | (uint32_t)(db + 32) << 7 | (bt ? 1u : 0u) << 13 |
           (uint32_t)e << 14;
}

/* LDS of ep_fix: the row-group table, candidate bases, the position
 * bitmap / list (ep_fix's LCAP words) and four counters */
struct EpfLds {
    uint32_t *goff, *gb, *gw, *cw, *cbase, *lst, *cnt;    /* goff / cbase 65, gb / gw / cw 64, cnt 4 */
    uint32_t *ws;                                          /* per wave: the unique-position scan */
};
/* k_dyn_row's block tasks: luma [0, 16 w), chroma AC from the next wave
 * boundary row_chroma0(w) on, so that every wave-pass is all luma or all
 * chroma (uniform branches and per-wave fetch offsets, no exec-mask split) */
__host__ __device__ inline int row_chroma0(int w) { return (16 * w + 63) & ~63; }
__host__ __device__ inline int row_vtasks(int w) { return row_chroma0(w) + 8 * w; }

/* threads of a k_dyn_row workgroup: about SCROLL_ROW_NP block tasks each */
__host__ __device__ inline int row_threads(int w)
{
    const int nt = row_vtasks(w), np = w > SCROLL_ROW_WIDE ? SCROLL_ROW_NP_WIDE : SCROLL_ROW_NP;
    const int a = (((nt + np - 1) / np) + 63) & ~63;
    const int b = (((nt + ROW_NPMAX - 1) / ROW_NPMAX) + 63) & ~63;      /* np <= ROW_NPMAX */
    const int t = a > b ? a : b;
    return t < ROW_MAXT ? t : ROW_MAXT;
}

/* The pixels of a block task: a = source rows, b = prediction rows (chroma:
 * the upper bilinear rows), c = the lower bilinear row of b[3] (chroma with
 * a fraction only; the lower row of b[i < 3] is b[i + 1]: both are the
 * chroma row after it through the same waypoint chain, k_dyn_rows) */
struct BlkPix {
    uint32_t a[4], b[4], c;
};

/* raw buffer descriptor over n bytes at p (gfx9 dword3: 32-bit data format) */
__device__ inline __amdgpu_buffer_rsrc_t buf_rsrc(const void *p, uint32_t n)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)n, 0x00020000);
}

/* A wave's fetch offsets (lane offsets into the frame's source / the
 * stream's reference pair) for the tasks of pass pb; pass q's tasks are T q
 * further on, and with T a multiple of 64 a task's position in its MB
 * (luma) or chroma quad (chroma) is the same in every pass and both its
 * byte offsets advance by exactly T q (16 k and 8 k both grow by T).  So the
 * per-pass advance and the row strides go in the uniform soffset: a pass's
 * eight (twelve) loads cost no vector instruction.  One set of registers,
 * reloaded when the wave's tasks turn from luma to chroma (once). */
struct FetchOff {
    uint32_t s, b[4], c;        /* source row 0; prediction rows; the lower bilinear row of b[3] */
    int pb;                     /* the pass they are for (uniform) */
};

/* luma task v (MB k = v / 16, raster block v % 16) of rect row ry; rt = the
 * row's 16 luma prediction rows (LDS, or k_dyn_rows' table in global memory) */
[[maybe_unused]] __device__ inline void fetch_luma(FetchOff &o, int v, int ry, const DynGeom &g, const uint32_t *rt)
{
    const int k = v >> 4, r = v & 15, bx = r & 3, by = r >> 2;
    o.s = (uint32_t)((16 * ry + 4 * by) * (16 * g.w) + 16 * k + 4 * bx);
    const uint32_t po = (uint32_t)(16 * (g.x0 + k) + 4 * bx);
#pragma unroll
    for (int i = 0; i < 4; ++i) o.b[i] = po + rt[4 * by + i];
    o.c = o.b[3];
}

/* chroma AC task e (MB e / 8, plane (e / 4) % 2, raster block e % 4); ru /
 * rd = the row's 8 upper / lower bilinear rows */
[[maybe_unused]] __device__ inline void fetch_chroma(FetchOff &o, int e, int ry, const DynGeom &g, uint32_t csz, const uint32_t *ru,
                                    const uint32_t *rd)
{
    const int ndt = g.w * g.h, k = e >> 3, p = (e >> 2) & 1, r = e & 3, bx = r & 1, by = r >> 1;
    o.s = (uint32_t)(256 * ndt + (p ? 64 * ndt : 0) + (8 * ry + 4 * by) * (8 * g.w) + 8 * k + 4 * bx);
    const uint32_t co = (uint32_t)p * csz + (uint32_t)(8 * (g.x0 + k) + 4 * bx);
#pragma unroll
    for (int i = 0; i < 4; ++i) o.b[i] = co + (ru[4 * by + i] & ROW_OFF);
    o.c = co + (rd[4 * by + 3] & ROW_OFF);
}

/* the loads of pass q (soffset = T (q - pb) + the row stride term).  Lanes
 * past the row's tasks load too: their offsets stay inside the frame's
 * source / the reference pair or read 0 past the descriptor (raw buffer
 * range check), and their results are never stored.  Chroma always loads
 * its lower row (used only with a fraction): no wait for the fraction */
[[maybe_unused]] __device__ inline void fetch_pass(const FetchOff &o, bool luma, uint32_t adv, uint32_t stride,
                                  __amdgpu_buffer_rsrc_t fs, __amdgpu_buffer_rsrc_t rb, BlkPix &px)
{
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        px.a[i] = __builtin_amdgcn_raw_buffer_load_b32(fs, o.s, adv + (uint32_t)i * stride, 0);
        px.b[i] = __builtin_amdgcn_raw_buffer_load_b32(rb, o.b[i], adv, 0);
    }
    px.c = luma ? 0u : __builtin_amdgcn_raw_buffer_load_b32(rb, o.c, adv, 0);
}
/* the same with the ninth load for luma too (o.c = o.b[3]; its value unused):
 * every pass issues nine loads (k_dyn_row's counted waits) */
[[maybe_unused]] __device__ inline void fetch_pass9(const FetchOff &o, uint32_t adv, uint32_t stride, __amdgpu_buffer_rsrc_t fs,
                                   __amdgpu_buffer_rsrc_t rb, BlkPix &px)
{
#ifdef SCROLL_ABL_NOLOAD
    /* profiling variant only: no pixel loads (values from the offsets), the
     * ceiling of any change to how the pixels are fetched */
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        px.a[i] = (o.s + adv + (uint32_t)i * stride) * 0x9e3779b1u;
        px.b[i] = (o.b[i] + adv) * 0x85ebca6bu;
    }
    px.c = o.c + adv;
    return;
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        px.a[i] = __builtin_amdgcn_raw_buffer_load_b32(fs, o.s, adv + (uint32_t)i * stride, 0);
        px.b[i] = __builtin_amdgcn_raw_buffer_load_b32(rb, o.b[i], adv, 0);
    }
    px.c = __builtin_amdgcn_raw_buffer_load_b32(rb, o.c, adv, 0);
}

/* round 6, an opt-in build (-DSCROLL_ROW_MFMA; the product path is the
 * vector form: the north star prescribes no MFMA for this integer path, and
 * the matrix-core form measured only 2.5 % faster): the
 * matrix-core levels (row_mfma.h).  A wave's pass = 64 tasks
 * = 4 tiles; lane (g = lane / 16, n = lane % 16) loads 16 bytes of one
 * source row, of its prediction row and (chroma) of the lower bilinear row:
 *   luma:   n = (MB m = n / 4 of the wave's four, block row n % 4), pixel
 *           row g of the block row; tile j = block column j;
 *   chroma: n = (plane n / 8, block row (n / 4) % 2, MB pair n % 4), pixel
 *           row g; tile j = (MB j / 2 of the pair, block column j % 2).
 * The offsets advance by T bytes per pass as FetchOff's (16 or 8 bytes per
 * MB, T / 16 or T / 8 MBs per pass) */
struct MFetch {
    uint32_t s, p, q;           /* source row; prediction row; its lower bilinear row (chroma) */
    int pb;
};
struct MPix {
    uint4 s, p, q;
};
[[maybe_unused]] __device__ inline void mfetch_luma(MFetch &o, int v0, int ry, const DynGeom &g, const uint32_t *rt, int lane)
{
    const int gq = lane >> 4, n = lane & 15, k = (v0 >> 4) + (n >> 2), y = 4 * (n & 3) + gq;
    o.s = (uint32_t)((16 * ry + y) * (16 * g.w) + 16 * k);
    o.p = (uint32_t)(16 * (g.x0 + k)) + rt[y];
    o.q = o.p;
}
[[maybe_unused]] __device__ inline void mfetch_chroma(MFetch &o, int e0, int ry, const DynGeom &g, uint32_t csz, const uint32_t *ru,
                                     const uint32_t *rd, int lane)
{
    const int ndt = g.w * g.h, gq = lane >> 4, n = lane & 15, p = n >> 3, by = (n >> 2) & 1;
    const int k = (e0 >> 3) + 2 * (n & 3), y = 4 * by + gq;
    o.s = (uint32_t)(256 * ndt + (p ? 64 * ndt : 0) + (8 * ry + y) * (8 * g.w) + 8 * k);
    const uint32_t co = (uint32_t)p * csz + (uint32_t)(8 * (g.x0 + k));
    o.p = co + (ru[y] & ROW_OFF);
    o.q = co + ((gq < 3 ? ru[y + 1] : rd[y]) & ROW_OFF);
}
[[maybe_unused]] __device__ inline void mfetch_pass(const MFetch &o, bool chroma, uint32_t adv, __amdgpu_buffer_rsrc_t fs,
                                   __amdgpu_buffer_rsrc_t rb, MPix &px)
{
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(fs, o.s, adv, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(rb, o.p, adv, 0);
    px.s = make_uint4(a[0], a[1], a[2], a[3]);
    px.p = make_uint4(b[0], b[1], b[2], b[3]);
    if (chroma) {
        const auto c = __builtin_amdgcn_raw_buffer_load_b128(rb, o.q, adv, 0);
        px.q = make_uint4(c[0], c[1], c[2], c[3]);
    } else {
        px.q = px.p;            /* every field written: the sets stay in registers */
    }
}
#ifdef SCROLL_ROW_MFMA
__constant__ KMat g_kmat = make_kmat();
#endif

/* ((8 - f) b + f c + 4) >> 3 for the four bytes of b, c: even and odd bytes
 * as two 16-bit halves each (at most 2,044: no carry between halves), two
 * 24-bit multiply-adds per half pair.  k_dyn_row's NALs only ever have f = 0
 * or 4 (full-pel luma motion: the chroma fraction is (4 mv) mod 8), where it
 * is b or the rounding byte average v_lerp_u8; this form is the guard */
__device__ inline uint32_t bilin4(uint32_t b, uint32_t c, uint32_t f)
{
    const uint32_t g = 8u - f;
    const uint32_t be = b & 0x00ff00ffu, bo = (b >> 8) & 0x00ff00ffu;
    const uint32_t ce = c & 0x00ff00ffu, co = (c >> 8) & 0x00ff00ffu;
    const uint32_t ve = __umul24(g, be) + __umul24(f, ce) + 0x00040004u;
    const uint32_t vo = __umul24(g, bo) + __umul24(f, co) + 0x00040004u;
    return ((ve >> 3) & 0x00ff00ffu) | (((vo >> 3) & 0x00ff00ffu) << 8);
}

/* i / NPC for a piece index of a rect row (i < NPC DYN_MAX_W): a 24-bit
 * multiply by the rounded-up reciprocal instead of the compiler's
 * quarter-rate high multiply */
static_assert(NPC == 26 && NPC * DYN_MAX_W < 18724, "div_npc's reciprocal (10083 / 2^18) is exact below 18724");
__device__ inline int div_npc(int i) { return (int)(__umul24((uint32_t)i, 10083u) >> 18); }

__device__ inline int row_slot(int task, int w)
{
    const int jj = task - 16 * w;                      /* < 0: luma */
    const bool l = jj < 0;
    const int k = l ? task >> 4 : jj >> 3, pc = l ? task & 15 : 18 + (jj & 7);
    return (int)__umul24((uint32_t)k, (uint32_t)NPC) + pc;   /* no quarter-rate multiply */
}

/* profiling variants only (tools/build_variant.sh, -DSCROLL_ABL_STOP=n):
 * the workgroup stops after phase n, for per-phase time and VALU counts */
#ifdef SCROLL_ABL_STOP
#define ROW_CUT(n) \
    if ((n) == SCROLL_ABL_STOP) return
#else
#define ROW_CUT(n) (void)0
#endif

/* grid (h, frames, streams), row_threads(w) threads, row_lds_bytes dynamic LDS.
 * GEN: the instantiation for the NALs k_dyn_rows flagged for the general
 * path (records from k_dyn_code_general); the other one codes the rest --
 * each returns at once for the other's NALs, and neither carries the
 * other's code (registers) */
template <bool GEN>
__global__ __launch_bounds__(ROW_MAXT) __attribute__((amdgpu_waves_per_eu(SCROLL_ROW_WAVES))) void k_dyn_row(DevStream *__restrict__ st,
                                                     const NalDesc *__restrict__ nal, int ld_nal,
                                                     const PlanPending *__restrict__ pend,
                                                     DynFrame *__restrict__ dfr, int ld_fr, DynGeom g,
                                                     const uint32_t *__restrict__ rows,
                                                     const uint8_t *__restrict__ src,
                                                     const uint8_t *__restrict__ refs,
                                                     const uint16_t *__restrict__ meta,
                                                     const uint2 *__restrict__ blo, const uint2 *__restrict__ bhi,
                                                     const uint4 *__restrict__ bwd,
                                                     unsigned long long *__restrict__ tcx, uint32_t epoch,
                                                     uint32_t *__restrict__ rowstage, uint32_t *__restrict__ gbits,
                                                     uint32_t *__restrict__ spill, uint32_t *__restrict__ ctr,
                                                     const uint4 *__restrict__ heads, uint64_t *__restrict__ stamps)
{
    __shared__ RowFixed L;
    extern __shared__ uint4 rdyn[];
    /* debug: realtime at entry and after each phase (tools/dyn_stamps.py) */
    /* (straight to the slot: an array of the six stamps was kept in scratch
     * memory, zeroed by every thread) */
    const uint64_t t_entry = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const int r = blockIdx.x, t = threadIdx.x, T = blockDim.x, lane = t & 63, wave = t >> 6, nwv = T >> 6;
    int f = blockIdx.y, s = blockIdx.z;
    if (GEN) {                          /* grid (h, record slots): the frames k_dyn_rows listed */
        const uint32_t j = blockIdx.y, n = min(__builtin_amdgcn_readfirstlane(ctr[1]), g.gen_cap);
        if (j >= n) return;
        const uint32_t q = __builtin_amdgcn_readfirstlane(ctr[DYN_CTR_LIST + j]);
        s = (int)(q / (uint32_t)ld_fr);
        f = (int)(q - (uint32_t)s * (uint32_t)ld_fr);
    }
    const size_t nb = (size_t)s * ld_fr + f;
    constexpr bool general = GEN;
    uint64_t *const stp = stamps && t == 0
                              ? stamps + (((size_t)s * gridDim.y + f) * g.ngroups + (max(1, (g.y0 + DYN_STATIC_ROWS - 1) /
                                                                                        DYN_STATIC_ROWS) + r)) * 8
                              : nullptr;
    if (stp) stp[0] = t_entry;
    const Rect R{g.x0, g.y0, g.w, g.h};
    const int w = R.w, ndt = R.w * R.h, row = R.y0 + r, npc = NPC * w, ntask = 24 * w;
    const int ng = g.ngroups;
    constexpr int SR = DYN_STATIC_ROWS;
    const int nA = max(1, (R.y0 + SR - 1) / SR);
    const DevStream *S = st + s;
    const int mbw = g.pw / 16;
    const uint32_t ysz = (uint32_t)g.pw * (uint32_t)g.ph, csz = ysz / 4;
    const int L0 = row_chroma0(w), nl = 16 * w, ntv = L0 + 8 * w;
    const int np = (ntv + T - 1) / T;                   /* passes over the (wave-aligned) tasks */
    const int wv0 = 64 * __builtin_amdgcn_readfirstlane(wave);
    /* the wave's kind in pass q: 0 luma, 1 chroma, 2 none (uniform) */
    auto kind_of = [&](int q) -> int {
        const int v0 = q * T + wv0;
        return v0 < nl ? 0 : (v0 < ntv ? 1 : 2);
    };
    const __amdgpu_buffer_rsrc_t fs = buf_rsrc(src + (size_t)s * g.src_ld + (size_t)f * g.src_fr, (uint32_t)g.src_fr);
    const __amdgpu_buffer_rsrc_t rb = buf_rsrc(refs + (size_t)s * g.ref_ld, 3u * ysz);
    /* pass 0's pixel loads go out first, their offsets from k_dyn_rows' row
     * table in global memory: they need neither the frame's DynFrame nor the
     * LDS copy of the table (a frame this instantiation does not code reads
     * a table k_dyn_rows did not write: offsets into the descriptors' ranges
     * or past them, which read 0; nothing is stored) */
#ifdef SCROLL_ROW_MFMA
    MFetch mo;
    mo.pb = -1;
    bool mo_chroma = false;
    MPix mx;
    if (!general) {
        const uint32_t *rtg = rows + nb * (size_t)(32 * g.h);
        const int k0 = kind_of(0);
        if (k0 == 0) {
            mfetch_luma(mo, wv0, r, g, rtg + 16 * r, lane);
            mo.pb = 0;
            mfetch_pass(mo, false, 0u, fs, rb, mx);
        } else if (k0 == 1) {
            mfetch_chroma(mo, wv0 - L0, r, g, csz, rtg + 16 * g.h + 8 * r, rtg + 24 * g.h + 8 * r, lane);
            mo.pb = 0;
            mo_chroma = true;
            mfetch_pass(mo, true, 0u, fs, rb, mx);
        }
    }
#else
    FetchOff fo;
    fo.pb = -1;
    bool fo_chroma = false;
    BlkPix nx;
    if (!general) {
        const uint32_t *rtg = rows + nb * (size_t)(32 * g.h);
        const int k0 = kind_of(0);
        if (k0 == 0) {
            fetch_luma(fo, t, r, g, rtg + 16 * r);
            fo.pb = 0;
            fetch_pass9(fo, 0u, (uint32_t)(16 * w), fs, rb, nx);
        } else if (k0 == 1) {
            fetch_chroma(fo, t - L0, r, g, csz, rtg + 16 * g.h + 8 * r, rtg + 24 * g.h + 8 * r);
            fo.pb = 0;
            fo_chroma = true;
            fetch_pass9(fo, 0u, (uint32_t)(8 * w), fs, rb, nx);
        }
    }
#endif
    const DynFrame df = dfr[nb];
    if (df.nal < 0 || ((df.err & DF_GENERAL) != 0) != GEN) return;

    uint4 *lv = rdyn;
    uint32_t *moff = reinterpret_cast<uint32_t *>(lv + npc);
    uint16_t *mt = reinterpret_cast<uint16_t *>(moff + w + 1), *lo = mt + npc, *off16 = lo + npc;
    uint16_t *order = off16;                          /* CAVLC phase only; off16 is phase 4's */
    uint8_t *ta = reinterpret_cast<uint8_t *>(off16 + npc), *cbpa = ta + 8 * w, *codea = cbpa + w;
    uint32_t *mbits = reinterpret_cast<uint32_t *>(ta);   /* phase 4 on: ta is dead after phase 3 */

    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    if (t == 0) {
        L.head_over = 0;
        L.ncand = 0;
    }
    if (t < 12) {                       /* the NAL's MB-head classes (k_dyn_rows) */
        const uint4 *hv = heads + nb * DYN_HEAD_VECS;
        const uint4 m = hv[t];
        const uint32_t hl = reinterpret_cast<const uint32_t *>(hv + 12)[t];
        L.hhi[t] = (uint64_t)m.x << 32 | m.y;
        L.hlo[t] = (uint64_t)m.z << 32 | m.w;
        L.hlen[t] = hl & 0x7fffffffu;
        if (hl >> 31) L.head_over = 1;                  /* after lane 0's 0 (same wave, same word) */
    }
    if (t < SORT_KEYS) L.kc[0][t] = 0u;
    if (t < NPC) L.pcd[t] = pc_desc(t);
    load_rowtabs(L.ptabs, t, T);
    for (int i = t; i < LVT_N / 2; i += T)      /* 8-byte aligned in LDS */
        reinterpret_cast<uint2 *>(L.lvt)[i] = reinterpret_cast<const uint2 *>(&g_lvt)[i];
    if (!general && t < 32) L.rt[t] = rows[nb * (size_t)(32 * g.h) + (t < 16 ? 16 * r + t : 16 * g.h + (t < 24 ? 8 * r + t - 16 : 8 * g.h + 8 * r + t - 24))];
    const NalDesc d = nal[(size_t)s * ld_nal + df.nal];

    /* ---- 1-2: records (levels -> CAVLC bodies) into LDS ---------------- */
    __syncthreads();                                    /* the row table (rt) */
    ROW_CUT(0);
    if (!general) {
        static_assert(ROW_MAXT % 64 == 0, "row_threads gives whole waves: the per-pass step T is a multiple of 64");
        /* the row's chroma fraction, the same for all its rows (one region,
         * one mv): 0 or 4 here (k_dyn_rows sends half-pel chains to the
         * general path) */
        const uint32_t frc = __builtin_amdgcn_readfirstlane((L.rt[16] >> 28) & 7u);
        /* the stream's rect QP (QP_MIN and up here: int8 levels) */
        const int qpy = __builtin_amdgcn_readfirstlane(S->dyn_qp);
        const QParams ql = g_qptab.q[qpy].l, qc = g_qptab.q[qpy].c;
#if defined(SCROLL_ROW_LVOLD) && !defined(SCROLL_ROW_MFMA)
        auto issue = [&](int q, BlkPix &px) {
            const int kd = kind_of(q);
            if (kd == 2) return;
            if (kd == 0 && fo.pb < 0) {
                fetch_luma(fo, q * T + t, r, g, L.rt);
                fo.pb = q;
            } else if (kd == 1 && !fo_chroma) {
                fetch_chroma(fo, q * T + t - L0, r, g, csz, L.rt + 16, L.rt + 24);
                fo.pb = q;
                fo_chroma = true;
            }
            fetch_pass(fo, kd == 0, (uint32_t)((q - fo.pb) * T), (uint32_t)(kd == 0 ? 16 * w : 8 * w), fs, rb, px);
        };
        /* counting sort on TotalCoeff class: a task's rank in its class from
         * an LDS atomic (the order inside a class does not matter), kept in
         * lo[] (phase 3's) until the class bases are known */
        auto compute = [&](int q, const BlkPix &px) {
            const int kd = kind_of(q);
            if (kd == 2) return;
            const int v = q * T + t;
            uint32_t pk[4];
            int w0 = 0;
            if (kd == 0) {
                levels_pk<true>(px.a, px.b, pk, w0, ql);
            } else {
                uint32_t pr[4];
                if (frc == 4u) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) pr[i] = __builtin_amdgcn_lerp(px.b[i], i < 3 ? px.b[i + 1] : px.c, 0x01010101u);
                } else if (frc == 0u) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) pr[i] = px.b[i];
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) pr[i] = bilin4(px.b[i], i < 3 ? px.b[i + 1] : px.c, frc);
                }
                levels_pk<false>(px.a, pr, pk, w0, qc);
            }
            const int e = v - L0;                           /* chroma task index */
            const bool ok = kd == 0 ? v < nl : e < 8 * w;
            if (ok) {
                const int n = nz_bytes(pk[0]) + nz_bytes(pk[1]) + nz_bytes(pk[2]) + nz_bytes(pk[3]);
                const int slot = kd == 0 ? (int)__umul24((uint32_t)(v >> 4), (uint32_t)NPC) + (v & 15)
                                         : (int)__umul24((uint32_t)(e >> 3), (uint32_t)NPC) + 18 + (e & 7);
                lv[slot] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                mt[slot] = (uint16_t)((uint32_t)min(n, 16) << 8);
                lo[slot] = (uint16_t)atomicAdd(&L.kc[0][SORT_KEYS - 1 - min(n, SORT_KEYS - 1)], 1u);
            }
            /* chroma DC: the quad's four DC coefficients -> 2x2 Hadamard,
             * quant -> levels as int16 in the DC slot (coded after the
             * barrier that publishes the CAVLC tables); quads are lane-aligned
             * (L0 and T are multiples of 64) */
            if (kd == 1) {
                const int qb = lane & ~3;
                const int d0 = __shfl(w0, qb, 64), d1 = __shfl(w0, qb + 1, 64);
                const int d2 = __shfl(w0, qb + 2, 64), d3 = __shfl(w0, qb + 3, 64);
                if (ok && (e & 3) == 0) {
                    const int k = e >> 3, p = (e >> 2) & 1;
                    const int q0 = quant_dc(d0 + d1 + d2 + d3, qc), q1 = quant_dc(d0 - d1 + d2 - d3, qc);
                    const int q2 = quant_dc(d0 + d1 - d2 - d3, qc), q3 = quant_dc(d0 - d1 - d2 + d3, qc);
                    lv[k * NPC + 16 + p] = make_uint4(((uint32_t)q0 & 0xffffu) | (uint32_t)q1 << 16,
                                                      ((uint32_t)q2 & 0xffffu) | (uint32_t)q3 << 16, 0u, 0u);
                    mt[k * NPC + 16 + p] =
                        (uint16_t)((uint32_t)((q0 != 0) + (q1 != 0) + (q2 != 0) + (q3 != 0)) << 8);
                }
            }
        };
        /* two pixel sets in turn: the next pass's loads are in flight while
         * this one is coded, with no register copies between passes */
        for (int pa = 0; pa < np; ++pa) {                  /* pass 0's loads are in flight already */
            const BlkPix cur = nx;
            if (pa + 1 < np) issue(pa + 1, nx);
            compute(pa, cur);
        }
#elif !defined(SCROLL_ROW_MFMA)
        /* round 6: a wave's passes are luma ones, then chroma ones, then
         * none (L0 and T are multiples of 64), so two loops whose kind is
         * known at compile time: no per-pass kind tests, and the compiler
         * schedules the next pass's loads and this pass's coding as one
         * straight block.  The next pass's loads are in flight while this
         * one is coded; qL / qC: this wave's luma / luma + chroma passes */
        const int qL = nl > wv0 ? (nl - wv0 + T - 1) / T : 0;
        const int qC = ntv > wv0 ? (ntv - wv0 + T - 1) / T : 0;
        auto issue_l = [&](int q, BlkPix &px) {
            fetch_pass9(fo, (uint32_t)((q - fo.pb) * T), (uint32_t)(16 * w), fs, rb, px);
        };
        auto issue_c = [&](int q, BlkPix &px) {
            if (!fo_chroma) {
                fetch_chroma(fo, q * T + t - L0, r, g, csz, L.rt + 16, L.rt + 24);
                fo.pb = q;
                fo_chroma = true;
            }
            fetch_pass9(fo, (uint32_t)((q - fo.pb) * T), (uint32_t)(8 * w), fs, rb, px);
        };
        /* the loads of pass q: luma, else chroma -- past the wave's tasks
         * too (offsets in the descriptors' ranges or read as 0 past them,
         * never used): every path issues the same nine loads, so the wait
         * for the other set before its coding counts nine, not zero */
        auto issue_any = [&](int q, BlkPix &px) {
            if (q < qL) issue_l(q, px);
            else issue_c(q, px);
        };
        /* a level record: packed levels, TotalCoeff, its rank in its class
         * (counting sort: the order inside a class does not matter) */
#ifdef SCROLL_ROW_OLDREC
        auto put_rec = [&](int slot, const uint32_t pk[4]) {
            const int n = nz_bytes(pk[0]) + nz_bytes(pk[1]) + nz_bytes(pk[2]) + nz_bytes(pk[3]);
            lv[slot] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            mt[slot] = (uint16_t)((uint32_t)min(n, 16) << 8);
            lo[slot] = (uint16_t)atomicAdd(&L.kc[0][SORT_KEYS - 1 - min(n, SORT_KEYS - 1)], 1u);
        };
#else
        /* round 6: mt holds the block's non-zero mask until its CAVLC body
         * (TotalCoeff = its popcount), so the body phase reads it instead of
         * deriving it from the levels again */
        const NzConst nzc = nz_const();
        auto put_rec = [&](int slot, const uint32_t pk[4]) {
            const uint4 p4 = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            const uint32_t nz = nz_mask16_c(p4, nzc);
            const int n = __builtin_popcount(nz);
            lv[slot] = p4;
            mt[slot] = (uint16_t)nz;
            /* a block without levels has no CAVLC body: no rank (its class
             * sorts last and is never read), and no same-address LDS atomic
             * of the many such lanes of a wave */
#ifndef SCROLL_ROW_RANK_ALL
            if (n)
#endif
                lo[slot] = (uint16_t)atomicAdd(&L.kc[0][SORT_KEYS - 1 - min(n, SORT_KEYS - 1)], 1u);
        };
#endif
        /* the quantisers' bias pairs pinned in VGPRs (full-rate v_bitop3) */
        const LevelsBias bl = levels_bias(ql), bc = levels_bias(qc);
        auto code_l = [&](int q, const BlkPix &px) {
            const int v = q * T + t;
            uint32_t pk[4];
            int w0 = 0;
            levels_pk<true>(px.a, px.b, pk, w0, ql, bl.k1, bl.k0);
            if (v < nl) put_rec((int)__umul24((uint32_t)(v >> 4), (uint32_t)NPC) + (v & 15), pk);
        };
        auto code_c = [&](int q, const BlkPix &px) {
            const int e = q * T + t - L0;                   /* chroma task index */
            uint32_t pr[4], pk[4];
            int w0 = 0;
            if (frc == 4u) {
#pragma unroll
                for (int i = 0; i < 4; ++i) pr[i] = __builtin_amdgcn_lerp(px.b[i], i < 3 ? px.b[i + 1] : px.c, 0x01010101u);
            } else if (frc == 0u) {
#pragma unroll
                for (int i = 0; i < 4; ++i) pr[i] = px.b[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) pr[i] = bilin4(px.b[i], i < 3 ? px.b[i + 1] : px.c, frc);
            }
            levels_pk<false>(px.a, pr, pk, w0, qc, bc.k1, bc.k0);
            const bool ok = e < 8 * w;
            if (ok) put_rec((int)__umul24((uint32_t)(e >> 3), (uint32_t)NPC) + 18 + (e & 7), pk);
#ifndef SCROLL_ROW_OLDREC
            /* chroma DC: the block's DC coefficient (|W0| <= 4080) as int16 i
             * of its plane's DC slot; the 2x2 Hadamard and quant follow the
             * loop, once per DC block (round 6: in the loop every chroma lane
             * ran them, masked to one lane of four) */
            if (ok) reinterpret_cast<int16_t *>(lv + (e >> 3) * NPC + 16 + ((e >> 2) & 1))[e & 3] = (int16_t)w0;
#else
            /* chroma DC: the quad's four DC coefficients -> 2x2 Hadamard,
             * quant -> levels as int16 in the DC slot (quads are lane-aligned) */
            const int qb = lane & ~3;
            const int d0 = __shfl(w0, qb, 64), d1 = __shfl(w0, qb + 1, 64);
            const int d2 = __shfl(w0, qb + 2, 64), d3 = __shfl(w0, qb + 3, 64);
            if (ok && (e & 3) == 0) {
                const int k = e >> 3, p = (e >> 2) & 1;
                const int q0 = quant_dc(d0 + d1 + d2 + d3, qc), q1 = quant_dc(d0 - d1 + d2 - d3, qc);
                const int q2 = quant_dc(d0 + d1 - d2 - d3, qc), q3 = quant_dc(d0 - d1 - d2 + d3, qc);
                lv[k * NPC + 16 + p] = make_uint4(((uint32_t)q0 & 0xffffu) | (uint32_t)q1 << 16,
                                                  ((uint32_t)q2 & 0xffffu) | (uint32_t)q3 << 16, 0u, 0u);
                mt[k * NPC + 16 + p] = (uint16_t)((uint32_t)((q0 != 0) + (q1 != 0) + (q2 != 0) + (q3 != 0)) << 8);
            }
#endif
        };
        /* two pixel sets in fixed roles (the passes unrolled by two): pass
         * q + 1's loads go into one while pass q is coded from the other --
         * no register copies between passes.  pass 0's loads are in flight */
        BlkPix A = nx, B;
        int q = 0;
        for (; q + 1 < qL; q += 2) {
            issue_l(q + 1, B);
            code_l(q, A);
            issue_any(q + 2, A);
            code_l(q + 1, B);
        }
        if (q < qL) {                                       /* an odd luma pass left */
            issue_any(q + 1, B);
            code_l(q, A);
            A = B;                                          /* once: the first chroma pass */
            ++q;
        }
        for (; q + 1 < qC; q += 2) {
            issue_c(q + 1, B);
            code_c(q, A);
            issue_c(q + 2, A);                              /* past the tasks: nine unused loads */
            code_c(q + 1, B);
        }
        if (q < qC) code_c(q, A);
        (void)np;
#else
        /* round 6: the levels on the matrix cores (row_mfma.h, MFetch): per
         * pass and wave 4 tiles of 16 blocks, each one MFMA, the quant of two
         * tiles per asm block, a lane-group transpose, then one block per
         * lane as before (put_rec).  The pass structure is the vector
         * form's: luma passes, then chroma ones, the next pass's loads in
         * flight while one is coded */
        const int qL = nl > wv0 ? (nl - wv0 + T - 1) / T : 0;
        const int qC = ntv > wv0 ? (ntv - wv0 + T - 1) / T : 0;
        const int gq = lane >> 4, ln = lane & 15;
        auto issue_l = [&](int q, MPix &px) { mfetch_pass(mo, false, (uint32_t)((q - mo.pb) * T), fs, rb, px); };
        auto issue_c = [&](int q, MPix &px) {
            if (!mo_chroma) {
                mfetch_chroma(mo, q * T + wv0 - L0, r, g, csz, L.rt + 16, L.rt + 24, lane);
                mo.pb = q;
                mo_chroma = true;
            }
            mfetch_pass(mo, true, (uint32_t)((q - mo.pb) * T), fs, rb, px);
        };
        auto issue_any = [&](int q, MPix &px) {
            if (q < qL) issue_l(q, px);
            else issue_c(q, px);
        };
        auto put_rec = [&](int slot, const uint32_t pk[4]) {
            const uint4 p4 = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            const uint32_t nz = nz_mask16(p4);
            const int n = __builtin_popcount(nz);
            lv[slot] = p4;
            mt[slot] = (uint16_t)nz;
            /* a block without levels has no CAVLC body: no rank (its class
             * sorts last and is never read), and no same-address LDS atomic
             * of the many such lanes of a wave */
#ifndef SCROLL_ROW_RANK_ALL
            if (n)
#endif
                lo[slot] = (uint16_t)atomicAdd(&L.kc[0][SORT_KEYS - 1 - min(n, SORT_KEYS - 1)], 1u);
        };
        const uint64_t aL = g_kmat.a[0][lane];
        const MQuant QL = mquant_of(gq, true, ql);
        auto code_l = [&](int q, const MPix &px) {
            uint32_t wd[4];
            {
                const mfma_v4i d0 = mtile(aL, px.s.x, px.p.x), d1 = mtile(aL, px.s.y, px.p.y);
                mquant2(d0, d1, QL, wd[0], wd[1]);
            }
            {
                const mfma_v4i d2 = mtile(aL, px.s.z, px.p.z), d3 = mtile(aL, px.s.w, px.p.w);
                mquant2(d2, d3, QL, wd[2], wd[3]);
            }
            mtranspose(wd);
            /* lane (gq, ln): block (MB ln / 4 of the pass's four, row ln % 4, column gq) */
            const int k = ((q * T + wv0) >> 4) + (ln >> 2);
            if (k < w) put_rec((int)__umul24((uint32_t)k, (uint32_t)NPC) + 4 * (ln & 3) + gq, wd);
        };
        auto code_c = [&](int q, const MPix &px, uint64_t aC, const MQuant &QC) {
            uint32_t pr[4];
            const uint32_t up[4] = {px.p.x, px.p.y, px.p.z, px.p.w}, dn[4] = {px.q.x, px.q.y, px.q.z, px.q.w};
            if (frc == 4u) {
#pragma unroll
                for (int j = 0; j < 4; ++j) pr[j] = __builtin_amdgcn_lerp(up[j], dn[j], 0x01010101u);
            } else if (frc == 0u) {
#pragma unroll
                for (int j = 0; j < 4; ++j) pr[j] = up[j];
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) pr[j] = bilin4(up[j], dn[j], frc);
            }
            const mfma_v4i d0 = mtile(aC, px.s.x, pr[0]), d1 = mtile(aC, px.s.y, pr[1]);
            const mfma_v4i d2 = mtile(aC, px.s.z, pr[2]), d3 = mtile(aC, px.s.w, pr[3]);
            const int kb = ((q * T + wv0 - L0) >> 3) + 2 * (ln & 3), pl = ln >> 3, by = (ln >> 2) & 1;
            /* the DC coefficients (row 15, lane group 3) as int16 into their
             * plane's DC slot: tile j = MB kb + j / 2, block column j % 2 */
            if (gq == 3) {
                const int dcv[4] = {d0[3], d1[3], d2[3], d3[3]};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int k = kb + (j >> 1);
                    if (k < w)
                        reinterpret_cast<int16_t *>(lv + (int)__umul24((uint32_t)k, (uint32_t)NPC) + 16 + pl)[2 * by + (j & 1)] =
                            (int16_t)dcv[j];
                }
            }
            uint32_t wd[4];
            mquant2(d0, d1, QC, wd[0], wd[1]);
            mquant2(d2, d3, QC, wd[2], wd[3]);
            mtranspose(wd);
            const int k = kb + (gq >> 1);
            if (k < w) put_rec((int)__umul24((uint32_t)k, (uint32_t)NPC) + 18 + 4 * pl + 2 * by + (gq & 1), wd);
        };
        MPix A = mx, B;
        int q = 0;
        for (; q + 1 < qL; q += 2) {
            issue_l(q + 1, B);
            code_l(q, A);
            issue_any(q + 2, A);
            code_l(q + 1, B);
        }
        if (q < qL) {                                       /* an odd luma pass left */
            issue_any(q + 1, B);
            code_l(q, A);
            A = B;                                          /* once: the first chroma pass */
            ++q;
        }
        if (q < qC) {
            const uint64_t aC = g_kmat.a[1][lane];
            const MQuant QC = mquant_of(gq, false, qc);
            for (; q + 1 < qC; q += 2) {
                issue_c(q + 1, B);
                code_c(q, A, aC, QC);
                issue_c(q + 2, A);                          /* past the tasks: unused loads */
                code_c(q + 1, B, aC, QC);
            }
            if (q < qC) code_c(q, A, aC, QC);
        }
        (void)np;
#endif
        __syncthreads();                                /* levels, TotalCoeffs, ptabs, counts */
        if (stp) stp[1] = __builtin_amdgcn_s_memrealtime();
        /* the row's bottom TotalCoeffs (luma 12-15, chroma AC raster 2, 3 of
         * each plane) for the row below: one granule per MB */
        const bool nopub = (g.debug & SCROLL_DEBUG_DYN_NOPUBLISH) && s == 0 && f == 0 && r == 0;   /* tests */
        if (t < w && r + 1 < R.h && !nopub) {
            const uint16_t *mk = mt + t * NPC;
            uint64_t v = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int pcA = e < 4 ? 12 + e : (e < 6 ? 16 + e : 18 + e);
#ifdef SCROLL_ROW_OLDREC
                v |= (uint64_t)(tc_of(mk[pcA]) & 31) << (5 * e);
#else
                v |= (uint64_t)__builtin_popcount(mk[pcA]) << (5 * e);    /* the block's non-zero mask */
#endif
            }
            lb_store(tcx + (nb * R.h + r) * (size_t)w + t, (uint64_t)(epoch & 0xffffffu) << 40 | v);
        }
        /* chroma DC blocks, whole (nC = -1) */
        if (t >= T - 2 * w) {
            const int i = t - (T - 2 * w), k = i >> 1, p = i & 1, sl = k * NPC + 16 + p;
            const uint4 q = lv[sl];
#ifdef SCROLL_ROW_OLDREC
            const int dq[4] = {(int)(int16_t)(q.x & 0xffffu), (int)(int16_t)(q.x >> 16),
                               (int)(int16_t)(q.y & 0xffffu), (int)(int16_t)(q.y >> 16)};
#else
            /* the four DC coefficients of the plane's 4x4 blocks (raster) ->
             * 2x2 Hadamard, quant (qbits + 1) */
            const int d0 = (int)(int16_t)(q.x & 0xffffu), d1 = (int)(int16_t)(q.x >> 16);
            const int d2 = (int)(int16_t)(q.y & 0xffffu), d3 = (int)(int16_t)(q.y >> 16);
            const int dq[4] = {quant_dc(d0 + d1 + d2 + d3, qc), quant_dc(d0 - d1 + d2 - d3, qc),
                               quant_dc(d0 + d1 - d2 - d3, qc), quant_dc(d0 - d1 - d2 + d3, qc)};
#endif
            CapSink cap{0, 0, 0};
            const int tc = cavlc_dc4(cap, L.ptabs, dq);
            if (cap.n <= 128) {
                mt[sl] = (uint16_t)(cap.n | (uint32_t)tc << 8);
                lv[sl] = body_msb(cap.hi, cap.lo, cap.n);
            } else {
                mt[sl] = (uint16_t)((uint32_t)tc << 8 | M_OVF);       /* the levels in lv */
#ifndef SCROLL_ROW_OLDREC
                lv[sl] = make_uint4(((uint32_t)dq[0] & 0xffffu) | (uint32_t)dq[1] << 16,
                                    ((uint32_t)dq[2] & 0xffffu) | (uint32_t)dq[3] << 16, 0u, 0u);
#endif
            }
        }
        if (t < SORT_KEYS) {                            /* class k = t: its base */
            const uint32_t tot = L.kc[0][t];
            uint32_t kb = tot;
#pragma unroll
            for (int dd = 1; dd < 32; dd <<= 1) {
                const uint32_t o = __shfl_up(kb, dd, 64);
                if (lane >= dd) kb += o;
            }
            L.kc[1][t] = kb - tot;
        }
        __syncthreads();
        for (int task = t; task < ntask; task += T) {       /* the slot, chroma flagged in bit 15 */
            const int slot = row_slot(task, w);
#ifdef SCROLL_ROW_OLDREC
            const int tcs = tc_of(mt[slot]);
#else
            const int tcs = __builtin_popcount(mt[slot]);
#endif
            if (tcs) {
                order[L.kc[1][SORT_KEYS - 1 - min(tcs, SORT_KEYS - 1)] + lo[slot]] =
                    (uint16_t)(slot | (task < 16 * w ? 0 : 0x8000));
#if SCROLL_LV_SWZ
                /* the record's dwords swizzled by its slot (lv_key): the
                 * CAVLC lanes read one level byte each from records on
                 * about consecutive slots (the sort's ranks follow the
                 * lanes), 16 bytes apart -- four banks -- so lanes 16 slots
                 * apart met in one bank; with dword d at d ^ key they don't */
                const uint32_t key = lv_key(slot);
                if (key) lv[slot] = lv_swz(lv[slot], key);
#endif
            }
        }
        __syncthreads();
    ROW_CUT(1);
        /* CAVLC bodies, largest TotalCoeff first */
        const int zbase = (int)L.kc[1][SORT_KEYS - 1];      /* blocks without levels sort last: no body */
        for (int pa = 0; pa < np; ++pa) {
            const int pos = pa * T + t;
            if (pos >= zbase) continue;
            const uint32_t oe = order[pos];
            const int slot = (int)(oe & 0x7fffu);
            const bool luma = !(oe & 0x8000u);
            CapSink cap{0, 0, 0};
            int t1 = 0;
            bool ok = true;
            /* total_zeros + run_before from the table: the load is in flight
             * during the trailing ones and the level loop */
#ifdef SCROLL_ROW_OLDREC
            const uint32_t nz = nz_mask16(lv[slot]);
#else
            const uint32_t nz = mt[slot];                   /* the non-zero mask (levels phase) */
#endif
            const uint32_t tzrb = g_tzrb[luma ? nz : 65536u + nz];
            const uint32_t key = SCROLL_LV_SWZ ? lv_key(slot) : 0u;
            const int tc = cavlc_body_t(cap, reinterpret_cast<const int8_t *>(lv + slot), nz, tzrb, t1, ok, L.lvt,
                                        key << 2);
            mt[slot] = ok ? (uint16_t)(cap.n | (uint32_t)tc << 8 | (uint32_t)t1 << 13)
                          : (uint16_t)((uint32_t)tc << 8 | (uint32_t)t1 << 13 | M_OVF);
            if (ok) lv[slot] = body_msb(cap.hi, cap.lo, cap.n);
            else if (key) lv[slot] = lv_swz(lv[slot], key);     /* rare: the levels stay, in plain order */
        }
    } else {
        /* general path: records of k_dyn_code_general */
        const int q0 = r * w;
        const size_t gs = df.rbsp_bytes;                /* its record slot (k_dyn_rows) */
        const uint16_t *M = meta + gs * (size_t)(NPC * ndt);
        const uint2 *BL = blo + gs * (size_t)(NPC * ndt), *BH = bhi + gs * (size_t)(NPC * ndt);
        for (int i = t; i < npc; i += T) {
            const int k = div_npc(i), pc = i - k * NPC;
            const int rec = rec_of(q0 + k, pc, ndt);
            const uint16_t mv = M[rec];
            mt[i] = mv;
            /* an empty body stored as zeros: phases 3 and 5 OR a piece's
             * first words whatever its length (stale LDS there was ORed into
             * the row's bits) */
            uint4 bv = make_uint4(0u, 0u, 0u, 0u);
            if ((mv & 255u) || (mv & M_OVF)) {
                const uint4 bd = get_body(BL, BH, rec, (mv & 255u) > 64u || (mv & M_OVF));
                bv = (mv & M_OVF) ? bd
                                  : body_msb((uint64_t)bd.z | (uint64_t)bd.w << 32,
                                             (uint64_t)bd.x | (uint64_t)bd.y << 32, mv & 255u);
            }
            lv[i] = bv;
        }
        for (int i = t; i < 8 * w; i += T) {
            const int k = i >> 3, e = i & 7;
            const int pcA = e < 4 ? 12 + e : (e < 6 ? 16 + e : 18 + e);
            ta[i] = r > 0 ? (uint8_t)tc_of(M[rec_of(q0 + k - w, pcA, ndt)]) : (uint8_t)0;
        }
    }
    /* top TotalCoeffs of the row above (normal path): its granules; the last
     * wave polls (the sort gives it the lightest blocks).  The wait is
     * bounded: past HANDOFF_TICKS the frame fails (DF_HANDOFF) and the row
     * finishes on zeros, so a missing granule costs one stream, not the GPU */
    if (!general && wave == nwv - 1) {
        /* waited time = the sum of the gaps between consecutive polls, a gap
         * over HANDOFF_GAP (the queue preempted or time-sliced: the row above
         * was paused too) not counted -- a slow-but-alive row above never
         * fails the stream on a shared GPU */
        uint64_t prev = r > 0 ? __builtin_amdgcn_s_memrealtime() : 0ull, waited = 0;
        bool late = false;
        for (int k = lane; k < w; k += 64) {
            uint64_t v = 0;
            if (r > 0) {
                const unsigned long long *p = tcx + (nb * R.h + r - 1) * (size_t)w + k;
                for (;;) {
                    v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((uint32_t)(v >> 40) == (epoch & 0xffffffu)) break;
                    const uint64_t now = __builtin_amdgcn_s_memrealtime(), gap = now - prev;
                    prev = now;
                    if (gap < HANDOFF_GAP) waited += gap;
                    if (waited > HANDOFF_TICKS) {
                        v = 0;
                        late = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) ta[8 * k + e] = (uint8_t)((v >> (5 * e)) & 31u);
        }
        if (__builtin_amdgcn_ballot_w64(late) != 0 && lane == 0) atomicOr(&dfr[nb].err, DF_HANDOFF);
    }
    const NalCtx c = nal_ctx(S, d, L.wo, L.wl, L.wv);
    const HeadCtx H = head_ctx(c);
    /* a piece's levels past 8 (16-bit records of the general path below
     * QP_MIN), nullptr for the int8 forms */
    const bool wide = GEN && __builtin_amdgcn_readfirstlane(S->dyn_qp) < QP_MIN;
    auto ovf_wide = [&](int k, int pc) -> const uint4 * {
        if (!wide) return nullptr;
        return bwd + (size_t)df.rbsp_bytes * (size_t)(NPC * ndt) + rec_of(r * w + k, pc, ndt);
    };
    __syncthreads();                                    /* records, top TotalCoeffs, waypoint table */
    if (stp) stp[2] = __builtin_amdgcn_s_memrealtime();
    ROW_CUT(2);

    /* ---- 3: coeff_token, piece lengths ----------------------------------- */
    const Tabs &TB = g_tabs;
    const PTabs &PT = *reinterpret_cast<const PTabs *>(&g_ptabs);       /* the rare overflow paths */
    const uint16_t(*ctab)[68] = L.ptabs.ct;
    /* one straight path for every piece class: its neighbours from pc_desc
     * (the per-class branches had made every wave run all of them) */
    const int nAe = R.x0 > 0 ? 0 : -1, nBe = row > 0 ? 0 : -1;
    /* piece i = k NPC + pc, D = its class's neighbour descriptor */
    auto token = [&](int i, int k, int pc, uint32_t D) {
        const uint32_t mv = mt[i];
        const int ia = max(i + (int)(D & 63u) - 32, 0), ib = max(i + (int)((D >> 7) & 63u) - 32, 0);
        const int tA = tc_of(mt[ia]), tB = tc_of(mt[ib]), tT = (int)ta[8 * k + (int)((D >> 14) & 7u)];
        const int nA = ((D & 64u) && k == 0) ? nAe : tA;
        const int nB = (D & 8192u) ? (r > 0 ? tT : nBe) : tB;
        /* both available: their rounded mean, else the available one (9.2.1);
         * as selects, no divergent branch */
        const int mean = (nA + nB + 1) >> 1, one = max(max(nA, nB), 0);
        const int nC0 = (nA | nB) >= 0 ? mean : one;
        const int nC = (D >> 17) ? -1 : nC0;
        const int tc = tc_of(mv), t1 = (int)((mv >> 13) & 3u);
        const uint32_t ce = ctab[nC < 0 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2))][4 * tc + t1];
        /* chroma DC: its body holds the whole block, token included */
        const uint32_t tl = nC < 0 ? 0u : (nC >= 8 ? 6u : ce >> 8);
        uint32_t len = tl + (mv & 255u);
        if (mv & M_OVF) len = ovf_bits(PT, TB, lv[i], ovf_wide(k, pc), pc, nC);   /* rare */
        uint32_t nc1 = (uint32_t)(nC + 1);
        if (!(mv & M_OVF) && nC >= 0 && len <= 128u) {
            /* the token goes in front of the body here, where its code is
             * at hand: the piece is then a bare MSB-first body of len bits
             * (nC field 0, as a chroma DC piece), and phase 5 writes it
             * without looking the token up again */
            const uint32_t tv = nC >= 8 ? (tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u) : (ce & 255u);
            const uint32_t tw = tv & low_mask((int)tl);
            const uint4 b = lv[i];
            lv[i] = make_uint4(__builtin_amdgcn_alignbit(tw, b.x, tl), __builtin_amdgcn_alignbit(b.x, b.y, tl),
                               __builtin_amdgcn_alignbit(b.y, b.z, tl), __builtin_amdgcn_alignbit(b.z, b.w, tl));
            mt[i] = (uint16_t)((mv & ~255u) | len);                 /* tc / t1 bits unchanged */
            nc1 = 0u;
        }
        lo[i] = (uint16_t)(len | nc1 << 11);
    };
    for (int i = t; i < npc; i += T) {
        const int k = div_npc(i), pc = i - k * NPC;
        token(i, k, pc, L.pcd[pc]);
    }
    __syncthreads();
    if (stp) stp[3] = __builtin_amdgcn_s_memrealtime();
    ROW_CUT(3);
    const bool head_over = L.head_over;
    auto head_bits = [&](int rr, int col) -> uint32_t {
        if (!head_over) return L.hlen[H.sel(rr, col)];
        CountSink cn{0};
        H.put_slow(cn, rr, col);
        return cn.n;
    };

    /* ---- 4: per MB cbp, code, piece offsets; the row's MB offsets ------- */
    for (int k = t; k < w; k += T) {
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
            const int rr = blk_raster(blk);
            const bool pres = (cbp_l >> (blk >> 2)) & 1;
            ok[rr] = pres ? (uint16_t)off : (uint16_t)0xffffu;
            off += pres ? (lk[rr] & LO_LEN) : 0u;
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
    /* the bit offset of column col in the row: a static column's head (+ its
     * coded_block_pattern '1') is the row's first / middle / last class, so
     * the static columns before the rect and after it are closed forms; the
     * rect's columns come from the scan below (moff) */
    const int x1 = R.x0 + w;
    const uint32_t h0 = head_bits(row, 0) + 1u;
    const uint32_t h1 = mbw >= 3 ? head_bits(row, 1) + 1u : 0u;
    const uint32_t h2 = mbw >= 2 ? head_bits(row, mbw - 1) + 1u : 0u;
    auto colpos = [&](int col) -> uint32_t {
        if (col <= R.x0) return col == 0 ? 0u : h0 + (uint32_t)(col - 1) * h1;
        if (col < x1) return moff[col - R.x0];
        return moff[w] + (uint32_t)(col - x1) * h1 + (col == mbw && x1 <= mbw - 1 ? h2 - h1 : 0u);
    };
    __syncthreads();
    const int gi = nA + r;
    if (wave == 0) {
        uint32_t carry = R.x0 == 0 ? 0u : h0 + (uint32_t)(R.x0 - 1) * h1;
        for (int k0 = 0; k0 < w; k0 += 64) {
            const int k = k0 + lane;
            const uint32_t len = k < w ? mbits[k] : 0u;
            const uint32_t incl = wave_incl_sum(len, lane);
            if (k < w) moff[k] = carry + incl - len;
            carry += __shfl(incl, 63, 64);
        }
        if (lane == 0) moff[w] = carry;
    }
    __syncthreads();
    if (stp) stp[4] = __builtin_amdgcn_s_memrealtime();
    ROW_CUT(4);
    const uint32_t bits = colpos(mbw);
    if (t == 0) gbits[nb * (size_t)ng + gi] = bits;

    /* ---- 5: bits -> the row's own row-stage words ------------------------ */
    const bool wwin = row_wide_win(w);
    uint32_t *const wb = wwin ? reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(rdyn) + row_wide_off(w)) : L.buf;
    const uint32_t GBW = wwin ? (uint32_t)ROW_GB_WIDE : (uint32_t)ROW_GB;
    uint32_t *out = rowstage + nb * g.rs_frame_words + rs_group_words(g, nA, gi);
    uint32_t epc = g.rs_row_words - EPC_ROW;            /* the EP-candidate record in the slot */
    bool lost = false;                                  /* no spill slot: the frame fails (DF_OVER) */
    if (((bits + 31u) >> 5) > epc) {
        /* the row outgrew its slot (sized for typical rows):
         * its bits go to a spill slot at the provable bound; the slot's
         * record word names it (k_dyn_epfix / the readers' rs_table follow) */
        if (t == 0) L.spill = atomicAdd(&ctr[0], 1u);
        __syncthreads();
        const uint32_t k = L.spill;
        uint32_t *fr = rowstage + nb * g.rs_frame_words;
        uint32_t *sp = spill + (size_t)k * g.rs_spill_words;
        /* none left, or out of the readers' reach (32-bit byte offsets from fr) */
        if (k >= g.rs_spill_cap || (uint64_t)(sp - fr) + g.rs_spill_words > 0x3fffffffull) {
            if (t == 0) atomicOr(&dfr[nb].err, DF_OVER);
            lost = true;
        } else {
            if (t == 0) out[epc] = 0x80000000u | (uint32_t)(sp - fr);
            out = sp;
            epc = g.rs_spill_words - EPC_ROW;
        }
    }
    const uint32_t nw = lost ? 0u : min((bits + 31u) >> 5, epc);     /* provable bound: never clipped */
    const int npass = (int)((nw + GBW - 1) / GBW);
    for (int pi = 0; pi < npass; ++pi) {
        const uint32_t p0 = (uint32_t)pi * GBW;
        const uint32_t n = min((uint32_t)GBW, nw - p0);
        for (uint32_t i = (uint32_t)t; i < n; i += (uint32_t)T) wb[i] = 0u;
        __syncthreads();
        const LdsOrWin win{wb, p0, n};
        /* MB heads (+ coded_block_pattern / mb_qp_delta) of every column:
         * in a one-pass row the class's MSB-first bits with the tail ORed
         * in, written as one piece */
        const bool one = npass == 1;
        for (int col = t; col < mbw; col += T) {
            const uint32_t pos = colpos(col);
            if (!one && (pos >= 32u * (p0 + n) || colpos(col + 1) <= 32u * p0)) continue;
            const int k = col - R.x0;
            const bool in = k >= 0 && k < w;
            if (one && !head_over) {
                const int cls = H.sel(row, col);
                const uint32_t hl = L.hlen[cls];
                uint32_t tv = 1u, tn = 1u;                      /* coded_block_pattern ue(0) */
                if (in) {
                    const uint32_t x = (uint32_t)codea[k] + 1u, lz = 31u - (uint32_t)__builtin_clz(x);
                    tv = x;
                    tn = 2u * lz + 1u;                          /* ue(code) */
                    if (cbpa[k]) {
                        tv = tv << 1 | 1u;                      /* mb_qp_delta se(0) */
                        ++tn;
                    }
                }
                if (hl + tn <= 128u) {
                    const uint64_t ha = L.hhi[cls], hb = L.hlo[cls];
                    const uint32_t t32 = tv << (32u - tn), q = hl >> 5, r = hl & 31u;
                    uint32_t wv[4] = {(uint32_t)(ha >> 32), (uint32_t)ha, (uint32_t)(hb >> 32), (uint32_t)hb};
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j)
                        wv[j] |= (j == q ? t32 >> r : 0u) | (j == q + 1u && r ? t32 << (32u - r) : 0u);
                    put_piece1(wb, pos, 0u, 0u, make_uint4(wv[0], wv[1], wv[2], wv[3]), hl + tn);
                    continue;
                }
            }
            WSink sk{win, 0, 0, 0};
            sk.start(pos);
            if (!head_over) {
                const int cls = H.sel(row, col);
                sk.put_cap(cap_of_msb(L.hhi[cls], L.hlo[cls], L.hlen[cls]));
            } else {
                H.put_slow(sk, row, col);
            }
            if (!in) {
                sk.put(1, 1);                           /* coded_block_pattern ue(0) */
            } else {
                put_ue(sk, (uint32_t)codea[k]);
                if (cbpa[k]) put_se(sk, 0);
            }
            sk.finish();
        }
        /* pieces (a row in one pass -- all of config 3's -- skips the
         * window tests) */
        for (int i = t; i < npc; i += T) {
            const uint32_t o = off16[i];
            if (o == 0xffffu) continue;
            const int k = div_npc(i), pc = i - k * NPC;
            const uint32_t e = lo[i], mv = mt[i];
            const uint32_t pos = moff[k] + o;
            if (!one && (pos >= 32u * (p0 + n) || pos + (e & LO_LEN) <= 32u * p0)) continue;
            const int nC = (int)(e >> 11) - 1;
            const uint4 bd = lv[i];
            if (!(mv & M_OVF)) {
                if (nC == -1) {                         /* a bare body (token in front since phase 3) */
                    if (one) put_piece1(wb, pos, 0u, 0u, bd, mv & 255u);
                    else put_piece(wb, p0, n, pos, 0u, 0u, bd, mv & 255u);
                } else {                                /* bodies over 128 - tl bits */
                    uint32_t tv = 0, tl = 0;
                    piece_token(ctab, mv, nC, tv, tl);
                    if (one) put_piece1(wb, pos, tv, tl, bd, mv & 255u);
                    else put_piece(wb, p0, n, pos, tv, tl, bd, mv & 255u);
                }
            } else {
                ovf_put(wb, p0, n, pos, PT, TB, bd, ovf_wide(k, pc), pc, nC);
            }
        }
        __syncthreads();
        flush_window(wb, n, p0, p0 + n >= nw, out, &L.ncand, out + epc, EPC_ROW - 1, t, T);
        __syncthreads();
    }
    if (t == 0 && !lost) out[epc] = L.ncand;
    if (stp) {
        stp[5] = __builtin_amdgcn_s_memrealtime();
        stp[6] = bits;
        stp[7] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);     /* HW_ID */
    }
}

/* ---------------------------------------------------------------------- */
/* reading a NAL's RBSP straight from its row groups                      */
/* ---------------------------------------------------------------------- */
/* A dynamic NAL's RBSP exists only as its row groups' words (each group
 * from bit 0 of its row-stage slot); the row groups' bit counts give their
 * offsets (one wave scan; ngroups <= 64).  An RBSP word is assembled from
 * the (one, at group seams two or more) row-stage words it spans -- a
 * funnel shift.  ep_scan reads 4 EPS_KW NT bytes at a time, EPS_KW words
 * per thread, word w of a chunk thread w % NT's (neighbouring lanes read
 * neighbouring row-stage words, the next chunk's loads in flight while this
 * one is scanned). */
#ifndef SCROLL_EPS_KW
#define SCROLL_EPS_KW 4
#endif
/* EPS_KW words per thread and chunk (4 or 8) */
constexpr int EPS_KW = SCROLL_EPS_KW;
static_assert(EPS_KW % 4 == 0, "the EP scan reads 16-byte LDS vectors");
/* the group tables live in dynamic LDS sized by the NAL's group count
 * (goff [ng + 1], gb / gw [ng], then cw [ng] and cbase [ng + 1] where a
 * kernel has them): the benched rects' few groups take little LDS, a whole
 * 4K frame's 137 fit too */
__host__ __device__ inline size_t gtab_bytes(int ng, bool epfix)
{
    return (size_t)4 * (epfix ? 5 * (size_t)ng + 2 : 3 * (size_t)ng + 1);
}
struct GTab {
    uint32_t *goff, *gb, *gw, *cw, *cbase;
};
__device__ inline GTab gtab_of(uint32_t *p, int ng)
{
    GTab T;
    T.goff = p;
    T.gb = p + ng + 1;
    T.gw = T.gb + ng;
    T.cw = T.gw + ng;
    T.cbase = T.cw + ng;
    return T;
}

/* the RBSP word (MSB first) at bit P (a multiple of 32) of a NAL whose row
 * groups have offsets goff, bit counts gb and row-stage words at fr + gw;
 * gg: the group holding P or before it, advanced */
__device__ inline uint32_t rs_word_span(uint32_t P, int &gg, int ng, uint32_t T, const uint32_t *goff,
                                       const uint32_t *gb, const uint32_t *gw, const uint32_t *fr)
{
    uint32_t acc = 0, filled = 0;
    while (filled < 32u && gg < ng && P + filled < T) {
        const uint32_t lp = P + filled - goff[gg];
        if (lp >= gb[gg]) {                             /* group done (or empty) */
            ++gg;
            continue;
        }
        const uint32_t take = min(32u - filled, gb[gg] - lp);
        const uint32_t *src = fr + gw[gg];
        const uint32_t i = lp >> 5, sh = lp & 31u;
        uint32_t x = src[i];
        if (sh) {
            x <<= sh;
            if (32u - sh < take) x |= src[i + 1] >> (32u - sh);
        }
        x &= take >= 32u ? 0xffffffffu : ~(0xffffffffu >> take);
        acc |= x >> filled;
        filled += take;
    }
    return acc;
}

/* last group with goff[g] <= P */
__device__ inline int rs_group_at(uint32_t P, int ng, const uint32_t *goff)
{
    int lo = 0, hi = ng;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (goff[mid] <= P) lo = mid;
        else hi = mid;
    }
    return lo;
}

/* the first source words of the EPS_KW words thread t (of NT) assembles
 * for the chunk at byte c0 (x1: the next word, where the shift needs it) */
struct ScanLoads {
    uint32_t x0[EPS_KW], x1[EPS_KW], y[EPS_KW];           /* y: the next group's first word (seam words) */
    int g[EPS_KW];
};

template <int NT>
__device__ inline void scan_load(ScanLoads &L, uint32_t c0, int t, int ng, uint32_t T, const uint32_t *goff,
                                   const uint32_t *gb, const uint32_t *gw, const uint32_t *fr, int &gcarry)
{
    /* a thread's words only move forward: its group search starts from
     * where the previous chunk's ended (no binary search per chunk) */
    const uint32_t P0 = c0 * 8u + 32u * (uint32_t)t;
    int gg = gcarry;
    while (gg + 1 < ng && goff[gg + 1] <= P0) ++gg;
#pragma unroll
    for (int k = 0; k < EPS_KW; ++k) {
        const uint32_t P = P0 + 32u * NT * (uint32_t)k;
        while (gg + 1 < ng && goff[gg + 1] <= P) ++gg;
        L.g[k] = gg;
        const uint32_t lp = P - goff[gg], i = lp >> 5;
        const uint32_t *src = fr + gw[gg];
        L.x0[k] = P < T && lp < gb[gg] ? src[i] : 0u;
        L.x1[k] = P < T && (lp & 31u) && 32u * (i + 1) < gb[gg] ? src[i + 1] : 0u;
        const bool seam = P < T && gb[gg] - lp < 32u && gg + 1 < ng;
        L.y[k] = seam ? fr[gw[gg + 1]] : 0u;
    }
    gcarry = gg;
}

/* the row-group table of NAL nb in LDS (wave 0, 64 groups per step with
 * the offset carried): goff = bit offsets (goff[ng] = RBSP bits incl. the
 * stop bit), gb = bit counts, gw = first row-stage words in the frame's
 * region, cw = the groups' EP-candidate records.  cnt (k_dyn_epfix): each
 * group's candidate count, read with the table (the record word is the
 * count unless it names a spill slot) */
__device__ inline void rs_table(const uint32_t *gbits, size_t nb, const DynGeom &g, const uint32_t *fr,
                                uint32_t *goff, uint32_t *gb, uint32_t *gw, uint32_t *cw, int t,
                                uint32_t *bad = nullptr, uint32_t *cnt = nullptr)
{
    const int ng = g.ngroups;
    constexpr int SR = DYN_STATIC_ROWS;
    const int nA = max(1, (g.y0 + SR - 1) / SR);
    if (t >= 64) return;
    uint32_t carry = 0;
    for (int g0 = 0; g0 < ng; g0 += 64) {
        const int gi = g0 + t;
        const bool in = gi < ng;
        const bool row = gi >= nA && gi < nA + g.h;
        uint32_t w = (uint32_t)rs_group_words(g, nA, gi), c = (uint32_t)rs_runs_words(g, nA, gi);
        /* both loads in flight together */
        const uint32_t b = in ? gbits[nb * (size_t)ng + gi] : 0u;
        uint32_t m = in && (row || cnt) ? fr[c] : 0u;
        const uint32_t incl = wave_incl_sum(b, t);
        if (in) {
            gb[gi] = b;
            goff[gi] = carry + incl - b;
            /* a rect row that outgrew its slot: its record word names the
             * spill slot (relative to fr) holding its bits and record */
            if (row && (m & 0x80000000u)) {
                /* bounds check of the spill slot the record names: slot k
                 * of the pool after the rs_frames frame regions, k <
                 * rs_spill_cap (k_dyn_row's claim is bounded the same
                 * way).  A record outside the pool is never followed: the
                 * group reads its own slot and the frame is flagged bad */
                const uint64_t base = ((uint64_t)g.rs_frames - nb) * g.rs_frame_words;
                const uint64_t rel = (uint64_t)(m & 0x7fffffffu) - base;
                if ((m & 0x7fffffffu) >= base && rel % g.rs_spill_words == 0 &&
                    rel / g.rs_spill_words < g.rs_spill_cap) {
                    w = m & 0x7fffffffu;
                    c = w + g.rs_spill_words - EPC_ROW;
                    if (cnt) m = fr[c];
                } else {
                    if (bad) *bad = 1u;
                    m = 0u;
                }
            }
            gw[gi] = w;
            if (cw) cw[gi] = c;
            if (cnt) cnt[gi] = m;
        }
        carry += __shfl(incl, 63, 64);
    }
    if (t == 0) goff[ng] = carry;
}

/* the RBSP word (MSB first) at bit P, a multiple of 32 (0 past the end) */
__device__ inline uint32_t rs_word(uint32_t P, int ng, uint32_t T, const uint32_t *goff, const uint32_t *gb,
                                   const uint32_t *gw, const uint32_t *fr)
{
    if (P >= T) return 0u;
    int gg = rs_group_at(P, ng, goff);
    return rs_word_span(P, gg, ng, T, goff, gb, gw, fr);
}

/* w[i] for i in 0..8 without indexing (three levels of selects) */
__device__ inline uint32_t pick9(const uint32_t w[9], uint32_t i)
{
    const uint32_t a = (i & 1u) ? w[1] : w[0], b = (i & 1u) ? w[3] : w[2];
    const uint32_t c = (i & 1u) ? w[5] : w[4], e = (i & 1u) ? w[7] : w[6];
    const uint32_t ab = (i & 2u) ? b : a, ce = (i & 2u) ? e : c;
    const uint32_t r = (i & 4u) ? ce : ab;
    return (i & 8u) ? w[8] : r;
}

/* nine row-stage words from byte offset wo of the frame's region */
__device__ inline void rs_load9(__amdgpu_buffer_rsrc_t rr, uint32_t wo, uint32_t x[9])
{
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(rr, wo, 0, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(rr, wo + 16u, 0, 0);
    x[0] = (uint32_t)a[0]; x[1] = (uint32_t)a[1]; x[2] = (uint32_t)a[2]; x[3] = (uint32_t)a[3];
    x[4] = (uint32_t)b[0]; x[5] = (uint32_t)b[1]; x[6] = (uint32_t)b[2]; x[7] = (uint32_t)b[3];
    x[8] = __builtin_amdgcn_raw_buffer_load_b32(rr, wo + 32u, 0, 0);
}

/* the 32 RBSP bytes from bit P (a multiple of 128) as eight words in memory
 * order.  Inside one row group: nine row-stage words funnel-shifted by the
 * group's bit phase (gg: the thread's group, carried forward).  Across one
 * group seam (a few windows per NAL): the first group's words up to the seam
 * and the next group's words from its bit 0, shifted into place.  Three or
 * more groups (groups under 256 bits: rare) word by word.  Bits past the
 * NAL's end are unspecified (never used). */
__device__ inline void rs_load8(uint32_t P, int &gg, int ng, uint32_t T, const uint32_t *goff, const uint32_t *gb,
                                const uint32_t *gw, const uint32_t *fr, __amdgpu_buffer_rsrc_t rr, uint32_t w[8])
{
    if (goff[gg] > P) gg = rs_group_at(P, ng, goff);     /* never for increasing P */
    while (gg + 1 < ng && goff[gg + 1] <= P) ++gg;
    const uint32_t lp = P - goff[gg];
    const uint32_t end = goff[gg] + gb[gg];              /* the group's end (bits) */
    const bool two = P + 256u > end && gg + 1 < ng && (gg + 2 >= ng || P + 256u <= goff[gg + 2]) &&
                     gb[gg + 1] >= 256u;
    if (P + 256u <= end || gg + 1 >= ng || two) {
        uint32_t x[9];
        rs_load9(rr, 4u * (gw[gg] + (lp >> 5)), x);
        const uint32_t sh = lp & 31u;
        uint32_t a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = sh ? __builtin_amdgcn_alignbit(x[k], x[k + 1], 32u - sh) : x[k];
        if (two) {
            /* m bits from this group, then the next group from its bit 0 */
            const uint32_t m = end - P, dw = (m + 31u) >> 5, r = m & 31u;
            uint32_t y[9];
            rs_load9(rr, 4u * gw[gg + 1], y);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t kk = (uint32_t)k;
                uint32_t v;
                if (32u * kk + 32u <= m) {
                    v = a[k];
                } else if (32u * kk >= m) {                 /* next-group bits 32 k - m .. */
                    const uint32_t i0 = kk - dw;
                    const uint32_t lo = pick9(y, i0), hi = pick9(y, i0 + 1u);
                    v = r ? __builtin_amdgcn_alignbit(lo, hi, r) : lo;
                } else {                                    /* the seam word */
                    const uint32_t keep = m - 32u * kk;     /* 1..31 bits of this group */
                    v = (a[k] & ~(0xffffffffu >> keep)) | (y[0] >> keep);
                }
                a[k] = v;
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = __builtin_bswap32(a[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t Pk = P + 32u * (uint32_t)k;
            int g2 = gg;
            w[k] = Pk < T ? __builtin_bswap32(rs_word_span(Pk, g2, ng, T, goff, gb, gw, fr)) : 0u;
        }
    }
}

/* ---------------------------------------------------------------------- */
/* ep_scan: a NAL's emulation-prevention positions, read straight from its  */
/* row groups -- no staged copy of the RBSP                                 */
/* ---------------------------------------------------------------------- */
/* Per chunk: every word from the row-stage word(s) it spans (a funnel
 * shift), the chunk's bytes in LDS, then the closed-form EP rule per byte.
 * The zero run before the chunk comes from a look-back over the RBSP before
 * it, and only when the chunk's first byte is <= 3 (otherwise no byte of the
 * chunk can depend on it). */
/* A NAL whose EP sites the candidate records cannot give (DF_EPSLOW: a
 * group over its record's candidate slots, or more positions than ep_fix's
 * set holds) is scanned whole by its own k_dyn_epfix workgroup (NT
 * threads), chunk after chunk, the next chunk's loads in flight; cbuf: NT
 * EPS_KW words of LDS, wmax: NT / 64 words, ep_n: an LDS counter.  The
 * positions go straight to the frame's EP list in any order (the gather
 * sorts a DF_EPSLOW list); returns the NAL's EP byte count.  (Round 4 had
 * this in a launch of its own over a device-side list, k_dyn_epscan: one
 * launch per compose for NALs that config 3 never has) */
template <int NT>
__device__ uint32_t ep_scan(const uint32_t *fr, int ng, uint32_t T, const uint32_t *goff, const uint32_t *gb,
                            const uint32_t *gw, uint32_t *cbuf, int *wmax, uint32_t &ep_n, uint32_t *eplist, int t, uint32_t ecap)
{
    constexpr int CH = NT * 4 * EPS_KW;                 /* bytes per chunk */
    const uint32_t nin = (T + 7) >> 3;                  /* bitwriter.c:103-111 */
    uint4 *cbuf4 = reinterpret_cast<uint4 *>(cbuf);
    if (t == 0) ep_n = 0;
    __syncthreads();
    ScanLoads ld;
    int gcarry = 0;
    if (nin > 0) {
        gcarry = rs_group_at(32u * (uint32_t)t, ng, goff);
        scan_load<NT>(ld, 0u, t, ng, T, goff, gb, gw, fr, gcarry);
    }
    for (uint32_t c0 = 0; c0 < nin; c0 += CH) {
        {
            const uint32_t P0 = c0 * 8u + 32u * (uint32_t)t;
#pragma unroll
            for (int k = 0; k < EPS_KW; ++k) {
                const uint32_t P = P0 + 32u * NT * (uint32_t)k;
                const int g0 = ld.g[k];
                const uint32_t lp = P - goff[g0], sh = lp & 31u;
                uint32_t v = 0;
                if (P < T) {
                    const uint32_t avail = gb[g0] - lp;
                    v = sh ? (ld.x0[k] << sh) | (ld.x1[k] >> (32u - sh)) : ld.x0[k];
                    if (avail < 32u) {
                        v &= ~(0xffffffffu >> avail);
                        if (goff[g0] + gb[g0] < T) {          /* the word crosses a group seam */
                            if (g0 + 1 < ng && gb[g0 + 1] >= 32u - avail) {
                                v |= ld.y[k] >> avail;      /* the next group's first bits */
                            } else {                        /* groups under 32 bits: rare */
                                int g2 = g0;
                                v = rs_word_span(P, g2, ng, T, goff, gb, gw, fr);
                            }
                        }
                    }
                }
                cbuf[t + NT * k] = __builtin_bswap32(v);    /* memory order */
            }
        }
        const uint32_t cn = c0 + CH;
        if (cn < nin) scan_load<NT>(ld, cn, t, ng, T, goff, gb, gw, fr, gcarry);
        lds_barrier();                                  /* the next chunk's loads stay in flight */
        /* the last non-zero RBSP byte before the chunk: needed only when its
         * first byte is <= 3 (else that byte is non-zero and no EP decision
         * of the chunk reaches behind it) */
        int lz = -1;
        if (t == 0 && c0 > 0 && (cbuf[0] & 255u) <= 3u) {
            for (int64_t P = 8ll * c0 - 32; P >= 0; P -= 32) {
                const uint32_t w = rs_word((uint32_t)P, ng, T, goff, gb, gw, fr);
                if (w) {
                    lz = (int)(P >> 3) + 3 - (__builtin_ctz(w) >> 3);
                    break;
                }
            }
        }
        /* emulation prevention of this thread's 4 EPS_KW contiguous bytes */
        const uint32_t ib = c0 + 4u * EPS_KW * (uint32_t)t;
        uint32_t wv[EPS_KW];
#pragma unroll
        for (int j = 0; j < EPS_KW / 4; ++j) {
            const uint4 a = cbuf4[(EPS_KW / 4) * t + j];
            wv[4 * j] = a.x; wv[4 * j + 1] = a.y; wv[4 * j + 2] = a.z; wv[4 * j + 3] = a.w;
        }
        int lnz = -1;
#pragma unroll
        for (int w = 0; w < EPS_KW; ++w) {
            const uint32_t m = ib + 4u * w < nin ? wv[w] : 0u;
            if (m) lnz = (int)(ib + 4u * w) + 3 - (__builtin_clz(m) >> 3);
        }
        if (t == 0 && lnz < 0) lnz = lz;                /* the run reaching back past the chunk */
        int ex, tot;
        block_excl_max<NT / 64, true>(lnz, wmax, ex, tot);   /* its barriers also free cbuf */
        int prev = t == 0 ? lz : ex;
        uint32_t ins = 0;
#pragma unroll
        for (int i = 0; i < 4 * EPS_KW; ++i) {
            const uint32_t gi2 = ib + (uint32_t)i;
            const uint32_t b = gi2 < nin ? (wv[i >> 2] >> (8 * (i & 3))) & 255u : 256u;   /* past the end: never */
            ins |= (ep_insert(b, (int)gi2 - 1 - prev) ? 1u : 0u) << i;
            prev = b ? (int)gi2 : prev;
        }
        if (ins) {
            uint32_t k = atomicAdd(&ep_n, (uint32_t)__builtin_popcount(ins));
            while (ins) {
                const int i = __builtin_ctz(ins);
                ins &= ins - 1u;
                if (k < ecap) eplist[k] = ib + (uint32_t)i;   /* RBSP index the 03 precedes */
                k++;
            }
        }
    }
    __syncthreads();
    return ep_n;
}

/* ---------------------------------------------------------------------- */
/* k_dyn_epfix: a NAL's RBSP size and EP positions from the candidates      */
/* ---------------------------------------------------------------------- */
/* One workgroup per dynamic NAL.  The row groups' bit counts place the
 * groups, which fixes every byte's phase; then
 *   - each candidate word (ep_quick) is read back from its group's
 *     row-stage words: its exact runs, each run's EP bytes by arithmetic;
 *   - each group seam (NAL start included) is decided from the RBSP itself
 *     (read from the row groups a word at a time): from the byte holding
 *     the seam, with the zero run before it looked up backwards, up to the
 *     first non-zero byte at or after the first byte wholly inside the group
 *     (closed form of nal.c:33-38, ep_insert).
 * Every other byte is preceded by a non-zero byte within fewer than 22 zero
 * bits.  A byte can be decided twice (a run's last byte at a seam): kept
 * once.  More candidates in a group than its record holds, or more than EPF_LIST
 * positions: DF_EPSLOW (the workgroup scans the NAL, ep_scan). */
#ifndef SCROLL_EPF_T
#define SCROLL_EPF_T 128
#endif
#ifndef SCROLL_EPF_LIST
#define SCROLL_EPF_LIST 2048
#endif
constexpr int EPF_T = SCROLL_EPF_T;

/* an EP position (RBSP byte index j) into k_dyn_epfix's set: a bitmap over
 * the NAL's bytes (bm: duplicates merge, the order comes with the
 * compaction) or, for NALs past the bitmap's reach, a list (count *nlst,
 * capacity lcap) */
__device__ inline void ep_put(uint32_t j, bool bm, uint32_t *lst, uint32_t *nlst, uint32_t lcap)
{
    if (bm) {
        atomicOr(&lst[j >> 5], 1u << (j & 31u));
    } else {
        const uint32_t q = atomicAdd(nlst, 1u);
        if (q < lcap) lst[q] = j;
    }
}

/* the RBSP bytes from byte B on, with the zero run before it: EP positions
 * -> the set (ep_put) until the first non-zero byte at or after byte Bend */
__device__ inline void ep_eval_bytes(uint32_t B, uint32_t Bend, uint32_t nin, int ng, uint32_t T,
                                     const uint32_t *goff, const uint32_t *gb, const uint32_t *gw,
                                     const uint32_t *fr, bool bm, uint32_t *lst, uint32_t *nlst, uint32_t lcap)
{
    uint32_t cw = 0, ci = 0xffffffffu;                  /* one RBSP word cached */
    auto byte_at = [&](uint32_t i) -> uint32_t {
        if ((i >> 2) != ci) {
            ci = i >> 2;
            cw = rs_word(32u * ci, ng, T, goff, gb, gw, fr);
        }
        return (cw >> (8u * (3u - (i & 3u)))) & 255u;
    };
    int k = 0;                                          /* zero bytes right before B */
    for (int64_t i = (int64_t)B - 1; i >= 0; --i) {
        if (byte_at((uint32_t)i)) break;
        ++k;
    }
    for (uint32_t i = B; i < nin; ++i) {
        const uint32_t b = byte_at(i);
        if (ep_insert(b, k)) ep_put(i, bm, lst, nlst, lcap);
        if (b == 0) {
            ++k;
        } else {
            if (i >= Bend) break;
            k = 0;
        }
    }
}

/* the group holding candidate i: the last g < ng with cbase[g] <= i (empty
 * groups have empty ranges) */
__device__ inline int cand_group(uint32_t i, int ng, const uint32_t *cbase)
{
    int lo = 0, hi = ng;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (cbase[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

/* ep_fix's list mode (NALs over 32 LCAP bytes) for lists of n <= LCAP -
 * 4 NT entries: the NAL's bytes in windows of the LDS after the list (HW
 * words from the first multiple of 4 NT past n); per window every thread
 * sets the bits of the listed positions lst[0, n) that fall in it, then the
 * window's compaction emits them in order into eplist (duplicates merged)
 * -- no sort.  (Measured in round 4: a bitonic sort of the list took 22 us
 * per config-5 NAL on average, 119 at p99.)  Returns the positions emitted */
template <int NT, int LCAP>
__device__ __attribute__((always_inline)) inline uint32_t ep_list_windows(uint32_t *lst, uint32_t n, uint32_t nin,
                                                                          uint32_t *eplist, uint32_t *ws, int t,
                                                                          int lane, int wave, uint32_t ecap)
{
    const uint32_t ws0 = (n + 4u * NT - 1u) / (4u * NT) * (4u * NT);
    const uint32_t HW = (uint32_t)LCAP - ws0, CH = HW / (uint32_t)NT;   /* multiples of 4 NT / 4 */
    uint32_t *win = lst + ws0;
    const uint4 *wv = reinterpret_cast<const uint4 *>(win) + (uint32_t)t * (CH / 4u);
    uint32_t base = 0;
    for (uint32_t w0 = 0; w0 < nin; w0 += 32u * HW) {
        for (uint32_t i = (uint32_t)t; i < HW / 4u; i += (uint32_t)NT)
            reinterpret_cast<uint4 *>(win)[i] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        for (uint32_t i = (uint32_t)t; i < n; i += (uint32_t)NT) {
            const uint32_t v = lst[i] - w0;
            if (v < 32u * HW) atomicOr(&win[v >> 5], 1u << (v & 31u));
        }
        __syncthreads();
        uint32_t mine = 0;
        for (uint32_t k = 0; k < CH / 4u; ++k) {
            const uint4 q = wv[k];
            mine += (uint32_t)(__builtin_popcount(q.x) + __builtin_popcount(q.y) + __builtin_popcount(q.z) +
                               __builtin_popcount(q.w));
        }
        const uint32_t incl = wave_incl_sum(mine, lane);
        if (lane == 63) ws[wave] = incl;
        __syncthreads();
        uint32_t ex = base, tot = 0;
        for (int q = 0; q < NT / 64; ++q) {
            if (q < wave) ex += ws[q];
            tot += ws[q];
        }
        ex += incl - mine;
        for (uint32_t k = 0; mine && k < CH / 4u; ++k) {
            const uint4 q = wv[k];
            const uint32_t wv4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                for (uint32_t m = wv4[e]; m; m &= m - 1u) {
                    if (ex < ecap)
                        eplist[ex] = w0 + 32u * ((uint32_t)t * CH + 4u * k + (uint32_t)e) + (uint32_t)__builtin_ctz(m);
                    ++ex;
                }
        }
        base += tot;
        __syncthreads();                                /* the window and ws are reused */
    }
    return base;
}

/* k_dyn_epfix's work for NAL nb (stream s), every thread of the workgroup
 * (NT of them, at least two waves) calling: size, EP positions sorted and
 * each once into the frame's EP list (g.ep_cap kept), DF_FIXED set.  The
 * step is a chain of dependent loads per NAL (the measured round-4 split:
 * table 2.3 us, counts 1.2, seams + candidates 14.6, sort 4.7 per
 * workgroup), so the work is laid out for few round trips: the candidate
 * counts come with the table (same wave, one sync), the seams take the last
 * wave while the others take the candidates two at a time with their loads
 * in flight together, and the positions go into a bitmap over the NAL's
 * bytes (no sort: the compaction scan emits them in order, duplicates
 * merged).  (Measured in round 4: run by each NAL's last row workgroup
 * inside k_dyn_row instead, the agent-scope release fence every row
 * workgroup then needs -- L2 write-back across the XCDs -- made k_dyn_row
 * 9.6 ms.) */
template <int NT, int LCAP>
__device__ inline void ep_fix(DevStream *st, DynFrame *DF, size_t nb, int s, const DynGeom &g,
                              const uint32_t *rowstage, const uint32_t *gbits, uint8_t *eps, const EpfLds &E,
                              int t, uint64_t *stp)
{
    static_assert(NT >= 128 && NT % 64 == 0, "ep_fix: one seam wave and at least one candidate wave");
    static_assert(LCAP % (4 * NT) == 0 && LCAP >= 8 * NT, "ep_fix: the bitmap in whole 16-byte chunks per thread");
    /* stp (debug, SCROLL_DEBUG_DYN_STAMPS): realtime at entry and after each
     * step (tools/dyn_stamps.py) */
    auto stamp = [&](int k) {
        if (stp && t == 0) stp[k] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    uint32_t *goff = E.goff, *gb = E.gb, *gw = E.gw, *cw = E.cw, *cbase = E.cbase, *lst = E.lst;
    uint32_t &nlst = E.cnt[0], &nu = E.cnt[1], &slow = E.cnt[2], &bad = E.cnt[3];
    const uint32_t lcap = LCAP;
    const uint32_t err0 = DF->err;
    if (err0 & (DF_OVER | DF_HANDOFF)) {                /* k_dyn_rows / k_dyn_row: pools exhausted,
                                                           or a row's wait expired */
        if (t == 0) {
            DF->rbsp_bytes = 0;
            DF->ep = 0;
            DF->err = err0 | DF_FIXED;
            atomicOr((unsigned int *)&st[s].err,
                     (err0 & DF_HANDOFF) ? SCROLL_DEVERR_HANDOFF : SCROLL_DEVERR_DYN);
        }
        return;
    }
    const int ng = g.ngroups;
    constexpr int SR = DYN_STATIC_ROWS;
    const int nA = max(1, (g.y0 + SR - 1) / SR);
    const uint32_t *fr = rowstage + nb * g.rs_frame_words;
    /* the bitmap starts empty (list mode overwrites what it uses) */
    for (uint32_t i = (uint32_t)t; i < lcap / 4u; i += (uint32_t)NT)
        reinterpret_cast<uint4 *>(lst)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (t < 64) {
        if (t == 0) bad = 0u;
        wave_sync();
        /* the groups' candidate counts (into cbase), then their bases */
        rs_table(gbits, nb, g, fr, goff, gb, gw, cw, t, &bad, cbase);
        wave_sync();
        uint32_t carry = 0;
        bool ov = false;
        for (int g0 = 0; g0 < ng; g0 += 64) {
            const int gi = g0 + t;
            const uint32_t c = gi < ng ? cbase[gi] : 0u;
            const uint32_t cmax = (gi >= nA && gi < nA + g.h) ? EPC_ROW - 1u : EPC_STATIC - 1u;
            const uint32_t cc = min(c, cmax);
            const uint32_t incl = wave_incl_sum(cc, t);
            if (gi < ng) cbase[gi] = carry + incl - cc;
            ov |= __builtin_amdgcn_ballot_w64(c > cmax) != 0;
            carry += __shfl(incl, 63, 64);
        }
        if (t == 0) {
            cbase[ng] = carry;
            slow = ov ? 1u : 0u;
            nlst = 0;
        }
    }
    __syncthreads();
    stamp(1);
    if (bad) {                                          /* a spill record outside the pool (never) */
        if (t == 0) {
            DF->err = DF_OVER | DF_FIXED;
            DF->rbsp_bytes = 0;
            DF->ep = 0;
            atomicOr((unsigned int *)&st[s].err, SCROLL_DEVERR_DYN);
        }
        return;
    }
    const uint32_t T = goff[ng];                        /* NAL RBSP bits incl. the stop bit */
    const uint32_t nin = (T + 7) >> 3;                  /* bitwriter.c:103-111 */
    if (((nin + 31u) & ~31u) > g.slot_bytes - DYN_OVF_BYTES) {   /* the cap the API sets */
        if (t == 0) {
            DF->err = DF_OVER | DF_FIXED;
            DF->rbsp_bytes = 0;
            DF->ep = 0;
            atomicOr((unsigned int *)&st[s].err, SCROLL_DEVERR_DYN);
        }
        return;
    }
    const uint32_t nbw = (nin + 31u) >> 5;              /* bitmap words */
    const bool bm = nbw <= lcap;
    const int wave = t >> 6, lane = t & 63;
    constexpr int NC = NT;                              /* candidate threads: all */
    const uint32_t nc = cbase[ng];
    if (!slow) {
        if (wave == NT / 64 - 1) {
            /* the seam before group k (0: NAL start): its bytes from the
             * RBSP.  (Measured in round 4: from a 64-bit register window of
             * the two groups, one round of loads -- the byte path remained
             * only for the NAL start -- 0.060 against 0.055 ms per launch:
             * shorter workgroups, but fewer of them resident) */
            for (int k = lane; k < ng; k += 64) {
                const uint32_t S = goff[k];
                if (S < T) ep_eval_bytes(S >> 3, (S + 7) >> 3, nin, ng, T, goff, gb, gw, fr, bm, lst, &nlst, lcap);
            }
            if (stp && lane == 0) stp[7] = __builtin_amdgcn_s_memrealtime();   /* the seam wave's end */
        }
        /* candidate words, CB per thread and pass: the index loads, then
         * the three data words of each, then the runs */
        constexpr int CB = NC >= 192 ? 2 : 4;
        for (uint32_t i0 = 0; i0 < nc; i0 += (uint32_t)(CB * NC)) {
            uint32_t wi[CB], gg[CB];
#pragma unroll
            for (int q = 0; q < CB; ++q) {
                const uint32_t ci = i0 + (uint32_t)(q * NC + t);
                gg[q] = ci < nc ? (uint32_t)cand_group(ci, ng, cbase) : 0u;
                wi[q] = ci < nc ? fr[cw[gg[q]] + 1u + (ci - cbase[gg[q]])] : 0xffffffffu;
            }
            uint32_t pw[CB], w[CB], nx[CB], nwd[CB];
#pragma unroll
            for (int q = 0; q < CB; ++q) {
                const uint32_t *src = fr + gw[gg[q]];
                nwd[q] = (gb[gg[q]] + 31u) >> 5;
                const bool ok = wi[q] < nwd[q];
                pw[q] = ok && wi[q] ? src[wi[q] - 1u] : 0u;
                w[q] = ok ? src[wi[q]] : 0u;
                nx[q] = ok && wi[q] + 1u < nwd[q] ? src[wi[q] + 1u] : 0u;
            }
#pragma unroll
            for (int q = 0; q < CB; ++q) {
                if (wi[q] >= nwd[q]) continue;
                const uint32_t bits = gb[gg[q]], O = goff[gg[q]], x = wi[q];
                const uint32_t *src = fr + gw[gg[q]];
                const uint32_t wd = ep_data(w[q], x, bits);
                const uint32_t nd = x + 1u < nwd[q] ? ep_data(nx[q], x + 1u, bits) : 0xffffffffu;
                uint32_t m = ep_run_starts(pw[q], wd, nd, x, bits);
                while (m) {                             /* usually one run */
                    const uint32_t a = (uint32_t)__builtin_clz(m);
                    m &= ~(0x80000000u >> a);
                    const uint64_t Y = ((uint64_t)wd << 32 | nd) << a;
                    uint32_t e = bits;
                    if (Y) {
                        e = 32u * x + a + (uint32_t)__builtin_clzll(Y);
                    } else {
                        for (uint32_t r = x + 2u; r < nwd[q]; ++r) {
                            const uint32_t v = ep_data(src[r], r, bits);
                            if (v) {
                                e = 32u * r + (uint32_t)__builtin_clz(v);
                                break;
                            }
                        }
                    }
                    const uint32_t A = (O + 32u * x + a + 7u) & ~7u, E2 = O + e;
                    for (uint32_t j = A + 16u; j + 6u <= E2; j += 16u) ep_put(j >> 3, bm, lst, &nlst, lcap);
                }
            }
        }
        stamp(4);                                       /* wave 0's candidates done */
    }
    __syncthreads();
    stamp(2);
    const uint32_t n = nlst;
    uint32_t *eplist = reinterpret_cast<uint32_t *>(eps + nb * eps_stride(g));
    if (slow || (!bm && n > lcap)) {                    /* the whole NAL scanned here */
        static_assert(NT * EPS_KW <= LCAP, "ep_scan's chunk buffer is the position set's LDS");
        __syncthreads();                                /* every thread is past the set */
        const uint32_t ne = ep_scan<NT>(fr, ng, T, goff, gb, gw, lst, reinterpret_cast<int *>(E.ws), nlst, eplist, t, g.ep_cap);
        if (t == 0) {
            DF->err = DF_EPSLOW | DF_FIXED;             /* the list unsorted: the gather sorts it */
            DF->rbsp_bytes = nin;
            DF->ep = ne;
        }
        return;
    }
    constexpr int CW = LCAP / NT;                       /* bitmap words per thread (whole bitmap) */
    if (!bm && n <= lcap - 4u * NT) {
        const uint32_t base = ep_list_windows<NT, LCAP>(lst, n, nin, eplist, E.ws, t, lane, wave, g.ep_cap);
        stamp(3);
        if (t == 0) nu = base;
    } else if (!bm) {
        /* a list too long to leave a window: a bitonic sort of the list
         * padded to a power of two (log^2 steps, one compare-exchange per
         * thread and step), then the first of each run of equal positions
         * goes to its rank */
        const uint32_t P = n <= 1u ? 1u : 1u << (32 - __builtin_clz(n - 1u));   /* <= lcap */
        for (uint32_t i = (uint32_t)t + n; i < P; i += (uint32_t)NT) lst[i] = 0xffffffffu;
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = (uint32_t)t; i < P; i += (uint32_t)NT) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const uint32_t a = lst[i], b = lst[l];
                        if ((a > b) == ((i & k) == 0u)) {
                            lst[i] = b;
                            lst[l] = a;
                        }
                    }
                }
                __syncthreads();
            }
        stamp(3);
        const uint32_t C = (n + (uint32_t)NT - 1u) / (uint32_t)NT, c0 = (uint32_t)t * C, c1 = min(c0 + C, n);
        uint32_t mine = 0;
        for (uint32_t i = c0; i < c1; ++i) mine += (i == 0u || lst[i] != lst[i - 1u]) ? 1u : 0u;
        uint32_t ex = 0;
        const uint32_t incl = wave_incl_sum(mine, lane);
        if (lane == 63) E.ws[wave] = incl;
        __syncthreads();
        for (int q = 0; q < wave; ++q) ex += E.ws[q];
        ex += incl - mine;
        if (t == NT - 1) nu = ex + mine;
        for (uint32_t i = c0; i < c1; ++i)
            if (i == 0u || lst[i] != lst[i - 1u]) {
                if (ex < g.ep_cap) eplist[ex] = lst[i];
                ++ex;
            }
    } else {
        stamp(3);
        /* bitmap mode: the threads' CW words held in registers, a scan,
         * then each chunk's positions in order from its rank */
        uint4 bw[CW / 4];
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < CW / 4; ++k) {
            bw[k] = reinterpret_cast<const uint4 *>(lst)[t * (CW / 4) + k];
            mine += (uint32_t)(__builtin_popcount(bw[k].x) + __builtin_popcount(bw[k].y) +
                               __builtin_popcount(bw[k].z) + __builtin_popcount(bw[k].w));
        }
        uint32_t ex = 0;
        {
            const uint32_t incl = wave_incl_sum(mine, lane);
            if (lane == 63) E.ws[wave] = incl;
            __syncthreads();
            for (int q = 0; q < wave; ++q) ex += E.ws[q];
            ex += incl - mine;
            if (t == NT - 1) nu = ex + mine;
        }
        if (mine) {
#pragma unroll
            for (int k = 0; k < CW / 4; ++k) {
                const uint32_t wv4[4] = {bw[k].x, bw[k].y, bw[k].z, bw[k].w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    for (uint32_t m = wv4[e]; m; m &= m - 1u) {
                        if (ex < g.ep_cap)
                            eplist[ex] = 32u * (uint32_t)(t * CW + 4 * k + e) + (uint32_t)__builtin_ctz(m);
                        ++ex;
                    }
            }
        }
    }
    __syncthreads();
    if (t == 0) {
        DF->err = DF_FIXED;                             /* clears DF_GENERAL */
        DF->rbsp_bytes = nin;
        DF->ep = nu;
        if (stp) stp[6] = (uint64_t)nc | (uint64_t)nu << 32;
    }
    stamp(5);
}

/* grid (frames, streams): one workgroup per NAL.  (Measured: one wave per
 * NAL, four NALs per workgroup, 0.138 against 0.086 ms -- each NAL's
 * candidate and seam loops then take several passes of 64 lanes.) */
constexpr int EPF_LIST = SCROLL_EPF_LIST;
/* waves per SIMD the epfix registers target (SCROLL_EPF_WAVES; 0: the
 * compiler's choice) */
#ifndef SCROLL_EPF_WAVES
#define SCROLL_EPF_WAVES 0
#endif
#if SCROLL_EPF_WAVES
#define EPF_ATTR __attribute__((amdgpu_waves_per_eu(SCROLL_EPF_WAVES)))
#else
#define EPF_ATTR
#endif
template <int NT, int LCAP>
__global__ __launch_bounds__(NT) EPF_ATTR void k_dyn_epfix(DevStream *__restrict__ st, DynFrame *__restrict__ dfr,
                                                     int ld_fr, int nframes, DynGeom g,
                                                     const uint32_t *__restrict__ rowstage,
                                                     const uint32_t *__restrict__ gbits, uint8_t *__restrict__ eps,
                                                     uint64_t *__restrict__ stamps)
{
    __shared__ __attribute__((aligned(16))) uint32_t lst[LCAP];   /* the position bitmap / list */
    extern __shared__ uint32_t gdyn[];                  /* the group tables (gtab_bytes); cbase: runs before group g */
    const GTab GT = gtab_of(gdyn, g.ngroups);
    uint32_t *goff = GT.goff, *gb = GT.gb, *gw = GT.gw, *cw = GT.cw, *cbase = GT.cbase;
    __shared__ uint32_t cnt[4], ws[NT / 64];
    const int f = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
    if (f >= nframes) return;
    const size_t nb = (size_t)s * ld_fr + f;
    DynFrame *DF = dfr + nb;
    if (DF->nal < 0) return;
    const EpfLds E{goff, gb, gw, cw, cbase, lst, cnt, ws};
    ep_fix<NT, LCAP>(st, DF, nb, s, g, rowstage, gbits, eps, E, t, stamps ? stamps + ((size_t)s * nframes + f) * 8 : nullptr);
}
/* the whole-picture rects' NALs (~300 KB at 720p) hold more EP bytes than
 * the 2,048-entry set (a quarter of p720full's frames had ~2,200: the whole
 * NAL then went through ep_scan and emit_serial, one workgroup each: gather
 * 1.17 + epfix 0.76 ms per step, now 0.18 + 0.10): an 8,192-entry set for
 * rects over EPF_BIG_MBS MBs.  Config 5 (2,209 MBs, 221 KB NALs: the bitmap
 * covers them) 2.93 -> 2.86 ms per step with it; config 3 (625 MBs) 1.47
 * -> 1.56 (fewer resident workgroups), so it keeps the small one.
 * SCROLL_EPF_BIG=0 / 1 forces the small / big form */
constexpr int EPF_BIG_LIST = 8192;
constexpr int EPF_BIG_MBS = 1024;
/* (measured, round 6: 256 threads per workgroup for launches of few NALs --
 * one frame per stream, 256 NALs, a workgroup per CU -- no change) */
inline bool epf_big_rect(int64_t mbs)
{
    static const int env = [] {
        const char *e = getenv("SCROLL_EPF_BIG");
        return e ? atoi(e) : -1;
    }();
    return env >= 0 ? env != 0 : mbs > EPF_BIG_MBS;
}

/* ---------------------------------------------------------------------- */
/* emit_serial: RBSP -> arena with start code, header, EP bytes            */
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

/* The NALs with more EP bytes than the gathers keep positions for
 * (ep_cap: past 2,048, or 4 under SCROLL_DEBUG_DYN_EPCAP4): one workgroup
 * streams the NAL through an LDS byte buffer, finding the EP sites on the
 * way.  Called by the gather workgroup of the NAL (z = 0) in place of its
 * chunk loop -- no launch of its own.  rowstage != nullptr: the dynamic
 * rect's NALs, whose RBSP lives only in their row groups (gbits, tables in
 * goff / gb / gw); else the staged RBSP of the hint / splice path.  ob: OBUF
 * bytes (16-byte aligned), wmax / wsum: NW words each, of the caller's LDS */
__device__ __attribute__((always_inline)) inline void emit_serial(const NalDesc &d, const DynFrame &df, size_t nb, int s,
                                                      const DynGeom &g, const uint8_t *__restrict__ stage,
                                                      const uint32_t *__restrict__ rowstage,
                                                      const uint32_t *__restrict__ gbits,
                                                      uint8_t *__restrict__ arena, uint64_t ld_arena,
                                                      uint32_t *goff, uint32_t *gb, uint32_t *gw, uint8_t *ob,
                                                      int32_t *wmax, uint32_t *wsum, int t)
{
    uint8_t *A = arena + (size_t)s * ld_arena;
    const uint64_t o0 = d.out_off, o1 = o0 + d.size;
    const bool RS = rowstage != nullptr;
    const uint8_t *in = RS ? nullptr : stage + nb * g.slot_bytes;
    const uint32_t *fr = RS ? rowstage + nb * g.rs_frame_words : nullptr;
    if (RS) rs_table(gbits, nb, g, fr, goff, gb, gw, nullptr, t);
    __syncthreads();
    const int ng = g.ngroups;
    const uint32_t T = RS ? goff[ng] : 0u;
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
            uint4 v = make_uint4(0, 0, 0, 0);
            if (n && RS) {
                const uint32_t P = 8u * ib;
                v = make_uint4(__builtin_bswap32(rs_word(P, ng, T, goff, gb, gw, fr)),
                               __builtin_bswap32(rs_word(P + 32u, ng, T, goff, gb, gw, fr)),
                               __builtin_bswap32(rs_word(P + 64u, ng, T, goff, gb, gw, fr)),
                               __builtin_bswap32(rs_word(P + 96u, ng, T, goff, gb, gw, fr)));
            } else if (n) {
                v = *reinterpret_cast<const uint4 *>(in + ib);
            }
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
static_assert(OBUF <= 4 * EPLIST_MAX && NW <= EPLIST_MAX, "emit_serial's buffers fit the gathers' LDS lists");

/* ---------------------------------------------------------------------- */
/* k_dyn_emit_gather: the same output for NALs with <= EPLIST_MAX EP bytes  */
/* (all in practice: 82 per config-3 frame).  k_dyn_epfix recorded where    */
/* the 03 bytes go; after sorting those positions once, every thread builds */
/* whole 16-byte arena chunks independently -- no barriers, no LDS byte     */
/* buffer: a chunk without an EP byte is a funnel shift of the row groups.  */
/* ---------------------------------------------------------------------- */
__device__ inline uint32_t pick4(const uint32_t w[8], int i)     /* w[i], i in 0..7, no indexing */
{
    const uint32_t a = (i & 1) ? w[1] : w[0], b = (i & 1) ? w[3] : w[2];
    const uint32_t c = (i & 1) ? w[5] : w[4], e = (i & 1) ? w[7] : w[6];
    const uint32_t ab = (i & 2) ? b : a, ce = (i & 2) ? e : c;
    return (i & 4) ? ce : ab;
}

#ifndef SCROLL_GATHER_Z
#define SCROLL_GATHER_Z 1
#endif
constexpr int GATHER_Z = SCROLL_GATHER_Z;             /* workgroups per NAL (2 and 4 measured slower) */

/* RS: the dynamic rect's NALs -- RBSP bytes assembled from the row groups
 * (rs_load8), EP lists at stage + DYN_OVF_BYTES per frame (k_dyn_epfix);
 * else the staged RBSP + slot-tail EP list of the hint / splice path */
template <int U, bool RS>
__global__ __launch_bounds__(DT) void k_dyn_emit_gather(const DevStream *__restrict__ st,
                                                        const NalDesc *__restrict__ nal, int ld_nal,
                                                        const DynFrame *__restrict__ dfr, int ld_fr,
                                                        DynGeom g, const uint8_t *__restrict__ stage,
                                                        const uint32_t *__restrict__ rowstage,
                                                        const uint32_t *__restrict__ gbits,
                                                        uint8_t *__restrict__ arena, uint64_t ld_arena,
                                                        uint64_t *__restrict__ stamps)
{
    __shared__ alignas(16) uint32_t raw[EPLIST_MAX];
    __shared__ uint32_t sp[EPLIST_MAX];
    extern __shared__ uint32_t gdyn[];                  /* RS: the group tables (gtab_bytes) */
    const GTab GT = gtab_of(gdyn, RS ? g.ngroups : 0);
    uint32_t *goff = GT.goff, *gb = GT.gb, *gw = GT.gw;
    const int s = blockIdx.y, f = dyn_frame_of(blockIdx.x, s), t = threadIdx.x;
    /* debug: realtime at entry / after the sort / at exit, EP count, HW_ID */
    uint64_t *stp = stamps && t == 0 && blockIdx.z == 0 ? stamps + ((size_t)s * gridDim.x + f) * 8 : nullptr;
    if (stp) stp[0] = __builtin_amdgcn_s_memrealtime();
    const DynFrame df = dfr[(size_t)s * ld_fr + f];
    const int j = df.nal;
    if (j < 0 || j >= st[s].nnal || (df.err & ~(DF_EPSLOW | DF_FIXED))) return;   /* nnal = 0: nothing committed */
    const uint32_t n = df.ep;
    const NalDesc d = nal[(size_t)s * ld_nal + j];
    if (d.slow != 2) return;
    const size_t nb = (size_t)s * ld_fr + f;
    if (n > min(ep_cap(g, RS), (uint32_t)EPLIST_MAX)) {     /* past the position list: streamed */
        if (blockIdx.z == 0)
            emit_serial(d, df, nb, s, g, stage, rowstage, gbits, arena, ld_arena, goff, gb, gw,
                        reinterpret_cast<uint8_t *>(raw), reinterpret_cast<int32_t *>(sp), sp + NW, t);
        return;
    }
    const uint8_t *in = RS ? nullptr : stage + nb * g.slot_bytes;
    const uint32_t *el = reinterpret_cast<const uint32_t *>(RS ? stage + nb * eps_stride(g)
                                                               : in + g.slot_bytes - DYN_OVF_BYTES);
    const uint32_t *fr = RS ? rowstage + nb * g.rs_frame_words : nullptr;
    if (RS) rs_table(gbits, nb, g, fr, goff, gb, gw, nullptr, t);
    /* ep_fix leaves the list sorted (not ep_scan, nor the hint / splice path) */
    const bool sorted = RS && !(df.err & DF_EPSLOW);
    for (uint32_t i = t; i < n; i += DT) (sorted ? sp : raw)[i] = el[i];
    __syncthreads();
    const int ng = RS ? g.ngroups : 0;
    const uint32_t T = RS ? goff[ng] : 0u;
    /* the frame's row groups, and spill slots up to 4 GB past them (k_dyn_row's bound) */
    const __amdgpu_buffer_rsrc_t rr = buf_rsrc(fr, RS ? 0xfffffffcu : 0u);
    int gcar = 0;                                            /* RS: the thread's row group */
    /* sort by rank (positions are distinct): sp[j] = j-th smallest */
    for (uint32_t i = t; i < (sorted ? 0u : n); i += DT) {
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
                if constexpr (RS) {
                    uint32_t w8[8];
                    rs_load8(8u * a0, gcar, ng, T, goff, gb, gw, fr, rr, w8);
                    x[u] = make_uint4(w8[0], w8[1], w8[2], w8[3]);
                    y[u] = make_uint4(w8[4], w8[5], w8[6], w8[7]);
                } else {
                    x[u] = *reinterpret_cast<const uint4 *>(in + a0);
                    if (a0 + 16 < nin) y[u] = *reinterpret_cast<const uint4 *>(in + a0 + 16);
                }
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
                /* RS: the <= 16 RBSP bytes of this chunk lie in the 32 from a0 */
                uint32_t w8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a0 = 0;
                if constexpr (RS) {
                    const int64_t ue = (int64_t)q0 - (int64_t)o0 - 5;
                    a0 = (uint32_t)(ue > 0 ? ue : 0) - kk;
                    a0 &= ~15u;
                    if (a0 < nin) rs_load8(8u * a0, gcar, ng, T, goff, gb, gw, fr, rr, w8);
                }
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
                    } else if constexpr (RS) {
                        const uint32_t r = (uint32_t)uu - kk - a0;           /* < 32 */
                        const uint32_t wd = pick4(w8, (int)(r >> 2));
                        v = (uint8_t)(wd >> (8u * (r & 3u)));
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
/* k_dyn_gather: the dynamic rect's NALs -> arena, one chunk per thread on  */
/* one straight path                                                        */
/* ---------------------------------------------------------------------- */
/* Round 4's replacement of k_dyn_emit_gather<., true> (≈440 VALU
 * instructions per 16-byte chunk there, in 64-bit index arithmetic, pick
 * trees and per-case branches).  Per 16-byte arena chunk inside the NAL:
 *   K  = EP bytes before it (coarse index per 2^cs EBSP bytes + a short
 *        step over the sorted positions); its first RBSP byte i0 = u0 - K;
 *   R  = the 128 RBSP bits from byte i0: five row-stage words of the group
 *        holding them funnel-shifted by the bit phase, merged at a group
 *        seam with the next group's first four words (a 128-bit shift and
 *        mask, computed by every lane: no branch);
 *   each EP byte inside the chunk (sorted list, usually none): the tail
 *   shifts right one byte and 03 goes in;
 *   R byte-swapped -> one 16-byte store.
 * Chunks at the NAL's ends (start code, header, the last partial chunk) and
 * chunks meeting three groups (groups under 128 bits: tiny rects) take a
 * byte loop.  Grid (frames, streams, Z): workgroup z owns 1/Z of the NAL's
 * chunks. */
/* workgroups per NAL (grid z): one per ~640 rect MBs -- a config-3 NAL
 * (25 x 25 MBs, ~116 KB) keeps one (Z = 2 measured equal), the whole-picture
 * rects of the fallback (80 x 45: ~350 KB per NAL, 1,024 NALs = 4 workgroups
 * per CU at Z = 1) take 5, at most 16 -- and at least GATHER_MIN_WG
 * workgroups in all (round 6: a compose of one frame per stream, 256 NALs,
 * had one workgroup per CU, 46 us of latency-bound gather).  nnal: the NAL
 * slots launched.  SCROLL_GATHER_Z overrides it */
constexpr int64_t GATHER_MIN_WG = 2048;
inline int gather_z(const DynGeom &g, int64_t nnal)
{
    static const int env = [] {
        const char *e = getenv("SCROLL_GATHER_Z");
        return e ? atoi(e) : 0;
    }();
    if (env > 0) return env < 64 ? env : 64;
    int64_t z = (int64_t)g.w * g.h / 640;
    if (nnal > 0 && z * nnal < GATHER_MIN_WG) z = (GATHER_MIN_WG + nnal - 1) / nnal;
    return (int)(z < 1 ? 1 : (z > 16 ? 16 : z));
}
/* Two chunk sets per thread in turn, the next chunk's loads in flight while
 * one is assembled (round 5: 0.142 against 0.146 ms per config-3 launch for
 * one chunk at a time, that form since removed).  Measured and not kept:
 * non-temporal arena stores (0.143), non-temporal row-stage loads (0.153) */

/* 128-bit helpers on four words, word 0 most significant */
struct W4 {
    uint32_t w[4];
};
/* x >> s (logical), 0 <= s < 128 */
__device__ inline W4 shr128(const W4 &x, uint32_t s)
{
    const uint32_t q = s >> 5, r = s & 31u;
    uint32_t a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        /* word k of the result: words k - q (hi part) and k - q - 1 */
        const int i = k - (int)q;
        const uint32_t hi = i >= 0 ? (i == 0 ? x.w[0] : (i == 1 ? x.w[1] : (i == 2 ? x.w[2] : x.w[3]))) : 0u;
        const int j = i - 1;
        const uint32_t lo = j >= 0 ? (j == 0 ? x.w[0] : (j == 1 ? x.w[1] : x.w[2])) : 0u;
        a[k] = r ? __builtin_amdgcn_alignbit(lo, hi, r) : hi;
    }
    return W4{{a[0], a[1], a[2], a[3]}};
}

__global__ __launch_bounds__(DT) __attribute__((amdgpu_waves_per_eu(8))) void k_dyn_gather(const DevStream *__restrict__ st,
                                                  const NalDesc *__restrict__ nal, int ld_nal,
                                                  const DynFrame *__restrict__ dfr, int ld_fr, DynGeom g,
                                                  const uint8_t *__restrict__ eps,
                                                  const uint32_t *__restrict__ rowstage,
                                                  const uint32_t *__restrict__ gbits,
                                                  uint8_t *__restrict__ arena, uint64_t ld_arena,
                                                  uint64_t *__restrict__ stamps)
{
    __shared__ alignas(16) uint32_t raw[EPLIST_MAX];
    __shared__ uint32_t sp[EPLIST_MAX + 1];
    extern __shared__ uint32_t gdyn[];                  /* the group tables (gtab_bytes) */
    const GTab GT = gtab_of(gdyn, g.ngroups);
    uint32_t *goff = GT.goff, *gb = GT.gb, *gw = GT.gw;
    const int s = blockIdx.y, f = dyn_frame_of(blockIdx.x, s), t = threadIdx.x;
    const DynFrame df = dfr[(size_t)s * ld_fr + f];
    const int j = df.nal;
    if (j < 0 || j >= st[s].nnal || (df.err & ~(DF_EPSLOW | DF_FIXED))) return;   /* nnal = 0: nothing committed */
    const uint32_t n = df.ep;
    const NalDesc d = nal[(size_t)s * ld_nal + j];
    if (d.slow != 2) return;
    const bool sorted = !(df.err & DF_EPSLOW);
    /* past the position list, or an unsorted list (ep_scan's) longer than
     * the LDS holds: streamed */
    /* positions per LDS window (SCROLL_DEBUG_DYN_EPWIN: 7, so the tests'
     * NALs take the window path) */
    const uint32_t wcap = (g.debug & SCROLL_DEBUG_DYN_EPWIN) ? 7u : (uint32_t)EPLIST_MAX - 1u;
    if (n > ep_cap(g, true) || (!sorted && n > wcap)) {
        if (blockIdx.z == 0)
            emit_serial(d, df, (size_t)s * ld_fr + f, s, g, nullptr, rowstage, gbits, arena, ld_arena, goff, gb,
                        gw, reinterpret_cast<uint8_t *>(raw), reinterpret_cast<int32_t *>(sp), sp + NW, t);
        return;
    }
    /* debug (SCROLL_DEBUG_DYN_STAMPS): realtime at entry, after the prologue, at the end */
    uint64_t *stp = stamps && blockIdx.z == 0 && t == 0 ? stamps + ((size_t)s * gridDim.x + blockIdx.x) * 8 : nullptr;
    if (stp) stp[0] = __builtin_amdgcn_s_memrealtime();
    const size_t nb = (size_t)s * ld_fr + f;
    const uint32_t *el = reinterpret_cast<const uint32_t *>(eps + nb * eps_stride(g));
    const uint32_t *fr = rowstage + nb * g.rs_frame_words;
    rs_table(gbits, nb, g, fr, goff, gb, gw, nullptr, t);
    const int ng = g.ngroups;
    const __amdgpu_buffer_rsrc_t rr = buf_rsrc(fr, 0xfffffffcu);   /* the frame's groups + spill slots */
    uint8_t *A = arena + (size_t)s * ld_arena;
    const uint64_t o0 = d.out_off, o1 = o0 + d.size;
    const uint8_t hdr[5] = {0, 0, 0, 1, nal_header_byte(0)};           /* nal.c:59-64 */
    const uint64_t cfirst = o0 >> 4;
    const uint32_t cnal = (uint32_t)(((o1 + 15) >> 4) - cfirst);
    const uint32_t per = (cnal + gridDim.z - 1) / gridDim.z;
    const uint32_t cbeg = per * blockIdx.z, cend = min(cnal, cbeg + per);
    /* EBSP index of chunk c's byte 0: 16 c - d0 (d0 = o0 - 16 cfirst + 5) */
    const int32_t d0 = (int32_t)(o0 - (cfirst << 4)) + 5;
    const int32_t nebsp = (int32_t)(d.size - 5);
    int gg = 0;                                              /* the thread's group, carried */
    /* The EP positions in LDS: the whole sorted list when it fits (every
     * benched NAL but the whole-picture rect's heaviest), else windows of the
     * workgroup's chunks whose EP bytes fit (round 6).  The j-th EP byte sits
     * at EBSP index el[j] + j; the LDS copy holds window positions j = kb + k
     * as sp[k] = el[kb + k] + kb, so sp[k] + k is that index and K (a local
     * count) + kb the EP bytes before a chunk.  raw: the window's coarse index
     * (EP bytes before EBSP index ub + (b << cs)) */
    const bool whole = n <= wcap;
    __shared__ uint32_t win[3];                              /* kb, m, ce of the next window */
    uint32_t kb = 0, T = 0;
    int32_t ub = 0;
    int cs = 8, nblk = 1;
    /* the NAL edges and three-group chunks: byte by byte */
    auto slow_chunk = [&](uint32_t c, uint32_t K) {
        uint8_t *q = A + ((cfirst + c) << 4);
        for (int b = 0; b < 16; ++b) {
            const uint64_t qa = ((cfirst + c) << 4) + (uint64_t)b;
            if (qa < o0 || qa >= o1) continue;
            const int32_t uu = (int32_t)(qa - o0) - 5;
            uint8_t v;
            if (uu < 0) {
                v = hdr[qa - o0];
            } else {
                while ((int32_t)(sp[K] + K) < uu) K++;
                if ((int32_t)(sp[K] + K) == uu) {
                    v = 3;
                } else {
                    const uint32_t ri = (uint32_t)uu - K - kb;
                    const uint32_t wd = rs_word(32u * (ri >> 2), ng, T, goff, gb, gw, fr);
                    v = (uint8_t)(wd >> (8u * (3u - (ri & 3u))));
                }
            }
            q[b] = v;
        }
    };
    /* chunk c's 128 RBSP bits from its loads (x: 160 bits of the group from
     * word lp >> 5, y: the next group's first 128 when the chunk runs past
     * rem bits), the EP bytes inside it, stored */
    auto fast_chunk = [&](uint32_t c, int32_t u0, uint32_t K, uint32_t lp, uint32_t rem, bool two, const uint32_t x[5],
                          const uint32_t yb[4]) {
        const uint32_t sh = lp & 31u;
        W4 R;
#pragma unroll
        for (int k = 0; k < 4; ++k) R.w[k] = sh ? __builtin_amdgcn_alignbit(x[k], x[k + 1], 32u - sh) : x[k];
        if (two) {                                           /* rem bits of this group, then the next */
            const W4 B = shr128(W4{{yb[0], yb[1], yb[2], yb[3]}}, rem);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t kb = 32u * (uint32_t)k;      /* bits of word k kept from this group */
                const uint32_t keep = rem <= kb ? 0u : (rem >= kb + 32u ? 32u : rem - kb);
                const uint32_t m = keep == 0u ? 0u : (keep == 32u ? 0xffffffffu : ~(0xffffffffu >> keep));
                R.w[k] = (R.w[k] & m) | B.w[k];
            }
        }
        /* the EP bytes inside the chunk: byte e becomes 03, the bytes from
         * e on move one byte later */
        for (uint32_t m = K;; ++m) {
            const int32_t e = (int32_t)(sp[m] + m) - u0;
            if (e >= 16) break;
            const W4 S = shr128(R, 8u);
            const uint32_t eb = 8u * (uint32_t)e;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t kb = 32u * (uint32_t)k;
                const uint32_t keep = eb <= kb ? 0u : (eb >= kb + 32u ? 32u : eb - kb);
                const uint32_t mk = keep == 0u ? 0u : (keep == 32u ? 0xffffffffu : ~(0xffffffffu >> keep));
                /* the 03 byte: bits [eb, eb + 8) */
                const uint32_t three = (eb >= kb && eb < kb + 32u) ? (3u << (24u - (eb - kb))) : 0u;
                const uint32_t mk2 = (eb >= kb && eb < kb + 32u) ? (0xff000000u >> (eb - kb)) : 0u;
                R.w[k] = (R.w[k] & mk) | (S.w[k] & ~mk & ~mk2) | three;
            }
        }
        *reinterpret_cast<uint4 *>(A + ((cfirst + c) << 4)) =
            make_uint4(__builtin_bswap32(R.w[0]), __builtin_bswap32(R.w[1]), __builtin_bswap32(R.w[2]),
                       __builtin_bswap32(R.w[3]));
    };
    /* two chunk sets in turn (no register copies between them): chunk c +
     * DT's search and loads go out before chunk c is assembled and stored.
     * Every chunk loads (the edge / past-the-end ones at word 0, unused), so
     * the number of loads in flight is fixed and the waits count them */
    struct GSet {
        uint32_t c, K, lp, rem;
        int32_t u0;
        bool fast, two, yv;                                  /* yv: y holds the next group's words */
        uint32_t x[5], y[4];
    };
    uint32_t wend = cend;                                    /* the window's chunk end */
    auto prep = [&](uint32_t c, GSet &S) {
        const int32_t u0 = 16 * (int32_t)c - d0, du = u0 - ub;
        uint32_t K = raw[du > 0 ? min(du >> cs, nblk - 1) : 0];
        uint32_t wo = 0u, yo = 0u;
        S.c = c;
        S.u0 = u0;
        S.fast = false;
        S.two = false;
        S.yv = false;
        S.lp = S.rem = 0u;
        if (c < wend && u0 >= 0 && u0 + 16 <= nebsp) {
            while ((int32_t)(sp[K] + K) < u0) K++;           /* sentinel stops it */
            const uint32_t i0 = (uint32_t)u0 - K - kb, P = 8u * i0;
            while (gg + 1 < ng && goff[gg + 1] <= P) ++gg;
            const uint32_t lp = P - goff[gg], rem = gb[gg] - lp;
            const bool two = rem < 128u;
            if (!two || gg + 1 >= ng || gb[gg + 1] >= 128u - rem) {
                S.fast = true;
                S.two = two;
                S.lp = lp;
                S.rem = rem;
                S.yv = two && gg + 1 < ng;
                wo = 4u * (gw[gg] + (lp >> 5));
                yo = S.yv ? 4u * gw[gg + 1] : wo;
            }
        }
        S.K = K;
        const auto xa = __builtin_amdgcn_raw_buffer_load_b128(rr, wo, 0, 0);
        const uint32_t x4 = __builtin_amdgcn_raw_buffer_load_b32(rr, wo + 16u, 0, 0);
        const auto y = __builtin_amdgcn_raw_buffer_load_b128(rr, yo, 0, 0);
        S.x[0] = (uint32_t)xa[0]; S.x[1] = (uint32_t)xa[1]; S.x[2] = (uint32_t)xa[2]; S.x[3] = (uint32_t)xa[3];
        S.x[4] = x4;
        S.y[0] = (uint32_t)y[0]; S.y[1] = (uint32_t)y[1]; S.y[2] = (uint32_t)y[2]; S.y[3] = (uint32_t)y[3];
    };
    auto finish = [&](GSet &S) {
        if (S.fast) {
            const uint32_t yb[4] = {S.yv ? S.y[0] : 0u, S.yv ? S.y[1] : 0u, S.yv ? S.y[2] : 0u, S.yv ? S.y[3] : 0u};
            fast_chunk(S.c, S.u0, S.K, S.lp, S.rem, S.two, S.x, yb);
        } else {
            slow_chunk(S.c, S.K);
        }
    };
    for (uint32_t cb = cbeg; cb < cend; cb = wend) {
        uint32_t m = n;
        if (whole) {
            kb = 0;
            wend = cend;
        } else {
            /* the window from chunk cb: its first EP byte kb (a binary search
             * in the sorted list), as many as the LDS holds, ending at the
             * chunk of the first one that does not fit (a chunk holds at most
             * 16 EP bytes, so a window is never empty) */
            __syncthreads();                                 /* the last window's sp / raw are done */
            if (t == 0) {
                const int32_t ulo = 16 * (int32_t)cb - d0;
                uint32_t lo = 0, hi = n;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if ((int32_t)(el[mid] + mid) < ulo) lo = mid + 1;
                    else hi = mid;
                }
                const uint32_t mm = min(n - lo, wcap);
                uint32_t ce = cend;
                if (lo + mm < n) ce = min(cend, max(cb + 1u, (uint32_t)((int32_t)(el[lo + mm] + lo + mm) + d0) >> 4));
                win[0] = lo;
                win[1] = mm;
                win[2] = ce;
            }
            __syncthreads();
            kb = win[0];
            m = win[1];
            wend = win[2];
        }
        for (uint32_t i = t; i < m; i += DT) (sorted ? sp : raw)[i] = el[kb + i] + kb;
        if (t == 0) sp[m] = 0x3fffffffu;                     /* sentinel: sp[m] + m never before a chunk */
        __syncthreads();
        for (uint32_t i = t; i < (sorted ? 0u : m); i += DT) {   /* ep_scan's lists (whole only): by rank */
            const uint32_t v = raw[i];
            uint32_t r = 0;
            for (uint32_t k = 0; k < m; ++k) r += raw[k] < v ? 1u : 0u;
            sp[r] = v;
        }
        __syncthreads();
        T = goff[ng];
        /* coarse index over the window's EBSP bytes from ub */
        ub = whole ? 0 : max(0, 16 * (int32_t)cb - d0);
        const uint32_t span = whole ? d.size : (uint32_t)(16 * (int32_t)wend - d0 - ub + 16);
        int lg = 0;
        while ((1u << lg) <= m) lg++;
        cs = 8;
        while ((span >> cs) >= (uint32_t)EPLIST_MAX) cs++;
        nblk = (int)(span >> cs) + 1;
        for (int bi = t; bi < nblk; bi += DT) {
            const uint32_t e0 = (uint32_t)ub + ((uint32_t)bi << cs);
            uint32_t K = 0;
            for (int b = lg - 1; b >= 0; --b) {
                const uint32_t k2 = K + (1u << b);
                K = k2 <= m && sp[k2 - 1] + (k2 - 1) < e0 ? k2 : K;
            }
            raw[bi] = K;
        }
        __syncthreads();
        if (stp && cb == cbeg) stp[1] = __builtin_amdgcn_s_memrealtime();
        GSet sa, sb;
        uint32_t c = cb + (uint32_t)t;
        if (c < wend) prep(c, sa);
        while (c < wend) {
            prep(c + DT, sb);
            finish(sa);
            c += DT;
            if (c >= wend) break;
            prep(c + DT, sa);
            finish(sb);
            c += DT;
        }
    }
    if (stamps) {                                            /* uniform */
        __syncthreads();
        if (stp) stp[2] = __builtin_amdgcn_s_memrealtime();
    }
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
int dyn_launch_code(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                    int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                    const DynGeom *g, const uint8_t *src, const uint8_t *refs, const DynScratch *x,
                    uint32_t epoch, int mbw, uint64_t *stamps, const DynFork *fk, hipEvent_t ev0, hipEvent_t ev1)
{
    if (nframes <= 0 || S <= 0) return 0;
    {                                   /* the tzrb table, once per device (and process) */
        static std::mutex mu;
        static uint64_t ready = 0;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev >= 64) return -1;
        std::lock_guard<std::mutex> lk(mu);
        if (!(ready >> dev & 1u)) {
            hipLaunchKernelGGL(k_tzrb_init, dim3((TZRB_N + 255) / 256), dim3(256), 0, hs);
            if (hipGetLastError() != hipSuccess || hipStreamSynchronize(hs) != hipSuccess) return -1;
            ready |= 1ull << dev;
        }
    }
    hipLaunchKernelGGL(k_dyn_rows, dim3(nframes, S), dim3(256), 0, hs, st, nal, ld_nal, pend, dfr, ld_fr,
                       *g, x->rows, x->ctr, x->heads);
    if (hipGetLastError() != hipSuccess) return -1;
    hipStream_t hg = hs;                /* the general path's stream */
    if (fk) {
        if (hipEventRecord(fk->e0, hs) != hipSuccess || hipStreamWaitEvent(fk->side, fk->e0, 0) != hipSuccess)
            return -1;
        hg = fk->side;
    }
    const int nchunk = (24 * g->w * g->h + CODE_T - 1) / CODE_T;
    hipLaunchKernelGGL(k_dyn_code_general, dim3(nchunk, CODE_GEN_Y), dim3(CODE_T), 0, hg, st, dfr, ld_fr,
                       pend, nal, ld_nal, *g, x->rows, src, refs, x->meta, x->body_lo, x->body_hi, x->body_w,
                       x->ctr);
    if (hipGetLastError() != hipSuccess) return -1;
    if (row_lds_bytes(g->w) > 65536) {
        /* wide rects (a whole 1280- or 4096-px row): dynamic LDS past the
         * 64 KB default, up to the CU's 160 KB (set_dyn_rect's bound) */
        const int rl = (int)row_lds_bytes(g->w);
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(&k_dyn_row<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, rl) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void *>(&k_dyn_row<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, rl) != hipSuccess)
            return -1;
    }
    if (ev0 && hipEventRecord(ev0, hs) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_dyn_row<false>, dim3(g->h, nframes, S), dim3(row_threads(g->w)),
                       row_lds_bytes(g->w), hs, st, nal, ld_nal, pend, dfr, ld_fr, *g, x->rows, src, refs,
                       x->meta, x->body_lo, x->body_hi, x->body_w, x->tcx, epoch, x->rowstage, x->gbits, x->spill,
                       x->ctr, x->heads, stamps);
    if (hipGetLastError() != hipSuccess) return -1;
    if (ev1 && hipEventRecord(ev1, hs) != hipSuccess) return -1;
    /* the general path: one row workgroup per record slot that may be taken */
    hipLaunchKernelGGL(k_dyn_row<true>, dim3(g->h, std::min<uint32_t>(g->gen_cap, (uint32_t)(nframes * S)), 1),
                       dim3(row_threads(g->w)),
                       row_lds_bytes(g->w), hg, st, nal, ld_nal, pend, dfr, ld_fr, *g, x->rows, src, refs,
                       x->meta, x->body_lo, x->body_hi, x->body_w, x->tcx, epoch, x->rowstage, x->gbits, x->spill,
                       x->ctr, x->heads, stamps);
    if (hipGetLastError() != hipSuccess) return -1;
    if (fk) {                           /* the static row groups beside the block coder too */
        if (dyn_launch_static(hg, nframes, S, st, nal, ld_nal, pend, dfr, ld_fr, g, x) ||
            hipEventRecord(fk->e1, hg) != hipSuccess)
            return -1;
    }
    return 0;
}

int dyn_launch_static(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal, int ld_nal,
                      const PlanPending *pend, DynFrame *dfr, int ld_fr, const DynGeom *g, const DynScratch *x)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_dyn_static, dim3(g->ngroups - g->h, nframes, S), dim3(GW), 0, hs, st, nal, ld_nal,
                       pend, dfr, ld_fr, *g, x->rowstage, x->gbits);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int dyn_launch_pack(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                    int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                    const DynGeom *g, const DynScratch *x, uint8_t *eps, uint64_t *stamps, const DynFork *fk)
{
    if (nframes <= 0 || S <= 0) return 0;
    if (fk) {                           /* k_dyn_static and the general path ran beside k_dyn_row */
        if (hipStreamWaitEvent(hs, fk->e1, 0) != hipSuccess) return -1;
    } else if (dyn_launch_static(hs, nframes, S, st, nal, ld_nal, pend, dfr, ld_fr, g, x)) {
        return -1;
    }
    if (g->ep_cap >= (uint32_t)EPF_BIG_LIST)
        hipLaunchKernelGGL((k_dyn_epfix<EPF_T, EPF_BIG_LIST>), dim3(nframes, S), dim3(EPF_T), gtab_bytes(g->ngroups, true),
                           hs, st, dfr, ld_fr, nframes, *g, x->rowstage, x->gbits, eps, stamps);
    else
        hipLaunchKernelGGL((k_dyn_epfix<EPF_T, EPF_LIST>), dim3(nframes, S), dim3(EPF_T), gtab_bytes(g->ngroups, true),
                           hs, st, dfr, ld_fr, nframes, *g, x->rowstage, x->gbits, eps, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int dyn_launch_emit(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal,
                    int ld_nal, const DynFrame *dfr, int ld_fr, const DynGeom *g,
                    const uint8_t *stage, const DynScratch *x, uint8_t *arena, uint64_t ld_arena,
                    uint64_t *stamps)
{
    if (nframes <= 0 || S <= 0) return 0;
    /* U chunks per thread and iteration, their loads in flight together:
     * one (fewer registers, more resident workgroups) for NALs up to ~64 KB
     * (config 3: 0.186 / 0.173 / 0.168 ms at U = 4 / 2 / 1), four for the
     * large rects (config 5: 0.45 ms at U = 4, 0.56 at U = 1) */
    const bool big = (int64_t)g->w * g->h > 1024;
    const uint32_t *rs = x ? x->rowstage : nullptr, *gbits = x ? x->gbits : nullptr;
    const dim3 grid(nframes, S, GATHER_Z);
    const size_t gl = x ? gtab_bytes(g->ngroups, false) : 0;     /* the group tables (RS) */
    if (x && !(g->debug & SCROLL_DEBUG_DYN_GATHER1))
        hipLaunchKernelGGL(k_dyn_gather, dim3(nframes, S, gather_z(*g, (int64_t)nframes * S)), dim3(DT), gl, hs, st, nal, ld_nal, dfr,
                           ld_fr, *g, stage, rs, gbits, arena, ld_arena, stamps);
    else if (x && big)
        hipLaunchKernelGGL((k_dyn_emit_gather<4, true>), grid, dim3(DT), gl, hs, st, nal, ld_nal, dfr, ld_fr, *g,
                           stage, rs, gbits, arena, ld_arena, stamps);
    else if (x)
        hipLaunchKernelGGL((k_dyn_emit_gather<1, true>), grid, dim3(DT), gl, hs, st, nal, ld_nal, dfr, ld_fr, *g,
                           stage, rs, gbits, arena, ld_arena, stamps);
    else if (big)
        hipLaunchKernelGGL((k_dyn_emit_gather<4, false>), grid, dim3(DT), 0, hs, st, nal, ld_nal, dfr, ld_fr,
                           *g, stage, rs, gbits, arena, ld_arena, stamps);
    else
        hipLaunchKernelGGL((k_dyn_emit_gather<1, false>), grid, dim3(DT), 0, hs, st, nal, ld_nal, dfr, ld_fr,
                           *g, stage, rs, gbits, arena, ld_arena, stamps);
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

void dyn_rowstage_geom(DynGeom *g, int mbw, int mbh)
{
    const int SR = DYN_STATIC_ROWS;
    const int above = g->y0 < SR ? g->y0 : SR, below0 = mbh - g->y0 - g->h;
    const int below = below0 < SR ? below0 : SR;
    const int maxrows = above > below ? above : below;
    auto words = [](uint64_t bits) { return (uint32_t)((((bits + 31) / 32) + 63) & ~(uint64_t)63); };
    /* + the group's EP-candidate record (EPC_ROW / EPC_STATIC words) at the slot end */
    g->rs_static_words = words((uint64_t)HDR_MAX + (uint64_t)maxrows * mbw * (HEAD_MAX + 1) + 64) + EPC_STATIC;
    /* a rect row's slot holds a typical row (SCROLL_DYN_ROW_KBITS per MB, ~2.5x
     * the synthetic source's mean); rows past it take a spill slot at the
     * provable bound (k_dyn_row) */
    g->rs_spill_words = words((uint64_t)mbw * (HEAD_MAX + 1) + (uint64_t)g->w * MB_BITS_MAX + 64) + EPC_ROW;
    g->rs_row_words = words((uint64_t)mbw * (HEAD_MAX + 1) + (uint64_t)g->w * SCROLL_DYN_ROW_KBITS + 64) + EPC_ROW;
    if (g->rs_row_words > g->rs_spill_words) g->rs_row_words = g->rs_spill_words;
    g->rs_frame_words = (uint64_t)(g->ngroups - g->h) * g->rs_static_words + (uint64_t)g->h * g->rs_row_words;
}

/* EP positions kept per frame by the rows' path (the list buffer's stride / 4) */
uint32_t dyn_ep_cap(int rw, int rh, int debug)
{
    return (debug & SCROLL_DEBUG_DYN_EPWIN) || epf_big_rect((int64_t)rw * rh) ? (uint32_t)EPF_BIG_LIST
                                                                            : (uint32_t)EPLIST_MAX;
}

size_t dyn_slot_bound(int mbw, int mbh, int rw, int rh)
{
    /* header + every MB head (+ cbp) + every dynamic MB at its provable
     * maximum + the stop word + 32 bytes of read-ahead */
    const size_t bits = (size_t)HDR_MAX + (size_t)mbw * mbh * (HEAD_MAX + 1) +
                        (size_t)rw * rh * MB_BITS_MAX + 64;
    return ((bits / 8 + 32 + DYN_OVF_BYTES) + 255) & ~(size_t)255;
}

/* profiling aid (tools/row_occupancy.py): resident k_dyn_row<false>
 * workgroups per CU for a w-MB rect row in an mbw-MB picture, with extra
 * bytes of dynamic LDS added (negative: removed) -- the HIP occupancy
 * calculator's answer for this very kernel (registers, static LDS) */
extern "C" int scroll_debug_row_occupancy(int w, int mbw, int extra_lds)
{
    int n = -1;
    (void)mbw;                              /* (round 4's LDS grew with the picture width) */
    const size_t lds = (size_t)((long)row_lds_bytes(w) + extra_lds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void *>(&k_dyn_row<false>),
                                                     row_threads(w), lds) != hipSuccess)
        return -1;
    return n;
}
