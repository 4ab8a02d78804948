/*
 * dyn_kernels.hip -- MI355X (gfx950) kernels of the dynamic-rect residual
 * coder (BASELINE configs 3-5).  A scroll NAL with the rect is no longer a
 * handful of periodic runs: every dynamic MB carries a CAVLC residual, and
 * 60 % of such NALs need emulation prevention.  So these NALs take their own
 * two kernels around the plan's sizing pass:
 *
 *   k_plan (state pass)   waypoint state machine, NalDesc per NAL
 *   k_dyn_stage           one workgroup per dynamic NAL: its whole RBSP into
 *                         a staging slot + its exact emulation-prevention count
 *   k_plan (size pass)    NAL sizes (dynamic: 5 + RBSP + EP), arena offsets
 *   k_emit                every other NAL (dynamic NALs are "external")
 *   k_dyn_emit            staged RBSP -> arena: start code, NAL header, EP
 *                         bytes, written in whole 128-byte lines
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

constexpr int WMB = DYN_WINDOW_MBS;     /* dynamic MBs per window: 24 x 10 = 240 block tasks */
static_assert(24 * WMB <= 256, "one block task per thread");
constexpr int WIN = DT;                 /* MBs per window (one MB per thread)    */
constexpr int HEAD_MAX = 160;           /* bits of one MB head (huge mvd: 2 x 63 + ref) */
constexpr int HDR_MAX = 1024;           /* slice header bits (8 waypoints + MMCO ~ 250) */
constexpr int BUF_WORDS = 1536;        /* 48 Kbit LDS bit buffer; larger windows take passes */
static_assert(BUF_WORDS * 32 > HDR_MAX + 64, "the slice header fits one buffer");
constexpr int OBUF = 6400;              /* k_dyn_emit: 127 carry + 5 + 4096 x 1.5 */

__device__ inline uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }

/* ---------------------------------------------------------------------- */
/* k_dyn_stage                                                             */
/* ---------------------------------------------------------------------- */
/* Block tasks of a window with nd dynamic MBs: luma first (lanes walk the
 * MBs' 4-pixel columns so a block row of the window is one contiguous
 * source read), then Cb, Cr. */
struct Task {
    int k, blk, bx, by, p;
    bool luma;
};

/* m4 = magic16(4 nd), m2 = magic16(2 nd): t < 240, divisors <= 40 */
__device__ inline Task task_of(int t, int nd, uint32_t m4, uint32_t m2)
{
    Task q;
    if (t < 16 * nd) {
        q.luma = true;
        q.p = 0;
        q.by = (int)div16((uint32_t)t, m4);
        const int c4 = t - q.by * 4 * nd;
        q.k = c4 >> 2;
        q.bx = c4 & 3;
        q.blk = 4 * q.by + q.bx;
    } else {
        const int u = t - 16 * nd;
        q.luma = false;
        q.p = (int)div16((uint32_t)u, m4);
        const int r = u - q.p * 4 * nd;
        q.by = (int)div16((uint32_t)r, m2);
        const int c2 = r - q.by * 2 * nd;
        q.k = c2 >> 1;
        q.bx = c2 & 1;
        q.blk = 16 + 4 * q.p + 2 * q.by + q.bx;
    }
    return q;
}

struct StageLds {
    uint32_t buf[BUF_WORDS];      /* NAL bits from word `bw` of the slot on       */
    uint32_t lv8[WMB * 24][4];    /* block levels, int8 packed, scan order        */
    uint8_t order[WMB * 24];      /* encode order: light blocks first, then heavy */
    uint32_t whc[NW];             /* heavy blocks per wave                        */
    int32_t dcraw[WMB][2][4];     /* chroma DC coefficients before the Hadamard   */
    int16_t dclv[WMB][2][4];
    alignas(16) uint8_t tc[WMB][32];   /* TotalCoeff per 4x4 block (24 used)      */
    uint8_t cbp[WMB];
    alignas(16) uint16_t blen[WMB][32];  /* pieces: luma raster 0..15, DC 16+p, AC 18+4p+kk */
    alignas(16) uint16_t boff[WMB][32];
    uint32_t exw[WIN];            /* MB lengths: in-wave exclusive prefix         */
    uint32_t wsum[NW];
    uint8_t ctx[DYN_CTX_MB][8];   /* bottom-row TotalCoeff of rect MBs (row ring) */
    uint16_t rmap[32 * DYN_MAX_H]; /* prediction rows of the rect, per frame row: picture << 15 | row;
                                      luma 16 h, chroma top 8 h, chroma bottom 8 h; 0xffff: half-pel */
    uint8_t lcarry[8];            /* right-column TotalCoeff of the last dyn MB   */
    int32_t wo[8], wl[8], wv[8];
    int32_t lnz_r, lnz_w;         /* last non-zero staged byte: before / of a flush */
    uint32_t ep_n;                /* EP positions recorded                         */
    int32_t general;              /* a half-pel waypoint step was met            */
    uint64_t hhi[12], hlo[12];    /* MB head codewords [row type 0..3][first / middle / last] */
    uint32_t hlen[12];
    int32_t head_over;            /* a head longer than 128 bits: compute per MB */
    PTabs ptabs;
};

constexpr int HEAVY_TC = 3;       /* blocks with more non-zero levels encode in the heavy group */

constexpr uint32_t DF_OVER = 1u, DF_GENERAL = 2u;   /* DynFrame.err bits */

/* windowed LDS OR: word i of the window's bit stream -> buf[i - lo] when in
 * [lo, lo + n) (one pass of a window larger than the buffer) */
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


/* GENERAL = false: every waypoint step is full-pel (always so for waypoints
 * the composer creates); a NAL that meets a half-pel step is flagged and
 * redone by the GENERAL instantiation, which evaluates the bilinear tree.
 *
 * Window pipeline (barriers: 4 per window):
 *   A(i)  block tasks: residual -> transform -> quant -> CAVLC rest (regs);
 *         flush of window i-1's whole words (staging + EP count)
 *   B(i)  nC + coeff_token, chroma DC; buffer rewind after the flush
 *   C(i)  MB heads (regs), cbp, piece offsets, in-wave scan of MB lengths
 *   D(i)  every piece ORed into the LDS bit buffer at its offset          */
#ifndef SCROLL_DYN_ABLATE
#define SCROLL_DYN_ABLATE 0         /* 1: honour the SCROLL_DEBUG_DYN_* ablation flags (profiling builds) */
#endif
#define ABL(flag) (SCROLL_DYN_ABLATE && (g.debug & (flag)))
#ifndef SCROLL_DYN_WAVES
#define SCROLL_DYN_WAVES 8          /* waves per SIMD the register budget targets */
#endif
template <bool GENERAL>
__global__ __launch_bounds__(DT, SCROLL_DYN_WAVES) void k_dyn_stage(DevStream *__restrict__ st,
                                                  const NalDesc *__restrict__ nal, int ld_nal,
                                                  const PlanPending *__restrict__ pend,
                                                  DynFrame *__restrict__ dfr, int ld_fr,
                                                  DynGeom g, const uint8_t *__restrict__ src,
                                                  const uint8_t *__restrict__ refs,
                                                  uint8_t *__restrict__ stage,
                                                  uint64_t *__restrict__ stamps)
{
    __shared__ StageLds L;
    /* debug: cycles per phase (A B C D, multi-pass), windows, total -> stamps */
    uint64_t ph[5] = {0, 0, 0, 0, 0}, t_start = 0, t_last = 0, nwin = 0;
    auto mark = [&](int k) {
        if (stamps) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            ph[k] += now - t_last;
            t_last = now;
        }
    };
    if (stamps) t_start = t_last = __builtin_amdgcn_s_memtime();
    const int s = blockIdx.y, f = dyn_frame_of(blockIdx.x, s), t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    DevStream *S = st + s;
    DynFrame *DF = dfr + (size_t)s * ld_fr + f;
    const int j = DF->nal;
    if (j < 0) return;
    if (GENERAL && !(DF->err & DF_GENERAL)) return;

    const Rect R{g.x0, g.y0, g.w, g.h};
    if (t == 0) {
        L.general = 0;
        L.lnz_r = -1;
        L.lnz_w = -1;
        L.head_over = 0;
        L.ep_n = 0;
    }
    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    for (int i = t; i < BUF_WORDS; i += DT) L.buf[i] = 0u;
    build_ptabs(*reinterpret_cast<const Tabs *>(&g_tabs), L.ptabs, t, DT);
    const NalDesc d = nal[(size_t)s * ld_nal + j];
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
    c.wp_off = L.wo;
    c.wp_lt = L.wl;
    c.wp_valid = L.wv;
    __syncthreads();

    /* slice header (h264_writer.c:549-553): thread 0 writes, all count */
    uint32_t F;
    {
        CountSink hc{0};
        emit_slice_header(hc, c);
        F = hc.n;
        if (t == 0) {
            LSink hs{{L.buf}, 0, 0, 0};
            hs.start(0);
            emit_slice_header(hs, c);
            hs.finish();
        }
    }

    const int w = c.w, h = c.h, mbw = w / 16, mbh = h / 16;
    const Regions rg = regions(c);
    const int a_end = (h - c.off) / 16;
    const int nrefs = 2 + c.nwp;
    const WpTab T{L.wo, L.wv, h};
    const uint8_t *rb = refs + (size_t)s * g.ref_ld;
    const size_t ysz = (size_t)w * h, csz = ysz / 4, pic = ysz + 2 * csz;
    const uint8_t *fs = src + (size_t)s * g.src_ld + (size_t)f * g.src_fr;
    const int lstride = 16 * R.w, cstride = 8 * R.w;
    const uint8_t *fcb = fs + (size_t)256 * R.w * R.h, *fcr = fcb + (size_t)64 * R.w * R.h;
    const int rmask = g.ring - 1;       /* TotalCoeff row ring: a power of two */
    /* the waypoint chain of every prediction row, once per NAL: frame row
     * -> (picture A / B, row) for luma, and for the two chroma rows of the
     * 1/8-pel bilinear (src/h264_writer.c:689-729 via dyn_device.h) */
    for (int i = t; i < 32 * R.h; i += DT) {
        uint16_t e;
        if (i < 16 * R.h) {
            const int Y = 16 * R.y0 + i, row = Y >> 4;
            const bool cA = row < a_end;
            int yo;
            const int b = luma_row(T, cA ? rg.ra : rg.rb, Y + (cA ? rg.mva : rg.mvb), yo);
            e = (uint16_t)(b << 15 | yo);
        } else {
            const int i2 = i - 16 * R.h, bot = i2 >= 8 * R.h;
            const int Y = 8 * R.y0 + (bot ? i2 - 8 * R.h : i2), row = Y >> 3;
            const bool cA = row < a_end;
            const int o = (4 * (cA ? rg.mva : rg.mvb)) >> 3;
            int yo;
            const int b = chroma_row(T, cA ? rg.ra : rg.rb, Y + o + bot, yo);
            e = b < 0 ? (uint16_t)0xffff : (uint16_t)(b << 15 | yo);
        }
        L.rmap[i] = e;
    }
    /* MB head codewords (mb_skip_run .. mvd, h264_writer.c:434-453): they
     * depend only on the row type -- row 0, steady A, A->B boundary, steady
     * B -- and on first / middle / last position */
    if (t < 12) {
        const int ty = t / 3, pos = t - 3 * ty;
        const int x = pos == 0 ? 0 : (pos == 1 ? min(1, mbw - 1) : mbw - 1);
        const bool cur = ty == 0 ? 0 < a_end : ty == 1;
        const bool abv = ty == 1 || ty == 2;
        const int ref = cur ? rg.ra : rg.rb, mv4 = 4 * (cur ? rg.mva : rg.mvb);
        const int aref = abv ? rg.ra : rg.rb, amv4 = 4 * (abv ? rg.mva : rg.mvb);
        int px, py;
        predict(x, ty == 0 ? 0 : 1, mbw, ref, mv4, aref, amv4, px, py);
        CapSink hc{0, 0, 0};
        put_mb_head(hc, ref, 0 - px, mv4 - py, nrefs);
        L.hhi[t] = hc.hi;
        L.hlo[t] = hc.lo;
        L.hlen[t] = hc.n;
        if (hc.over()) L.head_over = 1;
    }
    __syncthreads();
    const uint32_t m_mbw = magic32((uint32_t)mbw), m_rw = magic32((uint32_t)R.w);
    uint8_t *slot = stage + ((size_t)s * ld_fr + f) * g.slot_bytes;
    uint32_t *out = reinterpret_cast<uint32_t *>(slot);
    const uint32_t cap_words = (uint32_t)((g.slot_bytes - DYN_OVF_BYTES) / 4) - 4u;
    /* RBSP positions of the EP bytes (unsorted), for k_dyn_emit's gather */
    uint32_t *eplist = reinterpret_cast<uint32_t *>(slot + g.slot_bytes - DYN_OVF_BYTES);
    const Tabs &TB = g_tabs;            /* chroma DC and the rare > 128-bit blocks */
    const PTabs &PT = L.ptabs;

    uint32_t bw = 0;             /* staging word of buf[0]                        */
    uint32_t my_ep = 0;
    bool over = false;
    uint32_t pend_T = 0;         /* bits in buf awaiting the deferred flush (0: none) */

    /* whole words buf[0, n) -> staging words [gw0, gw0 + n), EP insertions
     * counted with the zero run looked up backwards in buf (L.lnz_r before
     * buf[0]); the last non-zero byte goes to L.lnz_w */
    auto flush_words = [&](uint32_t n, uint32_t gw0) {
        for (uint32_t jw = (uint32_t)t; jw < n; jw += DT) {
            const uint32_t wv = L.buf[jw];
            out[gw0 + jw] = __builtin_bswap32(wv);
            int prev = L.lnz_r;
            for (int jj = (int)jw - 1; jj >= 0; --jj) {
                const uint32_t pv = L.buf[jj];
                if (pv) {
                    prev = 4 * (int)(gw0 + jj) + last_nz_byte(pv);
                    break;
                }
            }
            const uint32_t gb = 4u * (gw0 + jw);
            my_ep += ep_word(wv, gb, 0xffffffffu, prev, eplist, &L.ep_n);
            if (wv) atomicMax(&L.lnz_w, (int)gb + last_nz_byte(wv));
        }
    };
    /* after a flush: carry the last non-zero byte forward */
    auto rewind_lnz = [&]() {
        if (t == 0) {
            L.lnz_r = max(L.lnz_r, L.lnz_w);
            L.lnz_w = -1;
        }
    };

    const int nmb = mbw * mbh, ndt = R.w * R.h;
    for (int m0 = 0; m0 < nmb;) {
        const int q0 = dyn_rank_m(R, mbw, m_mbw, m0);
        int m1 = min(m0 + WIN, nmb);
        if (q0 + WMB < ndt) m1 = min(m1, dyn_mb_m(R, mbw, m_rw, q0 + WMB));
        const int nd = dyn_rank_m(R, mbw, m_mbw, m1) - q0;
        const int nm = m1 - m0;
        const uint32_t m4 = nd ? magic16(4u * nd) : 0u, m2 = nd ? magic16(2u * nd) : 0u;
        /* rect coordinates (ry, cx) of dynamic MB k of the window */
        auto dcoord = [&](int k, int &ry, int &cx) {
            const int qq = q0 + k;
            ry = (int)div_m((uint32_t)qq, m_rw);
            cx = qq - ry * R.w;
        };
        nwin++;

        /* A: the previous window's whole words -> staging; then residual ->
         * transform -> quantised levels (int8 packed) and TotalCoeff to LDS */
        const uint32_t pnf = pend_T >> 5;
        uint32_t part = 0;
        if (pend_T) {
            flush_words(pnf, bw);
            part = L.buf[pnf];
        }
        CapSink bcap{0, 0, 0};
        bool heavy = false;
        if (t < 24 * nd) {
            const Task q = task_of(t, nd, m4, m2);
            int ry, cx;
            dcoord(q.k, ry, cx);
            const int row = R.y0 + ry, col = R.x0 + cx;
            const bool curA = row < a_end;
            const int ref = curA ? rg.ra : rg.rb, mvp = curA ? rg.mva : rg.mvb;
            int res[16], W[16];
            if (q.luma) {
                const uint8_t *sp = fs + (size_t)(16 * ry + 4 * q.by) * lstride + 16 * cx + 4 * q.bx;
                const int X = 16 * col + 4 * q.bx;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t e = L.rmap[16 * ry + 4 * q.by + i];
                    uint32_t sv = 0x80604020u + (uint32_t)(t + i), pv = 0x10203040u;
                    if (!ABL(SCROLL_DEBUG_DYN_NOLOAD)) {
                        sv = ld32(sp + (size_t)i * lstride);
                        pv = ld32(rb + (e >> 15) * (uint32_t)pic + (e & 0x7fffu) * (uint32_t)w + X);
                    }
#pragma unroll
                    for (int x = 0; x < 4; ++x)
                        res[4 * i + x] = (int)((sv >> (8 * x)) & 255u) - (int)((pv >> (8 * x)) & 255u);
                }
                fwd4x4(res, W);
                uint32_t pk[4] = {0, 0, 0, 0};
                int n = 0;
#pragma unroll
                for (int k2 = 0; k2 < 16; ++k2) {
                    const int v = quant(W[ZZ[k2]], ZZ[k2]);          /* |v| <= 78: int8 */
                    pk[k2 >> 2] |= ((uint32_t)v & 255u) << (8 * (k2 & 3));
                    n += v != 0;
                }
                *reinterpret_cast<uint4 *>(L.lv8[24 * q.k + q.blk]) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                heavy = n > HEAVY_TC;
                L.tc[q.k][q.blk] = (uint8_t)n;
                if (q.by == 3) L.ctx[(ry & rmask) * R.w + cx][q.bx] = (uint8_t)n;
            } else {
                const uint8_t *sp = (q.p ? fcr : fcb) + (size_t)(8 * ry + 4 * q.by) * cstride +
                                    8 * cx + 4 * q.bx;
                const int X = 8 * col + 4 * q.bx, Y = 8 * row + 4 * q.by;
                const int qq = 4 * mvp, o = qq >> 3, fr = qq & 7;
                const int cw = w / 2;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t sv = ABL(SCROLL_DEBUG_DYN_NOLOAD) ? 0x40506070u + (uint32_t)t
                                                                          : ld32(sp + (size_t)i * cstride);
                    const int ya = Y + i + o;
                    const uint32_t ea = L.rmap[16 * R.h + 8 * ry + 4 * q.by + i];
                    const uint32_t eb = fr ? L.rmap[24 * R.h + 8 * ry + 4 * q.by + i] : 0u;
                    const int ba = ea == 0xffffu ? -1 : (int)(ea >> 15), yoa = (int)(ea & 0x7fffu);
                    const int bb = eb == 0xffffu ? -1 : (int)(eb >> 15), yob = (int)(eb & 0x7fffu);
                    int pred[4];
                    if (!GENERAL && (ba < 0 || bb < 0)) {
                        L.general = 1;
                        pred[0] = pred[1] = pred[2] = pred[3] = 0;
                    } else if (ba >= 0 && bb >= 0) {
                        const uint8_t *cp = rb + ysz + (size_t)q.p * csz + X;
                        const bool nl = ABL(SCROLL_DEBUG_DYN_NOLOAD);
                        const uint32_t av =
                            nl ? 0x11223344u : ld32(cp + (uint32_t)ba * (uint32_t)pic + (uint32_t)yoa * (uint32_t)cw);
                        const uint32_t bv =
                            fr && !nl ? ld32(cp + (uint32_t)bb * (uint32_t)pic + (uint32_t)yob * (uint32_t)cw) : 0u;
#pragma unroll
                        for (int x = 0; x < 4; ++x) {
                            const int a = (int)((av >> (8 * x)) & 255u), b = (int)((bv >> (8 * x)) & 255u);
                            pred[x] = ((8 - fr) * a + fr * b + 4) >> 3;
                        }
                    } else {                       /* half-pel waypoint step: general path */
                        if constexpr (GENERAL) {
                            RefPics P;
                            P.w = w;
                            P.h = h;
                            for (int i2 = 0; i2 < 2; ++i2) {
                                P.pl[i2][0] = rb + i2 * pic;
                                P.pl[i2][1] = P.pl[i2][0] + ysz;
                                P.pl[i2][2] = P.pl[i2][1] + csz;
                            }
                            for (int x = 0; x < 4; ++x) {
                                const int a = chroma_px_any<9>(T, P, ref, 1 + q.p, X + x, ya);
                                const int b = fr ? chroma_px_any<9>(T, P, ref, 1 + q.p, X + x, ya + 1) : 0;
                                pred[x] = ((8 - fr) * a + fr * b + 4) >> 3;
                            }
                        }
                    }
#pragma unroll
                    for (int x = 0; x < 4; ++x) res[4 * i + x] = (int)((sv >> (8 * x)) & 255u) - pred[x];
                }
                fwd4x4(res, W);
                L.dcraw[q.k][q.p][2 * q.by + q.bx] = W[0];
                uint32_t pk[4] = {0, 0, 0, 0};
                int n = 0;
#pragma unroll
                for (int k2 = 1; k2 < 16; ++k2) {
                    const int v = quant(W[ZZ[k2]], ZZ[k2]);
                    pk[(k2 - 1) >> 2] |= ((uint32_t)v & 255u) << (8 * ((k2 - 1) & 3));
                    n += v != 0;
                }
                *reinterpret_cast<uint4 *>(L.lv8[24 * q.k + q.blk]) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                heavy = n > HEAVY_TC;
                L.tc[q.k][q.blk] = (uint8_t)n;
                if (q.by == 1) L.ctx[(ry & rmask) * R.w + cx][4 + 2 * q.p + q.bx] = (uint8_t)n;
            }
        }
        const uint64_t hb = __ballot(heavy);
        if (lane == 0) L.whc[wave] = (uint32_t)__popcll(hb);
        __syncthreads();
        mark(0);
        if (!GENERAL && L.general) {                /* uniform: read after the barrier */
            if (t == 0) DF->err = DF_GENERAL;
            return;
        }

        /* B: buffer rewind after the flush; nC, coded flags, coeff_token;
         * chroma DC Hadamard + quant + CAVLC */
        if (pend_T) {
            for (uint32_t jw = (uint32_t)t; jw <= pnf; jw += DT) L.buf[jw] = jw == 0 ? part : 0u;
            rewind_lnz();
            F = pend_T & 31u;
            bw += pnf;
            pend_T = 0;
        }
        /* encode order: light blocks (<= HEAVY_TC non-zero levels) first, so
         * the encode loop of a wave runs few iterations; heavy ones share the
         * last wave(s) */
        const int ntask = 24 * nd;
        if (t < ntask) {
            uint32_t hpre = 0, htot = 0;
#pragma unroll
            for (int w2 = 0; w2 < NW; ++w2) {
                hpre += w2 < wave ? L.whc[w2] : 0u;
                htot += L.whc[w2];
            }
            const uint32_t hr = hpre + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                           (uint32_t)(hb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hb, 0u));
            const uint32_t lr = (uint32_t)t - hr;
            L.order[heavy ? (uint32_t)ntask - htot + hr : lr] = (uint8_t)t;
        }
        if (t < 2 * nd) {
            const int k = t >> 1, p = t & 1;
            const int *dc = L.dcraw[k][p];
            const int f00 = dc[0] + dc[1] + dc[2] + dc[3], f01 = dc[0] - dc[1] + dc[2] - dc[3];
            const int f10 = dc[0] + dc[1] - dc[2] - dc[3], f11 = dc[0] - dc[1] - dc[2] + dc[3];
            const int dq[4] = {quant_dc(f00), quant_dc(f01), quant_dc(f10), quant_dc(f11)};
            int16_t *o = L.dclv[k][p];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = (int16_t)dq[i];
            CountSink dn{0};
            cavlc_dc4(dn, PT, dq);
            L.blen[k][16 + p] = (uint16_t)dn.n;
        }
        __syncthreads();

        /* B2: CAVLC of the block order[t] (token .. runs) into registers */
        /* the encoded block, packed to keep registers free across barriers:
         * bit 31 valid, 30 ok, 24..29 nC + 1, 16..23 MB of the window, 8..15
         * piece, 0..7 dynamic MB k */
        uint32_t enc = 0;
        if (t < ntask) {
            int enc_nc = 0, e_k = 0, e_pc = 0, e_u = 0, etask;
            bool enc_ok = true;
            etask = L.order[t];
            const Task q = task_of(etask, nd, m4, m2);
            int ry, cx;
            dcoord(q.k, ry, cx);
            const int row = R.y0 + ry, col = R.x0 + cx;
            e_k = q.k;
            e_pc = q.luma ? q.blk : 18 + (q.blk - 16);
            e_u = row * mbw + col - m0;                /* MB of the window */
            const bool ldyn = col > R.x0, lav = col > 0, tdyn = row > R.y0, tav = row > 0;
            const uint8_t *tc = L.tc[q.k];
            int nA, nB;
            bool coded;
            if (q.luma) {
                const int r = q.blk;
                nA = q.bx > 0 ? tc[r - 1]
                              : (ldyn ? (q.k > 0 ? L.tc[q.k - 1][r + 3] : L.lcarry[q.by]) : (lav ? 0 : -1));
                nB = q.by > 0 ? tc[r - 4]
                              : (tdyn ? L.ctx[((ry - 1) & rmask) * R.w + cx][q.bx] : (tav ? 0 : -1));
                const int b8 = 4 * (q.by & 2) + (q.bx & 2);
                coded = (tc[b8] | tc[b8 + 1] | tc[b8 + 4] | tc[b8 + 5]) != 0;
            } else {
                const int i = q.blk;
                nA = q.bx > 0 ? tc[i - 1]
                              : (ldyn ? (q.k > 0 ? L.tc[q.k - 1][i + 1] : L.lcarry[4 + 2 * q.p + q.by])
                                      : (lav ? 0 : -1));
                nB = q.by > 0 ? tc[i - 2]
                              : (tdyn ? L.ctx[((ry - 1) & rmask) * R.w + cx][4 + 2 * q.p + q.bx]
                                      : (tav ? 0 : -1));
                uint32_t any = 0;
#pragma unroll
                for (int k2 = 16; k2 < 24; ++k2) any |= tc[k2];
                coded = any != 0;
            }
            enc_nc = nc_of(nA, nB);
            if (coded && ABL(SCROLL_DEBUG_DYN_NOCAVLC)) {
                bcap.put(1, 1);
            } else if (coded) {
                const uint4 v4 = *reinterpret_cast<const uint4 *>(L.lv8[24 * q.k + q.blk]);
                const uint32_t pk[4] = {v4.x, v4.y, v4.z, v4.w};
                if (q.luma) cavlc_nz<16>(bcap, PT, pk, enc_nc, enc_ok);
                else cavlc_nz<15>(bcap, PT, pk, enc_nc, enc_ok);
            }
            L.blen[q.k][q.luma ? q.blk : 18 + (q.blk - 16)] = (uint16_t)bcap.n;
            enc = 0x80000000u | (enc_ok ? 0x40000000u : 0u) | (uint32_t)(enc_nc + 1) << 24 |
                  (uint32_t)e_u << 16 | (uint32_t)e_pc << 8 | (uint32_t)e_k;
        }
        __syncthreads();
        mark(1);

        /* C: MB heads, cbp, piece offsets; in-wave scan of the MB lengths */
        uint32_t mlen = 0;
        int kd = -1, hsel = 0, code = 0, cbp = 0;
        const bool head_over = L.head_over;        /* uniform */
        if (t < nm && ABL(SCROLL_DEBUG_DYN_NOHEAD)) {
            mlen = 1;
        } else if (t < nm) {
            const int m = m0 + t, row = (int)div_m((uint32_t)m, m_mbw), col = m - row * mbw;
            const bool curA = row < a_end, abvA = (row - 1) < a_end;
            hsel = 3 * (row == 0 ? 0 : (curA ? 1 : (abvA ? 2 : 3))) +
                   (col == 0 ? 0 : (col == mbw - 1 ? 2 : 1));
            CountSink mc{head_over ? 0u : L.hlen[hsel]};
            if (head_over) {                       /* > 128-bit heads: per MB */
                const int ref = curA ? rg.ra : rg.rb, mv4 = 4 * (curA ? rg.mva : rg.mvb);
                const int aref = abvA ? rg.ra : rg.rb, amv4 = 4 * (abvA ? rg.mva : rg.mvb);
                int px, py;
                predict(col, row, mbw, ref, mv4, aref, amv4, px, py);
                put_mb_head(mc, ref, 0 - px, mv4 - py, nrefs);
            }
            const bool isdyn = col >= R.x0 && col < R.x0 + R.w && row >= R.y0 && row < R.y0 + R.h;
            if (!isdyn) {
                mlen = mc.n + 1u;                  /* + coded_block_pattern ue(0) */
            } else {
                kd = (row - R.y0) * R.w + (col - R.x0) - q0;
                /* bulk LDS reads (no dependent chains): TotalCoeff, lengths */
                const uint4 t0 = *reinterpret_cast<const uint4 *>(L.tc[kd]);
                const uint2 t1 = *reinterpret_cast<const uint2 *>(L.tc[kd] + 16);
                const uint32_t tw[6] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y};
                int cbp_l = 0;
#pragma unroll
                for (int b8 = 0; b8 < 4; ++b8) {             /* rows 2(b8>>1), +1; cols 2(b8&1), +1 */
                    const int r0 = 2 * (b8 >> 1), sh = 16 * (b8 & 1);
                    if (((tw[r0] >> sh) & 0xffffu) | ((tw[r0 + 1] >> sh) & 0xffffu)) cbp_l |= 1 << b8;
                }
                const uint32_t ac = tw[4] | tw[5];
                const int16_t *dl = &L.dclv[kd][0][0];
                int anydc = 0;
#pragma unroll
                for (int k2 = 0; k2 < 8; ++k2) anydc |= dl[k2];
                const int cbp_c = ac ? 2 : (anydc ? 1 : 0);
                cbp = cbp_l | (cbp_c << 4);
                code = TB.cbp_code[cbp];
                L.cbp[kd] = (uint8_t)cbp;
                put_ue(mc, (uint32_t)code);
                if (cbp) put_se(mc, 0);            /* mb_qp_delta */
                uint32_t bl[32], bo[32];
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const uint4 x = reinterpret_cast<const uint4 *>(L.blen[kd])[v];
                    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        bl[8 * v + 2 * h] = xw[h] & 0xffffu;
                        bl[8 * v + 2 * h + 1] = xw[h] >> 16;
                    }
                }
                uint32_t off = mc.n;
#pragma unroll
                for (int blk = 0; blk < 16; ++blk) {       /* luma4x4BlkIdx order */
                    const int r = blk_raster(blk);
                    bo[r] = off;
                    off += bl[r];
                }
#pragma unroll
                for (int k2 = 16; k2 < 26; ++k2) {         /* Cb DC, Cr DC, Cb AC 0-3, Cr AC 0-3 */
                    bo[k2] = off;
                    off += (k2 < 18 ? cbp_c >= 1 : cbp_c == 2) ? bl[k2] : 0u;
                }
#pragma unroll
                for (int k2 = 26; k2 < 32; ++k2) bo[k2] = 0;
#pragma unroll
                for (int v = 0; v < 4; ++v)
                    reinterpret_cast<uint4 *>(L.boff[kd])[v] =
                        make_uint4(bo[8 * v] | bo[8 * v + 1] << 16, bo[8 * v + 2] | bo[8 * v + 3] << 16,
                                   bo[8 * v + 4] | bo[8 * v + 5] << 16, bo[8 * v + 6] | bo[8 * v + 7] << 16);
                mlen = off;
            }
        }
        {
            const uint32_t incl = wave_incl_sum(mlen, lane);
            L.exw[t] = incl - mlen;
            if (lane == 63) L.wsum[wave] = incl;
        }
        __syncthreads();
        mark(2);
        uint32_t wtot = 0, wpre[NW];
#pragma unroll
        for (int w2 = 0; w2 < NW; ++w2) {
            wpre[w2] = wtot;
            wtot += L.wsum[w2];
        }
        /* offset of MB u of the window */
        auto mbo = [&](int u) -> uint32_t {
            uint32_t pre = 0;
#pragma unroll
            for (int w2 = 0; w2 < NW; ++w2)
                if (w2 == (u >> 6)) pre = wpre[w2];
            return pre + L.exw[u];
        };
        const uint32_t Tb = F + wtot;
        if (bw + (Tb >> 5) + 2u > cap_words) {      /* uniform */
            over = true;
            break;
        }

        /* D: every piece ORed into the buffer; a window larger than the
         * buffer is written and flushed in passes of BUF_WORDS - 1 words */
        const uint32_t nw = (Tb + 31) >> 5;
        const bool single = nw <= (uint32_t)BUF_WORDS;
        const uint32_t PW = single ? (uint32_t)BUF_WORDS : (uint32_t)BUF_WORDS - 1u;
        const uint32_t my_mbo = t < nm ? mbo(t) : 0u;
        for (uint32_t p0 = 0; p0 < nw; p0 += PW) {
            const LdsOrWin win{L.buf, p0, PW};
            if (t < nm && !ABL(SCROLL_DEBUG_DYN_NOWRITE | SCROLL_DEBUG_DYN_NOHEAD)) {   /* MB head */
                WSink sk{win, 0, 0, 0};
                sk.start(F + my_mbo);
                if (!head_over) {
                    sk.put_cap(CapSink{L.hhi[hsel], L.hlo[hsel], L.hlen[hsel]});
                } else {
                    const int m = m0 + t, row = (int)div_m((uint32_t)m, m_mbw), col = m - row * mbw;
                    const bool curA = row < a_end, abvA = (row - 1) < a_end;
                    const int ref = curA ? rg.ra : rg.rb, mv4 = 4 * (curA ? rg.mva : rg.mvb);
                    const int aref = abvA ? rg.ra : rg.rb, amv4 = 4 * (abvA ? rg.mva : rg.mvb);
                    int px, py;
                    predict(col, row, mbw, ref, mv4, aref, amv4, px, py);
                    put_mb_head(sk, ref, 0 - px, mv4 - py, nrefs);
                }
                if (kd < 0) {
                    sk.put(1, 1);                  /* coded_block_pattern ue(0) */
                } else {
                    put_ue(sk, (uint32_t)code);
                    if (cbp) put_se(sk, 0);
                }
                sk.finish();
            }
            if ((enc >> 31) && bcap.n && !ABL(SCROLL_DEBUG_DYN_NOWRITE)) {
                const int e_k = (int)(enc & 255u), e_pc = (int)((enc >> 8) & 255u);
                WSink sk{win, 0, 0, 0};
                sk.start(F + mbo((int)((enc >> 16) & 255u)) + L.boff[e_k][e_pc]);
                if ((enc >> 30) & 1u) {
                    sk.put_cap(bcap);
                } else {                           /* > 128 bits: re-encode from LDS */
                    const int blk = e_pc < 16 ? e_pc : 16 + (e_pc - 18);
                    const int8_t *lv = reinterpret_cast<const int8_t *>(L.lv8[24 * e_k + blk]);
                    cavlc_block(sk, TB, lv, e_pc < 16 ? 16 : 15, (int)((enc >> 24) & 63u) - 1);
                }
                sk.finish();
            }
            if (t < 2 * nd && !ABL(SCROLL_DEBUG_DYN_NOWRITE)) {   /* chroma DC, from LDS */
                const int k = t >> 1, p = t & 1;
                if (L.cbp[k] >> 4) {
                    int ry, cx;
                    dcoord(k, ry, cx);
                    WSink sk{win, 0, 0, 0};
                    sk.start(F + mbo((R.y0 + ry) * mbw + R.x0 + cx - m0) + L.boff[k][16 + p]);
                    const int16_t *o = L.dclv[k][p];
                    const int dq[4] = {o[0], o[1], o[2], o[3]};
                    cavlc_dc4(sk, PT, dq);
                    sk.finish();
                }
            }
            if (nd > 0 && t < 8) {                 /* left context of the next window */
                const uint8_t *tc = L.tc[nd - 1];
                L.lcarry[t] = t < 4 ? tc[4 * t + 3] : tc[16 + 4 * ((t - 4) >> 1) + 2 * ((t - 4) & 1) + 1];
            }
            __syncthreads();
            if (single) {
                pend_T = Tb;                       /* flushed during the next A */
            } else {                               /* rare: flush this pass now */
                const uint32_t nfull = Tb >> 5;
                const uint32_t n = p0 < nfull ? min(PW, nfull - p0) : 0u;
                flush_words(n, bw + p0);
                const uint32_t lastp = (Tb & 31u) && nfull - p0 < PW ? L.buf[nfull - p0] : 0u;
                __syncthreads();
                rewind_lnz();
                for (uint32_t jw = (uint32_t)t; jw < (uint32_t)BUF_WORDS; jw += DT)
                    L.buf[jw] = jw == 0 && p0 + PW >= nw ? lastp : 0u;
                __syncthreads();
            }
        }
        if (!single) {
            bw += Tb >> 5;
            F = Tb & 31u;
        }
        mark(3);
        m0 = m1;
    }

    if (!over) {
        if (pend_T) {                              /* the last window's whole words */
            const uint32_t pnf = pend_T >> 5;
            flush_words(pnf, bw);
            const uint32_t part = L.buf[pnf];
            __syncthreads();
            rewind_lnz();
            if (t == 0) L.buf[0] = part;
            F = pend_T & 31u;
            bw += pnf;
            __syncthreads();
        }
        /* rbsp_stop_one_bit + alignment (bitwriter.c:103-111); F < 32 */
        if (t == 0) {
            const uint32_t wv = L.buf[0] | (1u << (31 - F));
            const uint32_t nb = (F + 1u + 7u) >> 3;
            out[bw] = __builtin_bswap32(wv);
            int prev = L.lnz_r;
            my_ep += ep_word(wv, 4u * bw, 4u * bw + nb, prev, eplist, &L.ep_n);
            DF->rbsp_bytes = 4u * bw + nb;
        }
    }
    uint32_t ex, tot;
    block_excl_sum(my_ep, L.wsum, ex, tot);
    if (stamps && t == 0) {
        uint64_t *o = stamps + ((size_t)s * gridDim.x + f) * 8;
        for (int k = 0; k < 5; ++k) o[k] = ph[k];
        o[5] = nwin;
        o[6] = __builtin_amdgcn_s_memtime() - t_start;
        o[7] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);     /* HW_ID */
    }
    if (t == 0) {
        DF->ep = tot;
        DF->err = over ? DF_OVER : 0u;
        if (over) atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_DYN);
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
    if (df.ep <= (uint32_t)EPLIST_MAX) return;               /* k_dyn_emit_gather's NAL */
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
/* (all in practice: 82 per config-3 frame).  k_dyn_stage recorded where    */
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
    uint64_t *stp = stamps && t == 0 ? stamps + ((size_t)s * gridDim.x + f) * 8 : nullptr;
    if (stp) stp[0] = __builtin_amdgcn_s_memrealtime();
    const DynFrame df = dfr[(size_t)s * ld_fr + f];
    const int j = df.nal;
    if (j < 0 || j >= st[s].nnal || df.err) return;          /* nnal = 0: nothing committed */
    const uint32_t n = df.ep;
    if (n > (uint32_t)EPLIST_MAX) return;                     /* k_dyn_emit's NAL */
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
    const uint64_t cend = (o1 + 15) >> 4;
    int lg = 0;                   /* binary-search steps: 2^lg > n */
    while ((1u << lg) <= n) lg++;
    for (uint64_t cb = (o0 >> 4) + (uint64_t)t; cb < cend; cb += (uint64_t)U * DT) {
        uint32_t Ku[U], epm[U], shv[U];
        bool inner[U];
        uint4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t q0 = (cb + (uint64_t)u * DT) << 4;
            const int64_t u0 = (int64_t)q0 - (int64_t)o0 - 5;        /* EBSP index of byte 0 */
            /* K = EP bytes before the chunk; the j-th sits at EBSP index
             * sp[j] + j (strictly increasing): branch-free binary search,
             * the U searches of an iteration are independent */
            uint32_t K = 0;
            for (int b = lg - 1; b >= 0; --b) {
                const uint32_t k2 = K + (1u << b);
                K = k2 <= n && (int64_t)(sp[k2 - 1] + (k2 - 1)) < u0 ? k2 : K;
            }
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
int dyn_launch_stage(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                     int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                     const DynGeom *g, const uint8_t *src, const uint8_t *refs, uint8_t *stage,
                     uint64_t *stamps)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_dyn_stage<false>, dim3(nframes, S), dim3(DT), 0, hs, st, nal, ld_nal, pend,
                       dfr, ld_fr, *g, src, refs, stage, stamps);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(k_dyn_stage<true>, dim3(nframes, S), dim3(DT), 0, hs, st, nal, ld_nal, pend,
                       dfr, ld_fr, *g, src, refs, stage, (uint64_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int dyn_launch_emit(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal,
                    int ld_nal, const DynFrame *dfr, int ld_fr, const DynGeom *g,
                    const uint8_t *stage, uint8_t *arena, uint64_t ld_arena, uint64_t *stamps)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_dyn_emit_gather, dim3(nframes, S), dim3(DT), 0, hs, st, nal, ld_nal, dfr,
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
     * maximum + the stop word + k_dyn_stage's 16-byte margin */
    const size_t bits = (size_t)HDR_MAX + (size_t)mbw * mbh * (HEAD_MAX + 1) +
                        (size_t)rw * rh * MB_BITS_MAX + 64;
    return ((bits / 8 + 32 + DYN_OVF_BYTES) + 255) & ~(size_t)255;
}
