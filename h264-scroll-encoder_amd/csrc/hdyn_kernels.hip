/*
 * hdyn_kernels.hip -- MI355X (gfx950) kernels of the dynamic rect under UI
 * hints: one per-frame hint record with the motion regions AND the dynamic
 * rect (docs/MASTER_DESIGN.md:58-64,109-113,121-146 of the reference, which
 * describes it in prose only).  Bits: oracle/splice_oracle.c
 * or_hint_dyn_scroll_nal; tests/test_gpu_hintdyn.py checks them bit-exact.
 *
 * The rect's MBs keep the hint field's (ref, mv) -- any motion, per MB --
 * and carry the residual of the source minus the prediction at that motion.
 * k_hdyn_code turns each such MB into the record a spliced MB has
 * (SpliceMbRec: motion, cbp, per piece TotalCoeff / TrailingOnes and the
 * CAVLC bits after coeff_token, which do not depend on nC), so the frame is
 * composed by k_splice_stage exactly like a spliced one: mb_skip_run, ref_idx
 * and mvd for the frame's hint mode, cbp, mb_qp_delta 0, coeff_token for the
 * composed nC.  The rect may sit anywhere in each frame (per stream and
 * frame, scroll_batch_set_dyn_rect_at).
 *
 * k_hdyn_code: one wave per rect MB.  Lanes 0..23 take its 4x4 blocks
 * (luma raster, then Cb / Cr AC raster): residual against the prediction --
 * full-pel luma, 1/8-pel 2-D bilinear chroma (8.4.2.2.2), samples clamped to
 * the picture, waypoints resolved through their own rows (luma_row /
 * chroma_px_any) -- 4x4 transform, quant; lanes 24 / 25 the chroma DC 2x2;
 * then every piece measures its body, the MB's bodies go to its region of
 * the word pool (LDS first), and lane 0 writes the record.  Roofline: the
 * per-pixel reference sampler makes it issue-bound; it is the combined
 * path's correctness-first version (no BASELINE config uses it).
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "dyn_device.h"
#include "hdyn_engine.h"
#include "hint_device.h"
#include "splice_engine.h"
#include "stage_util.h"

using namespace scroll;
using namespace scroll::dyn;
using namespace scroll::stage;
using namespace scroll::hint;

namespace {


__constant__ Tabs h_tabs = SCROLL_DYN_TABS;

constexpr int HD_T = 64;                /* one wave per MB */

struct HdynLds {
    uint32_t buf[HDYN_MB_WORDS_MAX];    /* the MB's piece bodies */
    ScrollHintRect rc[SCROLL_HINT_MAX_RECTS];
    int32_t wo[8], wl[8], wv[8];
    int32_t lev[26][16];                /* levels per piece, scan order */
    int32_t wdc[2][4];                  /* chroma AC blocks' DC coefficients */
    uint32_t len[26], off[27];
    uint8_t tc[26], t1[26];
};

__device__ inline void lds_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct LdsOrW {
    uint32_t *b;
    __device__ inline void operator()(uint32_t i, uint32_t v) const { atomicOr(&b[i], v); }
};

/* TrailingOnes (9.2.1) of a block in scan order */
__device__ inline int t1_of(const int32_t *c, int max)
{
    int t1 = 0;
    bool stop = false;
    for (int i = max - 1; i >= 0; --i) {
        if (!c[i] || stop || t1 >= 3) continue;
        if (c[i] == 1 || c[i] == -1) t1++;
        else stop = true;
    }
    return t1;
}

/* grid (w h, frames, streams), HD_T threads */
__global__ __launch_bounds__(HD_T) void k_hdyn_code(const DevStream *__restrict__ st,
                                                    const NalDesc *__restrict__ nal, int ld_nal,
                                                    const PlanPending *__restrict__ pend,
                                                    const DynFrame *__restrict__ dfr, int ld_fr,
                                                    const HintFrame *__restrict__ hf,
                                                    const ScrollHintRect *__restrict__ pool,
                                                    SpliceFrame *__restrict__ spf, DynGeom g,
                                                    const uint8_t *__restrict__ src,
                                                    const uint8_t *__restrict__ refs,
                                                    SpliceMbRec *__restrict__ rec, uint32_t *__restrict__ rbsp,
                                                    uint32_t mb_words)
{
    __shared__ HdynLds L;
    const int q = blockIdx.x, f = blockIdx.y, s = blockIdx.z, t = threadIdx.x;
    const size_t fi = (size_t)s * ld_fr + f;
    const DynFrame df = dfr[fi];
    if (df.nal < 0) return;                                 /* experiment mode: no scroll NAL */
    const SpliceFrame SF = spf[fi];
    if (SF.w <= 0) return;                                  /* no rect in this frame */
    const HintFrame H = hf[fi];
    /* the fallback (k_hint_fb): a dormant whole-picture region (SF.pad 1)
     * codes only in a frame that falls back, whose hint rects are dropped */
    const bool fb = (H.mode & HINT_MODE_FB) != 0;
    if ((SF.pad & 1) && !fb) return;
    const int nr = fb ? 0 : min((int)H.n, SCROLL_HINT_MAX_RECTS);
    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    for (int i = t; i < nr; i += HD_T) L.rc[i] = pool[H.first + i];
    for (uint32_t i = (uint32_t)t; i < mb_words; i += HD_T) L.buf[i] = 0u;
    lds_wave_sync();
    const DevStream *S = st + s;
    const NalDesc d = nal[(size_t)s * ld_nal + df.nal];
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
    const Regions rg = regions(c);
    const Layout lay{(c.h - c.off) / 16, rg.ra, 4 * rg.mva, rg.rb, 4 * rg.mvb};
    const int lx = q % SF.w, ly = q / SF.w, x = SF.x0 + lx, y = SF.y0 + ly;
    bool bad;
    const Mv me = field(L.rc, L.wv, nr, x, y, lay, c.nwp, bad);
    SpliceMbRec *R = rec + SF.rec_first + q;
    if (bad) {                                              /* k_splice_stage reports the reference */
        if (t == 0) {
            SpliceMbRec r{};
            r.ref = (int16_t)me.ref;
            r.mx = me.mx;
            r.my = me.my;
            *R = r;
        }
        return;
    }
    /* the frame's rect QP (scroll_batch_set_dyn_qp / _stream / _at) */
    const int qpy = __builtin_amdgcn_readfirstlane(SF.hd_qp);
    const QParams HQ = qparams_rt(qpy), HQC = qparams_rt(qp_chroma(qpy));
    const int mvx = me.mx / 4, mvy = me.my / 4, W = c.w, Hh = c.h;
    const uint32_t ysz = (uint32_t)W * (uint32_t)Hh;
    const uint8_t *rp = refs + (size_t)s * g.ref_ld;
    RefPics RP;
    for (int k = 0; k < 2; ++k) {
        RP.pl[k][0] = rp + (size_t)k * (ysz + ysz / 2);
        RP.pl[k][1] = RP.pl[k][0] + ysz;
        RP.pl[k][2] = RP.pl[k][1] + ysz / 4;
    }
    RP.w = W;
    RP.h = Hh;
    const WpTab T{L.wo, L.wv, Hh};
    const uint8_t *fs = src + (size_t)s * g.src_ld + (size_t)f * g.src_fr;
    const int lw = 16 * g.w, cw = 8 * g.w;

    /* ---- lanes 0..23: one 4x4 block each -------------------------------- */
    if (t < 24) {
        int res[16], Wc[16];
        if (t < 16) {
            const int bx = 4 * (t & 3), by = 4 * (t >> 2);
            for (int i = 0; i < 4; ++i) {
                int yo;
                const int b = luma_row(T, me.ref, 16 * y + by + i + mvy, yo);
                const uint8_t *prow = RP.pl[b][0] + (size_t)yo * W;
                const uint8_t *srow = fs + (size_t)(16 * ly + by + i) * lw + 16 * lx + bx;
                for (int j = 0; j < 4; ++j) {
                    const int X = clampi(16 * x + bx + j + mvx, 0, W - 1);
                    res[4 * i + j] = (int)srow[j] - (int)prow[X];
                }
            }
        } else {
            const int p = (t - 16) >> 2, k = (t - 16) & 3, bx = 4 * (k & 1), by = 4 * (k >> 1);
            const int qx = 4 * mvx, qy = 4 * mvy, fx = qx & 7, fy = qy & 7, wc = W / 2;
            const uint8_t *pl = fs + (size_t)lw * 16 * g.h + (size_t)p * cw * 8 * g.h;
            for (int i = 0; i < 4; ++i) {
                const uint8_t *srow = pl + (size_t)(8 * ly + by + i) * cw + 8 * lx + bx;
                const int yi = 8 * y + by + i + (qy >> 3);
                for (int j = 0; j < 4; ++j) {
                    const int xi = 8 * x + bx + j + (qx >> 3);
                    const int x0 = clampi(xi, 0, wc - 1), x1 = clampi(xi + 1, 0, wc - 1);
                    const int A = chroma_px_any<9>(T, RP, me.ref, 1 + p, x0, yi);
                    const int B = chroma_px_any<9>(T, RP, me.ref, 1 + p, x1, yi);
                    const int C = chroma_px_any<9>(T, RP, me.ref, 1 + p, x0, yi + 1);
                    const int D = chroma_px_any<9>(T, RP, me.ref, 1 + p, x1, yi + 1);
                    const int pr = ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C +
                                    fx * fy * D + 32) >> 6;
                    res[4 * i + j] = (int)srow[j] - pr;
                }
            }
        }
        fwd4x4(res, Wc);
        if (t < 16) {
            for (int k2 = 0; k2 < 16; ++k2) L.lev[t][k2] = quant(Wc[ZZ[k2]], ZZ[k2], HQ);
        } else {
            const int p = (t - 16) >> 2, k = (t - 16) & 3, pc = 18 + 4 * p + k;
            L.wdc[p][k] = Wc[0];
            for (int k2 = 1; k2 < 16; ++k2) L.lev[pc][k2 - 1] = quant(Wc[ZZ[k2]], ZZ[k2], HQC);
            L.lev[pc][15] = 0;
        }
    }
    lds_wave_sync();
    if (t == 24 || t == 25) {                               /* chroma DC 2x2 Hadamard */
        const int p = t - 24;
        const int d0 = L.wdc[p][0], d1 = L.wdc[p][1], d2 = L.wdc[p][2], d3 = L.wdc[p][3];
        L.lev[16 + p][0] = quant_dc(d0 + d1 + d2 + d3, HQC);
        L.lev[16 + p][1] = quant_dc(d0 - d1 + d2 - d3, HQC);
        L.lev[16 + p][2] = quant_dc(d0 + d1 - d2 - d3, HQC);
        L.lev[16 + p][3] = quant_dc(d0 - d1 - d2 + d3, HQC);
    }
    lds_wave_sync();

    /* ---- lanes 0..25: one piece each: TotalCoeff, TrailingOnes, body ---- */
    const int pc = t;
    int max = 0, nC = 0;
    if (pc < 26) {
        max = pc < 16 ? 16 : (pc < 18 ? 4 : 15);
        nC = pc == 16 || pc == 17 ? -1 : 0;
        int tc = 0;
        for (int k = 0; k < max; ++k) tc += L.lev[pc][k] != 0;
        const int t1 = t1_of(L.lev[pc], max);
        uint32_t tv;
        int tl;
        coeff_token(h_tabs, tc, t1, nC, tv, tl);
        CountSink cn{0};
        cavlc_block(cn, h_tabs, L.lev[pc], max, nC);
        L.tc[pc] = (uint8_t)tc;
        L.t1[pc] = (uint8_t)t1;
        L.len[pc] = cn.n - (uint32_t)tl;
    }
    lds_wave_sync();
    if (t == 0) {
        /* the bodies in syntax order (luma4x4BlkIdx, then chroma), as the
         * stage walks them from res_off (no coeff_tokens between them here) */
        uint32_t o = 0;
        for (int j = 0; j < 26; ++j) {
            const int q8 = j >> 2, q4 = j & 3;
            const int k = j < 16 ? 4 * ((q8 >> 1) * 2 + (q4 >> 1)) + (q8 & 1) * 2 + (q4 & 1) : j;
            L.off[k] = o;
            o += L.len[k];
        }
        L.off[26] = o;
    }
    lds_wave_sync();
    const bool over = L.off[26] > 32u * mb_words;
    if (over) {
        if (t == 0) atomicMax(&spf[fi].status, HDYN_STATUS_OVERFLOW);
        return;
    }
    if (pc < 26 && L.len[pc]) {
        uint32_t tv;
        int tl;
        coeff_token(h_tabs, L.tc[pc], L.t1[pc], nC, tv, tl);
        OrSink<LdsOrW> ws{LdsOrW{L.buf}, 0, 0, 0};
        ws.start(L.off[pc]);
        SkipSink<OrSink<LdsOrW>> sk{ws, (uint32_t)tl};
        cavlc_block(sk, h_tabs, L.lev[pc], max, nC);
        ws.finish();
    }
    lds_wave_sync();
    uint32_t *region = rbsp + SF.rbsp_word + (size_t)q * mb_words;
    const uint32_t nw = (L.off[26] + 31u) >> 5;
    for (uint32_t i = (uint32_t)t; i < nw; i += HD_T) region[i] = L.buf[i];
    if (t == 0) {
        SpliceMbRec r{};
        r.ref = (int16_t)me.ref;
        r.mx = me.mx;
        r.my = me.my;
        r.qpd = 0;
        int cbp_l = 0, dcn = 0, acn = 0;
        for (int k = 0; k < 16; ++k)
            if (L.tc[k]) cbp_l |= 1 << (2 * (k >> 3) + ((k & 3) >> 1));
        dcn = L.tc[16] + L.tc[17];
        for (int k = 18; k < 26; ++k) acn += L.tc[k];
        r.cbp = (uint8_t)(cbp_l | (acn ? 2 : (dcn ? 1 : 0)) << 4);
        if (r.cbp) atomicMin(&spf[fi].hd_first, (uint32_t)q);    /* the mb_qp_delta chain's first MB */
        uint32_t body = 0;
        r.res_off = 32u * (uint32_t)q * mb_words;      /* the bodies from here (res_len 0: no whole run) */
        for (int k = 0; k < 26; ++k) {
            r.tc[k] = L.tc[k];
            r.t1[k] = L.t1[k];
            r.bl[k] = (uint16_t)L.len[k];                /* no token bits before it */
            body += L.len[k];
        }
        r.body = (uint16_t)body;
        *R = r;
    }
}

/* grid (frames, streams): the frames' status back to OK before k_hdyn_code */
__global__ void k_hdyn_reset(SpliceFrame *__restrict__ spf, int ld_fr)
{
    SpliceFrame &F = spf[(size_t)blockIdx.y * ld_fr + blockIdx.x];
    if (F.w > 0) {
        F.status = SCROLL_SPLICE_OK;
        F.hd_first = ~0u;
    }
}

}  // namespace

int hdyn_launch_code(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal,
                     int ld_nal, const PlanPending *pend, const DynFrame *dfr, int ld_fr,
                     const HintFrame *hf, const ScrollHintRect *pool, SpliceFrame *spf,
                     const DynGeom *g, const uint8_t *src, const uint8_t *refs, SpliceMbRec *rec,
                     uint32_t *rbsp, uint32_t mb_words)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_hdyn_reset, dim3(nframes, S), dim3(1), 0, hs, spf, ld_fr);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(k_hdyn_code, dim3(g->w * g->h, nframes, S), dim3(HD_T), 0, hs, st, nal, ld_nal, pend,
                       dfr, ld_fr, hf, pool, spf, *g, src, refs, rec, rbsp, mb_words);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
