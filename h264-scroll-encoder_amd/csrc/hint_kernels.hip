/*
 * hint_kernels.hip -- MI355X (gfx950) kernel of the UI-hint P slice
 * (design only in the reference:
 * docs/MASTER_DESIGN.md:58-64,103-146).  With hints, a scroll NAL's MV field
 * is no longer two row-uniform regions: rects of MBs carry their own
 * (ref, mv) over the scroll layout, so neighbouring MBs predict from
 * different motion and (in the P_Skip mode) runs of MBs are skipped.  The
 * NALs take the staged path of the dynamic rect:
 *
 *   k_plan (state pass)  waypoint state machine, NalDesc per NAL
 *   k_hint_stage         one workgroup per scroll NAL: its whole RBSP into a
 *                        staging slot + its emulation-prevention positions
 *   k_plan (size pass)   NAL sizes (5 + RBSP + EP), arena offsets
 *   k_emit / k_dyn_emit_gather   waypoint NALs / staged NALs -> arena
 *
 * k_hint_stage codes 256 MBs per window, one per lane: the MB's and its
 * neighbours' (ref, mv) from the LDS rect list, the prediction (the
 * reference's get_mv_prediction, h264_writer.c:369-432, or the standard's
 * 8.4.1.3), the P_Skip decision (8.4.1.1), mb_skip_run by an exclusive
 * max-scan of coded MB indices, the codeword into a 128-bit register, its
 * offset by a sum-scan, then an LDS OR and a flush of whole words.  Bits:
 * oracle/hint_oracle.c; tests/test_gpu_hints.py checks them bit-exact.
 * Roofline: issue-bound per MB (rect lookups); HBM traffic is the NAL bytes
 * out.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "dyn_device.h"
#include "hint_device.h"
#include "hint_engine.h"
#include "splice_engine.h"
#include "stage_util.h"

using namespace scroll;
using namespace scroll::dyn;
using namespace scroll::stage;
using namespace scroll::hint;

namespace {

constexpr int HDR_BITS = 1024;          /* slice header bound (8 waypoints + MMCO ~ 250) */
constexpr int MB_BITS = 128;            /* one MB: run + type + ref + 2 mvd + cbp <= 110 */
constexpr int HB_WORDS = 1152;          /* LDS bit buffer: header + one window + carry */
static_assert(HB_WORDS * 32 >= HDR_BITS + DT * MB_BITS + 64, "a window fits the buffer");
constexpr int RING = 512;               /* MB motion ring: this window + the row above */
static_assert(RING >= DT + HINT_MAX_MBW + 1, "the row above a window stays in the ring");

struct HintLds {
    uint32_t buf[HB_WORDS];
    int32_t fr[RING], fx[RING], fy[RING];   /* motion of MB m at m % RING */
    ScrollHintRect rc[SCROLL_HINT_MAX_RECTS];
    int32_t wo[8], wl[8], wv[8];
    uint32_t wsum[NW];
    int32_t wmax[NW];
    int32_t lnz_r, lnz_w;         /* last non-zero staged byte: before / of a flush */
    uint32_t ep_n;                /* EP positions recorded                         */
    int32_t bad;                  /* an MB took a rect with an invalid reference   */
};

__global__ __launch_bounds__(DT) void k_hint_stage(DevStream *__restrict__ st,
                                                   const NalDesc *__restrict__ nal, int ld_nal,
                                                   const PlanPending *__restrict__ pend,
                                                   DynFrame *__restrict__ dfr, int ld_fr,
                                                   const HintFrame *__restrict__ hf,
                                                   const ScrollHintRect *__restrict__ pool,
                                                   uint8_t *__restrict__ stage, uint64_t slot_bytes)
{
    __shared__ HintLds L;
    const int s = blockIdx.y, f = dyn_frame_of(blockIdx.x, s), t = threadIdx.x;
    DevStream *S = st + s;
    DynFrame *DF = dfr + (size_t)s * ld_fr + f;
    const int j = DF->nal;
    if (j < 0) return;                                     /* experiment mode: no scroll NAL */
    const HintFrame H = hf[(size_t)s * ld_fr + f];
    if (H.mode & (HINT_MODE_SPLICED | HINT_MODE_FB)) return;   /* k_splice_stage's frame */
    const int nr = min((int)H.n, SCROLL_HINT_MAX_RECTS);
    const int hmode = H.mode & 0xff;
    const bool pskip = hmode == SCROLL_HINT_PSKIP;
    const bool spec = hmode != SCROLL_HINT_EXACT;
    if (t == 0) {
        L.lnz_r = -1;
        L.lnz_w = -1;
        L.ep_n = 0;
        L.bad = 0;
    }
    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    if (t < nr) L.rc[t] = pool[H.first + t];
    for (int i = t; i < HB_WORDS; i += DT) L.buf[i] = 0u;
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
    const int mbw = c.w / 16, mbh = c.h / 16, nmb = mbw * mbh;
    const Regions rg = regions(c);
    const Layout lay{(c.h - c.off) / 16, rg.ra, 4 * rg.mva, rg.rb, 4 * rg.mvb};
    const int nrefs = 2 + c.nwp;
    const uint32_t m_mbw = magic32((uint32_t)mbw);
    uint8_t *slot = stage + ((size_t)s * ld_fr + f) * slot_bytes;
    uint32_t *out = reinterpret_cast<uint32_t *>(slot);
    const uint32_t cap_words = (uint32_t)((slot_bytes - DYN_OVF_BYTES) / 4) - 4u;
    uint32_t *eplist = reinterpret_cast<uint32_t *>(slot + slot_bytes - DYN_OVF_BYTES);

    uint32_t bw = 0;             /* staging word of buf[0] */
    uint32_t my_ep = 0;
    bool over = false;
    int last = -1;               /* last coded MB before the window (uniform) */
    bool my_bad = false;
    for (int m0 = 0; m0 < nmb; m0 += DT) {
        const int m = m0 + t;
        CapSink cs{0, 0, 0};
        bool coded = false;
        Mv me{0, 0, 0};
        int px = 0, py = 0;
        if (m < nmb) {
            const int y = (int)div_m((uint32_t)m, m_mbw), x = m - y * mbw;
            bool bad;
            me = field(L.rc, L.wv, nr, x, y, lay, c.nwp, bad);
            my_bad |= bad;
            L.fr[m & (RING - 1)] = me.ref;
            L.fx[m & (RING - 1)] = me.mx;
            L.fy[m & (RING - 1)] = me.my;
        }
        __syncthreads();
        if (m < nmb) {
            /* neighbours from the ring: this window or the one(s) before */
            const int y = (int)div_m((uint32_t)m, m_mbw), x = m - y * mbw;
            auto at = [&](int k) { return Mv{L.fr[k & (RING - 1)], L.fx[k & (RING - 1)], L.fy[k & (RING - 1)]}; };
            const Mv none{-1, 0, 0};
            const Mv A = x > 0 ? at(m - 1) : none;
            const Mv B = y > 0 ? at(m - mbw) : none;
            const Mv C = y == 0 ? none : (x + 1 < mbw ? at(m - mbw + 1) : (x > 0 ? at(m - mbw - 1) : none));
            if (spec) {
                int sx, sy;
                pskip_mv(x > 0, y > 0, A, B, C, sx, sy);
                coded = !pskip || !(me.ref == 0 && me.mx == sx && me.my == sy);
                predict_spec(A, B, C, me.ref, px, py);
            } else {
                coded = true;
                predict_ref(A, B, C, me.ref, px, py);
            }
        }
        /* mb_skip_run = MBs since the previous coded one (7.3.4) */
        int excl, cmax;
        block_excl_max(coded ? m : -1, L.wmax, excl, cmax);
        if (coded) {
            put_ue(cs, (uint32_t)(m - max(excl, last) - 1));
            cs.put(1, 1);                                  /* mb_type P_L0_16x16 ue(0) */
            if (nrefs == 2) cs.put((uint32_t)(1 - (me.ref & 1)), 1);   /* te(), :441-445 */
            else if (nrefs > 2) put_ue(cs, (uint32_t)me.ref);
            put_se(cs, me.mx - px);
            put_se(cs, me.my - py);
            cs.put(1, 1);                                  /* coded_block_pattern ue(0) */
        }
        last = max(last, cmax);
        uint32_t off, T;
        block_excl_sum(cs.n, L.wsum, off, T);
        if (bw + ((F + T) >> 5) + 3u > cap_words) {        /* uniform */
            over = true;
            break;
        }
        if (cs.n) {
            LSink sk{{L.buf}, 0, 0, 0};
            sk.start(F + off);
            sk.put_cap(cs);
            sk.finish();
        }
        __syncthreads();
        /* whole words -> staging, EP positions with the zero run looked up
         * backwards in buf (L.lnz_r before buf[0]) */
        const uint32_t nf = (F + T) >> 5;
        for (uint32_t jw = (uint32_t)t; jw < nf; jw += DT) {
            const uint32_t wv = L.buf[jw];
            out[bw + jw] = __builtin_bswap32(wv);
            int prev = L.lnz_r;
            for (int jj = (int)jw - 1; jj >= 0; --jj) {
                const uint32_t pv = L.buf[jj];
                if (pv) {
                    prev = 4 * (int)(bw + jj) + last_nz_byte(pv);
                    break;
                }
            }
            const uint32_t gb = 4u * (bw + jw);
            my_ep += ep_word(wv, gb, 0xffffffffu, prev, eplist, &L.ep_n);
            if (wv) atomicMax(&L.lnz_w, (int)gb + last_nz_byte(wv));
        }
        const uint32_t part = L.buf[nf];
        __syncthreads();
        for (uint32_t jw = (uint32_t)t; jw <= nf; jw += DT) L.buf[jw] = jw == 0 ? part : 0u;
        if (t == 0) {
            L.lnz_r = max(L.lnz_r, L.lnz_w);
            L.lnz_w = -1;
        }
        F = (F + T) & 31u;
        bw += nf;
        __syncthreads();
    }
    if (my_bad) L.bad = 1;

    if (!over && t == 0) {
        /* trailing skipped MBs, rbsp_stop_one_bit + alignment (bitwriter.c:103-111) */
        LSink sk{{L.buf}, 0, 0, 0};
        sk.start(F);
        uint32_t nb = F + 1u;
        if (last < nmb - 1) {
            CountSink cc{0};
            put_ue(cc, (uint32_t)(nmb - 1 - last));
            put_ue(sk, (uint32_t)(nmb - 1 - last));
            nb += cc.n;
        }
        sk.put(1, 1);
        sk.finish();
        const uint32_t nbytes = (nb + 7u) >> 3;
        int prev = L.lnz_r;
        for (uint32_t k = 0; 4u * k < nbytes; ++k) {
            const uint32_t wv = L.buf[k];
            out[bw + k] = __builtin_bswap32(wv);
            my_ep += ep_word(wv, 4u * (bw + k), 4u * bw + nbytes, prev, eplist, &L.ep_n);
        }
        DF->rbsp_bytes = 4u * bw + nbytes;
    }
    uint32_t ex, tot;
    block_excl_sum(my_ep, L.wsum, ex, tot);
    if (t == 0) {
        const bool bad = L.bad != 0;
        DF->ep = tot;
        DF->err = over ? 1u : (bad ? 4u : 0u);
        if (over) atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_DYN);
        if (bad) atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_HINT);
    }
}

/* The conventional-encode fallback (docs/MASTER_DESIGN.md:220, "hints
 * missing/inconsistent -> full conventional encode"; scroll_batch_set_fallback):
 * one workgroup per scroll NAL, before the stage kernels.  A frame whose hint
 * record has an MB on a rect naming a reference the frame lacks -- the frames
 * that fail their stream with SCROLL_ERR_CONFIG otherwise -- is marked
 * HINT_MODE_FB: k_hint_stage leaves it, k_hdyn_code codes its whole picture
 * (the batch's rect is the picture) over the scroll frame's own motion (its
 * hint rects dropped) and k_splice_stage composes it in the frame's hint
 * mode.  The bit is the device's: set or cleared here every compose. */
__global__ __launch_bounds__(DT) void k_hint_fb(const DevStream *__restrict__ st,
                                                const NalDesc *__restrict__ nal, int ld_nal,
                                                const PlanPending *__restrict__ pend,
                                                const DynFrame *__restrict__ dfr, int ld_fr,
                                                HintFrame *__restrict__ hf,
                                                const ScrollHintRect *__restrict__ pool)
{
    __shared__ ScrollHintRect rc[SCROLL_HINT_MAX_RECTS];
    __shared__ int32_t wv[8];
    __shared__ int32_t any;
    const int s = blockIdx.y, f = blockIdx.x, t = threadIdx.x;
    const size_t fi = (size_t)s * ld_fr + f;
    const HintFrame H = hf[fi];
    const int j = dfr[fi].nal;
    const int nr = min((int)H.n, SCROLL_HINT_MAX_RECTS);
    bool bad = false;
    if (j >= 0 && nr > 0) {                                /* uniform */
        if (t < nr) rc[t] = pool[H.first + t];
        if (t < 8) wv[t] = pend[s].wv[t];
        if (t == 0) any = 0;
        __syncthreads();
        const DevStream *S = st + s;
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
        const Regions rg = regions(c);
        const Layout lay{(c.h - c.off) / 16, rg.ra, 4 * rg.mva, rg.rb, 4 * rg.mvb};
        const int mbw = c.w / 16, nmb = mbw * (c.h / 16);
        bool my = false;
        for (int m = t; m < nmb; m += DT) {
            bool b1;
            (void)field(rc, wv, nr, m % mbw, m / mbw, lay, c.nwp, b1);
            my |= b1;
        }
        if (my) any = 1;
        __syncthreads();
        bad = any != 0;
    }
    if (t == 0) {
        const int32_t mode = bad ? (H.mode | HINT_MODE_FB) : (H.mode & ~HINT_MODE_FB);
        if (mode != H.mode) hf[fi].mode = (int16_t)mode;
    }
}

}  // namespace

int hint_launch_fb(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal, int ld_nal,
                   const PlanPending *pend, const DynFrame *dfr, int ld_fr, HintFrame *hf,
                   const ScrollHintRect *pool)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_hint_fb, dim3(nframes, S), dim3(DT), 0, hs, st, nal, ld_nal, pend, dfr, ld_fr, hf, pool);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int hint_launch_stage(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                      int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                      const HintFrame *hf, const ScrollHintRect *pool, uint8_t *stage,
                      uint64_t slot_bytes)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_hint_stage, dim3(nframes, S), dim3(DT), 0, hs, st, nal, ld_nal, pend, dfr,
                       ld_fr, hf, pool, stage, slot_bytes);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t hint_slot_bound(int mbw, int mbh)
{
    const size_t bits = (size_t)HDR_BITS + (size_t)mbw * mbh * MB_BITS + 64;
    return ((bits / 8 + 64 + DYN_OVF_BYTES) + 255) & ~(size_t)255;
}
