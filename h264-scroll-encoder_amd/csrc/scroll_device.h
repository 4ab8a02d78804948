/*
 * scroll_device.h -- device-side building blocks of the P-slice composer
 * (gfx950, wave64).  Included by scroll_kernels.hip only.
 *
 * Reference path restated here (wreuven/h264-scroll-encoder):
 *   src/h264_writer.c:455-539  P slice headers            -> emit_slice_header
 *   src/h264_writer.c:362-432  MV prediction / median3    -> median3, predict
 *   src/h264_writer.c:434-453  P_L0_16x16 MB syntax       -> put_mb
 *   src/h264_writer.c:541-664  scroll P frame             -> build_nal / serial_nal
 *   src/h264_writer.c:678-782  waypoint P frame           -> build_nal / serial_nal (kind 1)
 *   src/bitwriter.c:50-111     ue/se/trailing bits        -> put_ue / put_se
 *   src/nal.c:24-84            start code + EP            -> prefix + EP automaton
 *
 * Key idea (DESIGN.md "row-class compaction"): every MB of a macroblock row
 * shares (ref_idx, mv) (src/h264_writer.c:601-617), so an MB's predictor
 * depends only on (x == 0, x == mbw-1, y == 0, region of its row, region of
 * the row above).  A frame therefore is a short list of RUNS, each one MB
 * codeword repeated k times.  The emit kernel random-accesses the slice bit
 * string through that list, so every lane produces 16 output bytes
 * independently -- no serial bit writer, no cross-lane scan.
 */
#ifndef SCROLL_DEVICE_H
#define SCROLL_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace scroll {

constexpr int MVL = 496;          /* MV_LIMIT_PX, include/h264_writer.h:24       */
constexpr int RUNS_MAX = 9;       /* runs per NAL on the fast path (row-class max) */
constexpr int HDR_WORDS = 8;      /* 256 bits: 40-bit NAL prefix + slice header
                                     (worst realistic case ~209 bits: 8 waypoints +
                                     MMCO; longer headers take the serial path)  */
constexpr int EP_ZERO_RUN = 22;   /* 00 00 0x (x<=3) needs >= 22 consecutive 0s   */

/* Per-NAL emission layout, built in LDS by one lane.  172 bytes = 43 dwords:
 * an odd stride keeps lanes that read different NALs on different banks.
 * Everything derivable from a run's codeword length (mul-high magic, the
 * pattern's continuation past 64 bits) lives in the per-wave LenLut. */
struct Lay {
    uint32_t nal_bits;            /* 8 * NAL bytes (prefix + RBSP incl. padding)  */
    uint32_t used_bits;           /* prefix + header + runs + stop bit            */
    uint32_t hdr_bits;            /* prefix (40) + slice header                   */
    uint32_t nruns;
    uint32_t hdr[HDR_WORDS];      /* prefix + header bits, MSB first              */
    uint32_t run_end[RUNS_MAX];   /* NAL bit where run r ends                     */
    uint32_t pat[RUNS_MAX][2];    /* run codeword repeated over 64 bits           */
    uint8_t len[RUNS_MAX];        /* codeword length (1..64)                      */
    uint8_t pad_[7];
};
static_assert(sizeof(Lay) == 172, "Lay stride must stay an odd number of dwords");

/* Per codeword length len in 1..64 (index len - 1): the mul-high magic
 * ceil(2^32 / len) and the pattern phases 64 / 96 / 128 / 160 mod len. */
struct LenLut {
    uint32_t magic[64];
    uint32_t mods[64];            /* bytes: 64%len | 96%len << 8 | 128%len << 16 | 160%len << 24 */
};

__device__ inline void lut_entry(uint32_t len, uint32_t &magic, uint32_t &mods)
{
    magic = len == 1 ? 0xffffffffu : 0xffffffffu / len + 1u;   /* ceil(2^32/len), len >= 2 */
    mods = (64u % len) | ((96u % len) << 8) | ((128u % len) << 16) | ((160u % len) << 24);
}

/* Everything the syntax of one NAL depends on. */
struct NalCtx {
    int w, h, log2_mfn, poc_type, log2_poc, deblock;
    int kind;                     /* 0 scroll, 1 waypoint                         */
    int off;                      /* offset_px                                    */
    int frame_num;                /* raw cfg->frame_num                           */
    int nwp;                      /* cfg->num_waypoints snapshot                  */
    const int32_t *wp_off, *wp_lt, *wp_valid;
    int qpd = 0;                  /* slice_qp_delta (the dynamic rect's QP - 26)  */
};

/* ---------------------------------------------------------------------- */
/* zero-run tracker over the RBSP: decides whether emulation prevention    */
/* can trigger (it cannot without >= 22 consecutive zero bits).            */
/* ---------------------------------------------------------------------- */
struct ZR {
    int cur, max;
};

__device__ inline void zr_push(ZR &z, uint64_t v, int n, uint32_t rep = 1)
{
    /* v: right-aligned n-bit field (1 <= n <= 64), repeated rep >= 1 times */
    uint64_t l = v << (64 - n);
    if (l == 0) {
        uint64_t add = (uint64_t)n * rep;
        z.cur = add > 0x40000000ull ? 0x40000000 : (int)(z.cur + add);
        if (z.cur > 0x40000000) z.cur = 0x40000000;
        return;
    }
    int lead = __clzll(l);
    int trail = __builtin_ctzll(l) - (64 - n);
    int m = z.cur + lead;
    if (n - 2 >= EP_ZERO_RUN) {               /* internal gaps can matter */
        uint64_t x = l & ~(0x8000000000000000ull >> lead);
        int prev = lead;
        while (x) {
            int p = __clzll(x);
            m = max(m, p - prev - 1);
            prev = p;
            x &= ~(0x8000000000000000ull >> p);
        }
    }
    if (rep > 1) m = max(m, trail + lead);
    z.max = max(z.max, m);
    z.cur = trail;
}

/* ---------------------------------------------------------------------- */
/* bit sinks                                                               */
/* ---------------------------------------------------------------------- */
__device__ inline uint32_t low_mask(int n) { return n >= 32 ? 0xffffffffu : ((1u << n) - 1u); }

/* header bits -> LDS words (STORE) or just counted.  CHECK tracks zero runs
 * and the HDR_WORDS bound; the emit kernel builds only NALs the plan kernel
 * already proved fast, so it skips both.  Words are assembled in a 64-bit
 * register and written whole (no LDS read-modify-write). */
template <bool STORE, bool CHECK>
struct HdrSink {
    uint32_t *w;
    int len;
    bool over;
    bool track;
    ZR zr;
    uint64_t acc;                  /* pending bits (len & 31), left-aligned */
    __device__ inline void put(uint32_t v, int n)
    {
        if (n <= 0) return;
        v &= low_mask(n);
        if (CHECK) {
            if (track) zr_push(zr, v, n);
            if (len + n > HDR_WORDS * 32) {
                over = true;
                len += n;
                return;
            }
        }
        if (STORE) {
            const int nacc = len & 31;
            acc |= ((uint64_t)v << (64 - n)) >> nacc;
            if (nacc + n >= 32) {
                w[len >> 5] = (uint32_t)(acc >> 32);
                acc <<= 32;
            }
        }
        len += n;
    }
    /* flush the partial word and zero the rest of the header words */
    __device__ inline void finish()
    {
        if (!STORE || over) return;
        int k = len >> 5;
        if (len & 31) w[k++] = (uint32_t)(acc >> 32);
        for (; k < HDR_WORDS; ++k) w[k] = 0u;
    }
};

/* one MB codeword, left-aligned in 64 bits */
struct CodeSink {
    uint64_t v;
    int len;
    bool over;
    __device__ inline void put(uint32_t x, int n)
    {
        if (n <= 0) return;
        x &= low_mask(n);
        if (len + n > 64) {
            over = true;
            len += n;
            return;
        }
        v |= ((uint64_t)x << (64 - n)) >> len;
        len += n;
    }
};

/* bitwriter.c:50-74: ue(v) = M zeros, then v+1 in M+1 bits (uint32 wrap kept) */
template <class S>
__device__ inline void put_ue(S &s, uint32_t v)
{
    if (v == 0) {
        s.put(1, 1);
        return;
    }
    uint32_t x = v + 1u;
    if (x == 0) {            /* v = 0xFFFFFFFF: reference writes one '0' bit */
        s.put(0, 1);
        return;
    }
    int m = 31 - __clz((int)x);
    if (m) s.put(0, m);
    s.put(x, m + 1);
}

/* bitwriter.c:91-101 */
template <class S>
__device__ inline void put_se(S &s, int32_t v)
{
    uint32_t k = v > 0 ? 2u * (uint32_t)v - 1u : (uint32_t)(-2 * (int64_t)v);
    put_ue(s, k);
}

/* h264_writer.c:455-488 (plain) and :490-539 (waypoint-aware) */
template <class S>
__device__ inline void emit_slice_header(S &s, const NalCtx &c)
{
    int fn = c.frame_num % (1 << c.log2_mfn);        /* :547 */
    bool wp_style = c.kind == 1 || c.nwp > 0;        /* :549-553, :687 */
    bool is_ref = c.kind == 1;
    put_ue(s, 0);                                    /* first_mb_in_slice */
    put_ue(s, 0);                                    /* slice_type P      */
    put_ue(s, 0);                                    /* pps_id            */
    s.put((uint32_t)(fn & ((1 << c.log2_mfn) - 1)), c.log2_mfn);
    if (c.poc_type == 0)
        s.put((uint32_t)((fn * 2) & ((1 << c.log2_poc) - 1)), c.log2_poc);
    s.put(1, 1);                                     /* override flag     */
    if (!wp_style) {
        put_ue(s, 1);
        s.put(1, 1);
        put_ue(s, 2); put_ue(s, 0);
        put_ue(s, 2); put_ue(s, 1);
        put_ue(s, 3);
        if (is_ref) s.put(0, 1);
    } else {
        put_ue(s, (uint32_t)(2 + c.nwp - 1));
        s.put(1, 1);
        put_ue(s, 2); put_ue(s, 0);
        put_ue(s, 2); put_ue(s, 1);
        for (int i = 0; i < c.nwp; ++i) {
            if (!c.wp_valid[i]) continue;
            put_ue(s, 2);
            put_ue(s, (uint32_t)c.wp_lt[i]);
        }
        put_ue(s, 3);
        if (is_ref) {                                /* lt_idx = 2 + nwp (:685) */
            int lt = 2 + c.nwp;
            s.put(1, 1);
            put_ue(s, 4); put_ue(s, (uint32_t)(lt + 1));
            put_ue(s, 6); put_ue(s, (uint32_t)lt);
            put_ue(s, 0);
        }
    }
    put_se(s, c.qpd);                                /* slice_qp_delta (0: h264_writer.c:486) */
    if (c.deblock) put_ue(s, 1);                     /* disable deblocking */
}

/* ---------------------------------------------------------------------- */
/* region split and waypoint choice: h264_writer.c:555-617 / :689-729      */
/* ---------------------------------------------------------------------- */
struct Regions {
    int ra, mva, rb, mvb;    /* ref_idx and mv_y (pixels) of region A / B */
};

__device__ inline Regions regions(const NalCtx &c)
{
    Regions r;
    int n = c.nwp;
    int wa = -1, woa = 0;
    if (c.off > MVL && (c.kind == 1 || n > 0)) {
        for (int i = 0; i < n; ++i) {
            if (!c.wp_valid[i]) continue;
            int wo = c.wp_off[i];
            if (wo <= c.off && wo > woa && c.off - wo <= MVL) {
                wa = i;
                woa = wo;
            }
        }
    }
    r.ra = wa >= 0 ? 2 + wa : 0;
    r.mva = wa >= 0 ? c.off - woa : c.off;
    r.rb = 1;
    r.mvb = c.off - c.h;
    if (c.kind == 0 && c.off - c.h < -MVL && n > 0) {
        for (int i = 0; i < n; ++i) {
            if (!c.wp_valid[i]) continue;
            int wo = c.wp_off[i];
            if (wo > c.off && c.off - wo >= -MVL) {   /* FIRST match (:584) */
                r.rb = 2 + i;
                r.mvb = c.off - wo;
                break;
            }
        }
    }
    return r;
}

/* median3, h264_writer.c:362-367 -- returns c when c < min(a, b) */
__device__ inline int median3(int a, int b, int c)
{
    if (a > b) { int t = a; a = b; b = t; }
    if (b > c) b = c;
    if (a > b) a = b;
    return b > a ? b : a;
}

/* get_mv_prediction, h264_writer.c:369-432, for a row-uniform MV field:
 * left neighbour = same row (ref, mvy); above / above-right / above-left
 * = row above (aref, amvy).  Every mv_x in the field is 0. */
__device__ inline void predict(int x, int y, int mbw, int ref, int mvy, int aref, int amvy,
                               int &px, int &py)
{
    bool avA = x > 0;
    bool avB = y > 0;
    bool avC = y > 0 && (x + 1 < mbw || x > 0);
    bool mA = avA;                       /* left always has the same ref */
    bool mB = avB && aref == ref;
    bool mC = avC && aref == ref;
    int na = (int)avA + (int)avB + (int)avC;
    int nm = (int)mA + (int)mB + (int)mC;
    px = 0;
    if (na == 0) {
        py = 0;
    } else if (na == 1) {
        if (avA) py = mA ? mvy : 0;
        else if (avB) py = mB ? amvy : 0;
        else py = mC ? amvy : 0;
    } else if (nm == 1) {
        py = mA ? mvy : (mB ? amvy : amvy);
    } else {
        py = median3(avA ? mvy : 0, avB ? amvy : 0, avC ? amvy : 0);
    }
}

/* mb_skip_run ue(0) (:630) + write_p16x16_mb (:434-453) */
template <class S>
__device__ inline void put_mb(S &s, int ref, int dx, int dy, int nrefs)
{
    s.put(1, 1);                         /* mb_skip_run = 0 */
    s.put(1, 1);                         /* mb_type P_L0_16x16 */
    if (nrefs == 2) s.put((uint32_t)(1 - (ref & 1)), 1);
    else if (nrefs > 2) put_ue(s, (uint32_t)ref);
    put_se(s, dx);
    put_se(s, dy);
    s.put(1, 1);                         /* coded_block_pattern = 0 */
}

__device__ inline uint8_t nal_header_byte(int kind)
{
    /* scroll: NAL_REF_IDC_NONE (:658); waypoint: NAL_REF_IDC_HIGH (:768); type 1 */
    return (uint8_t)(((kind == 1 ? 2 : 0) << 5) | 1);
}

/* ---------------------------------------------------------------------- */
/* run list construction                                                   */
/* ---------------------------------------------------------------------- */
__device__ inline void fill_pattern(uint32_t *p, uint64_t v, int len)
{
    uint64_t r = v;
    for (int rl = len; rl < 64; rl <<= 1) r |= r >> rl;
    p[0] = (uint32_t)(r >> 32);
    p[1] = (uint32_t)r;
}

/* bits [64, 96) of the repetition: the 64-bit pattern at phase 64 mod len
 * (< 32 for every len <= 64) */
__device__ inline uint32_t pattern_word2(uint32_t p0, uint32_t p1, uint32_t m64)
{
    return m64 ? __builtin_amdgcn_alignbit(p0, p1, 32 - m64) : p0;
}

template <bool CHECK>
struct RunAcc {
    Lay *L;
    int n;
    uint64_t last_v;
    int last_len;
    uint64_t pos;        /* NAL bit position */
    bool over;
    ZR *zr;
    __device__ inline void append(uint64_t v, int len, uint64_t rep)
    {
        if (rep == 0) return;
        if (CHECK)
            zr_push(*zr, v >> (64 - len), len, rep > 0xffffffffull ? 0xffffffffu : (uint32_t)rep);
        uint64_t end = pos + (uint64_t)len * rep;
        if (n > 0 && last_len == len && last_v == v) {
            if (L && !over) L->run_end[n - 1] = (uint32_t)end;
        } else if (n == RUNS_MAX) {
            over = true;
        } else {
            if (L) {
                L->len[n] = (uint8_t)len;
                L->run_end[n] = (uint32_t)end;
                fill_pattern(L->pat[n], v, len);
            }
            n++;
            last_v = v;
            last_len = len;
        }
        pos = end;
        if (pos >= 0x7fffffffull) over = true;
    }
};

/* codeword of MB (x, y) of a row group */
__device__ inline CodeSink mb_code(int x, int y, int mbw, int ref, int mv4, int aref, int amv4,
                                   int nrefs)
{
    int px, py;
    predict(x, y, mbw, ref, mv4, aref, amv4, px, py);
    CodeSink cs{0, 0, false};
    put_mb(cs, ref, 0 - px, mv4 - py, nrefs);
    return cs;
}

/* rows [y, y+count) of one class: all have region cur, row above region abv */
template <class RA>
__device__ inline bool emit_group(RA &ra, int mbw, int nrefs, int y, int count,
                                  int ref, int mv4, int aref, int amv4)
{
    if (count <= 0) return true;
    CodeSink F = mb_code(0, y, mbw, ref, mv4, aref, amv4, nrefs);
    CodeSink M = F, Lc = F;
    if (mbw >= 3) M = mb_code(1, y, mbw, ref, mv4, aref, amv4, nrefs);
    if (mbw >= 2) Lc = mb_code(mbw - 1, y, mbw, ref, mv4, aref, amv4, nrefs);
    if (F.over || M.over || Lc.over) return false;
    if (count == 1) {
        ra.append(F.v, F.len, 1);
        if (mbw >= 3) ra.append(M.v, M.len, (uint64_t)(mbw - 2));
        if (mbw >= 2) ra.append(Lc.v, Lc.len, 1);
        return true;
    }
    /* repeated rows: only uniform rows compact (always the case, see DESIGN) */
    bool uni = (F.len == M.len && F.v == M.v && F.len == Lc.len && F.v == Lc.v);
    if (!uni) return false;
    ra.append(F.v, F.len, (uint64_t)mbw * (uint64_t)count);
    return true;
}

/* Build (STORE) or measure the run layout of one NAL.  Returns true when the
 * fast path applies (no EP possible, codes <= 64 bits, <= RUNS_MAX runs,
 * header <= HDR_WORDS); *size = NAL bytes in that case.  The decision is the
 * same in the plan and emit kernels (it never depends on STORE). */
template <bool STORE, bool CHECK = true>
__device__ bool build_nal(const NalCtx &c, Lay *L, uint32_t *size)
{
    HdrSink<STORE, CHECK> hs{STORE ? L->hdr : nullptr, 0, false, false, {0, 0}, 0};
    hs.put(0, 24);                               /* 00 00 00 01 (nal.c:59-64) */
    hs.put(1, 8);
    hs.put(nal_header_byte(c.kind), 8);
    hs.track = true;
    emit_slice_header(hs, c);
    hs.finish();
    bool ok = !hs.over;
    ZR zr = hs.zr;
    RunAcc<CHECK> ra{STORE ? L : nullptr, 0, 0, 0, (uint64_t)hs.len, false, &zr};

    Regions rg = regions(c);
    int mbw = c.w / 16, mbh = c.h / 16;
    int a_end = (c.h - c.off) / 16;              /* :555 (C truncation) */
    if (ok && mbw > 0 && mbh > 0) {
        int nrefs = 2 + c.nwp;
        int rA = rg.ra, mA = rg.mva * 4, rB = rg.rb, mB = rg.mvb * 4;
        bool row0A = 0 < a_end;
        ok = ok && emit_group(ra, mbw, nrefs, 0, 1, row0A ? rA : rB, row0A ? mA : mB, 0, 0);
        if (mbh > 1) {
            int nAA = max(0, min(a_end, mbh) - 1);
            bool bnd = a_end >= 1 && a_end <= mbh - 1;
            int nBB = mbh - 1 - nAA - (bnd ? 1 : 0);
            ok = ok && emit_group(ra, mbw, nrefs, 1, nAA, rA, mA, rA, mA);
            if (bnd) ok = ok && emit_group(ra, mbw, nrefs, a_end, 1, rB, mB, rA, mA);
            ok = ok && emit_group(ra, mbw, nrefs, 1, nBB, rB, mB, rB, mB);
        }
    }
    ra.append(0x8000000000000000ull, 1, 1);      /* rbsp_stop_one_bit */
    ok = ok && !ra.over && (!CHECK || zr.max < EP_ZERO_RUN);
    uint64_t used = ra.pos;
    uint64_t nal_bits = (used + 7) & ~7ull;
    if (STORE && ok) {
        L->hdr_bits = (uint32_t)hs.len;
        L->used_bits = (uint32_t)used;
        L->nal_bits = (uint32_t)nal_bits;
        L->nruns = (uint32_t)ra.n;
    }
    *size = (uint32_t)(nal_bits >> 3);
    return ok;
}

/* ---------------------------------------------------------------------- */
/* random access into a NAL's bit string                                    */
/* ---------------------------------------------------------------------- */
__device__ inline uint32_t funnel(uint32_t a, uint32_t b, int sh)
{
    /* 32 bits starting sh bits into a:b (0 <= sh < 32) */
    return sh ? (a << sh) | (b >> (32 - sh)) : a;
}

__device__ inline uint32_t umod_small(uint32_t d, uint32_t len)
{
    if (d < (1u << 22)) {
        float inv = __builtin_amdgcn_rcpf((float)len);
        int32_t q = (int32_t)((float)d * inv);
        int32_t r = (int32_t)d - q * (int32_t)len;
        if (r < 0) r += (int32_t)len;
        if (r >= (int32_t)len) r -= (int32_t)len;
        return (uint32_t)r;
    }
    return d % len;
}

/* 32 bits of NAL bit string starting at bit b; zeros past used_bits */
__device__ inline uint32_t lay_bits32(const Lay *L, uint32_t b)
{
    uint32_t out = 0;
    int filled = 0;
    uint32_t used = L->used_bits;
    int r = -1;
    while (filled < 32) {
        uint32_t pos = b + (uint32_t)filled;
        if (pos >= used) break;
        uint32_t w, seg_end;
        if (pos < L->hdr_bits) {
            int k = (int)(pos >> 5);
            uint32_t nxt = (k + 1 < HDR_WORDS) ? L->hdr[k + 1] : 0u;
            w = funnel(L->hdr[k], nxt, (int)(pos & 31));
            seg_end = L->hdr_bits;
        } else {
            if (r < 0) r = 0;
            while (L->run_end[r] <= pos) r++;
            uint32_t start = r ? L->run_end[r - 1] : L->hdr_bits;
            uint32_t len = L->len[r];
            uint32_t phi = umod_small(pos - start, len);
            const uint32_t *p = L->pat[r];
            const uint32_t p2 = pattern_word2(p[0], p[1], 64u % len);
            w = phi < 32 ? funnel(p[0], p[1], (int)phi) : funnel(p[1], p2, (int)(phi - 32));
            seg_end = L->run_end[r];
        }
        uint32_t avail = seg_end - pos;
        int take = avail >= (uint32_t)(32 - filled) ? 32 - filled : (int)avail;
        if (take < 32) w &= ~(0xffffffffu >> take);
        out |= w >> filled;
        filled += take;
    }
    return out;
}


/* one byte of the tile at tile byte rel (fast NALs only) */
__device__ inline uint32_t tile_byte(const Lay *L, const int32_t *noff, int cnt, int &j,
                                     uint32_t rel)
{
    while (j + 1 < cnt && (uint32_t)noff[j + 1] <= rel) j++;
    return lay_bits32(&L[j], (rel - (uint32_t)noff[j]) * 8u) >> 24;
}


/* ---------------------------------------------------------------------- */
/* k_emit helpers: a PURE chunk (16 output bytes wholly inside one periodic */
/* run) is 4 funnel shifts of the run's 192-bit pattern expansion at phase  */
/* (bit offset into the run) mod len, the modulo by mul-high; a MIXED chunk */
/* ORs the masked pieces of every segment it meets (mixed_chunk).           */
/* ---------------------------------------------------------------------- */
__device__ inline uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

__device__ inline uint32_t mod_magic(uint32_t d, uint32_t len, uint32_t magic)
{
    uint32_t q = __umulhi(d, magic);                 /* floor(d/len) or +1 */
    int32_t r = (int32_t)(d - q * len);
    r += r < 0 ? (int32_t)len : 0;
    r -= r >= (int32_t)len ? (int32_t)len : 0;
    return (uint32_t)r;
}

__device__ inline uint32_t pat_window(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t phi)
{
    /* bits [phi, phi + 32) of the 96-bit pattern, phi < 64 */
    uint64_t hi = phi < 32 ? (((uint64_t)p0 << 32) | p1) : (((uint64_t)p1 << 32) | p2);
    return (uint32_t)(hi >> (32 - (phi & 31)));
}

/* 192-bit expansion of a run pattern: words 3..5 continue the repetition
 * (bits [96, 192)), so any 128-bit window at phase phi < 64 is 4 funnel
 * shifts of 5 consecutive words with ONE shift amount. */
__device__ inline void pattern192(uint32_t p0, uint32_t p1, uint32_t mods, uint32_t q[6])
{
    const uint32_t p2 = pattern_word2(p0, p1, mods & 255u);
    q[0] = p0;
    q[1] = p1;
    q[2] = p2;
    q[3] = pat_window(p0, p1, p2, (mods >> 8) & 255u);
    q[4] = pat_window(p0, p1, p2, (mods >> 16) & 255u);
    q[5] = pat_window(p0, p1, p2, mods >> 24);
}

/* 128 bits of a run's repetition starting at pattern phase phi (< len <= 64);
 * q = pattern192 of the run. */
__device__ inline void pure_words_phi(uint32_t phi, const uint32_t q[6], uint32_t w[4])
{
    const bool hi = phi >= 32;
    const uint32_t sh = phi & 31;
    uint32_t a[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) a[k] = hi ? q[k + 1] : q[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = sh ? __builtin_amdgcn_alignbit(a[k], a[k + 1], 32 - sh) : a[k];
}

/* 128 bits of a PURE chunk (wholly inside one periodic run) starting d bits
 * after the run's first bit; q = pattern192 of the run. */
__device__ inline void pure_words(uint32_t d, uint32_t len, uint32_t magic, const uint32_t q[6],
                                  uint32_t w[4])
{
    pure_words_phi(mod_magic(d, len, magic), q, w);      /* phase < len <= 64 */
}

/* bits [lo, hi) of a 32-bit word (MSB first), lo / hi clamped to [0, 32] */
__device__ inline uint32_t range_mask(int32_t lo, int32_t hi)
{
    lo = lo < 0 ? 0 : lo;
    hi = hi > 32 ? 32 : hi;
    if (hi <= lo) return 0u;
    const uint32_t b = hi >= 32 ? 0u : (0xffffffffu >> hi);
    return (0xffffffffu >> lo) & ~b;
}

__device__ inline int32_t clamp_bits(int64_t x)
{
    return x < -64 ? -64 : (x > 192 ? 192 : (int32_t)x);
}

/* 128 bits of the tile at tile bit x0 (x0 = 8 * (chunk byte - tile start),
 * negative before the tile start), j = the first layout that can hold a bit
 * of the chunk; noff[j] = layout j's first byte relative to the tile start
 * (negative for the previous tile's NALs), layouts j .. cnt-1 are read.  The chunk is the OR of the
 * pieces of every segment it meets -- header words, periodic runs, and the
 * same for the following NALs -- each run taken at its phase at x0 (a
 * negative offset when the run starts inside the chunk) and masked to its
 * bit range, so no per-word segment search is needed.  Bits past the last
 * NAL of the tile read as zero. */
__device__ inline void mixed_chunk(const Lay *L, const int32_t *noff, int cnt, int j, int64_t x0,
                                   const LenLut &T, uint32_t w[4])
{
    w[0] = w[1] = w[2] = w[3] = 0u;
    for (; j < cnt; ++j) {
        const int64_t nb = (int64_t)noff[j] * 8;
        if (nb >= x0 + 128) break;
        const Lay &Lj = L[j];
        const int64_t rel0 = x0 - nb;                    /* NAL bits, may be < 0 */
        if (rel0 >= (int64_t)Lj.nal_bits) continue;
        const uint32_t hb = Lj.hdr_bits;
        if (rel0 < (int64_t)hb) {
            const int32_t r0 = (int32_t)rel0;            /* (-128, 384) */
            const int32_t i0 = r0 >> 5;                  /* floor */
            const uint32_t sh = (uint32_t)r0 & 31u;
            uint32_t hw[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int32_t idx = i0 + k;
                hw[k] = (idx >= 0 && idx < HDR_WORDS) ? Lj.hdr[idx] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                w[k] |= sh ? __builtin_amdgcn_alignbit(hw[k], hw[k + 1], 32 - sh) : hw[k];
        }
        const uint32_t nr = Lj.nruns;
        uint32_t r = 0, s0 = hb;
        if (rel0 > (int64_t)hb) {           /* first run ending after rel0: independent loads */
#pragma unroll
            for (int q = 0; q < RUNS_MAX; ++q) {
                const uint32_t e = Lj.run_end[q];
                const bool past = (uint32_t)q < nr && (int64_t)e <= rel0;
                r += past ? 1u : 0u;
                s0 = past ? e : s0;
            }
        }
        for (; r < nr && (int64_t)s0 < rel0 + 128; ++r) {
            const uint32_t s1 = Lj.run_end[r];
            const uint32_t len = Lj.len[r], mag = T.magic[len - 1];
            const int64_t d = rel0 - (int64_t)s0;
            uint32_t phi;
            if (d >= 0) {
                phi = mod_magic((uint32_t)d, len, mag);
            } else {
                const uint32_t m = mod_magic((uint32_t)(-d), len, mag);
                phi = m ? len - m : 0u;
            }
            uint32_t q[6], pw[4];
            pattern192(Lj.pat[r][0], Lj.pat[r][1], T.mods[len - 1], q);
            pure_words_phi(phi, q, pw);
            const int32_t lo = clamp_bits((int64_t)s0 - rel0);
            const int32_t hi = clamp_bits((int64_t)s1 - rel0);
#pragma unroll
            for (int k = 0; k < 4; ++k) w[k] |= pw[k] & range_mask(lo - 32 * k, hi - 32 * k);
            s0 = s1;
        }
    }
}

/* pure chunk ranges of NAL j: run r covers arena bits [Aj + s0, Aj + s1);
 * its pure chunks are [ceil((Aj+s0)/128), floor((Aj+s1)/128)). */
__device__ inline void pure_range(uint64_t Aj, uint32_t s0, uint32_t s1, uint64_t &cp0,
                                  uint64_t &cp1)
{
    cp0 = (Aj + s0 + 127) >> 7;
    cp1 = (Aj + s1) >> 7;
    if (cp1 < cp0) cp1 = cp0;
}

/* ---------------------------------------------------------------------- */
/* k_emit tile plan (shared with the CPU test harness tests/hostsim).       */
/* Layout i of a tile is NAL t0 - SEAM_XB + i; the tile's own NALs are      */
/* layouts SEAM_XB .. SEAM_XB + cnt - 1; noff[i] = layout i's first byte     */
/* relative to the tile start B0.  Every 128-byte line in [line(B0),        */
/* line(B1)) is produced whole by the tile, the two seam lines included     */
/* when their neighbour bytes are available (see k_emit).                    */
/* ---------------------------------------------------------------------- */
constexpr int SEAM_XB = 2, SEAM_XA = 2;   /* neighbour layouts before / after */

struct Seams {
    bool head_full, head_rmw, tail_full;
    int hj;                 /* first layout feeding the head line          */
    int t_hi;               /* one past the last layout feeding the tail   */
    uint64_t cs, ce;        /* chunk range of the tile's single store pass */
};

/* lo / hi: valid layouts; slow_mask bit i: layout i is a serial-path NAL */
__device__ inline Seams seam_plan(uint64_t B0, uint64_t B1, int t0, int cnt, int nnal, int lo,
                                  int hi, const int32_t *noff, uint64_t slow_mask)
{
    Seams z;
    const uint64_t ls = B0 & ~127ull, le = (B1 + 127) & ~127ull;
    z.head_full = B0 == ls;
    z.head_rmw = false;
    z.tail_full = B1 == le;
    z.hj = SEAM_XB;
    z.t_hi = SEAM_XB + cnt;
    if (!z.head_full) {
        if (t0 == 0) {                          /* previous compose's bytes */
            z.head_full = z.head_rmw = true;
        } else {
            for (int i = SEAM_XB - 1; i >= lo; --i) {
                if ((slow_mask >> i) & 1ull) break;
                if ((int64_t)noff[i] <= (int64_t)ls - (int64_t)B0) {
                    z.head_full = true;
                    z.hj = i;
                    break;
                }
            }
        }
    }
    if (!z.tail_full) {
        if (t0 + cnt == nnal) {                 /* past the stream's end: zeros */
            z.tail_full = true;
        } else {
            for (int i = SEAM_XB + cnt; i < hi; ++i) {
                if ((slow_mask >> i) & 1ull) break;
                if ((int64_t)noff[i + 1] >= (int64_t)le - (int64_t)B0 ||
                    t0 - SEAM_XB + i == nnal - 1) {
                    z.tail_full = true;
                    z.t_hi = i + 1;
                    break;
                }
            }
        }
    }
    z.cs = z.head_full ? (ls >> 4) : ((B0 + 15) >> 4);
    z.ce = z.tail_full ? (le >> 4) : (B1 >> 4);
    if (z.ce < z.cs) z.ce = z.cs;
    return z;
}

/* chunks [own0, own1) whose first byte is in own NAL i (the first own NAL
 * also takes the head chunks, the last one the tail chunks) */
__device__ inline void owned_chunks(const Seams &z, uint64_t B0, const int32_t *noff, int i, int cnt,
                                    uint64_t &own0, uint64_t &own1)
{
    const uint64_t Aj = 8 * (B0 + (uint64_t)(int64_t)noff[i]);
    const uint64_t Aj1 = 8 * (B0 + (uint64_t)(int64_t)noff[i + 1]);
    own0 = i == SEAM_XB ? z.cs : (Aj + 127) >> 7;
    own1 = i == SEAM_XB + cnt - 1 ? z.ce : (Aj1 + 127) >> 7;
    if (own1 < own0) own1 = own0;
}

/* Walk the owned chunks of a fast NAL in order as entries: emit(r, c0, c1)
 * with r = run index for a PURE entry (chunks inside run r) or -1 for a
 * MIXED entry (a maximal gap between pure entries). */
template <class F>
__device__ inline void entry_walk(const Lay &Lj, uint64_t Aj, uint64_t own0, uint64_t own1, F &&emit)
{
    uint64_t prev = own0;
    uint32_t s0 = Lj.hdr_bits;
    for (uint32_t r = 0; r < Lj.nruns; ++r) {
        const uint32_t s1 = Lj.run_end[r];
        uint64_t cp0, cp1;
        pure_range(Aj, s0, s1, cp0, cp1);
        s0 = s1;
        if (cp1 <= cp0) continue;
        if (cp0 > prev) emit(-1, prev, cp0);
        emit((int)r, cp0, cp1);
        prev = cp1;
    }
    if (own1 > prev) emit(-1, prev, own1);
}

/* first layout holding a bit of chunk c (byte p = 16 c) of own NAL i */
__device__ inline uint32_t mixed_first(const Seams &z, uint64_t p, uint64_t B0, int i)
{
    return p < B0 ? (uint32_t)(z.head_rmw ? SEAM_XB : z.hj) : (uint32_t)i;
}

/* ---------------------------------------------------------------------- */
/* serial device path: exact restatement of the MB loop, any input          */
/* (long codes, emulation prevention, non-compactable fields)               */
/* ---------------------------------------------------------------------- */
struct EpCount {
    uint64_t n;
    int zeros;
    __device__ inline void byte(uint32_t v)
    {
        if (zeros >= 2 && v <= 3) {
            n++;
            zeros = 0;
        }
        n++;
        zeros = v ? 0 : zeros + 1;
    }
};

struct EpWrite {
    uint8_t *dst;
    uint64_t n;
    int zeros;
    __device__ inline void byte(uint32_t v)
    {
        if (zeros >= 2 && v <= 3) {              /* nal.c:33-38 */
            dst[n++] = 3;
            zeros = 0;
        }
        dst[n++] = (uint8_t)v;
        zeros = v ? 0 : zeros + 1;
    }
};

template <class B>
struct BitPump {
    B *b;
    uint64_t acc;
    int nacc;
    __device__ inline void put(uint32_t v, int n)
    {
        if (n <= 0) return;
        v &= low_mask(n);
        acc |= ((uint64_t)v << (64 - n)) >> nacc;
        nacc += n;
        while (nacc >= 8) {
            b->byte((uint32_t)(acc >> 56));
            acc <<= 8;
            nacc -= 8;
        }
    }
    __device__ inline void finish()
    {
        put(1, 1);                               /* bitwriter.c:103-111 */
        if (nacc) put(0, 8 - nacc);
    }
};

template <class B>
__device__ void serial_rbsp(const NalCtx &c, B &sink)
{
    BitPump<B> bp{&sink, 0, 0};
    emit_slice_header(bp, c);
    Regions rg = regions(c);
    int mbw = c.w / 16, mbh = c.h / 16;
    int a_end = (c.h - c.off) / 16;
    int nrefs = 2 + c.nwp;
    for (int y = 0; y < mbh; ++y) {
        bool curA = y < a_end, abvA = (y - 1) < a_end;
        int ref = curA ? rg.ra : rg.rb, mv4 = 4 * (curA ? rg.mva : rg.mvb);
        int aref = abvA ? rg.ra : rg.rb, amv4 = 4 * (abvA ? rg.mva : rg.mvb);
        for (int x = 0; x < mbw; ++x) {
            int px, py;
            predict(x, y, mbw, ref, mv4, aref, amv4, px, py);
            put_mb(bp, ref, 0 - px, mv4 - py, nrefs);
        }
    }
    bp.finish();
}

__device__ inline uint64_t serial_size(const NalCtx &c)
{
    EpCount ec{0, 0};
    serial_rbsp(c, ec);
    return 5 + ec.n;
}

__device__ inline void serial_write(const NalCtx &c, uint8_t *dst)
{
    dst[0] = 0; dst[1] = 0; dst[2] = 0; dst[3] = 1;
    dst[4] = nal_header_byte(c.kind);
    EpWrite ew{dst + 5, 0, 0};
    serial_rbsp(c, ew);
}

}  // namespace scroll
#endif
