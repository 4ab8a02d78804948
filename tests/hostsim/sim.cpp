/*
 * sim.cpp -- TEST-ONLY CPU harness around the product's device functions
 * (scroll_device.h).  Exposes:
 *   sim_nal():   one NAL via build_nal<true> + lay_bits32 (fast path) or the
 *                serial path, so tests can compare bytes with the oracle;
 *   sim_stream(): a whole stream produced tile by tile through k_emit's
 *                shared store plan (seam_plan / owned_chunks / entry_walk /
 *                mixed_chunk / pure_words), checked for coverage and for
 *                consistent duplicate seam-line writes.
 */
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <algorithm>
#include <array>
#include <vector>
#include "scroll_device.h"
#include "dyn_device.h"

using namespace scroll;

extern "C" {

/* returns NAL size; *fast = 1 if the run-layout path applied */
long sim_nal(int w, int h, int l2f, int poct, int l2p, int dbf, int kind, int off, int fn,
             int nwp, const int *wo, const int *wl, const int *wv, int force_serial,
             uint8_t *out, long cap, int *fast, int *nruns)
{
    NalCtx c{w, h, l2f, poct, l2p, dbf, kind, off, fn, nwp, wo, wl, wv};
    Lay L;
    memset(&L, 0, sizeof(L));
    uint32_t sz = 0;
    bool ok = !force_serial && build_nal<true>(c, &L, &sz);
    uint32_t sz2 = 0;
    bool ok2 = !force_serial && build_nal<false>(c, nullptr, &sz2);
    if (ok != ok2 || (ok && sz != sz2)) return -2;          /* plan/emit disagreement */
    if (ok) {                                 /* emit's unchecked build: same layout */
        Lay L3;
        memset(&L3, 0x5a, sizeof(L3));
        uint32_t sz3 = 0;
        build_nal<true, false>(c, &L3, &sz3);
        if (sz3 != sz || memcmp(&L3, &L, offsetof(Lay, run_end)) != 0) return -5;
        for (uint32_t r = 0; r < L.nruns; ++r)
            if (L3.run_end[r] != L.run_end[r] || L3.len[r] != L.len[r] ||
                memcmp(L3.pat[r], L.pat[r], sizeof(L.pat[r])) != 0)
                return -5;
    }
    *fast = ok;
    *nruns = ok ? (int)L.nruns : -1;
    if (ok) {
        if ((long)sz > cap) return -1;
        for (uint32_t i = 0; i < sz; i += 4) {
            uint32_t v = lay_bits32(&L, i * 8);
            for (int k = 0; k < 4 && i + k < sz; ++k) out[i + k] = (uint8_t)(v >> (24 - 8 * k));
        }
        /* bits past used must read as zero and the bit-granular reader must agree */
        for (uint32_t b = 0; b + 32 <= L.nal_bits; b += 7) {
            uint32_t v = lay_bits32(&L, b);
            uint32_t ref = 0;
            for (int k = 0; k < 32; ++k) {
                uint32_t bit = (out[(b + k) >> 3] >> (7 - ((b + k) & 7))) & 1;
                ref = (ref << 1) | bit;
            }
            if (v != ref) return -3;
        }
        return sz;
    }
    uint64_t n = serial_size(c);
    if ((long)n > cap) return -1;
    serial_write(c, out);
    return (long)n;
}

/* LenLut: mod_magic(d) == d % len for len 1..64 over small, near-2^31 and
 * random d; pattern phase bytes equal the direct modulo.  0 = ok. */
int sim_check_lut(void)
{
    LenLut T;
    for (uint32_t len = 1; len <= 64; ++len) lut_entry(len, T.magic[len - 1], T.mods[len - 1]);
    uint64_t x = 88172645463325252ull;
    for (uint32_t len = 1; len <= 64; ++len) {
        const uint32_t m = T.mods[len - 1];
        if ((m & 255u) != 64u % len || ((m >> 8) & 255u) != 96u % len ||
            ((m >> 16) & 255u) != 128u % len || (m >> 24) != 160u % len)
            return -1;
        for (uint32_t k = 0; k < 300000; ++k) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            const uint32_t d = k < 100000 ? k : (k < 200000 ? 0x7fffffffu - (k - 100000)
                                                            : (uint32_t)x);
            if (mod_magic(d, len, T.magic[len - 1]) != d % len) return -2;
        }
    }
    return 0;
}

/* k_emit's store plan over a whole stream: n fast NALs laid out from arena
 * byte base0 (bytes [0, base0) hold a previous compose), tiles of `tile`
 * NALs, each produced through the shared seam_plan / owned_chunks /
 * entry_walk / mixed_chunk / pure_words code exactly as one wave does.
 * out receives arena [0, base0 + total + 128).  Returns total, or
 *  -1 capacity, -2 a NAL not on the fast path, -4 a byte written twice with
 *  different values, -6 an output byte never written. */
long sim_stream(int w, int h, int l2f, int poct, int l2p, int dbf, int n, const int *kinds,
                const int *offs, const int *fns, const int *nwps, const int *wo, const int *wl,
                const int *wv, int base0, int tile, uint8_t *out, long cap)
{
    std::vector<Lay> La(n);
    std::vector<uint64_t> at(n + 1);
    at[0] = (uint64_t)base0;
    for (int i = 0; i < n; ++i) {
        NalCtx c{w, h, l2f, poct, l2p, dbf, kinds[i], offs[i], fns[i], nwps[i], wo, wl, wv};
        memset(&La[i], 0, sizeof(Lay));
        uint32_t sz;
        if (!build_nal<true, false>(c, &La[i], &sz)) return -2;
        at[i + 1] = at[i] + sz;
    }
    const uint64_t total = at[n] - (uint64_t)base0;
    const uint64_t span = at[n] + 128;
    if ((long)span > cap) return -1;
    std::vector<uint8_t> A(span + 256, 0xEE);
    for (int i = 0; i < base0; ++i) A[i] = (uint8_t)(i * 37 + 11);
    std::vector<int> wr(A.size(), -1);
    bool clash = false;
    auto put = [&](uint64_t x, uint8_t v) {
        if (wr[x] >= 0 && wr[x] != v) clash = true;
        wr[x] = v;
        A[x] = v;
    };
    LenLut T;
    for (uint32_t len = 1; len <= 64; ++len) lut_entry(len, T.magic[len - 1], T.mods[len - 1]);
    constexpr int XB = SEAM_XB, XA = SEAM_XA;
    for (int t0 = 0; t0 < n; t0 += tile) {
        const int cnt = std::min(tile, n - t0);
        const int lo = std::max(0, XB - t0), hi = XB + cnt + std::min(XA, n - t0 - cnt);
        std::vector<Lay> L(XB + tile + XA);
        std::vector<int32_t> noff(XB + tile + XA + 1, 0);
        const uint64_t B0 = at[t0], B1 = at[t0 + cnt];
        for (int i = lo; i < hi; ++i) {
            L[i] = La[t0 - XB + i];
            noff[i] = (int32_t)((int64_t)at[t0 - XB + i] - (int64_t)B0);
        }
        noff[hi] = (int32_t)((int64_t)at[t0 - XB + hi] - (int64_t)B0);
        const Seams z = seam_plan(B0, B1, t0, cnt, n, lo, hi, noff.data(), 0);
        struct E { uint32_t vs; int r, i; uint32_t mbase; };
        std::vector<E> ent;
        std::vector<std::pair<uint64_t, uint32_t>> mxl;    /* chunk, first layout */
        for (int i = XB; i < XB + cnt; ++i) {
            uint64_t own0, own1;
            owned_chunks(z, B0, noff.data(), i, cnt, own0, own1);
            const uint64_t Aj = 8 * (B0 + (uint64_t)(int64_t)noff[i]);
            entry_walk(L[i], Aj, own0, own1, [&](int r, uint64_t c0e, uint64_t c1e) {
                ent.push_back({(uint32_t)(c0e - z.cs), r, i, (uint32_t)mxl.size()});
                if (r < 0)
                    for (uint64_t c = c0e; c < c1e; ++c) mxl.push_back({c, mixed_first(z, c << 4, B0, i)});
            });
        }
        const int mix_hi = z.tail_full ? z.t_hi : XB + cnt;
        std::vector<std::array<uint32_t, 4>> mw(mxl.size());
        for (size_t k = 0; k < mxl.size(); ++k) {
            const uint64_t p = mxl[k].first << 4;
            uint32_t ww[4];
            mixed_chunk(L.data(), noff.data(), mix_hi, (int)mxl[k].second,
                        ((int64_t)p - (int64_t)B0) * 8, T, ww);
            if (z.head_rmw && p < B0) {
                const int32_t nb = (int32_t)(B0 - p);
                for (int q = 0; q < 4; ++q) {
                    uint32_t o = 0;
                    for (int b = 0; b < 4; ++b) o = (o << 8) | A[p + 4 * q + b];
                    ww[q] |= o & range_mask(0, 8 * nb - 32 * q);
                }
            }
            for (int q = 0; q < 4; ++q) mw[k][q] = ww[q];
        }
        const uint64_t nch = z.ce - z.cs;
        size_t e = 0;
        for (uint64_t v = 0; v < nch; ++v) {
            while (e + 1 < ent.size() && ent[e + 1].vs <= v) e++;
            uint32_t ww[4];
            const E &en = ent[e];
            if (en.r < 0) {
                for (int q = 0; q < 4; ++q) ww[q] = mw[en.mbase + (v - en.vs)][q];
            } else {
                const Lay &Lj = L[en.i];
                const uint32_t rs0 = en.r ? Lj.run_end[en.r - 1] : Lj.hdr_bits;
                const uint64_t Arun = 8 * (B0 + (uint64_t)(int64_t)noff[en.i]) + rs0;
                const uint32_t K = (uint32_t)((z.cs << 7) - Arun);
                const uint32_t len = Lj.len[en.r];
                uint32_t q6[6];
                pattern192(Lj.pat[en.r][0], Lj.pat[en.r][1], T.mods[len - 1], q6);
                pure_words(K + ((uint32_t)v << 7), len, T.magic[len - 1], q6, ww);
            }
            const uint64_t p = (z.cs + v) << 4;
            for (int b = 0; b < 16; ++b) put(p + b, (uint8_t)(ww[b >> 2] >> (24 - 8 * (b & 3))));
        }
        auto partial = [&](uint64_t pc) {
            uint32_t ww[4];
            mixed_chunk(L.data(), noff.data(), XB + cnt, XB, ((int64_t)(pc << 4) - (int64_t)B0) * 8, T, ww);
            for (int b = 0; b < 16; ++b) {
                const uint64_t x = (pc << 4) + b;
                if (x >= B0 && x < B1) put(x, (uint8_t)(ww[b >> 2] >> (24 - 8 * (b & 3))));
            }
        };
        const bool ph = !z.head_full && (B0 & 15);
        const bool pt = !z.tail_full && (B1 & 15) && (B1 >> 4) >= z.cs;
        if (ph) partial(B0 >> 4);
        if (pt && !(ph && (B1 >> 4) == (B0 >> 4))) partial(B1 >> 4);
    }
    if (clash) return -4;
    for (uint64_t x = (uint64_t)base0; x < at[n]; ++x)
        if (wr[x] < 0) return -6;
    memcpy(out, A.data(), span);
    return (long)total;
}


/* ---- dynamic-rect device functions (dyn_device.h) ---------------------- */
static const dyn::Tabs g_dyn_tabs = SCROLL_DYN_TABS;
static constexpr QParams Q26 = dyn::qparams(dyn::QP_DEFAULT);   /* the oracle checks run at QP 26 */

struct HostOr {
    uint32_t *b;
    void operator()(uint32_t i, uint32_t v) const { b[i] |= v; }
};

/* one CAVLC block at bit offset `start` of a zeroed MSB-first word buffer;
 * returns the bit count (must equal the CountSink pass) or -1 on mismatch */
long sim_cavlc(const int *coef, int max, int nC, int start, uint32_t *words, int *tc_out)
{
    dyn::CountSink cs{0};
    const int tc = dyn::cavlc_block(cs, g_dyn_tabs, coef, max, nC);
    dyn::OrSink<HostOr> os{{words}, 0, 0, 0};
    os.start((uint32_t)start);
    const int tc2 = dyn::cavlc_block(os, g_dyn_tabs, coef, max, nC);
    const uint32_t end = os.wi * 32u + (uint32_t)os.fill;
    os.finish();
    *tc_out = tc;
    if (tc != tc2 || end - (uint32_t)start != cs.n) return -1;
    return (long)cs.n;
}

/* luma: reference sample via luma_row; chroma: chroma_row where it applies
 * (else the general tree); planes[ri][p] of the two pictures */
int sim_ref_sample(int w, int h, const int *wo, const int *wv, int ri, int p, int x, int y,
                   const uint8_t *const *planes, int *fast)
{
    dyn::WpTab T{wo, wv, h};
    dyn::RefPics R;
    R.w = w;
    R.h = h;
    for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 3; ++k) R.pl[i][k] = planes[3 * i + k];
    int yo;
    if (p == 0) {
        const int b = dyn::luma_row(T, ri, y, yo);
        *fast = 1;
        return R.pl[b][0][(size_t)yo * w + x];
    }
    const int b = dyn::chroma_row(T, ri, y, yo);
    if (b >= 0) {
        *fast = 1;
        return R.pl[b][p][(size_t)yo * (w / 2) + x];
    }
    *fast = 0;
    return dyn::chroma_px_any<9>(T, R, ri, p, x, y);
}

/* forward transform + quantisation of one residual block (raster order in,
 * levels at raster positions out); dc: chroma DC quantiser of one value */
void sim_fwd_quant(const int *res, int *lv)
{
    int W[16];
    dyn::fwd4x4(res, W);
    for (int k = 0; k < 16; ++k) lv[k] = dyn::quant(W[k], k, Q26);
}

int sim_quant_dc(int w) { return dyn::quant_dc(w, Q26); }

int sim_ep_count(const uint8_t *b, int n)
{
    int prev = -1, c = 0;
    for (int i = 0; i < n; ++i) {
        c += dyn::ep_insert(b[i], i - 1 - prev);
        if (b[i]) prev = i;
    }
    return c;
}

/* the kernels' split form: cavlc_body (k_dyn_row's block phase: packed
 * int8 levels -> the nC-independent bits) + coeff_token (its token phase),
 * or cavlc_dc4 for chroma DC; must equal cavlc_block bit for bit.  Blocks
 * with levels outside int8 (the kernels' levels stay within +-78) or over
 * 128 body bits take cavlc_block, as the kernels' overflow path does. */
long sim_cavlc_split(const int *coef, int max, int nC, int start, uint32_t *words, int *tc_out)
{
    static dyn::PTabs P;
    static bool init = false;
    if (!init) {
        dyn::build_ptabs(g_dyn_tabs, P, 0, 1);
        init = true;
    }
    dyn::OrSink<HostOr> os{{words}, 0, 0, 0};
    os.start((uint32_t)start);
    if (max == 4) {
        dyn::CapSink cap{0, 0, 0};
        const int c[4] = {coef[0], coef[1], coef[2], coef[3]};
        *tc_out = dyn::cavlc_dc4(cap, P, c);
        os.put_cap(cap);
        os.finish();
        return (long)cap.n;
    }
    bool fits = true;
    uint32_t pw[4] = {0, 0, 0, 0};
    for (int i = 0; i < max; ++i) {
        fits = fits && coef[i] >= -128 && coef[i] <= 127;
        pw[i >> 2] |= ((uint32_t)coef[i] & 255u) << (8 * (i & 3));
    }
    dyn::CapSink cap{0, 0, 0};
    int t1 = 0, tc = 0;
    bool ok = false;
    if (fits) tc = dyn::cavlc_body(cap, P, make_uint4(pw[0], pw[1], pw[2], pw[3]), max, t1, ok);
    if (!ok) {                                        /* the overflow path: from the levels */
        *tc_out = dyn::cavlc_block(os, g_dyn_tabs, coef, max, nC);
        const uint32_t end = os.wi * 32u + (uint32_t)os.fill;
        os.finish();
        return (long)(end - (uint32_t)start);
    }
    uint32_t tv;
    int tl;
    dyn::coeff_token(g_dyn_tabs, tc, t1, nC, tv, tl);
    os.put(tv, tl);
    os.put_cap(cap);
    os.finish();
    *tc_out = tc;
    return (long)tl + (long)cap.n;
}

/* k_dyn_row's form: cavlc_body_t (levels as bytes with one guard byte
 * before them, total_zeros + run_before from tzrb_entry) + coeff_token; must
 * equal cavlc_block bit for bit (same overflow rule as sim_cavlc_split) */
long sim_cavlc_split_t(const int *coef, int max, int nC, int start, uint32_t *words, int *tc_out)
{
    dyn::OrSink<HostOr> os{{words}, 0, 0, 0};
    os.start((uint32_t)start);
    bool fits = max != 4;
    int8_t lb[17] = {0};
    lb[0] = 1;                                        /* the guard byte: any value */
    uint32_t nz = 0;
    for (int i = 0; i < max && fits; ++i) {
        fits = coef[i] >= -128 && coef[i] <= 127;
        lb[1 + i] = (int8_t)coef[i];
        if (coef[i]) nz |= 1u << i;
    }
    dyn::CapSink cap{0, 0, 0};
    int t1 = 0, tc = 0;
    bool ok = false;
    if (fits) {
        const uint32_t e = dyn::tzrb_entry(g_dyn_tabs, nz, max);
        static constexpr dyn::LvTab lvt = dyn::make_lvt();
        tc = dyn::cavlc_body_t(cap, lb + 1, nz, e, t1, ok, lvt.e);
    }
    if (!ok) {
        *tc_out = dyn::cavlc_block(os, g_dyn_tabs, coef, max, nC);
        const uint32_t end = os.wi * 32u + (uint32_t)os.fill;
        os.finish();
        return (long)(end - (uint32_t)start);
    }
    uint32_t tv;
    int tl;
    dyn::coeff_token(g_dyn_tabs, tc, t1, nC, tv, tl);
    os.put(tv, tl);
    os.put_cap(cap);
    os.finish();
    *tc_out = tc;
    return (long)tl + (long)cap.n;
}

/* k_dyn_row's packed-pair levels (levels_pk) against fwd4x4 + quant of the
 * same residual, n random 4x4 blocks (the extremes included): 0 = all equal,
 * else 1 + the failing block */
long sim_levels_pk(long n, unsigned seed)
{
    uint64_t x = seed * 0x9e3779b97f4a7c15ull + 1;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
    for (long it = 0; it < n; ++it) {
        uint32_t a[4], p[4];
        const int kind = (int)(it % 5);
        for (int i = 0; i < 4; ++i) {
            a[i] = rnd();
            p[i] = rnd();
            if (kind == 1) { a[i] = 0xffffffffu; p[i] = 0; }          /* max residual */
            if (kind == 2) { a[i] = 0; p[i] = 0xffffffffu; }          /* min residual */
            if (kind == 3) p[i] = a[i] ^ (rnd() & 0x07070707u);      /* small residuals */
            if (kind == 4) { a[i] = (i & 1) ? 0xff00ff00u : 0x00ff00ffu; p[i] = ~a[i]; }  /* checker */
        }
        for (int luma = 0; luma < 2; ++luma) {
            int res[16], W[16];
            for (int i = 0; i < 4; ++i)
                for (int c = 0; c < 4; ++c)
                    res[4 * i + c] = (int)((a[i] >> (8 * c)) & 255u) - (int)((p[i] >> (8 * c)) & 255u);
            dyn::fwd4x4(res, W);
            uint32_t want[4] = {0, 0, 0, 0};
            for (int k2 = luma ? 0 : 1; k2 < 16; ++k2) {
                const int v = dyn::quant(W[dyn::ZZ[k2]], dyn::ZZ[k2], Q26), o = luma ? k2 : k2 - 1;
                want[o >> 2] |= ((uint32_t)v & 255u) << (8 * (o & 3));
            }
            uint32_t got[4] = {0x5a5a5a5au, 0x5a5a5a5au, 0x5a5a5a5au, 0x5a5a5a5au};
            int w0 = 0;
            if (luma) dyn::levels_pk<true>(a, p, got, w0, Q26);
            else dyn::levels_pk<false>(a, p, got, w0, Q26);
            if (std::memcmp(want, got, sizeof want) != 0 || w0 != W[0]) return 1 + it;
        }
    }
    return 0;
}

/* tzrb_entry's longest code over every mask (luma 16, chroma AC 15) */
int sim_tzrb_maxlen(int max)
{
    int mx = 0;
    for (uint32_t nz = 0; nz < (1u << max); ++nz) {
        const uint32_t e = dyn::tzrb_entry(g_dyn_tabs, nz, max);
        mx = std::max(mx, 31 - __builtin_ctz(e));
    }
    return mx;
}

/* the compile-time packed tables the kernels copy (make_ptabs) equal the
 * runtime packing (build_ptabs): 1 if identical */
int sim_ptabs_match(void)
{
    dyn::PTabs a, b;
    std::memset(&a, 0xa5, sizeof a);
    dyn::build_ptabs(g_dyn_tabs, a, 0, 1);
    constexpr dyn::Tabs kt = SCROLL_DYN_TABS;
    constexpr dyn::PTabs kp = dyn::make_ptabs(kt);
    b = kp;
    return std::memcmp(a.ct, b.ct, sizeof a.ct) == 0 && std::memcmp(a.tz, b.tz, sizeof a.tz) == 0 &&
           std::memcmp(a.tzdc, b.tzdc, sizeof a.tzdc) == 0 && std::memcmp(a.rb, b.rb, sizeof a.rb) == 0;
}

long sim_cavlc_dc4(const int *coef, int start, uint32_t *words, int *tc_out)
{
    static dyn::PTabs P;
    static bool init = false;
    if (!init) {
        dyn::build_ptabs(g_dyn_tabs, P, 0, 1);
        init = true;
    }
    dyn::CapSink cap{0, 0, 0};
    int c[4] = {coef[0], coef[1], coef[2], coef[3]};
    *tc_out = dyn::cavlc_dc4(cap, P, c);
    dyn::OrSink<HostOr> os{{words}, 0, 0, 0};
    os.start((uint32_t)start);
    os.put_cap(cap);
    os.finish();
    return (long)cap.n;
}

}  // extern "C"
