/*
 * sim.cpp -- TEST-ONLY CPU harness around the product's device functions
 * (scroll_device.h).  Exposes:
 *   sim_nal():   one NAL via build_nal<true> + lay_bits32 (fast path) or the
 *                serial path, so tests can compare bytes with the oracle;
 *   sim_tile():  a sequence of NALs laid out as one k_emit tile and read back
 *                through pure_words()/mixed_chunk() at 16-byte granularity.
 */
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <vector>
#include "scroll_device.h"

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
            if (L3.run_end[r] != L.run_end[r] || L3.len[r] != L.len[r] || L3.magic[r] != L.magic[r] ||
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

/* Lay out n NALs (all fast) back to back starting at arena byte base0 and read
 * them with the k_emit chunk logic; out gets the concatenated bytes. */
long sim_tile(int w, int h, int l2f, int poct, int l2p, int dbf, int n, const int *kinds,
              const int *offs, const int *fns, const int *nwps, const int *wo, const int *wl,
              const int *wv, int base0, uint8_t *out, long cap)
{
    std::vector<Lay> L(n);
    std::vector<uint32_t> noff(n + 1);
    uint32_t pos = 0;
    for (int i = 0; i < n; ++i) {
        NalCtx c{w, h, l2f, poct, l2p, dbf, kinds[i], offs[i], fns[i], nwps[i], wo, wl, wv};
        memset(&L[i], 0, sizeof(Lay));
        uint32_t sz;
        if (!build_nal<true>(c, &L[i], &sz)) return -2;
        noff[i] = pos;
        pos += sz;
    }
    noff[n] = pos;
    if ((long)pos > cap) return -1;
    /* arena positions: tile starts at base0 (not 16-aligned in general) */
    uint64_t B0 = (uint64_t)base0, B1 = B0 + pos;
    std::vector<uint8_t> arena(B1 + 32, 0xEE);
    /* mirrors k_emit: classify owned chunks into pure / mixed, then both phases */
    const uint64_t c0 = B0 >> 4, c1 = (B1 + 15) >> 4;
    struct PE { uint32_t cb, n, j, r; };
    std::vector<PE> pes;
    std::vector<std::pair<uint32_t, int>> mxs;
    for (int lane = 0; lane < n; ++lane) {
        uint64_t Aj = 8 * (B0 + noff[lane]), Aj1 = 8 * (B0 + noff[lane + 1]);
        uint64_t own0 = lane == 0 ? c0 : (Aj + 127) >> 7;
        uint64_t own1 = lane == n - 1 ? c1 : (Aj1 + 127) >> 7;
        if (own1 < own0) own1 = own0;
        uint64_t prev = own0;
        uint32_t s0 = L[lane].hdr_bits;
        for (uint32_t r = 0; r <= L[lane].nruns; ++r) {
            uint64_t cp0 = own1, cp1 = own1;
            if (r < L[lane].nruns) {
                uint32_t s1 = L[lane].run_end[r];
                pure_range(Aj, s0, s1, cp0, cp1);
                s0 = s1;
                if (cp1 <= cp0) continue;
            }
            for (uint64_t c = prev; c < cp0; ++c) mxs.push_back({(uint32_t)(c - c0), lane});
            if (r < L[lane].nruns) pes.push_back({(uint32_t)(cp0 - c0), (uint32_t)(cp1 - cp0), (uint32_t)lane, r});
            prev = cp1;
        }
    }
    std::vector<int> owned(c1 - c0, 0);
    for (auto &e : pes) {
        const Lay &Lj = L[e.j];
        uint32_t rs0 = e.r ? Lj.run_end[e.r - 1] : Lj.hdr_bits;
        uint32_t len = Lj.len[e.r], magic = Lj.magic[e.r];
        uint64_t Arun = 8 * (B0 + noff[e.j]) + rs0;
        uint32_t q6[6];
        pattern192(Lj.pat[e.r][0], Lj.pat[e.r][1], Lj.pat[e.r][2], len, magic, q6);
        for (uint32_t k = 0; k < e.n; ++k) {
            uint64_t c = c0 + e.cb + k;
            owned[c - c0]++;
            uint32_t w[4];
            pure_words((uint32_t)((c << 7) - Arun), len, magic, q6, w);
            for (int q = 0; q < 16; ++q) arena[(c << 4) + q] = (uint8_t)(w[q >> 2] >> (24 - 8 * (q & 3)));
        }
    }
    for (auto &m : mxs) {
        uint64_t c = c0 + m.first, p = c << 4;
        owned[c - c0]++;
        uint32_t w[4];
        mixed_chunk(L.data(), noff.data(), n, m.second, ((int64_t)p - (int64_t)B0) * 8, w);
        for (int q = 0; q < 16; ++q) {
            uint64_t x = p + q;
            if (x < B0 || x >= B1) continue;
            arena[x] = (uint8_t)(w[q >> 2] >> (24 - 8 * (q & 3)));
        }
    }
    for (size_t k = 0; k < owned.size(); ++k)
        if (owned[k] != 1) return -4;                        /* every chunk exactly once */
    memcpy(out, arena.data() + B0, pos);
    return pos;
}

}  // extern "C"
