/*
 * sim.cpp -- TEST-ONLY CPU harness around the product's device functions
 * (scroll_device.h).  Exposes:
 *   sim_nal():   one NAL via build_nal<true> + lay_bits32 (fast path) or the
 *                serial path, so tests can compare bytes with the oracle;
 *   sim_tile():  a sequence of NALs laid out as one k_emit tile and read back
 *                through chunk_words()/tile_byte() at 16-byte granularity.
 */
#include <cstdio>
#include <cstdlib>
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
    for (uint64_t c = B0 >> 4; c < (B1 + 15) >> 4; ++c) {
        uint64_t p = c << 4;
        int j = 0;
        if (p >= B0 && p + 16 <= B1) {
            uint32_t wv4[4];
            chunk_words(L.data(), noff.data(), n, j, (uint32_t)(p - B0), wv4);
            for (int k = 0; k < 16; ++k) arena[p + k] = (uint8_t)(wv4[k >> 2] >> (24 - 8 * (k & 3)));
        } else {
            for (int k = 0; k < 16; ++k) {
                uint64_t q = p + k;
                if (q < B0 || q >= B1) continue;
                arena[q] = (uint8_t)tile_byte(L.data(), noff.data(), n, j, (uint32_t)(q - B0));
            }
        }
    }
    memcpy(out, arena.data() + B0, pos);
    return pos;
}

}  // extern "C"
