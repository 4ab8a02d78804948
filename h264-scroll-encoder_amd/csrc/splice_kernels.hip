/*
 * splice_kernels.hip -- MI355X (gfx950) kernels of the pre-encoded MB splice
 * (design only in the reference:
 * docs/MASTER_DESIGN.md:39-40,142-146,166-171 -- "transplant macroblock
 * payloads while rewriting addresses").  An external P slice coded for a
 * w x h MB picture (a conventional "dynamic encoder" ran on the rect) lands
 * in the rect of a composed scroll frame.  Bits: oracle/splice_oracle.c;
 * tests/test_gpu_splice.py checks them bit-exact.
 *
 *   k_splice_parse   one wave per spliced frame (a CAVLC slice is a
 *                    sequential bit string, so the parse is wave-uniform with
 *                    lane-parallel VLC table matching): emulation
 *                    prevention removed into the RBSP word pool, slice
 *                    header checked against the stream's SPS/PPS, then per
 *                    MB its motion (P_Skip 8.4.1.1 / median 8.4.1.3 in the
 *                    external picture), cbp, rebased mb_qp_delta and, per
 *                    residual block, (TotalCoeff, TrailingOnes) and where
 *                    the nC-independent rest of the block sits in the RBSP.
 *                    Runs once per change of the spliced slices.
 *   k_splice_stage   one workgroup per spliced scroll NAL, the UI-hint
 *                    staging (k_hint_stage) with variable-length MBs: a
 *                    counting sweep sizes every MB (head + re-contexted
 *                    coeff_tokens + copied block bodies), the NAL is zeroed,
 *                    a writing sweep ORs each MB's bits at its scanned
 *                    offset (block bodies funnel-shifted out of the RBSP),
 *                    then the emulation-prevention positions are recorded.
 *                    The emit kernels take the staged NAL from there.
 * Roofline: both are latency / issue bound and move only the slices' bytes;
 * the splice is not the benchmarked path.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>

#include "dyn_device.h"
#include "hint_device.h"
#include "splice_engine.h"
#include "stage_util.h"

using namespace scroll;
using namespace scroll::dyn;
using namespace scroll::stage;
using namespace scroll::hint;

namespace {

__constant__ Tabs SPT = SCROLL_DYN_TABS;

constexpr int RING = 512;               /* MB motion ring: this window + the row above */
static_assert(RING >= DT + 240 + 1, "the row above a window stays in the ring");

/* ------------------------------------------------------------------------ */
/* k_splice_parse                                                            */
/* ------------------------------------------------------------------------ */
__device__ inline int nc2(int nA, int nB)
{
    return nA >= 0 && nB >= 0 ? (nA + nB + 1) >> 1 : (nA >= 0 ? nA : (nB >= 0 ? nB : 0));
}

/* nC of piece i (luma raster 0..15, chroma AC 18..25) of an MB with
 * TotalCoeffs cur; left / top: the neighbour MBs' (nullptr: unavailable) */
template <class P>
__device__ inline int piece_nc(int i, const uint8_t *cur, P left, P top)
{
    if (i < 16) {
        const int bx = i & 3, by = i >> 2;
        return nc2(bx ? cur[i - 1] : (left ? (int)left[i + 3] : -1),
                   by ? cur[i - 4] : (top ? (int)top[i + 12] : -1));
    }
    const int k = (i - 18) & 3, bx = k & 1, by = k >> 1;
    return nc2(bx ? cur[i - 1] : (left ? (int)left[i + 1] : -1),
               by ? cur[i - 2] : (top ? (int)top[i + 2] : -1));
}

__device__ inline int blk_raster16(int blk)       /* luma4x4BlkIdx -> raster */
{
    const int q8 = blk >> 2, q4 = blk & 3;
    return 4 * ((q8 >> 1) * 2 + (q4 >> 1)) + (q8 & 1) * 2 + (q4 & 1);
}

/* the (sub-)partitions of an MB partitioned `part` (1 16x8, 2 8x16, 3
 * P_8x8 with sub_mb_types `sub`) in decoding order: f(bx, by, bw, bh,
 * mbPartIdx), 4x4-block units (Tables 7-13, 7-17) */
template <class Fn>
__device__ __attribute__((always_inline)) inline void for_parts(int part, uint32_t sub, Fn &&f)
{
    /* one call site of f: the geometry is computed per step (an unrolled
     * switch would inline f dozens of times) */
    const int n8 = part == 3 ? 4 : 2;
#pragma unroll 1
    for (int i = 0; i < n8; ++i) {
        const int st = part == 3 ? (int)((sub >> (2 * i)) & 3u) : 0;
        const int ns = st == 0 ? 1 : (st == 3 ? 4 : 2);
#pragma unroll 1
        for (int k = 0; k < ns; ++k) {
            int bx, by, bw, bh;
            if (part == 1) {
                bx = 0, by = 2 * i, bw = 4, bh = 2;
            } else if (part == 2) {
                bx = 2 * i, by = 0, bw = 2, bh = 4;
            } else {
                const int sx = (i & 1) * 2, sy = (i >> 1) * 2;
                bw = st == 0 || st == 1 ? 2 : 1;
                bh = st == 0 || st == 2 ? 2 : 1;
                bx = sx + (st == 2 ? k : (st == 3 ? (k & 1) : 0));
                by = sy + (st == 1 ? k : (st == 3 ? (k >> 1) : 0));
            }
            f(bx, by, bw, bh, i);
        }
    }
}

/* 4x4 blocks of a (sub-)partition as a mask (bit 4 y + x) */
__device__ inline uint32_t part_mask(int bx, int by, int bw, int bh)
{
    const uint32_t row = ((1u << bw) - 1u) << bx;
    uint32_t m = 0;
    for (int j = 0; j < bh; ++j) m |= row << (4 * (by + j));
    return m;
}

/* 8.4.1.3 for (sub-)partition mbPartIdx mp of an MB partitioned `part`,
 * neighbours nb(cx, cy) relative to the MB (6.4.11.7: C, else D) */
template <class NB>
__device__ __attribute__((always_inline)) inline void predict_part(int part, int mp, int bx, int by, int bw,
                                                                   int ref, NB &&nb, int &px, int &py)
{
    const Mv A = nb(bx - 1, by), B = nb(bx, by - 1);
    Mv C = nb(bx + bw, by - 1);
    if (C.ref == -1) C = nb(bx - 1, by - 1);            /* unavailable (an intra C is available) */
    const Mv d = part == 1 ? (mp ? A : B) : (mp ? C : A);
    if (part != 3 && d.ref == ref) {
        px = d.mx;
        py = d.my;
        return;
    }
    predict_spec(A, B, C, ref, px, py);
}

/* motion of a 4x4 block packed as mv x | y << 16 (quarter pels, |mv| <= 2^14) */
__device__ inline uint32_t pk_mv(int mx, int my) { return (uint32_t)(mx & 0xffff) | (uint32_t)my << 16; }
__device__ inline Mv unpk_mv(int ref, uint32_t v)
{
    return Mv{ref, (int)(int16_t)(v & 0xffffu), (int)(int16_t)(v >> 16)};
}

/* One wave parses one slice.  The slice is a sequential bit string, so the
 * parse itself is wave-uniform (scalar values, no divergence): the bit window
 * is 64 RBSP words held one per lane (readlane at the uniform bit position),
 * every VLC is matched by all lanes at once (lane e tests table entry e,
 * ballot), lane j keeps piece j's record fields, and the neighbour context
 * (motion of the two rows above, TotalCoeffs of the row above) sits in LDS. */
constexpr int PARSE_MAXW = 240;          /* external picture width limit (MBs) */

/* wave-uniform value to a scalar register */
__device__ inline uint32_t U(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
/* keep a (wave-uniform) value in a vector register: its arithmetic then runs
 * on the SIMD's VALU, of which a CU has four, instead of the CU's one SALU
 * that 16 parsing waves would otherwise queue on (and whose registers they
 * would run out of) */
template <class T>
__device__ inline void vpin(T &v)
{
    asm("" : "+v"(v));
}

/* The bit reader keeps the next 33..64 bits of the slice in a 64-bit vector
 * register pair (MSB-aligned; every lane holds the same value): a peek is a
 * shift, a read of up to 32 bits one 64-bit shift, and a word enters from the
 * window -- 64 RBSP words held one per lane, read by one v_readlane -- once
 * per 32 bits consumed.  Branches test readfirstlane'd values (uniform). */
struct SRd {
    const uint32_t *w;
    uint32_t nw, nbits;                  /* words, bits                               */
    uint64_t buf;                        /* the next nv bits at the top (VGPR)        */
    uint32_t nv, p;                      /* valid bits (>= 33 between reads), bits consumed (VGPR) */
    uint32_t wk, base, win;              /* next word; window: word base + lane       */
    bool bad;                            /* ue() without a 1 bit; p > nbits is checked per MB */
    /* the wait sits in the (rare) refill branch: otherwise the compiler
     * waits for vmcnt(0) before every readlane of the window -- and on gfx9
     * vmcnt also counts the record stores, so every read would wait for
     * the last MB's stores to drain */
    __device__ inline void fill(uint32_t k0)
    {
        base = k0;
        const uint32_t k = k0 + (uint32_t)(threadIdx.x & 63);
        win = k < nw ? w[k] : 0u;
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(win)::"memory");
    }
    __device__ inline uint32_t word(uint32_t k)
    {
        if (k - base >= 64u) fill(k);
        return (uint32_t)__builtin_amdgcn_readlane(win, k - base);
    }
    __device__ inline void init(const uint32_t *words, uint32_t nwords, uint32_t bits)
    {
        w = words;
        nw = nwords;
        nbits = bits;
        bad = false;
        fill(0);
        buf = (uint64_t)word(0) << 32 | word(1);
        nv = 64;
        p = 0;
        wk = 2;
        vpin(buf);
        vpin(nv);
        vpin(p);
    }
    __device__ inline uint32_t peek32() const { return (uint32_t)(buf >> 32); }
    __device__ inline uint32_t pos() const { return U(p); }
    __device__ inline void skip(uint32_t n)                  /* n <= 32 */
    {
        buf <<= n;
        nv -= n;
        p += n;
        if (U(nv) <= 32u) {
            buf |= (uint64_t)word(wk++) << (32u - nv);
            nv += 32u;
        }
    }
    __device__ inline bool over() const { return pos() > nbits; }
    __device__ inline uint32_t u(int n)                      /* 1 <= n <= 32; uniform */
    {
        const uint32_t v = U((uint32_t)(buf >> (64 - n)));
        skip((uint32_t)n);
        return v;
    }
    __device__ inline uint32_t ue()                          /* uniform */
    {
        const uint32_t x = peek32();
        const int z = (int)U((uint32_t)__clz((int)x));       /* 32 for x == 0 */
        if (z >= 32) {
            bad = true;
            return 0;
        }
        if (z < 16) {                    /* the whole code in x */
            const uint32_t v = U((x >> (31 - 2 * z)) - 1u);
            skip((uint32_t)(2 * z + 1));
            return v;
        }
        skip((uint32_t)z);
        return u(z + 1) - 1u;
    }
    __device__ inline int32_t se()
    {
        const uint32_t k = ue();
        return (k & 1u) ? (int32_t)((k + 1u) >> 1) : -(int32_t)(k >> 1);
    }
};

/* The CAVLC tables as v_readlane lookups indexed by the code's leading
 * zeros and the bits after its first 1 (Tables 9-5, 9-7/9-8, 9-9a, 9-10
 * have at most 3 / 2 such bits per leading-zero count), built per lane at
 * the kernel start from the coder's tables:
 *   ct[c]      coeff_token, class c (nC 0-1, 2-3, 4-7, -1): index lz * 8 +
 *              3 bits, 16-bit entries (lane i: i | i + 64), len << 8 | tc << 2 | t1
 *   tz0..2     total_zeros: (tc - 1) * 40 + min(lz, 9) * 4 + 2 bits, bytes
 *              (lane i byte j: index 256 v + 64 j + i), len << 4 | total_zeros
 *   tzd        chroma DC total_zeros: (tc - 1) * 16 + min(lz, 3) * 4 + 2 bits
 *   rb0, rb1   run_before: (min(zerosLeft, 7) - 1) * 48 + min(lz, 11) * 4 + 2 bits
 *   cbp        coded_block_pattern of codeNum lane (inter, Table 9-4)
 * (0: no code) */
struct LaneTabs {
    uint32_t ct0, ct1, ct2, ct3;
    uint32_t tz0, tz1, tz2, tzd, rb0, rb1;
    uint32_t cbp;
};

/* the 16-bit pattern `lz` zeros, a 1, then the top `nb` bits of n */
__device__ inline uint32_t vlc_pattern(int lz, uint32_t n, int nb)
{
    const int sh = 15 - lz - nb;
    return (1u << (15 - lz)) | (sh >= 0 ? n << sh : n >> -sh);
}

/* the entry (index) of the code among `cnt` (len, bits) that starts pattern x */
__device__ inline int vlc_find(uint32_t x, const uint8_t *len, const uint8_t *bits, int cnt)
{
    int e = -1;
    for (int i = 0; i < cnt; ++i) {
        const int l = len[i];
        if (l && e < 0 && (x >> (16 - l)) == bits[i]) e = i;
    }
    return e;
}

__device__ inline LaneTabs lane_tabs()
{
    const int lane = threadIdx.x & 63;
    LaneTabs T;
    auto ct = [&](int c) {
        uint32_t v = 0;
        for (int h = 0; h < 2; ++h) {
            const int idx = lane + 64 * h, lz = idx >> 3;
            if (lz > 15) continue;
            const uint32_t x = vlc_pattern(lz, (uint32_t)(idx & 7), 3);
            const int e = c < 3 ? vlc_find(x, SPT.ct_len[c], SPT.ct_bits[c], 68)
                                : vlc_find(x, SPT.ctdc_len, SPT.ctdc_bits, 20);
            if (e >= 0) {
                const int l = c < 3 ? SPT.ct_len[c][e] : SPT.ctdc_len[e];
                v |= (uint32_t)(l << 8 | (e >> 2) << 2 | (e & 3)) << (16 * h);
            }
        }
        return v;
    };
    T.ct0 = ct(0);
    T.ct1 = ct(1);
    T.ct2 = ct(2);
    T.ct3 = ct(3);
    auto bytes = [&](int v, auto entry) {         /* the 4 byte entries of lane, register v */
        uint32_t r = 0;
        for (int j = 0; j < 4; ++j) r |= (uint32_t)entry(256 * v + 64 * j + lane) << (8 * j);
        return r;
    };
    auto tz = [&](int idx) -> uint32_t {
        const int tc = idx / 40 + 1, q = idx % 40, lz = q >> 2;
        if (tc > 15) return 0u;
        const int e = vlc_find(vlc_pattern(lz, (uint32_t)(q & 3), 2), SPT.tz_len[tc - 1], SPT.tz_bits[tc - 1],
                               17 - tc < 16 ? 17 - tc : 16);
        return e < 0 ? 0u : (uint32_t)(SPT.tz_len[tc - 1][e] << 4 | e);
    };
    T.tz0 = bytes(0, tz);
    T.tz1 = bytes(1, tz);
    T.tz2 = bytes(2, tz);
    auto tzd = [&](int idx) -> uint32_t {
        const int tc = idx / 16 + 1, q = idx % 16, lz = q >> 2;
        if (tc > 3) return 0u;
        const int e = vlc_find(vlc_pattern(lz, (uint32_t)(q & 3), 2), SPT.tzdc_len[tc - 1], SPT.tzdc_bits[tc - 1],
                               5 - tc);
        return e < 0 ? 0u : (uint32_t)(SPT.tzdc_len[tc - 1][e] << 4 | e);
    };
    T.tzd = bytes(0, tzd);
    auto rb = [&](int idx) -> uint32_t {
        const int zl = idx / 48 + 1, q = idx % 48, lz = q >> 2;
        if (zl > 7) return 0u;
        const int e = vlc_find(vlc_pattern(lz, (uint32_t)(q & 3), 2), SPT.rb_len[zl - 1], SPT.rb_bits[zl - 1],
                               zl < 7 ? zl + 1 : 15);
        return e < 0 ? 0u : (uint32_t)(SPT.rb_len[zl - 1][e] << 4 | e);
    };
    T.rb0 = bytes(0, rb);
    T.rb1 = bytes(1, rb);
    uint32_t cb = 0xffu;
    for (int k = 0; k < 48; ++k)
        if (SPT.cbp_code[k] == (uint8_t)lane) cb = (uint32_t)k;
    T.cbp = cb;
    return T;
}

/* byte entry `idx` of a byte table spread over registers v0, v1, v2 */
__device__ inline uint32_t tab_byte(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t idx)
{
    const uint32_t v = idx < 256u ? v0 : (idx < 512u ? v1 : v2);
    return ((uint32_t)__builtin_amdgcn_readlane(v, idx & 63u) >> (8u * ((idx >> 6) & 3u))) & 255u;
}

/* leading zeros of the 32-bit peek, and the `nb` bits after its first 1
 * with the count clamped to lzmax (the bits then belong to no code) */
__device__ inline uint32_t lz_index(uint32_t x, int lzmax, int nb)
{
    const int lz = x ? __clz((int)x) : 32;
    const int l = lz < lzmax ? lz : lzmax;
    return (uint32_t)l << nb | ((x << (l + 1)) >> (32 - nb));
}

/* coeff_token (9.2.1) */
__device__ __attribute__((always_inline)) inline bool wrd_token(SRd &r, const LaneTabs &T, int nC, int &tc, int &t1)
{
    if (nC >= 8) {
        const uint32_t c = r.u(6);
        if (c == 3u) {
            tc = t1 = 0;
            return true;
        }
        tc = (int)(c >> 2) + 1;
        t1 = (int)(c & 3u);
        return t1 <= tc;
    }
    /* leading zeros and the 3 bits after the first 1, one readfirstlane */
    const uint32_t x = r.peek32();
    const uint32_t lzv = (uint32_t)__clz((int)x);            /* 32 for x == 0 */
    uint32_t idx = U(min(lzv, 16u) << 3 | ((x << (min(lzv, 15u) + 1u)) >> 29));
    if (idx >= 128u) {                   /* only chroma DC has an all-zero code ("0000000") */
        if (nC != -1) return false;
        idx = 120u;
    }
    const uint32_t v = nC == -1 ? T.ct3 : (nC < 2 ? T.ct0 : (nC < 4 ? T.ct1 : T.ct2));
    const uint32_t e = ((uint32_t)__builtin_amdgcn_readlane(v, idx & 63u) >> (idx & 64u ? 16 : 0)) & 0xffffu;
    if (!e) return false;
    r.skip(e >> 8);
    tc = (int)((e >> 2) & 31u);
    t1 = (int)(e & 3u);
    return true;
}

/* the body of a block (9.2.2-9.2.4), consumed, not kept: the levels are
 * vector arithmetic on the buffer, total_zeros / run_before table lookups */
__device__ __attribute__((always_inline)) inline bool wrd_body(SRd &r, const LaneTabs &T, int tc, int t1, int maxc)
{
    if (tc == 0) return true;
    r.skip((uint32_t)t1);
    uint32_t sl = (tc > 10 && t1 < 3) ? 1u : 0u, err = 0;
    vpin(sl);
    for (int k = t1; k < tc; ++k) {
        const uint32_t x = r.peek32();
        const uint32_t prefix = min((uint32_t)__clz((int)x), 16u);
        err |= prefix > 15u;
        uint32_t ssize = sl;
        ssize = prefix == 14u && sl == 0u ? 4u : ssize;
        ssize = prefix >= 15u ? 12u : ssize;
        /* level_suffix: the ssize bits after the prefix's 1 (<= 28 bits in all) */
        const uint32_t suf = (uint32_t)(((uint64_t)(x << min(prefix + 1u, 31u))) >> (32u - ssize));
        r.skip(min(prefix + 1u + ssize, 32u));
        uint32_t code = (min(prefix, 15u) << sl) + suf;
        code += prefix >= 15u && sl == 0u ? 15u : 0u;
        code += k == t1 && t1 < 3 ? 2u : 0u;
        const uint32_t a = (code + 2u) >> 1;                 /* |level| */
        sl = sl == 0u ? 1u : sl;
        sl += a > (3u << (sl - 1u)) && sl < 6u ? 1u : 0u;
    }
    if (U(err)) return false;                                /* level_prefix > 15: High profiles */
    uint32_t zl = 0;
    if (tc < maxc) {
        const uint32_t x = r.peek32();
        const uint32_t e = maxc == 4 ? tab_byte(T.tzd, T.tzd, T.tzd, U((uint32_t)(tc - 1) * 16u + lz_index(x, 3, 2)))
                                     : tab_byte(T.tz0, T.tz1, T.tz2, U((uint32_t)(tc - 1) * 40u + lz_index(x, 9, 2)));
        if (!e) return false;
        r.skip(e >> 4);
        zl = e & 15u;
    }
    for (int k = 0; k < tc - 1 && zl > 0u; ++k) {
        const uint32_t x = r.peek32();
        const uint32_t e = tab_byte(T.rb0, T.rb1, T.rb1, U((min(zl, 7u) - 1u) * 48u + lz_index(x, 11, 2)));
        if (!e || (e & 15u) > zl) return false;
        r.skip(e >> 4);
        zl -= e & 15u;
    }
    return true;
}

/* lane j: piece j of the MB being parsed */
struct PieceOut {
    uint32_t tc, t1, tl, len;                   /* tl: the coeff_token's bits */
};

/* one residual block: coeff_token, then the body; lane pi keeps the fields */
__device__ __attribute__((always_inline)) inline bool wrd_piece(SRd &r, const LaneTabs &T, int pi,
                                                                int nC, int maxc, PieceOut &po)
{
    int tc, t1;
    const uint32_t ps = r.p;
    if (!wrd_token(r, T, nC, tc, t1) || tc > maxc) return false;
    const uint32_t p0 = r.p;
    if (!wrd_body(r, T, tc, t1, maxc)) return false;
    if ((int)(threadIdx.x & 63) == pi) {
        po.tc = (uint32_t)tc;
        po.t1 = (uint32_t)t1;
        po.tl = p0 - ps;
        po.len = r.p - p0;
    }
    return true;
}

/* nC of piece pi from the TotalCoeffs of this MB (lanes' cur), the MB to the
 * left and the MB above (aA / aB: available -- inside the picture and the
 * slice) */
__device__ __attribute__((always_inline)) inline int nc_at(int pi, uint32_t cur, uint32_t left,
                                                           uint32_t top, bool aA, bool aB)
{
    int nA, nB;
    if (pi < 16) {
        const int bx = pi & 3, by = pi >> 2;
        nA = bx ? (int)__builtin_amdgcn_readlane(cur, pi - 1)
                : (aA ? (int)__builtin_amdgcn_readlane(left, pi + 3) : -1);
        nB = by ? (int)__builtin_amdgcn_readlane(cur, pi - 4)
                : (aB ? (int)__builtin_amdgcn_readlane(top, pi + 12) : -1);
    } else {
        const int k = (pi - 18) & 3, bx = k & 1, by = k >> 1;
        nA = bx ? (int)__builtin_amdgcn_readlane(cur, pi - 1)
                : (aA ? (int)__builtin_amdgcn_readlane(left, pi + 1) : -1);
        nB = by ? (int)__builtin_amdgcn_readlane(cur, pi - 2)
                : (aB ? (int)__builtin_amdgcn_readlane(top, pi + 2) : -1);
    }
    return nc2(nA, nB);
}

/* the pieces whose TotalCoeff an MB below reads (luma 12..15, chroma AC
 * 20, 21, 24, 25) -> slot 0..7; -1 for the others */
__device__ inline int tc_slot(int j)
{
    return j >= 12 && j < 16 ? j - 12 : ((j == 20 || j == 21) ? j - 16 : ((j == 24 || j == 25) ? j - 18 : -1));
}

/* coded_block_pattern of an Intra_4x4 MB by codeNum (Table 9-4, ChromaArrayType 1) */
__constant__ uint8_t CBP_INTRA[48] = {47, 31, 15, 0,  23, 27, 29, 30, 7,  11, 13, 14, 39, 43, 45, 46,
                                      16, 3,  5,  10, 12, 19, 21, 26, 28, 35, 37, 42, 44, 1,  2,  4,
                                      8,  17, 18, 20, 24, 6,  9,  22, 25, 32, 33, 34, 36, 40, 38, 41};

/* 7 KB: 16 parse workgroups fit a CU */
struct ParseLds {
    uint32_t rmv[PARSE_MAXW][4];         /* bottom 4x4 blocks of the MBs above (row y-1 ahead  */
    int8_t rrf[PARSE_MAXW][4];           /* of x, row y behind it): mv, ref                     */
    uint8_t tcrow[PARSE_MAXW][8];        /* their bottom pieces' TotalCoeffs (tc_slot)          */
    int8_t imrow[PARSE_MAXW][4];         /* their bottom Intra4x4PredModes (-1: not I_4x4)      */
    uint32_t cmv[16], lmv[4];            /* this MB's blocks as they decode; the left MB's right */
    int8_t crf[16], lrf[4];              /* column                                               */
    int8_t iml[4];                       /* the left MB's right-column Intra4x4PredModes         */
    uint32_t ulmv;                       /* block (3, 3) of the MB above-left (kept here, not in */
    int32_t ulrf;                        /* scalar registers: the parse is short of them)        */
};

/* k_splice_units: the NAL units of each listed frame's buffer -- Annex-B
 * units (00 00 01 / 00 00 00 01 start codes), or the whole buffer as one NAL
 * when it starts with none; trailing zero bytes of a unit belong to no unit
 * (7.4.1.2).  One workgroup per frame; the start codes are found 1,024
 * positions per pass and numbered in order by a workgroup scan.  A frame of
 * SPLICE_LANE_MIN slices or more puts its slices on the lane list. */
__global__ __launch_bounds__(DT) void k_splice_units(int n, const int32_t *__restrict__ list,
                                                     SpliceFrame *__restrict__ spf,
                                                     SpliceUnit *__restrict__ units,
                                                     int32_t *__restrict__ lanes)
{
    __shared__ uint32_t ws[NW];
    __shared__ uint32_t lbase;
    const int i = blockIdx.x, t = threadIdx.x;
    if (i >= n) return;
    SpliceFrame *F = spf + list[i];
    const uint8_t *p = F->nal;
    const uint32_t len = F->nal_len;
    const int w = F->w, h = F->h;
    const uint32_t cap = splice_unit_cap(w * h);
    SpliceUnit *UN = units + F->unit_first;
    const bool sc = len >= 3 && !p[0] && !p[1] && (p[2] == 1 || (len >= 4 && !p[2] && p[3] == 1));
    if (!sc) {
        if (t == 0) {
            UN[0].b = 0;
            UN[0].e = len;
            F->nunits = 1;
        }
        return;
    }
    uint32_t k = 0;                                   /* units so far (uniform) */
    /* aligned 16-byte lines, one per thread and pass (round 5; round 4 made
     * three byte loads per position): byte j of a line is the 01 of a start
     * code at position k - 2 when it is 01 after two zero bytes (SWAR tests
     * on whole dwords, the dword before the line loaded too) -- positions 0
     * .. len - 3 as before.  A line never leaves the pages of the bytes it
     * holds. */
    const uintptr_t pb = reinterpret_cast<uintptr_t>(p), a0 = pb & ~(uintptr_t)15, ae = pb + len;
    for (uintptr_t c = a0; c < ae; c += 16u * DT) {
        const uintptr_t A = c + 16u * (uintptr_t)t;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        uint32_t pw = 0;
        if (A < ae) {
            v = *reinterpret_cast<const uint4 *>(A);
            if (A > a0) pw = *reinterpret_cast<const uint32_t *>(A - 4);
        }
        const uint32_t W[4] = {v.x, v.y, v.z, v.w};
        const int64_t k0 = (int64_t)A - (int64_t)pb;
        uint32_t hit = 0, zp = zero_hi(pw);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t z = zero_hi(W[d]), e1 = zero_hi(W[d] ^ 0x01010101u);
            const uint32_t sc4 = e1 & __builtin_amdgcn_alignbyte(z, zp, 3u) & __builtin_amdgcn_alignbyte(z, zp, 2u);
            zp = z;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t kk = k0 + 4 * d + j;
                hit |= (((sc4 >> (8 * j + 7)) & 1u) && kk >= 2 && kk < (int64_t)len) ? 1u << (4 * d + j) : 0u;
            }
        }
        uint32_t ex, tot;
        block_excl_sum((uint32_t)__builtin_popcount(hit), ws, ex, tot);
        for (uint32_t m = hit; m; m &= m - 1u) {
            const uint32_t pos = (uint32_t)(k0 + __builtin_ctz(m) - 2), u = k + ex++;
            if (u < cap) UN[u].b = pos + 3u;
            if (u >= 1 && u - 1 < cap) UN[u - 1].e = pos;
        }
        k += tot;
    }
    if (t == 0 && k >= 1 && k - 1 < cap) UN[k - 1].e = len;
    __threadfence_block();
    __syncthreads();
    const uint32_t nu = min(k, cap);
    for (uint32_t u = (uint32_t)t; u < nu; u += DT) {
        const uint32_t b = UN[u].b;
        uint32_t e = UN[u].e;
        while (e > b && !p[e - 1]) --e;
        UN[u].e = e;
    }
    if (t == 0) {
        F->nunits = (int32_t)k;
        if (k >= SPLICE_LANE_MIN && k <= SPLICE_MAXU) lbase = (uint32_t)atomicAdd(&lanes[0], (int32_t)nu);
    }
    __syncthreads();
    if (k >= SPLICE_LANE_MIN && k <= SPLICE_MAXU)
        for (uint32_t u = (uint32_t)t; u < nu; u += DT) {
            lanes[1 + 2 * (lbase + u)] = i;
            lanes[2 + 2 * (lbase + u)] = (int32_t)u;
        }
}

/* k_splice_unesc: one wave per slice (a frame's slices dealt over the grid's
 * y waves): the NAL header checked, emulation prevention bytes out (7.4.1:
 * payload byte k >= 3 goes when it is 03 after two zero bytes), the bytes
 * MSB-first in words from word ceil(b / 4) of the frame's region on (b = the
 * unit's byte offset: a unit's RBSP never reaches the next unit's words), and
 * the position of its rbsp_stop_one_bit.  Round 5: each lane takes an aligned
 * 16-byte line of the payload per pass (one load; the two bytes before it
 * from the lane below), the removal test on whole dwords (SWAR), the kept
 * bytes through an LDS word window by a wave prefix count, whole words out;
 * the last non-zero byte comes from the pass, not from reading the words
 * back.  (Round 4: four byte loads and up to four byte stores per byte, the
 * region zeroed first: 0.34 ms per p720splicerows step.)  status:
 * SCROLL_SPLICE_ERR_NAL (a bad header), else 0 until the parse. */
__global__ __launch_bounds__(64) void k_splice_unesc(int n, const int32_t *__restrict__ list,
                                                     const SpliceFrame *__restrict__ spf,
                                                     SpliceUnit *__restrict__ units,
                                                     uint32_t *__restrict__ rbsp)
{
    /* the pass's output bytes at their MSB-first places (byte i at i ^ 3),
     * word 0 = the word carried from the pass before */
    __shared__ uint32_t ow[64 * 4 + 2];
    const int i = blockIdx.x, lane = threadIdx.x;
    if (i >= n) return;
    const SpliceFrame *F = spf + list[i];
    const int nu = min(F->nunits, (int)splice_unit_cap(F->w * F->h));
    uint8_t *ob = reinterpret_cast<uint8_t *>(ow);
    for (int u = (int)blockIdx.y; u < nu; u += (int)gridDim.y) {
        SpliceUnit *UN = units + F->unit_first + u;
        const uint32_t ub = U(UN->b);
        const uint8_t *p = F->nal + ub;
        const uint32_t len = U(UN->e) - ub;
        const uint32_t h0 = len ? U(p[0]) : 0u;
        const uint32_t w0 = (ub + 3u) >> 2;
        uint32_t nb = 0, end = 0;
        const bool ok = len >= 2 && !(h0 & 0x80) && ((h0 & 31) == 1 || (h0 & 31) == 5);   /* non-IDR / IDR slice */
        if (ok) {
            uint32_t *o = rbsp + F->rbsp_word + w0;
            /* aligned lines over payload bytes [1, len): a line never leaves
             * the pages of the bytes it holds */
            const uintptr_t pb = reinterpret_cast<uintptr_t>(p);
            const uintptr_t a0 = (pb + 1u) & ~(uintptr_t)15, ae = pb + len;
            uint32_t prevw = 0;                              /* lane 63's last dword of the pass before */
            uint32_t wout = 0, carry = 0;                    /* words written; bytes in the carried word */
            int64_t lastnz = -1;                             /* output index of the last non-zero byte */
            uint32_t lastv = 0;
            for (uintptr_t c = a0; c < ae; c += 64u * 16u) {
                const uintptr_t A = c + 16u * (uintptr_t)lane;
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (A < ae) v = *reinterpret_cast<const uint4 *>(A);
                const uint32_t W[4] = {v.x, v.y, v.z, v.w};
                uint32_t pw = __shfl_up(v.w, 1, 64);
                if (lane == 0) pw = prevw;
                prevw = __shfl(v.w, 63, 64);
                /* k = A + b - pb: kept iff 1 <= k < len and not (k >= 3, 03 after 00 00) */
                const int64_t k0 = (int64_t)A - (int64_t)pb;
                uint32_t keep = 0;
                uint32_t zp = zero_hi(pw);
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const uint32_t z = zero_hi(W[d]), e3 = zero_hi(W[d] ^ 0x03030303u);
                    const uint32_t rm = e3 & __builtin_amdgcn_alignbyte(z, zp, 3u) & __builtin_amdgcn_alignbyte(z, zp, 2u);
                    zp = z;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int64_t k = k0 + 4 * d + j;
                        const bool in = k >= 1 && k < (int64_t)len;
                        const bool gone = k >= 3 && ((rm >> (8 * j + 7)) & 1u);
                        keep |= (in && !gone) ? 1u << (4 * d + j) : 0u;
                    }
                }
                const uint32_t cnt = (uint32_t)__builtin_popcount(keep);
                const uint32_t incl = wave_incl_sum(cnt, lane);
                const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(incl, 63);
                /* the window: the carried word, then this pass's bytes */
                for (int q = lane; q < 64 * 4 + 2; q += 64)
                    if (q > 0) ow[q] = 0u;
                __syncthreads();
                uint32_t at = carry + incl - cnt;
                int64_t mylast = -1;
                uint32_t mylv = 0;
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if ((keep >> q) & 1u) {
                        const uint32_t bv = (W[q >> 2] >> (8 * (q & 3))) & 255u;
                        ob[at ^ 3u] = (uint8_t)bv;
                        if (bv) {
                            mylast = (int64_t)(4u * wout + at);
                            mylv = bv;
                        }
                        at++;
                    }
                __syncthreads();
                const uint32_t nbw = carry + tot, full = nbw >> 2;
                for (uint32_t q = (uint32_t)lane; q < full; q += 64) o[wout + q] = ow[q];
                /* the last non-zero byte so far: the highest lane that has one */
                const uint64_t bl = __ballot(mylast >= 0);
                if (bl) {
                    const int l = 63 - __builtin_clzll(bl);
                    lastnz = (int64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)mylast, l);
                    lastv = (uint32_t)__builtin_amdgcn_readlane(mylv, l);
                }
                const uint32_t cw = ow[full];                /* the partial word, carried */
                __syncthreads();
                if (lane == 0) ow[0] = cw;
                wout += full;
                carry = nbw & 3u;
                nb += tot;
                __syncthreads();
            }
            if (carry && lane == 0) o[wout] = ow[0];         /* the last word, zero-padded */
            nb = U(nb);
            if (lastnz >= 0) end = 8u * (uint32_t)lastnz + 7u - (uint32_t)__builtin_ctz(lastv);
        }
        if (lane == 0) {
            UN->w0 = w0;
            UN->nbytes = nb;
            UN->end = end;
            UN->status = ok ? SCROLL_SPLICE_OK : SCROLL_SPLICE_ERR_NAL;
            UN->bad = -1;
            UN->first = -1;
            UN->nmb = 0;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* k_splice_lanes: one slice per lane                                         */
/* ------------------------------------------------------------------------ */
/* Frames of many slices (one per MB row: the low-latency encoder mode) give
 * enough slices to parse one per LANE, each lane its own bit reader, VLC
 * lookups from LDS tables, its MB state in registers and lane-private LDS --
 * the wave then decodes 64 slices with the instructions the wave-uniform
 * parse spends on one.  A slice parsed here sees no MB above it in its own
 * slice (slices of at most w MBs: one per row, or shorter); the above-right
 * MB of its last MB can be its first MB, whose block (0, 3) it keeps.  A
 * slice that goes on past that (its MB m with m - w >= first) is handed back
 * (SPLICE_REDO) to the wave-uniform parse.  Bits and records: the same as
 * k_splice_parse's. */
constexpr int SPLICE_REDO = 99;
constexpr int LANE_WAVES = 1;
/* slices per wave: the lanes past it only build the tables.  The parse is a
 * chain of dependent loads per slice, and a frame batch has few slices per
 * SIMD (config-3 rows: 102,400 slices = 1.6 full waves per SIMD).  With the
 * records written field by field, fewer slices per wave had paid (4.40 /
 * 4.08 / 4.34 ms at 64 / 32 / 16 slices per wave): each bit-reader wait
 * also waited for the wave's scattered stores.  With the records staged in
 * LDS and written whole, 64 was best (p720splicerows, rocprofv3: 2.62-2.65 /
 * 3.33 / 3.62 ms at 64 / 32 / 16).  Round 6, with the 232-byte records (the
 * lane arrays a third smaller): 32 again, the whole step 5.06 -> 4.94 and
 * 5.07 -> 5.01 ms in two alternating A/Bs (24: 5.88, 16: 6.14, 48: 5.01;
 * profiles/r06v_splice_lpw.txt) */
#ifndef SCROLL_SPLICE_LPW
#define SCROLL_SPLICE_LPW 32
#endif
constexpr int LANE_ACTIVE = SCROLL_SPLICE_LPW;
static_assert(LANE_ACTIVE >= 1 && LANE_ACTIVE <= 64 && LANE_WAVES == 1, "k_splice_lanes: one wave, 1-64 slices");

struct LaneLds {
    uint16_t ct[4][128];                 /* coeff_token: lz 8 + 3 bits -> len << 8 | tc << 2 | t1 */
    uint8_t tz[15 * 40];                 /* total_zeros: (tc - 1) 40 + min(lz, 9) 4 + 2 bits -> len << 4 | tz */
    uint8_t tzd[3 * 16];                 /* chroma DC total_zeros */
    uint8_t rb[7 * 48];                  /* run_before: (min(zl, 7) - 1) 48 + min(lz, 11) 4 + 2 bits */
    uint8_t cbpi[48];                    /* inter codeNum -> coded_block_pattern */
    /* per active lane (LANE_ACTIVE; round 4 sized them for all 64) */
    uint8_t tcc[SPLICE_PIECES][LANE_ACTIVE];   /* the current MB's TotalCoeffs */
    uint32_t cmv[16][LANE_ACTIVE];             /* the current MB's blocks as they decode */
    int8_t crf[16][LANE_ACTIVE];
    int8_t im[16][LANE_ACTIVE];                /* the current MB's Intra4x4PredModes */
    /* the current MB's pieces -- TrailingOnes, body length and offset --
     * written to its record in whole lines when the MB is done: stored
     * field by field as parsed, 102 K lanes' open records (4.5 MB per XCD)
     * outgrew the L2 and reached HBM as partial lines, 5.5 GB of writes per
     * p720splicerows step for 0.9 GB of records */
    uint8_t t1s[SPLICE_PIECES + 1][LANE_ACTIVE];
    uint16_t bls[SPLICE_PIECES + 1][LANE_ACTIVE];   /* the record's bl words */
};

/* a lane's own bit reader: the next 33..64 bits in a 64-bit register, a
 * word loaded per 32 bits consumed (the next one already in flight) */
struct LRd {
    const uint32_t *w;
    uint32_t nw, nbits;
    uint64_t buf;
    uint32_t nv, p, wk, nxt, nxt2;
    bool bad;
    __device__ inline uint32_t word(uint32_t k) const { return k < nw ? w[k] : 0u; }
    __device__ inline void init(const uint32_t *words, uint32_t nwords, uint32_t bits)
    {
        w = words;
        nw = nwords;
        nbits = bits;
        bad = false;
        buf = (uint64_t)word(0) << 32 | word(1);
        nxt = word(2);
        nxt2 = word(3);
        nv = 64;
        p = 0;
        wk = 4;
    }
    __device__ inline uint32_t peek32() const { return (uint32_t)(buf >> 32); }
    __device__ inline void skip(uint32_t n)            /* n <= 32 */
    {
        buf <<= n;
        nv -= n;
        p += n;
        if (nv <= 32u) {
            buf |= (uint64_t)nxt << (32u - nv);
            nv += 32u;
            nxt = nxt2;
            nxt2 = word(wk++);
        }
    }
    __device__ inline bool over() const { return p > nbits; }
    __device__ inline uint32_t u(int n)                /* 1 <= n <= 32 */
    {
        const uint32_t v = (uint32_t)(buf >> (64 - n));
        skip((uint32_t)n);
        return v;
    }
    __device__ inline uint32_t ue()
    {
        const uint32_t x = peek32();
        const int z = x ? __clz((int)x) : 32;
        if (z >= 32) {
            bad = true;
            return 0;
        }
        if (z < 16) {
            const uint32_t v = (x >> (31 - 2 * z)) - 1u;
            skip((uint32_t)(2 * z + 1));
            return v;
        }
        skip((uint32_t)z);
        return u(z + 1) - 1u;
    }
    __device__ inline int32_t se()
    {
        const uint32_t k = ue();
        return (k & 1u) ? (int32_t)((k + 1u) >> 1) : -(int32_t)(k >> 1);
    }
};

__device__ inline void lane_tables(LaneLds &L, int t, int nt)
{
    for (int q = t; q < 4 * 128; q += nt) {
        const int c = q >> 7, idx = q & 127, lz = idx >> 3;
        uint16_t v = 0;
        if (lz <= 15) {
            const uint32_t x = vlc_pattern(lz, (uint32_t)(idx & 7), 3);
            const int e = c < 3 ? vlc_find(x, SPT.ct_len[c], SPT.ct_bits[c], 68) : vlc_find(x, SPT.ctdc_len, SPT.ctdc_bits, 20);
            if (e >= 0) {
                const int l = c < 3 ? SPT.ct_len[c][e] : SPT.ctdc_len[e];
                v = (uint16_t)(l << 8 | (e >> 2) << 2 | (e & 3));
            }
        }
        L.ct[c][idx] = v;
    }
    for (int q = t; q < 15 * 40; q += nt) {
        const int tc = q / 40 + 1, r = q % 40, lz = r >> 2;
        const int e = vlc_find(vlc_pattern(lz, (uint32_t)(r & 3), 2), SPT.tz_len[tc - 1], SPT.tz_bits[tc - 1],
                               17 - tc < 16 ? 17 - tc : 16);
        L.tz[q] = e < 0 ? 0 : (uint8_t)(SPT.tz_len[tc - 1][e] << 4 | e);
    }
    for (int q = t; q < 3 * 16; q += nt) {
        const int tc = q / 16 + 1, r = q % 16, lz = r >> 2;
        const int e = vlc_find(vlc_pattern(lz, (uint32_t)(r & 3), 2), SPT.tzdc_len[tc - 1], SPT.tzdc_bits[tc - 1], 5 - tc);
        L.tzd[q] = e < 0 ? 0 : (uint8_t)(SPT.tzdc_len[tc - 1][e] << 4 | e);
    }
    for (int q = t; q < 7 * 48; q += nt) {
        const int zl = q / 48 + 1, r = q % 48, lz = r >> 2;
        const int e = vlc_find(vlc_pattern(lz, (uint32_t)(r & 3), 2), SPT.rb_len[zl - 1], SPT.rb_bits[zl - 1],
                               zl < 7 ? zl + 1 : 15);
        L.rb[q] = e < 0 ? 0 : (uint8_t)(SPT.rb_len[zl - 1][e] << 4 | e);
    }
    for (int q = t; q < 48; q += nt) L.cbpi[SPT.cbp_code[q]] = (uint8_t)q;
}

/* one residual block of the lane's slice: coeff_token for nC, the body
 * (9.2.2-9.2.4) consumed; -> false on a decode failure */
__device__ inline bool lane_block(LRd &r, const LaneLds &L, int nC, int maxc, int &tc, int &t1, uint32_t &boff,
                                  uint32_t &blen)
{
    if (nC >= 8) {
        const uint32_t c = r.u(6);
        if (c == 3u) {
            tc = t1 = 0;
        } else {
            tc = (int)(c >> 2) + 1;
            t1 = (int)(c & 3u);
            if (t1 > tc) return false;
        }
    } else {
        const uint32_t x = r.peek32();
        const uint32_t lzv = x ? (uint32_t)__clz((int)x) : 32u;
        uint32_t idx = min(lzv, 16u) << 3 | ((x << (min(lzv, 15u) + 1u)) >> 29);
        if (idx >= 128u) {
            if (nC != -1) return false;
            idx = 120u;
        }
        const int c = nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
        const uint32_t e = L.ct[c][idx];
        if (!e) return false;
        r.skip(e >> 8);
        tc = (int)((e >> 2) & 31u);
        t1 = (int)(e & 3u);
    }
    if (tc > maxc) return false;
    boff = r.p;
    blen = 0;
    if (tc == 0) return true;
    r.skip((uint32_t)t1);
    uint32_t sl = (tc > 10 && t1 < 3) ? 1u : 0u;
    for (int k = t1; k < tc; ++k) {
        const uint32_t x = r.peek32();
        const uint32_t prefix = min(x ? (uint32_t)__clz((int)x) : 32u, 16u);
        if (prefix > 15u) return false;
        uint32_t ssize = sl;
        ssize = prefix == 14u && sl == 0u ? 4u : ssize;
        ssize = prefix >= 15u ? 12u : ssize;
        const uint32_t suf = ssize ? (x << (prefix + 1u)) >> (32u - ssize) : 0u;
        r.skip(prefix + 1u + ssize);
        uint32_t code = (min(prefix, 15u) << sl) + suf;
        code += prefix >= 15u && sl == 0u ? 15u : 0u;
        code += k == t1 && t1 < 3 ? 2u : 0u;
        const uint32_t a = (code + 2u) >> 1;
        sl = sl == 0u ? 1u : sl;
        sl += a > (3u << (sl - 1u)) && sl < 6u ? 1u : 0u;
    }
    uint32_t zl = 0;
    if (tc < maxc) {
        const uint32_t x = r.peek32();
        const uint32_t e = maxc == 4 ? L.tzd[(tc - 1) * 16 + lz_index(x, 3, 2)] : L.tz[(tc - 1) * 40 + lz_index(x, 9, 2)];
        if (!e) return false;
        r.skip(e >> 4);
        zl = e & 15u;
    }
    for (int k = 0; k < tc - 1 && zl > 0u; ++k) {
        const uint32_t x = r.peek32();
        const uint32_t e = L.rb[(min(zl, 7u) - 1u) * 48 + lz_index(x, 11, 2)];
        if (!e || (e & 15u) > zl) return false;
        r.skip(e >> 4);
        zl -= e & 15u;
    }
    blen = r.p - boff;
    return true;
}

/* an MB record's fixed fields in three wide stores (one lane per slice:
 * each store of the wave goes to 64 records, so field-by-field byte stores
 * had cost one store instruction per field) */
__device__ inline void store_mb_head(SpliceMbRec *R, int ref, int cbp, int qpd, int mx, int my, int skip, int part,
                                     uint32_t sub, int intra, uint32_t res_off, uint32_t res_len, uint32_t poff,
                                     uint32_t plen, uint32_t mbt, int cbp_code, int nbsame, int hasqpd, uint32_t body)
{
    uint4 *h = reinterpret_cast<uint4 *>(R);
    h[0] = make_uint4((uint32_t)(uint16_t)ref | (uint32_t)(cbp & 255) << 16 | (uint32_t)(qpd & 255) << 24, (uint32_t)mx,
                      (uint32_t)my,
                      (uint32_t)skip | (uint32_t)part << 8 | (sub & 255u) << 16 | (uint32_t)intra << 24);
    reinterpret_cast<uint2 *>(R)[9] = make_uint2(res_off, res_len);
    h[5] = make_uint4(poff, (plen & 0xffffu) | (mbt & 255u) << 16 | (uint32_t)(cbp_code & 255) << 24,
                      (uint32_t)(nbsame & 255) | (uint32_t)(hasqpd & 255) << 8 | (body & 0xffffu) << 16, 0u);
}

__global__ __launch_bounds__(64 * LANE_WAVES) void k_splice_lanes(const int32_t *__restrict__ list,
                                                                  const SpliceFrame *__restrict__ spf,
                                                                  SpliceUnit *__restrict__ units,
                                                                  const int32_t *__restrict__ lanes,
                                                                  const DevStream *__restrict__ st, int ld_fr,
                                                                  const uint32_t *__restrict__ rbsp,
                                                                  SpliceMbRec *__restrict__ recs)
{
    __shared__ LaneLds L;
    const int t = threadIdx.x, lane = t & 63;
    const int nl = lanes[0];
    const int stride = (int)gridDim.x * LANE_ACTIVE;
    if ((int)blockIdx.x * LANE_ACTIVE >= nl) return;
    lane_tables(L, t, (int)blockDim.x);
    __syncthreads();
    for (int q = t < LANE_ACTIVE ? (int)blockIdx.x * LANE_ACTIVE + t : nl; q < nl; q += stride) {
        const int idx = list[lanes[1 + 2 * q]], u = lanes[2 + 2 * q];
        const SpliceFrame *F = spf + idx;
        SpliceUnit *UN = units + F->unit_first + u;
        if (UN->status != SCROLL_SPLICE_OK) continue;            /* k_splice_unesc: not a slice NAL */
        const DevStream &S = st[idx / ld_fr];
        const int W = F->w, H = F->h, nmb = W * H;
        const int mbw_c = S.w / 16, x0c = F->x0, y0c = F->y0;
        SpliceMbRec *rec = recs + F->rec_first;
        const uint32_t w0 = UN->w0, nbytes = UN->nbytes, end = UN->end, base = 32u * w0;
        const uint32_t h0 = F->nal[UN->b];
        const int ref_idc = (int)(h0 >> 5) & 3;
        const bool idr = (h0 & 31u) == 5u;
        LRd r;
        r.init(rbsp + F->rbsp_word + w0, (nbytes + 3u) >> 2, 8u * nbytes);
        int status = SCROLL_SPLICE_ERR_HEADER, first = -1, m = 0, bad = -1;
        int fq_mb = -1, fq_qp = 0, last_qp = 0;
        int nrefs = 2;
        int qp = 0;
        bool go = true, islice = false;
        first = (int)r.ue();
        {
            const uint32_t stype = r.ue();
            islice = stype == 2 || stype == 7;
            if ((stype != 0 && stype != 5 && !islice) || (idr && !islice)) go = false;   /* P / I (IDR: I) */
        }
        if (go && r.ue() != 0) go = false;
        if (go) {
            r.skip(S.log2_mfn);
            if (idr) r.ue();                                   /* idr_pic_id */
            if (S.poc_type == 0) r.skip(S.log2_poc);
            if (!islice && r.u(1)) {
                const uint32_t k = r.ue();
                if (k > 31) go = false;
                nrefs = (int)k + 1;
            }
        }
        if (go && !islice && r.u(1)) {
            for (int k = 0;; ++k) {
                const uint32_t idc = r.ue();
                if (r.bad || r.over() || k > 32) {
                    status = SCROLL_SPLICE_ERR_SYNTAX;
                    go = false;
                    break;
                }
                if (idc == 3) break;
                if (idc != 2 || r.ue() != (uint32_t)k) {
                    go = false;
                    break;
                }
            }
        }
        if (go && ref_idc && idr) {
            r.skip(2);                                         /* no_output_of_prior_pics, long_term_reference */
        } else if (go && ref_idc && r.u(1)) {
            for (int k = 0;; ++k) {
                const uint32_t op = r.ue();
                if (r.bad || r.over() || k > 64 || op > 6) {
                    status = SCROLL_SPLICE_ERR_SYNTAX;
                    go = false;
                    break;
                }
                if (op == 0) break;
                if (op == 1 || op == 3) r.ue();
                if (op == 2) r.ue();
                if (op == 3 || op == 6) r.ue();
                if (op == 4) r.ue();
            }
        }
        if (go) {
            qp = 26 + r.se();
            if (qp < 0 || qp > 51) go = false;
        }
        if (go && S.deblock && r.ue() != 1) go = false;
        if (go) {
            status = SCROLL_SPLICE_ERR_SYNTAX;
            if (r.bad || r.over() || first < 0 || first >= nmb) go = false;
        }
        if (go) {
            const int m0 = first;
            m = m0;
            int x = m0 % W, y = m0 / W;
            int qp_c = 26;
            /* the left MB (available when aA): its right-column blocks,
             * right-column pieces' TotalCoeffs (3, 7, 11, 15, 19, 21, 23,
             * 25) and Intra4x4PredModes; the slice's first MB's block (0, 3)
             * (the above-right MB of an MB w - 1 later) */
            uint32_t lmv0 = 0, lmv1 = 0, lmv2 = 0, lmv3 = 0;
            int lrf0 = -1, lrf1 = -1, lrf2 = -1, lrf3 = -1;
            uint32_t ltc = 0, ltc2 = 0;                         /* bytes: 3 7 11 15 | 19 21 23 25 */
            uint32_t lim = 0xffffffffu;                         /* bytes: modes 3 7 11 15 (0xff: -1) */
            uint32_t fmv = 0;
            int frf = -1;
            const Mv none{-1, 0, 0};
            auto lmvq = [&](int q) { return q == 0 ? lmv0 : (q == 1 ? lmv1 : (q == 2 ? lmv2 : lmv3)); };
            auto lrfq = [&](int q) { return q == 0 ? lrf0 : (q == 1 ? lrf1 : (q == 2 ? lrf2 : lrf3)); };
            auto ltcq = [&](int pi) -> int {          /* the left MB's piece pi + 3 (luma) / pi + 1 (chroma) */
                if (pi < 16) return (int)((ltc >> (8 * (pi >> 2))) & 255u);
                const int k = (pi - 18) >> 1;          /* 18 -> 19, 20 -> 21, 22 -> 23, 24 -> 25 */
                return (int)((ltc2 >> (8 * k)) & 255u);
            };
            auto tcg = [&](int pi) -> int { return L.tcc[pi][lane]; };
            auto ncx = [&](int pi, bool aA) -> int {   /* no MB above in the slice: nB from this MB only */
                int nA, nB;
                if (pi < 16) {
                    const int bx = pi & 3, by = pi >> 2;
                    nA = bx ? tcg(pi - 1) : (aA ? ltcq(pi) : -1);
                    nB = by ? tcg(pi - 4) : -1;
                } else {
                    const int k = (pi - 18) & 3, bx = k & 1, by = k >> 1;
                    nA = bx ? tcg(pi - 1) : (aA ? ltcq(pi) : -1);
                    nB = by ? tcg(pi - 2) : -1;
                }
                return nc2(nA, nB);
            };
            auto next = [&]() {
                ++m;
                if (++x == W) {
                    x = 0;
                    ++y;
                }
            };
            bool fail = false;
            for (bool first_mb = true; !fail; first_mb = false) {
                if (r.p >= end && !first_mb) break;
                const uint32_t run = islice ? 0u : r.ue();            /* I slices: no mb_skip_run */
                if (r.bad || r.over() || run > (uint32_t)(nmb - m)) {
                    fail = true;
                    break;
                }
                for (uint32_t k = 0; k < run; ++k, next()) {           /* P_Skip */
                    if (m - W >= m0 && y > 0) {                        /* the MB above is in the slice */
                        status = SPLICE_REDO;
                        fail = true;
                        break;
                    }
                    const bool aA = x > 0 && m - 1 >= m0;
                    const int px = 0, py = 0;                          /* 8.4.1.1: the MB above unavailable */
                    SpliceMbRec *R = rec + m;
                    store_mb_head(R, 0, 0, 0, px, py, 1, 0, 0u, 0, 0u, 0u, 0u, 0u, 0u, 0, aA ? 1 : 0, 0, 0u);
                    /* the TotalCoeffs (its neighbours' nC) as 7 dword stores;
                     * t1 / blen / boff are read only for cbp's pieces */
                    uint32_t *tw = reinterpret_cast<uint32_t *>(R->tc);
#pragma unroll
                    for (int q = 0; q < (SPLICE_PIECES + 1) / 4; ++q) tw[q] = 0u;
                    const uint32_t v = pk_mv(px, py);
                    if (m == m0) {
                        fmv = v;
                        frf = 0;
                    }
                    lmv0 = lmv1 = lmv2 = lmv3 = v;
                    lrf0 = lrf1 = lrf2 = lrf3 = 0;
                    ltc = ltc2 = 0;
                    lim = 0xffffffffu;
                }
                if (fail) break;
                if (r.p >= end) {
                    if (run == 0) fail = true;
                    break;
                }
                if (m == nmb) {
                    fail = true;
                    break;
                }
                if (m - W >= m0 && y > 0) {
                    status = SPLICE_REDO;
                    fail = true;
                    break;
                }
                const bool aA = x > 0 && m - 1 >= m0, aC = y > 0 && x + 1 < W && m - W + 1 >= m0;
                const uint32_t mbt = r.ue() + (islice ? 5u : 0u);    /* an I slice's k: the P slice's 5 + k */
                if (r.bad || r.over() || mbt > 30u) {
                    fail = true;
                    break;
                }
                SpliceMbRec *R = rec + m;
                for (int j = 0; j < SPLICE_PIECES; ++j) L.tcc[j][lane] = 0;
                int cbp = 0, hasqpd = 0, qpd = 0, intra = 0, cbp_code = 0;
                uint32_t coded = 0, body = 0;                           /* pieces parsed, their body bits */
                uint32_t rs0 = 0, rsn = 0, poff = 0, plen = 0;
                uint32_t nim = 0xffffffffu;                             /* this MB's modes 3 7 11 15 */
                Mv me{0, 0, 0};
                int part = 0;
                uint32_t subv = 0;                                      /* P_8x8 sub_mb_types */
                if (mbt >= 5u) {
                    const int it = (int)mbt - 5;
                    intra = it == 0 ? 1 : (it == 25 ? 3 : 2);
                    me = Mv{SPLICE_REF_INTRA, 0, 0};
                    if (intra == 3) {
                        bool bad = false;
                        if (r.p & 7u) bad = r.u(8 - (int)(r.p & 7u)) != 0u;
                        poff = r.p;
                        for (int k = 0; k < 96; ++k) r.skip(32);
                        if (bad || r.over()) {
                            fail = true;
                            break;
                        }
                        for (int j = 0; j < SPLICE_PIECES; ++j) L.tcc[j][lane] = 16;
                    } else {
                        int m0d = -1, m3 = -1;
                        poff = r.p;
                        if (intra == 1) {
                            for (int blk = 0; blk < 16; ++blk) {
                                const int ri = blk_raster16(blk), bx = ri & 3, by = ri >> 2;
                                const int mA = bx ? (int)L.im[ri - 1][lane]
                                                  : (aA ? (int)(int8_t)((lim >> (8 * by)) & 255u) : -2);
                                const int mB = by ? (int)L.im[ri - 4][lane] : -2;
                                const int pm = (mA == -2 || mB == -2) ? 2 : min(mA < 0 ? 2 : mA, mB < 0 ? 2 : mB);
                                int md = pm;
                                if (!r.u(1)) {
                                    const int rem = (int)r.u(3);
                                    md = rem < pm ? rem : rem + 1;
                                }
                                L.im[ri][lane] = (int8_t)md;
                            }
                            m0d = L.im[0][lane];
                            m3 = L.im[3][lane];
                            nim = (uint32_t)(uint8_t)L.im[3][lane] | (uint32_t)(uint8_t)L.im[7][lane] << 8 |
                                  (uint32_t)(uint8_t)L.im[11][lane] << 16 | (uint32_t)(uint8_t)L.im[15][lane] << 24;
                        } else {
                            m0d = (it - 1) & 3;
                        }
                        const uint32_t cm = r.ue();
                        plen = r.p - poff;
                        if (r.bad || r.over() || cm > 3u) {
                            fail = true;
                            break;
                        }
                        bool na = cm == 0 || cm == 1 || cm == 3, nbb = cm == 0 || cm == 2 || cm == 3, nd = cm == 3,
                             nc = false;
                        if (intra == 1) {
                            na = nbb = true;
                            nd = nd || m0d == 4 || m0d == 5 || m0d == 6;
                            nc = m3 == 3 || m3 == 7;
                        } else {
                            na = na || m0d != 0;
                            nbb = nbb || m0d != 1;
                            nd = nd || m0d == 3;
                        }
                        auto same = [&](int dx, int dy, bool ext) {
                            const int X = x0c + x + dx, Y = y0c + y + dy;
                            return ext == (X >= 0 && Y >= 0 && X < mbw_c);
                        };
                        /* B and D are never in this slice here */
                        if ((na && !same(-1, 0, aA)) || (nbb && !same(0, -1, false)) || (nd && !same(-1, -1, false)) ||
                            (nc && !same(1, -1, aC))) {
                            status = SCROLL_SPLICE_ERR_MBTYPE;
                            bad = m | (int)mbt << 16;
                            fail = true;
                            break;
                        }
                        if (intra == 1) {
                            const uint32_t code = r.ue();
                            if (r.bad || r.over() || code > 47u) {
                                fail = true;
                                break;
                            }
                            cbp_code = (int)code;
                            cbp = CBP_INTRA[code];
                        } else {
                            cbp = ((it - 1) >= 12 ? 15 : 0) | (((it - 1) >> 2) % 3) << 4;
                        }
                        hasqpd = cbp || intra == 2;
                    }
                } else {
                    part = mbt == 4u ? 3 : (int)mbt;
                    uint32_t sub = 0;
                    const Mv A = aA ? unpk_mv(lrf0, lmv0) : none;
                    const Mv C = aC ? unpk_mv(frf, fmv) : none;
                    if (mbt == 0u) {
                        int ref = 0;
                        if (nrefs == 2) ref = 1 - (int)r.u(1);
                        else if (nrefs > 2) ref = (int)r.ue();
                        const int dx = r.se(), dy = r.se();
                        int px, py;
                        predict_spec(A, none, C, ref, px, py);
                        const long long mx = (long long)px + dx, my = (long long)py + dy;
                        if (ref >= nrefs || mx < -SPLICE_MAX_MV || mx > SPLICE_MAX_MV || my < -SPLICE_MAX_MV ||
                            my > SPLICE_MAX_MV) {
                            fail = true;
                            break;
                        }
                        me = Mv{ref, (int)mx, (int)my};
                    } else {
                        bool okp = true;
                        if (part == 3)
                            for (int k = 0; k < 4; ++k) {
                                const uint32_t stp = r.ue();
                                if (stp > 3u) okp = false;
                                sub |= (stp & 3u) << (2 * k);
                            }
                        const int nref = part == 3 ? 4 : 2;
                        uint32_t refw = 0;
                        if (mbt != 4u)
                            for (int k = 0; k < nref; ++k) {
                                int rf = 0;
                                if (nrefs == 2) rf = 1 - (int)r.u(1);
                                else if (nrefs > 2) rf = (int)r.ue();
                                if (rf >= nrefs) okp = false;
                                refw |= (uint32_t)(rf & 255) << (8 * k);
                            }
                        if (!okp) {
                            fail = true;
                            break;
                        }
                        uint32_t dn = 0;
                        /* block (cx, cy) relative to the MB: inside once decoded,
                         * the left MB's right column, the slice's first MB's
                         * block (0, 3) above-right; nothing else above */
                        auto nb = [&](int cx, int cy) -> Mv {
                            if (cy >= 0) {
                                if (cx >= 4) return none;
                                if (cx >= 0) {
                                    const int q2 = 4 * cy + cx;
                                    return (dn >> q2) & 1u ? unpk_mv(L.crf[q2][lane], L.cmv[q2][lane]) : none;
                                }
                                return aA ? unpk_mv(lrfq(cy), lmvq(cy)) : none;
                            }
                            if (cx >= 4) return aC ? unpk_mv(frf, fmv) : none;
                            return none;
                        };
                        for_parts(part, sub, [&](int bx, int by, int bw, int bh, int mp) {
                            const int rf = (int)((refw >> (8 * mp)) & 255u);
                            const int dx = r.se(), dy = r.se();
                            int px, py;
                            predict_part(part, mp, bx, by, bw, rf, nb, px, py);
                            const long long mx = (long long)px + dx, my = (long long)py + dy;
                            okp = okp && mx >= -SPLICE_MAX_MV && mx <= SPLICE_MAX_MV && my >= -SPLICE_MAX_MV &&
                                  my <= SPLICE_MAX_MV;
                            const uint32_t pm = part_mask(bx, by, bw, bh);
                            for (int q2 = 0; q2 < 16; ++q2)
                                if ((pm >> q2) & 1u) {
                                    L.cmv[q2][lane] = pk_mv((int)mx, (int)my);
                                    L.crf[q2][lane] = (int8_t)rf;
                                }
                            dn |= pm;
                        });
                        if (!okp || r.bad || r.over()) {
                            fail = true;
                            break;
                        }
                        me = unpk_mv(L.crf[0][lane], L.cmv[0][lane]);
                        /* the blocks' refs and motion in 8-byte stores */
                        uint2 *bw = reinterpret_cast<uint2 *>(R->bref);
#pragma unroll
                        for (int h2 = 0; h2 < 2; ++h2) {
                            uint32_t v0 = 0, v1 = 0;
#pragma unroll
                            for (int b2 = 0; b2 < 4; ++b2) {
                                v0 |= (uint32_t)(uint8_t)L.crf[8 * h2 + b2][lane] << (8 * b2);
                                v1 |= (uint32_t)(uint8_t)L.crf[8 * h2 + 4 + b2][lane] << (8 * b2);
                            }
                            bw[h2] = make_uint2(v0, v1);
                        }
                        uint2 *mw = reinterpret_cast<uint2 *>(R->bmv);
#pragma unroll
                        for (int h2 = 0; h2 < 8; ++h2) mw[h2] = make_uint2(L.cmv[2 * h2][lane], L.cmv[2 * h2 + 1][lane]);
                    }
                    subv = sub;
                    const uint32_t code = r.ue();
                    cbp = code < 48u ? (int)L.cbpi[code] : -1;
                    if (r.bad || r.over() || cbp < 0) {
                        fail = true;
                        break;
                    }
                    hasqpd = cbp != 0;
                }
                if (hasqpd) {
                    const int dq = r.se();
                    if (dq < -26 || dq > 25) {
                        fail = true;
                        break;
                    }
                    qp = (qp + dq + 52) % 52;
                    int d = qp - qp_c;
                    if (d < -26) d += 52;
                    if (d > 25) d -= 52;
                    qpd = d;
                    qp_c = qp;
                    if (fq_mb < 0) {
                        fq_mb = m;
                        fq_qp = qp;
                    }
                    last_qp = qp;
                    rs0 = r.p;
                    const int lmax = intra == 2 ? 15 : 16;
                    bool okr = true;
                    /* one piece in syntax order: TotalCoeff, TrailingOnes and
                     * where its body sits in the frame's RBSP */
                    auto lane_piece = [&](int pi, int nC, int maxc) {
                        if (!okr) return;
                        int tc, t1;
                        uint32_t bo, bl;
                        const uint32_t ps = r.p;
                        if (!lane_block(r, L, nC, maxc, tc, t1, bo, bl)) {
                            okr = false;
                            return;
                        }
                        L.tcc[pi][lane] = (uint8_t)tc;
                        L.t1s[pi][lane] = (uint8_t)t1;
                        L.bls[pi][lane] = (uint16_t)(bl | (bo - ps) << 11);
                        coded |= 1u << pi;
                        body += bl;
                    };
                    if (intra == 2) lane_piece(26, ncx(0, aA), 16);
                    for (int blk = 0; blk < 16; ++blk)
                        if (cbp & (1 << (blk >> 2))) {
                            const int pi = blk_raster16(blk);
                            lane_piece(pi, ncx(pi, aA), lmax);
                        }
                    if (cbp >> 4) {
                        lane_piece(16, -1, 4);
                        lane_piece(17, -1, 4);
                        if ((cbp >> 4) == 2)
                            for (int pi = 18; pi < 26; ++pi) lane_piece(pi, ncx(pi, aA), 15);
                    }
                    if (!okr) {
                        fail = true;
                        break;
                    }
                    rsn = r.p - rs0;
                }
                store_mb_head(R, me.ref, cbp, qpd, me.mx, me.my, 0, part, intra ? 0u : subv, intra, base + rs0, rsn,
                              base + poff, plen, mbt, cbp_code, aA ? 1 : 0, hasqpd, body);
                {
                    /* the TotalCoeffs as 7 dword stores (one byte store per
                     * piece had each wave store to 64 records 27 times); t1 /
                     * blen / boff are read only for cbp's pieces, all parsed */
                    uint32_t *tw = reinterpret_cast<uint32_t *>(R->tc);
#pragma unroll
                    for (int q = 0; q < (SPLICE_PIECES + 1) / 4; ++q) {
                        uint32_t v = 0;
#pragma unroll
                        for (int b2 = 0; b2 < 4; ++b2)
                            if (4 * q + b2 < SPLICE_PIECES) v |= (uint32_t)L.tcc[4 * q + b2][lane] << (8 * b2);
                        tw[q] = v;
                    }
                    if (hasqpd) {
                        /* the pieces' TrailingOnes (7 dwords), then bl [28] --
                         * record bytes 96 .. 152 -- as 3 16-byte stores and an
                         * 8-byte one; a piece the cbp leaves out carries a stale
                         * value, which no reader looks at */
                        uint32_t *t1w = reinterpret_cast<uint32_t *>(R->t1);
#pragma unroll
                        for (int q = 0; q < (SPLICE_PIECES + 1) / 4; ++q) {
                            uint32_t v = 0;
#pragma unroll
                            for (int b2 = 0; b2 < 4; ++b2) v |= (uint32_t)L.t1s[4 * q + b2][lane] << (8 * b2);
                            t1w[q] = v;
                        }
                        auto dw = [&](int d) -> uint32_t {          /* dword d of bytes 96 .. 152 */
                            return (uint32_t)L.bls[2 * d][lane] | (uint32_t)L.bls[2 * d + 1][lane] << 16;
                        };
                        uint4 *bq = reinterpret_cast<uint4 *>(R->bl);
#pragma unroll
                        for (int q = 0; q < 3; ++q) bq[q] = make_uint4(dw(4 * q), dw(4 * q + 1), dw(4 * q + 2), dw(4 * q + 3));
                        reinterpret_cast<uint2 *>(R->bl)[6] = make_uint2(dw(12), dw(13));
                    }
                }
                /* hand the context on */
                const bool parted = part != 0;
                if (m == m0) {
                    fmv = parted ? L.cmv[12][lane] : pk_mv(me.mx, me.my);
                    frf = parted ? L.crf[12][lane] : me.ref;
                }
                lmv0 = parted ? L.cmv[3][lane] : pk_mv(me.mx, me.my);
                lmv1 = parted ? L.cmv[7][lane] : lmv0;
                lmv2 = parted ? L.cmv[11][lane] : lmv0;
                lmv3 = parted ? L.cmv[15][lane] : lmv0;
                lrf0 = parted ? L.crf[3][lane] : me.ref;
                lrf1 = parted ? L.crf[7][lane] : lrf0;
                lrf2 = parted ? L.crf[11][lane] : lrf0;
                lrf3 = parted ? L.crf[15][lane] : lrf0;
                ltc = (uint32_t)L.tcc[3][lane] | (uint32_t)L.tcc[7][lane] << 8 | (uint32_t)L.tcc[11][lane] << 16 |
                      (uint32_t)L.tcc[15][lane] << 24;
                ltc2 = (uint32_t)L.tcc[19][lane] | (uint32_t)L.tcc[21][lane] << 8 | (uint32_t)L.tcc[23][lane] << 16 |
                       (uint32_t)L.tcc[25][lane] << 24;
                lim = nim;
                next();
            }
            if (!fail) {
                if (r.p != end || r.u(1) != 1u) fail = true;
                if (!fail && (r.p & 7u)) {
                    const int k = 8 - (int)(r.p & 7u);
                    if (r.u(k)) fail = true;
                }
                while (!fail && r.p < r.nbits)
                    if (r.u(8)) fail = true;
                if (!fail && !r.bad && !r.over()) status = SCROLL_SPLICE_OK;
            }
        }
        UN->first = first;
        UN->nmb = m - (first < 0 ? 0 : first);
        UN->status = status;
        UN->bad = bad;
        UN->fq_mb = fq_mb;
        UN->fq_qp = fq_qp;
        UN->last_qp = last_qp;
    }
}

/* k_splice_parse: one wave parses one slice (NAL unit; a frame's units are
 * dealt over the grid's y waves).  The slice is a sequential bit string, so
 * the parse itself is wave-uniform (scalar values, no divergence): the bit
 * window is 64 RBSP words held one per lane (readlane at the uniform bit
 * position), every VLC is matched by all lanes at once, lane j keeps piece
 * j's record fields, and the neighbour context (motion of the two rows above,
 * TotalCoeffs and Intra4x4PredModes of the row above) sits in LDS.  A
 * neighbour MB is available when it is inside the picture and not before the
 * slice's first MB (6.4.x); the slice's first_mb_in_slice, MB count and QP
 * ends go to its unit for k_splice_fix. */
__global__ __launch_bounds__(64) void k_splice_parse(int n, const int32_t *__restrict__ list,
                                                     SpliceFrame *__restrict__ spf,
                                                     SpliceUnit *__restrict__ units,
                                                     const DevStream *__restrict__ st, int ld_fr,
                                                     uint32_t *__restrict__ rbsp,
                                                     SpliceMbRec *__restrict__ recs)
{
    __shared__ ParseLds L;
    const int i = blockIdx.x, lane = threadIdx.x;
    if (i >= n) return;
    const int idx = list[i];
    SpliceFrame *F = spf + idx;
    const int W = F->w, H = F->h, nmb = W * H;
    const int nu = min(F->nunits, (int)splice_unit_cap(nmb));
    if ((int)blockIdx.y >= nu) return;
    const DevStream S = st[idx / ld_fr];
    const int mbw_c = S.w / 16, x0c = F->x0, y0c = F->y0;
    SpliceMbRec *rec = recs + F->rec_first;
    /* k_splice_unesc's bad NAL headers and the lanes' slices (unless handed
     * back) are done: no tables for a wave without a slice left */
    const bool lanef = F->nunits >= SPLICE_LANE_MIN && F->nunits <= SPLICE_MAXU;
    auto todo = [&](int u) {
        const int st0 = U(units[F->unit_first + u].status);
        return !(st0 == SCROLL_SPLICE_ERR_NAL || (lanef && st0 != SPLICE_REDO));
    };
    {
        bool any = false;
        for (int u = (int)blockIdx.y; u < nu && !any; u += (int)gridDim.y) any = todo(u);
        if (!any) return;
    }
    const LaneTabs T = lane_tabs();
    for (int u = (int)blockIdx.y; u < nu; u += (int)gridDim.y) {
    SpliceUnit *UN = units + F->unit_first + u;
    if (!todo(u)) continue;
    /* the NAL pointer is a generic one, so the compiler takes its bytes for
     * per-lane values: the header byte goes through readfirstlane, or every
     * branch on it -- and the whole bit reader after it -- turns divergent */
    const uint32_t h0 = U(F->nal[U(UN->b)]);
    int status = SCROLL_SPLICE_ERR_HEADER, first = -1, m = 0, bad = -1;
    int fq_mb = -1, fq_qp = 0, last_qp = 0;
    SRd r;
    const uint32_t w0 = U(UN->w0), nb = U(UN->nbytes), end = U(UN->end), base = 32u * w0;
    if (W > PARSE_MAXW) goto done;
    {
    const int ref_idc = (int)(h0 >> 5) & 3;
    const bool idr = (h0 & 31u) == 5u;
    r.init(rbsp + F->rbsp_word + w0, (nb + 3u) >> 2, 8u * nb);

    int nrefs = 2;                         /* the composer's PPS (h264_writer.c:114) */
    first = (int)r.ue();                                           /* first_mb_in_slice */
    bool islice;
    {
        const uint32_t stype = r.ue();
        islice = stype == 2 || stype == 7;
        if ((stype != 0 && stype != 5 && !islice) || (idr && !islice)) goto done;   /* P / I (IDR: I) */
    }
    if (r.ue() != 0) goto done;                                    /* pps id */
    r.skip(S.log2_mfn);
    if (idr) r.ue();                                               /* idr_pic_id */
    if (S.poc_type == 0) r.skip(S.log2_poc);
    if (!islice && r.u(1)) {
        const uint32_t k = r.ue();
        if (k > 31) goto done;
        nrefs = (int)k + 1;
    }
    if (!islice && r.u(1)) {               /* list modification: the composed list only */
        for (int k = 0;; ++k) {
            const uint32_t idc = r.ue();
            if (r.bad || r.over() || k > 32) {
                status = SCROLL_SPLICE_ERR_SYNTAX;
                goto done;
            }
            if (idc == 3) break;
            if (idc != 2 || r.ue() != (uint32_t)k) goto done;
        }
    }
    if (ref_idc && idr) {
        r.skip(2);                                                 /* no_output_of_prior_pics, long_term_reference */
    } else if (ref_idc && r.u(1)) {                                /* MMCO */
        for (int k = 0;; ++k) {
            const uint32_t op = r.ue();
            if (r.bad || r.over() || k > 64 || op > 6) {
                status = SCROLL_SPLICE_ERR_SYNTAX;
                goto done;
            }
            if (op == 0) break;
            if (op == 1 || op == 3) r.ue();
            if (op == 2) r.ue();
            if (op == 3 || op == 6) r.ue();
            if (op == 4) r.ue();
        }
    }
    int qp = 26 + r.se();
    if (qp < 0 || qp > 51) goto done;
    if (S.deblock && r.ue() != 1) goto done;
    status = SCROLL_SPLICE_ERR_SYNTAX;
    if (r.bad || r.over() || first < 0 || first >= nmb) goto done;   /* k_splice_fix: HEADER if out of order */
    {
        const int m0 = first;
        m = m0;
        int x = m0 % W, y = m0 / W;
        int qp_c = 26;                     /* composed chain from 26 (k_splice_fix rebases the first) */
        const Mv none{-1, 0, 0};
        uint32_t tc_left = 0;              /* lane j: TotalCoeff of piece j, MB to the left */
        bool aA = false, aB = false, aC = false, aD = false;
        auto avail = [&]() {
            aA = x > 0 && m - 1 >= m0;
            aB = y > 0 && m - W >= m0;
            aC = y > 0 && x + 1 < W && m - W + 1 >= m0;
            aD = x > 0 && y > 0 && m - W - 1 >= m0;
        };
        auto ul = [&]() { return unpk_mv(L.ulrf, L.ulmv); };     /* block (3, 3) of the MB above-left */
        /* whole-MB neighbours of MB (x, y): A = the left MB's block (3, 0),
         * B = the above MB's (0, 3), C = the above-right MB's (0, 3), else
         * D = the above-left MB's (3, 3) */
        auto ctx = [&](Mv &A, Mv &B, Mv &C) {
            A = aA ? unpk_mv(L.lrf[0], L.lmv[0]) : none;
            B = aB ? unpk_mv(L.rrf[x][0], L.rmv[x][0]) : none;
            C = aC ? unpk_mv(L.rrf[x + 1][0], L.rmv[x + 1][0]) : (aD ? ul() : none);
        };
        /* block (cx, cy) relative to MB (x, y) for a (sub-)partition (6.4.11.7):
         * inside the MB once decoded (done), right of it never */
        auto nb = [&](int cx, int cy, uint32_t done) -> Mv {
            if (cy >= 0) {
                if (cx >= 4) return none;
                if (cx >= 0) {
                    const int q = 4 * cy + cx;
                    return (done >> q) & 1u ? unpk_mv(L.crf[q], L.cmv[q]) : none;
                }
                return aA ? unpk_mv(L.lrf[cy], L.lmv[cy]) : none;
            }
            if (cx < 0) return aD ? ul() : none;
            if (cx < 4) return aB ? unpk_mv(L.rrf[x][cx], L.rmv[x][cx]) : none;
            return aC ? unpk_mv(L.rrf[x + 1][0], L.rmv[x + 1][0]) : none;
        };
        /* context for the MBs to come: the bottom row and right column of MB
         * (x, y) -- from one motion, or from the decoded blocks -- and its
         * Intra4x4PredModes (lane j: raster block j's; -1 not I_4x4) */
        auto finish = [&](bool parted, const Mv &me, int imode) {
            const int im3 = __shfl(imode, 4 * (lane & 3) + 3, 64), im12 = __shfl(imode, 12 + (lane & 3), 64);
            if (lane == 0) {                                  /* read before it is replaced */
                L.ulmv = L.rmv[x][3];
                L.ulrf = L.rrf[x][3];
            }
            if (lane < 4) {
                const uint32_t v = pk_mv(me.mx, me.my);
                L.rmv[x][lane] = parted ? L.cmv[12 + lane] : v;
                L.rrf[x][lane] = parted ? L.crf[12 + lane] : (int8_t)me.ref;
                L.lmv[lane] = parted ? L.cmv[4 * lane + 3] : v;
                L.lrf[lane] = parted ? L.crf[4 * lane + 3] : (int8_t)me.ref;
                L.iml[lane] = (int8_t)im3;
                L.imrow[x][lane] = (int8_t)im12;
            }
        };
        auto next = [&]() {
            ++m;
            if (++x == W) {
                x = 0;
                ++y;
            }
        };
        const int ts = tc_slot(lane);
        for (bool first_mb = true;; first_mb = false) {
            if (r.pos() >= end && !first_mb) break;
            const uint32_t run = islice ? 0u : r.ue();                  /* I slices: no mb_skip_run */
            if (r.bad || r.over() || run > (uint32_t)(nmb - m)) goto done;
            for (uint32_t k = 0; k < run; ++k, next()) {          /* P_Skip */
                avail();
                Mv A, B, C;
                ctx(A, B, C);
                int px, py;
                pskip_mv(aA, aB, A, B, C, px, py);
                SpliceMbRec *R = rec + m;
                if (lane == 0) {
                    R->ref = 0;
                    R->cbp = 0;
                    R->qpd = 0;
                    R->mx = px;
                    R->my = py;
                    R->skip = 1;
                    R->part = 0;
                    R->intra = 0;
                    R->hasqpd = 0;
                    R->nbsame = (uint8_t)((aA ? 1 : 0) | (aB ? 2 : 0));
                    R->res_len = 0;
                    R->body = 0;
                }
                if (lane < SPLICE_PIECES) {
                    R->tc[lane] = 0;
                    R->t1[lane] = 0;
                    R->bl[lane] = 0;
                }
                if (ts >= 0) L.tcrow[x][ts] = 0;
                tc_left = 0;
                finish(false, Mv{0, px, py}, -1);
            }
            if (r.pos() >= end) {                 /* skipped MBs end the slice (a run of 0 cannot) */
                if (run == 0) goto done;
                break;
            }
            if (m == nmb) goto done;
            avail();
            const uint32_t mbt = r.ue() + (islice ? 5u : 0u);          /* mb_type (Tables 7-13, 7-11) */
            if (r.bad || r.over() || mbt > 30) goto done;
            SpliceMbRec *R = rec + m;
            const uint8_t nbsame = (uint8_t)((aA ? 1 : 0) | (aB ? 2 : 0));
            /* lane j (12..15, 20, 21, 24, 25): piece j of the MB above, where
             * nc_at reads it */
            const uint32_t tc_top = aB && ts >= 0 ? L.tcrow[x][ts] : 0u;
            PieceOut po{0, 0, 0, 0};
            int cbp = 0, hasqpd = 0, qpd = 0, intra = 0, cbp_code = 0;
            uint32_t rs0 = 0, rsn = 0, poff = 0, plen = 0;
            if (mbt >= 5) {
                /* intra in a P slice (7.3.5.1): I_4x4, I_16x16, I_PCM */
                const int it = (int)mbt - 5;
                intra = it == 0 ? 1 : (it == 25 ? 3 : 2);
                int imode = -1;                                        /* lane j: raster block j's mode */
                if (intra == 3) {                                      /* I_PCM (7.3.5) */
                    bool bad = false;
                    if (r.pos() & 7u) bad = r.u(8 - (int)(r.pos() & 7u)) != 0u;   /* pcm_alignment_zero_bits */
                    poff = r.pos();
                    for (int k = 0; k < 96; ++k) r.skip(32);           /* 384 samples */
                    if (bad || r.over()) goto done;
                    po.tc = lane < SPLICE_PIECES ? 16u : 0u;           /* nC: 16 (9.2.1) */
                } else {
                    int m0d = -1, m3 = -1;                             /* modes of raster blocks 0, 3 */
                    poff = r.pos();
                    if (intra == 1) {
                        /* Intra4x4PredMode per block (8.3.1.1), luma4x4BlkIdx order;
                         * -2 unavailable, -1 not I_4x4 */
                        for (int blk = 0; blk < 16; ++blk) {
                            const int ri = blk_raster16(blk), bx = ri & 3, by = ri >> 2;
                            const int mA = bx ? __builtin_amdgcn_readlane(imode, ri - 1) : (aA ? (int)L.iml[by] : -2);
                            const int mB = by ? __builtin_amdgcn_readlane(imode, ri - 4)
                                              : (aB ? (int)L.imrow[x][bx] : -2);
                            const int pm = (mA == -2 || mB == -2) ? 2 : min(mA < 0 ? 2 : mA, mB < 0 ? 2 : mB);
                            int md = pm;
                            if (!r.u(1)) {
                                const int rem = (int)r.u(3);
                                md = rem < pm ? rem : rem + 1;
                            }
                            if (lane == ri) imode = md;
                        }
                        m0d = __builtin_amdgcn_readlane(imode, 0);
                        m3 = __builtin_amdgcn_readlane(imode, 3);
                    } else {
                        m0d = (it - 1) & 3;
                    }
                    const uint32_t cm = r.ue();                        /* intra_chroma_pred_mode */
                    plen = r.pos() - poff;
                    if (r.bad || r.over() || cm > 3u) goto done;
                    /* the neighbours its prediction reads have the same
                     * availability in the external and the composed picture */
                    bool na = cm == 0 || cm == 1 || cm == 3, nbb = cm == 0 || cm == 2 || cm == 3, nd = cm == 3,
                         nc = false;
                    if (intra == 1) {
                        na = nbb = true;
                        nd = nd || m0d == 4 || m0d == 5 || m0d == 6;
                        nc = m3 == 3 || m3 == 7;
                    } else {
                        na = na || m0d != 0;
                        nbb = nbb || m0d != 1;
                        nd = nd || m0d == 3;
                    }
                    auto same = [&](int dx, int dy, bool ext) {
                        const int X = x0c + x + dx, Y = y0c + y + dy;
                        return ext == (X >= 0 && Y >= 0 && X < mbw_c);
                    };
                    if ((na && !same(-1, 0, aA)) || (nbb && !same(0, -1, aB)) || (nd && !same(-1, -1, aD)) ||
                        (nc && !same(1, -1, aC))) {
                        status = SCROLL_SPLICE_ERR_MBTYPE;
                        bad = m | (int)mbt << 16;
                        goto done;
                    }
                    if (intra == 1) {
                        const uint32_t code = r.ue();
                        if (r.bad || r.over() || code > 47u) goto done;
                        cbp_code = (int)code;
                        cbp = CBP_INTRA[code];
                    } else {
                        cbp = ((it - 1) >= 12 ? 15 : 0) | (((it - 1) >> 2) % 3) << 4;
                    }
                    hasqpd = cbp || intra == 2;
                }
                if (lane == 0) {
                    R->ref = SPLICE_REF_INTRA;
                    R->mx = 0;
                    R->my = 0;
                    R->skip = 0;
                    R->part = 0;
                    R->sub = 0;
                }
                finish(false, Mv{SPLICE_REF_INTRA, 0, 0}, imode);
            } else {
                Mv me{0, 0, 0};
                const int part = mbt == 4 ? 3 : (int)mbt;
                uint32_t sub = 0;
                if (mbt == 0) {
                    int ref = 0;
                    if (nrefs == 2) ref = 1 - (int)r.u(1);
                    else if (nrefs > 2) ref = (int)r.ue();
                    const int dx = r.se(), dy = r.se();
                    Mv A, B, C;
                    ctx(A, B, C);
                    int px, py;
                    predict_spec(A, B, C, ref, px, py);
                    const long long mx = (long long)px + dx, my = (long long)py + dy;
                    if (ref >= nrefs || mx < -SPLICE_MAX_MV || mx > SPLICE_MAX_MV || my < -SPLICE_MAX_MV ||
                        my > SPLICE_MAX_MV)
                        goto done;
                    me = Mv{ref, (int)mx, (int)my};
                } else {
                    /* sub_mb_pred / mb_pred (7.3.5.1-2): sub_mb_types, ref_idx per
                     * mbPartIdx (P_8x8ref0: all 0), mvd per (sub-)partition */
                    if (part == 3)
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t stp = r.ue();
                            if (stp > 3u) goto done;
                            sub |= stp << (2 * k);
                        }
                    const int nref = part == 3 ? 4 : 2;
                    uint32_t refw = 0;                                 /* ref of mbPartIdx k: byte k */
                    if (mbt != 4)
                        for (int k = 0; k < nref; ++k) {
                            int rf = 0;
                            if (nrefs == 2) rf = 1 - (int)r.u(1);
                            else if (nrefs > 2) rf = (int)r.ue();
                            if (rf >= nrefs) goto done;
                            refw |= (uint32_t)rf << (8 * k);
                        }
                    uint32_t dn = 0;
                    bool ok = true;
                    for_parts(part, sub, [&](int bx, int by, int bw, int bh, int mp) {
                        const int rf = (int)((refw >> (8 * mp)) & 255u);
                        const int dx = r.se(), dy = r.se();
                        int px, py;
                        predict_part(part, mp, bx, by, bw, rf, [&](int cx, int cy) { return nb(cx, cy, dn); },
                                     px, py);
                        const long long mx = (long long)px + dx, my = (long long)py + dy;
                        ok = ok && mx >= -SPLICE_MAX_MV && mx <= SPLICE_MAX_MV && my >= -SPLICE_MAX_MV &&
                             my <= SPLICE_MAX_MV;
                        const uint32_t pm = part_mask(bx, by, bw, bh);
                        if (lane < 16 && ((pm >> lane) & 1u)) {
                            L.cmv[lane] = pk_mv((int)mx, (int)my);
                            L.crf[lane] = (int8_t)rf;
                        }
                        dn |= pm;
                    });
                    if (!ok || r.bad || r.over()) goto done;
                    me = unpk_mv(L.crf[0], L.cmv[0]);
                }
                /* the motion is final: record it and hand the context on now, so
                 * none of it stays live through the residual */
                if (lane == 0) {
                    R->ref = (int16_t)me.ref;
                    R->mx = me.mx;
                    R->my = me.my;
                    R->skip = 0;
                    R->part = (uint8_t)part;
                    R->sub = (uint8_t)sub;
                }
                if (part && lane < 16) {
                    R->bref[lane] = L.crf[lane];
                    R->bmv[lane] = L.cmv[lane];
                }
                finish(part != 0, me, -1);
                const uint32_t code = r.ue();
                cbp = code < 48u ? (int)__builtin_amdgcn_readlane(T.cbp, code) : -1;
                if (r.bad || r.over() || cbp < 0) goto done;
                hasqpd = cbp != 0;
            }
            if (hasqpd) {
                const int dq = r.se();
                if (dq < -26 || dq > 25) goto done;
                qp = (qp + dq + 52) % 52;
                int d = qp - qp_c;
                if (d < -26) d += 52;
                if (d > 25) d -= 52;
                qpd = d;
                qp_c = qp;
                if (fq_mb < 0) {
                    fq_mb = m;
                    fq_qp = qp;
                }
                last_qp = qp;
                rs0 = r.pos();
                /* the pieces in syntax order (7.3.5.3): (I_16x16 DC,) luma 4x4
                 * blocks of the coded 8x8s, chroma DC, chroma AC */
                const int lmax = intra == 2 ? 15 : 16;
                if (intra == 2 && !wrd_piece(r, T, 26, nc_at(0, po.tc, tc_left, tc_top, aA, aB), 16, po)) goto done;
                for (int blk = 0; blk < 16; ++blk) {
                    if (!(cbp & (1 << (blk >> 2)))) continue;
                    const int pi = blk_raster16(blk);
                    if (!wrd_piece(r, T, pi, nc_at(pi, po.tc, tc_left, tc_top, aA, aB), lmax, po)) goto done;
                }
                if (cbp >> 4) {
                    if (!wrd_piece(r, T, 16, -1, 4, po) || !wrd_piece(r, T, 17, -1, 4, po)) goto done;
                    if ((cbp >> 4) == 2)
                        for (int pi = 18; pi < 26; ++pi)
                            if (!wrd_piece(r, T, pi, nc_at(pi, po.tc, tc_left, tc_top, aA, aB), 15, po))
                                goto done;
                }
                rsn = r.pos() - rs0;
            }
            const uint32_t body = (uint32_t)__builtin_amdgcn_readlane(
                wave_incl_sum(lane < SPLICE_PIECES ? po.len : 0u, lane), 63);
            if (lane == 0) {
                R->cbp = (uint8_t)cbp;
                R->qpd = (int8_t)qpd;
                R->hasqpd = (uint8_t)hasqpd;
                R->body = (uint16_t)body;
                R->intra = (uint8_t)intra;
                R->mbt = (uint8_t)mbt;
                R->cbp_code = (uint8_t)cbp_code;
                R->poff = base + poff;
                R->plen = (uint16_t)plen;
                R->nbsame = nbsame;
                R->res_off = base + rs0;
                R->res_len = rsn;
            }
            if (lane < SPLICE_PIECES) {
                R->tc[lane] = (uint8_t)po.tc;
                R->t1[lane] = (uint8_t)po.t1;
                R->bl[lane] = (uint16_t)(po.len | po.tl << 11);
            }
            if (ts >= 0) L.tcrow[x][ts] = (uint8_t)po.tc;
            tc_left = po.tc;
            next();
        }
        /* rbsp_slice_trailing_bits (+ zero bytes of a byte stream) */
        if (r.pos() != end || r.u(1) != 1u) goto done;
        if (r.pos() & 7u) {
            const int k = 8 - (int)(r.pos() & 7u);
            if (r.u(k)) goto done;
        }
        while (r.pos() < r.nbits)
            if (r.u(8)) goto done;
        if (!r.bad && !r.over()) status = SCROLL_SPLICE_OK;
    }
    }
done:
    if (lane == 0) {
        UN->first = first;
        UN->nmb = m - (first < 0 ? 0 : first);
        UN->status = status;
        UN->bad = bad;
        UN->fq_mb = fq_mb;
        UN->fq_qp = fq_qp;
        UN->last_qp = last_qp;
    }
    }
}

/* k_splice_fix: one wave per frame walks its units in order -- each must
 * start at the MB after the previous one's last (else HEADER), the first
 * failing unit's status is the frame's, together they cover the picture --
 * and rebases the first mb_qp_delta of every slice on the QP chain of the
 * slices before it (composed slice QP 26). */
__global__ __launch_bounds__(64) void k_splice_fix(int n, const int32_t *__restrict__ list,
                                                   SpliceFrame *__restrict__ spf,
                                                   const SpliceUnit *__restrict__ units,
                                                   SpliceMbRec *__restrict__ recs, int32_t *__restrict__ lanes)
{
    const int i = blockIdx.x;
    if (i >= n || threadIdx.x != 0) return;
    if (i == 0) lanes[0] = 0;                           /* the lane list, empty for the next parse */
    SpliceFrame *F = spf + list[i];
    const int nmb = F->w * F->h, nall = F->nunits;
    const int nu = min(nall, (int)splice_unit_cap(nmb));
    const SpliceUnit *UN = units + F->unit_first;
    SpliceMbRec *rec = recs + F->rec_first;
    int status = SCROLL_SPLICE_OK, bad = -1;
    if (nall > SPLICE_MAXU || nall < 1) {
        status = SCROLL_SPLICE_ERR_NAL;
    } else {
        int expect = 0, qp_c = 26;
        for (int u = 0; u < nu; ++u) {
            const SpliceUnit un = UN[u];
            if (un.status == SCROLL_SPLICE_ERR_NAL) {
                status = un.status;
                break;
            }
            if (un.first != expect) {
                status = SCROLL_SPLICE_ERR_HEADER;
                break;
            }
            if (un.status != SCROLL_SPLICE_OK) {
                status = un.status;
                bad = un.status == SCROLL_SPLICE_ERR_MBTYPE ? un.bad : -1;
                break;
            }
            if (un.fq_mb >= 0) {
                int d = un.fq_qp - qp_c;
                if (d < -26) d += 52;
                if (d > 25) d -= 52;
                rec[un.fq_mb].qpd = (int8_t)d;
                qp_c = un.last_qp;
            }
            expect += un.nmb;
        }
        if (status == SCROLL_SPLICE_OK && (nall > nu || expect != nmb)) status = SCROLL_SPLICE_ERR_SYNTAX;
    }
    F->status = status;
    F->bad_mb = bad;
}

/* ------------------------------------------------------------------------ */
/* k_splice_stage                                                            */
/* ------------------------------------------------------------------------ */
constexpr int SPL_WB = 2048;                 /* writing sweep: LDS words per pass (64 Kbit) */
#ifndef SCROLL_STAGE_HEAD_LDS
#define SCROLL_STAGE_HEAD_LDS 1
#endif

/* ORs MSB-first words into LDS words [lo, lo + n) (others dropped: another pass) */
struct LdsWin {
    uint32_t *b;
    uint32_t lo, n;
    __device__ inline void operator()(uint32_t i, uint32_t v) const
    {
        const uint32_t k = i - lo;
        if (k < n && v) atomicOr(&b[k], v);
    }
};

struct SpliceLds {
    int32_t fr[RING], fx[RING], fy[RING];   /* motion of MB m at m % RING */
    int32_t fk[RING];                       /* its record if a partitioned spliced MB, else -1 */
    ScrollHintRect rc[SCROLL_HINT_MAX_RECTS];
    int32_t wo[8], wl[8], wv[8];
    uint32_t wsum[NW];
    int32_t wmax[NW];
    uint64_t pcm_mask[NW];                  /* I_PCM MBs of the window (alignment) */
    uint8_t pcm_key[DT];
    uint4 etc[RING];                        /* MB m's edge TotalCoeffs at m % RING (0: not spliced) */
    uint32_t wbuf[SPL_WB];                  /* the writing sweep's word window */
    PTabs pt;                               /* coeff_token (len << 8 | bits) */
    uint8_t cbpc[48];                       /* inter coded_block_pattern -> codeNum */
    uint32_t ep_n;
    int32_t bad;
    uint32_t carry;                         /* the partial word at the bit position (MSB first) */
#if SCROLL_STAGE_HEAD_LDS
    /* each lane's spliced MB record head (SPLICE_REC_HEAD bytes): held in
     * registers across the window it took the kernel to 252 VGPRs */
    alignas(16) uint8_t hdb[DT][SPLICE_REC_HEAD];
#endif
};
static_assert(offsetof(SpliceMbRec, bl) == SPLICE_REC_HEAD && sizeof(SpliceMbRec) == 232,
              "the stage copies a record's first SPLICE_REC_HEAD bytes in 16-byte loads");
static_assert(offsetof(SpliceMbRec, tc) % 4 == 0 && (SPLICE_PIECES + 1) % 4 == 0,
              "k_splice_lanes stores the TotalCoeffs as whole dwords");
static_assert(offsetof(SpliceMbRec, t1) % 4 == 0 && offsetof(SpliceMbRec, bl) == 96 &&
                  offsetof(SpliceMbRec, bref) == 152 && offsetof(SpliceMbRec, bmv) == 168 && (SPLICE_PIECES + 1) == 28,
              "k_splice_lanes' record stores: t1 in dwords, bl as 56 bytes from 96, bref / bmv in 8-byte stores");
static_assert(offsetof(SpliceMbRec, mx) == 4 && offsetof(SpliceMbRec, skip) == 12 && offsetof(SpliceMbRec, intra) == 15 &&
                  offsetof(SpliceMbRec, res_off) == 72 && offsetof(SpliceMbRec, poff) == 80 &&
                  offsetof(SpliceMbRec, mbt) == 86 && offsetof(SpliceMbRec, nbsame) == 88 &&
                  offsetof(SpliceMbRec, body) == 90,
              "store_mb_head's packing");

/* an MB's TotalCoeffs its right / lower neighbour reads for nC: x = pieces 3
 * 7 11 15, y = 19 21 23 25 (right column), z = 12 13 14 15, w = 20 21 24 25
 * (bottom row), a byte each */
__device__ inline uint4 edge_tc(const SpliceMbRec &h)
{
    auto b4 = [&](int a, int b, int c, int d) {
        return (uint32_t)h.tc[a] | (uint32_t)h.tc[b] << 8 | (uint32_t)h.tc[c] << 16 | (uint32_t)h.tc[d] << 24;
    };
    return make_uint4(b4(3, 7, 11, 15), b4(19, 21, 23, 25), b4(12, 13, 14, 15), b4(20, 21, 24, 25));
}

/* nC of piece i (luma raster 0..15, chroma AC 18..25) of MB h whose left /
 * top neighbours' edge TotalCoeffs are l / t (al / at: available) */
__device__ inline int nc_edge(int i, const SpliceMbRec &h, const uint4 &l, const uint4 &t, bool al, bool at)
{
    int nA, nB;
    if (i < 16) {
        const int bx = i & 3, by = i >> 2;
        nA = bx ? (int)h.tc[i - 1] : (al ? (int)((l.x >> (8 * by)) & 255u) : -1);
        nB = by ? (int)h.tc[i - 4] : (at ? (int)((t.z >> (8 * bx)) & 255u) : -1);
    } else {
        const int k = (i - 18) & 3, pl = (i - 18) >> 2, bx = k & 1, by = k >> 1;
        nA = bx ? (int)h.tc[i - 1] : (al ? (int)((l.y >> (8 * (2 * pl + by))) & 255u) : -1);
        nB = by ? (int)h.tc[i - 2] : (at ? (int)((t.w >> (8 * (2 * pl + bx))) & 255u) : -1);
    }
    return nc2(nA, nB);
}

/* ORs MSB-first words into the byte-order staging slot */
struct GlobOr {
    uint32_t *b;
    __device__ inline void operator()(uint32_t i, uint32_t v) const
    {
        if (v) atomicOr(&b[i], __builtin_bswap32(v));
    }
};
typedef OrSink<GlobOr> GSink;

/* n <= 32 bits at bit offset q of the RBSP words */
__device__ inline uint32_t bits_at(const uint32_t *w, uint32_t q)
{
    const uint32_t k = q >> 5, o = q & 31u;
    return o ? (w[k] << o) | (w[k + 1] >> (32u - o)) : w[k];
}

#ifndef SCROLL_STAGE_BL_PRELOAD
#define SCROLL_STAGE_BL_PRELOAD 1
#endif
/* SCROLL_STAGE_RWIN=1 (measured, not kept): the body reader below --
 * p720splicerows 5.09 -> 5.16 ms per step (profiles/r06s_stage_rwin.txt) */
#ifndef SCROLL_STAGE_RWIN
#define SCROLL_STAGE_RWIN 0
#endif

/* the writing sweep's reader of an MB's piece bodies: six RBSP words from
 * word wb in registers, moved on one word as a read passes word wb, the
 * word loaded then five words ahead -- the loads run ahead of the bits
 * instead of one load round trip per body, and a read always takes w0 / w1
 * (no selects: a select chain over the six became a scratch copy indexed
 * per lane).  Reads up to 6 words past the MB's last bit: the word pools
 * keep RWIN_SLACK_WORDS after their last unit */
static_assert(RWIN_SLACK_WORDS >= 6, "RWin reads up to 6 words past an MB's last bit");
struct RWin {
    const uint32_t *rb;
    uint32_t wb, w0, w1, w2, w3, w4, w5;
    __device__ inline void init(const uint32_t *r, uint32_t q)
    {
        rb = r;
        wb = q >> 5;
        w0 = rb[wb];
        w1 = rb[wb + 1];
        w2 = rb[wb + 2];
        w3 = rb[wb + 3];
        w4 = rb[wb + 4];
        w5 = rb[wb + 5];
    }
    /* the 32 bits from bit q (q >= 32 wb), MSB first */
    __device__ inline uint32_t at(uint32_t q)
    {
        while ((q >> 5) > wb) {
            w0 = w1;
            w1 = w2;
            w2 = w3;
            w3 = w4;
            w4 = w5;
            w5 = rb[wb + 6];
            ++wb;
        }
        const uint32_t o = q & 31u;
        return o ? __builtin_amdgcn_alignbit(w0, w1, 32u - o) : w0;
    }
};

/* n bits at bit q of the RBSP words, put */
template <class SK>
__device__ inline void put_rbsp(SK &sk, const uint32_t *rb, uint32_t q0, uint32_t n)
{
    if constexpr (__is_same(SK, CountSink)) {
        sk.n += n;
    } else {
        for (uint32_t k = 0; k < n; k += 32) {
            const int c = (int)min(32u, n - k);
            sk.put(bits_at(rb, q0 + k) >> (32 - c), c);
        }
    }
}

/* bits of one spliced MB after its head (inter: after the motion; intra:
 * after mb_type): an intra MB's prediction syntax (I_4x4: + its cbp codeNum)
 * or I_PCM's alignment (pad zero bits) and samples; an inter MB's cbp; then
 * mb_qp_delta and the pieces (I_16x16: its DC first).  An MB whose left and
 * top neighbours are spliced from the same slice (nbsame 3) sees the nC of
 * its external picture in every block: its residual is the external one bit
 * for bit and goes over as one run (parsed records only: res_len).  h: the
 * record's head in registers; the counting sweep takes the bodies' length
 * from h.body, the writing sweep each body's bits from the record (R) */
template <class SK>
__device__ inline void splice_tail(SK &sk, const SpliceMbRec &h, const SpliceMbRec *R, const uint4 &l,
                                   const uint4 &t, bool al, bool at, const SpliceLds &LS, const uint32_t *rb,
                                   uint32_t pad)
{
    constexpr bool count = __is_same(SK, CountSink);
    const int cbp = h.cbp;
    if (h.intra == 3) {
        sk.put(0u, (int)pad);                                  /* pcm_alignment_zero_bits */
        put_rbsp(sk, rb, h.poff, 384u * 8u);
        return;
    }
    if (h.intra) {
        put_rbsp(sk, rb, h.poff, h.plen);
        if (h.intra == 1) put_ue(sk, h.cbp_code);
        if (!h.hasqpd) return;
    } else {
        put_ue(sk, LS.cbpc[cbp]);
        if (!cbp) return;
    }
    put_se(sk, h.qpd);
    if ((h.nbsame & 3) == 3 && h.res_len) {
        put_rbsp(sk, rb, h.res_off, h.res_len);
        return;
    }
    if constexpr (count) sk.n += h.body;
    uint32_t rp = h.res_off;                    /* the external bits: pieces contiguous in syntax order */
    /* the pieces' u16 words, all at once (7 8-byte loads; records are 8-byte
     * aligned): per piece only its body's bit loads remain on the chain */
    uint32_t blw[(SPLICE_PIECES + 1) / 2] = {};
#if SCROLL_STAGE_BL_PRELOAD
    if constexpr (!count) {
        const uint2 *bq = reinterpret_cast<const uint2 *>(R->bl);
#pragma unroll
        for (int q = 0; q < (SPLICE_PIECES + 1) / 4; ++q) {
            const uint2 v = bq[q];
            blw[2 * q] = v.x;
            blw[2 * q + 1] = v.y;
        }
    }
#endif
    RWin win;
    if constexpr (!count) {
        if (SCROLL_STAGE_RWIN) win.init(rb, rp);
    }
    auto piece = [&](int i, int nC) {
        const int tc = h.tc[i], t1 = h.t1[i];
        uint32_t v, len;
        if (nC >= 8) {
            v = tc ? (uint32_t)(((tc - 1) << 2) | t1) : 3u;
            len = 6;
        } else {
            const uint32_t e = LS.pt.ct[nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2))][4 * tc + t1];
            v = e & 255u;
            len = e >> 8;
        }
        sk.put(v, (int)len);
        if constexpr (!count) {
            const uint32_t e = SCROLL_STAGE_BL_PRELOAD ? (blw[i >> 1] >> (16 * (i & 1))) & 0xffffu : R->bl[i];
            rp += e >> 11;                      /* past its external coeff_token */
            const uint32_t n = e & 2047u;
            if (SCROLL_STAGE_RWIN) {
                for (uint32_t k = 0; k < n; k += 32) {
                    const int c = (int)min(32u, n - k);
                    sk.put(win.at(rp + k) >> (32 - c), c);
                }
            } else {
                put_rbsp(sk, rb, rp, n);
            }
            rp += n;
        }
    };
    if (h.intra == 2) piece(26, nc_edge(0, h, l, t, al, at));
#pragma unroll
    for (int blk = 0; blk < 16; ++blk)
        if (cbp & (1 << (blk >> 2))) {
            const int i = blk_raster16(blk);
            piece(i, nc_edge(i, h, l, t, al, at));
        }
    if (cbp >> 4) {
        piece(16, -1);
        piece(17, -1);
        if ((cbp >> 4) == 2) {
#pragma unroll
            for (int i = 18; i < 26; ++i) piece(i, nc_edge(i, h, l, t, al, at));
        }
    }
}

#ifndef SCROLL_STAGE_WAVES
#define SCROLL_STAGE_WAVES 1
#endif
__global__ __launch_bounds__(DT) __attribute__((amdgpu_waves_per_eu(SCROLL_STAGE_WAVES))) void k_splice_stage(DevStream *__restrict__ st,
                                                     const NalDesc *__restrict__ nal, int ld_nal,
                                                     const PlanPending *__restrict__ pend,
                                                     DynFrame *__restrict__ dfr, int ld_fr,
                                                     const HintFrame *__restrict__ hf,
                                                     const ScrollHintRect *__restrict__ pool,
                                                     SpliceFrame *__restrict__ spf,
                                                     const SpliceMbRec *__restrict__ recs,
                                                     const uint32_t *__restrict__ rbsp,
                                                     uint8_t *__restrict__ stage, uint64_t slot_bytes)
{
    __shared__ SpliceLds L;
    const int s = blockIdx.y, f = dyn_frame_of(blockIdx.x, s), t = threadIdx.x;
    const size_t fi = (size_t)s * ld_fr + f;
    const HintFrame H = hf[fi];
    if (!(H.mode & (HINT_MODE_SPLICED | HINT_MODE_FB))) return;   /* k_hint_stage's frame */
    DevStream *S = st + s;
    DynFrame *DF = dfr + fi;
    const int j = DF->nal;
    if (j < 0) return;                                         /* experiment mode: no scroll NAL */
    const SpliceFrame SF = spf[fi];
    if (SF.status != SCROLL_SPLICE_OK) {                       /* the parse failed */
        if (t == 0) {
            DF->err = 8u;
            DF->ep = 0;
            atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_SPLICE);
        }
        return;
    }
    if (t == 0) spf[fi].stage_status = SCROLL_SPLICE_OK;
    const SpliceMbRec *rec = recs + SF.rec_first;
    const uint32_t *rb = rbsp + SF.rbsp_word;
    const int nr = (H.mode & HINT_MODE_FB) ? 0 : min((int)H.n, SCROLL_HINT_MAX_RECTS);   /* fallback: no rects */
    const int hmode = H.mode & 0xff;
    const bool pskip = hmode == SCROLL_HINT_PSKIP;
    const bool spec = hmode != SCROLL_HINT_EXACT;
    if (t == 0) {
        L.ep_n = 0;
        L.bad = 0;
        L.carry = 0u;
    }
    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    if (t < nr) L.rc[t] = pool[H.first + t];
    build_ptabs(SPT, L.pt, t, DT);
    if (t < 48) L.cbpc[t] = SPT.cbp_code[t];
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

    uint32_t F0;
    {
        CountSink hc{0};
        emit_slice_header(hc, c);
        F0 = hc.n;
    }
    const int mbw = c.w / 16, mbh = c.h / 16, nmb = mbw * mbh;
    const Regions rg = regions(c);
    const Layout lay{(c.h - c.off) / 16, rg.ra, 4 * rg.mva, rg.rb, 4 * rg.mvb};
    const int nrefs = 2 + c.nwp;
    const uint32_t m_mbw = magic32((uint32_t)mbw);
    uint8_t *slot = stage + fi * slot_bytes;
    uint32_t *out = reinterpret_cast<uint32_t *>(slot);
    const uint32_t cap_words = (uint32_t)((slot_bytes - DYN_OVF_BYTES) / 4) - 4u;
    uint32_t *eplist = reinterpret_cast<uint32_t *>(slot + slot_bytes - DYN_OVF_BYTES);

    bool my_bad = false, my_ref_bad = false;
    /* one sweep (round 5; round 4 counted the whole picture first, then
     * coded it again to write): each window's bits go out as soon as they
     * are placed, the word they share with the previous window carried in
     * LDS (L.carry), so no word is written twice concurrently and the slot
     * needs no zeroing; the slot's capacity is checked per window before
     * any store, and a frame that fails (capacity, hint, reference) has
     * written only inside its own slot and commits nothing */
    uint32_t pos = F0;             /* bits: header + MBs so far (uniform) */
    int last = -1;                 /* last coded MB before the window (uniform) */
    bool over = false;
    /* emulation prevention as the words go out (round 5; round 4 read the
     * slot back word by word after a fence, looking back for the last
     * non-zero byte through agent-scope loads): the last non-zero byte of
     * the words written so far (uniform) and this thread's insertions */
    int lnzb = -1;
    uint32_t my_ep = 0;
    for (int m0 = 0; m0 < nmb; m0 += DT) {
        /* the previous window's writing sweep still reads the ring (the
         * neighbour blocks of its partitioned MBs): wait before refilling */
        lds_barrier();
        const int m = m0 + t;
        int x = 0, y = 0, k = -1;
        Mv me{0, 0, 0};
        bool parted = false;
#if SCROLL_STAGE_HEAD_LDS
        SpliceMbRec &hd = *reinterpret_cast<SpliceMbRec *>(L.hdb[t]);   /* its head only */
#else
        SpliceMbRec hd;                                        /* a spliced MB's record head */
#endif
        uint4 et = make_uint4(0u, 0u, 0u, 0u);
        if (m < nmb) {
            y = (int)div_m((uint32_t)m, m_mbw);
            x = m - y * mbw;
            if (x >= SF.x0 && x < SF.x0 + SF.w && y >= SF.y0 && y < SF.y0 + SF.h) {
                k = (y - SF.y0) * SF.w + (x - SF.x0);
                const uint4 *hp = reinterpret_cast<const uint4 *>(rec + k);
#if SCROLL_STAGE_HEAD_LDS
#pragma unroll
                for (int q = 0; q < SPLICE_REC_HEAD / 16; ++q) reinterpret_cast<uint4 *>(L.hdb[t])[q] = hp[q];
#else
                uint4 hv[SPLICE_REC_HEAD / 16];
#pragma unroll
                for (int q = 0; q < SPLICE_REC_HEAD / 16; ++q) hv[q] = hp[q];
                __builtin_memcpy(&hd, hv, SPLICE_REC_HEAD);
#endif
                if (SF.hd_qp >= 0)                             /* the dynamic rect under hints: its QP chain */
                    hd.qpd = (int8_t)((uint32_t)k == SF.hd_first ? SF.hd_qp - 26 : 0);
                et = edge_tc(hd);
                const SpliceMbRec &mb = hd;
                me = Mv{mb.ref, mb.mx, mb.my};
                parted = mb.part != 0;
                auto valid = [&](int rf) {
                    const int wk = rf - 2;
                    return rf == 0 || rf == 1 || (wk >= 0 && wk < c.nwp && L.wv[wk]);
                };
                my_ref_bad |= !mb.intra && !valid(mb.ref);
                if (parted)
                    for (int q = 1; q < 16; ++q) my_ref_bad |= !valid(rec[k].bref[q]);   /* past the head */
            } else {
                bool bad;
                me = field(L.rc, L.wv, nr, x, y, lay, c.nwp, bad);
                my_bad |= bad;
            }
            L.fr[m & (RING - 1)] = me.ref;
            L.fx[m & (RING - 1)] = me.mx;
            L.fy[m & (RING - 1)] = me.my;
            L.fk[m & (RING - 1)] = parted ? k : -1;
            L.etc[m & (RING - 1)] = et;
        }
        __syncthreads();
        bool coded = false;
        int px = 0, py = 0;
        const Mv none{-1, 0, 0};
        /* 4x4 block (bx, by) of MB q (partitioned spliced MBs from their record) */
        auto blk = [&](int q, int bx, int by) {
            const int kk = L.fk[q & (RING - 1)];
            if (kk >= 0) return unpk_mv(rec[kk].bref[4 * by + bx], rec[kk].bmv[4 * by + bx]);
            return Mv{L.fr[q & (RING - 1)], L.fx[q & (RING - 1)], L.fy[q & (RING - 1)]};
        };
        if (m < nmb && !parted) {
            const Mv A = x > 0 ? blk(m - 1, 3, 0) : none;
            const Mv B = y > 0 ? blk(m - mbw, 0, 3) : none;
            const Mv C = y == 0 ? none
                                : (x + 1 < mbw ? blk(m - mbw + 1, 0, 3) : (x > 0 ? blk(m - mbw - 1, 3, 3) : none));
            if (spec) {
                int sx, sy;
                pskip_mv(x > 0, y > 0, A, B, C, sx, sy);
                coded = !pskip ||
                        !(me.ref == 0 && me.mx == sx && me.my == sy && (k < 0 || hd.cbp == 0));
                predict_spec(A, B, C, me.ref, px, py);
            } else {
                coded = true;
                predict_ref(A, B, C, me.ref, px, py);
            }
        }
        coded |= m < nmb && parted;                            /* predicted per partition */
        int excl, cmax;
        block_excl_max(coded ? m : -1, L.wmax, excl, cmax);
        /* the MB's bits: head, then (spliced) cbp / qp / pieces */
        /* the left / top MBs' edge TotalCoeffs (0 outside the rect) */
        const uint4 el = x > 0 ? L.etc[(m - 1) & (RING - 1)] : make_uint4(0u, 0u, 0u, 0u);
        const uint4 eu = y > 0 ? L.etc[(m - mbw) & (RING - 1)] : make_uint4(0u, 0u, 0u, 0u);
        /* a partitioned spliced MB's neighbour block (cx, cy) (6.4.11.7) */
        auto pnb = [&](int cx, int cy, uint32_t dn) {
            if (cy >= 0) {
                if (cx >= 4) return none;
                if (cx >= 0)
                    return (dn >> (4 * cy + cx)) & 1u ? unpk_mv(rec[k].bref[4 * cy + cx], rec[k].bmv[4 * cy + cx])
                                                      : none;
                return x > 0 ? blk(m - 1, 3, cy) : none;
            }
            if (y == 0) return none;
            if (cx < 0) return x > 0 ? blk(m - mbw - 1, 3, 3) : none;
            if (cx < 4) return blk(m - mbw, cx, 3);
            return x + 1 < mbw ? blk(m - mbw + 1, 0, 3) : none;
        };
        const bool intra = k >= 0 && hd.intra;
        uint32_t pcm_pad = 0;
        auto code_mb = [&](auto &sk) {
            put_ue(sk, (uint32_t)(m - max(excl, last) - 1));  /* mb_skip_run */
            if (intra) {
                put_ue(sk, hd.mbt);                            /* verbatim, like its prediction syntax */
                splice_tail(sk, hd, rec + k, el, eu, x > 0, y > 0, L, rb, pcm_pad);
                return;
            }
            if (parted) {
                const SpliceMbRec &mb = rec[k];
                const int part = mb.part;
                const uint32_t sub = mb.sub;
                put_ue(sk, (uint32_t)part);                    /* P_L0_L0_16x8 / 8x16, P_8x8 */
                if (part == 3)
                    for (int i = 0; i < 4; ++i) put_ue(sk, (sub >> (2 * i)) & 3u);
                for (int i = 0; i < (part == 3 ? 4 : 2); ++i) {  /* ref_idx per mbPartIdx */
                    const int q = part == 1 ? 8 * i : (part == 2 ? 2 * i : 2 * (i & 1) + 8 * (i >> 1));
                    const int rf = mb.bref[q];
                    if (nrefs == 2) sk.put((uint32_t)(1 - (rf & 1)), 1);
                    else put_ue(sk, (uint32_t)rf);
                }
                uint32_t dn = 0;
                for_parts(part, sub, [&](int bx, int by, int bw, int bh, int mp) {
                    const int q = 4 * by + bx;
                    const Mv v = unpk_mv(mb.bref[q], mb.bmv[q]);
                    int qx, qy;
                    predict_part(part, mp, bx, by, bw, v.ref, [&](int cx, int cy) { return pnb(cx, cy, dn); },
                                 qx, qy);
                    put_se(sk, v.mx - qx);
                    put_se(sk, v.my - qy);
                    dn |= part_mask(bx, by, bw, bh);
                });
            } else {
                sk.put(1, 1);                                  /* P_L0_16x16 */
                if (nrefs == 2) sk.put((uint32_t)(1 - (me.ref & 1)), 1);
                else if (nrefs > 2) put_ue(sk, (uint32_t)me.ref);
                put_se(sk, me.mx - px);
                put_se(sk, me.my - py);
            }
            if (k >= 0) splice_tail(sk, hd, rec + k, el, eu, x > 0, y > 0, L, rb, 0u);
            else sk.put(1, 1);                                 /* coded_block_pattern 0 */
        };
        CountSink cs{0};
        if (coded) code_mb(cs);
        /* I_PCM: pcm_alignment_zero_bits for its composed position.  Sizes
         * without them, scanned: the n-th I_PCM of the window starts its
         * samples at key_n + (pads before it) mod 8 with key_n = its
         * unpadded position mod 8, so pad_n = key_(n-1) - key_n mod 8
         * (key_0 = 0) */
        const bool pcm = coded && intra && hd.intra == 3;
        if (__syncthreads_or(pcm)) {
            uint32_t o0, t0;
            block_excl_sum(cs.n, L.wsum, o0, t0);
            CountSink hc{0};
            put_ue(hc, (uint32_t)(m - max(excl, last) - 1));
            put_ue(hc, 30u);
            const int lane = t & 63, wv = t >> 6;
            const uint64_t bl = __ballot(pcm);
            if (lane == 0) L.pcm_mask[wv] = bl;
            L.pcm_key[t] = (uint8_t)((pos + o0 + hc.n) & 7u);
            __syncthreads();
            if (pcm) {
                int prev = -1;
                const uint64_t below = bl & ((1ull << lane) - 1ull);
                if (below) {
                    prev = 64 * wv + 63 - __builtin_clzll(below);
                } else {
                    for (int w2 = wv - 1; w2 >= 0 && prev < 0; --w2)
                        if (L.pcm_mask[w2]) prev = 64 * w2 + 63 - __builtin_clzll(L.pcm_mask[w2]);
                }
                const uint32_t kp = prev >= 0 ? L.pcm_key[prev] : 0u;
                pcm_pad = (kp - L.pcm_key[t]) & 7u;
                cs.n += pcm_pad;
            }
            __syncthreads();
        }
        uint32_t off, T;
        block_excl_sum(cs.n, L.wsum, off, T);
            {
            /* the window's bits [pos, pos + T) -- window 0 from bit 0,
             * with the slice header -- through the LDS word window
             * (passes of SPL_WB words), then out with plain stores */
            const uint32_t wlo = m0 == 0 ? 0u : pos >> 5, whi = (pos + T + 31u) >> 5;
            if (whi + 2u > cap_words) over = true;             /* uniform */
            for (uint32_t b0 = wlo; b0 < whi && !over; b0 += SPL_WB) {
                const uint32_t n = min((uint32_t)SPL_WB, whi - b0);
                for (uint32_t i = (uint32_t)t; i < n; i += DT)
                    L.wbuf[i] = (b0 == wlo && i == 0 && m0 > 0) ? L.carry : 0u;
                __syncthreads();
                if (m0 == 0 && b0 == 0 && t == 0) {
                    OrSink<LdsWin> hs{LdsWin{L.wbuf, 0u, n}, 0, 0, 0};
                    hs.start(0);
                    emit_slice_header(hs, c);
                    hs.finish();
                }
                const uint32_t a0 = pos + off;
                if (coded && a0 < 32u * (b0 + n) && a0 + cs.n > 32u * b0) {
                    OrSink<LdsWin> sk{LdsWin{L.wbuf, b0, n}, 0, 0, 0};
                    sk.start(a0);
                    code_mb(sk);
                    sk.finish();
                }
                __syncthreads();
                /* the words final here (all but a last one the next window
                 * still ORs into): their 03 insertions, the last non-zero byte
                 * before each from a block max-scan and lnzb */
                const uint32_t nfin = (b0 + n == whi && ((pos + T) & 31u)) ? n - 1u : n;
                for (uint32_t c0 = 0; c0 < nfin; c0 += DT) {
                    const uint32_t i = c0 + (uint32_t)t;
                    const uint32_t wv = i < nfin ? L.wbuf[i] : 0u;
                    int ex, tot;
                    block_excl_max(wv ? (int)(4u * (b0 + i)) + last_nz_byte(wv) : -1, L.wmax, ex, tot);
                    int prev = max(ex, lnzb);
                    if (i < nfin) my_ep += ep_word(wv, 4u * (b0 + i), 0xffffffffu, prev, eplist, &L.ep_n);
                    lnzb = max(lnzb, tot);
                }
                for (uint32_t i = (uint32_t)t; i < n; i += DT) out[b0 + i] = __builtin_bswap32(L.wbuf[i]);
                if (b0 + n == whi && t == 0) L.carry = ((pos + T) & 31u) ? L.wbuf[n - 1] : 0u;
                __syncthreads();
            }
        }
        pos += T;
        last = max(last, cmax);
        if (over) break;
    }
    uint32_t run_bits = 0;
    if (last < nmb - 1) {
        CountSink cc{0};
        put_ue(cc, (uint32_t)(nmb - 1 - last));
        run_bits = cc.n;
    }
    const uint32_t total = pos + run_bits + 1u;     /* + rbsp_stop_one_bit */
    const int last_end = last;
    {
        const uint32_t nw = (total + 31u) >> 5;
        over |= nw + 2u > cap_words;
        if (my_bad) atomicOr(&L.bad, 1);
        if (my_ref_bad) atomicOr(&L.bad, 2);
        __syncthreads();
        const int bad = L.bad;
        if (over || bad) {
            if (t == 0) {
                DF->ep = 0;
                DF->err = over ? 1u : (bad & 1 ? 4u : 8u);
                if (over) atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_DYN);
                else if (bad & 1) atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_HINT);
                else {
                    atomicOr((unsigned int *)&S->err, SCROLL_DEVERR_SPLICE);
                    spf[fi].stage_status = SCROLL_SPLICE_ERR_REF;
                }
            }
            return;
        }
    }
    /* trailing skipped MBs, rbsp_stop_one_bit, alignment zeros, after the
     * carried word; the word after the last (the EP scan's look-ahead) 0 */
    const uint32_t nbytes = (total + 7u) >> 3;
    if (t == 0) {                                   /* the window buffer is free */
        const uint32_t w0 = pos >> 5;
        L.wbuf[0] = L.carry;
        L.wbuf[1] = 0u;
        OrSink<LdsWin> sk{LdsWin{L.wbuf, w0, 2u}, 0, 0, 0};
        sk.start(pos);
        if (run_bits) put_ue(sk, (uint32_t)(nmb - 1 - last_end));
        sk.put(1, 1);
        sk.finish();
        out[w0] = __builtin_bswap32(L.wbuf[0]);
        out[w0 + 1] = __builtin_bswap32(L.wbuf[1]);
        if (w0 + 2u <= ((total + 31u) >> 5)) out[w0 + 2] = 0u;
        int prev = lnzb;                            /* the last words' insertions (bytes < nbytes) */
        my_ep += ep_word(L.wbuf[0], 4u * w0, nbytes, prev, eplist, &L.ep_n);
        my_ep += ep_word(L.wbuf[1], 4u * (w0 + 1u), nbytes, prev, eplist, &L.ep_n);
    }
    uint32_t ex, tot;
    block_excl_sum(my_ep, L.wsum, ex, tot);
    if (t == 0) {
        DF->rbsp_bytes = nbytes;
        DF->ep = tot;
        DF->err = 0u;
    }
}

}  // namespace

int splice_launch_parse(hipStream_t hs, int n, int ymax, const int32_t *list, SpliceFrame *spf,
                        SpliceUnit *units, int32_t *lanes, size_t nslots, const DevStream *st, int ld_fr,
                        uint32_t *rbsp, SpliceMbRec *rec)
{
    if (n <= 0) return 0;
    const dim3 gy(n, (unsigned)std::max(1, std::min(ymax, 64)));
    hipLaunchKernelGGL(k_splice_units, dim3(n), dim3(DT), 0, hs, n, list, spf, units, lanes);
    hipLaunchKernelGGL(k_splice_unesc, gy, dim3(64), 0, hs, n, list, spf, units, rbsp);
    const unsigned lw = (unsigned)std::min<size_t>((nslots + LANE_ACTIVE - 1) / LANE_ACTIVE, 16384);
    hipLaunchKernelGGL(k_splice_lanes, dim3(std::max(lw, 1u)), dim3(64 * LANE_WAVES), 0, hs, list, spf, units, lanes, st,
                       ld_fr, rbsp, rec);
    hipLaunchKernelGGL(k_splice_parse, gy, dim3(64), 0, hs, n, list, spf, units, st, ld_fr, rbsp, rec);
    hipLaunchKernelGGL(k_splice_fix, dim3(n), dim3(64), 0, hs, n, list, spf, units, rec, lanes);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int splice_launch_stage(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                        int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                        const HintFrame *hf, const ScrollHintRect *pool, SpliceFrame *spf,
                        const SpliceMbRec *rec, const uint32_t *rbsp, uint8_t *stage,
                        uint64_t slot_bytes)
{
    if (nframes <= 0 || S <= 0) return 0;
    hipLaunchKernelGGL(k_splice_stage, dim3(nframes, S), dim3(DT), 0, hs, st, nal, ld_nal, pend,
                       dfr, ld_fr, hf, pool, spf, rec, rbsp, stage, slot_bytes);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t splice_slot_bound(int mbw, int mbh, int w, int h, size_t nal_bytes)
{
    /* header <= 1024 bits; every MB head <= 128 bits; a spliced MB adds its
     * body bits (<= the slice's) + 26 coeff_tokens (<= 16 bits each) +
     * cbp / mb_qp_delta (<= 24 bits) + a partitioned head (mb_type, 4
     * sub_mb_types, 4 ref_idx <= 64 bits; 16 mvd pairs <= 2 x 33 bits each) */
    const size_t bits = 1024 + (size_t)mbw * mbh * 128 + 8 * nal_bytes +
                        (size_t)w * h * (26 * 16 + 24 + 64 + 16 * 66) + 64;
    return ((bits / 8 + 64 + DYN_OVF_BYTES) + 255) & ~(size_t)255;
}
