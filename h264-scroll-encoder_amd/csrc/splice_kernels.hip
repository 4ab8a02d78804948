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

/* One wave parses one slice.  The slice is a sequential bit string, so the
 * parse itself is wave-uniform (scalar values, no divergence): the bit window
 * is 64 RBSP words held one per lane (readlane at the uniform bit position),
 * every VLC is matched by all lanes at once (lane e tests table entry e,
 * ballot), lane j keeps piece j's record fields, and the neighbour context
 * (motion of the two rows above, TotalCoeffs of the row above) sits in LDS. */
constexpr int PARSE_MAXW = 240;          /* external picture width limit (MBs) */

struct WRd {
    const uint32_t *w;
    uint32_t nw, nbits, p, base;
    uint32_t win;                        /* word base + lane */
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
    /* the 32 bits at p: words k, k + 1 of the window by readlane (scalar),
     * joined by a 64-bit scalar shift */
    __device__ inline uint32_t peek32()
    {
        uint32_t k = (p >> 5) - base;
        if (k >= 63u) {
            fill(p >> 5);
            k = 0;
        }
        const uint32_t a = (uint32_t)__builtin_amdgcn_readlane(win, k);
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(win, k + 1);
        const uint64_t ab = (uint64_t)a << 32 | b;
        return (uint32_t)((ab << (p & 31u)) >> 32);
    }
    __device__ inline uint32_t peek(int n) { return n ? peek32() >> (32 - n) : 0u; }
    __device__ inline void skip(int n) { p += (uint32_t)n; }
    __device__ inline bool over() const { return p > nbits; }
    __device__ inline uint32_t u(int n)
    {
        const uint32_t v = peek(n);
        skip(n);
        return v;
    }
    __device__ inline uint32_t ue()
    {
        const uint32_t x = peek32();
        if (!x) {
            bad = true;
            return 0;
        }
        const int z = __clz((int)x);
        if (z < 16) {                    /* the whole code in x */
            skip(2 * z + 1);
            return (x >> (31 - 2 * z)) - 1u;
        }
        skip(z);
        return u(z + 1) - 1u;
    }
    __device__ inline int32_t se()
    {
        const uint32_t k = ue();
        return (k & 1u) ? (int32_t)((k + 1u) >> 1) : -(int32_t)(k >> 1);
    }
};

/* first lane of a ballot, -1 if none */
__device__ inline int first_lane(uint64_t m) { return m ? __builtin_ctzll(m) : -1; }

/* The CAVLC tables in registers, lane e holding entry e of each (packed
 * len << 8 | bits, two 16-bit entries per register): a VLC match is then a
 * few VALU operations and a ballot, no memory access */
struct LaneTabs {
    uint32_t ct01, ct2d;          /* coeff_token nC 0-1 | 2-3 ; nC 4-7 | chroma DC, entry e */
    uint32_t cx01, cx2;           /* entries 64 + e (lanes 0..3)                             */
    /* total_zeros rows 2k | 2k+1, entry (total_zeros) e -- separate
     * registers: an array indexed by the row would live in scratch */
    uint32_t tz0, tz1, tz2, tz3, tz4, tz5, tz6, tz7;
    uint32_t tzd01, tzd2;         /* chroma DC total_zeros rows 0 | 1, 2                      */
    uint32_t rb0, rb1, rb2, rb3;  /* run_before rows 2k | 2k+1, entry (run) e                 */
    uint32_t cbp;                 /* coded_block_pattern -> codeNum, entry e < 48            */
};

__device__ inline uint32_t pk(int len, int bits) { return len ? (uint32_t)(len << 8 | bits) : 0u; }

__device__ inline LaneTabs lane_tabs()
{
    const int e = threadIdx.x & 63;
    LaneTabs T;
    T.ct01 = pk(SPT.ct_len[0][e], SPT.ct_bits[0][e]) | pk(SPT.ct_len[1][e], SPT.ct_bits[1][e]) << 16;
    T.ct2d = pk(SPT.ct_len[2][e], SPT.ct_bits[2][e]) |
             (e < 20 ? pk(SPT.ctdc_len[e], SPT.ctdc_bits[e]) << 16 : 0u);
    const int x = 64 + (e & 3);
    T.cx01 = e < 4 ? pk(SPT.ct_len[0][x], SPT.ct_bits[0][x]) | pk(SPT.ct_len[1][x], SPT.ct_bits[1][x]) << 16 : 0u;
    T.cx2 = e < 4 ? pk(SPT.ct_len[2][x], SPT.ct_bits[2][x]) : 0u;
    auto tzp = [e](int k) {
        const int r0 = 2 * k, r1 = 2 * k + 1;
        const uint32_t lo = e < 16 ? pk(SPT.tz_len[r0][e & 15], SPT.tz_bits[r0][e & 15]) : 0u;
        const uint32_t hi = e < 16 && r1 < 15 ? pk(SPT.tz_len[r1][e & 15], SPT.tz_bits[r1][e & 15]) : 0u;
        return lo | hi << 16;
    };
    T.tz0 = tzp(0);
    T.tz1 = tzp(1);
    T.tz2 = tzp(2);
    T.tz3 = tzp(3);
    T.tz4 = tzp(4);
    T.tz5 = tzp(5);
    T.tz6 = tzp(6);
    T.tz7 = tzp(7);
    T.tzd01 = e < 4 ? pk(SPT.tzdc_len[0][e & 3], SPT.tzdc_bits[0][e & 3]) |
                          pk(SPT.tzdc_len[1][e & 3], SPT.tzdc_bits[1][e & 3]) << 16 : 0u;
    T.tzd2 = e < 4 ? pk(SPT.tzdc_len[2][e & 3], SPT.tzdc_bits[2][e & 3]) : 0u;
    auto rbp = [e](int k) {
        const int r0 = 2 * k, r1 = 2 * k + 1;
        const uint32_t lo = e < 15 ? pk(SPT.rb_len[r0][e % 15], SPT.rb_bits[r0][e % 15]) : 0u;
        const uint32_t hi = e < 15 && r1 < 7 ? pk(SPT.rb_len[r1][e % 15], SPT.rb_bits[r1][e % 15]) : 0u;
        return lo | hi << 16;
    };
    T.rb0 = rbp(0);
    T.rb1 = rbp(1);
    T.rb2 = rbp(2);
    T.rb3 = rbp(3);
    T.cbp = e < 48 ? SPT.cbp_code[e] : 0xffffu;
    return T;
}

/* does the 16-bit lookahead x start with the packed code v? */
__device__ inline bool code_hit(uint32_t v, uint32_t x)
{
    const uint32_t len = (v >> 8) & 255u;
    return len && (x >> (16u - len)) == (v & 255u);
}

/* the ballot's entry, its packed code from the lane that holds it */
__device__ inline int match(uint32_t v, uint32_t x, uint32_t &len)
{
    const int e = first_lane(__ballot(code_hit(v, x)));
    if (e >= 0) len = (__builtin_amdgcn_readlane(v, e) >> 8) & 255u;
    return e;
}

/* 16-bit half h (uniform) of a packed register */
__device__ inline uint32_t half(uint32_t v, int h) { return h ? v >> 16 : v & 0xffffu; }

/* coeff_token (9.2.1): lane e tests entry e (4 * TotalCoeff + TrailingOnes) */
__device__ __attribute__((always_inline)) inline bool wrd_token(WRd &r, const LaneTabs &T, int nC, int &tc, int &t1)
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
    const uint32_t x = r.peek(16);
    const int tb = nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
    const uint32_t v = half(tb < 2 ? T.ct01 : T.ct2d, tb & 1);
    uint32_t len = 0;
    int e = match(v, x, len);
    if (e < 0 && tb != 3) {
        const uint32_t vx = half(tb < 2 ? T.cx01 : T.cx2, tb & 1);
        const int e2 = match(vx, x, len);
        e = e2 < 0 ? -1 : 64 + e2;
    }
    if (e < 0) return false;
    r.skip((int)len);
    tc = e >> 2;
    t1 = e & 3;
    return true;
}

/* the body of a block (9.2.2-9.2.4), consumed, not kept */
__device__ __attribute__((always_inline)) inline bool wrd_body(WRd &r, const LaneTabs &T, int tc, int t1, int maxc)
{
    const int lane = threadIdx.x & 63;
    if (tc == 0) return true;
    r.skip(t1);
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int k = t1; k < tc; ++k) {
        const uint32_t x = r.peek32();
        const int prefix = x ? __clz((int)x) : 32;
        if (prefix > 15) return false;                       /* High profiles only */
        r.skip(prefix + 1);
        int ssize = sl;
        if (prefix == 14 && sl == 0) ssize = 4;
        if (prefix >= 15) ssize = prefix - 3;
        int code = min(prefix, 15) << sl;
        if (ssize) code += (int)r.u(ssize);
        if (prefix >= 15 && sl == 0) code += 15;
        if (k == t1 && t1 < 3) code += 2;
        const int a = (code + 2) >> 1;                       /* |level| */
        if (sl == 0) sl = 1;
        if (a > (3 << (sl - 1)) && sl < 6) sl++;
    }
    int zl = 0;
    if (tc < maxc) {
        const uint32_t x = r.peek(16);
        const int row = tc - 1;
        uint32_t v;
        if (maxc == 4) {
            v = half(row < 2 ? T.tzd01 : T.tzd2, row & 1);
        } else {
            const int q = row >> 1;       /* uniform: a select tree, no indexing */
            const uint32_t w01 = q & 1 ? T.tz1 : T.tz0, w23 = q & 1 ? T.tz3 : T.tz2;
            const uint32_t w45 = q & 1 ? T.tz5 : T.tz4, w67 = q & 1 ? T.tz7 : T.tz6;
            const uint32_t w03 = q & 2 ? w23 : w01, w47 = q & 2 ? w67 : w45;
            v = half(q & 4 ? w47 : w03, row & 1);
        }
        if (lane > maxc - tc) v = 0;
        uint32_t len = 0;
        const int tz = match(v, x, len);
        if (tz < 0) return false;
        r.skip((int)len);
        zl = tz;
    }
    for (int k = 0; k < tc - 1 && zl > 0; ++k) {
        const uint32_t x = r.peek(16);
        const int zi = min(zl, 7) - 1;
        const int q = zi >> 1;
        const uint32_t w01 = q & 1 ? T.rb1 : T.rb0, w23 = q & 1 ? T.rb3 : T.rb2;
        uint32_t v = half(q & 2 ? w23 : w01, zi & 1);
        if (lane > zl) v = 0;
        uint32_t len = 0;
        const int run = match(v, x, len);
        if (run < 0) return false;
        r.skip((int)len);
        zl -= run;
    }
    return true;
}

/* lane j: piece j of the MB being parsed */
struct PieceOut {
    uint32_t tc, t1, off, len;
};

/* one residual block: coeff_token, then the body; lane pi keeps the fields */
__device__ __attribute__((always_inline)) inline bool wrd_piece(WRd &r, const LaneTabs &T, int pi,
                                                                int nC, int maxc, PieceOut &po)
{
    int tc, t1;
    if (!wrd_token(r, T, nC, tc, t1) || tc > maxc) return false;
    const uint32_t p0 = r.p;
    if (!wrd_body(r, T, tc, t1, maxc)) return false;
    if ((int)(threadIdx.x & 63) == pi) {
        po.tc = (uint32_t)tc;
        po.t1 = (uint32_t)t1;
        po.off = p0;
        po.len = r.p - p0;
    }
    return true;
}

/* nC of piece pi from the TotalCoeffs of this MB (lanes' cur), the MB to the
 * left and the MB above (-1: unavailable at the picture edge) */
__device__ __attribute__((always_inline)) inline int nc_at(int pi, uint32_t cur, uint32_t left,
                                                           uint32_t top, int x, int y)
{
    int nA, nB;
    if (pi < 16) {
        const int bx = pi & 3, by = pi >> 2;
        nA = bx ? (int)__builtin_amdgcn_readlane(cur, pi - 1)
                : (x ? (int)__builtin_amdgcn_readlane(left, pi + 3) : -1);
        nB = by ? (int)__builtin_amdgcn_readlane(cur, pi - 4)
                : (y ? (int)__builtin_amdgcn_readlane(top, pi + 12) : -1);
    } else {
        const int k = (pi - 18) & 3, bx = k & 1, by = k >> 1;
        nA = bx ? (int)__builtin_amdgcn_readlane(cur, pi - 1)
                : (x ? (int)__builtin_amdgcn_readlane(left, pi + 1) : -1);
        nB = by ? (int)__builtin_amdgcn_readlane(cur, pi - 2)
                : (y ? (int)__builtin_amdgcn_readlane(top, pi + 2) : -1);
    }
    return nc2(nA, nB);
}

/* wave-uniform (ref, mv) */
struct UMv {
    int ref, mx, my;
};

struct ParseLds {
    int32_t mref[2][PARSE_MAXW], mmx[2][PARSE_MAXW], mmy[2][PARSE_MAXW];  /* rows y-1, y by parity */
    uint8_t tcrow[PARSE_MAXW][SPLICE_PIECES];                              /* TotalCoeffs, row above */
};

__global__ __launch_bounds__(64) void k_splice_parse(int n, const int32_t *__restrict__ list,
                                                     SpliceFrame *__restrict__ spf,
                                                     const DevStream *__restrict__ st, int ld_fr,
                                                     uint32_t *__restrict__ rbsp,
                                                     SpliceMbRec *__restrict__ recs)
{
    __shared__ ParseLds L;
    const int i = blockIdx.x, lane = threadIdx.x;
    if (i >= n) return;
    const int idx = list[i];
    SpliceFrame *F = spf + idx;
    const DevStream S = st[idx / ld_fr];
    const uint8_t *p = F->nal;
    uint32_t len = F->nal_len;
    int status = SCROLL_SPLICE_ERR_NAL;
    if (len >= 4 && !p[0] && !p[1] && !p[2] && p[3] == 1) {
        p += 4;
        len -= 4;
    } else if (len >= 3 && !p[0] && !p[1] && p[2] == 1) {
        p += 3;
        len -= 3;
    }
    SpliceMbRec *rec = recs + F->rec_first;
    const int W = F->w, H = F->h, nmb = W * H;
    if (len < 2 || (p[0] & 0x80) || (p[0] & 31) != 1 || W > PARSE_MAXW) {
        if (lane == 0) F->status = len >= 2 && W > PARSE_MAXW ? SCROLL_SPLICE_ERR_HEADER : status;
        return;
    }
    const int ref_idc = (p[0] >> 5) & 3;
    /* emulation prevention bytes out (7.4.1): byte i of the payload goes
     * unless it is 03 after two zero bytes; 4 bytes per lane per pass, the
     * output index by a wave prefix count; bytes land MSB-first in words
     * (byte k at byte address k ^ 3) */
    uint32_t *o = rbsp + F->rbsp_word;
    const uint32_t nwmax = (len + 3u) / 4u + 2u;   /* = the host's region (splice_upload) */
    for (uint32_t k = (uint32_t)lane; k < nwmax; k += 64) o[k] = 0u;
    __syncthreads();
    uint8_t *ob = reinterpret_cast<uint8_t *>(o);
    uint32_t nb = 0;
    for (uint32_t c0 = 1; c0 < len; c0 += 256) {
        uint32_t keep = 0, cnt = 0;
        uint8_t by[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t k = c0 + 4u * (uint32_t)lane + (uint32_t)q;
            by[q] = k < len ? p[k] : 0;
            const bool ep = k < len && k >= 3 && by[q] == 3 && p[k - 1] == 0 && p[k - 2] == 0;
            const bool kp = k < len && !ep;
            keep |= kp ? 1u << q : 0u;
            cnt += kp ? 1u : 0u;
        }
        const uint32_t incl = wave_incl_sum(cnt, lane);
        uint32_t at = nb + incl - cnt;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (keep & (1u << q)) {
                ob[at ^ 3u] = by[q];
                at++;
            }
        nb += __builtin_amdgcn_readlane(incl, 63);
    }
    __syncthreads();
    nb = __builtin_amdgcn_readfirstlane(nb);
    WRd r{o, (nb + 3u) >> 2, 8u * nb, 0, 0, 0, false};
    r.fill(0);
    const LaneTabs T = lane_tabs();

    status = SCROLL_SPLICE_ERR_HEADER;
    int nrefs = 2;                         /* the composer's PPS (h264_writer.c:114) */
    int qp = 0;
    if (r.ue() != 0) goto done;                                    /* first_mb_in_slice */
    {
        const uint32_t stype = r.ue();
        if (stype != 0 && stype != 5) goto done;
    }
    if (r.ue() != 0) goto done;                                    /* pps id */
    r.skip(S.log2_mfn);
    if (S.poc_type == 0) r.skip(S.log2_poc);
    if (r.u(1)) {
        const uint32_t k = r.ue();
        if (k > 31) goto done;
        nrefs = (int)k + 1;
    }
    if (r.u(1)) {                          /* list modification: the composed list only */
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
    if (ref_idc && r.u(1)) {                                       /* MMCO */
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
    qp = 26 + r.se();
    if (qp < 0 || qp > 51) goto done;
    if (S.deblock && r.ue() != 1) goto done;
    status = SCROLL_SPLICE_ERR_SYNTAX;
    if (r.bad || r.over()) goto done;
    {
        int m = 0, qp_c = 26;
        const Mv none{-1, 0, 0};
        uint32_t tc_left = 0;              /* lane j: TotalCoeff of piece j, MB to the left */
        Mv left{-1, 0, 0};
        /* motion of MB (x, y) from the LDS rows */
        auto ctx = [&](int x, int y, Mv &A, Mv &B, Mv &C) {
            const int py = (y - 1) & 1;
            A = x ? left : none;
            auto at = [&](int xx) { return Mv{L.mref[py][xx], L.mmx[py][xx], L.mmy[py][xx]}; };
            B = y ? at(x) : none;
            C = y ? (x + 1 < W ? at(x + 1) : (x ? at(x - 1) : none)) : none;
        };
        auto finish = [&](int x, int y, const Mv &me) {    /* context for the MBs to come */
            if (lane == 0) {
                L.mref[y & 1][x] = me.ref;
                L.mmx[y & 1][x] = me.mx;
                L.mmy[y & 1][x] = me.my;
            }
            left = me;
        };
        while (m < nmb) {
            const uint32_t run = r.ue();
            if (r.bad || r.over() || run > (uint32_t)(nmb - m)) goto done;
            for (uint32_t k = 0; k < run; ++k, ++m) {             /* P_Skip */
                const int x = m % W, y = m / W;
                Mv A, B, C;
                ctx(x, y, A, B, C);
                int px, py;
                pskip_mv(x, y, A, B, C, px, py);
                SpliceMbRec *R = rec + m;
                if (lane == 0) {
                    R->ref = 0;
                    R->cbp = 0;
                    R->qpd = 0;
                    R->mx = px;
                    R->my = py;
                    R->skip = 1;
                }
                if (lane < SPLICE_PIECES) {
                    R->tc[lane] = 0;
                    R->t1[lane] = 0;
                    R->blen[lane] = 0;
                    R->boff[lane] = 0;
                    L.tcrow[x][lane] = 0;
                }
                tc_left = 0;
                finish(x, y, Mv{0, px, py});
            }
            if (m == nmb) break;
            const int x = m % W, y = m / W;
            if (r.ue() != 0) {                                     /* mb_type */
                status = r.bad || r.over() ? SCROLL_SPLICE_ERR_SYNTAX : SCROLL_SPLICE_ERR_MBTYPE;
                goto done;
            }
            int ref = 0;
            if (nrefs == 2) ref = 1 - (int)r.u(1);
            else if (nrefs > 2) ref = (int)r.ue();
            const int dx = r.se(), dy = r.se();
            Mv A, B, C;
            ctx(x, y, A, B, C);
            int px, py;
            predict_spec(A, B, C, ref, px, py);
            const long long mx = (long long)px + dx, my = (long long)py + dy;
            const uint32_t code = r.ue();
            const uint64_t cm = __ballot(T.cbp == code);
            const int cbp = first_lane(cm);
            if (r.bad || r.over() || ref >= nrefs || cbp < 0 || mx < -SPLICE_MAX_MV || mx > SPLICE_MAX_MV ||
                my < -SPLICE_MAX_MV || my > SPLICE_MAX_MV)
                goto done;
            int qpd = 0;
            /* lane j: piece j of this MB */
            uint32_t my_tc = 0, my_t1 = 0, my_off = 0, my_len = 0;
            if (cbp) {
                const int dq = r.se();
                if (dq < -26 || dq > 25) goto done;
                qp = (qp + dq + 52) % 52;
                int d = qp - qp_c;                                 /* composed chain from 26 */
                if (d < -26) d += 52;
                if (d > 25) d -= 52;
                qpd = d;
                qp_c = qp;
                const uint32_t tc_top = y && lane < SPLICE_PIECES ? L.tcrow[x][lane] : 0u;
                PieceOut po{0, 0, 0, 0};
                for (int blk = 0; blk < 16; ++blk) {
                    if (!(cbp & (1 << (blk >> 2)))) continue;
                    const int pi = blk_raster16(blk);
                    if (!wrd_piece(r, T, pi, nc_at(pi, po.tc, tc_left, tc_top, x, y), 16, po)) goto done;
                }
                if (cbp >> 4) {
                    if (!wrd_piece(r, T, 16, -1, 4, po) || !wrd_piece(r, T, 17, -1, 4, po)) goto done;
                    if ((cbp >> 4) == 2)
                        for (int pi = 18; pi < 26; ++pi)
                            if (!wrd_piece(r, T, pi, nc_at(pi, po.tc, tc_left, tc_top, x, y), 15, po))
                                goto done;
                }
                my_tc = po.tc;
                my_t1 = po.t1;
                my_off = po.off;
                my_len = po.len;
            }
            SpliceMbRec *R = rec + m;
            if (lane == 0) {
                R->ref = (int16_t)ref;
                R->cbp = (uint8_t)cbp;
                R->qpd = (int8_t)qpd;
                R->mx = (int32_t)mx;
                R->my = (int32_t)my;
                R->skip = 0;
            }
            if (lane < SPLICE_PIECES) {
                R->tc[lane] = (uint8_t)my_tc;
                R->t1[lane] = (uint8_t)my_t1;
                R->blen[lane] = (uint16_t)my_len;
                R->boff[lane] = my_off;
                L.tcrow[x][lane] = (uint8_t)my_tc;
            }
            tc_left = my_tc;
            finish(x, y, Mv{ref, (int)mx, (int)my});
            ++m;
        }
        /* rbsp_slice_trailing_bits (+ zero bytes of a byte stream) */
        if (r.u(1) != 1u) goto done;
        if (r.p & 7u) {
            const int k = 8 - (int)(r.p & 7u);
            if (r.u(k)) goto done;
        }
        while (r.p < r.nbits)
            if (r.u(8)) goto done;
        if (!r.bad && !r.over()) status = SCROLL_SPLICE_OK;
    }
done:
    if (lane == 0) F->status = status;
}

/* ------------------------------------------------------------------------ */
/* k_splice_stage                                                            */
/* ------------------------------------------------------------------------ */
struct SpliceLds {
    int32_t fr[RING], fx[RING], fy[RING];   /* motion of MB m at m % RING */
    ScrollHintRect rc[SCROLL_HINT_MAX_RECTS];
    int32_t wo[8], wl[8], wv[8];
    uint32_t wsum[NW];
    int32_t wmax[NW];
    uint32_t ep_n;
    int32_t bad;
};

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

/* bits of one spliced MB after its head: cbp, mb_qp_delta, pieces */
template <class SK>
__device__ inline void splice_tail(SK &sk, const SpliceMbRec &mb, const uint8_t *L, const uint8_t *T,
                                   const uint32_t *rb)
{
    const int cbp = mb.cbp;
    put_ue(sk, SPT.cbp_code[cbp]);
    if (!cbp) return;
    put_se(sk, mb.qpd);
    auto piece = [&](int i, int nC) {
        uint32_t v;
        int len;
        coeff_token(SPT, mb.tc[i], mb.t1[i], nC, v, len);
        sk.put(v, len);
        const uint32_t q0 = mb.boff[i];
        const int bl = mb.blen[i];
        if constexpr (__is_same(SK, CountSink)) {
            sk.n += (uint32_t)bl;
        } else {
            for (int k = 0; k < bl; k += 32) {
                const int c = min(32, bl - k);
                sk.put(bits_at(rb, q0 + (uint32_t)k) >> (32 - c), c);
            }
        }
    };
    for (int blk = 0; blk < 16; ++blk)
        if (cbp & (1 << (blk >> 2))) {
            const int i = blk_raster16(blk);
            piece(i, piece_nc(i, mb.tc, L, T));
        }
    if (cbp >> 4) {
        piece(16, -1);
        piece(17, -1);
        if ((cbp >> 4) == 2)
            for (int i = 18; i < 26; ++i) piece(i, piece_nc(i, mb.tc, L, T));
    }
}

__constant__ uint8_t ZERO_TC[SPLICE_PIECES] = {};

__global__ __launch_bounds__(DT) void k_splice_stage(DevStream *__restrict__ st,
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
    if (!(H.mode & HINT_MODE_SPLICED)) return;                 /* k_hint_stage's frame */
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
    const int nr = min((int)H.n, SCROLL_HINT_MAX_RECTS);
    const int hmode = H.mode & 0xff;
    const bool pskip = hmode == SCROLL_HINT_PSKIP;
    const bool spec = hmode != SCROLL_HINT_EXACT;
    if (t == 0) {
        L.ep_n = 0;
        L.bad = 0;
    }
    if (t < 8) {
        L.wo[t] = pend[s].wo[t];
        L.wl[t] = pend[s].wl[t];
        L.wv[t] = pend[s].wv[t];
    }
    if (t < nr) L.rc[t] = pool[H.first + t];
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
    uint32_t total = 0;            /* bits: header + MBs (uniform) */
    int last_end = -1;
    /* sweep 0 counts, sweep 1 writes at the counted offsets */
    for (int sweep = 0; sweep < 2; ++sweep) {
        uint32_t pos = F0;
        int last = -1;             /* last coded MB before the window (uniform) */
        if (sweep == 1 && t == 0) {
            GSink hs{{out}, 0, 0, 0};
            hs.start(0);
            emit_slice_header(hs, c);
            hs.finish();
        }
        for (int m0 = 0; m0 < nmb; m0 += DT) {
            const int m = m0 + t;
            int x = 0, y = 0, k = -1;
            Mv me{0, 0, 0};
            if (m < nmb) {
                y = (int)div_m((uint32_t)m, m_mbw);
                x = m - y * mbw;
                if (x >= SF.x0 && x < SF.x0 + SF.w && y >= SF.y0 && y < SF.y0 + SF.h) {
                    k = (y - SF.y0) * SF.w + (x - SF.x0);
                    const SpliceMbRec &mb = rec[k];
                    me = Mv{mb.ref, mb.mx, mb.my};
                    const int wk = mb.ref - 2;
                    my_ref_bad |= !(mb.ref == 0 || mb.ref == 1 || (wk >= 0 && wk < c.nwp && L.wv[wk]));
                } else {
                    bool bad;
                    me = field(L.rc, L.wv, nr, x, y, lay, c.nwp, bad);
                    my_bad |= bad;
                }
                L.fr[m & (RING - 1)] = me.ref;
                L.fx[m & (RING - 1)] = me.mx;
                L.fy[m & (RING - 1)] = me.my;
            }
            __syncthreads();
            bool coded = false;
            int px = 0, py = 0;
            if (m < nmb) {
                auto at = [&](int q) { return Mv{L.fr[q & (RING - 1)], L.fx[q & (RING - 1)], L.fy[q & (RING - 1)]}; };
                const Mv none{-1, 0, 0};
                const Mv A = x > 0 ? at(m - 1) : none;
                const Mv B = y > 0 ? at(m - mbw) : none;
                const Mv C = y == 0 ? none : (x + 1 < mbw ? at(m - mbw + 1) : (x > 0 ? at(m - mbw - 1) : none));
                if (spec) {
                    int sx, sy;
                    pskip_mv(x, y, A, B, C, sx, sy);
                    coded = !pskip ||
                            !(me.ref == 0 && me.mx == sx && me.my == sy && (k < 0 || rec[k].cbp == 0));
                    predict_spec(A, B, C, me.ref, px, py);
                } else {
                    coded = true;
                    predict_ref(A, B, C, me.ref, px, py);
                }
            }
            int excl, cmax;
            block_excl_max(coded ? m : -1, L.wmax, excl, cmax);
            /* the MB's bits: head, then (spliced) cbp / qp / pieces */
            const uint8_t *Lt = nullptr, *Tt = nullptr;
            if (k >= 0) {
                Lt = x == 0 ? nullptr : (x > SF.x0 ? rec[k - 1].tc : ZERO_TC);
                Tt = y == 0 ? nullptr : (y > SF.y0 ? rec[k - SF.w].tc : ZERO_TC);
            }
            auto code_mb = [&](auto &sk) {
                put_ue(sk, (uint32_t)(m - max(excl, last) - 1));  /* mb_skip_run */
                sk.put(1, 1);                                      /* P_L0_16x16 */
                if (nrefs == 2) sk.put((uint32_t)(1 - (me.ref & 1)), 1);
                else if (nrefs > 2) put_ue(sk, (uint32_t)me.ref);
                put_se(sk, me.mx - px);
                put_se(sk, me.my - py);
                if (k >= 0) splice_tail(sk, rec[k], Lt, Tt, rb);
                else sk.put(1, 1);                                 /* coded_block_pattern 0 */
            };
            CountSink cs{0};
            if (coded) code_mb(cs);
            uint32_t off, T;
            block_excl_sum(cs.n, L.wsum, off, T);
            if (sweep == 1 && coded) {
                GSink sk{{out}, 0, 0, 0};
                sk.start(pos + off);
                code_mb(sk);
                sk.finish();
            }
            pos += T;
            last = max(last, cmax);
        }
        if (sweep == 0) {
            /* trailing skipped MBs, rbsp_stop_one_bit, alignment */
            uint32_t nb = pos + 1u;
            if (last < nmb - 1) {
                CountSink cc{0};
                put_ue(cc, (uint32_t)(nmb - 1 - last));
                nb += cc.n;
            }
            total = nb;
            last_end = last;
            const uint32_t nw = (nb + 31u) >> 5;
            const bool over = nw + 2u > cap_words;
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
            for (uint32_t q = (uint32_t)t; q < nw + 1u; q += DT) out[q] = 0u;
            __threadfence();
            __syncthreads();
        }
    }
    /* trailing run + stop bit (thread 0; positions from the count) */
    if (t == 0) {
        uint32_t run_bits = 0;
        if (last_end < nmb - 1) {
            CountSink cc{0};
            put_ue(cc, (uint32_t)(nmb - 1 - last_end));
            run_bits = cc.n;
        }
        GSink sk{{out}, 0, 0, 0};
        sk.start(total - 1u - run_bits);
        if (run_bits) put_ue(sk, (uint32_t)(nmb - 1 - last_end));
        sk.put(1, 1);
        sk.finish();
    }
    __threadfence();
    __syncthreads();
    /* emulation prevention: per word, the zero run before it from the last
     * non-zero byte (looked up backwards) */
    const uint32_t nbytes = (total + 7u) >> 3, nw = (nbytes + 3u) >> 2;
    uint32_t my_ep = 0;
    for (uint32_t jw = (uint32_t)t; jw < nw; jw += DT) {
        const uint32_t wv = __builtin_bswap32(__hip_atomic_load(&out[jw], __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT));
        int prev = -1;
        for (int jj = (int)jw - 1; jj >= 0; --jj) {
            const uint32_t pv = __builtin_bswap32(
                __hip_atomic_load(&out[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (pv) {
                prev = 4 * jj + last_nz_byte(pv);
                break;
            }
        }
        my_ep += ep_word(wv, 4u * jw, nbytes, prev, eplist, &L.ep_n);
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

int splice_launch_parse(hipStream_t hs, int n, const int32_t *list, SpliceFrame *spf,
                        const DevStream *st, int ld_fr, uint32_t *rbsp, SpliceMbRec *rec)
{
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_splice_parse, dim3(n), dim3(64), 0, hs, n, list, spf, st, ld_fr, rbsp,
                       rec);
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
     * cbp / mb_qp_delta (<= 24 bits) */
    const size_t bits = 1024 + (size_t)mbw * mbh * 128 + 8 * nal_bytes +
                        (size_t)w * h * (26 * 16 + 24) + 64;
    return ((bits / 8 + 64 + DYN_OVF_BYTES) + 255) & ~(size_t)255;
}
