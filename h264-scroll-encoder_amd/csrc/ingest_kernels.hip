/*
 * ingest_kernels.hip -- MI355X (gfx950) stream ingest (SURVEY.md §8f rows
 * 3-4): composer_init + composer_write_header for many new streams at once.
 * Reference path, per stream (src/composer.c:127-253):
 *   parse_reference_file(A), (B)   nal_parser_next (src/nal_parser.c:28-65),
 *                                  ebsp_to_rbsp (:67-88), parse_sps / parse_pps
 *   composer_write_header          SPS + PPS (h264_writer.c:49-127),
 *                                  h264_rewrite_idr_frame (:242-294) of A,
 *                                  h264_rewrite_as_non_idr_i_frame (:296-350) of B
 * whose heavy part is a bit-serial copy of the whole slice body behind a new
 * header (copy_bits, :228-240) and the NAL framing with emulation prevention.
 *
 *   k_ing_scan    grid over every byte of every reference file: the
 *                 positions of the 00 00 01 patterns (a handful per file)
 *   k_ing_stream  one workgroup per new stream: lane 0 walks the NAL units
 *                 (first SPS / PPS / IDR, the reference's stop rules) and
 *                 parses SPS, PPS and both slice headers through an
 *                 unescaping bit reader; then the workgroup streams each
 *                 slice body in 4 KB EBSP windows: removal flags (closed form
 *                 of ebsp_to_rbsp) -> scan -> RBSP ring in LDS -> output
 *                 bytes = constant bit shift behind the new header -> EP
 *                 insertion (closed form of rbsp_to_ebsp from the last
 *                 non-zero byte, max-scan) -> arena.  Kept for slices over
 *                 16 MB and SCROLL_INGEST_SERIAL.
 *   segmented     (the default, below k_ing_stream) the same parse in
 *                 k_ing_head, each slice body cut into 16 KB segments
 *                 over many workgroups: k_ing_seg<FUSED> (summary,
 *                 look-back placement and write in one pass; round 4's
 *                 k_ing_seg<SUMMARY>, k_ing_fix, k_ing_seg<WRITE_STAGED>
 *                 stay for comparison, SCROLL_INGEST_THREEPASS).
 * Bits: byte-identical to the reference's composer_write_header output
 * (tests/test_gpu_ingest.py against oracle/scroll_oracle.c, pinned by the
 * reference's golden header files).  Roofline: HBM (files in, header NALs
 * out), DESIGN.md §5.
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "engine.h"
#include "ingest_engine.h"
#include "scroll_device.h"
#include "stage_util.h"

using namespace scroll;
using namespace scroll::stage;

namespace {

constexpr int WINB = DT * 16;           /* EBSP bytes per window: 16 per lane      */
constexpr int RING = 4 * WINB;          /* RBSP ring (power of two)                */
constexpr int OCH = WINB;               /* output bytes per emit chunk: 16 per lane */
constexpr int OBUF = OCH + OCH / 2 + 64; /* one chunk after EP (<= 1.5x)           */
constexpr int SCAN_W = 4;               /* k_ing_scan: windows per workgroup        */

/* ---------------------------------------------------------------------- */
/* k_ing_scan                                                              */
/* ---------------------------------------------------------------------- */
/* The 16 bytes of the aligned 16-byte chunk at absolute address a, with the
 * dword before it and the dword after, for the byte-pattern rules (start
 * codes, emulation-prevention removal).  Lanes of a wave hold consecutive
 * chunks, so the neighbours come over lanes; the wave's end lanes load them.
 * Only chunks / dwords holding a byte of the file [lo, hi) are read: no load
 * leaves the pages of the file's bytes.  Every lane of the wave calls it. */
struct Chunk16 {
    uint32_t w[4];
    uint32_t prev, next;
    __device__ inline uint32_t b(int q) const                /* byte q, -4 <= q < 20 */
    {
        const uint32_t x = q < 0 ? prev : q >= 16 ? next : w[q >> 2];
        return (x >> (8 * ((q + 4) & 3))) & 255u;
    }
};

__device__ inline Chunk16 load_chunk16(const uint8_t *a, const uint8_t *lo, const uint8_t *hi)
{
    Chunk16 c;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (a < hi && a + 16 > lo) v = *reinterpret_cast<const uint4 *>(a);
    c.w[0] = v.x;
    c.w[1] = v.y;
    c.w[2] = v.z;
    c.w[3] = v.w;
    const int lane = threadIdx.x & 63;
    c.prev = __shfl_up(v.w, 1, 64);
    c.next = __shfl_down(v.x, 1, 64);
    if (lane == 0) c.prev = (a - 1 >= lo && a - 1 < hi) ? *reinterpret_cast<const uint32_t *>(a - 4) : 0u;
    if (lane == 63) c.next = (a + 16 >= lo && a + 16 < hi) ? *reinterpret_cast<const uint32_t *>(a + 16) : 0u;
    return c;
}

__device__ inline const uint8_t *align16_down(const uint8_t *p)
{
    return reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)15);
}

__device__ inline uint32_t hi_to_bits4(uint32_t h)          /* bit k: byte k */
{
    return (h >> 7 | h >> 14 | h >> 21 | h >> 28) & 0xfu;
}

/* bits [lo, hi) of 16 */
__device__ inline uint32_t range16(int64_t lo, int64_t hi)
{
    const uint32_t l = (uint32_t)min(max(lo, (int64_t)0), (int64_t)16), h = (uint32_t)min(max(hi, (int64_t)0), (int64_t)16);
    return h > l ? ((1u << h) - 1u) & ~((1u << l) - 1u) : 0u;
}

__device__ inline uint32_t range16_32(int32_t lo, int32_t hi)
{
    const uint32_t l = (uint32_t)min(max(lo, 0), 16), h = (uint32_t)min(max(hi, 0), 16);
    return h > l ? ((1u << h) - 1u) & ~((1u << l) - 1u) : 0u;
}

/* bit q: byte q of the chunk (file index i0 + q) is an emulation-prevention
 * byte (nal_parser.c:72: 03 after 00 00, before a byte <= 3).  Per dword:
 * its own test, the zero tests of the bytes one and two before and the <= 3
 * test of the byte after, lined up with alignbyte */
__device__ inline uint32_t ep_removed16(const Chunk16 &c)
{
    const uint32_t E3[4] = {zero_hi(c.w[0] ^ 0x03030303u), zero_hi(c.w[1] ^ 0x03030303u),
                            zero_hi(c.w[2] ^ 0x03030303u), zero_hi(c.w[3] ^ 0x03030303u)};
    if ((E3[0] | E3[1] | E3[2] | E3[3]) == 0) return 0;   /* no 03 byte: the common case */
    const uint32_t W[6] = {c.prev, c.w[0], c.w[1], c.w[2], c.w[3], c.next};
    uint32_t Z[5], L3[6];
#pragma unroll
    for (int k = 0; k < 5; ++k) Z[k] = zero_hi(W[k]);
#pragma unroll
    for (int k = 1; k < 6; ++k) L3[k] = zero_hi(W[k] & 0xfcfcfcfcu);
    uint32_t rm = 0;
#pragma unroll
    for (int k = 1; k < 5; ++k) {
        const uint32_t r = E3[k - 1] & __builtin_amdgcn_alignbyte(Z[k], Z[k - 1], 3u) &
                           __builtin_amdgcn_alignbyte(Z[k], Z[k - 1], 2u) &
                           __builtin_amdgcn_alignbyte(L3[k + 1], L3[k], 1u);
        rm |= hi_to_bits4(r) << (4 * (k - 1));
    }
    return rm;                          /* the caller masks file indices [2, n - 1) */
}

__global__ __launch_bounds__(DT) void k_ing_scan(const uint8_t *__restrict__ in,
                                                 const IngestFile *__restrict__ files,
                                                 IngestScan *__restrict__ scan)
{
    const int fi = blockIdx.y;
    const IngestFile F = files[fi];
    const uint8_t *d = in + F.off, *hi = d + F.size;
    const uint8_t *w0 = align16_down(d) + (size_t)blockIdx.x * (SCAN_W * WINB);
    if (w0 >= hi) return;                                             /* uniform over the block */
    Chunk16 c[SCAN_W];                                                /* all loads in flight first */
#pragma unroll
    for (int j = 0; j < SCAN_W; ++j) c[j] = load_chunk16(w0 + j * WINB + 16u * threadIdx.x, d, hi);
#pragma unroll
    for (int j = 0; j < SCAN_W; ++j) {
        const int64_t i0 = w0 + j * WINB + 16u * threadIdx.x - d;
        const uint32_t W[5] = {c[j].w[0], c[j].w[1], c[j].w[2], c[j].w[3], c[j].next};
        uint32_t Z[5], E1[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            Z[k] = zero_hi(W[k]);
            E1[k] = zero_hi(W[k] ^ 0x01010101u);
        }
        uint32_t sc = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t r = Z[k] & __builtin_amdgcn_alignbyte(Z[k + 1], Z[k], 1u) &
                               __builtin_amdgcn_alignbyte(E1[k + 1], E1[k], 2u);
            sc |= hi_to_bits4(r) << (4 * k);
        }
        sc &= range16(-i0, (int64_t)F.size - 2 - i0);
        while (sc) {                                                  /* nal_parser.c:16-18 */
            const int q = __builtin_ctz(sc);
            sc &= sc - 1;
            const uint32_t k = atomicAdd(&scan[fi].n, 1u);
            if (k < (uint32_t)ING_SC_MAX) scan[fi].pos[k] = (uint32_t)(i0 + q);
        }
    }
}

/* ---------------------------------------------------------------------- */
/* serial parsing (lane 0)                                                 */
/* ---------------------------------------------------------------------- */
/* bit reader over an EBSP payload that removes emulation-prevention bytes
 * as ebsp_to_rbsp does (src/nal_parser.c:67-88); reads past the end give 0
 * (the reference's bitreader, :104-113) */
struct EbspReader {
    const uint8_t *d;
    uint64_t n, i;                /* next EBSP byte */
    int zeros;
    uint32_t cur;                 /* current RBSP byte                       */
    int bit;                      /* bits of cur consumed, 8 = need a byte   */
    bool eof;
    uint64_t rbsp_pos;            /* RBSP bytes fetched                      */
    __device__ void init(const uint8_t *p, uint64_t size)
    {
        d = p;
        n = size;
        i = 0;
        zeros = 0;
        bit = 8;
        eof = false;
        rbsp_pos = 0;
        cur = 0;
    }
    __device__ bool next_byte(uint32_t &v)
    {
        while (i < n) {
            const uint32_t b = d[i];
            if (zeros >= 2 && b == 3 && i + 1 < n && d[i + 1] <= 3) {
                zeros = 0;
                i++;
                continue;
            }
            zeros = b ? 0 : zeros + 1;
            i++;
            v = b;
            rbsp_pos++;
            return true;
        }
        return false;
    }
    __device__ uint32_t u1()
    {
        if (bit == 8) {
            if (eof || !next_byte(cur)) {
                eof = true;
                return 0;
            }
            bit = 0;
        }
        return (cur >> (7 - bit++)) & 1u;
    }
    __device__ uint32_t u(int k)
    {
        uint32_t v = 0;
        for (int q = 0; q < k; ++q) v = (v << 1) | u1();
        return v;
    }
    __device__ uint32_t ue()                 /* h264_writer.c:164-174 */
    {
        int lz = 0;
        while (u1() == 0 && lz < 32) lz++;
        if (lz == 0) return 0;
        return (1u << lz) - 1u + u(lz);
    }
    __device__ int32_t se()
    {
        const uint32_t k = ue();
        return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
    }
    /* RBSP bit position of the next bit to read */
    __device__ uint64_t pos() const { return 8 * rbsp_pos - (uint64_t)(bit == 8 ? 0 : 8 - bit); }
};

struct NalRange {
    uint64_t off, n;              /* payload after the NAL header byte, EBSP bytes */
    int found;
};

/* parse_reference_file's NAL walk (src/composer.c:62-108 over
 * nal_parser_next, src/nal_parser.c:28-65): first SPS / PPS / IDR */
__device__ int walk_nals(const uint8_t *d, uint64_t n, uint32_t *pos, int np, NalRange &sps,
                         NalRange &pps, NalRange &idr)
{
    for (int a = 1; a < np; ++a) {                         /* sort the pattern positions */
        const uint32_t v = pos[a];
        int b = a - 1;
        while (b >= 0 && pos[b] > v) {
            pos[b + 1] = pos[b];
            b--;
        }
        pos[b + 1] = v;
    }
    sps.found = pps.found = idr.found = 0;
    for (int k = 0; k < np; ++k) {
        const uint64_t s = (uint64_t)pos[k] + 3;          /* after 00 00 01 */
        uint64_t e = k + 1 < np ? (uint64_t)pos[k + 1] : n;
        while (e > s && d[e - 1] == 0) e--;                /* :46-48 */
        if (e <= s) break;                                 /* :50-53: the parser stops */
        const int type = d[s] & 31;
        NalRange r{s + 1, e - s - 1, 1};
        if (type == 7 && !sps.found) sps = r;
        else if (type == 8 && !pps.found) pps = r;
        else if (type == 5 && !idr.found) idr = r;
    }
    return sps.found && pps.found && idr.found ? 0 : -1;
}

struct SpsInfo {
    int w, h, l2f, poct, l2p;
};

__device__ int parse_sps(const uint8_t *p, uint64_t n, SpsInfo &o)   /* nal_parser.c:137-222 */
{
    EbspReader r;
    r.init(p, n);
    const int prof = (int)r.u(8);
    r.u(8);
    r.u(8);
    r.ue();
    if (prof == 100 || prof == 110 || prof == 122 || prof == 244 || prof == 44 || prof == 83 ||
        prof == 86 || prof == 118 || prof == 128 || prof == 138 || prof == 139 || prof == 134) {
        if (r.ue() == 3) r.u1();
        r.ue();
        r.ue();
        r.u1();
        if (r.u1()) return -1;                              /* scaling matrices */
    }
    o.l2f = (int)r.ue() + 4;
    o.poct = (int)r.ue();
    o.l2p = 0;
    if (o.poct == 0) o.l2p = (int)r.ue() + 4;
    else if (o.poct == 1) return -1;
    r.ue();
    r.u1();
    const int wm = (int)r.ue() + 1;
    int hm = (int)r.ue() + 1;
    if (!r.u1()) {
        r.u1();
        hm *= 2;
    }
    o.w = wm * 16;
    o.h = hm * 16;
    return 0;
}

__device__ int parse_pps(const uint8_t *p, uint64_t n, int &nref, int &dbf)   /* :224-276 */
{
    EbspReader r;
    r.init(p, n);
    r.ue();
    r.ue();
    r.u1();
    r.u1();
    if (r.ue() > 0) return -1;                             /* slice groups */
    nref = (int)r.ue();
    r.ue();
    r.u1();
    r.u(2);
    r.ue();
    r.ue();
    r.ue();
    dbf = (int)r.u1();
    return 0;
}

struct SliceHdr {
    uint64_t mb_start;            /* RBSP bit where the MB data begins */
    int32_t qpd, alpha, beta;
    uint32_t dbf;
};

/* parse_idr_slice_header (h264_writer.c:194-226) with the parse config */
__device__ void parse_idr(const uint8_t *p, uint64_t n, const SpsInfo &pc, int pdbf, SliceHdr &h)
{
    EbspReader r;
    r.init(p, n);
    r.ue();
    r.ue();
    r.ue();
    r.u(pc.l2f);
    r.ue();
    if (pc.poct == 0) r.u(pc.l2p);
    r.u1();
    r.u1();
    h.qpd = r.se();
    h.dbf = 0;
    h.alpha = h.beta = 0;
    if (pdbf) {
        h.dbf = r.ue();
        if (h.dbf != 1) {
            h.alpha = r.se();
            h.beta = r.se();
        }
    }
    h.mb_start = r.pos();
}

/* a small MSB-first bit string (headers: <= 256 bits) */
struct SmallBits {
    uint32_t w[8];
    int n;
    __device__ void clear()
    {
        for (int k = 0; k < 8; ++k) w[k] = 0;
        n = 0;
    }
    __device__ void put(uint32_t v, int k)       /* k <= 32 */
    {
        for (int q = k - 1; q >= 0; --q) {
            if ((v >> q) & 1u) w[n >> 5] |= 0x80000000u >> (n & 31);
            n++;
        }
    }
    __device__ uint32_t byte(int o) const { return (w[o >> 2] >> (24 - 8 * (o & 3))) & 255u; }
};

/* write-side headers of the composer (log2_max_frame_num 4, poc type 2:
 * src/composer.c:199-203).  rewrite_idr :262-283, rewrite_non_idr :314-339 */
__device__ void slice_header(SmallBits &b, bool idr, int dbf, const SliceHdr &h)
{
    b.clear();
    put_ue(b, 0);
    put_ue(b, 7);                                          /* SLICE_TYPE_I_ALL */
    put_ue(b, 0);
    if (idr) {
        b.put(0, 4);                                       /* frame_num 0 */
        put_ue(b, 0);                                      /* idr_pic_id */
        b.put(0, 1);
        b.put(1, 1);                                       /* long_term_reference_flag */
    } else {
        b.put(1, 4);                                       /* frame_num 1 */
        b.put(1, 1);                                       /* adaptive marking */
        put_ue(b, 4);
        put_ue(b, 2);
        put_ue(b, 6);
        put_ue(b, 1);
        put_ue(b, 0);
    }
    put_se(b, h.qpd);
    if (dbf) {
        put_ue(b, h.dbf);
        if (h.dbf != 1) {
            put_se(b, h.alpha);
            put_se(b, h.beta);
        }
    }
}

/* h264_generate_sps / _pps (h264_writer.c:49-127) */
__device__ void gen_sps(SmallBits &b, int w, int h)
{
    b.clear();
    b.put(66, 8);
    b.put(0xc0, 8);
    b.put(40, 8);
    put_ue(b, 0);
    put_ue(b, 0);
    put_ue(b, 2);
    put_ue(b, 2 + 8);
    b.put(0, 1);
    put_ue(b, (uint32_t)(w / 16 - 1));
    put_ue(b, (uint32_t)(h / 16 - 1));
    b.put(1, 1);
    b.put(1, 1);
    b.put(0, 1);
    b.put(0, 1);
    b.put(1, 1);                                           /* rbsp trailing */
    b.n = (b.n + 7) & ~7;
}

__device__ void gen_pps(SmallBits &b)
{
    b.clear();
    put_ue(b, 0);
    put_ue(b, 0);
    b.put(0, 1);
    b.put(0, 1);
    put_ue(b, 0);
    put_ue(b, 1);
    put_ue(b, 0);
    b.put(0, 1);
    b.put(0, 2);
    put_se(b, 0);
    put_se(b, 0);
    put_se(b, 0);
    b.put(1, 1);
    b.put(0, 1);
    b.put(0, 1);
    b.put(1, 1);
    b.n = (b.n + 7) & ~7;
}

/* nal_write_unit of a small RBSP (lane 0): start code, header, EP automaton */
__device__ uint64_t put_small_nal(uint8_t *A, uint64_t at, uint64_t cap, int ref_idc, int type,
                                  const SmallBits &b, bool &over)
{
    const int nb = b.n >> 3;
    if (at + 5 + 2 * (uint64_t)nb > cap) {
        over = true;
        return at;
    }
    A[at++] = 0;
    A[at++] = 0;
    A[at++] = 0;
    A[at++] = 1;
    A[at++] = (uint8_t)(((ref_idc & 3) << 5) | (type & 31));
    int zeros = 0;
    for (int k = 0; k < nb; ++k) {                         /* nal.c:24-50 */
        const uint32_t v = b.byte(k);
        if (zeros >= 2 && v <= 3) {
            A[at++] = 3;
            zeros = 0;
        }
        A[at++] = (uint8_t)v;
        zeros = v ? 0 : zeros + 1;
    }
    return at;
}

/* ---------------------------------------------------------------------- */
/* k_ing_stream                                                            */
/* ---------------------------------------------------------------------- */
struct IngLds {
    uint8_t ring[RING];           /* RBSP bytes, index k at k % RING          */
    uint8_t obuf[OBUF];           /* one output chunk after EP insertion       */
    uint32_t wsum[NW];
    int32_t wmax[NW];
    uint32_t pos[2][ING_SC_MAX];
    SmallBits hdr[2];             /* new slice headers of A and B             */
    uint8_t pre[2][40];           /* first output bytes (header + body mix)   */
    NalRange sps[2], pps[2], idr[2];
    SliceHdr sh[2];
    SpsInfo si[2];
    int32_t dbf, err;
};

/* one slice NAL: new header bits H ++ RBSP bits [mb_start, 8 R) of the EBSP
 * payload d[0, n), NAL-framed with EP into A[at, ...) */
__device__ uint64_t stream_slice(IngLds &L, const uint8_t *__restrict__ d, uint64_t n,
                                 const SmallBits &H, const uint8_t *pre, uint64_t mb_start,
                                 int ref_idc, int type, uint8_t *__restrict__ A, uint64_t at,
                                 uint64_t cap, bool &over)
{
    const int t = threadIdx.x;
    const int hlen = H.n;
    const int npre = (hlen + 7) >> 3;                       /* output bytes holding header bits */
    if (t == 0 && at + 5 <= cap) {
        A[at] = 0;
        A[at + 1] = 0;
        A[at + 2] = 0;
        A[at + 3] = 1;
        A[at + 4] = (uint8_t)(((ref_idc & 3) << 5) | (type & 31));
    }
    at += 5;
    uint64_t R = 0;               /* RBSP bytes produced (uniform) */
    uint64_t O = 0;               /* output RBSP bytes emitted      */
    int64_t lnz = -1;             /* output index of the last non-zero byte emitted */
    const uint32_t s = (uint32_t)((mb_start + 8 * (uint64_t)npre - (uint64_t)hlen) & 7u);
    /* output byte o >= npre takes RBSP bits [q, q + 8), q = 8 o - hlen + mb_start */
    for (uint64_t w0 = 0;; w0 += WINB) {
        const bool last = w0 + WINB >= n;
        /* 1. this window's RBSP bytes -> ring */
        int kept = 0;
        uint8_t v[16];
        uint32_t keepm = 0;
        const uint64_t i0 = w0 + 16u * (uint32_t)t;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint64_t i = i0 + (uint64_t)q;
            v[q] = 0;
            if (i < n) {
                const uint32_t b = d[i];
                v[q] = (uint8_t)b;
                const bool rm = b == 3 && i >= 2 && d[i - 1] == 0 && d[i - 2] == 0 && i + 1 < n &&
                                d[i + 1] <= 3;             /* nal_parser.c:72 */
                if (!rm) {
                    keepm |= 1u << q;
                    kept++;
                }
            }
        }
        uint32_t ex, tot;
        block_excl_sum((uint32_t)kept, L.wsum, ex, tot);
        {
            uint64_t k = R + ex;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if ((keepm >> q) & 1u) L.ring[(k++) & (RING - 1)] = v[q];
        }
        R += tot;
        __syncthreads();
        /* 2. output bytes whose source bytes are all in the ring */
        const uint64_t total_bits = 8 * R >= mb_start ? (uint64_t)hlen + 8 * R - mb_start : (uint64_t)hlen;
        uint64_t O_end;
        if (last) {
            O_end = (total_bits + 7) >> 3;
        } else {
            /* byte o needs RBSP byte ((8o - hlen + mb_start) >> 3) + 1 < R */
            const int64_t lim = (int64_t)(8 * (R - 1)) + (int64_t)hlen - (int64_t)mb_start - 8;
            O_end = lim < 8 * (int64_t)npre ? (uint64_t)npre : (uint64_t)(lim / 8);
            O_end = O_end > (uint64_t)npre ? O_end : (uint64_t)npre;
            if (O_end < O) O_end = O;
        }
        while (O < O_end) {
            const uint64_t oc = O_end - O < (uint64_t)OCH ? O_end - O : (uint64_t)OCH;
            /* each lane: 16 output bytes */
            uint8_t ob[16];
            int64_t my_lnz = -1;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint64_t o = O + 16u * (uint32_t)t + (uint64_t)q;
                uint32_t x = 0;
                if (o < O + oc) {
                    if (o < (uint64_t)npre) {
                        x = pre[o];
                    } else {
                        const uint64_t qb = 8 * o - (uint64_t)hlen + mb_start;
                        const uint64_t k = qb >> 3;
                        const uint32_t a = k < R ? L.ring[k & (RING - 1)] : 0u;
                        const uint32_t b = k + 1 < R ? L.ring[(k + 1) & (RING - 1)] : 0u;
                        x = ((a << s) | (b >> (8 - s))) & 255u;
                        if (8 * o + 8 > total_bits) x &= (0xff00u >> (total_bits - 8 * o)) & 255u;
                    }
                    if (x) my_lnz = (int64_t)o;
                }
                ob[q] = (uint8_t)x;
            }
            /* EP insertion: before byte o iff ob <= 3 and the zero run before o
             * (o - 1 - last non-zero) is even and >= 2 (nal.c:33-38) */
            int mx_ex, mx_tot;
            const int rel = my_lnz < 0 ? -1 : (int)(my_lnz - (int64_t)O);
            block_excl_max(rel, L.wmax, mx_ex, mx_tot);
            int64_t prev = mx_ex >= 0 ? (int64_t)O + mx_ex : lnz;
            uint32_t insm = 0;
            int nins = 0, nout = 0;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const uint64_t o = O + 16u * (uint32_t)t + (uint64_t)q;
                if (o < O + oc) {
                    const int64_t run = (int64_t)o - 1 - prev;
                    if (ob[q] <= 3 && run >= 2 && !(run & 1)) {
                        insm |= 1u << q;
                        nins++;
                    }
                    if (ob[q]) prev = (int64_t)o;
                    nout++;
                }
            }
            uint32_t oex, otot;
            block_excl_sum((uint32_t)(nout + nins), L.wsum, oex, otot);
            if (at + otot > cap) {
                over = true;
                return at;
            }
            {
                uint32_t k = oex;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    if (q >= nout) break;
                    if ((insm >> q) & 1u) L.obuf[k++] = 3;
                    L.obuf[k++] = ob[q];
                }
            }
            __syncthreads();
            for (uint32_t k = (uint32_t)t; k < otot; k += DT) A[at + k] = L.obuf[k];
            at += otot;
            if (mx_tot >= 0) lnz = (int64_t)O + mx_tot;
            O += oc;
            __syncthreads();
        }
        if (last) break;
    }
    return at;
}

__global__ __launch_bounds__(DT) void k_ing_stream(const uint8_t *__restrict__ in,
                                                   const IngestFile *__restrict__ files,
                                                   const IngestScan *__restrict__ scan,
                                                   IngestOut *__restrict__ outs,
                                                   uint8_t *__restrict__ arena, uint64_t ld_arena,
                                                   uint64_t cap, int first_stream)
{
    __shared__ IngLds L;
    const int k = blockIdx.x, t = threadIdx.x;
    uint8_t *A = arena + (size_t)(first_stream + k) * ld_arena;
    const uint8_t *d[2] = {in + files[2 * k].off, in + files[2 * k + 1].off};
    const uint64_t n[2] = {files[2 * k].size, files[2 * k + 1].size};
    if (t == 0) {
        L.err = ING_OK;
        for (int f = 0; f < 2 && L.err == ING_OK; ++f) {
            const int np = (int)scan[2 * k + f].n;
            if (np > ING_SC_MAX) {
                L.err = ING_ERR_NALS;
                break;
            }
            for (int q = 0; q < np; ++q) L.pos[f][q] = scan[2 * k + f].pos[q];
            if (walk_nals(d[f], n[f], L.pos[f], np, L.sps[f], L.pps[f], L.idr[f])) {
                L.err = ING_ERR_MISSING;
                break;
            }
            int nref, dbf;
            if (parse_sps(d[f] + L.sps[f].off, L.sps[f].n, L.si[f]) ||
                parse_pps(d[f] + L.pps[f].off, L.pps[f].n, nref, dbf)) {
                L.err = ING_ERR_PARSE;
                break;
            }
            if (f == 0) L.dbf = dbf;
        }
        if (L.err == ING_OK && (L.si[0].w != L.si[1].w || L.si[0].h != L.si[1].h))
            L.err = ING_ERR_DIMS;                          /* composer.c:177-186 */
        if (L.err == ING_OK) {
            for (int f = 0; f < 2; ++f) {                  /* both with A's parse config */
                parse_idr(d[f] + L.idr[f].off, L.idr[f].n, L.si[0], L.dbf, L.sh[f]);
                slice_header(L.hdr[f], f == 0, L.dbf, L.sh[f]);
                /* first output bytes: header bits, then the body's first bits */
                EbspReader r;
                r.init(d[f] + L.idr[f].off, L.idr[f].n);
                for (uint64_t q = 0; q < L.sh[f].mb_start; ++q) r.u1();
                SmallBits pb = L.hdr[f];
                const int npre = (pb.n + 7) >> 3;
                while (pb.n < 8 * npre && !r.eof) {
                    const uint32_t bit = r.u1();
                    if (r.eof) break;
                    pb.put(bit, 1);
                }
                for (int q = 0; q < npre; ++q) L.pre[f][q] = (uint8_t)pb.byte(q);
            }
        }
    }
    __syncthreads();
    IngestOut &o = outs[k];
    if (L.err != ING_OK) {
        if (t == 0) {
            o.err = L.err;
            o.bytes = 0;
        }
        return;
    }
    bool over = false;
    uint64_t at = 0;
    if (t == 0) {
        SmallBits b;
        gen_sps(b, L.si[0].w, L.si[0].h);
        at = put_small_nal(A, at, cap, 3, 7, b, over);
        gen_pps(b);
        at = put_small_nal(A, at, cap, 3, 8, b, over);
        L.wsum[0] = (uint32_t)at;
        L.wmax[0] = over ? 1 : 0;
    }
    __syncthreads();
    at = L.wsum[0];
    over = L.wmax[0] != 0;
    __syncthreads();
    for (int f = 0; f < 2 && !over; ++f)
        at = stream_slice(L, d[f] + L.idr[f].off, L.idr[f].n, L.hdr[f], L.pre[f], L.sh[f].mb_start,
                          3, f == 0 ? 5 : 1, A, at, cap, over);
    if (t == 0) {
        o.err = over ? ING_ERR_OVERFLOW : ING_OK;
        o.bytes = over ? 0 : at;
        o.w = L.si[0].w;
        o.h = L.si[0].h;
        o.deblock = L.dbf;
    }
}

/* ---------------------------------------------------------------------- */
/* segmented ingest: every slice body over many workgroups                 */
/* ---------------------------------------------------------------------- */
/* k_ing_stream streams a whole slice with one workgroup (one per stream: at
 * 256 new streams a quarter of the chip, 340 dependent windows each).  The
 * segmented path cuts each slice's EBSP into SEG-byte segments:
 *   k_ing_head        per stream: the parse and the SPS / PPS NAL units of
 *                     k_ing_stream, and a plan per slice (input range,
 *                     header bits, first output bytes)
 *   k_ing_seg<SUMMARY> per segment: its RBSP bytes (closed-form removal) and
 *                     its output bytes -- those RBSP bytes shifted behind the
 *                     new header -- summarised for emulation prevention:
 *                     first / last non-zero byte and the insertions after the
 *                     first, which do not depend on what came before
 *   k_ing_fix         per stream, serial over its segments: each one's
 *                     insertions before its first non-zero byte (closed form
 *                     in the last non-zero byte before it), hence its arena
 *                     offset; the byte counts and the arena bound
 *   k_ing_seg<WRITE_STAGED> per segment: the summary pass's bytes from
 *                     scratch (k_ing_seg<WRITE>: decoded again), with their 03s, to the
 *                     arena.
 * Bytes: identical to k_ing_stream's (tests/test_gpu_ingest.py checks both
 * against the oracle). */
constexpr uint32_t SEG = 16384;          /* EBSP bytes per segment                  */
constexpr uint32_t SEG_LA = 64;          /* EBSP bytes decoded past it (its successor's first RBSP byte) */

struct IngPlan {                         /* one slice of a new stream               */
    uint64_t in, n;                      /* EBSP payload in the input, bytes        */
    uint64_t mb_start;                   /* RBSP bit of the first MB                */
    uint64_t at;                         /* arena offset of the NAL (k_ing_fix)     */
    uint64_t R;                          /* RBSP bytes of the payload (k_ing_fix)   */
    uint32_t hlen, npre, nseg, ok;
    int32_t ref_idc, type;
    uint8_t pre[40];
};

struct IngSeg {
    uint32_t kept;                       /* RBSP bytes (the summary pass)           */
    uint32_t nout;                       /* output bytes it owns                    */
    int32_t f, vf, last;                 /* first non-zero output byte (relative to its first,
                                          * -1: none), its value, the last non-zero one */
    uint32_t cafter;                     /* EP insertions after the first non-zero byte */
    int64_t lnz;                         /* last non-zero output byte before it, relative (k_ing_fix) */
    uint64_t at;                         /* arena offset of its first output byte (k_ing_fix) */
    /* the one-pass path's hand-off (k_ing_seg<SEG_FUSED>): the summary
     * (hw[0..1]) and the chain state after the segment (hw[2..3]) as words
     * with a valid bit (63), written and polled with relaxed agent-scope
     * atomics -- no fence: an agent-scope release / acquire writes back /
     * invalidates the XCD's L2 (a first version that published a flag that
     * way, looking back one segment at a time from lane 0, took 3.1 ms per
     * call against 0.80 ms now).  Zeroed by k_ing_head. */
    unsigned long long hw[4];
};

/* the hand-off words: summary kept / nout / cafter (< 2^17 each), f + 1 /
 * last + 1 (< 2^17) / vf; state: bad, arena position; RBSP bytes (< 2^32)
 * and last non-zero output byte + 1 (< 2^31) of the slice so far */
__device__ inline uint64_t hw_s0(uint32_t kept, uint32_t nout, uint32_t cafter)
{
    return 1ull << 63 | (uint64_t)kept << 34 | (uint64_t)nout << 17 | cafter;
}
__device__ inline uint64_t hw_s1(int32_t f, int32_t last, int32_t vf)
{
    return 1ull << 63 | (uint64_t)(uint32_t)(f + 1) << 25 | (uint64_t)(uint32_t)(last + 1) << 8 | (uint32_t)vf;
}
__device__ inline uint64_t hw_p0(uint64_t pos, uint32_t bad) { return 1ull << 63 | (uint64_t)(bad != 0) << 62 | pos; }
__device__ inline uint64_t hw_p1(uint64_t R0, int64_t lnz) { return 1ull << 63 | R0 << 31 | (uint64_t)(lnz + 1); }
__device__ inline bool hw_valid(uint64_t a, uint64_t b) { return (a & b) >> 63; }
__device__ inline uint64_t hw_load(unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void hw_store(unsigned long long *p, uint64_t v)
{
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* the chain state over a new stream's segments, A's then B's (k_ing_fix's
 * serial loop as a step per segment): arena position, RBSP bytes and last
 * non-zero output byte of the slice so far, a header-longer-than-a-segment
 * flag */
struct IngChain {
    uint64_t pos, R0;
    int64_t lnz;
    uint32_t bad;
};

/* even numbers >= 2 in [a, b] */
__device__ inline int64_t evens_ge2(int64_t a, int64_t b)
{
    if (a < 2) a = 2;
    const int64_t f = a + (a & 1);
    return b < f ? 0 : (b - f) / 2 + 1;
}

/* segment c of slice P (summary kept / nout / f / vf / last / cafter) on
 * the chain: its arena offset and incoming last non-zero byte (relative to
 * its first output byte), then the state after it.  nal_at: the slice's NAL
 * offset (segment 0; A's from k_ing_head, B's where A ends) */
__device__ inline void ing_chain_step(IngChain &st, const IngPlan &P, uint32_t c, uint64_t nal_at, uint32_t kept,
                                      uint32_t nout, int32_t f, int32_t vf, int32_t last, uint32_t cafter,
                                      uint64_t &at, int64_t &lnz_rel)
{
    const int64_t D = (int64_t)P.hlen - (int64_t)P.mb_start, cd = (D + 7) >> 3;
    if (c == 0) {
        st.pos = nal_at + 5;
        st.R0 = 0;
        st.lnz = -1;
    }
    const int64_t o0 = c == 0 ? 0 : (int64_t)st.R0 + cd;
    if (c > 0 && o0 < (int64_t)P.npre) st.bad = 1;         /* a header longer than a segment's body */
    at = st.pos;
    lnz_rel = st.lnz - o0;
    const int64_t of = f >= 0 ? o0 + f : o0 + (int64_t)nout;   /* first non-zero (or the end) */
    int64_t ins = nout ? evens_ge2(o0 - 1 - st.lnz, of - 2 - st.lnz) : 0;   /* zero bytes o0 .. of - 1 */
    if (f >= 0) {
        const int64_t run = of - 1 - st.lnz;
        if (vf <= 3 && run >= 2 && !(run & 1)) ins++;
        ins += cafter;
        st.lnz = o0 + last;
    }
    st.pos += nout + (uint64_t)ins;
    st.R0 += kept;
}

__global__ __launch_bounds__(DT) void k_ing_head(const uint8_t *__restrict__ in,
                                                 const IngestFile *__restrict__ files,
                                                 const IngestScan *__restrict__ scan,
                                                 IngestOut *__restrict__ outs, IngPlan *__restrict__ plans,
                                                 IngSeg *__restrict__ segs, uint32_t *__restrict__ ticket,
                                                 uint32_t maxseg, uint8_t *__restrict__ arena,
                                                 uint64_t ld_arena, uint64_t cap, int first_stream)
{
    __shared__ IngLds L;
    const int k = blockIdx.x, t = threadIdx.x;
    uint8_t *A = arena + (size_t)(first_stream + k) * ld_arena;
    const uint8_t *d[2] = {in + files[2 * k].off, in + files[2 * k + 1].off};
    const uint64_t n[2] = {files[2 * k].size, files[2 * k + 1].size};
    /* the one-pass segments' hand-off flags and ticket (k_ing_seg<SEG_FUSED>) */
    for (uint32_t q = (uint32_t)t; q < 2 * maxseg; q += DT) {
        IngSeg &Q = segs[(size_t)2 * k * maxseg + q];
        Q.hw[0] = Q.hw[1] = Q.hw[2] = Q.hw[3] = 0ull;
    }
    if (k == 0 && t == 0 && ticket) *ticket = 0u;
    if (t != 0) return;
    int err = ING_OK;
    for (int f = 0; f < 2 && err == ING_OK; ++f) {
        const int np = (int)scan[2 * k + f].n;
        if (np > ING_SC_MAX) {
            err = ING_ERR_NALS;
            break;
        }
        for (int q = 0; q < np; ++q) L.pos[f][q] = scan[2 * k + f].pos[q];
        if (walk_nals(d[f], n[f], L.pos[f], np, L.sps[f], L.pps[f], L.idr[f])) {
            err = ING_ERR_MISSING;
            break;
        }
        int nref, dbf;
        if (parse_sps(d[f] + L.sps[f].off, L.sps[f].n, L.si[f]) ||
            parse_pps(d[f] + L.pps[f].off, L.pps[f].n, nref, dbf)) {
            err = ING_ERR_PARSE;
            break;
        }
        if (f == 0) L.dbf = dbf;
    }
    if (err == ING_OK && (L.si[0].w != L.si[1].w || L.si[0].h != L.si[1].h)) err = ING_ERR_DIMS;
    IngestOut &o = outs[k];
    if (err == ING_OK) {
        for (int f = 0; f < 2 && err == ING_OK; ++f) {          /* both with A's parse config */
            parse_idr(d[f] + L.idr[f].off, L.idr[f].n, L.si[0], L.dbf, L.sh[f]);
            slice_header(L.hdr[f], f == 0, L.dbf, L.sh[f]);
            EbspReader r;
            r.init(d[f] + L.idr[f].off, L.idr[f].n);
            for (uint64_t q = 0; q < L.sh[f].mb_start; ++q) r.u1();
            SmallBits pb = L.hdr[f];
            const int npre = (pb.n + 7) >> 3;
            while (pb.n < 8 * npre && !r.eof) {
                const uint32_t bit = r.u1();
                if (r.eof) break;
                pb.put(bit, 1);
            }
            IngPlan &P = plans[2 * k + f];
            P.in = files[2 * k + f].off + L.idr[f].off;
            P.n = L.idr[f].n;
            P.mb_start = L.sh[f].mb_start;
            P.hlen = (uint32_t)L.hdr[f].n;
            P.npre = (uint32_t)npre;
            P.nseg = (uint32_t)((P.n + SEG - 1) / SEG);
            if (P.nseg == 0) P.nseg = 1;
            if (P.nseg > maxseg) err = ING_ERR_NALS;       /* the host sized maxseg by the files */
            P.ref_idc = 3;
            P.type = f == 0 ? 5 : 1;
            for (int q = 0; q < npre && q < 40; ++q) P.pre[q] = (uint8_t)pb.byte(q);
        }
    }
    bool over = false;
    uint64_t at = 0;
    if (err == ING_OK) {
        SmallBits b;
        gen_sps(b, L.si[0].w, L.si[0].h);
        at = put_small_nal(A, at, cap, 3, 7, b, over);
        gen_pps(b);
        at = put_small_nal(A, at, cap, 3, 8, b, over);
        if (over) err = ING_ERR_OVERFLOW;
    }
    plans[2 * k].at = at;                                  /* A's NAL; k_ing_fix places B */
    plans[2 * k].ok = plans[2 * k + 1].ok = err == ING_OK;
    o.err = err;
    o.bytes = 0;
    o.w = L.si[0].w;
    o.h = L.si[0].h;
    o.deblock = L.dbf;
}

/* ---- workgroup scans of NV values at once (2 barriers for all) ---- */
template <int NV>
__device__ inline void block_excl_sum_v(const uint32_t (&v)[NV], uint32_t (*ws)[NW], uint32_t (&excl)[NV],
                                        uint32_t (&tot)[NV])
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        incl[j] = wave_incl_sum(v[j], lane);
        if (lane == 63) ws[j][wave] = incl[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        uint32_t pm = 0, tt = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint32_t x = ws[j][w];
            pm += w < wave ? x : 0u;
            tt += x;
        }
        excl[j] = pm + incl[j] - v[j];
        tot[j] = tt;
    }
    __syncthreads();
}

template <int NV>
__device__ inline void block_excl_max_v(const int (&v)[NV], int (*ws)[NW], int (&excl)[NV], int (&tot)[NV])
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        incl[j] = wave_incl_max(v[j], lane);
        if (lane == 63) ws[j][wave] = incl[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        int e = __shfl_up(incl[j], 1, 64);
        if (lane == 0) e = -1;
        int pm = -1, tt = -1;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const int x = ws[j][w];
            pm = w < wave ? max(pm, x) : pm;
            tt = max(tt, x);
        }
        excl[j] = max(pm, e);
        tot[j] = tt;
    }
    __syncthreads();
}

constexpr int NJ = (int)((SEG + SEG_LA + 15 + 16 * DT - 1) / (16 * DT));   /* 16-byte-per-lane windows */
constexpr uint32_t RBCAP = SEG + SEG_LA + 16;                            /* RBSP bytes kept in LDS   */

constexpr uint32_t SEG_LDS_BYTES = RBCAP + 48 + OBUF + 16;
struct SegLds {
    /* the segment's RBSP bytes (+ look-ahead), zeros after; once the output
     * bytes are in registers, the output bytes after EP at the arena's
     * phase (all windows, or one at a time past RBCAP + 48 when they do not
     * fit) */
    alignas(16) uint8_t rb[SEG_LDS_BYTES];
    uint32_t wsum[NJ + 1][NW];
    int32_t wmax[NJ][NW];
    int32_t wmin[1][NW];
};

/* One segment of a slice body: EBSP bytes [c SEG, (c + 1) SEG) of the
 * payload.  Its output bytes do not depend on the segments before: output
 * byte u (relative) is RBSP byte u and the next one (the look-ahead byte at
 * the end) shifted by the slice's constant s -- for segment 0 after the
 * npre header bytes -- so the summary pass summarises a segment without
 * knowing where it lands, and a write pass writes it where k_ing_fix
 * puts it.  Emulation prevention needs the last non-zero byte before each
 * byte: inside the segment a max-scan, from the segments before k_ing_fix's
 * lnz.  All windows of a phase share one workgroup scan. */
enum { SEG_SUMMARY = 0, SEG_WRITE = 1, SEG_WRITE_STAGED = 2, SEG_FUSED = 3 };

/* waves per SIMD k_ing_seg is compiled for: the fused pass held 128 VGPRs
 * (4 workgroups per CU) unbounded, while its LDS allows 6 */
#ifndef SCROLL_ING_WAVES
#define SCROLL_ING_WAVES 6
#endif

/* SEG_FUSED (round 5, the default): summary, place and write in one
 * workgroup, the output bytes never leaving registers.  Workgroups take
 * their segment from a ticket, in the order (stream's segment index over A
 * then B, stream), so every segment before it in its stream holds an earlier
 * ticket: it has started and publishes its summary without waiting for
 * anything.  A segment publishes its summary, looks back (decoupled
 * look-back) for the nearest earlier segment that has published its chain
 * state, steps the chain over the summaries in between (k_ing_fix's loop),
 * publishes its own state and writes.  The stream's last segment reports the
 * header's bytes.  Traffic: the file once here (and once in k_ing_scan), the
 * arena once -- 1.60x the algorithmic bytes; round 4's summary / fix /
 * staged-write passes also wrote and read back the output bytes (2.52x).
 * The look-back (wave 0, 64 segments per load) costs the workgroup about
 * two agent-scope round trips, hidden by 6 workgroups per CU (the output
 * bytes parked in LDS meanwhile): 0.80 ms per ingest720 call against the
 * three passes' 0.90 ms. */
constexpr uint64_t ING_WAIT_TICKS = 5000000ull;      /* 50 ms of waiting for an earlier segment: the stream fails */
constexpr uint64_t ING_WAIT_GAP = 100000ull;         /* a longer gap between two polls is a preemption, not counted */

template <int MODE>
__global__ __launch_bounds__(DT) __attribute__((amdgpu_waves_per_eu(SCROLL_ING_WAVES))) void k_ing_seg(const uint8_t *__restrict__ in,
                                                const IngPlan *__restrict__ plans,
                                                IngSeg *__restrict__ segs, uint32_t maxseg,
                                                uint8_t *__restrict__ arena, uint64_t ld_arena,
                                                int first_stream, uint8_t *__restrict__ stg,
                                                uint32_t *__restrict__ ticket, IngestOut *__restrict__ outs,
                                                uint64_t cap)
{
    constexpr bool WRITE = MODE != SEG_SUMMARY;
    constexpr bool FUSED = MODE == SEG_FUSED;
    __shared__ SegLds L;
    __shared__ uint32_t s_tk;
    __shared__ uint64_t s_at, s_nal;
    __shared__ int64_t s_lnz;
    __shared__ uint32_t s_skip;
    __shared__ int32_t s_vf;
    uint32_t c = blockIdx.x, p = blockIdx.y, v = 0, ntot = 0;
    const int t = threadIdx.x;
    if (FUSED) {                                            /* grid (2 maxseg, streams) */
        if (t == 0) s_tk = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint32_t tk = s_tk, k = tk % gridDim.y;
        v = tk / gridDim.y;
        const IngPlan &PA = plans[2 * k];
        if (!PA.ok) return;
        ntot = PA.nseg + plans[2 * k + 1].nseg;
        if (v >= ntot) return;
        p = v < PA.nseg ? 2 * k : 2 * k + 1;
        c = v < PA.nseg ? v : v - PA.nseg;
    }
    const IngPlan &P = plans[p];
    if (!P.ok || c >= P.nseg) return;
    IngSeg &G = segs[(size_t)p * maxseg + c];
    const uint8_t *d = in + P.in;
    const int64_t n = (int64_t)P.n;
    const bool lastseg = c + 1 == P.nseg;
    /* 1. RBSP bytes of [e0, e1) -> LDS; kept: those of [e0, es) */
    const int64_t e0 = (int64_t)c * SEG, es = min(n, e0 + (int64_t)SEG), e1 = min(n, e0 + (int64_t)(SEG + SEG_LA));
    const uint8_t *a0 = align16_down(d + e0), *hi = d + min(n, e1 + 1);
    /* the segment's output bytes (16 per lane and window, little-endian) */
    uint32_t ow[NJ][4];
    int64_t nout;
    uint32_t kept = 0;
    uint4 *sp = stg ? reinterpret_cast<uint4 *>(stg + ((size_t)p * maxseg + c) * (size_t)(NJ * OCH)) : nullptr;
    if (MODE != SEG_WRITE_STAGED) {
    uint32_t have;
    {
        uint32_t km[NJ], cnt[NJ + 1];
        cnt[NJ] = 0;
        Chunk16 ch[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) ch[j] = load_chunk16(a0 + 16 * (t + DT * j), d, hi);
        /* indices relative to e0, int32 */
        const int32_t e1r = (int32_t)(e1 - e0), esr = (int32_t)(es - e0);
        const int32_t rlo = (int32_t)max((int64_t)2 - e0, (int64_t)-64), rhi = (int32_t)min(n - 1 - e0, (int64_t)(1 << 20));
        const int32_t ia = (int32_t)(a0 - (d + e0)) + 16 * t;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int32_t i0 = ia + 16 * DT * j;
            km[j] = 0;
            uint32_t sm = 0;
            if (i0 + 16 > 0 && i0 < e1r) {
                const uint32_t rm = ep_removed16(ch[j]) & range16_32(rlo - i0, rhi - i0);
                km[j] = range16_32(-i0, e1r - i0) & ~rm;
                sm = range16_32(-i0, esr - i0) & ~rm;
            }
            cnt[j] = (uint32_t)__popc(km[j]);
            cnt[NJ] += (uint32_t)__popc(sm);
        }
        uint32_t ex[NJ + 1], tot[NJ + 1];
        block_excl_sum_v<NJ + 1>(cnt, L.wsum, ex, tot);
        uint32_t base = 0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            uint32_t at = base + ex[j];
            if (km[j] == 0xffffu && at + 16 <= RBCAP) {
                lds_put16(L.rb, at, ch[j].w);
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if ((km[j] >> q) & 1u) {
                        if (at < RBCAP) L.rb[at] = (uint8_t)ch[j].b(q);
                        at++;
                    }
            }
            base += tot[j];
        }
        have = min(base, RBCAP);
        kept = tot[NJ];
    }
    if (t < 48) L.rb[have + t] = 0;                         /* bytes past the end read as 0 */
    __syncthreads();
    /* 2. the segment's output bytes u = 0 .. nout - 1 */
    const int64_t hlen = P.hlen, npre = P.npre, mbs = (int64_t)P.mb_start, D = hlen - mbs;
    const int64_t cd = (D + 7) >> 3;                        /* ceil(D / 8) */
    const uint32_t s = (uint32_t)((-D) & 7);
    int64_t off = 0, ufast = 0, umask = INT64_MAX, total_bits = 0;
    if (c == 0) {
        off = -cd;                                          /* RBSP byte of output u: u - cd */
        ufast = npre;
        if (lastseg) {
            total_bits = 8 * (int64_t)kept >= mbs ? D + 8 * (int64_t)kept : hlen;
            nout = (total_bits + 7) >> 3;
            umask = total_bits >> 3;
        } else {
            nout = max((int64_t)kept + cd, npre);
        }
    } else {
        nout = kept;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int64_t u0 = (int64_t)OCH * j + 16 * t;
        ow[j][0] = ow[j][1] = ow[j][2] = ow[j][3] = 0;
        if (u0 >= nout) continue;
        if (u0 >= ufast && u0 + 16 <= umask) {
            /* RBSP bytes li0 .. li0 + 16 from five LDS dwords, then the bit
             * shift s of every byte with SWAR masks */
            const uint32_t li0 = (uint32_t)(u0 + off), m = li0 & 3u;
            const uint32_t *rw = reinterpret_cast<const uint32_t *>(L.rb) + (li0 >> 2);
            const uint32_t D0 = rw[0], D1 = rw[1], D2 = rw[2], D3 = rw[3], D4 = rw[4];
            const uint32_t E[5] = {__builtin_amdgcn_alignbyte(D1, D0, m), __builtin_amdgcn_alignbyte(D2, D1, m),
                                   __builtin_amdgcn_alignbyte(D3, D2, m), __builtin_amdgcn_alignbyte(D4, D3, m),
                                   D4 >> (8 * m)};
            const uint32_t mH = ((0xffu << s) & 0xffu) * 0x01010101u, mL = (0xffu >> (8 - s)) * 0x01010101u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t Y = __builtin_amdgcn_alignbyte(E[k + 1], E[k], 1u);
                ow[j][k] = ((E[k] << s) & mH) | (s ? (Y >> (8 - s)) & mL : 0u);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t u = u0 + q;
                uint32_t x;
                if (c == 0 && u < npre) {
                    x = P.pre[u];
                } else {
                    const int64_t k = u + off;
                    const uint32_t a = k >= 0 && k < (int64_t)have ? L.rb[k] : 0u;
                    const uint32_t b = k + 1 >= 0 && k + 1 < (int64_t)have ? L.rb[k + 1] : 0u;
                    x = ((a << s) | (b >> (8 - s))) & 255u;
                    if (u >= umask) x &= (0xff00u >> (total_bits - 8 * u)) & 255u;
                }
                ow[j][q >> 2] |= x << (8 * (q & 3));
            }
        }
    }
    } else {                                                /* the summary pass left them in stg */
        nout = G.nout;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const uint4 v = (int64_t)OCH * j + 16 * t < nout ? sp[(OCH / 16) * j + t] : make_uint4(0u, 0u, 0u, 0u);
            ow[j][0] = v.x;
            ow[j][1] = v.y;
            ow[j][2] = v.z;
            ow[j][3] = v.w;
        }
    }
    int my_l[NJ], my_f = INT32_MAX;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int64_t u0 = (int64_t)OCH * j + 16 * t;
        my_l[j] = -1;
        if (u0 >= nout) continue;
        if (MODE != SEG_WRITE_STAGED && u0 + 16 > nout) {  /* bytes past the segment's end */
            const int64_t keep = nout - u0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int64_t kb = keep - 4 * k;
                ow[j][k] &= kb >= 4 ? 0xffffffffu : kb <= 0 ? 0u : (1u << (8 * kb)) - 1;
            }
        }
        if (MODE == SEG_SUMMARY && sp) sp[(OCH / 16) * j + t] = make_uint4(ow[j][0], ow[j][1], ow[j][2], ow[j][3]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (ow[j][k]) {
                my_l[j] = 16 * t + 4 * k + 3 - (__builtin_clz(ow[j][k]) >> 3);
                if (my_f == INT32_MAX) my_f = OCH * j + 16 * t + 4 * k + (__builtin_ctz(ow[j][k]) >> 3);
            }
    }
    /* 3. emulation prevention (nal.c:33-38): before byte u iff it is <= 3 and
     * the zero run since the last non-zero byte is even and >= 2 */
    int lx[NJ], lt[NJ];
    block_excl_max_v<NJ>(my_l, L.wmax, lx, lt);
    const int32_t nout32 = (int32_t)nout;
    uint32_t nb[NJ + 1], insm[NJ];
    uint32_t naft = 0;
    int32_t before;
    /* lnz_in: the last non-zero output byte before the segment, relative */
    auto ep_pass = [&](int64_t lnz_in) {
    /* positions relative to the segment, int32; a last non-zero byte
     * further back than 4 bytes only matters through its parity */
    before = lnz_in >= -4 ? (int32_t)lnz_in : -4 - (int32_t)(lnz_in & 1);
    naft = 0;
    nb[NJ] = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int32_t u0 = OCH * j + 16 * t;
        int32_t prev = lx[j] >= 0 ? OCH * j + lx[j] : before;
        insm[j] = 0;
        const uint32_t valid = u0 >= nout32 ? 0u : u0 + 16 <= nout32 ? 0xffffu : (1u << (nout32 - u0)) - 1u;
        nb[j] = (uint32_t)__popc(valid);
        /* candidates: bytes <= 3 after two zero bytes (the bytes past nout
         * may pass too: the exact loop below skips them) */
        uint32_t cand = 0, zl = (prev < u0 - 1 ? 0x80000000u : 0u) | (prev < u0 - 2 ? 0x00800000u : 0u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t zk = zero_hi(ow[j][k]);
            cand |= zero_hi(ow[j][k] & 0xfcfcfcfcu) & __builtin_amdgcn_alignbyte(zk, zl, 3u) &
                    __builtin_amdgcn_alignbyte(zk, zl, 2u);
            zl = zk;
        }
        if (cand) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int32_t u = u0 + q;
                if (u < nout32) {
                    const uint32_t x = (ow[j][q >> 2] >> (8 * (q & 3))) & 255u;
                    const int32_t run = u - 1 - prev;
                    if (x <= 3 && run >= 2 && !(run & 1)) {
                        insm[j] |= 1u << q;
                        nb[j]++;
                        naft += prev >= 0 ? 1u : 0u;
                    }
                    if (x) prev = u;
                }
            }
        }
        if (lt[j] >= 0) before = OCH * j + lt[j];
    }
    };
    ep_pass(WRITE && !FUSED ? G.lnz : -((int64_t)1 << 40));
    int32_t my_first = -1, my_last = -1;
    uint32_t my_cafter = 0;
    if (!WRITE || FUSED) {
        uint32_t v1[1] = {naft}, e1v[1], t1v[1];
        int fv[1] = {my_f == INT32_MAX ? -1 : INT32_MAX - my_f}, fe[1], ft[1];
        block_excl_max_v<1>(fv, L.wmin, fe, ft);
        block_excl_sum_v<1>(v1, L.wsum, e1v, t1v);
        const int32_t first = ft[0] >= 0 ? INT32_MAX - ft[0] : -1;
        my_first = first;
        my_last = before >= 0 ? before : -1;
        my_cafter = t1v[0];
        if (t == 0) {
            G.kept = kept;
            G.nout = (uint32_t)nout;
            G.f = first;
            G.last = before >= 0 ? before : -1;
            G.cafter = t1v[0];
            if (first < 0) G.vf = 0;
        }
        if (first >= 0 && my_f == first) {                  /* the lane holding the first non-zero byte */
            const int j = first / OCH, q = first % OCH - 16 * t;
            uint32_t x = 0;
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (jj == j && k == (q >> 2)) x = (ow[jj][k] >> (8 * (q & 3))) & 255u;
            if (FUSED) s_vf = (int32_t)x;           /* published by lane 0 with the rest */
            else G.vf = (int32_t)x;
        }
        if (!FUSED) return;
    }
    uint64_t at = G.at;
    int64_t lnz_in = G.lnz;
    if (FUSED) {
        /* the output bytes wait in LDS (free: the RBSP bytes are consumed)
         * while wave 0 looks back -- kept in registers across it the pass
         * needed 128 VGPRs, 4 waves per SIMD */
        static_assert(NJ * DT * 16 <= SEG_LDS_BYTES, "the parked output bytes fit the LDS buffer");
        uint4 *park = reinterpret_cast<uint4 *>(L.rb);
#pragma unroll
        for (int j = 0; j < NJ; ++j) park[j * DT + t] = make_uint4(ow[j][0], ow[j][1], ow[j][2], ow[j][3]);
        __syncthreads();                                    /* s_vf */
        if (t < 64) {                                       /* wave 0: publish, look back, place */
            const int lane = t, k = (int)(p >> 1);
            const IngPlan &PA = plans[2 * k];
            IngSeg *SA = segs + (size_t)(2 * k) * maxseg, *SB = SA + maxseg;
            auto seg_at = [&](int64_t u) -> IngSeg & {
                return (uint32_t)u < PA.nseg ? SA[u] : SB[(uint32_t)u - PA.nseg];
            };
            const int32_t vf = my_first >= 0 ? s_vf : 0;
            if (lane == 0) {
                hw_store(&G.hw[0], hw_s0(kept, (uint32_t)nout, my_cafter));
                hw_store(&G.hw[1], hw_s1(my_first, my_last, vf));
            }
            /* the nearest earlier segment of the stream with its state (64
             * at a time; none: the chain starts at A's segment 0) */
            int64_t base = -1;
            uint64_t b0 = 0, b1 = 0;
            for (int64_t hi = (int64_t)v - 1; hi >= 0; hi -= 64) {
                const int64_t u = hi - lane;
                uint64_t q0 = 0, q1 = 0;
                if (u >= 0) {
                    q0 = hw_load(&seg_at(u).hw[2]);
                    q1 = hw_load(&seg_at(u).hw[3]);
                }
                const uint64_t m = __builtin_amdgcn_ballot_w64(u >= 0 && hw_valid(q0, q1));
                if (m) {
                    const int L = __builtin_ctzll(m);
                    base = hi - L;
                    b0 = __shfl(q0, L, 64);
                    b1 = __shfl(q1, L, 64);
                    break;
                }
            }
            IngChain st{0, 0, -1, 0};
            if (base >= 0) st = IngChain{b0 & ((1ull << 62) - 1), (b1 >> 31) & 0xffffffffull,
                                         (int64_t)(b1 & 0x7fffffffull) - 1, (uint32_t)((b0 >> 62) & 1u)};
            /* the summaries after it, 64 at a time (each published without
             * waiting for anything: the poll is bounded only against a
             * broken dispatch), stepped through in order */
            uint64_t prev = __builtin_amdgcn_s_memrealtime(), waited = 0, nal = 0;
            bool late = false;
            auto step_over = [&](int64_t w, uint64_t a0, uint64_t a1, uint64_t &at_o, int64_t &lr_o) {
                const bool inB = (uint32_t)w >= PA.nseg;
                const uint32_t cw = inB ? (uint32_t)w - PA.nseg : (uint32_t)w;
                if (cw == 0) nal = inB ? st.pos : PA.at;
                ing_chain_step(st, plans[2 * k + (inB ? 1 : 0)], cw, nal, (uint32_t)(a0 >> 34) & 0x1ffffu,
                               (uint32_t)(a0 >> 17) & 0x1ffffu, (int32_t)((a1 >> 25) & 0x1ffffu) - 1,
                               (int32_t)(a1 & 255u), (int32_t)((a1 >> 8) & 0x1ffffu) - 1, (uint32_t)a0 & 0x1ffffu,
                               at_o, lr_o);
            };
            uint64_t xat = 0;
            int64_t xl = -1;
            for (int64_t lo = base + 1; lo < (int64_t)v && !late; lo += 64) {
                const int64_t u = lo + lane;
                bool need = u < (int64_t)v;
                uint64_t q0 = 0, q1 = 0;
                for (;;) {
                    if (need) {
                        q0 = hw_load(&seg_at(u).hw[0]);
                        q1 = hw_load(&seg_at(u).hw[1]);
                        need = !hw_valid(q0, q1);
                    }
                    if (__builtin_amdgcn_ballot_w64(need) == 0) break;
                    const uint64_t now = __builtin_amdgcn_s_memrealtime(), gap = now - prev;
                    prev = now;
                    if (gap < ING_WAIT_GAP) waited += gap;
                    if (waited > ING_WAIT_TICKS) {
                        late = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (late) break;
                const int n = (int)min((int64_t)64, (int64_t)v - lo);
                for (int j = 0; j < n; ++j) {
                    uint64_t dat;
                    int64_t dl;
                    step_over(lo + j, __shfl(q0, j, 64), __shfl(q1, j, 64), dat, dl);
                }
            }
            step_over((int64_t)v, hw_s0(kept, (uint32_t)nout, my_cafter), hw_s1(my_first, my_last, vf), xat, xl);
            if (lane == 0) {
                if (!late) {
                    hw_store(&G.hw[2], hw_p0(st.pos, st.bad));
                    hw_store(&G.hw[3], hw_p1(st.R0, st.lnz));
                }
                s_nal = nal;
                s_at = xat;
                s_lnz = xl;
                /* nothing of a stream that fails is written past its arena */
                s_skip = late || st.bad || st.pos > cap;
                if (v + 1 == ntot || late) {                /* the stream's outcome */
                    if (late) outs[k].err = ING_ERR_WAIT;
                    else if (st.bad) outs[k].err = ING_ERR_PARSE;
                    else if (st.pos > cap) outs[k].err = ING_ERR_OVERFLOW;
                    if (!late && !st.bad && st.pos <= cap) outs[k].bytes = st.pos;
                }
            }
        }
        __syncthreads();
        if (s_skip) return;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const uint4 q = park[j * DT + t];
            ow[j][0] = q.x;
            ow[j][1] = q.y;
            ow[j][2] = q.z;
            ow[j][3] = q.w;
        }
        __syncthreads();                                    /* the staging below reuses the buffer */
        at = s_at;
        lnz_in = s_lnz;
        ep_pass(lnz_in);
    }
    /* 4. write, window by window, staged at the arena address's phase in
     * 16-byte lines: whole lines go out as one 16-byte store, the two end
     * lines (shared with the neighbouring segments) byte by byte */
    uint32_t ex[NJ + 1], tot[NJ + 1];
    block_excl_sum_v<NJ + 1>(nb, L.wsum, ex, tot);
    uint8_t *A = arena + (size_t)(first_stream + (int)(p >> 1)) * ld_arena;
    if (c == 0 && t == 0) {
        const uint64_t a5 = FUSED ? s_nal : P.at;
        A[a5] = 0;
        A[a5 + 1] = 0;
        A[a5 + 2] = 0;
        A[a5 + 3] = 1;
        A[a5 + 4] = (uint8_t)(((P.ref_idc & 3) << 5) | (P.type & 31));
    }
    auto put_lines = [&](const uint8_t *buf, uint32_t ph, uint32_t end, uint8_t *line0) {
        for (uint32_t l = (uint32_t)t; l < (end + 15) >> 4; l += DT) {
            const uint32_t b0 = 16 * l;
            if (b0 >= ph && b0 + 16 <= end) {
                *reinterpret_cast<uint4 *>(line0 + b0) = *reinterpret_cast<const uint4 *>(buf + b0);
            } else {
                for (uint32_t q = max(b0, ph); q < min(b0 + 16, end); ++q) line0[q] = buf[q];
            }
        }
    };
    auto stage = [&](uint8_t *buf, int j, uint32_t kq) {
        if (insm[j] == 0 && (int64_t)OCH * j + 16 * t + 16 <= nout) {
            lds_put16(buf, kq, ow[j]);
            return;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            if ((int64_t)OCH * j + 16 * t + q >= nout) break;
            if ((insm[j] >> q) & 1u) buf[kq++] = 3;
            buf[kq++] = (uint8_t)(ow[j][q >> 2] >> (8 * (q & 3)));
        }
    };
    uint32_t total = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) total += tot[j];
    const uint32_t ph0 = (uint32_t)(reinterpret_cast<uintptr_t>(A + at) & 15u);
    if (ph0 + total + 16 <= SEG_LDS_BYTES) {                /* all windows at once */
        uint32_t base = ph0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            stage(L.rb, j, base + ex[j]);
            base += tot[j];
        }
        __syncthreads();
        put_lines(L.rb, ph0, ph0 + total, A + at - ph0);
        return;
    }
    uint8_t *obuf = L.rb + RBCAP + 48;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        if ((int64_t)OCH * j >= nout) break;                /* uniform */
        const uint32_t ph = (uint32_t)(reinterpret_cast<uintptr_t>(A + at) & 15u);
        stage(obuf, j, ph + ex[j]);
        __syncthreads();
        put_lines(obuf, ph, ph + tot[j], A + at - ph);
        at += tot[j];
        __syncthreads();
    }
}

/* per stream, serial over the segments of A then B: RBSP prefix, output
 * offsets, the insertions before each segment's first non-zero byte (closed
 * form in the last non-zero byte before it), arena offsets, the bound */
constexpr int FIX_MAXSEG = 1024;             /* segments per slice staged in LDS (16 MB slices; larger files take k_ing_stream) */

struct FixSeg {
    uint32_t kept, nout, cafter;
    int32_t f, vf, last;
};

__global__ __launch_bounds__(64) void k_ing_fix(IngPlan *__restrict__ plans, IngSeg *__restrict__ segs,
                                                uint32_t maxseg, IngestOut *__restrict__ outs, uint64_t cap)
{
    __shared__ FixSeg S[FIX_MAXSEG];
    __shared__ uint64_t Sat[FIX_MAXSEG];
    __shared__ int64_t Slnz[FIX_MAXSEG];
    __shared__ uint64_t sh_at;
    __shared__ int sh_bad;
    const int k = blockIdx.x, t = threadIdx.x;
    IngPlan &PA = plans[2 * k], &PB = plans[2 * k + 1];
    if (!PA.ok) return;
    if (t == 0) {
        sh_at = PA.at;
        sh_bad = 0;
    }
    __syncthreads();
    for (int f = 0; f < 2; ++f) {
        IngPlan &P = f ? PB : PA;
        IngSeg *SG = segs + (size_t)(2 * k + f) * maxseg;
        const uint32_t ns = P.nseg;
        if (ns > (uint32_t)FIX_MAXSEG) {                    /* host keeps maxseg below; uniform */
            if (t == 0) sh_bad = 2;
            break;
        }
        for (uint32_t c = (uint32_t)t; c < ns; c += 64) {
            const IngSeg &G = SG[c];
            S[c] = FixSeg{G.kept, G.nout, G.cafter, G.f, G.vf, G.last};
        }
        __syncthreads();
        if (t == 0) {
            const int64_t D = (int64_t)P.hlen - (int64_t)P.mb_start, cd = (D + 7) >> 3;
            const uint64_t at = sh_at;
            P.at = at;
            uint64_t pos = at + 5, R0 = 0;
            int64_t lnz = -1;                               /* output index in the slice */
            for (uint32_t c = 0; c < ns; ++c) {
                const FixSeg G = S[c];
                const int64_t o0 = c == 0 ? 0 : (int64_t)R0 + cd;
                if (c > 0 && o0 < (int64_t)P.npre) sh_bad = 1;   /* a header longer than a segment's body */
                Sat[c] = pos;
                Slnz[c] = lnz - o0;
                const int64_t of = G.f >= 0 ? o0 + G.f : o0 + (int64_t)G.nout;   /* first non-zero (or the end) */
                /* zero bytes o0 .. of - 1: run o - 1 - lnz */
                int64_t ins = G.nout ? evens_ge2(o0 - 1 - lnz, of - 2 - lnz) : 0;
                if (G.f >= 0) {
                    const int64_t run = of - 1 - lnz;
                    if (G.vf <= 3 && run >= 2 && !(run & 1)) ins++;
                    ins += G.cafter;
                    lnz = o0 + G.last;
                }
                pos += G.nout + (uint64_t)ins;
                R0 += G.kept;
            }
            P.R = R0;
            sh_at = pos;
        }
        __syncthreads();
        for (uint32_t c = (uint32_t)t; c < ns; c += 64) {
            SG[c].at = Sat[c];
            SG[c].lnz = Slnz[c];
        }
        __syncthreads();
    }
    if (t == 0) {
        const bool over = sh_at > cap, bad = sh_bad != 0;
        if (over || bad) {
            PA.ok = PB.ok = 0;
            outs[k].err = bad ? ING_ERR_PARSE : ING_ERR_OVERFLOW;
            outs[k].bytes = 0;
        } else {
            outs[k].bytes = sh_at;
        }
    }
}

/* ---------------------------------------------------------------------- */
/* k_ing_update: mid-stream long-term reference ("atlas") updates          */
/* ---------------------------------------------------------------------- */
/* One workgroup per update of a live stream: the file's first SPS / PPS /
 * IDR (parse_reference_file's rules), the IDR slice parsed with the file's
 * own SPS / PPS (composer_init, composer.c:127-196), rewritten as a non-IDR I
 * frame with the STREAM's write config -- h264_rewrite_as_non_idr_i_frame
 * (h264_writer.c:296-350) with long_term_frame_idx `which` at the stream's
 * frame_num (mod 2^log2_max_frame_num, POC lsb 2 frame_num as the waypoint
 * frames, :683-687) -- appended at the stream's cursor.  Its MMCO 4
 * (max_long_term_frame_idx_plus1 2) drops the waypoints: the stream's
 * waypoint table empties and frame_num advances (:779-781).  Bits:
 * oracle/scroll_oracle.c or_update_ref. */
__device__ void update_header(SmallBits &b, const DevStream &S, int fn, int which, const SliceHdr &h)
{
    b.clear();
    put_ue(b, 0);
    put_ue(b, 7);                                          /* SLICE_TYPE_I_ALL */
    put_ue(b, 0);
    b.put((uint32_t)fn, S.log2_mfn);
    if (S.poc_type == 0) b.put((uint32_t)(2 * fn), S.log2_poc);
    b.put(1, 1);                                           /* adaptive_ref_pic_marking_mode_flag */
    put_ue(b, 4);
    put_ue(b, 2);
    put_ue(b, 6);
    put_ue(b, (uint32_t)which);
    put_ue(b, 0);
    put_se(b, h.qpd);
    if (S.deblock) {
        put_ue(b, h.dbf);
        if (h.dbf != 1) {
            put_se(b, h.alpha);
            put_se(b, h.beta);
        }
    }
}

__global__ __launch_bounds__(DT) void k_ing_update(const uint8_t *__restrict__ in,
                                                   const IngestFile *__restrict__ files,
                                                   const IngestScan *__restrict__ scan,
                                                   const int32_t *__restrict__ ups,
                                                   IngestOut *__restrict__ outs,
                                                   DevStream *__restrict__ st,
                                                   uint8_t *__restrict__ arena, uint64_t ld_arena)
{
    __shared__ IngLds L;
    __shared__ uint64_t s_at;
    const int k = blockIdx.x, t = threadIdx.x;
    const int s = ups[2 * k], which = ups[2 * k + 1];
    DevStream *S = st + s;
    uint8_t *A = arena + (size_t)s * ld_arena;
    const uint8_t *d = in + files[k].off;
    const uint64_t n = files[k].size;
    if (t == 0) {
        L.err = ING_OK;
        const int np = (int)scan[k].n;
        if (np > ING_SC_MAX) {
            L.err = ING_ERR_NALS;
        } else {
            for (int q = 0; q < np; ++q) L.pos[0][q] = scan[k].pos[q];
            int nref, dbf;
            if (walk_nals(d, n, L.pos[0], np, L.sps[0], L.pps[0], L.idr[0])) L.err = ING_ERR_MISSING;
            else if (parse_sps(d + L.sps[0].off, L.sps[0].n, L.si[0]) ||
                     parse_pps(d + L.pps[0].off, L.pps[0].n, nref, dbf))
                L.err = ING_ERR_PARSE;
            else if (L.si[0].w != S->w || L.si[0].h != S->h)
                L.err = ING_ERR_DIMS;
            else {
                parse_idr(d + L.idr[0].off, L.idr[0].n, L.si[0], dbf, L.sh[0]);
                const int fn = S->frame_num & ((1 << S->log2_mfn) - 1);
                update_header(L.hdr[0], *S, fn, which, L.sh[0]);
                EbspReader r;
                r.init(d + L.idr[0].off, L.idr[0].n);
                for (uint64_t q = 0; q < L.sh[0].mb_start; ++q) r.u1();
                SmallBits pb = L.hdr[0];
                const int npre = (pb.n + 7) >> 3;
                while (pb.n < 8 * npre && !r.eof) {
                    const uint32_t bit = r.u1();
                    if (r.eof) break;
                    pb.put(bit, 1);
                }
                for (int q = 0; q < npre; ++q) L.pre[0][q] = (uint8_t)pb.byte(q);
            }
        }
        s_at = S->out_pos;
    }
    __syncthreads();
    IngestOut &o = outs[k];
    if (L.err != ING_OK) {
        if (t == 0) {
            o.err = L.err;
            o.bytes = 0;
        }
        return;
    }
    const uint64_t at0 = s_at;
    bool over = false;
    const uint64_t at = stream_slice(L, d + L.idr[0].off, L.idr[0].n, L.hdr[0], L.pre[0], L.sh[0].mb_start, 3, 1,
                                     A, at0, S->out_cap, over);
    if (t == 0) {
        o.err = over ? ING_ERR_OVERFLOW : ING_OK;
        o.bytes = over ? 0 : at - at0;
        o.w = L.si[0].w;
        o.h = L.si[0].h;
        if (!over) {                                       /* commit */
            S->out_pos = at;
            S->undelivered += at - at0;
            S->frame_num += 1;
            S->nwp = 0;
            for (int q = 0; q < 8; ++q) S->wp_valid[q] = 0;
        }
    }
}

}  // namespace

int update_launch(hipStream_t hs, const uint8_t *in, const IngestFile *files, int n, uint64_t max_file,
                  IngestScan *scan, const int32_t *ups, IngestOut *outs, DevStream *st, uint8_t *arena,
                  uint64_t ld_arena)
{
    if (n <= 0) return 0;
    if (hipMemsetAsync(scan, 0, sizeof(IngestScan) * (size_t)n, hs) != hipSuccess) return -1;
    const uint32_t gx = (uint32_t)((max_file + 15 + SCAN_W * WINB - 1) / (SCAN_W * WINB));
    if (gx > 0) {
        hipLaunchKernelGGL(k_ing_scan, dim3(gx, n), dim3(DT), 0, hs, in, files, scan);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    hipLaunchKernelGGL(k_ing_update, dim3(n), dim3(DT), 0, hs, in, files, scan, ups, outs, st, arena, ld_arena);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int ingest_launch(hipStream_t hs, const uint8_t *in, const IngestFile *files, int nstreams,
                  uint64_t max_file, IngestScan *scan, IngestOut *outs, uint8_t *arena,
                  uint64_t ld_arena, uint64_t cap, int first_stream, void *work, size_t work_bytes, int mode)
{
    if (nstreams <= 0) return 0;
    if (hipMemsetAsync(scan, 0, sizeof(IngestScan) * 2 * (size_t)nstreams, hs) != hipSuccess)
        return -1;
    const uint32_t gx = (uint32_t)((max_file + 15 + SCAN_W * WINB - 1) / (SCAN_W * WINB));
    if (gx > 0) {
        hipLaunchKernelGGL(k_ing_scan, dim3(gx, 2 * nstreams), dim3(DT), 0, hs, in, files, scan);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    const uint32_t maxseg = (uint32_t)((max_file + SEG - 1) / SEG) + 1u;
    if (!work || maxseg > (uint32_t)FIX_MAXSEG) {   /* one workgroup per stream (SCROLL_INGEST_SERIAL, > 16 MB files) */
        hipLaunchKernelGGL(k_ing_stream, dim3(nstreams), dim3(DT), 0, hs, in, files, scan, outs, arena,
                           ld_arena, cap, first_stream);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    IngPlan *plans = reinterpret_cast<IngPlan *>(work);
    IngSeg *segs = reinterpret_cast<IngSeg *>(plans + 2 * (size_t)nstreams);
    const size_t base = 2 * (size_t)nstreams * (sizeof(IngPlan) + maxseg * sizeof(IngSeg));
    uint32_t *ticket = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(work) + base);
    if (work_bytes < base + 16) return -1;
    hipLaunchKernelGGL(k_ing_head, dim3(nstreams), dim3(DT), 0, hs, in, files, scan, outs, plans, segs,
                       mode == ING_ONEPASS ? ticket : nullptr, maxseg, arena, ld_arena, cap, first_stream);
    if (mode == ING_ONEPASS) {
        hipLaunchKernelGGL(k_ing_seg<SEG_FUSED>, dim3(2 * maxseg, nstreams), dim3(DT), 0, hs, in, plans, segs,
                           maxseg, arena, ld_arena, first_stream, nullptr, ticket, outs, cap);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    uint8_t *stg = nullptr;                 /* the summary pass's output bytes, when the scratch holds them */
    if (mode == ING_STAGED && work_bytes >= base + 2 * (size_t)nstreams * maxseg * (size_t)(NJ * OCH) + 16)
        stg = reinterpret_cast<uint8_t *>(((uintptr_t)work + base + 15) & ~(uintptr_t)15);
    hipLaunchKernelGGL(k_ing_seg<SEG_SUMMARY>, dim3(maxseg, 2 * nstreams), dim3(DT), 0, hs, in, plans, segs,
                       maxseg, arena, ld_arena, first_stream, stg, nullptr, nullptr, 0ull);
    hipLaunchKernelGGL(k_ing_fix, dim3(nstreams), dim3(64), 0, hs, plans, segs, maxseg, outs, cap);
    if (stg)
        hipLaunchKernelGGL(k_ing_seg<SEG_WRITE_STAGED>, dim3(maxseg, 2 * nstreams), dim3(DT), 0, hs, in, plans,
                           segs, maxseg, arena, ld_arena, first_stream, stg, nullptr, nullptr, 0ull);
    else
        hipLaunchKernelGGL(k_ing_seg<SEG_WRITE>, dim3(maxseg, 2 * nstreams), dim3(DT), 0, hs, in, plans, segs,
                           maxseg, arena, ld_arena, first_stream, stg, nullptr, nullptr, 0ull);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* scratch of the segmented path; 0 when ingest_launch takes the one-workgroup
 * path anyway (a slice over FIX_MAXSEG segments), which needs none */
size_t ingest_work_bytes(int nstreams, uint64_t max_file, int mode)
{
    const size_t maxseg = (size_t)((max_file + SEG - 1) / SEG) + 1u;
    if (maxseg > (size_t)FIX_MAXSEG) return 0;
    const size_t base = 2 * (size_t)nstreams * (sizeof(IngPlan) + maxseg * sizeof(IngSeg));
    return mode == ING_STAGED ? base + 2 * (size_t)nstreams * maxseg * (size_t)(NJ * OCH) + 16 : base + 16;
}
