/*
 * ipcm_kernels.hip -- MI355X (gfx950) kernels that write reference files
 * (SPS + PPS + IDR of I_PCM MBs) for arbitrary I420 pictures, the
 * experiment's h264_write_ipcm_mb / h264_write_idr_frame_* path
 * (experiments/scroll-encoder/src/h264_encoder.c:730-918) generalised from
 * one stripe colour per MB to the picture's own samples.  HBM-bound byte
 * work: every workgroup owns IPCM_CHUNK bytes of one file's RBSP.
 *
 *   pass 0  each chunk's RBSP bytes (staged from the picture into LDS: one
 *           16- / 8-byte load per source row segment of an MB record)
 *           -> its emulation-prevention count (closed form of nal.c:33-38,
 *           dyn::ep_insert, with the zero run looked up across the chunk)
 *   pass 1  the same bytes + the EP bytes at the chunk's output offset
 *           (prefix + RBSP offset + EP bytes of the earlier chunks);
 *           whole 16-byte lines stored aligned, edge lines byte by byte
 *   one pass (round 6, IP_ONEPASS, opt-in: SCROLL_IPCM_ONEPASS=1, when
 *           out_stride holds the worst case so no file can overflow; less
 *           traffic, more time -- scroll_kernels.hip): both in one workgroup -- the chunk's EP
 *           count published, the counts of the earlier chunks of its file
 *           found by a decoupled look-back (workgroups start in grid order,
 *           so every earlier chunk has started or will), the bytes written
 *           from registers.  The pictures are read once and nothing is
 *           staged: the count pass's RBSP copy (written, then read back) and
 *           its second reading of the pictures are gone
 *
 * The bits are those of oracle/scroll_oracle.c or_ipcm_picture_file
 * (tests/test_gpu_ipcm.py), which for the striped pictures is pinned to the
 * reference's I_PCM files (tests/golden).
 */
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "ipcm_engine.h"
#include "stage_util.h"

using namespace scroll::stage;

namespace {

constexpr int IT = IPCM_CHUNK / 16;         /* threads per workgroup            */
constexpr int IP_WAVES = IT / 64;
constexpr int LB = 64;                      /* look-back bytes staged before it */
constexpr uint32_t CH = IPCM_CHUNK;
static_assert(CH == 16 * IT, "16 RBSP bytes per thread");
constexpr uint64_t M386 = 5696951440ull;      /* ceil(2^41 / 386): j / 386 = j * M386 >> 41, j < 2^32 */
static_assert((uint64_t)M386 * 386u >= (1ull << 41), "magic");

/* RBSP byte cursor: MB m of the file, byte r of its 386-byte record
 * (0x0D, 0x00, 384 samples; MB 0's first two bytes belong to hdr) */
struct Cur {
    uint32_t m, r, mx, my;
};

__device__ inline Cur cur_at(const IpcmGeom &G, uint32_t j)     /* j = i - (nh - 2) */
{
    Cur c;
    c.m = (uint32_t)(((uint64_t)j * M386) >> 41);
    c.r = j - 386u * c.m;
    c.my = __umulhi(c.m, G.m_mbw);
    if (G.mbw == 1) c.my = c.m;
    c.mx = c.m - c.my * G.mbw;
    return c;
}

/* byte i of the RBSP with cursor c at i (when i >= nh) */
__device__ inline uint32_t rbsp_at(const IpcmGeom &G, const uint8_t *pic, uint32_t i, const Cur &c)
{
    if (i < G.nh) return G.hdr[i];
    if (i + 1u == G.rbsp_len) return 0x80u;                    /* rbsp_stop_one_bit + alignment */
    if (c.r < 2u) return c.r == 0u ? 0x0Du : 0x00u;            /* ue(25) + pcm_alignment_zero_bits */
    const uint32_t p = c.r - 2u;
    const uint32_t w = (uint32_t)G.w;
    size_t a;
    if (p < 256u) {
        a = (size_t)(16u * c.my + (p >> 4)) * w + 16u * c.mx + (p & 15u);
    } else {
        const uint32_t q = p - (p < 320u ? 256u : 320u);
        const size_t ysz = (size_t)w * (uint32_t)G.h;
        a = ysz + (p < 320u ? 0u : ysz / 4) + (size_t)(8u * c.my + (q >> 3)) * (w / 2) + 8u * c.mx + (q & 7u);
    }
    return pic[a];
}

enum { IP_COUNT = 0, IP_WRITE = 1, IP_WRITE_STAGED = 2, IP_ONEPASS = 3 };

/* the one-pass hand-off word of a chunk: the call's epoch (24 bits) << 40 |
 * inclusive flag << 39 | EP bytes (of the chunk alone, or of the file up to
 * and including it); relaxed agent-scope atomics, no fence (ingest's note:
 * an agent-scope release / acquire writes back / invalidates the XCD's L2) */
constexpr uint64_t IP_INCL = 1ull << 39, IP_VAL = IP_INCL - 1ull;
constexpr uint64_t IP_WAIT_TICKS = 5000000ull;        /* 50 ms of waiting for an earlier chunk: the call fails */
constexpr uint64_t IP_WAIT_GAP = 100000ull;           /* a longer gap between two polls is a preemption */
__device__ inline uint64_t ip_load(unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void ip_store(unsigned long long *p, uint64_t v)
{
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__global__ __launch_bounds__(IT) void k_ipcm(IpcmGeom G, const uint8_t *__restrict__ pics,
                                             uint32_t *__restrict__ counts, uint8_t *__restrict__ out,
                                             uint8_t *__restrict__ stg, uint64_t stg_stride,
                                             uint32_t *__restrict__ over, IpcmOnePass op)
{
    constexpr bool WRITE = MODE != IP_COUNT;
    constexpr bool ONE = MODE == IP_ONEPASS;
    if (!WRITE && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *over = 0u;   /* k_ipcm_size sets it */
    if (WRITE && !ONE && __builtin_amdgcn_readfirstlane(*over)) return;    /* a file past out_stride: none written */
    __shared__ alignas(16) uint8_t rb[LB + CH];
    __shared__ alignas(16) uint8_t ob[16 + CH + CH / 2 + 16];
    __shared__ int32_t wsm[IP_WAVES];
    __shared__ uint32_t wss[IP_WAVES];
    __shared__ int32_t deep;
    __shared__ uint32_t s_pre, s_late;
    const int t = threadIdx.x;
    const uint32_t c = blockIdx.x, n = blockIdx.y;
    /* one pass: the workgroups start in grid order (x fastest, in order on
     * each XCD), so every earlier chunk of the file has started or will start
     * without waiting for this one; the wait is bounded all the same.  (A
     * ticket from one global counter instead, as ingest takes its segments:
     * 86 K same-address atomics per call, 1.10 against 0.58 ms.) */
    if (ONE && c == 0 && n == 0 && t == 0) *over = 0u;   /* set only by a wait that expired */
    const uint8_t *pic = pics + (size_t)n * G.pic_stride;
    const uint32_t c0 = c * CH, c1 = min(c0 + CH, G.rbsp_len);
    uint8_t *S = stg ? stg + (size_t)n * stg_stride : nullptr;       /* the file's RBSP (count pass) */
    const uint32_t g0 = c0 + 16u * (uint32_t)t;
    const uint32_t nb = g0 < c1 ? min(16u, c1 - g0) : 0u;
    uint32_t qw[4];
    if (MODE != IP_WRITE_STAGED) {
        /* RBSP bytes [c0 - LB, c1) -> LDS.  The samples go by source row
         * segment (an MB record's 16 luma rows of 16 bytes, 8 + 8 chroma
         * rows of 8): one 16- or 8-byte load per segment, its bytes into LDS
         * at their RBSP offsets; a 33rd segment per record is its 0x0D 0x00.
         * The bytes of the first and the last chunk's ends -- before the RBSP
         * (a non-zero sentinel: the automaton starts with no zeros seen), the
         * slice header, the stop byte, past the end -- by the thread of their
         * index.  Each byte has one value. */
        const int64_t lo = (int64_t)c0 - LB;
        const uint32_t base = G.nh - 2u;
        if (c == 0 || c + 1 == G.nchunk) {
            for (uint32_t k = (uint32_t)t; k < (uint32_t)LB + CH; k += IT) {
                const int64_t i = lo + (int64_t)k;
                int v = -1;                                   /* -1: a record byte */
                if (i < 0) {
                    v = 0xff;
                } else if (i >= (int64_t)c1) {
                    v = 0;
                } else if ((uint32_t)i < G.nh) {
                    v = G.hdr[i];
                } else if ((uint32_t)i + 1u == G.rbsp_len) {
                    v = 0x80;                                 /* rbsp_stop_one_bit + alignment */
                }
                if (v >= 0) rb[k] = (uint8_t)v;
            }
        }
        /* the records that overlap [max(lo, nh), c1): 33 segments each */
        const int64_t s0 = lo > (int64_t)G.nh ? lo : (int64_t)G.nh;
        if (s0 < (int64_t)c1) {
            const uint32_t m0 = (uint32_t)((((uint64_t)s0 - base) * M386) >> 41);
            const uint32_t m1 = min((uint32_t)((((uint64_t)c1 - 1u - base) * M386) >> 41), G.nmb - 1u);
            const uint32_t w = (uint32_t)G.w, cw = w / 2u;
            const size_t ysz = (size_t)w * (uint32_t)G.h;
            const bool vec = (reinterpret_cast<uintptr_t>(pic) & 15u) == 0u;
            const uint32_t nseg = 33u * (m1 - m0 + 1u);
            for (uint32_t q = (uint32_t)t; q < nseg; q += IT) {
                const uint32_t mq = __umulhi(q, 130150525u);  /* q / 33 (q < 2^26) */
                const uint32_t m = m0 + mq, sg = q - 33u * mq;
                uint32_t off, len;
                uint32_t x[4] = {0, 0, 0, 0};
                if (sg == 32u) {                              /* ue(25) + pcm_alignment_zero_bits */
                    if (m == 0u) continue;                    /* MB 0's: in hdr */
                    off = 0u;
                    len = 2u;
                    x[0] = 0x0Du;
                } else {
                    uint32_t my = __umulhi(m, G.m_mbw);
                    if (G.mbw == 1) my = m;
                    const uint32_t mx = m - my * G.mbw;
                    size_t a;
                    if (sg < 16u) {
                        off = 2u + 16u * sg;
                        len = 16u;
                        a = (size_t)(16u * my + sg) * w + 16u * mx;
                    } else {
                        const uint32_t cr = sg & 7u;
                        off = (sg < 24u ? 258u : 322u) + 8u * cr;
                        len = 8u;
                        a = ysz + (sg < 24u ? 0u : ysz / 4) + (size_t)(8u * my + cr) * cw + 8u * mx;
                    }
                    const int64_t r0 = (int64_t)base + 386 * (int64_t)m + off;
                    if (r0 + len <= lo || r0 >= (int64_t)c1) continue;
                    if (vec) {
                        if (len == 16u) {
                            const uint4 u = *reinterpret_cast<const uint4 *>(pic + a);
                            x[0] = u.x, x[1] = u.y, x[2] = u.z, x[3] = u.w;
                        } else {
                            const uint2 u = *reinterpret_cast<const uint2 *>(pic + a);
                            x[0] = u.x, x[1] = u.y;
                        }
                    } else {
                        for (uint32_t b = 0; b < len; ++b) x[b >> 2] |= (uint32_t)pic[a + b] << (8u * (b & 3u));
                    }
                }
                const int64_t r0 = (int64_t)base + 386 * (int64_t)m + off;      /* its RBSP index */
                if (r0 + len <= lo || r0 >= (int64_t)c1) continue;
                if (r0 >= lo && r0 + 16 <= (int64_t)c1 && len == 16u) {
                    lds_put16(rb, (uint32_t)(r0 - lo), x);
                } else {
#pragma unroll
                    for (uint32_t b = 0; b < 16u; ++b) {
                        const int64_t i = r0 + b;
                        if (b < len && i >= lo && i < (int64_t)c1)
                            rb[(uint32_t)(i - lo)] = (uint8_t)(x[b >> 2] >> (8u * (b & 3u)));
                    }
                }
            }
        }
        __syncthreads();
        const uint4 q4 = *reinterpret_cast<const uint4 *>(&rb[LB + 16 * t]);
        qw[0] = q4.x, qw[1] = q4.y, qw[2] = q4.z, qw[3] = q4.w;
        if (MODE == IP_COUNT && S && nb) *reinterpret_cast<uint4 *>(S + g0) = q4;
    } else {
        /* the count pass's RBSP bytes; the look-back bytes the same way */
        uint4 q4 = nb ? *reinterpret_cast<const uint4 *>(S + g0) : make_uint4(0u, 0u, 0u, 0u);
        qw[0] = q4.x, qw[1] = q4.y, qw[2] = q4.z, qw[3] = q4.w;
        if (t < LB / 16)
            *reinterpret_cast<uint4 *>(&rb[16 * t]) =
                c0 > 0 ? *reinterpret_cast<const uint4 *>(S + c0 - LB + 16 * t) : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    if (nb < 16) {                                        /* bytes past the RBSP */
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int kb = (int)nb - 4 * k;
            qw[k] &= kb >= 4 ? 0xffffffffu : kb <= 0 ? 0u : (1u << (8 * kb)) - 1;
        }
    }
    /* look-back: the last non-zero byte before c0 (-1: the RBSP start), from
     * the LB staged bytes by the first LB / 16 lanes */
    if (t == 0) deep = -2;
    __syncthreads();
    if (t < LB / 16 && c0 > 0) {
        const uint4 v = *reinterpret_cast<const uint4 *>(&rb[16 * t]);
        const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
        int l = -2;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (vw[k]) l = (int)c0 - LB + 16 * t + 4 * k + 3 - (__builtin_clz(vw[k]) >> 3);
        atomicMax(&deep, l);
    }
    int mylast = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (qw[k]) mylast = (int)g0 + 4 * k + 3 - (__builtin_clz(qw[k]) >> 3);
    int pm, tmax;
    block_excl_max<IP_WAVES>(mylast, wsm, pm, tmax);                /* its barriers publish deep */
    int carry = -1;
    if (c0 > 0) {
        carry = deep;
        if (carry == -2) {                                /* LB zero bytes: rare (black pictures) */
            __syncthreads();
            if (t == 0) {
                int f = -1;
                for (int64_t i = (int64_t)c0 - LB - 1; i >= 0; --i) {
                    const uint32_t ii = (uint32_t)i;
                    uint32_t v;
                    if (MODE == IP_WRITE_STAGED) {
                        v = S[ii];
                    } else {
                        const uint32_t base = G.nh - 2u;
                        const Cur cu = cur_at(G, ii >= G.nh ? ii - base : 2u);
                        v = rbsp_at(G, pic, ii, cu);
                    }
                    if (v) {
                        f = (int)ii;
                        break;
                    }
                }
                deep = f;
            }
            __syncthreads();
            carry = deep;
        }
    }
    /* emulation prevention (nal.c:33-38): the exact loop only for lanes with
     * a byte <= 3 after two zero bytes */
    int prev = max(pm, carry);
    uint32_t epm = 0, cnt = 0;
    {
        uint32_t cand = 0, zl = (prev < (int)g0 - 1 ? 0x80000000u : 0u) | (prev < (int)g0 - 2 ? 0x00800000u : 0u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t zk = zero_hi(qw[k]);
            cand |= zero_hi(qw[k] & 0xfcfcfcfcu) & __builtin_amdgcn_alignbyte(zk, zl, 3u) &
                    __builtin_amdgcn_alignbyte(zk, zl, 2u);
            zl = zk;
        }
        if (cand) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if ((uint32_t)k >= nb) break;
                const uint32_t b = (qw[k >> 2] >> (8 * (k & 3))) & 255u;
                const int i = (int)(g0 + k);
                if (scroll::dyn::ep_insert(b, i - 1 - prev)) {
                    epm |= 1u << k;
                    cnt++;
                }
                if (b) prev = i;
            }
        }
    }
    uint32_t ex, tot;
    block_excl_sum<IP_WAVES>(cnt, wss, ex, tot);
    if (!WRITE) {
        if (t == 0) counts[(size_t)n * G.nchunk + c] = tot;
        return;
    }
    /* EP bytes of the earlier chunks of this file */
    uint32_t ptot;
    if (ONE) {
        if (t < 64) {                                   /* wave 0: publish, look back, publish */
            const int lane = t;
            const uint64_t tag = (uint64_t)op.epoch << 40;
            unsigned long long *H = op.hw + (size_t)n * G.nchunk;
            if (lane == 0) ip_store(&H[c], tag | (c == 0 ? IP_INCL : 0ull) | tot);
            uint64_t excl = 0, prevt = __builtin_amdgcn_s_memrealtime(), waited = 0;
            bool late = false;
            /* the earlier chunks 64 at a time, nearest first: the sum of
             * their counts down to the nearest one with its file prefix */
            for (int64_t hi = (int64_t)c - 1; hi >= 0 && !late;) {
                const int64_t u = hi - lane;
                uint64_t q = 0;
                bool val = u < 0;                       /* before chunk 0: nothing (never reached) */
                for (;;) {
                    if (!val) {
                        q = ip_load(&H[u]);
                        val = (q >> 40) == (uint64_t)op.epoch;
                    }
                    const uint64_t mi = __builtin_amdgcn_ballot_w64(u >= 0 && val && (q & IP_INCL));
                    const int li = mi ? __builtin_ctzll(mi) : 63;
                    const uint64_t needm = li == 63 ? ~0ull : ((2ull << li) - 1ull);
                    if ((__builtin_amdgcn_ballot_w64(val) & needm) == needm) {
                        const uint32_t v = (u >= 0 && lane <= li) ? (uint32_t)(q & IP_VAL) : 0u;
                        excl += __shfl(wave_incl_sum(v, lane), 63, 64);
                        hi = mi ? -1 : hi - 64;
                        break;
                    }
                    const uint64_t now = __builtin_amdgcn_s_memrealtime(), gap = now - prevt;
                    prevt = now;
                    if (gap < IP_WAIT_GAP) waited += gap;
                    if (waited > IP_WAIT_TICKS) {
                        late = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (lane == 0) {
                if (c > 0 && !late) ip_store(&H[c], tag | IP_INCL | (excl + tot));
                s_pre = (uint32_t)excl;
                s_late = late;
                if (late) {                             /* a broken dispatch: the call fails */
                    atomicOr(over, 1u);
                    if (op.sticky) atomicOr(op.sticky, 1u);
                }
                if (!late && c + 1 == G.nchunk) op.sizes[n] = (uint64_t)G.npre + G.rbsp_len + excl + tot;
            }
        }
        __syncthreads();
        if (s_late) return;
        ptot = s_pre;
    } else {
        uint32_t pre = 0;
        for (uint32_t k = (uint32_t)t; k < c; k += IT) pre += counts[(size_t)n * G.nchunk + k];
        uint32_t pex;
        block_excl_sum<IP_WAVES>(pre, wss, pex, ptot);
    }
    uint8_t *F = out + (size_t)n * G.out_stride;
    const uint64_t O = (uint64_t)G.npre + c0 + ptot;            /* file offset of RBSP byte c0 */
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(F + O) & 15u);
    if (c == 0)
        for (uint32_t k = (uint32_t)t; k < G.npre; k += IT) F[k] = G.pre[k];
    {
        uint32_t x = sh + 16u * (uint32_t)t + ex;
        if (epm == 0 && nb == 16u) {
            lds_put16(ob, x, qw);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if ((uint32_t)k >= nb) break;
                if ((epm >> k) & 1u) ob[x++] = 0x03;
                ob[x++] = (uint8_t)((qw[k >> 2] >> (8 * (k & 3))) & 255u);
            }
        }
    }
    __syncthreads();
    const uint32_t len = (c1 - c0) + tot, end = sh + len;
    uint8_t *L0 = F + (O - sh);
    for (uint32_t l = (uint32_t)t; 16u * l < end; l += IT) {
        const uint32_t a = 16u * l;
        if (a >= sh && a + 16u <= end) {
            *reinterpret_cast<uint4 *>(L0 + a) = *reinterpret_cast<const uint4 *>(&ob[a]);
        } else {
            for (uint32_t k = max(a, sh); k < min(a + 16u, end); ++k) L0[k] = ob[k];
        }
    }
}

/* grid (n): file n's size = prefix + RBSP + its chunks' EP bytes; any file
 * past out_stride sets *over (the write pass then writes nothing) and, for
 * the asynchronous calls, *sticky (read at the batch's next sync) */
__global__ __launch_bounds__(IT) void k_ipcm_size(IpcmGeom G, const uint32_t *__restrict__ counts,
                                                  uint64_t *__restrict__ sizes, uint32_t *__restrict__ over,
                                                  uint32_t *__restrict__ sticky)
{
    __shared__ uint32_t wss[IT / 64];
    const int t = threadIdx.x;
    const uint32_t n = blockIdx.x;
    uint32_t ep = 0;
    for (uint32_t k = (uint32_t)t; k < G.nchunk; k += IT) ep += counts[(size_t)n * G.nchunk + k];
    uint32_t ex, tot;
    block_excl_sum<IP_WAVES>(ep, wss, ex, tot);
    if (t == 0) {
        const uint64_t sz = (uint64_t)G.npre + G.rbsp_len + tot;
        sizes[n] = sz;
        if (sz > G.out_stride) {
            atomicOr(over, 1u);
            if (sticky) atomicOr(sticky, 1u);
        }
    }
}

}  // namespace

int ipcm_launch(hipStream_t hs, int pass, int n, const IpcmGeom *g, const uint8_t *pics,
                uint32_t *counts, uint8_t *out, uint8_t *stg, uint64_t stg_stride, uint64_t *sizes, uint32_t *over,
                uint32_t *sticky)
{
    if (n <= 0) return 0;
    const IpcmOnePass none{};
    if (pass == 0) {
        hipLaunchKernelGGL(k_ipcm<IP_COUNT>, dim3(g->nchunk, n), dim3(IT), 0, hs, *g, pics, counts, out, stg,
                           stg_stride, over, none);
        if (hipGetLastError() != hipSuccess) return -1;
        hipLaunchKernelGGL(k_ipcm_size, dim3(n), dim3(IT), 0, hs, *g, counts, sizes, over, sticky);
    } else if (stg) {
        hipLaunchKernelGGL(k_ipcm<IP_WRITE_STAGED>, dim3(g->nchunk, n), dim3(IT), 0, hs, *g, pics, counts, out,
                           stg, stg_stride, over, none);
    } else {
        hipLaunchKernelGGL(k_ipcm<IP_WRITE>, dim3(g->nchunk, n), dim3(IT), 0, hs, *g, pics, counts, out, stg,
                           stg_stride, over, none);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int ipcm_launch_onepass(hipStream_t hs, int n, const IpcmGeom *g, const uint8_t *pics, uint8_t *out,
                        uint32_t *over, const IpcmOnePass *op)
{
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_ipcm<IP_ONEPASS>, dim3(g->nchunk, n), dim3(IT), 0, hs, *g, pics, nullptr, out, nullptr,
                       0ull, over, *op);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
