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

constexpr int IT = 256;                     /* threads per workgroup            */
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

template <bool WRITE>
__global__ __launch_bounds__(IT) void k_ipcm(IpcmGeom G, const uint8_t *__restrict__ pics,
                                             uint32_t *__restrict__ counts, uint8_t *__restrict__ out)
{
    __shared__ alignas(16) uint8_t rb[LB + CH];
    __shared__ alignas(16) uint8_t ob[16 + CH + CH / 2 + 16];
    __shared__ int32_t wsm[IT / 64];
    __shared__ uint32_t wss[IT / 64];
    __shared__ int32_t deep;
    const int t = threadIdx.x;
    const uint32_t c = blockIdx.x, n = blockIdx.y;
    const uint8_t *pic = pics + (size_t)n * G.pic_stride;
    const uint32_t c0 = c * CH, c1 = min(c0 + CH, G.rbsp_len);

    /* RBSP bytes [c0 - LB, c1) -> LDS.  The samples go by source row
     * segment (an MB record's 16 luma rows of 16 bytes, 8 + 8 chroma rows of
     * 8): one 16- or 8-byte load per segment, its bytes into LDS at their
     * RBSP offsets; every other byte -- before the RBSP (a non-zero sentinel:
     * the automaton starts with no zeros seen), the slice header, the
     * records' 0x0D 0x00, the stop byte -- by the thread of its index.  Each
     * byte has exactly one writer. */
    {
        const int64_t lo = (int64_t)c0 - LB;
        const uint32_t base = G.nh - 2u;
        for (uint32_t k = (uint32_t)t; k < (uint32_t)LB + CH; k += IT) {
            const int64_t i = lo + (int64_t)k;
            int v = -1;                                       /* -1: a sample byte */
            if (i < 0) {
                v = 0xff;
            } else if (i >= (int64_t)c1) {
                v = 0;
            } else if ((uint32_t)i < G.nh) {
                v = G.hdr[i];
            } else if ((uint32_t)i + 1u == G.rbsp_len) {
                v = 0x80;                                     /* rbsp_stop_one_bit + alignment */
            } else {
                const uint32_t j = (uint32_t)i - base;
                const uint32_t r = j - 386u * (uint32_t)(((uint64_t)j * M386) >> 41);
                if (r < 2u) v = r == 0u ? 0x0D : 0x00;        /* ue(25) + pcm_alignment_zero_bits */
            }
            if (v >= 0) rb[k] = (uint8_t)v;
        }
        /* the records that overlap [max(lo, nh), c1): 32 segments each */
        const int64_t s0 = lo > (int64_t)G.nh ? lo : (int64_t)G.nh;
        if (s0 < (int64_t)c1) {
            const uint32_t m0 = (uint32_t)((((uint64_t)s0 - base) * M386) >> 41);
            const uint32_t m1 = min((uint32_t)((((uint64_t)c1 - 1u - base) * M386) >> 41), G.nmb - 1u);
            const uint32_t w = (uint32_t)G.w, cw = w / 2u;
            const size_t ysz = (size_t)w * (uint32_t)G.h;
            const bool vec = (reinterpret_cast<uintptr_t>(pic) & 15u) == 0u;
            const uint32_t nseg = 32u * (m1 - m0 + 1u);
            for (uint32_t q = (uint32_t)t; q < nseg; q += IT) {
                const uint32_t m = m0 + (q >> 5), sg = q & 31u;
                uint32_t my = __umulhi(m, G.m_mbw);
                if (G.mbw == 1) my = m;
                const uint32_t mx = m - my * G.mbw;
                uint32_t off, len;
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
                const int64_t r0 = (int64_t)base + 386 * (int64_t)m + off;      /* its RBSP index */
                if (r0 + len <= lo || r0 >= (int64_t)c1) continue;
                uint32_t x[4] = {0, 0, 0, 0};
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
#pragma unroll
                for (uint32_t b = 0; b < 16u; ++b) {
                    const int64_t i = r0 + b;
                    if (b < len && i >= lo && i < (int64_t)c1)
                        rb[(uint32_t)(i - lo)] = (uint8_t)(x[b >> 2] >> (8u * (b & 3u)));
                }
            }
        }
    }
    if (t == 0) deep = -2;
    __syncthreads();
    /* look-back: last non-zero byte before c0 (-1: the RBSP start) */
    int carry = -1;
    if (c0 > 0) {
        int lnz = -2;
#pragma unroll
        for (int k = 0; k < LB; ++k)
            if (rb[k]) lnz = (int)c0 - LB + k;
        if (lnz == -2) {                             /* LB zero bytes: rare (black pictures) */
            if (t == 0) {
                int64_t i = (int64_t)c0 - LB - 1;
                const uint32_t base = G.nh - 2u;
                int f = -1;
                for (; i >= 0; --i) {
                    const uint32_t ii = (uint32_t)i;
                    const Cur cu = cur_at(G, ii >= G.nh ? ii - base : 2u);
                    if (rbsp_at(G, pic, ii, cu)) {
                        f = (int)ii;
                        break;
                    }
                }
                deep = f;
            }
            __syncthreads();
            lnz = deep;
        }
        carry = lnz;
    }
    /* this thread's 16 bytes: last non-zero before them (block max-scan) */
    const uint32_t g0 = c0 + 16u * (uint32_t)t;
    const uint4 q4 = *reinterpret_cast<const uint4 *>(&rb[LB + 16 * t]);
    const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
    const uint32_t nb = g0 < c1 ? min(16u, c1 - g0) : 0u;
    int mylast = -1;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if ((uint32_t)k < nb && ((qw[k >> 2] >> (8 * (k & 3))) & 255u)) mylast = (int)(g0 + k);
    int pm, tmax;
    block_excl_max(mylast, wsm, pm, tmax);
    int prev = max(pm, carry);
    uint32_t epm = 0, cnt = 0;
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
    uint32_t ex, tot;
    block_excl_sum(cnt, wss, ex, tot);
    if (!WRITE) {
        if (t == 0) counts[(size_t)n * G.nchunk + c] = tot;
        return;
    }
    /* EP bytes of the earlier chunks of this file */
    uint32_t pre = 0;
    for (uint32_t k = (uint32_t)t; k < c; k += IT) pre += counts[(size_t)n * G.nchunk + k];
    uint32_t pex, ptot;
    block_excl_sum(pre, wss, pex, ptot);
    uint8_t *F = out + (size_t)n * G.out_stride;
    const uint64_t O = (uint64_t)G.npre + c0 + ptot;            /* file offset of RBSP byte c0 */
    const uint32_t sh = (uint32_t)(O & 15u);
    if (c == 0)
        for (uint32_t k = (uint32_t)t; k < G.npre; k += IT) F[k] = G.pre[k];
    {
        uint32_t x = sh + 16u * (uint32_t)t + ex;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if ((uint32_t)k >= nb) break;
            if ((epm >> k) & 1u) ob[x++] = 0x03;
            ob[x++] = (uint8_t)((qw[k >> 2] >> (8 * (k & 3))) & 255u);
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

}  // namespace

int ipcm_launch(hipStream_t hs, int pass, int n, const IpcmGeom *g, const uint8_t *pics,
                uint32_t *counts, uint8_t *out)
{
    if (n <= 0) return 0;
    if (pass == 0)
        hipLaunchKernelGGL(k_ipcm<false>, dim3(g->nchunk, n), dim3(IT), 0, hs, *g, pics, counts, out);
    else
        hipLaunchKernelGGL(k_ipcm<true>, dim3(g->nchunk, n), dim3(IT), 0, hs, *g, pics, counts, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
