/*
 * ipcm_engine.h -- reference pictures -> reference files on the GPU
 * (SURVEY §8f row 3): the experiment's I_PCM IDR writer
 * (experiments/scroll-encoder/src/h264_encoder.c:730-918, one stripe colour
 * per MB there) for arbitrary I420 pictures, as the SURVEY Appendix B harness
 * frames it: SPS + PPS + one IDR slice of I_PCM MBs.
 *
 * RBSP of the IDR slice: hdr[0, nh) = slice header (h264_encoder.c:622-662)
 * + MB 0's mb_type ue(25) + pcm_alignment_zero_bits; MB 0's 384 samples;
 * then per MB m >= 1 the bytes 0x0D 0x00 (ue(25) at a byte boundary + 7
 * alignment bits) and its 384 samples; the stop byte 0x80.  With
 * base = nh - 2, MB m's 386-byte record starts at RBSP byte base + 386 m.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#ifndef IPCM_CHUNK
#define IPCM_CHUNK 4096              /* RBSP bytes per workgroup (16 per thread) */
#endif
#define IPCM_PRE_MAX 96              /* SPS + PPS NAL units + IDR start code   */

typedef struct {
    int32_t w, h;
    uint32_t mbw, nmb;
    uint32_t m_mbw, m_386;           /* magic multipliers: / mbw, / 386        */
    uint64_t pic_stride, out_stride;
    uint32_t nh;                     /* header RBSP bytes (<= 16)              */
    uint32_t rbsp_len;               /* RBSP bytes including the stop byte     */
    uint32_t npre;                   /* file prefix bytes                      */
    uint32_t nchunk;                 /* IPCM_CHUNK chunks per file             */
    uint8_t hdr[16];
    uint8_t pre[IPCM_PRE_MAX];
} IpcmGeom;

/* pass 0: emulation-prevention bytes per chunk -> counts[n][nchunk] (and,
 * with stg, each file's RBSP -> stg + n * stg_stride, stg_stride >=
 * nchunk * IPCM_CHUNK, a multiple of 16), then each file's size -> sizes[n]
 * and *over = 1 if one exceeds out_stride (also *sticky, when given: never
 * cleared by the kernels); pass 1: files -> out (prefix, EBSP), from stg
 * when given, nothing when *over.  No host step between the passes.  0, or
 * -1 when a launch failed. */
int ipcm_launch(hipStream_t hs, int pass, int n, const IpcmGeom *g, const uint8_t *pics,
                uint32_t *counts, uint8_t *out, uint8_t *stg, uint64_t stg_stride, uint64_t *sizes,
                uint32_t *over, uint32_t *sticky);

/* the one pass (round 6): usable when out_stride >= ipcm_worst(g), so that no
 * file can overflow.  hw: n x nchunk hand-off words, tagged with epoch (24
 * bits, never 0, a new one per call; the words start zeroed); sizes: n u64;
 * *over (and *sticky) set only if a look-back wait expired (a broken
 * dispatch; no file of the call is then complete) */
typedef struct {
    unsigned long long *hw;
    uint32_t epoch;
    uint64_t *sizes;
    uint32_t *sticky;
} IpcmOnePass;
static inline uint64_t ipcm_worst(const IpcmGeom *g)
{
    return (uint64_t)g->npre + g->rbsp_len + (g->rbsp_len + 1u) / 2u;   /* an EP byte per two RBSP bytes at most */
}
int ipcm_launch_onepass(hipStream_t hs, int n, const IpcmGeom *g, const uint8_t *pics, uint8_t *out,
                        uint32_t *over, const IpcmOnePass *op);
