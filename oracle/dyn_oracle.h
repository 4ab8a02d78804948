/*
 * dyn_oracle.h -- CPU ORACLE (test infrastructure only): the dynamic-rect
 * residual coder of BASELINE configs 3-5.
 *
 * The reference has NO implementation of this path (SURVEY.md §0.4, §8c:
 * no forward transform, quantiser or CAVLC encoder exists anywhere in
 * wreuven/h264-scroll-encoder; the dynamic rect is prose in
 * docs/MASTER_DESIGN.md:35-56,142-171).  This restatement therefore DEFINES
 * the bits: parity is "unpinned".  Its CAVLC syntax is cross-checked against
 * the reference's own CAVLC parser (experiments/trans-resizer/trans_resizer.c
 * :549-755 copy_cavlc_block, :782-885 nC rules, :1362-1470
 * copy_inter_residual), compiled from the reference sources by
 * oracle/Makefile target `ref` (oracle/ref_cavlc.c), with fixtures in
 * tests/golden/.  The product (h264-scroll-encoder_amd/) never links this.
 *
 * Specification (H.264 Baseline/Main syntax, CAVLC):
 *  - dynamic MBs: MB coordinates inside the rect, in SCROLL NALs only
 *    (waypoint frames stay residual-free so they remain pure references).
 *    A dynamic MB keeps the (ref_idx, mv) of its row (the MV field and every
 *    scroll MB codeword are unchanged) and adds coded_block_pattern me(v),
 *    mb_qp_delta se(0) when cbp != 0, and the residual (7.3.5.3).
 *  - QP 26 (the composer's PPS: pic_init_qp_minus26 = 0, slice_qp_delta 0,
 *    src/h264_writer.c:118-120), chroma QP = QPc(26 + 0) = 26.
 *  - prediction from the decoded reference: full-pel luma (mv_y = 4 off),
 *    chroma 1/8-pel bilinear (8.4.2.2.2), coordinates clamped to the picture.
 *    Refs A/B are the I_PCM pictures; a waypoint (long-term ref 2+k) is the
 *    residual-free waypoint frame k, resolved recursively through its own
 *    row-uniform (ref, mv) (src/h264_writer.c:689-729).
 *  - residual = source - prediction; 4x4 forward core transform; quant
 *    Z = sign(W) ((|W| MF + f) >> qbits), qbits = 15 + QP/6, f = 2^qbits / 6;
 *    chroma DC: 2x2 Hadamard, (|F| MF0 + 2f) >> (qbits + 1).
 *  - CAVLC (9.2) with nC from left / top 4x4 neighbours; non-dynamic MBs
 *    count as available with TotalCoeff 0.
 *  - synthetic source: per stream s, frame t, pixel index i in
 *    plane-major raster order over the MB rect (luma, then Cb, then Cr):
 *      r = mix32(seed(s,t) + i * 0x9E3779B9), seed = 0x9E3779B9 s ^ 0x85EBCA6B t,
 *      Y  = clamp(128 + ((X + 2Y + 3t) & 63) - 32 + (r >> 28) - 8),
 *      Cb/Cr = clamp(128 + ((X + Y + t) & 15) - 8 + (r >> 30)),
 *    (X, Y) frame coordinates of the plane; mix32 = murmur3 fmix32.
 */
#ifndef DYN_ORACLE_H
#define DYN_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "scroll_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_dyn_rect_s {
    int x0, y0, w, h;             /* MB units */
    int qp;                       /* the rect's QP: 0 = 26 (the default), 1..51, or
                                   * OR_DYN_QP0 (-1) = QP 0.  Slice QP 26 + (QP - 26)
                                   * (slice_qp_delta) in or_scroll_nal_dyn, the MBs'
                                   * mb_qp_delta chain under hints; chroma at QPc
                                   * (Table 8-15).  Levels are clamped to
                                   * +-OR_LEVEL_MAX (only chroma DC below QPc 6
                                   * reaches it; luma levels stay <= 1632) */
} or_dyn_rect;
#define OR_DYN_QP0 (-1)
/* the largest |level| every CAVLC context codes with level_prefix <= 15
 * (9.2.2.1: levelCode (15 << suffixLength) + 4095, suffixLength 0: 30 + 4095,
 * so |level| <= 2063 always fits; baseline-profile streams allow no larger
 * prefix) */
#define OR_LEVEL_MAX 2063
int or_dyn_qp(const or_dyn_rect *r);             /* the rect's QP, 0..51 */

typedef struct {
    int w, h;                     /* luma size; chroma w/2 x h/2 */
    const uint8_t *y, *u, *v;     /* planes, strides w and w/2    */
} or_pic;

/* decoded pictures of reference A (idx 0) and B (idx 1) */
typedef struct or_refs_s {
    const or_pic *ab[2];
} or_refs;

uint32_t or_mix32(uint32_t x);
uint32_t or_dyn_seed(int s, int t);
/* source planes of the rect: luma 16w x 16h, then Cb, Cr 8w x 8h each
 * (384 w h bytes) */
void or_dyn_source(uint8_t *dst, int s, int t, const or_dyn_rect *r);
/* I_PCM striped picture planes (decoded = raw samples) of or_ipcm_striped */
void or_striped_planes(uint8_t *y, uint8_t *u, uint8_t *v, int w, int h, int which);

/* decoded sample of reference idx ri (0 A, 1 B, 2+k waypoint k), plane 0/1/2 */
int or_ref_sample(const or_cfg *c, const or_refs *R, int ri, int plane, int x, int y);

/* CAVLC residual block (9.2): coefficients in scan order, max = 16 / 15 /
 * 4 (chroma DC, nC = -1); returns TotalCoeff */
int or_cavlc_block(or_bits *b, const int *coef, int max, int nC);
/* code tables for decoders: coeff_token (Table 9-5), total_zeros (9-7,
 * 9-8, 9-9a), run_before (9-10): returns the length (0 = no such code) and
 * the bits; or_cbp_code: coded_block_pattern -> codeNum (Table 9-4 Inter) */
int or_ct_code(int tc, int t1, int nC, uint32_t *bits);
int or_tz_code(int tc, int tz, int maxc, uint32_t *bits);
int or_rb_code(int zl, int run, uint32_t *bits);
int or_cbp_code(int cbp);
/* forward 4x4 core transform + quantisation of a residual block (raster) */
void or_fwd4x4(const int res[16], int W[16]);
int or_quant(int w, int qp, int pos, int dc_chroma);
int or_qp_chroma(int qp);                 /* QPc (Table 8-15, chroma_qp_index_offset 0) */

/* scroll P NAL with the dynamic rect (src per or_dyn_source); r == NULL or
 * an empty rect gives exactly or_scroll_nal */
size_t or_scroll_nal_dyn(uint8_t *dst, size_t cap, or_cfg *c, int off, const or_dyn_rect *r,
                         const uint8_t *src, const or_refs *R);
/* composer_write_scroll_frame with the dynamic rect in the scroll NAL */
size_t or_compose_dyn(uint8_t *dst, size_t cap, or_cfg *c, int off, int mode,
                      const or_dyn_rect *r, const uint8_t *src, const or_refs *R, int *n_wp_out);

/* CPU baseline: frames/s of BASELINE config 3 (synthetic offsets and source,
 * striped refs) on nthreads pthreads */
double or_bench_compose_dyn(int nstreams, int nframes, int w, int h, int rx0, int ry0, int rw,
                            int rh, int nthreads, unsigned long long *bytes_out);

/* test hook: the residual bits of one dynamic MB (cbp + qp_delta + residual,
 * after the MB's mvd fields) for given quantised levels; tc_out receives
 * TotalCoeff of the 16 luma (raster) + 8 chroma AC blocks */
size_t or_dyn_mb_levels_bits(uint8_t *dst, size_t cap, const int luma[16][16],
                             const int cdc[2][4], const int cac[2][4][15],
                             const int nc_left[16 + 8], const int nc_top[16 + 8], int avail_l,
                             int avail_t, int *cbp_out, int tc_out[24], size_t *nbits);

/* test hook: called by or_scroll_nal_dyn for every dynamic MB before its
 * residual (cbp onwards) is written: MB (x, y), the residual's first bit in
 * the RBSP (slice header included, NAL header byte not), the levels
 * (luma[16][16] raster block / scan order, cdc[2][4], cac[2][4][15]) and the
 * left / top neighbours' TotalCoeffs (24 each, NULL = unavailable).  NULL
 * turns it off.  Not thread-safe: tests only. */
typedef void (*or_dyn_trace_fn)(int x, int y, long long bit, const int *luma, const int *cdc, const int *cac,
                                const int *tc_left, const int *tc_top);
void or_dyn_set_trace(or_dyn_trace_fn fn);

#ifdef __cplusplus
}
#endif
#endif
