/*
 * splice_engine.h -- host-side launchers of the pre-encoded MB splice
 * (splice_kernels.hip).  The batch (scroll_kernels.hip)
 * runs k_splice_parse when the spliced slices change and k_splice_stage
 * beside k_hint_stage between the plan's state and size passes.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "engine.h"

#define SPLICE_PIECES 26            /* 16 luma (raster), Cb DC, Cr DC, 4 Cb AC, 4 Cr AC */
#define SPLICE_MAX_MV 16383         /* |mv| of a spliced MB, quarter pels          */
#define HINT_MODE_SPLICED 0x100     /* HintFrame.mode bit: k_splice_stage stages it */

/* one spliced frame: rect, its external NAL (device memory), its RBSP in
 * the word pool (MSB-first words), its MB records, the parse status and the
 * last stage's (reference validity), SCROLL_SPLICE_*.  48 bytes. */
typedef struct {
    int32_t x0, y0, w, h;
    const uint8_t *nal;             /* device bytes: the NAL pool or the caller's */
    uint64_t rbsp_word;             /* words into the RBSP pool                   */
    uint32_t nal_len;
    uint32_t rec_first;             /* first MB record                            */
    int32_t status;                 /* k_splice_parse                             */
    int32_t stage_status;           /* k_splice_stage of the last compose         */
} SpliceFrame;

/* one external MB after parsing: motion (quarter pels), cbp, the composed
 * mb_qp_delta, and per piece its TotalCoeff, TrailingOnes and the bits after
 * coeff_token (offset and length in the RBSP).  A partitioned MB (part 1
 * 16x8, 2 8x16, 3 P_8x8 / P_8x8ref0 with sub_mb_type i in bits 2i..2i+1 of
 * sub) also carries the motion of each 4x4 block (raster; mv packed x | y
 * << 16); ref / mx / my are then block 0's.  312 bytes. */
typedef struct {
    int16_t ref;
    uint8_t cbp;
    int8_t qpd;
    int32_t mx, my;
    uint8_t skip, part, sub, pad;
    uint8_t tc[SPLICE_PIECES], t1[SPLICE_PIECES];
    uint16_t blen[SPLICE_PIECES];
    uint32_t boff[SPLICE_PIECES];
    int8_t bref[16];
    uint32_t bmv[16];
    uint32_t res_off, res_len;      /* the external residual's bits (0: not parsed / none) */
} SpliceMbRec;

/* 0, or -1 when the launch failed */
int splice_launch_parse(hipStream_t hs, int n, const int32_t *list, SpliceFrame *spf,
                        const DevStream *st, int ld_fr, uint32_t *rbsp, SpliceMbRec *rec);
int splice_launch_stage(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                        int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                        const HintFrame *hf, const ScrollHintRect *pool, SpliceFrame *spf,
                        const SpliceMbRec *rec, const uint32_t *rbsp, uint8_t *stage,
                        uint64_t slot_bytes);
/* staging bytes per frame that a spliced NAL of an mbw x mbh picture with a
 * w x h MB external slice of nal_bytes never exceeds */
size_t splice_slot_bound(int mbw, int mbh, int w, int h, size_t nal_bytes);
