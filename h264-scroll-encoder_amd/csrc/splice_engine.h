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

#define SPLICE_PIECES 27            /* 16 luma (raster; I_16x16: AC), Cb DC, Cr DC, 4 Cb AC, 4 Cr AC,
                                     * I_16x16 luma DC */
#define SPLICE_MAX_MV 16383         /* |mv| of a spliced MB, quarter pels          */
#define SPLICE_MAXU 1024            /* NAL units (slices) of one spliced picture   */
#define SPLICE_REF_INTRA (-2)       /* ref of an intra MB in the motion field:
                                     * available, never matching (8.4.1.3.1)      */
#define HINT_MODE_SPLICED 0x100     /* HintFrame.mode bit: k_splice_stage stages it */
#define HINT_MODE_FB 0x200          /* HintFrame.mode bit (device, k_hint_fb): the frame falls back to a
                                       whole-picture residual coding, its hint rects dropped */

/* unit slots of a spliced picture of nmb MBs: every slice holds an MB, so
 * slice nmb (if any) is the first one that cannot fit and fails the frame */
__host__ __device__ static inline uint32_t splice_unit_cap(int nmb)
{
    return (uint32_t)(nmb + 1 < SPLICE_MAXU ? nmb + 1 : SPLICE_MAXU);
}

/* one spliced frame: rect, its external NAL units (device memory), their
 * RBSPs in the word pool (MSB-first words; unit u's at word ceil(b_u / 4) of
 * the frame's region), its MB records and unit slots, the parse status and
 * the last stage's (reference validity), SCROLL_SPLICE_*.  56 bytes. */
typedef struct {
    int32_t x0, y0, w, h;
    const uint8_t *nal;             /* device bytes: the NAL pool or the caller's */
    uint64_t rbsp_word;             /* words into the RBSP pool                   */
    uint32_t nal_len;
    uint32_t rec_first;             /* first MB record                            */
    int32_t status;                 /* k_splice_fix                               */
    int32_t stage_status;           /* k_splice_stage of the last compose         */
    uint32_t unit_first;            /* first unit slot                            */
    int32_t nunits;                 /* NAL units found (k_splice_units; may exceed the slots) */
    /* the dynamic rect under hints (k_hdyn_code's frames; -1 for spliced
     * slices): its MBs' QP; the first of its MBs (raster) with a residual
     * (k_hdyn_reset: ~0, then atomicMin) carries mb_qp_delta hd_qp - 26, the
     * others 0 (the chain from the slice QP 26) */
    int32_t hd_qp;
    uint32_t hd_first;
    int32_t bad_mb;                 /* k_splice_fix: the first failing slice's SpliceUnit.bad */
    int32_t pad;
} SpliceFrame;

/* one NAL unit (slice) of a spliced picture: its bytes [b, e) of the
 * frame's buffer (after the start code, trailing zero bytes trimmed); from
 * k_splice_unesc its RBSP (words from w0 of the frame's region, nbytes
 * bytes) and the bit of its rbsp_stop_one_bit (end; 0: none); from its
 * parse: first_mb_in_slice, its MB count, status, and for the QP chain its
 * first MB with mb_qp_delta (-1: none), that MB's QP and the QP of its last
 * MB with mb_qp_delta.  48 bytes. */
typedef struct {
    uint32_t b, e;
    uint32_t w0, nbytes, end;
    int32_t first, nmb, status;
    int32_t fq_mb, fq_qp, last_qp;
    int32_t bad;                    /* SCROLL_SPLICE_ERR_MBTYPE: the refused MB (rect raster) | mb_type << 16; -1 */
} SpliceUnit;

/* frames of at least this many slices are parsed one slice per lane
 * (k_splice_lanes); the others, and slices the lanes hand back, one slice
 * per wave (k_splice_parse) */
#define SPLICE_LANE_MIN 4

/* one external MB after parsing: motion (quarter pels; intra: ref
 * SPLICE_REF_INTRA), cbp, the composed mb_qp_delta, and per piece its
 * TotalCoeff, TrailingOnes and the bits after coeff_token (bit offset into
 * the frame's RBSP region, length).  A partitioned MB (part 1 16x8, 2 8x16,
 * 3 P_8x8 / P_8x8ref0 with sub_mb_type i in bits 2i..2i+1 of sub) also
 * carries the motion of each 4x4 block (raster; mv packed x | y << 16); ref
 * / mx / my are then block 0's.  An intra MB (intra 1 I_4x4, 2 I_16x16, 3
 * I_PCM) keeps its mb_type, its prediction syntax's bits (poff, plen; I_PCM:
 * poff = its samples), I_4x4's cbp codeNum.  nbsame: bit 0 / 1 the left /
 * top MB is in the rect and the same slice.  232 bytes; the first 96 (motion,
 * cbp, TotalCoeffs, TrailingOnes, the intra / residual fields) are what the
 * stage's counting sweep reads; per piece a u16: its body's length in bits
 * (<= 625 with level_prefix <= 15) | the bits of its coeff_token in the
 * external slice (<= 16) << 11 -- the pieces are contiguous from res_off in
 * syntax order, so the writing sweep finds each body by a running sum (round
 * 6: a u16 length and a u32 offset per piece, 352-byte records); the blocks'
 * motion only for partitioned MBs. */
typedef struct {
    int16_t ref;
    uint8_t cbp;
    int8_t qpd;
    int32_t mx, my;
    uint8_t skip, part, sub, intra;
    uint8_t tc[SPLICE_PIECES + 1], t1[SPLICE_PIECES + 1];
    uint32_t res_off, res_len;      /* the residual after mb_qp_delta (len 0: none / not parsed); the pieces start there */
    uint32_t poff;
    uint16_t plen;
    uint8_t mbt, cbp_code;
    uint8_t nbsame, hasqpd;
    uint16_t body;                  /* bits of its pieces' bodies (after coeff_token) */
    uint32_t pad;                   /* -- the stage reads the 96 bytes up to here at once -- */
    uint16_t bl[SPLICE_PIECES + 1];
    int8_t bref[16];
    uint32_t bmv[16];
} SpliceMbRec;
#define SPLICE_REC_HEAD 96
/* RBSP word pools: words past the last unit that k_splice_stage's body
 * reader may load (splice_kernels.hip RWin) */
#define RWIN_SLACK_WORDS 8


/* 0, or -1 when the launch failed */
/* k_splice_units -> k_splice_unesc -> k_splice_lanes -> k_splice_parse ->
 * k_splice_fix over the n listed frames; ymax = the most unit slots of a
 * frame; lanes = the lane list (count word, zero between parses, then (list
 * index, unit) pairs; room for nslots) */
int splice_launch_parse(hipStream_t hs, int n, int ymax, const int32_t *list, SpliceFrame *spf,
                        SpliceUnit *units, int32_t *lanes, size_t nslots, const DevStream *st, int ld_fr,
                        uint32_t *rbsp, SpliceMbRec *rec);
int splice_launch_stage(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                        int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                        const HintFrame *hf, const ScrollHintRect *pool, SpliceFrame *spf,
                        const SpliceMbRec *rec, const uint32_t *rbsp, uint8_t *stage,
                        uint64_t slot_bytes);
/* staging bytes per frame that a spliced NAL of an mbw x mbh picture with a
 * w x h MB external slice of nal_bytes never exceeds */
size_t splice_slot_bound(int mbw, int mbh, int w, int h, size_t nal_bytes);
