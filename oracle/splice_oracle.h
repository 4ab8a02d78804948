/*
 * splice_oracle.h -- CPU ORACLE (test infrastructure only): the pre-encoded
 * MB splice.  Used only by tests/ as the checker of
 * k_splice_parse / k_splice_stage; the product library never links it.
 *
 * The reference designs this step but never implements it
 * (docs/MASTER_DESIGN.md:39-40 "splice the resulting encoded macroblocks into
 * the final frame", :142-146 "take the corresponding encoded macroblock
 * payload from the dynamic encoder output", :171 "encode in its own
 * coordinate system and transplant macroblock payloads while rewriting
 * addresses").  This file DEFINES that transplant ("parity unpinned",
 * DESIGN.md §10); tests/h264_pslice.py decodes both the external slice and
 * the composed NAL from the standard and checks that every spliced MB
 * decodes to the same (ref, mv, cbp, QP, coefficient levels).
 *
 * Input: one external P or I slice NAL (nal_unit_type 1, or 5 for an IDR
 * picture: a conventional encoder's first frame and scene cuts,
 * MASTER_DESIGN.md:39-40,85-90; CAVLC) coded for a
 * picture of w x h MBs with the composed stream's SPS/PPS fields
 * (log2_max_frame_num, POC type, num_ref_idx default, deblocking flag); the
 * rect [x0, x0 + w) x [y0, y0 + h) of the composed picture receives its MBs.
 * The picture may come as several slices (Annex-B NAL units one after
 * the other, in MB order, together covering the w x h MBs once: first slice
 * at MB 0, each next one at the MB after the previous one's last; any MB
 * boundary, e.g. one slice per MB row, MASTER_DESIGN.md:170,217).  Per
 * slice: no ref_pic_list_modification or one that restates the composed list
 * (op k: long_term_pic_num k, as the composer's own slices write it,
 * h264_writer.c:455-539), no deblocking when the PPS allows switching it off
 * (disable_deblocking_filter_idc 1, like the composer's own slices); MBs of
 * every P type (P_L0_16x16, P_L0_L0_16x8, P_L0_L0_8x16, P_8x8 with any
 * sub_mb_types, P_8x8ref0), P_Skip, and the intra types a P slice carries
 * (mb_type 5 I_4x4, 6..29 I_16x16, 30 I_PCM; the reference's own P-slice
 * walker takes all three, trans_resizer.c:1668-1748), any
 * coded_block_pattern, mb_qp_delta and CAVLC residual (level_prefix <= 15).
 * Neighbours in another slice are unavailable in the external picture
 * (6.4.x): motion prediction, P_Skip motion, nC and intra prediction see
 * them so.
 * Intra MBs: their sample prediction reads neighbour MBs, so an I_4x4 /
 * I_16x16 MB is spliced only where each neighbour MB its prediction uses
 * has the same availability in the external and the composed picture (a
 * neighbour inside the rect and the same slice: the same MB in both; outside
 * the rect it is available in the composed picture unless past its edge):
 * I_16x16 luma / chroma modes their A / B / D per mode (8.3.3, 8.3.4),
 * I_4x4 always A and B (intra mode prediction, 8.3.1.1), D when raster block
 * 0 uses a mode reading p[-1, -1] (4, 5, 6), C when raster block 3 uses one
 * reading above-right samples (3, 7).  So interior MBs of a one-slice picture
 * always qualify, the rect's left / top edge only at the composed picture's
 * edge, its right edge without above-right modes.  I_PCM anywhere.  Else
 * OR_SPLICE_ERR_MBTYPE.
 * Its ref_idx values index the composed stream's list (0 = A, 1 = B, 2 + i =
 * waypoint i) and its motion vectors are displacements in composed-picture
 * coordinates.
 *
 * An I slice (slice_type 2 / 7; IDR: idr_pic_id, the IDR dec_ref_pic_marking)
 * has no mb_skip_run and its MBs' mb_type k (Table 7-11: 0 I_4x4, 1-24
 * I_16x16, 25 I_PCM) is the P slice's intra mb_type 5 + k, under the same
 * availability rule (trans_resizer.c:1063 process_i_slice, :887-1058).
 * Transplant, per spliced MB (composed slice QP 26):
 *   - P_Skip becomes P_L0_16x16 with ref 0 and its P_Skip motion (8.4.1.1,
 *     evaluated in the external picture), cbp 0;
 *   - mb_skip_run, ref_idx te() (composed num_ref_idx = 2 + waypoints) and
 *     mvd (prediction in the composed picture: the reference's
 *     get_mv_prediction in EXACT mode, 8.4.1.3 in PSKIP mode) are re-coded;
 *   - a partitioned MB keeps its partitioning (P_8x8ref0 becomes P_8x8 with
 *     ref_idx 0 written) and codes every (sub-)partition's mvd against the
 *     8.4.1.3 prediction (directional 16x8 / 8x16 rules, 4x4-block
 *     neighbours, C -> D substitution, not-yet-decoded partitions
 *     unavailable) in the composed picture, in every mode; neighbours of
 *     any MB are the 4x4 blocks the standard names (A: left of the top-left
 *     block, B: above it, C: above-right of the top-right, D: above-left);
 *   - mb_qp_delta is rebased so each MB keeps its external QP;
 *   - every residual block keeps its bits after coeff_token verbatim (they do
 *     not depend on nC); coeff_token is re-coded for the nC of the composed
 *     picture (rect-edge neighbours are available MBs with TotalCoeff 0);
 *   - an intra MB keeps mb_type and its prediction syntax (I_4x4: the 16
 *     prev_intra4x4_pred_mode / rem fields, and intra_chroma_pred_mode) and
 *     I_4x4's coded_block_pattern codeNum verbatim; I_16x16's DC block is one
 *     more re-contexted piece; I_PCM is realigned (pcm_alignment_zero_bits
 *     for its composed position) and its 384 samples copied.  In the
 *     composed motion field an intra MB is available with refIdx -1, mv 0
 *     (8.4.1.3.1); it is never skipped.
 * MBs outside the rect follow the UI-hint composition (hint_oracle.h) of
 * the frame, whose neighbour predictions now see the spliced motion.
 */
#ifndef SPLICE_ORACLE_H
#define SPLICE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "hint_oracle.h"
#include "dyn_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

/* error codes (same values as SCROLL_SPLICE_ERR_* in include/composer_batch.h) */
#define OR_SPLICE_OK 0
#define OR_SPLICE_ERR_NAL 1      /* not a coded slice (nal_unit_type 1 or 5)      */
#define OR_SPLICE_ERR_HEADER 2   /* slice header outside the supported syntax     */
#define OR_SPLICE_ERR_MBTYPE 3   /* an intra MB whose prediction would change     */
#define OR_SPLICE_ERR_SYNTAX 4   /* malformed / truncated slice data              */
#define OR_SPLICE_ERR_REF 5      /* ref_idx not a valid reference of the frame    */

#define OR_SPLICE_PIECES 27      /* 16 luma (raster; I_16x16: AC), Cb DC, Cr DC, 4 Cb AC, 4 Cr AC,
                                  * I_16x16 luma DC */
#define OR_SPLICE_MAX_MV 16383   /* |mv| in quarter pels */

typedef struct {
    int x0, y0, w, h;            /* MB units in the composed picture */
    const uint8_t *nal;          /* the external NAL (leading Annex-B start code optional) */
    size_t n;
} or_splice;

/* one external MB after parsing */
typedef struct {
    int ref, mx, my;             /* quarter pels (partitioned: 4x4 block 0's) */
    int cbp, qp, qpd;            /* its QP and the composed mb_qp_delta      */
    int skip;                    /* P_Skip in the external slice             */
    uint8_t tc[OR_SPLICE_PIECES], t1[OR_SPLICE_PIECES];
    uint32_t boff[OR_SPLICE_PIECES], blen[OR_SPLICE_PIECES];  /* body bits in the RBSP */
    int part;                    /* 0 P_L0_16x16 / P_Skip, 1 16x8, 2 8x16, 3 P_8x8 (and P_8x8ref0) */
    int sub;                     /* P_8x8: sub_mb_type of 8x8 i in bits 2i..2i+1 (0 8x8, 1 8x4, 2 4x8, 3 4x4) */
    int bref[16], bmx[16], bmy[16];  /* motion per 4x4 block, raster order  */
    int intra;                   /* 0 inter / P_Skip, 1 I_4x4, 2 I_16x16, 3 I_PCM */
    int mbt;                     /* intra: its mb_type (5..30)                */
    uint32_t poff, plen;         /* intra: prediction syntax bits in the RBSP */
    int cbp_code;                /* I_4x4: coded_block_pattern codeNum        */
    uint32_t pcm;                /* I_PCM: byte offset of its samples in the RBSP */
    int hasqpd;                  /* carries mb_qp_delta                       */
} or_splice_mb;

/* Parse the external slice: mbs[w * h] (raster), its RBSP into rbsp (cap
 * >= n bytes), *rbsp_n = its bytes.  Returns OR_SPLICE_OK or an error. */
int or_splice_parse(const or_cfg *c, const or_splice *sp, or_splice_mb *mbs, uint8_t *rbsp,
                    size_t *rbsp_n);

/* The scroll NAL of a frame at offset `off` with hint rects r[0..n) in
 * `mode` (OR_HINT_EXACT / OR_HINT_PSKIP) and the splice sp (NULL = none);
 * frame_num++.  Returns the Annex-B bytes, or 0 with *err = OR_SPLICE_ERR_*
 * (or 1 + 0x100 for an invalid hint-rect reference); the state is then left
 * unchanged. */
size_t or_splice_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off, const or_hint_rect *r,
                            int n, int mode, const or_splice *sp, int *err);

/* composer_write_scroll_frame (src/composer.c:255-264) with that scroll NAL */
size_t or_compose_splice(uint8_t *dst, size_t cap, or_cfg *c, int off, int compose_mode,
                         const or_hint_rect *r, int n, int mode, const or_splice *sp, int *err);

/* ---- the dynamic rect under UI hints (docs/MASTER_DESIGN.md:58-64,
 * 109-113, 121-146: one per-frame hint record holds the motion regions AND
 * the dynamic rect; no reference implementation, this DEFINES the bits) ----
 * The frame's MV field is the UI-hint field (hint_oracle.h); the MBs of the
 * dynamic rect rc (its position may change from frame to frame and stream to
 * stream) keep their (ref, mv) from that field and carry the residual of the
 * rect source src (dyn_oracle.h layout for rc) minus the prediction at that
 * motion: full-pel luma, 1/8-pel 2-D bilinear chroma (8.4.2.2.2), samples
 * clamped to the picture, waypoints resolved through their own rows
 * (or_ref_sample); 4x4 transform + quant at QP 26 and CAVLC as in
 * dyn_oracle.h.  The MBs are then composed exactly like spliced MBs
 * (or_splice_scroll_nal): mb_skip_run / ref_idx / mvd for the frame's hint
 * mode (an MB without residual can be a P_Skip in OR_HINT_PSKIP), cbp,
 * mb_qp_delta 0, coeff_token for the composed nC.  rc NULL or empty: the
 * hint NAL.  Returns the Annex-B bytes, or 0 with *err (OR_SPLICE_ERR_REF:
 * a rect MB's hint reference is not valid in the frame). */
size_t or_hint_dyn_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off, const or_hint_rect *r,
                              int n, int mode, const or_dyn_rect *rc, const uint8_t *src,
                              const or_refs *R, int *err);
size_t or_compose_hint_dyn(uint8_t *dst, size_t cap, or_cfg *c, int off, int compose_mode,
                           const or_hint_rect *r, int n, int mode, const or_dyn_rect *rc,
                           const uint8_t *src, const or_refs *R, int *err);

/* after or_splice_parse (or a compose) failed with OR_SPLICE_ERR_MBTYPE: the
 * refused MB's index in the external picture | its P-slice mb_type << 16;
 * -1 otherwise (scroll_batch_splice_refusal's oracle) */
int or_splice_refused(void);

/* ---- test-input generator: a stand-in "dynamic encoder" (MASTER_DESIGN
 * §4.2) writing standard CAVLC P slices of a w x h MB picture with random
 * MBs, so the tests have external slices to splice ---- */
typedef struct {
    int nrefs;                   /* num_ref_idx_l0_active; 0 = the PPS default   */
    int max_ref;                 /* MB refs drawn from [0, max_ref]             */
    int skip_pm;                 /* per mille: MB coded as P_Skip              */
    int cbp_pm;                  /* per mille: MB with a residual              */
    int big_pm;                  /* per mille: level drawn large (escape codes) */
    int mv_range;                /* |mv| <= mv_range quarter pels               */
    int slice_qp_delta;
    int qp_jitter;               /* |mb_qp_delta| <= qp_jitter                  */
    int ref_idc;                 /* nal_ref_idc (adds dec_ref_pic_marking)      */
    int bad_mb;                  /* -1, or the MB coded with mb_type bad_type   */
    int bad_type;
    int list_mod;                /* 0 none, 1 the composed list restated (long-term
                                  * k at index k), 2 reversed (unsupported)      */
    int part_pm;                 /* per mille of coded MBs: P_L0_L0_16x8 / 8x16,
                                  * P_8x8 (random sub_mb_types) or P_8x8ref0     */
    int intra_pm;                /* per mille of coded MBs: I_4x4 / I_16x16 / I_PCM,
                                  * only where any rect placement splices them
                                  * (not on the picture's edges, the top MB row of
                                  * a slice, an I_4x4 not on the right column)   */
    int slice_rows;              /* 0: one slice; k: a slice per k MB rows       */
    int pcm_zero;                /* I_PCM samples all 0 (emulation prevention)   */
    int intra_types;             /* 0: all; else bit 0 I_4x4, 1 I_16x16, 2 I_PCM  */
    int islice;                  /* 0: P slices; 1: I slices (every MB intra: I_4x4 /
                                  * I_16x16 where any rect placement splices them,
                                  * else I_PCM -- the edge ring); 2: the same as an
                                  * IDR picture (nal_unit_type 5); 3: I slices of
                                  * intra_types everywhere, edge ring included (a
                                  * syntax check for the reference's I-slice walker) */
} or_ext_params;
size_t or_ext_slice(uint8_t *dst, size_t cap, const or_cfg *c, int w, int h, uint32_t seed,
                    const or_ext_params *p);

#ifdef __cplusplus
}
#endif
#endif
