/*
 * composer_batch.h -- ADDITIVE many-stream API (no reference counterpart).
 *
 * The reference API is synchronous, single-stream and single-frame
 * (include/composer.h:79, include/h264_writer.h:124).  Throughput on an
 * MI355X needs many (stream, frame) items per launch, so this header adds a
 * batch object that keeps every stream's ComposerConfig state, its scroll
 * offsets ("UI hints") and its Annex-B output arena resident in HBM:
 *
 *   scroll_batch_create()            one batch per GPU (device ordinal)
 *   scroll_batch_add_stream(cfg)     a stream = one ComposerConfig
 *   scroll_batch_set_offsets()       [streams][frames] offsets -> HBM
 *   scroll_batch_compose(n, stream)  async: GPU state machine (waypoints,
 *                                    frame_num) + P-slice kernels; appends
 *                                    n composed frames to every stream arena
 *   scroll_batch_sync()              wait + surface device error words
 *   scroll_batch_copy_output()       arena -> host
 *
 * Semantics per stream are exactly n calls of composer_write_scroll_frame
 * (src/composer.c:255-264), or of the experiment's loop body
 * (experiments/scroll-encoder/src/main.c:418-424) in SCROLL_MODE_EXPERIMENT.
 * Streams are independent; multi-GPU = one batch per device with a static
 * contiguous shard of the streams (no collective).
 *
 * All functions return SCROLL_OK (0) or a negative SCROLL_ERR_* code;
 * scroll_last_error() has the message.  No CPU fallback exists: without a
 * usable gfx950 device every compose call fails with SCROLL_ERR_NO_DEVICE.
 */
#ifndef COMPOSER_BATCH_H
#define COMPOSER_BATCH_H

#include <stddef.h>
#include <stdint.h>
#include "composer.h"
#include "h264_writer.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SCROLL_OK             0
#define SCROLL_ERR_NO_DEVICE (-1)
#define SCROLL_ERR_ARG       (-2)
#define SCROLL_ERR_OOM       (-3)
#define SCROLL_ERR_OVERFLOW  (-4)   /* output arena full (reference: assert abort) */
#define SCROLL_ERR_HIP       (-5)
#define SCROLL_ERR_CONFIG    (-6)   /* config outside the supported syntax range  */
#define SCROLL_ERR_DEVICE    (-7)   /* a device-side wait timed out (the dynamic rect's
                                       row hand-off): that stream committed nothing */

#define SCROLL_MODE_COMPOSER   0    /* waypoint NAL in addition to the scroll NAL */
#define SCROLL_MODE_EXPERIMENT 1    /* waypoint NAL instead of the scroll NAL     */

/* debug flags (tests / profiling ablations; outputs are wrong for 2, 4, 8) */
#define SCROLL_DEBUG_FORCE_SERIAL 1 /* every NAL through the serial device path   */
#define SCROLL_DEBUG_EMIT_NOSTORE 2 /* k_emit computes every chunk, stores none   */
#define SCROLL_DEBUG_EMIT_ZEROS   4 /* k_emit stores zero chunks, computes none   */
#define SCROLL_DEBUG_EMIT_BUILD   8 /* k_emit builds the layouts and stops        */
#define SCROLL_DEBUG_EMIT_NOPURE 16 /* k_emit skips the pure-chunk phase          */
#define SCROLL_DEBUG_EMIT_NOMIXED 32 /* k_emit skips the mixed-chunk phase        */
#define SCROLL_DEBUG_EMIT_STAMPS 64 /* k_emit records s_memtime per phase per wave */
#define SCROLL_DEBUG_EMIT_NOBYTES 128 /* k_emit skips the tile-end partial chunks  */
#define SCROLL_DEBUG_DYN_STAMPS 256 /* k_dyn_row / gather: realtime per phase    */
/* retired: runtime ablations of the earlier one-kernel dynamic coder (no
 * kernel reads them now; k_dyn_row's per-phase ablation is the compile-time
 * variant -DSCROLL_ABL_STOP=n).  Values kept so the flag numbering stays
 * stable. */
#define SCROLL_DEBUG_DYN_NOLOAD  512
#define SCROLL_DEBUG_DYN_NOCAVLC 1024
#define SCROLL_DEBUG_DYN_NOHEAD  2048
#define SCROLL_DEBUG_DYN_NOWRITE 4096
/* tests: the dynamic emit keeps at most 4 EP positions per NAL, so every NAL
 * with more emulation-prevention bytes takes the large-NAL path (k_dyn_emit,
 * otherwise only reached past 2,048 EP bytes); output unchanged */
#define SCROLL_DEBUG_DYN_EPCAP4 8192
/* tests: k_dyn_row of stream 0, frame 0, rect row 0 does not publish its
 * bottom TotalCoeffs, so row 1's bounded wait expires: stream 0 fails with
 * SCROLL_ERR_DEVICE, every other stream composes normally */
#define SCROLL_DEBUG_DYN_NOPUBLISH 16384
/* tests: the dynamic rect's NALs go to the arena through the round-3 gather
 * (k_dyn_emit_gather) instead of k_dyn_gather; output unchanged */
#define SCROLL_DEBUG_DYN_GATHER1 32768
/* tests: the dynamic rect's EP-position machinery of the whole-picture rects
 * on any rect -- the 8,192-entry epfix set and list, and k_dyn_gather's LDS
 * windows at 7 positions each (every NAL with more EP bytes is gathered
 * window by window); output unchanged.  Set before scroll_batch_set_dyn_rect */
#define SCROLL_DEBUG_DYN_EPWIN 65536

typedef struct ScrollBatch ScrollBatch;

typedef struct {
    int device;            /* HIP device ordinal                               */
    int max_streams;
    int max_frames;        /* max composed frames per scroll_batch_compose    */
    size_t arena_bytes;    /* device output arena per stream                   */
    int mode;              /* SCROLL_MODE_*                                    */
} ScrollBatchDesc;

const char *scroll_last_error(void);
int scroll_device_count(void);                 /* usable gfx950 devices (0 if none) */
const char *scroll_version(void);

int scroll_batch_create(ScrollBatch **out, const ScrollBatchDesc *desc);
void scroll_batch_destroy(ScrollBatch *b);
int scroll_batch_add_stream(ScrollBatch *b, const ComposerConfig *cfg); /* -> stream id */
int scroll_batch_num_streams(const ScrollBatch *b);
int scroll_batch_set_debug(ScrollBatch *b, int flags);

/* offsets: host array [num_streams][nframes] (row stride nframes) */
int scroll_batch_set_offsets(ScrollBatch *b, const int32_t *offsets, int nframes);
/* device array [num_streams][max_frames]; fill it from device code to skip H2D */
int32_t *scroll_batch_offsets_device(ScrollBatch *b);

/* async on hip_stream (hipStream_t; NULL = the batch's own stream) */
int scroll_batch_compose(ScrollBatch *b, int nframes, void *hip_stream);
/* flags: SCROLL_COMPOSE_REWIND = start every arena at 0 (the caller has
 * consumed the previous batch's bytes) -- device-side, no host sync. */
#define SCROLL_COMPOSE_REWIND 1
int scroll_batch_compose_ex(ScrollBatch *b, int nframes, void *hip_stream, int flags);
int scroll_batch_sync(ScrollBatch *b);

/* state after sync: ComposerConfig as the reference would hold it */
int scroll_batch_get_config(ScrollBatch *b, int s, ComposerConfig *cfg);
int scroll_batch_set_config(ScrollBatch *b, int s, const ComposerConfig *cfg);
size_t scroll_batch_output_size(ScrollBatch *b, int s);
int scroll_batch_copy_output(ScrollBatch *b, int s, size_t from, uint8_t *dst, size_t n);
const uint8_t *scroll_batch_output_device(ScrollBatch *b, int s);
/* Host delivery (the reference returns its bytes in host memory,
 * composer.c:255-291): pinned host buffers the device writes into, and the
 * bytes appended to every stream since its previous delivery (composes,
 * reference updates; a rewound arena starts over) packed into dst back to
 * back in stream order, asynchronously on hip_stream (NULL = the stream of
 * the last compose; another stream waits for it).  table (pinned, 1 + 2 S
 * u64) gets [0] = the packed size (~0: larger than cap, nothing written),
 * then per stream its offset in dst (16-byte aligned) and its byte count.
 * dst and cap 16-byte aligned.  Valid after scroll_batch_sync / a stream
 * sync; the arenas must not be rewritten before the copy has run. */
int scroll_host_alloc(void **p, size_t n);
void scroll_host_free(void *p);
int scroll_batch_output_to_host_async(ScrollBatch *b, uint8_t *dst, size_t cap, uint64_t *table,
                                      void *hip_stream);
int scroll_batch_reset_output(ScrollBatch *b);   /* rewind all arenas, keep state */

/* last compose: planned NAL units of stream s (kind/size/offset per NAL) */
int scroll_batch_nal_count(ScrollBatch *b, int s);
int scroll_batch_nal_info(ScrollBatch *b, int s, int i, int *kind, int *offset_px,
                          uint32_t *size, int *slow);

/* HIP-event timing of the last compose's kernels, on the launch stream:
 * which 0 = plan kernel(s), 1 = emit kernel, 2 = dyn stage, 3 = dyn emit,
 * 4 = dyn code (k_dyn_rows + k_dyn_code), 5 = dyn pack (k_dyn_group + k_dyn_ep).
 * Enable before compose: on = 1 every pair (kernel_ms and kernel_stats_ex
 * complete); on = 2 ("lite") only the dominant kernel's pair -- dyn code
 * (also reported as dyn stage) or emit -- into kernel_stats_ex, the others
 * 0: each event record is a marker packet that holds the queue between the
 * kernels, so a timed step with every pair runs ~ 40 us longer; 0 off.
 * kernel_ms returns -1 while lite timing is on (no per-kernel pairs exist). */
int scroll_batch_enable_timing(ScrollBatch *b, int on);
float scroll_batch_kernel_ms(ScrollBatch *b, int which);
/* all timed composes since the last call: summed plan / emit kernel ms and
 * the number of composes; the accumulators are reset afterwards */
int scroll_batch_kernel_stats(ScrollBatch *b, double *plan_ms, double *emit_ms, int *count);
/* SCROLL_DEBUG_EMIT_STAMPS: copy the per-wave phase stamps of the last
 * compose (8 x u64 per wave slot); returns the number of wave slots */
long long scroll_batch_debug_stamps(ScrollBatch *b, uint64_t *dst, long long max_slots);
/* bytes appended to every arena by the last compose (sum over streams) */
unsigned long long scroll_batch_last_bytes(ScrollBatch *b);
/* NAL units planned by the last compose (sum over streams) */
long long scroll_batch_last_nals(ScrollBatch *b);

/* ---- dynamic rect (BASELINE configs 3-5; no reference counterpart) ----
 * Every scroll NAL of the batch carries a rectangle of dynamic MBs: they keep
 * their row's (ref_idx, mv) and add coded_block_pattern, mb_qp_delta and a
 * CAVLC residual of (source - prediction) at QP 26 or the rect's QP
 * (scroll_batch_set_dyn_qp; bit-exact definition:
 * oracle/dyn_oracle.h).  Waypoint NALs stay residual-free.  All streams of
 * the batch must share one picture size; call after adding the streams.
 *
 *   scroll_batch_set_dyn_rect(b, x0, y0, w, h, slot)   MB units; w or h = 0
 *       turns the rect off.  slot = staging bytes per frame, 0 = a bound no
 *       NAL can exceed (larger ones fail with SCROLL_ERR_OVERFLOW).
 *   scroll_batch_set_dyn_refs(b, s, a, b)   decoded reference pictures A and
 *       B (I420, w*h*3/2 bytes each) of stream s, or of every stream (s = -1)
 *   source pixels: [stream][frame] blocks of 384*w*h bytes (the rect's luma
 *       16w x 16h, then Cb, Cr 8w x 8h), frame f = the f-th composed frame of
 *       the next compose: scroll_batch_set_dyn_source (host copy),
 *       scroll_batch_dyn_source_device (fill in place), or
 *       scroll_batch_dyn_source_synth (the synthetic source of SURVEY §8d for
 *       global stream ids stream_base + s and frame numbers t0 + f). */
int scroll_batch_set_dyn_rect(ScrollBatch *b, int x0, int y0, int w, int h, size_t slot_bytes);
int scroll_batch_set_dyn_refs(ScrollBatch *b, int s, const uint8_t *ref_a, const uint8_t *ref_b);
/*   scroll_batch_set_dyn_qp(b, qp)   the rect's QP, 0..51 (default 26), of
 *       every stream (and of streams added later), for the following
 *       composes: a stream's dynamic scroll NALs then carry slice_qp_delta =
 *       qp - 26 (chroma at QPc, Table 8-15) and their MBs mb_qp_delta 0;
 *       waypoint NALs and the P-only path are unchanged.  Below 22 a NAL's
 *       levels need 16 bits and it is coded on the general path (records in
 *       HBM); levels are clamped to +-2063, the largest every CAVLC context
 *       codes with level_prefix <= 15 (reached only by chroma DC below QPc 6).
 *   scroll_batch_set_dyn_qp_stream(b, s, qp)   the same for stream s.
 *   scroll_batch_set_dyn_qp_at(b, s, f, qp)    under UI hints (the rect in the
 *       frame's hint record): frame f of stream s at QP qp, -1 = the
 *       stream's.  There the slice QP stays 26 and the rect's first MB with a
 *       residual carries mb_qp_delta qp - 26, the others 0.
 *   A stream with the deblocking filter on (no
 *   deblocking_filter_control_present_flag, e.g. an ingested one) keeps QP 26:
 *   another QP would change the filtering of its scroll MBs (SCROLL_ERR_CONFIG). */
#define SCROLL_DYN_QP_MIN 0
#define SCROLL_DYN_QP_MAX 51
int scroll_batch_set_dyn_qp(ScrollBatch *b, int qp);
int scroll_batch_set_dyn_qp_stream(ScrollBatch *b, int s, int qp);
int scroll_batch_set_dyn_qp_at(ScrollBatch *b, int s, int f, int qp);
int scroll_batch_set_dyn_source(ScrollBatch *b, const uint8_t *src, int nframes);
/* Under UI hints (scroll_batch_set_hints) the rect's MBs keep the hint
 * field's (ref, mv) -- full-pel luma, 2-D 1/8-pel chroma prediction at that
 * motion -- and the rect may sit anywhere in each frame:
 *   scroll_batch_set_dyn_rect_at(b, s, f, x0, y0)   frame f of stream s puts
 *       the rect's w x h MBs at (x0, y0); x0 = -1: no rect in that frame.
 *       Positions other than set_dyn_rect's need hints at compose time
 *       (SCROLL_ERR_CONFIG otherwise); clear_hints resets them.
 * Each rect MB's residual bits get a region of slot_bytes / (w h) bytes
 * (64 to 2048; slot_bytes 0: 512, which saturated +-255 residuals stay well
 * inside); an MB that outgrows it fails the compose with SCROLL_ERR_OVERFLOW.
 * Bit-exact definition: oracle/splice_oracle.h or_hint_dyn_scroll_nal.
 * Not combinable with spliced slices (one rect per frame). */
int scroll_batch_set_dyn_rect_at(ScrollBatch *b, int s, int f, int x0, int y0);
/* The conventional-encode fallback (docs/MASTER_DESIGN.md:220: "if hints
 * missing/inconsistent -> full conventional encode"), opt-in:
 *   scroll_batch_set_fallback(b, 1)   with UI hints and a dynamic rect that
 *       is the whole picture (set_dyn_rect(b, 0, 0, width / 16, height / 16,
 *       ...): every frame's source is then a whole picture, as a conventional
 *       encoder's).  A frame whose hints put an MB on a rect naming a
 *       reference the frame lacks -- a frame that fails its stream with
 *       SCROLL_ERR_CONFIG without the flag -- is coded instead as a full
 *       P frame: its hint rects dropped, every MB on the scroll frame's own
 *       motion with the residual of the frame's source (the rect at (0, 0),
 *       whether or not set_dyn_rect_at placed it), in the frame's hint mode
 *       and rect QP.  Other frames are unchanged.  SCROLL_ERR_CONFIG when the
 *       rect is not the whole picture.
 *   scroll_batch_fallback_frame(b, s, f, &on)   after a compose: 1 when
 *       frame f of stream s fell back.
 * Bit-exact definition: oracle/splice_oracle.h or_compose_hint_dyn with no
 * hint rects and the whole-picture rect. */
int scroll_batch_set_fallback(ScrollBatch *b, int on);
int scroll_batch_fallback_frame(ScrollBatch *b, int s, int f, int *fell_back);
uint8_t *scroll_batch_dyn_source_device(ScrollBatch *b, size_t *stream_stride,
                                        size_t *frame_stride);
int scroll_batch_dyn_source_synth(ScrollBatch *b, int nframes, int stream_base, int t0);
/* last compose, frame f of stream s: staged RBSP bytes and EP bytes */
int scroll_batch_dyn_frame_info(ScrollBatch *b, int s, int f, uint32_t *rbsp_bytes,
                                uint32_t *ep_bytes);
/* last compose, all streams: staged RBSP bytes, EP bytes, dynamic NALs */
int scroll_batch_dyn_totals(ScrollBatch *b, unsigned long long *rbsp_bytes,
                            unsigned long long *ep_bytes, long long *dyn_nals);
/* HIP-event ms of the timed composes since the last call: plan (both
 * passes), emit, dyn stage (= dyn code + dyn pack), dyn emit, dyn code
 * (k_dyn_rows + k_dyn_code), dyn pack (k_dyn_group + k_dyn_ep); accumulators reset
 * afterwards */
int scroll_batch_kernel_stats_ex(ScrollBatch *b, double ms[6], int *count);

/* ---- UI hints (reference design docs/MASTER_DESIGN.md:
 * 58-64,103-146, no reference implementation) ----
 * Rectangles of MBs with their own reference and displacement, laid over
 * the scroll layout of the frame's offset: static chrome, a horizontally
 * scrolling row, a second pane.  MBs no rect covers keep the scroll frame's
 * (ref, mv).  Later rects lie on top.  Bit-exact definition:
 * oracle/hint_oracle.h.  Once hints are set, every scroll NAL of the batch
 * is coded per MB (waypoint NALs are unchanged); a frame without hints then
 * equals the reference's scroll frame byte for byte in SCROLL_HINT_EXACT.
 *
 *   modes: SCROLL_HINT_EXACT  the reference's MB syntax (mb_skip_run 0,
 *              get_mv_prediction of h264_writer.c:369-432) for any MV field;
 *          SCROLL_HINT_PSKIP  standard median prediction (H.264 8.4.1.3) and
 *              P_Skip runs for ref-0 MBs on their skip motion (8.4.1.1);
 *          SCROLL_HINT_SPEC   the reference's MB syntax (no skipped MBs) with
 *              the standard's median prediction: a standard decoder gets the
 *              intended motion for any MV field, and the plain scroll layout
 *              is still the reference's frame byte for byte (a row-uniform
 *              field never reaches the cases where get_mv_prediction departs
 *              from 8.4.1.3).
 *   scroll_batch_set_hints(b, s, f, rects, n, mode)   hints of frame f (the
 *       f-th frame of each following compose) of stream s; n <=
 *       SCROLL_HINT_MAX_RECTS; n = 0 gives the plain layout in `mode`.  A
 *       rect whose ref is not a valid reference of its frame (2 + i needs
 *       waypoint i) fails that stream's compose with SCROLL_ERR_CONFIG.
 *   scroll_batch_clear_hints(b)   back to plain scroll frames (k_emit path).
 * Pictures up to 240 MBs (3840 px) wide.
 * With a dynamic rect: see scroll_batch_set_dyn_rect_at. */
#define SCROLL_HINT_EXACT 0
#define SCROLL_HINT_PSKIP 1
#define SCROLL_HINT_SPEC 2
#define SCROLL_HINT_MAX_RECTS 64
#define SCROLL_HINT_MAX_MV 8192     /* |mv_x|, |mv_y| in pixels */
typedef struct ScrollHintRect {
    int16_t x0, y0, x1, y1;         /* MBs [x0, x1) x [y0, y1), clipped to the picture */
    int16_t ref;                    /* 0 = A, 1 = B, 2 + i = waypoint i               */
    int16_t reserved;               /* 0                                              */
    int32_t mv_x, mv_y;             /* pixels: MB (x, y) predicts from (16x + mv_x, 16y + mv_y) */
} ScrollHintRect;
int scroll_batch_set_hints(ScrollBatch *b, int s, int f, const ScrollHintRect *rects, int n,
                           int mode);
int scroll_batch_clear_hints(ScrollBatch *b);

/* ---- pre-encoded MB splice (reference design
 * docs/MASTER_DESIGN.md:39-40,87-90,142-146,166-171, no reference
 * implementation) ----
 * The MBs of an external P slice -- a conventional encoder's output for the
 * dynamic rect, coded as its own w x h MB picture -- are transplanted into
 * the rect [x0, x0 + w) x [y0, y0 + h) of frame f's scroll NAL: P_Skip MBs
 * become P_L0_16x16 with their skip motion, partitioned MBs keep their
 * partitioning (P_8x8ref0 written as P_8x8 with ref_idx 0), mb_skip_run /
 * ref_idx / every (sub-)partition's mvd are re-coded for the composed
 * picture (4x4-block neighbours, 8.4.1.3), mb_qp_delta rebased to the composed
 * slice QP, each residual block keeps its bits after coeff_token and gets
 * the coeff_token of its composed nC.  MBs outside the rect follow the frame's
 * UI hints (a splice turns the hint path on in SCROLL_HINT_SPEC, so a standard
 * decoder gets the spliced motion, and frames without a splice and without
 * hints still equal the reference's scroll frames; set_hints(.., NULL, 0,
 * SCROLL_HINT_PSKIP) adds P_Skip runs, SCROLL_HINT_EXACT the reference's own
 * predictor).
 * Bit-exact definition: oracle/splice_oracle.h.
 *
 * The external picture: one NAL (Annex-B start code optional), or several
 * Annex-B NAL units -- its slices, in MB order, each starting at the MB after
 * the previous one's last (first_mb_in_slice), together covering the w*h MBs
 * (at most 1,024 slices; each is parsed by its own wave); P slices or I
 * slices (nal_unit_type 1, or 5 for an IDR picture: a conventional encoder's
 * first frame and scene cuts; an I slice's MBs are the P slice's intra types,
 * without mb_skip_run), CAVLC, parsed with the composed stream's SPS/PPS (log2_max_frame_num, POC
 * type, 2 default references, disable_deblocking_filter_idc 1 when the
 * stream signals deblocking control); no ref_pic_list_modification, or one
 * that restates the composed list (op k: long_term_pic_num k, as the
 * composer's own slices write it); MBs of any inter type (P_L0_16x16,
 * P_L0_L0_16x8 / 8x16, P_8x8 with any sub_mb_types, P_8x8ref0), P_Skip, and
 * the intra types of a P slice (I_4x4, I_16x16, I_PCM) where the neighbour
 * MBs their sample prediction reads have the same availability in the
 * external and the composed picture (so not on the rect's left / top edge
 * unless that is the picture's, no above-right I_4x4 modes on its right
 * edge; I_PCM anywhere; splice_oracle.h has the rule);
 * ref_idx 0 = A, 1 = B, 2 + i = waypoint i of the composed stream; motion
 * vectors are displacements in the composed picture, |mv| <= 16383 quarter
 * pels; CAVLC level_prefix <= 15 (Baseline / Main).
 *
 *   scroll_batch_set_splice(b, s, f, x0, y0, w, h, nal, n)   frame f of
 *       stream s, for every following compose; n = 0 removes it.  The slice
 *       is parsed on the GPU by the next compose; a slice outside the
 *       supported syntax, or a reference the frame does not have, fails that
 *       stream's compose with SCROLL_ERR_CONFIG (nothing of the batch is
 *       written for the stream) and scroll_batch_splice_status gives the
 *       reason (SCROLL_SPLICE_ERR_*).
 *   scroll_batch_clear_splices(b)   remove every splice (hints stay).
 * The staging slots grow to the largest spliced NAL's bound (about the
 * external slice plus 16 bytes per picture MB) for every (stream, frame). */
#define SCROLL_SPLICE_MAX_BYTES   ((uint64_t)1 << 29)   /* n < 512 MiB: 32-bit bit offsets */
#define SCROLL_SPLICE_OK          0
#define SCROLL_SPLICE_ERR_NAL     1   /* not a coded slice (nal_unit_type 1 / 5), or
                                       * more than 1,024 slices                      */
#define SCROLL_SPLICE_ERR_HEADER  2   /* slice header outside the supported syntax  */
#define SCROLL_SPLICE_ERR_MBTYPE  3   /* an intra MB whose prediction would change   */
#define SCROLL_SPLICE_ERR_SYNTAX  4   /* malformed, truncated or MB count mismatch   */
#define SCROLL_SPLICE_ERR_REF     5   /* ref_idx not a valid reference of the frame  */
int scroll_batch_set_splice(ScrollBatch *b, int s, int f, int x0, int y0, int w, int h,
                            const uint8_t *nal, size_t n);
/* the same for many frames at once, the NALs already in device memory (e.g.
 * a dynamic encoder's output arena on the same GPU): nal = device pointer,
 * read by the next compose (keep it valid and unchanged until that compose
 * has been synced); n = 0 removes the entry's splice.  Each call marks the
 * slices changed, so the next compose parses them again (new content in
 * place needs only another call). */
typedef struct ScrollSpliceDesc {
    int32_t s, f;                   /* stream, frame                              */
    int32_t x0, y0, w, h;           /* MB rect                                    */
    const uint8_t *nal;             /* device pointer to the external NAL         */
    uint64_t n;                     /* its bytes                                  */
} ScrollSpliceDesc;
int scroll_batch_set_splices_device(ScrollBatch *b, int n, const ScrollSpliceDesc *d);
int scroll_batch_clear_splices(ScrollBatch *b);
/* after sync: SCROLL_SPLICE_* of frame f of stream s in the last compose
 * (SCROLL_SPLICE_OK also when the frame has no splice) */
int scroll_batch_splice_status(ScrollBatch *b, int s, int f, int *status);
/* the same, and for SCROLL_SPLICE_ERR_MBTYPE the refused MB: its position in
 * the external picture (MB units) and its mb_type in P-slice numbering (5
 * I_4x4, 6..29 I_16x16; an I slice's k is 5 + k) -- the MB a caller can
 * re-code as I_PCM or with a mode that reads no neighbour across the rect's
 * edge (the margin ring, docs/MASTER_DESIGN.md:54-56); -1 otherwise */
int scroll_batch_splice_refusal(ScrollBatch *b, int s, int f, int *status, int *mb_x, int *mb_y, int *mb_type);

/* ---- stream ingest on the GPU ----
 * Batched composer_init + composer_write_header (reference src/composer.c:
 * 127-253): n new streams from their reference files (Annex-B with SPS, PPS
 * and an IDR slice: A and B), parsed and rewritten on the GPU.  Each new
 * stream's arena starts with SPS + PPS + IDR A (long-term 0) + non-IDR I B
 * (long-term 1), byte-identical to the reference; its config is the one
 * composer_init derives (log2_max_frame_num 4, POC type 2, A's deblocking
 * flag; frame_num 2 after the header).  Synchronous.  On an error no stream
 * is added and the message names the first failing one (missing NAL unit,
 * unsupported SPS/PPS, A/B size mismatch, header larger than the arena).
 *   scroll_batch_ingest(b, n, a, na, b_, nb, &first)   host files
 *   scroll_batch_ingest_device(b, n, d_files, desc, &first)   files already in
 *       device memory: desc[4k..4k+3] = offset, size of A, offset, size of B
 * The new streams get ids first .. first + n - 1.
 * Device scratch, kept by the batch for later calls: 2 n x 1.25 x the LARGEST
 * file's bytes (each slice body's 16 KB segments keep their output bytes
 * between the summary and the write pass, every file sized like the largest)
 * while that stays under 8 GB and under 4 x the input's bytes + 256 MB, else a
 * few hundred bytes per segment of the largest file (the write pass decodes
 * again).  Slices over 16 MB go one workgroup per stream, without scratch. */
int scroll_batch_ingest(ScrollBatch *b, int n, const uint8_t *const *ref_a, const size_t *na,
                        const uint8_t *const *ref_b, const size_t *nb, int *first);
int scroll_batch_ingest_device(ScrollBatch *b, int n, const uint8_t *d_files,
                               const uint64_t *desc, int *first);

/* Mid-stream long-term reference ("atlas") update -- SURVEY 8f row 3; the
 * reference only installs A / B at composer_write_header.  Entry k: the IDR
 * picture of Annex-B file k (parse_reference_file's rules, parsed with the
 * file's own SPS / PPS) becomes a non-IDR I frame of stream streams[k]
 * marked long_term_frame_idx which[k] (0 = A, 1 = B): the reference's
 * h264_rewrite_as_non_idr_i_frame (h264_writer.c:296-350) with the index as
 * a parameter, at the stream's frame_num, written with the stream's config,
 * appended after everything composed so far.  Its MMCO 4
 * (max_long_term_frame_idx_plus1 = 2) drops the stream's waypoints, so the
 * stream continues with an empty waypoint table and frame_num + 1; later
 * scroll frames predict from the new picture.  Streams distinct per call;
 * the picture must have the stream's size.  Synchronous; status[k] (may be
 * NULL) = 0 or the ingest error class (1 missing NAL, 2 refused SPS / PPS,
 * 3 size, 4 too many NALs, 5 arena full: nothing appended).  For a batch
 * with a dynamic rect also give the stream its new pictures
 * (scroll_batch_set_dyn_refs): prediction reads those. */
int scroll_batch_update_refs(ScrollBatch *b, int n, const int *streams, const int *which,
                             const uint8_t *const *files, const size_t *sizes, int *status);
/* the same from files already on the device (desc: offset, size per entry) */
int scroll_batch_update_refs_device(ScrollBatch *b, int n, const int *streams, const int *which,
                                    const uint8_t *d_files, const uint64_t *desc, int *status);
/* with timing enabled: summed ms of the ingest kernels (HIP events on the
 * batch's stream) and the number of ingest calls since the last call */
int scroll_batch_ingest_stats(ScrollBatch *b, double *ms, int *count);

/* ---- reference files from pictures on the GPU ----
 * The experiment's I_PCM reference writer (experiments/scroll-encoder/src/
 * h264_encoder.c:730-918: SPS + PPS + an IDR slice of I_PCM MBs, as the
 * SURVEY Appendix B harness frames it) generalised from one stripe colour per
 * MB to any I420 picture: n pictures at d_pics + i * pic_stride (Y w*h, then
 * Cb, Cr w*h/4 each, device memory) become n Annex-B files at d_out + i *
 * out_stride (device memory); sizes[i] (host) receives each file's bytes.
 * The files are what scroll_batch_ingest_device reads, so new streams (or a
 * new long-term reference picture) go from pixels to a composing stream
 * without leaving the GPU.  Synchronous; SCROLL_ERR_OVERFLOW (the sizes are
 * filled, nothing written) when a file exceeds out_stride -- at most
 * 1.5 x (w*h*193/128) + 128 bytes.  w, h multiples of 16, < 65536 MBs.
 * Device scratch, kept by the batch: the files' RBSP bytes (n x about 1.5 x
 * w*h, 4 KB aligned) while under 4 GB, which the write pass reads instead of
 * generating them again. */
int scroll_batch_ipcm_files_device(ScrollBatch *b, int n, int w, int h, const uint8_t *d_pics,
                                   size_t pic_stride, uint8_t *d_out, size_t out_stride,
                                   uint64_t *sizes);
/* the same without the host step: the sizes go to d_sizes (device, n u64)
 * and the call returns once its launches are queued on the batch's stream;
 * a file past out_stride (that call then writes no file) is reported by the
 * next scroll_batch_sync as SCROLL_ERR_OVERFLOW.  For pipelines that feed
 * the files straight to scroll_batch_ingest_device; the scratch is the
 * batch's, so calls of one batch run in stream order. */
int scroll_batch_ipcm_files_device_async(ScrollBatch *b, int n, int w, int h, const uint8_t *d_pics,
                                         size_t pic_stride, uint8_t *d_out, size_t out_stride,
                                         uint64_t *d_sizes);
/* with timing enabled: summed kernel ms of the calls above since the last
 * call (both passes) and the number of calls */
int scroll_batch_ipcm_stats(ScrollBatch *b, double *ms, int *count);

/* Composer-level batch: offsets[i] composed on cs[i], i < n, in
 * order; Composers may repeat.  Output lands in each Composer's buffer before
 * return (equivalent to n composer_write_scroll_frame calls + a flush). */
int composer_batch_write_scroll_frames(Composer *const *cs, const int *offsets, int n,
                                       int flags);
/* Force queued frames of c onto the GPU now (0 or SCROLL_ERR_*). */
int composer_flush(Composer *c);

#ifdef __cplusplus
}
#endif
#endif /* COMPOSER_BATCH_H */
