/*
 * engine.h -- internal interface between the host C drop-in layer
 * (composer.c, h264_writer.c) and the HIP engine (scroll_kernels.hip).
 * Not installed; the public ABI is the headers in include/.
 */
#ifndef SCROLL_ENGINE_H
#define SCROLL_ENGINE_H

#include <stddef.h>
#include <stdint.h>
#include "composer_batch.h"
#include "qparams.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device-resident per-stream state (one ComposerConfig + output arena).
 * 256 bytes, kept in HBM for the whole life of a ScrollBatch. */
typedef struct {
    int32_t w, h;                 /* cfg->width / cfg->height (pixels)          */
    int32_t log2_mfn;             /* log2_max_frame_num                         */
    int32_t poc_type;             /* pic_order_cnt_type                         */
    int32_t log2_poc;             /* log2_max_pic_order_cnt_lsb                 */
    int32_t deblock;              /* deblocking_filter_control_present_flag     */
    int32_t frame_num;            /* cfg->frame_num (monotonic, % on use)       */
    int32_t nwp;                  /* cfg->num_waypoints                         */
    int32_t wp_off[8];
    int32_t wp_lt[8];
    int32_t wp_valid[8];
    uint64_t out_pos;             /* bytes used in this stream's arena          */
    uint64_t out_cap;             /* arena capacity                             */
    int32_t frames;               /* composed frames requested in this batch    */
    int32_t nnal;                 /* NAL units planned in this batch            */
    int32_t nal_wp;               /* waypoint NAL units planned in this batch   */
    int32_t err;                  /* SCROLL_DEVERR_* bits                       */
    int32_t frames_written;       /* Composer::frames_written analogue          */
    int32_t n_slow;               /* NALs routed to the serial device path      */
    uint64_t batch_bytes;         /* bytes appended by this batch               */
    uint64_t undelivered;         /* arena bytes not yet packed to the host (output_to_host) */
    int32_t dyn_qp;               /* the dynamic rect's QP, 0..51 (scroll_batch_set_dyn_qp) */
    uint32_t pad[17];
} DevStream;

/* One planned NAL unit (32 bytes). */
typedef struct {
    uint64_t out_off;             /* byte offset in the stream arena            */
    uint32_t size;                /* bytes incl. 4-byte start code + NAL header */
    int32_t off;                  /* scroll offset (px)                         */
    int32_t frame_num;            /* raw cfg->frame_num when written            */
    uint8_t kind;                 /* 0 scroll P, 1 waypoint P                   */
    uint8_t nwp;                  /* cfg->num_waypoints snapshot                */
    uint8_t slow;                 /* 1: serial device path, 2: dynamic rect     */
    uint8_t pad0;
    uint32_t frame;               /* composed-frame index within the batch      */
    uint32_t pad1;
} NalDesc;

#define SCROLL_DEVERR_OVERFLOW 1u   /* arena too small (reference: assert)        */
#define SCROLL_DEVERR_CONFIG   2u   /* unsupported config (e.g. log2 fields)      */
#define SCROLL_DEVERR_DYN      4u   /* a dynamic NAL outgrew its staging slot     */
#define SCROLL_DEVERR_HINT     8u   /* a hint rect names an invalid reference     */
#define SCROLL_DEVERR_SPLICE  16u   /* a spliced slice failed (parse / reference) */
#define SCROLL_DEVERR_HANDOFF 32u   /* k_dyn_row's wait for the row above timed out */
#define SCROLL_DEVERR_STAGED   (SCROLL_DEVERR_DYN | SCROLL_DEVERR_HINT | SCROLL_DEVERR_SPLICE | \
                                SCROLL_DEVERR_HANDOFF)   /* nothing committed */

/* k_plan state pass -> size pass: the stream's planned totals and the final
 * waypoint table (committed only by the size pass).  128 bytes. */
typedef struct {
    int32_t nnal, nwp_end, fn_end, nalwp;
    int32_t wo[8], wl[8], wv[8];
    int32_t pad[4];
} PlanPending;

/* per composed frame with the dynamic rect: its scroll NAL (-1: none, the
 * experiment mode replaced it), staged RBSP bytes, emulation-prevention
 * bytes to insert, staging overflow.  16 bytes. */
typedef struct {
    int32_t nal;
    uint32_t rbsp_bytes;
    uint32_t ep;
    uint32_t err;
} DynFrame;

/* dynamic rect geometry and buffer strides (one per batch) */
#define DYN_MAX_W 256               /* rect width limit (MBs): a whole 4096-px row */
#define DYN_MAX_H 256               /* rect height limit (MBs): a whole 4K frame   */
#define DYN_MAX_MBW 512             /* picture width limit with the rect (MBs)   */
#define DYN_MAX_MBH 512             /* picture height limit with the rect (MBs)  */
#ifndef DYN_STATIC_ROWS
/* MB rows per static row group (k_dyn_static, one wave each): round 6 64 ->
 * 16, config 5's 88 static rows in 6 groups instead of 2 (2.872 -> 2.833 ms
 * per step; 8: the same, 32: 2.891; 4 measured slower in round 3) */
#define DYN_STATIC_ROWS 16
#endif
#define DYN_PIECES 26               /* coded pieces per dynamic MB: 16 luma, 2 DC, 8 AC */
#define DYN_OVF_BYTES 8192          /* staging-slot tail: levels of > 128-bit blocks */
#ifndef SCROLL_DYN_ROW_KBITS
#define SCROLL_DYN_ROW_KBITS 1280   /* rect-row slot bits per MB (typical; more: a spill slot) */
#endif
typedef struct {
    int32_t x0, y0, w, h;           /* rect, MB units                             */
    int32_t pw, ph;                 /* the streams' picture size (pixels)         */
    int32_t ngroups;                /* k_dyn_group row groups per NAL (dyn_groups) */
    int32_t qp;                     /* the rect's QP (slice_qp_delta qp - 26)     */
    QParams ql, qc;                 /* its luma / chroma (QPc) quantisers          */
    int32_t debug;                  /* SCROLL_DEBUG_DYN_* ablation bits           */
    uint64_t src_ld, src_fr;        /* source bytes per stream / per frame        */
    uint64_t ref_ld;                /* reference-pair bytes per stream (0 shared) */
    uint64_t slot_bytes;            /* staging bytes per frame                    */
    uint32_t rs_static_words;       /* row-stage words per static row group       */
    uint32_t rs_row_words;          /* row-stage words per rect row               */
    uint64_t rs_frame_words;        /* row-stage words per frame (all row groups) */
    uint32_t rs_spill_words;        /* a spill slot: one rect row at its provable bound */
    uint32_t rs_spill_cap;          /* spill slots after the frames' regions       */
    uint32_t gen_cap;               /* general-path record slots (NALs)           */
    uint32_t rs_frames;             /* frame regions before the spill slots (S F)  */
    uint32_t ep_cap;                /* EP positions kept per frame (the dyn path's list; 4 ep_cap bytes a frame) */
} DynGeom;

/* hints of one composed frame: rects [first, first + n) of the batch's rect
 * pool, SCROLL_HINT_* mode.  8 bytes. */
typedef struct {
    int32_t first;
    int16_t n;
    int16_t mode;
} HintFrame;

enum { SCROLL_PLAN_COMPOSER = 0, SCROLL_PLAN_EXPERIMENT = 1, SCROLL_PLAN_EXPLICIT = 2 };

/* Synchronous single-stream helpers used by the drop-in entry points.
 * All return SCROLL_OK or a negative SCROLL_ERR_*. */

/* Plan + emit explicit NALs (h264_write_scroll_p_frame / _waypoint_) for one
 * config.  dst receives the Annex-B bytes. */
int scroll_engine_write_nals(const ComposerConfig *cfg, const NalDesc *nals, int n,
                             uint8_t *dst, size_t cap, size_t *written);

/* Composer semantics for one or many streams: cfgs[i] composes frames[i]
 * offsets from offs[i]; output appended to dsts[i] (capacity caps[i]),
 * *written[i] bytes; cfgs updated (frame_num, waypoints); wp_offsets_out
 * (optional, per stream up to nframes entries, -1 terminated) receives the
 * offsets at which waypoint NALs were written (for the reference's stdout). */
int scroll_engine_compose(ComposerConfig *const *cfgs, const int *const *offs,
                          const int *frames, int nstreams, int mode,
                          uint8_t *const *dsts, const size_t *caps, size_t *written,
                          int **wp_offsets_out);

#ifdef __cplusplus
}
#endif
#endif
