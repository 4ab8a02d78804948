/*
 * scroll_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference composer's hot path
 * (wreuven/h264-scroll-encoder @ 2026-01-30), used ONLY by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * The product library (h264-scroll-encoder_amd/) never links or calls it.
 *
 * Parity pinning: this restatement is checked against golden vectors produced
 * by the reference C compiled from /root/reference sources (oracle/Makefile
 * target `ref`, outputs in oracle/_ref/, fixtures in tests/golden/, generated
 * by tests/golden/make_golden.py).  The dynamic-rect residual coder has no
 * reference implementation: it is "parity unpinned" (see DESIGN.md).
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef SCROLL_ORACLE_H
#define SCROLL_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MV_LIMIT 496   /* include/h264_writer.h:24 */
#define OR_MAX_WP   8     /* include/h264_writer.h:27 */

/* Per-stream writer state: mirrors ComposerConfig (include/h264_writer.h:30-59). */
typedef struct {
    int w, h;                 /* pixels */
    int log2_mfn;             /* log2_max_frame_num */
    int poc_type;
    int log2_poc;             /* log2_max_pic_order_cnt_lsb */
    int num_ref_default_m1;
    int deblock;              /* deblocking_filter_control_present_flag */
    int frame_num;
    int idr_pic_id;
    int nwp;                  /* num_waypoints */
    int wp_off[OR_MAX_WP];
    int wp_lt[OR_MAX_WP];
    int wp_valid[OR_MAX_WP];
} or_cfg;

/* composer_config_init (src/h264_writer.c:13-28) */
void or_cfg_init(or_cfg *c, int w, int h);

/* ---- bit writer restatement (src/bitwriter.c) ---- */
typedef struct {
    uint8_t *buf;
    size_t cap;     /* bytes */
    size_t nbits;   /* bits written */
} or_bits;
void or_bits_init(or_bits *b, uint8_t *buf, size_t cap);
void or_put(or_bits *b, uint32_t v, int n);      /* bitwriter_write_bits :25-32 */
void or_ue(or_bits *b, uint32_t v);              /* bitwriter_write_ue   :50-74 */
void or_se(or_bits *b, int32_t v);               /* bitwriter_write_se   :91-101 */
void or_trailing(or_bits *b);                    /* :103-111 */
size_t or_bytes(or_bits *b);                     /* bitwriter_get_size :124-131 */
/* slice header of a scroll P frame (src/h264_writer.c:549-553) */
void or_scroll_header(or_bits *b, const or_cfg *c);
void or_scroll_header_qpd(or_bits *b, const or_cfg *c, int qpd);   /* slice_qp_delta qpd */

/* ---- NAL framing restatement (src/nal.c) ---- */
size_t or_rbsp_to_ebsp(uint8_t *dst, size_t cap, const uint8_t *src, size_t n); /* :24-50 */
size_t or_nal(uint8_t *dst, size_t cap, int ref_idc, int type,
              const uint8_t *rbsp, size_t n);                                    /* :52-84 */

/* ---- P-frame writers (src/h264_writer.c) ---- */
/* h264_write_scroll_p_frame :541-664 ; appends one Annex-B NAL, frame_num++ */
size_t or_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off);
/* h264_write_waypoint_p_frame :678-782 ; registers waypoint, frame_num++ */
size_t or_waypoint_nal(uint8_t *dst, size_t cap, or_cfg *c, int off);
/* h264_needs_waypoint :666-676 */
int or_needs_waypoint(const or_cfg *c, int off);

/* ---- MB-layer pieces shared with the UI-hint restatement (hint_oracle.c) ---- */
/* MVInfo (src/h264_writer.c:356-360); mx, my in quarter pels */
typedef struct {
    int mx, my, ref, avail;
} or_mvi;
/* get_mv_prediction (src/h264_writer.c:369-432) with median3 (:362-367) */
void or_predict(int x, int y, int mbw, const or_mvi *above, const or_mvi *left,
                int ref, int *px, int *py);
/* region split (:555) and waypoint choice for A (:558-571) and B (:573-588)
 * of a scroll frame at offset off; mv in pixels */
void or_scroll_regions(const or_cfg *c, int off, int *a_end, int *ra, int *mva, int *rb,
                       int *mvb);

/* One composed frame.
 * mode 0 = composer_write_scroll_frame (src/composer.c:255-264): optional
 *          waypoint NAL *then* the scroll NAL.
 * mode 1 = experiment loop (experiments/scroll-encoder/src/main.c:418-424):
 *          waypoint NAL *instead of* the scroll NAL.
 * Returns bytes appended; *n_wp_out (optional) = waypoint NALs written. */
size_t or_compose(uint8_t *dst, size_t cap, or_cfg *c, int off, int mode, int *n_wp_out);

/* ---- cold path: headers, I-frame rewrite, I_PCM refs ---- */
size_t or_sps(uint8_t *rbsp, size_t cap, int w, int h);   /* h264_writer.c:49-100 */
size_t or_pps(uint8_t *rbsp, size_t cap);                 /* h264_writer.c:105-127 */
/* h264_rewrite_idr_frame :242-294 / h264_rewrite_as_non_idr_i_frame :296-350 */
size_t or_rewrite_idr(uint8_t *dst, size_t cap, or_cfg *wr, const or_cfg *pc,
                      const uint8_t *rbsp, size_t n);
size_t or_rewrite_non_idr(uint8_t *dst, size_t cap, or_cfg *wr, const or_cfg *pc,
                          const uint8_t *rbsp, size_t n, int frame_num);
/* mid-stream long-term reference update (scroll_oracle.c): the file's IDR
 * as a non-IDR I frame marked long-term `which`, waypoints dropped */
size_t or_update_ref(uint8_t *dst, size_t cap, or_cfg *c, const uint8_t *file, size_t n, int which);
/* I_PCM striped reference (experiments/scroll-encoder/src/h264_encoder.c:730-918).
 * which = 0: IDR with stripes (y1..cr3), which = 1: non-IDR I frame. */
size_t or_ipcm_striped(uint8_t *dst, size_t cap, or_cfg *c, int which,
                       const uint8_t yuv[9]);
/* SPS+PPS+I_PCM striped A (IDR) or B (IDR) file, as a harness would write it
 * (SURVEY Appendix B).  which=0 -> colours of frame A, 1 -> frame B. */
size_t or_ipcm_ref_file(uint8_t *dst, size_t cap, int w, int h, int which);

/* The same file for an arbitrary I420 picture (Y w*h, Cb, Cr w*h/4 each):
 * SPS + PPS + IDR whose I_PCM MBs carry the picture's samples
 * (h264_encoder.c:730-753 generalised from one colour per MB).  For the
 * striped pictures it equals or_ipcm_ref_file. */
size_t or_ipcm_picture_file(uint8_t *dst, size_t cap, int w, int h, const uint8_t *pic);

/* ---- ingest (src/nal_parser.c) ---- */
size_t or_ebsp_to_rbsp(uint8_t *dst, const uint8_t *src, size_t n);   /* :67-88 */

/* Whole-composer run: composer_init (src/composer.c:127-222) from two Annex-B
 * buffers, composer_write_header (:232-253), nframes x composer_write_scroll_frame
 * with the CLI triangle scroll (src/main.c:109-128). Returns bytes or 0 on error. */
size_t or_composer_run(uint8_t *dst, size_t cap,
                       const uint8_t *ref_a, size_t na,
                       const uint8_t *ref_b, size_t nb,
                       int nframes, int speed);

/* Experiment test-mode run (experiments/scroll-encoder/src/main.c:198-429,
 * striped, start offset 496, waypoint instead of scroll). */
size_t or_experiment_run(uint8_t *dst, size_t cap, int w, int h, int nframes, int speed);

/* Synthetic many-stream workload of SURVEY 8(d) config 2:
 * stream s: speed 1+(s%8), phase (97*s) mod (2H); off_i = tri(i*v+phase, H). */
int or_tri(int x, int m);
int or_synthetic_offset(int s, int i, int h);

/* CPU baseline timer: compose nframes for each of nstreams fresh streams
 * (state as after composer_write_header), nthreads pthreads, streams split
 * contiguously.  Returns composed frames/s; *bytes_out = total bytes. */
double or_bench_compose(int nstreams, int nframes, int w, int h, int nthreads,
                        int warmup_frames, unsigned long long *bytes_out);

#ifdef __cplusplus
}
#endif
#endif
