/*
 * hint_oracle.h -- CPU ORACLE (test infrastructure only) for the UI-hint
 * P slice (docs/MASTER_DESIGN.md:58-64,103-146 of the
 * reference).  Used only by tests/ as the checker of k_hint_stage; the product
 * library never links it.
 *
 * The reference has no implementation of UI hints, so this file DEFINES the
 * bits ("parity unpinned" for hinted layouts).  Two anchors pin
 * it anyway:
 *   - a frame whose hints restate the scroll layout (or that has no hints) is
 *     byte-identical to h264_write_scroll_p_frame (src/h264_writer.c:541-664),
 *     checked against or_scroll_nal, itself pinned by the reference's golden
 *     vectors;
 *   - tests/h264_pslice.py decodes the MV field of a hinted NAL from the
 *     standard (mb_skip_run 7.3.4, P_Skip 8.4.1.1, median prediction 8.4.1.3)
 *     or with the reference's own predictor, and must get the hinted layout.
 *
 * Semantics.  A hint rect covers MBs [x0, x1) x [y0, y1) (MB units, clipped
 * to the picture) and gives them reference `ref` (0 = A, 1 = B, 2 + i =
 * waypoint i, which must be valid in the frame) and displacement (mv_x, mv_y)
 * in pixels: the MB at (16x, 16y) is predicted from (16x + mv_x, 16y + mv_y)
 * of that reference.  Later rects lie on top of earlier ones.  MBs no rect
 * covers keep the scroll layout of the frame's offset (region A / B with the
 * reference's waypoint choice), so static chrome, a horizontally scrolling
 * row or a second scroll pane are overlays on the ordinary scroll frame.
 *
 * Modes:
 *   OR_HINT_EXACT  every MB is P_L0_16x16 preceded by mb_skip_run 0 and
 *                  predicted with the reference's get_mv_prediction
 *                  (h264_writer.c:369-432, non-standard median3) -- the
 *                  reference's MB syntax, generalised to any MV field;
 *   OR_HINT_PSKIP  standard MV prediction (8.4.1.3) and P_Skip: an MB with
 *                  ref 0 whose mv equals the P_Skip motion (8.4.1.1) is
 *                  skipped; runs of skipped MBs are coded with mb_skip_run.
 *   OR_HINT_SPEC   the reference's MB syntax (every MB P_L0_16x16 after
 *                  mb_skip_run 0) with the standard's MV prediction
 *                  (8.4.1.3): decodable by a standard decoder for any MV
 *                  field, and byte-identical to the reference's scroll frame
 *                  for the plain scroll layout (a row-uniform field never
 *                  reaches the cases where get_mv_prediction departs from
 *                  the standard).
 */
#ifndef HINT_ORACLE_H
#define HINT_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#include "scroll_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OR_HINT_EXACT 0
#define OR_HINT_PSKIP 1
#define OR_HINT_SPEC 2

/* layout-identical to ScrollHintRect (include/composer_batch.h) */
typedef struct {
    int16_t x0, y0, x1, y1;
    int16_t ref, reserved;
    int32_t mv_x, mv_y;
} or_hint_rect;

/* The scroll NAL of a frame at offset `off` with hint rects r[0..n) in mode
 * `mode`; frame_num++ like or_scroll_nal.  Returns the Annex-B bytes, or 0
 * when an MB takes a rect whose ref is not a valid reference of the frame
 * (*err = 1; the state is then left unchanged). */
size_t or_hint_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off,
                          const or_hint_rect *r, int n, int mode, int *err);

/* composer_write_scroll_frame (src/composer.c:255-264) with the scroll NAL
 * replaced by or_hint_scroll_nal; compose mode as or_compose. */
size_t or_compose_hint(uint8_t *dst, size_t cap, or_cfg *c, int off, int compose_mode,
                       const or_hint_rect *r, int n, int mode, int *err);

/* the MV field the hints give a frame: per MB (ref, mv_x, mv_y) in pixels,
 * row-major, out[3 * mbw * mbh]; returns 0, or -1 on an invalid ref */
int or_hint_field(const or_cfg *c, int off, const or_hint_rect *r, int n, int32_t *out);

/* motion helpers shared with the splice restatement (splice_oracle.c):
 * the topmost rect holding MB (x, y) (returns 1; else 0 and the scroll row's
 * motion, mv in pixels); reference validity; neighbours A, B, C-or-D of
 * 8.4.1.3.2 (unavailable: avail 0); median prediction 8.4.1.3 and P_Skip
 * motion 8.4.1.1 (quarter pels) */
int or_hint_motion(const or_hint_rect *r, int n, int x, int y, int a_end, int ra, int mva,
                   int rb, int mvb, int *ref, int *mx, int *my);
int or_ref_valid(const or_cfg *c, int ref);
void or_neighbours(int x, int y, int mbw, const or_mvi *above, const or_mvi *left, or_mvi *A,
                   or_mvi *B, or_mvi *C);
void or_spec_predict(const or_mvi *A, const or_mvi *B, const or_mvi *C, int ref, int *px,
                     int *py);
void or_pskip_motion(int x, int y, const or_mvi *A, const or_mvi *B, const or_mvi *C, int *px,
                     int *py);

#ifdef __cplusplus
}
#endif
#endif
