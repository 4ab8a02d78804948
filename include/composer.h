/*
 * composer.h -- drop-in for the reference's include/composer.h (:23-101).
 *
 * The Composer struct is caller-allocated in the reference (src/main.c:94),
 * so its layout is ABI and is kept byte-identical.  GPU-side state lives in a
 * library registry keyed by the Composer pointer, never inside the struct.
 *
 * composer_write_scroll_frame() is the hot entry.  In libh264scroll.so it
 * records the offset; the queued frames are composed on the MI355X in one
 * batch (GPU state machine + P-slice kernels) and appended to the Composer's
 * output buffer at the next composer_get_output_size / composer_get_output /
 * composer_write_to_file / composer_finish call, or when the queue is full.
 * Bytes are identical to the reference's; only the moment they land differs
 * (and the "Waypoint at offset" stdout lines are printed at that moment).
 */
#ifndef COMPOSER_H
#define COMPOSER_H

#include <stddef.h>
#include <stdint.h>
#include "h264_writer.h"
#include "nal.h"

#ifdef __cplusplus
extern "C" {
#endif

/* reference include/composer.h:23-49 */
typedef struct {
    ComposerConfig cfg;         /* our stream parameters              */
    ComposerConfig parse_cfg;   /* parameters of the input encoder    */

    uint8_t *ref_a_rbsp;        /* IDR RBSP of reference A            */
    size_t ref_a_size;
    uint8_t *ref_b_rbsp;        /* IDR RBSP of reference B            */
    size_t ref_b_size;

    uint8_t *orig_sps;
    size_t orig_sps_size;
    uint8_t *orig_pps;
    size_t orig_pps_size;

    NALWriter nw;
    uint8_t *output_buffer;
    size_t output_capacity;
    uint8_t *rbsp_temp;
    size_t rbsp_capacity;

    int frames_written;
} Composer;

int composer_init(Composer *c, const char *ref_a_path, const char *ref_b_path);   /* :59 */
int composer_get_width(Composer *c);                                             /* :64 */
int composer_get_height(Composer *c);                                            /* :65 */
void composer_write_header(Composer *c);                                         /* :72 */
void composer_write_scroll_frame(Composer *c, int offset_px);                    /* :79 HOT */
size_t composer_get_output_size(Composer *c);                                    /* :84 */
uint8_t *composer_get_output(Composer *c);                                       /* :89 */
int composer_write_to_file(Composer *c, const char *path);                       /* :96 */
void composer_finish(Composer *c);                                               /* :101 */

#ifdef __cplusplus
}
#endif
#endif /* COMPOSER_H */
