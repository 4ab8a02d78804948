/*
 * ref_frames.c -- golden-vector harness for the REFERENCE composer (test
 * infrastructure).  Compiled by oracle/Makefile against the reference's own
 * sources under /root/reference/src (never copied), output to oracle/_ref/.
 *
 * stdin : one case per line
 *   W H log2_mfn poc_type log2_poc deblock frame_num nwp
 *   (wp_off wp_lt wp_valid) x 8   kind offset
 *   kind 0 = h264_write_scroll_p_frame, 1 = h264_write_waypoint_p_frame,
 *        2 = composer_write_scroll_frame semantics (src/composer.c:255-264)
 * stdout: per case one line "<hex bytes> <frame_num after> <nwp after>"
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "h264_writer.h"
#include "nal.h"

int main(void)
{
    size_t cap = 64u << 20;
    uint8_t *out = malloc(cap);
    uint8_t *rb = malloc(4u << 20);
    int v[8 + 24 + 2];
    for (;;) {
        int got = 0;
        for (int i = 0; i < 34; ++i) {
            if (scanf("%d", &v[i]) != 1) break;
            got++;
        }
        if (got != 34) break;
        ComposerConfig c;
        composer_config_init(&c, v[0], v[1]);
        composer_config_set_sps_params(&c, v[2], v[3], v[4]);
        composer_config_set_pps_params(&c, 1, v[5]);
        c.frame_num = v[6];
        c.num_waypoints = v[7];
        for (int i = 0; i < 8; ++i) {
            c.waypoints[i].offset_px = v[8 + 3 * i];
            c.waypoints[i].long_term_idx = v[9 + 3 * i];
            c.waypoints[i].valid = v[10 + 3 * i];
        }
        int kind = v[32], off = v[33];
        NALWriter nw;
        nal_writer_init(&nw, out, cap, rb, 4u << 20);
        if (kind == 0) {
            h264_write_scroll_p_frame(&nw, &c, off);
        } else if (kind == 1) {
            h264_write_waypoint_p_frame(&nw, &c, off);
        } else {
            if (h264_needs_waypoint(&c, off))
                h264_write_waypoint_p_frame(&nw, &c, off);
            h264_write_scroll_p_frame(&nw, &c, off);
        }
        size_t n = nal_writer_get_size(&nw);
        for (size_t i = 0; i < n; ++i) printf("%02x", out[i]);
        printf(" %d %d\n", c.frame_num, c.num_waypoints);
    }
    free(out);
    free(rb);
    return 0;
}
