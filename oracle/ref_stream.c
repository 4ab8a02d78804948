/*
 * ref_stream.c -- golden-vector harness: one synthetic stream through the
 * REFERENCE composer (test infrastructure).  Built by oracle/Makefile against
 * /root/reference/src objects; output to oracle/_ref/.
 *
 * usage: ref_stream W H stream_id nframes
 * State = ComposerConfig as composer_init + composer_write_header leave it
 * (src/composer.c:199-203, frame_num 2).  Offsets follow SURVEY 8(d):
 * speed 1+(s%8), phase (97*s) mod 2H, triangle 0..H.
 * stdout: one hex line per composed frame (composer_write_scroll_frame).
 */
#include <stdio.h>
#include <stdlib.h>
#include "h264_writer.h"
#include "nal.h"

static int tri(int x, int m)
{
    int c = 2 * m, p = x % c;
    return p < m ? p : c - p;
}

int main(int argc, char **argv)
{
    if (argc != 5) return 1;
    int w = atoi(argv[1]), h = atoi(argv[2]), s = atoi(argv[3]), nf = atoi(argv[4]);
    size_t cap = 8u << 20;
    uint8_t *out = malloc(cap), *rb = malloc(1u << 20);
    ComposerConfig c;
    composer_config_init(&c, w, h);
    composer_config_set_sps_params(&c, 4, 2, 4);
    composer_config_set_pps_params(&c, 1, 1);
    c.frame_num = 2;
    for (int i = 0; i < nf; ++i) {
        int off = tri(i * (1 + s % 8) + (97 * s) % (2 * h), h);
        NALWriter nw;
        nal_writer_init(&nw, out, cap, rb, 1u << 20);
        if (h264_needs_waypoint(&c, off))
            h264_write_waypoint_p_frame(&nw, &c, off);
        h264_write_scroll_p_frame(&nw, &c, off);
        size_t n = nal_writer_get_size(&nw);
        for (size_t k = 0; k < n; ++k) printf("%02x", out[k]);
        printf("\n");
    }
    free(out);
    free(rb);
    return 0;
}
