/*
 * ref_ipcm.c -- reference I_PCM striped reference-frame writer (test
 * infrastructure).  Linked against the reference
 * experiment's own objects built from /root/reference/experiments/
 * scroll-encoder/src by oracle/Makefile into oracle/_ref/.
 *
 * usage: ref_ipcm W H which out.h264     (which 0 = colours A, 1 = colours B)
 */
#include <stdio.h>
#include <stdlib.h>
#include "h264_encoder.h"
#include "nal.h"

int main(int argc, char **argv)
{
    if (argc != 5) {
        fprintf(stderr, "usage: %s W H which out\n", argv[0]);
        return 1;
    }
    int w = atoi(argv[1]), h = atoi(argv[2]), which = atoi(argv[3]);
    size_t cap = (size_t)(w / 16) * (size_t)(h / 16) * 400 + (1u << 20);
    uint8_t *out = malloc(cap), sps[256], pps[256];
    uint8_t *rb = malloc(1u << 20);
    NALWriter nw;
    nal_writer_init(&nw, out, cap, rb, 1u << 20);
    H264EncoderConfig cfg;
    h264_encoder_init(&cfg, w, h);
    size_t s = h264_generate_sps(sps, sizeof(sps), w, h);
    nal_write_unit(&nw, 3, 7, sps, s, 1);
    s = h264_generate_pps(pps, sizeof(pps));
    nal_write_unit(&nw, 3, 8, pps, s, 1);
    if (which == 0)
        h264_write_idr_frame_striped(&nw, &cfg, 81, 90, 240, 145, 54, 34, 41, 240, 110);
    else
        h264_write_idr_frame_striped(&nw, &cfg, 210, 16, 146, 170, 166, 16, 106, 202, 222);
    FILE *f = fopen(argv[4], "wb");
    if (!f) return 1;
    fwrite(out, 1, nal_writer_get_size(&nw), f);
    fclose(f);
    free(out);
    free(rb);
    return 0;
}
