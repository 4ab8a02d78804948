/*
 * composer_cli.c -- the reference `composer` CLI (src/main.c:32-141) rebuilt
 * against libh264scroll.so: same options, same triangle scroll, same output
 * file.  Scroll frames are composed on the MI355X.
 */
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>

#include "composer.h"

static void usage(const char *p)
{
    printf("Usage: %s --ref-a FILE --ref-b FILE [-n FRAMES] [-s SPEED] [-o OUT]\n", p);
}

int main(int argc, char **argv)
{
    const char *ra = NULL, *rb = NULL, *out = "output.h264";
    int frames = 250, speed = 4;
    static struct option lo[] = {{"ref-a", required_argument, 0, 'a'},
                                 {"ref-b", required_argument, 0, 'b'},
                                 {"frames", required_argument, 0, 'n'},
                                 {"speed", required_argument, 0, 's'},
                                 {"output", required_argument, 0, 'o'},
                                 {"help", no_argument, 0, 'h'},
                                 {0, 0, 0, 0}};
    int o;
    while ((o = getopt_long(argc, argv, "a:b:n:s:o:h", lo, NULL)) != -1) {
        switch (o) {
        case 'a': ra = optarg; break;
        case 'b': rb = optarg; break;
        case 'n': frames = atoi(optarg); break;
        case 's': speed = atoi(optarg); break;
        case 'o': out = optarg; break;
        case 'h': usage(argv[0]); return 0;
        default: usage(argv[0]); return 1;
        }
    }
    if (!ra || !rb) {
        fprintf(stderr, "Error: --ref-a and --ref-b are required\n\n");
        usage(argv[0]);
        return 1;
    }
    if (frames <= 0 || speed <= 0) {
        fprintf(stderr, "Error: --frames and --speed must be positive\n");
        return 1;
    }
    Composer c;
    if (composer_init(&c, ra, rb) < 0) return 1;
    int h = composer_get_height(&c);
    printf("Generating %d frames, scroll speed %d px/frame\n", frames, speed);
    printf("Max scroll offset: %d pixels\n", h);
    composer_write_header(&c);
    for (int i = 0; i < frames; ++i) {
        int cyc = 2 * h, pos = (i * speed) % cyc;
        composer_write_scroll_frame(&c, pos < h ? pos : cyc - pos);
    }
    int rc = composer_write_to_file(&c, out);
    composer_finish(&c);
    return rc < 0 ? 1 : 0;
}
