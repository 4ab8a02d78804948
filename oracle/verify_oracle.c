/*
 * verify_oracle.c -- CPU ORACLE (test infrastructure only): whole-step
 * checkers, see verify_oracle.h.  The product never links this file.
 */
#include "verify_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* src/composer.c:255-264: an optional waypoint frame (h264_writer.c:666-676
 * decides; :772-777 registers it while fewer than 8 exist; :780 frame_num++)
 * then the scroll frame (:662 frame_num++); experiment mode writes the
 * waypoint frame instead of the scroll frame */
void or_compose_state(or_cfg *c, int off, int mode)
{
    if (or_needs_waypoint(c, off)) {
        if (c->nwp < OR_MAX_WP) {
            c->wp_off[c->nwp] = off;
            c->wp_lt[c->nwp] = 2 + c->nwp;
            c->wp_valid[c->nwp] = 1;
            c->nwp++;
        }
        c->frame_num++;
        if (mode == 1) return;
    }
    c->frame_num++;
}

typedef struct {
    int s0, s1, F, mode, stream_base, t0, passes;
    or_cfg *cfgs;
    const int32_t *offs;
    const or_dyn_rect *r;
    const or_refs *const *R;
    const or_refs *R_shared;
    uint8_t *out;
    size_t stride;
    size_t *sizes;
    int rc;
} or_verify_job;

static void *or_verify_worker(void *arg)
{
    or_verify_job *j = (or_verify_job *)arg;
    const int dyn = j->r && j->r->w > 0 && j->r->h > 0;
    const size_t sb = dyn ? (size_t)384 * j->r->w * j->r->h : 0;
    uint8_t *src = dyn ? (uint8_t *)malloc(sb) : NULL;
    /* one composed frame (waypoint + scroll NAL) at most: 4 KB + 6 bytes per
     * MB per NAL, 2 KB per dynamic MB */
    const size_t fcap = 2 * (4096 + (size_t)(j->cfgs[j->s0].w / 16) * (j->cfgs[j->s0].h / 16) * 6) +
                        (dyn ? (size_t)j->r->w * j->r->h * 2048 : 0);
    uint8_t *tmp = (uint8_t *)malloc(fcap);
    for (int s = j->s0; s < j->s1 && !j->rc; ++s) {
        or_cfg *c = &j->cfgs[s];
        const int32_t *o = j->offs + (size_t)s * j->F;
        for (int p = 0; p + 1 < j->passes; ++p)
            for (int f = 0; f < j->F; ++f) or_compose_state(c, o[f], j->mode);
        uint8_t *dst = j->out + (size_t)s * j->stride;
        size_t n = 0;
        const or_refs *R = j->R ? j->R[s] : j->R_shared;
        for (int f = 0; f < j->F; ++f) {
            size_t k;
            if (dyn) {
                or_dyn_source(src, j->stream_base + s, j->t0 + f, j->r);
                k = or_compose_dyn(tmp, fcap, c, o[f], j->mode, j->r, src, R, NULL);
            } else {
                k = or_compose(tmp, fcap, c, o[f], j->mode, NULL);
            }
            if (j->stride - n < k) {
                j->rc = -1;
                break;
            }
            memcpy(dst + n, tmp, k);
            n += k;
        }
        j->sizes[s] = n;
    }
    free(tmp);
    free(src);
    return NULL;
}

int or_verify_compose(int S, int F, or_cfg *cfgs, const int32_t *offs, int mode,
                      const or_dyn_rect *r, int stream_base, int t0, const or_refs *const *R,
                      const or_refs *R_shared, int passes, uint8_t *out, size_t stride,
                      size_t *sizes, int nthreads)
{
    if (S <= 0) return 0;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > S) nthreads = S;
    if (passes < 1) passes = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    or_verify_job *jobs = (or_verify_job *)calloc((size_t)nthreads, sizeof(or_verify_job));
    for (int t = 0; t < nthreads; ++t) {
        or_verify_job *j = &jobs[t];
        j->s0 = (int)((long long)S * t / nthreads);
        j->s1 = (int)((long long)S * (t + 1) / nthreads);
        j->F = F;
        j->mode = mode;
        j->stream_base = stream_base;
        j->t0 = t0;
        j->passes = passes;
        j->cfgs = cfgs;
        j->offs = offs;
        j->r = r;
        j->R = R;
        j->R_shared = R_shared;
        j->out = out;
        j->stride = stride;
        j->sizes = sizes;
        pthread_create(&th[t], NULL, or_verify_worker, j);
    }
    int rc = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    free(th);
    free(jobs);
    return rc;
}
