/*
 * composer.c -- ABI of include/composer.h (+ Composer-level batch entry of
 * include/composer_batch.h).
 *
 * composer_init / composer_write_header are the cold path (reference
 * src/composer.c:127-253) and run on the host.  composer_write_scroll_frame
 * (reference :255-264) is the hot entry: it queues the offset in a registry
 * keyed by the Composer pointer (the caller-allocated struct stays
 * byte-identical); queued frames are composed on the GPU in one batch by
 * scroll_engine_compose() -- the waypoint state machine runs in the plan
 * kernel -- and appended to c->nw.output when an accessor needs the bytes.
 */
#include "composer.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../engine.h"
#include "composer_batch.h"
#include "nal_parser.h"

#define OUTPUT_BUFFER_SIZE (64 * 1024 * 1024)   /* reference :8 */
#define RBSP_BUFFER_SIZE (4 * 1024 * 1024)      /* reference :9 */
#define QUEUE_FLUSH_FRAMES 8192

/* ------------------------------------------------------------------------ */
/* pending-frame registry                                                    */
/* ------------------------------------------------------------------------ */
typedef struct {
    Composer *c;
    int *off;
    int n, cap;
} Pending;

static pthread_mutex_t g_reg_mu = PTHREAD_MUTEX_INITIALIZER;
static Pending *g_reg;
static int g_nreg, g_capreg;

static Pending *reg_find(Composer *c, int create)
{
    for (int i = 0; i < g_nreg; ++i)
        if (g_reg[i].c == c) return &g_reg[i];
    if (!create) return NULL;
    if (g_nreg == g_capreg) {
        g_capreg = g_capreg ? 2 * g_capreg : 16;
        g_reg = (Pending *)realloc(g_reg, (size_t)g_capreg * sizeof(Pending));
    }
    Pending *p = &g_reg[g_nreg++];
    memset(p, 0, sizeof(*p));
    p->c = c;
    return p;
}

static void reg_drop(Composer *c)
{
    for (int i = 0; i < g_nreg; ++i) {
        if (g_reg[i].c != c) continue;
        free(g_reg[i].off);
        g_reg[i] = g_reg[g_nreg - 1];
        g_nreg--;
        return;
    }
}

static void pend_push(Pending *p, int off)
{
    if (p->n == p->cap) {
        p->cap = p->cap ? 2 * p->cap : 256;
        p->off = (int *)realloc(p->off, (size_t)p->cap * sizeof(int));
    }
    p->off[p->n++] = off;
}

/* compose every queued frame of the given registry entries on the GPU */
static int flush_entries(Pending **ps, int n)
{
    if (n == 0) return SCROLL_OK;
    ComposerConfig **cfgs = (ComposerConfig **)calloc((size_t)n, sizeof(*cfgs));
    const int **offs = (const int **)calloc((size_t)n, sizeof(*offs));
    int *frames = (int *)calloc((size_t)n, sizeof(int));
    uint8_t **dsts = (uint8_t **)calloc((size_t)n, sizeof(*dsts));
    size_t *caps = (size_t *)calloc((size_t)n, sizeof(size_t));
    size_t *written = (size_t *)calloc((size_t)n, sizeof(size_t));
    int **wps = (int **)calloc((size_t)n, sizeof(*wps));
    for (int i = 0; i < n; ++i) {
        Composer *c = ps[i]->c;
        cfgs[i] = &c->cfg;
        offs[i] = ps[i]->off;
        frames[i] = ps[i]->n;
        dsts[i] = c->nw.output + c->nw.output_pos;
        caps[i] = c->nw.output_capacity - c->nw.output_pos;
        wps[i] = (int *)malloc(((size_t)ps[i]->n + 1) * sizeof(int));
    }
    int rc = scroll_engine_compose(cfgs, offs, frames, n, SCROLL_MODE_COMPOSER, dsts, caps,
                                   written, wps);
    if (rc == SCROLL_OK) {
        for (int i = 0; i < n; ++i) {
            Composer *c = ps[i]->c;
            c->nw.output_pos += written[i];
            c->frames_written += ps[i]->n;
            for (int k = 0; wps[i][k] >= 0; ++k)       /* reference :259 stdout line */
                printf("  Waypoint at offset %d\n", wps[i][k]);
            ps[i]->n = 0;
        }
    }
    for (int i = 0; i < n; ++i) free(wps[i]);
    free(cfgs); free(offs); free(frames); free(dsts); free(caps); free(written); free(wps);
    return rc;
}

static void flush_or_die(Composer *c)
{
    pthread_mutex_lock(&g_reg_mu);
    Pending *p = reg_find(c, 0);
    int rc = SCROLL_OK;
    if (p && p->n) rc = flush_entries(&p, 1);
    pthread_mutex_unlock(&g_reg_mu);
    if (rc != SCROLL_OK) {
        fprintf(stderr, "libh264scroll: composing queued frames on the GPU failed: %s\n",
                scroll_last_error());
        abort();
    }
}

int composer_flush(Composer *c)
{
    pthread_mutex_lock(&g_reg_mu);
    Pending *p = reg_find(c, 0);
    int rc = SCROLL_OK;
    if (p && p->n) rc = flush_entries(&p, 1);
    pthread_mutex_unlock(&g_reg_mu);
    return rc;
}

int composer_batch_write_scroll_frames(Composer *const *cs, const int *offsets, int n, int flags)
{
    (void)flags;
    if (n < 0 || (n && (!cs || !offsets))) return SCROLL_ERR_ARG;
    pthread_mutex_lock(&g_reg_mu);
    Pending **ps = (Pending **)calloc((size_t)(n ? n : 1), sizeof(Pending *));
    int np = 0;
    for (int i = 0; i < n; ++i) {
        Pending *p = reg_find(cs[i], 1);
        pend_push(p, offsets[i]);
        int seen = 0;
        for (int k = 0; k < np; ++k) seen |= ps[k] == p;
        if (!seen) ps[np++] = p;
    }
    int rc = flush_entries(ps, np);
    free(ps);
    pthread_mutex_unlock(&g_reg_mu);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* cold path (reference src/composer.c:14-253)                               */
/* ------------------------------------------------------------------------ */
static uint8_t *load_file(const char *path, size_t *size)
{
    FILE *f = fopen(path, "rb");
    if (!f) {
        fprintf(stderr, "Error: Cannot open %s\n", path);
        return NULL;
    }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    *size = sz > 0 ? (size_t)sz : 0;
    uint8_t *d = (uint8_t *)malloc(*size ? *size : 1);
    if (d && *size && fread(d, 1, *size, f) != *size) {
        fprintf(stderr, "Error: Failed to read %s\n", path);
        free(d);
        d = NULL;
    }
    fclose(f);
    return d;
}

typedef struct {
    int w, h, l2f, poct, l2p, nref, dbf;
} RefParams;

/* first SPS / PPS / IDR of an Annex-B buffer (reference :45-125) */
static int parse_reference(const uint8_t *d, size_t n, uint8_t **sps, size_t *nsps, uint8_t **pps,
                           size_t *npps, uint8_t **idr, size_t *nidr, RefParams *rp)
{
    NALParser np;
    NALUnit u;
    uint8_t *tmp = (uint8_t *)malloc(n ? n : 1);
    int got_sps = 0, got_pps = 0, got_idr = 0;
    nal_parser_init(&np, d, n);
    while (nal_parser_next(&np, &u)) {
        uint8_t **dst = NULL;
        size_t *dn = NULL;
        if (u.nal_unit_type == NAL_TYPE_SPS && !got_sps) {
            size_t rn = ebsp_to_rbsp(tmp, u.data, u.size);
            if (parse_sps(tmp, rn, &rp->w, &rp->h, &rp->l2f, &rp->poct, &rp->l2p) < 0) {
                fprintf(stderr, "Error: Failed to parse SPS\n");
                free(tmp);
                return -1;
            }
            dst = sps; dn = nsps; got_sps = 1;
            *dst = (uint8_t *)malloc(rn ? rn : 1);
            memcpy(*dst, tmp, rn);
            *dn = rn;
        } else if (u.nal_unit_type == NAL_TYPE_PPS && !got_pps) {
            size_t rn = ebsp_to_rbsp(tmp, u.data, u.size);
            if (parse_pps(tmp, rn, &rp->nref, &rp->dbf) < 0) {
                fprintf(stderr, "Error: Failed to parse PPS\n");
                free(tmp);
                return -1;
            }
            dst = pps; dn = npps; got_pps = 1;
            *dst = (uint8_t *)malloc(rn ? rn : 1);
            memcpy(*dst, tmp, rn);
            *dn = rn;
        } else if (u.nal_unit_type == NAL_TYPE_IDR && !got_idr) {
            size_t rn = ebsp_to_rbsp(tmp, u.data, u.size);
            *idr = (uint8_t *)malloc(rn ? rn : 1);
            memcpy(*idr, tmp, rn);
            *nidr = rn;
            got_idr = 1;
        }
    }
    free(tmp);
    if (!got_sps || !got_pps || !got_idr) {
        fprintf(stderr, "Error: Reference file missing SPS/PPS/IDR\n");
        return -1;
    }
    return 0;
}

int composer_init(Composer *c, const char *ref_a_path, const char *ref_b_path)
{
    memset(c, 0, sizeof(*c));
    pthread_mutex_lock(&g_reg_mu);
    reg_drop(c);                       /* a recycled struct starts with an empty queue */
    pthread_mutex_unlock(&g_reg_mu);
    size_t na = 0, nb = 0;
    uint8_t *a = load_file(ref_a_path, &na);
    uint8_t *b = load_file(ref_b_path, &nb);
    if (!a || !b) {
        free(a);
        free(b);
        return -1;
    }
    RefParams ra, rb;
    memset(&ra, 0, sizeof(ra));
    memset(&rb, 0, sizeof(rb));
    if (parse_reference(a, na, &c->orig_sps, &c->orig_sps_size, &c->orig_pps, &c->orig_pps_size,
                        &c->ref_a_rbsp, &c->ref_a_size, &ra) < 0) {
        free(a);
        free(b);
        return -1;
    }
    uint8_t *tsps = NULL, *tpps = NULL;
    size_t ntsps = 0, ntpps = 0;
    if (parse_reference(b, nb, &tsps, &ntsps, &tpps, &ntpps, &c->ref_b_rbsp, &c->ref_b_size, &rb) < 0) {
        free(a);
        free(b);
        return -1;
    }
    free(tsps);
    free(tpps);
    free(a);
    free(b);
    if (ra.w != rb.w || ra.h != rb.h) {
        fprintf(stderr, "Error: Reference frame dimensions don't match\n");
        fprintf(stderr, "  RefA: %dx%d, RefB: %dx%d\n", ra.w, ra.h, rb.w, rb.h);
        return -1;
    }
    composer_config_init(&c->parse_cfg, ra.w, ra.h);
    composer_config_set_sps_params(&c->parse_cfg, ra.l2f, ra.poct, ra.l2p);
    composer_config_set_pps_params(&c->parse_cfg, ra.nref, ra.dbf);
    composer_config_init(&c->cfg, ra.w, ra.h);
    composer_config_set_sps_params(&c->cfg, 4, 2, 4);          /* reference :201 */
    composer_config_set_pps_params(&c->cfg, 1, ra.dbf);        /* reference :203 */
    c->output_capacity = OUTPUT_BUFFER_SIZE;
    c->output_buffer = (uint8_t *)malloc(c->output_capacity);
    c->rbsp_capacity = RBSP_BUFFER_SIZE;
    c->rbsp_temp = (uint8_t *)malloc(c->rbsp_capacity);
    if (!c->output_buffer || !c->rbsp_temp) {
        fprintf(stderr, "Error: Failed to allocate output buffers\n");
        return -1;
    }
    nal_writer_init(&c->nw, c->output_buffer, c->output_capacity, c->rbsp_temp, c->rbsp_capacity);
    printf("Composer initialized: %dx%d\n", ra.w, ra.h);
    return 0;
}

int composer_get_width(Composer *c) { return c->cfg.width; }

int composer_get_height(Composer *c) { return c->cfg.height; }

void composer_write_header(Composer *c)
{
    flush_or_die(c);                   /* keep stream order if frames were queued */
    size_t n = h264_generate_sps(c->rbsp_temp, c->rbsp_capacity, c->cfg.width, c->cfg.height);
    nal_write_unit(&c->nw, NAL_REF_IDC_HIGHEST, NAL_TYPE_SPS, c->rbsp_temp, n, 1);
    n = h264_generate_pps(c->rbsp_temp, c->rbsp_capacity);
    nal_write_unit(&c->nw, NAL_REF_IDC_HIGHEST, NAL_TYPE_PPS, c->rbsp_temp, n, 1);
    h264_rewrite_idr_frame(&c->nw, &c->cfg, &c->parse_cfg, c->ref_a_rbsp, c->ref_a_size);
    h264_rewrite_as_non_idr_i_frame(&c->nw, &c->cfg, &c->parse_cfg, c->ref_b_rbsp, c->ref_b_size, 1);
    printf("Header written: SPS + PPS + 2 reference frames\n");
}

/* HOT ENTRY (reference :255-264): queue; the GPU composes at flush time. */
void composer_write_scroll_frame(Composer *c, int offset_px)
{
    pthread_mutex_lock(&g_reg_mu);
    Pending *p = reg_find(c, 1);
    pend_push(p, offset_px);
    int rc = SCROLL_OK;
    if (p->n >= QUEUE_FLUSH_FRAMES) rc = flush_entries(&p, 1);
    pthread_mutex_unlock(&g_reg_mu);
    if (rc != SCROLL_OK) {
        fprintf(stderr, "libh264scroll: composing queued frames on the GPU failed: %s\n",
                scroll_last_error());
        abort();
    }
}

size_t composer_get_output_size(Composer *c)
{
    flush_or_die(c);
    return nal_writer_get_size(&c->nw);
}

uint8_t *composer_get_output(Composer *c)
{
    flush_or_die(c);
    return nal_writer_get_output(&c->nw);
}

int composer_write_to_file(Composer *c, const char *path)
{
    flush_or_die(c);
    FILE *f = fopen(path, "wb");
    if (!f) {
        fprintf(stderr, "Error: Cannot create %s\n", path);
        return -1;
    }
    size_t n = c->nw.output_pos;
    if (fwrite(c->output_buffer, 1, n, f) != n) {
        fprintf(stderr, "Error: Failed to write %s\n", path);
        fclose(f);
        return -1;
    }
    fclose(f);
    printf("Written %zu bytes to %s\n", n, path);
    return 0;
}

void composer_finish(Composer *c)
{
    pthread_mutex_lock(&g_reg_mu);
    reg_drop(c);                       /* frames never read back are dropped, as freed */
    pthread_mutex_unlock(&g_reg_mu);
    free(c->ref_a_rbsp);
    free(c->ref_b_rbsp);
    free(c->orig_sps);
    free(c->orig_pps);
    free(c->output_buffer);
    free(c->rbsp_temp);
    memset(c, 0, sizeof(*c));
}
