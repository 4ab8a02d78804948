/*
 * scroll_oracle.c -- CPU ORACLE (test infrastructure only; see scroll_oracle.h).
 *
 * Restates, in plain C, the reference composer path:
 *   src/bitwriter.c, src/nal.c, src/h264_writer.c, src/composer.c,
 *   src/nal_parser.c, experiments/scroll-encoder/src/{h264_encoder,main}.c
 * of wreuven/h264-scroll-encoder.  The per-macroblock loop is kept in the
 * reference's own shape (row buffers of neighbour MV info) on purpose: it is
 * the independent check of the GPU path's row-class compaction.
 */
#include "scroll_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------ */
/* configuration: src/h264_writer.c:13-44                                    */
/* ------------------------------------------------------------------------ */
void or_cfg_init(or_cfg *c, int w, int h)
{
    memset(c, 0, sizeof(*c));
    c->w = w;
    c->h = h;
    c->log2_mfn = 4;
    c->poc_type = 2;
    c->log2_poc = 4;
    c->num_ref_default_m1 = 1;
    c->deblock = 1;
}

/* ------------------------------------------------------------------------ */
/* bits: src/bitwriter.c:13-131 (MSB-first, partial byte zero-padded)        */
/* ------------------------------------------------------------------------ */
void or_bits_init(or_bits *b, uint8_t *buf, size_t cap)
{
    b->buf = buf;
    b->cap = cap;
    b->nbits = 0;
}

static void or_bit(or_bits *b, int bit)
{
    size_t byte = b->nbits >> 3;
    int sh = 7 - (int)(b->nbits & 7);
    if (byte >= b->cap)
        abort();                       /* reference: assert (bitwriter.c:18) */
    if (sh == 7)
        b->buf[byte] = 0;
    if (bit & 1)
        b->buf[byte] |= (uint8_t)(1u << sh);
    b->nbits++;
}

void or_put(or_bits *b, uint32_t v, int n)
{
    for (int i = n - 1; i >= 0; --i)
        or_bit(b, (int)((v >> i) & 1u));
}

void or_ue(or_bits *b, uint32_t v)
{
    /* Exp-Golomb: M zeros, then (v+1) in M+1 bits, M = floor(log2(v+1)).
     * bitwriter.c:50-74 computes v+1 in uint32 (wraps for 0xFFFFFFFF). */
    if (v == 0) {
        or_bit(b, 1);
        return;
    }
    uint32_t x = v + 1u;
    int m = 0;
    for (uint32_t t = x; t > 1; t >>= 1)
        m++;
    for (int i = 0; i < m; ++i)
        or_bit(b, 0);
    or_put(b, x, m + 1);
}

void or_se(or_bits *b, int32_t v)
{
    /* bitwriter.c:91-101: v>0 -> 2v-1, else -2v (uint32 arithmetic) */
    uint32_t k = v > 0 ? 2u * (uint32_t)v - 1u : (uint32_t)(-2 * (int64_t)v);
    or_ue(b, k);
}

void or_trailing(or_bits *b)
{
    or_bit(b, 1);
    while (b->nbits & 7)
        or_bit(b, 0);
}

size_t or_bytes(or_bits *b)
{
    return (b->nbits + 7) >> 3;
}

/* ------------------------------------------------------------------------ */
/* NAL framing: src/nal.c:24-84                                              */
/* ------------------------------------------------------------------------ */
size_t or_rbsp_to_ebsp(uint8_t *dst, size_t cap, const uint8_t *src, size_t n)
{
    size_t o = 0;
    int zeros = 0;
    for (size_t i = 0; i < n; ++i) {
        uint8_t v = src[i];
        if (zeros >= 2 && v <= 3) {
            if (o >= cap) abort();
            dst[o++] = 3;
            zeros = 0;
        }
        if (o >= cap) abort();
        dst[o++] = v;
        zeros = v ? 0 : zeros + 1;
    }
    return o;
}

size_t or_nal(uint8_t *dst, size_t cap, int ref_idc, int type,
              const uint8_t *rbsp, size_t n)
{
    /* every caller on this path uses the 4-byte start code */
    if (cap < 5) abort();
    dst[0] = 0; dst[1] = 0; dst[2] = 0; dst[3] = 1;
    dst[4] = (uint8_t)(((ref_idc & 3) << 5) | (type & 31));
    return 5 + or_rbsp_to_ebsp(dst + 5, cap - 5, rbsp, n);
}

/* ------------------------------------------------------------------------ */
/* P slice headers: src/h264_writer.c:455-539                                */
/* ------------------------------------------------------------------------ */
static void or_frame_poc(or_bits *b, const or_cfg *c, int fn)
{
    int nb = c->log2_mfn;
    or_put(b, (uint32_t)(fn & ((1 << nb) - 1)), nb);
    if (c->poc_type == 0) {
        int pb = c->log2_poc;
        or_put(b, (uint32_t)((fn * 2) & ((1 << pb) - 1)), pb);
    }
}

/* :455-488 -- two long-term refs, no waypoints */
static void or_hdr_plain(or_bits *b, const or_cfg *c, int fn, int is_ref, int qpd)
{
    or_ue(b, 0);
    or_ue(b, 0);           /* SLICE_TYPE_P */
    or_ue(b, 0);
    or_frame_poc(b, c, fn);
    or_bit(b, 1);
    or_ue(b, 1);
    or_bit(b, 1);
    or_ue(b, 2); or_ue(b, 0);
    or_ue(b, 2); or_ue(b, 1);
    or_ue(b, 3);
    if (is_ref)
        or_bit(b, 0);
    or_se(b, qpd);         /* slice_qp_delta (0; the dynamic rect's QP - 26) */
    if (c->deblock)
        or_ue(b, 1);
}

/* :490-539 -- waypoint-aware list, optional MMCO marking */
static void or_hdr_wp(or_bits *b, const or_cfg *c, int fn, int is_ref, int lt_idx, int qpd)
{
    or_ue(b, 0);
    or_ue(b, 0);
    or_ue(b, 0);
    or_frame_poc(b, c, fn);
    or_bit(b, 1);
    or_ue(b, (uint32_t)(2 + c->nwp - 1));
    or_bit(b, 1);
    or_ue(b, 2); or_ue(b, 0);
    or_ue(b, 2); or_ue(b, 1);
    for (int i = 0; i < c->nwp; ++i) {
        if (!c->wp_valid[i]) continue;
        or_ue(b, 2);
        or_ue(b, (uint32_t)c->wp_lt[i]);
    }
    or_ue(b, 3);
    if (is_ref) {
        if (lt_idx >= 0) {
            or_bit(b, 1);
            or_ue(b, 4); or_ue(b, (uint32_t)(lt_idx + 1));
            or_ue(b, 6); or_ue(b, (uint32_t)lt_idx);
            or_ue(b, 0);
        } else {
            or_bit(b, 0);
        }
    }
    or_se(b, qpd);         /* slice_qp_delta (0; the dynamic rect's QP - 26) */
    if (c->deblock)
        or_ue(b, 1);
}

/* ------------------------------------------------------------------------ */
/* MV prediction: src/h264_writer.c:356-432                                  */
/* ------------------------------------------------------------------------ */

/* median3 :362-367 -- NOT a true median (returns c when c < min(a,b)) */
static int or_median3(int a, int b, int c)
{
    if (a > b) { int t = a; a = b; b = t; }
    if (b > c) b = c;
    if (a > b) a = b;
    return b > a ? b : a;
}

void or_predict(int x, int y, int mbw, const or_mvi *above, const or_mvi *left,
                int ref, int *px, int *py)
{
    or_mvi n[3];
    int avail[3] = {0, 0, 0}, match[3] = {0, 0, 0};
    memset(n, 0, sizeof(n));
    if (x > 0 && left->avail) {                       /* A: left */
        n[0] = *left; avail[0] = 1;
    }
    if (y > 0 && above[x].avail) {                    /* B: above */
        n[1] = above[x]; avail[1] = 1;
    }
    if (y > 0 && x + 1 < mbw && above[x + 1].avail) { /* C: above-right */
        n[2] = above[x + 1]; avail[2] = 1;
    } else if (y > 0 && x > 0 && above[x - 1].avail) {/* D: above-left */
        n[2] = above[x - 1]; avail[2] = 1;
    }
    int na = 0, nm = 0;
    for (int k = 0; k < 3; ++k) {
        match[k] = avail[k] && n[k].ref == ref;
        na += avail[k];
        nm += match[k];
    }
    if (na == 0) {
        *px = 0; *py = 0;
    } else if (na == 1) {
        int k = avail[0] ? 0 : (avail[1] ? 1 : 2);
        *px = match[k] ? n[k].mx : 0;
        *py = match[k] ? n[k].my : 0;
    } else if (nm == 1) {
        int k = match[0] ? 0 : (match[1] ? 1 : 2);
        *px = n[k].mx;
        *py = n[k].my;
    } else {
        *px = or_median3(avail[0] ? n[0].mx : 0, avail[1] ? n[1].mx : 0, avail[2] ? n[2].mx : 0);
        *py = or_median3(avail[0] ? n[0].my : 0, avail[1] ? n[1].my : 0, avail[2] ? n[2].my : 0);
    }
}

/* write_p16x16_mb :434-453 preceded by mb_skip_run ue(0) (:630) */
static void or_mb(or_bits *b, int ref, int dx, int dy, int nrefs)
{
    or_ue(b, 0);              /* mb_skip_run (P_Skip disabled) */
    or_ue(b, 0);              /* mb_type P_L0_16x16 */
    if (nrefs == 2)
        or_bit(b, 1 - (ref & 1));
    else if (nrefs > 2)
        or_ue(b, (uint32_t)ref);
    or_se(b, dx);
    or_se(b, dy);
    or_ue(b, 0);              /* coded_block_pattern = 0 */
}

/* MB loop shared by :595-646 and :712-756.  region A rows use (ra, mva),
 * region B rows use (rb, mvb); mv in pixels, written in quarter-pel. */
static void or_mb_loop(or_bits *b, const or_cfg *c, int a_end,
                       int ra, int mva, int rb, int mvb)
{
    int mbw = c->w / 16, mbh = c->h / 16;
    or_mvi *above = (or_mvi *)calloc((size_t)(mbw > 0 ? mbw : 1), sizeof(or_mvi));
    or_mvi *cur = (or_mvi *)calloc((size_t)(mbw > 0 ? mbw : 1), sizeof(or_mvi));
    int nrefs = 2 + c->nwp;
    for (int y = 0; y < mbh; ++y) {
        or_mvi left;
        memset(&left, 0, sizeof(left));
        for (int x = 0; x < mbw; ++x) {
            int ref = y < a_end ? ra : rb;
            int my = (y < a_end ? mva : mvb) * 4;
            int px, py;
            or_predict(x, y, mbw, above, &left, ref, &px, &py);
            or_mb(b, ref, 0 - px, my - py, nrefs);
            cur[x].mx = 0;
            cur[x].my = my;
            cur[x].ref = ref;
            cur[x].avail = 1;
            left = cur[x];
        }
        or_mvi *t = above; above = cur; cur = t;
    }
    free(above);
    free(cur);
}

/* slice header of a scroll (non-reference) P frame, :549-553 (slice_qp_delta
 * qpd: 0 as the reference writes it; a dynamic rect's QP - 26) */
void or_scroll_header_qpd(or_bits *b, const or_cfg *c, int qpd)
{
    int fn = c->frame_num % (1 << c->log2_mfn);
    if (c->nwp > 0)
        or_hdr_wp(b, c, fn, 0, -1, qpd);
    else
        or_hdr_plain(b, c, fn, 0, qpd);
}

void or_scroll_header(or_bits *b, const or_cfg *c) { or_scroll_header_qpd(b, c, 0); }

/* :541-664 */
size_t or_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off)
{
    size_t rcap = 64 + (size_t)(c->w / 16) * (size_t)(c->h / 16) * 24;
    uint8_t *rbsp = (uint8_t *)malloc(rcap);
    or_bits b;
    or_bits_init(&b, rbsp, rcap);
    int fn = c->frame_num % (1 << c->log2_mfn);
    if (c->nwp > 0)
        or_hdr_wp(&b, c, fn, 0, -1, 0);
    else
        or_hdr_plain(&b, c, fn, 0, 0);

    int a_end, ra, mva, rb, mvb;
    or_scroll_regions(c, off, &a_end, &ra, &mva, &rb, &mvb);
    or_mb_loop(&b, c, a_end, ra, mva, rb, mvb);
    or_trailing(&b);
    size_t n = or_nal(dst, cap, 0, 1, rbsp, or_bytes(&b));
    free(rbsp);
    c->frame_num++;
    return n;
}

/* region split and waypoint choice of a scroll frame, :555-617 */
void or_scroll_regions(const or_cfg *c, int off, int *a_end_out, int *ra_out, int *mva_out,
                       int *rb_out, int *mvb_out)
{
    /* A-region waypoint (:558-571): best valid wo <= off, wo > best, off-wo <= 496 */
    int wa = -1, woa = 0;
    if (off > OR_MV_LIMIT && c->nwp > 0) {
        for (int i = 0; i < c->nwp; ++i) {
            if (!c->wp_valid[i]) continue;
            int wo = c->wp_off[i];
            if (wo <= off && wo > woa && off - wo <= OR_MV_LIMIT) {
                wa = i; woa = wo;
            }
        }
    }
    /* B-region waypoint (:573-588): FIRST valid wo > off with off-wo >= -496 */
    int wb = -1, wob = 0;
    if (off - c->h < -OR_MV_LIMIT && c->nwp > 0) {
        for (int i = 0; i < c->nwp; ++i) {
            if (!c->wp_valid[i]) continue;
            int wo = c->wp_off[i];
            if (wo > off && off - wo >= -OR_MV_LIMIT) {
                wb = i; wob = wo;
                break;
            }
        }
    }
    *a_end_out = (c->h - off) / 16;
    *ra_out = wa >= 0 ? 2 + wa : 0;
    *mva_out = wa >= 0 ? off - woa : off;
    *rb_out = wb >= 0 ? 2 + wb : 1;
    *mvb_out = wb >= 0 ? off - wob : off - c->h;
}

/* :666-676 */
int or_needs_waypoint(const or_cfg *c, int off)
{
    if (off == 0 || off % OR_MV_LIMIT != 0)
        return 0;
    for (int i = 0; i < c->nwp; ++i)
        if (c->wp_valid[i] && c->wp_off[i] == off)
            return 0;
    return 1;
}

/* :678-782 */
size_t or_waypoint_nal(uint8_t *dst, size_t cap, or_cfg *c, int off)
{
    size_t rcap = 64 + (size_t)(c->w / 16) * (size_t)(c->h / 16) * 24;
    uint8_t *rbsp = (uint8_t *)malloc(rcap);
    or_bits b;
    or_bits_init(&b, rbsp, rcap);
    int fn = c->frame_num % (1 << c->log2_mfn);
    int lt = 2 + c->nwp;
    or_hdr_wp(&b, c, fn, 1, lt, 0);
    int a_end = (c->h - off) / 16;
    int wa = -1, woa = 0;
    if (off > OR_MV_LIMIT) {
        for (int i = 0; i < c->nwp; ++i) {
            if (!c->wp_valid[i]) continue;
            int wo = c->wp_off[i];
            if (wo <= off && wo > woa && off - wo <= OR_MV_LIMIT) {
                wa = i; woa = wo;
            }
        }
    }
    int ra = wa >= 0 ? 2 + wa : 0, mva = wa >= 0 ? off - woa : off;
    or_mb_loop(&b, c, a_end, ra, mva, 1, off - c->h);   /* B always ref 1 (:726-729) */
    or_trailing(&b);
    size_t n = or_nal(dst, cap, 2, 1, rbsp, or_bytes(&b));
    free(rbsp);
    if (c->nwp < OR_MAX_WP) {                             /* :772-777 */
        c->wp_off[c->nwp] = off;
        c->wp_lt[c->nwp] = lt;
        c->wp_valid[c->nwp] = 1;
        c->nwp++;
    }
    c->frame_num++;
    return n;
}

size_t or_compose(uint8_t *dst, size_t cap, or_cfg *c, int off, int mode, int *n_wp_out)
{
    size_t n = 0;
    int nw = 0;
    if (or_needs_waypoint(c, off)) {
        n += or_waypoint_nal(dst, cap, c, off);
        nw = 1;
        if (mode == 1) {
            if (n_wp_out) *n_wp_out = nw;
            return n;
        }
    }
    n += or_scroll_nal(dst + n, cap - n, c, off);
    if (n_wp_out) *n_wp_out = nw;
    return n;
}

/* ------------------------------------------------------------------------ */
/* headers: src/h264_writer.c:49-127                                         */
/* ------------------------------------------------------------------------ */
size_t or_sps(uint8_t *rbsp, size_t cap, int w, int h)
{
    or_bits b;
    or_bits_init(&b, rbsp, cap);
    or_put(&b, 66, 8);
    or_put(&b, 0xc0, 8);
    or_put(&b, 40, 8);
    or_ue(&b, 0);
    or_ue(&b, 0);
    or_ue(&b, 2);
    or_ue(&b, 2 + OR_MAX_WP);
    or_bit(&b, 0);
    or_ue(&b, (uint32_t)(w / 16 - 1));
    or_ue(&b, (uint32_t)(h / 16 - 1));
    or_bit(&b, 1);
    or_bit(&b, 1);
    or_bit(&b, 0);
    or_bit(&b, 0);
    or_trailing(&b);
    return or_bytes(&b);
}

size_t or_pps(uint8_t *rbsp, size_t cap)
{
    or_bits b;
    or_bits_init(&b, rbsp, cap);
    or_ue(&b, 0);
    or_ue(&b, 0);
    or_bit(&b, 0);
    or_bit(&b, 0);
    or_ue(&b, 0);
    or_ue(&b, 1);
    or_ue(&b, 0);
    or_bit(&b, 0);
    or_put(&b, 0, 2);
    or_se(&b, 0);
    or_se(&b, 0);
    or_se(&b, 0);
    or_bit(&b, 1);
    or_bit(&b, 0);
    or_bit(&b, 0);
    or_trailing(&b);
    return or_bytes(&b);
}

/* ------------------------------------------------------------------------ */
/* bit reader (src/h264_writer.c:141-192, src/nal_parser.c:93-135)           */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t *p;
    size_t n;
    size_t pos;   /* bit position */
} or_rd;

static int or_rbit(or_rd *r)
{
    if ((r->pos >> 3) >= r->n) return 0;          /* EOF reads as 0 */
    int v = (r->p[r->pos >> 3] >> (7 - (r->pos & 7))) & 1;
    r->pos++;
    return v;
}
static uint32_t or_rbits(or_rd *r, int n)
{
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | (uint32_t)or_rbit(r);
    return v;
}
static uint32_t or_rue(or_rd *r)
{
    int lz = 0;
    while (or_rbit(r) == 0 && lz < 32) lz++;
    if (lz == 0) return 0;
    return (1u << lz) - 1u + or_rbits(r, lz);
}
static int32_t or_rse(or_rd *r)
{
    uint32_t k = or_rue(r);
    return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
}

typedef struct {
    size_t mb_start;
    int32_t qpd;
    uint32_t dbf;
    int32_t alpha, beta;
} or_slice_hdr;

/* parse_idr_slice_header :194-226 */
static void or_parse_idr(const uint8_t *rbsp, size_t n, const or_cfg *pc, or_slice_hdr *h)
{
    or_rd r = {rbsp, n, 0};
    memset(h, 0, sizeof(*h));
    or_rue(&r); or_rue(&r); or_rue(&r);
    or_rbits(&r, pc->log2_mfn);
    or_rue(&r);
    if (pc->poc_type == 0) or_rbits(&r, pc->log2_poc);
    or_rbit(&r); or_rbit(&r);
    h->qpd = or_rse(&r);
    if (pc->deblock) {
        h->dbf = or_rue(&r);
        if (h->dbf != 1) {
            h->alpha = or_rse(&r);
            h->beta = or_rse(&r);
        }
    }
    h->mb_start = r.pos;
}

static void or_copy_bits(or_bits *b, const uint8_t *src, size_t n, size_t from)
{
    or_rd r = {src, n, from};
    size_t total = n * 8;
    for (size_t i = from; i < total; ++i) or_bit(b, or_rbit(&r));
}

static void or_tail_fields(or_bits *b, const or_cfg *wr, const or_slice_hdr *h)
{
    or_se(b, h->qpd);
    if (wr->deblock) {
        or_ue(b, h->dbf);
        if (h->dbf != 1) {
            or_se(b, h->alpha);
            or_se(b, h->beta);
        }
    }
}

size_t or_rewrite_idr(uint8_t *dst, size_t cap, or_cfg *wr, const or_cfg *pc,
                      const uint8_t *rbsp, size_t n)
{
    or_slice_hdr h;
    or_parse_idr(rbsp, n, pc, &h);
    size_t oc = n + 256;
    uint8_t *o = (uint8_t *)malloc(oc);
    or_bits b;
    or_bits_init(&b, o, oc);
    or_ue(&b, 0);
    or_ue(&b, 7);
    or_ue(&b, 0);
    or_put(&b, 0, wr->log2_mfn);
    or_ue(&b, (uint32_t)wr->idr_pic_id);
    if (wr->poc_type == 0) or_put(&b, 0, wr->log2_poc);
    or_bit(&b, 0);
    or_bit(&b, 1);
    or_tail_fields(&b, wr, &h);
    or_copy_bits(&b, rbsp, n, h.mb_start);
    size_t r = or_nal(dst, cap, 3, 5, o, or_bytes(&b));
    free(o);
    wr->frame_num = 1;
    return r;
}

static size_t or_rewrite_non_idr_lt(uint8_t *dst, size_t cap, or_cfg *wr, const or_cfg *pc,
                                    const uint8_t *rbsp, size_t n, int frame_num, int lt_idx);

size_t or_rewrite_non_idr(uint8_t *dst, size_t cap, or_cfg *wr, const or_cfg *pc,
                          const uint8_t *rbsp, size_t n, int frame_num)
{
    return or_rewrite_non_idr_lt(dst, cap, wr, pc, rbsp, n, frame_num, 1);
}

/* the same with long_term_frame_idx lt_idx in the MMCO 6 (the reference
 * writes 1, :328) */
static size_t or_rewrite_non_idr_lt(uint8_t *dst, size_t cap, or_cfg *wr, const or_cfg *pc,
                                    const uint8_t *rbsp, size_t n, int frame_num, int lt_idx)
{
    or_slice_hdr h;
    or_parse_idr(rbsp, n, pc, &h);
    size_t oc = n + 256;
    uint8_t *o = (uint8_t *)malloc(oc);
    or_bits b;
    or_bits_init(&b, o, oc);
    or_ue(&b, 0);
    or_ue(&b, 7);
    or_ue(&b, 0);
    or_put(&b, (uint32_t)frame_num, wr->log2_mfn);
    if (wr->poc_type == 0) or_put(&b, (uint32_t)(frame_num * 2), wr->log2_poc);
    or_bit(&b, 1);
    or_ue(&b, 4); or_ue(&b, 2);
    or_ue(&b, 6); or_ue(&b, (uint32_t)lt_idx);
    or_ue(&b, 0);
    or_tail_fields(&b, wr, &h);
    or_copy_bits(&b, rbsp, n, h.mb_start);
    size_t r = or_nal(dst, cap, 3, 1, o, or_bytes(&b));
    free(o);
    wr->frame_num = frame_num + 1;
    return r;
}

/* ------------------------------------------------------------------------ */
/* I_PCM striped frames: experiments/scroll-encoder/src/h264_encoder.c        */
/* ------------------------------------------------------------------------ */
static void or_ipcm_mb(or_bits *b, uint8_t y, uint8_t cb, uint8_t cr)  /* :730-753 */
{
    or_ue(b, 25);
    while (b->nbits & 7) or_bit(b, 0);
    for (int i = 0; i < 256; ++i) or_put(b, y, 8);
    for (int i = 0; i < 64; ++i) or_put(b, cb, 8);
    for (int i = 0; i < 64; ++i) or_put(b, cr, 8);
}

size_t or_ipcm_striped(uint8_t *dst, size_t cap, or_cfg *c, int which, const uint8_t yuv[9])
{
    int mbw = c->w / 16, mbh = c->h / 16;
    size_t rc = (size_t)mbw * (size_t)mbh * 400 + 1024;
    uint8_t *o = (uint8_t *)malloc(rc);
    or_bits b;
    or_bits_init(&b, o, rc);
    int fn = which == 0 ? 0 : c->frame_num;
    if (which == 0) c->frame_num = 0;
    or_ue(&b, 0);
    or_ue(&b, 7);
    or_ue(&b, 0);
    or_put(&b, (uint32_t)fn, c->log2_mfn);
    if (which == 0) {                       /* IDR header :622-662 */
        or_ue(&b, (uint32_t)c->idr_pic_id);
        if (c->poc_type == 0) or_put(&b, 0, c->log2_poc);
        or_bit(&b, 0);
        or_bit(&b, 1);
    } else {                                /* non-IDR header :667-715 */
        if (c->poc_type == 0) or_put(&b, (uint32_t)(fn * 2), c->log2_poc);
        or_bit(&b, 1);
        or_ue(&b, 4); or_ue(&b, 2);
        or_ue(&b, 6); or_ue(&b, 1);
        or_ue(&b, 0);
    }
    or_se(&b, 0);
    if (c->deblock) or_ue(&b, 1);
    int third = mbh / 3;                    /* :816-829 */
    for (int y = 0; y < mbh; ++y) {
        int s = y < third ? 0 : (y < 2 * third ? 1 : 2);
        for (int x = 0; x < mbw; ++x)
            or_ipcm_mb(&b, yuv[3 * s], yuv[3 * s + 1], yuv[3 * s + 2]);
    }
    or_trailing(&b);
    size_t r = which == 0 ? or_nal(dst, cap, 3, 5, o, or_bytes(&b))
                          : or_nal(dst, cap, 3, 1, o, or_bytes(&b));
    free(o);
    if (which == 0) c->frame_num = 1; else c->frame_num++;
    return r;
}

/* experiments/scroll-encoder/src/main.c:234-243 colours */
static const uint8_t OR_STRIPES_A[9] = {81, 90, 240, 145, 54, 34, 41, 240, 110};
static const uint8_t OR_STRIPES_B[9] = {210, 16, 146, 170, 166, 16, 106, 202, 222};

static size_t or_sps_pps(uint8_t *dst, size_t cap, int w, int h)
{
    uint8_t tmp[256];
    size_t n = or_sps(tmp, sizeof(tmp), w, h);
    size_t o = or_nal(dst, cap, 3, 7, tmp, n);
    n = or_pps(tmp, sizeof(tmp));
    o += or_nal(dst + o, cap - o, 3, 8, tmp, n);
    return o;
}

size_t or_ipcm_ref_file(uint8_t *dst, size_t cap, int w, int h, int which)
{
    or_cfg c;
    or_cfg_init(&c, w, h);
    size_t o = or_sps_pps(dst, cap, w, h);
    /* both refs are written as IDR frames */
    o += or_ipcm_striped(dst + o, cap - o, &c, 0, which == 0 ? OR_STRIPES_A : OR_STRIPES_B);
    return o;
}

/* An arbitrary I420 picture as one IDR of I_PCM MBs: the IDR header of
 * or_ipcm_striped (h264_encoder.c:622-662) and h264_write_ipcm_mb (:730-753)
 * with the picture's own samples in place of a stripe colour (raster order
 * inside the MB: 256 luma, 64 Cb, 64 Cr). */
size_t or_ipcm_picture_file(uint8_t *dst, size_t cap, int w, int h, const uint8_t *pic)
{
    or_cfg c;
    or_cfg_init(&c, w, h);
    size_t o = or_sps_pps(dst, cap, w, h);
    const int mbw = w / 16, mbh = h / 16;
    const uint8_t *Y = pic, *U = pic + (size_t)w * h, *V = U + (size_t)w * h / 4;
    size_t rc = (size_t)mbw * (size_t)mbh * 400 + 1024;
    uint8_t *rb = (uint8_t *)malloc(rc);
    or_bits b;
    or_bits_init(&b, rb, rc);
    or_ue(&b, 0);
    or_ue(&b, 7);
    or_ue(&b, 0);
    or_put(&b, 0, c.log2_mfn);
    or_ue(&b, (uint32_t)c.idr_pic_id);
    if (c.poc_type == 0) or_put(&b, 0, c.log2_poc);
    or_put(&b, 0, 1);
    or_put(&b, 1, 1);
    or_se(&b, 0);
    if (c.deblock) or_ue(&b, 1);
    for (int my = 0; my < mbh; ++my)
        for (int mx = 0; mx < mbw; ++mx) {
            or_ue(&b, 25);
            while (b.nbits & 7) or_put(&b, 0, 1);
            for (int i = 0; i < 256; ++i) or_put(&b, Y[(size_t)(16 * my + i / 16) * w + 16 * mx + i % 16], 8);
            for (int i = 0; i < 64; ++i) or_put(&b, U[(size_t)(8 * my + i / 8) * (w / 2) + 8 * mx + i % 8], 8);
            for (int i = 0; i < 64; ++i) or_put(&b, V[(size_t)(8 * my + i / 8) * (w / 2) + 8 * mx + i % 8], 8);
        }
    or_trailing(&b);
    o += or_nal(dst + o, cap - o, 3, 5, rb, or_bytes(&b));
    free(rb);
    return o;
}

/* ------------------------------------------------------------------------ */
/* ingest: src/nal_parser.c:14-276                                           */
/* ------------------------------------------------------------------------ */
size_t or_ebsp_to_rbsp(uint8_t *dst, const uint8_t *src, size_t n)
{
    size_t o = 0;
    int zeros = 0;
    for (size_t i = 0; i < n; ++i) {
        if (zeros >= 2 && src[i] == 3 && i + 1 < n && src[i + 1] <= 3) {
            zeros = 0;
            continue;
        }
        dst[o++] = src[i];
        zeros = src[i] ? 0 : zeros + 1;
    }
    return o;
}

/* start code scan (:14-26); returns index after the start code or n */
static size_t or_find_sc(const uint8_t *d, size_t n, size_t from)
{
    for (size_t i = from; i + 2 < n; ++i) {
        if (d[i] == 0 && d[i + 1] == 0) {
            if (d[i + 2] == 1) return i + 3;
            if (i + 3 < n && d[i + 2] == 0 && d[i + 3] == 1) return i + 4;
        }
    }
    return n;
}

/* nal_parser_next (:28-65). Returns 1 and fills (type, payload) or 0. */
static int or_next_nal(const uint8_t *d, size_t n, size_t *pos, int *type,
                       const uint8_t **pl, size_t *pn)
{
    size_t s = or_find_sc(d, n, *pos);
    if (s >= n) return 0;
    size_t e = n;
    for (size_t i = s; i + 2 < n; ++i) {
        if (d[i] == 0 && d[i + 1] == 0 &&
            (d[i + 2] == 1 || (i + 3 < n && d[i + 2] == 0 && d[i + 3] == 1))) {
            e = i;
            break;
        }
    }
    while (e > s && d[e - 1] == 0) e--;
    if (e <= s) {
        *pos = e;
        return 0;
    }
    *type = d[s] & 31;
    *pl = d + s + 1;
    *pn = e - s - 1;
    *pos = e;
    return 1;
}

/* parse_sps (:137-222) */
static int or_parse_sps(const uint8_t *p, size_t n, int *w, int *h, int *l2f, int *poct, int *l2p)
{
    or_rd r = {p, n, 0};
    int prof = (int)or_rbits(&r, 8);
    or_rbits(&r, 8);
    or_rbits(&r, 8);
    or_rue(&r);
    if (prof == 100 || prof == 110 || prof == 122 || prof == 244 || prof == 44 ||
        prof == 83 || prof == 86 || prof == 118 || prof == 128 || prof == 138 ||
        prof == 139 || prof == 134) {
        if (or_rue(&r) == 3) or_rbit(&r);
        or_rue(&r);
        or_rue(&r);
        or_rbit(&r);
        if (or_rbit(&r)) return -1;
    }
    *l2f = (int)or_rue(&r) + 4;
    *poct = (int)or_rue(&r);
    *l2p = 0;
    if (*poct == 0) *l2p = (int)or_rue(&r) + 4;
    else if (*poct == 1) return -1;
    or_rue(&r);
    or_rbit(&r);
    int wm = (int)or_rue(&r) + 1;
    int hm = (int)or_rue(&r) + 1;
    if (!or_rbit(&r)) {
        or_rbit(&r);
        hm *= 2;
    }
    *w = wm * 16;
    *h = hm * 16;
    return 0;
}

/* parse_pps (:224-276) */
static int or_parse_pps(const uint8_t *p, size_t n, int *nref, int *dbf)
{
    or_rd r = {p, n, 0};
    or_rue(&r); or_rue(&r);
    or_rbit(&r); or_rbit(&r);
    if (or_rue(&r) > 0) return -1;
    *nref = (int)or_rue(&r);
    or_rue(&r);
    or_rbit(&r);
    or_rbits(&r, 2);
    or_rue(&r); or_rue(&r); or_rue(&r);
    *dbf = or_rbit(&r);
    return 0;
}

typedef struct {
    int w, h, l2f, poct, l2p, nref, dbf;
    uint8_t *idr;
    size_t nidr;
} or_refinfo;

/* parse_reference_file (src/composer.c:45-125) */
static int or_parse_ref(const uint8_t *d, size_t n, or_refinfo *ri)
{
    int got_sps = 0, got_pps = 0, got_idr = 0, type;
    const uint8_t *pl;
    size_t pn, pos = 0;
    uint8_t *tmp = (uint8_t *)malloc(n ? n : 1);
    memset(ri, 0, sizeof(*ri));
    while (or_next_nal(d, n, &pos, &type, &pl, &pn)) {
        if (type == 7 && !got_sps) {
            size_t rn = or_ebsp_to_rbsp(tmp, pl, pn);
            if (or_parse_sps(tmp, rn, &ri->w, &ri->h, &ri->l2f, &ri->poct, &ri->l2p) < 0) {
                free(tmp);
                return -1;
            }
            got_sps = 1;
        } else if (type == 8 && !got_pps) {
            size_t rn = or_ebsp_to_rbsp(tmp, pl, pn);
            if (or_parse_pps(tmp, rn, &ri->nref, &ri->dbf) < 0) {
                free(tmp);
                return -1;
            }
            got_pps = 1;
        } else if (type == 5 && !got_idr) {
            size_t rn = or_ebsp_to_rbsp(tmp, pl, pn);
            ri->idr = (uint8_t *)malloc(rn ? rn : 1);
            memcpy(ri->idr, tmp, rn);
            ri->nidr = rn;
            got_idr = 1;
        }
    }
    free(tmp);
    if (!got_sps || !got_pps || !got_idr) {
        free(ri->idr);
        ri->idr = NULL;
        return -1;
    }
    return 0;
}

size_t or_composer_run(uint8_t *dst, size_t cap,
                       const uint8_t *ref_a, size_t na,
                       const uint8_t *ref_b, size_t nb,
                       int nframes, int speed)
{
    or_refinfo a, b;
    if (or_parse_ref(ref_a, na, &a) < 0) return 0;
    if (or_parse_ref(ref_b, nb, &b) < 0) {
        free(a.idr);
        return 0;
    }
    if (a.w != b.w || a.h != b.h) {
        free(a.idr);
        free(b.idr);
        return 0;
    }
    or_cfg pc, wc;
    or_cfg_init(&pc, a.w, a.h);                     /* composer.c:193-196 */
    pc.log2_mfn = a.l2f; pc.poc_type = a.poct; pc.log2_poc = a.l2p;
    pc.num_ref_default_m1 = a.nref; pc.deblock = a.dbf;
    or_cfg_init(&wc, a.w, a.h);                     /* composer.c:199-203 */
    wc.log2_mfn = 4; wc.poc_type = 2; wc.log2_poc = 4;
    wc.num_ref_default_m1 = 1; wc.deblock = a.dbf;

    size_t o = or_sps_pps(dst, cap, a.w, a.h);      /* composer_write_header */
    o += or_rewrite_idr(dst + o, cap - o, &wc, &pc, a.idr, a.nidr);
    o += or_rewrite_non_idr(dst + o, cap - o, &wc, &pc, b.idr, b.nidr, 1);
    for (int i = 0; i < nframes; ++i) {
        int off = or_tri(i * speed, a.h);           /* src/main.c:109-120 */
        o += or_compose(dst + o, cap - o, &wc, off, 0, NULL);
    }
    free(a.idr);
    free(b.idr);
    return o;
}

/* Mid-stream long-term reference ("atlas") update -- no reference function:
 * the file's IDR picture (parse_reference_file's rules, parsed with its own
 * SPS / PPS like composer_init, src/composer.c:127-196) written as a non-IDR
 * I frame of stream c, h264_rewrite_as_non_idr_i_frame (h264_writer.c:296-350)
 * with long_term_frame_idx `which` (0 = A, 1 = B) at the stream's frame_num
 * (mod 2^log2_max_frame_num, POC lsb 2 frame_num, as the waypoint frames,
 * :683-687); its MMCO 4 (max_long_term_frame_idx_plus1 2) drops every
 * waypoint, so c loses its waypoints and frame_num advances (:779-781).  0
 * (c unchanged) if the file is refused or its picture size differs. */
size_t or_update_ref(uint8_t *dst, size_t cap, or_cfg *c, const uint8_t *file, size_t n, int which)
{
    or_refinfo ri;
    if (which < 0 || which > 1 || or_parse_ref(file, n, &ri) < 0) return 0;
    if (ri.w != c->w || ri.h != c->h) {
        free(ri.idr);
        return 0;
    }
    or_cfg pc;
    or_cfg_init(&pc, ri.w, ri.h);
    pc.log2_mfn = ri.l2f; pc.poc_type = ri.poct; pc.log2_poc = ri.l2p;
    pc.num_ref_default_m1 = ri.nref; pc.deblock = ri.dbf;
    const int fn = c->frame_num % (1 << c->log2_mfn);
    const int fn_next = c->frame_num + 1;
    size_t r = or_rewrite_non_idr_lt(dst, cap, c, &pc, ri.idr, ri.nidr, fn, which);
    free(ri.idr);
    c->frame_num = fn_next;
    c->nwp = 0;
    for (int k = 0; k < OR_MAX_WP; ++k) c->wp_valid[k] = 0;
    return r;
}

size_t or_experiment_run(uint8_t *dst, size_t cap, int w, int h, int nframes, int speed)
{
    or_cfg c;
    or_cfg_init(&c, w, h);
    size_t o = or_sps_pps(dst, cap, w, h);
    o += or_ipcm_striped(dst + o, cap - o, &c, 0, OR_STRIPES_A);
    o += or_ipcm_striped(dst + o, cap - o, &c, 1, OR_STRIPES_B);
    int maxo = h - 16;                              /* main.c:387 */
    for (int i = 0; i < nframes; ++i) {
        int off = or_tri(i * speed + OR_MV_LIMIT, maxo);   /* main.c:402-415 */
        o += or_compose(dst + o, cap - o, &c, off, 1, NULL);
    }
    return o;
}

/* triangle scroll 0 -> m -> 0 (src/main.c:388-396) */
int or_tri(int x, int m)
{
    int cyc = 2 * m;
    int p = x % cyc;
    return p < m ? p : cyc - p;
}

int or_synthetic_offset(int s, int i, int h)
{
    int v = 1 + (s % 8);
    int phase = (97 * s) % (2 * h);
    return or_tri(i * v + phase, h);
}

/* ------------------------------------------------------------------------ */
/* CPU baseline timer                                                        */
/* ------------------------------------------------------------------------ */
typedef struct {
    int s0, s1, nframes, w, h, warm;
    unsigned long long bytes;
    long long frames;
} or_job;

static void or_stream_init(or_cfg *c, int w, int h)
{
    or_cfg_init(c, w, h);
    c->frame_num = 2;    /* state after composer_write_header */
}

static void *or_worker(void *arg)
{
    or_job *j = (or_job *)arg;
    size_t cap = (size_t)(j->w / 16) * (size_t)(j->h / 16) * 24 + 4096;
    uint8_t *buf = (uint8_t *)malloc(cap * 2);
    for (int s = j->s0; s < j->s1; ++s) {
        or_cfg c;
        or_stream_init(&c, j->w, j->h);
        for (int i = 0; i < j->nframes; ++i) {
            size_t n = or_compose(buf, cap * 2, &c, or_synthetic_offset(s, i, j->h), 0, NULL);
            j->bytes += n;
            j->frames++;
        }
    }
    free(buf);
    return NULL;
}

static double or_now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

double or_bench_compose(int nstreams, int nframes, int w, int h, int nthreads,
                        int warmup_frames, unsigned long long *bytes_out)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > nstreams) nthreads = nstreams;
    if (warmup_frames > 0) {
        or_job wj = {0, 1, warmup_frames, w, h, 0, 0, 0};
        or_worker(&wj);
    }
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    or_job *jobs = (or_job *)calloc((size_t)nthreads, sizeof(or_job));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].s0 = (int)((long long)nstreams * t / nthreads);
        jobs[t].s1 = (int)((long long)nstreams * (t + 1) / nthreads);
        jobs[t].nframes = nframes;
        jobs[t].w = w;
        jobs[t].h = h;
    }
    double t0 = or_now();
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, or_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    double dt = or_now() - t0;
    unsigned long long bytes = 0;
    long long frames = 0;
    for (int t = 0; t < nthreads; ++t) {
        bytes += jobs[t].bytes;
        frames += jobs[t].frames;
    }
    if (bytes_out) *bytes_out = bytes;
    free(th);
    free(jobs);
    return dt > 0 ? (double)frames / dt : 0.0;
}
