/*
 * splice_oracle.c -- CPU ORACLE (test infrastructure only): the pre-encoded
 * MB splice.  See splice_oracle.h for the semantics and what pins the bits.
 * The slice parse follows ITU-T H.264 7.3.3 (slice header), 7.3.4 (slice
 * data), 7.3.5 (macroblock layer), 7.3.5.3 / 9.2 (CAVLC residual) and
 * 8.4.1.1 / 8.4.1.3 (P_Skip motion, median prediction); the composed MB
 * loop follows the UI-hint restatement (hint_oracle.c), itself the
 * reference's scroll frame (src/h264_writer.c:595-646) generalised.
 */
#include "splice_oracle.h"

#include <stdlib.h>
#include <string.h>

#include "dyn_oracle.h"

/* ------------------------------------------------------------------------ */
/* RBSP bit reader                                                           */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t *d;
    size_t nbits, p;
    int bad;                     /* read past the end */
} rd_t;

static uint32_t rd_peek(const rd_t *r, int n)
{
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) {
        const size_t q = r->p + (size_t)i;
        const uint32_t bit = q < r->nbits ? (uint32_t)(r->d[q >> 3] >> (7 - (q & 7))) & 1u : 0u;
        v = (v << 1) | bit;
    }
    return v;
}

static uint32_t rd_u(rd_t *r, int n)
{
    const uint32_t v = rd_peek(r, n);
    r->p += (size_t)n;
    if (r->p > r->nbits) r->bad = 1;
    return v;
}

static uint32_t rd_ue(rd_t *r)
{
    int z = 0;
    while (!r->bad && rd_u(r, 1) == 0)
        if (++z > 31) {
            r->bad = 1;
            return 0;
        }
    if (r->bad || z == 0) return 0;
    return ((1u << z) - 1u) + rd_u(r, z);
}

static int32_t rd_se(rd_t *r)
{
    const uint32_t k = rd_ue(r);
    return (k & 1u) ? (int32_t)((k + 1u) >> 1) : -(int32_t)(k >> 1);
}

/* consume (bits, len) if the stream continues with it */
static int rd_match(rd_t *r, uint32_t bits, int len)
{
    if (len <= 0 || rd_peek(r, len) != bits) return 0;
    r->p += (size_t)len;
    if (r->p > r->nbits) r->bad = 1;
    return 1;
}

/* emulation prevention removal (7.4.1: 0x000003 -> 0x0000) */
static size_t sp_unescape(uint8_t *dst, const uint8_t *src, size_t n)
{
    size_t o = 0;
    int zeros = 0;
    for (size_t i = 0; i < n; ++i) {
        if (zeros >= 2 && src[i] == 3) {
            zeros = 0;
            continue;
        }
        dst[o++] = src[i];
        zeros = src[i] ? 0 : zeros + 1;
    }
    return o;
}

/* ------------------------------------------------------------------------ */
/* CAVLC block: coeff_token, then the nC-independent body (9.2)              */
/* ------------------------------------------------------------------------ */
static int sp_block(rd_t *r, int nC, int maxc, uint8_t *tc_o, uint8_t *t1_o, uint32_t *boff,
                    uint32_t *blen)
{
    int tc = -1, t1 = 0;
    const int tcmax = nC == -1 ? 4 : 16;
    for (int c = 0; c <= tcmax && tc < 0; ++c)
        for (int o = 0; o <= 3 && o <= c; ++o) {
            uint32_t b;
            const int len = or_ct_code(c, o, nC, &b);
            if (rd_match(r, b, len)) {
                tc = c;
                t1 = o;
                break;
            }
        }
    if (tc < 0 || tc > maxc || r->bad) return -1;
    *boff = (uint32_t)r->p;
    if (tc > 0) {
        for (int k = 0; k < t1; ++k) rd_u(r, 1);                 /* trailing_ones_sign_flag */
        int sl = (tc > 10 && t1 < 3) ? 1 : 0;
        for (int k = t1; k < tc; ++k) {
            int prefix = 0;                                       /* level_prefix (9.2.2.1) */
            while (!r->bad && rd_u(r, 1) == 0)
                if (++prefix > 15) return -1;                     /* > 15: High profiles only */
            if (r->bad) return -1;
            int ssize = sl;
            if (prefix == 14 && sl == 0) ssize = 4;
            if (prefix >= 15) ssize = prefix - 3;
            int code = (prefix < 15 ? prefix : 15) << sl;
            if (ssize) code += (int)rd_u(r, ssize);
            if (prefix >= 15 && sl == 0) code += 15;
            if (k == t1 && t1 < 3) code += 2;
            const int L = (code & 1) ? -((code + 1) >> 1) : (code + 2) >> 1;
            if (sl == 0) sl = 1;
            if ((L < 0 ? -L : L) > (3 << (sl - 1)) && sl < 6) sl++;
        }
        int tz = 0;
        if (tc < maxc) {                                          /* total_zeros */
            tz = -1;
            for (int z = 0; z <= maxc - tc; ++z) {
                uint32_t b;
                if (rd_match(r, b, or_tz_code(tc, z, maxc, &b))) {
                    tz = z;
                    break;
                }
            }
            if (tz < 0) return -1;
        }
        int zl = tz;
        for (int k = 0; k < tc - 1 && zl > 0; ++k) {              /* run_before */
            int run = -1;
            for (int q = 0; q <= zl && q <= 14; ++q) {
                uint32_t b;
                if (rd_match(r, b, or_rb_code(zl, q, &b))) {
                    run = q;
                    break;
                }
            }
            if (run < 0) return -1;
            zl -= run;
        }
    }
    *blen = (uint32_t)(r->p - *boff);
    *tc_o = (uint8_t)tc;
    *t1_o = (uint8_t)t1;
    return r->bad ? -1 : 0;
}

static int sp_nc(int nA, int nB)
{
    if (nA >= 0 && nB >= 0) return (nA + nB + 1) >> 1;
    if (nA >= 0) return nA;
    if (nB >= 0) return nB;
    return 0;
}

/* nC of piece i (luma raster 0..15, chroma AC 18..25) of an MB with
 * TotalCoeffs cur; left / top = the neighbour MBs' or NULL (unavailable) */
static int sp_piece_nc(int i, const uint8_t *cur, const uint8_t *left, const uint8_t *top)
{
    if (i < 16) {
        const int bx = i & 3, by = i >> 2;
        const int nA = bx ? cur[i - 1] : (left ? left[i + 3] : -1);
        const int nB = by ? cur[i - 4] : (top ? top[i + 12] : -1);
        return sp_nc(nA, nB);
    }
    if (i < 18) return -1;
    const int k = (i - 18) & 3, bx = k & 1, by = k >> 1;
    const int nA = bx ? cur[i - 1] : (left ? left[i + 1] : -1);
    const int nB = by ? cur[i - 2] : (top ? top[i + 2] : -1);
    return sp_nc(nA, nB);
}

/* luma4x4BlkIdx -> raster index */
static int sp_blk_raster(int blk)
{
    const int q8 = blk >> 2, q4 = blk & 3;
    return 4 * ((q8 >> 1) * 2 + (q4 >> 1)) + (q8 & 1) * 2 + (q4 & 1);
}

/* the residual of one MB (7.3.5.3) in piece order; 0 or -1 */
static int sp_residual(rd_t *r, int cbp, or_splice_mb *mb, const uint8_t *left, const uint8_t *top)
{
    for (int blk = 0; blk < 16; ++blk) {
        if (!(cbp & (1 << (blk >> 2)))) continue;
        const int i = sp_blk_raster(blk);
        if (sp_block(r, sp_piece_nc(i, mb->tc, left, top), 16, &mb->tc[i], &mb->t1[i],
                     &mb->boff[i], &mb->blen[i]))
            return -1;
    }
    if (cbp >> 4) {
        for (int i = 16; i < 18; ++i)
            if (sp_block(r, -1, 4, &mb->tc[i], &mb->t1[i], &mb->boff[i], &mb->blen[i])) return -1;
        if ((cbp >> 4) == 2)
            for (int i = 18; i < 26; ++i)
                if (sp_block(r, sp_piece_nc(i, mb->tc, left, top), 15, &mb->tc[i], &mb->t1[i],
                             &mb->boff[i], &mb->blen[i]))
                    return -1;
    }
    return 0;
}

static int sp_cbp_of_code(uint32_t code)
{
    for (int cbp = 0; cbp < 48; ++cbp)
        if ((uint32_t)or_cbp_code(cbp) == code) return cbp;
    return -1;
}

/* ------------------------------------------------------------------------ */
/* partitions and 4x4-block motion (7.3.5.1-2, Tables 7-13 / 7-17, 6.4.11.7, */
/* 8.4.1.3)                                                                   */
/* ------------------------------------------------------------------------ */
typedef struct {
    int bx, by, bw, bh;          /* 4x4-block units inside the MB */
    int mb_part;                 /* mbPartIdx (8x8 index for P_8x8) */
} sp_part;

/* the (sub-)partitions of an MB in decoding order */
static int sp_partitions(int part, int sub, sp_part *o)
{
    int n = 0;
    if (part == 0) {
        o[n++] = (sp_part){0, 0, 4, 4, 0};
    } else if (part == 1) {                                       /* 16x8 */
        o[n++] = (sp_part){0, 0, 4, 2, 0};
        o[n++] = (sp_part){0, 2, 4, 2, 1};
    } else if (part == 2) {                                       /* 8x16 */
        o[n++] = (sp_part){0, 0, 2, 4, 0};
        o[n++] = (sp_part){2, 0, 2, 4, 1};
    } else {
        for (int i = 0; i < 4; ++i) {
            const int sx = (i & 1) * 2, sy = (i >> 1) * 2, st = (sub >> (2 * i)) & 3;
            if (st == 0) {
                o[n++] = (sp_part){sx, sy, 2, 2, i};
            } else if (st == 1) {                                 /* 8x4 */
                o[n++] = (sp_part){sx, sy, 2, 1, i};
                o[n++] = (sp_part){sx, sy + 1, 2, 1, i};
            } else if (st == 2) {                                 /* 4x8 */
                o[n++] = (sp_part){sx, sy, 1, 2, i};
                o[n++] = (sp_part){sx + 1, sy, 1, 2, i};
            } else {
                for (int k = 0; k < 4; ++k) o[n++] = (sp_part){sx + (k & 1), sy + (k >> 1), 1, 1, i};
            }
        }
    }
    return n;
}

/* motion per 4x4 block of a picture of W MBs across; sid (NULL: one slice)
 * the slice of each MB, cur the current one -- an MB of another slice is
 * unavailable (6.4.x) */
typedef struct {
    int W;
    or_mvi *f;
    const int *sid;
    int cur;
} sp_field;

static or_mvi *sp_at(const sp_field *F, int x, int y, int bx, int by)
{
    return &F->f[(size_t)(4 * y + by) * 4 * (size_t)F->W + 4 * (size_t)x + (size_t)bx];
}

/* the block at (cx, cy) relative to MB (x, y) (cx, cy in -1..4): outside
 * the MB the neighbour MB's block, inside it only once decoded (bit
 * 4 cy + cx of done); unavailable: ref -1, mv 0 */
static or_mvi sp_nb(const sp_field *F, int x, int y, int cx, int cy, unsigned done)
{
    const or_mvi none = {0, 0, -1, 0};
    if (cy >= 0 && cx >= 4) return none;                          /* right: later in order */
    if (cy >= 0 && cx >= 0) return (done >> (4 * cy + cx)) & 1u ? *sp_at(F, x, y, cx, cy) : none;
    const int nx = x + (cx < 0 ? -1 : (cx >= 4 ? 1 : 0)), ny = y + (cy < 0 ? -1 : 0);
    if (nx < 0 || ny < 0 || nx >= F->W) return none;
    if (F->sid && F->sid[(size_t)ny * F->W + nx] != F->cur) return none;
    return *sp_at(F, nx, ny, (cx + 4) & 3, (cy + 4) & 3);
}

/* neighbours of a whole-MB partition: A, B, C (D when C is unavailable) */
static void sp_nb16(const sp_field *F, int x, int y, or_mvi *A, or_mvi *B, or_mvi *C, or_mvi *Cr,
                    or_mvi *D)
{
    *A = sp_nb(F, x, y, -1, 0, 0);
    *B = sp_nb(F, x, y, 0, -1, 0);
    *Cr = sp_nb(F, x, y, 4, -1, 0);
    *D = sp_nb(F, x, y, -1, -1, 0);
    *C = Cr->avail ? *Cr : *D;
}

/* 8.4.1.3 for (sub-)partition p of an MB partitioned `part` */
static void sp_mvp(const sp_field *F, int x, int y, unsigned done, int part, const sp_part *p, int ref,
                   int *px, int *py)
{
    const or_mvi A = sp_nb(F, x, y, p->bx - 1, p->by, done);
    const or_mvi B = sp_nb(F, x, y, p->bx, p->by - 1, done);
    or_mvi C = sp_nb(F, x, y, p->bx + p->bw, p->by - 1, done);
    if (!C.avail) C = sp_nb(F, x, y, p->bx - 1, p->by - 1, done);
    const or_mvi *d = NULL;
    if (part == 1) d = p->mb_part == 0 ? &B : &A;                  /* 16x8 */
    if (part == 2) d = p->mb_part == 0 ? &A : &C;                  /* 8x16 */
    if (d && d->avail && d->ref == ref) {
        *px = d->mx;
        *py = d->my;
        return;
    }
    or_spec_predict(&A, &B, &C, ref, px, py);
}

static void sp_fill(const sp_field *F, int x, int y, const sp_part *p, or_mvi v, unsigned *done)
{
    for (int j = 0; j < p->bh; ++j)
        for (int i = 0; i < p->bw; ++i) {
            *sp_at(F, x, y, p->bx + i, p->by + j) = v;
            *done |= 1u << (4 * (p->by + j) + p->bx + i);
        }
}

/* coded_block_pattern of an Intra_4x4 MB (Table 9-4, ChromaArrayType 1) */
static const uint8_t SP_CBP_INTRA[48] = {47, 31, 15, 0,  23, 27, 29, 30, 7,  11, 13, 14, 39, 43, 45, 46,
                                         16, 3,  5,  10, 12, 19, 21, 26, 28, 35, 37, 42, 44, 1,  2,  4,
                                         8,  17, 18, 20, 24, 6,  9,  22, 25, 32, 33, 34, 36, 40, 38, 41};

/* the NAL units of a splice buffer: Annex-B units (00 00 01 / 00 00 00 01
 * start codes), or the whole buffer as one NAL when it starts with none;
 * trailing zero bytes of a unit belong to no unit (7.4.1.2) */
static int sp_units(const uint8_t *p, size_t n, size_t *ub, size_t *ue, int cap)
{
    if (!(n >= 3 && !p[0] && !p[1] && (p[2] == 1 || (n >= 4 && !p[2] && p[3] == 1)))) {
        ub[0] = 0;
        ue[0] = n;
        return 1;
    }
    int k = 0;
    size_t i = 0;
    while (i + 3 <= n) {
        if (!p[i] && !p[i + 1] && p[i + 2] == 1) {
            if (k > 0) {
                size_t e = i;
                while (e > ub[k - 1] && !p[e - 1]) --e;
                ue[k - 1] = e;
            }
            if (k == cap) return -1;
            ub[k++] = i + 3;
            i += 3;
        } else {
            ++i;
        }
    }
    if (k > 0) {
        size_t e = n;
        while (e > ub[k - 1] && !p[e - 1]) --e;
        ue[k - 1] = e;
    }
    return k;
}

/* index of the last 1 bit of an RBSP (its rbsp_stop_one_bit), or -1 */
static long sp_stop_bit(const uint8_t *d, size_t nb)
{
    for (size_t i = nb; i-- > 0;)
        if (d[i]) return (long)(8 * i + 7 - (size_t)__builtin_ctz(d[i]));
    return -1;
}

/* availability of neighbour MB (x + dx, y + dy) of rect MB (x, y): in the
 * external picture (inside the rect and the same slice) and in the composed
 * one (inside the composed picture); 1 when they agree */
static int sp_same_avail(const or_cfg *c, const or_splice *sp, const int *sid, int x, int y, int dx, int dy)
{
    const int nx = x + dx, ny = y + dy;
    const int ext = nx >= 0 && ny >= 0 && nx < sp->w && sid[(size_t)ny * sp->w + nx] == sid[(size_t)y * sp->w + x];
    const int X = sp->x0 + nx, Y = sp->y0 + ny;
    const int comp = X >= 0 && Y >= 0 && X < c->w / 16;
    return ext == comp;
}

/* an intra MB's prediction reads the same neighbours in both pictures
 * (splice_oracle.h): modes = its Intra4x4PredModes (raster; I_4x4), or the
 * I_16x16 luma mode in modes[0]; cm = intra_chroma_pred_mode */
static int sp_intra_ok(const or_cfg *c, const or_splice *sp, const int *sid, int x, int y, int type,
                       const int *modes, int cm)
{
    int a = 0, b = 0, d = 0, cc = 0;
    if (cm == 0) a = b = 1;                                       /* chroma DC, horizontal, vertical, plane */
    else if (cm == 1) a = 1;
    else if (cm == 2) b = 1;
    else a = b = d = 1;
    if (type == 1) {
        a = b = 1;                                                /* mode prediction (8.3.1.1) */
        if (modes[0] == 4 || modes[0] == 5 || modes[0] == 6) d = 1;
        if (modes[3] == 3 || modes[3] == 7) cc = 1;
    } else {
        const int lm = modes[0];                                  /* 8.3.3: vertical, horizontal, DC, plane */
        if (lm == 0) b = 1;
        else if (lm == 1) a = 1;
        else if (lm == 2) a = b = 1;
        else a = b = d = 1;
    }
    return (!a || sp_same_avail(c, sp, sid, x, y, -1, 0)) && (!b || sp_same_avail(c, sp, sid, x, y, 0, -1)) &&
           (!d || sp_same_avail(c, sp, sid, x, y, -1, -1)) && (!cc || sp_same_avail(c, sp, sid, x, y, 1, -1));
}

/* P_Skip motion (8.4.1.1) from the availability of A and B (slices) */
static void sp_pskip(const or_mvi *A, const or_mvi *B, const or_mvi *C, int *px, int *py)
{
    if (!A->avail || !B->avail || (A->ref == 0 && A->mx == 0 && A->my == 0) ||
        (B->ref == 0 && B->mx == 0 && B->my == 0)) {
        *px = 0;
        *py = 0;
        return;
    }
    or_spec_predict(A, B, C, 0, px, py);
}

/* the MB the last parse refused with OR_SPLICE_ERR_MBTYPE: its index in the
 * external picture | its (P-slice) mb_type << 16, or -1 */
static __thread int sp_refused = -1;
int or_splice_refused(void) { return sp_refused; }

int or_splice_parse(const or_cfg *c, const or_splice *sp, or_splice_mb *mbs, uint8_t *rbsp,
                    size_t *rbsp_n)
{
    enum { MAXU = 1024 };
    size_t ub[MAXU], ue[MAXU];
    *rbsp_n = 0;
    sp_refused = -1;
    const int nu = sp_units(sp->nal, sp->n, ub, ue, MAXU);
    if (nu <= 0) return OR_SPLICE_ERR_NAL;
    const int W = sp->w, H = sp->h, nmb = W * H;
    memset(mbs, 0, sizeof(*mbs) * (size_t)nmb);
    int *sid = (int *)malloc(sizeof(int) * (size_t)nmb);
    int8_t(*im)[16] = malloc((size_t)nmb * 16);                   /* Intra4x4PredMode, -1: not I_4x4 */
    for (int k = 0; k < nmb; ++k) sid[k] = -1;
    sp_field F = {W, (or_mvi *)calloc((size_t)nmb * 16, sizeof(or_mvi)), sid, 0};
    int err = OR_SPLICE_OK, m = 0, qp_c = 26;
    size_t rb0 = 0;                                               /* this slice's RBSP in rbsp[] */
    for (int u = 0; u < nu && !err; ++u) {
        const uint8_t *p = sp->nal + ub[u];
        const size_t n = ue[u] - ub[u];
        const int nut = p[0] & 31;
        if (n < 2 || (p[0] & 0x80) || (nut != 1 && nut != 5)) {  /* non-IDR or IDR slice */
            err = OR_SPLICE_ERR_NAL;
            break;
        }
        const int ref_idc = (p[0] >> 5) & 3, idr = nut == 5;
        const size_t rn = sp_unescape(rbsp + rb0, p + 1, n - 1);
        /* bit positions are kept relative to the whole rbsp[] (all slices) */
        rd_t r = {rbsp, (rb0 + rn) * 8, rb0 * 8, 0};
        const long stop = sp_stop_bit(rbsp + rb0, rn);
        const size_t end = stop < 0 ? 0 : rb0 * 8 + (size_t)stop;
        rb0 += rn;
        *rbsp_n = rb0;
        /* slice header (7.3.3) with the composed stream's SPS / PPS fields */
        const uint32_t first = rd_ue(&r);
        if (first != (uint32_t)m) {                               /* slices in order, no gap */
            err = OR_SPLICE_ERR_HEADER;
            break;
        }
        const uint32_t st = rd_ue(&r);
        const int islice = st == 2 || st == 7;
        if ((st != 0 && st != 5 && !islice) || (idr && !islice) || rd_ue(&r) != 0) {
            err = OR_SPLICE_ERR_HEADER;                           /* P / I, pic_parameter_set_id 0 */
            break;
        }
        rd_u(&r, c->log2_mfn);                                    /* frame_num */
        if (idr) rd_ue(&r);                                       /* idr_pic_id */
        if (c->poc_type == 0) rd_u(&r, c->log2_poc);              /* pic_order_cnt_lsb */
        int nrefs = c->num_ref_default_m1 + 1;
        if (!islice && rd_u(&r, 1)) {                             /* num_ref_idx_active_override */
            const uint32_t k = rd_ue(&r);
            if (k > 31) {
                err = OR_SPLICE_ERR_HEADER;
                break;
            }
            nrefs = (int)k + 1;
        }
        if (!islice && rd_u(&r, 1)) {                             /* ref_pic_list_modification */
            /* only the composer's own list (h264_writer.c:455-539): op k puts
             * long_term_pic_num k at index k -- the composed list itself */
            for (int k = 0;; ++k) {
                const uint32_t idc = rd_ue(&r);
                if (r.bad || k > 32) {
                    err = OR_SPLICE_ERR_SYNTAX;
                    break;
                }
                if (idc == 3) break;
                if (idc != 2 || rd_ue(&r) != (uint32_t)k) {
                    err = OR_SPLICE_ERR_HEADER;
                    break;
                }
            }
            if (err) break;
        }
        if (ref_idc && idr) {
            rd_u(&r, 2);                                          /* no_output_of_prior_pics, long_term_reference */
        } else if (ref_idc && rd_u(&r, 1)) {                      /* adaptive_ref_pic_marking */
            for (int k = 0;; ++k) {
                const uint32_t op = rd_ue(&r);
                if (r.bad || k > 64 || op > 6) {
                    err = OR_SPLICE_ERR_SYNTAX;
                    break;
                }
                if (op == 0) break;
                if (op == 1 || op == 3) rd_ue(&r);
                if (op == 2) rd_ue(&r);
                if (op == 3 || op == 6) rd_ue(&r);
                if (op == 4) rd_ue(&r);
            }
            if (err) break;
        }
        int qp = 26 + rd_se(&r);                                  /* pic_init_qp 26 + slice_qp_delta */
        if (qp < 0 || qp > 51) {
            err = OR_SPLICE_ERR_HEADER;
            break;
        }
        if (c->deblock && rd_ue(&r) != 1) {
            err = OR_SPLICE_ERR_HEADER;
            break;
        }
        if (r.bad) {
            err = OR_SPLICE_ERR_SYNTAX;
            break;
        }
        F.cur = u;
        /* slice data (7.3.4): MBs until the stop bit (more_rbsp_data) */
        int first_mb = 1;
        while (!err) {
            if (r.p >= end && !first_mb) break;
            first_mb = 0;
            const uint32_t run = islice ? 0u : rd_ue(&r);         /* I slices: no mb_skip_run */
            if (r.bad || run > (uint32_t)(nmb - m)) {
                err = OR_SPLICE_ERR_SYNTAX;
                break;
            }
            for (uint32_t k = 0; k < run; ++k, ++m) {             /* P_Skip (8.4.1.1) */
                const int x = m % W, y = m / W;
                sid[m] = u;
                or_mvi A, B, C, Cr, D;
                sp_nb16(&F, x, y, &A, &B, &C, &Cr, &D);
                int px, py;
                sp_pskip(&A, &B, &C, &px, &py);
                or_splice_mb *mb = &mbs[m];
                mb->ref = 0;
                mb->mx = px;
                mb->my = py;
                mb->qp = qp;
                mb->skip = 1;
                memset(im[m], -1, 16);
                for (int b = 0; b < 16; ++b) {
                    mb->bmx[b] = px;
                    mb->bmy[b] = py;
                    *sp_at(&F, x, y, b & 3, b >> 2) = (or_mvi){px, py, 0, 1};
                }
            }
            if (r.p >= end) {                                     /* skipped MBs end the slice; */
                if (!run) err = OR_SPLICE_ERR_SYNTAX;             /* a run of 0 precedes an MB  */
                break;
            }
            if (m == nmb) {
                err = OR_SPLICE_ERR_SYNTAX;
                break;
            }
            const int x = m % W, y = m / W;
            sid[m] = u;
            or_splice_mb *mb = &mbs[m];
            const uint8_t *L = x && sid[m - 1] == u ? mbs[m - 1].tc : NULL;
            const uint8_t *T = y && sid[m - W] == u ? mbs[m - W].tc : NULL;
            /* mb_type (Table 7-13, 7-11; an I slice's k is the P slice's 5 + k) */
            const uint32_t mbt = rd_ue(&r) + (islice ? 5u : 0u);
            if (r.bad || mbt > 30 || (islice && mbt < 5)) {
                err = OR_SPLICE_ERR_SYNTAX;
                break;
            }
            memset(im[m], -1, 16);
            if (mbt >= 5) {
                /* intra in a P slice (7.3.5.1): I_4x4, I_16x16, I_PCM */
                const int it = (int)mbt - 5;
                mb->intra = it == 0 ? 1 : (it == 25 ? 3 : 2);
                mb->mbt = (int)mbt;
                mb->ref = -1;
                for (int b = 0; b < 16; ++b) {
                    mb->bref[b] = -1;
                    *sp_at(&F, x, y, b & 3, b >> 2) = (or_mvi){0, 0, -1, 1};
                }
                if (mb->intra == 3) {                             /* I_PCM (7.3.5) */
                    while (r.p & 7)
                        if (rd_u(&r, 1)) err = OR_SPLICE_ERR_SYNTAX;  /* pcm_alignment_zero_bit */
                    mb->pcm = (uint32_t)(r.p >> 3);
                    r.p += 384 * 8;
                    if (r.p > r.nbits) r.bad = 1;
                    for (int i = 0; i < OR_SPLICE_PIECES; ++i) mb->tc[i] = 16;   /* nC: 16 (9.2.1) */
                    mb->qp = qp;
                    if (r.bad) err = OR_SPLICE_ERR_SYNTAX;
                    ++m;
                    continue;
                }
                int modes[16], cm;
                mb->poff = (uint32_t)r.p;
                if (mb->intra == 1) {
                    /* Intra4x4PredMode per block (8.3.1.1), luma4x4BlkIdx order */
                    for (int blk = 0; blk < 16; ++blk) {
                        const int ri = sp_blk_raster(blk), bx = ri & 3, by = ri >> 2;
                        int mA = -2, mB = -2;                     /* -2 unavailable, -1 not I_4x4 */
                        if (bx) mA = im[m][ri - 1];
                        else if (x && sid[m - 1] == u) mA = im[m - 1][ri + 3];
                        if (by) mB = im[m][ri - 4];
                        else if (y && sid[m - W] == u) mB = im[m - W][ri + 12];
                        const int pm = (mA == -2 || mB == -2) ? 2 : ((mA < 0 ? 2 : mA) < (mB < 0 ? 2 : mB)
                                                                         ? (mA < 0 ? 2 : mA) : (mB < 0 ? 2 : mB));
                        int md = pm;
                        if (!rd_u(&r, 1)) {
                            const int rem = (int)rd_u(&r, 3);
                            md = rem < pm ? rem : rem + 1;
                        }
                        im[m][ri] = (int8_t)md;
                    }
                    for (int k = 0; k < 16; ++k) modes[k] = im[m][k];
                } else {
                    modes[0] = (it - 1) & 3;
                }
                cm = (int)rd_ue(&r);                              /* intra_chroma_pred_mode */
                mb->plen = (uint32_t)r.p - mb->poff;
                if (r.bad || cm > 3) {
                    err = OR_SPLICE_ERR_SYNTAX;
                    break;
                }
                if (!sp_intra_ok(c, sp, sid, x, y, mb->intra, modes, cm)) {
                    err = OR_SPLICE_ERR_MBTYPE;
                    sp_refused = m | (int)mbt << 16;
                    break;
                }
                int cbp;
                if (mb->intra == 1) {
                    const uint32_t code = rd_ue(&r);
                    if (r.bad || code > 47) {
                        err = OR_SPLICE_ERR_SYNTAX;
                        break;
                    }
                    mb->cbp_code = (int)code;
                    cbp = SP_CBP_INTRA[code];
                } else {
                    cbp = ((it - 1) >= 12 ? 15 : 0) | (((it - 1) >> 2) % 3) << 4;
                }
                mb->cbp = cbp;
                if (cbp || mb->intra == 2) {
                    const int dq = rd_se(&r);                     /* mb_qp_delta */
                    if (dq < -26 || dq > 25) {
                        err = OR_SPLICE_ERR_SYNTAX;
                        break;
                    }
                    qp = (qp + dq + 52) % 52;
                    int d = qp - qp_c;
                    if (d < -26) d += 52;
                    if (d > 25) d -= 52;
                    mb->qpd = d;
                    mb->hasqpd = 1;
                    qp_c = qp;
                    int e = 0;
                    if (mb->intra == 2) {                         /* Intra16x16DCLevel: nC of block 0 */
                        e = sp_block(&r, sp_piece_nc(0, mb->tc, L, T), 16, &mb->tc[26], &mb->t1[26], &mb->boff[26],
                                     &mb->blen[26]);
                        if (!e && (cbp & 15))                     /* Intra16x16ACLevel */
                            for (int blk = 0; blk < 16 && !e; ++blk) {
                                const int ri = sp_blk_raster(blk);
                                e = sp_block(&r, sp_piece_nc(ri, mb->tc, L, T), 15, &mb->tc[ri], &mb->t1[ri],
                                             &mb->boff[ri], &mb->blen[ri]);
                            }
                        if (!e && (cbp >> 4)) {
                            for (int i = 16; i < 18 && !e; ++i)
                                e = sp_block(&r, -1, 4, &mb->tc[i], &mb->t1[i], &mb->boff[i], &mb->blen[i]);
                            if (!e && (cbp >> 4) == 2)
                                for (int i = 18; i < 26 && !e; ++i)
                                    e = sp_block(&r, sp_piece_nc(i, mb->tc, L, T), 15, &mb->tc[i], &mb->t1[i],
                                                 &mb->boff[i], &mb->blen[i]);
                        }
                    } else {
                        e = sp_residual(&r, cbp, mb, L, T);
                    }
                    if (e) {
                        err = OR_SPLICE_ERR_SYNTAX;
                        break;
                    }
                }
                mb->qp = qp;
                if (r.bad) err = OR_SPLICE_ERR_SYNTAX;
                ++m;
                continue;
            }
            const int part = mbt == 4 ? 3 : (int)mbt;
            int sub = 0;
            if (part == 3)                                        /* sub_mb_pred (7.3.5.2) */
                for (int i = 0; i < 4; ++i) {
                    const uint32_t st2 = rd_ue(&r);
                    if (st2 > 3) err = OR_SPLICE_ERR_SYNTAX;
                    sub |= (int)(st2 & 3u) << (2 * i);
                }
            const int nref = part == 0 ? 1 : (part == 3 ? 4 : 2);
            int refs[4] = {0, 0, 0, 0};
            if (mbt != 4)
                for (int i = 0; i < nref; ++i) {                  /* ref_idx_l0: te() */
                    if (nrefs == 2) refs[i] = 1 - (int)rd_u(&r, 1);
                    else if (nrefs > 2) refs[i] = (int)rd_ue(&r);
                    if (refs[i] >= nrefs) err = OR_SPLICE_ERR_SYNTAX;
                }
            sp_part ps[16];
            const int np = sp_partitions(part, sub, ps);
            unsigned done = 0;
            for (int k = 0; k < np && !err; ++k) {               /* mvd_l0 per (sub-)partition */
                const int ref = refs[ps[k].mb_part];
                const int dx = rd_se(&r), dy = rd_se(&r);
                int px, py;
                sp_mvp(&F, x, y, done, part, &ps[k], ref, &px, &py);
                const long long mx = (long long)px + dx, my = (long long)py + dy;
                if (r.bad || mx < -OR_SPLICE_MAX_MV || mx > OR_SPLICE_MAX_MV || my < -OR_SPLICE_MAX_MV ||
                    my > OR_SPLICE_MAX_MV) {
                    err = OR_SPLICE_ERR_SYNTAX;
                    break;
                }
                sp_fill(&F, x, y, &ps[k], (or_mvi){(int)mx, (int)my, ref, 1}, &done);
            }
            const int cbp = sp_cbp_of_code(rd_ue(&r));
            if (err || r.bad || cbp < 0) {
                err = OR_SPLICE_ERR_SYNTAX;
                break;
            }
            for (int b = 0; b < 16; ++b) {
                const or_mvi v = *sp_at(&F, x, y, b & 3, b >> 2);
                mb->bref[b] = v.ref;
                mb->bmx[b] = v.mx;
                mb->bmy[b] = v.my;
            }
            mb->part = part;
            mb->sub = sub;
            mb->ref = mb->bref[0];
            mb->mx = mb->bmx[0];
            mb->my = mb->bmy[0];
            mb->cbp = cbp;
            if (cbp) {
                const int dq = rd_se(&r);                         /* mb_qp_delta */
                if (dq < -26 || dq > 25) {
                    err = OR_SPLICE_ERR_SYNTAX;
                    break;
                }
                qp = (qp + dq + 52) % 52;
                int d = qp - qp_c;                                /* composed chain from 26 */
                if (d < -26) d += 52;
                if (d > 25) d -= 52;
                mb->qpd = d;
                mb->hasqpd = 1;
                qp_c = qp;
                if (sp_residual(&r, cbp, mb, L, T)) {
                    err = OR_SPLICE_ERR_SYNTAX;
                    break;
                }
            }
            mb->qp = qp;
            ++m;
        }
        if (err) break;
        /* rbsp_slice_trailing_bits: the stop bit, alignment zeros (zero bytes
         * after it are tolerated: trailing_zero_8bits of a byte stream) */
        if (r.p != end || rd_u(&r, 1) != 1) {
            err = OR_SPLICE_ERR_SYNTAX;
            break;
        }
        while (r.p & 7)
            if (rd_u(&r, 1)) err = OR_SPLICE_ERR_SYNTAX;
        while (!err && r.p < r.nbits)
            if (rd_u(&r, 8)) err = OR_SPLICE_ERR_SYNTAX;
        if (r.bad) err = OR_SPLICE_ERR_SYNTAX;
    }
    if (!err && m != nmb) err = OR_SPLICE_ERR_SYNTAX;             /* the slices cover the picture */
    free(F.f);
    free(sid);
    free(im);
    return err;
}

/* ------------------------------------------------------------------------ */
/* composed scroll NAL                                                        */
/* ------------------------------------------------------------------------ */
static void sp_copy_bits(or_bits *b, const uint8_t *src, uint32_t off, uint32_t len)
{
    rd_t r = {src, (size_t)off + len, off, 0};
    while (len) {
        const int k = len > 16 ? 16 : (int)len;
        or_put(b, rd_u(&r, k), k);
        len -= (uint32_t)k;
    }
}

static void sp_piece(or_bits *b, const or_splice_mb *mb, int i, int nC, const uint8_t *rbsp)
{
    uint32_t bits;
    const int len = or_ct_code(mb->tc[i], mb->t1[i], nC, &bits);
    or_put(b, bits, len);
    sp_copy_bits(b, rbsp, mb->boff[i], mb->blen[i]);
}

/* the scroll NAL with the MBs of rect [x0, x0 + w) x [y0, y0 + h) taken
 * from mbs[] (their piece bodies in erb, erb_n bytes); shared by the splice
 * and the hinted dynamic rect (or_hint_dyn_scroll_nal) */
static size_t sp_compose(uint8_t *dst, size_t cap, or_cfg *c, int off, const or_hint_rect *r, int n,
                         int mode, int x0, int y0, int w, int h, const or_splice_mb *mbs,
                         const uint8_t *erb, size_t erb_n, int *err)
{
    *err = 0;
    const int mbw = c->w / 16, mbh = c->h / 16, nrefs = 2 + c->nwp;
    const int has = w > 0 && h > 0;
    const struct { int x0, y0, w, h; } rect = {x0, y0, w, h}, *sp = &rect;
    int a_end, ra, mva, rb, mvb;
    or_scroll_regions(c, off, &a_end, &ra, &mva, &rb, &mvb);
    size_t rcap = 64 + (size_t)mbw * mbh * 24 + (has ? erb_n * 2 + (size_t)w * h * 64 : 0);
    uint8_t *rbsp = (uint8_t *)malloc(rcap);
    sp_field F = {mbw, (or_mvi *)calloc((size_t)mbw * mbh * 16, sizeof(or_mvi)), NULL, 0};
    uint8_t(*tabove)[OR_SPLICE_PIECES] = calloc((size_t)mbw, OR_SPLICE_PIECES);
    uint8_t(*tcur)[OR_SPLICE_PIECES] = calloc((size_t)mbw, OR_SPLICE_PIECES);
    or_bits b;
    or_bits_init(&b, rbsp, rcap);
    or_scroll_header(&b, c);
    int run = 0, bad_hint = 0, bad_ref = 0;
    for (int y = 0; y < mbh; ++y) {
        for (int x = 0; x < mbw; ++x) {
            const or_splice_mb *mb = NULL;
            if (has && x >= sp->x0 && x < sp->x0 + sp->w && y >= sp->y0 && y < sp->y0 + sp->h)
                mb = &mbs[(size_t)(y - sp->y0) * sp->w + (x - sp->x0)];
            if (mb && mb->intra) {
                /* an intra MB: mb_type, its prediction syntax (and I_4x4's cbp
                 * codeNum) verbatim, the residual re-contexted; I_PCM
                 * realigned.  Available with refIdx -1, mv 0 for the motion
                 * prediction of the MBs after it (8.4.1.3.1) */
                or_ue(&b, (uint32_t)run);                         /* mb_skip_run */
                run = 0;
                or_ue(&b, (uint32_t)mb->mbt);
                memset(tcur[x], 0, OR_SPLICE_PIECES);
                if (mb->intra == 3) {
                    while (b.nbits & 7) or_put(&b, 0, 1);         /* pcm_alignment_zero_bit */
                    sp_copy_bits(&b, erb, 8u * mb->pcm, 384u * 8u);
                    memset(tcur[x], 16, OR_SPLICE_PIECES);
                } else {
                    sp_copy_bits(&b, erb, mb->poff, mb->plen);
                    if (mb->intra == 1) or_ue(&b, (uint32_t)mb->cbp_code);
                    memcpy(tcur[x], mb->tc, OR_SPLICE_PIECES);
                    const uint8_t *L = x ? tcur[x - 1] : NULL, *T = y ? tabove[x] : NULL;
                    const int cbp = mb->cbp;
                    if (mb->hasqpd) {
                        or_se(&b, mb->qpd);
                        if (mb->intra == 2) sp_piece(&b, mb, 26, sp_piece_nc(0, tcur[x], L, T), erb);
                        for (int blk = 0; blk < 16; ++blk)
                            if (cbp & (1 << (blk >> 2))) {
                                const int i = sp_blk_raster(blk);
                                sp_piece(&b, mb, i, sp_piece_nc(i, tcur[x], L, T), erb);
                            }
                        if (cbp >> 4) {
                            sp_piece(&b, mb, 16, -1, erb);
                            sp_piece(&b, mb, 17, -1, erb);
                            if ((cbp >> 4) == 2)
                                for (int i = 18; i < 26; ++i) sp_piece(&b, mb, i, sp_piece_nc(i, tcur[x], L, T), erb);
                        }
                    }
                }
                for (int k = 0; k < 16; ++k) *sp_at(&F, x, y, k & 3, k >> 2) = (or_mvi){0, 0, -1, 1};
                continue;
            }
            int ref, mx, my, cbp = 0;
            const int part = mb ? mb->part : 0;
            if (mb) {
                ref = mb->ref;
                mx = mb->mx;
                my = mb->my;
                cbp = mb->cbp;
                for (int k = 0; k < (part ? 16 : 1); ++k)
                    if (!or_ref_valid(c, part ? mb->bref[k] : ref)) bad_ref = 1;
            } else {
                if (or_hint_motion(r, n, x, y, a_end, ra, mva, rb, mvb, &ref, &mx, &my) &&
                    !or_ref_valid(c, ref))
                    bad_hint = 1;
                mx *= 4;
                my *= 4;
            }
            int px = 0, py = 0, coded = 1;
            or_mvi A, B, C, Cr, D;
            sp_nb16(&F, x, y, &A, &B, &C, &Cr, &D);
            if (part) {
                coded = 1;                                        /* predicted per partition */
            } else if (mode != OR_HINT_EXACT) {
                int sx, sy;
                or_pskip_motion(x, y, &A, &B, &C, &sx, &sy);
                coded = mode == OR_HINT_SPEC || !(ref == 0 && mx == sx && my == sy && cbp == 0);
                or_spec_predict(&A, &B, &C, ref, &px, &py);
            } else {
                /* the reference's get_mv_prediction over the neighbour blocks:
                 * above[x - 1 .. x + 1] = D, B, C at a stand-in x = 1 of 3 */
                const or_mvi ab[3] = {D, B, Cr};
                or_predict(1, y, 3, ab, &A, ref, &px, &py);
            }
            memset(tcur[x], 0, OR_SPLICE_PIECES);
            if (coded) {
                or_ue(&b, (uint32_t)run);                         /* mb_skip_run */
                run = 0;
                if (part) {
                    sp_part ps[16];
                    const int np = sp_partitions(part, mb->sub, ps), nref = part == 3 ? 4 : 2;
                    or_ue(&b, (uint32_t)part);                    /* P_L0_L0_16x8 / 8x16, P_8x8 */
                    if (part == 3)
                        for (int i = 0; i < 4; ++i) or_ue(&b, (uint32_t)((mb->sub >> (2 * i)) & 3));
                    for (int i = 0; i < nref; ++i) {              /* ref_idx_l0 per mbPartIdx */
                        int k = 0;
                        while (ps[k].mb_part != i) ++k;
                        const int rf = mb->bref[4 * ps[k].by + ps[k].bx];
                        if (nrefs == 2) or_put(&b, (uint32_t)(1 - (rf & 1)), 1);
                        else or_ue(&b, (uint32_t)rf);
                    }
                    unsigned done = 0;
                    for (int k = 0; k < np; ++k) {                /* mvd per (sub-)partition */
                        const int q = 4 * ps[k].by + ps[k].bx;
                        const or_mvi v = {mb->bmx[q], mb->bmy[q], mb->bref[q], 1};
                        int qx, qy;
                        sp_mvp(&F, x, y, done, part, &ps[k], v.ref, &qx, &qy);
                        or_se(&b, v.mx - qx);
                        or_se(&b, v.my - qy);
                        sp_fill(&F, x, y, &ps[k], v, &done);
                    }
                } else {
                    or_ue(&b, 0);                                 /* P_L0_16x16 */
                    if (nrefs == 2) or_put(&b, (uint32_t)(1 - (ref & 1)), 1);
                    else if (nrefs > 2) or_ue(&b, (uint32_t)ref);
                    or_se(&b, mx - px);
                    or_se(&b, my - py);
                }
                or_ue(&b, (uint32_t)or_cbp_code(cbp));
                if (cbp) {
                    or_se(&b, mb->qpd);
                    memcpy(tcur[x], mb->tc, OR_SPLICE_PIECES);
                    const uint8_t *L = x ? tcur[x - 1] : NULL, *T = y ? tabove[x] : NULL;
                    for (int blk = 0; blk < 16; ++blk)
                        if (cbp & (1 << (blk >> 2))) {
                            const int i = sp_blk_raster(blk);
                            sp_piece(&b, mb, i, sp_piece_nc(i, tcur[x], L, T), erb);
                        }
                    if (cbp >> 4) {
                        sp_piece(&b, mb, 16, -1, erb);
                        sp_piece(&b, mb, 17, -1, erb);
                        if ((cbp >> 4) == 2)
                            for (int i = 18; i < 26; ++i)
                                sp_piece(&b, mb, i, sp_piece_nc(i, tcur[x], L, T), erb);
                    }
                }
            } else {
                run++;                                            /* P_Skip */
            }
            if (!part)
                for (int k = 0; k < 16; ++k) *sp_at(&F, x, y, k & 3, k >> 2) = (or_mvi){mx, my, ref, 1};
        }
        uint8_t(*tt)[OR_SPLICE_PIECES] = tabove;
        tabove = tcur;
        tcur = tt;
    }
    if (run > 0) or_ue(&b, (uint32_t)run);
    or_trailing(&b);
    size_t nb = 0;
    if (bad_ref) {
        *err = OR_SPLICE_ERR_REF;
    } else if (bad_hint) {
        *err = 0x101;
    } else {
        nb = or_nal(dst, cap, 0, 1, rbsp, or_bytes(&b));
        c->frame_num++;
    }
    free(rbsp);
    free(F.f);
    free(tabove);
    free(tcur);
    return nb;
}

size_t or_splice_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off, const or_hint_rect *r,
                            int n, int mode, const or_splice *sp, int *err)
{
    *err = 0;
    const int mbw = c->w / 16, mbh = c->h / 16;
    const int has = sp && sp->w > 0 && sp->h > 0;
    if (!has) return sp_compose(dst, cap, c, off, r, n, mode, 0, 0, 0, 0, NULL, NULL, 0, err);
    if (sp->x0 < 0 || sp->y0 < 0 || sp->x0 + sp->w > mbw || sp->y0 + sp->h > mbh) {
        *err = OR_SPLICE_ERR_HEADER;
        return 0;
    }
    or_splice_mb *mbs = (or_splice_mb *)malloc(sizeof(*mbs) * (size_t)sp->w * (size_t)sp->h);
    uint8_t *erb = (uint8_t *)malloc(sp->n + 8);
    size_t rn;
    const int e = or_splice_parse(c, sp, mbs, erb, &rn);
    size_t nb = 0;
    if (e)
        *err = e;
    else
        nb = sp_compose(dst, cap, c, off, r, n, mode, sp->x0, sp->y0, sp->w, sp->h, mbs, erb, sp->n, err);
    free(mbs);
    free(erb);
    return nb;
}

size_t or_compose_splice(uint8_t *dst, size_t cap, or_cfg *c, int off, int compose_mode,
                         const or_hint_rect *r, int n, int mode, const or_splice *sp, int *err)
{
    *err = 0;
    size_t nb = 0;
    if (or_needs_waypoint(c, off)) {                              /* src/composer.c:255-264 */
        nb += or_waypoint_nal(dst, cap, c, off);
        if (compose_mode == 1) return nb;
    }
    const size_t k = or_splice_scroll_nal(dst + nb, cap - nb, c, off, r, n, mode, sp, err);
    return k ? nb + k : 0;
}

/* ------------------------------------------------------------------------ */
/* the dynamic rect under UI hints (or_hint_dyn_scroll_nal)                   */
/* ------------------------------------------------------------------------ */
static const int HD_ZZ[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};

/* TrailingOnes of a block in scan order (9.2.1: up to 3 +-1 levels from the
 * last non-zero one down) */
static int hd_t1(const int *coef, int max)
{
    int t1 = 0;
    for (int i = max - 1; i >= 0 && t1 < 3; --i) {
        if (!coef[i]) continue;
        if (coef[i] != 1 && coef[i] != -1) break;
        t1++;
    }
    return t1;
}

/* a block's piece: TotalCoeff, TrailingOnes and its bits after coeff_token
 * appended to erb (nC does not change them: coded here at nC 0 / -1) */
static void hd_piece(or_bits *erb, or_splice_mb *mb, int i, const int *coef, int max)
{
    uint8_t tmp[128];
    or_bits tb;
    or_bits_init(&tb, tmp, sizeof(tmp));
    const int nC = max == 4 ? -1 : 0;
    const int tc = or_cavlc_block(&tb, coef, max, nC);
    const int t1 = hd_t1(coef, max);
    uint32_t tv;
    const int tl = or_ct_code(tc, t1, nC, &tv);
    mb->tc[i] = (uint8_t)tc;
    mb->t1[i] = (uint8_t)t1;
    mb->boff[i] = (uint32_t)erb->nbits;
    mb->blen[i] = (uint32_t)(tb.nbits - (size_t)tl);
    for (size_t p = (size_t)tl; p < tb.nbits;) {              /* copy the body bits */
        const int k = tb.nbits - p > 16 ? 16 : (int)(tb.nbits - p);
        uint32_t v = 0;
        for (int j = 0; j < k; ++j) v = v << 1 | ((tmp[(p + j) >> 3] >> (7 - ((p + j) & 7))) & 1u);
        or_put(erb, v, k);
        p += (size_t)k;
    }
}

/* the prediction sample of reference ref at (x, y) of plane 0 (luma,
 * full-pel displacement in pixels) or 1 / 2 (chroma, 1/8-pel 2-D bilinear,
 * 8.4.2.2.2), displacement (mvx, mvy) in luma pixels */
static int hd_pred(const or_cfg *c, const or_refs *R, int ref, int plane, int x, int y, int mvx, int mvy)
{
    if (plane == 0) return or_ref_sample(c, R, ref, 0, x + mvx, y + mvy);
    const int qx = 4 * mvx, qy = 4 * mvy, fx = qx & 7, fy = qy & 7;
    const int xi = x + (qx >> 3), yi = y + (qy >> 3);
    const int A = or_ref_sample(c, R, ref, plane, xi, yi), B = or_ref_sample(c, R, ref, plane, xi + 1, yi);
    const int C = or_ref_sample(c, R, ref, plane, xi, yi + 1), D = or_ref_sample(c, R, ref, plane, xi + 1, yi + 1);
    return ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6;
}

/* the record of dynamic MB (x, y) at motion (ref, mvx, mvy) px */
static void hd_mb(const or_cfg *c, const or_refs *R, const or_dyn_rect *rc, const uint8_t *src, int x,
                  int y, int ref, int mvx, int mvy, or_splice_mb *mb, or_bits *erb)
{
    const int lw = 16 * rc->w, cw = 8 * rc->w;
    const uint8_t *sy = src, *su = src + (size_t)lw * 16 * rc->h, *sv = su + (size_t)cw * 8 * rc->h;
    const int lx0 = 16 * (x - rc->x0), ly0 = 16 * (y - rc->y0);
    const int qp = or_dyn_qp(rc), qpc = or_qp_chroma(qp);
    int luma[16][16], cdc[2][4], cac[2][4][15];
    for (int r = 0; r < 16; ++r) {
        const int bx = 4 * (r % 4), by = 4 * (r / 4);
        int res[16], W[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                res[4 * i + j] = sy[(size_t)(ly0 + by + i) * lw + lx0 + bx + j] -
                                 hd_pred(c, R, ref, 0, 16 * x + bx + j, 16 * y + by + i, mvx, mvy);
        or_fwd4x4(res, W);
        for (int k = 0; k < 16; ++k) luma[r][k] = or_quant(W[HD_ZZ[k]], qp, HD_ZZ[k], 0);
    }
    const int cx0 = 8 * (x - rc->x0), cy0 = 8 * (y - rc->y0);
    for (int p = 0; p < 2; ++p) {
        const uint8_t *spl = p ? sv : su;
        int dc[4];
        for (int k = 0; k < 4; ++k) {
            const int bx = 4 * (k % 2), by = 4 * (k / 2);
            int res[16], W[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j)
                    res[4 * i + j] = spl[(size_t)(cy0 + by + i) * cw + cx0 + bx + j] -
                                     hd_pred(c, R, ref, 1 + p, 8 * x + bx + j, 8 * y + by + i, mvx, mvy);
            or_fwd4x4(res, W);
            dc[k] = W[0];
            for (int i = 1; i < 16; ++i) cac[p][k][i - 1] = or_quant(W[HD_ZZ[i]], qpc, HD_ZZ[i], 0);
        }
        cdc[p][0] = or_quant(dc[0] + dc[1] + dc[2] + dc[3], qpc, 0, 1);
        cdc[p][1] = or_quant(dc[0] - dc[1] + dc[2] - dc[3], qpc, 0, 1);
        cdc[p][2] = or_quant(dc[0] + dc[1] - dc[2] - dc[3], qpc, 0, 1);
        cdc[p][3] = or_quant(dc[0] - dc[1] - dc[2] + dc[3], qpc, 0, 1);
    }
    memset(mb, 0, sizeof(*mb));
    mb->ref = ref;
    mb->mx = 4 * mvx;
    mb->my = 4 * mvy;
    mb->qp = qp;
    int cbp_l = 0, dcn = 0, acn = 0;
    for (int r = 0; r < 16; ++r) {
        hd_piece(erb, mb, r, luma[r], 16);
        if (mb->tc[r]) cbp_l |= 1 << (2 * (r / 8) + (r % 4) / 2);
    }
    for (int p = 0; p < 2; ++p) {
        hd_piece(erb, mb, 16 + p, cdc[p], 4);
        dcn += mb->tc[16 + p];
        for (int k = 0; k < 4; ++k) {
            hd_piece(erb, mb, 18 + 4 * p + k, cac[p][k], 15);
            acn += mb->tc[18 + 4 * p + k];
        }
    }
    mb->cbp = cbp_l | (acn ? 2 : (dcn ? 1 : 0)) << 4;
}

size_t or_hint_dyn_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off, const or_hint_rect *r,
                              int n, int mode, const or_dyn_rect *rc, const uint8_t *src, const or_refs *R,
                              int *err)
{
    *err = 0;
    const int mbw = c->w / 16, mbh = c->h / 16;
    if (!rc || rc->w <= 0 || rc->h <= 0)
        return sp_compose(dst, cap, c, off, r, n, mode, 0, 0, 0, 0, NULL, NULL, 0, err);
    if (rc->x0 < 0 || rc->y0 < 0 || rc->x0 + rc->w > mbw || rc->y0 + rc->h > mbh) {
        *err = OR_SPLICE_ERR_HEADER;
        return 0;
    }
    int a_end, ra, mva, rb, mvb;
    or_scroll_regions(c, off, &a_end, &ra, &mva, &rb, &mvb);
    const size_t nmb = (size_t)rc->w * rc->h, ecap = nmb * OR_SPLICE_PIECES * 64 + 64;
    or_splice_mb *mbs = (or_splice_mb *)malloc(sizeof(*mbs) * nmb);
    uint8_t *erb = (uint8_t *)calloc(ecap, 1);
    or_bits eb;
    or_bits_init(&eb, erb, ecap);
    for (int y = rc->y0; y < rc->y0 + rc->h; ++y)
        for (int x = rc->x0; x < rc->x0 + rc->w; ++x) {
            int ref, mvx, mvy;
            or_hint_motion(r, n, x, y, a_end, ra, mva, rb, mvb, &ref, &mvx, &mvy);
            or_splice_mb *mb = &mbs[(size_t)(y - rc->y0) * rc->w + (x - rc->x0)];
            if (!or_ref_valid(c, ref)) {            /* an invalid hint reference: no residual */
                memset(mb, 0, sizeof(*mb));
                mb->ref = ref;
                mb->mx = 4 * mvx;
                mb->my = 4 * mvy;
                continue;
            }
            hd_mb(c, R, rc, src, x, y, ref, mvx, mvy, mb, &eb);
        }
    /* mb_qp_delta: the chain of the coded MBs (raster order) from the slice
     * QP 26 -- the first one carries QP - 26, the rest 0 */
    for (size_t i = 0, qp_c = 26; i < nmb; ++i) {
        or_splice_mb *mb = &mbs[i];
        if (!mb->cbp) continue;
        mb->qpd = mb->qp - (int)qp_c;
        mb->hasqpd = 1;
        qp_c = (size_t)mb->qp;
    }
    const size_t nb = sp_compose(dst, cap, c, off, r, n, mode, rc->x0, rc->y0, rc->w, rc->h, mbs, erb,
                                 or_bytes(&eb), err);
    free(mbs);
    free(erb);
    return nb;
}

size_t or_compose_hint_dyn(uint8_t *dst, size_t cap, or_cfg *c, int off, int compose_mode,
                           const or_hint_rect *r, int n, int mode, const or_dyn_rect *rc,
                           const uint8_t *src, const or_refs *R, int *err)
{
    *err = 0;
    size_t nb = 0;
    if (or_needs_waypoint(c, off)) {                              /* src/composer.c:255-264 */
        nb += or_waypoint_nal(dst, cap, c, off);
        if (compose_mode == 1) return nb;
    }
    const size_t k = or_hint_dyn_scroll_nal(dst + nb, cap - nb, c, off, r, n, mode, rc, src, R, err);
    return k ? nb + k : 0;
}

/* ------------------------------------------------------------------------ */
/* test-input generator                                                       */
/* ------------------------------------------------------------------------ */
static uint32_t sp_rng(uint32_t *s)
{
    uint32_t x = *s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return *s = x;
}

static int sp_level(uint32_t *s, const or_ext_params *p)
{
    const int sign = (sp_rng(s) & 1) ? -1 : 1;
    if ((int)(sp_rng(s) % 1000) < p->big_pm) return sign * (16 + (int)(sp_rng(s) % 2000));
    if (sp_rng(s) % 3 == 0) return sign * (2 + (int)(sp_rng(s) % 6));
    return sign;
}

static void sp_rand_block(uint32_t *s, const or_ext_params *p, int *coef, int maxc)
{
    memset(coef, 0, sizeof(int) * (size_t)maxc);
    const int k = (sp_rng(s) & 3) ? (int)(sp_rng(s) % 4) : (int)(sp_rng(s) % (unsigned)(maxc + 1));
    for (int i = 0; i < k; ++i) coef[sp_rng(s) % (unsigned)maxc] = sp_level(s, p);
}

/* the slice header of the stand-in encoder's slices */
static void ext_header(or_bits *b, const or_cfg *c, const or_ext_params *p, int first, int nrefs, int nrefs_def)
{
    or_ue(b, (uint32_t)first);                                    /* first_mb_in_slice */
    if (p->islice) {                                              /* I (7: all of the picture) */
        or_ue(b, 7);
        or_ue(b, 0);                                              /* pps id */
        or_put(b, 0, c->log2_mfn);
        if (p->islice == 2) or_ue(b, 1);                          /* idr_pic_id */
        if (c->poc_type == 0) or_put(b, 0, c->log2_poc);
        if (p->islice == 2) or_put(b, 0, 2);                      /* no_output_of_prior_pics, long_term_reference */
        else if (p->ref_idc) or_put(b, 0, 1);                     /* sliding window */
        or_se(b, p->slice_qp_delta);
        if (c->deblock) or_ue(b, 1);
        return;
    }
    or_ue(b, 0);                                                  /* P */
    or_ue(b, 0);                                                  /* pps id */
    or_put(b, 0, c->log2_mfn);
    if (c->poc_type == 0) or_put(b, 0, c->log2_poc);
    if (nrefs != nrefs_def) {
        or_put(b, 1, 1);
        or_ue(b, (uint32_t)(nrefs - 1));
    } else {
        or_put(b, 0, 1);
    }
    if (p->list_mod) {                                            /* ref_pic_list_modification */
        or_put(b, 1, 1);
        for (int k = 0; k < nrefs; ++k) {
            or_ue(b, 2);                                          /* long_term_pic_num */
            or_ue(b, (uint32_t)(p->list_mod == 2 ? nrefs - 1 - k : k));
        }
        or_ue(b, 3);
    } else {
        or_put(b, 0, 1);
    }
    if (p->ref_idc) or_put(b, 0, 1);                              /* sliding window */
    or_se(b, p->slice_qp_delta);
    if (c->deblock) or_ue(b, 1);
}

/* an intra MB of the stand-in encoder (type 1 I_4x4, 2 I_16x16, 3 I_PCM, or
 * mbt_force 5..30), its modes predicted as the parse does (8.3.1.1) */
static void ext_intra(or_bits *b, uint32_t *s, const or_ext_params *p, int type, int mbt_force, int x, int y,
                      int W, const int *sid, int8_t (*im)[16], uint8_t (*tcs)[OR_SPLICE_PIECES], int *qp)
{
    const int m = y * W + x, u = sid[m];
    const uint8_t *L = x && sid[m - 1] == u ? tcs[m - 1] : NULL, *T = y && sid[m - W] == u ? tcs[m - W] : NULL;
    uint8_t *t = tcs[m];
    memset(t, 0, OR_SPLICE_PIECES);
    memset(im[m], -1, 16);
    if (mbt_force) type = mbt_force == 5 ? 1 : (mbt_force == 30 ? 3 : 2);
    const uint32_t mo = p->islice ? 5u : 0u;                      /* I slice: mb_type k = P's 5 + k */
    if (type == 3) {
        or_ue(b, 30 - mo);
        while (b->nbits & 7) or_put(b, 0, 1);
        for (int k = 0; k < 384; ++k) or_put(b, p->pcm_zero ? 0u : (sp_rng(s) & 255u), 8);
        memset(t, 16, OR_SPLICE_PIECES);
        return;
    }
    int coef[16];
    if (type == 1) {
        or_ue(b, 5 - mo);
        for (int blk = 0; blk < 16; ++blk) {
            const int ri = sp_blk_raster(blk), bx = ri & 3, by = ri >> 2;
            int mA = -2, mB = -2;
            if (bx) mA = im[m][ri - 1];
            else if (x && sid[m - 1] == u) mA = im[m - 1][ri + 3];
            if (by) mB = im[m][ri - 4];
            else if (y && sid[m - W] == u) mB = im[m - W][ri + 12];
            const int a = mA < 0 ? 2 : mA, bb = mB < 0 ? 2 : mB;
            const int pm = (mA == -2 || mB == -2) ? 2 : (a < bb ? a : bb);
            const int md = (sp_rng(s) % 3 == 0) ? pm : (int)(sp_rng(s) % 9);
            if (md == pm) {
                or_put(b, 1, 1);
            } else {
                or_put(b, 0, 1);
                or_put(b, (uint32_t)(md < pm ? md : md - 1), 3);
            }
            im[m][ri] = (int8_t)md;
        }
        or_ue(b, sp_rng(s) % 4);                                  /* intra_chroma_pred_mode */
        const int cbp = (int)(sp_rng(s) % 48);
        int code = 0;
        while (SP_CBP_INTRA[code] != cbp) ++code;
        or_ue(b, (uint32_t)code);
        if (!cbp) return;
        const int j = p->qp_jitter;
        int nq = *qp + (j ? (int)(sp_rng(s) % (uint32_t)(2 * j + 1)) - j : 0);
        nq = nq < 0 ? 0 : (nq > 51 ? 51 : nq);
        or_se(b, nq - *qp);
        *qp = nq;
        for (int blk = 0; blk < 16; ++blk) {
            if (!(cbp & (1 << (blk >> 2)))) continue;
            const int i = sp_blk_raster(blk);
            sp_rand_block(s, p, coef, 16);
            t[i] = (uint8_t)or_cavlc_block(b, coef, 16, sp_piece_nc(i, t, L, T));
        }
        if (cbp >> 4) {
            for (int i = 16; i < 18; ++i) {
                sp_rand_block(s, p, coef, 4);
                or_cavlc_block(b, coef, 4, -1);
            }
            if ((cbp >> 4) == 2)
                for (int i = 18; i < 26; ++i) {
                    sp_rand_block(s, p, coef, 15);
                    t[i] = (uint8_t)or_cavlc_block(b, coef, 15, sp_piece_nc(i, t, L, T));
                }
        }
        return;
    }
    /* I_16x16: prediction mode, chroma cbp, luma cbp in the mb_type */
    const int it = mbt_force ? mbt_force - 6 : (int)(sp_rng(s) % 24);
    const int cbl = it >= 12 ? 15 : 0, cbc = (it >> 2) % 3;
    or_ue(b, (uint32_t)(6 + it) - mo);
    or_ue(b, sp_rng(s) % 4);                                      /* intra_chroma_pred_mode */
    const int j = p->qp_jitter;
    int nq = *qp + (j ? (int)(sp_rng(s) % (uint32_t)(2 * j + 1)) - j : 0);
    nq = nq < 0 ? 0 : (nq > 51 ? 51 : nq);
    or_se(b, nq - *qp);                                           /* mb_qp_delta: always */
    *qp = nq;
    sp_rand_block(s, p, coef, 16);                                /* Intra16x16DCLevel */
    or_cavlc_block(b, coef, 16, sp_piece_nc(0, t, L, T));
    if (cbl)
        for (int blk = 0; blk < 16; ++blk) {                      /* Intra16x16ACLevel */
            const int i = sp_blk_raster(blk);
            sp_rand_block(s, p, coef, 15);
            t[i] = (uint8_t)or_cavlc_block(b, coef, 15, sp_piece_nc(i, t, L, T));
        }
    if (cbc) {
        for (int i = 16; i < 18; ++i) {
            sp_rand_block(s, p, coef, 4);
            or_cavlc_block(b, coef, 4, -1);
        }
        if (cbc == 2)
            for (int i = 18; i < 26; ++i) {
                sp_rand_block(s, p, coef, 15);
                t[i] = (uint8_t)or_cavlc_block(b, coef, 15, sp_piece_nc(i, t, L, T));
            }
    }
}

/* the stand-in encoder's NAL header: IDR pictures are nal_unit_type 5, a
 * reference (nal_ref_idc 3 unless given) */
static int ext_nut(const or_ext_params *p) { return p->islice == 2 ? 5 : 1; }
static int ext_ref_idc(const or_ext_params *p) { return p->islice == 2 && !p->ref_idc ? 3 : p->ref_idc; }

size_t or_ext_slice(uint8_t *dst, size_t cap, const or_cfg *c, int W, int H, uint32_t seed,
                    const or_ext_params *p)
{
    uint32_t s = seed * 2654435761u + 0x9E3779B9u;
    if (!s) s = 1;
    const int nmb = W * H, nrefs_def = c->num_ref_default_m1 + 1;
    const int nrefs = p->nrefs ? p->nrefs : nrefs_def;
    const size_t rcap = 64 + (size_t)nmb * 8192;
    uint8_t *rbsp = (uint8_t *)malloc(rcap);
    int *sid = (int *)malloc(sizeof(int) * (size_t)nmb);
    int8_t(*im)[16] = malloc((size_t)nmb * 16);
    or_bits b;
    or_bits_init(&b, rbsp, rcap);
    int qp = 26 + p->slice_qp_delta, slice = 0, top = 0;          /* top: the slice's first MB row */
    ext_header(&b, c, p, 0, nrefs, nrefs_def);
    sp_field F = {W, (or_mvi *)calloc((size_t)nmb * 16, sizeof(or_mvi)), sid, 0};
    uint8_t(*tcs)[OR_SPLICE_PIECES] = calloc((size_t)nmb, OR_SPLICE_PIECES);
    size_t nb = 0;
    int run = 0;
    const int rg = p->mv_range;
    for (int m = 0; m < nmb; ++m) {
        const int x = m % W, y = m / W;
        if (p->slice_rows > 0 && x == 0 && y > 0 && y % p->slice_rows == 0) {
            /* the next slice: this one ends (pending skips, trailing bits) */
            if (run > 0) or_ue(&b, (uint32_t)run);
            run = 0;
            or_trailing(&b);
            nb += or_nal(dst + nb, cap - nb, ext_ref_idc(p), ext_nut(p), rbsp, or_bytes(&b));
            or_bits_init(&b, rbsp, rcap);
            ext_header(&b, c, p, m, nrefs, nrefs_def);
            qp = 26 + p->slice_qp_delta;
            F.cur = ++slice;
            top = y;
        }
        sid[m] = slice;
        memset(im[m], -1, 16);
        or_mvi A, B, C, Cr, D;
        sp_nb16(&F, x, y, &A, &B, &C, &Cr, &D);
        if (m == p->bad_mb && (p->bad_type < 5 || p->bad_type > 30)) {
            or_ue(&b, (uint32_t)run);
            or_ue(&b, (uint32_t)p->bad_type);
            or_put(&b, sp_rng(&s), 32);
            run = 0;
            break;
        }
        const int forced = m == p->bad_mb ? p->bad_type : 0;     /* a valid intra MB of that type here */
        if (p->islice) {                                          /* every MB intra, no mb_skip_run */
            const int interior = x > 0 && x < W - 1 && y > top;
            const int k = (int)(sp_rng(&s) % 5);
            const int ty = p->intra_types ? p->intra_types : 7;
            int type = forced ? 0 : 3;                            /* the edge ring: I_PCM */
            if (!forced && (interior || p->islice == 3)) {
                type = k < 2 ? 1 : (k < 4 ? 2 : 3);
                if (!(ty >> (type - 1) & 1)) type = (ty & 2) ? 2 : ((ty & 1) ? 1 : 3);
            }
            ext_intra(&b, &s, p, type, forced, x, y, W, sid, im, tcs, &qp);
            for (int q = 0; q < 16; ++q) *sp_at(&F, x, y, q & 3, q >> 2) = (or_mvi){0, 0, -1, 1};
            continue;
        }
        if (!forced && (int)(sp_rng(&s) % 1000) < p->skip_pm) {
            int px, py;
            sp_pskip(&A, &B, &C, &px, &py);
            for (int k = 0; k < 16; ++k) *sp_at(&F, x, y, k & 3, k >> 2) = (or_mvi){px, py, 0, 1};
            memset(tcs[m], 0, OR_SPLICE_PIECES);
            run++;
            continue;
        }
        /* intra where any rect placement splices it (splice_oracle.h) */
        if (forced || (p->intra_pm > 0 && (int)(sp_rng(&s) % 1000) < p->intra_pm)) {
            const int interior = x > 0 && x < W - 1 && y > top;
            const int k = (int)(sp_rng(&s) % 5);
            int type = !interior ? 3 : (k < 2 ? 1 : (k < 4 ? 2 : 3));
            const int ty = p->intra_types ? p->intra_types : 7;
            if (!(ty >> (type - 1) & 1)) type = (ty & 2) && interior ? 2 : ((ty & 1) && interior ? 1 : ((ty & 4) ? 3 : 0));
            if (!forced && type == 0) {                           /* no allowed type here: inter */
                goto inter;
            }
            or_ue(&b, (uint32_t)run);
            run = 0;
            ext_intra(&b, &s, p, type, forced, x, y, W, sid, im, tcs, &qp);
            for (int q = 0; q < 16; ++q) *sp_at(&F, x, y, q & 3, q >> 2) = (or_mvi){0, 0, -1, 1};
            continue;
        }
    inter:;
        int ref = (int)(sp_rng(&s) % (uint32_t)(p->max_ref + 1));
        if (ref >= nrefs) ref = nrefs - 1;
        const int mx = rg ? (int)(sp_rng(&s) % (uint32_t)(2 * rg + 1)) - rg : 0;
        const int my = rg ? (int)(sp_rng(&s) % (uint32_t)(2 * rg + 1)) - rg : 0;
        /* a partitioned MB (drawn only when part_pm > 0: the other
         * parameters keep their slices bit for bit) */
        int mbt = 0;
        if (p->part_pm > 0 && (int)(sp_rng(&s) % 1000) < p->part_pm) mbt = 1 + (int)(sp_rng(&s) % 4);
        const int cbp = (int)(sp_rng(&s) % 1000) < p->cbp_pm ? 1 + (int)(sp_rng(&s) % 47) : 0;
        or_ue(&b, (uint32_t)run);
        run = 0;
        or_ue(&b, (uint32_t)mbt);
        if (mbt == 0) {
            int px, py;
            or_spec_predict(&A, &B, &C, ref, &px, &py);
            if (nrefs == 2) or_put(&b, (uint32_t)(1 - ref), 1);
            else if (nrefs > 2) or_ue(&b, (uint32_t)ref);
            or_se(&b, mx - px);
            or_se(&b, my - py);
            for (int k = 0; k < 16; ++k) *sp_at(&F, x, y, k & 3, k >> 2) = (or_mvi){mx, my, ref, 1};
        } else {
            const int part = mbt == 4 ? 3 : mbt;
            int sub = 0, refs[4] = {ref, ref, ref, ref};
            if (part == 3)
                for (int i = 0; i < 4; ++i) {
                    const int st = (int)(sp_rng(&s) % 4);
                    sub |= st << (2 * i);
                    or_ue(&b, (uint32_t)st);
                }
            const int nref = part == 3 ? 4 : 2;
            for (int i = 0; i < nref; ++i) {
                refs[i] = mbt == 4 ? 0 : (int)(sp_rng(&s) % (uint32_t)(p->max_ref + 1));
                if (refs[i] >= nrefs) refs[i] = nrefs - 1;
                if (mbt == 4) continue;
                if (nrefs == 2) or_put(&b, (uint32_t)(1 - refs[i]), 1);
                else if (nrefs > 2) or_ue(&b, (uint32_t)refs[i]);
            }
            sp_part ps[16];
            const int np = sp_partitions(part, sub, ps);
            unsigned done = 0;
            for (int k = 0; k < np; ++k) {
                /* motion near the MB's own draw, so predictions and mvds vary */
                const int vx = mx + (rg ? (int)(sp_rng(&s) % 17) - 8 : 0);
                const int vy = my + (rg ? (int)(sp_rng(&s) % 17) - 8 : 0);
                const int rf = refs[ps[k].mb_part];
                int px, py;
                sp_mvp(&F, x, y, done, part, &ps[k], rf, &px, &py);
                or_se(&b, vx - px);
                or_se(&b, vy - py);
                sp_fill(&F, x, y, &ps[k], (or_mvi){vx, vy, rf, 1}, &done);
            }
        }
        or_ue(&b, (uint32_t)or_cbp_code(cbp));
        uint8_t *t = tcs[m];
        memset(t, 0, OR_SPLICE_PIECES);
        if (cbp) {
            const int j = p->qp_jitter;
            int nq = qp + (j ? (int)(sp_rng(&s) % (uint32_t)(2 * j + 1)) - j : 0);
            nq = nq < 0 ? 0 : (nq > 51 ? 51 : nq);
            or_se(&b, nq - qp);
            qp = nq;
            const uint8_t *L = x && sid[m - 1] == slice ? tcs[m - 1] : NULL;
            const uint8_t *T = y && sid[m - W] == slice ? tcs[m - W] : NULL;
            int coef[16];
            for (int blk = 0; blk < 16; ++blk) {
                if (!(cbp & (1 << (blk >> 2)))) continue;
                const int i = sp_blk_raster(blk);
                sp_rand_block(&s, p, coef, 16);
                t[i] = (uint8_t)or_cavlc_block(&b, coef, 16, sp_piece_nc(i, t, L, T));
            }
            if (cbp >> 4) {
                for (int i = 16; i < 18; ++i) {
                    sp_rand_block(&s, p, coef, 4);
                    or_cavlc_block(&b, coef, 4, -1);
                }
                if ((cbp >> 4) == 2)
                    for (int i = 18; i < 26; ++i) {
                        sp_rand_block(&s, p, coef, 15);
                        t[i] = (uint8_t)or_cavlc_block(&b, coef, 15, sp_piece_nc(i, t, L, T));
                    }
            }
        }
    }
    if (run > 0) or_ue(&b, (uint32_t)run);
    or_trailing(&b);
    nb += or_nal(dst + nb, cap - nb, ext_ref_idc(p), ext_nut(p), rbsp, or_bytes(&b));
    free(rbsp);
    free(F.f);
    free(tcs);
    free(sid);
    free(im);
    return nb;
}
