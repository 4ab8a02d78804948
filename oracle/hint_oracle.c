/*
 * hint_oracle.c -- CPU ORACLE (test infrastructure only): the UI-hint P
 * slice.  See hint_oracle.h for the semantics and how the bits are pinned.
 * The MB loop follows src/h264_writer.c:595-646 (scroll frame); the P_Skip
 * mode follows ITU-T H.264 7.3.4 (mb_skip_run), 8.4.1.1 (P_Skip motion) and
 * 8.4.1.3 (median prediction).
 */
#include "hint_oracle.h"

#include <stdlib.h>
#include <string.h>

/* MV field of the frame: hints over the scroll layout of `off` */
static int field_at(const or_hint_rect *r, int n, int x, int y, int a_end, int ra, int mva,
                    int rb, int mvb, int *ref, int *mx, int *my)
{
    for (int i = n - 1; i >= 0; --i) {
        if (x >= r[i].x0 && x < r[i].x1 && y >= r[i].y0 && y < r[i].y1) {
            *ref = r[i].ref;
            *mx = r[i].mv_x;
            *my = r[i].mv_y;
            return 1;
        }
    }
    *ref = y < a_end ? ra : rb;                        /* h264_writer.c:601-620 */
    *mx = 0;
    *my = y < a_end ? mva : mvb;
    return 0;
}

static int ref_valid(const or_cfg *c, int ref)
{
    if (ref == 0 || ref == 1) return 1;
    int i = ref - 2;
    return i >= 0 && i < c->nwp && c->wp_valid[i];
}

int or_hint_field(const or_cfg *c, int off, const or_hint_rect *r, int n, int32_t *out)
{
    int a_end, ra, mva, rb, mvb;
    or_scroll_regions(c, off, &a_end, &ra, &mva, &rb, &mvb);
    int mbw = c->w / 16, mbh = c->h / 16, bad = 0;
    for (int y = 0; y < mbh; ++y)
        for (int x = 0; x < mbw; ++x) {
            int ref, mx, my;
            if (field_at(r, n, x, y, a_end, ra, mva, rb, mvb, &ref, &mx, &my) && !ref_valid(c, ref))
                bad = 1;
            int32_t *o = out + 3 * ((size_t)y * mbw + x);
            o[0] = ref;
            o[1] = mx;
            o[2] = my;
        }
    return bad ? -1 : 0;
}

/* ---- standard motion vector prediction (8.4.1.3), 16x16 partitions ---- */
static int med3(int a, int b, int c)
{
    int lo = a < b ? a : b, hi = a < b ? b : a;
    return c < lo ? lo : (c > hi ? hi : c);
}

/* neighbours A (left), B (above), C (above-right, else D above-left) of the
 * MB at (x, y); unavailable ones have ref -1 and mv 0 */
static void neighbours(int x, int y, int mbw, const or_mvi *above, const or_mvi *left,
                       or_mvi *A, or_mvi *B, or_mvi *C)
{
    const or_mvi none = {0, 0, -1, 0};
    *A = x > 0 ? *left : none;
    *B = y > 0 ? above[x] : none;
    if (y > 0 && x + 1 < mbw)
        *C = above[x + 1];
    else if (y > 0 && x > 0)
        *C = above[x - 1];                              /* 8.4.1.3.2: D replaces C */
    else
        *C = none;
}

static void spec_mvp(const or_mvi *A0, const or_mvi *B0, const or_mvi *C0, int ref, int *px,
                     int *py)
{
    or_mvi A = *A0, B = *B0, C = *C0;
    if (!B.avail && !C.avail && A.avail) {             /* 8.4.1.3.1 */
        B = A;
        C = A;
    }
    int ma = A.avail && A.ref == ref, mb = B.avail && B.ref == ref, mc = C.avail && C.ref == ref;
    if (ma + mb + mc == 1) {
        const or_mvi *k = ma ? &A : (mb ? &B : &C);
        *px = k->mx;
        *py = k->my;
        return;
    }
    *px = med3(A.avail ? A.mx : 0, B.avail ? B.mx : 0, C.avail ? C.mx : 0);
    *py = med3(A.avail ? A.my : 0, B.avail ? B.my : 0, C.avail ? C.my : 0);
}

/* 8.4.1.1: motion of a P_Skip MB */
static void pskip_mv(int x, int y, const or_mvi *A, const or_mvi *B, const or_mvi *C, int *px,
                     int *py)
{
    if (x == 0 || y == 0 || (A->ref == 0 && A->mx == 0 && A->my == 0) ||
        (B->ref == 0 && B->mx == 0 && B->my == 0)) {
        *px = 0;
        *py = 0;
        return;
    }
    spec_mvp(A, B, C, 0, px, py);
}

/* exported for the splice restatement (splice_oracle.c) */
int or_hint_motion(const or_hint_rect *r, int n, int x, int y, int a_end, int ra, int mva,
                   int rb, int mvb, int *ref, int *mx, int *my)
{
    return field_at(r, n, x, y, a_end, ra, mva, rb, mvb, ref, mx, my);
}
int or_ref_valid(const or_cfg *c, int ref) { return ref_valid(c, ref); }
void or_neighbours(int x, int y, int mbw, const or_mvi *above, const or_mvi *left, or_mvi *A,
                   or_mvi *B, or_mvi *C)
{
    neighbours(x, y, mbw, above, left, A, B, C);
}
void or_spec_predict(const or_mvi *A, const or_mvi *B, const or_mvi *C, int ref, int *px, int *py)
{
    spec_mvp(A, B, C, ref, px, py);
}
void or_pskip_motion(int x, int y, const or_mvi *A, const or_mvi *B, const or_mvi *C, int *px,
                     int *py)
{
    pskip_mv(x, y, A, B, C, px, py);
}

size_t or_hint_scroll_nal(uint8_t *dst, size_t cap, or_cfg *c, int off,
                          const or_hint_rect *r, int n, int mode, int *err)
{
    if (err) *err = 0;
    int a_end, ra, mva, rb, mvb;
    or_scroll_regions(c, off, &a_end, &ra, &mva, &rb, &mvb);
    int mbw = c->w / 16, mbh = c->h / 16, nrefs = 2 + c->nwp;
    size_t rcap = 64 + (size_t)mbw * (size_t)mbh * 24;
    uint8_t *rbsp = (uint8_t *)malloc(rcap);
    or_mvi *above = (or_mvi *)calloc((size_t)mbw, sizeof(or_mvi));
    or_mvi *cur = (or_mvi *)calloc((size_t)mbw, sizeof(or_mvi));
    or_bits b;
    or_bits_init(&b, rbsp, rcap);
    or_scroll_header(&b, c);                            /* :549-553 */
    int run = 0, bad = 0;
    for (int y = 0; y < mbh; ++y) {
        or_mvi left = {0, 0, -1, 0};
        for (int x = 0; x < mbw; ++x) {
            int ref, mx, my;
            if (field_at(r, n, x, y, a_end, ra, mva, rb, mvb, &ref, &mx, &my) &&
                !ref_valid(c, ref))
                bad = 1;
            mx *= 4;                                    /* quarter pels */
            my *= 4;
            int px, py;
            if (mode != OR_HINT_EXACT) {
                or_mvi A, B, C;
                neighbours(x, y, mbw, above, &left, &A, &B, &C);
                int sx, sy;
                pskip_mv(x, y, &A, &B, &C, &sx, &sy);
                if (mode == OR_HINT_PSKIP && ref == 0 && mx == sx && my == sy) {
                    run++;                              /* P_Skip */
                } else {
                    spec_mvp(&A, &B, &C, ref, &px, &py);
                    or_ue(&b, (uint32_t)run);           /* mb_skip_run */
                    run = 0;
                    or_ue(&b, 0);                       /* mb_type P_L0_16x16 */
                    if (nrefs == 2) or_put(&b, (uint32_t)(1 - (ref & 1)), 1);
                    else if (nrefs > 2) or_ue(&b, (uint32_t)ref);
                    or_se(&b, mx - px);
                    or_se(&b, my - py);
                    or_ue(&b, 0);                       /* coded_block_pattern 0 */
                }
            } else {                                    /* :630, :434-453 */
                or_predict(x, y, mbw, above, &left, ref, &px, &py);
                or_ue(&b, 0);
                or_ue(&b, 0);
                if (nrefs == 2) or_put(&b, (uint32_t)(1 - (ref & 1)), 1);
                else if (nrefs > 2) or_ue(&b, (uint32_t)ref);
                or_se(&b, mx - px);
                or_se(&b, my - py);
                or_ue(&b, 0);
            }
            cur[x].mx = mx;
            cur[x].my = my;
            cur[x].ref = ref;
            cur[x].avail = 1;
            left = cur[x];
        }
        or_mvi *t = above;
        above = cur;
        cur = t;
    }
    if (run > 0) or_ue(&b, (uint32_t)run);              /* trailing skipped MBs */
    or_trailing(&b);
    size_t nb = 0;
    if (bad) {
        if (err) *err = 1;
    } else {
        nb = or_nal(dst, cap, 0, 1, rbsp, or_bytes(&b));
        c->frame_num++;
    }
    free(rbsp);
    free(above);
    free(cur);
    return nb;
}

size_t or_compose_hint(uint8_t *dst, size_t cap, or_cfg *c, int off, int compose_mode,
                       const or_hint_rect *r, int n, int mode, int *err)
{
    if (err) *err = 0;
    size_t nb = 0;
    if (or_needs_waypoint(c, off)) {                    /* src/composer.c:255-264 */
        nb += or_waypoint_nal(dst, cap, c, off);
        if (compose_mode == 1) return nb;
    }
    size_t k = or_hint_scroll_nal(dst + nb, cap - nb, c, off, r, n, mode, err);
    return k ? nb + k : 0;
}
