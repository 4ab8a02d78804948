/*
 * ref_cavlc.c -- TEST INFRASTRUCTURE: the reference's own CAVLC P-slice
 * parser (experiments/trans-resizer/trans_resizer.c:1486-1787
 * process_p_slice -> :1362-1470 copy_inter_residual -> :612-755
 * copy_cavlc_block, nC rules :782-885) driven over the MB layer of a slice,
 * to cross-check the syntax of the dynamic-rect residual coder (which has
 * no reference implementation).  Compiled in place from the reference
 * sources by `make -C oracle ref`; never copied into this repository.
 * trans_resizer's geometry is fixed at 320x320 (20x20 MBs).
 */
#define main trans_resizer_main
#include "trans_resizer.c"
#undef main

/* parse the MB layer starting at bit start_bit of rbsp; returns
 * process_p_slice's status (0 ok) and the bit position where it stopped */
int ref_cavlc_parse(const uint8_t *rbsp, size_t n, size_t start_bit, int num_ref,
                    size_t *end_bit)
{
    BitReader br;
    bitreader_init(&br, rbsp, n);
    for (size_t i = 0; i < start_bit; ++i) bitreader_read_bit(&br);
    size_t cap = n * 4 + 65536;
    uint8_t *out = (uint8_t *)malloc(cap);
    BitWriter bw;
    bitwriter_init(&bw, out, cap);
    free(top_mb_ctx);
    top_mb_ctx = NULL;
    top_mb_ctx_size = 0;
    int rc = process_p_slice(&br, &bw, num_ref);
    *end_bit = bitreader_get_bit_position(&br);
    free(out);
    return rc;
}

/* the same for an I slice's MB layer (process_i_slice :1063-1360: a whole
 * 20x20-MB picture, mb_type / prediction modes / cbp / residuals), its
 * debug output silenced */
static int quiet_begin(void);
static void quiet_end(int saved);
int ref_cavlc_parse_i(const uint8_t *rbsp, size_t n, size_t start_bit, size_t *end_bit)
{
    BitReader br;
    bitreader_init(&br, rbsp, n);
    for (size_t i = 0; i < start_bit; ++i) bitreader_read_bit(&br);
    size_t cap = n * 4 + ((size_t)16 << 20);     /* + the walker's I_PCM padding MBs per row */
    uint8_t *out = (uint8_t *)malloc(cap);
    BitWriter bw;
    bitwriter_init(&bw, out, cap);
    free(top_mb_ctx);
    top_mb_ctx = NULL;
    top_mb_ctx_size = 0;
    fflush(stdout);
    const int saved = quiet_begin();
    const int rc = process_i_slice(&br, &bw);
    fflush(stdout);
    quiet_end(saved);
    *end_bit = bitreader_get_bit_position(&br);
    free(out);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* value-level check of one inter MB's residual (cbp me(v), mb_qp_delta,      */
/* blocks), every decode step a reference function                          */
/* ------------------------------------------------------------------------ */
/* compute_luma_nC prints a debug line for raster block 13 (:823-831): the
 * calls below run with stderr on /dev/null */
#include <fcntl.h>
#include <unistd.h>
static int quiet_begin(void)
{
    fflush(stderr);
    int saved = dup(2), nul = open("/dev/null", O_WRONLY);
    if (nul >= 0) {
        dup2(nul, 2);
        close(nul);
    }
    return saved;
}
static void quiet_end(int saved)
{
    fflush(stderr);
    if (saved >= 0) {
        dup2(saved, 2);
        close(saved);
    }
}

/* The residual bits of one inter MB (after its mvd fields) in rbsp from bit
 * start: coded_block_pattern through bitreader_read_ue + cbp_inter_table
 * (:284-288), mb_qp_delta through bitreader_read_se, then the blocks in
 * copy_inter_residual's order (:1388-1446) with its nC rules
 * (compute_luma_nC :782, compute_chroma_nC :841) over the neighbour
 * TotalCoeffs tcl / tct (16 luma raster + Cb AC 4 + Cr AC 4 of the left / top
 * MB; avail_l / avail_t = 0: that neighbour does not exist).  Per coded block
 * (at most 26) rec[i] = {id, nC, tc, t1, start, token_end, end}: id = luma
 * raster 0-15, 16 / 17 chroma DC Cb / Cr, 18 + 4 p + k chroma AC; tc, t1 and
 * token_end from read_coeff_token (:549), end from copy_cavlc_block (:612,
 * the reference's whole-block parse incl. levels).  Returns the number of
 * blocks, or -1 (a decode failed); *cbp_out, *qpd_out. */
int ref_cavlc_mb(const uint8_t *rbsp, size_t n, size_t start, int avail_l, int avail_t, const int tcl[24],
                 const int tct[24], int *cbp_out, int *qpd_out, long long rec[26][7])
{
    BitReader br;
    bitreader_init(&br, rbsp, n);
    for (size_t i = 0; i < start; ++i) bitreader_read_bit(&br);
    size_t cap = n * 4 + 65536;
    uint8_t *out = (uint8_t *)malloc(cap);
    BitWriter bw;
    bitwriter_init(&bw, out, cap);
    const int q = quiet_begin();
    int nb = 0, rc = 0;
    const uint32_t code = br_read_ue(&br);
    const int cbp = code < 48 ? cbp_inter_table[code] : -1;
    *cbp_out = cbp;
    *qpd_out = 0;
    if (cbp < 0) {
        rc = -1;
        goto done;
    }
    if (cbp == 0) goto done;
    *qpd_out = br_read_se(&br);
    MBCoeffContext L, T, C;
    memset(&L, 0, sizeof L);
    memset(&T, 0, sizeof T);
    memset(&C, 0, sizeof C);
    for (int i = 0; i < 16; ++i) {
        L.luma_tc[i] = tcl[i];
        T.luma_tc[i] = tct[i];
    }
    for (int p = 0; p < 2; ++p)
        for (int k = 0; k < 4; ++k) {
            L.chroma_tc[p][k] = tcl[16 + 4 * p + k];
            T.chroma_tc[p][k] = tct[16 + 4 * p + k];
        }
    /* compute_*_nC take mb_col > 0 && left != NULL for the left MB */
    const MBCoeffContext *left = avail_l ? &L : NULL, *top = avail_t ? &T : NULL;
    const int mb_col = avail_l ? 1 : 0;
    static const int s2r[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};
    for (int b = 0; b < 26 && rc == 0; ++b) {
        int id, nC, maxc;
        if (b < 16) {
            if (!((cbp & 15) >> (b >> 2) & 1)) continue;
            id = s2r[b];
            nC = compute_luma_nC(id, mb_col, &C, left, top);
            maxc = 16;
        } else if (b < 18) {
            if (((cbp >> 4) & 3) == 0) continue;
            id = b;
            nC = -1;
            maxc = 4;
        } else {
            if (((cbp >> 4) & 3) != 2) continue;
            id = b;
            const int p = (b - 18) >> 2, k = (b - 18) & 3;
            nC = compute_chroma_nC(p, k, mb_col, &C, left, top);
            maxc = 15;
        }
        const size_t bs = br.byte_pos;
        const int bb = br.bit_pos;
        const long long s0 = (long long)bitreader_get_bit_position(&br);
        int tc = 0, t1 = 0;
        if (read_coeff_token(&br, nC, &tc, &t1) < 0) {
            rc = -1;
            break;
        }
        const long long te = (long long)bitreader_get_bit_position(&br);
        br.byte_pos = bs;
        br.bit_pos = bb;
        const int tcc = copy_cavlc_block(&br, &bw, nC, maxc);
        if (tcc < 0 || tcc != tc) {
            rc = -1;
            break;
        }
        if (id < 16) C.luma_tc[id] = tc;
        else if (id >= 18) C.chroma_tc[(id - 18) >> 2][(id - 18) & 3] = tc;
        long long *r = rec[nb++];
        r[0] = id;
        r[1] = nC;
        r[2] = tc;
        r[3] = t1;
        r[4] = s0;
        r[5] = te;
        r[6] = (long long)bitreader_get_bit_position(&br);
    }
done:
    quiet_end(q);
    free(out);
    return rc < 0 ? -1 : nb;
}

/* The level values of one block as the reference's own level parser reads
 * them.  copy_cavlc_block (:612) traces each levelCode it decodes (:690-693)
 * for blocks that start at bytes 96-110 of its reader; the block (at bit pos
 * of rbsp) is copied to byte 100 of a scratch buffer, parsed there with
 * stderr on a temporary file, and the traced levelCodes are read back.
 * Returns the number of levels (TotalCoeff - TrailingOnes), -1 on failure;
 * codes[] the levelCodes in coding order, signs = the TrailingOnes sign bits
 * (first one in bit t1 - 1), *tc_out. */
#include <stdlib.h>
int ref_cavlc_levels(const uint8_t *rbsp, size_t n, size_t pos, int nC, int maxc, int codes[16], int *signs,
                     int *tc_out)
{
    const size_t nb = n - pos / 8 + 8, off = 100;
    uint8_t *buf = (uint8_t *)calloc(off + nb + 8, 1);
    memcpy(buf + off, rbsp + pos / 8, n - pos / 8);
    BitReader br;
    bitreader_init(&br, buf, off + nb);
    br.byte_pos = off;
    br.bit_pos = (int)(pos & 7);
    size_t cap = nb * 4 + 4096;
    uint8_t *out = (uint8_t *)malloc(cap);
    BitWriter bw;
    bitwriter_init(&bw, out, cap);
    char path[] = "/tmp/ref_cavlc_XXXXXX";
    const int fd = mkstemp(path);
    int nl = -1;
    if (fd >= 0) {
        fflush(stderr);
        const int saved = dup(2);
        dup2(fd, 2);
        /* TrailingOnes and their sign bits first (read_coeff_token, then the
         * raw sign bits as copy_cavlc_block copies them, :638-639) */
        int tc = 0, t1 = 0;
        const int ok = read_coeff_token(&br, nC, &tc, &t1) >= 0;
        int sg = 0;
        for (int i = 0; ok && i < t1; ++i) sg = sg << 1 | bitreader_read_bit(&br);
        br.byte_pos = off;
        br.bit_pos = (int)(pos & 7);
        const int tcc = ok ? copy_cavlc_block(&br, &bw, nC, maxc) : -1;
        fflush(stderr);
        dup2(saved, 2);
        close(saved);
        if (tcc >= 0) {
            *tc_out = tcc;
            *signs = sg;
            nl = 0;
            FILE *f = fdopen(fd, "r");
            char line[512];
            rewind(f);
            while (fgets(line, sizeof line, f)) {
                const char *p = strstr(line, "levelCode=");
                if (p && nl < 16) codes[nl++] = atoi(p + 10);
            }
            fclose(f);
            if (nl != tcc - t1) nl = -1;
        } else {
            close(fd);
        }
        unlink(path);
    }
    free(out);
    free(buf);
    return nl;
}

/* total_zeros (decode_total_zeros :467) and the run_before values
 * (decode_run_before :514, while zeros are left, at most tc - 1) of a block
 * with TotalCoeff tc whose levels end at bit pos; returns the number of runs
 * read (-1 on a decode failure), *tz_out, runs[], *end_out */
int ref_cavlc_tail(const uint8_t *rbsp, size_t n, size_t pos, int tc, int maxc, int *tz_out, int runs[16],
                   size_t *end_out)
{
    BitReader br;
    bitreader_init(&br, rbsp, n);
    for (size_t i = 0; i < pos; ++i) bitreader_read_bit(&br);
    const int q = quiet_begin();
    int nr = 0;
    const int tz = tc < maxc ? decode_total_zeros(&br, tc, maxc) : 0;
    if (tz < 0) {
        quiet_end(q);
        return -1;
    }
    int zl = tz;
    for (int i = 0; i < tc - 1 && zl > 0; ++i) {
        const int run = decode_run_before(&br, zl);
        if (run < 0) {
            quiet_end(q);
            return -1;
        }
        runs[nr++] = run;
        zl -= run;
    }
    quiet_end(q);
    *tz_out = tz;
    *end_out = bitreader_get_bit_position(&br);
    return nr;
}
