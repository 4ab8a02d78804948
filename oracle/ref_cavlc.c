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
