/*
 * nal_parser.c -- host Annex-B ingest (ABI of include/nal_parser.h).
 * Behaviour of the reference src/nal_parser.c:4-276 (start-code scan,
 * trailing-zero strip, EBSP -> RBSP, minimal SPS/PPS parse incl. its quirk
 * of reading the PPS se(v) fields as ue(v), which consumes the same bits).
 * Runs once per stream in composer_init.
 */
#include "nal_parser.h"

#include <string.h>

#include "bitwriter.h"

void nal_parser_init(NALParser *parser, const uint8_t *data, size_t size)
{
    parser->data = data;
    parser->size = size;
    parser->pos = 0;
}

/* index just after the next 00 00 01 / 00 00 00 01 at or after `from`, else n */
static size_t sc_after(const uint8_t *d, size_t n, size_t from)
{
    for (size_t i = from; i + 2 < n; ++i) {
        if (d[i] != 0 || d[i + 1] != 0) continue;
        if (d[i + 2] == 1) return i + 3;
        if (i + 3 < n && d[i + 2] == 0 && d[i + 3] == 1) return i + 4;
    }
    return n;
}

/* index of the next start code (its first zero) at or after `from`, else n */
static size_t sc_begin(const uint8_t *d, size_t n, size_t from)
{
    for (size_t i = from; i + 2 < n; ++i) {
        if (d[i] != 0 || d[i + 1] != 0) continue;
        if (d[i + 2] == 1 || (i + 3 < n && d[i + 2] == 0 && d[i + 3] == 1)) return i;
    }
    return n;
}

int nal_parser_next(NALParser *parser, NALUnit *unit)
{
    const uint8_t *d = parser->data;
    size_t n = parser->size;
    size_t s = sc_after(d, n, parser->pos);
    if (s >= n) return 0;
    size_t e = sc_begin(d, n, s);
    while (e > s && d[e - 1] == 0) e--;
    parser->pos = e;
    if (e <= s) return 0;
    unit->nal_ref_idc = (d[s] >> 5) & 3;
    unit->nal_unit_type = d[s] & 31;
    unit->data = d + s + 1;
    unit->size = e - s - 1;
    return 1;
}

size_t ebsp_to_rbsp(uint8_t *rbsp, const uint8_t *ebsp, size_t ebsp_size)
{
    size_t o = 0;
    int zeros = 0;
    for (size_t i = 0; i < ebsp_size; ++i) {
        uint8_t v = ebsp[i];
        if (zeros >= 2 && v == 3 && i + 1 < ebsp_size && ebsp[i + 1] <= 3) {
            zeros = 0;
            continue;
        }
        rbsp[o++] = v;
        zeros = v ? 0 : zeros + 1;
    }
    return o;
}

static int high_profile(int p)
{
    static const int hp[] = {100, 110, 122, 244, 44, 83, 86, 118, 128, 138, 139, 134};
    for (size_t i = 0; i < sizeof(hp) / sizeof(hp[0]); ++i)
        if (hp[i] == p) return 1;
    return 0;
}

int parse_sps(const uint8_t *rbsp, size_t size, int *width, int *height,
              int *log2_max_frame_num, int *pic_order_cnt_type, int *log2_max_pic_order_cnt_lsb)
{
    BitReader br;
    bitreader_init(&br, rbsp, size);
    int profile = (int)bitreader_read_bits(&br, 8);
    bitreader_read_bits(&br, 16);                  /* constraint flags + level_idc */
    bitreader_read_ue(&br);                        /* seq_parameter_set_id */
    if (high_profile(profile)) {
        if (bitreader_read_ue(&br) == 3) bitreader_read_bit(&br);
        bitreader_read_ue(&br);
        bitreader_read_ue(&br);
        bitreader_read_bit(&br);
        if (bitreader_read_bit(&br)) return -1;    /* scaling matrices unsupported */
    }
    *log2_max_frame_num = (int)bitreader_read_ue(&br) + 4;
    *pic_order_cnt_type = (int)bitreader_read_ue(&br);
    *log2_max_pic_order_cnt_lsb = 0;
    if (*pic_order_cnt_type == 0)
        *log2_max_pic_order_cnt_lsb = (int)bitreader_read_ue(&br) + 4;
    else if (*pic_order_cnt_type == 1)
        return -1;
    bitreader_read_ue(&br);                        /* max_num_ref_frames */
    bitreader_read_bit(&br);                       /* gaps flag */
    int wmbs = (int)bitreader_read_ue(&br) + 1;
    int hmap = (int)bitreader_read_ue(&br) + 1;
    if (!bitreader_read_bit(&br)) {                /* frame_mbs_only_flag */
        bitreader_read_bit(&br);
        hmap *= 2;
    }
    *width = wmbs * 16;
    *height = hmap * 16;
    return 0;
}

int parse_pps(const uint8_t *rbsp, size_t size, int *num_ref_idx_l0_default_minus1,
              int *deblocking_filter_control_present_flag)
{
    BitReader br;
    bitreader_init(&br, rbsp, size);
    bitreader_read_ue(&br);                        /* pps id */
    bitreader_read_ue(&br);                        /* sps id */
    bitreader_read_bits(&br, 2);                   /* entropy + bottom_field flags */
    if (bitreader_read_ue(&br) > 0) return -1;     /* slice groups unsupported */
    *num_ref_idx_l0_default_minus1 = (int)bitreader_read_ue(&br);
    bitreader_read_ue(&br);
    bitreader_read_bits(&br, 3);                   /* weighted_pred + bipred_idc */
    bitreader_read_ue(&br);                        /* pic_init_qp_minus26  (se) */
    bitreader_read_ue(&br);                        /* pic_init_qs_minus26  (se) */
    bitreader_read_ue(&br);                        /* chroma_qp_index_offset (se) */
    *deblocking_filter_control_present_flag = bitreader_read_bit(&br);
    return 0;
}
