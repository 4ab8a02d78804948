/*
 * h264_writer.c -- ABI of include/h264_writer.h.
 *
 *   cold, host:  composer_config_*, h264_generate_sps/pps, I-frame rewrites,
 *                h264_needs_waypoint (reference src/h264_writer.c:13-350,666-676)
 *   HOT, GPU:    h264_write_scroll_p_frame, h264_write_waypoint_p_frame
 *                (reference :541-664, :678-782) -> scroll_engine_write_nals()
 *                -> k_plan + k_emit on the MI355X.  No CPU fallback: if the
 *                engine fails the call aborts with a message, like the
 *                reference's capacity asserts.
 */
#include "h264_writer.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../engine.h"

void composer_config_init(ComposerConfig *cfg, int width, int height)
{
    memset(cfg, 0, sizeof(*cfg));
    cfg->width = width;
    cfg->height = height;
    cfg->mb_width = width / 16;
    cfg->mb_height = height / 16;
    cfg->log2_max_frame_num = 4;
    cfg->pic_order_cnt_type = 2;
    cfg->log2_max_pic_order_cnt_lsb = 4;
    cfg->num_ref_idx_l0_default_minus1 = 1;
    cfg->deblocking_filter_control_present_flag = 1;
}

void composer_config_set_sps_params(ComposerConfig *cfg, int log2_max_frame_num,
                                    int pic_order_cnt_type, int log2_max_pic_order_cnt_lsb)
{
    cfg->log2_max_frame_num = log2_max_frame_num;
    cfg->pic_order_cnt_type = pic_order_cnt_type;
    cfg->log2_max_pic_order_cnt_lsb = log2_max_pic_order_cnt_lsb;
}

void composer_config_set_pps_params(ComposerConfig *cfg, int num_ref_idx_l0_default_minus1,
                                    int deblocking_filter_control_present_flag)
{
    cfg->num_ref_idx_l0_default_minus1 = num_ref_idx_l0_default_minus1;
    cfg->deblocking_filter_control_present_flag = deblocking_filter_control_present_flag;
}

/* Baseline SPS: profile 66, constraint 0xc0, level 40, log2_max_frame_num 4,
 * poc type 2, max_num_ref_frames 2 + MAX_WAYPOINTS (reference :49-100). */
size_t h264_generate_sps(uint8_t *rbsp, size_t capacity, int width, int height)
{
    BitWriter bw;
    bitwriter_init(&bw, rbsp, capacity);
    bitwriter_write_bits(&bw, (66u << 16) | (0xc0u << 8) | 40u, 24);
    bitwriter_write_ue(&bw, 0);                       /* sps id */
    bitwriter_write_ue(&bw, 0);                       /* log2_max_frame_num_minus4 */
    bitwriter_write_ue(&bw, 2);                       /* pic_order_cnt_type */
    bitwriter_write_ue(&bw, 2 + MAX_WAYPOINTS);       /* max_num_ref_frames */
    bitwriter_write_bit(&bw, 0);                      /* gaps */
    bitwriter_write_ue(&bw, (uint32_t)(width / 16 - 1));
    bitwriter_write_ue(&bw, (uint32_t)(height / 16 - 1));
    bitwriter_write_bits(&bw, 0xC, 4);                /* frame_mbs_only 1, direct_8x8 1, crop 0, vui 0 */
    bitwriter_write_trailing_bits(&bw);
    return bitwriter_get_size(&bw);
}

/* Baseline PPS, CAVLC, 2 default refs, deblocking control present (:105-127) */
size_t h264_generate_pps(uint8_t *rbsp, size_t capacity)
{
    BitWriter bw;
    bitwriter_init(&bw, rbsp, capacity);
    bitwriter_write_ue(&bw, 0);                       /* pps id */
    bitwriter_write_ue(&bw, 0);                       /* sps id */
    bitwriter_write_bits(&bw, 0, 2);                  /* CAVLC, no bottom_field_pic_order */
    bitwriter_write_ue(&bw, 0);                       /* one slice group */
    bitwriter_write_ue(&bw, 1);                       /* num_ref_idx_l0_default_active_minus1 */
    bitwriter_write_ue(&bw, 0);
    bitwriter_write_bits(&bw, 0, 3);                  /* weighted pred / bipred */
    bitwriter_write_se(&bw, 0);
    bitwriter_write_se(&bw, 0);
    bitwriter_write_se(&bw, 0);
    bitwriter_write_bits(&bw, 4, 3);                  /* deblock ctrl 1, constrained intra 0, redundant 0 */
    bitwriter_write_trailing_bits(&bw);
    return bitwriter_get_size(&bw);
}

/* ---------------- I-frame rewrite (cold; reference :133-350) ---------------- */
typedef struct {
    size_t mb_start;
    int32_t qp_delta;
    uint32_t dbf_idc;
    int32_t alpha, beta;
} IdrHeader;

static void parse_idr_header(const uint8_t *rbsp, size_t n, const ComposerConfig *pc, IdrHeader *h)
{
    BitReader br;
    bitreader_init(&br, rbsp, n);
    memset(h, 0, sizeof(*h));
    bitreader_read_ue(&br);                           /* first_mb_in_slice */
    bitreader_read_ue(&br);                           /* slice_type */
    bitreader_read_ue(&br);                           /* pps id */
    bitreader_read_bits(&br, pc->log2_max_frame_num);
    bitreader_read_ue(&br);                           /* idr_pic_id */
    if (pc->pic_order_cnt_type == 0) bitreader_read_bits(&br, pc->log2_max_pic_order_cnt_lsb);
    bitreader_read_bits(&br, 2);                      /* no_output_of_prior_pics, long_term_ref */
    h->qp_delta = bitreader_read_se(&br);
    if (pc->deblocking_filter_control_present_flag) {
        h->dbf_idc = bitreader_read_ue(&br);
        if (h->dbf_idc != 1) {
            h->alpha = bitreader_read_se(&br);
            h->beta = bitreader_read_se(&br);
        }
    }
    h->mb_start = bitreader_get_bit_position(&br);
}

static void write_tail_fields(BitWriter *bw, const ComposerConfig *wc, const IdrHeader *h)
{
    bitwriter_write_se(bw, h->qp_delta);
    if (wc->deblocking_filter_control_present_flag) {
        bitwriter_write_ue(bw, h->dbf_idc);
        if (h->dbf_idc != 1) {
            bitwriter_write_se(bw, h->alpha);
            bitwriter_write_se(bw, h->beta);
        }
    }
}

/* Bulk copy of src bits [from, 8n) onto bw: byte-wise funnel shifts instead
 * of the reference's bit-serial copy_bits (:228-240); same result. */
static void copy_tail_bits(BitWriter *bw, const uint8_t *src, size_t n, size_t from)
{
    size_t total = n * 8;
    if (from >= total) return;
    size_t lead = (8 - (from & 7)) & 7;
    if (lead > total - from) lead = total - from;
    if (lead) bitwriter_write_bits(bw, src[from >> 3] & ((1u << lead) - 1u), (int)lead);
    size_t pos = from + lead;
    if (bw->bit_pos == 0) {
        size_t nb = (total - pos) >> 3;
        if (bw->byte_pos + nb > bw->capacity) {
            fprintf(stderr, "libh264scroll: BitWriter overflow\n");
            abort();
        }
        memcpy(bw->buffer + bw->byte_pos, src + (pos >> 3), nb);
        bw->byte_pos += nb;
        pos += nb * 8;
    } else {
        for (; pos + 8 <= total; pos += 8) bitwriter_write_bits(bw, src[pos >> 3], 8);
    }
    if (pos < total) bitwriter_write_bits(bw, src[pos >> 3] >> (8 - (total - pos)), (int)(total - pos));
}

size_t h264_rewrite_idr_frame(NALWriter *nw, ComposerConfig *write_cfg, ComposerConfig *parse_cfg,
                              const uint8_t *rbsp, size_t rbsp_size)
{
    IdrHeader h;
    parse_idr_header(rbsp, rbsp_size, parse_cfg, &h);
    size_t cap = rbsp_size + 256;
    uint8_t *out = (uint8_t *)malloc(cap);
    BitWriter bw;
    bitwriter_init(&bw, out, cap);
    bitwriter_write_ue(&bw, 0);
    bitwriter_write_ue(&bw, SLICE_TYPE_I_ALL);
    bitwriter_write_ue(&bw, 0);
    bitwriter_write_bits(&bw, 0, write_cfg->log2_max_frame_num);
    bitwriter_write_ue(&bw, (uint32_t)write_cfg->idr_pic_id);
    if (write_cfg->pic_order_cnt_type == 0)
        bitwriter_write_bits(&bw, 0, write_cfg->log2_max_pic_order_cnt_lsb);
    bitwriter_write_bits(&bw, 1, 2);                  /* no_output_of_prior 0, long_term_ref 1 */
    write_tail_fields(&bw, write_cfg, &h);
    copy_tail_bits(&bw, rbsp, rbsp_size, h.mb_start);
    size_t n = nal_write_unit(nw, NAL_REF_IDC_HIGHEST, NAL_TYPE_IDR, out, bitwriter_get_size(&bw), 1);
    free(out);
    write_cfg->frame_num = 1;
    return n;
}

size_t h264_rewrite_as_non_idr_i_frame(NALWriter *nw, ComposerConfig *write_cfg,
                                       ComposerConfig *parse_cfg, const uint8_t *rbsp,
                                       size_t rbsp_size, int frame_num)
{
    IdrHeader h;
    parse_idr_header(rbsp, rbsp_size, parse_cfg, &h);
    size_t cap = rbsp_size + 256;
    uint8_t *out = (uint8_t *)malloc(cap);
    BitWriter bw;
    bitwriter_init(&bw, out, cap);
    bitwriter_write_ue(&bw, 0);
    bitwriter_write_ue(&bw, SLICE_TYPE_I_ALL);
    bitwriter_write_ue(&bw, 0);
    bitwriter_write_bits(&bw, (uint32_t)frame_num, write_cfg->log2_max_frame_num);
    if (write_cfg->pic_order_cnt_type == 0)
        bitwriter_write_bits(&bw, (uint32_t)(frame_num * 2), write_cfg->log2_max_pic_order_cnt_lsb);
    bitwriter_write_bit(&bw, 1);                      /* adaptive_ref_pic_marking */
    bitwriter_write_ue(&bw, 4);                       /* MMCO 4: max LT idx + 1 = 2 */
    bitwriter_write_ue(&bw, 2);
    bitwriter_write_ue(&bw, 6);                       /* MMCO 6: this picture -> LT idx 1 */
    bitwriter_write_ue(&bw, 1);
    bitwriter_write_ue(&bw, 0);                       /* end */
    write_tail_fields(&bw, write_cfg, &h);
    copy_tail_bits(&bw, rbsp, rbsp_size, h.mb_start);
    size_t n = nal_write_unit(nw, NAL_REF_IDC_HIGHEST, NAL_TYPE_SLICE, out, bitwriter_get_size(&bw), 1);
    free(out);
    write_cfg->frame_num = frame_num + 1;
    return n;
}

/* ---------------- waypoint bookkeeping (host; reference :666-676) ---------------- */
int h264_needs_waypoint(ComposerConfig *cfg, int offset_px)
{
    if (offset_px == 0 || offset_px % MV_LIMIT_PX != 0) return 0;
    for (int i = 0; i < cfg->num_waypoints; ++i)
        if (cfg->waypoints[i].valid && cfg->waypoints[i].offset_px == offset_px) return 0;
    return 1;
}

/* ---------------- HOT PATH: GPU ---------------- */
static size_t gpu_write(NALWriter *nw, ComposerConfig *cfg, int kind, int offset_px)
{
    NalDesc d;
    memset(&d, 0, sizeof(d));
    d.kind = (uint8_t)kind;
    d.off = offset_px;
    d.frame_num = cfg->frame_num;
    d.nwp = (uint8_t)(cfg->num_waypoints < 0 ? 0 : cfg->num_waypoints);
    size_t written = 0;
    int rc = scroll_engine_write_nals(cfg, &d, 1, nw->output + nw->output_pos,
                                      nw->output_capacity - nw->output_pos, &written);
    if (rc != SCROLL_OK) {
        fprintf(stderr, "libh264scroll: %s failed on the GPU path: %s\n",
                kind ? "h264_write_waypoint_p_frame" : "h264_write_scroll_p_frame",
                scroll_last_error());
        abort();
    }
    nw->output_pos += written;
    return written;
}

size_t h264_write_scroll_p_frame(NALWriter *nw, ComposerConfig *cfg, int offset_px)
{
    size_t n = gpu_write(nw, cfg, 0, offset_px);
    cfg->frame_num++;                                 /* :662 */
    return n;
}

size_t h264_write_waypoint_p_frame(NALWriter *nw, ComposerConfig *cfg, int offset_px)
{
    size_t n = gpu_write(nw, cfg, 1, offset_px);
    if (cfg->num_waypoints < MAX_WAYPOINTS) {         /* :772-777 */
        WaypointInfo *w = &cfg->waypoints[cfg->num_waypoints];
        w->offset_px = offset_px;
        w->long_term_idx = 2 + cfg->num_waypoints;
        w->valid = 1;
        cfg->num_waypoints++;
    }
    cfg->frame_num++;
    return n;
}
