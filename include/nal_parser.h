/*
 * nal_parser.h -- drop-in for the reference's include/nal_parser.h (:13-56).
 * Annex-B ingest used by composer_init (host, once per stream).
 */
#ifndef NAL_PARSER_H
#define NAL_PARSER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reference include/nal_parser.h:13-19 */
typedef struct {
    int nal_ref_idc;
    int nal_unit_type;
    const uint8_t *data;    /* payload after the NAL header byte */
    size_t size;            /* payload size (EBSP)               */
    size_t rbsp_size;       /* not filled by nal_parser_next (as in the reference) */
} NALUnit;

/* reference include/nal_parser.h:21-25 */
typedef struct {
    const uint8_t *data;
    size_t size;
    size_t pos;
} NALParser;

void nal_parser_init(NALParser *parser, const uint8_t *data, size_t size);  /* :28 */
int nal_parser_next(NALParser *parser, NALUnit *unit);                       /* :31 */
size_t ebsp_to_rbsp(uint8_t *rbsp, const uint8_t *ebsp, size_t ebsp_size);   /* :34 */
int parse_sps(const uint8_t *rbsp, size_t size,
              int *width, int *height,
              int *log2_max_frame_num,
              int *pic_order_cnt_type,
              int *log2_max_pic_order_cnt_lsb);                              /* :41 */
int parse_pps(const uint8_t *rbsp, size_t size,
              int *num_ref_idx_l0_default_minus1,
              int *deblocking_filter_control_present_flag);                  /* :52 */

#ifdef __cplusplus
}
#endif
#endif /* NAL_PARSER_H */
