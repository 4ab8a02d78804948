/*
 * nal.h -- drop-in for the reference's include/nal.h (:28-73).
 * Host utility entry points (header/IDR cold path, caller-built NALs).
 */
#ifndef NAL_H
#define NAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* NAL unit types, reference include/nal.h:10-15 */
#define NAL_TYPE_SLICE          1
#define NAL_TYPE_IDR            5
#define NAL_TYPE_SEI            6
#define NAL_TYPE_SPS            7
#define NAL_TYPE_PPS            8
#define NAL_TYPE_AUD            9

/* nal_ref_idc values, reference include/nal.h:20-23 */
#define NAL_REF_IDC_NONE        0
#define NAL_REF_IDC_LOW         1
#define NAL_REF_IDC_HIGH        2
#define NAL_REF_IDC_HIGHEST     3

/* reference include/nal.h:28-35 */
typedef struct {
    uint8_t *output;        /* Annex-B stream being appended to */
    size_t output_capacity;
    size_t output_pos;
    uint8_t *rbsp;          /* scratch RBSP buffer */
    size_t rbsp_capacity;
} NALWriter;

void nal_writer_init(NALWriter *nw, uint8_t *output, size_t output_capacity,
                     uint8_t *rbsp_temp, size_t rbsp_capacity);           /* :38 */
size_t nal_write_unit(NALWriter *nw, int nal_ref_idc, int nal_type,
                      const uint8_t *rbsp, size_t rbsp_size,
                      int use_long_startcode);                             /* :56 */
size_t nal_writer_get_size(NALWriter *nw);                                 /* :61 */
uint8_t *nal_writer_get_output(NALWriter *nw);                             /* :64 */
size_t rbsp_to_ebsp(uint8_t *ebsp, size_t ebsp_capacity,
                    const uint8_t *rbsp, size_t rbsp_size);                /* :72 */

#ifdef __cplusplus
}
#endif
#endif /* NAL_H */
