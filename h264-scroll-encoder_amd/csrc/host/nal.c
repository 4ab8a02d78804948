/*
 * nal.c -- host NAL framing utilities (ABI of include/nal.h).
 * Behaviour of the reference src/nal.c:5-92: Annex-B start code, header
 * byte (ref_idc << 5 | type), RBSP -> EBSP with 0x03 emulation prevention.
 * The GPU path applies the same framing inside its kernels.
 */
#include "nal.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void nal_fail(void)
{
    fprintf(stderr, "libh264scroll: NALWriter capacity exceeded\n");
    abort();                                   /* reference: assert() */
}

void nal_writer_init(NALWriter *nw, uint8_t *output, size_t output_capacity,
                     uint8_t *rbsp_temp, size_t rbsp_capacity)
{
    nw->output = output;
    nw->output_capacity = output_capacity;
    nw->output_pos = 0;
    nw->rbsp = rbsp_temp;
    nw->rbsp_capacity = rbsp_capacity;
}

size_t rbsp_to_ebsp(uint8_t *ebsp, size_t ebsp_capacity, const uint8_t *rbsp, size_t rbsp_size)
{
    size_t o = 0;
    unsigned zeros = 0;
    size_t i = 0;
    while (i < rbsp_size) {
        /* copy a run that cannot need a 0x03 in one go */
        if (zeros < 2) {
            const uint8_t *z = (const uint8_t *)memchr(rbsp + i, 0, rbsp_size - i);
            size_t run = z ? (size_t)(z - (rbsp + i)) : rbsp_size - i;
            if (run) {
                if (o + run > ebsp_capacity) nal_fail();
                memcpy(ebsp + o, rbsp + i, run);
                o += run;
                i += run;
                zeros = 0;
                continue;
            }
        }
        uint8_t v = rbsp[i++];
        if (zeros >= 2 && v <= 3) {
            if (o >= ebsp_capacity) nal_fail();
            ebsp[o++] = 3;
            zeros = 0;
        }
        if (o >= ebsp_capacity) nal_fail();
        ebsp[o++] = v;
        zeros = v ? 0 : zeros + 1;
    }
    return o;
}

size_t nal_write_unit(NALWriter *nw, int nal_ref_idc, int nal_type, const uint8_t *rbsp,
                      size_t rbsp_size, int use_long_startcode)
{
    size_t start = nw->output_pos;
    size_t sc = use_long_startcode ? 4 : 3;
    if (nw->output_pos + sc + 1 > nw->output_capacity) nal_fail();
    if (use_long_startcode) nw->output[nw->output_pos++] = 0;
    nw->output[nw->output_pos++] = 0;
    nw->output[nw->output_pos++] = 0;
    nw->output[nw->output_pos++] = 1;
    nw->output[nw->output_pos++] = (uint8_t)(((nal_ref_idc & 3) << 5) | (nal_type & 31));
    nw->output_pos += rbsp_to_ebsp(nw->output + nw->output_pos,
                                   nw->output_capacity - nw->output_pos, rbsp, rbsp_size);
    return nw->output_pos - start;
}

size_t nal_writer_get_size(NALWriter *nw)
{
    return nw->output_pos;
}

uint8_t *nal_writer_get_output(NALWriter *nw)
{
    return nw->output;
}
