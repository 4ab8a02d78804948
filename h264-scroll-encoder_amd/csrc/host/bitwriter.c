/*
 * bitwriter.c -- host BitWriter / BitReader (ABI of include/bitwriter.h).
 *
 * Behaviour of the reference src/bitwriter.c:5-224 (same struct state after
 * every call, same capacity aborts), written as chunked bit insertion rather
 * than a bit-at-a-time loop.  Used by the cold paths (SPS/PPS, I-frame
 * rewrite) and by callers that build their own NAL units; the P-slice hot
 * path is generated on the GPU and never comes through here.
 */
#include "bitwriter.h"

#include <stdio.h>
#include <stdlib.h>

static void bw_fail(const char *what)
{
    fprintf(stderr, "libh264scroll: BitWriter %s\n", what);
    abort();                                   /* reference: assert() */
}

void bitwriter_init(BitWriter *bw, uint8_t *buffer, size_t capacity)
{
    bw->buffer = buffer;
    bw->capacity = capacity;
    bw->byte_pos = 0;
    bw->bit_pos = 0;
    bw->current_byte = 0;
}

/* append the low n bits of v (n <= 32), MSB first */
static void bw_append(BitWriter *bw, uint32_t v, int n)
{
    while (n > 0) {
        int room = 8 - bw->bit_pos;
        int take = n < room ? n : room;
        uint32_t chunk = (v >> (n - take)) & ((1u << take) - 1u);
        bw->current_byte = (uint8_t)((bw->current_byte << take) | chunk);
        bw->bit_pos += take;
        n -= take;
        if (bw->bit_pos == 8) {
            if (bw->byte_pos >= bw->capacity) bw_fail("overflow");
            bw->buffer[bw->byte_pos++] = bw->current_byte;
            bw->current_byte = 0;
            bw->bit_pos = 0;
        }
    }
}

void bitwriter_write_bit(BitWriter *bw, int bit)
{
    bw_append(bw, (uint32_t)(bit & 1), 1);
}

void bitwriter_write_bits(BitWriter *bw, uint32_t value, int n)
{
    if (n < 1 || n > 32) bw_fail("write_bits: n out of 1..32");
    bw_append(bw, value, n);
}

void bitwriter_write_ue(BitWriter *bw, uint32_t value)
{
    if (value == 0) {
        bw_append(bw, 1, 1);
        return;
    }
    uint32_t x = value + 1u;             /* wraps to 0 for 0xFFFFFFFF, as the reference */
    int m = 0;
    for (uint32_t t = x; t > 1; t >>= 1) m++;
    if (m) bw_append(bw, 0, m);
    bw_append(bw, x, m + 1);
}

void bitwriter_write_se(BitWriter *bw, int32_t value)
{
    uint32_t k = value > 0 ? 2u * (uint32_t)value - 1u : (uint32_t)(-2 * (int64_t)value);
    bitwriter_write_ue(bw, k);
}

void bitwriter_write_trailing_bits(BitWriter *bw)
{
    bw_append(bw, 1, 1);
    if (bw->bit_pos) bw_append(bw, 0, 8 - bw->bit_pos);
}

void bitwriter_flush(BitWriter *bw)
{
    if (bw->bit_pos > 0) {
        if (bw->byte_pos >= bw->capacity) bw_fail("overflow");
        bw->buffer[bw->byte_pos++] = (uint8_t)(bw->current_byte << (8 - bw->bit_pos));
        bw->current_byte = 0;
        bw->bit_pos = 0;
    }
}

size_t bitwriter_get_size(BitWriter *bw)
{
    /* pads the partial byte in place without advancing (reference :124-131) */
    if (bw->bit_pos > 0)
        bw->buffer[bw->byte_pos] = (uint8_t)(bw->current_byte << (8 - bw->bit_pos));
    return bw->byte_pos + (bw->bit_pos > 0 ? 1 : 0);
}

size_t bitwriter_get_bit_position(BitWriter *bw)
{
    return bw->byte_pos * 8 + (size_t)bw->bit_pos;
}

int bitwriter_is_byte_aligned(BitWriter *bw)
{
    return bw->bit_pos == 0;
}

/* ---------------- reader (reference :145-224) ---------------- */
void bitreader_init(BitReader *br, const uint8_t *buffer, size_t size)
{
    br->buffer = buffer;
    br->size = size;
    br->byte_pos = 0;
    br->bit_pos = 0;
}

int bitreader_read_bit(BitReader *br)
{
    if (br->byte_pos >= br->size) return 0;     /* EOF reads as 0 */
    int bit = (br->buffer[br->byte_pos] >> (7 - br->bit_pos)) & 1;
    if (++br->bit_pos == 8) {
        br->bit_pos = 0;
        br->byte_pos++;
    }
    return bit;
}

uint32_t bitreader_read_bits(BitReader *br, int n)
{
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | (uint32_t)bitreader_read_bit(br);
    return v;
}

uint32_t bitreader_read_ue(BitReader *br)
{
    int lz = 0;
    while (bitreader_read_bit(br) == 0 && lz < 32) lz++;
    if (lz == 0) return 0;
    return (1u << lz) - 1u + bitreader_read_bits(br, lz);
}

int32_t bitreader_read_se(BitReader *br)
{
    uint32_t k = bitreader_read_ue(br);
    return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
}

size_t bitreader_get_bit_position(BitReader *br)
{
    return br->byte_pos * 8 + (size_t)br->bit_pos;
}

int bitreader_is_byte_aligned(BitReader *br)
{
    return br->bit_pos == 0;
}

size_t bitreader_get_remaining_bytes(BitReader *br)
{
    return br->bit_pos ? br->size - br->byte_pos - 1 : br->size - br->byte_pos;
}

const uint8_t *bitreader_get_pointer(BitReader *br)
{
    return br->buffer + br->byte_pos;
}
