/*
 * bitwriter.h -- drop-in for the reference's include/bitwriter.h (:17-91).
 *
 * Same types, same field order and same signatures, so code compiled against
 * the reference header links against libh264scroll.so unchanged.  These are
 * HOST utility entry points (the composer's cold paths and any caller that
 * builds its own NAL units use them); the P-frame hot path never goes through
 * them -- it is generated on the GPU (see composer_batch.h).
 */
#ifndef BITWRITER_H
#define BITWRITER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reference include/bitwriter.h:17-23 */
typedef struct {
    uint8_t *buffer;        /* destination bytes                          */
    size_t capacity;        /* destination size                           */
    size_t byte_pos;        /* completed bytes                            */
    int bit_pos;            /* bits held in current_byte (0..7)           */
    uint8_t current_byte;   /* byte under construction, MSB first         */
} BitWriter;

void bitwriter_init(BitWriter *bw, uint8_t *buffer, size_t capacity);      /* :26 */
void bitwriter_write_bits(BitWriter *bw, uint32_t value, int n);           /* :29, n in 1..32 */
void bitwriter_write_bit(BitWriter *bw, int bit);                          /* :32 */
void bitwriter_write_ue(BitWriter *bw, uint32_t value);                    /* :35 */
void bitwriter_write_se(BitWriter *bw, int32_t value);                     /* :38 */
void bitwriter_write_trailing_bits(BitWriter *bw);                         /* :41 */
void bitwriter_flush(BitWriter *bw);                                       /* :44 */
size_t bitwriter_get_size(BitWriter *bw);                                  /* :47 */
size_t bitwriter_get_bit_position(BitWriter *bw);                          /* :50 */
int bitwriter_is_byte_aligned(BitWriter *bw);                              /* :53 */

/* reference include/bitwriter.h:59-64 */
typedef struct {
    const uint8_t *buffer;
    size_t size;
    size_t byte_pos;
    int bit_pos;
} BitReader;

void bitreader_init(BitReader *br, const uint8_t *buffer, size_t size);    /* :67 */
uint32_t bitreader_read_bits(BitReader *br, int n);                        /* :70 */
int bitreader_read_bit(BitReader *br);                                     /* :73 */
uint32_t bitreader_read_ue(BitReader *br);                                 /* :76 */
int32_t bitreader_read_se(BitReader *br);                                  /* :79 */
size_t bitreader_get_bit_position(BitReader *br);                          /* :82 */
int bitreader_is_byte_aligned(BitReader *br);                              /* :85 */
size_t bitreader_get_remaining_bytes(BitReader *br);                       /* :88 */
const uint8_t *bitreader_get_pointer(BitReader *br);                       /* :91 */

#ifdef __cplusplus
}
#endif
#endif /* BITWRITER_H */
