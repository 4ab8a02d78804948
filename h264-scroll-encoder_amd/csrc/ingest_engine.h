/*
 * ingest_engine.h -- device-side types and launcher of the stream ingest
 * (ingest_kernels.hip): batched composer_init + composer_write_header.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "engine.h"

#define ING_SC_MAX 64               /* 00 00 01 patterns kept per reference file */

enum {
    ING_OK = 0,
    ING_ERR_MISSING = 1,            /* no SPS / PPS / IDR (composer.c:116-120)   */
    ING_ERR_PARSE = 2,              /* parse_sps / parse_pps refused the file    */
    ING_ERR_DIMS = 3,               /* A and B differ in size (composer.c:177)   */
    ING_ERR_NALS = 4,               /* more than ING_SC_MAX NAL units in a file  */
    ING_ERR_OVERFLOW = 5,           /* the header does not fit the arena         */
    ING_ERR_WAIT = 6,               /* a segment waited too long for an earlier one (k_ing_seg) */
};

typedef struct {
    uint64_t off, size;             /* bytes of the file in the input buffer     */
} IngestFile;

typedef struct {
    uint32_t n;                     /* patterns found (may exceed ING_SC_MAX)    */
    uint32_t pos[ING_SC_MAX];
} IngestScan;

typedef struct {
    int32_t err;                    /* ING_*                                     */
    int32_t w, h, deblock;          /* stream config from reference A            */
    uint64_t bytes;                 /* header bytes written to the arena         */
} IngestOut;

/* files[2 k], files[2 k + 1] = reference A, B of new stream first_stream + k;
 * header bytes at the start of its arena.  0, or -1 when a launch failed. */
int ingest_launch(hipStream_t hs, const uint8_t *in, const IngestFile *files, int nstreams,
                  uint64_t max_file, IngestScan *scan, IngestOut *outs, uint8_t *arena,
                  uint64_t ld_arena, uint64_t cap, int first_stream, void *work, size_t work_bytes, int mode);
/* the segmented path's passes: one (summary, placement and write in one
 * workgroup per segment, the default), or round 4's three -- summary, serial
 * placement per stream, write -- whose write pass reads the summary pass's
 * output bytes back (staged) or decodes the segment again */
enum { ING_ONEPASS = 0, ING_STAGED = 1, ING_RECOMPUTE = 2 };
/* device scratch of the segmented path (work; nullptr: one workgroup per
 * stream) for mode ING_* */
size_t ingest_work_bytes(int nstreams, uint64_t max_file, int mode);

/* mid-stream long-term reference updates (k_ing_update): files[k] -> a
 * non-IDR I frame of stream ups[2 k] marked long-term ups[2 k + 1],
 * appended at its cursor (streams distinct).  0, or -1 when a launch failed. */
int update_launch(hipStream_t hs, const uint8_t *in, const IngestFile *files, int n, uint64_t max_file,
                  IngestScan *scan, const int32_t *ups, IngestOut *outs, DevStream *st, uint8_t *arena,
                  uint64_t ld_arena);
