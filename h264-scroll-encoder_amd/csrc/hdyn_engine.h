/*
 * hdyn_engine.h -- host-side launcher of the dynamic rect under UI hints
 * (hdyn_kernels.hip).  The batch runs k_hdyn_code between the plan's state
 * pass and k_splice_stage, which composes the rect's MBs like spliced ones.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "engine.h"
#include "splice_engine.h"

#define HDYN_MB_WORDS_MAX 512       /* body words per MB the coder's LDS holds     */
#define HDYN_MB_WORDS_MIN 16        /* an explicit slot_bytes: 64 bytes and up      */
#define HDYN_MB_WORDS_DEFAULT 128   /* slot_bytes 0: 512 bytes per MB (noise against
                                     * +-255 residuals needs ~420 on average)        */
#define HDYN_STATUS_OVERFLOW 100    /* SpliceFrame.status: an MB outgrew its region */

/* 0, or -1 when the launch failed.  rec: w h records per frame from
 * SpliceFrame.rec_first; rbsp: mb_words words per MB from rbsp_word */
int hdyn_launch_code(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal,
                     int ld_nal, const PlanPending *pend, const DynFrame *dfr, int ld_fr,
                     const HintFrame *hf, const ScrollHintRect *pool, SpliceFrame *spf,
                     const DynGeom *g, const uint8_t *src, const uint8_t *refs, SpliceMbRec *rec,
                     uint32_t *rbsp, uint32_t mb_words);
