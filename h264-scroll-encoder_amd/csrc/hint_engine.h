/*
 * hint_engine.h -- host-side launcher of the UI-hint stage kernel
 * (hint_kernels.hip); the batch (scroll_kernels.hip) drives it between the
 * plan's state and size passes, like the dynamic-rect coder.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "engine.h"

#define HINT_MAX_MBW 240            /* MBs per row k_hint_stage's motion ring holds (3840 px) */

/* 0, or -1 when the launch failed */
int hint_launch_stage(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                      int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                      const HintFrame *hf, const ScrollHintRect *pool, uint8_t *stage,
                      uint64_t slot_bytes);
/* the conventional-encode fallback: frames whose hints name a reference the
 * frame lacks get HintFrame.mode |= HINT_MODE_FB (the others have it cleared) */
int hint_launch_fb(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal, int ld_nal,
                   const PlanPending *pend, const DynFrame *dfr, int ld_fr, HintFrame *hf,
                   const ScrollHintRect *pool);
/* staging bytes per frame that no hinted NAL of an mbw x mbh picture exceeds */
size_t hint_slot_bound(int mbw, int mbh);
