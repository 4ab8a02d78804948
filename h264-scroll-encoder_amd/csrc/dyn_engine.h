/*
 * dyn_engine.h -- engine-internal launchers of the dynamic-rect kernels
 * (dyn_kernels.hip), used by the batch engine (scroll_kernels.hip).
 */
#ifndef SCROLL_DYN_ENGINE_H
#define SCROLL_DYN_ENGINE_H

#include <hip/hip_runtime.h>
#include "engine.h"

/* all return 0, or -1 when the launch failed */
/* per-batch scratch of the dynamic-rect coder: prediction
 * rows (32 h u32 per NAL), block records of the general-path NALs
 * (DYN_PIECES per dynamic MB: a u16 meta and a 16-byte body; gen_cap NAL
 * slots taken per compose), row stage (+ spill slots) */
typedef struct {
    uint32_t *rows;
    uint16_t *meta;
    uint2 *body_lo, *body_hi;       /* record bodies: bits 0..63, bits 64..127 */
    uint4 *body_w;                  /* below QP_MIN: levels 8..15 (int16) of > 128-bit blocks */
    uint4 *heads;                   /* per frame: the 12 MB-head classes (k_dyn_rows -> k_dyn_row), HEAD_WORDS */
    unsigned long long *tcx;        /* k_dyn_row: per (frame, rect row, MB) bottom TotalCoeffs */
    uint32_t *rowstage;             /* per (frame, row group): its bits from bit 0 (rs_frame_words) */
    uint32_t *gbits;                /* per (frame, row group): its bit count */
    uint32_t *spill;                /* rs_spill_cap spill slots (rect rows over their slot) */
    uint32_t *ctr;                  /* per compose: [0] spill slots taken, [1] general records taken,
                                     * [2], [3] unused, [DYN_CTR_LIST + k] the frame (s ld_fr + f)
                                     * holding general record k */
    uint32_t ctr_frames;            /* frames the lists hold (S ld_fr) */
    uint32_t epoch;                 /* look-back epoch of the last compose (24 bits, never 0) */
} DynScratch;
#define DYN_HEAD_VECS 16             /* heads[] per frame: 12 classes MSB first, then their lengths */
#define DYN_CTR_LIST 4               /* ctr[]: the lists (the counters zeroed per compose: 4 words) */

/* a second HIP stream beside the block coder: after k_dyn_rows it takes the
 * general path (k_dyn_code_general, k_dyn_row<true>) and k_dyn_static, which
 * k_dyn_row<false> does not wait for; k_dyn_epfix waits for both (e1) */
typedef struct {
    hipStream_t side;
    hipEvent_t e0, e1;
} DynFork;
/* k_dyn_rows + k_dyn_code_general (records of the general-path NALs) +
 * k_dyn_row (every rect row: block coding + packing -> its row-stage bits);
 * fk != NULL: the fork above (k_dyn_static then runs on the side stream);
 * ev0 / ev1 != NULL: recorded right before / after k_dyn_row (the bench's
 * lite timing: that kernel alone) */
int dyn_launch_code(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                    int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                    const DynGeom *g, const uint8_t *src, const uint8_t *refs, const DynScratch *x,
                    uint32_t epoch, int mbw, uint64_t *stamps, const DynFork *fk, hipEvent_t ev0 = nullptr,
                    hipEvent_t ev1 = nullptr);
/* k_dyn_static (static row groups) + k_dyn_epfix: RBSP sizes and EP
 * positions (eps: DYN_OVF_BYTES per frame) straight from the row groups */
/* k_dyn_static alone (the static row groups: header, rows above / below the
 * rect).  (Measured in round 4: on a second HIP stream beside the block
 * coder, 1.69 against 1.67 ms per step -- no gain) */
int dyn_launch_static(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal, int ld_nal,
                      const PlanPending *pend, DynFrame *dfr, int ld_fr, const DynGeom *g, const DynScratch *x);
int dyn_launch_pack(hipStream_t hs, int nframes, int S, DevStream *st, const NalDesc *nal,
                    int ld_nal, const PlanPending *pend, DynFrame *dfr, int ld_fr,
                    const DynGeom *g, const DynScratch *x, uint8_t *eps, uint64_t *stamps, const DynFork *fk);
/* k_dyn_gather (k_dyn_emit_gather on the hint / splice path): x != NULL -- the dynamic rect (RBSP from
 * the row groups, EP lists in stage = eps); x == NULL -- the staged RBSP of
 * the hint / splice path (slot_bytes per frame, EP list in the slot tail) */
int dyn_launch_emit(hipStream_t hs, int nframes, int S, const DevStream *st, const NalDesc *nal,
                    int ld_nal, const DynFrame *dfr, int ld_fr, const DynGeom *g,
                    const uint8_t *stage, const DynScratch *x, uint8_t *arena, uint64_t ld_arena,
                    uint64_t *stamps);
int dyn_launch_synth(hipStream_t hs, int nframes, int S, uint8_t *src, const DynGeom *g,
                     int stream_base, int t0);

/* row-stage geometry (rs_* fields) of a rect in an mbw x mbh picture */
void dyn_rowstage_geom(DynGeom *g, int mbw, int mbh);
/* staging bytes per frame that no dynamic NAL can exceed */
size_t dyn_slot_bound(int mbw, int mbh, int rw, int rh);
/* EP positions kept per frame for an rw x rh MB rect on the rows' path
 * (DynGeom.ep_cap; the list buffer holds 4 ep_cap bytes per frame;
 * SCROLL_DEBUG_DYN_EPWIN: the large form on any rect) */
uint32_t dyn_ep_cap(int rw, int rh, int debug);

#endif
