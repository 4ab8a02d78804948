/*
 * verify_oracle.h -- CPU ORACLE (test infrastructure only): whole-step
 * checkers for the benchmarked workloads.  Used by tests/ (parity at the
 * benchmarked scale) and by bench.py after its timed region (the "verified"
 * field of the bench line); the product never links it.
 *
 * A bench step composes the same F offsets per stream again and again (the
 * arenas are rewound, the stream state -- frame_num, waypoints -- carries
 * on), so the bytes of the k-th pass depend on the state the k-1 earlier
 * passes left.  or_compose_state advances that state without writing a
 * byte (a restatement of the state side of src/composer.c:255-264 and
 * src/h264_writer.c:662,666-676,772-777; tests check it against or_compose).
 */
#ifndef VERIFY_ORACLE_H
#define VERIFY_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "dyn_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

/* the state change of or_compose(.., c, off, mode, ..) without its bytes */
void or_compose_state(or_cfg *c, int off, int mode);

/* S streams, stream s starting from cfgs[s] (advanced in place):
 * `passes` compositions of the F offsets offs[s * F .. s * F + F); the
 * bytes of the last pass go to out + s * stride, their count to sizes[s].
 * r == NULL or r->w == 0: P-only (or_compose); else or_compose_dyn with the
 * synthetic source of dyn_oracle.h for stream stream_base + s, frame t0 + f,
 * and reference pictures R[s] (R_shared when R == NULL).  nthreads pthreads
 * over the streams.  Returns 0, or -1 when a stream's bytes exceed stride. */
int or_verify_compose(int S, int F, or_cfg *cfgs, const int32_t *offs, int mode,
                      const or_dyn_rect *r, int stream_base, int t0, const or_refs *const *R,
                      const or_refs *R_shared, int passes, uint8_t *out, size_t stride,
                      size_t *sizes, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
