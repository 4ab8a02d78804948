/*
 * scroll_kernels.hip -- MI355X (gfx950) engine of the many-stream scroll
 * composer: plan kernel (per-stream state machine + exact NAL sizes + output
 * offsets), emit kernel (random-access bit generation, 16 B per lane) and the
 * host-side batch engine behind include/composer_batch.h.
 *
 * Reference hot path: src/composer.c:255-264 -> src/h264_writer.c:541-782 ->
 * src/bitwriter.c -> src/nal.c:52-84.  See DESIGN.md for the data layout and
 * the roofline of each kernel.
 */
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "dyn_engine.h"
#include "hint_engine.h"
#include "splice_engine.h"
#include "hdyn_engine.h"
#include "ingest_engine.h"
#include "ipcm_engine.h"
#include "engine.h"
#include "scroll_device.h"

#include "dyn_device.h"

using namespace scroll;

static_assert(sizeof(DevStream) == 256, "DevStream must stay 256 B");
static_assert(sizeof(NalDesc) == 32, "NalDesc must stay 32 B");

namespace {

#ifndef SCROLL_TILE
#define SCROLL_TILE 16
#endif
#ifndef SCROLL_EMIT_WAVES
#define SCROLL_EMIT_WAVES 1
#endif
constexpr int TILE = SCROLL_TILE;              /* NAL units per wave tile in k_emit */
constexpr int EMIT_WAVES = SCROLL_EMIT_WAVES;  /* waves per k_emit workgroup        */
#ifndef SCROLL_PLAN_THREADS
#define SCROLL_PLAN_THREADS 1024   /* 16 waves: the NAL sizing pass is latency-bound */
#endif
constexpr int PLAN_THREADS = SCROLL_PLAN_THREADS;
constexpr int PLAN_REWIND = 1 << 8;   /* k_plan flag: arena restarts at 0 */
constexpr int PLAN_STATE = 1 << 9;    /* phase 1 only -> PlanPending (dynamic rect)   */
constexpr int PLAN_SIZE = 1 << 10;    /* phase 2 only, from PlanPending              */
constexpr int PLAN_DYN = 1 << 11;     /* scroll NALs carry the dynamic rect          */

/* ---------------------------------------------------------------------- */
/* helpers                                                                 */
/* ---------------------------------------------------------------------- */
__device__ inline uint64_t lanemask_lt()
{
    uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ inline uint64_t wave_incl_scan(uint64_t v, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ inline void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline NalCtx make_ctx(const int32_t *cfg, const int32_t *wo, const int32_t *wl,
                                  const int32_t *wv, const NalDesc &d)
{
    NalCtx c;
    c.w = cfg[0];
    c.h = cfg[1];
    c.log2_mfn = cfg[2];
    c.poc_type = cfg[3];
    c.log2_poc = cfg[4];
    c.deblock = cfg[5];
    c.kind = d.kind;
    c.off = d.off;
    c.frame_num = d.frame_num;
    c.nwp = d.nwp;
    c.wp_off = wo;
    c.wp_lt = wl;
    c.wp_valid = wv;
    return c;
}

/* ---------------------------------------------------------------------- */
/* k_plan: one workgroup per stream.                                       */
/*  phase 1 (wave 0): composer_write_scroll_frame state machine over the   */
/*          stream's offsets (src/composer.c:255-264, h264_writer.c:666-676,*/
/*          :772-777) -> one NalDesc per NAL unit, frame_num per NAL.       */
/*  phase 2 (all waves): exact size of every NAL (run layout, or the serial */
/*          path when emulation prevention / long codes are possible), and  */
/*          a block scan -> byte offset of every NAL in the stream arena.   */
/* With the dynamic rect the kernel runs twice around the dynamic coder: a  */
/* pass (PLAN_STATE: phase 1, totals + final table to PlanPending, frame -> */
/* scroll NAL map to DynFrame) and a size pass (PLAN_SIZE: phase 2, sizes   */
/* of dynamic NALs from DynFrame).                                          */
/* ---------------------------------------------------------------------- */
__global__ __launch_bounds__(PLAN_THREADS) void k_plan(DevStream *__restrict__ st,
                                                       const int32_t *__restrict__ offs,
                                                       int ld_off, NalDesc *__restrict__ nal,
                                                       int ld_nal, int nframes, int mode,
                                                       int flags, PlanPending *__restrict__ pend,
                                                       DynFrame *__restrict__ dfr, int ld_fr,
                                                       const uint32_t *__restrict__ pool_ctr = nullptr,
                                                       uint32_t spill_cap = 0, uint32_t gen_cap = 0,
                                                       uint32_t *__restrict__ ctr_zero = nullptr)
{
    const int s = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ int32_t s_cfg[8];
    __shared__ int32_t s_wo[8], s_wl[8], s_wv[8];
    __shared__ int32_t s_nnal, s_nwp_end, s_fn_end, s_nalwp;
    __shared__ uint64_t s_wsum[PLAN_THREADS / 64];
    __shared__ uint64_t s_carry;
    __shared__ int32_t s_nslow;

    DevStream *S = st + s;
    if (tid < 8) {
        s_wo[tid] = S->wp_off[tid];
        s_wl[tid] = S->wp_lt[tid];
        s_wv[tid] = S->wp_valid[tid];
    }
    /* the dynamic rect's per-compose counters (spill / record slots),
     * zeroed here rather than by a fill launch of their own */
    if (ctr_zero && s == 0 && tid < DYN_CTR_LIST) ctr_zero[tid] = 0u;
    if (tid == 0) {
        s_cfg[0] = S->w; s_cfg[1] = S->h; s_cfg[2] = S->log2_mfn; s_cfg[3] = S->poc_type;
        s_cfg[4] = S->log2_poc; s_cfg[5] = S->deblock; s_cfg[6] = S->frame_num; s_cfg[7] = S->nwp;
        s_carry = 0;
        s_nslow = 0;
        if ((flags & PLAN_REWIND) && !(flags & PLAN_STATE)) {
            S->out_pos = 0;
            S->undelivered = 0;
        }
        /* the dynamic rect ran out of a scratch pool somewhere in this
         * compose: no stream commits, so the same compose can be retried
         * once the batch has grown its pools */
        if ((flags & PLAN_SIZE) && pool_ctr && (pool_ctr[0] > spill_cap || pool_ctr[1] > gen_cap))
            S->err |= SCROLL_DEVERR_DYN;
    }
    const int F = nframes >= 0 ? nframes : S->frames;
    NalDesc *N = nal + (size_t)s * ld_nal;
    __syncthreads();
    const uint64_t out0 = S->out_pos;

    if (flags & PLAN_SIZE) {
        if (tid < 8) {
            s_wo[tid] = pend[s].wo[tid];
            s_wl[tid] = pend[s].wl[tid];
            s_wv[tid] = pend[s].wv[tid];
        }
        if (tid == 0) {
            s_nnal = pend[s].nnal;
            s_nwp_end = pend[s].nwp_end;
            s_fn_end = pend[s].fn_end;
            s_nalwp = pend[s].nalwp;
        }
    } else if (mode == SCROLL_PLAN_EXPLICIT) {
        if (tid == 0) {
            s_nnal = S->nnal;
            s_nwp_end = s_cfg[7];
            s_fn_end = s_cfg[6];
            s_nalwp = 0;
        }
    } else if (wave == 0) {
        /* waypoint table held in registers with static indices (no scratch) */
        int wo[8], wl[8], wv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            wo[k] = s_wo[k];
            wl[k] = s_wl[k];
            wv[k] = s_wv[k];
        }
        int n = s_cfg[7];
        const int fn0 = s_cfg[6];
        int nalc = 0, nalwp = 0;
        const int32_t *O = offs + (size_t)s * ld_off;
        for (int base = 0; base < F; base += 64) {
            int i = base + lane;
            bool valid = i < F;
            int off = valid ? O[i] : 0;
            bool cand = valid && off != 0 && (off % MVL) == 0;   /* h264_writer.c:667-668 */
            uint64_t mask = __ballot(cand);
            int my_n = n, has_wp = 0, wp_nb = 0;
            while (mask) {
                int jl = __ffsll((unsigned long long)mask) - 1;
                mask &= mask - 1;
                int offj = __shfl(off, jl, 64);
                bool need = true;
#pragma unroll
                for (int k = 0; k < 8; ++k)                       /* :670-674 */
                    if (k < n && wv[k] && wo[k] == offj) need = false;
                if (need) {
                    if (lane == jl) {
                        has_wp = 1;
                        wp_nb = n;
                    }
                    if (n < 8) {                                  /* :772-777 */
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if (k == n) {
                                wo[k] = offj;
                                wl[k] = 2 + n;
                                wv[k] = 1;
                            }
                        n++;
                    }
                    if (lane >= jl) my_n = n;
                }
            }
            uint64_t vmask = __ballot(valid), wmask = __ballot(has_wp != 0);
            uint64_t lt = lanemask_lt();
            if (mode == SCROLL_PLAN_COMPOSER) {
                int first = nalc + __popcll(vmask & lt) + __popcll(wmask & lt);
                if (valid) {
                    if (has_wp) {
                        NalDesc d{};
                        d.kind = 1; d.off = off; d.frame_num = fn0 + first; d.nwp = (uint8_t)wp_nb;
                        d.frame = (uint32_t)i;
                        N[first] = d;
                    }
                    NalDesc d{};
                    d.kind = 0; d.off = off; d.frame_num = fn0 + first + has_wp;
                    d.nwp = (uint8_t)my_n; d.frame = (uint32_t)i;
                    N[first + has_wp] = d;
                    if (flags & PLAN_DYN) dfr[(size_t)s * ld_fr + i].nal = first + has_wp;
                }
                nalc += __popcll(vmask) + __popcll(wmask);
            } else {   /* experiment: waypoint NAL replaces the scroll NAL */
                int idx = nalc + __popcll(vmask & lt);
                if (valid) {
                    NalDesc d{};
                    d.kind = has_wp ? 1 : 0; d.off = off; d.frame_num = fn0 + idx;
                    d.nwp = (uint8_t)(has_wp ? wp_nb : my_n); d.frame = (uint32_t)i;
                    N[idx] = d;
                    if (flags & PLAN_DYN) dfr[(size_t)s * ld_fr + i].nal = has_wp ? -1 : idx;
                }
                nalc += __popcll(vmask);
            }
            nalwp += __popcll(wmask);
        }
        if (lane < 8) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (k == lane) {
                    s_wo[k] = wo[k];
                    s_wl[k] = wl[k];
                    s_wv[k] = wv[k];
                }
        }
        if (lane == 0) {
            s_nnal = nalc;
            s_nwp_end = n;
            s_fn_end = fn0 + nalc;
            s_nalwp = nalwp;
        }
    }
    __syncthreads();
    if (flags & PLAN_STATE) {
        if (tid < 8) {
            pend[s].wo[tid] = s_wo[tid];
            pend[s].wl[tid] = s_wl[tid];
            pend[s].wv[tid] = s_wv[tid];
        }
        if (tid == 0) {
            pend[s].nnal = s_nnal;
            pend[s].nwp_end = s_nwp_end;
            pend[s].fn_end = s_fn_end;
            pend[s].nalwp = s_nalwp;
        }
        return;
    }

    /* phase 2: sizes + offsets.  Every NAL reads the FINAL table: entries are
     * only appended, and a NAL only looks at its first nwp entries. */
    const int nnal = s_nnal;
    for (int t = 0; t < nnal; t += PLAN_THREADS) {
        int j = t + tid;
        uint64_t sz = 0;
        int slow = 0;
        if (j < nnal) {
            NalDesc d = N[j];
            NalCtx c = make_ctx(s_cfg, s_wo, s_wl, s_wv, d);
            uint32_t fsz = 0;
            const bool dyn = (flags & PLAN_DYN) && d.kind == 0;
            bool fast = !dyn && !(flags & SCROLL_DEBUG_FORCE_SERIAL) && build_nal<false>(c, nullptr, &fsz);
            if (dyn) {
                const DynFrame df = dfr[(size_t)s * ld_fr + d.frame];
                sz = 5u + (uint64_t)df.rbsp_bytes + df.ep;     /* start code + header + EBSP */
                slow = 2;
            } else if (fast) {
                sz = fsz;
            } else {
                sz = serial_size(c);
                slow = 1;
            }
        }
        uint64_t inc = wave_incl_scan(sz, lane);
        if (lane == 63) s_wsum[wave] = inc;
        int ns = __popcll(__ballot(slow == 1));
        if (lane == 0 && ns) atomicAdd(&s_nslow, ns);
        __syncthreads();
        uint64_t before = s_carry;
        for (int w = 0; w < wave; ++w) before += s_wsum[w];
        if (j < nnal) {
            N[j].out_off = out0 + before + inc - sz;
            N[j].size = (uint32_t)sz;
            N[j].slow = (uint8_t)slow;
        }
        __syncthreads();
        if (tid == 0) {
            uint64_t tot = 0;
            for (int w = 0; w < PLAN_THREADS / 64; ++w) tot += s_wsum[w];
            s_carry += tot;
        }
        __syncthreads();
    }

    if (tid == 0) {
        uint64_t total = s_carry;
        S->n_slow = s_nslow;
        if (out0 + total > S->out_cap || (S->err & SCROLL_DEVERR_STAGED)) {
            if (!(S->err & SCROLL_DEVERR_STAGED))
                S->err |= SCROLL_DEVERR_OVERFLOW;   /* nothing committed, nothing emitted */
            S->nnal = 0;
            S->batch_bytes = 0;
        } else {
            S->out_pos = out0 + total;
            S->batch_bytes = total;
            S->undelivered += total;
            S->nnal = nnal;
            S->nal_wp = s_nalwp;
            S->frame_num = s_fn_end;
            S->nwp = s_nwp_end;
            if (mode != SCROLL_PLAN_EXPLICIT) S->frames_written += F;
        }
    }
    if (tid < 8 && mode != SCROLL_PLAN_EXPLICIT && out0 + s_carry <= S->out_cap &&
        !(S->err & SCROLL_DEVERR_STAGED)) {
        S->wp_off[tid] = s_wo[tid];
        S->wp_lt[tid] = s_wl[tid];
        S->wp_valid[tid] = s_wv[tid];
    }
}

/* ---------------------------------------------------------------------- */
/* k_emit: one wave per tile of TILE consecutive NAL units of one stream.   */
/*                                                                          */
/* Rule: every 128-byte line of an arena is written whole, by one wave, in  */
/* one pass.  A line written in pieces at different times (16- to 64-byte   */
/* holes filled later) costs the memory system up to 2x (DESIGN.md §6,      */
/* tools/store_floor.hip).  So:                                             */
/*  1. lanes build the run layouts of the tile's NALs plus up to XB / XA    */
/*     neighbour NALs, which supply the bytes of the two seam lines the     */
/*     tile shares with the adjacent tiles;                                 */
/*  2. the wave's chunk range covers whole lines [line(B0), line(B1)).      */
/*     Chunks are classified into PURE entries (runs of chunks inside one   */
/*     periodic run) and MIXED entries (runs of chunks holding NAL headers, */
/*     run boundaries, NAL boundaries, seam bytes);                         */
/*  3. mixed chunks are computed, one lane each, into LDS;                  */
/*  4. one pass streams every chunk of the range in order, 4 groups of 64   */
/*     chunks per iteration: each lane finds its entry (entry-start flag    */
/*     map + mbcnt), pulls the entry data by ds_bpermute and either expands */
/*     the run pattern at its phase or copies its mixed words from LDS.     */
/* Seam lines: both neighbours compute the identical full line and write    */
/* it (benign duplicate); a side whose neighbour bytes cannot be computed   */
/* here (serial-path or too many tiny neighbour NALs) writes only its own   */
/* bytes of that line.  A stream's first tile in a launch merges the line   */
/* head from memory (the previous compose's bytes); its last tile zero-     */
/* fills its line tail (arena slack).  Tiles holding a serial-path NAL use  */
/* the generic byte path and the owning lane writes that NAL serially;     */
/* dynamic-rect NALs (slow = 2) are written by k_dyn_gather.                */
/* ---------------------------------------------------------------------- */
constexpr int PURE_U = 4;         /* 64-chunk groups per stream iteration      */
constexpr int XB = SEAM_XB, XA = SEAM_XA;   /* neighbour layouts before / after the tile */
constexpr int NL = XB + TILE + XA;
constexpr int MAXPE = 8 * TILE;   /* pure + mixed entries per wave             */
constexpr int MAXMX = 6 * TILE;   /* mixed chunks per wave (~3-4 per NAL)      */
constexpr uint32_t PE_VS_MASK = (1u << 22) - 1;   /* chunks of a tile < 2^22   */
constexpr uint32_t PE_MIXED = 15u;                /* run field of a mixed entry */
static_assert(NL <= 64, "layout index is 6 bits and one lane builds each layout");
static_assert(PURE_U == 4, "the flag map packs 4 groups per lane dword");

struct EmitWaveLds {
    Lay lay[NL];
    int32_t noff[NL + 1];         /* layout i's first byte - B0 (signed)       */
    uint32_t pe_cb[MAXPE];        /* mixed entry: index of its first chunk in mw */
    uint32_t pe_vj[MAXPE];        /* first chunk (rel cs) | layout << 22 | run << 28 */
    uint32_t mx[MAXMX];           /* mixed chunk: (chunk rel cs) << 6 | first layout */
    alignas(16) uint32_t mw[MAXMX][4];   /* mixed chunk words, MSB first (ds_read_b128) */
    uint32_t flg[64];             /* stream loop: entry-start flags, byte 4 p + u
                                     = an entry starts at chunk v0 + 64 u + p   */
};

/* 16-B global store to an integer address (address space 1: a
 * global_store, not flat) */
__device__ inline void store_raw(uint64_t addr, const uint32_t o[4])
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) u32x4 gu32x4;
    u32x4 v;
    v.x = o[0];
    v.y = o[1];
    v.z = o[2];
    v.w = o[3];
    *reinterpret_cast<gu32x4 *>(addr) = v;
}

/* MSB-first words of a chunk whose bytes < first are outside this wave */
__device__ inline void store_bytes(uint8_t *A, uint64_t p, uint64_t lo, uint64_t hi,
                                   const uint32_t w[4])
{
    for (int k = 0; k < 16; ++k) {
        const uint64_t x = p + (uint64_t)k;
        if (x < lo || x >= hi) continue;
        A[x] = (uint8_t)(w[k >> 2] >> (24 - 8 * (k & 3)));
    }
}

__global__ __launch_bounds__(EMIT_WAVES * 64) void k_emit(const DevStream *__restrict__ st,
                                                          const NalDesc *__restrict__ nal,
                                                          int ld_nal, uint8_t *__restrict__ arena,
                                                          uint64_t ld_arena, int flags,
                                                          uint64_t *__restrict__ dbg)
{
    __shared__ EmitWaveLds s_w[EMIT_WAVES];
    __shared__ int32_t s_cfg[8], s_wo[8], s_wl[8], s_wv[8];
    __shared__ LenLut s_lut;

    const int s = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = (int)uni((uint32_t)(tid >> 6));      /* wave-uniform -> SGPR */
    const DevStream *S = st + s;
    const int t0 = (blockIdx.x * EMIT_WAVES + wave) * TILE;
    /* lane i <-> layout i <-> NAL t0 - XB + i.  Every start-up load in one
     * memory round trip: the descriptors (bounded by the descriptor
     * capacity; lanes past nnal are ignored below), the stream config and
     * its waypoint table. */
    const int ti = t0 - XB + lane;
    NalDesc d{};
    if (lane < NL && ti >= 0 && ti < ld_nal) d = nal[(size_t)s * ld_nal + ti];
    if (tid < 8) {
        s_wo[tid] = S->wp_off[tid];
        s_wl[tid] = S->wp_lt[tid];
        s_wv[tid] = S->wp_valid[tid];
    }
    if (tid == 0) {
        s_cfg[0] = S->w; s_cfg[1] = S->h; s_cfg[2] = S->log2_mfn; s_cfg[3] = S->poc_type;
        s_cfg[4] = S->log2_poc; s_cfg[5] = S->deblock;
    }
    if (tid < 64) lut_entry((uint32_t)tid + 1u, s_lut.magic[tid], s_lut.mods[tid]);
    const int nnal = S->nnal;
    __syncthreads();
    if (t0 >= nnal) return;
    const int cnt = min(TILE, nnal - t0);
    const int lo = max(0, XB - t0);                       /* first valid layout   */
    const int hi = XB + cnt + min(XA, nnal - t0 - cnt);   /* one past the last    */
    const LenLut &T = s_lut;
    EmitWaveLds &W = s_w[wave];
    const bool stamps = (flags & SCROLL_DEBUG_EMIT_STAMPS) && dbg;
    uint64_t *stamp = dbg + ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * EMIT_WAVES + wave) * 8;
    auto mark = [&](int k) {
        if (stamps) {
            uint64_t t = __builtin_amdgcn_s_memtime();
            if (lane == 0) stamp[k] = t;
        }
    };
    mark(0);
    if (stamps && lane == 0) stamp[5] = __builtin_amdgcn_s_memrealtime();
    Lay *L = W.lay;
    int32_t *noff = W.noff;
    uint8_t *A = arena + (size_t)s * ld_arena;

    /* 1. layouts (own NALs + neighbours) */
    const uint64_t B0 = ((uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)(d.out_off >> 32), XB) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)d.out_off, XB);
    const bool valid = lane >= lo && lane < hi;
    const bool own = lane >= XB && lane < XB + cnt;
    bool my_slow = false;
    NalCtx my_ctx;
    if (valid) {
        my_ctx = make_ctx(s_cfg, s_wo, s_wl, s_wv, d);
        my_slow = d.slow != 0;
        if (!my_slow) {
            uint32_t sz;
            build_nal<true, false>(my_ctx, &L[lane], &sz);   /* plan proved it fast */
        } else {
            L[lane].nal_bits = d.size * 8u;
            L[lane].used_bits = 0;
            L[lane].hdr_bits = 0;
            L[lane].nruns = 0;
        }
        noff[lane] = (int32_t)(int64_t)(d.out_off - B0);
        if (lane == hi - 1) noff[hi] = (int32_t)(int64_t)(d.out_off + d.size - B0);
    }
    const uint64_t slow_mask = __ballot(valid && my_slow);
    const bool any_slow = (slow_mask >> XB) & ((cnt == 64 ? 0ull : (1ull << cnt)) - 1ull) ? true : false;
    wave_lds_sync();
    mark(1);
    if (flags & SCROLL_DEBUG_EMIT_BUILD) return;

    const uint64_t B1 = B0 + (uint64_t)(int64_t)noff[XB + cnt];

    /* seam lines (scroll_device.h seam_plan): head bytes [line(B0), B0)
     * from memory (a stream's first tile) or from previous layouts; tail
     * bytes [B1, line end) zero (last tile) or from next layouts */
    const Seams z = seam_plan(B0, B1, t0, cnt, nnal, lo, hi, noff, slow_mask);
    const bool head_full = z.head_full, tail_full = z.tail_full;
    const uint64_t cs = z.cs, ce = z.ce;
    const uint64_t nch = ce - cs;

    /* 2. classify the owned chunks of every own NAL into entries */
    uint32_t npe = 0, nmx = 0;
    uint64_t own0 = 0, own1 = 0, Aj = 0;
    if (own && !my_slow) {
        owned_chunks(z, B0, noff, lane, cnt, own0, own1);
        Aj = 8 * (B0 + (uint64_t)(int64_t)noff[lane]);
        entry_walk(L[lane], Aj, own0, own1, [&](int r, uint64_t c0e, uint64_t c1e) {
            npe++;
            if (r < 0) nmx += (uint32_t)(c1e - c0e);
        });
    }
    const uint32_t pe_inc = (uint32_t)wave_incl_scan(npe, lane);
    const uint32_t mx_inc = (uint32_t)wave_incl_scan(nmx, lane);
    const uint32_t tot_pe = uni((uint32_t)__shfl(pe_inc, 63, 64));
    const uint32_t tot_mx = uni((uint32_t)__shfl(mx_inc, 63, 64));
    const bool generic = any_slow || (B1 - B0) >= (1ull << 26) || nch >= (1ull << 22) ||
                         tot_pe > (uint32_t)MAXPE || tot_mx > (uint32_t)MAXMX;

    if (!generic) {
        if (own) {
            uint32_t e = pe_inc - npe, m = mx_inc - nmx;
            entry_walk(L[lane], Aj, own0, own1, [&](int r, uint64_t c0e, uint64_t c1e) {
                W.pe_vj[e] = (uint32_t)(c0e - cs) | ((uint32_t)lane << 22) |
                             ((r < 0 ? PE_MIXED : (uint32_t)r) << 28);
                W.pe_cb[e] = m;
                e++;
                if (r < 0)
                    for (uint64_t c = c0e; c < c1e; ++c)
                        W.mx[m++] = ((uint32_t)(c - cs) << 6) | mixed_first(z, c << 4, B0, lane);
            });
        }
        wave_lds_sync();
        mark(2);

        /* 3. mixed chunks -> LDS (head chunks merge the bytes before B0 from
         * memory on the launch's first tile) */
        const int mix_hi = tail_full ? z.t_hi : XB + cnt;
        const uint32_t mx_end = (flags & SCROLL_DEBUG_EMIT_NOMIXED) ? 0u : tot_mx;
        for (uint32_t k = (uint32_t)lane; k < mx_end; k += 64) {
            const uint32_t mm = W.mx[k];
            const uint64_t p = (cs + (mm >> 6)) << 4;
            uint32_t w[4];
            mixed_chunk(L, noff, mix_hi, (int)(mm & 63u), ((int64_t)p - (int64_t)B0) * 8, T, w);
            if (z.head_rmw && p < B0) {
                const uint4 old = *reinterpret_cast<const uint4 *>(A + p);
                const uint32_t ow[4] = {__builtin_bswap32(old.x), __builtin_bswap32(old.y),
                                        __builtin_bswap32(old.z), __builtin_bswap32(old.w)};
                const int32_t nb = (int32_t)(B0 - p);          /* bytes kept, 1..15 */
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    w[q] |= ow[q] & range_mask(0, 8 * nb - 32 * q);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) W.mw[k][q] = w[q];
        }
        wave_lds_sync();
        mark(3);
        if (stamps && lane == 0) stamp[6] = ((uint64_t)nch << 32) | tot_mx;

        /* 4. stream.  Lane k of a window holds entry ebase + k: first chunk
         * vs (relative to cs), and for a pure entry K = run bit of chunk cs
         * (mod 2^32; chunk cs + v starts at run bit K + 128 v), code len,
         * magic, pattern192; for a mixed entry len = 0 and K + v = the mw
         * index of chunk cs + v. */
        uint32_t ebase = 0;
        uint32_t e_vs = 0xffffffffu, e_K = 0, e_len = 0, e_mag = 0, e_q[6] = {0, 0, 0, 0, 0, 0};
        auto load_window = [&](uint32_t base) {
            const uint32_t idx = base + (uint32_t)lane;
            e_vs = 0xffffffffu;
            if (idx < tot_pe) {
                const uint32_t vj = W.pe_vj[idx];
                const uint32_t vs = vj & PE_VS_MASK;
                const int j = (int)((vj >> 22) & 63u);
                const uint32_t r = vj >> 28;
                e_vs = vs;
                if (r == PE_MIXED) {
                    e_len = 0;
                    e_mag = 0;
                    e_K = W.pe_cb[idx] - vs;
#pragma unroll
                    for (int z = 0; z < 6; ++z) e_q[z] = 0;
                } else {
                    const Lay &Lj = L[j];
                    const uint32_t rs0 = r ? Lj.run_end[r - 1] : Lj.hdr_bits;
                    const uint64_t Arun = 8 * (B0 + (uint64_t)(int64_t)noff[j]) + rs0;
                    e_K = (uint32_t)((cs << 7) - Arun);        /* chunk cs + v: bit K + 128 v */
                    e_len = Lj.len[r];
                    e_mag = T.magic[e_len - 1];
                    pattern192(Lj.pat[r][0], Lj.pat[r][1], T.mods[e_len - 1], e_q);
                }
            }
        };
        /* the 4 words of chunk v from entry data (len 0 = mixed) */
        auto words = [&](uint32_t v, uint32_t K, uint32_t len, uint32_t mag, const uint32_t q[6],
                         uint32_t w[4]) {
            pure_words(K + (v << 7), len ? len : 1u, mag, q, w);
            if (__ballot(len == 0u)) {                  /* some lane in a mixed entry */
                const uint32_t mi = len ? 0u : min(K + v, (uint32_t)MAXMX - 1u);
                const uint4 mv = *reinterpret_cast<const uint4 *>(W.mw[mi]);
                w[0] = len ? w[0] : mv.x;
                w[1] = len ? w[1] : mv.y;
                w[2] = len ? w[2] : mv.z;
                w[3] = len ? w[3] : mv.w;
            }
        };
        const uint32_t nv = (flags & SCROLL_DEBUG_EMIT_NOPURE) ? 0u : (uint32_t)nch;
        const bool do_store = !(flags & SCROLL_DEBUG_EMIT_NOSTORE);
        if (nv) load_window(0);
        auto store4 = [&](uint32_t (&w)[PURE_U][4], const uint32_t (&vv)[PURE_U]) {
            if (do_store) {
                /* byte-swap all groups first and keep them live together, so
                 * the stores read distinct registers (no WAR stall behind a
                 * queued store) */
                uint32_t o[PURE_U][4];
#pragma unroll
                for (int u = 0; u < PURE_U; ++u)
#pragma unroll
                    for (int k = 0; k < 4; ++k) o[u][k] = __builtin_bswap32(w[u][k]);
                uint64_t ptr[PURE_U];
#pragma unroll
                for (int u = 0; u < PURE_U; ++u) {
                    ptr[u] = (uint64_t)(uintptr_t)A + ((cs + vv[u]) << 4);
                    asm volatile("" : "+v"(o[u][0]), "+v"(o[u][1]), "+v"(o[u][2]), "+v"(o[u][3]),
                                 "+v"(ptr[u]));
                }
#pragma unroll
                for (int u = 0; u < PURE_U; ++u) store_raw(ptr[u], o[u]);
                asm volatile("" ::"v"(o[PURE_U - 1][0]), "v"(ptr[0]));
            } else {
#pragma unroll
                for (int u = 0; u < PURE_U; ++u)
                    asm volatile("" ::"v"(w[u][0]), "v"(w[u][1]), "v"(w[u][2]), "v"(w[u][3]));
            }
        };

        for (uint32_t v0 = 0; v0 < nv; v0 += 64u * PURE_U) {
            const uint32_t vlast = min(v0 + 64u * PURE_U, nv) - 1u;
            uint64_t m = __ballot(e_vs <= vlast);
            if ((m >> 63) && ebase + 64 < tot_pe) {
                /* the window must hold every entry of the iteration */
                const uint32_t ks = ebase + (uint32_t)__popcll(__ballot(e_vs <= v0)) - 1u;
                if (ks != ebase) {
                    ebase = ks;
                    load_window(ebase);
                    m = __ballot(e_vs <= vlast);
                }
            }
            uint32_t w[PURE_U][4], vv[PURE_U];
            if ((m >> 63) && ebase + 64 < tot_pe) {
                /* > 64 entries in 256 chunks (tiny NALs): group by group,
                 * entry by entry, reloading the window as needed */
#pragma unroll
                for (int u = 0; u < PURE_U; ++u) {
                    const uint32_t v = min(v0 + 64u * (uint32_t)u + (uint32_t)lane, vlast);
                    vv[u] = v;
                    const uint32_t g = min(v0 + 64u * (uint32_t)u, vlast);
                    /* move the window to start at the entry holding g, so it
                     * holds all (<= 64) entries of the group */
                    for (;;) {
                        const uint64_t b = __ballot(e_vs <= g);
                        if (!(b >> 63) || ebase + 64 >= tot_pe) break;
                        ebase += 63;                      /* every entry starts <= g */
                        load_window(ebase);
                    }
                    const uint32_t ks = ebase + (uint32_t)__popcll(__ballot(e_vs <= g)) - 1u;
                    if (ks != ebase) {
                        ebase = ks;
                        load_window(ebase);
                    }
                    const uint32_t k0 = 0u;
                    const uint32_t k1 = (uint32_t)__popcll(__ballot(e_vs <= min(g + 63u, vlast))) - 1u;
                    uint32_t kk = k0;
                    for (uint32_t jb = k0 + 1; jb <= k1; ++jb)
                        kk += v >= (uint32_t)__builtin_amdgcn_readlane((int)e_vs, (int)jb) ? 1u : 0u;
                    const int src = (int)(kk << 2);
                    uint32_t q[6];
#pragma unroll
                    for (int z = 0; z < 6; ++z) q[z] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_q[z]);
                    words(v, (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_K),
                          (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_len),
                          (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_mag), q, w[u]);
                }
                store4(w, vv);
                continue;
            }
            const uint32_t ks0 = (uint32_t)__popcll(__ballot(e_vs <= v0)) - 1u;  /* window index */
            const bool starts = e_vs > v0 && e_vs <= vlast;
            if (__ballot(starts) == 0) {
                /* one entry covers the whole iteration: SGPR operands */
                const uint32_t K = (uint32_t)__builtin_amdgcn_readlane((int)e_K, (int)ks0);
                const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)e_len, (int)ks0);
                const uint32_t mag = (uint32_t)__builtin_amdgcn_readlane((int)e_mag, (int)ks0);
                uint32_t q[6];
#pragma unroll
                for (int z = 0; z < 6; ++z) q[z] = (uint32_t)__builtin_amdgcn_readlane((int)e_q[z], (int)ks0);
#pragma unroll
                for (int u = 0; u < PURE_U; ++u) {
                    vv[u] = min(v0 + 64u * (uint32_t)u + (uint32_t)lane, vlast);
                    words(vv[u], K, len, mag, q, w[u]);
                }
            } else {
                /* entry-start flags of the 4 groups -> per-lane entry index
                 * (window lane) by one ballot + mbcnt per group */
                W.flg[lane] = 0u;
                if (starts) {
                    const uint32_t rel = e_vs - v0;
                    reinterpret_cast<uint8_t *>(W.flg)[(rel & 63u) * 4u + (rel >> 6)] = 1;
                }
                wave_lds_sync();
                const uint32_t f4 = W.flg[lane];
                uint32_t base = ks0;
#pragma unroll
                for (int u = 0; u < PURE_U; ++u) {
                    const uint32_t fu = (f4 >> (8 * u)) & 255u;
                    const uint64_t B = __ballot(fu != 0u);
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(B >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)B, 0u));
                    const uint32_t kk = base + below + fu;
                    base += (uint32_t)__popcll(B);
                    vv[u] = min(v0 + 64u * (uint32_t)u + (uint32_t)lane, vlast);
                    const int src = (int)(kk << 2);
                    uint32_t q[6];
#pragma unroll
                    for (int z = 0; z < 6; ++z) q[z] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_q[z]);
                    words(vv[u], (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_K),
                          (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_len),
                          (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)e_mag), q, w[u]);
                }
            }
            store4(w, vv);
        }

        /* partial chunks of a seam line whose neighbour bytes are not
         * available here: own bytes only */
        if (!(flags & SCROLL_DEBUG_EMIT_NOBYTES)) {
            const bool ph = !head_full && (B0 & 15);
            const bool pt = !tail_full && (B1 & 15) && (B1 >> 4) >= cs;
            const uint64_t pc = lane == 0 ? (B0 >> 4) : (B1 >> 4);
            if ((lane == 0 && ph) || (lane == 1 && pt && !(ph && (B1 >> 4) == (B0 >> 4)))) {
                uint32_t w[4];
                mixed_chunk(L, noff, XB + cnt, XB, ((int64_t)(pc << 4) - (int64_t)B0) * 8, T, w);
                store_bytes(A, pc << 4, B0, B1, w);
            }
        }
    } else {
        /* generic byte path: the bytes of every own run-layout NAL, one
         * byte per lane; serial-path and dynamic-rect NALs are written by
         * their own writers (below / k_dyn_gather) */
        const Lay *Lo = L + XB;
        const int32_t *no = noff + XB;
        for (int jn = 0; jn < cnt; ++jn) {
            if ((slow_mask >> (XB + jn)) & 1ull) continue;
            const uint32_t r0 = (uint32_t)no[jn], r1 = (uint32_t)no[jn + 1];
            for (uint32_t rel = r0 + (uint32_t)lane; rel < r1; rel += 64) {
                int jj = jn;
                A[B0 + rel] = (uint8_t)tile_byte(Lo, no, cnt, jj, rel);
            }
        }
    }
    mark(4);
    if (stamps && lane == 0) {
        uint64_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);      /* HW_ID */
        uint64_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((15 << 11) | 20);    /* XCC_ID */
        stamp[7] = (__builtin_amdgcn_s_memrealtime() & 0xffffffffull) | (hw << 32);
        stamp[6] = (stamp[6] & 0x00ffffffffffffffull) | ((xcc & 0xff) << 56);
    }
    if (own && d.slow == 1) serial_write(my_ctx, A + d.out_off);
}

/* ---------------------------------------------------------------------- */
/* host engine                                                             */
/* ---------------------------------------------------------------------- */
thread_local char g_err[512];

void set_err(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            set_err("%s failed: %s", #x, hipGetErrorString(e_));                   \
            return SCROLL_ERR_HIP;                                                 \
        }                                                                          \
    } while (0)

int usable_devices(std::vector<int> *ids)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_err("no HIP device visible (libh264scroll needs an MI355X / gfx950)");
        return 0;
    }
    int ok = 0;
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) != hipSuccess) continue;
        if (strncmp(p.gcnArchName, "gfx950", 6) == 0) {
            ok++;
            if (ids) ids->push_back(i);
        }
    }
    if (!ok) set_err("no gfx950 device among %d HIP devices", n);
    return ok;
}

int check_cfg(const ComposerConfig *c)
{
    if (c->log2_max_frame_num < 1 || c->log2_max_frame_num > 16 ||
        (c->pic_order_cnt_type == 0 &&
         (c->log2_max_pic_order_cnt_lsb < 1 || c->log2_max_pic_order_cnt_lsb > 16)) ||
        c->num_waypoints < 0 || c->num_waypoints > MAX_WAYPOINTS || c->width < 0 ||
        c->height < 0) {
        set_err("unsupported ComposerConfig (log2 fields must be 1..16, num_waypoints 0..8)");
        return SCROLL_ERR_CONFIG;
    }
    return SCROLL_OK;
}

void cfg_to_dev(const ComposerConfig *c, DevStream *d)
{
    d->w = c->width;
    d->h = c->height;
    d->log2_mfn = c->log2_max_frame_num;
    d->poc_type = c->pic_order_cnt_type;
    d->log2_poc = c->log2_max_pic_order_cnt_lsb;
    d->deblock = c->deblocking_filter_control_present_flag;
    d->frame_num = c->frame_num;
    d->nwp = c->num_waypoints;
    for (int i = 0; i < 8; ++i) {
        d->wp_off[i] = c->waypoints[i].offset_px;
        d->wp_lt[i] = c->waypoints[i].long_term_idx;
        d->wp_valid[i] = c->waypoints[i].valid;
    }
}

void dev_to_cfg(const DevStream *d, ComposerConfig *c)
{
    c->frame_num = d->frame_num;
    c->num_waypoints = d->nwp;
    for (int i = 0; i < 8; ++i) {
        c->waypoints[i].offset_px = d->wp_off[i];
        c->waypoints[i].long_term_idx = d->wp_lt[i];
        c->waypoints[i].valid = d->wp_valid[i];
    }
}

}  // namespace

/* ======================================================================== */
/* ScrollBatch                                                              */
/* ======================================================================== */
constexpr int NEV = 7;
struct ScrollBatch {
    int device = 0;
    int mode = SCROLL_MODE_COMPOSER;
    int max_streams = 0, max_frames = 0, nstreams = 0;
    int debug = 0;
    size_t arena_bytes = 0, ld_arena = 0;
    int ld_nal = 0;
    DevStream *d_st = nullptr;
    DevStream *h_st = nullptr;
    int32_t *d_off = nullptr;
    NalDesc *d_nal = nullptr;
    uint8_t *d_arena = nullptr;
    hipStream_t own = nullptr;
    hipStream_t last = nullptr;
    hipEvent_t ev[NEV] = {};
    int timing = 0;
    int timed_pending = 0;
    float ms[6] = {0, 0, 0, 0, 0, 0};  /* plan, emit, dyn stage, dyn emit, dyn code, dyn pack */
    std::vector<hipEvent_t> ring;      /* NEV events per timed compose, pending */
    std::vector<uint8_t> ring_dyn;     /* per pending compose: 1 the dynamic-rect pipeline ran, 2 lite timing */
    int ev_dyn = 0;                    /* the same for b->ev */
    int ring_used = 0;
    double acc_ms[6] = {0, 0, 0, 0, 0, 0};
    int acc_n = 0;
    int host_valid = 1;
    int last_plan_mode = SCROLL_PLAN_COMPOSER;
    int last_nframes = 0;
    std::vector<NalDesc> nal_cache;
    int nal_cache_valid = 0;
    uint64_t *d_dbg = nullptr;
    size_t dbg_slots = 0;
    /* dynamic rect (configs 3-5) */
    PlanPending *d_pend = nullptr;
    int dyn_on = 0;
    int dyn_pw = 0, dyn_ph = 0;        /* picture size every stream must have      */
    int dyn_refs = 0;                  /* 0 unset, 1 shared pair, 2 per stream     */
    DynGeom geo{};
    DynFrame *d_dfr = nullptr;
    uint8_t *d_src = nullptr, *d_refs = nullptr, *d_stage = nullptr;
    DynScratch dx{};                   /* rows, block records, look-back words of the dynamic coder */
    /* UI hints: staged like the dynamic rect (shares
     * d_dfr, d_stage and geo.slot_bytes; the two are exclusive) */
    int hint_on = 0;
    int hint_dirty = 0;
    int hint_max_mb = 0;               /* MBs per picture the slots are sized for */
    std::vector<std::vector<ScrollHintRect>> h_hint;   /* [s * max_frames + f] */
    std::vector<int16_t> h_hint_mode;
    HintFrame *d_hf = nullptr;
    ScrollHintRect *d_pool = nullptr;
    size_t pool_cap = 0;
    /* pre-encoded MB splice: frames of the hint path
     * whose rect comes from an external slice */
    struct SpliceHost {
        int x0 = 0, y0 = 0, w = 0, h = 0;
        std::vector<uint8_t> nal;      /* host bytes (scroll_batch_set_splice)          */
        const uint8_t *dnal = nullptr; /* or device bytes (scroll_batch_set_splices_device) */
        size_t n = 0;
    };
    std::vector<SpliceHost> h_sp;      /* [s * max_frames + f]; w = 0: none */
    /* the dynamic rect under UI hints (hdyn_kernels.hip): with both on,
     * every frame's rect MBs are coded by k_hdyn_code into splice records
     * (d_sp_rec, word pool d_sp_rbsp) and composed by k_splice_stage */
    std::vector<int32_t> h_dyn_pos;    /* [2 (s * max_frames + f)]: rect origin, x0 < 0: none */
    int fallback = 0;                  /* scroll_batch_set_fallback: k_hint_fb before the stage kernels */
    DynFork fork{};                    /* SCROLL_DYN_FORK=1: the general path + static groups beside k_dyn_row */
    std::vector<int32_t> h_dyn_qp;     /* [s * max_frames + f]: the frame's rect QP under hints, -1: the stream's */
    int dyn_pos_custom = 0;            /* some frame's origin differs from the batch rect */
    int dyn_qp = 26;                   /* the rect's QP (scroll_batch_set_dyn_qp)          */
    int hd_dirty = 0;                  /* d_spf / HintFrame of the combined frames out of date */
    uint32_t hd_mb_words = 0;          /* pool words per rect MB */
    size_t dyn_cap = 0;                /* the dynamic rect's own staging cap (geo.slot_bytes without hints) */
    int sp_n = 0;                      /* spliced frames                           */
    int sp_dirty = 0;                  /* upload + parse before the next compose   */
    int sp_parse = 0;                  /* k_splice_parse pending                   */
    SpliceFrame *d_spf = nullptr;      /* [max_streams * max_frames]               */
    uint8_t *d_sp_nal = nullptr;
    uint32_t *d_sp_rbsp = nullptr;
    SpliceMbRec *d_sp_rec = nullptr;
    int32_t *d_sp_list = nullptr;
    SpliceUnit *d_sp_units = nullptr;  /* NAL unit slots (splice_unit_cap per frame) */
    int32_t *d_sp_lanes = nullptr;     /* lane list: count (zero between parses), (list index, unit) pairs */
    size_t sp_lanes_cap = 0, sp_nslots = 0;
    int sp_ymax = 1;                   /* most unit slots of a frame (parse grid y)  */
    size_t sp_nal_cap = 0, sp_rbsp_cap = 0, sp_rec_cap = 0, sp_list_cap = 0, sp_units_cap = 0;
    /* stream ingest: scratch, grown on demand */
    uint8_t *d_ing_in = nullptr;
    size_t ing_in_cap = 0;
    IngestFile *d_ing_files = nullptr;
    IngestScan *d_ing_scan = nullptr;
    IngestOut *d_ing_out = nullptr;
    int ing_cap = 0;
    void *d_ing_work = nullptr;                 /* segmented ingest scratch */
    size_t ing_work_bytes = 0;
    hipEvent_t ing_ev[2] = {};         /* timing: around the ingest kernels */
    /* reference files from pictures: EP count per chunk */
    uint32_t *d_ipcm_cnt = nullptr;
    size_t ipcm_cap = 0;
    uint8_t *d_ipcm_stg = nullptr;              /* count pass RBSP for the write pass */
    size_t ipcm_stg_cap = 0;
    /* the one pass: the chunks' hand-off words */
    unsigned long long *d_ipcm_hw = nullptr;
    size_t ipcm_hw_cap = 0;
    uint32_t ipcm_epoch = 0;
    double ipcm_ms = 0.0;
    int ipcm_n = 0;
    /* the asynchronous I_PCM calls since the last sync: their overflow flag
     * (checked at the sync) and, with timing, their event pairs */
    uint32_t *ipcm_over = nullptr;      /* = d_ipcm_sticky while calls are pending */
    uint32_t *d_ipcm_sticky = nullptr;
    size_t ipcm_over_stride = 0;
    std::vector<hipEvent_t> ipcm_ev;    /* pairs, reused */
    size_t ipcm_ev_used = 0;
    double ing_ms = 0.0;
    int ing_n = 0;
    /* host delivery: per-stream (offset, bytes) table of the last packing */
    int dyn_grow = 0;                  /* the dynamic rect's pools at their bounds (after running out) */
    int32_t *d_upd = nullptr;          /* reference updates: (stream, which) per entry */
    size_t upd_cap = 0;
    uint64_t *d_out_tab = nullptr;
    size_t out_tab_cap = 0;
    hipEvent_t out_ev = nullptr;
};

/* event pairs of one compose.  Dynamic rect: plan = [0,1) + [2,3), dyn
 * stage [1,2), emit [3,4), dyn emit [4,5).  Otherwise only events 0, 1, 4
 * are recorded (fewer markers between the kernels): plan [0,1), emit [1,4).
 * lite (scroll_batch_enable_timing(b, 2)): only the dominant kernel's pair,
 * dyn code [1,6) (reported as dyn stage too) or emit [1,4) -- each event
 * record is a marker packet that holds the queue for microseconds, so the
 * full set costs a timed step ~ 40 us of gaps between its kernels */
static void event_ms(const hipEvent_t *e, bool dyn, bool lite, float out[6])
{
    auto el = [&](int a, int b) {
        float v = 0.0f;
        return hipEventElapsedTime(&v, e[a], e[b]) == hipSuccess ? v : 0.0f;
    };
    if (lite) {
        for (int k = 0; k < 6; ++k) out[k] = 0.0f;
        if (dyn) out[2] = out[4] = el(1, 6);
        else out[1] = el(1, 4);
        return;
    }
    if (dyn) {
        out[0] = el(0, 1) + el(2, 3);
        out[1] = el(3, 4);
        out[2] = el(1, 2);
        out[3] = el(4, 5);
        out[4] = el(1, 6);
        out[5] = el(6, 2);
    } else {
        out[0] = el(0, 1);
        out[1] = el(1, 4);
        out[2] = out[3] = out[4] = out[5] = 0.0f;
    }
}

/* timing-only events: no system-scope fence on record (no cache writeback /
 * invalidate between the kernels being timed) */
static hipError_t timing_event(hipEvent_t *e)
{
    return hipEventCreateWithFlags(e, hipEventDisableSystemFence);
}

extern "C" {

const char *scroll_last_error(void) { return g_err; }

const char *scroll_version(void) { return "h264scroll-amd 0.1 (gfx950)"; }

int scroll_device_count(void) { return usable_devices(nullptr); }

int scroll_batch_create(ScrollBatch **out, const ScrollBatchDesc *desc)
{
    if (!out || !desc || desc->max_streams <= 0 || desc->max_frames <= 0 ||
        desc->arena_bytes == 0 ||
        (desc->mode != SCROLL_MODE_COMPOSER && desc->mode != SCROLL_MODE_EXPERIMENT)) {
        set_err("scroll_batch_create: bad descriptor");
        return SCROLL_ERR_ARG;
    }
    *out = nullptr;
    std::vector<int> ids;
    if (!usable_devices(&ids)) return SCROLL_ERR_NO_DEVICE;
    int n = 0;
    (void)hipGetDeviceCount(&n);
    if (desc->device < 0 || desc->device >= n) {
        set_err("scroll_batch_create: device %d out of range (%d visible)", desc->device, n);
        return SCROLL_ERR_ARG;
    }
    bool ok = false;
    for (int i : ids) ok |= (i == desc->device);
    if (!ok) {
        set_err("scroll_batch_create: device %d is not gfx950", desc->device);
        return SCROLL_ERR_NO_DEVICE;
    }
    HIPCHK(hipSetDevice(desc->device));
    ScrollBatch *b = new ScrollBatch();
    b->device = desc->device;
    b->mode = desc->mode;
    b->max_streams = desc->max_streams;
    b->max_frames = desc->max_frames;
    b->arena_bytes = desc->arena_bytes;
    /* >= 128 B slack past out_cap: k_emit writes whole 128-byte lines and
     * zero-fills the tail of a stream's last line */
    b->ld_arena = (desc->arena_bytes + 128 + 255) & ~(size_t)255;
    b->ld_nal = 2 * desc->max_frames;
    size_t S = (size_t)desc->max_streams;
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMalloc(&b->d_st, S * sizeof(DevStream));
    if (e == hipSuccess) e = hipHostMalloc(&b->h_st, S * sizeof(DevStream), hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(&b->d_off, S * (size_t)desc->max_frames * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&b->d_nal, S * (size_t)b->ld_nal * sizeof(NalDesc));
    if (e == hipSuccess) e = hipMalloc(&b->d_arena, S * b->ld_arena);
    if (e == hipSuccess) e = hipMalloc(&b->d_pend, S * sizeof(PlanPending));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&b->own, hipStreamNonBlocking);
    for (int i = 0; i < NEV && e == hipSuccess; ++i) e = timing_event(&b->ev[i]);
    if (e == hipSuccess) e = hipMemset(b->d_st, 0, S * sizeof(DevStream));
    if (e == hipSuccess) e = hipMemset(b->d_off, 0, S * (size_t)desc->max_frames * sizeof(int32_t));
    if (e != hipSuccess) {
        set_err("scroll_batch_create: %s", hipGetErrorString(e));
        scroll_batch_destroy(b);
        return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
    }
    memset(b->h_st, 0, S * sizeof(DevStream));
    b->last = b->own;
    *out = b;
    return SCROLL_OK;
}

void scroll_batch_destroy(ScrollBatch *b)
{
    if (!b) return;
    (void)hipSetDevice(b->device);
    if (b->own) (void)hipStreamSynchronize(b->own);
    for (int i = 0; i < NEV; ++i)
        if (b->ev[i]) (void)hipEventDestroy(b->ev[i]);
    for (hipEvent_t e : b->ring) (void)hipEventDestroy(e);
    if (b->fork.side) {
        (void)hipStreamSynchronize(b->fork.side);
        (void)hipStreamDestroy(b->fork.side);
        (void)hipEventDestroy(b->fork.e0);
        (void)hipEventDestroy(b->fork.e1);
    }
    if (b->own) (void)hipStreamDestroy(b->own);
    (void)hipFree(b->d_st);
    (void)hipHostFree(b->h_st);
    (void)hipFree(b->d_off);
    (void)hipFree(b->d_nal);
    (void)hipFree(b->d_arena);
    (void)hipFree(b->d_out_tab);
    (void)hipFree(b->d_upd);
    if (b->out_ev) (void)hipEventDestroy(b->out_ev);
    (void)hipFree(b->d_pend);
    (void)hipFree(b->d_dfr);
    (void)hipFree(b->d_src);
    (void)hipFree(b->d_refs);
    (void)hipFree(b->d_stage);
    (void)hipFree(b->d_hf);
    (void)hipFree(b->d_pool);
    (void)hipFree(b->d_spf);
    (void)hipFree(b->d_sp_nal);
    (void)hipFree(b->d_sp_rbsp);
    (void)hipFree(b->d_sp_rec);
    (void)hipFree(b->d_sp_list);
    (void)hipFree(b->d_sp_units);
    (void)hipFree(b->d_sp_lanes);
    (void)hipFree(b->d_ing_in);
    (void)hipFree(b->d_ipcm_cnt);
    (void)hipFree(b->d_ipcm_stg);
    (void)hipFree(b->d_ipcm_hw);
    (void)hipFree(b->d_ing_files);
    (void)hipFree(b->d_ing_scan);
    (void)hipFree(b->d_ing_out);
    (void)hipFree(b->d_ing_work);
    for (hipEvent_t e : b->ing_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : b->ipcm_ev)
        if (e) (void)hipEventDestroy(e);
    (void)hipFree(b->d_ipcm_sticky);
    if (b->d_dbg) (void)hipFree(b->d_dbg);
    delete b;
}

int scroll_batch_num_streams(const ScrollBatch *b) { return b ? b->nstreams : 0; }

int scroll_batch_set_debug(ScrollBatch *b, int flags)
{
    if (!b) return SCROLL_ERR_ARG;
    b->debug = flags;
    return SCROLL_OK;
}

static int dyn_grow_pools(ScrollBatch *b);

static int ipcm_async_check(ScrollBatch *b);

static int batch_host_sync(ScrollBatch *b)
{
    if (b->host_valid) return SCROLL_OK;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipStreamSynchronize(b->last));
    HIPCHK(hipMemcpy(b->h_st, b->d_st, (size_t)b->nstreams * sizeof(DevStream),
                     hipMemcpyDeviceToHost));
    b->host_valid = 1;
    return SCROLL_OK;
}

int scroll_batch_add_stream(ScrollBatch *b, const ComposerConfig *cfg)
{
    if (!b || !cfg) return SCROLL_ERR_ARG;
    if (b->nstreams >= b->max_streams) {
        set_err("scroll_batch_add_stream: batch full (%d streams)", b->max_streams);
        return SCROLL_ERR_ARG;
    }
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (b->dyn_on && (cfg->width != b->dyn_pw || cfg->height != b->dyn_ph)) {
        set_err("scroll_batch_add_stream: the dynamic rect needs %dx%d streams", b->dyn_pw,
                b->dyn_ph);
        return SCROLL_ERR_CONFIG;
    }
    if (b->hint_on && ((cfg->width / 16) * (cfg->height / 16) > b->hint_max_mb ||
                       cfg->width / 16 > HINT_MAX_MBW)) {
        set_err("scroll_batch_add_stream: hint staging slots hold %d MBs per picture, %d per row",
                b->hint_max_mb, HINT_MAX_MBW);
        return SCROLL_ERR_CONFIG;
    }
    rc = batch_host_sync(b);
    if (rc) return rc;
    int s = b->nstreams;
    DevStream *d = &b->h_st[s];
    if (b->dyn_qp != 26 && !cfg->deblocking_filter_control_present_flag) {
        set_err("scroll_batch_add_stream: a stream with the deblocking filter on (no "
                "deblocking_filter_control_present_flag) needs the rect at QP 26, the batch's is %d",
                b->dyn_qp);
        return SCROLL_ERR_CONFIG;
    }
    memset(d, 0, sizeof(*d));
    cfg_to_dev(cfg, d);
    d->dyn_qp = b->dyn_qp;
    d->out_pos = 0;
    d->out_cap = b->arena_bytes;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpy(b->d_st + s, d, sizeof(DevStream), hipMemcpyHostToDevice));
    b->nstreams++;
    return s;
}

int scroll_batch_get_config(ScrollBatch *b, int s, ComposerConfig *cfg)
{
    if (!b || !cfg || s < 0 || s >= b->nstreams) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    const DevStream *d = &b->h_st[s];
    composer_config_init(cfg, d->w, d->h);
    cfg->log2_max_frame_num = d->log2_mfn;
    cfg->pic_order_cnt_type = d->poc_type;
    cfg->log2_max_pic_order_cnt_lsb = d->log2_poc;
    cfg->deblocking_filter_control_present_flag = d->deblock;
    dev_to_cfg(d, cfg);
    return SCROLL_OK;
}

int scroll_batch_set_config(ScrollBatch *b, int s, const ComposerConfig *cfg)
{
    if (!b || !cfg || s < 0 || s >= b->nstreams) return SCROLL_ERR_ARG;
    int rc = check_cfg(cfg);
    if (rc) return rc;
    rc = batch_host_sync(b);
    if (rc) return rc;
    DevStream *d = &b->h_st[s];
    if (!cfg->deblocking_filter_control_present_flag) {
        /* the guard of add_stream / set_dyn_qp*: the loop filter on keeps the
         * stream's rect, and every per-frame rect QP of it, at 26 */
        bool bad = d->dyn_qp != 26;
        const size_t F = (size_t)b->max_frames, i0 = (size_t)s * F;
        for (size_t f = 0; !bad && f < F && i0 + f < b->h_dyn_qp.size(); ++f) {
            const int q = b->h_dyn_qp[i0 + f];
            bad = q >= 0 && q != 26;
        }
        if (bad) {
            set_err("scroll_batch_set_config: stream %d's rect QP is not 26: it cannot turn the deblocking "
                    "filter on (no deblocking_filter_control_present_flag)", s);
            return SCROLL_ERR_CONFIG;
        }
    }
    cfg_to_dev(cfg, d);
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpy(b->d_st + s, d, sizeof(DevStream), hipMemcpyHostToDevice));
    return SCROLL_OK;
}

int scroll_batch_set_offsets(ScrollBatch *b, const int32_t *offsets, int nframes)
{
    if (!b || !offsets || nframes < 0 || nframes > b->max_frames) return SCROLL_ERR_ARG;
    if (nframes == 0 || b->nstreams == 0) return SCROLL_OK;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpy2D(b->d_off, (size_t)b->max_frames * sizeof(int32_t), offsets,
                       (size_t)nframes * sizeof(int32_t), (size_t)nframes * sizeof(int32_t),
                       (size_t)b->nstreams, hipMemcpyHostToDevice));
    return SCROLL_OK;
}

int32_t *scroll_batch_offsets_device(ScrollBatch *b) { return b ? b->d_off : nullptr; }

static void fold_ring(ScrollBatch *b)
{
    for (int i = 0; i + NEV <= b->ring_used; i += NEV) {
        float m[6];
        event_ms(&b->ring[i], (b->ring_dyn[i / NEV] & 1) != 0, (b->ring_dyn[i / NEV] & 2) != 0, m);
        for (int k = 0; k < 6; ++k) b->acc_ms[k] += m[k];
        b->acc_n++;
    }
    b->ring_used = 0;
}

static int ring_events(ScrollBatch *b, hipEvent_t **evs)
{
    if ((size_t)b->ring_used + NEV > b->ring.size()) {
        if (b->ring.size() >= (size_t)NEV * 256) {   /* bound: fold pending timings first */
            HIPCHK(hipStreamSynchronize(b->last));
            fold_ring(b);
        } else {
            for (int i = 0; i < NEV; ++i) {
                hipEvent_t e;
                HIPCHK(timing_event(&e));
                b->ring.push_back(e);
            }
            b->ring_dyn.push_back(0);
        }
    }
    *evs = &b->ring[b->ring_used];
    b->ring_used += NEV;
    return SCROLL_OK;
}

static int launch(ScrollBatch *b, int nframes, int plan_mode, int nal_max, hipStream_t hs,
                  int plan_flags = 0)
{
    int S = b->nstreams;
    if (S == 0) return SCROLL_OK;
    hipEvent_t *rev = nullptr;
    if (b->timing) {
        int rc = ring_events(b, &rev);
        if (rc) return rc;
    }
    const bool hint = b->hint_on && plan_mode != SCROLL_PLAN_EXPLICIT;
    const bool dyn = (b->dyn_on || hint) && plan_mode != SCROLL_PLAN_EXPLICIT;   /* staged NALs */
    const bool lite = b->timing == 2;
    /* lite with the row coder: its pair goes right around k_dyn_row
     * (dyn_launch_code), not around the whole code step */
    const bool lite_row = lite && dyn && !hint;
    auto mark = [&](int k) -> int {
        if (!b->timing || (!dyn && k != 0 && k != 1 && k != 4)) return SCROLL_OK;
        if (lite) {                     /* the dominant kernel's pair, ring only */
            if ((k == 1 || k == (dyn ? 6 : 4)) && !lite_row) HIPCHK(hipEventRecord(rev[k], hs));
            return SCROLL_OK;
        }
        HIPCHK(hipEventRecord(b->ev[k], hs));
        HIPCHK(hipEventRecord(rev[k], hs));
        return SCROLL_OK;
    };
    if (b->timing) {
        b->ring_dyn[(b->ring_used - NEV) / NEV] = (uint8_t)((dyn ? 1 : 0) | (lite ? 2 : 0));
        if (!lite) b->ev_dyn = dyn ? 1 : 0;
    }
    const int ld_fr = b->max_frames;
    int rc = mark(0);
    if (rc) return rc;
    if (!dyn) {
        hipLaunchKernelGGL(k_plan, dim3(S), dim3(PLAN_THREADS), 0, hs, b->d_st, b->d_off,
                           b->max_frames, b->d_nal, b->ld_nal, nframes, plan_mode,
                           b->debug | plan_flags, b->d_pend, b->d_dfr, ld_fr);
        HIPCHK(hipGetLastError());
        if ((rc = mark(1)) || (rc = mark(2)) || (rc = mark(3))) return rc;
    } else {
        const bool dyn_rect = b->dyn_on && !hint;
        hipLaunchKernelGGL(k_plan, dim3(S), dim3(PLAN_THREADS), 0, hs, b->d_st, b->d_off,
                           b->max_frames, b->d_nal, b->ld_nal, nframes, plan_mode,
                           b->debug | plan_flags | PLAN_STATE | PLAN_DYN, b->d_pend, b->d_dfr,
                           ld_fr, nullptr, 0u, 0u, dyn_rect ? b->dx.ctr : nullptr);
        HIPCHK(hipGetLastError());
        if ((rc = mark(1))) return rc;
        uint64_t *stamps = nullptr;
        if (b->debug & SCROLL_DEBUG_DYN_STAMPS) {   /* k_dyn_emit_gather's, then k_dyn_group's */
            const size_t slots = (2 + (size_t)b->geo.ngroups) * (size_t)nframes * S;
            if (slots > b->dbg_slots) {
                if (b->d_dbg) (void)hipFree(b->d_dbg);
                HIPCHK(hipMalloc(&b->d_dbg, slots * 8 * sizeof(uint64_t)));
                b->dbg_slots = slots;
            }
            HIPCHK(hipMemsetAsync(b->d_dbg, 0, slots * 8 * sizeof(uint64_t), hs));
            stamps = b->d_dbg + 2 * (size_t)nframes * S * 8;
        }
        b->geo.debug = b->debug;
        if (hint) {
            if (b->sp_parse) {
                if (splice_launch_parse(hs, b->sp_n, b->sp_ymax, b->d_sp_list, b->d_spf, b->d_sp_units,
                                        b->d_sp_lanes, b->sp_nslots, b->d_st, ld_fr, b->d_sp_rbsp, b->d_sp_rec)) {
                    set_err("k_splice_parse launch: %s", hipGetErrorString(hipGetLastError()));
                    return SCROLL_ERR_HIP;
                }
                b->sp_parse = 0;
            }
            if (b->fallback && b->dyn_on &&
                hint_launch_fb(hs, nframes, S, b->d_st, b->d_nal, b->ld_nal, b->d_pend, b->d_dfr, ld_fr,
                               b->d_hf, b->d_pool)) {
                set_err("k_hint_fb launch: %s", hipGetErrorString(hipGetLastError()));
                return SCROLL_ERR_HIP;
            }
            if (hint_launch_stage(hs, nframes, S, b->d_st, b->d_nal, b->ld_nal, b->d_pend,
                                  b->d_dfr, ld_fr, b->d_hf, b->d_pool, b->d_stage,
                                  b->geo.slot_bytes)) {
                set_err("k_hint_stage launch: %s", hipGetErrorString(hipGetLastError()));
                return SCROLL_ERR_HIP;
            }
            const bool combined = b->dyn_on;
            if (combined &&
                hdyn_launch_code(hs, nframes, S, b->d_st, b->d_nal, b->ld_nal, b->d_pend, b->d_dfr, ld_fr,
                                 b->d_hf, b->d_pool, b->d_spf, &b->geo, b->d_src, b->d_refs,
                                 b->d_sp_rec, b->d_sp_rbsp, b->hd_mb_words)) {
                set_err("k_hdyn_code launch: %s", hipGetErrorString(hipGetLastError()));
                return SCROLL_ERR_HIP;
            }
            if ((b->sp_n > 0 || combined) &&
                splice_launch_stage(hs, nframes, S, b->d_st, b->d_nal, b->ld_nal, b->d_pend,
                                    b->d_dfr, ld_fr, b->d_hf, b->d_pool, b->d_spf, b->d_sp_rec,
                                    b->d_sp_rbsp, b->d_stage, b->geo.slot_bytes)) {
                set_err("k_splice_stage launch: %s", hipGetErrorString(hipGetLastError()));
                return SCROLL_ERR_HIP;
            }
            if ((rc = mark(6))) return rc;
        } else {
            b->dx.epoch = b->dx.epoch % 0xffffffu + 1u;    /* look-back epoch, never 0 */
            /* (a pipeline over stream chunks, the coder of one chunk beside the
             * packing of the one before on a second HIP stream, measured slower
             * at 2 / 4 / 8 chunks: DESIGN.md §6; the device-side frame lists
             * are batch-wide, so the launches below cover the whole batch) */
            const DynGeom &G = b->geo;
            /* SCROLL_DYN_FORK=1: the general path and the static groups on a
             * second stream beside k_dyn_row (created on first use) */
            const DynFork *fk = nullptr;
            static const bool fork_on = [] {
                const char *e = getenv("SCROLL_DYN_FORK");
                return e && e[0] == '1';
            }();
            if (fork_on) {
                if (!b->fork.side) {
                    HIPCHK(hipStreamCreateWithFlags(&b->fork.side, hipStreamNonBlocking));
                    HIPCHK(hipEventCreateWithFlags(&b->fork.e0, hipEventDisableTiming));
                    HIPCHK(hipEventCreateWithFlags(&b->fork.e1, hipEventDisableTiming));
                }
                fk = &b->fork;
            }
            if (dyn_launch_code(hs, nframes, S, b->d_st, b->d_nal, b->ld_nal, b->d_pend, b->d_dfr, ld_fr, &G,
                                b->d_src, b->d_refs, &b->dx, b->dx.epoch, b->dyn_pw / 16, stamps, fk,
                                lite_row ? rev[1] : nullptr, lite_row ? rev[6] : nullptr)) {
                set_err("k_dyn_code launch: %s", hipGetErrorString(hipGetLastError()));
                return SCROLL_ERR_HIP;
            }
            if ((rc = mark(6))) return rc;
            if (dyn_launch_pack(hs, nframes, S, b->d_st, b->d_nal, b->ld_nal, b->d_pend, b->d_dfr, ld_fr, &G,
                                &b->dx, b->d_stage, stamps ? b->d_dbg : nullptr, fk)) {
                set_err("k_dyn_static / k_dyn_epfix launch: %s", hipGetErrorString(hipGetLastError()));
                return SCROLL_ERR_HIP;
            }
        }
        if ((rc = mark(2))) return rc;
        hipLaunchKernelGGL(k_plan, dim3(S), dim3(PLAN_THREADS), 0, hs, b->d_st, b->d_off,
                           b->max_frames, b->d_nal, b->ld_nal, nframes, plan_mode,
                           b->debug | plan_flags | PLAN_SIZE | PLAN_DYN, b->d_pend, b->d_dfr,
                           ld_fr, (b->dyn_on && !b->hint_on) ? (const uint32_t *)b->dx.ctr : nullptr,
                           b->geo.rs_spill_cap, b->geo.gen_cap);
        HIPCHK(hipGetLastError());
        if ((rc = mark(3))) return rc;
    }
    int per_wg = EMIT_WAVES * TILE;
    int gx = (nal_max + per_wg - 1) / per_wg;
    if (gx > 0 && (b->debug & SCROLL_DEBUG_EMIT_STAMPS)) {
        size_t slots = (size_t)gx * S * EMIT_WAVES;
        if (slots > b->dbg_slots) {
            if (b->d_dbg) (void)hipFree(b->d_dbg);
            HIPCHK(hipMalloc(&b->d_dbg, slots * 8 * sizeof(uint64_t)));
            b->dbg_slots = slots;
        }
        HIPCHK(hipMemsetAsync(b->d_dbg, 0, slots * 8 * sizeof(uint64_t), hs));
    }
    if (gx > 0) {
        hipLaunchKernelGGL(k_emit, dim3(gx, S), dim3(EMIT_WAVES * 64), 0, hs, b->d_st, b->d_nal,
                           b->ld_nal, b->d_arena, (uint64_t)b->ld_arena, b->debug, b->d_dbg);
        HIPCHK(hipGetLastError());
    }
    if ((rc = mark(4))) return rc;
    if (dyn && dyn_launch_emit(hs, nframes, S, b->d_st, b->d_nal, b->ld_nal, b->d_dfr, ld_fr,
                               &b->geo, b->d_stage, hint ? nullptr : &b->dx, b->d_arena,
                               (uint64_t)b->ld_arena,
                               (b->debug & SCROLL_DEBUG_DYN_STAMPS) && b->d_dbg
                                   ? b->d_dbg + (size_t)nframes * S * 8 : nullptr)) {
        set_err("k_dyn_gather launch: %s", hipGetErrorString(hipGetLastError()));
        return SCROLL_ERR_HIP;
    }
    if ((rc = mark(5))) return rc;
    if (b->timing == 1) b->timed_pending = 1;
    b->host_valid = 0;
    b->nal_cache_valid = 0;
    b->last = hs;
    return SCROLL_OK;
}

static int hint_upload(ScrollBatch *b);
static int splice_upload(ScrollBatch *b);
static int hd_upload(ScrollBatch *b);
static int splice_frame_status(ScrollBatch *b, size_t i, int *status);
static const char *splice_msg(int e);

int scroll_batch_compose(ScrollBatch *b, int nframes, void *hip_stream)
{
    return scroll_batch_compose_ex(b, nframes, hip_stream, 0);
}

int scroll_batch_compose_ex(ScrollBatch *b, int nframes, void *hip_stream, int flags)
{
    if (!b || nframes < 0 || nframes > b->max_frames) {
        set_err("scroll_batch_compose: nframes %d out of range", nframes);
        return SCROLL_ERR_ARG;
    }
    if (b->dyn_on && !b->dyn_refs) {
        set_err("scroll_batch_compose: dynamic rect without reference pictures");
        return SCROLL_ERR_CONFIG;
    }
    HIPCHK(hipSetDevice(b->device));
    const bool combined = b->hint_on && b->dyn_on;
    if (b->dyn_pos_custom && !b->hint_on) {
        set_err("scroll_batch_compose: per-frame dynamic rect positions need UI hints "
                "(scroll_batch_set_hints)");
        return SCROLL_ERR_CONFIG;
    }
    if (b->hint_on && b->sp_dirty) {
        int rc = splice_upload(b);
        if (rc) return rc;
        if (combined) b->hd_dirty = 1;
    }
    if (combined && b->hd_dirty) {
        int rc = hd_upload(b);
        if (rc) return rc;
    }
    if (b->hint_on && b->hint_dirty) {
        int rc = hint_upload(b);
        if (rc) return rc;
    }
    hipStream_t hs = hip_stream ? (hipStream_t)hip_stream : b->own;
    int plan = b->mode == SCROLL_MODE_EXPERIMENT ? SCROLL_PLAN_EXPERIMENT : SCROLL_PLAN_COMPOSER;
    int nal_max = plan == SCROLL_PLAN_COMPOSER ? 2 * nframes : nframes;
    b->last_plan_mode = plan;
    b->last_nframes = nframes;
    return launch(b, nframes, plan, nal_max, hs,
                  (flags & SCROLL_COMPOSE_REWIND) ? PLAN_REWIND : 0);
}

int scroll_batch_sync(ScrollBatch *b)
{
    if (!b) return SCROLL_ERR_ARG;
    {
        int rc0 = batch_host_sync(b);
        if (rc0) return rc0;
        if ((rc0 = ipcm_async_check(b))) return rc0;
    }
    if (b->timed_pending) {
        event_ms(b->ev, b->ev_dyn != 0, false, b->ms);
        b->timed_pending = 0;
    }
    int rc = SCROLL_OK;
    for (int s = 0; s < b->nstreams; ++s) {
        if (!b->h_st[s].err) continue;
        if (rc == SCROLL_OK && (b->h_st[s].err & SCROLL_DEVERR_HANDOFF)) {
            set_err("stream %d: a dynamic-rect row waited past its bound for the row above's "
                    "TotalCoeffs (k_dyn_row hand-off); the stream committed nothing", s);
            rc = SCROLL_ERR_DEVICE;
        } else if (rc == SCROLL_OK && (b->h_st[s].err & SCROLL_DEVERR_SPLICE)) {
            int st = 0, ff = 0;
            for (; ff < b->max_frames && !st; ++ff)
                if (splice_frame_status(b, (size_t)s * b->max_frames + ff, &st)) break;
            if (st == HDYN_STATUS_OVERFLOW) {
                set_err("stream %d frame %d: a dynamic-rect MB under hints outgrew its %u-byte "
                        "region (raise slot_bytes of scroll_batch_set_dyn_rect)", s, ff - 1,
                        4u * b->hd_mb_words);
                rc = SCROLL_ERR_OVERFLOW;
            } else {
                set_err("stream %d frame %d: %s: %s", s, ff - 1,
                        b->dyn_on ? "dynamic rect under hints" : "spliced slice", splice_msg(st));
                rc = SCROLL_ERR_CONFIG;
            }
        } else if (rc == SCROLL_OK && (b->h_st[s].err & SCROLL_DEVERR_HINT)) {
            set_err("stream %d: a hint rect names a reference that is not valid in its frame "
                    "(ref 2 + i needs waypoint i)", s);
            rc = SCROLL_ERR_CONFIG;
        } else if (rc == SCROLL_OK && (b->h_st[s].err & SCROLL_DEVERR_DYN)) {
            uint32_t used[2] = {0, 0};
            if (b->dyn_on && !b->hint_on && b->dx.ctr)
                HIPCHK(hipMemcpy(used, b->dx.ctr, sizeof(used), hipMemcpyDeviceToHost));
            if (used[0] > b->geo.rs_spill_cap || used[1] > b->geo.gen_cap) {
                /* content past the typical-size pools: grow them to their
                 * bound for the next compose (this one committed nothing for
                 * the stream) */
                const int grc = dyn_grow_pools(b);
                set_err("stream %d: the dynamic rect's %s pool ran out (%u of %u); %s", s,
                        used[0] > b->geo.rs_spill_cap ? "row-stage spill" : "general-path record",
                        used[0] > b->geo.rs_spill_cap ? used[0] : used[1],
                        used[0] > b->geo.rs_spill_cap ? b->geo.rs_spill_cap : b->geo.gen_cap,
                        grc ? "growing it failed" : "grown: compose again");
            } else {
                set_err("stream %d: a staged NAL outgrew its staging slot (%llu bytes)", s,
                        (unsigned long long)b->geo.slot_bytes);
            }
            rc = SCROLL_ERR_OVERFLOW;
        } else if (rc == SCROLL_OK) {
            set_err("stream %d: output arena overflow (%llu bytes used, capacity %llu)", s,
                    (unsigned long long)b->h_st[s].out_pos,
                    (unsigned long long)b->h_st[s].out_cap);
            rc = SCROLL_ERR_OVERFLOW;
        }
        b->h_st[s].err = 0;                      /* reported once, then cleared */
        HIPCHK(hipMemcpy(&b->d_st[s].err, &b->h_st[s].err, sizeof(int32_t),
                         hipMemcpyHostToDevice));
    }
    if (rc) return rc;
    return SCROLL_OK;
}

size_t scroll_batch_output_size(ScrollBatch *b, int s)
{
    if (!b || s < 0 || s >= b->nstreams || batch_host_sync(b)) return 0;
    return (size_t)b->h_st[s].out_pos;
}

int scroll_batch_copy_output(ScrollBatch *b, int s, size_t from, uint8_t *dst, size_t n)
{
    if (!b || s < 0 || s >= b->nstreams || (!dst && n)) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    if (from + n > b->h_st[s].out_pos) {
        set_err("scroll_batch_copy_output: range beyond stream output");
        return SCROLL_ERR_ARG;
    }
    if (n == 0) return SCROLL_OK;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpy(dst, b->d_arena + (size_t)s * b->ld_arena + from, n, hipMemcpyDeviceToHost));
    return SCROLL_OK;
}

/* ------------------------ host delivery (PCIe) ----------------------------- */
/* The reference hands its bytes over in host memory (composer.c:255-291).
 * scroll_batch_output_to_host_async packs the bytes appended to every stream
 * since its previous delivery (DevStream.undelivered) into pinned host memory, device-side and asynchronously: one
 * workgroup scans the streams' byte counts (16-byte aligned offsets) into the
 * host table, then every stream's bytes are read from its arena and stored
 * straight into the pinned buffer by (8, S) workgroups of 16-byte chunks --
 * no host sync between the compose and the copy, and the host never needs
 * the sizes before the bytes land. */
namespace {
constexpr int OUT_Z = 8;
__global__ __launch_bounds__(1024) void k_out_table(DevStream *__restrict__ st, int S, uint64_t cap,
                                                    uint64_t *__restrict__ dtab, uint64_t *__restrict__ htab)
{
    __shared__ uint64_t s_w[16], s_carry;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t == 0) s_carry = 0;
    __syncthreads();
    for (int s0 = 0; s0 < S; s0 += 1024) {
        const int s = s0 + t;
        const uint64_t n = s < S ? st[s].undelivered : 0, a = (n + 15) & ~(uint64_t)15;
        const uint64_t inc = wave_incl_scan(a, lane);
        if (lane == 63) s_w[wave] = inc;
        __syncthreads();
        uint64_t before = s_carry;
        for (int w = 0; w < wave; ++w) before += s_w[w];
        if (s < S) {
            dtab[1 + 2 * (size_t)s] = htab[1 + 2 * (size_t)s] = before + inc - a;
            dtab[2 + 2 * (size_t)s] = htab[2 + 2 * (size_t)s] = n;
        }
        __syncthreads();
        if (t == 0)
            for (int w = 0; w < 16; ++w) s_carry += s_w[w];
        __syncthreads();
    }
    if (t == 0) {
        /* total: its aligned size, or ~0 when it does not fit (nothing copied,
         * the bytes stay undelivered) */
        const uint64_t tot = s_carry <= cap ? s_carry : ~(uint64_t)0;
        dtab[0] = htab[0] = tot;
    }
    if (s_carry <= cap)
        for (int s = t; s < S; s += 1024) st[s].undelivered = 0;
}

/* grid (OUT_Z, S): stream s's last-compose bytes -> dst + its offset, one
 * 16-byte chunk per thread and iteration: two aligned arena loads and a
 * byte funnel shift (bytes past n are don't-care: the table has n) */
__global__ __launch_bounds__(256) void k_out_copy(const DevStream *__restrict__ st, const uint8_t *__restrict__ arena,
                                                  uint64_t ld_arena, uint64_t arena_end,
                                                  const uint64_t *__restrict__ dtab, uint8_t *__restrict__ dst)
{
    const int s = blockIdx.y;
    if (dtab[0] == ~(uint64_t)0) return;
    const uint64_t n = dtab[2 + 2 * (size_t)s], o = dtab[1 + 2 * (size_t)s];
    const uint64_t from = (uint64_t)s * ld_arena + st[s].out_pos - n;   /* arena byte of the first new byte */
    uint4 *d = reinterpret_cast<uint4 *>(dst + o);
    const uint32_t q = (uint32_t)(from & 15u) >> 2, rb = (uint32_t)from & 3u;
    const uint64_t base = from & ~(uint64_t)15;
    const uint4 *a = reinterpret_cast<const uint4 *>(arena + base);
    const uint64_t nch = (n + 15) / 16;
    for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < nch; j += (uint64_t)OUT_Z * 256) {
        const uint4 x = a[j];
        const uint4 y = (q | rb) && base + 16 * (j + 2) <= arena_end ? a[j + 1] : x;
        const uint32_t w0 = x.x, w1 = x.y, w2 = x.z, w3 = x.w, w4 = y.x, w5 = y.y, w6 = y.z, w7 = y.w;
        /* word k of the output = bytes 4 (q + k) + rb .. of w[] */
        auto pick = [&](uint32_t i) -> uint32_t {        /* w[i], i <= 7, by selects */
            const uint32_t lo = i & 1u ? (i & 2u ? w3 : w1) : (i & 2u ? w2 : w0);
            const uint32_t hi = i & 1u ? (i & 2u ? w7 : w5) : (i & 2u ? w6 : w4);
            return i & 4u ? hi : lo;
        };
        uint32_t o4[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t lo = pick(q + k), hi = pick(q + k + 1u);
            o4[k] = rb ? __builtin_amdgcn_alignbyte(hi, lo, rb) : lo;
        }
        d[j] = make_uint4(o4[0], o4[1], o4[2], o4[3]);
    }
}
}  // namespace

int scroll_host_alloc(void **p, size_t n)
{
    if (!p) return SCROLL_ERR_ARG;
    *p = nullptr;
    hipError_t e = hipHostMalloc(p, n ? n : 1, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        set_err("scroll_host_alloc(%zu): %s", n, hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
    }
    return SCROLL_OK;
}

void scroll_host_free(void *p)
{
    if (p) (void)hipHostFree(p);
}

int scroll_batch_output_to_host_async(ScrollBatch *b, uint8_t *dst, size_t cap, uint64_t *table, void *hip_stream)
{
    if (!b || !dst || !table || (cap & 15) || (reinterpret_cast<uintptr_t>(dst) & 15)) {
        set_err("scroll_batch_output_to_host_async: bad arguments (dst / cap must be 16-byte aligned)");
        return SCROLL_ERR_ARG;
    }
    HIPCHK(hipSetDevice(b->device));
    hipStream_t hs = hip_stream ? (hipStream_t)hip_stream : (b->last ? b->last : b->own);
    if (b->last && hs != b->last) {                 /* after the last compose */
        if (!b->out_ev) HIPCHK(hipEventCreateWithFlags(&b->out_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(b->out_ev, b->last));
        HIPCHK(hipStreamWaitEvent(hs, b->out_ev, 0));
    }
    const size_t S = (size_t)b->nstreams;
    if (b->out_tab_cap < 1 + 2 * S) {
        (void)hipFree(b->d_out_tab);
        b->d_out_tab = nullptr;
        b->out_tab_cap = 0;
        HIPCHK(hipMalloc(&b->d_out_tab, (1 + 2 * S) * sizeof(uint64_t)));
        b->out_tab_cap = 1 + 2 * S;
    }
    hipLaunchKernelGGL(k_out_table, dim3(1), dim3(1024), 0, hs, b->d_st, (int)S, (uint64_t)cap, b->d_out_tab,
                       table);
    HIPCHK(hipGetLastError());
    if (S) {
        hipLaunchKernelGGL(k_out_copy, dim3(OUT_Z, (unsigned)S), dim3(256), 0, hs, b->d_st, b->d_arena,
                           (uint64_t)b->ld_arena, (uint64_t)b->max_streams * b->ld_arena, b->d_out_tab, dst);
        HIPCHK(hipGetLastError());
    }
    b->last = hs;
    b->host_valid = 0;      /* k_out_table zeroes DevStream.undelivered: the next sync waits for
                               the copy and refreshes the host mirror before anything uploads it */
    return SCROLL_OK;
}

const uint8_t *scroll_batch_output_device(ScrollBatch *b, int s)
{
    if (!b || s < 0 || s >= b->nstreams) return nullptr;
    return b->d_arena + (size_t)s * b->ld_arena;
}

int scroll_batch_reset_output(ScrollBatch *b)
{
    if (!b) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    for (int s = 0; s < b->nstreams; ++s) b->h_st[s].out_pos = b->h_st[s].undelivered = 0;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpy(b->d_st, b->h_st, (size_t)b->nstreams * sizeof(DevStream),
                     hipMemcpyHostToDevice));
    return SCROLL_OK;
}

static int load_nals(ScrollBatch *b)
{
    if (b->nal_cache_valid) return SCROLL_OK;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    b->nal_cache.resize((size_t)b->nstreams * b->ld_nal);
    HIPCHK(hipMemcpy(b->nal_cache.data(), b->d_nal, b->nal_cache.size() * sizeof(NalDesc),
                     hipMemcpyDeviceToHost));
    b->nal_cache_valid = 1;
    return SCROLL_OK;
}

int scroll_batch_nal_count(ScrollBatch *b, int s)
{
    if (!b || s < 0 || s >= b->nstreams) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    return b->h_st[s].nnal;
}

int scroll_batch_nal_info(ScrollBatch *b, int s, int i, int *kind, int *offset_px,
                          uint32_t *size, int *slow)
{
    if (!b || s < 0 || s >= b->nstreams) return SCROLL_ERR_ARG;
    int rc = load_nals(b);
    if (rc) return rc;
    if (i < 0 || i >= b->h_st[s].nnal) return SCROLL_ERR_ARG;
    const NalDesc &d = b->nal_cache[(size_t)s * b->ld_nal + i];
    if (kind) *kind = d.kind;
    if (offset_px) *offset_px = d.off;
    if (size) *size = d.size;
    if (slow) *slow = d.slow;
    return SCROLL_OK;
}

int scroll_batch_kernel_stats(ScrollBatch *b, double *plan_ms, double *emit_ms, int *count)
{
    if (!b) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(b->last));
    fold_ring(b);
    if (plan_ms) *plan_ms = b->acc_ms[0];
    if (emit_ms) *emit_ms = b->acc_ms[1];
    if (count) *count = b->acc_n;
    for (int k = 0; k < 6; ++k) b->acc_ms[k] = 0;
    b->acc_n = 0;
    return SCROLL_OK;
}

int scroll_batch_kernel_stats_ex(ScrollBatch *b, double ms[6], int *count)
{
    if (!b || !ms) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(b->last));
    fold_ring(b);
    for (int k = 0; k < 6; ++k) {
        ms[k] = b->acc_ms[k];
        b->acc_ms[k] = 0;
    }
    if (count) *count = b->acc_n;
    b->acc_n = 0;
    return SCROLL_OK;
}

long long scroll_batch_debug_stamps(ScrollBatch *b, uint64_t *dst, long long max_slots)
{
    if (!b || batch_host_sync(b) || !b->d_dbg) return 0;
    long long n = (long long)b->dbg_slots < max_slots ? (long long)b->dbg_slots : max_slots;
    if (hipMemcpy(dst, b->d_dbg, (size_t)n * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost) !=
        hipSuccess)
        return 0;
    return n;
}

unsigned long long scroll_batch_last_bytes(ScrollBatch *b)
{
    if (!b || batch_host_sync(b)) return 0;
    unsigned long long t = 0;
    for (int s = 0; s < b->nstreams; ++s) t += b->h_st[s].batch_bytes;
    return t;
}

long long scroll_batch_last_nals(ScrollBatch *b)
{
    if (!b || batch_host_sync(b)) return -1;
    long long t = 0;
    for (int s = 0; s < b->nstreams; ++s) t += b->h_st[s].nnal;
    return t;
}

/* ------------------------------ dynamic rect ----------------------------- */
static void dyn_release(ScrollBatch *b)
{
    if (!b->hint_on) {                 /* else they are the hint path's */
        (void)hipFree(b->d_dfr);
        (void)hipFree(b->d_stage);
        b->d_dfr = nullptr;
        b->d_stage = nullptr;
    }
    (void)hipFree(b->d_src);
    (void)hipFree(b->d_refs);
    (void)hipFree(b->dx.rows);
    (void)hipFree(b->dx.meta);
    (void)hipFree(b->dx.body_lo);
    (void)hipFree(b->dx.body_hi);
    (void)hipFree(b->dx.body_w);
    (void)hipFree(b->dx.heads);
    (void)hipFree(b->dx.tcx);
    (void)hipFree(b->dx.rowstage);
    (void)hipFree(b->dx.ctr);
    (void)hipFree(b->dx.gbits);
    b->d_src = b->d_refs = nullptr;
    b->dx = DynScratch{};
    b->dyn_on = 0;
    b->dyn_refs = 0;
    b->h_dyn_pos.clear();
    b->h_dyn_qp.clear();
    b->dyn_pos_custom = 0;
    if (b->hint_on) {                  /* the combined frames become plain hint frames */
        b->geo.x0 = b->geo.y0 = b->geo.w = b->geo.h = 0;
        b->sp_dirty = 1;                   /* d_spf back to the (no) splices */
        b->hint_dirty = 1;
    }
}

static int hd_setup(ScrollBatch *b);
static int sp_grow(void **p, size_t *cap, size_t n, size_t size);

static size_t round256(size_t n) { return (n + 255) & ~(size_t)255; }

static size_t dyn_pair_bytes(const ScrollBatch *b)
{
    return round256((size_t)3 * b->dyn_pw * b->dyn_ph);   /* A and B, I420 each */
}

int scroll_batch_set_dyn_rect(ScrollBatch *b, int x0, int y0, int w, int h, size_t slot_bytes)
{
    if (!b || x0 < 0 || y0 < 0 || w < 0 || h < 0) return SCROLL_ERR_ARG;
    if (b->hint_on && b->sp_n > 0 && w > 0 && h > 0) {
        set_err("scroll_batch_set_dyn_rect: not combinable with spliced slices (clear them first)");
        return SCROLL_ERR_CONFIG;
    }
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    dyn_release(b);
    if (w == 0 || h == 0) return SCROLL_OK;
    if (b->nstreams == 0) {
        set_err("scroll_batch_set_dyn_rect: add the streams first");
        return SCROLL_ERR_ARG;
    }
    const int pw = b->h_st[0].w, ph = b->h_st[0].h;
    for (int s = 1; s < b->nstreams; ++s)
        if (b->h_st[s].w != pw || b->h_st[s].h != ph) {
            set_err("scroll_batch_set_dyn_rect: streams of one batch must share the picture size");
            return SCROLL_ERR_CONFIG;
        }
    const int mbw = pw / 16, mbh = ph / 16;
    /* prediction rows are byte offsets into a reference pair below 2^28 */
    if ((pw & 15) || (ph & 15) || x0 + w > mbw || y0 + h > mbh || w > DYN_MAX_W || h > DYN_MAX_H ||
        mbw > DYN_MAX_MBW || mbh > DYN_MAX_MBH ||
        (size_t)3 * pw * ph >= ((size_t)1 << 28)) {
        set_err("scroll_batch_set_dyn_rect: rect (%d,%d %dx%d MBs) not supported in %dx%d", x0, y0,
                w, h, pw, ph);
        return SCROLL_ERR_CONFIG;
    }
    DynGeom g{};
    g.x0 = x0;
    g.y0 = y0;
    g.pw = pw;
    g.ph = ph;
    g.w = w;
    g.h = h;
    g.qp = b->dyn_qp;
    g.ql = scroll::dyn::qparams(g.qp);
    g.qc = scroll::dyn::qparams(scroll::dyn::qp_chroma(g.qp));
    {
        const int sr = DYN_STATIC_ROWS;
        const int na = (y0 + sr - 1) / sr, nbl = (mbh - y0 - h + sr - 1) / sr;
        g.ngroups = (na > 1 ? na : 1) + h + (nbl > 1 ? nbl : 1);
    }
    g.src_fr = (uint64_t)384 * w * h;
    g.src_ld = round256((size_t)b->max_frames * g.src_fr);
    g.ref_ld = 0;
    g.slot_bytes = slot_bytes ? round256(slot_bytes + DYN_OVF_BYTES) : dyn_slot_bound(mbw, mbh, w, h);
    g.ep_cap = dyn_ep_cap(w, h, b->debug);
    dyn_rowstage_geom(&g, mbw, mbh);
    b->dyn_pw = pw;
    b->dyn_ph = ph;
    const size_t S = (size_t)b->max_streams, F = (size_t)b->max_frames;
    hipError_t e = hipSuccess;
    if (!b->hint_on) {                 /* with hints: the hint path's DynFrames and slots */
        e = hipMalloc(&b->d_dfr, S * F * sizeof(DynFrame));
        /* the RBSP is never staged (k_dyn_epfix / k_dyn_emit_gather read the
         * row groups): per frame only its EP list; slot_bytes stays the cap */
        if (e == hipSuccess) e = hipMalloc(&b->d_stage, S * F * (size_t)4 * g.ep_cap);
        if (e == hipSuccess) e = hipMemset(b->d_dfr, 0, S * F * sizeof(DynFrame));
    }
    if (e == hipSuccess) e = hipMalloc(&b->d_src, S * g.src_ld);
    if (e == hipSuccess) e = hipMalloc(&b->d_refs, S * dyn_pair_bytes(b));
    if (e == hipSuccess) e = hipMalloc(&b->dx.rows, S * F * 32 * h * sizeof(uint32_t));
    /* scratch sized for typical content: general-path record
     * slots for 1/64 of the frames (those NALs need half-pel chroma steps the
     * composer's own waypoints never make), spill slots for 1/32 of the rect
     * rows; a compose that runs out fails the frames concerned with
     * SCROLL_ERR_OVERFLOW and the next compose has pools at their bound */
    g.gen_cap = (uint32_t)std::min(S * F, std::max<size_t>(32, S * F / 64));
    g.rs_spill_cap = g.rs_row_words < g.rs_spill_words
                         ? (uint32_t)std::min(S * F * (size_t)h, std::max<size_t>(2048, S * F * (size_t)h / 32))
                         : 0u;
    g.rs_frames = (uint32_t)(S * F);
    if (b->dyn_grow) {                 /* pools at their bounds (ran out before) */
        g.gen_cap = (uint32_t)(S * F);
        if (g.rs_spill_cap) g.rs_spill_cap = (uint32_t)(S * F * (size_t)h);
    }
    const size_t nrec = (size_t)g.gen_cap * DYN_PIECES * w * h;
    if (e == hipSuccess) e = hipMalloc(&b->dx.meta, nrec * sizeof(uint16_t));
    if (e == hipSuccess) e = hipMalloc(&b->dx.body_lo, nrec * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&b->dx.body_hi, nrec * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&b->dx.body_w, nrec * sizeof(uint4));
    const size_t ng = (size_t)g.ngroups;
    if (e == hipSuccess) e = hipMalloc(&b->dx.heads, S * F * DYN_HEAD_VECS * sizeof(uint4));
    if (e == hipSuccess) e = hipMalloc(&b->dx.tcx, S * F * w * h * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(b->dx.tcx, 0, S * F * w * h * sizeof(unsigned long long));
    const size_t rs_words = S * F * g.rs_frame_words + (size_t)g.rs_spill_cap * g.rs_spill_words;
    if (e == hipSuccess) e = hipMalloc(&b->dx.rowstage, rs_words * sizeof(uint32_t));
    if (e == hipSuccess) b->dx.spill = b->dx.rowstage + S * F * g.rs_frame_words;
    /* counters and the general-record list (dyn_engine.h) */
    if (e == hipSuccess) e = hipMalloc(&b->dx.ctr, (DYN_CTR_LIST + S * F) * sizeof(uint32_t));
    b->dx.ctr_frames = (uint32_t)(S * F);
    if (e == hipSuccess) e = hipMalloc(&b->dx.gbits, S * F * ng * sizeof(uint32_t));
    b->dx.epoch = 0;
    if (e == hipSuccess) e = hipMemset(b->d_src, 0, S * g.src_ld);
    if (e == hipSuccess) e = hipMemset(b->d_refs, 0, S * dyn_pair_bytes(b));
    if (e != hipSuccess) {
        set_err("scroll_batch_set_dyn_rect: %s", hipGetErrorString(e));
        dyn_release(b);
        return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
    }
    b->dyn_cap = g.slot_bytes;
    if (b->hint_on) g.slot_bytes = b->geo.slot_bytes;   /* the hint path's slots (grown by hd_setup) */
    b->geo = g;
    b->dyn_on = 1;
    b->h_dyn_pos.assign(2 * S * F, 0);
    b->h_dyn_qp.assign(S * F, -1);
    for (size_t i = 0; i < S * F; ++i) {
        b->h_dyn_pos[2 * i] = x0;
        b->h_dyn_pos[2 * i + 1] = y0;
    }
    b->dyn_pos_custom = 0;
    b->hd_mb_words = slot_bytes == 0 ? HDYN_MB_WORDS_DEFAULT
                                     : (uint32_t)std::min<size_t>(HDYN_MB_WORDS_MAX,
                                                                  std::max<size_t>(HDYN_MB_WORDS_MIN,
                                                                                   slot_bytes / (4 * (size_t)w * h)));
    if (b->hint_on) return hd_setup(b);
    return SCROLL_OK;
}

int scroll_batch_set_dyn_rect_at(ScrollBatch *b, int s, int f, int x0, int y0)
{
    if (!b || !b->dyn_on || s < 0 || s >= b->nstreams || f < 0 || f >= b->max_frames) {
        set_err("scroll_batch_set_dyn_rect_at: no dynamic rect, or stream / frame out of range");
        return SCROLL_ERR_ARG;
    }
    const int mbw = b->dyn_pw / 16, mbh = b->dyn_ph / 16;
    if (x0 >= 0 && (y0 < 0 || x0 + b->geo.w > mbw || y0 + b->geo.h > mbh)) {
        set_err("scroll_batch_set_dyn_rect_at: rect at (%d, %d) leaves the picture", x0, y0);
        return SCROLL_ERR_ARG;
    }
    int rc = batch_host_sync(b);
    if (rc) return rc;
    const size_t i = (size_t)s * b->max_frames + f;
    b->h_dyn_pos[2 * i] = x0 < 0 ? -1 : x0;
    b->h_dyn_pos[2 * i + 1] = x0 < 0 ? -1 : y0;
    if (x0 != b->geo.x0 || (x0 >= 0 && y0 != b->geo.y0)) b->dyn_pos_custom = 1;
    b->hd_dirty = 1;
    b->hint_dirty = 1;
    return SCROLL_OK;
}

/* the conventional-encode fallback (docs/MASTER_DESIGN.md:220): needs the
 * dynamic rect to be the whole picture, so that every frame's source is a
 * whole picture a conventional encoder would have */
int scroll_batch_set_fallback(ScrollBatch *b, int on)
{
    if (!b) return SCROLL_ERR_ARG;
    if (on && (!b->dyn_on || b->geo.x0 != 0 || b->geo.y0 != 0 || b->geo.w != b->dyn_pw / 16 ||
               b->geo.h != b->dyn_ph / 16)) {
        set_err("scroll_batch_set_fallback: needs the dynamic rect to be the whole picture "
                "(scroll_batch_set_dyn_rect(b, 0, 0, width / 16, height / 16, ...))");
        return SCROLL_ERR_CONFIG;
    }
    int rc = batch_host_sync(b);
    if (rc) return rc;
    b->fallback = on ? 1 : 0;
    b->hd_dirty = 1;
    return SCROLL_OK;
}

int scroll_batch_fallback_frame(ScrollBatch *b, int s, int f, int *fell_back)
{
    if (!b || !fell_back || s < 0 || s >= b->nstreams || f < 0 || f >= b->max_frames) return SCROLL_ERR_ARG;
    *fell_back = 0;
    if (!b->hint_on || !b->d_hf) return SCROLL_OK;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HintFrame H;
    HIPCHK(hipMemcpy(&H, b->d_hf + (size_t)s * b->max_frames + f, sizeof(H), hipMemcpyDeviceToHost));
    *fell_back = (H.mode & HINT_MODE_FB) ? 1 : 0;
    return SCROLL_OK;
}

/* the general-path record pool and the row-stage spill pool at their
 * bounds (a slot for every NAL / rect row), keeping source and references */
static int dyn_grow_pools(ScrollBatch *b)
{
    if (!b->dyn_on || b->dyn_grow) return SCROLL_OK;
    HIPCHK(hipSetDevice(b->device));
    DynGeom g = b->geo;
    const size_t S = (size_t)b->max_streams, F = (size_t)b->max_frames, nmb = (size_t)g.w * g.h;
    g.gen_cap = (uint32_t)(S * F);
    if (g.rs_spill_cap) g.rs_spill_cap = (uint32_t)(S * F * (size_t)g.h);
    const size_t nrec = (size_t)g.gen_cap * DYN_PIECES * nmb;
    const size_t rs_words = S * F * g.rs_frame_words + (size_t)g.rs_spill_cap * g.rs_spill_words;
    uint16_t *meta = nullptr;
    uint2 *lo = nullptr, *hi = nullptr;
    uint4 *wd = nullptr;
    uint32_t *rs = nullptr;
    hipError_t e = hipMalloc(&meta, nrec * sizeof(uint16_t));
    if (e == hipSuccess) e = hipMalloc(&lo, nrec * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&hi, nrec * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&wd, nrec * sizeof(uint4));
    if (e == hipSuccess) e = hipMalloc(&rs, rs_words * sizeof(uint32_t));
    if (e != hipSuccess) {
        (void)hipFree(meta);
        (void)hipFree(lo);
        (void)hipFree(hi);
        (void)hipFree(wd);
        (void)hipFree(rs);
        (void)hipGetLastError();
        return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
    }
    (void)hipFree(b->dx.meta);
    (void)hipFree(b->dx.body_lo);
    (void)hipFree(b->dx.body_hi);
    (void)hipFree(b->dx.body_w);
    (void)hipFree(b->dx.rowstage);
    b->dx.meta = meta;
    b->dx.body_lo = lo;
    b->dx.body_hi = hi;
    b->dx.body_w = wd;
    b->dx.rowstage = rs;
    b->dx.spill = rs + S * F * g.rs_frame_words;
    b->geo.gen_cap = g.gen_cap;
    b->geo.rs_spill_cap = g.rs_spill_cap;
    b->dyn_grow = 1;
    return SCROLL_OK;
}

int scroll_batch_set_dyn_refs(ScrollBatch *b, int s, const uint8_t *ref_a, const uint8_t *ref_b)
{
    if (!b || !b->dyn_on || !ref_a || !ref_b || s < -1 || s >= b->nstreams) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    const size_t pic = (size_t)3 * b->dyn_pw * b->dyn_ph / 2, pair = dyn_pair_bytes(b);
    if (s >= 0 && b->dyn_refs == 1)                      /* shared -> per stream */
        for (int k = 1; k < b->nstreams; ++k)
            HIPCHK(hipMemcpy(b->d_refs + k * pair, b->d_refs, pair, hipMemcpyDeviceToDevice));
    uint8_t *dst = b->d_refs + (s < 0 ? 0 : (size_t)s * pair);
    HIPCHK(hipMemcpy(dst, ref_a, pic, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(dst + pic, ref_b, pic, hipMemcpyHostToDevice));
    if (s < 0) {
        b->dyn_refs = 1;
        b->geo.ref_ld = 0;
    } else {
        b->dyn_refs = 2;
        b->geo.ref_ld = pair;
    }
    return SCROLL_OK;
}

int scroll_batch_set_dyn_source(ScrollBatch *b, const uint8_t *src, int nframes)
{
    if (!b || !b->dyn_on || !src || nframes < 0 || nframes > b->max_frames) return SCROLL_ERR_ARG;
    if (nframes == 0) return SCROLL_OK;
    HIPCHK(hipSetDevice(b->device));
    const size_t row = (size_t)nframes * b->geo.src_fr;
    HIPCHK(hipMemcpy2D(b->d_src, b->geo.src_ld, src, row, row, (size_t)b->nstreams,
                       hipMemcpyHostToDevice));
    return SCROLL_OK;
}

uint8_t *scroll_batch_dyn_source_device(ScrollBatch *b, size_t *stream_stride, size_t *frame_stride)
{
    if (!b || !b->dyn_on) return nullptr;
    if (stream_stride) *stream_stride = b->geo.src_ld;
    if (frame_stride) *frame_stride = b->geo.src_fr;
    return b->d_src;
}

int scroll_batch_dyn_source_synth(ScrollBatch *b, int nframes, int stream_base, int t0)
{
    if (!b || !b->dyn_on || nframes < 0 || nframes > b->max_frames) return SCROLL_ERR_ARG;
    HIPCHK(hipSetDevice(b->device));
    if (dyn_launch_synth(b->own, nframes, b->nstreams, b->d_src, &b->geo, stream_base, t0)) {
        set_err("k_dyn_synth launch: %s", hipGetErrorString(hipGetLastError()));
        return SCROLL_ERR_HIP;
    }
    HIPCHK(hipStreamSynchronize(b->own));
    return SCROLL_OK;
}

int scroll_batch_dyn_frame_info(ScrollBatch *b, int s, int f, uint32_t *rbsp_bytes,
                                uint32_t *ep_bytes)
{
    if (!b || !(b->dyn_on || b->hint_on) || s < 0 || s >= b->nstreams || f < 0 ||
        f >= b->max_frames)
        return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    DynFrame d;
    HIPCHK(hipMemcpy(&d, b->d_dfr + (size_t)s * b->max_frames + f, sizeof(d),
                     hipMemcpyDeviceToHost));
    if (rbsp_bytes) *rbsp_bytes = d.rbsp_bytes;
    if (ep_bytes) *ep_bytes = d.ep;
    return d.nal < 0 ? 1 : SCROLL_OK;
}

int scroll_batch_dyn_totals(ScrollBatch *b, unsigned long long *rbsp_bytes,
                            unsigned long long *ep_bytes, long long *dyn_nals)
{
    if (!b || !(b->dyn_on || b->hint_on)) return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    const size_t S = (size_t)b->nstreams, F = (size_t)b->max_frames;
    std::vector<DynFrame> v(S * F);
    HIPCHK(hipMemcpy(v.data(), b->d_dfr, v.size() * sizeof(DynFrame), hipMemcpyDeviceToHost));
    unsigned long long r = 0, e = 0;
    long long n = 0;
    for (size_t s = 0; s < S; ++s)
        for (int f = 0; f < b->last_nframes; ++f) {
            const DynFrame &d = v[s * F + (size_t)f];
            if (d.nal < 0) continue;
            r += d.rbsp_bytes;
            e += d.ep;
            n++;
        }
    if (rbsp_bytes) *rbsp_bytes = r;
    if (ep_bytes) *ep_bytes = e;
    if (dyn_nals) *dyn_nals = n;
    return SCROLL_OK;
}

/* --------------------------------- UI hints -------------------------------- */
static void hint_release(ScrollBatch *b)
{
    (void)hipFree(b->d_dfr);
    (void)hipFree(b->d_stage);
    (void)hipFree(b->d_hf);
    (void)hipFree(b->d_pool);
    b->d_dfr = nullptr;
    b->d_stage = nullptr;
    b->d_hf = nullptr;
    b->d_pool = nullptr;
    b->pool_cap = 0;
    b->hint_on = 0;
    b->hint_dirty = 0;
    b->h_hint.clear();
    b->h_hint_mode.clear();
    (void)hipFree(b->d_spf);
    (void)hipFree(b->d_sp_nal);
    (void)hipFree(b->d_sp_rbsp);
    (void)hipFree(b->d_sp_rec);
    (void)hipFree(b->d_sp_list);
    (void)hipFree(b->d_sp_units);
    (void)hipFree(b->d_sp_lanes);
    b->d_spf = nullptr;
    b->d_sp_nal = nullptr;
    b->d_sp_rbsp = nullptr;
    b->d_sp_rec = nullptr;
    b->d_sp_list = nullptr;
    b->d_sp_units = nullptr;
    b->d_sp_lanes = nullptr;
    b->sp_nal_cap = b->sp_rbsp_cap = b->sp_rec_cap = b->sp_list_cap = b->sp_units_cap = b->sp_lanes_cap = 0;
    b->sp_nslots = 0;
    b->h_sp.clear();
    b->sp_n = 0;
    b->sp_dirty = 0;
    b->sp_parse = 0;
}

/* host hint tables -> d_hf (per frame) + d_pool (all rects) */
static int hint_upload(ScrollBatch *b)
{
    const size_t n = b->h_hint.size();
    std::vector<HintFrame> hf(n);
    std::vector<ScrollHintRect> pool;
    for (size_t i = 0; i < n; ++i) {
        hf[i].first = (int32_t)pool.size();
        hf[i].n = (int16_t)b->h_hint[i].size();
        hf[i].mode = b->h_hint_mode[i];
        if (i < b->h_sp.size() && b->h_sp[i].w > 0) hf[i].mode |= HINT_MODE_SPLICED;
        if (b->dyn_on && 2 * i < b->h_dyn_pos.size() && b->h_dyn_pos[2 * i] >= 0)
            hf[i].mode |= HINT_MODE_SPLICED;   /* the rect's MBs: k_hdyn_code's records */
        pool.insert(pool.end(), b->h_hint[i].begin(), b->h_hint[i].end());
    }
    if (pool.size() > b->pool_cap) {
        (void)hipFree(b->d_pool);
        b->d_pool = nullptr;
        b->pool_cap = 0;
        hipError_t e = hipMalloc(&b->d_pool, pool.size() * sizeof(ScrollHintRect));
        if (e != hipSuccess) {
            set_err("scroll_batch_compose: hint rects: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->pool_cap = pool.size();
    }
    HIPCHK(hipMemcpy(b->d_hf, hf.data(), n * sizeof(HintFrame), hipMemcpyHostToDevice));
    if (!pool.empty())
        HIPCHK(hipMemcpy(b->d_pool, pool.data(), pool.size() * sizeof(ScrollHintRect),
                         hipMemcpyHostToDevice));
    b->hint_dirty = 0;
    return SCROLL_OK;
}

/* the dynamic rect under hints: record / word pools for every frame's rect
 * MBs, staging slots grown to the largest NAL such a frame composes */
static int hd_setup(ScrollBatch *b)
{
    const size_t S = (size_t)b->max_streams, F = (size_t)b->max_frames;
    const size_t nmb = (size_t)b->geo.w * b->geo.h;
    const size_t words = S * F * nmb * b->hd_mb_words + 2 + RWIN_SLACK_WORDS;   /* + the stage's look-ahead */
    int rc;
    if (!b->d_spf) {
        HIPCHK(hipMalloc(&b->d_spf, S * F * sizeof(SpliceFrame)));
        HIPCHK(hipMemset(b->d_spf, 0, S * F * sizeof(SpliceFrame)));
    }
    if ((rc = sp_grow((void **)&b->d_sp_rbsp, &b->sp_rbsp_cap, words, sizeof(uint32_t))) ||
        (rc = sp_grow((void **)&b->d_sp_rec, &b->sp_rec_cap, S * F * nmb, sizeof(SpliceMbRec))))
        return rc;
    const size_t slot = splice_slot_bound(b->dyn_pw / 16, b->dyn_ph / 16, b->geo.w, b->geo.h,
                                          nmb * 4 * b->hd_mb_words);
    if (slot > b->geo.slot_bytes) {
        void *ns = nullptr;
        hipError_t e = hipMalloc(&ns, S * F * slot);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            set_err("dynamic rect under hints: staging (%zu bytes per frame): %s", slot,
                    hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        (void)hipFree(b->d_stage);
        b->d_stage = (uint8_t *)ns;
        b->geo.slot_bytes = slot;
    }
    b->hd_dirty = 1;
    b->hint_dirty = 1;
    return SCROLL_OK;
}

/* every frame's rect position -> d_spf (records and words at fixed places) */
static int hd_upload(ScrollBatch *b)
{
    const size_t S = (size_t)b->max_streams, F = (size_t)b->max_frames;
    const size_t nmb = (size_t)b->geo.w * b->geo.h;
    std::vector<SpliceFrame> spf(S * F);
    for (size_t i = 0; i < S * F; ++i) {
        SpliceFrame &o = spf[i];
        o = SpliceFrame{};
        const bool dormant = b->h_dyn_pos[2 * i] < 0;
        if (dormant && !b->fallback) continue;
        /* the fallback: a frame without the rect keeps a dormant whole-picture
         * region (pad 1) that k_hdyn_code codes only if k_hint_fb marks it */
        o.x0 = dormant ? 0 : b->h_dyn_pos[2 * i];
        o.y0 = dormant ? 0 : b->h_dyn_pos[2 * i + 1];
        o.pad = dormant ? 1 : 0;
        o.w = b->geo.w;
        o.h = b->geo.h;
        o.rbsp_word = i * nmb * b->hd_mb_words;
        o.rec_first = (uint32_t)(i * nmb);
        const int fq = i < b->h_dyn_qp.size() ? b->h_dyn_qp[i] : -1;
        const size_t st = i / F;
        o.hd_qp = fq >= 0 ? fq : (st < (size_t)b->nstreams ? b->h_st[st].dyn_qp : b->dyn_qp);
    }
    HIPCHK(hipMemcpy(b->d_spf, spf.data(), S * F * sizeof(SpliceFrame), hipMemcpyHostToDevice));
    b->hd_dirty = 0;
    return SCROLL_OK;
}

/* the rect's QP of stream s (every stream: s < 0); with the deblocking
 * filter on (no deblocking_filter_control_present_flag: ingested streams may
 * have it) a QP other than 26 would change the filtering of the scroll
 * region's MBs (their QP follows the slice / the coded MBs before them), so
 * it is refused for such streams */
static int set_stream_qp(ScrollBatch *b, int s, int qp, const char *who)
{
    if (!b || qp < SCROLL_DYN_QP_MIN || qp > SCROLL_DYN_QP_MAX || s >= b->nstreams) {
        set_err("%s: QP %d outside %d..%d or stream %d out of range", who, qp, SCROLL_DYN_QP_MIN,
                SCROLL_DYN_QP_MAX, s);
        return SCROLL_ERR_ARG;
    }
    const int s0 = s < 0 ? 0 : s, s1 = s < 0 ? b->nstreams : s + 1;
    for (int k = s0; k < s1; ++k)
        if (qp != 26 && !b->h_st[k].deblock) {
            set_err("%s: stream %d has the deblocking filter on (no "
                    "deblocking_filter_control_present_flag): its rect codes at QP 26", who, k);
            return SCROLL_ERR_CONFIG;
        }
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    for (int k = s0; k < s1; ++k) {
        b->h_st[k].dyn_qp = qp;
        HIPCHK(hipMemcpy(&b->d_st[k].dyn_qp, &qp, sizeof(int32_t), hipMemcpyHostToDevice));
    }
    if (s < 0) b->dyn_qp = qp;         /* streams added later */
    b->hd_dirty = 1;                   /* under hints: frames without their own QP follow the stream */
    return SCROLL_OK;
}

int scroll_batch_set_dyn_qp(ScrollBatch *b, int qp)
{
    return set_stream_qp(b, -1, qp, "scroll_batch_set_dyn_qp");
}

int scroll_batch_set_dyn_qp_stream(ScrollBatch *b, int s, int qp)
{
    if (!b || s < 0) {
        set_err("scroll_batch_set_dyn_qp_stream: bad stream");
        return SCROLL_ERR_ARG;
    }
    return set_stream_qp(b, s, qp, "scroll_batch_set_dyn_qp_stream");
}

int scroll_batch_set_dyn_qp_at(ScrollBatch *b, int s, int f, int qp)
{
    if (!b || !b->hint_on || !b->dyn_on || s < 0 || s >= b->nstreams || f < 0 || f >= b->max_frames ||
        qp < -1 || qp > SCROLL_DYN_QP_MAX) {
        set_err("scroll_batch_set_dyn_qp_at: needs UI hints and the dynamic rect; stream / frame / QP "
                "(-1, 0..%d) out of range", SCROLL_DYN_QP_MAX);
        return SCROLL_ERR_ARG;
    }
    if (qp >= 0 && qp != 26 && !b->h_st[s].deblock) {
        set_err("scroll_batch_set_dyn_qp_at: stream %d has the deblocking filter on: its rect codes at QP 26",
                s);
        return SCROLL_ERR_CONFIG;
    }
    int rc = batch_host_sync(b);
    if (rc) return rc;
    const size_t i = (size_t)s * b->max_frames + f;
    if (b->h_dyn_qp.size() < (size_t)b->max_streams * b->max_frames)
        b->h_dyn_qp.assign((size_t)b->max_streams * b->max_frames, -1);
    b->h_dyn_qp[i] = qp;
    b->hd_dirty = 1;
    return SCROLL_OK;
}

int scroll_batch_set_hints(ScrollBatch *b, int s, int f, const ScrollHintRect *rects, int n,
                           int mode)
{
    if (!b || s < 0 || s >= b->nstreams || f < 0 || f >= b->max_frames || n < 0 ||
        n > SCROLL_HINT_MAX_RECTS || (n > 0 && !rects) ||
        (mode != SCROLL_HINT_EXACT && mode != SCROLL_HINT_PSKIP && mode != SCROLL_HINT_SPEC)) {
        set_err("scroll_batch_set_hints: bad arguments");
        return SCROLL_ERR_ARG;
    }
    for (int i = 0; i < n; ++i) {
        const ScrollHintRect &r = rects[i];
        if (r.ref < 0 || r.ref >= 2 + 8 || r.mv_x < -SCROLL_HINT_MAX_MV ||
            r.mv_x > SCROLL_HINT_MAX_MV || r.mv_y < -SCROLL_HINT_MAX_MV ||
            r.mv_y > SCROLL_HINT_MAX_MV) {
            set_err("scroll_batch_set_hints: rect %d: ref %d / mv (%d, %d) out of range", i,
                    r.ref, r.mv_x, r.mv_y);
            return SCROLL_ERR_ARG;
        }
    }
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    if (!b->hint_on) {
        int mb = 0;
        for (int k = 0; k < b->nstreams; ++k) {
            mb = std::max(mb, (b->h_st[k].w / 16) * (b->h_st[k].h / 16));
            if (b->h_st[k].w / 16 > HINT_MAX_MBW) {
                set_err("scroll_batch_set_hints: stream %d is wider than %d MBs", k, HINT_MAX_MBW);
                return SCROLL_ERR_CONFIG;
            }
        }
        const size_t slot = hint_slot_bound(1, mb);     /* slots from the MB count only */
        const size_t S = (size_t)b->max_streams, F = (size_t)b->max_frames;
        hipError_t e = hipSuccess;
        if (b->dyn_on) {
            /* the dynamic rect's DynFrames stay; its EP-list buffer becomes
             * the hint path's staging slots (hd_setup grows them for the rect) */
            void *ns = nullptr;
            e = hipMalloc(&ns, S * F * slot);
            if (e == hipSuccess) e = hipMalloc(&b->d_hf, S * F * sizeof(HintFrame));
            if (e != hipSuccess) {
                (void)hipFree(ns);
                (void)hipFree(b->d_hf);
                b->d_hf = nullptr;
                (void)hipGetLastError();
                set_err("scroll_batch_set_hints: %s", hipGetErrorString(e));
                return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
            }
            (void)hipFree(b->d_stage);
            b->d_stage = (uint8_t *)ns;
        } else {
            e = hipMalloc(&b->d_dfr, S * F * sizeof(DynFrame));
            if (e == hipSuccess) e = hipMalloc(&b->d_stage, S * F * slot);
            if (e == hipSuccess) e = hipMalloc(&b->d_hf, S * F * sizeof(HintFrame));
            if (e == hipSuccess) e = hipMemset(b->d_dfr, 0, S * F * sizeof(DynFrame));
            if (e != hipSuccess) {
                set_err("scroll_batch_set_hints: %s", hipGetErrorString(e));
                hint_release(b);
                return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
            }
            b->geo = DynGeom{};
        }
        b->geo.slot_bytes = slot;
        b->hint_max_mb = mb;
        b->h_hint.assign(S * F, {});
        b->h_hint_mode.assign(S * F, (int16_t)SCROLL_HINT_EXACT);
        b->hint_on = 1;
        if (b->dyn_on && (rc = hd_setup(b))) return rc;
    }
    const size_t i = (size_t)s * b->max_frames + f;
    b->h_hint[i].assign(rects, rects + n);
    b->h_hint_mode[i] = (int16_t)mode;
    b->hint_dirty = 1;
    return SCROLL_OK;
}

int scroll_batch_clear_hints(ScrollBatch *b)
{
    if (!b) return SCROLL_ERR_ARG;
    if (!b->hint_on) return SCROLL_OK;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    hint_release(b);
    if (b->dyn_on) {                   /* the dynamic rect alone again: its DynFrames + EP lists */
        const size_t S = (size_t)b->max_streams, F = (size_t)b->max_frames;
        hipError_t e = hipMalloc(&b->d_dfr, S * F * sizeof(DynFrame));
        if (e == hipSuccess) e = hipMalloc(&b->d_stage, S * F * (size_t)4 * b->geo.ep_cap);
        if (e == hipSuccess) e = hipMemset(b->d_dfr, 0, S * F * sizeof(DynFrame));
        if (e != hipSuccess) {
            set_err("scroll_batch_clear_hints: %s", hipGetErrorString(e));
            dyn_release(b);
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->geo.slot_bytes = b->dyn_cap;
        if (b->dyn_pos_custom) {
            for (size_t i = 0; i < S * F; ++i) {
                b->h_dyn_pos[2 * i] = b->geo.x0;
                b->h_dyn_pos[2 * i + 1] = b->geo.y0;
            }
            b->dyn_pos_custom = 0;
        }
    }
    return SCROLL_OK;
}

/* ------------------------- pre-encoded MB splice --------------------------- */
/* grow a device buffer to n elements of `size` bytes (contents dropped) */
static int sp_grow(void **p, size_t *cap, size_t n, size_t size)
{
    if (n <= *cap) return SCROLL_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, std::max<size_t>(n, 1) * size);
    if (e != hipSuccess) {
        set_err("splice: %s", hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
    }
    *cap = n;
    return SCROLL_OK;
}

/* host splices -> device (table, NAL pool, pools sized for the parse) and
 * staging slots grown to the largest spliced NAL's bound; k_splice_parse
 * runs on the next compose's stream */
static int splice_upload(ScrollBatch *b)
{
    const size_t S = (size_t)b->max_streams, F = (size_t)b->max_frames;
    std::vector<SpliceFrame> spf(S * F);
    for (SpliceFrame &o : spf) o.hd_qp = -1;             /* spliced slices keep their own QP chain */
    std::vector<int32_t> list;
    std::vector<uint8_t> pool;
    size_t words = 0, recs = 0, nunits = 0, slot = b->geo.slot_bytes;
    int ymax = 1;
    std::vector<size_t> pool_off(b->h_sp.size(), 0);
    for (size_t i = 0; i < b->h_sp.size(); ++i) {
        const ScrollBatch::SpliceHost &h = b->h_sp[i];
        SpliceFrame &o = spf[i];
        o = SpliceFrame{};
        o.hd_qp = -1;
        if (h.w <= 0) continue;
        o.x0 = h.x0;
        o.y0 = h.y0;
        o.w = h.w;
        o.h = h.h;
        o.nal_len = (uint32_t)h.n;
        o.rbsp_word = words;
        o.rec_first = (uint32_t)recs;
        if (!h.dnal) {                 /* host bytes -> the NAL pool */
            pool_off[i] = pool.size();
            pool.insert(pool.end(), h.nal.begin(), h.nal.end());
            pool.resize((pool.size() + 3) & ~(size_t)3);
        }
        words += (h.n + 3) / 4 + 2;    /* k_splice_parse's units stay below (len + 2) / 4 + 1 words */
        recs += (size_t)h.w * h.h;
        o.unit_first = (uint32_t)nunits;
        nunits += splice_unit_cap(h.w * h.h);
        ymax = std::max(ymax, (int)splice_unit_cap(h.w * h.h));
        list.push_back((int32_t)i);
        const DevStream &d = b->h_st[i / F];
        slot = std::max(slot, splice_slot_bound(d.w / 16, d.h / 16, h.w, h.h, h.n));
    }
    int rc;
    if (!b->d_spf) {
        HIPCHK(hipMalloc(&b->d_spf, S * F * sizeof(SpliceFrame)));
    }
    if ((rc = sp_grow((void **)&b->d_sp_nal, &b->sp_nal_cap, pool.size(), 1)) ||
        (rc = sp_grow((void **)&b->d_sp_rbsp, &b->sp_rbsp_cap, words + RWIN_SLACK_WORDS, sizeof(uint32_t))) ||
        (rc = sp_grow((void **)&b->d_sp_rec, &b->sp_rec_cap, recs, sizeof(SpliceMbRec))) ||
        (rc = sp_grow((void **)&b->d_sp_list, &b->sp_list_cap, list.size(), sizeof(int32_t))) ||
        (rc = sp_grow((void **)&b->d_sp_units, &b->sp_units_cap, nunits, sizeof(SpliceUnit))))
        return rc;
    if (1 + 2 * nunits > b->sp_lanes_cap) {
        if ((rc = sp_grow((void **)&b->d_sp_lanes, &b->sp_lanes_cap, 1 + 2 * nunits, sizeof(int32_t)))) return rc;
        HIPCHK(hipMemset(b->d_sp_lanes, 0, sizeof(int32_t)));     /* k_splice_fix keeps it zero after */
    }
    b->sp_nslots = nunits;
    if (slot > b->geo.slot_bytes) {
        /* the new slots first: on failure the old ones, the hints and the
         * splices stay as they were (sp_dirty stays set: the next compose
         * tries again, or the caller clears / shrinks the splices) */
        void *ns = nullptr;
        hipError_t e = hipMalloc(&ns, S * F * slot);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            set_err("scroll_batch_compose: splice staging (%zu bytes per frame): %s", slot,
                    hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        (void)hipFree(b->d_stage);
        b->d_stage = (uint8_t *)ns;
        b->geo.slot_bytes = slot;
    }
    for (size_t i = 0; i < b->h_sp.size(); ++i)
        if (b->h_sp[i].w > 0) spf[i].nal = b->h_sp[i].dnal ? b->h_sp[i].dnal : b->d_sp_nal + pool_off[i];
    HIPCHK(hipMemcpy(b->d_spf, spf.data(), S * F * sizeof(SpliceFrame), hipMemcpyHostToDevice));
    if (!pool.empty())
        HIPCHK(hipMemcpy(b->d_sp_nal, pool.data(), pool.size(), hipMemcpyHostToDevice));
    if (!list.empty())
        HIPCHK(hipMemcpy(b->d_sp_list, list.data(), list.size() * sizeof(int32_t),
                         hipMemcpyHostToDevice));
    b->sp_n = (int)list.size();
    b->sp_ymax = ymax;
    b->sp_parse = b->sp_n > 0;
    b->sp_dirty = 0;
    return SCROLL_OK;
}

int scroll_batch_set_splice(ScrollBatch *b, int s, int f, int x0, int y0, int w, int h,
                            const uint8_t *nal, size_t n)
{
    if (!b || s < 0 || s >= b->nstreams || f < 0 || f >= b->max_frames ||
        (n > 0 && (!nal || w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || n >= SCROLL_SPLICE_MAX_BYTES))) {
        set_err("scroll_batch_set_splice: bad arguments");
        return SCROLL_ERR_ARG;
    }
    if (n > 0 && (x0 + w > b->h_st[s].w / 16 || y0 + h > b->h_st[s].h / 16)) {
        set_err("scroll_batch_set_splice: rect (%d, %d) %dx%d MBs outside the %dx%d picture", x0,
                y0, w, h, b->h_st[s].w, b->h_st[s].h);
        return SCROLL_ERR_ARG;
    }
    if (b->dyn_on) {
        set_err("scroll_batch_set_splice: not combinable with a dynamic rect (one spliced rect per frame)");
        return SCROLL_ERR_CONFIG;
    }
    if (n == 0 && !b->hint_on) return SCROLL_OK;
    if (!b->hint_on) {                 /* the splice rides on the hint path, SPEC by default */
        int rc = scroll_batch_set_hints(b, s, f, nullptr, 0, SCROLL_HINT_SPEC);
        if (rc) return rc;
        std::fill(b->h_hint_mode.begin(), b->h_hint_mode.end(), (int16_t)SCROLL_HINT_SPEC);
    } else {
        int rc = batch_host_sync(b);
        if (rc) return rc;
    }
    const size_t i = (size_t)s * b->max_frames + f;
    if (b->h_sp.size() < (size_t)b->max_streams * b->max_frames)
        b->h_sp.resize((size_t)b->max_streams * b->max_frames);
    ScrollBatch::SpliceHost &sp = b->h_sp[i];
    if (n == 0) {
        sp = ScrollBatch::SpliceHost{};
    } else {
        sp.x0 = x0;
        sp.y0 = y0;
        sp.w = w;
        sp.h = h;
        sp.nal.assign(nal, nal + n);
        sp.dnal = nullptr;
        sp.n = n;
    }
    b->sp_dirty = 1;
    b->hint_dirty = 1;
    return SCROLL_OK;
}

int scroll_batch_set_splices_device(ScrollBatch *b, int n, const ScrollSpliceDesc *d)
{
    if (!b || n < 0 || (n > 0 && !d)) {
        set_err("scroll_batch_set_splices_device: bad arguments");
        return SCROLL_ERR_ARG;
    }
    for (int k = 0; k < n; ++k) {
        const ScrollSpliceDesc &e = d[k];
        const bool on = e.n > 0;
        if (e.s < 0 || e.s >= b->nstreams || e.f < 0 || e.f >= b->max_frames ||
            (on && (!e.nal || e.w <= 0 || e.h <= 0 || e.x0 < 0 || e.y0 < 0 ||
                    e.n >= SCROLL_SPLICE_MAX_BYTES || e.x0 + e.w > b->h_st[e.s].w / 16 ||
                    e.y0 + e.h > b->h_st[e.s].h / 16))) {
            set_err("scroll_batch_set_splices_device: entry %d: bad stream / frame / rect / size", k);
            return SCROLL_ERR_ARG;
        }
    }
    if (n == 0) return SCROLL_OK;
    if (b->dyn_on) {
        set_err("scroll_batch_set_splices_device: not combinable with a dynamic rect (one spliced rect per frame)");
        return SCROLL_ERR_CONFIG;
    }
    if (!b->hint_on) {
        int rc = scroll_batch_set_hints(b, d[0].s, d[0].f, nullptr, 0, SCROLL_HINT_SPEC);
        if (rc) return rc;
        std::fill(b->h_hint_mode.begin(), b->h_hint_mode.end(), (int16_t)SCROLL_HINT_SPEC);
    } else {
        int rc = batch_host_sync(b);
        if (rc) return rc;
    }
    if (b->h_sp.size() < (size_t)b->max_streams * b->max_frames)
        b->h_sp.resize((size_t)b->max_streams * b->max_frames);
    for (int k = 0; k < n; ++k) {
        const ScrollSpliceDesc &e = d[k];
        ScrollBatch::SpliceHost &sp = b->h_sp[(size_t)e.s * b->max_frames + e.f];
        sp = ScrollBatch::SpliceHost{};
        if (e.n == 0) continue;
        sp.x0 = e.x0;
        sp.y0 = e.y0;
        sp.w = e.w;
        sp.h = e.h;
        sp.dnal = e.nal;
        sp.n = (size_t)e.n;
    }
    b->sp_dirty = 1;
    b->hint_dirty = 1;
    return SCROLL_OK;
}

int scroll_batch_clear_splices(ScrollBatch *b)
{
    if (!b) return SCROLL_ERR_ARG;
    if (b->h_sp.empty()) return SCROLL_OK;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    b->h_sp.clear();
    b->sp_dirty = 1;
    b->hint_dirty = 1;
    return SCROLL_OK;
}

static int splice_frame_status(ScrollBatch *b, size_t i, int *status)
{
    *status = SCROLL_SPLICE_OK;
    const bool on = (i < b->h_sp.size() && b->h_sp[i].w > 0) ||
                    (b->hint_on && b->dyn_on && 2 * i < b->h_dyn_pos.size() && b->h_dyn_pos[2 * i] >= 0);
    if (!b->d_spf || !on) return SCROLL_OK;
    SpliceFrame sf;
    HIPCHK(hipMemcpy(&sf, b->d_spf + i, sizeof(sf), hipMemcpyDeviceToHost));
    *status = sf.status ? sf.status : sf.stage_status;
    return SCROLL_OK;
}

int scroll_batch_splice_status(ScrollBatch *b, int s, int f, int *status)
{
    if (!b || !status || s < 0 || s >= b->nstreams || f < 0 || f >= b->max_frames)
        return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    return splice_frame_status(b, (size_t)s * b->max_frames + f, status);
}

int scroll_batch_splice_refusal(ScrollBatch *b, int s, int f, int *status, int *mb_x, int *mb_y, int *mb_type)
{
    if (!b || !status || s < 0 || s >= b->nstreams || f < 0 || f >= b->max_frames)
        return SCROLL_ERR_ARG;
    int rc = batch_host_sync(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    const size_t i = (size_t)s * b->max_frames + f;
    rc = splice_frame_status(b, i, status);
    if (rc) return rc;
    int x = -1, y = -1, t = -1;
    if (*status == SCROLL_SPLICE_ERR_MBTYPE && b->d_spf) {
        SpliceFrame sf;
        HIPCHK(hipMemcpy(&sf, b->d_spf + i, sizeof(sf), hipMemcpyDeviceToHost));
        if (sf.bad_mb >= 0 && sf.w > 0) {
            const int m = sf.bad_mb & 0xffff;
            x = m % sf.w;
            y = m / sf.w;
            t = sf.bad_mb >> 16;
        }
    }
    if (mb_x) *mb_x = x;
    if (mb_y) *mb_y = y;
    if (mb_type) *mb_type = t;
    return SCROLL_OK;
}

static const char *splice_msg(int e)
{
    switch (e) {
    case SCROLL_SPLICE_ERR_NAL: return "not a coded slice of an IDR or non-IDR picture (or more than 1,024 slices)";
    case SCROLL_SPLICE_ERR_HEADER: return "slice header outside the supported syntax, or slices out of order";
    case SCROLL_SPLICE_ERR_MBTYPE: return "an intra MB whose prediction reads other samples in the composed picture";
    case SCROLL_SPLICE_ERR_SYNTAX: return "malformed or truncated slice data, or slices not covering the rect's MBs";
    case SCROLL_SPLICE_ERR_REF: return "a ref_idx that is not a valid reference of the frame";
    default: return "unknown";
    }
}

/* ------------------------------ stream ingest ------------------------------ */
static const char *ing_msg(int e)
{
    switch (e) {
    case ING_ERR_MISSING: return "reference file missing SPS/PPS/IDR";
    case ING_ERR_PARSE: return "unsupported SPS/PPS (scaling matrices, POC type 1 or slice groups)";
    case ING_ERR_DIMS: return "reference frame dimensions don't match";
    case ING_ERR_NALS: return "too many NAL units in a reference file";
    case ING_ERR_OVERFLOW: return "header larger than the stream arena";
    case ING_ERR_WAIT: return "a segment of the header waited too long for the one before it";
    default: return "ingest failed";
    }
}

int scroll_batch_ingest_device(ScrollBatch *b, int n, const uint8_t *d_files, const uint64_t *desc,
                               int *first)
{
    if (!b || n < 0 || (n > 0 && (!d_files || !desc))) return SCROLL_ERR_ARG;
    if (b->nstreams + n > b->max_streams) {
        set_err("scroll_batch_ingest: %d + %d streams exceed the batch (%d)", b->nstreams, n,
                b->max_streams);
        return SCROLL_ERR_ARG;
    }
    int rc = batch_host_sync(b);
    if (rc) return rc;
    if (first) *first = b->nstreams;
    if (n == 0) return SCROLL_OK;
    HIPCHK(hipSetDevice(b->device));
    if (n > b->ing_cap) {
        (void)hipFree(b->d_ing_files);
        (void)hipFree(b->d_ing_scan);
        (void)hipFree(b->d_ing_out);
        b->d_ing_files = nullptr;
        b->d_ing_scan = nullptr;
        b->d_ing_out = nullptr;
        b->ing_cap = 0;
        hipError_t e = hipMalloc(&b->d_ing_files, 2 * (size_t)n * sizeof(IngestFile));
        if (e == hipSuccess) e = hipMalloc(&b->d_ing_scan, 2 * (size_t)n * sizeof(IngestScan));
        if (e == hipSuccess) e = hipMalloc(&b->d_ing_out, (size_t)n * sizeof(IngestOut));
        if (e != hipSuccess) {
            set_err("scroll_batch_ingest: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->ing_cap = n;
    }
    std::vector<IngestFile> files(2 * (size_t)n);
    uint64_t maxf = 0, totf = 0;
    for (int k = 0; k < 2 * n; ++k) {
        files[k].off = desc[2 * k];
        files[k].size = desc[2 * k + 1];
        maxf = std::max(maxf, files[k].size);
        totf += files[k].size;
    }
    const bool serial = getenv("SCROLL_INGEST_SERIAL") != nullptr;
    /* the one-pass segments (default); round 4's three passes for
     * comparison (tests): SCROLL_INGEST_THREEPASS=1 stages the output bytes
     * while that scratch (every file sized like the largest, ~1.25x per
     * segment) stays within 4x the input plus 256 MB and under 8 GB, and
     * otherwise -- or with SCROLL_INGEST_RECOMPUTE=1 -- decodes again */
    int mode = ING_ONEPASS;
    if (getenv("SCROLL_INGEST_THREEPASS") || getenv("SCROLL_INGEST_RECOMPUTE")) {
        const size_t stg_bytes = ingest_work_bytes(n, maxf, ING_STAGED);
        mode = getenv("SCROLL_INGEST_RECOMPUTE") == nullptr && stg_bytes <= ((size_t)8 << 30) &&
                       stg_bytes <= 4 * (size_t)totf + ((size_t)256 << 20)
                   ? ING_STAGED
                   : ING_RECOMPUTE;
    }
    const size_t wb = serial ? 0 : ingest_work_bytes(n, maxf, mode);
    if (wb > b->ing_work_bytes) {
        (void)hipFree(b->d_ing_work);
        b->d_ing_work = nullptr;
        b->ing_work_bytes = 0;
        hipError_t e = hipMalloc(&b->d_ing_work, wb);
        if (e != hipSuccess) {
            set_err("scroll_batch_ingest: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->ing_work_bytes = wb;
    }
    hipStream_t hs = b->own;
    HIPCHK(hipMemcpyAsync(b->d_ing_files, files.data(), files.size() * sizeof(IngestFile),
                          hipMemcpyHostToDevice, hs));
    if (b->timing) {
        for (hipEvent_t &e : b->ing_ev)
            if (!e) HIPCHK(timing_event(&e));
        HIPCHK(hipEventRecord(b->ing_ev[0], hs));
    }
    if (ingest_launch(hs, d_files, b->d_ing_files, n, maxf, b->d_ing_scan, b->d_ing_out,
                      b->d_arena, (uint64_t)b->ld_arena, (uint64_t)b->arena_bytes, b->nstreams,
                      serial ? nullptr : b->d_ing_work, wb, mode)) {
        set_err("ingest launch: %s", hipGetErrorString(hipGetLastError()));
        return SCROLL_ERR_HIP;
    }
    if (b->timing) HIPCHK(hipEventRecord(b->ing_ev[1], hs));
    std::vector<IngestOut> outs((size_t)n);
    HIPCHK(hipMemcpyAsync(outs.data(), b->d_ing_out, outs.size() * sizeof(IngestOut),
                          hipMemcpyDeviceToHost, hs));
    HIPCHK(hipStreamSynchronize(hs));
    if (b->timing) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, b->ing_ev[0], b->ing_ev[1]) == hipSuccess) {
            b->ing_ms += ms;
            b->ing_n++;
        }
    }
    for (int k = 0; k < n; ++k) {
        if (outs[k].err != ING_OK) {
            set_err("scroll_batch_ingest: new stream %d: %s", k, ing_msg(outs[k].err));
            /* a segment's bounded look-back wait is a device hand-off failure,
             * not a bad file (as k_dyn_row's DF_HANDOFF) */
            return outs[k].err == ING_ERR_OVERFLOW ? SCROLL_ERR_OVERFLOW
                   : outs[k].err == ING_ERR_WAIT   ? SCROLL_ERR_DEVICE
                                                   : SCROLL_ERR_CONFIG;
        }
        if ((b->dyn_on && (outs[k].w != b->dyn_pw || outs[k].h != b->dyn_ph)) ||
            (b->hint_on && ((outs[k].w / 16) * (outs[k].h / 16) > b->hint_max_mb ||
                            outs[k].w / 16 > HINT_MAX_MBW))) {
            set_err("scroll_batch_ingest: new stream %d (%dx%d) does not fit the batch's "
                    "dynamic rect / hint slots", k, outs[k].w, outs[k].h);
            return SCROLL_ERR_CONFIG;
        }
    }
    /* the config composer_init derives (src/composer.c:193-203), frame_num 2
     * after composer_write_header */
    const int s0 = b->nstreams;
    for (int k = 0; k < n; ++k) {
        /* the rule add_stream enforces: the loop filter on (no
         * deblocking_filter_control_present_flag) keeps the rect at QP 26 */
        if (b->dyn_qp != 26 && !outs[k].deblock) {
            set_err("scroll_batch_ingest: new stream %d has the deblocking filter on (no "
                    "deblocking_filter_control_present_flag); the batch's rect QP is %d, not 26", k, b->dyn_qp);
            return SCROLL_ERR_CONFIG;
        }
    }
    for (int k = 0; k < n; ++k) {
        ComposerConfig cfg;
        composer_config_init(&cfg, outs[k].w, outs[k].h);
        composer_config_set_sps_params(&cfg, 4, 2, 4);
        composer_config_set_pps_params(&cfg, 1, outs[k].deblock);
        cfg.frame_num = 2;
        if ((rc = check_cfg(&cfg))) return rc;
        DevStream *d = &b->h_st[s0 + k];
        memset(d, 0, sizeof(*d));
        cfg_to_dev(&cfg, d);
        d->dyn_qp = b->dyn_qp;              /* the batch's rect QP, as add_stream sets it */
        d->out_pos = outs[k].bytes;
        d->undelivered = outs[k].bytes;     /* SPS + PPS + A + B go out with the first delivery */
        d->out_cap = b->arena_bytes;
    }
    HIPCHK(hipMemcpy(b->d_st + s0, b->h_st + s0, (size_t)n * sizeof(DevStream),
                     hipMemcpyHostToDevice));
    b->nstreams += n;
    return SCROLL_OK;
}

int scroll_batch_ingest_stats(ScrollBatch *b, double *ms, int *count)
{
    if (!b) return SCROLL_ERR_ARG;
    if (ms) *ms = b->ing_ms;
    if (count) *count = b->ing_n;
    b->ing_ms = 0.0;
    b->ing_n = 0;
    return SCROLL_OK;
}

/* ------------------- reference files from pictures (I_PCM) ------------------ */
/* the I_PCM files of n pictures; sizes: host (synchronous call) or device
 * (d_sizes, asynchronous: the overflow check waits for the next sync) */
static int ipcm_files(ScrollBatch *b, int n, int w, int h, const uint8_t *d_pics, size_t pic_stride, uint8_t *d_out,
                      size_t out_stride, uint64_t *sizes, uint64_t *d_sizes_out)
{
    const bool async = d_sizes_out != nullptr;
    if (!b || n < 0 || (n > 0 && (!d_pics || !d_out || !(sizes || d_sizes_out)))) return SCROLL_ERR_ARG;
    if (n == 0) return SCROLL_OK;
    const size_t nmb = (size_t)(w / 16) * (size_t)(h / 16);
    if (w <= 0 || h <= 0 || (w & 15) || (h & 15) || nmb >= 65536 ||
        pic_stride < (size_t)w * h * 3 / 2) {
        set_err("scroll_batch_ipcm_files: %dx%d pictures (stride %zu) not supported", w, h, pic_stride);
        return SCROLL_ERR_ARG;
    }
    if (!async) {
        int rc = batch_host_sync(b);
        if (rc) return rc;
    }
    HIPCHK(hipSetDevice(b->device));
    if (async && !b->ipcm_over) {                   /* the sticky overflow flag (read at the next sync) */
        if (!b->d_ipcm_sticky) HIPCHK(hipMalloc(&b->d_ipcm_sticky, sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(b->d_ipcm_sticky, 0, sizeof(uint32_t), b->own));
    }
    IpcmGeom g{};
    g.w = w;
    g.h = h;
    g.mbw = (uint32_t)(w / 16);
    g.nmb = (uint32_t)nmb;
    g.m_mbw = g.mbw <= 1 ? 0u : 0xffffffffu / g.mbw + 1u;
    g.m_386 = 0;
    g.pic_stride = pic_stride;
    g.out_stride = out_stride;
    /* prefix: SPS, PPS (h264_generate_sps / _pps, identical in the composer
     * and the experiment) as NAL units, then the IDR's start code + header */
    {
        uint8_t rbsp[64];
        NALWriter nw;
        uint8_t tmp[64];
        nal_writer_init(&nw, g.pre, IPCM_PRE_MAX, tmp, sizeof(tmp));
        size_t k = h264_generate_sps(rbsp, sizeof(rbsp), w, h);
        nal_write_unit(&nw, 3, 7, rbsp, k, 1);
        k = h264_generate_pps(rbsp, sizeof(rbsp));
        nal_write_unit(&nw, 3, 8, rbsp, k, 1);
        size_t o = nal_writer_get_size(&nw);
        const uint8_t idr[5] = {0, 0, 0, 1, (uint8_t)(3 << 5 | 5)};
        memcpy(g.pre + o, idr, 5);
        g.npre = (uint32_t)(o + 5);
    }
    /* IDR slice header with the experiment's defaults (h264_encoder.c:12-29,
     * :622-662) + MB 0's mb_type ue(25) and alignment (:730-736) */
    {
        BitWriter bw;
        bitwriter_init(&bw, g.hdr, sizeof(g.hdr));
        bitwriter_write_ue(&bw, 0);          /* first_mb_in_slice */
        bitwriter_write_ue(&bw, 7);          /* slice_type I (all) */
        bitwriter_write_ue(&bw, 0);          /* pic_parameter_set_id */
        bitwriter_write_bits(&bw, 0, 4);     /* frame_num, log2_max_frame_num 4 */
        bitwriter_write_ue(&bw, 0);          /* idr_pic_id */
        bitwriter_write_bit(&bw, 0);         /* no_output_of_prior_pics_flag */
        bitwriter_write_bit(&bw, 1);         /* long_term_reference_flag */
        bitwriter_write_se(&bw, 0);          /* slice_qp_delta */
        bitwriter_write_ue(&bw, 1);          /* disable_deblocking_filter_idc */
        bitwriter_write_ue(&bw, 25);         /* mb_type I_PCM */
        while (!bitwriter_is_byte_aligned(&bw)) bitwriter_write_bit(&bw, 0);
        g.nh = (uint32_t)bitwriter_get_size(&bw);
    }
    g.rbsp_len = (uint32_t)(g.nh - 2 + 386 * nmb + 1);
    g.nchunk = (g.rbsp_len + IPCM_CHUNK - 1) / IPCM_CHUNK;
    /* counts [n][nchunk] u32, then sizes [n] u64, then the over flag */
    const size_t cnt_bytes = ((size_t)n * g.nchunk * sizeof(uint32_t) + 7) & ~(size_t)7;
    const size_t need = cnt_bytes + (size_t)n * sizeof(uint64_t) + sizeof(uint64_t);
    if (need > b->ipcm_cap && async && b->ipcm_over) {
        /* an earlier asynchronous call may still use the scratch */
        HIPCHK(hipStreamSynchronize(b->own));
    }
    if (need > b->ipcm_cap) {
        (void)hipFree(b->d_ipcm_cnt);
        b->d_ipcm_cnt = nullptr;
        b->ipcm_cap = 0;
        hipError_t e = hipMalloc(&b->d_ipcm_cnt, need);
        if (e != hipSuccess) {
            set_err("scroll_batch_ipcm_files: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->ipcm_cap = need;
    }
    /* SCROLL_IPCM_ONEPASS=1: the one pass when no file can overflow
     * out_stride -- 1.54x the algorithmic bytes instead of 2.50x, but 0.67
     * against 0.57 ms per ipcm720 call (its look-back holds each workgroup
     * for a round trip; profiles/r06o_ipcm_onepass.txt), so not the default */
    const bool one = getenv("SCROLL_IPCM_ONEPASS") != nullptr && out_stride >= ipcm_worst(&g);
    if (one && (size_t)n * g.nchunk > b->ipcm_hw_cap) {
        if (async && b->ipcm_over) HIPCHK(hipStreamSynchronize(b->own));
        (void)hipFree(b->d_ipcm_hw);
        b->d_ipcm_hw = nullptr;
        b->ipcm_hw_cap = 0;
        const size_t words = (size_t)n * g.nchunk;
        hipError_t e = hipMalloc(&b->d_ipcm_hw, words * sizeof(unsigned long long));
        if (e != hipSuccess) {
            set_err("scroll_batch_ipcm_files: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        HIPCHK(hipMemsetAsync(b->d_ipcm_hw, 0, words * sizeof(unsigned long long), b->own));
        b->ipcm_hw_cap = words;
    }
    /* the write pass reads the count pass's RBSP while that scratch stays
     * under 4 GB, else it generates the bytes again */
    const uint64_t stg_stride = (uint64_t)g.nchunk * IPCM_CHUNK;
    const size_t stg_need = (size_t)n * stg_stride;
    uint8_t *stg = nullptr;
    if (!one && getenv("SCROLL_IPCM_RECOMPUTE") == nullptr && stg_need <= ((size_t)4 << 30)) {
        if (stg_need > b->ipcm_stg_cap) {
            (void)hipFree(b->d_ipcm_stg);
            b->d_ipcm_stg = nullptr;
            b->ipcm_stg_cap = 0;
            if (hipMalloc(&b->d_ipcm_stg, stg_need) == hipSuccess) b->ipcm_stg_cap = stg_need;
            else (void)hipGetLastError();               /* no scratch: the generating write pass */
        }
        if (b->d_ipcm_stg) stg = b->d_ipcm_stg;
    }
    hipStream_t hs = b->own;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (b->timing && !async) {
        for (hipEvent_t &e : b->ing_ev)                  /* created lazily, shared with ingest */
            if (!e) HIPCHK(timing_event(&e));
        e0 = b->ing_ev[0];
        e1 = b->ing_ev[1];
    } else if (b->timing) {                             /* a pair per call, read at the stats */
        if (b->ipcm_ev.size() < b->ipcm_ev_used + 2) {
            for (int k = 0; k < 2; ++k) {
                hipEvent_t e;
                HIPCHK(timing_event(&e));
                b->ipcm_ev.push_back(e);
            }
        }
        e0 = b->ipcm_ev[b->ipcm_ev_used];
        e1 = b->ipcm_ev[b->ipcm_ev_used + 1];
        b->ipcm_ev_used += 2;
    }
    if (async && b->last && b->last != hs) {
        /* a compose queued on a caller's stream: own waits for it, so that
         * b->last = own below still covers it (the next sync must not copy
         * d_st back while that compose runs) */
        if (!b->out_ev) HIPCHK(hipEventCreateWithFlags(&b->out_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(b->out_ev, b->last));
        HIPCHK(hipStreamWaitEvent(hs, b->out_ev, 0));
    }
    if (e0) HIPCHK(hipEventRecord(e0, hs));
    uint64_t *d_sizes = async ? d_sizes_out
                              : reinterpret_cast<uint64_t *>(reinterpret_cast<uint8_t *>(b->d_ipcm_cnt) + cnt_bytes);
    uint32_t *d_over = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(b->d_ipcm_cnt) + cnt_bytes +
                                                    (size_t)n * sizeof(uint64_t));
    /* count pass, sizes and the overflow check, write pass: no host step in
     * between (the write pass writes nothing when a file is over) */
    uint32_t *sticky = async ? b->d_ipcm_sticky : nullptr;
    if (one) {
        b->ipcm_epoch = b->ipcm_epoch % 0xffffffu + 1u;          /* 24 bits, never 0 */
        const IpcmOnePass op{b->d_ipcm_hw, b->ipcm_epoch, d_sizes, sticky};
        if (ipcm_launch_onepass(hs, n, &g, d_pics, d_out, d_over, &op)) {
            set_err("ipcm launch: %s", hipGetErrorString(hipGetLastError()));
            return SCROLL_ERR_HIP;
        }
    } else if (ipcm_launch(hs, 0, n, &g, d_pics, b->d_ipcm_cnt, d_out, stg, stg_stride, d_sizes, d_over, sticky) ||
               ipcm_launch(hs, 1, n, &g, d_pics, b->d_ipcm_cnt, d_out, stg, stg_stride, d_sizes, d_over, sticky)) {
        set_err("ipcm launch: %s", hipGetErrorString(hipGetLastError()));
        return SCROLL_ERR_HIP;
    }
    if (e1) HIPCHK(hipEventRecord(e1, hs));
    if (async) {
        /* nothing comes back now: the overflow flag is read at the next sync */
        b->ipcm_over = b->d_ipcm_sticky;
        b->ipcm_over_stride = out_stride;
        b->last = hs;
        b->host_valid = 0;
        return SCROLL_OK;
    }
    uint32_t over_flag = 0;
    HIPCHK(hipMemcpyAsync(sizes, d_sizes, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost, hs));
    HIPCHK(hipMemcpyAsync(&over_flag, d_over, sizeof(uint32_t), hipMemcpyDeviceToHost, hs));
    HIPCHK(hipStreamSynchronize(hs));
    if (e0) {
        float ms = 0.0f;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        b->ipcm_ms += ms;
        b->ipcm_n++;
    }
    if (over_flag) {
        int over = 0;
        while (over < n && sizes[over] <= out_stride) ++over;
        set_err("scroll_batch_ipcm_files: file %d needs %llu bytes, out_stride is %zu", over,
                (unsigned long long)sizes[over < n ? over : 0], out_stride);
        return SCROLL_ERR_OVERFLOW;
    }
    return SCROLL_OK;
}

int scroll_batch_ipcm_files_device(ScrollBatch *b, int n, int w, int h, const uint8_t *d_pics,
                                   size_t pic_stride, uint8_t *d_out, size_t out_stride,
                                   uint64_t *sizes)
{
    return ipcm_files(b, n, w, h, d_pics, pic_stride, d_out, out_stride, sizes, nullptr);
}

int scroll_batch_ipcm_files_device_async(ScrollBatch *b, int n, int w, int h, const uint8_t *d_pics,
                                         size_t pic_stride, uint8_t *d_out, size_t out_stride,
                                         uint64_t *d_sizes)
{
    if (!b || (n > 0 && !d_sizes)) return SCROLL_ERR_ARG;
    return ipcm_files(b, n, w, h, d_pics, pic_stride, d_out, out_stride, nullptr, d_sizes);
}

/* the asynchronous I_PCM calls' outcome (scroll_batch_sync): their overflow
 * flag, after the stream is idle */
static int ipcm_async_check(ScrollBatch *b)
{
    if (!b->ipcm_over) return SCROLL_OK;
    uint32_t over = 0;
    HIPCHK(hipStreamSynchronize(b->own));
    HIPCHK(hipMemcpy(&over, b->ipcm_over, sizeof(over), hipMemcpyDeviceToHost));
    b->ipcm_over = nullptr;
    if (over) {
        set_err("scroll_batch_ipcm_files_device_async: a file exceeded out_stride (%zu bytes): "
                "its call wrote no file", b->ipcm_over_stride);
        return SCROLL_ERR_OVERFLOW;
    }
    return SCROLL_OK;
}

int scroll_batch_ipcm_stats(ScrollBatch *b, double *ms, int *count)
{
    if (!b) return SCROLL_ERR_ARG;
    if (b->ipcm_ev_used) {                              /* the asynchronous calls' pairs */
        HIPCHK(hipStreamSynchronize(b->own));
        for (size_t k = 0; k + 1 < b->ipcm_ev_used; k += 2) {
            float v = 0.0f;
            HIPCHK(hipEventElapsedTime(&v, b->ipcm_ev[k], b->ipcm_ev[k + 1]));
            b->ipcm_ms += v;
            b->ipcm_n++;
        }
        b->ipcm_ev_used = 0;
    }
    if (ms) *ms = b->ipcm_ms;
    if (count) *count = b->ipcm_n;
    b->ipcm_ms = 0.0;
    b->ipcm_n = 0;
    return SCROLL_OK;
}

int scroll_batch_ingest(ScrollBatch *b, int n, const uint8_t *const *ref_a, const size_t *na,
                        const uint8_t *const *ref_b, const size_t *nb, int *first)
{
    if (!b || n < 0 || (n > 0 && (!ref_a || !na || !ref_b || !nb))) return SCROLL_ERR_ARG;
    if (n == 0) return scroll_batch_ingest_device(b, 0, nullptr, nullptr, first);
    std::vector<uint64_t> desc(4 * (size_t)n);
    size_t tot = 0;
    for (int k = 0; k < n; ++k) {
        if ((na[k] && !ref_a[k]) || (nb[k] && !ref_b[k])) return SCROLL_ERR_ARG;
        desc[4 * k] = tot;
        desc[4 * k + 1] = na[k];
        tot += (na[k] + 255) & ~(size_t)255;
        desc[4 * k + 2] = tot;
        desc[4 * k + 3] = nb[k];
        tot += (nb[k] + 255) & ~(size_t)255;
    }
    HIPCHK(hipSetDevice(b->device));
    if (tot > b->ing_in_cap) {
        (void)hipFree(b->d_ing_in);
        b->d_ing_in = nullptr;
        b->ing_in_cap = 0;
        hipError_t e = hipMalloc(&b->d_ing_in, tot);
        if (e != hipSuccess) {
            set_err("scroll_batch_ingest: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->ing_in_cap = tot;
    }
    for (int k = 0; k < n; ++k) {
        if (na[k]) HIPCHK(hipMemcpy(b->d_ing_in + desc[4 * k], ref_a[k], na[k], hipMemcpyHostToDevice));
        if (nb[k]) HIPCHK(hipMemcpy(b->d_ing_in + desc[4 * k + 2], ref_b[k], nb[k], hipMemcpyHostToDevice));
    }
    return scroll_batch_ingest_device(b, n, b->d_ing_in, desc.data(), first);
}

/* mid-stream long-term reference updates (k_ing_update, ingest_kernels.hip) */
int scroll_batch_update_refs_device(ScrollBatch *b, int n, const int *streams, const int *which,
                                    const uint8_t *d_files, const uint64_t *desc, int *status)
{
    if (!b || n < 0 || (n > 0 && (!streams || !which || !d_files || !desc))) return SCROLL_ERR_ARG;
    std::vector<uint8_t> seen((size_t)b->nstreams, 0);
    for (int k = 0; k < n; ++k) {
        if (streams[k] < 0 || streams[k] >= b->nstreams || which[k] < 0 || which[k] > 1 || seen[streams[k]]) {
            set_err("scroll_batch_update_refs: entry %d: bad or repeated stream / which", k);
            return SCROLL_ERR_ARG;
        }
        seen[streams[k]] = 1;
    }
    if (n == 0) return SCROLL_OK;
    HIPCHK(hipSetDevice(b->device));
    if (n > b->ing_cap) {
        (void)hipFree(b->d_ing_files);
        (void)hipFree(b->d_ing_scan);
        (void)hipFree(b->d_ing_out);
        b->d_ing_files = nullptr;
        b->d_ing_scan = nullptr;
        b->d_ing_out = nullptr;
        b->ing_cap = 0;
        hipError_t e = hipMalloc(&b->d_ing_files, 2 * (size_t)n * sizeof(IngestFile));
        if (e == hipSuccess) e = hipMalloc(&b->d_ing_scan, 2 * (size_t)n * sizeof(IngestScan));
        if (e == hipSuccess) e = hipMalloc(&b->d_ing_out, (size_t)n * sizeof(IngestOut));
        if (e != hipSuccess) {
            set_err("scroll_batch_update_refs: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->ing_cap = n;
    }
    if ((size_t)n > b->upd_cap) {
        (void)hipFree(b->d_upd);
        b->d_upd = nullptr;
        b->upd_cap = 0;
        HIPCHK(hipMalloc(&b->d_upd, 2 * (size_t)n * sizeof(int32_t)));
        b->upd_cap = (size_t)n;
    }
    std::vector<IngestFile> files((size_t)n);
    std::vector<int32_t> ups(2 * (size_t)n);
    uint64_t maxf = 0;
    for (int k = 0; k < n; ++k) {
        files[k].off = desc[2 * k];
        files[k].size = desc[2 * k + 1];
        maxf = std::max(maxf, files[k].size);
        ups[2 * k] = streams[k];
        ups[2 * k + 1] = which[k];
    }
    hipStream_t hs = b->last ? b->last : b->own;   /* after the pending composes */
    HIPCHK(hipMemcpyAsync(b->d_ing_files, files.data(), files.size() * sizeof(IngestFile),
                          hipMemcpyHostToDevice, hs));
    HIPCHK(hipMemcpyAsync(b->d_upd, ups.data(), ups.size() * sizeof(int32_t), hipMemcpyHostToDevice, hs));
    if (update_launch(hs, d_files, b->d_ing_files, n, maxf, b->d_ing_scan, b->d_upd, b->d_ing_out, b->d_st,
                      b->d_arena, (uint64_t)b->ld_arena)) {
        set_err("reference update launch: %s", hipGetErrorString(hipGetLastError()));
        return SCROLL_ERR_HIP;
    }
    std::vector<IngestOut> outs((size_t)n);
    HIPCHK(hipMemcpyAsync(outs.data(), b->d_ing_out, outs.size() * sizeof(IngestOut), hipMemcpyDeviceToHost, hs));
    HIPCHK(hipStreamSynchronize(hs));
    b->host_valid = 0;
    b->nal_cache_valid = 0;
    int rc = SCROLL_OK;
    for (int k = 0; k < n; ++k) {
        if (status) status[k] = outs[k].err;
        if (outs[k].err != ING_OK && rc == SCROLL_OK) {
            set_err("scroll_batch_update_refs: stream %d: %s", streams[k],
                    outs[k].err == ING_ERR_DIMS ? "picture size differs from the stream's" : ing_msg(outs[k].err));
            rc = outs[k].err == ING_ERR_OVERFLOW ? SCROLL_ERR_OVERFLOW : SCROLL_ERR_CONFIG;
        }
    }
    return rc;
}

int scroll_batch_update_refs(ScrollBatch *b, int n, const int *streams, const int *which,
                             const uint8_t *const *files, const size_t *sizes, int *status)
{
    if (!b || n < 0 || (n > 0 && (!files || !sizes))) return SCROLL_ERR_ARG;
    std::vector<uint64_t> desc(2 * (size_t)n);
    size_t tot = 0;
    for (int k = 0; k < n; ++k) {
        if (sizes[k] && !files[k]) return SCROLL_ERR_ARG;
        desc[2 * k] = tot;
        desc[2 * k + 1] = sizes[k];
        tot += (sizes[k] + 255) & ~(size_t)255;
    }
    if (n == 0) return SCROLL_OK;
    int rc = batch_host_sync(b);                  /* the input buffer may be in use */
    if (rc) return rc;
    HIPCHK(hipSetDevice(b->device));
    if (tot > b->ing_in_cap) {
        (void)hipFree(b->d_ing_in);
        b->d_ing_in = nullptr;
        b->ing_in_cap = 0;
        hipError_t e = hipMalloc(&b->d_ing_in, tot);
        if (e != hipSuccess) {
            set_err("scroll_batch_update_refs: %s", hipGetErrorString(e));
            return e == hipErrorOutOfMemory ? SCROLL_ERR_OOM : SCROLL_ERR_HIP;
        }
        b->ing_in_cap = tot;
    }
    for (int k = 0; k < n; ++k)
        if (sizes[k]) HIPCHK(hipMemcpy(b->d_ing_in + desc[2 * k], files[k], sizes[k], hipMemcpyHostToDevice));
    return scroll_batch_update_refs_device(b, n, streams, which, b->d_ing_in, desc.data(), status);
}

int scroll_batch_enable_timing(ScrollBatch *b, int on)
{
    if (!b) return SCROLL_ERR_ARG;
    b->timing = on;
    return SCROLL_OK;
}

float scroll_batch_kernel_ms(ScrollBatch *b, int which)
{
    if (!b || which < 0 || which > 5) return -1.0f;
    if (b->timing == 2) return -1.0f;           /* lite: no per-kernel pairs (kernel_stats_ex has the dominant one) */
    if (batch_host_sync(b)) return -1.0f;
    if (b->timed_pending) {
        event_ms(b->ev, b->ev_dyn != 0, false, b->ms);
        b->timed_pending = 0;
    }
    return b->ms[which];
}

/* ======================================================================== */
/* synchronous helpers for the drop-in entry points (engine.h)              */
/* ======================================================================== */
static std::mutex g_mu;

struct TempBatch {
    ScrollBatch *b = nullptr;
    int streams = 0, frames = 0;
    size_t arena = 0;
    int mode = -1;
};
static TempBatch g_tmp;

static int temp_batch(int streams, int frames, size_t arena, int mode, ScrollBatch **out)
{
    TempBatch &t = g_tmp;
    if (!t.b || t.streams < streams || t.frames < frames || t.arena < arena || t.mode != mode) {
        if (t.b) scroll_batch_destroy(t.b);
        t.b = nullptr;
        ScrollBatchDesc d;
        d.device = 0;
        std::vector<int> ids;
        if (!usable_devices(&ids)) return SCROLL_ERR_NO_DEVICE;
        d.device = ids[0];
        d.max_streams = streams > t.streams ? streams : t.streams;
        d.max_frames = frames > t.frames ? frames : t.frames;
        d.arena_bytes = arena > t.arena ? arena : t.arena;
        d.mode = mode;
        int rc = scroll_batch_create(&t.b, &d);
        if (rc) return rc;
        t.streams = d.max_streams;
        t.frames = d.max_frames;
        t.arena = d.arena_bytes;
        t.mode = mode;
    }
    t.b->nstreams = 0;
    t.b->host_valid = 1;
    *out = t.b;
    return SCROLL_OK;
}

static size_t round_arena(size_t n)
{
    size_t a = 1u << 20;
    while (a < n) a <<= 1;
    return a;
}

int scroll_engine_write_nals(const ComposerConfig *cfg, const NalDesc *nals, int n,
                             uint8_t *dst, size_t cap, size_t *written)
{
    std::lock_guard<std::mutex> lk(g_mu);
    *written = 0;
    int rc = check_cfg(cfg);
    if (rc) return rc;
    ScrollBatch *b;
    rc = temp_batch(1, n, round_arena(cap), SCROLL_MODE_COMPOSER, &b);
    if (rc) return rc;
    DevStream *d = &b->h_st[0];
    if (b->dyn_qp != 26 && !cfg->deblocking_filter_control_present_flag) {
        set_err("scroll_batch_add_stream: a stream with the deblocking filter on (no "
                "deblocking_filter_control_present_flag) needs the rect at QP 26, the batch's is %d",
                b->dyn_qp);
        return SCROLL_ERR_CONFIG;
    }
    memset(d, 0, sizeof(*d));
    cfg_to_dev(cfg, d);
    d->dyn_qp = b->dyn_qp;
    d->out_pos = 0;
    d->out_cap = cap;
    d->nnal = n;
    b->nstreams = 1;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpyAsync(b->d_st, d, sizeof(DevStream), hipMemcpyHostToDevice, b->own));
    HIPCHK(hipMemcpyAsync(b->d_nal, nals, (size_t)n * sizeof(NalDesc), hipMemcpyHostToDevice,
                          b->own));
    rc = launch(b, 0, SCROLL_PLAN_EXPLICIT, n, b->own);
    if (rc) return rc;
    rc = scroll_batch_sync(b);
    if (rc) return rc;
    size_t tot = (size_t)b->h_st[0].out_pos;
    HIPCHK(hipMemcpy(dst, b->d_arena, tot, hipMemcpyDeviceToHost));
    *written = tot;
    return SCROLL_OK;
}

int scroll_engine_compose(ComposerConfig *const *cfgs, const int *const *offs, const int *frames,
                          int nstreams, int mode, uint8_t *const *dsts, const size_t *caps,
                          size_t *written, int **wp_offsets_out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    int fmax = 0;
    size_t cmax = 0;
    for (int i = 0; i < nstreams; ++i) {
        written[i] = 0;
        int rc = check_cfg(cfgs[i]);
        if (rc) return rc;
        if (frames[i] > fmax) fmax = frames[i];
        if (caps[i] > cmax) cmax = caps[i];
    }
    if (nstreams == 0 || fmax == 0) return SCROLL_OK;
    ScrollBatch *b;
    int rc = temp_batch(nstreams, fmax, round_arena(cmax), mode, &b);
    if (rc) return rc;
    std::vector<int32_t> off((size_t)nstreams * fmax, 0);
    for (int i = 0; i < nstreams; ++i) {
        DevStream *d = &b->h_st[i];
        memset(d, 0, sizeof(*d));
        cfg_to_dev(cfgs[i], d);
        d->out_pos = 0;
        d->out_cap = caps[i];
        d->frames = frames[i];
        memcpy(&off[(size_t)i * fmax], offs[i], (size_t)frames[i] * sizeof(int32_t));
    }
    b->nstreams = nstreams;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipMemcpyAsync(b->d_st, b->h_st, (size_t)nstreams * sizeof(DevStream),
                          hipMemcpyHostToDevice, b->own));
    HIPCHK(hipMemcpy2DAsync(b->d_off, (size_t)b->max_frames * sizeof(int32_t), off.data(),
                            (size_t)fmax * sizeof(int32_t), (size_t)fmax * sizeof(int32_t),
                            (size_t)nstreams, hipMemcpyHostToDevice, b->own));
    int plan = mode == SCROLL_MODE_EXPERIMENT ? SCROLL_PLAN_EXPERIMENT : SCROLL_PLAN_COMPOSER;
    rc = launch(b, -1, plan, plan == SCROLL_PLAN_COMPOSER ? 2 * fmax : fmax, b->own);
    if (rc) return rc;
    rc = scroll_batch_sync(b);
    if (rc) return rc;
    if (wp_offsets_out) {
        rc = load_nals(b);
        if (rc) return rc;
    }
    for (int i = 0; i < nstreams; ++i) {
        size_t tot = (size_t)b->h_st[i].out_pos;
        if (tot) {
            HIPCHK(hipMemcpy(dsts[i], b->d_arena + (size_t)i * b->ld_arena, tot,
                             hipMemcpyDeviceToHost));
        }
        written[i] = tot;
        dev_to_cfg(&b->h_st[i], cfgs[i]);
        if (wp_offsets_out && wp_offsets_out[i]) {
            int k = 0;
            for (int j = 0; j < b->h_st[i].nnal; ++j) {
                const NalDesc &nd = b->nal_cache[(size_t)i * b->ld_nal + j];
                if (nd.kind == 1) wp_offsets_out[i][k++] = nd.off;
            }
            wp_offsets_out[i][k] = -1;
        }
    }
    return SCROLL_OK;
}

}  // extern "C"
