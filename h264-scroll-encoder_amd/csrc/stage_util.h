/*
 * stage_util.h -- device helpers shared by the kernels that stage a whole
 * NAL's RBSP in a slot (k_dyn_group / k_dyn_ep, k_hint_stage) and by k_dyn_emit_gather:
 * workgroup scans, the LDS OR bit sink, the emulation-prevention recorder
 * and the XCD-mixing frame rotation.  Workgroups are NW waves of 64.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dyn_device.h"
#include "engine.h"

namespace scroll {
namespace stage {

using dyn::ep_insert;
using dyn::OrSink;

constexpr int DT = 256;                         /* threads per staging workgroup */
constexpr int NW = DT / 64;
constexpr int EPLIST_MAX = DYN_OVF_BYTES / 4;   /* EP positions kept per NAL (slot tail) */
/* NALs with more EP bytes than this go to emit_serial (SCROLL_DEBUG_DYN_EPCAP4
 * lowers it so the tests reach that path) */
__device__ inline uint32_t ep_cap(const DynGeom &g, bool rs)
{
    return (g.debug & SCROLL_DEBUG_DYN_EPCAP4) ? 4u : (rs ? g.ep_cap : (uint32_t)EPLIST_MAX);
}
/* bytes of a frame's EP list in the dynamic rect's list buffer (the rows'
 * path: k_dyn_epfix writes it, k_dyn_gather reads it) */
__host__ __device__ inline size_t eps_stride(const DynGeom &g) { return (size_t)4 * g.ep_cap; }

__device__ inline int wave_incl_max(int v, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(v, d, 64);
        if (lane >= d) v = max(v, u);
    }
    return v;
}

__device__ inline uint32_t wave_incl_sum(uint32_t v, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    return v;
}

/* workgroup barrier for LDS hand-offs only: waits for this wave's LDS
 * operations, not for its global loads and stores (__syncthreads' release
 * fence waits for every outstanding vector-memory operation, which would
 * also drain prefetched loads and fire-and-forget stores).  The "memory"
 * clobber keeps the compiler from moving memory accesses across it. */
__device__ inline void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

/* exclusive prefix max over the workgroup (identity -1) and the total;
 * ends with a barrier so `ws` can be reused.  LDS: the barriers are
 * lds_barrier (global operations stay in flight) */
template <int NWV = NW, bool LDS = false>
__device__ inline void block_excl_max(int v, int *ws, int &excl, int &tot)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_max(v, lane);
    if (lane == 63) ws[wave] = incl;
    int e = __shfl_up(incl, 1, 64);
    if (lane == 0) e = -1;
    if (LDS) lds_barrier();
    else __syncthreads();
    int pm = -1, t = -1;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
        if (w < wave) pm = max(pm, ws[w]);
        t = max(t, ws[w]);
    }
    excl = max(pm, e);
    tot = t;
    if (LDS) lds_barrier();
    else __syncthreads();
}

template <int NWV = NW>
__device__ inline void block_excl_sum(uint32_t v, uint32_t *ws, uint32_t &excl, uint32_t &tot)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_sum(v, lane);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    uint32_t pm = 0, t = 0;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
        if (w < wave) pm += ws[w];
        t += ws[w];
    }
    excl = pm + incl - v;
    tot = t;
    __syncthreads();
}

struct LdsOr {
    uint32_t *b;
    __device__ inline void operator()(uint32_t i, uint32_t v) const { atomicOr(&b[i], v); }
};
typedef OrSink<LdsOr> LSink;

__device__ inline int last_nz_byte(uint32_t w)      /* MSB-first byte index, w != 0 */
{
    return 3 - (__builtin_ctz(w) >> 3);
}

/* number of EP insertions among the 4 bytes of MSB-first word w whose
 * global indices start at g (only bytes < lim count); prev = index of the
 * last non-zero byte before them, updated */
__device__ inline uint32_t ep_word(uint32_t w, uint32_t g, uint32_t lim, int &prev,
                                   uint32_t *list = nullptr, uint32_t *cnt = nullptr)
{
    uint32_t n = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t gi = g + (uint32_t)i;
        if (gi >= lim) break;
        const uint32_t b = (w >> (24 - 8 * i)) & 255u;
        if (ep_insert(b, (int)gi - 1 - prev)) {
            n++;
            if (list) {                              /* RBSP index the 03 precedes */
                const uint32_t k = atomicAdd(cnt, 1u);
                if (k < (uint32_t)EPLIST_MAX) list[k] = gi;
            }
        }
        if (b) prev = (int)gi;
    }
    return n;
}

/* Workgroup (x, s) -> frame: rotated by the stream so that consecutive
 * workgroups -- which the dispatcher deals round-robin to the 8 XCDs --
 * mix frame indices; the residual cost of a frame depends on t, and without
 * the rotation frame f of every stream lands on XCD f % 8 (frames >= 8). */
__device__ inline int dyn_frame_of(int x, int s)
{
    const int F = (int)gridDim.x;
    int r = x + (s & 7);                     /* uniform: no integer division */
    while (r >= F) r -= F;
    return __builtin_amdgcn_readfirstlane(r);
}

/* SWAR byte tests in "high bit" form: bit 8k + 7 set iff byte k passes */
__device__ inline uint32_t zero_hi(uint32_t x)
{
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

/* the 16 bytes w (little-endian) to buf[at, at + 16), any alignment: the
 * three whole dwords inside as dword writes, the bytes of the two end dwords
 * (shared with the neighbouring lanes) one by one */
__device__ inline void lds_put16(uint8_t *buf, uint32_t at, const uint32_t (&w)[4])
{
    const uint32_t m = at & 3u;
    uint32_t *dw = reinterpret_cast<uint32_t *>(buf + (at - m));
    if (m == 0) {
        dw[0] = w[0];
        dw[1] = w[1];
        dw[2] = w[2];
        dw[3] = w[3];
        return;
    }
    uint8_t *b = buf + (at - m);
    for (uint32_t k = m; k < 4; ++k) b[k] = (uint8_t)(w[0] >> (8 * (k - m)));
    dw[1] = __builtin_amdgcn_alignbyte(w[1], w[0], 4u - m);
    dw[2] = __builtin_amdgcn_alignbyte(w[2], w[1], 4u - m);
    dw[3] = __builtin_amdgcn_alignbyte(w[3], w[2], 4u - m);
    for (uint32_t k = 0; k < m; ++k) b[16 + k] = (uint8_t)(w[3] >> (8 * (4 - m + k)));
}

}  // namespace stage
}  // namespace scroll
