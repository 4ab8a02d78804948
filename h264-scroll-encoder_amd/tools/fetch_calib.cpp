/*
 * fetch_calib.cpp -- calibration of the rocprofv3 HBM counters (FETCH_SIZE,
 * WRITE_SIZE) for the access widths this repo's kernels use.
 *
 * MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of a
 * wide (16 B per lane) coalesced streaming read on gfx950, WRITE_SIZE is
 * exact for 16-B-per-lane stores, and "other access widths are
 * uncalibrated: calibrate on a known byte count in your own access pattern".
 * k_dyn_row reads its pixels with 4-byte buffer loads, k_ipcm and the ingest
 * read bytes and 8-byte words, the row stage is written in 4-byte words.
 *
 * Each kernel below touches exactly BYTES bytes of a buffer far larger than
 * the Infinity Cache (every line once, whole waves over contiguous bytes),
 * at one access width; run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc
 * WRITE_SIZE` (separate passes), and tools/calib_summary.py divides the
 * counter by the known bytes: the correction factor per width.
 *
 * Build: hipcc --offload-arch=gfx950 -O3 fetch_calib.cpp -o fetch_calib
 */
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr size_t BYTES = (size_t)1 << 30;   /* 1 GiB per kernel: 4x the Infinity Cache */
constexpr int TPB = 256;

/* reads: every lane W bytes per step, grid-stride over the buffer; the sum
 * goes to one word per block (so the loads are not dead) */
template <typename V>
__global__ __launch_bounds__(TPB) void k_read(const V *__restrict__ p, size_t n, uint32_t *__restrict__ out)
{
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) {
        const V v = p[i];
        const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
        if constexpr (sizeof(V) >= 4) {
#pragma unroll
            for (size_t k = 0; k < sizeof(V) / 4; ++k) acc += w[k];
        } else {
            acc += (uint32_t)v;
        }
    }
    if (acc == 0x9e3779b1u) out[blockIdx.x] = acc;     /* never (the buffer is zero): keeps the loads */
}

/* writes: every lane W bytes per step */
template <typename V>
__global__ __launch_bounds__(TPB) void k_write(V *__restrict__ p, size_t n, V v)
{
    for (size_t i = (size_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (size_t)gridDim.x * TPB) p[i] = v;
}

struct u64x2 {
    uint64_t a, b;
};

int main()
{
    uint8_t *buf = nullptr;
    uint32_t *out = nullptr;
    CHK(hipMalloc(&buf, BYTES));
    CHK(hipMalloc(&out, 1 << 20));
    CHK(hipMemset(buf, 0, BYTES));
    CHK(hipDeviceSynchronize());
    const int grid = 256 * 8 * 4;                /* 8 workgroups per CU, 4 rounds of grid stride */
    /* the dispatch order is the order of the lines calib_summary.py reads */
    hipLaunchKernelGGL(k_read<uint8_t>, dim3(grid), dim3(TPB), 0, 0, buf, BYTES, out);
    hipLaunchKernelGGL(k_read<uint32_t>, dim3(grid), dim3(TPB), 0, 0, (const uint32_t *)buf, BYTES / 4, out);
    hipLaunchKernelGGL(k_read<uint2>, dim3(grid), dim3(TPB), 0, 0, (const uint2 *)buf, BYTES / 8, out);
    hipLaunchKernelGGL(k_read<uint4>, dim3(grid), dim3(TPB), 0, 0, (const uint4 *)buf, BYTES / 16, out);
    hipLaunchKernelGGL(k_write<uint8_t>, dim3(grid), dim3(TPB), 0, 0, buf, BYTES, (uint8_t)0);
    hipLaunchKernelGGL(k_write<uint32_t>, dim3(grid), dim3(TPB), 0, 0, (uint32_t *)buf, BYTES / 4, 0u);
    hipLaunchKernelGGL(k_write<uint2>, dim3(grid), dim3(TPB), 0, 0, (uint2 *)buf, BYTES / 8, make_uint2(0, 0));
    hipLaunchKernelGGL(k_write<uint4>, dim3(grid), dim3(TPB), 0, 0, (uint4 *)buf, BYTES / 16, make_uint4(0, 0, 0, 0));
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    printf("{\"bytes_per_kernel\": %zu}\n", BYTES);
    CHK(hipFree(buf));
    CHK(hipFree(out));
    return 0;
}
