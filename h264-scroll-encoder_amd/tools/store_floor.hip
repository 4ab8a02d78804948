// store_floor.hip -- profiling aid: the store-only floor of k_emit's output
// pattern.  Each 1-wave workgroup streams one tile (TILE NAL units of about
// `nal_bytes` each) of one stream's arena with 16-B-per-lane dwordx4 stores,
// exactly the tile geometry of k_emit on the bench workload; optional LDS
// reservation reproduces k_emit's occupancy, optional spin emulates compute
// between stores.  Prints ms and GB/s per variant.
//
//   hipcc -O3 --offload-arch=gfx950 -o store_floor store_floor.hip && ./store_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int LDS_BYTES>
__global__ __launch_bounds__(64) void k_store(uint8_t *arena, uint64_t ld_arena, uint64_t tile_bytes,
                                              int tiles, int unroll, int spin)
{
    __shared__ uint32_t pad[LDS_BYTES / 4 > 0 ? LDS_BYTES / 4 : 1];
    const int lane = threadIdx.x;
    if (LDS_BYTES > 4) pad[lane] = lane;
    const int t = blockIdx.x;
    if (t >= tiles) return;
    uint8_t *A = arena + (uint64_t)blockIdx.y * ld_arena;
    const uint64_t B0 = (uint64_t)t * tile_bytes, B1 = B0 + tile_bytes;
    const uint64_t c0 = (B0 + 15) >> 4, c1 = B1 >> 4;
    uint32_t x = lane * 2654435761u + t;
    for (uint64_t c = c0; c < c1; c += 64u * unroll) {
        for (int u = 0; u < unroll; ++u) {
            const uint64_t cc = c + 64u * u + lane;
            if (cc < c1) {
                uint4 o = make_uint4(x, x ^ 1, x ^ 2, x ^ 3);
                *reinterpret_cast<uint4 *>(A + (cc << 4)) = o;
            }
        }
        for (int k = 0; k < spin; ++k) x = x * 1664525u + 1013904223u;
    }
    if (LDS_BYTES > 4 && x == 0xdeadbeef) arena[0] = (uint8_t)pad[(lane + 1) & 63];
}

int main()
{
    const int streams = 256, nal = 1056, tile = 32;
    const uint64_t nal_bytes = 2833, tile_bytes = tile * nal_bytes;
    const int tiles = (nal + tile - 1) / tile;
    const uint64_t ld = 1024ull * 2 * (64 + 80 * 45) + (1 << 16);
    uint8_t *d;
    CK(hipMalloc(&d, ld * streams));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)tiles * streams * tile_bytes;
    struct V { const char *name; int lds; int unroll; int spin; };
    V vs[] = {{"lds0 u1", 0, 1, 0}, {"lds0 u4", 0, 4, 0}, {"lds12k u1", 1, 1, 0},
              {"lds12k u4", 1, 4, 0}, {"lds12k u4 spin64", 1, 4, 64},
              {"lds12k u4 spin256", 1, 4, 256}};
    for (int rep = 0; rep < 2; ++rep)
        for (auto &v : vs) {
            float best = 1e9f;
            for (int it = 0; it < 5; ++it) {
                CK(hipEventRecord(e0));
                if (v.lds)
                    hipLaunchKernelGGL(k_store<11904>, dim3(tiles, streams), dim3(64), 0, 0, d, ld,
                                       tile_bytes, tiles, v.unroll, v.spin);
                else
                    hipLaunchKernelGGL(k_store<0>, dim3(tiles, streams), dim3(64), 0, 0, d, ld,
                                       tile_bytes, tiles, v.unroll, v.spin);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("%-20s %.4f ms  %.1f GB/s\n", v.name, best, bytes / best / 1e6);
        }
    CK(hipFree(d));
    return 0;
}
