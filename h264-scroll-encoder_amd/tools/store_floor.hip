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
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int LDS_BYTES>
__global__ __launch_bounds__(64) void k_store(uint8_t *arena, uint64_t ld_arena, uint64_t tile_bytes,
                                              int tiles, int unroll, int spin, int per_lane,
                                              int skew, int hole, int holew, int before)
{
    __shared__ uint32_t pad[LDS_BYTES / 4 > 0 ? LDS_BYTES / 4 : 1];
    const int lane = threadIdx.x;
    if (LDS_BYTES > 4) pad[lane] = lane;
    const int t = blockIdx.x;
    if (t >= tiles) return;
    uint8_t *A = arena + (uint64_t)blockIdx.y * ld_arena;
    const uint64_t B0 = (uint64_t)t * tile_bytes + 16u * skew, B1 = B0 + tile_bytes - 16u * skew;
    const uint64_t c0 = (B0 + 15) >> 4, c1 = B1 >> 4;
    uint32_t x = lane * 2654435761u + t;
    /* hole > 0: every hole-th block of holew chunks is skipped by the
     * streaming pass and written by a scattered pass (one lane per skipped
     * chunk) after it, or before it when `before` */
    if (hole > 0 && before) {
        const uint64_t h0 = (c0 / holew + hole - 1) / hole;
        for (uint64_t h = h0 * holew + lane; (h / holew) * hole * holew < c1; h += 64) {
            const uint64_t cc = (h / holew) * hole * holew + h % holew;
            if (cc < c0 || cc >= c1) continue;
            uint4 o = make_uint4(x, x ^ 5, x ^ 6, x ^ 7);
            *reinterpret_cast<uint4 *>(A + (cc << 4)) = o;
        }
    }
    for (uint64_t c = c0; c < c1; c += 64u * unroll) {
        for (int u = 0; u < unroll; ++u) {
            /* per_lane consecutive chunks per lane: lane stride 16 * per_lane bytes */
            const uint64_t cc = per_lane == 1 ? c + 64u * u + lane
                                              : c + (uint64_t)(u / per_lane) * 64u * per_lane +
                                                    (uint64_t)lane * per_lane + (u % per_lane);
            if (cc < c1 && !(hole > 0 && (cc / holew) % hole == 0)) {
                uint4 o = make_uint4(x, x ^ 1, x ^ 2, x ^ 3);
                *reinterpret_cast<uint4 *>(A + (cc << 4)) = o;
            }
        }
        for (int k = 0; k < spin; ++k) x = x * 1664525u + 1013904223u;
    }
    if (hole > 0 && !before) {
        const uint64_t h0 = (c0 / holew + hole - 1) / hole;
        for (uint64_t h = h0 * holew + lane; (h / holew) * hole * holew < c1; h += 64) {
            const uint64_t cc = (h / holew) * hole * holew + h % holew;
            if (cc < c0 || cc >= c1) continue;
            uint4 o = make_uint4(x, x ^ 5, x ^ 6, x ^ 7);
            *reinterpret_cast<uint4 *>(A + (cc << 4)) = o;
        }
    }
    if (LDS_BYTES > 4 && x == 0xdeadbeef) arena[0] = (uint8_t)pad[(lane + 1) & 63];
}

int main(int argc, char **argv)
{
    const int only = argc > 1 ? atoi(argv[1]) : -1;   /* run one variant (profiling) */
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
    struct V { const char *name; int lds; int unroll; int spin; int per_lane; int skew; int hole;
               int holew; int before; };
    V vs[] = {{"u4", 1, 4, 0, 1, 0, 0, 1, 0},
              {"hole 1/31 16B after", 1, 4, 0, 1, 0, 31, 1, 0},
              {"hole 1/31 16B before", 1, 4, 0, 1, 0, 31, 1, 1},
              {"hole 1/31 32B after", 1, 4, 0, 1, 0, 31, 2, 0},
              {"hole 1/31 64B after", 1, 4, 0, 1, 0, 31, 4, 0},
              {"hole 1/31 128B after", 1, 4, 0, 1, 0, 31, 8, 0},
              {"hole 1/31 256B after", 1, 4, 0, 1, 0, 31, 16, 0},
              {"hole 1/500 16B after", 1, 4, 0, 1, 0, 500, 1, 0},
              {"hole 1/31 16B unroll1", 1, 1, 0, 1, 0, 31, 1, 0}};
    int vi = -1;
    for (int rep = 0; rep < 2; ++rep)
        for (auto &v : vs) {
            vi = (vi + 1) % (int)(sizeof(vs) / sizeof(vs[0]));
            if (only >= 0 && vi != only) continue;
            float best = 1e9f;
            for (int it = 0; it < 5; ++it) {
                CK(hipEventRecord(e0));
                if (v.lds)
                    hipLaunchKernelGGL(k_store<11904>, dim3(tiles, streams), dim3(64), 0, 0, d, ld,
                                       tile_bytes, tiles, v.unroll, v.spin, v.per_lane, v.skew, v.hole, v.holew, v.before);
                else
                    hipLaunchKernelGGL(k_store<0>, dim3(tiles, streams), dim3(64), 0, 0, d, ld,
                                       tile_bytes, tiles, v.unroll, v.spin, v.per_lane, v.skew,
                                       v.hole, v.holew, v.before);
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
