/*
 * TEST-ONLY shim: lets g++ compile the product's device header
 * (h264-scroll-encoder_amd/csrc/scroll_device.h) on the CPU so its run-layout
 * and bit-extraction logic can be unit-tested without a GPU.  Never linked
 * into libh264scroll.so; the GPU tests (tests/test_gpu_*.py) are the parity
 * evidence for the real kernels.
 */
#pragma once
#include <algorithm>
#include <cstdint>
#define __device__
#define __host__
using std::max;
using std::min;
static inline int __clzll(uint64_t x) { return x ? __builtin_clzll(x) : 64; }
static inline int __clz(int x) { return x ? __builtin_clz((unsigned)x) : 32; }
static inline float __builtin_amdgcn_rcpf(float x) { return 1.0f / x; }
static inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
static inline uint32_t __umul24(uint32_t a, uint32_t b) { return (a & 0xffffffu) * (b & 0xffffffu); }
struct uint4 {
    uint32_t x, y, z, w;
};
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
static inline int __mul24(int a, int b) { return ((int)((uint32_t)a << 8) >> 8) * ((int)((uint32_t)b << 8) >> 8); }
static inline int __builtin_amdgcn_readfirstlane(int x) { return x; }
static inline uint32_t __builtin_amdgcn_alignbit(uint32_t a, uint32_t b, uint32_t s)
{ return (uint32_t)((((uint64_t)a << 32) | b) >> (s & 31)); }
