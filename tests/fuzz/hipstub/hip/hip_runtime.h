// Host stand-in for <hip/hip_runtime.h> so redisson_amd/csrc/sk_device.h compiles as plain C++ for the CPU checks
// of its hash arithmetic (dev_hash_host.cpp).  Only what sk_device.h uses: the qualifiers and three builtins.
#pragma once
#include <stdint.h>
#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
// v_alignbyte_b32: (hi:lo >> 8 * (sel & 3)) low 32 bits
struct uint4 {
    uint32_t x, y, z, w;
};
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
struct Dim3 {
    uint32_t x = 0, y = 0, z = 0;
};
static const Dim3 threadIdx, blockDim;   // stage_keys is not called on the host
static inline void __syncthreads() {}
static inline uint32_t __builtin_amdgcn_alignbyte(uint32_t hi, uint32_t lo, uint32_t sel) {
    return uint32_t(((uint64_t(hi) << 32) | lo) >> (8 * (sel & 3)));
}
static inline uint32_t __builtin_amdgcn_readfirstlane(uint32_t x) { return x; } // one lane on the host
static inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return uint64_t((unsigned __int128)a * b >> 64); }
