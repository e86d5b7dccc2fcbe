// micro_lines.hip -- which random-access forms move more lines per second on
// gfx950 (follow-up to micro_random.hip): cache-scope variants of random
// loads, and byte vs whole-line random stores / read-modify-writes.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
template <int SCOPE> // 0 plain, 1 agent-scope relaxed atomic load, 2 system-scope
__global__ void k_load(const uint32_t *t, uint64_t words, uint64_t n, int per, uint32_t *out, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t acc = 0;
    for (int j = 0; j < per; j++) {
        const uint32_t *p = t + mix(seed + i * per + j) % words;
        if (SCOPE == 0) acc += *p;
        else if (SCOPE == 1) acc += __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else acc += __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (acc == 0xffffffff) out[0] = acc;
}
__global__ void k_store_byte(uint8_t *t, uint64_t bytes, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) t[mix(seed + i) % bytes] = uint8_t(i);
}
// 8 lanes write one random 128-B line whole (16 B each)
__global__ void k_store_line(uint4 *t, uint64_t lines, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t l = i >> 3;
    if (l >= n) return;
    uint64_t line = mix(seed + l) % lines;
    t[line * 8 + (i & 7)] = make_uint4(uint32_t(i), 1, 2, 3);
}
__global__ void k_rmw_byte(uint8_t *t, uint64_t bytes, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t a = mix(seed + i) % bytes;
    t[a] = uint8_t(t[a] + 1);
}
// 8 lanes read a random line, then write it back whole
__global__ void k_rmw_line(uint4 *t, uint64_t lines, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t l = i >> 3;
    if (l >= n) return;
    uint4 *p = t + (mix(seed + l) % lines) * 8 + (i & 7);
    uint4 v = *p;
    v.x += 1;
    *p = v;
}

int main() {
    const uint64_t big = 1600ull << 20, bloom = 534ull << 20;
    uint8_t *t;
    uint32_t *o;
    hipMalloc(&t, big);
    hipMemset(t, 1, big);
    hipMalloc(&o, 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char *name, auto fn, double units, const char *unit) {
        fn();
        hipDeviceSynchronize();
        float best = 1e9;
        for (int r = 0; r < 5; r++) {
            hipEventRecord(a);
            fn();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        printf("%-52s %9.1f us  %8.2f G%s/s\n", name, best * 1e3, units / (best * 1e-3) / 1e9, unit);
    };
    const uint64_t n = 1ull << 22;
    unsigned g = unsigned((n + 255) / 256);
    timeit("load u32 x6 rand 534MB plain", [&] { k_load<0><<<g, 256>>>((uint32_t *)t, bloom / 4, n, 6, o, 1); },
           6.0 * n, "load");
    timeit("load u32 x6 rand 534MB agent-scope atomic (sc1)",
           [&] { k_load<1><<<g, 256>>>((uint32_t *)t, bloom / 4, n, 6, o, 1); }, 6.0 * n, "load");
    timeit("load u32 x6 rand 534MB system-scope atomic (sc0 sc1)",
           [&] { k_load<2><<<g, 256>>>((uint32_t *)t, bloom / 4, n, 6, o, 1); }, 6.0 * n, "load");
    timeit("store byte rand 1.6GB", [&] { k_store_byte<<<g, 256>>>(t, big, n, 2); }, n, "store");
    timeit("store whole 128-B line rand 1.6GB (8 lanes)",
           [&] { k_store_line<<<unsigned(n * 8 / 256), 256>>>((uint4 *)t, big / 128, n, 3); }, n, "line");
    timeit("rmw byte rand 1.6GB", [&] { k_rmw_byte<<<g, 256>>>(t, big, n, 4); }, n, "rmw");
    timeit("rmw whole 128-B line rand 1.6GB (8 lanes)",
           [&] { k_rmw_line<<<unsigned(n * 8 / 256), 256>>>((uint4 *)t, big / 128, n, 5); }, n, "line");
    return 0;
}
