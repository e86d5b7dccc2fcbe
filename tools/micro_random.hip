// micro_random.hip -- primitive costs behind the sketch kernels on gfx950:
// random byte loads / byte stores / u32 atomics over a large table.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void k_load(const uint8_t *t, uint64_t bytes, uint64_t n, int per, uint32_t *out, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t acc = 0;
    for (int j = 0; j < per; j++) acc += t[mix(seed + i * per + j) % bytes];
    if (acc == 0xffffffff) out[0] = acc;
}
__global__ void k_load_dep(const uint8_t *t, uint64_t bytes, uint64_t n, int per, uint32_t *out, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t acc = 0;
    for (int j = 0; j < per; j++) acc += t[(mix(seed + i * per + j) + acc) % bytes];
    if (acc == 0xffffffff) out[0] = acc;
}
__global__ void k_store(uint8_t *t, uint64_t bytes, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    t[mix(seed + i) % bytes] = uint8_t(i);
}
__global__ void k_rmw(uint8_t *t, uint64_t bytes, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t a = mix(seed + i) % bytes;
    uint8_t v = t[a];
    if (v < (i & 63)) t[a] = uint8_t(i & 63);
}
__global__ void k_atomic_or(uint32_t *t, uint64_t words, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    atomicOr(&t[mix(seed + i) % words], 1u << (i & 31));
}
__global__ void k_atomic_or_ret(uint32_t *t, uint64_t words, uint64_t n, uint32_t *out, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t o = atomicOr(&t[mix(seed + i) % words], 1u << (i & 31));
    if (o == 0xdeadbeef) out[0] = o;
}
__global__ void k_load_nt(const uint8_t *t, uint64_t bytes, uint64_t n, int per, uint32_t *out, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t acc = 0;
    for (int j = 0; j < per; j++) acc += __builtin_nontemporal_load(t + mix(seed + i * per + j) % bytes);
    if (acc == 0xffffffff) out[0] = acc;
}
__global__ void k_load16(const uint4 *t, uint64_t n16, uint64_t n, int per, uint32_t *out, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t acc = 0;
    for (int j = 0; j < per; j++) { uint4 v = t[mix(seed + i * per + j) % n16]; acc += v.x ^ v.w; }
    if (acc == 0xffffffff) out[0] = acc;
}
// each lane's 6 probes land in one 4 KiB page (what a page-blocked layout would give)
__global__ void k_load_page(const uint8_t *t, uint64_t bytes, uint64_t n, int per, uint32_t *out, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t base = (mix(seed + i) % (bytes >> 12)) << 12;
    uint32_t acc = 0;
    for (int j = 0; j < per; j++) acc += t[base + (mix(seed + i * per + j) & 4095)];
    if (acc == 0xffffffff) out[0] = acc;
}
__global__ void k_stream(const uint4 *a, uint64_t n, uint4 *b) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
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
        printf("%-48s %9.1f us  %8.2f G%s/s\n", name, best * 1e3, units / (best * 1e-3) / 1e9, unit);
    };
    for (uint64_t n : {1ull << 20, 1ull << 22}) {
        unsigned g = unsigned((n + 255) / 256);
        char nm[128];
        snprintf(nm, sizeof nm, "load 1B x1 rand 1.6GB n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_load<<<g, 256>>>(t, big, n, 1, o, 1); }, n, "load");
        snprintf(nm, sizeof nm, "load 1B x6 rand 534MB (indep) n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_load<<<g, 256>>>(t, bloom, n, 6, o, 2); }, 6.0 * n, "load");
        snprintf(nm, sizeof nm, "load 1B x6 rand 534MB (dependent) n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_load_dep<<<g, 256>>>(t, bloom, n, 6, o, 3); }, 6.0 * n, "load");
        snprintf(nm, sizeof nm, "load 1B x6 rand 128MB (indep) n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_load<<<g, 256>>>(t, 128ull << 20, n, 6, o, 2); }, 6.0 * n, "load");
        snprintf(nm, sizeof nm, "store 1B rand 1.6GB n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_store<<<g, 256>>>(t, big, n, 4); }, n, "store");
        snprintf(nm, sizeof nm, "load+cond store 1B rand 1.6GB n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_rmw<<<g, 256>>>(t, big, n, 5); }, n, "rmw");
        snprintf(nm, sizeof nm, "atomicOr u32 noret rand 1.6GB n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_atomic_or<<<g, 256>>>((uint32_t *)t, big / 4, n, 6); }, n, "atom");
        snprintf(nm, sizeof nm, "atomicOr u32 ret rand 1.6GB n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_atomic_or_ret<<<g, 256>>>((uint32_t *)t, big / 4, n, o, 7); }, n, "atom");
        snprintf(nm, sizeof nm, "atomicOr u32 ret rand 32MB n=%llu", (unsigned long long)n);
        timeit(nm, [&] { k_atomic_or_ret<<<g, 256>>>((uint32_t *)t, (32ull << 20) / 4, n, o, 8); }, n, "atom");
    }
    {
        uint64_t n = 1ull << 22;
        unsigned g = unsigned((n + 255) / 256);
        for (uint64_t tb : {2ull << 20, 16ull << 20, 64ull << 20}) {
            char nm[128];
            snprintf(nm, sizeof nm, "load 1B x6 rand %lluMB (indep) n=4M", (unsigned long long)(tb >> 20));
            timeit(nm, [&] { k_load<<<g, 256>>>(t, tb, n, 6, o, 2); }, 6.0 * n, "load");
            snprintf(nm, sizeof nm, "atomicOr ret rand %lluMB n=4M", (unsigned long long)(tb >> 20));
            timeit(nm, [&] { k_atomic_or_ret<<<g, 256>>>((uint32_t *)t, tb / 4, n, o, 9); }, n, "atom");
        }
        timeit("load 1B x6 nontemporal 534MB n=4M", [&] { k_load_nt<<<g, 256>>>(t, bloom, n, 6, o, 2); }, 6.0 * n, "load");
        timeit("load 16B x6 rand 534MB n=4M", [&] { k_load16<<<g, 256>>>((const uint4 *)t, bloom / 16, n, 6, o, 2); }, 6.0 * n, "load");
        timeit("load 1B x6 same-4KiB-page 534MB n=4M", [&] { k_load_page<<<g, 256>>>(t, bloom, n, 6, o, 2); }, 6.0 * n, "load");
        timeit("load 1B x6 rand 534MB n=4M block=64", [&] { k_load<<<unsigned(n / 64), 64>>>(t, bloom, n, 6, o, 2); }, 6.0 * n, "load");
        timeit("load 1B x6 rand 534MB n=4M block=1024", [&] { k_load<<<unsigned(n / 1024), 1024>>>(t, bloom, n, 6, o, 2); }, 6.0 * n, "load");
    }
    uint64_t nv = (512ull << 20) / 16;
    timeit("stream copy 512MB (read+write GB/s)", [&] { k_stream<<<unsigned(nv / 256), 256>>>((uint4 *)t, nv, (uint4 *)(t + (768ull << 20))); }, 1024.0 * (1 << 20), "B");
    return 0;
}
