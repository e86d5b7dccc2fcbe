// micro_alloc.hip -- does the allocation's memory type change the random
// line-request ceiling on gfx950?  Random 1-B loads (6 independent per lane,
// the Bloom-contains shape), 1-B stores and 1-B read-modify-writes over a
// 534 MB table (the C3 filter) allocated with hipMalloc and with each
// hipExtMallocWithFlags type.  Prints one line per (type, op).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

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
__global__ void k_fill(uint4 *t, uint64_t n16) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n16) t[i] = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
}

int main() {
    const uint64_t bytes = 534ull << 20, n = 1ull << 22;
    uint32_t *o;
    if (hipMalloc(&o, 64) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct Kind {
        const char *name;
        int flags; // -1: hipMalloc
    } kinds[] = {{"hipMalloc", -1},
                 {"ext Default", hipDeviceMallocDefault},
                 {"ext Finegrained", hipDeviceMallocFinegrained},
                 {"ext Uncached", hipDeviceMallocUncached},
                 {"ext Contiguous", hipDeviceMallocContiguous}};
    unsigned g = unsigned(n / 256);
    for (auto &k : kinds) {
        uint8_t *t = nullptr;
        hipError_t e = k.flags < 0 ? hipMalloc(&t, bytes) : hipExtMallocWithFlags((void **)&t, bytes, unsigned(k.flags));
        if (e != hipSuccess) {
            printf("%-18s alloc failed: %s\n", k.name, hipGetErrorString(e));
            continue;
        }
        k_fill<<<unsigned((bytes / 16 + 255) / 256), 256>>>((uint4 *)t, bytes / 16);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        auto timeit = [&](const char *op, auto fn, double units) {
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
            printf("%-18s %-28s %9.1f us %8.2f G/s\n", k.name, op, best * 1e3, units / (best * 1e-3) / 1e9);
        };
        timeit("load 1B x6 rand (4M lanes)", [&] { k_load<<<g, 256>>>(t, bytes, n, 6, o, 2); }, 6.0 * n);
        timeit("store 1B rand (4M)", [&] { k_store<<<g, 256>>>(t, bytes, n, 4); }, double(n));
        timeit("load+cond store 1B (4M)", [&] { k_rmw<<<g, 256>>>(t, bytes, n, 5); }, double(n));
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        hipFree(t);
    }
    return 0;
}
