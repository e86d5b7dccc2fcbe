// Dev micro-benchmark: issue rate of the 32-bit integer multiplies the Bloom / HLL hashes are built from
// (v_mul_lo_u32, v_mul_hi_u32, v_mad_u64_u32) against v_add_u32, 8 independent chains per lane, every CU busy.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/mulrate tools/micro/mulrate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ void __launch_bounds__(256) k_rate(uint32_t iters, uint32_t seed, uint32_t *out) {
    uint32_t a[8];
    uint64_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        a[i] = seed + threadIdx.x * 8 + i;
        w[i] = a[i];
    }
    const uint32_t k = seed | 1u;
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                // inline asm: one instruction per step, none folded away by the compiler
                if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(k));
                if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(k));
                if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(k));
                if (OP == 3) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "v"(k) : "vcc");
            }
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= a[i] ^ uint32_t(w[i]) ^ uint32_t(w[i] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP> float run(uint32_t *d, int grid, uint32_t iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, 4u, 7u, d); // warm
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, iters, 7u, d);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    const int grid = 256 * 16; // 16 workgroups of 256 per CU
    const uint32_t iters = 2000;
    uint32_t *d;
    if (hipMalloc(&d, size_t(grid) * 256 * 4) != hipSuccess) return 1;
    const double ops = double(grid) * 256 * iters * 16 * 8; // lane-ops
    const char *names[4] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32"};
    float t[4] = {run<0>(d, grid, iters), run<1>(d, grid, iters), run<2>(d, grid, iters), run<3>(d, grid, iters)};
    for (int i = 0; i < 4; i++)
        printf("%-24s %8.3f ms  %8.1f G lane-ops/s  %.2fx the add time\n", names[i], t[i], ops / (t[i] * 1e-3) / 1e9,
               t[i] / t[0]);
    (void)hipFree(d);
    return 0;
}
