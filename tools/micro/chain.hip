// Micro-benchmark: MurmurHash64A's sequential state chain h = (h ^ k) * m over precomputed k[] (one wave).
// Variant S: uniform loads (s_load) + SALU 64-bit chain.  Variant V: one lane, VALU chain (as the round-2 chain kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_fill(uint64_t *k, uint64_t n) {
    uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
    if (i < n) { uint64_t x = i * 0x9E3779B97F4A7C15ull; x ^= x >> 31; k[i] = x * 0xc6a4a7935bd1e995ull; }
}

template <int U>
__global__ void __launch_bounds__(64) k_chain_s(const uint64_t *__restrict__ k, uint64_t n, uint64_t h0, uint64_t *__restrict__ out) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = h0;
    uint64_t i = 0;
    for (; i + U <= n; i += U) {
        uint64_t kv[U];
#pragma unroll
        for (int q = 0; q < U; q++) kv[q] = k[i + q];
#pragma unroll
        for (int q = 0; q < U; q++) h = (h ^ kv[q]) * m;
    }
    for (; i < n; i++) h = (h ^ k[i]) * m;
    if (threadIdx.x == 0) out[0] = h;
}


template <int U>
__global__ void __launch_bounds__(64) k_chain_sp(const uint64_t *__restrict__ k, uint64_t n, uint64_t h0, uint64_t *__restrict__ out) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = h0;
    uint64_t i = 0;
    if (n >= 2 * U) {
        uint64_t kv[U], kn[U];
#pragma unroll
        for (int q = 0; q < U; q++) kv[q] = k[q];
        for (; i + 2 * U <= n; i += U) {
#pragma unroll
            for (int q = 0; q < U; q++) kn[q] = k[i + U + q];
#pragma unroll
            for (int q = 0; q < U; q++) h = (h ^ kv[q]) * m;
#pragma unroll
            for (int q = 0; q < U; q++) kv[q] = kn[q];
        }
#pragma unroll
        for (int q = 0; q < U; q++) h = (h ^ kv[q]) * m;
        i += U;
    }
    for (; i < n; i++) h = (h ^ k[i]) * m;
    if (threadIdx.x == 0) out[0] = h;
}


// compute floors: k generated in registers (k_i = i * c), no loads
__global__ void __launch_bounds__(64) k_floor_s64(uint64_t n, uint64_t h0, uint64_t *__restrict__ out) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = h0, kk = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < n; i += 4) {
#pragma unroll
        for (int q = 0; q < 4; q++) { h = (h ^ kk) * m; kk += 0x9E3779B97F4A7C15ull; }
    }
    if (threadIdx.x == 0) out[0] = h;
}
__global__ void __launch_bounds__(64) k_floor_s32(uint64_t n, uint32_t h0, uint64_t *__restrict__ out) {
    const uint32_t m = 0x5bd1e995u;
    uint32_t h = h0, kk = 0x7F4A7C15u;
    for (uint64_t i = 0; i < n; i += 4) {
#pragma unroll
        for (int q = 0; q < 4; q++) { h = (h ^ kk) * m; kk += 0x7F4A7C15u; }
    }
    if (threadIdx.x == 0) out[0] = h;
}
__global__ void __launch_bounds__(64) k_floor_v32(uint64_t n, uint32_t h0, uint64_t *__restrict__ out) {
    const uint32_t m = 0x5bd1e995u;
    uint32_t h = h0 + threadIdx.x, kk = 0x7F4A7C15u + threadIdx.x;   // lane-varying: stays on the VALU
    for (uint64_t i = 0; i < n; i += 4) {
#pragma unroll
        for (int q = 0; q < 4; q++) { h = (h ^ kk) * m; kk += 0x7F4A7C15u; }
    }
    if (threadIdx.x == 0) out[0] = h;
}

__global__ void __launch_bounds__(64) k_chain_v(const uint64_t *__restrict__ k, uint64_t n, uint64_t h0, uint64_t *__restrict__ out) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    if (threadIdx.x != 0) return;
    uint64_t h = h0;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t kv[8];
#pragma unroll
        for (int q = 0; q < 8; q++) kv[q] = k[i + q];
#pragma unroll
        for (int q = 0; q < 8; q++) h = (h ^ kv[q]) * m;
    }
    for (; i < n; i++) h = (h ^ k[i]) * m;
    out[0] = h;
}

int main() {
    const uint64_t n = 5161578; // the C1 Q1 element's 8-byte blocks
    uint64_t *k, *o;
    CK(hipMalloc(&k, n * 8)); CK(hipMalloc(&o, 64));
    hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, 0, k, n);
    std::vector<uint64_t> hk(n);
    CK(hipMemcpy(hk.data(), k, n * 8, hipMemcpyDeviceToHost));
    uint64_t ref = 0x1234;
    for (uint64_t i = 0; i < n; i++) ref = (ref ^ hk[i]) * 0xc6a4a7935bd1e995ull;
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](const char *name, auto fn) {
        for (int r = 0; r < 3; r++) {
            CK(hipMemset(o, 0, 64));
            CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            uint64_t got; CK(hipMemcpy(&got, o, 8, hipMemcpyDeviceToHost));
            printf("%-10s %8.2f ms  %s\n", name, ms, got == ref ? "ok" : "MISMATCH");
        }
        return 0;
    };
    run("valu", [&] { hipLaunchKernelGGL(k_chain_v, dim3(1), dim3(64), 0, 0, k, n, 0x1234ull, o); });
    run("salu_u8", [&] { hipLaunchKernelGGL(k_chain_s<8>, dim3(1), dim3(64), 0, 0, k, n, 0x1234ull, o); });
    run("salu_u16", [&] { hipLaunchKernelGGL(k_chain_s<16>, dim3(1), dim3(64), 0, 0, k, n, 0x1234ull, o); });
    run("salu_u32", [&] { hipLaunchKernelGGL(k_chain_s<32>, dim3(1), dim3(64), 0, 0, k, n, 0x1234ull, o); });
    auto tfloor = [&](const char *name, auto fn) {
        for (int r = 0; r < 2; r++) {
            CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            printf("%-10s %8.2f ms  (%.1f ns/step)\n", name, ms, ms * 1e6 / n);
        }
        return 0;
    };
    tfloor("floor_s64", [&] { hipLaunchKernelGGL(k_floor_s64, dim3(1), dim3(64), 0, 0, n, 0x1234ull, o); });
    tfloor("floor_s32", [&] { hipLaunchKernelGGL(k_floor_s32, dim3(1), dim3(64), 0, 0, n, 0x1234u, o); });
    tfloor("floor_v32", [&] { hipLaunchKernelGGL(k_floor_v32, dim3(1), dim3(64), 0, 0, n, 0x1234u, o); });
    run("salu_p8", [&] { hipLaunchKernelGGL(k_chain_sp<8>, dim3(1), dim3(64), 0, 0, k, n, 0x1234ull, o); });
    run("salu_p16", [&] { hipLaunchKernelGGL(k_chain_sp<16>, dim3(1), dim3(64), 0, 0, k, n, 0x1234ull, o); });
    return 0;
}
