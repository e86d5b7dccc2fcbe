// Micro-benchmark (dev tool): the PFADD line apply's register-line traffic, u8 lines (128 B per 128 registers,
// 16 KiB per sketch) against Redis's packed 6-bit lines (96 B per 128 registers, 12 KiB per sketch: a line at
// byte 96 L straddles 128-B cache lines for L % 4 in {1, 2}).  One 256-thread workgroup per fine bucket (coarse bucket
// b, 128 sketches), each reading its 128 lines (line (b - rot(s)) & 127 of sketch s) and storing them back changed.
// Grid orders: "bucket-major" (the apply's: f = b * nsub + sub) and "xcd" (the 128 buckets of one sketch group
// consecutive on one XCD, so neighbouring lines' shared 128-B cache lines meet in one L2).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/packed_lines tools/micro/packed_lines.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHK(x)                                                                                                         \
    do {                                                                                                               \
        hipError_t e = (x);                                                                                            \
        if (e != hipSuccess) {                                                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                                     \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t rot(uint32_t s) { return (s * 0x9E3779B1u) >> 25; }

__device__ __forceinline__ uint32_t fine_of(uint32_t bx, uint32_t nsub, int xcd) {
    if (!xcd) return bx; // f = b * nsub + sub
    // bx = 8 * (grp * 128 + b) + x, sub = grp * 8 + x
    const uint32_t x = bx & 7u, j = bx >> 3, b = j & 127u, grp = j >> 7;
    return b * nsub + grp * 8 + x;
}

// u8 lines: 8 threads x 16 B per line, 32 lines per pass of 256 threads
__global__ void __launch_bounds__(256) k_u8(uint8_t *arena, uint32_t nsub, uint32_t nslab, int xcd) {
    __shared__ uint4 lds[128 * 8];
    const uint32_t f = fine_of(blockIdx.x, nsub, xcd), b = f / nsub, sub = f % nsub;
    if (sub >= nsub) return;
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t q = threadIdx.x + j * 256, i = q >> 3, s = sub * 128 + i;
        if (s < nslab)
            v[j] = reinterpret_cast<const uint4 *>(arena + uint64_t(s) * 16384 + (((b - rot(s)) & 127u) << 7))[q & 7];
    }
#pragma unroll
    for (int j = 0; j < 4; j++) lds[threadIdx.x + j * 256] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t q = threadIdx.x + j * 256, i = q >> 3, s = sub * 128 + i;
        uint4 x = lds[q ^ 1];
        x.x += 1;
        if (s < nslab)
            reinterpret_cast<uint4 *>(arena + uint64_t(s) * 16384 + (((b - rot(s)) & 127u) << 7))[q & 7] = x;
    }
}

// packed lines: 8 threads x 12 B (three dwords: 16 registers) per line
__global__ void __launch_bounds__(256) k_p6(uint8_t *arena, uint32_t nsub, uint32_t nslab, int xcd) {
    __shared__ uint4 lds[128 * 8];
    const uint32_t f = fine_of(blockIdx.x, nsub, xcd), b = f / nsub, sub = f % nsub;
    if (sub >= nsub) return;
    uint32_t w[4][3];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t q = threadIdx.x + j * 256, i = q >> 3, s = sub * 128 + i;
        if (s < nslab) {
            const uint32_t *p = reinterpret_cast<const uint32_t *>(arena + uint64_t(s) * 12288 +
                                                                   ((b - rot(s)) & 127u) * 96 + (q & 7) * 12);
            w[j][0] = p[0];
            w[j][1] = p[1];
            w[j][2] = p[2];
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) lds[threadIdx.x + j * 256] = make_uint4(w[j][0], w[j][1], w[j][2], 0);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t q = threadIdx.x + j * 256, i = q >> 3, s = sub * 128 + i;
        uint4 x = lds[q ^ 1];
        x.x += 1;
        if (s < nslab) {
            uint32_t *p = reinterpret_cast<uint32_t *>(arena + uint64_t(s) * 12288 + ((b - rot(s)) & 127u) * 96 +
                                                       (q & 7) * 12);
            p[0] = x.x;
            p[1] = x.y;
            p[2] = x.z;
        }
    }
}

int main(int argc, char **argv) {
    const uint32_t nslab = argc > 1 ? atoi(argv[1]) : 100000;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const uint32_t nsub = (nslab + 127) / 128, nsubx = (nsub + 7) / 8 * 8;
    uint8_t *a = nullptr;
    CHK(hipMalloc(&a, uint64_t(nsubx) * 128 * 16384));
    CHK(hipMemset(a, 0, uint64_t(nsubx) * 128 * 16384));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int kind = 0; kind < 2; kind++)
        for (int xcd = 0; xcd < 2; xcd++) {
            const uint32_t grid = xcd ? 128 * nsubx : 128 * nsub;
            const uint32_t ns = xcd ? nsubx : nsub;
            auto run = [&] {
                if (kind == 0) hipLaunchKernelGGL(k_u8, dim3(grid), dim3(256), 0, 0, a, ns, nslab, xcd);
                else hipLaunchKernelGGL(k_p6, dim3(grid), dim3(256), 0, 0, a, ns, nslab, xcd);
            };
            run();
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0));
            for (int r = 0; r < reps; r++) run();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            const double lines = double(nslab) * 128, bytes = lines * (kind ? 96 : 128) * 2;
            printf("%s %-12s %u sketches: %.3f ms per pass, %.0f GB/s of line bytes (%.0f B per line each way)\n",
                   kind ? "packed6" : "u8     ", xcd ? "xcd-order" : "bucket-major", nslab, ms, bytes / ms / 1e6,
                   kind ? 96.0 : 128.0);
        }
    CHK(hipFree(a));
    return 0;
}
