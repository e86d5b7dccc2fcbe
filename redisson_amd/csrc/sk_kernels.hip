// sk_kernels.hip -- CDNA4 (gfx950) kernels of the sketch engine.
//
// Layout in HBM (see DESIGN.md "Data layout"):
//   HLL arena   : Redis's dense register bodies, 12,288 B (16384 x 6 bits) per slab,
//                 slab id -> arena + id * 12288 (SK_SLAB_BYTES; GET copies it).
//   bit strings : one buffer per key, Redis MSB-first bytes, capacity a
//                 multiple of 16 B, bytes in [len, cap) kept zero; a device
//                 directory {ptr, len, cap} per string id, len grown by
//                 atomicMax (sdsgrowzero semantics).
//
// Sequential-reply semantics inside a batch (PFADD's 1/0, SETBIT's old bit,
// Bloom add's "a probe saw 0") are made exact by a stable radix sort on the
// touched slot (rocPRIM) followed by a segment-head walk in batch order; the
// final state (max / OR) needs no atomics because each slot has one head.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>

#include "sk_device.h"
#include "sk_internal.h"

namespace sk {

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 0x7fffffffu) {
    uint64_t g = (n + block - 1) / block;
    if (g == 0) g = 1;
    return g > cap ? cap : unsigned(g);
}

// ------------------------------------------------------------------ the HLL arena: Redis's dense registers
// A slab is the 12,288-B register body of Redis's dense encoding (HLL_DENSE_GET/SET_REGISTER, hyperloglog.c):
// register i in bits [6i, 6i + 6) of the body, LSB first.  So 16 registers are exactly 12 bytes (three u32 words) and
// a 128-register line exactly 96 bytes; GET / DUMP / SAVE copy the body as it is.  The arena ends with 16 B of
// padding (a field read takes the byte after its own).
#define SK_SLAB_BYTES 12288u
__device__ __forceinline__ uint8_t *slab_at(uint8_t *arena, uint64_t slab) { return arena + slab * SK_SLAB_BYTES; }
__device__ __forceinline__ const uint8_t *slab_at(const uint8_t *arena, uint64_t slab) {
    return arena + slab * SK_SLAB_BYTES;
}
// the slab of a caller's handle (slab | generation << 24).  The empty asm keeps the mask: hipcc (ROCm 7.2) compiles
// `(h & 0xffffff) * 12288` into one v_mad_u64_u32 of the UNMASKED h, so a handle with a nonzero generation addressed
// 12288 x 2^24 x gen bytes past its slab (a memory aperture violation on the GPU, round 6; tools/micro: the 4-line
// reproducer in DESIGN "The packed arena").  With the barrier the AND is materialised before the multiply.
__device__ __forceinline__ uint64_t slab_of(uint32_t handle) {
    uint32_t s = handle & SK_SLAB_MASK;
    __asm__ volatile("" : "+v"(s));
    return s;
}
// register r of a slab (two byte loads: the field may straddle a byte boundary)
__device__ __forceinline__ uint32_t reg_get(const uint8_t *slab, uint32_t r) {
    const uint32_t bit = 6u * r, by = bit >> 3;
    return ((uint32_t(slab[by]) | (uint32_t(slab[by + 1]) << 8)) >> (bit & 7u)) & 63u;
}
// register r of a slab from `old` to old ^ x: device-scope XORs on its aligned word(s).  Other registers of the same
// words may change at the same time (their own XORs commute with this one); the caller is this register's only
// writer and knows its value.
__device__ __forceinline__ void reg_xor(uint8_t *slab, uint32_t r, uint32_t x) {
    if (!x) return;
    uint32_t *w = reinterpret_cast<uint32_t *>(slab);
    const uint32_t bit = 6u * r, wi = bit >> 5, sh = bit & 31u;
    atomicXor(&w[wi], x << sh);
    if (sh > 26u) atomicXor(&w[wi + 1], x >> (32u - sh));
}
// 16 registers <-> their 12 bytes: a 16-B vector of u8 registers <-> three u32 words
__device__ __forceinline__ void pack16(uint4 r, uint32_t *w) {
    const uint32_t b0 = r.x, b1 = r.y, b2 = r.z, b3 = r.w;
    auto g = [](uint32_t v, int i) { return (v >> (8 * i)) & 63u; };
    w[0] = g(b0, 0) | g(b0, 1) << 6 | g(b0, 2) << 12 | g(b0, 3) << 18 | g(b1, 0) << 24 | (g(b1, 1) & 3u) << 30;
    w[1] = g(b1, 1) >> 2 | g(b1, 2) << 4 | g(b1, 3) << 10 | g(b2, 0) << 16 | g(b2, 1) << 22 | (g(b2, 2) & 15u) << 28;
    w[2] = g(b2, 2) >> 4 | g(b2, 3) << 2 | g(b3, 0) << 8 | g(b3, 1) << 14 | g(b3, 2) << 20 | g(b3, 3) << 26;
}
__device__ __forceinline__ uint4 unpack16(uint32_t w0, uint32_t w1, uint32_t w2) {
    auto q = [](uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return a | b << 8 | c << 16 | d << 24; };
    const uint32_t r0 = w0 & 63u, r1 = (w0 >> 6) & 63u, r2 = (w0 >> 12) & 63u, r3 = (w0 >> 18) & 63u;
    const uint32_t r4 = (w0 >> 24) & 63u, r5 = (w0 >> 30) | ((w1 & 15u) << 2), r6 = (w1 >> 4) & 63u;
    const uint32_t r7 = (w1 >> 10) & 63u, r8 = (w1 >> 16) & 63u, r9 = (w1 >> 22) & 63u;
    const uint32_t r10 = (w1 >> 28) | ((w2 & 3u) << 4), r11 = (w2 >> 2) & 63u, r12 = (w2 >> 8) & 63u;
    const uint32_t r13 = (w2 >> 14) & 63u, r14 = (w2 >> 20) & 63u, r15 = w2 >> 26;
    return make_uint4(q(r0, r1, r2, r3), q(r4, r5, r6, r7), q(r8, r9, r10, r11), q(r12, r13, r14, r15));
}
// group g (16 registers) of a packed body: three word loads (nontemporal: streamed once)
__device__ __forceinline__ uint4 grp_load_nt(const uint8_t *body, uint32_t g) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(body) + 3 * g;
    return unpack16(__builtin_nontemporal_load(w), __builtin_nontemporal_load(w + 1), __builtin_nontemporal_load(w + 2));
}
__device__ __forceinline__ uint4 grp_load(const uint8_t *body, uint32_t g) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(body) + 3 * g;
    return unpack16(w[0], w[1], w[2]);
}
__device__ __forceinline__ void grp_store(uint8_t *body, uint32_t g, uint4 r) {
    uint32_t p[3];
    pack16(r, p);
    uint32_t *w = reinterpret_cast<uint32_t *>(body) + 3 * g;
    w[0] = p[0];
    w[1] = p[1];
    w[2] = p[2];
}

// ------------------------------------------------------------------ PFADD
// hllPatLen: register index = low 14 bits; rho = 1 + trailing zeros of
// bits 14.. with the version's sentinel (3.2: bit 63 -> rho <= 50,
// >= 5.0: bit 64 of the shifted hash at HLL_Q=50 -> rho <= 51).
__device__ __forceinline__ void hll_pat(uint64_t h, int v5, uint32_t *reg, uint32_t *rho) {
    *reg = uint32_t(h & 16383u);
    uint64_t x = (h >> 14) | (v5 ? (1ull << 50) : (1ull << 49));
    *rho = 1u + uint32_t(__builtin_ctzll(x));
}

// Bloom add: the string length follows the largest probed bit = the last sorted key
__global__ void k_len_from_last_key(const uint64_t *keys, uint64_t m, uint64_t *d_len) {
    uint64_t need = (keys[m - 1] >> 35) + 1; // (idx >> 3) + 1 with idx = key >> 32
    atomicMax((unsigned long long *)d_len, (unsigned long long)need);
}


// ------------------------------------------------- PFADD, partition path
// Two launches, no global scan and no sort:
//   k_pfp_hash   one workgroup per SK_PFP_EPB elements: hash, bucket each
//                record by its register slot (every record of a slot lands in
//                one bucket), counting-sort the block's records by bucket in
//                LDS, store them as one coalesced chunk plus the block's
//                bucket start offsets (bucket-major table S[b][block]);
//   k_pfp_apply  one workgroup per bucket: gather the bucket's segment from
//                every block chunk into LDS, chain the records of a slot with
//                an LDS hash table; the earliest (lowest seq) record of each
//                slot loads R0 and writes the final max, and a record replies
//                1 iff its rho beats R0 and every earlier rho of its slot --
//                the sequential PFADD result with one random load + one store
//                per touched register and no global atomics.
//   rec = slot << 26 | seq << 6 | rho   (slot <= 38 bits, seq < 2^20)
// Buckets larger than SK_PFP_CAP (hot registers, skew) are resolved by the
// same workgroup from a (slot, rho) -> min seq table (pfp_big_resolve).
#ifndef SK_PFP_NB
#define SK_PFP_NB 512     // buckets (~n/512 records each; ~8 records = one 64-B line per block segment)
#endif
#define SK_PFP_TPB 1024   // threads per hash workgroup (16 waves: one per CU hides the latency)
#define SK_PFP_EPB 4096   // elements per line-schedule hash workgroup (12-bit element-in-block)
#ifndef SK_PFQ_EPB
#define SK_PFQ_EPB 4096   // elements per partition-path hash workgroup (2048, two per CU: slower, r06s)
#endif
#define SK_PFQ_TPS (SK_PFP_ATPB * SK_PFQ_EPB >> 20) // apply threads per hash block (n <= 2^20)
#define SK_PFP_ATPB 1024  // threads per apply workgroup (4 per block segment)
#define SK_PFP_CAP 4096   // records one apply workgroup holds in LDS
#define SK_PFP_HT 4096    // LDS hash-chain heads
#define SK_PFP_STAGE (4 * SK_STAGE_WORDS) // LDS key window (u64 words) for SK_PFP_TPB elements
static_assert(SK_PFQ_TPS >= 1 && (SK_PFQ_TPS & (SK_PFQ_TPS - 1)) == 0 && SK_PFQ_TPS <= 64 &&
              SK_PFP_ATPB / SK_PFQ_TPS * SK_PFQ_EPB >= (1 << 20), "apply threads per hash block");
static_assert(SK_PFP_NB <= SK_PFP_TPB, "one bucket per hash thread in the start scan");
static_assert(SK_PFP_CAP < 0xffff, "u16 chain links");
// a bucket takes whole runs of 32 registers of a sketch: the records of a hot sketch (C1, a Zipf head) in one
// bucket then read their registers from one 32-B piece, so a wave's register loads coalesce into one request.
// Run g of sketch s goes to bucket (g + hash(s)) % 512: the 512 runs of every sketch cover the 512 buckets once
// each (one hot sketch fills every bucket evenly), and sketches are rotated against each other.
static_assert(SK_PFP_NB == 512 || SK_PFP_NB == 1024, "16384 registers = 512 runs of 32 (or 1024 of 16)");
__device__ __forceinline__ uint32_t pfp_bucket(uint64_t slot) {
    constexpr uint32_t LNB = SK_PFP_NB == 512 ? 9 : 10, RB = 14 - LNB;
    const uint32_t run = uint32_t(slot >> RB) & (SK_PFP_NB - 1u), rot = (uint32_t(slot >> 14) * 0x9E3779B1u) >> (32 - LNB);
    return (run + rot) & (SK_PFP_NB - 1u);
}
__device__ __forceinline__ uint32_t pfp_ht(uint64_t slot) {
    return uint32_t((slot * 0xC2B2AE3D27D4EB4Full) >> 52); // 12 bits
}

// exclusive scan of one value per thread over a workgroup of NT threads;
// `wsum` is LDS scratch of NT/64 words; returns the exclusive prefix, *total = sum
template <int NT> __device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wsum, uint32_t *total) {
    uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        uint32_t y = __shfl_up(x, s);
        if (lane >= uint32_t(s)) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
        uint32_t t = wsum[i];
        base += i < int(w) ? t : 0u;
        tot += t;
    }
    __syncthreads(); // wsum reusable
    *total = tot;
    return base + x - v;
}

// Key bytes are staged through two LDS windows: the global loads of window
// e+1 are issued (into registers) before round e is hashed, so one barrier
// per round is the only wait; every element's offsets and slab id are loaded
// up front.  Windows that do not fit fall back to direct global reads.
#define SK_PFP_WIN 5056 // u64 words per key window (39.5 KiB: 1024 keys of mean length <= ~39 B; two hash workgroups per CU)
#define SK_PFP_WVEC ((SK_PFP_WIN * 8 / 16 + SK_PFP_TPB - 1) / SK_PFP_TPB) // 16-B vectors per thread per window (loads and stores stop at the window's vectors)
__device__ __forceinline__ bool pfp_win_fits(uint64_t lo, uint64_t hi) {
    return (hi - (lo & ~uint64_t(15))) + 32 <= uint64_t(SK_PFP_WIN) * 8;
}
__device__ __forceinline__ void pfp_win_load(const uint8_t *bytes, uint64_t lo, uint64_t hi, uint4 (&v)[SK_PFP_WVEC]) {
    uint64_t a0 = lo & ~uint64_t(15);
    uint32_t nvec = uint32_t((hi - a0 + 15) >> 4);
    const uint4 *src = reinterpret_cast<const uint4 *>(bytes + a0);
#pragma unroll
    for (int q = 0; q < SK_PFP_WVEC; q++) {
        uint32_t idx = threadIdx.x + q * SK_PFP_TPB;
        v[q] = idx < nvec ? src[idx] : make_uint4(0, 0, 0, 0);
    }
}
// stores the window and the 16 zero bytes after it (readers look up to 15 B past a key)
__device__ __forceinline__ void pfp_win_store(uint64_t lo, uint64_t hi, const uint4 (&v)[SK_PFP_WVEC], uint64_t *buf) {
    uint32_t nvec = uint32_t((hi - (lo & ~uint64_t(15)) + 15) >> 4);
    uint4 *dst = reinterpret_cast<uint4 *>(buf);
#pragma unroll
    for (int q = 0; q < SK_PFP_WVEC; q++) {
        uint32_t idx = threadIdx.x + q * SK_PFP_TPB;
        if (idx <= nvec) dst[idx] = v[q];
    }
}

// line schedule (sketch-major group apply, below): coarse bucket of a register = its 128-register line, rotated
// per sketch, so bucket b holds exactly one line of every sketch and a hot sketch spreads over all 128 buckets
#define SK_PFL_NB 128 // coarse buckets = register lines per sketch
#define SK_PFL_LB 7   // log2 registers per line: 128 registers = one 128-B line (64-register pieces at 256 buckets:
                      // apply 1.62 vs 1.31 ms per 64 M, Zipf no better)
static_assert((SK_PFL_NB << SK_PFL_LB) == 16384, "the lines tile a sketch");
__device__ __forceinline__ uint32_t pfl_rot(uint32_t slab) { return (slab * 0x9E3779B1u) >> (32 - 7); }
static_assert(SK_PFL_NB == 128, "pfl_rot draws 7 bits");
__device__ __forceinline__ uint32_t pfl_bucket(uint32_t slab, uint32_t reg) {
    return ((reg >> SK_PFL_LB) + pfl_rot(slab)) & (SK_PFL_NB - 1);
}
__device__ __forceinline__ uint32_t pfl_slotb(uint64_t key) { // key = slab_low << 14 | reg -> the register in LDS
    return uint32_t(key >> 14) << SK_PFL_LB | (uint32_t(key) & ((1u << SK_PFL_LB) - 1));
}

#ifndef SK_PFL_C6
#define SK_PFL_C6 0        // the line hash's block chunks as 6-B records too: measured slower (region pass 0.35 -> 0.445 ms)
#endif
// k_pfl_hash's records: slab << 32 | reg << 18 | rho << 12 | element-in-block, read back by the region pass with
// reg's line bits zero in the 6-B form (the coarse bucket and the slab fix them).  6-B form: a u32 plane of the
// low 32 bits with slab_low7 in bits 25..31, and a u16 plane of slab >> 7 (slab ids >= 2^23 kept as 2^23 - 1, which
// is past every store's slab count, so those records are still dropped).
struct PflChunk {
    uint64_t *p;
    uint64_t cap; // records: hash blocks x SK_PFP_EPB
    __device__ __forceinline__ void put(uint64_t i, uint64_t r) const {
        if (SK_PFL_C6) {
            uint32_t slab = uint32_t(r >> 32);
            slab = slab < (1u << 23) ? slab : (1u << 23) - 1u;
            reinterpret_cast<uint32_t *>(p)[i] = (slab << 25) | (uint32_t(r) & ((1u << 25) - 1u));
            reinterpret_cast<uint16_t *>(reinterpret_cast<uint32_t *>(p) + cap)[i] = uint16_t(slab >> 7);
        } else {
            p[i] = r;
        }
    }
    __device__ __forceinline__ uint64_t get(uint64_t i) const {
        if (SK_PFL_C6) {
            const uint32_t lo = reinterpret_cast<const uint32_t *>(p)[i];
            const uint32_t hi = reinterpret_cast<const uint16_t *>(reinterpret_cast<const uint32_t *>(p) + cap)[i];
            return (uint64_t((hi << 7) | (lo >> 25)) << 32) | (lo & ((1u << 25) - 1u));
        }
        return p[i];
    }
};

// NBK buckets; LINE = false: the partition path (records slot << 26 | seq << 6 | rho, pfp_bucket),
// LINE = true: the line schedule (records slab << 32 | reg << 18 | rho << 12 | element-in-block, pfl_bucket)
template <int NBK, bool LINE, int EPB>
__device__ __forceinline__ void pfp_hash_impl(uint64_t n, const uint32_t *__restrict__ key_ids,
                                              const uint64_t *__restrict__ off, const uint8_t *__restrict__ bytes,
                                              int v5, uint64_t *__restrict__ chunks, uint32_t *__restrict__ S,
                                              uint32_t nblocks, uint16_t *__restrict__ pos,
                                              uint32_t *__restrict__ big_alloc, const uint64_t *__restrict__ pre_h) {
    // the block's records reuse the key windows' LDS once the last round is hashed: 98 KiB in all, so a hash
    // workgroup (the next batch, on the third stream) fits on a CU beside an apply workgroup (61.5 KiB)
    // bucket counts and starts as u16 (<= EPB): counted with u32 adds on the pairs' words; the scan's wave sums sit
    // at the end of the second key window (free once the last round is hashed).  80 KiB in all: two hash workgroups
    // per CU.
    __shared__ uint32_t h32[NBK / 2];
    __shared__ uint64_t win[2][SK_PFP_WIN];
    static_assert(EPB <= 2 * SK_PFP_WIN && EPB <= 0xffff && NBK % 2 == 0, "records fit the windows");
    uint16_t *h = reinterpret_cast<uint16_t *>(h32);
    uint32_t *wsum = reinterpret_cast<uint32_t *>(&win[1][SK_PFP_WIN - SK_PFP_TPB / 128]);
    static_assert(EPB * 8 <= SK_PFP_WIN * 8 * 2 - SK_PFP_TPB / 16, "records clear of the wave sums");
    uint64_t *lrec = &win[0][0];
    for (uint32_t b = threadIdx.x; b < NBK / 2; b += SK_PFP_TPB) h32[b] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        big_alloc[0] = 0;
        if (LINE) big_alloc[1] = big_alloc[2] = 0; // the line plan's heavy / light counters
    }
    constexpr int PER = EPB / SK_PFP_TPB;
    const uint64_t base = uint64_t(blockIdx.x) * EPB;
    const uint64_t rounds = (n - base + SK_PFP_TPB - 1) / SK_PFP_TPB;
    const int nr = rounds < PER ? int(rounds) : PER;
    uint64_t wb[PER + 1], oa[PER], ob[PER];
    uint32_t kid[PER];
#pragma unroll
    for (int e = 0; e <= PER; e++) {
        uint64_t i0 = base + uint64_t(e) * SK_PFP_TPB;
        wb[e] = off[i0 < n ? i0 : n];
    }
#pragma unroll
    for (int e = 0; e < PER; e++) {
        uint64_t i = base + uint64_t(e) * SK_PFP_TPB + threadIdx.x;
        oa[e] = ob[e] = 0;
        kid[e] = 0;
        if (i < n) {
            oa[e] = off[i];
            ob[e] = off[i + 1];
            kid[e] = key_ids[i] & SK_SLAB_MASK;
        }
    }
    uint4 v[SK_PFP_WVEC];
    if (pfp_win_fits(wb[0], wb[1])) {
        pfp_win_load(bytes, wb[0], wb[1], v);
        pfp_win_store(wb[0], wb[1], v, win[0]);
    }
    __syncthreads(); // h zeroed, window 0 staged
    uint64_t r[PER];
    uint32_t bk[PER], rk[PER];
#pragma unroll
    for (int e = 0; e < PER; e++) {
        r[e] = ~0ull;
        bk[e] = rk[e] = 0;
        if (e >= nr) continue; // uniform
        bool pre = e + 1 < nr && pfp_win_fits(wb[e + 1], wb[e + 2]);
        if (pre) pfp_win_load(bytes, wb[e + 1], wb[e + 2], v);
        uint64_t i = base + uint64_t(e) * SK_PFP_TPB + threadIdx.x;
        if (i < n) {
            uint32_t len = uint32_t(ob[e] - oa[e]);
            uint64_t hh = (pre_h && len >= SK_LONG_ELEM) ? pre_h[i] // hashed by the bit-round scan (k_ms_rounds)
                          : pfp_win_fits(wb[e], wb[e + 1])
                              ? murmur64a_r(LdsReader{win[e & 1], uint32_t(wb[e] & 15u) + uint32_t(oa[e] - wb[e])},
                                            len, 0xadc83b19ull)
                              : murmur64a(bytes + oa[e], len, 0xadc83b19ull);
            uint32_t reg, rho;
            hll_pat(hh, v5, &reg, &rho);
            if (LINE) {
                r[e] = (uint64_t(kid[e]) << 32) | (uint64_t(reg) << 18) | (rho << 12) | uint32_t(i - base);
                bk[e] = pfl_bucket(kid[e], reg);
            } else {
                uint64_t slot = (uint64_t(kid[e]) << 14) | reg;
                r[e] = (slot << 26) | (i << 6) | rho;
                bk[e] = pfp_bucket(slot);
            }
            const uint32_t hs = (bk[e] & 1u) << 4;
            rk[e] = (atomicAdd(&h32[bk[e] >> 1], 1u << hs) >> hs) & 0xffffu;
        }
        if (pre) pfp_win_store(wb[e + 1], wb[e + 2], v, win[(e + 1) & 1]);
        __syncthreads(); // window e+1 staged; window e free for round e+2
    }
    // bucket starts (one bucket per thread), row NBK = the block's total
    uint32_t c0 = threadIdx.x < NBK ? h[threadIdx.x] : 0u, tot;
    uint32_t st0 = block_exscan<SK_PFP_TPB>(c0, wsum, &tot);
    if (threadIdx.x < NBK) {
        h[threadIdx.x] = st0;
        S[uint64_t(threadIdx.x) * nblocks + blockIdx.x] = st0;
    }
    if (threadIdx.x == 0) S[uint64_t(NBK) * nblocks + blockIdx.x] = tot;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < PER; e++)
        if (r[e] != ~0ull) {
            uint32_t p = h[bk[e]] + rk[e];
            lrec[p] = r[e];
            if (pos) pos[base + uint64_t(e) * SK_PFP_TPB + threadIdx.x] = uint16_t(p);
        }
    __syncthreads();
    if (LINE && SK_PFL_C6) {
        const PflChunk ch{chunks, uint64_t(nblocks) * EPB};
        for (uint32_t t = threadIdx.x; t < tot; t += SK_PFP_TPB) ch.put(base + t, lrec[t]);
        return;
    }
    uint64_t *dst = chunks + base;
    for (uint32_t t = threadIdx.x; t < tot; t += SK_PFP_TPB) dst[t] = lrec[t];
}

__global__ void __launch_bounds__(SK_PFP_TPB) k_pfp_hash(uint64_t n, const uint32_t *__restrict__ key_ids,
                                                         const uint64_t *__restrict__ off,
                                                         const uint8_t *__restrict__ bytes, int v5,
                                                         uint64_t *__restrict__ chunks, uint32_t *__restrict__ S,
                                                         uint32_t nblocks, uint16_t *__restrict__ pos,
                                                         uint32_t *__restrict__ big_alloc,
                                                         const uint64_t *__restrict__ pre_h) {
    pfp_hash_impl<SK_PFP_NB, false, SK_PFQ_EPB>(n, key_ids, off, bytes, v5, chunks, S, nblocks, pos, big_alloc, pre_h);
}
__global__ void __launch_bounds__(SK_PFP_TPB) k_pfl_hash(uint64_t n, const uint32_t *__restrict__ key_ids,
                                                         const uint64_t *__restrict__ off,
                                                         const uint8_t *__restrict__ bytes, int v5,
                                                         uint64_t *__restrict__ chunks, uint32_t *__restrict__ S,
                                                         uint32_t nblocks, uint32_t *__restrict__ big_alloc) {
    pfp_hash_impl<SK_PFL_NB, true, SK_PFP_EPB>(n, key_ids, off, bytes, v5, chunks, S, nblocks, nullptr, big_alloc, nullptr);
}

// Replies back to batch order: rep holds them in chunk order (written by
// k_pfp_apply as runs per block segment), pos maps element -> chunk slot.
__global__ void __launch_bounds__(SK_PFP_TPB) k_pfp_reply(uint64_t n, const uint8_t *__restrict__ rep,
                                                          const uint16_t *__restrict__ pos,
                                                          const uint32_t *__restrict__ cmd_of,
                                                          uint8_t *__restrict__ changed) {
    __shared__ uint8_t lr[SK_PFQ_EPB];
    const uint64_t base = uint64_t(blockIdx.x) * SK_PFQ_EPB;
    const uint32_t m = uint32_t(n - base < SK_PFQ_EPB ? n - base : SK_PFQ_EPB);
    for (uint32_t t = threadIdx.x; t < m; t += SK_PFP_TPB) lr[t] = rep[base + t];
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < m; t += SK_PFP_TPB) {
        uint64_t i = base + t;
        uint8_t v = lr[pos[i]];
        if (!cmd_of) changed[i] = v;
        else if (v) changed[cmd_of[i]] = 1; // multi-element commands: OR over their elements
    }
}

// ---- long elements (RHyperLogLog.addAll, quirk Q1: ONE element = the Jackson array of every value, ~41 MB at
// C1, M:RedissonHyperLogLog.java:70-76).  MurmurHash64A's state chain h_{i+1} = x_i * m, x_i = h_i ^ k_i, with the
// per-block transform k_i = mix(block i), is sequential in i -- but not bit by bit.  m is odd, so bit j of x * m is
// x_j ^ bit_j((x mod 2^j) * m): with p_i = (x_i mod 2^j) * m,
//     h_{i+1,j} = h_{i,j} ^ d_i,   d_i = k_{i,j} ^ p_{i,j},
// i.e. once bits < j of every x_i are known, bit j of every state h_i is a prefix XOR over i of d.  The chain
// becomes 64 rounds (one per bit) of a device-wide XOR scan over the blocks; each round then sets bit j of every
// x_i (p_i += m << j where x_{i,j} = 1).  A thread owns SK_MS_S consecutive blocks (their p_i in registers, their
// k bits as one word per round from bit planes written by k_ms_planes), a workgroup SK_MS_BPW blocks; across
// workgroups each round is a decoupled look-back over per-(workgroup, round) flags.  Workgroups take ordered ids
// from a counter, so one only waits on workgroups already running; every wait is bounded (err flag, never a hang).
#define SK_MS_S 32
#define SK_MS_TPB 1024
#define SK_MS_BPW (SK_MS_S * SK_MS_TPB)
#define SK_MS_AGG (1u << 30)
#define SK_MS_INCL (1u << 31)
#define SK_MS_SPIN (1u << 20)

// meta: which[n_long] (element index in the batch), first_wg[n_long + 1] (workgroup prefix over the elements), then
// at the next even word the u64 plane offsets poff[n_long + 1] (prefix of 64 * ceil(blocks / 32) words)
__device__ __forceinline__ const uint64_t *ms_poff(const uint32_t *meta, uint32_t n_long) {
    return reinterpret_cast<const uint64_t *>(meta + ((2 * n_long + 2) & ~1u));
}
__device__ __forceinline__ uint32_t ms_elem_of(const uint32_t *first_wg, uint32_t n_long, uint32_t w) {
    uint32_t lo = 0, hi = n_long; // first_wg[lo] <= w < first_wg[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (first_wg[mid] <= w) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(SK_MS_TPB) k_ms_planes(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off,
                                                         const uint32_t *__restrict__ meta, uint32_t n_long,
                                                         uint32_t *__restrict__ plane) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const uint32_t *which = meta, *first_wg = meta + n_long;
    const uint32_t w = blockIdx.x, e = ms_elem_of(first_wg, n_long, w);
    const uint64_t o = off[which[e]], nb = (off[which[e] + 1] - o) >> 3;
    const uint64_t nw = (nb + SK_MS_S - 1) / SK_MS_S; // words per plane
    const uint64_t g = uint64_t(w - first_wg[e]) * SK_MS_TPB + threadIdx.x;
    if (g >= nw) return;
    uint32_t *pl = plane + ms_poff(meta, n_long)[e];
    uint32_t word[64];
#pragma unroll
    for (int j = 0; j < 64; j++) word[j] = 0;
#pragma unroll 1
    for (uint32_t t = 0; t < SK_MS_S; t++) {
        const uint64_t b = g * SK_MS_S + t;
        if (b >= nb) break;
        uint64_t k = ldu64(bytes + o + 8 * b);
        k *= m;
        k ^= k >> 47;
        k *= m;
#pragma unroll
        for (int j = 0; j < 64; j++) word[j] |= uint32_t((k >> j) & 1u) << t;
    }
#pragma unroll
    for (int j = 0; j < 64; j++) pl[uint64_t(j) * nw + g] = word[j];
}

// flags: [n_wg][64] round flags, then the id counter and the err word (zeroed by the launcher)
__global__ void __launch_bounds__(SK_MS_TPB) k_ms_rounds(const uint8_t *__restrict__ bytes, const uint64_t *__restrict__ off,
                                                         const uint32_t *__restrict__ meta, uint32_t n_long,
                                                         uint32_t n_wg, const uint32_t *__restrict__ plane,
                                                         uint32_t *__restrict__ flags, uint64_t seed,
                                                         uint64_t *__restrict__ out_h, uint32_t spin_max) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    __shared__ uint32_t s_id, s_wpar[2][SK_MS_TPB / 64], s_ex[2];
    uint32_t *ctr = flags + uint64_t(n_wg) * 64, *err = ctr + 1;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_id = atomicAdd(ctr, 1u);
    __syncthreads();
    const uint32_t w = s_id;
    const uint32_t *which = meta, *first_wg = meta + n_long;
    const uint32_t e = ms_elem_of(first_wg, n_long, w);
    const uint32_t w0 = first_wg[e], nwg = first_wg[e + 1] - w0, lw = w - w0;
    const uint64_t o = off[which[e]], len = off[which[e] + 1] - o, nb = len >> 3;
    const uint64_t nw = (nb + SK_MS_S - 1) / SK_MS_S;
    const uint64_t g = uint64_t(lw) * SK_MS_TPB + threadIdx.x;
    const bool has = g < nw; // threads past the element's last block carry d = 0
    const uint32_t *pl = plane + ms_poff(meta, n_long)[e] + (has ? g : 0);
    const uint64_t first_b = g * SK_MS_S;
    const uint32_t valid = first_b >= nb ? 0u : (nb - first_b >= SK_MS_S ? 0xffffffffu
                                                                          : (1u << uint32_t(nb - first_b)) - 1u);
    const uint64_t h0 = seed ^ (len * m);
    uint64_t p[SK_MS_S];
#pragma unroll
    for (int t = 0; t < SK_MS_S; t++) p[t] = 0;
    uint64_t fin = 0;
    uint32_t kw = has ? pl[0] : 0u;
#pragma unroll 1
    for (uint32_t j = 0; j < 64; j++) {
        const uint32_t kcur = kw;
        if (has && j + 1 < 64) kw = pl[uint64_t(j + 1) * nw]; // next round's word, in flight during this round
        uint32_t pw = 0;
#pragma unroll
        for (int t = 0; t < SK_MS_S; t++) {
            const uint32_t half = j < 32 ? uint32_t(p[t]) : uint32_t(p[t] >> 32);
            pw |= ((half >> (j & 31u)) & 1u) << t;
        }
        const uint32_t dm = (kcur ^ pw) & valid;
        uint32_t inc = dm;
        inc ^= inc << 1;
        inc ^= inc << 2;
        inc ^= inc << 4;
        inc ^= inc << 8;
        inc ^= inc << 16;
        const uint64_t bal = __ballot(inc >> 31);
        const uint32_t lane_ex = uint32_t(__popcll(bal & ((1ull << lane) - 1ull))) & 1u;
        if (lane == 0) s_wpar[j & 1][wave] = uint32_t(__popcll(bal)) & 1u;
        __syncthreads();
        uint32_t wave_ex = 0, wg_tot = 0;
#pragma unroll
        for (uint32_t v = 0; v < SK_MS_TPB / 64; v++) {
            const uint32_t x = s_wpar[j & 1][v];
            wave_ex ^= v < wave ? x : 0u;
            wg_tot ^= x;
        }
        if (wave == 0) {
            uint32_t *fl = flags + uint64_t(w) * 64 + j;
            uint32_t ex = 0;
            if (lw == 0) {
                if (lane == 0) __hip_atomic_store(fl, SK_MS_INCL | wg_tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (lane == 0) __hip_atomic_store(fl, SK_MS_AGG | wg_tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                int64_t pos = int64_t(w) - 1;
                uint32_t spins = 0;
                for (;;) { // look back over predecessors of this element, 64 at a time
                    const int64_t q = pos - int64_t(lane);
                    const uint32_t f = q >= int64_t(w0)
                        ? __hip_atomic_load(flags + uint64_t(q) * 64 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : SK_MS_INCL;
                    const uint64_t inc_b = __ballot((f & SK_MS_INCL) != 0), rdy = __ballot(f != 0);
                    const uint32_t stop = inc_b ? uint32_t(__ffsll((long long)inc_b)) - 1u : 64u;
                    const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1ull);
                    if ((rdy & need) != need) {
                        if (++spins > spin_max) { // a predecessor never published: report, do not hang
                            if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                        continue;
                    }
                    ex ^= uint32_t(__popcll(__ballot(f & 1u) & need)) & 1u;
                    if (stop < 64) break;
                    pos -= 64;
                }
                if (lane == 0)
                    __hip_atomic_store(fl, SK_MS_INCL | (ex ^ wg_tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (lane == 0) s_ex[j & 1] = ex;
        }
        __syncthreads();
        const uint32_t ex = s_ex[j & 1];
        if (threadIdx.x == 0 && lw == nwg - 1) fin |= uint64_t(((h0 >> j) & 1u) ^ ex ^ wg_tot) << j;
        const uint32_t c = uint32_t((h0 >> j) & 1u) ^ ex ^ wave_ex ^ lane_ex;
        const uint32_t hm = (inc << 1) ^ (c ? 0xffffffffu : 0u); // bit t: bit j of the state before block t
        const uint32_t xm = (hm ^ kcur) & valid;
        const uint64_t mj = m << j;
#pragma unroll
        for (int t = 0; t < SK_MS_S; t++) p[t] += ((xm >> t) & 1u) ? mj : 0ull;
    }
    if (threadIdx.x == 0 && lw == nwg - 1) {
        uint64_t h = fin;
        const unsigned tail = unsigned(len & 7u);
        if (tail) {
            h ^= low_bytes(ldu64(bytes + o + 8 * nb), tail);
            h *= m;
        }
        h ^= h >> 47;
        h *= m;
        h ^= h >> 47;
        out_h[which[e]] = h;
    }
}

// ---- oversized buckets: a record replies 1 iff rho > R0 and it is the
// earliest record of its slot with a rho >= its own; the workgroup builds the
// table (slot, rho) -> min seq (LDS open addressing, SK_BIG_PROBE slots, then
// a global table of 2*cnt entries carved from a per-batch arena) and answers
// from it.  The slot's last prefix maximum (max rho, its earliest record)
// stores the register: one writer per slot.
#define SK_BIG_LDS 4096
#define SK_BIG_PROBE 32
#define SK_BIG_EMPTY 0xffffffffffffffffull
__device__ __forceinline__ uint32_t big_hash(uint64_t key) {
    return uint32_t((key * 0x9E3779B97F4A7C15ull) >> 32);
}
__device__ __forceinline__ uint32_t gload_u32(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long gload_u64(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct BigTable {
    unsigned long long *lk; // LDS keys
    uint32_t *lv;           // LDS min seq
    unsigned long long *gk; // global keys
    uint32_t *gv;
    uint32_t S;
    uint32_t L = SK_BIG_LDS; // LDS slots (power of two)

    __device__ void insert(uint64_t key, uint32_t seq) const {
        uint32_t h = big_hash(key);
        for (uint32_t p = 0; p < SK_BIG_PROBE; p++) {
            uint32_t s = (h + p) & (L - 1);
            unsigned long long k = lk[s];
            if (k == SK_BIG_EMPTY) k = atomicCAS(&lk[s], SK_BIG_EMPTY, (unsigned long long)key);
            if (k == SK_BIG_EMPTY || k == key) {
                atomicMin(&lv[s], seq);
                return;
            }
        }
        for (uint32_t s = h % S;; s = s + 1 == S ? 0 : s + 1) { // S >= 2 x distinct keys: terminates
            unsigned long long k = atomicCAS(&gk[s], SK_BIG_EMPTY, (unsigned long long)key);
            if (k == SK_BIG_EMPTY || k == key) {
                atomicMin(&gv[s], seq);
                return;
            }
        }
    }
    // min seq of key, or 0xffffffff if absent (after the insert phase's barrier)
    __device__ uint32_t find(uint64_t key) const {
        uint32_t h = big_hash(key);
        for (uint32_t p = 0; p < SK_BIG_PROBE; p++) {
            uint32_t s = (h + p) & (L - 1);
            unsigned long long k = lk[s];
            if (k == key) return lv[s];
            if (k == SK_BIG_EMPTY) return 0xffffffffu; // slots only fill: the key was never inserted
        }
        for (uint32_t s = h % S;; s = s + 1 == S ? 0 : s + 1) {
            unsigned long long k = gload_u64(&gk[s]);
            if (k == key) return gload_u32(&gv[s]);
            if (k == SK_BIG_EMPTY) return 0xffffffffu;
        }
    }
};

// this thread's records: seg[t0], seg[t0 + 4], ... below seg_cnt; cnt = the bucket's total
// register rises for the HLL string writer (sk_hll_exact_strings): the record of every element that raised its
// register, in no particular order (the host sorts by seq)
__device__ __forceinline__ void pfp_event(uint64_t *ev, uint32_t *ev_n, uint64_t rec) {
    if (ev) ev[atomicAdd(ev_n, 1u)] = rec;
}

__device__ void pfp_big_resolve(const uint64_t *seg, uint32_t t0, uint32_t seg_cnt, uint32_t cnt, void *smem,
                                uint32_t *big_alloc, uint64_t *big_keys, uint32_t *big_vals, uint8_t *arena,
                                uint8_t *__restrict__ rep_seg, uint8_t *__restrict__ changed, uint64_t *ev,
                                uint32_t *ev_n) {
    __shared__ uint32_t gbase;
    unsigned long long *lk = reinterpret_cast<unsigned long long *>(smem);
    uint32_t *lv = reinterpret_cast<uint32_t *>(lk + SK_BIG_LDS);
    if (threadIdx.x == 0) gbase = atomicAdd(big_alloc, 2 * cnt);
    for (uint32_t s = threadIdx.x; s < SK_BIG_LDS; s += blockDim.x) lk[s] = SK_BIG_EMPTY, lv[s] = 0xffffffffu;
    __syncthreads();
    BigTable T{lk, lv, reinterpret_cast<unsigned long long *>(big_keys) + gbase, big_vals + gbase, 2 * cnt};
    for (uint32_t s = threadIdx.x; s < T.S; s += blockDim.x) T.gk[s] = SK_BIG_EMPTY, T.gv[s] = 0xffffffffu;
    __threadfence();
    __syncthreads();
    for (uint32_t t = t0; t < seg_cnt; t += SK_PFQ_TPS) {
        uint64_t r = seg[t];
        T.insert(((r >> 26) << 6) | (r & 63u), uint32_t((r >> 6) & 0xfffffu));
    }
    __threadfence();
    __syncthreads();
    for (uint32_t t = t0; t < seg_cnt; t += SK_PFQ_TPS) { // replies (the arena is only read)
        uint64_t r = seg[t], slot = r >> 26;
        uint32_t rho = uint32_t(r & 63u), seq = uint32_t((r >> 6) & 0xfffffu);
        bool first = rho > reg_get(slab_at(arena, slot >> 14), uint32_t(slot) & 16383u);
        // v = rho: no earlier equal rho; v > rho: no earlier larger one
        for (uint32_t v = rho; v < 52 && first; v++) first = T.find((slot << 6) | v) >= seq;
        if (first) pfp_event(ev, ev_n, r);
        if (changed) changed[seq] = first ? 1 : 0;
        else rep_seg[t] = first ? 1 : 0;
    }
    __syncthreads();
    for (uint32_t t = t0; t < seg_cnt; t += SK_PFQ_TPS) { // the slot's writer
        uint64_t r = seg[t], slot = r >> 26;
        uint32_t rho = uint32_t(r & 63u), seq = uint32_t((r >> 6) & 0xfffffu);
        if (T.find((slot << 6) | rho) != seq) continue;
        bool top = true;
        for (uint32_t v = rho + 1; v < 52 && top; v++) top = T.find((slot << 6) | v) == 0xffffffffu;
        if (!top) continue;
        uint8_t *sl = slab_at(arena, slot >> 14);
        const uint32_t cur = reg_get(sl, uint32_t(slot) & 16383u); // this thread is the register's only writer
        if (rho > cur) reg_xor(sl, uint32_t(slot) & 16383u, cur ^ rho);
    }
}

// One workgroup per bucket.  Gather: threads 4j..4j+3 copy block j's segment
// of the bucket into LDS and load each record's register (R0) right away --
// records of one slot all live in this workgroup and the arena is written
// only after the last barrier, so every load of a slot sees its pre-batch
// value, and the R0 latency overlaps the chain building.  Then the chain walk
// gives each record the max rho of its slot's earlier records and of the
// whole slot; replies and the slot's one register store follow.
__global__ void __launch_bounds__(SK_PFP_ATPB) __attribute__((amdgpu_waves_per_eu(8))) k_pfp_apply(const uint64_t *__restrict__ chunks,
                                                           const uint32_t *__restrict__ S, uint32_t nblocks,
                                                           uint8_t *arena, uint8_t *__restrict__ rep,
                                                           uint32_t *big_alloc, uint64_t *big_keys,
                                                           uint32_t *big_vals, uint8_t *__restrict__ changed,
                                                           uint64_t *ev, uint32_t *ev_n) {
    constexpr uint32_t kSmem = SK_PFP_CAP * 8 + SK_PFP_CAP * 2 + SK_PFP_HT * 4 + SK_PFP_CAP;
    static_assert(kSmem >= SK_BIG_LDS * 12, "big-bucket table shares the LDS");
    __shared__ uint64_t smem[(kSmem + 7) / 8];
    __shared__ uint32_t wsum[SK_PFP_ATPB / 64];
    uint64_t *R = smem;
    uint16_t *nxt = reinterpret_cast<uint16_t *>(R + SK_PFP_CAP);
    uint32_t *head = reinterpret_cast<uint32_t *>(nxt + SK_PFP_CAP);
    uint8_t *r0 = reinterpret_cast<uint8_t *>(head + SK_PFP_HT);
    uint32_t b = blockIdx.x, j = threadIdx.x / SK_PFQ_TPS, sub = threadIdx.x % SK_PFQ_TPS;
    uint32_t lo = 0, c = 0;
    if (j < nblocks) {
        lo = S[uint64_t(b) * nblocks + j];
        c = S[uint64_t(b + 1) * nblocks + j] - lo;
    }
    uint32_t cnt;
    uint32_t dst = block_exscan<SK_PFP_ATPB>(sub ? 0u : c, wsum, &cnt);
    dst = __shfl(dst, int((threadIdx.x & 63u) & ~(SK_PFQ_TPS - 1u))); // the group's start (from its sub 0 lane)
    if (cnt == 0) return; // uniform
    const uint64_t *seg = chunks + uint64_t(j) * SK_PFQ_EPB + lo;
    if (cnt > SK_PFP_CAP) {
        pfp_big_resolve(seg, sub, c, cnt, smem, big_alloc, big_keys, big_vals, arena,
                        rep + uint64_t(j) * SK_PFQ_EPB + lo, changed, ev, ev_n);
        return;
    }
    for (uint32_t t = threadIdx.x; t < SK_PFP_HT; t += SK_PFP_ATPB) head[t] = 0xffffu;
    uint32_t t = sub;
    for (; t + SK_PFQ_TPS < c; t += 2 * SK_PFQ_TPS) { // two records per step: both loads, then both register loads
        uint64_t ra = seg[t], rb = seg[t + SK_PFQ_TPS];
        const uint32_t va = reg_get(slab_at(arena, ra >> 40), uint32_t(ra >> 26) & 16383u);
        const uint32_t vb = reg_get(slab_at(arena, rb >> 40), uint32_t(rb >> 26) & 16383u);
        R[dst + t] = ra;
        R[dst + t + SK_PFQ_TPS] = rb;
        r0[dst + t] = uint8_t(va);
        r0[dst + t + SK_PFQ_TPS] = uint8_t(vb);
    }
    if (t < c) {
        uint64_t ra = seg[t];
        R[dst + t] = ra;
        r0[dst + t] = uint8_t(reg_get(slab_at(arena, ra >> 40), uint32_t(ra >> 26) & 16383u));
    }
    __syncthreads();
    for (uint32_t u = threadIdx.x; u < cnt; u += SK_PFP_ATPB)
        nxt[u] = uint16_t(atomicExch(&head[pfp_ht(R[u] >> 26)], u));
    __syncthreads();
    constexpr int PER = SK_PFP_CAP / SK_PFP_ATPB;
    uint64_t wslot[PER];
    uint32_t wx[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        wx[q] = 0;
        wslot[q] = 0;
        uint32_t tq = threadIdx.x + q * SK_PFP_ATPB;
        if (tq >= cnt) continue;
        uint64_t rt = R[tq], slot = rt >> 26, seq = (rt >> 6) & 0xfffffu;
        uint32_t rho = uint32_t(rt & 63u);
        uint32_t p = 0, m = rho;
        bool earliest = true;
        for (uint32_t u = head[pfp_ht(slot)]; u != 0xffffu; u = nxt[u]) {
            uint64_t ru = R[u];
            if ((ru >> 26) != slot) continue;
            uint32_t rhou = uint32_t(ru & 63u);
            uint64_t sequ = (ru >> 6) & 0xfffffu;
            m = rhou > m ? rhou : m;
            if (sequ < seq) {
                p = rhou > p ? rhou : p;
                earliest = false;
            }
        }
        uint32_t R0 = r0[tq];
        uint8_t reply = rho > (R0 > p ? R0 : p);
        if (reply) pfp_event(ev, ev_n, rt);
        if (changed) changed[seq] = reply; // one element per command: straight to batch order
        else r0[tq] = reply;               // the reply replaces R0 (read by this thread only)
        if (earliest && m > R0) {          // the slot's one writer: register R0 -> m
            wslot[q] = slot;
            wx[q] = R0 ^ m;
        }
    }
    // the slots' writes: device-scope XORs on the fields' words (neighbouring slots share words; XORs commute).
    // Merging them per word in LDS and storing whole words was slower: apply 82.8 vs 74.1 us per 1 M (C2, one RBatch
    // per call, profiles/r06_ab/r06k_ab_*)
#pragma unroll
    for (int q = 0; q < PER; q++)
        if (wx[q]) reg_xor(slab_at(arena, wslot[q] >> 14), uint32_t(wslot[q]) & 16383u, wx[q]);
    if (changed) return;
    __syncthreads();
    uint8_t *rs = rep + uint64_t(j) * SK_PFQ_EPB + lo; // replies as runs, in the chunk's order
    for (uint32_t u = sub; u < c; u += SK_PFQ_TPS) rs[u] = r0[dst + u];
}

// ---------------------------------------------------------------- PFADD, line schedule (group apply)
// For a large device batch (many RBatches of one-element commands group-committed into one call, up to 2^26
// elements) registers are applied sketch-major with the registers held in LDS, instead of one random register
// line read and written per element:
//   k_pfl_hash     as k_pfp_hash, 128 coarse buckets: bucket b holds line (b - rot(s)) & 127 of every sketch s
//   k_pfl_tot      records per region = (coarse bucket b, tile of tb hash blocks), from the hash blocks' segments
//   k_pfl_region   one workgroup per region: its segments into registers, counting-sorted in LDS by fine bucket
//                  (b, p >> sh), written back as ONE contiguous region of rec2 (tile-major runs: region (b, t) holds
//                  the runs (b, t, fine bucket) back to back) plus the region's fine-bucket starts C2[region][sub]
//                  rec2 = slab_low << 46 | reg << 32 | rho << 26 | seq (26 bits), stored as 6 B (PflRec)
//   k_pfl_fill     replies pre-filled with the call's default (the majority reply of the previous call)
//   k_pfl_apply    one workgroup per fine bucket: its 2^sh lines (one per sketch, 16 KiB) into LDS with its
//                  records (one run per tile), the records chained per register in LDS, the sequential replies (rho
//                  beats the register and every earlier rho of it; only replies != the default are stored), the
//                  lines that changed stored back.
// A region's records are binomial in the register index whatever the key skew (a sketch's 128 lines sit in 128
// distinct coarse buckets), so at tb = 448 blocks (~14.3 k records) a region fits LDS; only a region swollen by one
// element repeated thousands of times takes the two-pass streaming path.  The region layout replaces a global
// count pass + scan + a scatter of partial-line pieces (0.77 ms per 64 M, r02) with one read and one contiguous
// write of the records.
// Runs are in tile order and tiles in batch order, so a fine bucket larger than one chunk is applied in chunks of
// whole runs with the LDS registers carried over; a single run larger than a chunk is resolved with the (slot,
// rho) -> min seq table of pfp_big_resolve, against the LDS registers.
#ifndef SK_PFL_SH
#define SK_PFL_SH 7        // largest fine bucket = 2^SH sketches (128 lines of 128 B = 16 KiB of registers); a call
                           // uses sh <= SH sketches per fine bucket, sized so a fine bucket expects <= ~768 records
#endif
#ifndef SK_PFL_EXP
#define SK_PFL_EXP 600     // records a fine bucket is sized to expect (one chunk of SK_PFL_CAP with margin)
#endif
#define SK_PFL_TILE 448    // hash blocks per run tile (default; SK_PFL_TILE): ~14.3 k records per region
#define SK_PFL_RTPB 1024   // region threads: one hash-block segment each
#ifndef SK_PFL_RPER
#define SK_PFL_RPER 16     // records per region thread held in registers
#endif
#define SK_PFL_RCAP (SK_PFL_RTPB * SK_PFL_RPER) // most records of a one-piece region
#ifndef SK_PFL_ATPB
#define SK_PFL_ATPB 256    // apply threads (five apply workgroups per CU)
#endif
#ifndef SK_PFL_CAP
#define SK_PFL_CAP 768     // records per apply chunk (a fine bucket expects <= ~600: six apply workgroups per CU)
#endif
#ifndef SK_PFL_HT
#define SK_PFL_HT 256      // chain heads per chunk (LDS: six apply workgroups per CU)
#endif
#define SK_PFL_MAXSUB 8192 // fine buckets per coarse bucket (2^20 sketches)
#define SK_PFL_TMAX 1024   // largest run tile (hash blocks): one segment per region thread
#ifndef SK_PFL_NTMAX
#define SK_PFL_NTMAX 64    // most tiles per call (the apply's run table; 5 apply workgroups per CU need <= 32 KiB of LDS)
#endif
#ifndef SK_PFL_LDS
#define SK_PFL_LDS (160 * 1024 - 9 * 1024) // dynamic LDS of a region workgroup: records + fine-bucket counts
#endif
#ifndef SK_PFL_XORD
#define SK_PFL_XORD 8      // the apply's XCD order: fine buckets per XCD block (0: bucket-major, the round-5 order)
#endif
#ifndef SK_PFL_WFU
#define SK_PFL_WFU 4       // wave-loaded pair steps in flight per thread
#endif
#ifndef SK_PFL_WAVELD
#define SK_PFL_WAVELD 1    // the apply's big runs: a wave's packed pairs as three coalesced word loads + ds_bpermute
#endif
#ifndef SK_PFL_R6
#define SK_PFL_R6 2        // rec2 as 6-B records packed back to back (0: u64)
#endif
// rec2 record slot i.  The region pass writes the records sorted; the apply reads them back as the u64
// slab_low << 46 | reg << 32 | rho << 26 | seq, with reg's line bits zero in the 6-B forms (a fine bucket holds one
// line of each of its sketches, so slab_low and the register's place in its line name the register): lo = the low
// 32 bits, hi = slab_low << 7 | register in its line.  The buffer holds u64[cap] in every form.
//   2: record i at bytes [6i, 6i + 6): lo then hi for even i, hi then lo for odd i, so both are aligned loads and
//      a fine bucket's run (~16 records) spans as few 128-B lines as its 96 bytes allow;
//   (a u32 plane and a u16 plane instead, tried first: a run then touches lines of both planes, and r05req counted
//   17 % more read requests in the apply than with u64 records; packed, 4 % fewer.)
struct PflRec {
    uint64_t *p;
    uint64_t cap; // records the buffer holds (the call's hash blocks x SK_PFP_EPB)
    __device__ __forceinline__ void put(uint64_t i, uint64_t r) const {
        const uint32_t lo = uint32_t(r);
        const uint16_t hi = uint16_t((uint32_t(r >> 46) << SK_PFL_LB) | (uint32_t(r >> 32) & ((1u << SK_PFL_LB) - 1)));
        if (SK_PFL_R6 == 2) {
            const uint64_t odd = i & 1u;
            reinterpret_cast<uint32_t *>(p)[(3 * i + odd) >> 1] = lo;
            reinterpret_cast<uint16_t *>(p)[3 * i + 2 * (1 - odd)] = hi;
        } else {
            p[i] = r;
        }
    }
    // SK_PFL_R6 == 2: records 2P and 2P + 1 as three whole words (lo, hi | hi' << 16, lo')
    __device__ __forceinline__ void put_pair(uint64_t P, uint64_t r0, uint64_t r1) const {
        auto hi = [](uint64_t r) {
            return (uint32_t(r >> 46) << SK_PFL_LB) | (uint32_t(r >> 32) & ((1u << SK_PFL_LB) - 1));
        };
        uint32_t *w = reinterpret_cast<uint32_t *>(p) + 3 * P;
        w[0] = uint32_t(r0);
        w[1] = hi(r0) | (hi(r1) << 16);
        w[2] = uint32_t(r1);
    }
    // records 2P and 2P + 1
    __device__ __forceinline__ void get_pair(uint32_t P, uint64_t *r0, uint64_t *r1) const { // slots < 2^26
        if (SK_PFL_R6 == 2) {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(p) + 3 * P;
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
            *r0 = unpack(w0, w1 & 0xffffu);
            *r1 = unpack(w2, w1 >> 16);
        } else {
            *r0 = p[2 * P];
            *r1 = p[2 * P + 1];
        }
    }
    __device__ __forceinline__ static uint64_t unpack(uint32_t lo, uint32_t hi) {
        return (uint64_t(hi >> SK_PFL_LB) << 46) | (uint64_t(hi & ((1u << SK_PFL_LB) - 1)) << 32) | lo;
    }
    __device__ __forceinline__ uint64_t get(uint64_t i) const {
        uint32_t lo, hi;
        if (SK_PFL_R6 == 2) {
            const uint64_t odd = i & 1u;
            lo = reinterpret_cast<const uint32_t *>(p)[(3 * i + odd) >> 1];
            hi = reinterpret_cast<const uint16_t *>(p)[3 * i + 2 * (1 - odd)];
        } else {
            return p[i];
        }
        return unpack(lo, hi);
    }
};
static_assert(SK_PFL_SH + SK_PFL_LB <= 16, "6-B records: slab_low and the register in its line fit 16 bits");
__device__ __forceinline__ uint32_t pfl_ht(uint64_t key) {
    static_assert((SK_PFL_HT & (SK_PFL_HT - 1)) == 0, "power-of-two chain heads");
    return uint32_t((key * 0xC2B2AE3D27D4EB4Full) >> (64 - __builtin_ctz(SK_PFL_HT)));
}

// Fine buckets take sketches by a permuted slab id, p = slab * pa mod 2^pk (pa odd, a bijection): slabs are
// handed out in key-creation order, so consecutive slabs -- a batch of tenants created together, the head of a
// Zipf key space -- would otherwise share fine buckets and pile their records onto a few workgroups.
struct PflPerm {
    uint32_t pa, pai, mask; // multiplier, its inverse mod 2^pk, 2^pk - 1
    uint32_t nslab;         // slab ids >= nslab (never handed out) are dropped, their replies 0
    __device__ __forceinline__ uint32_t fwd(uint32_t slab) const { return (slab * pa) & mask; }
    __device__ __forceinline__ uint32_t inv(uint32_t p) const { return (p * pai) & mask; }
};

// records of region (b, t) = sum over the tile's blocks of segment b's length; grid (ntile, 128)
__global__ void __launch_bounds__(256) k_pfl_tot(const uint32_t *__restrict__ S, uint32_t nblk, uint32_t tb,
                                                 uint32_t ntile, uint32_t *__restrict__ tot) {
    __shared__ uint32_t wsum[256 / 64];
    const uint32_t t = blockIdx.x, b = blockIdx.y, b0 = t * tb, b1 = b0 + tb < nblk ? b0 + tb : nblk;
    uint32_t s = 0;
    for (uint32_t blk = b0 + threadIdx.x; blk < b1; blk += 256)
        s += S[uint64_t(b + 1) * nblk + blk] - S[uint64_t(b) * nblk + blk];
    uint32_t total;
    block_exscan<256>(s, wsum, &total);
    if (threadIdx.x == 0) tot[b * ntile + t] = total;
}

// The region's record x: segment lo with segp[lo] <= x < segp[lo + 1] (binary search over the tile's prefix)
__device__ __forceinline__ uint64_t pfl_region_rec(const PflChunk chunks, const uint32_t *segp,
                                                   const uint32_t *segs, uint32_t nb, uint32_t b0, uint32_t x,
                                                   uint32_t *blk) {
    uint32_t lo = 0, hi = nb;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (segp[mid] <= x) lo = mid;
        else hi = mid;
    }
    *blk = b0 + lo;
    return chunks.get(uint64_t(b0 + lo) * SK_PFP_EPB + segs[lo] + (x - segp[lo]));
}

// One workgroup per region g = b * ntile + t.  Dynamic LDS: cap records (u64) + nsub + 1 counts.
// Outputs: rbase[g] (the region's first rec2 slot), C2[g][0..nsub] (exclusive starts of the fine buckets' runs
// inside the region, [nsub] = records kept), rec2[rbase + ...] the runs; dropped records (slab >= nslab) reply 0.
#ifndef SK_PFL_RWPE
#define SK_PFL_RWPE 4      // region waves per SIMD the register budget is sized for (one 1024-thread workgroup per CU)
#endif
__global__ void __launch_bounds__(SK_PFL_RTPB) __attribute__((amdgpu_waves_per_eu(SK_PFL_RWPE))) k_pfl_region(const PflChunk chunks,
                                                            const uint32_t *__restrict__ S, uint32_t nblk, uint32_t tb,
                                                            uint32_t ntile, uint32_t nsub, uint32_t sh, PflPerm pm,
                                                            uint32_t cap, const uint32_t *__restrict__ tot,
                                                            uint32_t *__restrict__ rbase, uint32_t *__restrict__ C2,
                                                            PflRec rec2,
                                                            uint8_t *__restrict__ changed, int probe) {
    extern __shared__ uint64_t dyn64[];
    uint64_t *sorted = dyn64;
    uint32_t *hist = reinterpret_cast<uint32_t *>(dyn64 + cap);
    __shared__ uint32_t segp[SK_PFL_TMAX + 1], segs[SK_PFL_TMAX];
    __shared__ uint32_t wsum[SK_PFL_RTPB / 64];
    const uint32_t tid = threadIdx.x, g = blockIdx.x, b = g / ntile, t = g % ntile;
    const uint32_t b0 = t * tb, nb = (b0 + tb < nblk ? b0 + tb : nblk) - b0;
    // the segment table loads first (independent of the region base below)
    uint32_t st = 0, len = 0;
    if (tid < nb) {
        st = S[uint64_t(b) * nblk + b0 + tid];
        len = S[uint64_t(b + 1) * nblk + b0 + tid] - st;
    }
    // this region's base: the records of every region before it (b-major, tile minor)
    uint32_t acc = 0;
    for (uint32_t i = tid; i < g; i += SK_PFL_RTPB) acc += tot[i];
    uint32_t base;
    block_exscan<SK_PFL_RTPB>(acc, wsum, &base);
    if (tid < nb) segs[tid] = st;
    uint32_t m;
    const uint32_t ex = block_exscan<SK_PFL_RTPB>(len, wsum, &m);
    if (tid < nb) segp[tid] = ex;
    for (uint32_t x = tid; x <= nsub; x += SK_PFL_RTPB) hist[x] = 0;
    if (tid == 0) {
        segp[nb] = m;
        rbase[g] = base;
    }
    __syncthreads();
    uint32_t *C = C2 + uint64_t(g) * (nsub + 1);
    // a record of the region -> its rec2 value (fine bucket in sub), or ~0 for a dropped record
    auto conv = [&](uint64_t rr, uint32_t blk, uint32_t *sub) -> uint64_t {
        const uint32_t seq = blk * SK_PFP_EPB + uint32_t(rr & 4095u);
        if (uint32_t(rr >> 32) >= pm.nslab) { // ids beyond the store's slabs are dropped
            if (changed) changed[seq] = 0;
            return ~0ull;
        }
        const uint32_t slab = pm.fwd(uint32_t(rr >> 32)), reg = uint32_t(rr >> 18) & 16383u,
                       rho = uint32_t(rr >> 12) & 63u;
        *sub = slab >> sh;
        return (uint64_t(slab & ((1u << sh) - 1)) << 46) | (uint64_t(reg) << 32) | (uint64_t(rho) << 26) | seq;
    };
    // exclusive scan of hist[0..nsub) in place (nsub <= 8 per thread), hist[nsub] = total; also written to C
    auto scan_hist = [&]() {
        constexpr int HP = SK_PFL_MAXSUB / SK_PFL_RTPB;
        uint32_t v[HP], s = 0;
#pragma unroll
        for (int q = 0; q < HP; q++) {
            const uint32_t x = tid * HP + q;
            v[q] = x < nsub ? hist[x] : 0u;
            s += v[q];
        }
        uint32_t total;
        uint32_t e = block_exscan<SK_PFL_RTPB>(s, wsum, &total);
#pragma unroll
        for (int q = 0; q < HP; q++) {
            const uint32_t x = tid * HP + q;
            if (x < nsub) {
                hist[x] = e;
                C[x] = e;
            }
            e += v[q];
        }
        if (tid == 0) {
            hist[nsub] = total;
            C[nsub] = total;
        }
        __syncthreads();
    };
    if (m <= cap) { // one piece: every record in registers, ranked by its fine bucket, placed in LDS, written out
        // each record's segment from a u16 map in the (still free) sort area: one LDS read instead of a binary
        // search over the tile's segments
        static_assert(SK_PFL_TMAX <= 65536, "seg_of: u16 segment numbers");
        uint16_t *seg_of = reinterpret_cast<uint16_t *>(sorted); // m <= cap records: 2 m of the 8 cap bytes
        if (tid < nb)
            for (uint32_t u = ex; u < ex + len; u++) seg_of[u] = uint16_t(tid);
        __syncthreads();
        uint64_t r[SK_PFL_RPER];
        uint32_t rk[SK_PFL_RPER];
#pragma unroll
        for (int q = 0; q < SK_PFL_RPER; q++) {
            const uint32_t x = tid + q * SK_PFL_RTPB;
            r[q] = ~0ull;
            if (x < m) {
                if (probe & 2048) { // dev ablation: no record loads (a record of block b0, timing only)
                    r[q] = (uint64_t(x % pm.nslab) << 32) | (uint64_t(x & 16383) << 18) | (1u << 12) | (x & 4095);
                    rk[q] = b0;
                    continue;
                }
                const uint32_t lo = seg_of[x];
                r[q] = chunks.get(uint64_t(b0 + lo) * SK_PFP_EPB + segs[lo] + (x - segp[lo]));
                rk[q] = b0 + lo;
            }
        }
#pragma unroll
        for (int q = 0; q < SK_PFL_RPER; q++) {
            if (r[q] == ~0ull) continue;
            uint32_t sub = 0;
            r[q] = conv(r[q], rk[q], &sub);
            if (r[q] != ~0ull) rk[q] = atomicAdd(&hist[sub], 1u) | (sub << 14);
        }
        __syncthreads();
        scan_hist();
#pragma unroll
        for (int q = 0; q < SK_PFL_RPER; q++)
            if (r[q] != ~0ull) sorted[hist[rk[q] >> 14] + (rk[q] & 16383u)] = r[q];
        __syncthreads();
        const uint32_t kept = hist[nsub];
        if (probe & 1024) return; // dev ablation: no write-out
        if (SK_PFL_R6 != 2) {
            for (uint32_t i = tid; i < kept; i += SK_PFL_RTPB) rec2.put(base + i, sorted[i]);
            return;
        }
        // packed records: whole pairs as three words each; an odd first or last record alone (its pair is shared
        // with the neighbouring region)
        const uint64_t a = base, e = uint64_t(base) + kept, a2 = a + (a & 1u), e2 = e - (e & 1u);
        if (kept && (a & 1u) && tid == 0) rec2.put(a, sorted[0]);
        if (kept && (e & 1u) && e - 1 >= a2 && tid == 1) rec2.put(e - 1, sorted[e - 1 - a]);
        for (uint64_t P = a2 / 2 + tid; P < e2 / 2; P += SK_PFL_RTPB)
            rec2.put_pair(P, sorted[2 * P - a], sorted[2 * P + 1 - a]);
        return;
    }
    // swollen region (one element repeated in many blocks): count every piece, then place every piece; the runs
    // keep piece (= batch) order
    for (uint32_t p0 = 0; p0 < m; p0 += cap) {
#pragma unroll 4
        for (int q = 0; q < SK_PFL_RPER; q++) {
            const uint32_t x = p0 + tid + q * SK_PFL_RTPB;
            if (x >= m || x - p0 >= cap) continue;
            uint32_t blk, sub = 0;
            const uint64_t rr = conv(pfl_region_rec(chunks, segp, segs, nb, b0, x, &blk), blk, &sub);
            if (rr != ~0ull) atomicAdd(&hist[sub], 1u);
        }
    }
    __syncthreads();
    scan_hist();
    uint32_t *lcnt = reinterpret_cast<uint32_t *>(sorted); // cap * 8 >= nsub * 4 bytes
    for (uint32_t x = tid; x < nsub; x += SK_PFL_RTPB) lcnt[x] = 0;
    __syncthreads();
    for (uint32_t p0 = 0; p0 < m; p0 += cap) {
#pragma unroll 4
        for (int q = 0; q < SK_PFL_RPER; q++) {
            const uint32_t x = p0 + tid + q * SK_PFL_RTPB;
            if (x >= m || x - p0 >= cap) continue;
            uint32_t blk, sub = 0;
            const uint64_t rr = conv(pfl_region_rec(chunks, segp, segs, nb, b0, x, &blk), blk, &sub);
            if (rr != ~0ull) rec2.put(base + hist[sub] + atomicAdd(&lcnt[sub], 1u), rr);
        }
        __syncthreads();
        for (uint32_t x = tid; x < nsub; x += SK_PFL_RTPB) {
            hist[x] += lcnt[x];
            lcnt[x] = 0;
        }
        __syncthreads();
    }
}

// Reply default: the apply stores only replies that differ from it, after k_pfl_fill wrote it everywhere.  It is
// the majority reply of the previous call, from counters a sample of apply workgroups (1 in 16) kept: rc[16 p ..
// 16 p + 8) ones and [16 p + 8, 16 p + 16) replies, parity p alternating per call (this call reads p and fills
// p ^ 1, which its fill zeroed).
__device__ __forceinline__ uint32_t pfl_dflt(const uint32_t *rc, uint32_t p) {
    uint32_t ones = 0, all = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        ones += rc[16 * p + i];
        all += rc[16 * p + 8 + i];
    }
    return 2 * ones > all ? 1u : 0u;
}
__global__ void __launch_bounds__(256) k_pfl_fill(uint8_t *__restrict__ changed, uint64_t n, uint32_t *rc,
                                                  uint32_t p) {
    const uint32_t v = pfl_dflt(rc, p) * 0x01010101u;
    if (blockIdx.x == 0 && threadIdx.x < 16) rc[16 * (p ^ 1) + threadIdx.x] = 0;
    const uint64_t a = (16 - (reinterpret_cast<uintptr_t>(changed) & 15)) & 15; // bytes before the first 16-B word
    const uint64_t head = a < n ? a : n, nv = (n - head) >> 4;
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x, stride = uint64_t(gridDim.x) * 256;
    uint4 *w = reinterpret_cast<uint4 *>(changed + head);
    for (uint64_t j = i; j < nv; j += stride) w[j] = make_uint4(v, v, v, v);
    if (i < head) changed[i] = uint8_t(v);
    if (i < ((n - head) & 15)) changed[head + nv * 16 + i] = uint8_t(v);
}

#ifndef SK_PFL_DG
#define SK_PFL_DG 1        // 16-B words per dirty flag: the apply stores back the 16-B pieces of its lines that changed
#endif
#define PFL_DWORDS ((16384 / 16 / SK_PFL_DG + 31) / 32)
// The apply's lines stay packed in LDS (Redis's layout, 24 words per 128-register line, line i at word 24 i): a
// chunk touches ~600 of the 16384 registers it holds, so reading and writing those fields costs less than unpacking
// every line to bytes and packing the changed ones back.  Register slotb = line << 7 | register-in-line.
__device__ __forceinline__ uint32_t lds_reg_get(const uint32_t *lw, uint32_t slotb) {
    const uint32_t bit = 6u * (slotb & 127u), w = (slotb >> 7) * 24u + (bit >> 5), sh = bit & 31u;
    uint32_t v = lw[w] >> sh;
    if (sh > 26u) v |= lw[w + 1] << (32u - sh);
    return v & 63u;
}
// field slotb from `old` to old ^ x (LDS XORs: neighbours of the same words may change at the same time)
__device__ __forceinline__ void lds_reg_xor(uint32_t *lw, uint32_t slotb, uint32_t x) {
    const uint32_t bit = 6u * (slotb & 127u), w = (slotb >> 7) * 24u + (bit >> 5), sh = bit & 31u;
    atomicXor(&lw[w], x << sh);
    if (sh > 26u) atomicXor(&lw[w + 1], x >> (32u - sh));
}
__device__ __forceinline__ void pfl_mark(uint32_t *dirty, uint32_t slotb) { // register slotb of the LDS lines changed
    const uint32_t piece = slotb / (16 * SK_PFL_DG);
    atomicOr(&dirty[piece >> 5], 1u << (piece & 31u));
}

// one chunk of records R[0..cnt) (every record of its registers with a smaller seq is in this chunk or was
// applied to `reg` before): chains per register, sequential replies, final register values into `reg` (LDS).
// Caller syncs before (R loaded, heads cleared) and after; `fill` runs between the chain build and the walk (the
// caller's register lines, loaded into registers before, go to LDS while the chains are built).  `put` stores a
// reply (only those that differ from the call's default when the replies were pre-filled).
template <class Fill, class Put>
__device__ __forceinline__ void pfl_chunk(const uint64_t *R, uint32_t cnt, uint16_t *nxt, uint32_t *head,
                                          uint8_t *fin, uint32_t *lw, uint32_t *dirty, Fill fill, Put put) {
    for (uint32_t u = threadIdx.x; u < cnt; u += SK_PFL_ATPB)
        nxt[u] = uint16_t(atomicExch(&head[pfl_ht(R[u] >> 32)], u));
    fill();
    __syncthreads();
    for (uint32_t u = threadIdx.x; u < cnt; u += SK_PFL_ATPB) {
        const uint64_t rt = R[u], key = rt >> 32, seq = rt & 0x3ffffffu;
        const uint32_t rho = uint32_t(rt >> 26) & 63u;
        uint32_t p = 0, m = rho;
        bool earliest = true;
        for (uint32_t w = head[pfl_ht(key)]; w != 0xffffu; w = nxt[w]) {
            const uint64_t rw = R[w];
            if ((rw >> 32) != key) continue;
            const uint32_t rhow = uint32_t(rw >> 26) & 63u;
            m = rhow > m ? rhow : m;
            if ((rw & 0x3ffffffu) < seq) {
                p = rhow > p ? rhow : p;
                earliest = false;
            }
        }
        const uint32_t slotb = pfl_slotb(key);
        const uint32_t R0 = lds_reg_get(lw, slotb);
        put(uint32_t(seq), uint32_t(rho > (R0 > p ? R0 : p)));
        fin[u] = earliest && m > R0 ? uint8_t(m ^ R0) : uint8_t(0); // the register's change, as an XOR
    }
    __syncthreads();
    for (uint32_t u = threadIdx.x; u < cnt; u += SK_PFL_ATPB)
        if (fin[u]) {
            const uint32_t slotb = pfl_slotb(R[u] >> 32);
            lds_reg_xor(lw, slotb, fin[u]);
            pfl_mark(dirty, slotb);
        }
}

// Heavy fine buckets first: the apply's grid starts with hmax "heavy slots"; the plan lists the fine buckets of more
// than one chunk (C1, a Zipf head's lines -- they run longest) in order[0..H), H = ctr[0], and heavy slot k applies
// order[k].  The rest of the grid is the fine buckets in their own order; a heavy one there exits at once.  A
// uniform call has H = 0: its heavy slots exit and nothing else is indirected.
__global__ void __launch_bounds__(256) k_pfl_plan(const uint32_t *__restrict__ C2, uint32_t ntile, uint32_t nsub,
                                                  uint32_t nf, uint32_t hmax, uint32_t *ctr,
                                                  uint32_t *__restrict__ order) {
    __shared__ uint32_t wsum[256 / 64], base;
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    uint32_t cnt = 0;
    if (f < nf) {
        const uint32_t b = f / nsub, sub = f % nsub;
        for (uint32_t t = 0; t < ntile; t++) {
            const uint32_t *c = C2 + uint64_t(b * ntile + t) * (nsub + 1) + sub;
            cnt += c[1] - c[0];
        }
    }
    const bool heavy = cnt > SK_PFL_CAP;
    uint32_t th;
    const uint32_t ph = block_exscan<256>(heavy ? 1u : 0u, wsum, &th);
    if (threadIdx.x == 0) base = th ? atomicAdd(ctr, th) : 0u;
    __syncthreads();
    if (heavy && base + ph < hmax) order[base + ph] = f; // hmax bounds the heavy buckets (n / (CAP + 1))
}

#ifndef SK_PFL_AWPE
#define SK_PFL_AWPE 6      // apply waves per SIMD the register budget allows (6: <= 80 VGPRs; 7 needs <= 72)
#endif
__global__ void __launch_bounds__(SK_PFL_ATPB) __attribute__((amdgpu_waves_per_eu(SK_PFL_AWPE))) k_pfl_apply(const PflRec rec2,
                                                           const uint32_t *__restrict__ rbase,
                                                           const uint32_t *__restrict__ C2, uint32_t ntile,
                                                           uint32_t nsub, uint32_t sh, PflPerm pm, uint32_t nslab,
                                                           uint8_t *arena,
                                                           uint8_t *__restrict__ changed, uint32_t *big_alloc,
                                                           uint64_t *big_keys, uint32_t *big_vals, int probe,
                                                           uint32_t hmax, const uint32_t *order_n,
                                                           const uint32_t *__restrict__ order, uint32_t *rc,
                                                           uint32_t par) {
    constexpr uint32_t NL = 1u << SK_PFL_SH;
    constexpr uint32_t kWork = SK_PFL_CAP * 8 + SK_PFL_CAP * 2 + SK_PFL_HT * 4 + SK_PFL_CAP;
    constexpr uint32_t kBigL = 512;        // LDS slots of the big-run table
    static_assert(kWork >= kBigL * 12, "the big-run table shares the chunk LDS");
    constexpr uint32_t LW = (1u << SK_PFL_LB) / 16; // 16-B words per line
    __shared__ uint32_t lw[NL * 24];           // packed line of sketch slab0 + i at lw[24 i] (12-B group q at 3q)
    __shared__ uint64_t work[(kWork + 7) / 8]; // chunk records, chains, final values (or the big-run table)
    __shared__ uint32_t dirty[PFL_DWORDS]; // bit per SK_PFL_DG-word piece of the lines: changed, stored back
    __shared__ uint32_t rs[SK_PFL_NTMAX], rp[SK_PFL_NTMAX + 1]; // the fine bucket's run per tile: start, prefix
    __shared__ uint32_t wsum[SK_PFL_ATPB / 64];
    uint64_t *R = work;
    uint16_t *nxt = reinterpret_cast<uint16_t *>(R + SK_PFL_CAP);
    uint32_t *head = reinterpret_cast<uint32_t *>(nxt + SK_PFL_CAP);
    uint8_t *fin = reinterpret_cast<uint8_t *>(head + SK_PFL_HT);

    uint32_t f;
    if (blockIdx.x < hmax) { // a heavy slot
        if (blockIdx.x >= order_n[0]) return; // uniform
        f = order[blockIdx.x];
    } else {
        // XCD-aware order (hmax is a multiple of 8, so j % 8 is the workgroup's XCD): the 128 coarse buckets of one
        // group of fine buckets run back to back on one XCD, so the 96-B packed lines of neighbouring buckets -- which
        // share 128-B cache lines for line % 4 in {1, 2} -- meet in that XCD's L2 and each cache line is read once
        const uint32_t j = blockIdx.x - hmax;
#if SK_PFL_XORD == 0
        f = j; // bucket-major: f = b * nsub + sub
        if (f >= SK_PFL_NB * nsub) return;
#else
        // XCD x takes blocks of SK_PFL_XORD consecutive fine buckets of each coarse bucket; on it, b advances every
        // SK_PFL_XORD workgroups: the block's record runs lie side by side in each region (shared record lines) and a
        // sketch's neighbouring lines come SK_PFL_XORD workgroups apart (shared packed-line lines in its L2)
        constexpr uint32_t SB = SK_PFL_XORD;
        const uint32_t x = j & 7u, jj = j >> 3, grp = jj / (SK_PFL_NB * SB), w = jj % (SK_PFL_NB * SB);
        const uint32_t sub_ = (grp * 8u + x) * SB + w % SB;
        if (sub_ >= nsub) return;
        f = (w / SB) * nsub + sub_;
#endif
    }
    const uint32_t b = f / nsub, sub = f % nsub;
    const uint32_t slab0 = sub << sh, nsl = 1u << sh; // permuted ids slab0 + i, i < nsl
    // line i of the bucket: the 96 packed bytes of registers (b - rot(s)) * 128 .. + 127 of sketch s; LDS word q of the
    // lines (16 u8 registers) <-> packed group q % LW (12 B) of line q / LW
    auto line = [&](uint32_t i) -> uint8_t * {
        const uint32_t s = pm.inv(slab0 + i);
        return slab_at(arena, s) + ((b - pfl_rot(s)) & (SK_PFL_NB - 1)) * (SK_SLAB_BYTES / SK_PFL_NB);
    };
    constexpr int LQ = (NL * LW + SK_PFL_ATPB - 1) / SK_PFL_ATPB;
    uint4 lv[LQ]; // the packed group's three words (w unused) until fill_lines unpacks them
    auto load_lines = [&] {
#pragma unroll
        for (int j = 0; j < LQ; j++) {
            const uint32_t q = threadIdx.x + j * SK_PFL_ATPB;
            if (q < nsl * LW && pm.inv(slab0 + q / LW) < nslab) {
                if (probe & 4) {
                    lv[j] = make_uint4(0, 0, 0, 0);
                } else {
                    const uint32_t *w = reinterpret_cast<const uint32_t *>(line(q / LW)) + 3 * (q % LW);
                    lv[j] = make_uint4(w[0], w[1], w[2], 0);
                }
            }
        }
    };
    uint32_t st = 0, len = 0;
    if (threadIdx.x < ntile) {
        const uint32_t g = b * ntile + threadIdx.x;
        const uint32_t *c = C2 + uint64_t(g) * (nsub + 1) + sub;
        const uint32_t c0 = c[0];
        st = rbase[g] + c0;
        len = c[1] - c0;
        rs[threadIdx.x] = st;
    }
    uint32_t cnt;
    const uint32_t ex = block_exscan<SK_PFL_ATPB>(len, wsum, &cnt);
    if (cnt == 0) return; // uniform
    if (hmax && blockIdx.x >= hmax && cnt > SK_PFL_CAP) return; // applied by a heavy slot
    if (threadIdx.x < ntile) rp[threadIdx.x] = ex;
    if (probe & 256) return; // dev ablation: run table only
    // record u of the fine bucket (u < cnt): run t with rp[t] <= u < rp[t + 1].  A one-chunk bucket reads t from
    // run_of[u] (filled below, one LDS read per record); chunked buckets search rp (fixed steps, no branches)
    static_assert(SK_PFL_NTMAX <= 128, "run_of holds u8 run numbers; 7 search steps");
    uint8_t *run_of = fin; // the records' run numbers (u < cnt), read before the chunk's walk writes fin
    auto rec_at = [&](uint32_t u) -> uint64_t {
        uint32_t lo = 0;
#pragma unroll
        for (uint32_t step = 64; step; step >>= 1)
            if (lo + step < ntile && rp[lo + step] <= u) lo += step;
        return rec2.get(rs[lo] + (u - rp[lo]));
    };
    auto rec_one = [&](uint32_t u) -> uint64_t {
        const uint32_t t = run_of[u];
        return rec2.get(rs[t] + (u - rp[t]));
    };
    if (cnt <= SK_PFL_CAP && threadIdx.x < ntile)
        for (uint32_t u = ex; u < ex + len; u++) run_of[u] = uint8_t(threadIdx.x);
    const uint32_t dflt = (probe & 32) ? pfl_dflt(rc, par) : 2u; // 2: no default, every reply stored
    const bool sample = (probe & 32) && (blockIdx.x & 15u) == 0;
    uint32_t nrep = 0, nones = 0; // replies made by this thread and how many were 1 (sampled workgroups)
    auto put = [&](uint32_t seq, uint32_t rep) {
        if (!(probe & 64) && rep != dflt) changed[seq] = uint8_t(rep); // probe & 64: dev ablation, no reply stores
        if (sample) {
            nrep++;
            nones += rep;
        }
    };
    for (uint32_t i = threadIdx.x; i < PFL_DWORDS; i += SK_PFL_ATPB) dirty[i] = 0;
    for (uint32_t t = threadIdx.x; t < SK_PFL_HT; t += SK_PFL_ATPB) head[t] = 0xffffu;
    if (threadIdx.x == 0) rp[ntile] = cnt;
    __syncthreads();
    if (cnt <= SK_PFL_CAP) { // the whole fine bucket is one chunk: records and lines in one round trip
        load_lines();
        constexpr int RU = SK_PFL_CAP / SK_PFL_ATPB; // every record load in flight at once
        uint64_t rv[RU];
#pragma unroll
        for (int q = 0; q < RU; q++) {
            const uint32_t u = q * SK_PFL_ATPB + threadIdx.x;
            if (u < cnt) rv[q] = rec_one(u);
        }
#pragma unroll
        for (int q = 0; q < RU; q++) {
            const uint32_t u = q * SK_PFL_ATPB + threadIdx.x;
            if (u < cnt) R[u] = rv[q];
        }
        auto fill_lines = [&] {
#pragma unroll
            for (int j = 0; j < LQ; j++) {
                const uint32_t q = threadIdx.x + j * SK_PFL_ATPB;
                if (q < nsl * LW && pm.inv(slab0 + q / LW) < nslab) {
                    lw[3 * q] = lv[j].x;
                    lw[3 * q + 1] = lv[j].y;
                    lw[3 * q + 2] = lv[j].z;
                }
            }
        };
        __syncthreads();
        if (probe & 128) return; // dev ablation: run table, lines and records loaded, nothing applied
        pfl_chunk(R, cnt, nxt, head, fin, lw, dirty, fill_lines, put);
    } else {
        for (uint32_t q = threadIdx.x; q < nsl * LW; q += SK_PFL_ATPB)
            if (pm.inv(slab0 + q / LW) < nslab) {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(line(q / LW)) + 3 * (q % LW);
                lw[3 * q] = w[0];
                lw[3 * q + 1] = w[1];
                lw[3 * q + 2] = w[2];
            }
        __syncthreads();
        uint32_t t0 = 0;
        while (t0 < ntile) { // uniform: chunks of whole runs, in tile (= batch) order
            const uint32_t a = rp[t0];
            uint32_t t1 = t0 + 1;
            while (t1 < ntile && rp[t1 + 1] - a <= SK_PFL_CAP) t1++;
            const uint32_t k = rp[t1] - a;
            if (k <= SK_PFL_CAP) {
                constexpr int CU = SK_PFL_CAP / SK_PFL_ATPB;
                uint64_t rr[CU];
#pragma unroll
                for (int q = 0; q < CU; q++) {
                    const uint32_t u = q * SK_PFL_ATPB + threadIdx.x;
                    if (u < k) rr[q] = rec_at(a + u);
                }
#pragma unroll
                for (int q = 0; q < CU; q++) {
                    const uint32_t u = q * SK_PFL_ATPB + threadIdx.x;
                    if (u < k) R[u] = rr[q];
                }
                __syncthreads();
                pfl_chunk(R, k, nxt, head, fin, lw, dirty, [] {}, put);
            } else { // one run larger than a chunk (t1 == t0 + 1), contiguous from rs[t0]
                const uint64_t run0 = rs[t0];
                auto run = [&](uint32_t u) -> uint64_t { return rec2.get(run0 + u); };
                // only records above their register can rise, and only they can stop a later record from rising:
                // the rest reply 0 now; the candidates are resolved as a chunk when they fit (a hot sketch whose
                // registers are already high has few), else with the (slot, rho) -> min seq table
                __shared__ uint32_t ncand;
                if (threadIdx.x == 0) ncand = 0;
                __syncthreads();
                // records in pairs (a packed pair is three aligned words: one load), FU of them in flight per
                // thread; the run's slots [run0, run0 + k) may start and end inside a pair
                constexpr int FU = SK_PFL_R6 == 2 && SK_PFL_WAVELD ? SK_PFL_WFU : 4;
                auto consider = [&](uint64_t r) { // a record of the run: a candidate, or its reply is 0 now
                    if (r == ~0ull) return;
                    const uint64_t key = r >> 32;
                    if (((r >> 26) & 63u) > lds_reg_get(lw, pfl_slotb(key))) {
                        const uint32_t i = atomicAdd(&ncand, 1u);
                        if (i < SK_PFL_CAP) R[i] = r;
                    } else {
                        put(uint32_t(r & 0x3ffffffu), 0u);
                    }
                };
                const uint32_t r0s = rs[t0], r1s = r0s + k, pe0 = r0s >> 1, pe1 = (r1s + 1) >> 1; // slots < 2^26
                for (uint32_t p0 = pe0; p0 < pe1; p0 += FU * SK_PFL_ATPB) {
#if SK_PFL_R6 == 2 && SK_PFL_WAVELD
                    // packed: each wave reads its 64 pairs (192 words) as three coalesced word loads, and every lane
                    // gathers its pair's three words from the holders (ds_bpermute)
                    const uint32_t lane = threadIdx.x & 63u;
                    uint32_t a[FU][3];
#pragma unroll
                    for (int q = 0; q < FU; q++) {
                        const uint32_t Pq = p0 + q * SK_PFL_ATPB + (threadIdx.x - lane); // the wave's first pair
                        const uint32_t lim = pe1 > Pq ? 3 * (pe1 - Pq) : 0u;             // its words in the run
                        const uint32_t *wb = reinterpret_cast<const uint32_t *>(rec2.p) + 3 * uint64_t(Pq);
#pragma unroll
                        for (int j = 0; j < 3; j++) a[q][j] = lane + 64 * j < lim ? wb[lane + 64 * j] : 0u;
                    }
#pragma unroll
                    for (int q = 0; q < FU; q++) {
                        // lane l takes the wave's records l and 64 + l (consecutive lanes, consecutive records)
                        auto take = [&](uint32_t d) -> uint32_t { // word d of the wave's 192
                            const int src = int(d & 63u) << 2;
                            const uint32_t x0 = __builtin_amdgcn_ds_bpermute(src, int(a[q][0])),
                                           x1 = __builtin_amdgcn_ds_bpermute(src, int(a[q][1])),
                                           x2 = __builtin_amdgcn_ds_bpermute(src, int(a[q][2]));
                            return d < 64 ? x0 : d < 128 ? x1 : x2;
                        };
                        const uint32_t Pq = p0 + q * SK_PFL_ATPB + (threadIdx.x - lane), odd = lane & 1u;
#pragma unroll
                        for (int m = 0; m < 2; m++) {
                            const uint32_t pr = (lane >> 1) + 32u * m;           // the record's pair in the wave
                            const uint32_t lo = take(3 * pr + 2 * odd), hw = take(3 * pr + 1);
                            const uint32_t slot = 2 * (Pq + pr) + odd;
                            if (Pq + pr < pe1 && slot >= r0s && slot < r1s)
                                consider(PflRec::unpack(lo, odd ? hw >> 16 : hw & 0xffffu));
                        }
                    }
#else
                    uint64_t rr[2 * FU];
#pragma unroll
                    for (int q = 0; q < FU; q++) {
                        const uint32_t P = p0 + q * SK_PFL_ATPB + threadIdx.x;
                        rr[2 * q] = rr[2 * q + 1] = ~0ull;
                        if (P < pe1) rec2.get_pair(P, &rr[2 * q], &rr[2 * q + 1]);
                        if (2 * P < r0s) rr[2 * q] = ~0ull;
                        if (2 * P + 1 >= r1s) rr[2 * q + 1] = ~0ull;
                    }
#pragma unroll
                    for (int q = 0; q < 2 * FU; q++) consider(rr[q]);
#endif
                }
                __syncthreads();
                const uint32_t nc = ncand;
                if (nc <= SK_PFL_CAP) {
                    pfl_chunk(R, nc, nxt, head, fin, lw, dirty, [] {}, put);
                } else {
                __shared__ uint32_t gbase;
                unsigned long long *lk = reinterpret_cast<unsigned long long *>(work);
                uint32_t *lv = reinterpret_cast<uint32_t *>(lk + kBigL);
                if (threadIdx.x == 0) gbase = atomicAdd(big_alloc, 2 * k);
                for (uint32_t s = threadIdx.x; s < kBigL; s += SK_PFL_ATPB) lk[s] = SK_BIG_EMPTY, lv[s] = 0xffffffffu;
                __syncthreads();
                BigTable T{lk, lv, reinterpret_cast<unsigned long long *>(big_keys) + gbase, big_vals + gbase, 2 * k,
                           kBigL};
                for (uint32_t s = threadIdx.x; s < T.S; s += SK_PFL_ATPB) T.gk[s] = SK_BIG_EMPTY, T.gv[s] = 0xffffffffu;
                __threadfence();
                __syncthreads();
                auto cand = [&](uint64_t r) {
                    const uint64_t key = r >> 32;
                    return ((r >> 26) & 63u) > lds_reg_get(lw, pfl_slotb(key));
                };
                for (uint32_t u = threadIdx.x; u < k; u += SK_PFL_ATPB) {
                    const uint64_t r = run(u);
                    if (cand(r)) T.insert(((r >> 32) << 6) | ((r >> 26) & 63u), uint32_t(r & 0x3ffffffu));
                }
                __threadfence();
                __syncthreads();
                for (uint32_t u = threadIdx.x; u < k; u += SK_PFL_ATPB) { // replies (registers only read)
                    const uint64_t r = run(u), key = r >> 32;
                    if (!cand(r)) continue;
                    const uint32_t rho = uint32_t(r >> 26) & 63u, seq = uint32_t(r & 0x3ffffffu);
                    bool first = true;
                    for (uint32_t v = rho; v < 52 && first; v++) first = T.find((key << 6) | v) >= seq;
                    put(seq, first ? 1u : 0u);
                }
                __syncthreads();
                for (uint32_t u = threadIdx.x; u < k; u += SK_PFL_ATPB) { // the register's writer: its top record
                    const uint64_t r = run(u), key = r >> 32;
                    if (!cand(r)) continue;
                    const uint32_t rho = uint32_t(r >> 26) & 63u, seq = uint32_t(r & 0x3ffffffu);
                    if (T.find((key << 6) | rho) != seq) continue;
                    bool top = true;
                    for (uint32_t v = rho + 1; v < 52 && top; v++) top = T.find((key << 6) | v) == 0xffffffffu;
                    const uint32_t slotb = pfl_slotb(key);
                    const uint32_t cur = lds_reg_get(lw, slotb); // this thread is the register's only writer
                    if (top && rho > cur) {
                        lds_reg_xor(lw, slotb, cur ^ rho);
                        pfl_mark(dirty, slotb);
                    }
                }
                }
            }
            __syncthreads();
            for (uint32_t t = threadIdx.x; t < SK_PFL_HT; t += SK_PFL_ATPB) head[t] = 0xffffu;
            __syncthreads();
            t0 = t1;
        }
    }
    __syncthreads();
    if (sample) { // the reply mix of a sample of fine buckets decides the next call's default
        uint32_t tot, ones;
        block_exscan<SK_PFL_ATPB>(nrep, wsum, &tot);
        block_exscan<SK_PFL_ATPB>(nones, wsum, &ones);
        if (threadIdx.x == 0) {
            const uint32_t sh8 = (blockIdx.x >> 4) & 7u, q = 16 * (par ^ 1);
            atomicAdd(&rc[q + sh8], ones);
            atomicAdd(&rc[q + 8 + sh8], tot);
        }
    }
    if (probe & 4) return;
    for (uint32_t q = threadIdx.x; q < nsl * LW; q += SK_PFL_ATPB) // the changed 16-register groups (12 B each)
        if ((dirty[(q / SK_PFL_DG) >> 5] >> ((q / SK_PFL_DG) & 31u)) & 1u) {
            uint32_t *w = reinterpret_cast<uint32_t *>(line(q / LW)) + 3 * (q % LW);
            w[0] = lw[3 * q];
            w[1] = lw[3 * q + 1];
            w[2] = lw[3 * q + 2];
        }
}

// streamed-once 16-B load with the nontemporal hint (native vector type for the builtin)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4 *p) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// -------------------------------------------------------------- exact register sums (PFCOUNT, redis 3.x)
// The 3.x estimator needs only E = sum 2^-r[j] and the zero count (hllDenseSum).  With every register <= 39,
// S = E * 2^40 = sum 2^(40 - r[j]) is an integer < 2^55, and the host's E = S * 2^-40 is bit-identical to Redis's
// register-order double sum (every partial sum is a multiple of 2^-39 below 2^14: exact in 53 bits).
// One wave per key, 12 fully coalesced 16-B loads per lane: lane l holds chunks c = it * 64 + l of the 12,288-B body.
// Chunk c holds the registers whose 6-bit fields start in its bits: 22 of them when c % 3 == 0 (the 22nd straddles
// into chunk c + 1, whose first word comes from the next lane, or for lane 63 from lane 0's next chunk), else 21
// starting 4 (c % 3 == 1) or 2 (c % 3 == 2) bits in.  Registers are taken two at a time: the 12-bit pair indexes a
// 4,160-entry u64 table in LDS (built by each workgroup once) holding 2^(40 - a) + 2^(40 - b) in bits [0, 48), the
// pair's zero count at bit 48 and its count of registers >= 40 at bit 56 (entries 4096 + r: one register, the odd
// one of a 21-register chunk).  So a pair costs one extract, one LDS read and one 64-bit add.  Two accumulators (even
// and odd chunks, <= 132 registers each) keep the three fields from carrying into each other.
// out[2k] = S (0 when a register is >= 40), out[2k + 1] = zeros | (a register >= 40) << 32: the host then takes
// Redis's register-order sum instead.
#define SK_SUM_LUT (4096 + 64)
__device__ __forceinline__ uint64_t sum_term(uint32_t r) {
    return (r < 40u ? (1ull << (40u - r)) : 0ull) + (uint64_t(r == 0u) << 48) + (uint64_t(r >= 40u) << 56);
}
__global__ void __launch_bounds__(256) k_hll_sum(uint64_t n, const uint32_t *__restrict__ ids,
                                                 const uint8_t *__restrict__ arena, uint64_t *__restrict__ out) {
    __shared__ uint64_t lut[SK_SUM_LUT];
    for (uint32_t i = threadIdx.x; i < SK_SUM_LUT; i += 256)
        lut[i] = i < 4096u ? sum_term(i & 63u) + sum_term(i >> 6) : sum_term(i - 4096u);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, l3 = lane % 3u;
    for (uint64_t key = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6); key < n; key += uint64_t(gridDim.x) * 4) {
        const uint4 *base = reinterpret_cast<const uint4 *>(slab_at(arena, slab_of(ids[key])));
        uint4 v[12];
#pragma unroll
        for (int it = 0; it < 12; it++) v[it] = ld_nt(base + it * 64 + lane);
        uint64_t acc[2] = {0ull, 0ull};
#pragma unroll
        for (int it = 0; it < 12; it++) {
            const uint32_t m3 = (uint32_t(it) + l3) % 3u; // chunk % 3 (64 = 1 mod 3)
            const uint32_t o = m3 == 0u ? 0u : (m3 == 1u ? 4u : 2u);
            const uint32_t nx_same = uint32_t(__shfl(int(v[it].x), int((lane + 1u) & 63u)));
            const uint32_t nx_next = it + 1 < 12 ? __builtin_amdgcn_readfirstlane(v[it + 1 < 12 ? it + 1 : it].x) : 0u;
            const uint32_t w4 = lane == 63u ? nx_next : nx_same;
            // the chunk's 160-bit window shifted so that its first register starts at bit 0
            const uint32_t s[5] = {__builtin_amdgcn_alignbit(v[it].y, v[it].x, o),
                                   __builtin_amdgcn_alignbit(v[it].z, v[it].y, o),
                                   __builtin_amdgcn_alignbit(v[it].w, v[it].z, o),
                                   __builtin_amdgcn_alignbit(w4, v[it].w, o), w4 >> o};
#pragma unroll
            for (int p = 0; p < 11; p++) {
                const int bit = 12 * p, q = bit >> 5, sh = bit & 31;
                uint32_t x = (sh <= 20 ? (s[q] >> sh) : __builtin_amdgcn_alignbit(s[q + 1], s[q], sh)) & 0xfffu;
                if (p == 10) x = o == 0u ? x : 4096u + (x & 63u); // register 20 alone
                acc[it & 1] += lut[x];
            }
        }
        uint64_t S = (acc[0] & 0xffffffffffffull) + (acc[1] & 0xffffffffffffull);
        uint32_t zeros = uint32_t((acc[0] >> 48) & 255u) + uint32_t((acc[1] >> 48) & 255u);
        uint32_t big = uint32_t(acc[0] >> 56) + uint32_t(acc[1] >> 56);
#pragma unroll
        for (int o = 32; o; o >>= 1) {
            S += __shfl_xor(S, o);
            zeros += __shfl_xor(zeros, o);
            big += __shfl_xor(big, o);
        }
        if (lane == 0) {
            out[2 * key] = big ? 0ull : S;
            out[2 * key + 1] = uint64_t(zeros) | (uint64_t(big ? 1u : 0u) << 32);
        }
    }
}

// -------------------------------------------------------------- histogram
// 64-bin register histogram per key, one wave per key and no barriers (the input of the >= 5.0 estimator).
// Each lane owns a column of a bin-major LDS table h[64][64] (u32, 16 KiB per wave) and counts its 256 registers
// into it with return-less LDS adds: the address is bin * 256 + lane * 4, so the 64 lanes of one add always hit
// 64 different banks whatever the values, zeros included (no branch).  Lane b then sums row b (bin b) with 16-B
// reads, rotated per lane, and clears it.  LDS instructions of one wave execute in order, so the next key's adds
// land after this key's reads.  The next key's 16 KiB loads while the table is summed (a second key in registers,
// loading while this one is counted, measured the same).  10 waves per CU (the LDS): 48 % of wave cycles parked,
// LDS array 39 % busy, VALU 27 % (profiles/r03j_hist_sq_summary.json).
// PK: slabs ids[k] of the packed arena; else u8 register arrays (ids[k] = 0 with the array as `arena`: a union's
// temporary registers, sk_hll_count_registers_dev)
// Round 6: 16-bit halves of 8 KiB per wave (20 waves per CU): row r & 31 of lane l counts bin r in its low half and
// bin r + 32 in its high half.  Registers >= 32 need 31 leading zero bits of a hash, so a lane whose 16-register
// group holds none (one test of the fields' bit 5 per group) adds a constant 1 at row (r & 31) -- a 5-bit field
// extract and one shift-or per register -- and only a group with one takes the per-register increment.  Lanes 2 x
// 32 then sum the two halves of each row.  (u32 counters, 64 rows at 16 KiB per wave: 0.290 ms per 100 k keys;
// bins 2i / 2i + 1 in the halves with a computed increment per register: 0.276 ms.)
template <bool PK>
__global__ void __launch_bounds__(64) k_hll_hist(uint64_t n, const uint32_t *__restrict__ ids,
                                                   const uint8_t *__restrict__ arena, uint32_t *__restrict__ hist) {
    __shared__ uint4 h4[32 * 16];
    uint32_t *h = reinterpret_cast<uint32_t *>(h4);
    const uint32_t lane = threadIdx.x, l4 = lane * 4u;
#pragma unroll
    for (int j = 0; j < 8; j++) h4[lane + 64 * j] = make_uint4(0, 0, 0, 0);
    // a lane's 16 groups of 16 registers: groups it * 64 + lane (packed: three words each; u8: one 16-B vector)
    auto load = [&](uint64_t key, uint32_t (&v)[16][4]) {
        if constexpr (PK) {
            const uint32_t *base = reinterpret_cast<const uint32_t *>(slab_at(arena, slab_of(ids[key])));
#pragma unroll
            for (int it = 0; it < 16; it++)
#pragma unroll
                for (int q = 0; q < 3; q++) v[it][q] = __builtin_nontemporal_load(base + 3 * (it * 64 + lane) + q);
        } else {
            const uint4 *base = reinterpret_cast<const uint4 *>(arena + (uint64_t(ids[key] & SK_SLAB_MASK) << 14));
#pragma unroll
            for (int it = 0; it < 16; it++) {
                const uint4 x = ld_nt(base + it * 64 + lane);
                v[it][0] = x.x, v[it][1] = x.y, v[it][2] = x.z, v[it][3] = x.w;
            }
        }
    };
    auto add = [&](uint32_t byteaddr, uint32_t inc) {
        __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(h) + byteaddr), inc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    };
    auto count = [&](uint64_t key, const uint32_t (&v)[16][4]) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 16; it++) {
            uint32_t src[16], pos[16];
            bool big;
            if constexpr (PK) {
                const uint32_t w0 = v[it][0], w1 = v[it][1], w2 = v[it][2];
                // bit 5 of fields 0-4 / 6-9 (+ field 5's) / 10-15: any register >= 32 in the group
                big = ((w0 & 0x20820820u) | (w1 & 0x08208208u) | (w2 & 0x82082082u)) != 0u;
                const uint32_t x5 = __builtin_amdgcn_alignbit(w1, w0, 30), x10 = __builtin_amdgcn_alignbit(w2, w1, 28);
                const uint32_t sw[16] = {w0, w0, w0, w0, w0, x5, w1, w1, w1, w1, x10, w2, w2, w2, w2, w2};
                const uint32_t sp[16] = {0, 6, 12, 18, 24, 0, 4, 10, 16, 22, 0, 2, 8, 14, 20, 26};
#pragma unroll
                for (int j = 0; j < 16; j++) src[j] = sw[j], pos[j] = sp[j];
            } else {
                big = ((v[it][0] | v[it][1] | v[it][2] | v[it][3]) & 0x20202020u) != 0u;
#pragma unroll
                for (int j = 0; j < 16; j++) src[j] = v[it][j >> 2], pos[j] = 8u * (j & 3);
            }
            if (!big) { // row = the field's low 5 bits, +1 in the low half
#pragma unroll
                for (int j = 0; j < 16; j++) add((__builtin_amdgcn_ubfe(src[j], pos[j], 5) << 8) | l4, 1u);
            } else {
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const uint32_t r = __builtin_amdgcn_ubfe(src[j], pos[j], 6);
                    add(((r & 31u) << 8) | l4, (r & 32u) ? 65536u : 1u);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // lanes b and b + 32 sum the two halves of row b & 31, then add each other's: bin b in the low half, b + 32 in
        // the high (64 lanes x <= 256 registers per bin: no carry out of a half)
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t q = (lane & 31u) * 16 + (lane >> 5) * 8 + ((j + lane) & 7u);
            const uint4 x = h4[q];
            c += x.x + x.y + x.z + x.w;
            h4[q] = make_uint4(0, 0, 0, 0);
        }
        c += __shfl_xor(c, 32);
        hist[key * 64 + lane] = lane < 32u ? c & 0xffffu : c >> 16;
    };
    const uint64_t G = gridDim.x;
    uint32_t v[16][4];
    uint64_t key = blockIdx.x;
    if (key < n) load(key, v);
    for (; key < n; key += G) {
        count(key, v);
        if (key + G < n) load(key + G, v);
    }
}

// ------------------------------------------------------------------ union
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t bytemax(uint32_t a, uint32_t b) {
    const uint32_t m = 0x00ff00ffu;
    us2 al = __builtin_bit_cast(us2, a & m), bl = __builtin_bit_cast(us2, b & m);
    us2 ah = __builtin_bit_cast(us2, (a >> 8) & m), bh = __builtin_bit_cast(us2, (b >> 8) & m);
    uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(al, bl));
    uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(ah, bh));
    return lo | (hi << 8);
}
__device__ __forceinline__ uint4 bytemax4(uint4 a, uint4 b) {
    return make_uint4(bytemax(a.x, b.x), bytemax(a.y, b.y), bytemax(a.z, b.z), bytemax(a.w, b.w));
}

// grid (4, G): block (x, g) covers 4096 registers (256 lanes x 16 registers) of the union of sources
// [g*per, (g+1)*per) and writes partial[g] as u8 registers.  Sources are slabs ids[k] of the packed arena (PK: 12-B
// groups, unpacked in registers), or consecutive u8 register arrays of 16 KiB (ids == null: the form the next tree
// level reads; or one caller array, sk_hll_merge_registers_dev).
// PK keeps the running max as 8 pairs of u16 lanes (registers 2j, 2j + 1 of the group: one v_pk_max_u16 each), each
// source's 12 bytes going straight into that form (two field extracts and a shift-or per pair), and converts to u8 once
__device__ __forceinline__ void grp_pairs(uint32_t w0, uint32_t w1, uint32_t w2, us2 (&p)[8]) {
    const uint32_t x[8] = {w0, w0 >> 12, __builtin_amdgcn_alignbit(w1, w0, 24), w1 >> 4,
                           w1 >> 16, __builtin_amdgcn_alignbit(w2, w1, 28), w2 >> 8, w2 >> 20};
#pragma unroll
    for (int j = 0; j < 8; j++)
        p[j] = __builtin_bit_cast(us2, (x[j] & 63u) | (((x[j] >> 6) & 63u) << 16));
}
template <bool PK>
__global__ void __launch_bounds__(256) k_hll_union_partial(uint64_t n, const uint32_t *__restrict__ ids,
                                                           const uint8_t *__restrict__ base, uint64_t per,
                                                           uint8_t *__restrict__ partial) {
    unsigned lane16 = blockIdx.x * 256 + threadIdx.x; // group of 16 registers within the key
    uint64_t g = blockIdx.y, k0 = g * per, k1 = k0 + per;
    if (k1 > n) k1 = n;
    uint64_t k = k0;
    // the next step's slab ids are loaded while this step's 8 vectors are in flight (the id loads used to sit in
    // front of every step's vector loads)
    auto idof = [&](uint64_t kk) -> uint64_t { return ids ? slab_of(ids[kk]) : kk; };
    uint64_t idn[8];
    if (k + 8 <= k1)
#pragma unroll
        for (int j = 0; j < 8; j++) idn[j] = idof(k + j);
    if constexpr (PK) {
        us2 acc[8];
#pragma unroll
        for (int j = 0; j < 8; j++) acc[j] = us2{0, 0};
        auto fold = [&](uint32_t w0, uint32_t w1, uint32_t w2) {
            us2 p[8];
            grp_pairs(w0, w1, w2, p);
#pragma unroll
            for (int j = 0; j < 8; j++) acc[j] = __builtin_elementwise_max(acc[j], p[j]);
        };
        auto wp = [&](uint64_t id) { return reinterpret_cast<const uint32_t *>(slab_at(base, id)) + 3 * lane16; };
        for (; k + 8 <= k1; k += 8) { // 8 independent groups in flight per lane
            uint32_t a[8][3];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t *w = wp(idn[j]);
                a[j][0] = __builtin_nontemporal_load(w);
                a[j][1] = __builtin_nontemporal_load(w + 1);
                a[j][2] = __builtin_nontemporal_load(w + 2);
            }
            if (k + 16 <= k1)
#pragma unroll
                for (int j = 0; j < 8; j++) idn[j] = idof(k + 8 + j);
#pragma unroll
            for (int j = 0; j < 8; j++) fold(a[j][0], a[j][1], a[j][2]);
        }
        for (; k < k1; k++) {
            const uint32_t *w = wp(idof(k));
            fold(__builtin_nontemporal_load(w), __builtin_nontemporal_load(w + 1), __builtin_nontemporal_load(w + 2));
        }
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; q++) { // bytes 0 and 2 of pair 2q (registers 4q, 4q + 1), then of pair 2q + 1
            const uint32_t lo = __builtin_bit_cast(uint32_t, acc[2 * q]), hi = __builtin_bit_cast(uint32_t, acc[2 * q + 1]);
            o[q] = __builtin_amdgcn_perm(hi, lo, 0x06040200u);
        }
        reinterpret_cast<uint4 *>(partial + g * 16384)[lane16] = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
        uint4 acc = make_uint4(0, 0, 0, 0);
        auto ld = [&](uint64_t id) -> uint4 { return ld_nt(reinterpret_cast<const uint4 *>(base + (id << 14)) + lane16); };
        for (; k + 8 <= k1; k += 8) { // 8 independent loads in flight per lane
            uint4 a[8];
#pragma unroll
            for (int j = 0; j < 8; j++) a[j] = ld(idn[j]);
            if (k + 16 <= k1)
#pragma unroll
                for (int j = 0; j < 8; j++) idn[j] = idof(k + 8 + j);
            acc = bytemax4(acc, bytemax4(bytemax4(bytemax4(a[0], a[1]), bytemax4(a[2], a[3])),
                                         bytemax4(bytemax4(a[4], a[5]), bytemax4(a[6], a[7]))));
        }
        for (; k < k1; k++) acc = bytemax4(acc, ld(idof(k)));
        reinterpret_cast<uint4 *>(partial + g * 16384)[lane16] = acc;
    }
}

// out = max(include_out ? out : 0, partial[0..G)) for a small G (the tree root); PKOUT: out is a packed slab (the
// PFMERGE destination), else u8 registers
template <bool PKOUT>
__global__ void __launch_bounds__(256) k_hll_union_final(uint64_t G, const uint8_t *__restrict__ partial,
                                                         uint8_t *__restrict__ out, int include_out) {
    unsigned lane16 = blockIdx.x * 256 + threadIdx.x;
    uint4 acc = make_uint4(0, 0, 0, 0);
    if (include_out) acc = PKOUT ? grp_load(out, lane16) : reinterpret_cast<const uint4 *>(out)[lane16];
    const uint4 *pp = reinterpret_cast<const uint4 *>(partial) + lane16;
    uint64_t g = 0;
    for (; g + 8 <= G; g += 8) { // 8 partials in flight (one at a time took 12 us for 31 partials at C4)
        uint4 a[8];
#pragma unroll
        for (int j = 0; j < 8; j++) a[j] = pp[(g + j) * 1024];
        acc = bytemax4(acc, bytemax4(bytemax4(bytemax4(a[0], a[1]), bytemax4(a[2], a[3])),
                                     bytemax4(bytemax4(a[4], a[5]), bytemax4(a[6], a[7]))));
    }
    for (; g < G; g++) acc = bytemax4(acc, pp[g * 1024]);
    if (PKOUT) grp_store(out, lane16, acc);
    else reinterpret_cast<uint4 *>(out)[lane16] = acc;
}

// The arena holds Redis's dense bodies, so SAVE / DUMP of many HLLs and the bulk restore of a snapshot (sk_rdb.h) are
// gathers / scatters of 12,288-B bodies: 768 16-B vectors per key, one per thread.
// out[i * 12288 ..) = the dense body of slab ids[i] (generation bits masked off)
__global__ void __launch_bounds__(256) k_hll_pack(uint64_t n, const uint32_t *__restrict__ ids,
                                                  const uint8_t *__restrict__ arena, uint32_t *__restrict__ out) {
    const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x, key = t / 768, v = t % 768;
    if (key >= n) return;
    reinterpret_cast<uint4 *>(out)[key * 768 + v] =
        reinterpret_cast<const uint4 *>(slab_at(arena, slab_of(ids[key])))[v];
}
// slab ids[i] = the dense body in[i * 12288 ..)
__global__ void __launch_bounds__(256) k_hll_unpack(uint64_t n, const uint32_t *__restrict__ ids,
                                                    const uint32_t *__restrict__ in, uint8_t *__restrict__ arena) {
    const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x, key = t / 768, v = t % 768;
    if (key >= n) return;
    reinterpret_cast<uint4 *>(slab_at(arena, slab_of(ids[key])))[v] =
        reinterpret_cast<const uint4 *>(in)[key * 768 + v];
}

// ------------------------------------------------------------------ Bloom
__device__ __forceinline__ void bloom_hashes(const uint8_t *p, uint32_t len, uint64_t *h1, uint64_t *h2) {
    *h1 = xxh64(p, len);
    *h2 = farm_uo64(p, len);
}

// contains: probes 0..k-2 only (the k-th GETBIT reply is dropped by
// result.subList(1, size-1), M:RedissonBloomFilter.java:155), in order, and
// an element stops at its first 0 bit (the fewest line fetches: fetching
// 2, 3 or all probes per round measured 8 %, 13 % and 38 % slower at C3).
// Members need k-1 probes, non-members ~2 at fill 0.5.
//
// k_bloom_contains: one element per thread -- a wave lives as long as its
// slowest lane, so early-exit lanes sit idle.
// k_bloom_contains_q: a wave hashes 64*EPT elements into LDS, then runs a
// probe queue: every iteration each busy lane issues one probe, and lanes
// whose element finished take the next one (ballot + prefix count, no
// atomics), so nearly every lane of every load instruction is a useful probe.
// Measured at C3 (1M contains, k = 7, fill 0.5): 112 us one-per-thread, 113
// queue with 4 elements per lane, 110 with 2 -- the chip-wide rate of random
// line requests (~55 G/s), not idle lanes, bounds it.
// WORDS: key window (u64 words)
template <int WORDS>
__device__ __forceinline__ void bloom_contains_body(uint64_t n, const uint64_t *__restrict__ off,
                                                    const uint8_t *__restrict__ bytes, const uint8_t *__restrict__ bits,
                                                    const uint64_t *__restrict__ d_len, uint64_t size, uint64_t magic,
                                                    int k, uint8_t *__restrict__ out) {
    __shared__ uint64_t lds[WORDS];
    uint64_t e0 = uint64_t(blockIdx.x) * blockDim.x, e1 = e0 + blockDim.x < n ? e0 + blockDim.x : n;
    uint64_t lo = off[e0], hi = off[e1];
    bool staged = (hi - (lo & ~uint64_t(15))) + 32 <= uint64_t(WORDS) * 8;
    uint32_t wbase = staged ? stage_keys(bytes, lo, hi, lds) : 0u;
    uint64_t i = e0 + threadIdx.x;
    if (i >= n) return;
    uint64_t o = off[i];
    uint32_t len = uint32_t(off[i + 1] - o);
    uint64_t h1, h2;
    if (staged) {
        LdsReader rd{lds, wbase + uint32_t(o - lo)};
        h1 = xxh64_r(rd, len);
        h2 = farm_uo64_r(rd, len);
    } else {
        bloom_hashes(bytes + o, len, &h1, &h2);
    }
    uint64_t slen = *d_len;
    BloomIdx bi(h1, h2, size, magic);
    uint8_t r = 1;
    for (int j = 0; j < k - 1; j++) {
        if (!get_bit(bits, slen, bi.r)) {
            r = 0;
            break;
        }
        bi.next(j);
    }
    out[i] = r;
}

__global__ void __launch_bounds__(256) k_bloom_contains(uint64_t n, const uint64_t *__restrict__ off,
                                                        const uint8_t *__restrict__ bytes,
                                                        const uint8_t *__restrict__ bits,
                                                        const uint64_t *__restrict__ d_len, uint64_t size,
                                                        uint64_t magic, int k, uint8_t *__restrict__ out) {
    bloom_contains_body<SK_STAGE_WORDS>(n, off, bytes, bits, d_len, size, magic, k, out);
}
// split schedule (SK_BLOOM_SCHED=3): k_bloom_hash writes (h1, h2) per element
// (16 B, coalesced), k_bloom_probe_h walks the probes with few registers, so
// the request-bound half runs at full occupancy and the compute-bound half can
// overlap another stream's request-bound kernel.
__global__ void __launch_bounds__(256) k_bloom_hash(uint64_t n, const uint64_t *__restrict__ off,
                                                    const uint8_t *__restrict__ bytes, uint4 *__restrict__ hh) {
    __shared__ uint64_t lds[SK_STAGE_WORDS];
    uint64_t e0 = uint64_t(blockIdx.x) * blockDim.x, e1 = e0 + blockDim.x < n ? e0 + blockDim.x : n;
    uint64_t lo = off[e0], hi = off[e1];
    bool staged = stage_fits(lo, hi);
    uint32_t wbase = staged ? stage_keys(bytes, lo, hi, lds) : 0u;
    uint64_t i = e0 + threadIdx.x;
    if (i >= n) return;
    uint64_t o = off[i];
    uint32_t len = uint32_t(off[i + 1] - o);
    uint64_t h1, h2;
    if (staged) {
        LdsReader rd{lds, wbase + uint32_t(o - lo)};
        h1 = xxh64_r(rd, len);
        h2 = farm_uo64_r(rd, len);
    } else {
        bloom_hashes(bytes + o, len, &h1, &h2);
    }
    hh[i] = make_uint4(uint32_t(h1), uint32_t(h1 >> 32), uint32_t(h2), uint32_t(h2 >> 32));
}
__global__ void __launch_bounds__(256) k_bloom_probe_h(uint64_t n, const uint4 *__restrict__ hh,
                                                       const uint8_t *__restrict__ bits,
                                                       const uint64_t *__restrict__ d_len, uint64_t size,
                                                       uint64_t magic, int k, uint8_t *__restrict__ out) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 v = hh[i];
    uint64_t h1 = uint64_t(v.x) | uint64_t(v.y) << 32, h2 = uint64_t(v.z) | uint64_t(v.w) << 32;
    uint64_t slen = *d_len;
    BloomIdx bi(h1, h2, size, magic);
    uint8_t r = 1;
    for (int j = 0; j < k - 1; j++) {
        if (!get_bit(bits, slen, bi.r)) {
            r = 0;
            break;
        }
        bi.next(j);
    }
    out[i] = r;
}
template <int EPT>
__global__ void __launch_bounds__(256) k_bloom_contains_q(uint64_t n, const uint64_t *__restrict__ off,
                                                          const uint8_t *__restrict__ bytes,
                                                          const uint8_t *__restrict__ bits,
                                                          const uint64_t *__restrict__ d_len, uint64_t size,
                                                          uint64_t magic, int k, uint8_t *__restrict__ out) {
    __shared__ uint64_t lds[SK_STAGE_WORDS];
    __shared__ uint64_t H1[256 * EPT], H2[256 * EPT];
    uint64_t base = uint64_t(blockIdx.x) * (256 * EPT);
    for (int e = 0; e < EPT; e++) { // hash 256 elements per round (keys staged in LDS)
        uint64_t e0 = base + uint64_t(e) * 256;
        if (e0 >= n) break; // uniform
        uint64_t e1 = e0 + 256 < n ? e0 + 256 : n;
        uint64_t lo = off[e0], hi = off[e1];
        bool staged = stage_fits(lo, hi);
        __syncthreads(); // the previous round's readers are done
        uint32_t wbase = staged ? stage_keys(bytes, lo, hi, lds) : 0u;
        uint64_t i = e0 + threadIdx.x;
        if (i < n) {
            uint64_t o = off[i];
            uint32_t len = uint32_t(off[i + 1] - o);
            uint64_t h1, h2;
            if (staged) {
                LdsReader rd{lds, wbase + uint32_t(o - lo)};
                h1 = xxh64_r(rd, len);
                h2 = farm_uo64_r(rd, len);
            } else {
                bloom_hashes(bytes + o, len, &h1, &h2);
            }
            H1[e * 256 + threadIdx.x] = h1;
            H2[e * 256 + threadIdx.x] = h2;
        }
    }
    __syncthreads();
    // wave w owns local elements [first, first + cnt)
    const uint32_t lane = threadIdx.x & 63u, first = (threadIdx.x >> 6) * (64u * EPT);
    uint64_t avail = n - base;
    uint32_t cnt = avail > first ? uint32_t(avail - first < 64u * EPT ? avail - first : 64u * EPT) : 0u;
    uint8_t *o = out + base + first;
    const int np = k - 1;
    if (np <= 0) { // k = 1: no reply is kept, contains is true (Q2)
        for (uint32_t t = lane; t < cnt; t += 64) o[t] = 1;
        return;
    }
    const uint64_t slen = *d_len;
    uint32_t cursor = 64, cur = lane;
    bool active = lane < cnt;
    uint64_t a1 = 0, a2 = 0, h = 0;
    int j = 0;
    if (active) {
        a1 = H1[first + cur];
        a2 = H2[first + cur];
        h = a1;
    }
    while (true) {
        bool freed = !active;
        if (active) {
            int bit = get_bit(bits, slen, mod_invariant(h & 0x7fffffffffffffffull, size, magic));
            if (!bit || j == np - 1) {
                o[cur] = uint8_t(bit);
                freed = true;
            } else {
                h += (j & 1) ? a1 : a2;
                j++;
            }
        }
        uint64_t mask = __ballot(freed);
        if (freed) {
            uint32_t e = cursor + uint32_t(__popcll(mask & ((1ull << lane) - 1ull)));
            active = e < cnt;
            if (active) {
                cur = e;
                a1 = H1[first + e];
                a2 = H2[first + e];
                h = a1;
                j = 0;
            }
        }
        cursor += uint32_t(__popcll(mask));
        if (__ballot(active) == 0) break;
    }
}

// ------------------------------------------- Bloom contains, region schedule
// For large contains batches (n >> filter lines / probes) the one-element-
// per-thread kernel pays one 128-B HBM line request per probe: the C3 array
// (534 MB, ~4.2 M lines) sees ~1 probe per line per 1 M batch, so no line is
// ever reused and the chip-wide random-request rate (~54 G/s) bounds it.
// The region schedule turns the probes around: probes are bucketed by the
// 128 KiB region of the bit array they fall in, and one workgroup per region
// loads its region into LDS once (a coalesced stream) and answers every probe
// of the batch that falls there from LDS.  HBM then sees the keys, the probe
// records (4 B per probe, written and read once, coalesced) and the array once
// per batch, instead of a line per probe.
//   k_bloom_rc_hash   one 1024-thread workgroup per RC_EPB elements: XXH64 +
//                     farmhashuo, the k-1 probes that decide contains (Q2),
//                     an LDS counting sort of the block's probes by region,
//                     stored as one coalesced chunk of u32 records
//                     (bit-in-region << 12 | element-in-block) plus the
//                     block's column of the region-major segment table S[region][block] = start | count<<16;
//                     out[i] = 1 for every element.
//   k_bloom_rc_probe  one 1024-thread workgroup per region: the region's
//                     128 KiB into LDS, then the region's segment of every
//                     block chunk; a probe on a 0 bit stores out[elem] = 0
//                     (contains is the AND of its probes; every writer of an
//                     element writes the same 0, so the order is free).
// Regions of one XCD are consecutive (blockIdx % 8 -> XCD under round-robin
// dispatch; speed only, never correctness): the ~32 workgroups an XCD runs at
// once read neighbouring segments of each block chunk, which share lines.
#ifndef SK_BLOOM_PRE
#define SK_BLOOM_PRE 1                // shared-prefix hash path (sk_device.h bloom_hashes_pre)
#endif
#ifndef SK_RC_ABL
// dev ablations of the contains chain (results discarded): 1 no reply stores, 2 no record loads, 4 no region load,
// 8 no hash arithmetic, 16 no segment-table stores, 32 no record stores, 64 no add reply stores; of the add apply:
// 128 records gathered from one contiguous run, 256 no windows (region and segment table only), 512 no chain walk;
// 1024: the probe reads each (block, region) segment from a region-major position ((r * NB + j) * CH / NR words,
// as a region-major record arena would place it: a wave's segments adjacent) -- a timing probe, results discarded;
// of the probe's zero lists: 2048 no word tests, 4096 no scan or list entries, 8192 no list sort or write-back;
// of the hash: 16384 no per-round barrier
#define SK_RC_ABL 0
#endif
#ifndef SK_RC_LATERANK
// contains hash: 1 = the hashing rounds only count each probe's region (return-less LDS adds), and the records take
// their places with returning adds on the region cursors after the scan (the ranks leave the rounds' critical path)
#define SK_RC_LATERANK 0
#endif
#ifndef SK_RC_STILE
// The hash blocks write their segment entries interleaved by SK_RC_STILE regions, St[(r / T * NB + block) * T + r % T]:
// a block's entries for T consecutive regions are one 128-B line (coalesced stores; a region-major row per region
// made every entry a separate partial line, 0.12 ms of the contains hash per 32 M).  k_rc_stranspose then turns
// them into the region-major rows S[r * NB + block] the probe / apply stream (their rows read as columns of the
// interleaved table cost the probe 0.15 ms).  1: the hash writes the rows itself, no transpose.
#define SK_RC_STILE 32
#endif
#ifndef SK_RC_STAMP
#define SK_RC_STAMP 0 // dev: s_memtime stamps of the contains hash blocks' phases (thread 0 of each block)
#endif
#if SK_RC_STAMP
__device__ unsigned long long sk_rc_stamps[8192 * 8];
#define RC_STAMP(k)                                                                                                    \
    do {                                                                                                               \
        if (!ADD && threadIdx.x == 0 && jb < 8192) sk_rc_stamps[jb * 8 + (k)] = __builtin_amdgcn_s_memtime();          \
    } while (0)
extern "C" hipError_t sk_rc_stamp_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sk_rc_stamps), sizeof(sk_rc_stamps), 0, hipMemcpyDeviceToHost);
}
#else
#define RC_STAMP(k) do { } while (0)
#endif
__host__ __device__ __forceinline__ uint64_t rc_sidx(uint32_t r, uint32_t j, uint32_t NB) {
    return (uint64_t(r / SK_RC_STILE) * NB + j) * SK_RC_STILE + (r % SK_RC_STILE);
}
#ifndef RC_RB
#define RC_RB 20                      // region = 2^20 bits = 128 KiB
#endif
#define RC_TPB 1024
#define RC_EPB 4096                   // elements per hash block (12-bit element-in-block)
#ifndef RC_PMAX
#define RC_PMAX 8                     // probes per element handled here (k <= 9)
#endif
#ifndef RC_NRMAX
#define RC_NRMAX 4096                 // regions (bit arrays <= 2^32 bits)
#endif
#define RC_ROUNDS (RC_EPB / RC_TPB)
// add: elements per hash block.  4096 while the block's records (4096 x k u32) fit LDS beside the key windows and
// the region counts (k <= RA_K4), else 2048: twice the records per (block, region) segment and half the segment
// table -- the apply's cost is per record and per segment (C3 fill: 5.5 vs 3.9 G adds/s, r03)
#define RA_K4 7
__host__ __device__ constexpr uint32_t ra_bufw(uint32_t epb, uint32_t pmax) { // u64 words: two key windows, then
    return epb * pmax / 2 > 2 * SK_PFP_WIN ? epb * pmax / 2 : 2 * SK_PFP_WIN;  // the block's records (epb x pmax u32)
}
#define RA_RB 19                      // add: region = 2^19 bits = 64 KiB (the apply keeps a window of records too)
#define RA_NRMAX 8192
#define RA_SEGMAX 512                 // add: longest (block, region) segment the apply's windows take
#define RC_BUFW 16384                 // u64 words: two key windows, then the block's records (RC_EPB*RC_PMAX u32)
static_assert(2 * SK_PFP_WIN <= RC_BUFW && RC_EPB * RC_PMAX * 4 <= RC_BUFW * 8, "hash block LDS");
static_assert(RC_EPB * RC_PMAX < 65536, "segment starts/counts are u16");
static_assert(4096 * 2 <= 8192, "add records: bit << 13 | element << 1 | last (element < 4096)");
static_assert(ra_bufw(4096, RA_K4) * 8 + RA_NRMAX * 4 <= 150 * 1024 && RA_K4 <= RC_PMAX, "add hash block LDS");
static_assert(RC_TPB == SK_PFP_TPB, "key windows sized for SK_PFP_TPB threads");

// ADD: AEPB = the add's elements per block (4096 for k <= RA_K4, else 2048)
// CPM: contains probes held per element (6 for k <= 7, the bench's C3 filter; else RC_PMAX): the probes' indexes
// and ranks stay in registers across the block's rounds, so holding no more than needed keeps the kernel spill-free
template <bool ADD, uint32_t AEPB = 2048, uint32_t CPM = RC_PMAX>
__global__ void __launch_bounds__(RC_TPB) k_bloom_rc_hash(uint64_t n, const uint64_t *__restrict__ off,
                                                          const uint8_t *__restrict__ bytes, uint64_t size,
                                                          uint64_t magic, uint32_t P, uint32_t NR, uint32_t NB,
                                                          uint32_t *__restrict__ S, uint32_t *__restrict__ chunks,
                                                          uint8_t *__restrict__ out, uint32_t *__restrict__ flag,
                                                          uint32_t piece) {
    constexpr uint32_t EPB = ADD ? AEPB : RC_EPB;
    constexpr uint32_t PM = ADD ? (AEPB == 4096 ? RA_K4 : RC_PMAX) : CPM; // probes per element held
    static_assert(PM <= RC_PMAX, "probes held");
    static_assert(!ADD || AEPB == 2048 || AEPB == 4096, "add blocks");
    constexpr int ROUNDS = int(EPB / RC_TPB);
    constexpr uint32_t RB = ADD ? RA_RB : RC_RB, NRMAX = ADD ? RA_NRMAX : RC_NRMAX, RPT = NRMAX / RC_TPB;
    __shared__ uint32_t hist[NRMAX];
    // block j: consecutive blocks on one XCD (blockIdx % 8 groups, speed only), so the ~32 blocks an XCD runs at
    // once write neighbouring words of each region's row of S and those lines fill in its L2
    const uint32_t jq = (NB + 7) / 8, jb = (blockIdx.x & 7u) * jq + (blockIdx.x >> 3);
    if (jb >= NB) return; // uniform
    RC_STAMP(0);
    __shared__ uint32_t wsum[RC_TPB / 64];
    __shared__ uint64_t buf[ra_bufw(EPB, PM)]; // two key windows, then the block's records (EPB x PM u32)
    uint64_t *win[2] = {buf, buf + SK_PFP_WIN};
    uint32_t *lrec = reinterpret_cast<uint32_t *>(buf); // after the last hash round
    for (uint32_t r = threadIdx.x; r < NR; r += RC_TPB) hist[r] = 0;
    const uint64_t base = uint64_t(jb) * EPB;
    const uint64_t rounds = (n - base + RC_TPB - 1) / RC_TPB;
    const int nr = rounds < ROUNDS ? int(rounds) : ROUNDS;
    uint64_t wb[ROUNDS + 1];
#pragma unroll
    for (int e = 0; e <= ROUNDS; e++) {
        uint64_t i0 = base + uint64_t(e) * RC_TPB;
        wb[e] = off[i0 < n ? i0 : n];
    }
    // this thread's element offsets, one round ahead (the next round's are loaded while this round hashes; holding
    // all rounds' offsets in registers made the kernel spill)
    uint64_t oa_c = 0, ob_c = 0;
    {
        const uint64_t i = base + threadIdx.x;
        if (i < n) {
            oa_c = off[i];
            ob_c = off[i + 1];
        }
    }
    uint4 v[SK_PFP_WVEC];
    const bool fit0 = pfp_win_fits(wb[0], wb[1]);
    if (fit0) {
        pfp_win_load(bytes, wb[0], wb[1], v);
        pfp_win_store(wb[0], wb[1], v, win[0]);
    }
    __syncthreads(); // hist zeroed, window 0 staged
    RC_STAMP(1);
#if SK_BLOOM_PRE
    // the block's first element's 16 leading bytes: the shared-prefix pattern (bloom_hashes_pre)
    const BloomPre bpre = fit0 ? bloom_pre(LdsReader{win[0], uint32_t(wb[0] & 15u)}.u64(0),
                                          LdsReader{win[0], uint32_t(wb[0] & 15u)}.u64(8))
                              : bloom_pre(ldu64(bytes + wb[0]), ldu64(bytes + wb[0] + 8));
#endif
    // probe p of round e: bit index (< 2^32: sizes <= 4,294,967,294) and its rank in its region
    uint32_t ix[ROUNDS][PM], rk[ROUNDS][(PM + 1) / 2]; // u16 ranks, two per word
#pragma unroll
    for (int e = 0; e < ROUNDS; e++) {
#pragma unroll
        for (int q = 0; q < int(PM); q++) ix[e][q] = 0;
#pragma unroll
        for (int q = 0; q < int(PM + 1) / 2; q++) rk[e][q] = 0;
        if (e >= nr) continue; // uniform
        bool pre = e + 1 < nr && pfp_win_fits(wb[e + 1], wb[e + 2]);
        if (pre) pfp_win_load(bytes, wb[e + 1], wb[e + 2], v);
        uint64_t oa_n = 0, ob_n = 0;
        if (e + 1 < nr) {
            const uint64_t i1 = base + uint64_t(e + 1) * RC_TPB + threadIdx.x;
            if (i1 < n) {
                oa_n = off[i1];
                ob_n = off[i1 + 1];
            }
        }
        const uint64_t oa = oa_c, ob = ob_c;
        oa_c = oa_n;
        ob_c = ob_n;
        uint64_t i = base + uint64_t(e) * RC_TPB + threadIdx.x;
        if (i < n) {
            uint32_t len = uint32_t(ob - oa);
            uint64_t h1, h2;
            if (pfp_win_fits(wb[e], wb[e + 1])) {
                LdsReader rd{win[e & 1], uint32_t(wb[e] & 15u) + uint32_t(oa - wb[e])};
#if SK_RC_ABL & 8
                (void)rd;
                h1 = (oa + len) * 0x9e3779b97f4a7c15ull;
                h2 = (h1 ^ (h1 >> 29)) * 0xbf58476d1ce4e5b9ull;
#elif SK_BLOOM_PRE
                bloom_hashes_pre(rd, len, bpre, &h1, &h2);
#else
                h1 = xxh64_r(rd, len);
                h2 = farm_uo64_r(rd, len);
#endif
            } else {
                bloom_hashes(bytes + oa, len, &h1, &h2);
            }
            if (!ADD) out[i] = 1;
            BloomIdx32 bi(h1, h2, size, magic); // sizes < 2^32 (the records hold 32-bit indexes)
#pragma unroll
            for (int p = 0; p < int(PM); p++) {
                if (uint32_t(p) >= P) break;
                uint32_t idx = uint32_t(bi.r);
                ix[e][p] = idx;
                if (!ADD && SK_RC_LATERANK) { // a count only (a return-less LDS add): ranks come at placement
                    atomicAdd(&hist[idx >> RB], 1u);
                } else {
                    uint32_t rank = atomicAdd(&hist[idx >> RB], 1u);
                    rk[e][p >> 1] |= rank << ((p & 1) * 16);
                }
                bi.next(p);
            }
        }
        if (pre) pfp_win_store(wb[e + 1], wb[e + 2], v, win[(e + 1) & 1]);
#if !(SK_RC_ABL & 16384) // timing probe: no per-round barrier (keys read from a window that may not be staged)
        __syncthreads(); // window e+1 staged; window e free for round e+2
#endif
    }
    RC_STAMP(2);
    // segment starts: RPT consecutive regions per thread
    uint32_t c4[RPT], s4 = 0;
#pragma unroll
    for (uint32_t q = 0; q < RPT; q++) {
        uint32_t r = threadIdx.x * RPT + q;
        c4[q] = r < NR ? hist[r] : 0u;
        s4 += c4[q];
    }
    uint32_t tot;
    uint32_t st = block_exscan<RC_TPB>(s4, wsum, &tot);
#pragma unroll
    for (uint32_t q = 0; q < RPT; q++) { // S is region-major: S[r * NB + block]
        uint32_t r = threadIdx.x * RPT + q;
        if (r < NR) {
            if (ADD && c4[q] > RA_SEGMAX) atomicMin(flag, piece); // the apply's windows assume short segments
            hist[r] = st;
            if (!(SK_RC_ABL & 16) || ADD) S[rc_sidx(r, jb, NB)] = st | (c4[q] << 16);
        }
        st += c4[q];
    }
    __syncthreads();
    RC_STAMP(3);
#pragma unroll
    for (int e = 0; e < ROUNDS; e++) {
        uint64_t i = base + uint64_t(e) * RC_TPB + threadIdx.x;
        if (e >= nr || i >= n) continue;
#pragma unroll
        for (int p = 0; p < int(PM); p++) {
            if (uint32_t(p) >= P) break;
            uint32_t idx = ix[e][p], rank = (rk[e][p >> 1] >> ((p & 1) * 16)) & 0xffffu;
            const uint32_t el = uint32_t(e) * RC_TPB + threadIdx.x;
            if (!ADD && SK_RC_LATERANK) { // contains: a segment's order is free (the probe ANDs)
                lrec[atomicAdd(&hist[idx >> RB], 1u)] = (idx << 12) | el;
                continue;
            }
            lrec[hist[idx >> RB] + rank] =
                ADD ? (idx << 13) | (el << 1) | (uint32_t(p) + 1 == P ? 1u : 0u) : (idx << 12) | el;
        }
    }
    __syncthreads();
    RC_STAMP(4);
    uint4 *dst = reinterpret_cast<uint4 *>(chunks + uint64_t(jb) * EPB * P);
    const uint4 *src = reinterpret_cast<const uint4 *>(lrec);
    if (!(SK_RC_ABL & 32) || ADD)
        for (uint32_t t = threadIdx.x; t < (tot + 3) / 4; t += RC_TPB) dst[t] = src[t];
    RC_STAMP(5);
}

// St (interleaved by SK_RC_STILE regions) -> S (region-major rows): one 128 x T tile of (block, region) entries per
// workgroup (16 KiB: a 4 KiB tile per workgroup left the copy launch-bound), both sides moved as 16-B vectors
// (4 consecutive entries of a block's T-region line in, 4 consecutive blocks of a region's row out; scalar when
// NB is not a multiple of 4, i.e. a small last piece)
#define RC_STJ 128
__global__ void __launch_bounds__(256) k_rc_stranspose(const uint32_t *__restrict__ St, uint32_t *__restrict__ S,
                                                       uint32_t NB, uint32_t NR) {
    constexpr uint32_t T = SK_RC_STILE, TJ = RC_STJ;
    static_assert(T == 1 || (T % 4 == 0 && TJ % 4 == 0), "16-B vectors on both sides"); // T = 1: never launched
    __shared__ uint32_t tile[TJ][T + 1];
    const uint32_t j0 = blockIdx.x * TJ, rt = blockIdx.y;
    for (uint32_t e = threadIdx.x; e < TJ * T / 4; e += 256) {
        const uint32_t jj = (4 * e) / T, rr = (4 * e) % T;
        if (j0 + jj < NB) {
            const uint4 v = *reinterpret_cast<const uint4 *>(St + (uint64_t(rt) * NB + j0 + jj) * T + rr);
            tile[jj][rr] = v.x;
            tile[jj][rr + 1] = v.y;
            tile[jj][rr + 2] = v.z;
            tile[jj][rr + 3] = v.w;
        }
    }
    __syncthreads();
    if ((NB & 3u) == 0) {
        for (uint32_t e = threadIdx.x; e < TJ * T / 4; e += 256) {
            const uint32_t rr = (4 * e) / TJ, jj = (4 * e) % TJ, r = rt * T + rr;
            if (r < NR && j0 + jj < NB) // NB, j0 and jj are multiples of 4: the 4 blocks are all < NB
                *reinterpret_cast<uint4 *>(S + uint64_t(r) * NB + j0 + jj) =
                    make_uint4(tile[jj][rr], tile[jj + 1][rr], tile[jj + 2][rr], tile[jj + 3][rr]);
        }
    } else {
        for (uint32_t e = threadIdx.x; e < TJ * T; e += 256) {
            const uint32_t rr = e / TJ, jj = e % TJ, r = rt * T + rr;
            if (r < NR && j0 + jj < NB) S[uint64_t(r) * NB + j0 + jj] = tile[jj][rr];
        }
    }
}

// regions of XCD group x = blockIdx % 8 are [x*q, (x+1)*q), taken in order
__device__ __forceinline__ uint32_t rc_region(uint32_t b, uint32_t NR) {
    uint32_t q = (NR + 7) / 8;
    return (b & 7u) * q + (b >> 3);
}

// One thread per (block, region) segment, RC_JB blocks at once: the segment's
// records are read as RC_SEGV aligned 16-B vectors (the segment starts at any
// word), so a lane issues 4 vector loads instead of one load per record; a
// segment that does not fit them (rare: > 13 records) finishes word by word.
// The region's own stream is issued before the segment loads and lands in
// LDS while they are in flight.
#ifndef RC_SEGV
#define RC_SEGV 4
#endif
#define RC_JB 2
__device__ __forceinline__ void rc_test(const uint8_t *fb, uint32_t x, uint8_t *ob) {
    uint32_t bit = x >> 12;
    if (!((fb[bit >> 3] >> (7u - (bit & 7u))) & 1u) && (!(SK_RC_ABL & 1) || x == 0xffffffffu)) ob[x & 0xfffu] = 0;
}
// Per thread: the segment-table words of every block it serves are loaded up front (with the region's own
// stream); then the record vectors of RC_JB segments are loaded one step ahead of the segments being tested,
// so a lane always has a step of loads in flight while it tests from LDS.
#define RC_SMAX 8 // blocks per thread: pieces of <= 32 M elements = 8192 blocks
#ifndef RC_PF
#define RC_PF 3   // steps of segment loads in flight per thread (2: one step ahead)
#endif
__device__ __forceinline__ void rc_load_seg(const uint32_t *chunks, uint64_t CH, uint32_t j, uint32_t seg,
                                            uint4 (&w)[RC_SEGV], uint32_t r = 0, uint32_t NB = 0, uint32_t NR = 1) {
    uint32_t st = seg & 0xffffu, cnt = seg >> 16;
#if SK_RC_ABL & 1024
    uint64_t w0 = (uint64_t(r) * NB + j) * CH / NR;
    const uint64_t wmax = uint64_t(NB) * CH - 4 * RC_SEGV - 4;
    w0 = (w0 < wmax ? w0 : wmax) & ~uint64_t(3);
    const uint4 *cv = reinterpret_cast<const uint4 *>(chunks + w0);
    if (j >= NB) cv = reinterpret_cast<const uint4 *>(chunks); // seg == 0: nothing read
#else
    (void)r;
    (void)NB;
    (void)NR;
    const uint4 *cv = reinterpret_cast<const uint4 *>(chunks + uint64_t(j) * CH) + (st >> 2);
#endif
    uint32_t nv = ((st & 3u) + cnt + 3u) >> 2; // vectors covering the segment
#if SK_RC_ABL & 2
    (void)cv;
#pragma unroll
    for (int q = 0; q < RC_SEGV; q++) {
        const uint32_t h = (seg ^ j) * 2654435761u + uint32_t(q) * 0x9e3779b9u;
        w[q] = uint32_t(q) < nv ? make_uint4(h, h * 3u, h * 5u, h * 7u) : make_uint4(0, 0, 0, 0);
    }
#else
#pragma unroll
    for (int q = 0; q < RC_SEGV; q++) w[q] = uint32_t(q) < nv ? cv[q] : make_uint4(0, 0, 0, 0);
#endif
}
__device__ __forceinline__ void rc_test_seg(const uint8_t *fb, const uint32_t *chunks, uint64_t CH, uint32_t j,
                                            uint32_t seg, const uint4 (&w)[RC_SEGV], uint8_t *out) {
    const uint32_t st = seg & 0xffffu, cnt = seg >> 16, o = st & 3u;
    uint8_t *ob = out + uint64_t(j) * RC_EPB;
    // word t of the vectors is a record of this segment iff o <= t < o + cnt
    constexpr uint32_t NW = 4 * RC_SEGV;
    const uint32_t end = o + cnt < NW ? o + cnt : NW, inreg = end - o;
#pragma unroll
    for (int q = 0; q < RC_SEGV; q++) {
        if (4 * q >= o && 4 * q < end) rc_test(fb, w[q].x, ob);
        if (4 * q + 1 >= o && 4 * q + 1 < end) rc_test(fb, w[q].y, ob);
        if (4 * q + 2 >= o && 4 * q + 2 < end) rc_test(fb, w[q].z, ob);
        if (4 * q + 3 >= o && 4 * q + 3 < end) rc_test(fb, w[q].w, ob);
    }
    if (cnt > inreg) { // long segment (rare): the rest word by word
        const uint32_t *cs = chunks + uint64_t(j) * CH + st;
        for (uint32_t s = inreg; s < cnt; s++) rc_test(fb, cs[s], ob);
    }
}
// Zero lists (SK_RC_ZL): a probe on a 0 bit no longer stores its element's reply byte (one random byte store per
// zero hit: ~19 M per 32 M piece at C3, a third of the probe's time, r04 ablation).  The workgroup appends the
// element's piece-local index to an LDS list instead (one LDS atomic per wave and step); at the end it counting-
// sorts the list by reply group (RC_GB hash blocks) into the free region area and writes it as one contiguous run
// per region, Z[region][...], with the row GT[region][group] = start | count << 16.  k_bloom_rc_zero then takes
// one reply group per workgroup: the group's zero entries from every region go into an LDS byte map, and the
// replies are ANDed in as coalesced 16-B vectors.  A region with more zero hits than the list holds (a sparse
// filter) stores the rest directly, as before; the AND keeps those.
#ifndef SK_RC_ZL
#define SK_RC_ZL 1
#endif
#define RC_GB 16                         // hash blocks per reply group: 64 Ki replies, a 64 KiB LDS map
#define RC_NG (RC_SMAX * RC_TPB / RC_GB) // reply groups per piece (<= 512)
#ifndef RC_ZCAP
#define RC_ZCAP 7424                     // zero-list entries per region (LDS beside the 128 KiB region)
#endif
static_assert((1u << (RC_RB - 3)) >= RC_ZCAP * 4, "the sorted list fits the region area");
// SK_RC_TV: the probe's word tests without branches, and the wave scan of the zero-hit counts on DPP row shifts and
// broadcasts (6 adds) instead of six shuffles through LDS
#ifndef SK_RC_TV
#define SK_RC_TV 1
#endif
// inclusive sum over the 64 lanes of a wave: row_shr 1, 2, 4, 8 inside each row of 16, then row_bcast 15 and 31
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xf, 0xf, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xf, 0xf, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xf, 0xf, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xf, 0xf, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xa, 0xf, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xc, 0xf, false));
    return x;
}
// the zero hits of one segment (the words the unrolled test found on 0 bits): the wave's counts are scanned, one
// lane reserves the wave's slots, and every lane writes its entries; entries past the list's end store directly
__device__ __forceinline__ void rc_test_seg_zl(const uint8_t *fb, const uint32_t *chunks, uint64_t CH, uint32_t j,
                                               uint32_t seg, const uint4 (&w)[RC_SEGV], uint8_t *out, uint32_t *zl,
                                               uint32_t *zn, uint32_t *gt_row) {
    const uint32_t st = seg & 0xffffu, cnt = seg >> 16, o = st & 3u;
    constexpr uint32_t NW = 4 * RC_SEGV;
    const uint32_t end = o + cnt < NW ? o + cnt : NW, inreg = end - o;
    auto zero = [&](uint32_t x) {
        const uint32_t bit = x >> 12;
        return !((fb[bit >> 3] >> (7u - (bit & 7u))) & 1u);
    };
    uint32_t mask = 0;
#if SK_RC_ABL & 2048
    // timing probe: no word tests (the loads stay live; ~1 in 10 records reported zero)
    (void)end;
    (void)zero;
    mask = ((w[0].x ^ w[1].y ^ w[2].z ^ w[3].w) % 10u == 0u ? 1u : 0u) << o;
#elif SK_RC_TV
    // every word tested without a branch (a word outside the segment reads some byte of the region: x >> 15 <
    // 128 Ki), then masked to the segment's words [o, end)
    auto zb = [&](uint32_t x) { return ((uint32_t(fb[x >> 15]) << ((x >> 12) & 7u)) & 0x80u) ^ 0x80u; };
#pragma unroll
    for (int q = 0; q < RC_SEGV; q++) {
        const uint32_t t = 4u * uint32_t(q);
        mask |= (zb(w[q].x) | zb(w[q].y) << 1 | zb(w[q].z) << 2 | zb(w[q].w) << 3) >> 7 << t;
    }
    mask &= ((1u << end) - 1u) & ~((1u << o) - 1u); // end <= 16
    (void)zero;
#else
#pragma unroll
    for (int q = 0; q < RC_SEGV; q++) {
        const uint32_t t = 4u * uint32_t(q);
        if (t >= o && t < end && zero(w[q].x)) mask |= 1u << t;
        if (t + 1 >= o && t + 1 < end && zero(w[q].y)) mask |= 2u << t;
        if (t + 2 >= o && t + 2 < end && zero(w[q].z)) mask |= 4u << t;
        if (t + 3 >= o && t + 3 < end && zero(w[q].w)) mask |= 8u << t;
    }
#endif
#if SK_RC_ABL & 4096
    // timing probe: no zero-list scan or entries (the hits are folded into one word)
    if (mask == (seg ^ 0x5bd1e995u)) zl[0] = j; // (a condition the compiler cannot fold away)
    return;
#endif
    const uint32_t k = __popc(mask);
#if SK_RC_TV
    const uint32_t x = wave_incl_scan(k);
    // the wave's total (uniform) reserved by lane 0 (every lane of the wave is active here)
    const uint32_t tot = uint32_t(__builtin_amdgcn_readlane(int(x), 63));
    uint32_t base = 0;
    if (tot) {
        if ((threadIdx.x & 63u) == 0u) base = atomicAdd(zn, tot);
        base = uint32_t(__builtin_amdgcn_readlane(int(base), 0));
    }
    base += x - k;
    {
        // the wave's entries are in lane (= block) order and its 64 blocks are 4 whole reply groups (RC_GB = 16), so
        // each group's entries are one run of the list: GT[region][group] = start | count << 16, clipped at the
        // list's end (entries past it are stored directly)
        static_assert(RC_GB == 16, "4 reply groups per wave");
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t g0 = uint32_t(__builtin_amdgcn_readlane(int(base), 0)),
                       g1 = uint32_t(__builtin_amdgcn_readlane(int(base), 16)),
                       g2 = uint32_t(__builtin_amdgcn_readlane(int(base), 32)),
                       g3 = uint32_t(__builtin_amdgcn_readlane(int(base), 48)),
                       ge = uint32_t(__builtin_amdgcn_readlane(int(base + k), 63));
        if (lane < 4) {
            uint32_t a = lane == 0 ? g0 : lane == 1 ? g1 : lane == 2 ? g2 : g3;
            uint32_t b = lane == 0 ? g1 : lane == 1 ? g2 : lane == 2 ? g3 : ge;
            a = a < RC_ZCAP ? a : RC_ZCAP;
            b = b < RC_ZCAP ? b : RC_ZCAP;
            gt_row[((j - lane) >> 4) + lane] = a | ((b - a) << 16);
        }
    }
#else
    (void)gt_row;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t x = k;
#pragma unroll
    for (int s2 = 1; s2 < 64; s2 <<= 1) {
        const uint32_t y = __shfl_up(x, s2);
        if (lane >= uint32_t(s2)) x += y;
    }
    uint32_t base = 0;
    if (lane == 63 && x) base = atomicAdd(zn, x);
    base = __shfl(base, 63) + (x - k);
#endif
    const uint32_t e0 = j * RC_EPB;
    uint8_t *ob = out + uint64_t(j) * RC_EPB;
#if SK_RC_TV
    if (tot == 0 || uint32_t(__builtin_amdgcn_readlane(int(base + k), 63)) <= RC_ZCAP) {
        // uniform: all of the wave's entries fit (or there are none).  Every word is written, a hit to its list slot
        // and a miss to the lane's spare slot past the list: no branches, and the 64 spare slots are distinct words
        if (tot) {
            const uint32_t spare = RC_ZCAP + (threadIdx.x & 63u);
            uint32_t pos = base;
            auto put1 = [&](uint32_t word, uint32_t t) {
                const uint32_t hit = (mask >> t) & 1u;
                zl[hit ? pos : spare] = (e0 & ~0xfffu) | (word & 0xfffu);
                pos += hit;
            };
#pragma unroll
            for (int q = 0; q < RC_SEGV; q++) {
                const uint32_t t = 4u * uint32_t(q);
                put1(w[q].x, t);
                put1(w[q].y, t + 1);
                put1(w[q].z, t + 2);
                put1(w[q].w, t + 3);
            }
        }
        if (cnt > inreg) { // long segment (rare): the rest word by word, direct stores
            const uint32_t *cs = chunks + uint64_t(j) * CH + st;
            for (uint32_t s2 = inreg; s2 < cnt; s2++) rc_test(fb, cs[s2], ob);
        }
        return;
    }
#endif
    auto put = [&](uint32_t word) {
        const uint32_t el = word & 0xfffu;
        if (base < RC_ZCAP) zl[base] = e0 + el;
        else ob[el] = 0;
        base++;
    };
#pragma unroll
    for (int q = 0; q < RC_SEGV; q++) {
        const uint32_t t = 4u * uint32_t(q);
        if (mask & (1u << t)) put(w[q].x);
        if (mask & (2u << t)) put(w[q].y);
        if (mask & (4u << t)) put(w[q].z);
        if (mask & (8u << t)) put(w[q].w);
    }
    if (cnt > inreg) { // long segment (rare): the rest word by word, direct stores
        const uint32_t *cs = chunks + uint64_t(j) * CH + st;
        for (uint32_t s2 = inreg; s2 < cnt; s2++) rc_test(fb, cs[s2], ob);
    }
}
__global__ void __launch_bounds__(RC_TPB) k_bloom_rc_probe(uint32_t NB, uint32_t NR, const uint32_t *__restrict__ S,
                                                           const uint32_t *__restrict__ chunks, uint32_t P,
                                                           const uint8_t *__restrict__ bits, uint64_t cap_bytes,
                                                           uint8_t *__restrict__ out, uint32_t *__restrict__ Z,
                                                           uint32_t *__restrict__ GT) {
    __shared__ uint4 filt[(1u << (RC_RB - 3)) / 16];
    constexpr uint32_t NV = (1u << (RC_RB - 3)) / 16, VPT = NV / RC_TPB;
    const uint32_t r = rc_region(blockIdx.x, NR);
    if (r >= NR) return; // uniform
#if SK_RC_ZL
    __shared__ uint32_t zl[RC_ZCAP + 64]; // + one spare word per lane (SK_RC_TV)
    __shared__ uint32_t zn;
    if (threadIdx.x == 0) zn = 0;
#if !SK_RC_TV
    __shared__ uint32_t gcnt[RC_NG];
    __shared__ uint32_t wsum[RC_TPB / 64];
    for (uint32_t g = threadIdx.x; g < RC_NG; g += RC_TPB) gcnt[g] = 0;
#endif
#else
    (void)Z;
    (void)GT;
#endif
    const uint64_t b0 = uint64_t(r) << (RC_RB - 3);
    const uint4 *src = reinterpret_cast<const uint4 *>(bits + b0);
    {
        uint4 fv[VPT];
#pragma unroll
        for (uint32_t q = 0; q < VPT; q++) { // bytes past the buffer read as 0 (they are past the string)
            uint32_t v = threadIdx.x + q * RC_TPB;
#if SK_RC_ABL & 4
            fv[q] = make_uint4(~0u, ~((v * 2654435761u) & 0x01010101u), ~0u, ~(r & 0x10u)); // ~1 in 64 bits 0
            (void)src;
#else
            fv[q] = b0 + uint64_t(v) * 16 < cap_bytes ? ld_nt(src + v) : make_uint4(0, 0, 0, 0);
#endif
        }
        // NB <= RC_SMAX * RC_TPB (the host cuts batches into pieces)
        uint32_t seg0[RC_SMAX];
#pragma unroll
        for (int u = 0; u < RC_SMAX; u++) {
            uint32_t j = threadIdx.x + u * RC_TPB;
            seg0[u] = j < NB ? S[uint64_t(r) * NB + j] : 0u; // coalesced: S is region-major
        }
        // a ring of RC_PF steps of segment vectors: the first RC_PF - 1 steps are issued before the region's bits
        // land in LDS, and each step then issues the loads RC_PF - 1 steps ahead of the one it tests
        const uint64_t CH = uint64_t(RC_EPB) * P;
        uint4 w[RC_PF][RC_SEGV];
#pragma unroll
        for (int u = 0; u < RC_PF - 1; u++)
            rc_load_seg(chunks, CH, threadIdx.x + u * RC_TPB, seg0[u], w[u], r, NB, NR);
#pragma unroll
        for (uint32_t q = 0; q < VPT; q++) filt[threadIdx.x + q * RC_TPB] = fv[q];
        __syncthreads();
        const uint8_t *fb = reinterpret_cast<const uint8_t *>(filt);
#pragma unroll
        for (int u = 0; u < RC_SMAX; u++) {
            if (uint32_t(u) * RC_TPB >= NB) break; // no thread has a block at this step (uniform)
            if (u + RC_PF - 1 < RC_SMAX)
                rc_load_seg(chunks, CH, threadIdx.x + (u + RC_PF - 1) * RC_TPB, seg0[u + RC_PF - 1],
                            w[(u + RC_PF - 1) % RC_PF], r, NB, NR);
#if SK_RC_ZL
            rc_test_seg_zl(fb, chunks, CH, threadIdx.x + u * RC_TPB, seg0[u], w[u % RC_PF], out, zl, &zn,
                           GT + uint64_t(r) * RC_NG);
#else
            rc_test_seg(fb, chunks, CH, threadIdx.x + u * RC_TPB, seg0[u], w[u % RC_PF], out);
#endif
        }
    }
#if SK_RC_ABL & 8192
    return; // timing probe: no zero-list sort or write-back
#endif
#if SK_RC_ZL && SK_RC_TV
    __syncthreads(); // every test done: the list is complete, already in reply-group runs (GT written per wave)
    const uint32_t nz = zn < RC_ZCAP ? zn : RC_ZCAP;
    uint32_t *zdst = Z + uint64_t(r) * RC_ZCAP;
    for (uint32_t i = threadIdx.x; i < nz; i += RC_TPB) zdst[i] = zl[i];
#elif SK_RC_ZL
    __syncthreads(); // every test done: the list is complete and the region area is free
    const uint32_t nz = zn < RC_ZCAP ? zn : RC_ZCAP;
    constexpr uint32_t ZPT = (RC_ZCAP + RC_TPB - 1) / RC_TPB;
    constexpr uint32_t GSH = 12 + 4; // log2(RC_EPB * RC_GB)
    static_assert((RC_EPB * RC_GB) == (1u << GSH), "reply group size");
    uint32_t zv[ZPT], zr[ZPT];
#pragma unroll
    for (uint32_t q = 0; q < ZPT; q++) { // rank of each entry inside its group
        const uint32_t i = threadIdx.x + q * RC_TPB;
        zv[q] = i < nz ? zl[i] : 0u;
        zr[q] = i < nz ? atomicAdd(&gcnt[zv[q] >> GSH], 1u) : 0u;
    }
    __syncthreads();
    const uint32_t ng = (NB + RC_GB - 1) / RC_GB;
    const uint32_t c = threadIdx.x < ng ? gcnt[threadIdx.x] : 0u;
    uint32_t tot;
    const uint32_t gs = block_exscan<RC_TPB>(c, wsum, &tot);
    if (threadIdx.x < ng) {
        gcnt[threadIdx.x] = gs;
        GT[uint64_t(r) * RC_NG + threadIdx.x] = gs | (c << 16);
    }
    __syncthreads();
    uint32_t *sorted = reinterpret_cast<uint32_t *>(filt);
#pragma unroll
    for (uint32_t q = 0; q < ZPT; q++) {
        const uint32_t i = threadIdx.x + q * RC_TPB;
        if (i < nz) sorted[gcnt[zv[q] >> GSH] + zr[q]] = zv[q];
    }
    __syncthreads();
    uint32_t *zdst = Z + uint64_t(r) * RC_ZCAP;
    for (uint32_t i = threadIdx.x; i < nz; i += RC_TPB) zdst[i] = sorted[i];
#endif
}

#if SK_RC_ZL && SK_RC_TV
// SK_RC_PERSIST: the probe as one workgroup per CU looping over regions, with the next region's bits loaded into
// registers while the current region's segments are tested, so a region's load no longer stands between two
// regions (one workgroup fits a CU: the 128 KiB region plus the zero list).  The steps run as a rolled loop of two
// (a ring of two segment-vector sets, the segment-table words two steps ahead), which keeps the bits' 32 registers
// beside the ring inside the 128 a 1024-thread workgroup allows (a ring of three spills).
#ifndef SK_RC_PERSIST
#define SK_RC_PERSIST 1
#endif
#ifndef RC_PSLOTS
#define RC_PSLOTS 32 // workgroups per XCD group (8 x 32 = 256 = one per CU)
#endif
#ifndef SK_RC_PCOL
// 1: the probe reads the hash blocks' interleaved segment table St itself (no k_rc_stranspose): an XCD group starts
// on a multiple of SK_RC_STILE regions, so its 32 workgroups test one interleave group's regions at a time and the
// group's lines of St (a block's entries for those regions, 128 B) are fetched into that XCD's L2 once.  Measured
// slower (probe 0.684 -> 0.809 ms per 32 M for the transpose's ~0.03 ms, r05dg): 0 keeps the transpose
#define SK_RC_PCOL 0
#endif
#ifndef RC_PTPB
#define RC_PTPB 1024 // threads per workgroup
#endif
#ifndef RC_PRING
#define RC_PRING 2   // segment-vector sets in flight (3 at 512 threads)
#endif
// TPB threads (1024: 128 registers per lane, a ring of two; 512: 256 registers, a ring of three) per workgroup
template <uint32_t TPB, int RING>
__global__ void __launch_bounds__(TPB) k_bloom_rc_probe_p(uint32_t NB, uint32_t NR, const uint32_t *__restrict__ S,
                                                          const uint32_t *__restrict__ chunks, uint32_t P,
                                                          const uint8_t *__restrict__ bits, uint64_t cap_bytes,
                                                          uint8_t *__restrict__ out, uint32_t *__restrict__ Z,
                                                          uint32_t *__restrict__ GT) {
    static_assert(RING == 2 || RING == 3, "segment-vector sets in flight");
    __shared__ uint4 filt[(1u << (RC_RB - 3)) / 16];
    __shared__ uint32_t zl[RC_ZCAP + 64]; // + one spare word per lane
    __shared__ uint32_t zn;
    constexpr uint32_t NV = (1u << (RC_RB - 3)) / 16, VPT = NV / TPB;
    // XCD group x = blockIdx % 8 owns regions [x*q, (x+1)*q); its nslot workgroups take them interleaved, so the
    // ~32 regions an XCD works on at once are neighbours (their segments share lines of the block chunks)
    const uint32_t xg = blockIdx.x & 7u, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
    const uint32_t q = SK_RC_PCOL ? ((NR + 7) / 8 + SK_RC_STILE - 1) / SK_RC_STILE * SK_RC_STILE : (NR + 7) / 8;
    auto region = [&](uint32_t i) -> uint32_t {
        const uint32_t t = slot + nslot * i, rr = xg * q + t;
        return t < q && rr < NR ? rr : NR;
    };
    uint32_t r = region(0);
    if (r >= NR) return; // uniform
    uint4 fv[VPT];
    auto load_bits = [&](uint32_t rr) {
        const uint64_t b0 = uint64_t(rr) << (RC_RB - 3);
        const uint4 *src = reinterpret_cast<const uint4 *>(bits + b0);
#pragma unroll
        for (uint32_t q2 = 0; q2 < VPT; q2++) { // bytes past the buffer read as 0 (they are past the string)
            const uint32_t v = threadIdx.x + q2 * TPB;
            fv[q2] = b0 + uint64_t(v) * 16 < cap_bytes ? ld_nt(src + v) : make_uint4(0, 0, 0, 0);
        }
    };
    load_bits(r);
    if (threadIdx.x == 0) zn = 0;
    const uint64_t CH = uint64_t(RC_EPB) * P;
    const uint8_t *fb = reinterpret_cast<const uint8_t *>(filt);
    const uint32_t nsteps = (NB + TPB - 1) / TPB; // NB <= RC_SMAX * RC_TPB
    for (uint32_t i = 0; r < NR; i++) {
        const uint32_t *Srow = S + uint64_t(r) * NB;
        auto seg_of = [&](uint32_t u) -> uint32_t { // this thread's segment-table word of step u (0 past the end)
            const uint32_t j = threadIdx.x + u * TPB;
            if (SK_RC_PCOL) return u < nsteps && j < NB ? S[rc_sidx(r, j, NB)] : 0u;
            return u < nsteps && j < NB ? Srow[j] : 0u;
        };
        auto ld = [&](uint32_t u, uint32_t sg, uint4 (&w)[RC_SEGV]) { // sg = 0 past the end: nothing read
            rc_load_seg(chunks, CH, threadIdx.x + u * TPB, sg, w);
        };
        uint32_t *gt = GT + uint64_t(r) * RC_NG;
        auto test = [&](uint32_t u, uint32_t sg, const uint4 (&w)[RC_SEGV]) {
            if (u < nsteps) // uniform
                rc_test_seg_zl(fb, chunks, CH, threadIdx.x + u * TPB, sg, w, out, zl, &zn, gt);
        };
        uint4 wa[RC_SEGV], wb[RC_SEGV];
        uint32_t sa = seg_of(0), sb = seg_of(1);
        ld(0, sa, wa);
        if constexpr (RING == 3) ld(1, sb, wb);
#pragma unroll
        for (uint32_t q2 = 0; q2 < VPT; q2++) filt[threadIdx.x + q2 * TPB] = fv[q2];
        const uint32_t rn = region(i + 1);
        if (rn < NR) load_bits(rn); // uniform: in flight while this region is tested
        __syncthreads();            // the region's bits staged; the list empty
        if constexpr (RING == 2) {
#pragma unroll 1
            for (uint32_t u = 0; u < nsteps; u += 2) { // step u from wa, u + 1 from wb; loads one step ahead
                const uint32_t s2 = seg_of(u + 2);
                ld(u + 1, sb, wb);
                test(u, sa, wa);
                const uint32_t s3 = seg_of(u + 3);
                ld(u + 2, s2, wa);
                test(u + 1, sb, wb);
                sa = s2;
                sb = s3;
            }
        } else {
            uint4 wc[RC_SEGV];
            uint32_t sc = seg_of(2);
#pragma unroll 1
            for (uint32_t u = 0; u < nsteps; u += 3) { // steps u, u + 1, u + 2 from wa, wb, wc; loads two ahead
                const uint32_t s3 = seg_of(u + 3);
                ld(u + 2, sc, wc);
                test(u, sa, wa);
                const uint32_t s4 = seg_of(u + 4);
                ld(u + 3, s3, wa);
                test(u + 1, sb, wb);
                const uint32_t s5 = seg_of(u + 5);
                ld(u + 4, s4, wb);
                test(u + 2, sc, wc);
                sa = s3;
                sb = s4;
                sc = s5;
            }
        }
        __syncthreads(); // every test done: the list complete (in reply-group runs), the bits free
        const uint32_t nz = zn < RC_ZCAP ? zn : RC_ZCAP;
        uint32_t *zdst = Z + uint64_t(r) * RC_ZCAP;
        for (uint32_t t = threadIdx.x; t < nz; t += TPB) zdst[t] = zl[t];
        __syncthreads(); // every thread has read zn and the list
        if (threadIdx.x == 0) zn = 0;
        r = rn;
    }
}
#endif

// One reply group (RC_GB hash blocks, 64 Ki elements) per workgroup: its zero entries from every region's list
// (GT[region][group] names the run) clear bits of an 8 KiB LDS bitmap of the group's replies, which is then ANDed
// into out with 16-B vectors.  Each thread's run descriptors are loaded up front (independent loads in flight), and
// groups of one XCD are consecutive (speed only): their runs of one region are neighbours.
#ifndef RC_ZTPB
#define RC_ZTPB 512
#endif
__global__ void __launch_bounds__(RC_ZTPB) k_bloom_rc_zero(uint32_t NB, uint32_t NR, uint64_t n,
                                                           const uint32_t *__restrict__ Z,
                                                           const uint32_t *__restrict__ GT,
                                                           uint8_t *__restrict__ out) {
    constexpr uint32_t GE = RC_EPB * RC_GB; // replies per group
    constexpr uint32_t RPT = RC_NRMAX / RC_ZTPB;
    __shared__ uint32_t bm[GE / 32];
    const uint32_t ng = (NB + RC_GB - 1) / RC_GB;
    const uint32_t g = rc_region(blockIdx.x, ng);
    if (g >= ng) return; // uniform
    uint32_t t[RPT];
#pragma unroll
    for (uint32_t q = 0; q < RPT; q++) {
        const uint32_t rr = threadIdx.x + q * RC_ZTPB;
        t[q] = rr < NR ? GT[uint64_t(rr) * RC_NG + g] : 0u;
    }
    for (uint32_t v = threadIdx.x; v < GE / 32; v += RC_ZTPB) bm[v] = ~0u;
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < RPT; q++) {
        const uint32_t rr = threadIdx.x + q * RC_ZTPB, st = t[q] & 0xffffu, c = t[q] >> 16;
        const uint32_t *zs = Z + uint64_t(rr) * RC_ZCAP + st;
        uint32_t i = 0;
        for (; i + 4 <= c; i += 4) { // four list loads in flight
            const uint32_t a0 = zs[i] & (GE - 1), a1 = zs[i + 1] & (GE - 1), a2 = zs[i + 2] & (GE - 1),
                           a3 = zs[i + 3] & (GE - 1);
            atomicAnd(&bm[a0 >> 5], ~(1u << (a0 & 31u)));
            atomicAnd(&bm[a1 >> 5], ~(1u << (a1 & 31u)));
            atomicAnd(&bm[a2 >> 5], ~(1u << (a2 & 31u)));
            atomicAnd(&bm[a3 >> 5], ~(1u << (a3 & 31u)));
        }
        for (; i < c; i++) {
            const uint32_t e = zs[i] & (GE - 1);
            atomicAnd(&bm[e >> 5], ~(1u << (e & 31u)));
        }
    }
    __syncthreads();
    const uint64_t e0 = uint64_t(g) * GE;
    const uint64_t ne = n - e0 < GE ? n - e0 : GE;
    uint8_t *ob = out + e0;
    // reply byte i &= bit i: 16 replies per 16-B vector from one 16-bit piece of the bitmap
    auto spread = [](uint32_t b4) { // 4 bits -> 4 bytes of 0 / 1
        return (b4 & 1u) | ((b4 & 2u) << 7) | ((b4 & 4u) << 14) | ((b4 & 8u) << 21);
    };
    if ((reinterpret_cast<uintptr_t>(ob) & 15u) == 0) {
        for (uint32_t v = threadIdx.x; v < ne / 16; v += RC_ZTPB) {
            const uint32_t w16 = (bm[v >> 1] >> ((v & 1u) * 16u)) & 0xffffu;
            const uint4 a = reinterpret_cast<const uint4 *>(ob)[v];
            reinterpret_cast<uint4 *>(ob)[v] = make_uint4(a.x & spread(w16 & 15u), a.y & spread((w16 >> 4) & 15u),
                                                          a.z & spread((w16 >> 8) & 15u), a.w & spread(w16 >> 12));
        }
        for (uint32_t i = uint32_t(ne / 16) * 16 + threadIdx.x; i < ne; i += RC_ZTPB)
            ob[i] &= uint8_t((bm[i >> 5] >> (i & 31u)) & 1u);
    } else {
        for (uint32_t i = threadIdx.x; i < ne; i += RC_ZTPB) ob[i] &= uint8_t((bm[i >> 5] >> (i & 31u)) & 1u);
    }
}

// ---------------------------------------------- Bloom add, region schedule
// The add side of the region schedule (the rocPRIM sort path is left for k > RC_PMAX and for the rare piece with
// a segment longer than RA_SEGMAX, i.e. one element repeated hundreds of times in one block):
//   k_bloom_rc_hash<true>  as for contains, with all k probes, 4096 (k <= RA_K4) or 2048 elements per block, records
//                          bit-in-region << 12 | element-in-block << 1 | (probe == k-1); a segment longer than
//                          RA_SEGMAX raises *flag, and the host then takes the sort path for that piece.
//   k_bloom_ra_apply       one workgroup per region.  Reference semantics (M:RedissonBloomFilter.java:94-113,
//                          oracle bloom_add): the batch's SETBITs run in (element, probe) order, each replies the
//                          bit before it, and add() is true iff one of probes 0..k-2 replied 0.  So a probe is the
//                          setter of its bit iff the bit is 0 before the batch and no probe with a smaller
//                          (block, element) key touched it (two probes of one element on one bit share the key: the
//                          non-last one answers).
// A region's records are taken in windows of whole segments in block order (= batch order).  Inside a window the
// records of a bit are chained in LDS and each looks for a smaller key on its chain; the window's setters then set
// their bits, which later windows see.  A dense region (>= RA_DENSE records) keeps its 128 KiB of bits in LDS
// (one coalesced load and store); a sparse one reads and sets the words in place (device-scope atomics: a
// region's words belong to its workgroup alone).  Every probe extends the string to its byte (SETBIT grows it).
#define RA_CAP 8192   // records per window (LDS)
#define RA_HT 4096    // chain heads
#define RA_DENSE 1024 // records from which the region's bits are staged in LDS
#ifndef RA_JPT
#define RA_JPT 4      // blocks per thread (block j = q * RC_TPB + thread): pieces of <= 4096 blocks (8 M elements)
#endif
#define RA_NONE 0xffffffffu
#ifndef RA_GQ
#define RA_GQ 8       // record loads in flight per thread in a window's gather (RA_RPT: all of them)
#endif
#ifndef RA_SKIPSET
#define RA_SKIPSET 1  // records on bits already set are not chained
#endif
#define RA_RPT (RA_CAP / RC_TPB)
#ifndef SK_RA_OL
#define SK_RA_OL 1    // add replies through one lists (k_bloom_ra_one) instead of a random byte store per new element
#endif
#define RA_GSH 16     // one list groups: 64 Ki elements of the piece (the reply bytes one k_bloom_ra_one workgroup writes)
#define RA_NG 256     // groups per piece (<= 4096 blocks x 4096 elements / 64 Ki)
static_assert(RA_CAP >= 2 * RA_SEGMAX && RA_CAP % RC_TPB == 0 && RA_CAP < 0xffff, "windows: u16 links");
static_assert(RA_JPT * RC_TPB * 4096ull <= (uint64_t(RA_NG) << RA_GSH), "one-list groups of a piece");
static_assert(RA_JPT * RC_TPB <= 65536, "block numbers: u16 in the window, 16 bits of the order key");

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}
__device__ __forceinline__ uint32_t ra_mask(uint32_t b) { return (0x80u >> (b & 7u)) << (((b >> 3) & 3u) * 8u); }
template <uint32_t AEPB> __device__ __forceinline__ uint32_t ra_key(uint32_t blk, uint32_t x) {
    return (blk << (AEPB == 4096 ? 12 : 11)) | ((x >> 1) & (AEPB - 1));
}

template <uint32_t AEPB>
__global__ void __launch_bounds__(RC_TPB) k_bloom_ra_apply(uint32_t NB, uint32_t NR, const uint32_t *__restrict__ S,
                                                           const uint32_t *__restrict__ chunks, uint32_t P,
                                                           uint8_t *bits, uint64_t cap_bytes,
                                                           unsigned long long *d_len, uint8_t *__restrict__ out,
                                                           const uint32_t *stop, uint32_t piece,
                                                           int big, uint32_t *__restrict__ Z, uint32_t *zalloc,
                                                           uint64_t *__restrict__ GT) {
    constexpr uint32_t NW = 1u << (RA_RB - 5); // u32 words per region
    __shared__ uint32_t filt[NW];
    __shared__ uint32_t rec[RA_CAP];
    __shared__ uint16_t blk[RA_CAP];
    __shared__ uint16_t nxt[RA_CAP];
    __shared__ uint32_t head[RA_HT];
    __shared__ uint32_t wsum[RC_TPB / 64];
    __shared__ uint32_t wbase, wend, maxb;
#if SK_RA_OL
    // one list: the piece-local indexes of the elements this region makes "new" (a setter among probes 0..k-2), in
    // record order = block order, so each reply group is one run of the region's list (gfirst / glast); the run
    // table GT[group][region] tells k_bloom_ra_one where.  The list lives in Z from a slot range the workgroup
    // reserves (<= its records).
    __shared__ uint32_t wc[RA_RPT * (RC_TPB / 64)], gfirst[RA_NG], glast[RA_NG], zbase, wtot;
    uint32_t zn = 0, lastg = RA_NONE; // the region's list so far and its last entry's group (uniform, per thread)
    const uint32_t ng = uint32_t((uint64_t(NB) * AEPB + (1u << RA_GSH) - 1) >> RA_GSH);
#endif
    const uint32_t r = rc_region(blockIdx.x, NR);
    if (r >= NR || *stop <= piece) return; // uniform (stop: a hash pass of this or an earlier piece saw a long segment)
    const uint64_t b0 = uint64_t(r) << (RA_RB - 3);
    uint32_t *gw = reinterpret_cast<uint32_t *>(bits + b0);
    constexpr uint32_t VT = NW / 4 / RC_TPB;
    uint4 t[VT]; // big pieces: the region's bits are loaded while the segment table is scanned
    if (big) {
        const uint4 *src = reinterpret_cast<const uint4 *>(gw);
#pragma unroll
        for (uint32_t q = 0; q < VT; q++) { // no branch around the loads: all in flight
            const uint32_t v = threadIdx.x + q * RC_TPB;
            const bool ok = b0 + uint64_t(v) * 16 < cap_bytes;
            t[q] = src[ok ? v : 0u];
            if (!ok) t[q] = make_uint4(0, 0, 0, 0);
        }
    }
    const uint32_t CH = AEPB * P; // words per block chunk (NB * CH < 2^32: pieces of <= 16 M elements)
    uint32_t sg[RA_JPT], pre[RA_JPT], total = 0;
#pragma unroll
    for (int q = 0; q < RA_JPT; q++) {
        uint32_t j = uint32_t(q) * RC_TPB + threadIdx.x;
        sg[q] = j < NB ? S[uint64_t(r) * NB + j] : 0u;
    }
#pragma unroll
    for (int q = 0; q < RA_JPT; q++) { // segment positions in block order: row q = blocks q*RC_TPB..
        pre[q] = total;
        if (uint32_t(q) * RC_TPB >= NB) continue; // uniform
        uint32_t tq, e = block_exscan<RC_TPB>(sg[q] >> 16, wsum, &tq);
        pre[q] = total + e;
        total += tq;
    }
    if (total == 0) { // uniform: no probe in this region
#if SK_RA_OL
        for (uint32_t g = threadIdx.x; g < ng; g += RC_TPB) GT[uint64_t(g) * NR + r] = 0;
#endif
        return;
    }
#if SK_RA_OL
    for (uint32_t g = threadIdx.x; g < RA_NG; g += RC_TPB) gfirst[g] = RA_NONE;
    if (threadIdx.x == 0) zbase = atomicAdd(zalloc, total);
#endif
    const bool dense = big || total >= RA_DENSE;
    if (dense) { // bytes past the buffer read as 0 and are not written back
        uint4 *fv = reinterpret_cast<uint4 *>(filt);
        if (!big) {
            const uint4 *src = reinterpret_cast<const uint4 *>(gw);
#pragma unroll
            for (uint32_t q = 0; q < VT; q++) {
                const uint32_t v = threadIdx.x + q * RC_TPB;
                const bool ok = b0 + uint64_t(v) * 16 < cap_bytes;
                t[q] = src[ok ? v : 0u];
                if (!ok) t[q] = make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < VT; q++) fv[threadIdx.x + q * RC_TPB] = t[q];
    }
    for (uint32_t t = threadIdx.x; t < RA_HT; t += RC_TPB) head[t] = RA_NONE;
    if (threadIdx.x == 0) maxb = 0;
    uint32_t mymax = 0;
    bool anyset = false;
    constexpr uint32_t W = RA_CAP - RA_SEGMAX;
    for (uint32_t lo = 0; lo < ((SK_RC_ABL & 256) ? 0u : total); lo += W) {
        if (total <= W) { // one window: [0, total), known without the atomics (the usual case)
            if (threadIdx.x == 0) {
                wbase = 0;
                wend = total;
            }
            __syncthreads(); // bits staged, heads cleared
        } else {
            if (threadIdx.x == 0) {
                wbase = RA_NONE;
                wend = 0;
            }
            __syncthreads(); // (first window: bits staged, heads cleared)
            // the window = the segments starting in [lo, lo + W), laid out from the first one's start (a segment that
            // starts in the previous window belongs to it whole).  Reduced per thread, then per wave, then one LDS
            // atomic per wave: one atomic per segment on the same two words serialized ~8 k LDS atomics per window
            uint32_t mn = RA_NONE, mx = 0;
#pragma unroll
            for (int q = 0; q < RA_JPT; q++) {
                const uint32_t cnt = sg[q] >> 16;
                if (cnt == 0 || pre[q] < lo || pre[q] >= lo + W) continue;
                mn = pre[q] < mn ? pre[q] : mn;
                mx = pre[q] + cnt > mx ? pre[q] + cnt : mx;
            }
            mn = wave_min_u32(mn);
            mx = wave_max_u32(mx);
            if ((threadIdx.x & 63u) == 0 && mx) {
                atomicMin(&wbase, mn);
                atomicMax(&wend, mx);
            }
            __syncthreads();
        }
        const uint32_t base = wbase; // RA_NONE: no segment starts here (wend = 0, nw = 0)
        const uint32_t nw = base == RA_NONE ? 0u : wend - base; // <= W + RA_SEGMAX = RA_CAP
        // a record whose bit is already set (before the batch or by an earlier window) is never a setter, and a
        // record on an unset bit only looks for smaller keys on its own bit: the former stay off the chains
#pragma unroll
        for (int q = 0; q < RA_JPT; q++) { // owners write each record's chunk word index
            const uint32_t cnt = sg[q] >> 16;
            if (cnt == 0 || pre[q] < lo || pre[q] >= lo + W) continue;
            const uint32_t j = uint32_t(q) * RC_TPB + threadIdx.x, d = pre[q] - base;
            const uint32_t src = j * CH + (sg[q] & 0xffffu);
#pragma unroll 1
            for (uint32_t u = 0; u < cnt; u++) {
                rec[d + u] = src + u;
                blk[d + u] = uint16_t(j);
            }
        }
        __syncthreads();
        // this thread's records u = thread + q * RC_TPB stay in registers (xs) with their bit's word (ws) from the
        // link to the set: the scan and the set read no record back, and every load of a step is in flight at once
        uint32_t xs[RA_RPT], ws[RA_RPT];
#pragma unroll
        for (uint32_t g = 0; g < RA_RPT; g += RA_GQ) { // RA_GQ gathers in flight
#pragma unroll
            for (uint32_t q = 0; q < RA_GQ; q++) {
                const uint32_t u = threadIdx.x + (g + q) * RC_TPB;
#if SK_RC_ABL & 128
                xs[g + q] = u < nw ? chunks[(uint64_t(r) * W + lo + u) % (uint64_t(NB) * CH)] : 0u;
#else
                xs[g + q] = u < nw ? chunks[rec[u]] : 0u;
#endif
            }
#pragma unroll
            for (uint32_t q = 0; q < RA_GQ; q++) {
                const uint32_t u = threadIdx.x + (g + q) * RC_TPB, b = xs[g + q] >> 13;
                ws[g + q] = ~0u;
                if (u < nw) {
                    rec[u] = xs[g + q];
                    ws[g + q] = dense ? filt[b >> 5]
                                      : __hip_atomic_load(gw + (b >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
#pragma unroll
            for (uint32_t q = 0; q < RA_GQ; q++) {
                const uint32_t u = threadIdx.x + (g + q) * RC_TPB, b = xs[g + q] >> 13;
                if (u >= nw) continue;
                mymax = b > mymax ? b : mymax;
                if (RA_SKIPSET && (ws[g + q] & ra_mask(b))) nxt[u] = 0xffffu;
                else nxt[u] = uint16_t(atomicExch(&head[b & (RA_HT - 1)], u));
            }
        }
        __syncthreads();
        uint32_t first = 0; // bit q: record q of this thread sets its bit
#if SK_RA_OL
        uint32_t one = 0; // bit q: record q makes its element new
#endif
#pragma unroll
        for (uint32_t q = 0; q < RA_RPT; q++) {
            const uint32_t u = threadIdx.x + q * RC_TPB, xu = xs[q], b = xu >> 13;
            if (u >= nw || (ws[q] & ra_mask(b))) continue; // set before this probe: not a setter
            const uint32_t key = ra_key<AEPB>(blk[u], xu);
            bool f = true;
            uint32_t steps = 0; // a chain holds <= nw records: a longer walk is a broken chain, reported, never a hang
            for (uint32_t v = (SK_RC_ABL & 512) ? RA_NONE : head[b & (RA_HT - 1)]; v < RA_CAP && f; v = nxt[v]) { // RA_NONE / 0xffff end a chain
                const uint32_t xv = rec[v];
                if ((xv >> 13) == b && ra_key<AEPB>(blk[v], xv) < key) f = false;
                if (++steps > RA_CAP) {
                    atomicOr(const_cast<uint32_t *>(stop) + 2, 1u);
                    break;
                }
            }
            if (!f) continue;
            first |= 1u << q;
#if SK_RA_OL
            if (!(xu & 1u)) one |= 1u << q;
#else
            if (!(xu & 1u) && (!(SK_RC_ABL & 64) || xu == 0xfffffffeu)) out[uint64_t(blk[u]) * AEPB + ((xu >> 1) & (AEPB - 1))] = 1;
#endif
        }
        __syncthreads(); // every probe of the window has read the bits
#if SK_RA_OL
        const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
        const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
        for (uint32_t q = 0; q < RA_RPT; q++) { // this window's new elements per (record row q, wave)
            const uint64_t bal = __ballot((one >> q) & 1u);
            if (lane == 0) wc[q * (RC_TPB / 64) + wv] = uint32_t(__popcll(bal));
        }
#endif
#pragma unroll
        for (uint32_t q = 0; q < RA_RPT; q++) {
            const uint32_t u = threadIdx.x + q * RC_TPB, b = xs[q] >> 13;
            if (u >= nw) continue;
            if (first & (1u << q)) {
                anyset = true;
                if (dense) atomicOr(&filt[b >> 5], ra_mask(b));
                else __hip_atomic_fetch_or(gw + (b >> 5), ra_mask(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            head[b & (RA_HT - 1)] = RA_NONE;
        }
#if SK_RA_OL
        __syncthreads(); // the (row, wave) counts are in; the window's records are no longer read: rec is free
        if (threadIdx.x < 64) { // exclusive scan of the 128 counts in (row, wave) = record order
            const uint32_t a = wc[2 * threadIdx.x], c = wc[2 * threadIdx.x + 1];
            uint32_t x = a + c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o);
                if (threadIdx.x >= uint32_t(o)) x += y;
            }
            wc[2 * threadIdx.x] = x - a - c;
            wc[2 * threadIdx.x + 1] = x - c;
            if (threadIdx.x == 63) wtot = x;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < RA_RPT; q++) { // the window's new elements in record order into rec
            const uint64_t bal = __ballot((one >> q) & 1u);
            const uint32_t u = threadIdx.x + q * RC_TPB; // blk[] holds the window's blocks until its next fill
            if ((one >> q) & 1u)
                rec[wc[q * (RC_TPB / 64) + wv] + uint32_t(__popcll(bal & below))] =
                    uint32_t(blk[u]) * AEPB + ((xs[q] >> 1) & (AEPB - 1));
        }
        __syncthreads();
        { // appended to the list, group runs marked; rec is rewritten only after the next window's first barrier
            const uint32_t nt = wtot;
            for (uint32_t i = threadIdx.x; i < nt; i += RC_TPB) {
                const uint32_t e = rec[i], g = e >> RA_GSH;
                Z[zbase + zn + i] = e;
                if (i == 0 ? (zn == 0 || lastg != g) : (rec[i - 1] >> RA_GSH) != g) gfirst[g] = zn + i;
                if (i + 1 == nt || (rec[i + 1] >> RA_GSH) != g) glast[g] = zn + i + 1;
            }
            if (nt) {
                lastg = rec[nt - 1] >> RA_GSH;
                zn += nt;
            }
        }
#endif
    }
    mymax = wave_max_u32(mymax);
    if ((threadIdx.x & 63u) == 0) atomicMax(&maxb, mymax);
    const bool changed = __syncthreads_or(anyset);
#if SK_RA_OL
    for (uint32_t g = threadIdx.x; g < ng; g += RC_TPB)
        GT[uint64_t(g) * NR + r] = gfirst[g] == RA_NONE ? 0ull
                                                        : uint64_t(zbase + gfirst[g]) | uint64_t(glast[g] - gfirst[g]) << 32;
#endif
    if (threadIdx.x == 0) atomicMax(d_len, (unsigned long long)(b0 + (maxb >> 3) + 1));
    if (dense && changed) {
        uint4 *dst = reinterpret_cast<uint4 *>(gw);
        const uint4 *fv = reinterpret_cast<const uint4 *>(filt);
#pragma unroll
        for (uint32_t v = threadIdx.x; v < NW / 4; v += RC_TPB)
            if (b0 + uint64_t(v) * 16 < cap_bytes) dst[v] = fv[v];
    }
}

// One reply group (64 Ki elements of the piece) per workgroup: every region's run of the group's new elements sets
// bits of an 8 KiB LDS bitmap, then the group's reply bytes are written whole (16-B vectors: no partial lines).
// Replaces one random byte store per new element in k_bloom_ra_apply (their partial-line write-backs were ~1.5 GB
// of the apply's 2.1 GB written per 16 M piece).  A stopped piece (sort-path fallback) is left to the host.
#define RA_OTPB 1024
__global__ void __launch_bounds__(RA_OTPB) k_bloom_ra_one(uint32_t NR, uint64_t n, const uint32_t *__restrict__ Z,
                                                          uint64_t zcap, const uint64_t *__restrict__ GT,
                                                          uint8_t *__restrict__ out, const uint32_t *stop,
                                                          uint32_t piece) {
    constexpr uint32_t GE = 1u << RA_GSH, RPT = RA_NRMAX / RA_OTPB;
    __shared__ uint32_t bm[GE / 32];
    const uint32_t ng = uint32_t((n + GE - 1) >> RA_GSH), g = rc_region(blockIdx.x, ng);
    if (g >= ng || *stop <= piece) return; // uniform
    uint64_t t[RPT]; // this thread's run descriptors, every load in flight before the first run is read
#pragma unroll
    for (uint32_t q = 0; q < RPT; q++) {
        const uint32_t rr = threadIdx.x + q * RA_OTPB;
        t[q] = rr < NR ? GT[uint64_t(g) * NR + rr] : 0ull;
    }
    for (uint32_t v = threadIdx.x; v < GE / 32; v += RA_OTPB) bm[v] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < RPT; q++) {
        const uint32_t st = uint32_t(t[q]);
        uint32_t c = uint32_t(t[q] >> 32);
        if (uint64_t(st) + c > zcap) { // a run past the lists: reported, never read
            atomicOr(const_cast<uint32_t *>(stop) + 2, 2u);
            c = 0;
        }
        const uint32_t *zs = Z + st;
        uint32_t i = 0;
        for (; i + 4 <= c; i += 4) { // four loads in flight
            const uint32_t a0 = zs[i], a1 = zs[i + 1], a2 = zs[i + 2], a3 = zs[i + 3];
            atomicOr(&bm[(a0 & (GE - 1)) >> 5], 1u << (a0 & 31u));
            atomicOr(&bm[(a1 & (GE - 1)) >> 5], 1u << (a1 & 31u));
            atomicOr(&bm[(a2 & (GE - 1)) >> 5], 1u << (a2 & 31u));
            atomicOr(&bm[(a3 & (GE - 1)) >> 5], 1u << (a3 & 31u));
        }
        for (; i < c; i++) {
            const uint32_t e = zs[i] & (GE - 1);
            atomicOr(&bm[e >> 5], 1u << (e & 31u));
        }
    }
    __syncthreads();
    const uint64_t e0 = uint64_t(g) * GE;
    const uint64_t ne = n - e0 < GE ? n - e0 : GE;
    uint8_t *ob = out + e0;
    auto spread = [](uint32_t b4) { // 4 bits -> 4 bytes of 0 / 1
        return (b4 & 1u) | ((b4 & 2u) << 7) | ((b4 & 4u) << 14) | ((b4 & 8u) << 21);
    };
    if ((reinterpret_cast<uintptr_t>(ob) & 15u) == 0) {
        for (uint32_t v = threadIdx.x; v < ne / 16; v += RA_OTPB) {
            const uint32_t w16 = (bm[v >> 1] >> ((v & 1u) * 16u)) & 0xffffu;
            reinterpret_cast<uint4 *>(ob)[v] = make_uint4(spread(w16 & 15u), spread((w16 >> 4) & 15u),
                                                          spread((w16 >> 8) & 15u), spread(w16 >> 12));
        }
        for (uint32_t i = uint32_t(ne / 16) * 16 + threadIdx.x; i < ne; i += RA_OTPB)
            ob[i] = uint8_t((bm[i >> 5] >> (i & 31u)) & 1u);
    } else {
        for (uint32_t i = threadIdx.x; i < ne; i += RA_OTPB) ob[i] = uint8_t((bm[i >> 5] >> (i & 31u)) & 1u);
    }
}

// add, pass 1: all k probes -> key = idx << 32 | (elem*k + j)
__global__ void __launch_bounds__(256) k_bloom_probes(uint64_t n, const uint64_t *__restrict__ off,
                                                      const uint8_t *__restrict__ bytes, uint64_t size,
                                                      uint64_t magic, int k, uint64_t *__restrict__ keys) {
    __shared__ uint64_t lds[SK_STAGE_WORDS];
    uint64_t e0 = uint64_t(blockIdx.x) * blockDim.x, e1 = e0 + blockDim.x < n ? e0 + blockDim.x : n;
    uint64_t lo = off[e0], hi = off[e1];
    bool staged = stage_fits(lo, hi);
    uint32_t wbase = staged ? stage_keys(bytes, lo, hi, lds) : 0u;
    uint64_t i = e0 + threadIdx.x;
    if (i >= n) return;
    uint64_t o = off[i];
    uint32_t len = uint32_t(off[i + 1] - o);
    uint64_t h1, h2;
    if (staged) {
        LdsReader rd{lds, wbase + uint32_t(o - lo)};
        h1 = xxh64_r(rd, len);
        h2 = farm_uo64_r(rd, len);
    } else {
        bloom_hashes(bytes + o, len, &h1, &h2);
    }
    BloomIdx bi(h1, h2, size, magic);
    uint64_t pos = i * uint64_t(k);
    for (int j = 0; j < k; j++) {
        keys[pos + j] = (bi.r << 32) | (pos + j);
        bi.next(j);
    }
}

// Probe bit indexes of n elements, element-major: idx[i * np + j] = probe j of element i (RedissonBloomFilter.hash,
// M:RedissonBloomFilter.java:116-131), np <= k.  The input of the range-sharded filter's router
// (redisson_amd/cluster.py RangeShardedBloom): every probe travels to the GPU that owns its bit.
__global__ void __launch_bounds__(256) k_bloom_indexes(uint64_t n, const uint64_t *__restrict__ off,
                                                       const uint8_t *__restrict__ bytes, uint64_t size,
                                                       uint64_t magic, int np, uint64_t *__restrict__ idx) {
    __shared__ uint64_t lds[SK_STAGE_WORDS];
    uint64_t e0 = uint64_t(blockIdx.x) * blockDim.x, e1 = e0 + blockDim.x < n ? e0 + blockDim.x : n;
    uint64_t lo = off[e0], hi = off[e1];
    bool staged = stage_fits(lo, hi);
    uint32_t wbase = staged ? stage_keys(bytes, lo, hi, lds) : 0u;
    uint64_t i = e0 + threadIdx.x;
    if (i >= n) return;
    uint64_t o = off[i];
    uint32_t len = uint32_t(off[i + 1] - o);
    uint64_t h1, h2;
    if (staged) {
        LdsReader rd{lds, wbase + uint32_t(o - lo)};
        h1 = xxh64_r(rd, len);
        h2 = farm_uo64_r(rd, len);
    } else {
        bloom_hashes(bytes + o, len, &h1, &h2);
    }
    BloomIdx bi(h1, h2, size, magic);
    for (int j = 0; j < np; j++) {
        idx[i * uint64_t(np) + j] = bi.r;
        bi.next(j);
    }
}
// Host ingress in prefix form (sk_pfadd_ids_prefix, sk_bloom_*_prefix): element i = prefix ‖ suffix bytes
// [soff[i], soff[i+1]) (u32 offsets, relative to soff[0]); rebuilt here into the (u64 offsets, bytes) form every hash
// kernel reads.  One thread per element.
__global__ void __launch_bounds__(256) k_expand_prefix(uint64_t n, SkPrefix pre, const uint32_t *__restrict__ soff,
                                                       const uint8_t *__restrict__ sbytes, uint64_t *__restrict__ off,
                                                       uint8_t *__restrict__ bytes) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i > n) return;
    const uint32_t s0 = soff[0], a = soff[i] - s0;
    const uint64_t o = i * pre.len + a;
    off[i] = o;
    if (i == n) return;
    const uint32_t b = soff[i + 1] - s0;
    const uint8_t *pp = reinterpret_cast<const uint8_t *>(pre.w);
    for (uint32_t j = 0; j < pre.len; j++) bytes[o + j] = pp[j];
    for (uint32_t j = a; j < b; j++) bytes[o + pre.len + (j - a)] = sbytes[j];
}

// out[i] = AND(in[i * group .. i * group + take)) ^ invert: a contains reply (AND of probes 0..k-2) or an add reply
// (one of probes 0..k-2 replied 0) from per-probe bits in element-major order
__global__ void __launch_bounds__(256) k_reduce_groups_u8(uint64_t n, uint32_t group, uint32_t take, uint32_t invert,
                                                          const uint8_t *__restrict__ in, uint8_t *__restrict__ out) {
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
        const uint8_t *p = in + i * group;
        uint32_t a = 1;
        for (uint32_t j = 0; j < take; j++) a &= p[j] ? 1u : 0u;
        out[i] = uint8_t(a ^ invert);
    }
}

// add, pass 2 (after a stable sort on idx): the earliest probe of each bit
// sees the pre-batch bit; every later probe of the same bit sees 1.  Keys are
// sorted by bit index, so every probe of one 32-bit word is in one run and the
// run's first thread is the word's only writer: one plain load + store per
// touched word, no atomics.
__global__ void __launch_bounds__(256) k_bloom_apply(uint64_t m, const uint64_t *__restrict__ keys, uint8_t *bits,
                                                     uint64_t *d_len, int k, uint8_t *__restrict__ out) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint64_t key = keys[i], idx = key >> 32;
    uint32_t mask;
    uint32_t *wp = bit_word(bits, idx, &mask);
    if (i > 0) {
        uint32_t pm;
        if (bit_word(bits, keys[i - 1] >> 32, &pm) == wp) return; // not the first probe of this word
    }
    const uint32_t old = *wp;
    uint32_t set = 0;
    uint64_t prev_idx = ~0ull;
    for (uint64_t u = i; u < m; u++) {
        uint64_t ku = keys[u], iu = ku >> 32;
        uint32_t mu;
        if (bit_word(bits, iu, &mu) != wp) break;
        if (iu != prev_idx) { // the earliest probe of this bit (stable sort: batch order within a bit)
            prev_idx = iu;
            uint32_t pos = uint32_t(ku & 0xffffffffu), e = pos / uint32_t(k), j = pos - e * uint32_t(k);
            if (!(old & mu) && int(j) <= k - 2) out[e] = 1;
            set |= mu;
        }
    }
    if ((old | set) != old) *wp = old | set;
}

// ------------------------------------------------------------ bit strings
struct DirEnt {
    uint8_t *ptr;
    uint64_t len;
    uint64_t cap;
};

__global__ void __launch_bounds__(256) k_getbit_multi(uint64_t n, const uint32_t *__restrict__ sid,
                                                      const uint64_t *__restrict__ offs,
                                                      const DirEnt *__restrict__ dir, uint8_t *__restrict__ out) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s = sid[i];
    if (s == 0xffffffffu) { // missing key
        out[i] = 0;
        return;
    }
    out[i] = uint8_t(get_bit(dir[s].ptr, dir[s].len, offs[i]));
}

__global__ void __launch_bounds__(256) k_getbit_single(uint64_t n, const uint64_t *__restrict__ offs,
                                                       const uint8_t *__restrict__ buf,
                                                       const uint64_t *__restrict__ d_len, uint8_t *__restrict__ out) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = uint8_t(get_bit(buf, *d_len, offs[i]));
}

// SETBIT, pass 1: key = (string id << 36 | offset) sorted stably with the
// command index as value; pass 2: segment heads walk the ops in order.
__global__ void __launch_bounds__(256) k_setbit_keys(uint64_t n, const uint32_t *__restrict__ sid,
                                                     const uint64_t *__restrict__ offs, uint64_t *__restrict__ keys,
                                                     uint32_t *__restrict__ vals) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = (uint64_t(sid ? sid[i] : 0u) << 36) | offs[i];
    vals[i] = uint32_t(i);
}

__global__ void __launch_bounds__(256) k_setbit_apply(uint64_t n, const uint64_t *__restrict__ keys,
                                                      const uint32_t *__restrict__ vals,
                                                      const uint8_t *__restrict__ values, uint8_t value_all,
                                                      DirEnt *dir, uint8_t *__restrict__ out_old) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t key = keys[i];
        if (i == 0 || keys[i - 1] != key) {
            uint32_t s = uint32_t(key >> 36);
            uint64_t off = key & ((1ull << 36) - 1);
            DirEnt d = dir[s];
            uint32_t mask;
            uint32_t *wp = bit_word(d.ptr, off, &mask);
            uint32_t cur = (*wp & mask) ? 1u : 0u; // only this head writes this bit
            uint32_t c0 = cur;
            for (uint64_t j = i; j < n; j++) {
                if (j != i && keys[j] != key) break;
                uint32_t c = vals[j];
                if (out_old) out_old[c] = uint8_t(cur);
                cur = values ? (values[c] & 1u) : value_all;
            }
            if (cur != c0) {
                if (cur) atomicOr(wp, mask);
                else atomicAnd(wp, ~mask);
            }
        }
    }
}

// SETBIT of one value with no replies (SETBIT_VOID, M:RedissonBitSet.java:79-81): order-free.
// (the string length is raised by the host from the validated max offset)
__global__ void __launch_bounds__(256) k_setbit_void(uint64_t n, const uint64_t *__restrict__ offs, uint8_t *buf,
                                                     uint32_t value) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t off = offs[i];
        uint32_t mask;
        uint32_t *wp = bit_word(buf, off, &mask);
        if (value) atomicOr(wp, mask);
        else atomicAnd(wp, ~mask);
    }
}

// SETBIT_VOID in bulk (a dense batch: >= 2 ops per 128-B line of the string, C5's 64 M ops on 2^34 bits give 4): the
// ops sorted by 32 KiB region (a radix sort on the offset's region bits only), then one workgroup per region with
// ops stages the region in LDS, ORs (ANDs) its ops in with LDS atomics and writes it back.  The string streams in
// and out once instead of taking one random device-scope atomic per op; the result is the same set of bits (one
// value, so the ops commute).
#define SBV_RB 18   // region = 2^18 bits = 32 KiB of LDS
#define SBV_TPB 256
__global__ void __launch_bounds__(256) k_sbv_starts(uint64_t n, const uint64_t *__restrict__ keys, uint32_t NR,
                                                    uint32_t *__restrict__ start) {
    const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = uint32_t(keys[i] >> SBV_RB);
    const uint32_t rp = i ? uint32_t(keys[i - 1] >> SBV_RB) + 1u : 0u; // regions rp..r start at op i
    for (uint32_t q = rp; q <= r; q++) start[q] = uint32_t(i);
    if (i == n - 1)
        for (uint32_t q = r + 1; q <= NR; q++) start[q] = uint32_t(n);
}
__global__ void __launch_bounds__(SBV_TPB) k_sbv_apply(const uint64_t *__restrict__ keys,
                                                       const uint32_t *__restrict__ start, uint8_t *buf, uint64_t cap,
                                                       uint32_t value) {
    constexpr uint32_t RBYTES = 1u << (SBV_RB - 3), NV = RBYTES / 16, VPT = NV / SBV_TPB;
    __shared__ uint4 reg4[NV];
    const uint32_t r = blockIdx.x, lo = start[r], hi = start[r + 1];
    if (lo == hi) return; // uniform: no op in this region
    const uint64_t b0 = uint64_t(r) * RBYTES; // < cap: an op's byte lies in the region
    uint4 *src = reinterpret_cast<uint4 *>(buf + b0);
    const uint32_t nv = cap - b0 >= RBYTES ? NV : uint32_t((cap - b0) / 16); // cap is a multiple of 16
    if (nv == NV) { // a whole region: every load issued before the first LDS store
        uint4 t[VPT];
#pragma unroll
        for (uint32_t q = 0; q < VPT; q++) t[q] = src[threadIdx.x + q * SBV_TPB];
#pragma unroll
        for (uint32_t q = 0; q < VPT; q++) reg4[threadIdx.x + q * SBV_TPB] = t[q];
    } else {
        for (uint32_t v = threadIdx.x; v < nv; v += SBV_TPB) reg4[v] = src[v];
    }
    __syncthreads();
    uint32_t *w = reinterpret_cast<uint32_t *>(reg4);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += SBV_TPB) {
        const uint32_t lb = uint32_t(keys[i] - (uint64_t(r) << SBV_RB));
        const uint32_t byte = lb >> 3, mask = 1u << ((byte & 3u) * 8u + (7u - (lb & 7u))); // bit_word's layout
        if (value) atomicOr(&w[byte >> 2], mask);
        else atomicAnd(&w[byte >> 2], ~mask);
    }
    __syncthreads();
    for (uint32_t v = threadIdx.x; v < nv; v += SBV_TPB) src[v] = reg4[v];
}

// Dense SETBIT_VOID without a library sort (r05).  The ops of one value commute, so the apply needs each 32 KiB
// region's in-region bit offsets in any order, never a sorted op list.  Three passes of u32 records
// rec = (region % SBV_G) << 18 | bit-in-region, each written once and read once (the rocPRIM radix sort moved the 8-B
// offsets through two scatter passes and a histogram pass, ~45 % of the streaming rate):
//   k_sbv_part   per block of SBV_E ops: coarse bucket = region / SBV_G (8 MiB of string), LDS counting sort,
//                one coalesced chunk per block + S[bucket][block] = start | count << 16, tot[bucket][tile] += count
//   k_sbv_fine   per (tile of T blocks, bucket): the bucket's segments of the tile sorted by region in LDS and
//                stored as one piece at pbase[bucket][tile] with its region starts rs[bucket][tile][0..SBV_G]
//   k_sbv_runs   per region: its run from every tile's piece of its bucket applied to the region staged in LDS
#define SBV_E 16384   // ops per partition block (1024 threads x 16 in registers)
#define SBV_PTPB 1024
#define SBV_PPT (SBV_E / SBV_PTPB)
#define SBV_G 256     // regions per coarse bucket (record: 8 + 18 bits)
#define SBV_TMAX 256  // partition blocks per fine-sort tile (a call takes T = NC / 2: E * T / NC = 8 k records per
                      // (tile, bucket) piece on average, whatever the string's size)
#define SBV_FCAP 16384 // records a fine-sort workgroup places through LDS (more: placed by atomics, in pieces)
#define SBV_NCMAX 4096 // coarse buckets (strings <= 2^38 bits)
#define SBV_NTMAXR 256 // tiles per call
static_assert(SBV_E <= 65535 && SBV_G * (1u << SBV_RB) <= (1ull << 32), "record and segment packing");

// Records: u32 rec = (region % SBV_G) << 18 | bit-in-region (SETBIT_VOID: the ops of one value commute), or u64 with
// that word on top and seq << 1 | value below (SETBIT with replies, k_sbr_runs: the seq orders one bit's ops; the
// partition need not be stable).  `vrb` (optional): per-op base of the op's key in the call's virtual region space
// (0xffffffff: an op that failed validation, dropped); `vals` (optional): per-op values, else `value_all`.
template <typename R> __device__ __forceinline__ uint32_t sbv_key(R r) { return uint32_t(uint64_t(r) >> (sizeof(R) == 8 ? 32 : 0)); }
template <typename R> constexpr uint32_t sbv_fcap() { return sizeof(R) == 8 ? SBV_FCAP / 2 : SBV_FCAP; } // 64 KiB of LDS

template <typename R>
__global__ void __launch_bounds__(SBV_PTPB) k_sbv_part(uint64_t n, const uint64_t *__restrict__ offs,
                                                       const uint32_t *__restrict__ vrb, const uint8_t *__restrict__ vals,
                                                       uint32_t value_all, uint32_t NC, uint32_t NB, uint32_t T,
                                                       uint32_t ntile, R *__restrict__ chunks, uint32_t *__restrict__ S,
                                                       uint32_t *__restrict__ tot) {
    extern __shared__ uint32_t dyn32[];
    uint32_t *hist = dyn32;
    R *lrec = reinterpret_cast<R *>(dyn32 + ((NC + 3) & ~3u));
    __shared__ uint32_t wsum[SBV_PTPB / 64];
    const uint32_t blk = blockIdx.x;
    const uint64_t base = uint64_t(blk) * SBV_E;
    for (uint32_t b = threadIdx.x; b < NC; b += SBV_PTPB) hist[b] = 0;
    __syncthreads();
    R rec[SBV_PPT];
    uint32_t bk[SBV_PPT];
#pragma unroll
    for (int q = 0; q < SBV_PPT; q++) {
        const uint64_t i = base + uint64_t(q) * SBV_PTPB + threadIdx.x;
        bk[q] = 0xffffffffu;
        if (i < n) {
            const uint64_t o = offs[i];
            const uint32_t vb = vrb ? vrb[i] : 0u;
            if (vb != 0xffffffffu) {
                const uint32_t r = vb + uint32_t(o >> SBV_RB);
                const uint32_t key = ((r % SBV_G) << SBV_RB) | uint32_t(o & ((1u << SBV_RB) - 1u));
                if constexpr (sizeof(R) == 8)
                    rec[q] = (uint64_t(key) << 32) | (uint32_t(i) << 1) | (vals ? vals[i] & 1u : value_all);
                else
                    rec[q] = key;
                const uint32_t b = r / SBV_G;
                bk[q] = b | (atomicAdd(&hist[b], 1u) << 16); // rank < SBV_E
            }
        }
    }
    __syncthreads();
    // bucket starts: consecutive buckets per thread
    const uint32_t per = (NC + SBV_PTPB - 1) / SBV_PTPB;
    uint32_t s4 = 0;
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t b = threadIdx.x * per + k;
        s4 += b < NC ? hist[b] : 0u;
    }
    uint32_t total;
    uint32_t st = block_exscan<SBV_PTPB>(s4, wsum, &total);
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t b = threadIdx.x * per + k;
        if (b < NC) {
            const uint32_t c = hist[b];
            hist[b] = st;
            S[uint64_t(b) * NB + blk] = st | (c << 16);
            if (c) atomicAdd(&tot[uint64_t(b) * ntile + blk / T], c);
            st += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < SBV_PPT; q++)
        if (bk[q] != 0xffffffffu) lrec[hist[bk[q] & 0xffffu] + (bk[q] >> 16)] = rec[q];
    __syncthreads();
    R *dst = chunks + base;
    for (uint32_t t = threadIdx.x; t < total; t += SBV_PTPB) dst[t] = lrec[t];
}

template <typename R>
__global__ void __launch_bounds__(SBV_PTPB) k_sbv_fine(uint32_t NC, uint32_t NB, uint32_t T, uint32_t ntile,
                                                       const R *__restrict__ chunks,
                                                       const uint32_t *__restrict__ S,
                                                       const uint32_t *__restrict__ tot, uint32_t *__restrict__ pbase,
                                                       uint32_t *__restrict__ rs, R *__restrict__ out) {
    constexpr uint32_t FCAP = sbv_fcap<R>();
    __shared__ uint32_t segp[SBV_TMAX + 1], segs[SBV_TMAX], hist[SBV_G + 1], cur[SBV_G];
    __shared__ R sorted[FCAP];
    __shared__ uint32_t wsum[SBV_PTPB / 64];
    const uint32_t t = blockIdx.x, g = blockIdx.y, b0 = t * T;
    const uint32_t nb = (b0 + T < NB ? b0 + T : NB) - b0;
    // the piece's base: every record of the tile's earlier blocks, then the tile's records of buckets before g
    uint32_t acc = 0;
    for (uint32_t gg = threadIdx.x; gg < g; gg += SBV_PTPB) acc += tot[uint64_t(gg) * ntile + t];
    uint32_t pre;
    block_exscan<SBV_PTPB>(acc, wsum, &pre);
    const uint32_t base = t * T * SBV_E + pre; // < n < 2^32
    uint32_t len = 0, st0 = 0;
    if (threadIdx.x < nb) {
        const uint32_t e = S[uint64_t(g) * NB + b0 + threadIdx.x];
        st0 = e & 0xffffu;
        len = e >> 16;
    }
    uint32_t m;
    const uint32_t ex = block_exscan<SBV_PTPB>(len, wsum, &m);
    if (threadIdx.x < nb) {
        segp[threadIdx.x] = ex;
        segs[threadIdx.x] = st0;
    }
    if (threadIdx.x == 0) {
        segp[nb] = m;
        pbase[uint64_t(g) * ntile + t] = base;
    }
    for (uint32_t x = threadIdx.x; x <= SBV_G; x += SBV_PTPB) hist[x] = 0;
    __syncthreads();
    auto rec_at = [&](uint32_t x) { // record x of the piece: segment lo with segp[lo] <= x < segp[lo + 1]
        uint32_t lo = 0, hi = nb;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (segp[mid] <= x) lo = mid;
            else hi = mid;
        }
        return chunks[uint64_t(b0 + lo) * SBV_E + segs[lo] + (x - segp[lo])];
    };
    constexpr int RP = FCAP / SBV_PTPB;
    R rv[RP];
    uint32_t rk[RP];
    const bool small = m <= FCAP;
    if (small) {
#pragma unroll
        for (int q = 0; q < RP; q++) {
            const uint32_t x = threadIdx.x + q * SBV_PTPB;
            if (x < m) {
                rv[q] = rec_at(x);
                rk[q] = atomicAdd(&hist[sbv_key(rv[q]) >> SBV_RB], 1u);
            }
        }
    } else { // an oversized piece (skew): count first, place by atomics below
        for (uint32_t x = threadIdx.x; x < m; x += SBV_PTPB) atomicAdd(&hist[sbv_key(rec_at(x)) >> SBV_RB], 1u);
    }
    __syncthreads();
    uint32_t tot2;
    const uint32_t c = threadIdx.x < SBV_G ? hist[threadIdx.x] : 0u;
    const uint32_t gs = block_exscan<SBV_PTPB>(c, wsum, &tot2);
    uint32_t *rsp = rs + (uint64_t(g) * ntile + t) * (SBV_G + 1);
    if (threadIdx.x < SBV_G) {
        hist[threadIdx.x] = gs;
        cur[threadIdx.x] = gs;
        rsp[threadIdx.x] = gs;
    }
    if (threadIdx.x == 0) rsp[SBV_G] = m;
    __syncthreads();
    if (small) {
#pragma unroll
        for (int q = 0; q < RP; q++) {
            const uint32_t x = threadIdx.x + q * SBV_PTPB;
            if (x < m) sorted[hist[sbv_key(rv[q]) >> SBV_RB] + rk[q]] = rv[q];
        }
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < m; x += SBV_PTPB) out[uint64_t(base) + x] = sorted[x];
    } else {
        for (uint32_t x = threadIdx.x; x < m; x += SBV_PTPB) {
            const R r = rec_at(x);
            out[uint64_t(base) + atomicAdd(&cur[sbv_key(r) >> SBV_RB], 1u)] = r;
        }
    }
}

// one workgroup per region: its runs (one per tile) of its bucket's pieces, applied to the region in LDS
__global__ void __launch_bounds__(SBV_TPB) k_sbv_runs(uint32_t ntile, const uint32_t *__restrict__ pbase,
                                                      const uint32_t *__restrict__ rs,
                                                      const uint32_t *__restrict__ recs, uint8_t *buf, uint64_t cap,
                                                      uint32_t value) {
    constexpr uint32_t RBYTES = 1u << (SBV_RB - 3), NV = RBYTES / 16, VPT = NV / SBV_TPB;
    __shared__ uint4 reg4[NV];
    __shared__ uint32_t rlo[SBV_NTMAXR], rn[SBV_NTMAXR + 1];
    __shared__ uint32_t wsum[SBV_TPB / 64];
    const uint32_t r = blockIdx.x, g = r / SBV_G, rr = r % SBV_G;
    uint32_t lo = 0, c = 0;
    if (threadIdx.x < ntile) {
        const uint32_t *q = rs + (uint64_t(g) * ntile + threadIdx.x) * (SBV_G + 1) + rr;
        lo = pbase[uint64_t(g) * ntile + threadIdx.x] + q[0];
        c = q[1] - q[0];
    }
    uint32_t total;
    const uint32_t ex = block_exscan<SBV_TPB>(c, wsum, &total);
    if (total == 0) return; // uniform: no op in this region
    if (threadIdx.x < ntile) {
        rlo[threadIdx.x] = lo;
        rn[threadIdx.x] = ex;
    }
    if (threadIdx.x == 0) rn[ntile] = total;
    const uint64_t b0 = uint64_t(r) * RBYTES; // < cap: an op's byte lies in the region
    uint4 *src = reinterpret_cast<uint4 *>(buf + b0);
    const uint32_t nv = cap - b0 >= RBYTES ? NV : uint32_t((cap - b0) / 16); // cap is a multiple of 16
    if (nv == NV) { // a whole region: every load issued before the first LDS store
        uint4 tv[VPT];
#pragma unroll
        for (uint32_t q = 0; q < VPT; q++) tv[q] = src[threadIdx.x + q * SBV_TPB];
#pragma unroll
        for (uint32_t q = 0; q < VPT; q++) reg4[threadIdx.x + q * SBV_TPB] = tv[q];
    } else {
        for (uint32_t v = threadIdx.x; v < nv; v += SBV_TPB) reg4[v] = src[v];
    }
    __syncthreads();
    uint32_t *w = reinterpret_cast<uint32_t *>(reg4);
    for (uint32_t i = threadIdx.x; i < total; i += SBV_TPB) {
        uint32_t t = 0; // the run of record i (ntile <= SBV_NTMAXR: fixed-step search)
#pragma unroll
        for (uint32_t step = SBV_NTMAXR / 2; step; step >>= 1)
            if (t + step < ntile && rn[t + step] <= i) t += step;
        const uint32_t lb = recs[rlo[t] + (i - rn[t])] & ((1u << SBV_RB) - 1u);
        const uint32_t byte = lb >> 3, mask = 1u << ((byte & 3u) * 8u + (7u - (lb & 7u))); // bit_word's layout
        if (value) atomicOr(&w[byte >> 2], mask);
        else atomicAnd(&w[byte >> 2], ~mask);
    }
    __syncthreads();
    for (uint32_t v = threadIdx.x; v < nv; v += SBV_TPB) src[v] = reg4[v];
}

// SETBIT with replies (M:RedissonBitSet.java:79-81 with a reply, RBatch SETBIT; the reference's pipeline executes
// the ops in batch order, each replying the bit before it) over the same region partition, u64 records carrying the
// op's seq and value.  One workgroup per 32 KiB region of the call's virtual region space (every key touched gets a
// range of regions, `seg`): the region's bits staged in LDS, its records sorted by (bit, seq) in LDS (bitonic), then
// each op replies the value of the op before it on the same bit -- or the bit as the batch found it -- and the last
// op of each bit leaves its value.  A region with more than SBR_RCAP ops (a skewed batch) sorts them in global memory
// first: LDS-sorted chunks, then merge-path passes, through the partition's free chunk buffer at the same slots.
#define SBR_TPB 1024
#define SBR_RCAP 4096
struct SbrSeg { // a key's range of virtual regions: [rb, next seg's rb) -> its string
    uint64_t rb;
    uint8_t *ptr;
    uint64_t cap;
};
__device__ __forceinline__ void lds_bitonic_u64(uint64_t *a, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < P / 2; t += SBR_TPB) {
                const uint32_t i = ((t & ~(j - 1u)) << 1) | (t & (j - 1u)), l = i + j;
                const bool up = (i & k) == 0;
                const uint64_t x = a[i], y = a[l];
                if ((x > y) == up) {
                    a[i] = y;
                    a[l] = x;
                }
            }
            __syncthreads();
        }
}
// The same sort for P <= SBR_TPB keys held one per thread (threads >= P hold ~0 and only ever pair with each other):
// the exchange stages within a wave (j < 64) go through shuffles with no barrier, the wider ones through two
// alternating LDS buffers (one barrier each) -- 10 barriers for 1024 keys instead of 55
__device__ __forceinline__ uint64_t bitonic_regs_u64(uint64_t x, uint32_t P, uint64_t *buf) {
    const uint32_t t = threadIdx.x;
    uint32_t nb = 0;
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            uint64_t y;
            if (j >= 64) { // uniform
                uint64_t *b = buf + nb * SBR_TPB;
                nb ^= 1u;
                b[t] = x;
                __syncthreads();
                y = b[t ^ j];
            } else {
                const uint32_t hi = uint32_t(__shfl_xor(int(uint32_t(x >> 32)), int(j)));
                const uint32_t lo = uint32_t(__shfl_xor(int(uint32_t(x)), int(j)));
                y = (uint64_t(hi) << 32) | lo;
            }
            const bool up = (t & k) == 0, lower = (t & j) == 0;
            const uint64_t mn = x < y ? x : y, mx = x < y ? y : x;
            x = lower == up ? mn : mx;
        }
    return x;
}
__global__ void __launch_bounds__(SBR_TPB) k_sbr_runs(uint32_t ntile, const uint32_t *__restrict__ pbase,
                                                      const uint32_t *__restrict__ rs, uint64_t *recs, uint64_t *scr,
                                                      const SbrSeg *__restrict__ seg, uint32_t nseg,
                                                      uint8_t *__restrict__ out) {
    constexpr uint32_t RBYTES = 1u << (SBV_RB - 3), NV = RBYTES / 16, VPT = NV / SBR_TPB;
    constexpr uint64_t KMASK = 0x0003ffffffffffffull; // bit-in-region << 32 | seq << 1 | value
    __shared__ uint4 reg4[NV];
    __shared__ uint64_t key[SBR_RCAP + 2];
    __shared__ uint32_t rlo[SBV_NTMAXR], rn[SBV_NTMAXR + 1];
    __shared__ uint32_t wsum[SBR_TPB / 64];
    const uint32_t r = blockIdx.x, g = r / SBV_G, rr = r % SBV_G;
    uint32_t lo = 0, c = 0;
    if (threadIdx.x < ntile) {
        const uint32_t *q = rs + (uint64_t(g) * ntile + threadIdx.x) * (SBV_G + 1) + rr;
        lo = pbase[uint64_t(g) * ntile + threadIdx.x] + q[0];
        c = q[1] - q[0];
    }
    uint32_t total;
    const uint32_t ex = block_exscan<SBR_TPB>(c, wsum, &total);
    if (total == 0) return; // uniform: no op in this region
    if (threadIdx.x < ntile) {
        rlo[threadIdx.x] = lo;
        rn[threadIdx.x] = ex;
    }
    if (threadIdx.x == 0) rn[ntile] = total;
    // the key this region belongs to (largest rb <= r)
    uint32_t sl = 0, sh = nseg;
    while (sh - sl > 1) {
        const uint32_t mid = (sl + sh) >> 1;
        if (seg[mid].rb <= r) sl = mid;
        else sh = mid;
    }
    const uint64_t srb = seg[sl].rb, scap = seg[sl].cap;
    uint8_t *const sptr = seg[sl].ptr;
    const uint64_t b0 = (uint64_t(r) - srb) * RBYTES; // < cap: an op's byte lies in the region
    uint4 *src = reinterpret_cast<uint4 *>(sptr + b0);
    const uint32_t nv = scap - b0 >= RBYTES ? NV : uint32_t((scap - b0) / 16); // cap is a multiple of 16
    if (nv == NV) { // a whole region: both loads issued before the LDS stores
        static_assert(VPT == 2, "two 16-B vectors per thread");
        const uint4 t0 = src[threadIdx.x], t1 = src[threadIdx.x + SBR_TPB];
        reg4[threadIdx.x] = t0;
        reg4[threadIdx.x + SBR_TPB] = t1;
    } else {
        for (uint32_t v = threadIdx.x; v < nv; v += SBR_TPB) reg4[v] = src[v];
    }
    __syncthreads();
    uint32_t *w = reinterpret_cast<uint32_t *>(reg4);
    auto slot = [=](uint32_t i) __attribute__((always_inline)) -> uint64_t { // the partition slot of the region's record i (its tile's run)
        uint32_t t = 0;
#pragma unroll
        for (uint32_t step = SBV_NTMAXR / 2; step; step >>= 1)
            if (t + step < ntile && rn[t + step] <= i) t += step;
        return uint64_t(rlo[t]) + (i - rn[t]);
    };
    auto bit_of = [](uint32_t lb) __attribute__((always_inline)) { // LDS word and mask of bit lb (bit_word's layout)
        const uint32_t byte = lb >> 3;
        return 1u << ((byte & 3u) * 8u + (7u - (lb & 7u)));
    };
    // replies and final bits of sorted records key[1 .. m] (key[0] = the record before them or ~0, key[m + 1] the one
    // after or ~0): phase A reads the bits as the batch found them, phase B writes each bit's last value
    auto apply_sorted = [=](uint32_t m) __attribute__((always_inline)) {
        for (uint32_t i = threadIdx.x; i < m; i += SBR_TPB) {
            const uint64_t k = key[i + 1], kp = key[i];
            const uint32_t lb = uint32_t(k >> 32);
            const uint32_t rep = (kp >> 32) == lb ? uint32_t(kp) & 1u : (w[lb >> 5] & bit_of(lb)) ? 1u : 0u;
            if (out) out[uint32_t(k) >> 1] = uint8_t(rep);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += SBR_TPB) {
            const uint64_t k = key[i + 1], kn = key[i + 2];
            const uint32_t lb = uint32_t(k >> 32);
            if ((kn >> 32) != lb) {
                if (uint32_t(k) & 1u) atomicOr(&w[lb >> 5], bit_of(lb));
                else atomicAnd(&w[lb >> 5], ~bit_of(lb));
            }
        }
        __syncthreads();
    };
    if (total <= SBR_TPB) { // one key per thread: sorted in registers and shuffles
        uint32_t P = 2;
        while (P < total) P <<= 1;
        uint64_t x = threadIdx.x < total ? recs[slot(threadIdx.x)] & KMASK : ~0ull;
        static_assert(2 * SBR_TPB <= SBR_RCAP + 2, "two exchange buffers in key[]");
        x = bitonic_regs_u64(x, P, key);
        __syncthreads(); // the exchange buffers read
        if (threadIdx.x < P) key[threadIdx.x + 1] = x;
        if (threadIdx.x == 0) key[0] = ~0ull;
        __syncthreads();
        if (threadIdx.x == 0) key[total + 1] = ~0ull;
        __syncthreads();
        apply_sorted(total);
    } else if (total <= SBR_RCAP) {
        uint32_t P = 2;
        while (P < total) P <<= 1;
        for (uint32_t i = threadIdx.x; i < P; i += SBR_TPB) key[i + 1] = i < total ? recs[slot(i)] & KMASK : ~0ull;
        if (threadIdx.x == 0) key[0] = ~0ull;
        __syncthreads();
        lds_bitonic_u64(key + 1, P);
        if (threadIdx.x == 0) key[total + 1] = ~0ull;
        __syncthreads();
        apply_sorted(total);
    } else {
        // 1) LDS-sorted chunks of SBR_RCAP: recs -> scr
        for (uint32_t c0 = 0; c0 < total; c0 += SBR_RCAP) {
            const uint32_t m = total - c0 < SBR_RCAP ? total - c0 : SBR_RCAP;
            uint32_t P = 2;
            while (P < m) P <<= 1;
            for (uint32_t i = threadIdx.x; i < P; i += SBR_TPB) key[i + 1] = i < m ? recs[slot(c0 + i)] & KMASK : ~0ull;
            __syncthreads();
            lds_bitonic_u64(key + 1, P);
            for (uint32_t i = threadIdx.x; i < m; i += SBR_TPB) scr[slot(c0 + i)] = key[i + 1];
            __syncthreads();
        }
        // 2) merge passes (merge path per thread), src <-> dst
        uint64_t *a = scr, *b = recs;
        for (uint32_t wd = SBR_RCAP; wd < total; wd <<= 1) {
            for (uint32_t p0 = 0; p0 < total; p0 += 2 * wd) {
                const uint32_t a1 = p0 + wd < total ? p0 + wd : total, b1 = p0 + 2 * wd < total ? p0 + 2 * wd : total;
                const uint32_t la = a1 - p0, lb = b1 - a1, len = la + lb;
                const uint32_t d0 = uint32_t(uint64_t(len) * threadIdx.x / SBR_TPB);
                const uint32_t d1 = uint32_t(uint64_t(len) * (threadIdx.x + 1) / SBR_TPB);
                uint32_t x = d0 > lb ? d0 - lb : 0u, y = d0 < la ? d0 : la; // A items taken before output d0
                while (x < y) {
                    const uint32_t mid = (x + y) >> 1;
                    if (a[slot(p0 + mid)] < a[slot(a1 + (d0 - 1 - mid))]) x = mid + 1;
                    else y = mid;
                }
                uint32_t i = x, j = d0 - x;
                for (uint32_t d = d0; d < d1; d++) {
                    const bool ta = j >= lb || (i < la && a[slot(p0 + i)] < a[slot(a1 + j)]);
                    b[slot(p0 + d)] = ta ? a[slot(p0 + i)] : a[slot(a1 + j)];
                    i += ta ? 1u : 0u;
                    j += ta ? 0u : 1u;
                }
            }
            __syncthreads();
            uint64_t *t_ = a;
            a = b;
            b = t_;
        }
        // 3) the sorted records, chunk by chunk, with their neighbours across chunk ends
        for (uint32_t c0 = 0; c0 < total; c0 += SBR_RCAP) {
            const uint32_t m = total - c0 < SBR_RCAP ? total - c0 : SBR_RCAP;
            for (uint32_t i = threadIdx.x; i < m; i += SBR_TPB) key[i + 1] = a[slot(c0 + i)];
            if (threadIdx.x == 0) key[0] = c0 ? a[slot(c0 - 1)] : ~0ull;
            if (threadIdx.x == 1) key[m + 1] = c0 + m < total ? a[slot(c0 + m)] : ~0ull;
            __syncthreads();
            apply_sorted(m);
        }
    }
    for (uint32_t v = threadIdx.x; v < nv; v += SBR_TPB) src[v] = reg4[v];
}

// RBitSet.set(from, to) / clear(from, to) (M:RedissonBitSet.java:202-228:
// one SETBIT_VOID per bit): bits [from, to) of an MSB-first string set to
// `value`.  One lane per 16-B vector; vectors inside the range are stored
// whole, the two edge vectors are masked per byte.  The buffer capacity is a
// multiple of 16 B, so whole-vector access stays in bounds.
__global__ void __launch_bounds__(256) k_bit_range(uint8_t *buf, uint64_t from, uint64_t to, uint32_t value) {
    uint64_t v0 = (from >> 3) >> 4;
    uint64_t v = v0 + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (v > ((to - 1) >> 3) >> 4) return;
    uint64_t b0 = v << 4;
    uint4 *p = reinterpret_cast<uint4 *>(buf) + v;
    if (b0 * 8 >= from && (b0 + 16) * 8 <= to) {
        uint32_t f = value ? 0xffffffffu : 0u;
        *p = make_uint4(f, f, f, f);
        return;
    }
    uint4 w = *p;
    uint8_t *bytes = reinterpret_cast<uint8_t *>(&w);
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint64_t lo = (b0 + j) * 8, hi = lo + 8; // the byte's bit range [lo, hi)
        uint64_t a = from > lo ? from : lo, b = to < hi ? to : hi;
        if (a >= b) continue;
        // MSB-first: bit i of the byte has mask 0x80 >> i
        uint32_t mask = (0xffu >> (a - lo)) & (0xffu << (hi - b)) & 0xffu;
        bytes[j] = value ? uint8_t(bytes[j] | mask) : uint8_t(bytes[j] & ~mask);
    }
    *p = w;
}

// max of a u64 array (offset validation / capacity sizing)
// 16-B loads, SK_MX_UNROLL in flight per lane (one element by itself when v is not 16-B aligned, and an odd last one)
#define SK_MX_UNROLL 4
__global__ void __launch_bounds__(256) k_max_u64(uint64_t n, const uint64_t *__restrict__ v, uint64_t *out) {
    constexpr uint32_t U = SK_MX_UNROLL;
    uint64_t m = 0;
    const uint64_t lead = (reinterpret_cast<uintptr_t>(v) & 15u) && n ? 1u : 0u;
    const uint64_t nv = (n - lead) / 2; // 16-B pairs after the lead element
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (lead) m = v[0];
        if ((n - lead) & 1u) m = v[n - 1] > m ? v[n - 1] : m;
    }
    const ulonglong2 *w = reinterpret_cast<const ulonglong2 *>(v + lead);
    const uint64_t step = uint64_t(gridDim.x) * (256 * U);
    uint64_t i = uint64_t(blockIdx.x) * (256 * U) + threadIdx.x;
    for (; i + 256 * (U - 1) < nv; i += step) {
        ulonglong2 x[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) x[u] = w[i + 256 * u];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint64_t a = x[u].x > x[u].y ? x[u].x : x[u].y;
            m = a > m ? a : m;
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) { // this lane's part of the last, partial chunk (later chunks start past nv)
        const uint64_t t = i + 256 * u;
        if (t < nv) {
            const uint64_t a = w[t].x > w[t].y ? w[t].x : w[t].y;
            m = a > m ? a : m;
        }
    }
    for (int s = 32; s > 0; s >>= 1) {
        uint64_t o = __shfl_xor(m, s);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned long long *)out, (unsigned long long)m);
}

// BITCOUNT: SK_BC_UNROLL independent 16-B loads per lane per step (one
// coalesced 4 KiB row per unroll slot and workgroup), popcount, wave reduce,
// one atomic per wave.
#define SK_BC_UNROLL 8
__global__ void __launch_bounds__(256) k_bitcount(const uint8_t *__restrict__ buf, uint64_t len,
                                                  unsigned long long *out) {
    uint64_t nvec = len >> 4;
    uint64_t c = 0;
    const uint4 *v = reinterpret_cast<const uint4 *>(buf);
    const uint64_t step = uint64_t(gridDim.x) * (256 * SK_BC_UNROLL);
    uint64_t i = uint64_t(blockIdx.x) * (256 * SK_BC_UNROLL) + threadIdx.x;
    for (; i + 256 * (SK_BC_UNROLL - 1) < nvec; i += step) {
        uint4 x[SK_BC_UNROLL];
#pragma unroll
        for (int u = 0; u < SK_BC_UNROLL; u++) x[u] = ld_nt(v + i + 256 * u);
#pragma unroll
        for (int u = 0; u < SK_BC_UNROLL; u++) c += __popc(x[u].x) + __popc(x[u].y) + __popc(x[u].z) + __popc(x[u].w);
    }
    for (int u = 0; u < SK_BC_UNROLL; u++, i += 256) // the last partial step
        if (i < nvec) {
            uint4 x = v[i];
            c += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
        }
    if (blockIdx.x == 0) // tail bytes
        for (uint64_t b = (nvec << 4) + threadIdx.x; b < len; b += blockDim.x) c += __popc(buf[b]);
    for (int s = 32; s > 0; s >>= 1) c += __shfl_xor(c, s);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

// BITOP over maxlen bytes; sources shorter than maxlen read as 0.  Source
// pointers / lengths are cached in LDS; steps every source covers take the
// straight 16 B path with SK_BO_UNROLL chunks per lane in flight per source.
#define SK_BITOP_MAXSRC 64
__device__ __forceinline__ uint4 bitop_src_chunk(const uint8_t *p, uint64_t l, uint64_t b0) {
    if (b0 + 16 <= l) return *reinterpret_cast<const uint4 *>(p + b0);
    uint8_t tmp[16];
    for (int q = 0; q < 16; q++) tmp[q] = (b0 + q < l) ? p[b0 + q] : 0;
    return *reinterpret_cast<uint4 *>(tmp);
}
__device__ __forceinline__ uint4 bitop_combine(int op, uint4 acc, uint4 x) {
    if (op == 0) return make_uint4(acc.x & x.x, acc.y & x.y, acc.z & x.z, acc.w & x.w);
    if (op == 1) return make_uint4(acc.x | x.x, acc.y | x.y, acc.z | x.z, acc.w | x.w);
    return make_uint4(acc.x ^ x.x, acc.y ^ x.y, acc.z ^ x.z, acc.w ^ x.w);
}
#define SK_BO_UNROLL 4
__device__ __forceinline__ uint4 bitop_not(uint4 a) { return make_uint4(~a.x, ~a.y, ~a.z, ~a.w); }
// NT: nontemporal result stores (+2-3 % on C5 AND4 / OR2 over plain stores; 8 chunks per
// lane or a 16384-workgroup grid: no change, profiles/r01_ab/bitop/).
// One step = U (SK_BO_UNROLL) coalesced 4 KiB rows per workgroup; a lane reads
// and writes the same 16-B chunks, so dest may alias a source (BITOP in place).
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_bitop(int op, uint32_t nsrc, const uint8_t *const *__restrict__ srcs,
                                               const uint64_t *__restrict__ lens, uint64_t maxlen, uint8_t *dst) {
    __shared__ const uint8_t *P[SK_BITOP_MAXSRC];
    __shared__ uint64_t L[SK_BITOP_MAXSRC];
    if (threadIdx.x < nsrc) {
        P[threadIdx.x] = srcs[threadIdx.x];
        L[threadIdx.x] = lens[threadIdx.x];
    }
    __syncthreads();
    uint64_t minlen = L[0];
    for (uint32_t s = 1; s < nsrc; s++) minlen = L[s] < minlen ? L[s] : minlen;
    const uint64_t nvec = (maxlen + 15) >> 4, step = uint64_t(gridDim.x) * (256 * U);
    for (uint64_t base = uint64_t(blockIdx.x) * (256 * U); base < nvec; base += step) {
        const uint64_t i0 = base + threadIdx.x;
        uint4 acc[U];
        if ((base + 256 * U) * 16 <= minlen) { // every source covers the whole step (uniform)
            const uint4 *p0 = reinterpret_cast<const uint4 *>(P[0]) + i0;
#pragma unroll
            for (int u = 0; u < U; u++) acc[u] = ld_nt(p0 + 256 * u);
            if (op == 3)
#pragma unroll
                for (int u = 0; u < U; u++) acc[u] = bitop_not(acc[u]);
            for (uint32_t s = 1; s < nsrc; s++) {
                const uint4 *ps = reinterpret_cast<const uint4 *>(P[s]) + i0;
                uint4 x[U];
#pragma unroll
                for (int u = 0; u < U; u++) x[u] = ld_nt(ps + 256 * u);
#pragma unroll
                for (int u = 0; u < U; u++) acc[u] = bitop_combine(op, acc[u], x[u]);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                uint4 *d = reinterpret_cast<uint4 *>(dst) + i0 + 256 * u;
                if (NT) {
                    u32x4 w = {acc[u].x, acc[u].y, acc[u].z, acc[u].w};
                    __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(d));
                } else {
                    *d = acc[u];
                }
            }
            continue;
        }
        for (int u = 0; u < U; u++) { // ragged edge: sources shorter than maxlen read as 0
            uint64_t i = i0 + 256 * u;
            if (i >= nvec) break;
            uint64_t bb = i << 4;
            uint4 a = bitop_src_chunk(P[0], L[0], bb);
            if (op == 3) a = bitop_not(a);
            for (uint32_t s = 1; s < nsrc; s++) a = bitop_combine(op, a, bitop_src_chunk(P[s], L[s], bb));
            if (bb + 16 <= maxlen) {
                reinterpret_cast<uint4 *>(dst)[i] = a;
            } else {
                const uint8_t *ab = reinterpret_cast<const uint8_t *>(&a);
                for (int q = 0; q < 16; q++)
                    if (bb + q < maxlen) dst[bb + q] = ab[q];
            }
        }
    }
}

// ------------------------------------------------- synthetic input generator
// Counter-based SplitMix64: element i = mix(seed + (i+1)*golden), the same
// sequence sk_gen_jackson_longs produces on the host, rendered as Jackson's
// default-typed Long ["java.lang.Long",<v>] (bench/test inputs only).
__device__ __forceinline__ int64_t splitmix_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return int64_t(z ^ (z >> 31));
}
__device__ __forceinline__ unsigned dec_len(int64_t v) {
    uint64_t u = v < 0 ? (~uint64_t(v) + 1) : uint64_t(v);
    unsigned d = 1;
    while (u >= 10) {
        u /= 10;
        d++;
    }
    return d + (v < 0);
}
__global__ void __launch_bounds__(256) k_gen_len(uint64_t n, uint64_t seed, const uint64_t *__restrict__ idx,
                                                 uint64_t first, uint64_t *__restrict__ lens) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t v = splitmix_at(seed, idx ? idx[i] : first + i);
    lens[i] = 18 + dec_len(v) + 1;
}
__global__ void __launch_bounds__(256) k_gen_write(uint64_t n, uint64_t seed, const uint64_t *__restrict__ idx,
                                                   uint64_t first, const uint64_t *__restrict__ off,
                                                   uint8_t *__restrict__ out) {
    uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t v = splitmix_at(seed, idx ? idx[i] : first + i);
    const char pre[] = "[\"java.lang.Long\",";
    uint8_t *p = out + off[i];
    for (int q = 0; q < 18; q++) p[q] = uint8_t(pre[q]);
    unsigned L = dec_len(v);
    uint64_t u = v < 0 ? (~uint64_t(v) + 1) : uint64_t(v);
    uint8_t *d = p + 18;
    if (v < 0) d[0] = '-';
    for (unsigned q = L; q > unsigned(v < 0); q--) {
        d[q - 1] = uint8_t('0' + u % 10);
        u /= 10;
    }
    p[18 + L] = ']';
}

// -------------------------------------------------------------- range-sharded RBitSet routing (C5 across GPUs)
// A SETBIT / GETBIT batch submitted on one rank is split by owner shard (shard s holds bits [s * shard_bits,
// (s + 1) * shard_bits) of the logical string) into ONE buffer: shard 0's ops, then shard 1's, ..., each in batch
// order, as shard-local offsets.  Blocks of SK_RT_EPB ops; a thread takes SK_RT_PER consecutive ops, so the stable
// rank of an op inside its block is the thread's exclusive prefix for its shard plus its running count.  The
// replies come back in the same layout and k_unroute gathers them to batch order (each block reads one contiguous
// segment per shard).
#define SK_RT_TPB 256
#define SK_RT_PER 16
#define SK_RT_EPB (SK_RT_TPB * SK_RT_PER)
#define SK_RT_MAXW 8
__device__ __forceinline__ uint32_t rt_shard(uint64_t off, uint64_t shard_bits, uint32_t world) {
    const uint64_t s = off / shard_bits;
    return s < world ? uint32_t(s) : world; // world: out of range
}
// ops per (shard, block) -> cnt[s * nblk + blk]; *bad = 1 if an offset is past the last shard
__global__ void __launch_bounds__(SK_RT_TPB) k_route_count(uint64_t n, const uint64_t *__restrict__ offs,
                                                           uint64_t shard_bits, uint32_t world, uint32_t nblk,
                                                           uint32_t *__restrict__ cnt, uint32_t *bad) {
    __shared__ uint32_t h[SK_RT_MAXW + 1];
    if (threadIdx.x <= SK_RT_MAXW) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i0 = uint64_t(blockIdx.x) * SK_RT_EPB + uint64_t(threadIdx.x) * SK_RT_PER;
    uint32_t c[SK_RT_MAXW + 1] = {};
#pragma unroll
    for (int q = 0; q < SK_RT_PER; q++) {
        const uint64_t i = i0 + q;
        if (i < n) {
            const uint32_t sh = rt_shard(offs[i], shard_bits, world);
#pragma unroll
            for (int w = 0; w <= SK_RT_MAXW; w++) c[w] += sh == uint32_t(w);
        }
    }
#pragma unroll
    for (int w = 0; w <= SK_RT_MAXW; w++)
        if (c[w]) atomicAdd(&h[w], c[w]);
    __syncthreads();
    if (threadIdx.x < world) cnt[uint64_t(threadIdx.x) * nblk + blockIdx.x] = h[threadIdx.x];
    if (threadIdx.x == 0 && h[world]) *bad = 1;
}
// base = exclusive scan of cnt (shard-major); send[base + rank] = shard-local offset (values alongside if given),
// dst[i] = the op's slot in send
__global__ void __launch_bounds__(SK_RT_TPB) k_route_scatter(uint64_t n, const uint64_t *__restrict__ offs,
                                                             const uint8_t *__restrict__ vals, uint64_t shard_bits,
                                                             uint32_t world, uint32_t nblk,
                                                             const uint32_t *__restrict__ base,
                                                             uint64_t *__restrict__ send, uint8_t *__restrict__ svals,
                                                             uint32_t *__restrict__ dst) {
    __shared__ uint32_t wsum[SK_RT_TPB / 64];
    const uint64_t i0 = uint64_t(blockIdx.x) * SK_RT_EPB + uint64_t(threadIdx.x) * SK_RT_PER;
    uint64_t o[SK_RT_PER];
    uint32_t c[SK_RT_MAXW] = {};
#pragma unroll
    for (int q = 0; q < SK_RT_PER; q++) {
        const uint64_t i = i0 + q;
        o[q] = i < n ? offs[i] : ~0ull;
        const uint32_t sh = i < n ? rt_shard(o[q], shard_bits, world) : world;
#pragma unroll
        for (int w = 0; w < SK_RT_MAXW; w++) c[w] += sh == uint32_t(w);
    }
    uint32_t pre[SK_RT_MAXW];
#pragma unroll
    for (int w = 0; w < SK_RT_MAXW; w++) {
        uint32_t tot;
        pre[w] = uint32_t(w) < world ? base[uint64_t(w) * nblk + blockIdx.x] + block_exscan<SK_RT_TPB>(c[w], wsum, &tot)
                                     : 0u;
    }
#pragma unroll
    for (int q = 0; q < SK_RT_PER; q++) {
        const uint64_t i = i0 + q;
        if (i >= n) continue;
        const uint32_t sh = rt_shard(o[q], shard_bits, world);
        if (sh >= world) continue;
        uint32_t d = 0;
#pragma unroll
        for (int w = 0; w < SK_RT_MAXW; w++)
            if (sh == uint32_t(w)) d = pre[w]++;
        send[d] = o[q] - uint64_t(sh) * shard_bits;
        if (vals) svals[d] = vals[i];
        dst[i] = d;
    }
}
// out[i] = rep[dst[i]]: replies back to batch order
__global__ void __launch_bounds__(256) k_unroute(uint64_t n, const uint32_t *__restrict__ dst,
                                                 const uint8_t *__restrict__ rep, uint8_t *__restrict__ out) {
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
        out[i] = rep[dst[i]];
}

// ================================================================ launchers
#define SK_LAUNCH_CHECK()                                                                                              \
    do {                                                                                                               \
        hipError_t e__ = hipGetLastError();                                                                            \
        if (e__ != hipSuccess) return e__;                                                                             \
    } while (0)




uint64_t long_elem_bytes() { return SK_LONG_ELEM; }

uint32_t murmur_long_wgs(uint64_t len) { return uint32_t(((len >> 3) + SK_MS_BPW - 1) / SK_MS_BPW); }
uint64_t murmur_long_plane_words(uint64_t len) { return 64 * (((len >> 3) + SK_MS_S - 1) / SK_MS_S); }

hipError_t launch_murmur_long(hipStream_t st, uint32_t n_long, uint32_t n_wg, const uint8_t *bytes,
                              const uint64_t *off, const uint32_t *meta, uint32_t *plane, uint32_t *flags,
                              uint64_t *out_h) {
    if (!n_long) return hipSuccess;
    hipError_t r = hipMemsetAsync(flags, 0, (uint64_t(n_wg) * 64 + 2) * 4, st);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL(k_ms_planes, dim3(n_wg), dim3(SK_MS_TPB), 0, st, bytes, off, meta, n_long, plane);
    SK_LAUNCH_CHECK();
    // SK_MS_SPIN_DEV: a test-only lower wait bound, so the host's recompute path is exercised
    static const uint32_t spin = getenv("SK_MS_SPIN_DEV") ? uint32_t(strtoul(getenv("SK_MS_SPIN_DEV"), nullptr, 10))
                                                          : SK_MS_SPIN;
    hipLaunchKernelGGL(k_ms_rounds, dim3(n_wg), dim3(SK_MS_TPB), 0, st, bytes, off, meta, n_long, n_wg,
                       (const uint32_t *)plane, flags, 0xadc83b19ull, out_h, spin);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

uint32_t pfp_blocks(uint64_t n) { return uint32_t((n + SK_PFQ_EPB - 1) / SK_PFQ_EPB); } // partition path
uint32_t pfp_buckets() { return SK_PFP_NB; }
uint32_t pfp_epb() { return SK_PFQ_EPB; }
static uint32_t pfl_blocks(uint64_t n) { return uint32_t((n + SK_PFP_EPB - 1) / SK_PFP_EPB); } // line schedule


// hash + block-local bucket sort -> per-bucket LDS resolve; one launcher per stage so each is timed
hipError_t launch_pfp_hash(hipStream_t st, uint64_t n, const uint32_t *key_ids, const uint64_t *off,
                           const uint8_t *bytes, int v5, uint64_t *chunks, uint32_t *S, uint16_t *pos,
                           uint32_t *big_alloc, const uint64_t *pre) {
    uint32_t nb = pfp_blocks(n);
    hipLaunchKernelGGL(k_pfp_hash, dim3(nb), dim3(SK_PFP_TPB), 0, st, n, key_ids, off, bytes, v5, chunks, S, nb, pos,
                       big_alloc, pre);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_pfp_apply(hipStream_t st, uint64_t n, const uint64_t *chunks, const uint32_t *S, uint8_t *arena,
                            uint8_t *rep, uint32_t *big_alloc, uint64_t *big_keys, uint32_t *big_vals,
                            uint8_t *changed, uint64_t *ev, uint32_t *ev_n) {

    hipLaunchKernelGGL(k_pfp_apply, dim3(SK_PFP_NB), dim3(SK_PFP_ATPB), 0, st, chunks, S, pfp_blocks(n), arena, rep,
                       big_alloc, big_keys, big_vals, changed, ev, ev_n);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_pfp_reply(hipStream_t st, uint64_t n, const uint8_t *rep, const uint16_t *pos,
                            const uint32_t *cmd_of, uint8_t *changed) {
    hipLaunchKernelGGL(k_pfp_reply, dim3(pfp_blocks(n)), dim3(SK_PFP_TPB), 0, st, n, rep, pos, cmd_of, changed);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

// line schedule: layout of one call's scratch (PflDims) and its stages
PflDims pfl_dims(uint64_t n, uint32_t nslab, uint32_t tile_blocks) {
    PflDims d;
    d.nblk = pfl_blocks(n);
    // permutation over 2^pk >= nslab ids (>= one fine bucket); a fine bucket = 2^sh consecutive permuted ids, of which
    // nslab / 2^pk are live: it expects n * 2^sh / (128 * 2^pk) records.  Keep that <= ~600 (one chunk of
    // SK_PFL_CAP with margin), within the LDS lines (2^SK_PFL_SH) and the region's fine-bucket counts (MAXSUB)
    uint32_t pk0 = 0;
    while (pk0 < 32 && (1ull << pk0) < nslab) pk0++;
    d.sh = SK_PFL_SH;
    while (d.sh > 0 && double(n) * double(1u << d.sh) > double(SK_PFL_EXP) * SK_PFL_NB * double(1ull << std::max(pk0, d.sh)) &&
           (1ull << (std::max(pk0, d.sh - 1) - (d.sh - 1))) <= SK_PFL_MAXSUB)
        d.sh--;
    // the inverse of an odd pa mod 2^32 by Newton steps
    d.pk = std::max(pk0, d.sh);
    d.pm_mask = d.pk >= 32 ? 0xffffffffu : uint32_t((1ull << d.pk) - 1);
    d.pa = 0x9E3779B1u;
    uint32_t inv = d.pa; // x <- x (2 - a x): correct bits double each step
    for (int it = 0; it < 5; it++) inv *= 2u - d.pa * inv;
    d.pai = inv;
    d.nsub = uint32_t((uint64_t(d.pm_mask) + 1) >> d.sh);
    d.nslab = nslab;
    d.nf = uint64_t(SK_PFL_NB) * d.nsub;
    // region capacity in LDS: records (u64) + nsub + 1 counts; the tile keeps a region's binomial record count
    // (mean 32 tb) 6 sigma below it
    uint64_t cap = (uint64_t(SK_PFL_LDS) - 4ull * (d.nsub + 1)) / 8;
    d.rcap = uint32_t(std::min<uint64_t>(cap & ~uint64_t(1023), SK_PFL_RCAP));
    d.tb = tile_blocks ? tile_blocks : SK_PFL_TILE;
    while (d.tb > 64 && 32.0 * d.tb + 6.0 * std::sqrt(32.0 * d.tb) > double(d.rcap)) d.tb -= 32;
    if (d.tb > SK_PFL_TMAX) d.tb = SK_PFL_TMAX;
    if (d.tb < (d.nblk + SK_PFL_NTMAX - 1) / SK_PFL_NTMAX) d.tb = (d.nblk + SK_PFL_NTMAX - 1) / SK_PFL_NTMAX;
    d.ntile = (d.nblk + d.tb - 1) / d.tb;
    d.nreg = SK_PFL_NB * d.ntile;
    d.c_words = 2 * uint64_t(d.nreg) + uint64_t(d.nreg) * (d.nsub + 1);
    d.chunk_bytes = uint64_t(d.nblk) * SK_PFP_EPB * 8;
    d.S_bytes = uint64_t(SK_PFL_NB + 1) * d.nblk * 4;
    return d;
}
uint32_t pfl_max_slabs() { return (SK_PFL_MAXSUB << SK_PFL_SH) / 2; } // the permuted id range is < 2 x nslab

hipError_t launch_pfl_hash(hipStream_t st, uint64_t n, const uint32_t *key_ids, const uint64_t *off,
                           const uint8_t *bytes, int v5, uint64_t *chunks, uint32_t *S, uint32_t *big_alloc) {
    uint32_t nb = pfl_blocks(n);
    hipLaunchKernelGGL(k_pfl_hash, dim3(nb), dim3(SK_PFP_TPB), 0, st, n, key_ids, off, bytes, v5, chunks, S, nb,
                       big_alloc);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_pfl_part(hipStream_t st, const PflDims &d, const uint64_t *chunks, const uint32_t *S, uint32_t *C,
                           uint64_t *rec2, uint8_t *changed) {
    if (d.nsub > SK_PFL_MAXSUB || d.tb > SK_PFL_TMAX || d.ntile > SK_PFL_NTMAX || d.rcap < SK_PFL_RTPB)
        return hipErrorInvalidValue; // pfl_dims never produces these (the caller checks pfl_dims_ok)
    uint32_t *tot = C, *rbase = C + d.nreg, *C2 = C + 2 * d.nreg;
    hipLaunchKernelGGL(k_pfl_tot, dim3(d.ntile, SK_PFL_NB), dim3(256), 0, st, S, d.nblk, d.tb, d.ntile, tot);
    SK_LAUNCH_CHECK();
    const uint32_t lds = d.rcap * 8 + (d.nsub + 1) * 4;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pfl_region),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, SK_PFL_LDS);
        if (e != hipSuccess) return e;
        attr = true;
    }
    static const int probe_flags = getenv("SK_PFL_PROBE") ? atoi(getenv("SK_PFL_PROBE")) : 0; // dev ablations
    hipLaunchKernelGGL(k_pfl_region, dim3(d.nreg), dim3(SK_PFL_RTPB), lds, st,
                       PflChunk{const_cast<uint64_t *>(chunks), uint64_t(d.nblk) * SK_PFP_EPB}, S, d.nblk, d.tb, d.ntile,
                       d.nsub, d.sh, PflPerm{d.pa, d.pai, d.pm_mask, d.nslab}, d.rcap, tot, rbase, C2,
                       PflRec{rec2, uint64_t(d.nblk) * SK_PFP_EPB},
                       changed, probe_flags);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}
bool pfl_dims_ok(const PflDims &d) {
    return d.nsub <= SK_PFL_MAXSUB && d.tb <= SK_PFL_TMAX && d.ntile <= SK_PFL_NTMAX && d.rcap >= SK_PFL_RTPB;
}

hipError_t launch_pfl_fill(hipStream_t st, uint8_t *changed, uint64_t n, uint32_t *rc, uint32_t par) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_pfl_fill, dim3(grid_for((n + 15) / 16, 256, 4096)), dim3(256), 0, st, changed, n, rc, par);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_pfl_apply(hipStream_t st, const PflDims &d, const uint64_t *rec2, const uint32_t *C, uint32_t nslab,
                            uint8_t *arena, uint8_t *changed, uint32_t *big_alloc, uint64_t *big_keys,
                            uint32_t *big_vals, int flags, uint32_t *order, uint32_t *rc, uint32_t par) {
    static const int probe_flags = getenv("SK_PFL_PROBE") ? atoi(getenv("SK_PFL_PROBE")) : 0; // dev ablations
    const uint32_t *rbase = C + d.nreg, *C2 = C + 2 * d.nreg;
    // heavy slots: at most n / (CAP + 1) fine buckets hold more than one chunk
    const uint32_t hmax = order ? uint32_t(std::min<uint64_t>(d.nf, uint64_t(d.nblk) * SK_PFP_EPB / (SK_PFL_CAP + 1)))
                                : 0u;
    if (order) {
        hipLaunchKernelGGL(k_pfl_plan, dim3(uint32_t((d.nf + 255) / 256)), dim3(256), 0, st, C2, d.ntile, d.nsub,
                           uint32_t(d.nf), hmax, big_alloc + 1, order);
        SK_LAUNCH_CHECK();
    }
    // see k_pfl_apply's XCD order: heavy slots a multiple of 8, the fine buckets padded to whole XCD blocks
    const uint32_t sbx = SK_PFL_XORD ? 8u * SK_PFL_XORD : 1u;
    const uint32_t hmax8 = (hmax + 7u) & ~7u, nsubx = uint32_t((d.nsub + sbx - 1) / sbx * sbx);
    hipLaunchKernelGGL(k_pfl_apply, dim3(uint32_t(SK_PFL_NB) * nsubx + hmax8), dim3(SK_PFL_ATPB), 0, st,
                       PflRec{const_cast<uint64_t *>(rec2), uint64_t(d.nblk) * SK_PFP_EPB}, rbase, C2, d.ntile,
                       d.nsub, d.sh, PflPerm{d.pa, d.pai, d.pm_mask, d.nslab}, nslab, arena, changed, big_alloc,
                       big_keys, big_vals, flags | probe_flags, hmax8, big_alloc + 1, order, rc, par);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t sort_keys_size(uint64_t n, unsigned begin_bit, unsigned end_bit, size_t *bytes) {
    size_t sz = 0;
    hipError_t e = rocprim::radix_sort_keys(nullptr, sz, (const uint64_t *)nullptr, (uint64_t *)nullptr, size_t(n),
                                            begin_bit, end_bit);
    *bytes = sz;
    return e;
}

hipError_t sort_keys(hipStream_t st, void *tmp, size_t tmp_bytes, const uint64_t *in, uint64_t *out, uint64_t n,
                     unsigned begin_bit, unsigned end_bit) {
    if (!n) return hipSuccess;
    size_t sz = tmp_bytes;
    return rocprim::radix_sort_keys(tmp, sz, in, out, size_t(n), begin_bit, end_bit, st);
}

hipError_t sort_pairs_size(uint64_t n, unsigned begin_bit, unsigned end_bit, size_t *bytes) {
    size_t sz = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, sz, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                             (const uint32_t *)nullptr, (uint32_t *)nullptr, size_t(n), begin_bit,
                                             end_bit);
    *bytes = sz;
    return e;
}

hipError_t sort_pairs(hipStream_t st, void *tmp, size_t tmp_bytes, const uint64_t *kin, uint64_t *kout,
                      const uint32_t *vin, uint32_t *vout, uint64_t n, unsigned begin_bit, unsigned end_bit) {
    if (!n) return hipSuccess;
    size_t sz = tmp_bytes;
    return rocprim::radix_sort_pairs(tmp, sz, kin, kout, vin, vout, size_t(n), begin_bit, end_bit, st);
}

hipError_t sort_pairs64_size(uint64_t n, size_t *bytes) {
    size_t sz = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, sz, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                             (const uint64_t *)nullptr, (uint64_t *)nullptr, size_t(n), 0, 64);
    *bytes = sz;
    return e;
}

hipError_t sort_pairs64(hipStream_t st, void *tmp, size_t tmp_bytes, const uint64_t *kin, uint64_t *kout,
                        const uint64_t *vin, uint64_t *vout, uint64_t n) {
    if (!n) return hipSuccess;
    size_t sz = tmp_bytes;
    return rocprim::radix_sort_pairs(tmp, sz, kin, kout, vin, vout, size_t(n), 0, 64, st);
}

hipError_t launch_hll_sum(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *arena, uint64_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_hll_sum, dim3(grid_for((n + 3) / 4, 1, 1024)), dim3(256), 0, st, n, ids, arena, out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hll_pack(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *arena, uint8_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_hll_pack, dim3(uint32_t(n * 3)), dim3(256), 0, st, n, ids, arena,
                       reinterpret_cast<uint32_t *>(out));
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hll_unpack(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *in, uint8_t *arena) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_hll_unpack, dim3(uint32_t(n * 3)), dim3(256), 0, st, n, ids,
                       reinterpret_cast<const uint32_t *>(in), arena);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_hll_hist(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *arena, uint32_t *hist,
                           int packed) {
    if (!n) return hipSuccess;
    if (packed)
        hipLaunchKernelGGL(k_hll_hist<true>, dim3(grid_for(n, 1, 8192)), dim3(64), 0, st, n, ids, arena, hist);
    else
        hipLaunchKernelGGL(k_hll_hist<false>, dim3(grid_for(n, 1, 8192)), dim3(64), 0, st, n, ids, arena, hist);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

// Union as a max-tree: level 0 reduces the slabs into <= max_groups partials
// (>= 64 sources per workgroup column), each further level reduces 64:1 until
// <= 64 remain, and the root folds them (and `out` when include_out) into out.
// `partial` holds max_groups + max_groups/64 + 1 arrays of 16 KiB.
hipError_t launch_hll_union(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *src, uint8_t *partial,
                            uint64_t max_groups, uint8_t *out, int include_out, int src_packed, int out_packed) {
    if (!n) {
        if (!include_out) return hipMemsetAsync(out, 0, out_packed ? SK_SLAB_BYTES : 16384u, st);
        return hipSuccess;
    }
    const uint32_t *cur_ids = ids;
    const uint8_t *cur = src;
    uint64_t cur_n = n;
    bool pk = src_packed != 0;
    uint8_t *bufs[2] = {partial, partial + max_groups * 16384};
    int which = 0;
    auto partial_pass = [&](uint64_t per, uint64_t G) {
        if (pk)
            hipLaunchKernelGGL(k_hll_union_partial<true>, dim3(4, unsigned(G)), dim3(256), 0, st, cur_n, cur_ids, cur,
                               per, bufs[which]);
        else
            hipLaunchKernelGGL(k_hll_union_partial<false>, dim3(4, unsigned(G)), dim3(256), 0, st, cur_n, cur_ids, cur,
                               per, bufs[which]);
        cur = bufs[which];
        cur_ids = nullptr;
        pk = false; // the partials are u8
        which ^= 1;
    };
    while (cur_n > 64) {
        uint64_t per = (cur_n + max_groups - 1) / max_groups;
        if (per < 64) per = 64;
        uint64_t G = (cur_n + per - 1) / per;
        partial_pass(per, G);
        SK_LAUNCH_CHECK();
        cur_n = G;
    }
    if (cur_ids || pk) { // n <= 64 sources not yet in u8 partial form: one partial, then the root
        partial_pass(cur_n, 1);
        SK_LAUNCH_CHECK();
        cur_n = 1;
    }
    if (out_packed)
        hipLaunchKernelGGL(k_hll_union_final<true>, dim3(4), dim3(256), 0, st, cur_n, cur, out, include_out);
    else
        hipLaunchKernelGGL(k_hll_union_final<false>, dim3(4), dim3(256), 0, st, cur_n, cur, out, include_out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_bloom_contains(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes,
                                 const uint8_t *bits, const uint64_t *d_len, uint64_t size, uint64_t magic, int k,
                                 uint8_t *out, int sched, void *scratch) {
    if (!n) return hipSuccess;
    if (sched == 3 && scratch) { // split: hash pass, then probe pass
        hipLaunchKernelGGL(k_bloom_hash, dim3(grid_for(n, 256)), dim3(256), 0, st, n, off, bytes,
                           reinterpret_cast<uint4 *>(scratch));
        SK_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_bloom_probe_h, dim3(grid_for(n, 256)), dim3(256), 0, st, n,
                           reinterpret_cast<const uint4 *>(scratch), bits, d_len, size, magic, k, out);
    } else if (sched == 1) // probe queue, 4 elements per lane (A/B: not faster at C3 -- line requests bound both)
        hipLaunchKernelGGL(k_bloom_contains_q<4>, dim3(grid_for(n, 1024)), dim3(256), 0, st, n, off, bytes, bits,
                           d_len, size, magic, k, out);
    else // one element per thread
        hipLaunchKernelGGL(k_bloom_contains, dim3(grid_for(n, 256)), dim3(256), 0, st, n, off,
                           bytes, bits, d_len, size, magic, k, out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

uint32_t rc_blocks(uint64_t n) { return uint32_t((n + RC_EPB - 1) / RC_EPB); }
uint32_t rc_regions(uint64_t size) { return uint32_t((size + (1ull << RC_RB) - 1) >> RC_RB); }
uint32_t rc_max_probes() { return RC_PMAX; }
uint64_t rc_chunk_words(int k) { return uint64_t(RC_EPB) * uint64_t(k - 1); }

static uint32_t ra_epb(int k) { return k <= RA_K4 ? 4096u : 2048u; }
uint32_t ra_blocks(uint64_t n, int k) { return uint32_t((n + ra_epb(k) - 1) / ra_epb(k)); }
uint64_t rc_seg_words(uint32_t nb, uint32_t nr) {
    return uint64_t(nb) * ((nr + SK_RC_STILE - 1) / SK_RC_STILE * SK_RC_STILE);
}
bool rc_seg_interleaved() { return SK_RC_STILE > 1; }
// the contains probe reads the interleaved table itself (no transpose before it)
bool rc_probe_reads_st() { return SK_RC_STILE > 1 && SK_RC_PCOL && SK_RC_ZL && SK_RC_TV && SK_RC_PERSIST; }
hipError_t launch_rc_stranspose(hipStream_t st, uint32_t nb, uint32_t nr, const uint32_t *St, uint32_t *S) {
    if (SK_RC_STILE == 1) return hipSuccess;
    hipLaunchKernelGGL(k_rc_stranspose, dim3((nb + RC_STJ - 1) / RC_STJ, (nr + SK_RC_STILE - 1) / SK_RC_STILE), dim3(256), 0, st,
                       St, S, nb, nr);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}
uint32_t ra_regions(uint64_t size) { return uint32_t((size + (1ull << RA_RB) - 1) >> RA_RB); }
uint64_t ra_piece(int k) { return uint64_t(RA_JPT) * RC_TPB * ra_epb(k); }
uint64_t ra_chunk_words(int k) { return uint64_t(ra_epb(k)) * uint64_t(k); }
uint32_t ra_max_probes() { return RC_PMAX; }

// Bloom add, region schedule: records u32[ra_blocks(n) * ra_chunk_words(k)], S u32[regions * blocks], *flag = 0 before
hipError_t launch_bloom_ra_hash(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                                uint64_t magic, int k, uint32_t *S, uint32_t *recs, uint32_t *stop, uint32_t piece) {
    if (!n) return hipSuccess;
    uint32_t NB = ra_blocks(n, k);
    if (ra_epb(k) == 4096)
        hipLaunchKernelGGL((k_bloom_rc_hash<true, 4096>), dim3(8 * ((NB + 7) / 8)), dim3(RC_TPB), 0, st, n, off, bytes,
                           size, magic, uint32_t(k), ra_regions(size), NB, S, recs, nullptr, stop, piece);
    else
        hipLaunchKernelGGL((k_bloom_rc_hash<true, 2048>), dim3(8 * ((NB + 7) / 8)), dim3(RC_TPB), 0, st, n, off, bytes,
                           size, magic, uint32_t(k), ra_regions(size), NB, S, recs, nullptr, stop, piece);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

uint64_t ra_group_table_words(uint64_t size) { return uint64_t(RA_NG) * ra_regions(size); }
hipError_t launch_bloom_ra_apply(hipStream_t st, uint64_t n, uint64_t size, int k, const uint32_t *S,
                                 const uint32_t *recs, uint8_t *bits, uint64_t cap_bytes, uint64_t *d_len,
                                 uint8_t *out, const uint32_t *stop, uint32_t piece, uint32_t *Z, uint32_t *zalloc,
                                 uint64_t *GT) {
    if (!n) return hipSuccess;
    uint32_t NR = ra_regions(size);
    // every region of a big piece expects >= RA_DENSE records: its bits are loaded up front
    const int big = n * uint64_t(k) >= uint64_t(2 * RA_DENSE) * NR;
#if SK_RA_OL
    hipError_t e = hipMemsetAsync(zalloc, 0, 4, st);
    if (e != hipSuccess) return e;
#endif
    if (ra_epb(k) == 4096)
        hipLaunchKernelGGL(k_bloom_ra_apply<4096>, dim3(8 * ((NR + 7) / 8)), dim3(RC_TPB), 0, st, ra_blocks(n, k), NR, S,
                           recs, uint32_t(k), bits, cap_bytes, reinterpret_cast<unsigned long long *>(d_len), out,
                           stop, piece, big, Z, zalloc, GT);
    else
        hipLaunchKernelGGL(k_bloom_ra_apply<2048>, dim3(8 * ((NR + 7) / 8)), dim3(RC_TPB), 0, st, ra_blocks(n, k), NR, S,
                           recs, uint32_t(k), bits, cap_bytes, reinterpret_cast<unsigned long long *>(d_len), out,
                           stop, piece, big, Z, zalloc, GT);
    SK_LAUNCH_CHECK();
#if SK_RA_OL
    const uint32_t ng = uint32_t((n + (1u << RA_GSH) - 1) >> RA_GSH);
    hipLaunchKernelGGL(k_bloom_ra_one, dim3(8 * ((ng + 7) / 8)), dim3(RA_OTPB), 0, st, NR, n, Z,
                       uint64_t(ra_blocks(n, k)) * ra_chunk_words(k), GT, out, stop, piece);
    SK_LAUNCH_CHECK();
#endif
    return hipSuccess;
}

// region schedule: records u32[blocks * RC_EPB * (k-1)], S u32[regions * blocks]
hipError_t launch_bloom_rc_hash(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                                uint64_t magic, int k, uint32_t *S, uint32_t *recs, uint8_t *out) {
    if (!n) return hipSuccess;
    uint32_t NB = rc_blocks(n);
    if (k - 1 <= 6)
        hipLaunchKernelGGL((k_bloom_rc_hash<false, 2048, 6>), dim3(8 * ((NB + 7) / 8)), dim3(RC_TPB), 0, st, n, off,
                           bytes, size, magic, uint32_t(k - 1), rc_regions(size), NB, S, recs, out, nullptr, 0u);
    else
        hipLaunchKernelGGL(k_bloom_rc_hash<false>, dim3(8 * ((NB + 7) / 8)), dim3(RC_TPB), 0, st, n, off, bytes, size,
                           magic, uint32_t(k - 1), rc_regions(size), NB, S, recs, out, nullptr, 0u);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}
hipError_t launch_bloom_rc_probe(hipStream_t st, uint64_t n, uint64_t size, int k, const uint32_t *S,
                                 const uint32_t *recs, const uint8_t *bits, uint64_t cap_bytes, uint8_t *out,
                                 uint32_t *Z, uint32_t *GT) {
    if (!n) return hipSuccess;
    uint32_t NR = rc_regions(size), NB = rc_blocks(n);
#if SK_RC_ZL && SK_RC_TV && SK_RC_PERSIST
    const uint32_t slots = std::min<uint32_t>(RC_PSLOTS, (NR + 7) / 8); // workgroups per XCD group
    hipLaunchKernelGGL((k_bloom_rc_probe_p<RC_PTPB, RC_PRING>), dim3(8 * slots), dim3(RC_PTPB), 0, st, NB, NR, S,
                       recs, uint32_t(k - 1), bits, cap_bytes, out, Z, GT);
#else
    hipLaunchKernelGGL(k_bloom_rc_probe, dim3(8 * ((NR + 7) / 8)), dim3(RC_TPB), 0, st, NB, NR, S, recs,
                       uint32_t(k - 1), bits, cap_bytes, out, Z, GT);
#endif
    SK_LAUNCH_CHECK();
#if SK_RC_ZL
    const uint32_t ng = (NB + RC_GB - 1) / RC_GB;
    hipLaunchKernelGGL(k_bloom_rc_zero, dim3(8 * ((ng + 7) / 8)), dim3(RC_ZTPB), 0, st, NB, NR, n, Z, GT, out);
    SK_LAUNCH_CHECK();
#endif
    return hipSuccess;
}
uint64_t rc_zero_list_words(uint64_t size) { return SK_RC_ZL ? uint64_t(rc_regions(size)) * RC_ZCAP : 1; }
uint64_t rc_group_table_words(uint64_t size) { return SK_RC_ZL ? uint64_t(rc_regions(size)) * RC_NG : 1; }

hipError_t launch_bloom_probes(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                               uint64_t magic, int k, uint64_t *keys) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bloom_probes, dim3(grid_for(n, 256)), dim3(256), 0, st, n, off, bytes, size, magic, k, keys);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_bloom_indexes(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                                uint64_t magic, int np, uint64_t *idx) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_bloom_indexes, dim3(grid_for(n, 256)), dim3(256), 0, st, n, off, bytes, size, magic, np, idx);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}
hipError_t launch_expand_prefix(hipStream_t st, uint64_t n, const SkPrefix &pre, const uint32_t *soff,
                                const uint8_t *sbytes, uint64_t *off, uint8_t *bytes) {
    hipLaunchKernelGGL(k_expand_prefix, dim3(grid_for(n + 1, 256)), dim3(256), 0, st, n, pre, soff, sbytes, off, bytes);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}
hipError_t launch_reduce_groups_u8(hipStream_t st, uint64_t n, uint32_t group, uint32_t take, uint32_t invert,
                                   const uint8_t *in, uint8_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_reduce_groups_u8, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, n, group, take, invert, in,
                       out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_bloom_apply(hipStream_t st, uint64_t m, const uint64_t *keys, uint8_t *bits, uint64_t *d_len, int k,
                              uint8_t *out) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_bloom_apply, dim3(grid_for(m, 256)), dim3(256), 0, st, m, keys, bits, d_len, k, out);
    SK_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_len_from_last_key, dim3(1), dim3(1), 0, st, keys, m, d_len);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_getbit_multi(hipStream_t st, uint64_t n, const uint32_t *sid, const uint64_t *offs, const void *dir,
                               uint8_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_getbit_multi, dim3(grid_for(n, 256)), dim3(256), 0, st, n, sid, offs,
                       reinterpret_cast<const DirEnt *>(dir), out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_getbit_single(hipStream_t st, uint64_t n, const uint64_t *offs, const uint8_t *buf,
                                const uint64_t *d_len, uint8_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_getbit_single, dim3(grid_for(n, 256)), dim3(256), 0, st, n, offs, buf, d_len, out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_setbit_keys(hipStream_t st, uint64_t n, const uint32_t *sid, const uint64_t *offs, uint64_t *keys,
                              uint32_t *vals) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_setbit_keys, dim3(grid_for(n, 256)), dim3(256), 0, st, n, sid, offs, keys, vals);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_setbit_apply(hipStream_t st, uint64_t n, const uint64_t *keys, const uint32_t *vals,
                               const uint8_t *values, uint8_t value_all, void *dir, uint8_t *out_old) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_setbit_apply, dim3(grid_for(n, 256)), dim3(256), 0, st, n, keys, vals, values, value_all,
                       reinterpret_cast<DirEnt *>(dir), out_old);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_setbit_void(hipStream_t st, uint64_t n, const uint64_t *offs, uint8_t *buf, uint32_t value) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_setbit_void, dim3(grid_for(n, 256)), dim3(256), 0, st, n, offs, buf, value);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

uint32_t sbv_region_bits() { return SBV_RB; }
hipError_t launch_setbit_void_regions(hipStream_t st, uint64_t n, const uint64_t *keys, uint64_t max_off,
                                      uint32_t *start, uint8_t *buf, uint64_t cap, uint32_t value) {
    if (!n) return hipSuccess;
    const uint32_t NR = uint32_t(max_off >> SBV_RB) + 1;
    hipLaunchKernelGGL(k_sbv_starts, dim3(grid_for(n, 256)), dim3(256), 0, st, n, keys, NR, start);
    SK_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sbv_apply, dim3(NR), dim3(SBV_TPB), 0, st, keys, start, buf, cap, value);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

// dense SETBIT_VOID through the hand-written region partition: scratch = sbv_part_scratch_bytes(n, max_off) bytes
static void sbv_dims(uint64_t n, uint64_t max_off, uint64_t *NR, uint64_t *NC, uint64_t *NB, uint64_t *T,
                     uint64_t *ntile) {
    *NR = (max_off >> SBV_RB) + 1;
    *NC = (*NR + SBV_G - 1) / SBV_G;
    *NB = (n + SBV_E - 1) / SBV_E;
    *T = std::min<uint64_t>(SBV_TMAX, std::max<uint64_t>(1, *NC / 2));
    *ntile = (*NB + *T - 1) / *T;
}
uint64_t sbv_part_scratch_bytes(uint64_t n, uint64_t max_off) {
    uint64_t NR, NC, NB, T, ntile;
    sbv_dims(n, max_off, &NR, &NC, &NB, &T, &ntile);
    return 4 * (2 * NB * SBV_E + NC * NB + NC * ntile * (2 + SBV_G + 1)) + 64;
}
bool sbv_part_ok(uint64_t n, uint64_t max_off) {
    uint64_t NR, NC, NB, T, ntile;
    sbv_dims(n, max_off, &NR, &NC, &NB, &T, &ntile);
    return n < (1ull << 32) && NC <= SBV_NCMAX && ntile <= SBV_NTMAXR;
}
hipError_t launch_setbit_void_part(hipStream_t st, uint64_t n, const uint64_t *offs, uint64_t max_off, void *scratch,
                                   uint8_t *buf, uint64_t cap, uint32_t value) {
    if (!n) return hipSuccess;
    uint64_t NR_, NC_, NB_, T_, nt_;
    sbv_dims(n, max_off, &NR_, &NC_, &NB_, &T_, &nt_);
    const uint32_t NR = uint32_t(NR_), NC = uint32_t(NC_), NB = uint32_t(NB_), T = uint32_t(T_), ntile = uint32_t(nt_);
    uint32_t *chunks = static_cast<uint32_t *>(scratch), *recs = chunks + uint64_t(NB) * SBV_E;
    uint32_t *S = recs + uint64_t(NB) * SBV_E, *tot = S + uint64_t(NC) * NB, *pbase = tot + uint64_t(NC) * ntile;
    uint32_t *rs = pbase + uint64_t(NC) * ntile;
    hipError_t e = hipMemsetAsync(tot, 0, uint64_t(NC) * ntile * 4, st);
    if (e != hipSuccess) return e;
    const size_t lds = (((NC + 3) & ~3u) + SBV_E) * 4;
    hipLaunchKernelGGL(k_sbv_part<uint32_t>, dim3(NB), dim3(SBV_PTPB), lds, st, n, offs, nullptr, nullptr, 0u, NC, NB,
                       T, ntile, chunks, S, tot);
    SK_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sbv_fine<uint32_t>, dim3(ntile, NC), dim3(SBV_PTPB), 0, st, NC, NB, T, ntile, chunks, S, tot,
                       pbase, rs, recs);
    SK_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sbv_runs, dim3(NR), dim3(SBV_TPB), 0, st, ntile, pbase, rs, recs, buf, cap, value);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

// SETBIT with replies over the region partition (u64 records): NRv virtual regions, segments sorted by rb
uint64_t sbr_scratch_bytes(uint64_t n, uint64_t NRv) {
    uint64_t NR, NC, NB, T, ntile;
    sbv_dims(n, (NRv << SBV_RB) - 1, &NR, &NC, &NB, &T, &ntile);
    return 8 * (2 * NB * SBV_E) + 4 * (NC * NB + NC * ntile * (2 + SBV_G + 1)) + 64;
}
bool sbr_ok(uint64_t n, uint64_t NRv) {
    uint64_t NR, NC, NB, T, ntile;
    if (!NRv || NRv > (uint64_t(SBV_NCMAX) * SBV_G)) return false;
    sbv_dims(n, (NRv << SBV_RB) - 1, &NR, &NC, &NB, &T, &ntile);
    return n <= (1ull << 30) && NC <= SBV_NCMAX && ntile <= SBV_NTMAXR;
}
hipError_t launch_setbit_regions(hipStream_t st, uint64_t n, const uint64_t *offs, const uint32_t *vrb,
                                 const uint8_t *vals, uint32_t value_all, uint64_t NRv, const void *seg, uint32_t nseg,
                                 void *scratch, uint8_t *out) {
    if (!n) return hipSuccess;
    uint64_t NR_, NC_, NB_, T_, nt_;
    sbv_dims(n, (NRv << SBV_RB) - 1, &NR_, &NC_, &NB_, &T_, &nt_);
    const uint32_t NR = uint32_t(NR_), NC = uint32_t(NC_), NB = uint32_t(NB_), T = uint32_t(T_), ntile = uint32_t(nt_);
    uint64_t *chunks = static_cast<uint64_t *>(scratch), *recs = chunks + uint64_t(NB) * SBV_E;
    uint32_t *S = reinterpret_cast<uint32_t *>(recs + uint64_t(NB) * SBV_E), *tot = S + uint64_t(NC) * NB;
    uint32_t *pbase = tot + uint64_t(NC) * ntile, *rs = pbase + uint64_t(NC) * ntile;
    hipError_t e = hipMemsetAsync(tot, 0, uint64_t(NC) * ntile * 4, st);
    if (e != hipSuccess) return e;
    const size_t lds = ((NC + 3) & ~3u) * 4 + size_t(SBV_E) * 8;
    static bool attr = false;
    if (!attr) {
        e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sbv_part<uint64_t>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(((SBV_NCMAX + 3) & ~3u) * 4 + SBV_E * 8));
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(k_sbv_part<uint64_t>, dim3(NB), dim3(SBV_PTPB), lds, st, n, offs, vrb, vals, value_all & 1u, NC,
                       NB, T, ntile, chunks, S, tot);
    SK_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sbv_fine<uint64_t>, dim3(ntile, NC), dim3(SBV_PTPB), 0, st, NC, NB, T, ntile, chunks, S, tot,
                       pbase, rs, recs);
    SK_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sbr_runs, dim3(NR), dim3(SBR_TPB), 0, st, ntile, pbase, rs, recs, chunks,
                       static_cast<const SbrSeg *>(seg), nseg, out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_bit_range(hipStream_t st, uint8_t *buf, uint64_t from, uint64_t to, uint32_t value) {
    if (from >= to) return hipSuccess;
    uint64_t nvec = (((to - 1) >> 3) >> 4) - ((from >> 3) >> 4) + 1;
    hipLaunchKernelGGL(k_bit_range, dim3(grid_for(nvec, 256)), dim3(256), 0, st, buf, from, to, value);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_max_u64(hipStream_t st, uint64_t n, const uint64_t *v, uint64_t *out) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    if (e != hipSuccess || !n) return e;
    hipLaunchKernelGGL(k_max_u64, dim3(grid_for((n + 1) / 2, 256 * SK_MX_UNROLL, 2048)), dim3(256), 0, st, n, v, out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_bitcount(hipStream_t st, const uint8_t *buf, uint64_t len, uint64_t *out) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    if (e != hipSuccess || !len) return e;
    hipLaunchKernelGGL(k_bitcount, dim3(grid_for((len + 15) / 16, 256 * SK_BC_UNROLL, 2048)), dim3(256), 0, st, buf, len,
                       (unsigned long long *)out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_bitop(hipStream_t st, int op, uint32_t nsrc, const uint8_t *const *srcs, const uint64_t *lens,
                        uint64_t maxlen, uint8_t *dst) {
    if (!maxlen) return hipSuccess;
    hipLaunchKernelGGL((k_bitop<SK_BO_UNROLL, true>), dim3(grid_for((maxlen + 15) / 16, 256 * SK_BO_UNROLL, 4096)),
                       dim3(256), 0, st, op, nsrc, srcs, lens, maxlen, dst);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t gen_jackson_scan_size(uint64_t n, size_t *bytes) {
    size_t sz = 0;
    hipError_t e = rocprim::inclusive_scan(nullptr, sz, (const uint64_t *)nullptr, (uint64_t *)nullptr, size_t(n),
                                           rocprim::plus<uint64_t>());
    *bytes = sz;
    return e;
}

// lens: scratch u64[n]; off: u64[n+1]
hipError_t launch_gen_jackson(hipStream_t st, uint64_t n, uint64_t seed, const uint64_t *idx, uint64_t first,
                              uint64_t *lens, void *tmp, size_t tmp_bytes, uint64_t *off, uint8_t *out) {
    if (!n) return hipMemsetAsync(off, 0, 8, st);
    hipLaunchKernelGGL(k_gen_len, dim3(grid_for(n, 256)), dim3(256), 0, st, n, seed, idx, first, lens);
    SK_LAUNCH_CHECK();
    hipError_t e = hipMemsetAsync(off, 0, 8, st);
    if (e != hipSuccess) return e;
    size_t sz = tmp_bytes;
    e = rocprim::inclusive_scan(tmp, sz, lens, off + 1, size_t(n), rocprim::plus<uint64_t>(), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gen_write, dim3(grid_for(n, 256)), dim3(256), 0, st, n, seed, idx, first, off, out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}


// routing: cnt u32[world * nblk + 1] scratch, tmp rocprim scratch; base written in place of cnt
uint32_t route_blocks(uint64_t n) { return uint32_t((n + SK_RT_EPB - 1) / SK_RT_EPB); }
uint32_t route_max_world() { return SK_RT_MAXW; }
hipError_t route_scan_size(uint64_t m, size_t *bytes) {
    size_t sz = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, sz, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u, size_t(m),
                                           rocprim::plus<uint32_t>());
    *bytes = sz;
    return e;
}
hipError_t launch_route(hipStream_t st, uint64_t n, const uint64_t *offs, const uint8_t *vals, uint64_t shard_bits,
                        uint32_t world, uint32_t *cnt, uint32_t *base, void *tmp, size_t tmp_bytes, uint32_t *bad,
                        uint64_t *send, uint8_t *svals, uint32_t *dst) {
    if (!n) return hipSuccess;
    if (world > SK_RT_MAXW || !world) return hipErrorInvalidValue;
    const uint32_t nblk = route_blocks(n);
    hipLaunchKernelGGL(k_route_count, dim3(nblk), dim3(SK_RT_TPB), 0, st, n, offs, shard_bits, world, nblk, cnt, bad);
    SK_LAUNCH_CHECK();
    size_t sz = tmp_bytes;
    hipError_t e = rocprim::exclusive_scan(tmp, sz, cnt, base, 0u, size_t(world) * nblk + 1, rocprim::plus<uint32_t>(),
                                           st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_route_scatter, dim3(nblk), dim3(SK_RT_TPB), 0, st, n, offs, vals, shard_bits, world, nblk,
                       base, send, svals, dst);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}
hipError_t launch_unroute(hipStream_t st, uint64_t n, const uint32_t *dst, const uint8_t *rep, uint8_t *out) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_unroute, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, n, dst, rep, out);
    SK_LAUNCH_CHECK();
    return hipSuccess;
}

} // namespace sk
