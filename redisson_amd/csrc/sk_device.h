// sk_device.h -- device-side byte readers and hash functions for gfx950.
//
// Keys arrive as (off u64[n+1], bytes u8[]) with arbitrary byte alignment
// (Jackson-encoded Longs are 20-39 B).  Rather than byte loads, every 8-byte
// block is assembled from two naturally aligned 8-byte loads and a funnel
// shift, so a key costs ~len/8+2 dword-pair loads that hit L1 for neighbours.
// Contract: byte buffers carry >= 16 readable bytes of padding after the last
// key (the library's staging buffers do; _dev callers must).
//
// Hash functions restate the third-party algorithms on the path (the oracle
// in oracle/sketch_oracle.c is the CPU checker; this file never calls it):
//   murmur64a  -- redis 3.2 hyperloglog.c MurmurHash64A (PFADD)
//   xxh64      -- OpenHFT xx_r39() (M:RedissonBloomFilter.java:117)
//   farm_uo64  -- OpenHFT farmUo() = farmhashuo::Hash64 (:118)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sk {

// HLL slab handles from sk_hll_resolve carry the slab's generation in the top 8 bits (stale caller-cached ids
// are rejected by the host entry points); kernels index the arena with the low 24 bits
#define SK_SLAB_MASK 0xffffffu
// elements at least this long are hashed by the bit-round scan (k_ms_rounds) before the PFADD hash pass
#define SK_LONG_ELEM (uint64_t(1) << 16)

__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, unsigned sh) {
    // (lo >> sh) | (hi << (64 - sh)) for sh = 8 * (0..7): the 32-bit word pair picked by sh >= 32, then two
    // byte-aligned 32-bit funnel shifts (v_alignbyte_b32) -- full-rate 32-bit ops instead of three 64-bit shifts
    const bool up = sh & 32u;
    const uint32_t w1 = uint32_t(lo >> 32), w2 = uint32_t(hi);
    const uint32_t a0 = up ? w1 : uint32_t(lo), a1 = up ? w2 : w1, a2 = up ? uint32_t(hi >> 32) : w2;
    const uint32_t b = (sh >> 3) & 3u;
    return uint64_t(__builtin_amdgcn_alignbyte(a1, a0, b)) | (uint64_t(__builtin_amdgcn_alignbyte(a2, a1, b)) << 32);
}

// unaligned little-endian 8-byte load (over-reads < 16 B past p)
__device__ __forceinline__ uint64_t ldu64(const uint8_t *p) {
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint64_t *q = reinterpret_cast<const uint64_t *>(a & ~uintptr_t(7));
    unsigned sh = unsigned(a & 7) * 8u;
    return funnel(q[0], q[1], sh);
}
__device__ __forceinline__ uint32_t ldu32(const uint8_t *p) { return uint32_t(ldu64(p)); }

// Sequential reader: each next() costs one aligned load.
struct Stream {
    const uint64_t *q;
    uint64_t cur;
    unsigned sh;
    __device__ __forceinline__ explicit Stream(const uint8_t *p) {
        uintptr_t a = reinterpret_cast<uintptr_t>(p);
        q = reinterpret_cast<const uint64_t *>(a & ~uintptr_t(7));
        sh = unsigned(a & 7) * 8u;
        cur = q[0];
    }
    __device__ __forceinline__ uint64_t next() {
        uint64_t nxt = *++q;
        uint64_t v = funnel(cur, nxt, sh);
        cur = nxt;
        return v;
    }
};

__device__ __forceinline__ uint64_t low_bytes(uint64_t v, unsigned nbytes) {
    // keep the low nbytes (0..7) bytes
    return nbytes ? (v & (~0ull >> (64 - 8 * nbytes))) : 0ull;
}

// ------------------------------------------------------- key byte readers
// Hash functions are written against a Reader: u64(p) = 8 little-endian
// bytes starting at byte position p of the key.  GlobalReader reads HBM
// directly (two aligned loads + funnel shift); LdsReader reads a workgroup's
// key bytes that were staged into LDS with coalesced 16-byte loads
// (stage_keys below), which turns ~len/8 scattered line requests per lane into
// ~1 coalesced request per 16 bytes per workgroup.
struct GlobalReader {
    const uint8_t *base;
    __device__ __forceinline__ uint64_t u64(uint32_t p) const { return ldu64(base + p); }
};
struct LdsReader {
    const uint64_t *lds; // __shared__ words
    uint32_t base;       // byte position of the key inside the staged window
    __device__ __forceinline__ uint64_t u64(uint32_t p) const {
        uint32_t a = base + p;
        uint32_t q = a >> 3, sh = (a & 7u) * 8u;
        return funnel(lds[q], lds[q + 1], sh);
    }
};

// Stage bytes [lo, hi) of a global buffer into LDS words and zero the next
// 16 B (readers look up to 15 B past a key's end, masked); returns the byte
// position of `lo` inside the window (lo rounded down to 16 B).  Global reads
// stay below hi + 16 (the buffers' padding contract).  All threads of the
// workgroup must call it; ends with a barrier.
__device__ __forceinline__ uint32_t stage_keys(const uint8_t *bytes, uint64_t lo, uint64_t hi, uint64_t *lds) {
    uint64_t a0 = lo & ~uint64_t(15);
    uint32_t nvec = uint32_t((hi - a0 + 15) >> 4);
    const uint4 *src = reinterpret_cast<const uint4 *>(bytes + a0);
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
    for (uint32_t v = threadIdx.x; v <= nvec; v += blockDim.x) dst[v] = v < nvec ? src[v] : make_uint4(0, 0, 0, 0);
    __syncthreads();
    return uint32_t(lo - a0);
}
// LDS window (u64 words) for one 256-element workgroup: room for keys of
// mean length <= ~90 B; larger windows fall back to GlobalReader.
#define SK_STAGE_WORDS 3072
__device__ __forceinline__ bool stage_fits(uint64_t lo, uint64_t hi) {
    return (hi - (lo & ~uint64_t(15))) + 32 <= uint64_t(SK_STAGE_WORDS) * 8;
}

// ---------------------------------------------------------------- Murmur
template <class R> __device__ __forceinline__ uint64_t murmur64a_r(const R &rd, uint32_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = seed ^ (uint64_t(len) * m);
    uint32_t nb = len >> 3;
    for (uint32_t i = 0; i < nb; i++) {
        uint64_t k = rd.u64(8 * i);
        k *= m;
        k ^= k >> 47;
        k *= m;
        h ^= k;
        h *= m;
    }
    unsigned tail = len & 7u;
    if (tail) {
        h ^= low_bytes(rd.u64(8 * nb), tail);
        h *= m;
    }
    h ^= h >> 47;
    h *= m;
    h ^= h >> 47;
    return h;
}

__device__ __forceinline__ uint64_t murmur64a(const uint8_t *data, uint32_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = seed ^ (uint64_t(len) * m);
    Stream s(data);
    uint32_t nb = len >> 3;
    for (uint32_t i = 0; i < nb; i++) {
        uint64_t k = s.next();
        k *= m;
        k ^= k >> 47;
        k *= m;
        h ^= k;
        h *= m;
    }
    unsigned tail = len & 7u;
    if (tail) {
        h ^= low_bytes(s.next(), tail);
        h *= m;
    }
    h ^= h >> 47;
    h *= m;
    h ^= h >> 47;
    return h;
}

// ---------------------------------------------------------------- XXH64
#define SK_XP1 0x9E3779B185EBCA87ull
#define SK_XP2 0xC2B2AE3D27D4EB4Full
#define SK_XP3 0x165667B19E3779F9ull
#define SK_XP4 0x85EBCA77C2B2AE63ull
#define SK_XP5 0x27D4EB2F165667C5ull

__device__ __forceinline__ uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t rotr(uint64_t x, int r) { return (x >> r) | (x << (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * SK_XP2;
    acc = rotl(acc, 31);
    return acc * SK_XP1;
}
__device__ __forceinline__ uint64_t xmerge(uint64_t acc, uint64_t v) {
    acc ^= xround(0, v);
    return acc * SK_XP1 + SK_XP4;
}

// the part after the stripes: h already holds the stripes' merge (or seed + P5) plus len; bytes [pos, pos + rem)
template <class R> __device__ __forceinline__ uint64_t xxh64_tail(const R &rd, uint64_t h, uint32_t pos, uint32_t rem) {
    while (rem >= 8) {
        h ^= xround(0, rd.u64(pos));
        h = rotl(h, 27) * SK_XP1 + SK_XP4;
        pos += 8;
        rem -= 8;
    }
    if (rem) {
        uint64_t w = rd.u64(pos); // the last 1..7 bytes, low-aligned
        if (rem >= 4) {
            h ^= (w & 0xffffffffull) * SK_XP1;
            h = rotl(h, 23) * SK_XP2 + SK_XP3;
            w >>= 32;
            rem -= 4;
        }
        while (rem) {
            h ^= (w & 0xffull) * SK_XP5;
            h = rotl(h, 11) * SK_XP1;
            w >>= 8;
            rem--;
        }
    }
    h ^= h >> 33;
    h *= SK_XP2;
    h ^= h >> 29;
    h *= SK_XP3;
    h ^= h >> 32;
    return h;
}
template <class R> __device__ __forceinline__ uint64_t xxh64_r(const R &rd, uint32_t len) {
    const uint64_t seed = 0;
    uint64_t h;
    uint32_t pos = 0, rem = len;
    if (len >= 32) {
        uint64_t v1 = seed + SK_XP1 + SK_XP2, v2 = seed + SK_XP2, v3 = seed, v4 = seed - SK_XP1;
        do {
            v1 = xround(v1, rd.u64(pos));
            v2 = xround(v2, rd.u64(pos + 8));
            v3 = xround(v3, rd.u64(pos + 16));
            v4 = xround(v4, rd.u64(pos + 24));
            pos += 32;
            rem -= 32;
        } while (rem >= 32);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + SK_XP5;
    }
    return xxh64_tail(rd, h + len, pos, rem);
}
__device__ __forceinline__ uint64_t xxh64(const uint8_t *p, uint32_t len) { return xxh64_r(GlobalReader{p}, len); }

// ---------------------------------------------------------------- FarmHash
#define SK_K0 0xc3a5c85c97cb3127ull
#define SK_K1 0xb492b66fbe98f273ull
#define SK_K2 0x9ae16a3b2f90404full

__device__ __forceinline__ uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }
__device__ __forceinline__ uint64_t hl16(uint64_t u, uint64_t v, uint64_t mul) {
    uint64_t a = (u ^ v) * mul;
    a ^= (a >> 47);
    uint64_t b = (v ^ a) * mul;
    b ^= (b >> 47);
    return b * mul;
}
struct P2 {
    uint64_t first, second;
};
template <class R> __device__ __forceinline__ P2 weak32(const R &rd, uint32_t s, uint64_t a, uint64_t b) {
    uint64_t w = rd.u64(s), x = rd.u64(s + 8), y = rd.u64(s + 16), z = rd.u64(s + 24);
    a += w;
    b = rotr(b + a + z, 21);
    uint64_t c = a;
    a += x;
    a += y;
    b += rotr(a, 44);
    return P2{a + z, b + c};
}

template <class R> __device__ __forceinline__ uint64_t farm_na_short(const R &rd, uint32_t len) {
    const uint32_t s = 0;
    // farmhashna::Hash64 for len <= 64
    if (len <= 16) {
        if (len >= 8) {
            uint64_t mul = SK_K2 + uint64_t(len) * 2;
            uint64_t a = rd.u64(s) + SK_K2;
            uint64_t b = rd.u64(s + len - 8);
            uint64_t c = rotr(b, 37) * mul + a;
            uint64_t d = (rotr(a, 25) + b) * mul;
            return hl16(c, d, mul);
        }
        if (len >= 4) {
            uint64_t mul = SK_K2 + uint64_t(len) * 2;
            uint64_t a = uint32_t(rd.u64(s));
            return hl16(uint64_t(len) + (a << 3), uint32_t(rd.u64(s + len - 4)), mul);
        }
        if (len > 0) {
            uint64_t w = rd.u64(s);
            uint32_t a = uint32_t(w & 0xff), b = uint32_t((w >> (8 * (len >> 1))) & 0xff),
                     c = uint32_t((w >> (8 * (len - 1))) & 0xff);
            uint32_t y = a + (b << 8);
            uint32_t z = len + (c << 2);
            return shift_mix(uint64_t(y) * SK_K2 ^ uint64_t(z) * SK_K0) * SK_K2;
        }
        return SK_K2;
    }
    uint64_t mul = SK_K2 + uint64_t(len) * 2;
    if (len <= 32) {
        uint64_t a = rd.u64(s) * SK_K1;
        uint64_t b = rd.u64(s + 8);
        uint64_t c = rd.u64(s + len - 8) * mul;
        uint64_t d = rd.u64(s + len - 16) * SK_K2;
        return hl16(rotr(a + b, 43) + rotr(c, 30) + d, a + rotr(b + SK_K2, 18) + c, mul);
    }
    uint64_t a = rd.u64(s) * SK_K2;
    uint64_t b = rd.u64(s + 8);
    uint64_t c = rd.u64(s + len - 8) * mul;
    uint64_t d = rd.u64(s + len - 16) * SK_K2;
    uint64_t y = rotr(a + b, 43) + rotr(c, 30) + d;
    uint64_t z = hl16(y, a + rotr(b + SK_K2, 18) + c, mul);
    uint64_t e = rd.u64(s + 16) * mul;
    uint64_t f = rd.u64(s + 24);
    uint64_t g = (y + rd.u64(s + len - 32)) * mul;
    uint64_t h = (z + rd.u64(s + len - 24)) * mul;
    return hl16(rotr(e + f, 43) + rotr(g, 30) + h, e + rotr(f + a, 18) + g, mul);
}

__device__ __forceinline__ uint64_t uo_H(uint64_t x, uint64_t y, uint64_t mul, int r) {
    uint64_t a = (x ^ y) * mul;
    a ^= (a >> 47);
    uint64_t b = (y ^ a) * mul;
    return rotr(b, r) * mul;
}

// farmhashuo::Hash64WithSeeds(s, len, 81, 0) for len > 64 (inlined into the out-of-line pair below; called from
// the other kernels through farm_uo_long)
template <class R> __device__ __forceinline__ uint64_t farm_uo_long_body(const R &rd, uint32_t len) {
    uint32_t s = 0;
    const uint64_t seed0 = 81, seed1 = 0;
    uint64_t x = seed0;
    uint64_t y = seed1 * SK_K2 + 113;
    uint64_t z = shift_mix(y * SK_K2) * SK_K2;
    P2 v{seed0, seed1}, w{0, 0};
    uint64_t u = x - z;
    x *= SK_K2;
    uint64_t mul = SK_K2 + (u & 0x82);
    uint32_t nblk = (len - 1) / 64;
    const uint32_t last64 = len - 64;
    for (uint32_t blk = 0; blk < nblk; blk++, s += 64) {
        uint64_t a0 = rd.u64(s), a1 = rd.u64(s + 8), a2 = rd.u64(s + 16), a3 = rd.u64(s + 24);
        uint64_t a4 = rd.u64(s + 32), a5 = rd.u64(s + 40), a6 = rd.u64(s + 48), a7 = rd.u64(s + 56);
        x += a0 + a1;
        y += a2;
        z += a3;
        v.first += a4;
        v.second += a5 + a1;
        w.first += a6;
        w.second += a7;
        x = rotr(x, 26);
        x *= 9;
        y = rotr(y, 29);
        z *= mul;
        v.first = rotr(v.first, 33);
        v.second = rotr(v.second, 30);
        w.first ^= x;
        w.first *= 9;
        z = rotr(z, 32);
        z += w.second;
        w.second += z;
        z *= 9;
        uint64_t t = u;
        u = y;
        y = t;
        z += a0 + a6;
        v.first += a2;
        v.second += a3;
        w.first += a4;
        w.second += a5 + a6;
        x += a1;
        y += a7;
        y += v.first;
        v.first += x - y;
        v.second += w.first;
        w.first += v.second;
        w.second += x - y;
        x += w.second;
        w.second = rotr(w.second, 34);
        t = u;
        u = z;
        z = t;
    }
    s = last64;
    u *= 9;
    v.second = rotr(v.second, 28);
    v.first = rotr(v.first, 20);
    w.first += ((len - 1) & 63);
    u += y;
    y += u;
    x = rotr(y - x + v.first + rd.u64(s + 8), 37) * mul;
    y = rotr(y ^ v.second ^ rd.u64(s + 48), 42) * mul;
    x ^= w.second * 9;
    y += v.first + rd.u64(s + 40);
    z = rotr(z + w.first, 33) * mul;
    v = weak32(rd, s, v.second * mul, x + w.first);
    w = weak32(rd, s + 32, z + w.second, y + rd.u64(s + 16));
    return uo_H(hl16(v.first + x, w.first ^ y, mul) + z - u, uo_H(v.second + w.second, x, mul, 30) ^ w.first,
                mul, 31);
}

template <class R> __device__ __noinline__ uint64_t farm_uo_long(const R rd, uint32_t len) {
    return farm_uo_long_body(rd, len);
}
template <class R> __device__ __forceinline__ uint64_t farm_uo64_r(const R &rd, uint32_t len) {
    return len <= 64 ? farm_na_short(rd, len) : farm_uo_long(rd, len);
}
__device__ __forceinline__ uint64_t farm_uo64(const uint8_t *s, uint32_t len) {
    return farm_uo64_r(GlobalReader{s}, len);
}

// ---------------------------------------------------------------- Bloom hash pair, shared 16-byte prefix
// Codec-encoded elements share their first bytes: every Jackson Long is `["java.lang.Long",<digits>]`, 20-39 B
// (SURVEY A3), and a typed object starts with its class name.  For 33 <= len <= 63, XXH64 runs one 32-byte stripe,
// whose lanes v1 / v2 take bytes 0-15 alone, and farmhashna's 33-64 path multiplies bytes 0-7 by K2 and combines
// them with bytes 8-15 before anything else.  So an element whose first 16 bytes equal a block-uniform pattern
// (taken from the block's first element, precomputed on the scalar unit) reuses v1, v2, their merge terms and
// farm's prefix terms: 9 of its ~40 64-bit multiplies.  Any other element takes the full functions.  Results are
// identical either way (the same arithmetic, evaluated once per block instead of once per element).
struct BloomPre {
    uint64_t w0, w1;       // the pattern: bytes 0-7 and 8-15
    uint64_t R12, M1, M2;  // XXH64: rotl(v1, 1) + rotl(v2, 7); xround(0, v1); xround(0, v2)
    uint64_t FA, FY0, FZ0; // farmhashna 33-64: a = w0 * K2; rotr(a + w1, 43); a + rotr(w1 + K2, 18)
};
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    return uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(x))) |
           (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(x >> 32))) << 32);
}
// w0 / w1: the same 16 bytes in every lane of the wave (the block's first element, read by every lane)
__device__ __forceinline__ BloomPre bloom_pre(uint64_t w0, uint64_t w1) {
    BloomPre p;
    p.w0 = uniform64(w0);
    p.w1 = uniform64(w1);
    const uint64_t v1 = xround(SK_XP1 + SK_XP2, p.w0), v2 = xround(SK_XP2, p.w1);
    p.R12 = rotl(v1, 1) + rotl(v2, 7);
    p.M1 = xround(0, v1);
    p.M2 = xround(0, v2);
    p.FA = p.w0 * SK_K2;
    p.FY0 = rotr(p.FA + p.w1, 43);
    p.FZ0 = p.FA + rotr(p.w1 + SK_K2, 18);
    return p;
}
// the generic pair, out of line: elements off the shared prefix are rare in a codec's batch, and keeping this code
// out of the hash kernels' round loop keeps the loop unrolled and its registers spill-free
template <class R> __device__ __noinline__ P2 bloom_hash_pair(const R rd, uint32_t len) {
    return P2{xxh64_r(rd, len), len <= 64 ? farm_na_short(rd, len) : farm_uo_long_body(rd, len)}; // a leaf: no stack
}
template <class R>
__device__ __forceinline__ void bloom_hashes_pre(const R &rd, uint32_t len, const BloomPre &pre, uint64_t *h1,
                                                 uint64_t *h2) {
    if (len >= 33 && len <= 63 && rd.u64(0) == pre.w0 && rd.u64(8) == pre.w1) {
        // XXH64 (xxh64_r): one stripe with v1 / v2 from the pattern
        const uint64_t b2 = rd.u64(16), b3 = rd.u64(24);
        const uint64_t v3 = xround(0, b2), v4 = xround(0 - SK_XP1, b3);
        uint64_t h = pre.R12 + rotl(v3, 12) + rotl(v4, 18);
        h = (h ^ pre.M1) * SK_XP1 + SK_XP4; // xmerge(h, v1)
        h = (h ^ pre.M2) * SK_XP1 + SK_XP4; // xmerge(h, v2)
        h = xmerge(h, v3);
        h = xmerge(h, v4);
        *h1 = xxh64_tail(rd, h + len, 32, len - 32);
        // farmhashna::Hash64, 33 <= len <= 64 (farm_na_short) with a / b from the pattern
        const uint64_t mul = SK_K2 + uint64_t(len) * 2;
        const uint64_t c = rd.u64(len - 8) * mul;
        const uint64_t d = rd.u64(len - 16) * SK_K2;
        const uint64_t y = pre.FY0 + rotr(c, 30) + d;
        const uint64_t z = hl16(y, pre.FZ0 + c, mul);
        const uint64_t e = b2 * mul, f = b3;
        const uint64_t g = (y + rd.u64(len - 32)) * mul;
        const uint64_t hh = (z + rd.u64(len - 24)) * mul;
        *h2 = hl16(rotr(e + f, 43) + rotr(g, 30) + hh, e + rotr(f + pre.FA, 18) + g, mul);
        return;
    }
    const P2 h = bloom_hash_pair(rd, len);
    *h1 = h.first;
    *h2 = h.second;
}

// ---------------------------------------------------------------- misc
// x % d for x < 2^63 using a precomputed M = floor((2^64-1)/d): q_est is
// at most 2 below the true quotient, so two conditional subtractions fix it.
__device__ __forceinline__ uint64_t mod_invariant(uint64_t x, uint64_t d, uint64_t M) {
    uint64_t q = __umul64hi(x, M);
    uint64_t r = x - q * d;
    if (r >= d) r -= d;
    if (r >= d) r -= d;
    return r;
}

// Redisson's probe indexes (M:RedissonBloomFilter.java hash(): index_i = (h_i & Long.MAX_VALUE) % size with
// h_0 = h1, h_{i+1} = h_i + (i even ? h2 : h1), wrapping) at two 64-bit reductions per element instead of one per
// probe.  m_i = h_i mod 2^63 steps by D = d mod 2^63 (d = h2 or h1), wrapping at 2^63, so
//   index_{i+1} = index_i + (D mod size) - [m_i + D >= 2^63] * (2^63 mod size)   (then one correction into [0, size)).
// Sizes are < 2^62 (Redis strings: <= 2^32 bits), so the sum fits a signed 64-bit word.
struct BloomIdx {
    uint64_t m, r, size, D1, D2, A1, A2, C;
    __device__ __forceinline__ BloomIdx(uint64_t h1, uint64_t h2, uint64_t size_, uint64_t magic) : size(size_) {
        const uint64_t MAXL = 0x7fffffffffffffffull;
        D1 = h1 & MAXL;
        D2 = h2 & MAXL;
        A1 = mod_invariant(D1, size, magic);
        A2 = mod_invariant(D2, size, magic);
        C = mod_invariant(MAXL, size, magic) + 1; // 2^63 mod size (uniform)
        if (C == size) C = 0;
        m = D1;
        r = A1;
    }
    // index of probe p+1 from that of probe p
    __device__ __forceinline__ void next(int p) {
        const uint64_t D = (p & 1) ? D1 : D2, A = (p & 1) ? A1 : A2;
        const uint64_t s = m + D;
        const bool w = s >= (1ull << 63);
        m = w ? s - (1ull << 63) : s;
        int64_t t = int64_t(r + A) - (w ? int64_t(C) : 0);
        if (t < 0) t += int64_t(size);
        else if (t >= int64_t(size)) t -= int64_t(size);
        r = uint64_t(t);
    }
};

// The same walk for sizes < 2^32 (every Redis bit string: Bloom sizes are <= 4,294,967,294), the index arithmetic
// in 32-bit words: r + A < 2 size is reduced with one conditional subtraction (its carry out of 32 bits included),
// then C is taken off modulo size.  Only the 63-bit m stays 64-bit.
struct BloomIdx32 {
    uint64_t m, D1, D2;
    uint32_t r, A1, A2, B1, B2, size; // B = (A - C) mod size: the step when m wraps past 2^63
    __device__ __forceinline__ BloomIdx32(uint64_t h1, uint64_t h2, uint64_t size_, uint64_t magic)
        : size(uint32_t(size_)) {
        const uint64_t MAXL = 0x7fffffffffffffffull;
        D1 = h1 & MAXL;
        D2 = h2 & MAXL;
        A1 = uint32_t(mod_invariant(D1, size_, magic));
        A2 = uint32_t(mod_invariant(D2, size_, magic));
        uint64_t c = mod_invariant(MAXL, size_, magic) + 1; // 2^63 mod size (uniform)
        const uint32_t C = c == size_ ? 0u : uint32_t(c);
        B1 = A1 >= C ? A1 - C : A1 - C + size;
        B2 = A2 >= C ? A2 - C : A2 - C + size;
        m = D1;
        r = A1;
    }
    // index += (D mod size) - [m + D >= 2^63] * (2^63 mod size), mod size: one step term chosen by the wrap, then
    // one conditional subtraction (r + a < 2 * size; the carry out of 32 bits counts too)
    __device__ __forceinline__ void next(int p) {
        const uint64_t D = (p & 1) ? D1 : D2;
        const uint64_t s = m + D;
        const bool w = (s >> 63) != 0;
        m = s & 0x7fffffffffffffffull;
        const uint32_t a = w ? ((p & 1) ? B1 : B2) : ((p & 1) ? A1 : A2);
        const uint32_t x = r + a;
        r = (x < r || x >= size) ? x - size : x;
    }
};

// Redis bit strings are MSB-first: bit i lives in byte i>>3 at mask 0x80>>(i&7)
__device__ __forceinline__ int get_bit(const uint8_t *buf, uint64_t len, uint64_t idx) {
    uint64_t byte = idx >> 3;
    if (byte >= len) return 0;
    return (buf[byte] >> (7 - unsigned(idx & 7))) & 1;
}
// word-aligned address + mask of bit idx inside a little-endian u32
__device__ __forceinline__ uint32_t *bit_word(uint8_t *buf, uint64_t idx, uint32_t *mask) {
    uint64_t byte = idx >> 3;
    *mask = 1u << (unsigned(byte & 3) * 8u + (7u - unsigned(idx & 7)));
    return reinterpret_cast<uint32_t *>(buf + (byte & ~uint64_t(3)));
}

} // namespace sk
