/*
 * sketch_oracle.c -- CPU restatement (plain C99) of the Redisson sketch path.
 * TEST INFRASTRUCTURE ONLY: see sketch_oracle.h for the rules and the pins.
 *
 * Every function names the reference file:line (M: = /root/reference/src/main/
 * java/org/redisson/) or the third-party algorithm it restates.  Third-party
 * code is NOT in /root/reference; it is restated from the published
 * algorithms (redis-server 3.2.0 hyperloglog.c / bitops.c, OpenHFT
 * zero-allocation-hashing 0.5 = XXH64 + Google farmhash).
 */
#include "sketch_oracle.h"
#include <math.h>
#include <string.h>

static inline uint64_t ld64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v; /* x86-64 / gfx950 are little endian: matches Fetch()/read64 LE */
}
static inline uint32_t ld32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
/* farmhash's Rotate() is a right rotation */
static inline uint64_t rotr64(uint64_t x, int r) { return r == 0 ? x : ((x >> r) | (x << (64 - r))); }

/* ------------------------------------------------------------------ */
/* MurmurHash64A (Austin Appleby), as vendored in redis 3.2 hyperloglog.c,
 * little-endian path.  Called by hllPatLen with seed 0xadc83b19.        */
uint64_t or_murmur64a(const uint8_t *data, int64_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ULL;
    const int r = 47;
    uint64_t h = seed ^ ((uint64_t)len * m);
    const uint8_t *end = data + (len - (len & 7));
    while (data != end) {
        uint64_t k = ld64(data);
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
        data += 8;
    }
    switch (len & 7) {
    case 7: h ^= (uint64_t)data[6] << 48; /* fallthrough */
    case 6: h ^= (uint64_t)data[5] << 40; /* fallthrough */
    case 5: h ^= (uint64_t)data[4] << 32; /* fallthrough */
    case 4: h ^= (uint64_t)data[3] << 24; /* fallthrough */
    case 3: h ^= (uint64_t)data[2] << 16; /* fallthrough */
    case 2: h ^= (uint64_t)data[1] << 8;  /* fallthrough */
    case 1: h ^= (uint64_t)data[0]; h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}

/* SMHasher VerificationTest: keys {}, {0}, {0,1}, ... {0..254} hashed with
 * seed 256-i, the 256 x 8-byte results hashed with seed 0; first 4 bytes LE. */
uint32_t or_murmur64a_verification(void) {
    uint8_t key[256], hashes[256 * 8];
    memset(key, 0, sizeof key);
    for (int i = 0; i < 256; i++) {
        key[i] = (uint8_t)i;
        uint64_t h = or_murmur64a(key, i, (uint64_t)(256 - i));
        memcpy(&hashes[i * 8], &h, 8);
    }
    uint64_t f = or_murmur64a(hashes, 256 * 8, 0);
    return (uint32_t)(f & 0xffffffffu);
}

/* ------------------------------------------------------------------ */
/* XXH64 (Yann Collet) = OpenHFT LongHashFunction.xx_r39() with seed 0,
 * called at M:RedissonBloomFilter.java:117.                             */
#define XP1 0x9E3779B185EBCA87ULL
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL
static inline uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * XP2;
    acc = rotl64(acc, 31);
    return acc * XP1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t v) {
    acc ^= xround(0, v);
    return acc * XP1 + XP4;
}
uint64_t or_xxh64(const uint8_t *p, uint64_t len, uint64_t seed) {
    const uint8_t *end = p + len;
    uint64_t h;
    if (len >= 32) {
        const uint8_t *limit = end - 32;
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        do {
            v1 = xround(v1, ld64(p));
            v2 = xround(v2, ld64(p + 8));
            v3 = xround(v3, ld64(p + 16));
            v4 = xround(v4, ld64(p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += len;
    while (p + 8 <= end) {
        h ^= xround(0, ld64(p));
        h = rotl64(h, 27) * XP1 + XP4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)ld32(p) * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * XP5;
        h = rotl64(h, 11) * XP1;
        p++;
    }
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

/* ------------------------------------------------------------------ */
/* Google farmhash: farmhashna::Hash64 and farmhashuo::Hash64 (= OpenHFT
 * LongHashFunction.farmUo(), called at M:RedissonBloomFilter.java:118). */
static const uint64_t k0 = 0xc3a5c85c97cb3127ULL;
static const uint64_t k1 = 0xb492b66fbe98f273ULL;
static const uint64_t k2 = 0x9ae16a3b2f90404fULL;

static inline uint64_t shift_mix(uint64_t v) { return v ^ (v >> 47); }
static inline uint64_t hash_len16_mul(uint64_t u, uint64_t v, uint64_t mul) {
    uint64_t a = (u ^ v) * mul;
    a ^= (a >> 47);
    uint64_t b = (v ^ a) * mul;
    b ^= (b >> 47);
    b *= mul;
    return b;
}
static inline uint64_t hash_len16(uint64_t u, uint64_t v) {
    return hash_len16_mul(u, v, 0x9ddfea08eb382d69ULL); /* Hash128to64 */
}
static uint64_t hash_len_0to16(const uint8_t *s, uint64_t len) {
    if (len >= 8) {
        uint64_t mul = k2 + len * 2;
        uint64_t a = ld64(s) + k2;
        uint64_t b = ld64(s + len - 8);
        uint64_t c = rotr64(b, 37) * mul + a;
        uint64_t d = (rotr64(a, 25) + b) * mul;
        return hash_len16_mul(c, d, mul);
    }
    if (len >= 4) {
        uint64_t mul = k2 + len * 2;
        uint64_t a = ld32(s);
        return hash_len16_mul(len + (a << 3), ld32(s + len - 4), mul);
    }
    if (len > 0) {
        uint8_t a = s[0], b = s[len >> 1], c = s[len - 1];
        uint32_t y = (uint32_t)a + ((uint32_t)b << 8);
        uint32_t z = (uint32_t)len + ((uint32_t)c << 2);
        return shift_mix((uint64_t)y * k2 ^ (uint64_t)z * k0) * k2;
    }
    return k2;
}
static uint64_t hash_len_17to32(const uint8_t *s, uint64_t len) {
    uint64_t mul = k2 + len * 2;
    uint64_t a = ld64(s) * k1;
    uint64_t b = ld64(s + 8);
    uint64_t c = ld64(s + len - 8) * mul;
    uint64_t d = ld64(s + len - 16) * k2;
    return hash_len16_mul(rotr64(a + b, 43) + rotr64(c, 30) + d,
                          a + rotr64(b + k2, 18) + c, mul);
}
static uint64_t na_hash_len_33to64(const uint8_t *s, uint64_t len) {
    uint64_t mul = k2 + len * 2;
    uint64_t a = ld64(s) * k2;
    uint64_t b = ld64(s + 8);
    uint64_t c = ld64(s + len - 8) * mul;
    uint64_t d = ld64(s + len - 16) * k2;
    uint64_t y = rotr64(a + b, 43) + rotr64(c, 30) + d;
    uint64_t z = hash_len16_mul(y, a + rotr64(b + k2, 18) + c, mul);
    uint64_t e = ld64(s + 16) * mul;
    uint64_t f = ld64(s + 24);
    uint64_t g = (y + ld64(s + len - 32)) * mul;
    uint64_t h = (z + ld64(s + len - 24)) * mul;
    return hash_len16_mul(rotr64(e + f, 43) + rotr64(g, 30) + h,
                          e + rotr64(f + a, 18) + g, mul);
}
typedef struct { uint64_t first, second; } u64pair;
static inline u64pair weak32(uint64_t w, uint64_t x, uint64_t y, uint64_t z, uint64_t a, uint64_t b) {
    a += w;
    b = rotr64(b + a + z, 21);
    uint64_t c = a;
    a += x;
    a += y;
    b += rotr64(a, 44);
    u64pair r = {a + z, b + c};
    return r;
}
static inline u64pair weak32s(const uint8_t *s, uint64_t a, uint64_t b) {
    return weak32(ld64(s), ld64(s + 8), ld64(s + 16), ld64(s + 24), a, b);
}

uint64_t or_farmhash_na64(const uint8_t *s, uint64_t len) {
    const uint64_t seed = 81;
    if (len <= 32) {
        return len <= 16 ? hash_len_0to16(s, len) : hash_len_17to32(s, len);
    } else if (len <= 64) {
        return na_hash_len_33to64(s, len);
    }
    uint64_t x = seed;
    uint64_t y = seed * k1 + 113;
    uint64_t z = shift_mix(y * k2 + 113) * k2;
    u64pair v = {0, 0}, w = {0, 0};
    x = x * k2 + ld64(s);
    const uint8_t *end = s + ((len - 1) / 64) * 64;
    const uint8_t *last64 = end + ((len - 1) & 63) - 63;
    do {
        x = rotr64(x + y + v.first + ld64(s + 8), 37) * k1;
        y = rotr64(y + v.second + ld64(s + 48), 42) * k1;
        x ^= w.second;
        y += v.first + ld64(s + 40);
        z = rotr64(z + w.first, 33) * k1;
        v = weak32s(s, v.second * k1, x + w.first);
        w = weak32s(s + 32, z + w.second, y + ld64(s + 16));
        uint64_t t = z; z = x; x = t;
        s += 64;
    } while (s != end);
    uint64_t mul = k1 + ((z & 0xff) << 1);
    s = last64;
    w.first += ((len - 1) & 63);
    v.first += w.first;
    w.first += v.first;
    x = rotr64(x + y + v.first + ld64(s + 8), 37) * mul;
    y = rotr64(y + v.second + ld64(s + 48), 42) * mul;
    x ^= w.second * 9;
    y += v.first * 9 + ld64(s + 40);
    z = rotr64(z + w.first, 33) * mul;
    v = weak32s(s, v.second * mul, x + w.first);
    w = weak32s(s + 32, z + w.second, y + ld64(s + 16));
    { uint64_t t = z; z = x; x = t; }
    return hash_len16_mul(hash_len16_mul(v.first, w.first, mul) + shift_mix(y) * k0 + z,
                          hash_len16_mul(v.second, w.second, mul) + x, mul);
}

static inline uint64_t uo_H(uint64_t x, uint64_t y, uint64_t mul, int r) {
    uint64_t a = (x ^ y) * mul;
    a ^= (a >> 47);
    uint64_t b = (y ^ a) * mul;
    return rotr64(b, r) * mul;
}

static uint64_t uo_hash64_with_seeds(const uint8_t *s, uint64_t len, uint64_t seed0, uint64_t seed1) {
    /* len > 64 only (len <= 64 goes to farmhashna in Hash64) */
    uint64_t x = seed0;
    uint64_t y = seed1 * k2 + 113;
    uint64_t z = shift_mix(y * k2) * k2;
    u64pair v = {seed0, seed1}, w = {0, 0};
    uint64_t u = x - z;
    x *= k2;
    uint64_t mul = k2 + (u & 0x82);
    const uint8_t *end = s + ((len - 1) / 64) * 64;
    const uint8_t *last64 = end + ((len - 1) & 63) - 63;
    do {
        uint64_t a0 = ld64(s), a1 = ld64(s + 8), a2 = ld64(s + 16), a3 = ld64(s + 24);
        uint64_t a4 = ld64(s + 32), a5 = ld64(s + 40), a6 = ld64(s + 48), a7 = ld64(s + 56);
        x += a0 + a1;
        y += a2;
        z += a3;
        v.first += a4;
        v.second += a5 + a1;
        w.first += a6;
        w.second += a7;

        x = rotr64(x, 26);
        x *= 9;
        y = rotr64(y, 29);
        z *= mul;
        v.first = rotr64(v.first, 33);
        v.second = rotr64(v.second, 30);
        w.first ^= x;
        w.first *= 9;
        z = rotr64(z, 32);
        z += w.second;
        w.second += z;
        z *= 9;
        { uint64_t t = u; u = y; y = t; }

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
        w.second = rotr64(w.second, 34);
        { uint64_t t = u; u = z; z = t; }
        s += 64;
    } while (s != end);
    s = last64;
    u *= 9;
    v.second = rotr64(v.second, 28);
    v.first = rotr64(v.first, 20);
    w.first += ((len - 1) & 63);
    u += y;
    y += u;
    x = rotr64(y - x + v.first + ld64(s + 8), 37) * mul;
    y = rotr64(y ^ v.second ^ ld64(s + 48), 42) * mul;
    x ^= w.second * 9;
    y += v.first + ld64(s + 40);
    z = rotr64(z + w.first, 33) * mul;
    v = weak32s(s, v.second * mul, x + w.first);
    w = weak32s(s + 32, z + w.second, y + ld64(s + 16));
    return uo_H(hash_len16_mul(v.first + x, w.first ^ y, mul) + z - u,
                uo_H(v.second + w.second, x, mul, 30) ^ w.first, mul, 31);
}

uint64_t or_farmhash_uo64(const uint8_t *s, uint64_t len) {
    return len <= 64 ? or_farmhash_na64(s, len) : uo_hash64_with_seeds(s, len, 81, 0);
}

/* ------------------------------------------------------------------ */
/* CRC16-XMODEM, M:connection/CRC16.java:23-61 (table-free bitwise form of
 * the same polynomial 0x1021, init 0, no reflection).                    */
uint32_t or_crc16(const uint8_t *p, uint64_t len) {
    uint32_t crc = 0;
    for (uint64_t i = 0; i < len; i++) {
        crc ^= (uint32_t)p[i] << 8;
        for (int b = 0; b < 8; b++)
            crc = (crc & 0x8000) ? ((crc << 1) ^ 0x1021) : (crc << 1);
        crc &= 0xffff;
    }
    return crc;
}

/* M:cluster/ClusterConnectionManager.java:543-558.  indexOf('{'), then the
 * FIRST '}' anywhere (not the first after '{'); substring(start+1,end)
 * throws when end == -1 or end < start+1 -> reported as -1 here.  '{' and
 * '}' never occur inside UTF-8 multi-byte sequences, so byte search equals
 * Java's char search for key.getBytes() in UTF-8.                        */
int32_t or_calc_slot(const uint8_t *key, uint64_t len) {
    int64_t start = -1, end = -1;
    for (uint64_t i = 0; i < len; i++)
        if (key[i] == '{') { start = (int64_t)i; break; }
    if (start != -1) {
        for (uint64_t i = 0; i < len; i++)
            if (key[i] == '}') { end = (int64_t)i; break; }
        if (end < start + 1) return -1;
        return (int32_t)(or_crc16(key + start + 1, (uint64_t)(end - start - 1)) % 16384);
    }
    return (int32_t)(or_crc16(key, len) % 16384);
}

/* ------------------------------------------------------------------ */
/* redis hyperloglog.c hllPatLen.  3.2.0: hash |= 1<<63, scan from bit 14.
 * >=5.0: hash >>= 14; hash |= 1<<HLL_Q (Q=50); scan from bit 0.         */
int or_hll_patlen(const uint8_t *ele, uint64_t len, int redis_major, int64_t *reg) {
    uint64_t hash = or_murmur64a(ele, (int64_t)len, 0xadc83b19ULL);
    uint64_t index = hash & (OR_HLL_REGISTERS - 1);
    int count = 1;
    if (redis_major >= 5) {
        hash >>= 14;
        hash |= (uint64_t)1 << 50;
        uint64_t bit = 1;
        while ((hash & bit) == 0) { count++; bit <<= 1; }
    } else {
        hash |= (uint64_t)1 << 63;
        uint64_t bit = OR_HLL_REGISTERS;
        while ((hash & bit) == 0) { count++; bit <<= 1; }
    }
    *reg = (int64_t)index;
    return count;
}

int or_hll_add(uint8_t *regs, const uint8_t *ele, uint64_t len, int redis_major) {
    int64_t idx;
    int cnt = or_hll_patlen(ele, len, redis_major, &idx);
    if (regs[idx] < cnt) {
        regs[idx] = (uint8_t)cnt;
        return 1;
    }
    return 0;
}

/* pfaddCommand: key created -> updated++; each element hllAdd()==1 ->
 * updated++; reply updated ? 1 : 0.  Commands applied in batch order
 * (M:command/CommandBatchService.java:163-171 ordering).                */
void or_pfadd_batch(uint8_t *regs_base, uint8_t *exists, uint32_t n_cmds,
                    const uint32_t *key_ids, const uint32_t *elem_counts,
                    const uint64_t *elem_off, const uint8_t *elem_bytes,
                    int redis_major, uint8_t *out_changed) {
    uint64_t e = 0;
    for (uint32_t c = 0; c < n_cmds; c++) {
        uint32_t key = key_ids[c];
        uint8_t *regs = regs_base + (uint64_t)key * OR_HLL_REGISTERS;
        int updated = 0;
        if (!exists[key]) { exists[key] = 1; updated = 1; }
        for (uint32_t j = 0; j < elem_counts[c]; j++, e++) {
            uint64_t o = elem_off[e], l = elem_off[e + 1] - o;
            if (or_hll_add(regs, elem_bytes + o, l, redis_major)) updated = 1;
        }
        out_changed[c] = (uint8_t)updated;
    }
}

static double PE[64];
static int pe_init = 0;
static void init_pe(void) {
    if (pe_init) return;
    PE[0] = 1;
    for (int j = 1; j < 64; j++) PE[j] = 1.0 / (double)(1ULL << j);
    pe_init = 1;
}

/* hllDenseSum (16 registers per iteration, paired sums, left-assoc),
 * hllSparseSum (VAL runs in order, ez added at the end) and hllRawSum
 * (byte order, zero words skipped, ez added at the end).               */
double or_hll_sum(const uint8_t *regs, int encoding, int *ezp) {
    init_pe();
    double E = 0;
    int ez = 0;
    if (encoding == 1) {
        for (int j = 0; j < 1024; j++) {
            const uint8_t *r = regs + j * 16;
            for (int t = 0; t < 16; t++)
                if (r[t] == 0) ez++;
            E += (PE[r[0]] + PE[r[1]]) + (PE[r[2]] + PE[r[3]]) + (PE[r[4]] + PE[r[5]]) +
                 (PE[r[6]] + PE[r[7]]) + (PE[r[8]] + PE[r[9]]) + (PE[r[10]] + PE[r[11]]) +
                 (PE[r[12]] + PE[r[13]]) + (PE[r[14]] + PE[r[15]]);
        }
    } else if (encoding == 0) {
        /* sparse: VAL(v,runlen) adds PE[v]*runlen; all terms exact (v<=32) */
        int i = 0;
        while (i < OR_HLL_REGISTERS) {
            uint8_t v = regs[i];
            int run = 1;
            if (v == 0) {
                while (i + run < OR_HLL_REGISTERS && regs[i + run] == 0) run++;
                ez += run;
            } else {
                while (run < 4 && i + run < OR_HLL_REGISTERS && regs[i + run] == v) run++;
                E += PE[v] * run;
            }
            i += run;
        }
        E += ez;
    } else {
        for (int j = 0; j < OR_HLL_REGISTERS / 8; j++) {
            const uint8_t *b = regs + j * 8;
            if (ld64(b) == 0) {
                ez += 8;
            } else {
                for (int t = 0; t < 8; t++) {
                    if (b[t]) E += PE[b[t]];
                    else ez++;
                }
            }
        }
        E += ez;
    }
    *ezp = ez;
    return E;
}

static double hll_sigma(double x) {
    if (x == 1.) return INFINITY;
    double zPrime, y = 1, z = x;
    do {
        x *= x;
        zPrime = z;
        z += x * y;
        y += y;
    } while (zPrime != z);
    return z;
}
static double hll_tau(double x) {
    if (x == 0. || x == 1.) return 0.;
    double zPrime, y = 1.0, z = 1 - x;
    do {
        x = sqrt(x);
        zPrime = z;
        y *= 0.5;
        z -= pow(1 - x, 2) * y;
    } while (zPrime != z);
    return z / 3;
}

static uint64_t count_from_hist_v5(const uint32_t *hist) {
    double m = OR_HLL_REGISTERS, z;
    z = m * hll_tau((m - hist[51]) / m);
    for (int j = 50; j >= 1; --j) {
        z += hist[j];
        z *= 0.5;
    }
    z += m * hll_sigma(hist[0] / m);
    return (uint64_t)llroundl(0.721347520444481703680 * m * m / z);
}

/* hllCount (redis 3.2 / 4.0 estimator, or >=5.0 Ertl estimator) */
uint64_t or_hll_count(const uint8_t *regs, int encoding, int redis_major) {
    double m = OR_HLL_REGISTERS;
    if (redis_major >= 5) {
        uint32_t hist[64];
        or_hll_histogram(regs, hist);
        return count_from_hist_v5(hist);
    }
    double alpha = 0.7213 / (1 + 1.079 / m);
    int ez;
    double E = or_hll_sum(regs, encoding, &ez);
    E = (1 / E) * alpha * m * m;
    if (E < m * 2.5 && ez != 0) {
        E = m * log(m / ez);
    } else if (m == 16384 && E < 72000) {
        double bias = 5.9119 * 1.0e-18 * (E * E * E * E) - 1.4253 * 1.0e-12 * (E * E * E) +
                      1.2940 * 1.0e-7 * (E * E) - 5.2921 * 1.0e-3 * E + 83.3216;
        E -= E * (bias / 100);
    }
    return (uint64_t)E;
}

void or_hll_histogram(const uint8_t *regs, uint32_t *hist64) {
    memset(hist64, 0, 64 * sizeof(uint32_t));
    for (int i = 0; i < OR_HLL_REGISTERS; i++) hist64[regs[i] & 63]++;
}

void or_hll_union(const uint8_t *const *regs, uint32_t n, uint8_t *out) {
    memset(out, 0, OR_HLL_REGISTERS);
    for (uint32_t k = 0; k < n; k++) {
        if (!regs[k]) continue; /* missing key = empty HLL */
        for (int i = 0; i < OR_HLL_REGISTERS; i++)
            if (regs[k][i] > out[i]) out[i] = regs[k][i];
    }
}

/* HLL_DENSE_SET_REGISTER / GET: register i at bit 6*i, LSB-first in bytes */
void or_hll_dense_pack(const uint8_t *regs, uint8_t *out) {
    memset(out, 0, OR_HLL_DENSE_BYTES);
    for (int i = 0; i < OR_HLL_REGISTERS; i++) {
        unsigned byte = (unsigned)(i * 6) / 8, fb = (unsigned)(i * 6) & 7;
        unsigned v = regs[i] & 63;
        out[byte] |= (uint8_t)(v << fb);
        if (fb > 2) out[byte + 1] |= (uint8_t)(v >> (8 - fb));
    }
}
void or_hll_dense_unpack(const uint8_t *in, uint8_t *regs) {
    for (int i = 0; i < OR_HLL_REGISTERS; i++) {
        unsigned byte = (unsigned)(i * 6) / 8, fb = (unsigned)(i * 6) & 7;
        unsigned b0 = in[byte];
        unsigned b1 = (byte + 1 < OR_HLL_DENSE_BYTES) ? in[byte + 1] : 0;
        regs[i] = (uint8_t)(((b0 >> fb) | (b1 << (8 - fb))) & 63);
    }
}

/* ------------------------------------------------------------------ */
/* Redis HLL strings as redis-server 3.2 writes them (hyperloglog.c):     */
/* createHLLObject (sparse XZERO runs, cached card 0), hllSparseSet        */
/* (split the opcode covering the register, promote to dense past          */
/* hll_sparse_max_bytes = 3000 or a value > 32, merge adjacent VAL          */
/* opcodes over <= 5 opcodes from the previous one), hllSparseToDense,     */
/* and the cached-cardinality bytes of PFADD / PFCOUNT / PFMERGE.          */
/* s: a buffer of >= 16 + 12288 + 8 bytes; *len: the string's length.      */
#define OR_HDR 16
#define OR_SPARSE_MAX_BYTES 3000
#define OR_IS_ZERO(p) (((*(p)) & 0xc0) == 0)
#define OR_IS_XZERO(p) (((*(p)) & 0xc0) == 0x40)
#define OR_IS_VAL(p) ((*(p)) & 0x80)
#define OR_ZERO_LEN(p) (((*(p)) & 0x3f) + 1)
#define OR_XZERO_LEN(p) (((((*(p)) & 0x3f) << 8) | (*((p) + 1))) + 1)
#define OR_VAL_VALUE(p) ((((*(p)) >> 2) & 0x1f) + 1)
#define OR_VAL_LEN(p) (((*(p)) & 0x3) + 1)
static void or_val_set(uint8_t *p, int val, int len) { *p = (uint8_t)((((val) - 1) << 2 | ((len) - 1)) | 0x80); }
static void or_zero_set(uint8_t *p, int len) { *p = (uint8_t)((len) - 1); }
static void or_xzero_set(uint8_t *p, int len) {
    int l = len - 1;
    p[0] = (uint8_t)((l >> 8) | 0x40);
    p[1] = (uint8_t)(l & 0xff);
}
static unsigned or_dense_get(const uint8_t *regs, long i) {
    unsigned byte = (unsigned)(i * 6) / 8, fb = (unsigned)(i * 6) & 7;
    unsigned b0 = regs[byte], b1 = byte + 1 < OR_HLL_DENSE_BYTES ? regs[byte + 1] : 0;
    return ((b0 >> fb) | (b1 << (8 - fb))) & 63;
}
static void or_dense_set(uint8_t *regs, long i, unsigned v) {
    unsigned byte = (unsigned)(i * 6) / 8, fb = (unsigned)(i * 6) & 7;
    regs[byte] &= (uint8_t)~(63u << fb);
    regs[byte] |= (uint8_t)(v << fb);
    if (fb > 2) {
        regs[byte + 1] &= (uint8_t)~(63u >> (8 - fb));
        regs[byte + 1] |= (uint8_t)(v >> (8 - fb));
    }
}

uint64_t or_hllstr_new(uint8_t *s) {
    memset(s, 0, OR_HDR);
    memcpy(s, "HYLL", 4);
    s[4] = 1; /* HLL_SPARSE; card bytes 0 */
    or_xzero_set(s + OR_HDR, 16384);
    return OR_HDR + 2;
}

int or_hllstr_to_dense(uint8_t *s, uint64_t *len) {
    if (s[4] == 0) return 0;
    uint8_t dense[OR_HLL_DENSE_BYTES];
    memset(dense, 0, sizeof dense);
    long idx = 0;
    const uint8_t *p = s + OR_HDR, *end = s + *len;
    while (p < end) {
        if (OR_IS_ZERO(p)) {
            idx += OR_ZERO_LEN(p);
            p++;
        } else if (OR_IS_XZERO(p)) {
            idx += OR_XZERO_LEN(p);
            p += 2;
        } else {
            int run = OR_VAL_LEN(p), v = OR_VAL_VALUE(p);
            while (run--) {
                if (idx < OR_HLL_REGISTERS) or_dense_set(dense, idx, (unsigned)v);
                idx++;
            }
            p++;
        }
    }
    if (idx != OR_HLL_REGISTERS) return -1;
    s[4] = 0; /* header (magic, unused bytes, cached card) kept */
    memcpy(s + OR_HDR, dense, sizeof dense);
    *len = OR_HDR + OR_HLL_DENSE_BYTES;
    return 0;
}

/* hllSparseSet / hllDenseSet: 1 if the register rose, 0 if not, -1 corrupted */
int or_hllstr_set(uint8_t *s, uint64_t *len, long index, uint8_t count) {
    if (s[4] == 0) {
        uint8_t *regs = s + OR_HDR;
        if (or_dense_get(regs, index) >= count) return 0;
        or_dense_set(regs, index, count);
        return 1;
    }
    if (count > 32) goto promote;
    {
        uint8_t *sparse = s + OR_HDR, *p = sparse, *end = s + *len, *prev = NULL, *next;
        long first = 0, span = 0, runlen;
        int is_zero = 0, is_xzero = 0, is_val = 0;
        while (p < end) {
            long oplen = 1;
            if (OR_IS_ZERO(p)) span = OR_ZERO_LEN(p);
            else if (OR_IS_VAL(p)) span = OR_VAL_LEN(p);
            else span = OR_XZERO_LEN(p), oplen = 2;
            if (index <= first + span - 1) break;
            prev = p;
            p += oplen;
            first += span;
        }
        if (span == 0 || p >= end) return -1;
        next = OR_IS_XZERO(p) ? p + 2 : p + 1;
        if (next >= end) next = NULL;
        if (OR_IS_ZERO(p)) is_zero = 1, runlen = OR_ZERO_LEN(p);
        else if (OR_IS_XZERO(p)) is_xzero = 1, runlen = OR_XZERO_LEN(p);
        else is_val = 1, runlen = OR_VAL_LEN(p);
        if (is_val) {
            int oldcount = OR_VAL_VALUE(p);
            if (oldcount >= count) return 0;
            if (runlen == 1) {
                or_val_set(p, count, 1);
                goto updated;
            }
        }
        if (is_zero && runlen == 1) {
            or_val_set(p, count, 1);
            goto updated;
        }
        {
            uint8_t seq[5], *n = seq;
            long last = first + span - 1, l;
            if (is_zero || is_xzero) {
                if (index != first) {
                    l = index - first;
                    if (l > 64) or_xzero_set(n, (int)l), n += 2;
                    else or_zero_set(n, (int)l), n++;
                }
                or_val_set(n, count, 1), n++;
                if (index != last) {
                    l = last - index;
                    if (l > 64) or_xzero_set(n, (int)l), n += 2;
                    else or_zero_set(n, (int)l), n++;
                }
            } else {
                int curval = OR_VAL_VALUE(p);
                if (index != first) or_val_set(n, curval, (int)(index - first)), n++;
                or_val_set(n, count, 1), n++;
                if (index != last) or_val_set(n, curval, (int)(last - index)), n++;
            }
            long seqlen = n - seq, oldlen = is_xzero ? 2 : 1, deltalen = seqlen - oldlen;
            if (deltalen > 0 && (long)*len + deltalen > OR_SPARSE_MAX_BYTES) goto promote;
            if (deltalen && next) memmove(next + deltalen, next, (size_t)(end - next));
            *len = (uint64_t)((long)*len + deltalen);
            memcpy(p, seq, (size_t)seqlen);
            end += deltalen;
        }
    updated:
        p = prev ? prev : sparse;
        {
            int scanlen = 5;
            while (p < end && scanlen--) {
                if (OR_IS_XZERO(p)) {
                    p += 2;
                    continue;
                } else if (OR_IS_ZERO(p)) {
                    p++;
                    continue;
                }
                if (p + 1 < end && OR_IS_VAL(p + 1)) {
                    int v1 = OR_VAL_VALUE(p), v2 = OR_VAL_VALUE(p + 1);
                    if (v1 == v2) {
                        int l2 = OR_VAL_LEN(p) + OR_VAL_LEN(p + 1);
                        if (l2 <= 4) {
                            or_val_set(p + 1, v1, l2);
                            memmove(p, p + 1, (size_t)(end - p));
                            *len -= 1;
                            end--;
                            continue;
                        }
                    }
                }
                p++;
            }
        }
        s[15] |= 0x80; /* HLL_INVALIDATE_CACHE */
        return 1;
    }
promote:
    if (or_hllstr_to_dense(s, len) != 0) return -1;
    or_dense_set(s + OR_HDR, index, count);
    return 1;
}

/* pfaddCommand on one key: created -> updated; each element hllAdd; updated -> cache invalidated.  Returns
 * the reply (1/0), -1 on a corrupted string. */
int or_hllstr_pfadd(uint8_t *s, uint64_t *len, int created, uint32_t n, const uint64_t *off, const uint8_t *bytes,
                    int redis_major) {
    int updated = created;
    for (uint32_t j = 0; j < n; j++) {
        int64_t idx;
        int cnt = or_hll_patlen(bytes + off[j], off[j + 1] - off[j], redis_major, &idx);
        int r = or_hllstr_set(s, len, (long)idx, (uint8_t)cnt);
        if (r < 0) return -1;
        updated |= r;
    }
    if (updated) s[15] |= 0x80;
    return updated;
}

/* registers of an HLL string (dense or sparse); -1 corrupted */
int or_hllstr_registers(const uint8_t *s, uint64_t len, uint8_t *regs) {
    if (s[4] == 0) {
        or_hll_dense_unpack(s + OR_HDR, regs);
        return 0;
    }
    long idx = 0;
    const uint8_t *p = s + OR_HDR, *end = s + len;
    while (p < end) {
        if (OR_IS_ZERO(p)) {
            int r = OR_ZERO_LEN(p);
            if (idx + r > OR_HLL_REGISTERS) return -1;
            memset(regs + idx, 0, (size_t)r), idx += r, p++;
        } else if (OR_IS_XZERO(p)) {
            int r = OR_XZERO_LEN(p);
            if (idx + r > OR_HLL_REGISTERS) return -1;
            memset(regs + idx, 0, (size_t)r), idx += r, p += 2;
        } else {
            int r = OR_VAL_LEN(p);
            if (idx + r > OR_HLL_REGISTERS) return -1;
            memset(regs + idx, OR_VAL_VALUE(p), (size_t)r), idx += r, p++;
        }
    }
    return idx == OR_HLL_REGISTERS ? 0 : -1;
}

/* ------------------------------------------------------------------ */
/* RedissonBloomFilter (M:RedissonBloomFilter.java)                      */

/* optimalNumOfBits :74-78 ; (long) truncation of a double */
int64_t or_bloom_optimal_bits(int64_t n, double p) {
    if (p == 0) p = 4.9e-324; /* Double.MIN_VALUE */
    return (int64_t)((double)(-n) * log(p) / (log(2) * log(2)));
}
/* optimalNumOfHashFunctions :69-71 ; Math.round = floor(x + 0.5) */
int32_t or_bloom_optimal_k(int64_t n, int64_t m) {
    double x = (double)m / (double)n * log(2);
    int64_t r = (int64_t)floor(x + 0.5);
    int32_t k = (int32_t)r;
    return k > 1 ? k : 1;
}
/* hash :116-131 */
void or_bloom_indexes(const uint8_t *e, uint64_t len, int32_t k, int64_t size, int64_t *out) {
    uint64_t h1 = or_xxh64(e, len, 0);
    uint64_t h2 = or_farmhash_uo64(e, len);
    uint64_t h = h1;
    for (int32_t i = 0; i < k; i++) {
        out[i] = (int64_t)((h & 0x7fffffffffffffffULL) % (uint64_t)size);
        h += (i % 2 == 0) ? h2 : h1;
    }
}
/* count :188-199 */
int32_t or_bloom_count(int64_t size, int32_t k, int64_t bitcount) {
    double r = (double)(-size) / ((double)k) * log(1 - (double)bitcount / ((double)size));
    /* Java (int) of a double: NaN -> 0, saturating, else truncation */
    if (r != r) return 0;
    if (r >= 2147483647.0) return 2147483647;
    if (r <= -2147483648.0) return (int32_t)(-2147483647 - 1);
    return (int32_t)r;
}

int or_getbit(const uint8_t *buf, uint64_t len, uint64_t off) {
    uint64_t byte = off >> 3;
    if (byte >= len) return 0;
    return (buf[byte] >> (7 - (off & 7))) & 1;
}
int or_setbit(uint8_t *buf, uint64_t *len, uint64_t off, int val) {
    uint64_t byte = off >> 3;
    if (byte >= *len) *len = byte + 1; /* sdsgrowzero: new bytes are zero */
    int bit = 7 - (int)(off & 7);
    int old = (buf[byte] >> bit) & 1;
    buf[byte] = (uint8_t)((buf[byte] & ~(1 << bit)) | ((val & 1) << bit));
    return old;
}

/* add :80-114 -> k SETBIT, reply = any of probes 0..k-2 saw 0 (Q2) */
void or_bloom_add_batch(uint8_t *buf, uint64_t *strlen_bytes, int64_t size, int32_t k,
                        uint32_t n, const uint64_t *elem_off, const uint8_t *elem_bytes,
                        uint8_t *out) {
    int64_t idx[256];
    for (uint32_t e = 0; e < n; e++) {
        uint64_t o = elem_off[e], l = elem_off[e + 1] - o;
        int32_t kk = k > 256 ? 256 : k;
        or_bloom_indexes(elem_bytes + o, l, kk, size, idx);
        int r = 0;
        for (int32_t i = 0; i < kk; i++) {
            int old = or_setbit(buf, strlen_bytes, (uint64_t)idx[i], 1);
            if (i <= kk - 2 && old == 0) r = 1;
        }
        out[e] = (uint8_t)r;
    }
}
/* contains :133-168 -> k GETBIT, reply = AND of probes 0..k-2 (Q2) */
void or_bloom_contains_batch(const uint8_t *buf, uint64_t strlen_bytes, int64_t size, int32_t k,
                             uint32_t n, const uint64_t *elem_off, const uint8_t *elem_bytes,
                             uint8_t *out) {
    int64_t idx[256];
    for (uint32_t e = 0; e < n; e++) {
        uint64_t o = elem_off[e], l = elem_off[e + 1] - o;
        int32_t kk = k > 256 ? 256 : k;
        or_bloom_indexes(elem_bytes + o, l, kk, size, idx);
        int r = 1;
        for (int32_t i = 0; i <= kk - 2; i++)
            if (!or_getbit(buf, strlen_bytes, (uint64_t)idx[i])) { r = 0; break; }
        out[e] = (uint8_t)r;
    }
}

uint64_t or_bitcount(const uint8_t *buf, uint64_t len) {
    uint64_t c = 0;
    for (uint64_t i = 0; i < len; i++) c += (uint64_t)__builtin_popcount(buf[i]);
    return c;
}

/* bitopCommand: missing/short sources read as 0, result length = max len */
uint64_t or_bitop(int op, uint8_t *dst, const uint8_t *const *srcs, const uint64_t *lens, uint32_t n) {
    uint64_t maxlen = 0;
    for (uint32_t j = 0; j < n; j++)
        if (lens[j] > maxlen) maxlen = lens[j];
    for (uint64_t b = 0; b < maxlen; b++) {
        uint8_t out = (lens[0] <= b) ? 0 : srcs[0][b];
        if (op == 3) out = (uint8_t)~out;
        for (uint32_t i = 1; i < n; i++) {
            uint8_t byte = (lens[i] <= b) ? 0 : srcs[i][b];
            if (op == 0) out &= byte;
            else if (op == 1) out |= byte;
            else if (op == 2) out ^= byte;
        }
        dst[b] = out;
    }
    return maxlen;
}
