/*
 * oracle_mt.c -- whole-host CPU baseline: the oracle's PFADD and Bloom contains
 * loops on T host threads.  TEST/BENCH INFRASTRUCTURE ONLY (bench.py's
 * cpu_baseline leg); the product path never links it.
 *
 * It models SURVEY 8(d)'s "whole host" reference variant: one single-threaded
 * redis-server per core with the client routing each command to its key's
 * owner (M:cluster/ClusterConnectionManager.java:543-558 slot routing, here
 * key id % T).  Each thread applies the commands of the keys it owns in batch
 * order (or_pfadd_batch semantics, sketch_oracle.c), so registers and replies
 * equal the single-threaded oracle's.  Bloom contains only reads the bit
 * array: the batch is split into T contiguous ranges.
 *
 * The *_gen_mt functions are the full-size checkers of tests/test_full_size.py:
 * they generate each element themselves (or_gen_jackson_long, the same
 * SplitMix64 -> Jackson Long byte stream the engine's generator produces), so a
 * 10^8-element check needs no element buffer on the host.  The state they build
 * is order-free (register max, bit OR) or per-owner ordered (PFADD replies).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <stdint.h>

#include "sketch_oracle.h"

typedef struct {
    int t, T;
    uint8_t *regs_base, *exists, *out;
    uint32_t n;
    const uint32_t *key_ids;
    const uint64_t *off;
    const uint8_t *bytes;
    int redis_major;
    /* contains */
    const uint8_t *buf;
    uint64_t strlen_bytes;
    int64_t size;
    int32_t k;
    /* PFADD: the commands of owner t are own[own_start[t] .. own_start[t + 1]) (routed once, in batch order) */
    const uint32_t *own, *own_start;
} mt_arg;

#define OR_MT_MAX_THREADS 1024

static void *pfadd_owned(void *p) {
    mt_arg *a = (mt_arg *)p;
    for (uint32_t j = a->own_start[a->t]; j < a->own_start[a->t + 1]; j++) {
        uint32_t c = a->own[j];
        uint32_t key = a->key_ids[c];
        uint8_t *regs = a->regs_base + (uint64_t)key * OR_HLL_REGISTERS;
        int updated = 0;
        if (!a->exists[key]) {
            a->exists[key] = 1;
            updated = 1;
        }
        uint64_t o = a->off[c];
        if (or_hll_add(regs, a->bytes + o, a->off[c + 1] - o, a->redis_major)) updated = 1;
        a->out[c] = (uint8_t)updated;
    }
    return NULL;
}

static void *contains_range(void *p) {
    mt_arg *a = (mt_arg *)p;
    uint64_t lo = (uint64_t)a->n * (uint64_t)a->t / (uint64_t)a->T;
    uint64_t hi = (uint64_t)a->n * (uint64_t)(a->t + 1) / (uint64_t)a->T;
    or_bloom_contains_batch(a->buf, a->strlen_bytes, a->size, a->k, (uint32_t)(hi - lo), a->off + lo, a->bytes,
                            a->out + lo);
    return NULL;
}

static void run(int T, mt_arg *base, void *(*fn)(void *)) {
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)T);
    mt_arg *args = (mt_arg *)malloc(sizeof(mt_arg) * (size_t)T);
    for (int t = 0; t < T; t++) {
        args[t] = *base;
        args[t].t = t;
        args[t].T = T;
        pthread_create(&th[t], NULL, fn, &args[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    free(th);
    free(args);
}
static int clampMT(int T) { return T < 1 ? 1 : (T > OR_MT_MAX_THREADS ? OR_MT_MAX_THREADS : T); }

/* one element per command; regs_base: n_keys x 16384 registers, exists: n_keys flags */
void or_pfadd_owned_mt(uint8_t *regs_base, uint8_t *exists, uint32_t n, const uint32_t *key_ids,
                       const uint64_t *elem_off, const uint8_t *elem_bytes, int redis_major, uint8_t *out,
                       int nthreads) {
    mt_arg a = {0};
    a.regs_base = regs_base;
    a.exists = exists;
    a.out = out;
    a.n = n;
    a.key_ids = key_ids;
    a.off = elem_off;
    a.bytes = elem_bytes;
    a.redis_major = redis_major;
    /* client-side routing (key id % T), once per batch: each owner's commands in batch order */
    int T = clampMT(nthreads);
    uint32_t *start = (uint32_t *)calloc((size_t)T + 1, sizeof(uint32_t));
    uint32_t *own = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)n + 1));
    for (uint32_t c = 0; c < n; c++) start[key_ids[c] % (uint32_t)T + 1]++;
    for (int t = 0; t < T; t++) start[t + 1] += start[t];
    uint32_t *pos = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)T);
    memcpy(pos, start, sizeof(uint32_t) * (size_t)T);
    for (uint32_t c = 0; c < n; c++) own[pos[key_ids[c] % (uint32_t)T]++] = c;
    a.own = own;
    a.own_start = start;
    run(T, &a, pfadd_owned);
    free(pos);
    free(own);
    free(start);
}

void or_bloom_contains_mt(const uint8_t *buf, uint64_t strlen_bytes, int64_t size, int32_t k, uint32_t n,
                          const uint64_t *elem_off, const uint8_t *elem_bytes, uint8_t *out, int nthreads) {
    mt_arg a = {0};
    a.buf = buf;
    a.strlen_bytes = strlen_bytes;
    a.size = size;
    a.k = k;
    a.n = n;
    a.off = elem_off;
    a.bytes = elem_bytes;
    a.out = out;
    run(clampMT(nthreads), &a, contains_range);
}


/* ------------------------------------------------------------------ */
/* synthetic elements: element i of stream `seed` is
 *   v = SplitMix64 output i = mix(seed + (i + 1) * 0x9E3779B97F4A7C15)
 * rendered as Jackson's default-typed Long ["java.lang.Long",v]
 * (M:codec/JsonJacksonCodec.java:103-106; SURVEY 8d synthetic inputs).    */
uint32_t or_gen_jackson_long(uint64_t seed, uint64_t i, uint8_t *out) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    static const char pre[] = "[\"java.lang.Long\",";
    memcpy(out, pre, 18);
    int nl = snprintf((char *)out + 18, 24, "%lld", (long long)(int64_t)z);
    out[18 + nl] = ']';
    return (uint32_t)(18 + nl + 1);
}

typedef struct {
    int t, T;
    uint64_t n, seed, first;
    const uint64_t *idx;
    const uint32_t *key_ids;
    uint8_t *regs, *exists, *out;
    int redis_major;
    int64_t size;
    int32_t k;
    uint64_t strlen_bytes, maxbyte;
    uint64_t ones;
} gen_arg;

static void run_gen(int T, gen_arg *base, gen_arg *args, void *(*fn)(void *)) {
    pthread_t th[256];
    for (int t = 0; t < T; t++) {
        args[t] = *base;
        args[t].t = t;
        args[t].T = T;
        pthread_create(&th[t], NULL, fn, &args[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
}
static int clampT(int T) { return T < 1 ? 1 : (T > 256 ? 256 : T); }

static void *pfadd_gen(void *p) {
    gen_arg *a = (gen_arg *)p;
    uint8_t e[48];
    for (uint64_t c = 0; c < a->n; c++) {
        uint32_t key = a->key_ids[c];
        if ((int)(key % (uint32_t)a->T) != a->t) continue;
        uint32_t len = or_gen_jackson_long(a->seed, a->first + c, e);
        int updated = 0;
        if (!a->exists[key]) {
            a->exists[key] = 1;
            updated = 1;
        }
        if (or_hll_add(a->regs + (uint64_t)key * OR_HLL_REGISTERS, e, len, a->redis_major)) updated = 1;
        a->out[c] = (uint8_t)updated;
        a->ones += (uint64_t)updated;
    }
    return NULL;
}
/* PFADD of generated elements first..first+n-1, element c into key_ids[c]; returns the number of 1 replies */
uint64_t or_pfadd_gen_mt(uint8_t *regs_base, uint8_t *exists, uint64_t n, const uint32_t *key_ids, uint64_t seed,
                         uint64_t first, int redis_major, uint8_t *out, int nthreads) {
    int T = clampT(nthreads);
    gen_arg a, args[256];
    memset(&a, 0, sizeof a);
    a.n = n;
    a.key_ids = key_ids;
    a.seed = seed;
    a.first = first;
    a.regs = regs_base;
    a.exists = exists;
    a.out = out;
    a.redis_major = redis_major;
    run_gen(T, &a, args, pfadd_gen);
    uint64_t ones = 0;
    for (int t = 0; t < T; t++) ones += args[t].ones;
    return ones;
}

static void *union_gen(void *p) {
    gen_arg *a = (gen_arg *)p;
    uint8_t e[48];
    uint64_t lo = a->n * (uint64_t)a->t / (uint64_t)a->T, hi = a->n * (uint64_t)(a->t + 1) / (uint64_t)a->T;
    for (uint64_t c = lo; c < hi; c++) {
        uint32_t len = or_gen_jackson_long(a->seed, a->first + c, e);
        or_hll_add(a->regs, e, len, a->redis_major);
    }
    return NULL;
}
/* registers of the union of every HLL the generated elements went into (= the HLL of all of them) */
void or_hll_union_gen_mt(uint8_t *regs_out, uint64_t n, uint64_t seed, uint64_t first, int redis_major,
                         int nthreads) {
    int T = clampT(nthreads);
    static uint8_t priv[256][OR_HLL_REGISTERS];
    gen_arg a, args[256];
    memset(&a, 0, sizeof a);
    a.n = n;
    a.seed = seed;
    a.first = first;
    a.redis_major = redis_major;
    pthread_t th[256];
    for (int t = 0; t < T; t++) {
        memset(priv[t], 0, OR_HLL_REGISTERS);
        args[t] = a;
        args[t].t = t;
        args[t].T = T;
        args[t].regs = priv[t];
        pthread_create(&th[t], NULL, union_gen, &args[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < T; t++)
        for (int r = 0; r < OR_HLL_REGISTERS; r++)
            if (priv[t][r] > regs_out[r]) regs_out[r] = priv[t][r];
}

static void *bloom_add_gen(void *p) {
    gen_arg *a = (gen_arg *)p;
    uint8_t e[48];
    int64_t idx[256];
    int32_t kk = a->k > 256 ? 256 : a->k;
    uint64_t lo = a->n * (uint64_t)a->t / (uint64_t)a->T, hi = a->n * (uint64_t)(a->t + 1) / (uint64_t)a->T;
    for (uint64_t c = lo; c < hi; c++) {
        uint32_t len = or_gen_jackson_long(a->seed, a->first + c, e);
        or_bloom_indexes(e, len, kk, a->size, idx);
        for (int32_t j = 0; j < kk; j++) {
            uint64_t b = (uint64_t)idx[j] >> 3;
            __atomic_fetch_or(&a->regs[b], (uint8_t)(0x80u >> ((uint64_t)idx[j] & 7u)), __ATOMIC_RELAXED);
            if (b + 1 > a->maxbyte) a->maxbyte = b + 1;
        }
    }
    return NULL;
}
/* bit array after RBloomFilter.add of the generated elements (bits: (size+7)/8 zeroed bytes);
 * returns the Redis string length (highest byte SETBIT touched + 1) */
uint64_t or_bloom_add_gen_mt(uint8_t *bits, int64_t size, int32_t k, uint64_t seed, uint64_t first, uint64_t n,
                             int nthreads) {
    int T = clampT(nthreads);
    gen_arg a, args[256];
    memset(&a, 0, sizeof a);
    a.n = n;
    a.seed = seed;
    a.first = first;
    a.regs = bits;
    a.size = size;
    a.k = k;
    run_gen(T, &a, args, bloom_add_gen);
    uint64_t m = 0;
    for (int t = 0; t < T; t++)
        if (args[t].maxbyte > m) m = args[t].maxbyte;
    return m;
}

/* RBloomFilter.add of generated elements first..first+n-1 in batch order with every reply (one thread: a reply
 * depends on every earlier element); bits: (size+7)/8 zeroed bytes; returns the Redis string length */
uint64_t or_bloom_add_gen_seq(uint8_t *bits, int64_t size, int32_t k, uint64_t seed, uint64_t first, uint64_t n,
                              uint8_t *out) {
    uint8_t e[48];
    uint64_t len = 0;
    for (uint64_t c = 0; c < n; c++) {
        uint64_t off[2] = {0, 0};
        off[1] = or_gen_jackson_long(seed, first + c, e);
        or_bloom_add_batch(bits, &len, size, k, 1, off, e, out + c);
    }
    return len;
}

/* the same for element numbers idx[0..n) of stream `seed` (repeats allowed), continuing the string in bits/len */
uint64_t or_bloom_add_idx_seq(uint8_t *bits, uint64_t len, int64_t size, int32_t k, uint64_t seed,
                              const uint64_t *idx, uint64_t n, uint8_t *out) {
    uint8_t e[48];
    for (uint64_t c = 0; c < n; c++) {
        uint64_t off[2] = {0, 0};
        off[1] = or_gen_jackson_long(seed, idx[c], e);
        or_bloom_add_batch(bits, &len, size, k, 1, off, e, out + c);
    }
    return len;
}

static void *bloom_contains_gen(void *p) {
    gen_arg *a = (gen_arg *)p;
    uint8_t e[48];
    uint64_t lo = a->n * (uint64_t)a->t / (uint64_t)a->T, hi = a->n * (uint64_t)(a->t + 1) / (uint64_t)a->T;
    for (uint64_t c = lo; c < hi; c++) {
        uint64_t off[2] = {0, 0};
        off[1] = or_gen_jackson_long(a->seed, a->idx[c], e);
        or_bloom_contains_batch(a->regs, a->strlen_bytes, a->size, a->k, 1, off, e, a->out + c);
    }
    return NULL;
}
/* RBloomFilter.contains of generated elements idx[0..n) (element numbers of stream `seed`) */
void or_bloom_contains_gen_mt(const uint8_t *bits, uint64_t strlen_bytes, int64_t size, int32_t k, uint64_t seed,
                              const uint64_t *idx, uint64_t n, uint8_t *out, int nthreads) {
    int T = clampT(nthreads);
    gen_arg a, args[256];
    memset(&a, 0, sizeof a);
    a.n = n;
    a.seed = seed;
    a.idx = idx;
    a.regs = (uint8_t *)bits;
    a.strlen_bytes = strlen_bytes;
    a.size = size;
    a.k = k;
    a.out = out;
    run_gen(T, &a, args, bloom_contains_gen);
}

static void *setbits(void *p) {
    gen_arg *a = (gen_arg *)p;
    uint64_t lo = a->n * (uint64_t)a->t / (uint64_t)a->T, hi = a->n * (uint64_t)(a->t + 1) / (uint64_t)a->T;
    for (uint64_t c = lo; c < hi; c++) {
        uint64_t o = a->idx[c];
        __atomic_fetch_or(&a->regs[o >> 3], (uint8_t)(0x80u >> (o & 7u)), __ATOMIC_RELAXED);
    }
    return NULL;
}
/* SETBIT key off 1 for every offset (MSB-first bytes, buf sized past the largest offset) */
void or_setbits_mt(uint8_t *buf, const uint64_t *offsets, uint64_t n, int nthreads) {
    int T = clampT(nthreads);
    gen_arg a, args[256];
    memset(&a, 0, sizeof a);
    a.n = n;
    a.idx = offsets;
    a.regs = buf;
    run_gen(T, &a, args, setbits);
}
