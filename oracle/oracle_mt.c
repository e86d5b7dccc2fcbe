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
 */
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
} mt_arg;

static void *pfadd_owned(void *p) {
    mt_arg *a = (mt_arg *)p;
    for (uint32_t c = 0; c < a->n; c++) {
        uint32_t key = a->key_ids[c];
        if ((int)(key % (uint32_t)a->T) != a->t) continue;
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
    pthread_t th[256];
    mt_arg args[256];
    if (T > 256) T = 256;
    if (T < 1) T = 1;
    for (int t = 0; t < T; t++) {
        args[t] = *base;
        args[t].t = t;
        args[t].T = T;
        pthread_create(&th[t], NULL, fn, &args[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
}

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
    run(nthreads, &a, pfadd_owned);
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
    run(nthreads, &a, contains_range);
}
