/*
 * sketch_oracle.h -- CPU restatement of the arithmetic behind Redisson's
 * probabilistic-structure path (RHyperLogLog / RBitSet / RBloomFilter).
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / CPU comparator.  The product (redisson_amd, include/redisson_sketch.h)
 * never links, loads or calls it.
 *
 * What it restates (file:line in the reference, M: = src/main/java/org/redisson/):
 *   - CRC16-XMODEM + calcSlot:  M:connection/CRC16.java:23-61,
 *                               M:cluster/ClusterConnectionManager.java:543-558
 *   - Bloom sizing / indexes / count:  M:RedissonBloomFilter.java:69-78,116-131,188-199
 *   - Bloom add/contains reply rule (Q2, subList(1,size-1)):
 *                               M:RedissonBloomFilter.java:102,155
 *   - HLL command mapping:      M:RedissonHyperLogLog.java:66-97
 *   - BitSet command mapping:   M:RedissonBitSet.java:53-268
 * and the third-party arithmetic those call (not in /root/reference):
 *   - redis-server 3.2.0 hyperloglog.c: MurmurHash64A (seed 0xadc83b19),
 *     hllPatLen, PFADD/PFCOUNT/PFMERGE, hllDenseSum / hllRawSum order,
 *     the <=4.0 estimator (linear counting + bias polynomial) and the >=5.0
 *     Ertl estimator (hllSigma / hllTau).
 *   - redis-server 3.2.0 bitops.c: SETBIT/GETBIT/BITCOUNT/BITOP/STRLEN.
 *   - net.openhft:zero-allocation-hashing 0.5: xx_r39() = XXH64 seed 0,
 *     farmUo() = farmhashuo::Hash64 (len<=64 -> farmhashna::Hash64).
 *
 * Pins (see DESIGN.md "Oracle"):
 *   - MurmurHash64A: SMHasher verification value 0x1F0D3804.
 *   - XXH64: python xxhash 3.8.1 (tests/test_oracle_pins.py).
 *   - farmhashna::Hash64 (= farmUo for len<=64): Guava FarmHashFingerprint64
 *     published known answers; farmUo for len>64 is parity UNPINNED.
 *   - CRC16-XMODEM check value crc16("123456789") = 0x31C3.
 *   - Reference functional tests (T:RedissonHyperLogLogTest, ...BloomFilterTest,
 *     ...BitSetTest) re-expressed in tests/test_oracle_reference_cases.py.
 */
#ifndef SKETCH_ORACLE_H
#define SKETCH_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_HLL_REGISTERS 16384
#define OR_HLL_DENSE_BYTES 12288

/* ---- hashes ---- */
uint64_t or_murmur64a(const uint8_t *key, int64_t len, uint64_t seed);
uint32_t or_murmur64a_verification(void);
uint64_t or_xxh64(const uint8_t *p, uint64_t len, uint64_t seed);
uint64_t or_farmhash_na64(const uint8_t *s, uint64_t len);
uint64_t or_farmhash_uo64(const uint8_t *s, uint64_t len);

/* ---- cluster slot ---- */
uint32_t or_crc16(const uint8_t *p, uint64_t len);
/* returns slot in [0,16384), or -1 where Java's substring would throw */
int32_t or_calc_slot(const uint8_t *key, uint64_t len);

/* ---- HyperLogLog ---- */
/* redis_major: 3 (reference CI pin, sentinel bit 63) or >=5 (HLL_Q sentinel) */
int or_hll_patlen(const uint8_t *ele, uint64_t len, int redis_major, int64_t *reg);
/* one element into unpacked u8 registers; returns 1 iff a register rose */
int or_hll_add(uint8_t *regs, const uint8_t *ele, uint64_t len, int redis_major);
/* batch of PFADD commands; regs_base = n_keys * 16384 unpacked registers;
 * exists[key] (0/1) is updated (a PFADD creates its key -> reply 1). */
void or_pfadd_batch(uint8_t *regs_base, uint8_t *exists, uint32_t n_cmds,
                    const uint32_t *key_ids, const uint32_t *elem_counts,
                    const uint64_t *elem_off, const uint8_t *elem_bytes,
                    int redis_major, uint8_t *out_changed);
/* encoding: 0 = sparse order, 1 = dense order (hllDenseSum), 2 = raw order (hllRawSum) */
double or_hll_sum(const uint8_t *regs, int encoding, int *ez);
uint64_t or_hll_count(const uint8_t *regs, int encoding, int redis_major);
void or_hll_histogram(const uint8_t *regs, uint32_t *hist64);
/* union of n register arrays -> out (max); what multi-key PFCOUNT / PFMERGE do */
void or_hll_union(const uint8_t *const *regs, uint32_t n, uint8_t *out);
void or_hll_dense_pack(const uint8_t *regs, uint8_t *out12288);
void or_hll_dense_unpack(const uint8_t *in12288, uint8_t *regs);
/* Redis HLL strings as redis-server 3.2 writes them (sparse writer) */
uint64_t or_hllstr_new(uint8_t *s);
int or_hllstr_to_dense(uint8_t *s, uint64_t *len);
int or_hllstr_set(uint8_t *s, uint64_t *len, long index, uint8_t count);
int or_hllstr_pfadd(uint8_t *s, uint64_t *len, int created, uint32_t n, const uint64_t *off, const uint8_t *bytes,
                    int redis_major);
int or_hllstr_registers(const uint8_t *s, uint64_t len, uint8_t *regs);

/* ---- Bloom filter (RedissonBloomFilter) ---- */
int64_t or_bloom_optimal_bits(int64_t n, double p);
int32_t or_bloom_optimal_k(int64_t n, int64_t m);
void or_bloom_indexes(const uint8_t *e, uint64_t len, int32_t k, int64_t size, int64_t *out);
int32_t or_bloom_count(int64_t size, int32_t k, int64_t bitcount);
/* batch add / contains on a raw MSB-first bit string (buf has capacity for
 * size bits; *strlen_bytes is the Redis string length, grown by SETBIT). */
void or_bloom_add_batch(uint8_t *buf, uint64_t *strlen_bytes, int64_t size, int32_t k,
                        uint32_t n, const uint64_t *elem_off, const uint8_t *elem_bytes,
                        uint8_t *out);
void or_bloom_contains_batch(const uint8_t *buf, uint64_t strlen_bytes, int64_t size, int32_t k,
                             uint32_t n, const uint64_t *elem_off, const uint8_t *elem_bytes,
                             uint8_t *out);

/* ---- bit strings (redis bitops.c) ---- */
int or_getbit(const uint8_t *buf, uint64_t len, uint64_t off);
/* buf must have capacity > off/8; returns old bit; grows *len */
int or_setbit(uint8_t *buf, uint64_t *len, uint64_t off, int val);
uint64_t or_bitcount(const uint8_t *buf, uint64_t len);
/* op: 0 AND, 1 OR, 2 XOR, 3 NOT; dst must hold max(lens) bytes; returns maxlen */
uint64_t or_bitop(int op, uint8_t *dst, const uint8_t *const *srcs, const uint64_t *lens, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
