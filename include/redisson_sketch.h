/*
 * redisson_sketch.h -- C ABI of the MI355X sketch engine (libredisson_sketch.so).
 *
 * Drop-in boundary for Redisson's probabilistic-structure path.  Every entry
 * point replaces a (RedisCommand, key, params) triple that Redisson's L3
 * executor would otherwise send over Netty to redis-server
 * (M:command/CommandAsyncService.java:378 async(...), and the batch hook
 * M:command/CommandBatchService.java:91-111,184).  M: = /root/reference/src/
 * main/java/org/redisson/.  The Java side (JNI shim) applies
 * the codec / param-encoding rules first (M:client/handler/CommandEncoder.java:
 * 73-94), so every "element" below is already the exact byte string Redis
 * would have hashed.
 *
 * Conventions
 *   - Plain pointers and sizes only.  "Host" buffers are caller-owned and only
 *     read/written during the call.  Functions suffixed _dev take DEVICE
 *     pointers (already resident in HBM on this context's GPU) and enqueue on
 *     the context's stream; they return after completion unless noted.
 *   - Variable-length byte strings are passed as (off u64[n+1], bytes u8[]):
 *     item i = bytes[off[i] .. off[i+1]).  Device byte buffers must have 16
 *     readable bytes of padding after the last item.
 *   - Every function returns SK_OK (0) or a negative SK_E* status;
 *     sk_last_error() gives the Redis-compatible message (Java maps it to
 *     RedisException, M:client/handler/CommandDecoder.java:239-241).
 *   - A context is bound to one GPU.  Calls on one context are serialized
 *     internally (thread-safe).  Multi-GPU: one context per device, keys
 *     routed by sk_owner() = calcSlot(key) % n_gpus (north_star partitioner).
 */
#ifndef REDISSON_SKETCH_H
#define REDISSON_SKETCH_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (message text = what redis-server / Redisson raises) ---- */
#define SK_OK 0
#define SK_EWRONGTYPE (-1) /* "WRONGTYPE Operation against a key holding the wrong kind of value"
                              (HLL ops: "Key is not a valid HyperLogLog string value.") */
#define SK_ERANGE (-2)     /* "ERR bit offset is not an integer or out of range" */
#define SK_ECONFIG (-3)    /* "Bloom filter config has been changed" (M:RedissonBloomFilter.java:108,183) */
#define SK_ENOTINIT (-4)   /* "Bloom filter is not initialized!" (IllegalStateException, :217,284) */
#define SK_EDEVICE (-5)    /* HIP runtime / device failure */
#define SK_EINVAL (-6)     /* bad argument */
#define SK_ENOMEM (-7)     /* device or host allocation failed */
#define SK_ESYNTAX (-8)    /* "ERR BITOP NOT must be called with a single source key." */
#define SK_ETOOBIG (-9)    /* "Bloom filter can't be greater than 4294967294. ..." (IllegalArgumentException, :72-74) */
#define SK_ECORRUPT (-10)  /* "INVALIDOBJ Corrupted HLL object detected" (a SET string with the HYLL magic
                              whose registers do not decode) */
#define SK_ESTALE (-11)    /* a caller-cached HLL slab id (sk_pfadd_ids / sk_pfcount_ids) whose key was deleted,
                              replaced or flushed: drop the cached id and resolve the key by name again */
#define SK_EBUSYKEY (-12)  /* "BUSYKEY Target key name already exists." (RESTORE without REPLACE) */
#define SK_EPAYLOAD (-13)  /* "ERR DUMP payload version or checksum are wrong" / a malformed RDB file */

#define SK_TYPE_NONE 0
#define SK_TYPE_HLL 1    /* string holding a HyperLogLog (PFADD/PFMERGE created it) */
#define SK_TYPE_STRING 2 /* plain string: RBitSet / Bloom filter bit array */
#define SK_TYPE_HASH 3   /* a Bloom filter config "{name}__config" (sk_type, sk_scan) */

#define SK_BITOP_AND 0
#define SK_BITOP_OR 1
#define SK_BITOP_XOR 2
#define SK_BITOP_NOT 3

#define SK_HLL_REGISTERS 16384
#define SK_HLL_DENSE_SIZE (16 + 12288) /* "HYLL" header + 6-bit dense registers */

typedef struct sk_ctx sk_ctx;

typedef struct sk_config {
    int device;              /* HIP device ordinal */
    int redis_major;         /* 3 = redis 3.2.0 semantics (reference CI pin, R:.travis.yml:23-24);
                                >= 5: HLL_Q sentinel in hllPatLen + Ertl estimator */
    uint64_t max_bit_offset; /* exclusive SETBIT/GETBIT offset limit; 0 -> 2^32 (redis 3.2: 512 MB strings) */
    uint64_t hll_capacity;   /* initial HLL slab capacity (16 KiB each); 0 -> 1024 */
    uint64_t max_batch;      /* largest single device batch (elements); 0 -> 1<<22 */
} sk_config;

/* ---- lifecycle ---- */
int sk_open(const sk_config *cfg, sk_ctx **out);
int sk_close(sk_ctx *ctx);
const char *sk_last_error(sk_ctx *ctx);
const char *sk_strerror(int status);
void *sk_stream(sk_ctx *ctx); /* the context's hipStream_t (for event timing) */
int sk_sync(sk_ctx *ctx);

/* ---- host-only helpers (no GPU needed) ---- */
/* visible HIP devices (0 without a GPU) */
int sk_device_count(void);
/* CRC16-XMODEM, M:connection/CRC16.java:55-61 */
uint32_t sk_crc16(const uint8_t *bytes, uint64_t len);
/* ClusterConnectionManager.calcSlot, M:cluster/ClusterConnectionManager.java:543-558;
 * -1 where Java's substring() throws (a '}' before the '{', or none). */
int32_t sk_calc_slot(const uint8_t *key, uint64_t len);
/* partitioner: owning GPU = calcSlot % n_gpus (-1 if calcSlot throws) */
int32_t sk_owner(const uint8_t *key, uint64_t len, int32_t n_gpus);
/* sk_owner of n keys (off u64[n+1], bytes) into out[n] */
int sk_owner_many(uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes, int32_t n_gpus, int32_t *out);
/* RedissonBloomFilter.optimalNumOfBits / optimalNumOfHashFunctions (:69-78) */
int64_t sk_bloom_optimal_bits(int64_t expected_insertions, double false_probability);
int32_t sk_bloom_optimal_k(int64_t expected_insertions, int64_t bits);
/* hllCount from a 64-bin register histogram (exact when no register >= 40
 * under redis 3.x; always under >= 5).  encoding 0 sparse / 1 dense / 2 raw. */
uint64_t sk_hll_estimate_hist(const uint32_t *hist64, int redis_major);

/* ---- key directory (one keyspace per context, like one redis db) ---- */
/* type of key (SK_TYPE_*) */
int sk_type(sk_ctx *ctx, const uint8_t *key, uint64_t len, int *out_type);
/* types of n keys in one call (SK_TYPE_*; 3 = a Bloom filter's name) */
int sk_type_many(sk_ctx *ctx, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes, int32_t *out_types);
/* DEL k1..kn -> number removed (RedissonObject.delete / RBitSet.clear, M:RedissonBitSet.java:250) */
int sk_del(sk_ctx *ctx, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes, uint64_t *out_removed);
/* FLUSHALL: remove every key and Bloom config of the context */
int sk_flushall(sk_ctx *ctx);
/* resolve HLL names to slab ids, creating empty HLLs for missing names (what
 * PFADD / PFMERGE do).  out_created[i] = 1 if this call created it. */
int sk_hll_resolve(sk_ctx *ctx, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes,
                   uint32_t *out_ids, uint8_t *out_created);
/* handles of existing HLL keys, creating nothing: out_ids[i] = 0xffffffff for a
 * missing key (PFCOUNT / countWith semantics: missing keys are empty); a key
 * holding a plain string fails with SK_EWRONGTYPE.  Parallel directory pass
 * for >= 64k keys (cross-GPU countWith over 1M tenants, cluster.py). */
int sk_hll_lookup(sk_ctx *ctx, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes, uint32_t *out_ids);

/* ---- RHyperLogLog (M:RedissonHyperLogLog.java:66-97) ---- */
/* Batch of PFADD commands in RBatch order.  Command c targets key c and adds
 * elem_counts[c] elements (consecutive in elem_off/elem_bytes).  out_changed[c]
 * = PFADD reply (1 if a register rose or the key was created), with exact
 * sequential semantics inside the batch. */
int sk_pfadd(sk_ctx *ctx, uint32_t n_cmds, const uint64_t *key_off, const uint8_t *key_bytes,
             const uint32_t *elem_counts, const uint64_t *elem_off, const uint8_t *elem_bytes,
             uint8_t *out_changed);
/* sk_pfadd with keys pre-resolved to slab ids by sk_hll_resolve (the Java
 * executor caches name -> id per tenant, SURVEY 8(b) "key names resolved to
 * slab ids on the Java side"); host buffers, same replies.  An id is valid
 * while its key owns the slab: after DEL, SET, a BITOP / flushall that
 * replaced the key, the call fails with SK_ESTALE (nothing is written) and
 * the caller drops its cached id and resolves the name again.  Replaces the PFADD
 * round trip of M:RedissonHyperLogLog.java:66-68 / M:RedissonBatch.java:76-83. */
int sk_pfadd_ids(sk_ctx *ctx, uint32_t n_cmds, const uint32_t *key_ids, const uint32_t *elem_counts,
                 const uint64_t *elem_off, const uint8_t *elem_bytes, uint8_t *out_changed);
/* Host ingress in prefix form (the group-commit path of GpuBatchCoalescer and the Bloom coalescer): n one-element
 * commands whose elements share the byte prefix prefix[0..prefix_len) (prefix_len <= 255: a codec's type header --
 * every Jackson Long is ["java.lang.Long",<digits>]); element i = prefix followed by suffix bytes
 * [suffix_off[i], suffix_off[i+1]) (u32 offsets into suffix_bytes, which keeps >= 16 B of readable padding).  Only
 * the suffixes and the u32 offsets cross the host link; the elements are rebuilt on the device and the replies are
 * those of the same commands through sk_pfadd_ids / sk_bloom_add / sk_bloom_contains. */
int sk_pfadd_ids_prefix(sk_ctx *ctx, uint32_t n, const uint32_t *key_ids, const uint8_t *prefix, uint32_t prefix_len,
                        const uint32_t *suffix_off, const uint8_t *suffix_bytes, uint8_t *out_changed);
/* PFADD of one element per command, keys pre-resolved to slab ids (all
 * existing); device-resident inputs.  d_out_changed u8[n] on device.
 * Replies are the sequential replies of the n commands in order, so a caller
 * may group-commit many RBatches into one call.  Calls of >= 4 M commands
 * (SK_PFL_MIN) and >= 160 per sketch of the store (SK_PFL_RATIO) are
 * applied with the line schedule: register lines streamed
 * once per call instead of once per element (DESIGN.md "PFADD group commit"). */
int sk_pfadd_dev(sk_ctx *ctx, uint64_t n, const uint32_t *d_key_ids, const uint64_t *d_elem_off,
                 const uint8_t *d_elem_bytes, uint64_t elem_bytes_len, uint8_t *d_out_changed);
/* Batch of PFCOUNT commands: command c counts the union of nkeys[c] keys
 * (1 = RHyperLogLog.count, >1 = countWith).  Missing keys count as empty. */
int sk_pfcount(sk_ctx *ctx, uint32_t n_cmds, const uint32_t *nkeys, const uint64_t *key_off,
               const uint8_t *key_bytes, int64_t *out_counts);
/* RHyperLogLog.count (M:RedissonHyperLogLog.java:78-81) of n keys given by
 * slab ids from sk_hll_resolve (cached by the caller, as for sk_pfadd_ids):
 * out[i] = PFCOUNT of key_ids[i].  One histogram launch, estimates on host
 * threads.  Ids no key holds fail with SK_ESTALE (as for sk_pfadd_ids). */
int sk_pfcount_ids(sk_ctx *ctx, uint64_t n, const uint32_t *key_ids, int64_t *out);
/* per-key exact register sums for slab ids (device in / device out u64[2n]): d_out[2i] = sum of 2^(40 - r) over the
 * registers, d_out[2i+1] = zero registers | (a register >= 40) << 32.  Without such a register,
 * E = d_out[2i] * 2^-40 is bit-identical to redis 3.x hllDenseSum (the PFCOUNT path of sk_pfcount /
 * sk_pfcount_ids under redis_major 3); with one, d_out[2i] is not meaningful */
int sk_hll_sum_dev(sk_ctx *ctx, uint64_t n, const uint32_t *d_key_ids, uint64_t *d_out);
/* per-key 64-bin register histograms for slab ids (device in / device out u32[n*64]) */
int sk_hll_histogram_dev(sk_ctx *ctx, uint64_t n, const uint32_t *d_key_ids, uint32_t *d_hist);
/* PFMERGE dest src1..srcn (dest included in the max, becomes dense) */
int sk_pfmerge(sk_ctx *ctx, const uint8_t *dest, uint64_t dest_len, uint32_t n_src,
               const uint64_t *src_off, const uint8_t *src_bytes);
/* union of n slab ids into a 16384-byte register array on device (d_out);
 * building block of the cross-GPU merge (then RCCL uint8 max all-reduce). */
int sk_hll_union_dev(sk_ctx *ctx, uint64_t n, const uint32_t *d_key_ids, uint8_t *d_out);
/* the local step of countWith / PFMERGE over keys sharded by calcSlot % n_gpus: register max of the existing
 * HLLs among keys[0..n) owned by `rank` into d_out (16384 B device); *n_used = HLLs merged
 * (replaces, per shard, the name resolution of M:RedissonHyperLogLog.java:86-97) */
int sk_hll_union_keys(sk_ctx *ctx, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes, int32_t n_gpus,
                      int32_t rank, uint8_t *d_out, uint32_t *n_used);
/* PFCOUNT of 16384 raw registers in device memory (multi-key PFCOUNT semantics: the union's estimate); the
 * last step of the cross-GPU countWith after the MAX all-reduce (M:RedissonHyperLogLog.java:83-89) */
int sk_hll_count_registers_dev(sk_ctx *ctx, const uint8_t *d_regs, int64_t *out_count);
/* pinned host memory (hipHostMalloc) for inputs the caller fills in place -- the JNI side wraps it in a direct
 * ByteBuffer for the group-commit coalescer -- so their H2D needs no staging copy.  Pageable inputs of >= 4 MiB
 * are staged by the library through two pinned buffers (host threads fill one while the other is copied). */
int sk_host_alloc(sk_ctx *ctx, uint64_t bytes, void **out_ptr);
int sk_host_free(sk_ctx *ctx, void *ptr);
/* HLL keyspace epoch: changes whenever an HLL key is created or removed.  A caller that caches the slab ids
 * of a key set on the device (the cross-GPU countWith of cluster.py through sk_hll_union_dev) re-resolves
 * the set when the epoch moved: the ids then still name exactly the set's existing HLLs. */
int sk_hll_epoch(sk_ctx *ctx, uint64_t *out_epoch);
/* write 16384 unpacked registers (device pointer) into a key as max (PFMERGE of a raw array) */
int sk_hll_merge_registers_dev(sk_ctx *ctx, const uint8_t *key, uint64_t len, const uint8_t *d_regs);
/* parity readback: 16384 unpacked registers of an HLL key (zeros if missing) */
int sk_hll_registers(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint8_t *out16384);

/* ---- RBitSet (M:RedissonBitSet.java:53-268) ---- */
/* batch of SETBIT in order; out_old[i] = previous bit (SETBIT reply), may be NULL */
int sk_setbit(sk_ctx *ctx, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes,
              const uint64_t *offsets, const uint8_t *values, uint8_t *out_old);
/* batch of GETBIT */
int sk_getbit(sk_ctx *ctx, uint32_t n, const uint64_t *key_off, const uint8_t *key_bytes,
              const uint64_t *offsets, uint8_t *out_bits);
/* RBitSet.set(from, to) / clear(from, to) (M:RedissonBitSet.java:194-228, one
 * SETBIT_VOID per bit in a pipeline): bits [from, to) := value; from >= to is a
 * no-op.  Offsets outside [0, max_bit_offset) fail with SK_ERANGE after the
 * in-range bits are applied (a pipeline runs the other commands). */
int sk_set_bit_range(sk_ctx *ctx, const uint8_t *key, uint64_t len, int64_t from, int64_t to, int value);
/* single-key device-resident variants for the bulk path (C5) */
/* SETBIT with one value per op (d_values u8[n], device); old bits in d_out_old (may be NULL) */
int sk_setbit_values_dev(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint64_t n, const uint64_t *d_offsets,
                         const uint8_t *d_values, uint8_t *d_out_old);
/* RBitSet range-sharded over the GPUs (C5 across GPUs; M:RedissonBitSet.java:53-81 GETBIT / SETBIT): shard s of
 * `world` holds logical bits [s * shard_bits, (s + 1) * shard_bits).  sk_route_bits splits a device batch of logical
 * offsets (n < 2^32) stably by shard: d_send = shard 0's ops, then shard 1's, ..., as shard-local offsets in batch
 * order (d_send_values alongside when d_values != NULL), d_dst[i] = op i's slot, out_counts[s] = ops of shard s
 * (host u64[world]); an offset >= world * shard_bits fails with SK_ERANGE.  sk_alltoallv exchanges the parts over
 * the context's RCCL communicator (per-peer byte counts; displacements = their prefix sums), the owner applies its
 * ops with sk_setbit_dev / sk_getbit_dev, the replies travel back the same way, and sk_unroute_u8 puts them in
 * batch order: d_out[i] = d_rep[d_dst[i]]. */
int sk_route_bits(sk_ctx *ctx, uint64_t n, const uint64_t *d_offsets, const uint8_t *d_values, uint64_t shard_bits,
                  int32_t world, uint64_t *d_send, uint8_t *d_send_values, uint32_t *d_dst, uint64_t *out_counts);
int sk_unroute_u8(sk_ctx *ctx, uint64_t n, const uint32_t *d_dst, const uint8_t *d_rep, uint8_t *d_out);
/* One RBloomFilter range-sharded over the GPUs (redisson_amd/cluster.py RangeShardedBloom; RedissonBloomFilter.add /
 * contains, M:RedissonBloomFilter.java:80-168): sk_bloom_indexes_dev writes the probe bit indexes of n device
 * elements, element-major (d_idx u64[n * nprobe]: probes 0..nprobe-1 of hash(), :116-131, nprobe <= k); they are
 * routed to the shards that own them like SETBIT / GETBIT (sk_route_bits ...), and sk_reduce_groups_u8 turns the
 * per-probe replies back in element order into one reply per element: d_out[i] = AND(d_in[i * group ..
 * i * group + take)) ^ invert -- contains = AND of probes 0..k-2 (Q2), add = one of probes 0..k-2 was 0. */
int sk_bloom_indexes_dev(sk_ctx *ctx, uint64_t n, const uint64_t *d_off, const uint8_t *d_bytes, int64_t size,
                         int32_t k, int32_t nprobe, uint64_t *d_idx);
int sk_reduce_groups_u8(sk_ctx *ctx, uint64_t n, uint32_t group, uint32_t take, int invert, const uint8_t *d_in,
                        uint8_t *d_out);
int sk_alltoallv(sk_ctx *ctx, const void *d_send, const uint64_t *send_bytes, void *d_recv,
                 const uint64_t *recv_bytes);
int sk_setbit_dev(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint64_t n, const uint64_t *d_offsets,
                  uint8_t value, uint8_t *d_out_old);
int sk_getbit_dev(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint64_t n, const uint64_t *d_offsets,
                  uint8_t *d_out_bits);
int sk_bitcount(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint64_t *out);
int sk_strlen(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint64_t *out);
/* BITOP op dest src1..srcn -> out_len = result length (0 deletes dest) */
int sk_bitop(sk_ctx *ctx, int op, const uint8_t *dest, uint64_t dest_len, uint32_t n_src,
             const uint64_t *src_off, const uint8_t *src_bytes, uint64_t *out_len);
/* GET: HLL keys -> dense "HYLL" string (12304 B); strings -> raw bytes.
 * *out_len = length (or -1 when the key does not exist); copies min(cap, len). */
int sk_get(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint8_t *buf, uint64_t cap, int64_t *out_len);
/* SET key raw-bytes (RBitSet.set(BitSet), M:RedissonBitSet.java:211-214) */
int sk_set(sk_ctx *ctx, const uint8_t *key, uint64_t len, const uint8_t *val, uint64_t val_len);
/* GET / SET of a bit string with the value in DEVICE memory of this context's
 * GPU (cross-GPU BITOP / Bloom union, redisson_amd/cluster.py: a shard or an
 * operand gathered with sk_allgather becomes a local string, no host copy).
 * sk_get_dev on an HLL key: SK_EWRONGTYPE. */
int sk_get_dev(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint8_t *d_buf, uint64_t cap, int64_t *out_len);
int sk_set_dev(sk_ctx *ctx, const uint8_t *key, uint64_t len, const uint8_t *d_val, uint64_t val_len);
/* RBitSet.length() Lua script (M:RedissonBitSet.java:180-192), same result and errors */
int sk_bitset_length(sk_ctx *ctx, const uint8_t *key, uint64_t len, int64_t *out);

/* ---- RBloomFilter (M:RedissonBloomFilter.java) ---- */
/* tryInit :223-252 -> *out_ok 1 if created, 0 if a config already existed */
int sk_bloom_try_init(sk_ctx *ctx, const uint8_t *name, uint64_t len, int64_t expected_insertions,
                      double false_probability, int *out_ok);
/* readConfig :206-221 (SK_ENOTINIT if absent) */
int sk_bloom_config(sk_ctx *ctx, const uint8_t *name, uint64_t len, int64_t *size, int32_t *hash_iterations,
                    int64_t *expected_insertions, double *false_probability);
/* add :80-114 / contains :133-168 for n encoded elements, checked against the
 * caller's (size, k) like addConfigCheck :180-186 (SK_ECONFIG on mismatch). */
int sk_bloom_add(sk_ctx *ctx, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                 const uint64_t *elem_off, const uint8_t *elem_bytes, uint8_t *out);
int sk_bloom_contains(sk_ctx *ctx, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                      const uint64_t *elem_off, const uint8_t *elem_bytes, uint8_t *out);
int sk_bloom_add_prefix(sk_ctx *ctx, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                        const uint8_t *prefix, uint32_t prefix_len, const uint32_t *suffix_off,
                        const uint8_t *suffix_bytes, uint8_t *out);
int sk_bloom_contains_prefix(sk_ctx *ctx, const uint8_t *name, uint64_t len, int64_t size, int32_t k, uint32_t n,
                             const uint8_t *prefix, uint32_t prefix_len, const uint32_t *suffix_off,
                             const uint8_t *suffix_bytes, uint8_t *out);
int sk_bloom_add_dev(sk_ctx *ctx, const uint8_t *name, uint64_t len, uint64_t n, const uint64_t *d_elem_off,
                     const uint8_t *d_elem_bytes, uint64_t elem_bytes_len, uint8_t *d_out);
int sk_bloom_contains_dev(sk_ctx *ctx, const uint8_t *name, uint64_t len, uint64_t n, const uint64_t *d_elem_off,
                          const uint8_t *d_elem_bytes, uint64_t elem_bytes_len, uint8_t *d_out);
/* count :188-199 */
int sk_bloom_count(sk_ctx *ctx, const uint8_t *name, uint64_t len, int32_t *out);

/* ---- device memory and timing on the context's device / stream ---- */
int sk_dev_alloc(sk_ctx *ctx, uint64_t bytes, void **out);
int sk_dev_free(sk_ctx *ctx, void *p);
int sk_h2d(sk_ctx *ctx, void *d_dst, const void *src, uint64_t n);
int sk_d2h(sk_ctx *ctx, void *dst, const void *d_src, uint64_t n);
int sk_d2d(sk_ctx *ctx, void *d_dst, const void *d_src, uint64_t n);
int sk_dev_memset(sk_ctx *ctx, void *d_p, int value, uint64_t n);
/* async mode: sk_pfadd_dev / sk_bloom_contains_dev / sk_bloom_add_dev return
 * once enqueued (inputs must stay valid until sk_sync); default off */
/* Redis HLL strings byte for byte (off by default; set while no HLL key exists, or SK_HLL_EXACT_STRINGS=1):
 * keys keep redis-server 3.2's sparse encoding until hllSparseSet would promote them (3000 bytes or a register
 * past 32), and the 8 cached-cardinality bytes follow PFADD / single-key PFCOUNT / PFMERGE, so sk_get returns
 * what GET on redis-server returns (M:RedissonBitSet.java:88-91).  Costs one logged record per register rise
 * and a host replay per PFADD batch; the partition path is used for every batch. */
int sk_hll_exact_strings(sk_ctx *ctx, int on);
int sk_set_async(sk_ctx *ctx, int on);
/* completion tickets (with sk_set_async): a ticket covers everything enqueued on
 * the context so far.  sk_poll never blocks and releases a finished ticket;
 * sk_wait blocks (without holding the context lock) and releases it. */
int sk_ticket(sk_ctx *ctx, uint64_t *out_ticket);
int sk_poll(sk_ctx *ctx, uint64_t ticket, int *out_done);
int sk_wait(sk_ctx *ctx, uint64_t ticket);
/* HIP events on the context stream: 16 slots; elapsed(a, b) waits for b */
int sk_timer_record(sk_ctx *ctx, int slot);
int sk_timer_elapsed(sk_ctx *ctx, int slot_a, int slot_b, float *ms);
/* per-kernel device time inside the library (event pairs around each launch
 * of a phase): "pfadd_hash", "pfadd_sort", "pfadd_apply", "hll_hist",
 * "hll_union", "bloom_contains", "bloom_probes", "bloom_sort", "bloom_apply",
 * "setbit", "getbit", "bitcount", "bitop", "pfadd_claim", "pfadd_commit",
 * "pfp_hash", "pfp_apply", "pfp_reply", "bloom_rc_hash", "bloom_rc_probe",
 * "pfadd_long", "bloom_ra_hash", "bloom_ra_apply", "pfl_hash", "pfl_part",
 * "pfl_apply" (k_pfl_plan + k_pfl_apply), "hll_sum", "pfl_fill" (the
 * line schedule's default-reply fill);
 * chains: "bloom_contains" (every kernel of one contains call), "pfadd" (every
 * kernel of one sk_pfadd_dev batch).  "pfadd_long_fallback" is a count, not a
 * time: calls whose long elements (>= 64 KiB) were re-hashed per thread because
 * a look-back wait of the bit-round scan ran out (the call still succeeds) */
int sk_prof_enable(sk_ctx *ctx, int on);
/* time only the named phases while profiling is on ("a,b,c"; NULL: every phase) */
int sk_prof_only(sk_ctx *ctx, const char *phase);
int sk_prof_reset(sk_ctx *ctx);
int sk_prof_read(sk_ctx *ctx, const char *phase, uint64_t *launches, double *total_ms);

/* ---- persistence: redis-server's own formats (SURVEY 5 "Checkpoint / resume", 8(f) rank 1) ----
 * Replaces redis-server's RDB persistence behind the keys the store holds (Redisson's tests drive it through
 * RedisRunner's nosave / appendonly / dbfilename options, T:RedisRunner.java:68,174,339,497; the values are the GET /
 * SET byte forms, M:RedissonBitSet.java:88-91,211-214, and the Bloom config hash, M:RedissonBloomFilter.java:
 * 231-256).  Every value is written as redis-server 3.2 writes it (RDB_VERSION 7): HLLs and bit strings as strings
 * (an HLL is its GET bytes: the dense `HYLL` encoding, or the sparse string in exact mode), a Bloom filter's
 * "{name}__config" as a hash in HMSET order.  Reading accepts redis-server 3.2-5.0 output of those two types
 * (integer- and LZF-encoded strings, ziplist hashes).  A restored string that is a Redis HLL becomes an HLL key at
 * once when that leaves GET's bytes unchanged (exact mode, or the dense encoding with a stale cache: what this store
 * writes), else on its first HLL command, as after SET. */

/* SCAN: up to `count` keys from `cursor` (0 = start); *next_cursor = 0 when the scan is done.  Every key present
 * for the whole scan is returned once: a key's position is a hash of its name, so it holds across type changes
 * (a string adopted as an HLL) and replacement; keys sharing a position are never split between calls (a call may
 * then return fewer than `count`).  names: the key bytes, name_off u64[*out_n + 1] into it (stops early rather
 * than pass names_cap); types: SK_TYPE_HLL / SK_TYPE_STRING / SK_TYPE_HASH (a Bloom filter config). */
int sk_scan(sk_ctx *ctx, uint64_t cursor, uint32_t count, uint64_t *next_cursor, uint32_t *out_n,
            uint64_t *name_off, uint8_t *names, uint64_t names_cap, int32_t *types);
/* DBSIZE: the number of keys the store holds (HLLs, strings, Bloom filter configs), O(1) */
int sk_dbsize(sk_ctx *ctx, uint64_t *out);
/* DUMP key: the redis-server DUMP payload (type, value, RDB version, CRC64).  *out_len = its size (-1: no such
 * key); at most cap bytes are copied (call with cap = 0 to size the buffer). */
int sk_dump(sk_ctx *ctx, const uint8_t *key, uint64_t len, uint8_t *buf, uint64_t cap, int64_t *out_len);
/* RESTORE key 0 payload [REPLACE]: SK_EBUSYKEY if the key exists and !replace, SK_EPAYLOAD for a bad payload. */
int sk_restore(sk_ctx *ctx, const uint8_t *key, uint64_t len, const uint8_t *payload, uint64_t plen, int replace);
/* SAVE: every key of the store into an RDB file at `path` (written in place; HLLs packed to their dense bodies
 * on the GPU in bulk), plus n_extra caller-held keys: 2 * n_extra items in (off, bytes), key i then its DUMP
 * payload (the RESP front-end's small hashes).  *out_keys = keys written. */
int sk_save(sk_ctx *ctx, const char *path, uint32_t n_extra, const uint64_t *extra_off, const uint8_t *extra_bytes,
            uint64_t *out_keys);
/* Load an RDB file (this store's SAVE, or redis-server's dump.rdb holding strings and hashes) into the context;
 * keys in the file replace existing ones.  take (optional): offered every hash value first as a DUMP payload;
 * returning 1 keeps it out of the store (the RESP front-end holds its own hashes), 0 lets the store keep it (a
 * Bloom filter config), < 0 fails the load.  Expire times in the file are ignored (no TTL is served). */
typedef int (*sk_take_fn)(void *user, const uint8_t *key, uint64_t klen, const uint8_t *payload, uint64_t plen);
int sk_load(sk_ctx *ctx, const char *path, sk_take_fn take, void *user, uint64_t *out_keys);

/* ---- cross-GPU exchange: RCCL over xGMI (one context per GPU / process) ---- */
int sk_comm_unique_id(uint8_t *out128);
int sk_comm_init(sk_ctx *ctx, int nranks, int rank, const uint8_t *id128);
/* register-wise max of n bytes in place (cross-GPU PFMERGE / countWith) */
int sk_allreduce_max_u8(sk_ctx *ctx, uint8_t *d_buf, uint64_t n);
/* sum of n u64 in place (BITCOUNT of a range-sharded bitset) */
int sk_allreduce_sum_u64(sk_ctx *ctx, uint64_t *d_buf, uint64_t n);
/* gather bytes_per_rank from every rank into d_recv (rank-major) */
int sk_allgather(sk_ctx *ctx, const void *d_send, void *d_recv, uint64_t bytes_per_rank);

/* ---- bench / test helpers ---- */
/* Jackson default-typing bytes of Longs, ["java.lang.Long",<v>] (M:codec/JsonJacksonCodec.java:
 * 86-117, Long forced typed :103-106), for SplitMix64(seed) values; host buffers.
 * Call with bytes == NULL to get the offsets (and total size in off[n]). */
int sk_gen_jackson_longs(uint64_t seed, uint64_t n, uint64_t *off, uint8_t *bytes);
/* device variant: element j = value #(d_idx ? d_idx[j] : first + j) of the same
 * counter-based sequence; d_off u64[n+1], d_bytes sized n*39 + 16. */
int sk_gen_jackson_longs_dev(sk_ctx *ctx, uint64_t seed, const uint64_t *d_idx, uint64_t first, uint64_t n,
                             uint64_t *d_off, uint8_t *d_bytes);

#ifdef __cplusplus
}
#endif
#endif
