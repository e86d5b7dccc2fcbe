// sk_internal.h -- launchers exported by sk_kernels.hip to the store/executor.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace sk {


uint32_t pfp_blocks(uint64_t n);
uint32_t pfp_buckets();
uint32_t pfp_epb();
// pre: per-element hashes of the elements >= long_elem_bytes() (k_ms_planes + k_ms_rounds), or null
hipError_t launch_pfp_hash(hipStream_t st, uint64_t n, const uint32_t *key_ids, const uint64_t *off,
                           const uint8_t *bytes, int v5, uint64_t *chunks, uint32_t *S, uint16_t *pos,
                           uint32_t *big_alloc, const uint64_t *pre = nullptr);
uint64_t long_elem_bytes();
// MurmurHash64A (seed 0xadc83b19) of long elements into out_h[which[i]] by 64 bit rounds of an XOR scan.
// meta = which[n_long], first_wg[n_long + 1] (murmur_long_wgs(len) workgroups per element, n_wg in all), then at
// the next even word u64 poff[n_long + 1] (prefix of murmur_long_plane_words(len)); plane: poff[n_long] words;
// flags: n_wg * 64 + 2 words, flags[n_wg * 64 + 1] != 0 after the run = a look-back wait ran out (hashes invalid)
uint32_t murmur_long_wgs(uint64_t len);
uint64_t murmur_long_plane_words(uint64_t len);
hipError_t launch_murmur_long(hipStream_t st, uint32_t n_long, uint32_t n_wg, const uint8_t *bytes,
                              const uint64_t *off, const uint32_t *meta, uint32_t *plane, uint32_t *flags,
                              uint64_t *out_h);
hipError_t launch_pfp_apply(hipStream_t st, uint64_t n, const uint64_t *chunks, const uint32_t *S, uint8_t *arena,
                            uint8_t *rep, uint32_t *big_alloc, uint64_t *big_keys, uint32_t *big_vals,
                            uint8_t *changed, uint64_t *ev = nullptr,
                            uint32_t *ev_n = nullptr); // changed != null: replies straight to batch order (no k_pfp_reply)
hipError_t launch_pfp_reply(hipStream_t st, uint64_t n, const uint8_t *rep, const uint16_t *pos,
                            const uint32_t *cmd_of, uint8_t *changed);
// PFADD line schedule (one element per command, n <= 2^26, <= pfl_max_slabs() sketches): hash into 128 line
// buckets, sort each (bucket, tile of hash blocks) region by fine bucket (2^sh sketches) in LDS, apply each fine
// bucket with its lines in LDS
struct PflDims {
    uint32_t nblk, tb, ntile, nsub;  // hash blocks, blocks per run tile, tiles, fine buckets per bucket
    uint32_t sh;                     // 2^sh sketches per fine bucket
    uint32_t pk, pa, pai, pm_mask;   // fine buckets by permuted slab id: slab * pa mod 2^pk
    uint32_t nslab;
    uint32_t rcap, nreg;             // records a region holds in LDS; regions (128 x ntile)
    uint64_t nf;                     // fine buckets
    uint64_t c_words;                // C: region totals, region bases (nreg each), then C2[nreg][nsub + 1]
    uint64_t chunk_bytes, S_bytes;
};
PflDims pfl_dims(uint64_t n, uint32_t nslab, uint32_t tile_blocks = 0); // 0: the default tile
bool pfl_dims_ok(const PflDims &d);
uint32_t pfl_max_slabs();
hipError_t launch_pfl_hash(hipStream_t st, uint64_t n, const uint32_t *key_ids, const uint64_t *off,
                           const uint8_t *bytes, int v5, uint64_t *chunks, uint32_t *S, uint32_t *big_alloc);
// region totals + region sort; C u32[c_words], rec2 u64[nblk * SK_PFP_EPB] (u64 records or the 6-B planes); dropped records (slab >= nslab) reply 0 in changed
hipError_t launch_pfl_part(hipStream_t st, const PflDims &d, const uint64_t *chunks, const uint32_t *S, uint32_t *C,
                           uint64_t *rec2, uint8_t *changed);
// replies pre-filled with the call's default reply (rc: u32[32] reply-mix counters, par: this call's parity)
hipError_t launch_pfl_fill(hipStream_t st, uint8_t *changed, uint64_t n, uint32_t *rc, uint32_t par);
// big tables: 2 entries per record of the call (u64 keys, u32 values)
hipError_t launch_pfl_apply(hipStream_t st, const PflDims &d, const uint64_t *rec2, const uint32_t *C, uint32_t nslab,
                            uint8_t *arena, uint8_t *changed, uint32_t *big_alloc, uint64_t *big_keys,
                            uint32_t *big_vals, int flags, // flags & 32: replies pre-filled, only others stored
                            uint32_t *order,               // u32[nf]: dispatch order (heavy fine buckets first)
                            uint32_t *rc, uint32_t par);
hipError_t sort_keys_size(uint64_t n, unsigned begin_bit, unsigned end_bit, size_t *bytes);
hipError_t sort_keys(hipStream_t st, void *tmp, size_t tmp_bytes, const uint64_t *in, uint64_t *out, uint64_t n,
                     unsigned begin_bit, unsigned end_bit);
hipError_t sort_pairs64_size(uint64_t n, size_t *bytes);
hipError_t sort_pairs64(hipStream_t st, void *tmp, size_t tmp_bytes, const uint64_t *kin, uint64_t *kout,
                        const uint64_t *vin, uint64_t *vout, uint64_t n);
hipError_t sort_pairs_size(uint64_t n, unsigned begin_bit, unsigned end_bit, size_t *bytes);
hipError_t sort_pairs(hipStream_t st, void *tmp, size_t tmp_bytes, const uint64_t *kin, uint64_t *kout,
                      const uint32_t *vin, uint32_t *vout, uint64_t n, unsigned begin_bit, unsigned end_bit);
// per key: out[2k] = sum 2^(40 - r) over the registers, out[2k+1] = zeros | (a register >= 40) << 32 (PFCOUNT 3.x)
hipError_t launch_hll_sum(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *arena, uint64_t *out);
// 64-bin register histograms: slabs ids[] of the packed arena (packed), or u8 register arrays (ids[k] = 0)
hipError_t launch_hll_hist(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *arena, uint32_t *hist,
                           int packed);
// Redis dense HLL bodies in bulk (SAVE / DUMP / snapshot restore): out / in hold n x 12,288 B (16-B aligned), n < 2^30
hipError_t launch_hll_pack(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *arena, uint8_t *out);
hipError_t launch_hll_unpack(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *in, uint8_t *arena);
// out = max over sources (include_out: and out): sources are slabs ids[] of the packed arena (src_packed) or u8
// register arrays (ids null: consecutive 16 KiB arrays); out is a packed slab (out_packed) or 16384 u8 registers
hipError_t launch_hll_union(hipStream_t st, uint64_t n, const uint32_t *ids, const uint8_t *src, uint8_t *partial,
                            uint64_t max_groups, uint8_t *out, int include_out, int src_packed, int out_packed);
// scratch: 16 B per element, used by the split schedule (sched 3) only
hipError_t launch_bloom_contains(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes,
                                 const uint8_t *bits, const uint64_t *d_len, uint64_t size, uint64_t magic, int k,
                                 uint8_t *out, int sched, void *scratch = nullptr);
// contains, region schedule (large batches): hash + bucket probes by 128 KiB region, then one LDS-resident
// region per workgroup; records u32[rc_blocks(n) * rc_chunk_words(k)], S u32[rc_regions(size) * rc_blocks(n)]
uint32_t rc_blocks(uint64_t n);
uint32_t rc_regions(uint64_t size);
uint32_t rc_max_probes();
uint64_t rc_chunk_words(int k);
hipError_t launch_bloom_rc_hash(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                                uint64_t magic, int k, uint32_t *S, uint32_t *recs, uint8_t *out);
hipError_t launch_bloom_rc_probe(hipStream_t st, uint64_t n, uint64_t size, int k, const uint32_t *S,
                                 const uint32_t *recs, const uint8_t *bits, uint64_t cap_bytes, uint8_t *out,
                                 uint32_t *Z, uint32_t *GT);
// a shared element prefix (host ingress in prefix form), passed by value to the expand kernel
struct SkPrefix {
    uint64_t w[32]; // prefix bytes, <= 255
    uint32_t len;
};
hipError_t launch_expand_prefix(hipStream_t st, uint64_t n, const SkPrefix &pre, const uint32_t *soff,
                                const uint8_t *sbytes, uint64_t *off, uint8_t *bytes);
hipError_t launch_bloom_indexes(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                                uint64_t magic, int np, uint64_t *idx);
hipError_t launch_reduce_groups_u8(hipStream_t st, uint64_t n, uint32_t group, uint32_t take, uint32_t invert,
                                   const uint8_t *in, uint8_t *out);
// contains zero lists (k_bloom_rc_probe -> k_bloom_rc_zero): u32 words of the per-region lists and the group table
uint64_t rc_zero_list_words(uint64_t size);
uint64_t rc_group_table_words(uint64_t size);
// Bloom add, region schedule: pieces of <= ra_piece() elements; k <= rc_max_probes()
uint32_t ra_blocks(uint64_t n, int k);
uint64_t rc_seg_words(uint32_t nb, uint32_t nr); // u32 words of a hash's interleaved segment table (nb blocks, nr regions)
bool rc_seg_interleaved();
bool rc_probe_reads_st();                        // the hash writes an interleaved table (then launch_rc_stranspose)
hipError_t launch_rc_stranspose(hipStream_t st, uint32_t nb, uint32_t nr, const uint32_t *St, uint32_t *S);
uint32_t ra_regions(uint64_t size);
uint64_t ra_piece(int k);
uint64_t ra_chunk_words(int k);
uint32_t ra_max_probes();
hipError_t launch_bloom_ra_hash(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                                uint64_t magic, int k, uint32_t *S, uint32_t *recs, uint32_t *stop, uint32_t piece);
// Z u32[ra_chunk_words(k) x blocks] (one lists, <= the records), zalloc u32 scratch counter,
// GT u64[ra_group_table_words(size)] (one-list run table); out must be zeroed before (a stopped piece writes nothing)
uint64_t ra_group_table_words(uint64_t size);
hipError_t launch_bloom_ra_apply(hipStream_t st, uint64_t n, uint64_t size, int k, const uint32_t *S,
                                 const uint32_t *recs, uint8_t *bits, uint64_t cap_bytes, uint64_t *d_len,
                                 uint8_t *out, const uint32_t *stop, uint32_t piece, uint32_t *Z, uint32_t *zalloc,
                                 uint64_t *GT);
hipError_t launch_bloom_probes(hipStream_t st, uint64_t n, const uint64_t *off, const uint8_t *bytes, uint64_t size,
                               uint64_t magic, int k, uint64_t *keys);
hipError_t launch_bloom_apply(hipStream_t st, uint64_t m, const uint64_t *keys, uint8_t *bits, uint64_t *d_len, int k,
                              uint8_t *out);
hipError_t launch_getbit_multi(hipStream_t st, uint64_t n, const uint32_t *sid, const uint64_t *offs, const void *dir,
                               uint8_t *out);
hipError_t launch_getbit_single(hipStream_t st, uint64_t n, const uint64_t *offs, const uint8_t *buf,
                                const uint64_t *d_len, uint8_t *out);
hipError_t launch_setbit_keys(hipStream_t st, uint64_t n, const uint32_t *sid, const uint64_t *offs, uint64_t *keys,
                              uint32_t *vals);
hipError_t launch_setbit_apply(hipStream_t st, uint64_t n, const uint64_t *keys, const uint32_t *vals,
                               const uint8_t *values, uint8_t value_all, void *dir, uint8_t *out_old);
hipError_t launch_setbit_void(hipStream_t st, uint64_t n, const uint64_t *offs, uint8_t *buf, uint32_t value);
// dense SETBIT_VOID: keys = the offsets grouped by 2^sbv_region_bits()-bit region (ascending), start u32[regions + 1]
uint32_t sbv_region_bits();
hipError_t launch_setbit_void_regions(hipStream_t st, uint64_t n, const uint64_t *keys, uint64_t max_off,
                                      uint32_t *start, uint8_t *buf, uint64_t cap, uint32_t value);
// dense SETBIT_VOID, hand-written region partition (k_sbv_part -> k_sbv_fine -> k_sbv_runs) in a scratch of
// sbv_part_scratch_bytes(n, max_off) bytes; sbv_part_ok: the call's size fits the partition's tables
uint64_t sbv_part_scratch_bytes(uint64_t n, uint64_t max_off);
bool sbv_part_ok(uint64_t n, uint64_t max_off);
hipError_t launch_setbit_void_part(hipStream_t st, uint64_t n, const uint64_t *offs, uint64_t max_off, void *scratch,
                                   uint8_t *buf, uint64_t cap, uint32_t value);
// SETBIT with replies (and SETBIT_VOID of several keys or values) through the region partition with u64 records
// (k_sbv_part<u64> -> k_sbv_fine<u64> -> k_sbr_runs): op i sets bit offs[i] of the key whose virtual regions start at
// vrb[i] (nullptr: one key at 0; 0xffffffff: op skipped) to vals[i] (nullptr: value_all), replying the bit before it
// in batch order into out[i] (nullptr: none).  seg: SbrSeg[nseg] {u64 rb, u8 *ptr, u64 cap} sorted by rb.
struct SbrSegH {
    uint64_t rb;
    uint8_t *ptr;
    uint64_t cap;
};
uint64_t sbr_scratch_bytes(uint64_t n, uint64_t NRv);
bool sbr_ok(uint64_t n, uint64_t NRv);
hipError_t launch_setbit_regions(hipStream_t st, uint64_t n, const uint64_t *offs, const uint32_t *vrb,
                                 const uint8_t *vals, uint32_t value_all, uint64_t NRv, const void *seg, uint32_t nseg,
                                 void *scratch, uint8_t *out);
hipError_t launch_bit_range(hipStream_t st, uint8_t *buf, uint64_t from, uint64_t to, uint32_t value);
hipError_t launch_max_u64(hipStream_t st, uint64_t n, const uint64_t *v, uint64_t *out);
hipError_t launch_bitcount(hipStream_t st, const uint8_t *buf, uint64_t len, uint64_t *out);
hipError_t launch_bitop(hipStream_t st, int op, uint32_t nsrc, const uint8_t *const *srcs, const uint64_t *lens,
                        uint64_t maxlen, uint8_t *dst);

hipError_t gen_jackson_scan_size(uint64_t n, size_t *bytes);
hipError_t launch_gen_jackson(hipStream_t st, uint64_t n, uint64_t seed, const uint64_t *idx, uint64_t first,
                              uint64_t *lens, void *tmp, size_t tmp_bytes, uint64_t *off, uint8_t *out);

// range-sharded RBitSet routing: stable split of a batch by shard (offset / shard_bits < world <= route_max_world());
// cnt u32[world * route_blocks(n) + 1] (the last word zero), base the same size; *bad = 1 for an offset past the
// last shard; send u64[n] shard-local offsets grouped by shard, svals (if vals) alongside, dst u32[n] each op's slot
uint32_t route_blocks(uint64_t n);
uint32_t route_max_world();
hipError_t route_scan_size(uint64_t m, size_t *bytes);
hipError_t launch_route(hipStream_t st, uint64_t n, const uint64_t *offs, const uint8_t *vals, uint64_t shard_bits,
                        uint32_t world, uint32_t *cnt, uint32_t *base, void *tmp, size_t tmp_bytes, uint32_t *bad,
                        uint64_t *send, uint8_t *svals, uint32_t *dst);
hipError_t launch_unroute(hipStream_t st, uint64_t n, const uint32_t *dst, const uint8_t *rep, uint8_t *out);

} // namespace sk
