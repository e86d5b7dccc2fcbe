"""Full-size parity at BASELINE.json's configurations, on the device.

The oracle cannot replay 10^9 commands in seconds, so these tests keep the size dimension of each config (100 k
tenant arena, the 2^32-class Bloom array, 1 M tenant HLLs, 2^34-bit bitsets) and check the state through
properties that do not need a sequential replay of everything:
- register arrays and Bloom / bitset bit arrays are order-free (max, OR): the threaded checkers of
  oracle/oracle_mt.c rebuild them from the same generated elements and the whole arrays are compared;
- PFADD replies depend on order only within a key: a checker thread owns whole keys and applies their commands in
  batch order, so every reply is compared;
- PFCOUNT / countWith / bloom count follow from the compared arrays.
Elements are the SplitMix64 -> Jackson Long stream of the bench (generated on the device by the engine and on the
host by the checker), so no element buffer is ever shipped.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M = 1 << 20


def _engine(**kw):
    from redisson_amd import SketchEngine

    return SketchEngine(device=0, **kw)


@pytest.mark.parametrize("per_call", [M, 64 * M], ids=["partition_1M", "lines_64M"])
def test_c2_pfadd_100k_tenants_full_arena(O, per_call):
    """C2: 100 k tenants (1.6 GB of registers), 128 M single-element PFADDs, one 1 M RBatch per call (partition
    path) or 64 RBatches group-committed per call (line schedule): every reply, every register of every tenant,
    every per-key PFCOUNT and the union count equal the oracle's."""
    T, NB, seed = 100_000, 128 * M // per_call, 0x5EED2002
    names = ["tenant:%d:hll" % t for t in range(T)]
    eng = _engine(hll_capacity=T + 16, max_batch=per_call)
    try:
        ids = eng.hll_resolve(names)
        kid = np.random.default_rng(22).integers(0, T, NB * per_call).astype(np.uint32)
        got = np.zeros(NB * per_call, dtype=np.uint8)
        d_out = eng.alloc(per_call)
        for b in range(NB):
            off, byt, tot = eng.gen_jackson_longs_dev(seed, per_call, first=b * per_call)
            d_ids = eng.to_device(ids[kid[b * per_call:(b + 1) * per_call]])
            eng.pfadd_dev(per_call, d_ids, off, byt, tot, d_out)
            got[b * per_call:(b + 1) * per_call] = d_out.download(np.uint8, per_call)
            for x in (off, byt, d_ids):
                x.free()
        regs = np.zeros((T, 16384), dtype=np.uint8)
        exists = np.zeros(T, dtype=np.uint8)
        want, ones = O.pfadd_gen(regs, exists, kid, seed, 0)
        assert int(got.sum()) == ones
        assert np.array_equal(got, want), "PFADD replies differ at %s" % np.flatnonzero(got != want)[:8]
        for t in range(T):
            r = eng.hll_registers(names[t])
            if not np.array_equal(r, regs[t]):
                raise AssertionError("registers of %s differ at %s" % (names[t], np.flatnonzero(r != regs[t])[:8]))
        counts = eng.pfcount([[nm] for nm in names])
        assert counts == [O.count_regs(regs[t], 1) for t in range(T)]
        assert eng.pfcount([names]) == [O.count_regs(regs.max(axis=0), 2)]
    finally:
        eng.close()


def test_c3_bloom_full_size_bit_array(O):
    """C3 as stated: tryInit(425 M, 0.008) -> m = 4,271,038,538 bits, k = 7 (a 534 MB array, indexes past 2^32); 1 B
    adds in 8 M batches (the array ends ~81 % set): the whole bit array (GET) and its Redis length equal the
    oracle's; 32 M contains (half members; the region schedule) equal the oracle's replies, members all true;
    count() follows BITCOUNT."""
    seed, NA, CH, NC = 0x5EED2003, 1_000_000_000, 8 * M, 32 * M
    eng = _engine(max_batch=CH)
    try:
        assert eng.bloom_try_init("c3", 425_000_000, 0.008)
        size, k, _, _ = eng.bloom_config("c3")
        assert (size, k) == (4_271_038_538, 7)
        d_out = eng.alloc(CH)
        for s in range(0, NA, CH):
            n = min(CH, NA - s)
            off, byt, tot = eng.gen_jackson_longs_dev(seed, n, first=s)
            eng.bloom_add_dev("c3", n, off, byt, tot, d_out)
            off.free()
            byt.free()
        bits, ln = O.bloom_add_gen(size, k, seed, 0, NA)
        got = eng.get("c3")
        assert len(got) == ln
        g = np.frombuffer(got, dtype=np.uint8)
        if not np.array_equal(g, bits[:ln]):
            raise AssertionError("Bloom bit array differs at bytes %s" % np.flatnonzero(g != bits[:ln])[:8])
        del g, got
        rng = np.random.default_rng(33)
        idx = np.where(rng.random(NC) < 0.5, rng.integers(0, NA, NC, dtype=np.uint64),
                       rng.integers(1 << 40, 1 << 41, NC, dtype=np.uint64)).astype(np.uint64)
        d_idx = eng.to_device(idx)
        off, byt, tot = eng.gen_jackson_longs_dev(seed, NC, d_idx=d_idx)
        d_c = eng.alloc(NC)
        eng.bloom_contains_dev("c3", NC, off, byt, tot, d_c)
        got_c = d_c.download(np.uint8, NC)
        want_c = O.bloom_contains_gen(bits, ln, size, k, seed, idx)
        assert np.array_equal(got_c, want_c), "contains differs at %s" % np.flatnonzero(got_c != want_c)[:8]
        assert got_c[idx < NA].all()
        bc = int(np.bitwise_count(bits[:ln]).sum(dtype=np.uint64))
        assert eng.bitcount("c3") == bc
        assert eng.bloom_count("c3") == O.bloom_count(size, k, bc)
    finally:
        eng.close()


def test_c4_union_over_1m_tenant_hlls(O):
    """C4 (one GPU's shard at full count): 1 M tenant HLLs (16 GB arena), 256 M elements; countWith over all 1 M
    keys and PFMERGE into a destination equal the oracle's union registers and estimate."""
    T, N, seed = 1_000_000, 256 * M, 0x5EED2004
    names = ["c4:%d" % t for t in range(T)]
    eng = _engine(hll_capacity=T + 16, max_batch=8 * M)
    try:
        ids = eng.hll_resolve(names)
        kid = np.random.default_rng(44).integers(0, T, N).astype(np.uint32)
        d_out = eng.alloc(8 * M)
        for s in range(0, N, 8 * M):
            off, byt, tot = eng.gen_jackson_longs_dev(seed, 8 * M, first=s)
            d_ids = eng.to_device(ids[kid[s:s + 8 * M]])
            eng.pfadd_dev(8 * M, d_ids, off, byt, tot, d_out)
            for x in (off, byt, d_ids):
                x.free()
        union = O.hll_union_gen(N, seed)
        assert eng.pfcount([names]) == [O.count_regs(union, 2)]
        eng.pfmerge("c4:dest", names)
        assert np.array_equal(eng.hll_registers("c4:dest"), union)
        assert eng.pfcount([["c4:dest"]]) == [O.count_regs(union, 1)]
    finally:
        eng.close()


def test_c5_bitsets_2p34_bits(O):
    """C5: two RBitSets of 2^34 bits (2 GiB each), 64 M random SETBITs each; GETBIT of 16 M offsets, BITCOUNT,
    length, GET, and BITOP AND / OR / NOT over the full strings equal the oracle's."""
    NBITS, NS, NG = 1 << 34, 64 * M, 16 * M
    rng = np.random.default_rng(55)
    eng = _engine(max_bit_offset=NBITS, max_batch=NS)
    try:
        host = {}
        for key in ("c5:a", "c5:b"):
            offs = rng.integers(0, NBITS, NS, dtype=np.uint64)
            if key == "c5:a":
                offs[0] = NBITS - 1   # a reaches the last byte of the 2 GiB string
            d = eng.to_device(offs)
            eng.setbit_dev(key, NS, d, 1)
            d.free()
            buf = np.zeros(NBITS // 8 + 16, dtype=np.uint8)
            O.setbits(buf, offs)
            host[key] = (buf, int(offs.max() >> np.uint64(3)) + 1, offs)
        a, la, offs_a = host["c5:a"]
        b, lb, _ = host["c5:b"]
        q = np.concatenate([offs_a[:NG // 2], rng.integers(0, NBITS, NG // 2, dtype=np.uint64)])
        d_q, d_o = eng.to_device(q), eng.alloc(NG)
        eng.getbit_dev("c5:a", NG, d_q, d_o)
        byte = a[(q >> np.uint64(3)).astype(np.int64)]
        want = (byte >> (np.uint64(7) - (q & np.uint64(7))).astype(np.uint8)) & np.uint8(1)
        assert np.array_equal(d_o.download(np.uint8, NG), want)
        for key, (buf, ln, _) in host.items():
            assert eng.strlen(key) == ln
            assert eng.bitcount(key) == int(np.bitwise_count(buf[:ln]).sum(dtype=np.uint64))
        assert np.array_equal(np.frombuffer(eng.get("c5:a"), np.uint8), a[:la])
        L = max(la, lb)
        for op, ref in (("AND", lambda: a[:L] & b[:L]), ("OR", lambda: a[:L] | b[:L])):
            assert eng.bitop(op, "c5:" + op, ["c5:a", "c5:b"]) == L
            got = np.frombuffer(eng.get("c5:" + op), np.uint8)
            assert np.array_equal(got, ref()), op
            del got
        assert eng.bitop("NOT", "c5:NOT", ["c5:b"]) == lb
        assert np.array_equal(np.frombuffer(eng.get("c5:NOT"), np.uint8), ~b[:lb])
    finally:
        eng.close()
