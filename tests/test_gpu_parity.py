"""GPU parity: HIP path (through the C ABI) vs the CPU oracle, bit-exact.

Seeded inputs at sizes the oracle finishes in seconds; edge cases the
reference path has (empty / ragged / long elements, intra-batch register and
bit collisions, missing keys, maximum offsets)."""
import numpy as np
import pytest

from redisson_amd import RedisException, gen_jackson_longs

pytestmark = pytest.mark.gpu


def _elems(seed, n):
    off, buf = gen_jackson_longs(seed, n)
    return [buf[off[i]:off[i + 1]].tobytes() for i in range(n)]


def _ragged(rng, n, maxlen=200):
    lens = rng.integers(0, maxlen, n)
    return [rng.integers(0, 256, l, dtype=np.uint8).tobytes() for l in lens]


# ------------------------------------------------------------------- PFADD
@pytest.mark.parametrize("nkeys,n", [(1, 5000), (7, 20000), (300, 30000), (100, 200000), (5, 10000)])
def test_pfadd_registers_and_replies(engine, O, nkeys, n):
    rng = np.random.default_rng(nkeys)
    elems = _elems(0x5EED0000 + nkeys, n)
    # duplicates -> replies 0, same-register collisions inside the batch
    elems += [elems[i] for i in rng.integers(0, n, n // 5)]
    keys = [b"pf:%d:%d" % (nkeys, rng.integers(0, nkeys)) for _ in elems]
    got = engine.pfadd(keys, [[e] for e in elems])
    ref = O.HLLStore()
    want = ref.pfadd(keys, [[e] for e in elems])
    assert got == want
    for k in set(keys):
        np.testing.assert_array_equal(engine.hll_registers(k), ref.regs[k])


def test_pfadd_multi_element_and_ragged(engine, O):
    rng = np.random.default_rng(7)
    keys, elems = [], []
    for c in range(400):
        keys.append(b"rag:%d" % (c % 13))
        elems.append(_ragged(rng, int(rng.integers(0, 6))))   # includes 0-element commands
    got = engine.pfadd(keys, elems)
    ref = O.HLLStore()
    assert got == ref.pfadd(keys, elems)
    for k in set(keys):
        np.testing.assert_array_equal(engine.hll_registers(k), ref.regs[k])


def test_pfadd_dense_single_key_sequential(engine, O):
    # C1 shape, small: many elements into ONE key -> long same-register segments
    elems = _elems(0x5EED0001, 60000)
    keys = [b"c1"] * len(elems)
    got = engine.pfadd(keys, [[e] for e in elems])
    ref = O.HLLStore()
    assert got == ref.pfadd(keys, [[e] for e in elems])
    np.testing.assert_array_equal(engine.hll_registers(b"c1"), ref.regs[b"c1"])


def test_pfcount_single_and_union(engine, O):
    rng = np.random.default_rng(3)
    ref = O.HLLStore()
    keys = [b"cnt:%d" % i for i in range(20)]
    for ci, k in enumerate(keys):
        m = int(10 ** rng.uniform(0, 5))
        es = _elems(1000 + ci, m)
        engine.pfadd([k] * m, [[e] for e in es])
        ref.pfadd([k] * m, [[e] for e in es])
    cmds = [[k] for k in keys] + [keys[:3], keys, [b"missing"], [b"missing", keys[4]]]
    assert engine.pfcount(cmds) == [ref.count(c) for c in cmds]


def test_pfcount_register_ge_40_order_fallback(engine, O):
    # craft an element whose rho >= 40 is astronomically rare; instead merge a
    # raw register array with values >= 40 through the device merge entry
    regs = np.zeros(16384, dtype=np.uint8)
    rng = np.random.default_rng(11)
    regs[:] = rng.integers(0, 12, 16384)
    regs[[5, 77, 9000]] = [40, 45, 50]
    d = engine.to_device(regs)
    engine.hll_merge_registers_dev(b"big40", d)
    np.testing.assert_array_equal(engine.hll_registers(b"big40"), regs)
    assert engine.pfcount([[b"big40"]]) == [O.count_regs(regs, 1)]        # dense order
    assert engine.pfcount([[b"big40", b"nokey2"]]) == [O.count_regs(regs, 2)]  # raw order


def test_pfmerge(engine, O):
    ref = O.HLLStore()
    srcs = [b"m:%d" % i for i in range(6)]
    for i, k in enumerate(srcs):
        es = _elems(77 + i, 3000)
        engine.pfadd([k] * len(es), [[e] for e in es])
        ref.pfadd([k] * len(es), [[e] for e in es])
    engine.pfadd([b"m:dest"], [[b"x"]])
    ref.pfadd([b"m:dest"], [[b"x"]])
    engine.pfmerge(b"m:dest", [b"m:dest"] + srcs + [b"m:absent"])
    ref.merge(b"m:dest", [b"m:dest"] + srcs + [b"m:absent"])
    np.testing.assert_array_equal(engine.hll_registers(b"m:dest"), ref.regs[b"m:dest"])
    assert engine.pfcount([[b"m:dest"]]) == [ref.count([b"m:dest"])]


def test_hll_wrongtype(engine):
    engine.setbit([b"wt:str"], [3], [1])
    with pytest.raises(RedisException, match="HyperLogLog"):
        engine.pfadd([b"wt:str"], [[b"a"]])


def test_pfadd_dev_path(engine, O):
    n, nkeys = 50000, 37
    off, buf = gen_jackson_longs(0x5EED0002, n)
    rng = np.random.default_rng(5)
    kid = rng.integers(0, nkeys, n).astype(np.uint32)
    names = [b"dev:%d" % i for i in range(nkeys)]
    ids = engine.hll_resolve(names)
    d_ids = engine.to_device(ids[kid])
    d_off = engine.to_device(off)
    d_buf = engine.to_device(buf, pad=16)
    d_out = engine.alloc(n)
    engine.pfadd_dev(n, d_ids, d_off, d_buf, int(off[-1]), d_out)
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    assert np.array_equal(d_out.download(np.uint8, n), want)
    for i, nm in enumerate(names):
        np.testing.assert_array_equal(engine.hll_registers(nm), regs[i])
    # histogram + host estimator == oracle count
    d_hist = engine.alloc(nkeys * 64 * 4)
    engine.hll_histogram_dev(nkeys, engine.to_device(ids), d_hist)
    h = d_hist.download(np.uint32).reshape(nkeys, 64)
    for i in range(nkeys):
        assert np.array_equal(h[i], np.bincount(regs[i], minlength=64)), i
        assert engine.estimate_hist(h[i]) == O.count_regs(regs[i], 1)


def test_hll_histogram_many_keys(engine, O):
    """More keys than histogram workgroups (each loops over keys and reuses its cleared LDS table), with the ids
    in a shuffled order and repeated: every row equals np.bincount of the key's registers."""
    n, nkeys = 600_000, 20_000
    off, buf = gen_jackson_longs(0x5EED0021, n)
    rng = np.random.default_rng(21)
    kid = rng.integers(0, nkeys, n).astype(np.uint32)
    names = [b"hh:%d" % i for i in range(nkeys)]
    ids = engine.hll_resolve(names)
    d_out = engine.alloc(n)
    engine.pfadd_dev(n, engine.to_device(ids[kid]), engine.to_device(off), engine.to_device(buf, pad=16),
                     int(off[-1]), d_out)
    regs, _ = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    order = np.concatenate([rng.permutation(nkeys), rng.integers(0, nkeys, 3000)]).astype(np.int64)
    d_hist = engine.alloc(len(order) * 64 * 4)
    engine.hll_histogram_dev(len(order), engine.to_device(ids[order]), d_hist)
    h = d_hist.download(np.uint32).reshape(len(order), 64)
    want = np.stack([np.bincount(regs[i], minlength=64) for i in order]).astype(np.uint32)
    np.testing.assert_array_equal(h, want)


def test_hll_histogram_high_registers(engine, O):
    """k_hll_hist counts a register r at row r & 31 (+1 in the low half, +65536 for r >= 32 in the high half) and takes
    the per-register increment only in 16-register groups holding a register >= 32: keys whose every group has one
    (registers uniform over 0..63), keys with a few high registers (single groups on the slow path), and keys with
    none; packed arena rows (k_hll_hist<true>) equal np.bincount, and the u8 form (k_hll_hist<false>, PFCOUNT of a
    raw register array, registers clamped to Redis's 0..51) gives the oracle's redis >= 5 count, whose q + 1 bin (51)
    weighs on the estimate."""
    from redisson_amd import SketchEngine
    rng = np.random.default_rng(78)
    regs = []
    for i in range(24):
        kind = i % 3
        if kind == 0:
            r = rng.integers(0, 64, 16384, dtype=np.uint8)
        elif kind == 1:
            r = rng.integers(0, 32, 16384, dtype=np.uint8)
            hot = rng.integers(0, 16384, 1 + i)
            r[hot] = rng.integers(32, 64, len(hot), dtype=np.uint8)
            r[hot[:1]] = 51
        else:
            r = rng.integers(0, 32, 16384, dtype=np.uint8)
        regs.append(r)
    names = [b"hh64:%d" % i for i in range(len(regs))]
    ids = engine.hll_resolve(names)
    for nm, r in zip(names, regs):
        d = engine.to_device(r)
        engine.hll_merge_registers_dev(nm, d)
        d.free()
    d_hist = engine.alloc(len(regs) * 64 * 4)
    engine.hll_histogram_dev(len(regs), engine.to_device(ids), d_hist)
    h = d_hist.download(np.uint32).reshape(len(regs), 64)
    want = np.stack([np.bincount(r, minlength=64) for r in regs]).astype(np.uint32)
    np.testing.assert_array_equal(h, want)
    e5 = SketchEngine(device=0, redis_major=5)
    try:
        for r in regs:
            r = np.minimum(r, 51).astype(np.uint8)   # registers a redis >= 5 histogram holds (q + 2 = 52 bins)
            d = e5.to_device(r)
            assert e5.hll_count_registers_dev(d) == O.count_regs(r, 1, 5)
            d.free()
    finally:
        e5.close()


# ------------------------------------------------------------------- Bloom
@pytest.mark.parametrize("n_exp,p", [(100, 0.03), (20000, 0.01), (5000, 0.5)])
def test_bloom_add_contains(engine, O, n_exp, p):
    name = "bf:%d:%s" % (n_exp, p)
    assert engine.bloom_try_init(name, n_exp, p)
    size, k, _, _ = engine.bloom_config(name)
    bits = O.BitString()
    rng = np.random.default_rng(n_exp)
    elems = _elems(n_exp, n_exp) + _ragged(rng, 300)           # includes >64 B (farmUo long path)
    elems += [elems[i] for i in rng.integers(0, len(elems), 200)]  # in-batch duplicates
    assert engine.bloom_add(name, size, k, elems) == bits.bloom_add(size, k, elems)
    probe = elems[::3] + _elems(n_exp + 1, 3000)
    assert engine.bloom_contains(name, size, k, probe) == bits.bloom_contains(size, k, probe)
    assert engine.get(name) == bits.bytes()
    assert engine.bitcount(name) == bits.bitcount()
    assert engine.bloom_count(name) == O.bloom_count(size, k, bits.bitcount())


def test_bloom_k1_and_config_errors(engine, O):
    from redisson_amd import IllegalStateException
    assert engine.bloom_try_init("bfk1", 10, 0.9)   # k == 1: add never true, contains always true
    size, k, _, _ = engine.bloom_config("bfk1")
    assert k == 1
    bits = O.BitString()
    els = [b"a", b"b", b"c"]
    assert engine.bloom_contains("bfk1", size, k, els) == bits.bloom_contains(size, k, els) == [True] * 3
    assert engine.bloom_add("bfk1", size, k, els) == bits.bloom_add(size, k, els)
    with pytest.raises(RedisException, match="Bloom filter config has been changed"):
        engine.bloom_add("bfk1", size + 1, k, els)
    with pytest.raises(IllegalStateException):
        engine.bloom_config("nobf")


# ------------------------------------------------------------------- bits
def test_setbit_getbit_sequential(engine, O):
    rng = np.random.default_rng(9)
    n = 20000
    keys = [b"bs:%d" % rng.integers(0, 5) for _ in range(n)]
    offs = rng.integers(0, 5000, n)
    vals = rng.integers(0, 2, n)
    got = engine.setbit(keys, offs, vals)
    ref = {}
    want = []
    for k, o, v in zip(keys, offs, vals):
        want.append(ref.setdefault(k, O.BitString()).setbit(int(o), int(v)))
    assert got == want
    for k, b in ref.items():
        assert engine.get(k) == b.bytes()
        assert engine.strlen(k) == len(b.bytes())
        assert engine.bitcount(k) == b.bitcount()
    q = rng.integers(0, 6000, 3000)
    qk = [b"bs:%d" % rng.integers(0, 6) for _ in q]   # bs:5 missing -> 0
    assert engine.getbit(qk, q) == [ref[k].getbit(int(o)) if k in ref else 0 for k, o in zip(qk, q)]


def test_bit_offset_limits(engine):
    top = 2 * 2147483647                       # RedissonBitSetTest.testIndexRange
    assert engine.getbit([b"lim"], [top]) == [0]
    engine.setbit([b"lim"], [top], [1])
    assert engine.getbit([b"lim"], [top]) == [1]
    with pytest.raises(RedisException, match="bit offset is not an integer or out of range"):
        engine.setbit([b"lim"], [1 << 32], [1])


def test_bitop(engine, O):
    rng = np.random.default_rng(2)
    data = {b"op:a": rng.integers(0, 256, 1000, dtype=np.uint8).tobytes(),
            b"op:b": rng.integers(0, 256, 37, dtype=np.uint8).tobytes(),
            b"op:c": rng.integers(0, 256, 4099, dtype=np.uint8).tobytes()}
    for k, v in data.items():
        engine.set(k, v)
    for op in ["AND", "OR", "XOR"]:
        srcs = [b"op:a", b"op:b", b"op:missing", b"op:c"]
        n = engine.bitop(op, b"op:dst:" + op.encode(), srcs)
        want = O.bitop(op, [data.get(s) for s in srcs])
        assert n == len(want)
        assert engine.get(b"op:dst:" + op.encode()) == want
    engine.bitop("NOT", b"op:a", [b"op:a"])
    assert engine.get(b"op:a") == O.bitop("NOT", [data[b"op:a"]])
    with pytest.raises(RedisException, match="BITOP NOT"):
        engine.bitop("NOT", b"x", [b"op:a", b"op:b"])
    # empty result deletes the destination
    assert engine.bitop("OR", b"op:c", [b"op:none1", b"op:none2"]) == 0
    assert engine.get(b"op:c") is None


def test_bulk_setbit_getbit_dev(engine):
    rng = np.random.default_rng(4)
    n = 1 << 16
    offs = rng.integers(0, 1 << 24, n).astype(np.uint64)
    d = engine.to_device(offs)
    engine.setbit_dev(b"bulk", n, d, 1)
    out = engine.alloc(n)
    engine.getbit_dev(b"bulk", n, d, out)
    assert int(out.download(np.uint8, n).sum()) == n
    assert engine.bitcount(b"bulk") == len(np.unique(offs))
    # with replies: first occurrence sees 0, repeats see 1
    offs2 = np.concatenate([offs[:100], offs[:100], rng.integers(1 << 24, 1 << 25, 100)]).astype(np.uint64)
    old = engine.alloc(len(offs2))
    engine.setbit_dev(b"bulk", len(offs2), engine.to_device(offs2), 0, old)
    o = old.download(np.uint8, len(offs2))
    assert o[:100].all() and not o[100:200].any()


def test_setbit_dev_max_offset_any_alignment(engine):
    """The batch's max offset (string growth, range check) is found with 16-B loads: at every start alignment and
    odd / even counts the string grows to exactly the highest op's byte."""
    rng = np.random.default_rng(12)
    for n in (1, 2, 3, 64, 1001, 100000):
        offs = rng.integers(0, 1 << 20, n + 1).astype(np.uint64)
        for lead in (0, 1):
            hi = int(rng.integers(1 << 21, 1 << 22))
            o = offs.copy()
            o[lead + int(rng.integers(0, n))] = hi          # the max somewhere in the n ops
            d = engine.to_device(o)
            key = b"mx:%d:%d" % (n, lead)
            engine.setbit_dev(key, n, d.ptr + 8 * lead, 1)
            assert engine.strlen(key) == hi // 8 + 1, (n, lead)
            d.free()


def test_dense_setbit_void_regions(engine):
    """A dense SETBIT_VOID batch (>= 2 ops per 128-B line, >= 256 regions of 32 KiB: the region path, k_sbv_apply)
    sets and then clears exactly the bits the per-op atomics would: repeated offsets, the first and last bit of the
    string, a last region cut short by the string's length, and a clear batch over a set string."""
    rng = np.random.default_rng(8)
    nbits = (1 << 27) - 12345                     # 16 MiB string: 512 regions, the last one partial
    offs = rng.integers(0, nbits, 3 << 20).astype(np.uint64)
    offs[:3] = [0, nbits - 1, 0]
    offs[3:1000] = offs[1000:1997]                # repeats
    engine.setbit_dev(b"dense", len(offs), engine.to_device(offs), 1)
    want = np.zeros((nbits + 7) // 8, dtype=np.uint8)
    np.bitwise_or.at(want, (offs >> np.uint64(3)).astype(np.int64),
                     (np.uint8(1) << (np.uint8(7) - (offs & np.uint64(7)).astype(np.uint8))).astype(np.uint8))
    assert engine.strlen(b"dense") == len(want)
    assert np.array_equal(np.frombuffer(engine.get(b"dense"), np.uint8), want)
    clr = np.concatenate([offs[: 1 << 20], rng.integers(0, nbits, 1 << 20).astype(np.uint64)])
    engine.setbit_dev(b"dense", len(clr), engine.to_device(clr), 0)
    np.bitwise_and.at(want, (clr >> np.uint64(3)).astype(np.int64),
                      (~(np.uint8(1) << (np.uint8(7) - (clr & np.uint64(7)).astype(np.uint8)))).astype(np.uint8))
    assert np.array_equal(np.frombuffer(engine.get(b"dense"), np.uint8), want)
    assert engine.bitcount(b"dense") == int(np.bitwise_count(want).sum(dtype=np.uint64))


@pytest.mark.parametrize("part", ["1", "0"])
def test_dense_setbit_void_partition_skew(O, part):
    """The hand-written region partition of dense SETBIT_VOID (k_sbv_part / k_sbv_fine / k_sbv_runs; "0": the
    rocPRIM radix-sort form it replaced) with 70 % of a 4 M-op call on one 32 KiB region: the fine-sort pieces of
    that region's bucket overflow the LDS and take the atomic placement; the string ends mid-region; set, then
    clear; the bytes equal numpy's."""
    import os

    from redisson_amd import SketchEngine

    os.environ["SK_SBV_PART"] = part
    try:
        eng = SketchEngine(device=0, max_batch=8 << 20)
    finally:
        del os.environ["SK_SBV_PART"]
    try:
        rng = np.random.default_rng(81)
        nbits = (1 << 28) + 777                       # 1025 regions, 5 coarse buckets, the last region partial
        n = 4 << 20
        offs = rng.integers(0, nbits, n).astype(np.uint64)
        hot = rng.random(n) < 0.7
        offs[hot] = (np.uint64(3) << np.uint64(18)) + rng.integers(0, 1 << 18, int(hot.sum())).astype(np.uint64)
        offs[0] = nbits - 1
        want = np.zeros((nbits + 7) // 8, dtype=np.uint8)
        for key, val, ops in ((b"skew", 1, offs), (b"skew", 0, offs[::3])):
            eng.setbit_dev(key, len(ops), eng.to_device(ops), val)
            m = (np.uint8(1) << (np.uint8(7) - (ops & np.uint64(7)).astype(np.uint8))).astype(np.uint8)
            if val:
                np.bitwise_or.at(want, (ops >> np.uint64(3)).astype(np.int64), m)
            else:
                np.bitwise_and.at(want, (ops >> np.uint64(3)).astype(np.int64), ~m)
            assert np.array_equal(np.frombuffer(eng.get(b"skew"), np.uint8), want)
        assert eng.bitcount(b"skew") == int(np.bitwise_count(want).sum(dtype=np.uint64))
    finally:
        eng.close()


def test_async_pfadd_and_read_stream(engine, O):
    """Async mode: PFADD batches (one overflowing the in-LDS conflict replay)
    interleaved with Bloom contains on the read stream and Bloom adds; the
    deferred settle and the stream ordering give the sequential results."""
    nkeys = 30
    names = [b"as:%d" % i for i in range(nkeys)]
    ids = engine.hll_resolve(names)
    assert engine.bloom_try_init("as:bf", 50000, 0.01)
    size, k, _, _ = engine.bloom_config("as:bf")
    bits = O.BitString()
    rng = np.random.default_rng(21)
    batches, outs, keep = [], [], []
    ref_regs = np.zeros((nkeys, 16384), dtype=np.uint8)
    exists = np.zeros(nkeys, dtype=np.uint8)
    engine.set_async(True)
    try:
        for b, n in enumerate([20000, 300000, 5000]):
            off, buf = gen_jackson_longs(0x5EED0100 + b, n)
            kid = rng.integers(0, nkeys, n).astype(np.uint32)
            d = [engine.to_device(ids[kid]), engine.to_device(off), engine.to_device(buf, pad=16), engine.alloc(n)]
            engine.pfadd_dev(n, d[0], d[1], d[2], int(off[-1]), d[3])
            # Bloom: add on the main stream, contains on the read stream
            eoff, ebuf = gen_jackson_longs(0x5EED0200 + b, 4000)
            e = [engine.to_device(eoff), engine.to_device(ebuf, pad=16), engine.alloc(4000), engine.alloc(4000)]
            engine.bloom_add_dev("as:bf", 4000, e[0], e[1], int(eoff[-1]), e[2])
            engine.bloom_contains_dev("as:bf", 4000, e[0], e[1], int(eoff[-1]), e[3])
            batches.append((kid, off, buf, n, eoff, ebuf))
            keep.append((d, e))
        engine.sync()
    finally:
        engine.set_async(False)
    for (kid, off, buf, n, eoff, ebuf), (d, e) in zip(batches, keep):
        counts = np.ones(n, dtype=np.uint32)
        want = np.zeros(n, dtype=np.uint8)
        O.lib().or_pfadd_batch(ref_regs.ctypes.data, exists.ctypes.data, n, kid.ctypes.data, counts.ctypes.data,
                               off.ctypes.data, buf.ctypes.data, 3, want.ctypes.data)
        assert np.array_equal(d[3].download(np.uint8, n), want)
        els = [ebuf[eoff[i]:eoff[i + 1]].tobytes() for i in range(4000)]
        assert list(e[2].download(np.uint8, 4000).astype(bool)) == bits.bloom_add(size, k, els)
        assert list(e[3].download(np.uint8, 4000).astype(bool)) == bits.bloom_contains(size, k, els)
    for i, nm in enumerate(names):
        np.testing.assert_array_equal(engine.hll_registers(nm), ref_regs[i])
    assert engine.get("as:bf") == bits.bytes()


def test_redis5_semantics(O):
    """redis_major=5: HLL_Q sentinel in hllPatLen and the Ertl estimator."""
    from redisson_amd import SketchEngine
    e5 = SketchEngine(device=0, redis_major=5)
    try:
        ref = O.HLLStore(5)
        keys = [b"v5:%d" % i for i in range(6)]
        for i, k in enumerate(keys):
            m = [10, 1000, 20000, 100000, 3, 0][i]
            els = _elems(4000 + i, m)
            if els:
                e5.pfadd([k] * m, [[x] for x in els])
                ref.pfadd([k] * m, [[x] for x in els])
        live = [k for k in keys if k in ref.regs]
        for k in live:
            np.testing.assert_array_equal(e5.hll_registers(k), ref.regs[k])
        assert e5.pfcount([[k] for k in live]) == [ref.count([k]) for k in live]
        assert e5.pfcount([live]) == [ref.count(live)]
    finally:
        e5.close()


def test_edge_cases(engine, O):
    # empty batches are no-ops
    assert engine.pfadd([], []) == []
    assert engine.getbit([], []) == []
    assert engine.pfcount([]) == []
    # zero-length elements and very long elements (global-reader path, farmUo > 64)
    rng = np.random.default_rng(1)
    els = [b"", b"x", bytes(64), bytes(65), rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()] * 3
    keys = [b"edge:%d" % (i % 2) for i in range(len(els))]
    ref = O.HLLStore()
    assert engine.pfadd(keys, [[e] for e in els]) == ref.pfadd(keys, [[e] for e in els])
    for k in set(keys):
        np.testing.assert_array_equal(engine.hll_registers(k), ref.regs[k])
    assert engine.bloom_try_init("edge:bf", 1000, 0.01)
    size, k, _, _ = engine.bloom_config("edge:bf")
    bits = O.BitString()
    assert engine.bloom_add("edge:bf", size, k, els) == bits.bloom_add(size, k, els)
    assert engine.bloom_contains("edge:bf", size, k, els[::-1]) == bits.bloom_contains(size, k, els[::-1])
    # PFCOUNT of a missing key, union with only missing keys
    assert engine.pfcount([[b"edge:none"], [b"edge:none", b"edge:none2"]]) == [0, 0]
    # DEL returns the count and frees slabs for reuse (zeroed)
    assert engine.delete([b"edge:0", b"edge:0", b"edge:none"]) == 1
    assert engine.pfadd([b"edge:new"], [[b"a"]]) == [True]
    assert engine.pfcount([[b"edge:new"]]) == [1]
    # STRLEN of an HLL is its dense size; GET of a missing key is None
    assert engine.strlen(b"edge:new") == 12304
    assert engine.get(b"edge:none") is None


@pytest.mark.parametrize("direct,pipe", [("1", "0"), ("0", "0"), ("1", "1")])
def test_pfadd_paths_agree(O, direct, pipe):
    """The partition path (replies stored by k_pfp_apply, or restored by k_pfp_reply) on the packed 6-bit arena gives
    the oracle's registers and replies, dense and sparse, with intra-batch collisions (neighbouring registers of one
    word rising in one batch: the packed writes are XORs on shared words) and an oversized partition bucket.  (The
    claim / commit and sorted paths of rounds 1-5 were retired with the u8 arena.)"""
    import os
    from redisson_amd import SketchEngine
    env = {"SK_PFP_DIRECT": direct, "SK_PFP_PIPE": pipe}   # pipe: device batches hashed on a second stream
    os.environ.update(env)
    try:
        e = SketchEngine(device=0)
    finally:
        for v in env:
            del os.environ[v]
    try:
        for nkeys, n, dup in [(300, 40000, 0.2), (3, 60000, 0.1), (1, 3000, 0.0)]:
            rng = np.random.default_rng(nkeys)
            els = _elems(0x5EED0300 + nkeys, n)
            els += [els[i] for i in rng.integers(0, n, int(n * dup))]
            names = [b"pp:%d:%d" % (nkeys, i) for i in range(nkeys)]
            ids = e.hll_resolve(names)
            kid = rng.integers(0, nkeys, len(els)).astype(np.uint32)
            off, buf = O.pack(els)
            d = [e.to_device(ids[kid]), e.to_device(off), e.to_device(buf, pad=16), e.alloc(len(els))]
            e.pfadd_dev(len(els), d[0], d[1], d[2], int(off[-1]), d[3])
            regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
            assert np.array_equal(d[3].download(np.uint8, len(els)), want)
            for i, nm in enumerate(names):
                np.testing.assert_array_equal(e.hll_registers(nm), regs[i])
            # host path with multi-element commands through the same path
            keys = [names[i % nkeys] for i in range(500)]
            el2 = [[bytes([j % 256, i % 256]) * (j % 7) for j in range(i % 5)] for i in range(500)]
            ref = O.HLLStore()
            ref.regs = {nm: e.hll_registers(nm).copy() for nm in names}
            assert e.pfadd(keys, el2) == ref.pfadd(keys, el2)
            for nm in names:
                np.testing.assert_array_equal(e.hll_registers(nm), ref.regs[nm])
        # one register hit by 5000 copies of one element: oversized partition bucket -> host sort
        same = [b"same-element"] * 5000
        off, buf = O.pack(same)
        ids = e.hll_resolve([b"pp:same"])
        d = [e.to_device(np.repeat(ids, 5000)), e.to_device(off), e.to_device(buf, pad=16), e.alloc(5000)]
        e.pfadd_dev(5000, d[0], d[1], d[2], int(off[-1]), d[3])
        r = d[3].download(np.uint8, 5000)
        assert r[0] == 1 and not r[1:].any()
    finally:
        e.close()


def _pfp_bucket(slots):
    """k_pfp_hash's bucket of a register slot (sk_kernels.hip pfp_bucket)."""
    with np.errstate(over="ignore"):
        return (np.asarray(slots, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(55)


def test_pfadd_partition_oversized_buckets(engine, O):
    """Buckets far past the apply pass's LDS capacity, with more distinct
    (slot, rho) pairs than k_pfp_big's LDS table (its global table), plus one
    hot register hit thousands of times: replies and registers still exact."""
    nkeys = 1000
    names = [b"ob:%d" % i for i in range(nkeys)]
    ids = engine.hll_resolve(names)
    pool = _elems(0x5EED0400, 120000)
    by_reg = {}
    for e in pool:
        by_reg.setdefault(O.hll_patlen(e)[0], []).append(e)
    rng = np.random.default_rng(44)
    kids, els = [], []
    for target in (5, 300):
        kk, rr = np.meshgrid(np.arange(nkeys, dtype=np.uint64), np.arange(16384, dtype=np.uint64), indexing="ij")
        slots = ((ids[kk.astype(np.int64)] & 0xFFFFFF).astype(np.uint64) << np.uint64(14)) | rr
        hit = np.argwhere(_pfp_bucket(slots) == target)
        for ki, r in hit:
            cand = by_reg.get(int(r), [])
            for e in cand[: int(rng.integers(1, 5))]:
                for _ in range(int(rng.integers(1, 3))):
                    kids.append(ki)
                    els.append(e)
    hot = pool[7]
    kids += [3] * 6000
    els += [hot] * 6000
    perm = rng.permutation(len(els))
    kid = np.asarray(kids, dtype=np.uint32)[perm]
    els = [els[i] for i in perm]
    assert len(els) < (1 << 20)
    off, buf = O.pack(els)
    d = [engine.to_device(ids[kid]), engine.to_device(off), engine.to_device(buf, pad=16), engine.alloc(len(els))]
    engine.pfadd_dev(len(els), d[0], d[1], d[2], int(off[-1]), d[3])
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    assert np.array_equal(d[3].download(np.uint8, len(els)), want)
    for i, nm in enumerate(names):
        np.testing.assert_array_equal(engine.hll_registers(nm), regs[i])


@pytest.mark.parametrize("sched", ["0", "1", "3"])
def test_bloom_contains_kernels_agree(O, sched):
    """Every Bloom contains schedule (one element per thread, probe queue, split hash/probe passes) gives the oracle's replies, for k = 1 (Q2: always true), small
    and large k, ragged and empty elements, batch sizes off the tile size."""
    import os
    from redisson_amd import SketchEngine
    os.environ["SK_BLOOM_SCHED"] = sched
    try:
        e = SketchEngine(device=0)
    finally:
        del os.environ["SK_BLOOM_SCHED"]
    try:
        rng = np.random.default_rng(int(sched) + 90)
        for n_exp, p, n_add, n_probe in [(5000, 0.5, 3000, 777), (20000, 0.01, 15000, 5001),
                                         (3000, 1e-6, 2000, 3333), (100, 0.03, 60, 1)]:
            name = "bq:%s:%d" % (sched, n_exp)
            assert e.bloom_try_init(name, n_exp, p)
            size, k, _, _ = e.bloom_config(name)
            bits = O.BitString()
            added = _elems(0x5EED0500 + n_exp, n_add)
            assert e.bloom_add(name, size, k, added) == bits.bloom_add(size, k, added)
            probe = [added[i] for i in rng.integers(0, n_add, n_probe // 2)] + _ragged(rng, n_probe - n_probe // 2)
            assert e.bloom_contains(name, size, k, probe) == bits.bloom_contains(size, k, probe)
            off, buf = O.pack(probe)
            d = [e.to_device(off), e.to_device(buf, pad=16), e.alloc(len(probe))]
            e.bloom_contains_dev(name, len(probe), d[0], d[1], int(off[-1]), d[2])
            assert list(d[2].download(np.uint8, len(probe)).astype(bool)) == bits.bloom_contains(size, k, probe)
    finally:
        e.close()


def test_set_bit_range(engine, O):
    """RBitSet.set(from, to) / clear(from, to): one range-fill kernel gives the
    string the reference's per-bit SETBIT_VOID batch gives (growth included),
    and out-of-range offsets fail after the in-range bits are applied."""
    rng = np.random.default_rng(12)
    ref = O.BitString()
    key = b"rng:bits"
    cases = [(3, 10, 1), (0, 8, 1), (5, 6, 0), (7, 9, 0), (100, 1000, 1), (120, 900, 0), (127, 129, 1),
             (1000, 1000, 1), (2000, 1999, 1), (4096 * 8 - 3, 4096 * 8 + 133, 1), (17, 4096 * 8 + 5, 0)]
    cases += [(int(a), int(a + rng.integers(1, 3000)), int(rng.integers(0, 2))) for a in rng.integers(0, 40000, 40)]
    for frm, to, v in cases:
        engine.set_bit_range(key, frm, to, v)
        for i in range(frm, to):
            ref.setbit(i, v)
        assert engine.get(key) == ref.bytes(), (frm, to, v)
    # clear on a missing key grows it with zero bytes, like SETBIT x 0
    engine.set_bit_range(b"rng:empty", 0, 20, 0)
    assert engine.get(b"rng:empty") == bytes(3)
    # out of range: the valid part is applied, then the offset error
    lim = 1 << 32
    with pytest.raises(RedisException, match="bit offset"):
        engine.set_bit_range(b"rng:neg", -5, 4, 1)
    assert engine.get(b"rng:neg") == bytes([0xF0])
    with pytest.raises(RedisException, match="bit offset"):
        engine.set_bit_range(b"rng:big", lim - 2, lim + 3, 1)
    assert engine.strlen(b"rng:big") == lim // 8
    assert engine.getbit([b"rng:big"] * 3, [lim - 3, lim - 2, lim - 1]) == [0, 1, 1]
    engine.delete([b"rng:big"])


def test_completion_tickets(engine, O):
    """Async submission + tickets: PFADD on the main stream and Bloom contains on
    the read stream complete under one ticket; poll never blocks; results exact."""
    import time
    n, nkeys = 200000, 64
    off, buf = gen_jackson_longs(0x5EED0700, n)
    rng = np.random.default_rng(70)
    kid = rng.integers(0, nkeys, n).astype(np.uint32)
    names = [b"tk:%d" % i for i in range(nkeys)]
    ids = engine.hll_resolve(names)
    assert engine.bloom_try_init("tk:bf", 100000, 0.01)
    size, k, _, _ = engine.bloom_config("tk:bf")
    els = _elems(0x5EED0701, 5000)
    bits = O.BitString()
    want_add = bits.bloom_add(size, k, els[:3000])
    want_has = bits.bloom_contains(size, k, els)
    eo, eb = O.pack(els)
    d = [engine.to_device(ids[kid]), engine.to_device(off), engine.to_device(buf, pad=16), engine.alloc(n),
         engine.to_device(eo), engine.to_device(eb, pad=16), engine.alloc(5000), engine.alloc(5000)]
    a_off = engine.to_device(eo[:3001])
    engine.set_async(True)
    try:
        engine.bloom_add_dev("tk:bf", 3000, a_off, d[5], int(eo[3000]), d[6])
        engine.pfadd_dev(n, d[0], d[1], d[2], int(off[-1]), d[3])
        engine.bloom_contains_dev("tk:bf", 5000, d[4], d[5], int(eo[-1]), d[7])
        t = engine.ticket()
        t0 = time.time()
        while not engine.poll(t):
            assert time.time() - t0 < 30, "ticket never completed"
            time.sleep(0.0005)
        with pytest.raises(RedisException, match="unknown ticket"):
            engine.poll(t)                      # released once seen done
        engine.wait(engine.ticket())            # nothing new: completes at once
    finally:
        engine.set_async(False)
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    assert np.array_equal(d[3].download(np.uint8, n), want)
    for i, nm in enumerate(names):
        np.testing.assert_array_equal(engine.hll_registers(nm), regs[i])
    assert list(d[6].download(np.uint8, 3000).astype(bool)) == want_add
    assert list(d[7].download(np.uint8, 5000).astype(bool)) == want_has


@pytest.mark.parametrize("encoding", ["dense", "sparse"])
def test_hll_string_restore(engine, O, encoding):
    """A Redis HLL string SET on a key (a redis-server dump, sparse or dense)
    becomes an HLL on the first HLL command, with the registers it encodes;
    PFCOUNT / PFADD / PFMERGE continue from them exactly."""
    rng = np.random.default_rng(31 if encoding == "dense" else 32)
    regs = np.zeros(16384, dtype=np.uint8)
    hit = rng.integers(0, 16384, 900)
    regs[hit] = rng.integers(1, 33, 900)
    if encoding == "dense":
        regs[[3, 4]] = [45, 50]                       # dense only: values above the sparse limit
    key = b"restore:" + encoding.encode()
    engine.set(key, O.hll_string(regs, encoding, card=12345))
    assert engine.pfcount([[key]]) == [O.count_regs(regs, 1)]
    np.testing.assert_array_equal(engine.hll_registers(key), regs)
    els = _elems(0x5EED0800, 3000)
    ref = O.HLLStore()
    ref.regs[key] = regs.copy()
    assert engine.pfadd([key] * len(els), [[e] for e in els]) == ref.pfadd([key] * len(els), [[e] for e in els])
    np.testing.assert_array_equal(engine.hll_registers(key), ref.regs[key])
    # GET gives the dense form back; it decodes to the same registers
    np.testing.assert_array_equal(O.hll_decode(engine.get(key)), ref.regs[key])


def test_hll_string_invalid(engine, O):
    engine.set(b"notahll", b"hello world, not an HLL")
    with pytest.raises(RedisException, match="not a valid HyperLogLog"):
        engine.pfadd([b"notahll"], [[b"x"]])
    assert engine.get(b"notahll") == b"hello world, not an HLL"      # untouched
    regs = np.zeros(16384, dtype=np.uint8)
    regs[100] = 5
    bad = O.hll_string(regs, "sparse")[:-1]            # the last opcode cut: registers do not add up to 16384
    engine.set(b"corrupt", bad)
    with pytest.raises(RedisException, match="INVALIDOBJ"):
        engine.pfcount([[b"corrupt"]])
    dense_short = O.hll_string(regs, "dense")[:-1]
    engine.set(b"shortdense", dense_short)
    with pytest.raises(RedisException, match="not a valid HyperLogLog"):
        engine.pfmerge(b"m", [b"shortdense"])


def test_pfadd_multi_launch_zipf(engine, O):
    """A 1.5 M-element device batch (two partition launches, the second seeing
    the first's registers) over Zipf(1.1)-skewed tenants (SURVEY 8d C2 variant):
    replies and registers exact."""
    n, nkeys = 1_500_000, 2000
    off, buf = gen_jackson_longs(0x5EED0900, n)
    rng = np.random.default_rng(90)
    kid = (np.minimum(rng.zipf(1.1, n), nkeys) - 1).astype(np.uint32)
    names = [b"zipf:%d" % i for i in range(nkeys)]
    ids = engine.hll_resolve(names)
    d = [engine.to_device(ids[kid]), engine.to_device(off), engine.to_device(buf, pad=16), engine.alloc(n)]
    engine.pfadd_dev(n, d[0], d[1], d[2], int(off[-1]), d[3])
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    assert np.array_equal(d[3].download(np.uint8, n), want)
    for i in np.unique(kid)[:200]:
        np.testing.assert_array_equal(engine.hll_registers(names[i]), regs[i])
    hot = int(np.bincount(kid).argmax())
    np.testing.assert_array_equal(engine.hll_registers(names[hot]), regs[hot])


def test_pfadd_ids_matches_names_and_oracle(O):
    """sk_pfadd_ids (slab ids from sk_hll_resolve, host buffers) gives the oracle's replies and registers, for
    one-element commands (the shipped-as-is chunk), multi-element and empty commands (the re-packed chunk) and a
    batch split into several device batches (max_batch); an id never handed out fails with SK_ESTALE."""
    from redisson_amd import SketchEngine
    from redisson_amd.engine import RedisException
    e = SketchEngine(device=0, max_batch=3000)
    try:
        rng = np.random.default_rng(404)
        names = [b"ids:%d" % i for i in range(37)]
        ref = O.HLLStore()
        ref.pfadd(names, [[] for _ in names])          # created by the resolve below
        ids = e.hll_resolve(names)
        els = _elems(0x5EED0404, 12000)
        # one element per command, 8000 commands in 3 device batches
        kid = rng.integers(0, len(names), 8000)
        cmds = [[els[i]] for i in range(8000)]
        assert e.pfadd_ids(ids[kid], cmds) == ref.pfadd([names[k] for k in kid], cmds)
        # ragged commands (0..5 elements), repeats of earlier elements
        kid2 = rng.integers(0, len(names), 1500)
        cmds2 = [[els[int(j)] for j in rng.integers(0, 12000, int(rng.integers(0, 6)))] for _ in kid2]
        assert e.pfadd_ids(ids[kid2], cmds2) == ref.pfadd([names[k] for k in kid2], cmds2)
        for i, nm in enumerate(names):
            np.testing.assert_array_equal(e.hll_registers(nm), ref.regs[nm])
        # the name path over the same store agrees
        cmds3 = [[x] for x in _elems(0x5EED0405, 4000)]
        kid3 = rng.integers(0, len(names), 4000)
        assert e.pfadd([names[k] for k in kid3], cmds3) == ref.pfadd([names[k] for k in kid3], cmds3)
        with pytest.raises(RedisException, match="not held by a key"):
            e.pfadd_ids(np.array([1 << 20], dtype=np.uint32), [[b"x"]])
    finally:
        e.close()


def test_pfadd_names_large_batch_parallel_lookup(engine, O):
    """A name batch >= 64k commands takes the parallel directory lookup: keys that exist, keys created in the
    middle of the batch (reply 1 only for the first command on them) and repeats give the oracle's replies."""
    rng = np.random.default_rng(405)
    names = [b"big:%d" % i for i in range(3000)]
    ref = O.HLLStore()
    old = names[:1500]
    e0 = _elems(0x5EED0406, 1500)
    assert engine.pfadd(old, [[x] for x in e0]) == ref.pfadd(old, [[x] for x in e0])
    n = 100_000
    kid = rng.integers(0, len(names), n)
    els = _elems(0x5EED0407, n)
    keys = [names[k] for k in kid]
    assert engine.pfadd(keys, [[x] for x in els]) == ref.pfadd(keys, [[x] for x in els])
    for nm in names[::97]:
        np.testing.assert_array_equal(engine.hll_registers(nm), ref.regs[nm])


def test_pfcount_ids_many_keys(O):
    """sk_pfcount_ids over 40k slab ids (threaded estimates): empty keys, keys of 1..600 elements, and two keys
    holding registers >= 40 (the register-order sum, run after the threaded pass) give the oracle's counts; the
    name path (sk_pfcount) agrees; an id never handed out fails."""
    from redisson_amd import SketchEngine
    from redisson_amd.engine import RedisException
    e = SketchEngine(device=0)
    try:
        rng = np.random.default_rng(406)
        nk = 40_000
        names = [b"cnt:%d" % i for i in range(nk)]
        ids = e.hll_resolve(names)
        per = rng.integers(0, 600, nk)
        per[: nk // 4] = 0
        kid = np.repeat(np.arange(nk), per)
        rng.shuffle(kid)
        off, buf = O.pack(_elems(0x5EED0409, len(kid)))
        d = [e.to_device(ids[kid].astype(np.uint32)), e.to_device(off), e.to_device(buf, pad=16), e.alloc(len(kid))]
        e.pfadd_dev(len(kid), d[0], d[1], d[2], int(off[-1]), d[3])
        regs, _ = O.HLLStore().pfadd_bulk(kid, off, buf, nk)
        big = np.zeros(16384, dtype=np.uint8)
        big[:] = rng.integers(0, 12, 16384)
        big[[5, 77, 9000]] = [40, 45, 50]
        for j in (7, nk - 3):
            e.hll_merge_registers_dev(names[j], e.to_device(big))
            regs[j] = np.maximum(regs[j], big)
        want = [O.count_regs(regs[i], 1) for i in range(nk)]
        assert list(e.pfcount_ids(ids)) == want
        sub = rng.integers(0, nk, 3000)
        assert e.pfcount([[names[i]] for i in sub]) == [want[i] for i in sub]
        # >= 64k keys by name (the parallel directory pass): singles twice, missing keys, 3-key unions
        pairs = rng.integers(0, nk, (200, 2))
        cmds = [[nm] for nm in names] * 2 + [[b"absent:1"]] + \
               [[names[a], names[b], b"absent:%d" % a] for a, b in pairs]
        exp = want * 2 + [0] + [O.count_regs(np.maximum(regs[a], regs[b]), 2) for a, b in pairs]
        assert e.pfcount(cmds) == exp
        with pytest.raises(RedisException, match="not held by a key"):
            e.pfcount_ids(np.array([1 << 22], dtype=np.uint32))
    finally:
        e.close()


def test_pfadd_mixed_batch_wrongtype_skips_one_command(engine, O):
    """A PFADD batch with a command on a bit string fails that command alone (pipeline semantics): the other
    commands (one element each, and a multi-element one) still update their registers exactly."""
    engine.setbit([b"mx:str"], [5], [1])
    els = _elems(0x5EED0410, 3000)
    keys = [b"mx:%d" % (i % 7) for i in range(3000)]
    keys[1234] = b"mx:str"
    cmds = [[x] for x in els]
    cmds[10] = els[:50]
    with pytest.raises(RedisException, match="HyperLogLog"):
        engine.pfadd(keys, cmds)
    ref = O.HLLStore()
    keep = [i for i in range(3000) if i != 1234]
    ref.pfadd([keys[i] for i in keep], [cmds[i] for i in keep])
    for k in set(keys) - {b"mx:str"}:
        np.testing.assert_array_equal(engine.hll_registers(k), ref.regs[k])


def test_stale_slab_id_rejected(O):
    """a cached slab handle whose key was deleted (or replaced by SET, or flushed) is rejected with
    SK_ESTALE and writes nothing, even after another key reuses the slab (the handle's generation byte differs);
    resolving the name again works."""
    from redisson_amd import SketchEngine
    from redisson_amd.engine import RedisException
    e = SketchEngine(device=0)
    try:
        [old] = e.hll_resolve([b"st:a"])
        assert e.pfadd_ids(np.array([old], np.uint32), [[b"x1"]]) == [1]
        assert e.delete([b"st:a"]) == 1
        [new] = e.hll_resolve([b"st:b"])          # the freed slab is handed out again, one generation on
        assert new & 0xFFFFFF == old & 0xFFFFFF and new != old
        before = e.hll_registers(b"st:b").copy()
        assert not before.any()
        with pytest.raises(RedisException, match="not held by a key"):
            e.pfadd_ids(np.array([old], np.uint32), [[b"x2"]])
        with pytest.raises(RedisException, match="not held by a key"):
            e.pfcount_ids(np.array([old], np.uint32))
        np.testing.assert_array_equal(e.hll_registers(b"st:b"), before)
        # the id is live again through its new owner
        assert e.pfadd_ids(np.array([new], np.uint32), [[b"x3"]]) == [1]
        ref = O.HLLStore()
        ref.pfadd([b"st:b"], [[b"x3"]])
        np.testing.assert_array_equal(e.hll_registers(b"st:b"), ref.regs[b"st:b"])
        # SET over the HLL and FLUSHALL free the slab too
        e.set(b"st:b", b"plain")
        with pytest.raises(RedisException, match="not held by a key"):
            e.pfadd_ids(np.array([new], np.uint32), [[b"x4"]])
        [c] = e.hll_resolve([b"st:c"])
        e.flushall()
        with pytest.raises(RedisException, match="not held by a key"):
            e.pfcount_ids(np.array([c], np.uint32))
    finally:
        e.close()


_LONG_FALLBACK = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
from redisson_amd import SketchEngine
e = SketchEngine(device=0)
ref = O.HLLStore()
rng = np.random.default_rng(5)
elems = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
         for n in (3_000_003, 37, 1_048_583, 65_536, 2_500_000, 5)]
keys = [b"lf:%d" % (i % 2) for i in range(len(elems))]
assert e.pfadd(keys, [[x] for x in elems]) == ref.pfadd(keys, [[x] for x in elems])
for k in set(keys):
    np.testing.assert_array_equal(e.hll_registers(k), ref.regs[k])
n_fb, _ = e.prof_read("pfadd_long_fallback")
e.close()
print("fallbacks", n_fb)
"""


def test_pfadd_long_elements_lookback_fallback():
    """a look-back wait of the bit-round scan that runs out (a delayed predecessor workgroup, e.g. on a
    GPU shared by two processes) must not fail the PFADD.  A child process forces a zero wait bound
    (SK_MS_SPIN_DEV=0): the long elements are then re-hashed per thread, and replies and registers still equal the
    oracle's."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SK_MS_SPIN_DEV="0")
    r = subprocess.run([sys.executable, "-c", _LONG_FALLBACK, root], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    n_fb = int(r.stdout.split("fallbacks")[1])
    assert n_fb >= 1, r.stdout   # the zero bound made some workgroup give up waiting


def test_pfadd_long_elements_workgroup_hash(O):
    """C1's addAll (quirk Q1: ONE element = the Jackson array of 1M Longs, ~40 MB) and a batch mixing elements
    of 64 KiB .. 3 MB with short ones: elements >= 64 KiB are hashed by the bit-round scan (k_ms_planes +
    k_ms_rounds: 256 KiB per workgroup, a look-back across workgroups), so the cases straddle workgroup boundaries
    and every tail length; replies and registers equal the oracle's."""
    import time

    from redisson_amd import JLong, JsonJacksonCodec, SketchEngine
    e = SketchEngine(device=0)
    try:
        vals = np.random.default_rng(1).integers(-(1 << 63), (1 << 63) - 1, 1 << 20, dtype=np.int64)
        blob = JsonJacksonCodec().encode(["hll:c1q"] + [JLong(int(v)) for v in vals])
        assert len(blob) > 30_000_000
        ref = O.HLLStore()
        e.pfadd([b"hll:c1q"], [[blob[:100]]])              # warm the path
        ref.pfadd([b"hll:c1q"], [[blob[:100]]])
        e.prof_reset()
        e.prof_enable(True)
        t0 = time.perf_counter()
        got = e.pfadd([b"hll:c1q"], [[blob]])
        dt = time.perf_counter() - t0
        e.prof_enable(False)
        n_l, ms_l = e.prof_read("pfadd_long")
        assert n_l == 1 and ms_l < 10.0, (n_l, ms_l)        # the bit-round hash: ~0.3 ms for the 41 MB element
        assert got == ref.pfadd([b"hll:c1q"], [[blob]])
        np.testing.assert_array_equal(e.hll_registers(b"hll:c1q"), ref.regs[b"hll:c1q"])
        assert e.pfcount([[b"hll:c1q"]]) == [ref.count([b"hll:c1q"])]
        assert dt < 1.0, dt                                  # host-timed, H2D of 40 MB included
        rng = np.random.default_rng(3)
        elems = []
        for i in range(40):
            n = int(rng.choice([5, 37, 65536, 65537, 200_001, 262_144, 262_136, 524_288 + 8, 3_000_003])) + i % 8
            elems.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        keys = [b"long:%d" % (i % 3) for i in range(40)]
        assert e.pfadd(keys, [[x] for x in elems]) == ref.pfadd(keys, [[x] for x in elems])
        for k in set(keys):
            np.testing.assert_array_equal(e.hll_registers(k), ref.regs[k])
    finally:
        e.close()


def test_stale_handle_after_generation_wrap(engine):
    """A slab whose 8-bit generation would wrap is retired instead of reused: a handle cached before
    300 delete / re-create cycles of its key is still refused with SK_ESTALE, and no cycle reuses its slab."""
    from redisson_amd.engine import RedisException

    k = b"wrap:key"
    h0 = engine.hll_resolve([k])[0]
    seen = set()
    for _ in range(300):
        engine.delete([k])
        h = int(engine.hll_resolve([k])[0])
        seen.add(h)
        with pytest.raises(RedisException, match="not held by a key"):
            engine.pfadd_ids(np.array([h0], dtype=np.uint32), [[b"e"]])
    assert int(h0) not in seen
    engine.delete([k])


def test_hll_sum_kernel_exact(engine, O):
    """k_hll_sum (the PFCOUNT path under redis 3.x): per-key S = sum 2^(40-r), zero count and the register >= 40
    flag against numpy on keys with every register value 0..63; PFCOUNT of each key equals the oracle (the keys
    holding a register >= 40 take the register-order sum)."""
    rng = np.random.default_rng(77)
    names = [b"hsum:%d" % i for i in range(40)]
    ids = engine.hll_resolve(names)
    regs = []
    for i, nm in enumerate(names):
        top = 20 if i % 4 else 63                      # every 4th key reaches registers >= 40
        r = rng.integers(0, top + 1, 16384, dtype=np.uint8)
        r[rng.random(16384) < (i % 5) / 5] = 0
        d = engine.to_device(r)
        engine.hll_merge_registers_dev(nm, d)
        d.free()
        regs.append(r)
    d_ids, d_out = engine.to_device(ids), engine.alloc(16 * len(names))
    engine.hll_sum_dev(len(names), d_ids, d_out)
    got = d_out.download(np.uint64, 2 * len(names))
    for i, r in enumerate(regs):
        assert int(got[2 * i + 1]) & 0xffffffff == int((r == 0).sum())
        assert int(got[2 * i + 1]) >> 32 == int(r.max() >= 40)
        if r.max() < 40:
            assert int(got[2 * i]) == int(sum(1 << (40 - int(v)) for v in r))
    assert [int(x) for x in engine.pfcount_ids(ids)] == [O.count_regs(r, 1) for r in regs]
    d_ids.free(); d_out.free()


def test_prefix_form_ingress_matches_oracle(O):
    """Host ingress in prefix form (sk_pfadd_ids_prefix, sk_bloom_add_prefix, sk_bloom_contains_prefix: element =
    shared prefix + suffix, rebuilt on the device) gives the oracle's replies, registers and bit array: Jackson Longs
    split at their type header, an empty suffix, an empty prefix, a batch over several device batches (max_batch), a
    long element (the full-element fallback) and a stale handle."""
    from redisson_amd import SketchEngine
    from redisson_amd.engine import RedisException
    e = SketchEngine(device=0, max_batch=3000)
    try:
        rng = np.random.default_rng(505)
        names = [b"pfx:%d" % i for i in range(29)]
        ref = O.HLLStore()
        ref.pfadd(names, [[] for _ in names])
        ids = e.hll_resolve(names)
        els = _elems(0x5EED0505, 8000)
        pre = b'["java.lang.Long",'
        assert all(x.startswith(pre) for x in els)
        kid = rng.integers(0, len(names), 8000)
        got = e.pfadd_ids_prefix(ids[kid], pre, [x[len(pre):] for x in els])
        assert got == ref.pfadd([names[k] for k in kid], [[x] for x in els])
        # an empty suffix, an empty prefix, repeats
        odd = [pre, pre + b"1]", els[0]]
        kid2 = rng.integers(0, len(names), len(odd))
        assert e.pfadd_ids_prefix(ids[kid2], pre, [x[len(pre):] for x in odd]) == \
            ref.pfadd([names[k] for k in kid2], [[x] for x in odd])
        assert e.pfadd_ids_prefix(ids[kid2], b"", odd) == ref.pfadd([names[k] for k in kid2], [[x] for x in odd])
        # a long element (>= 64 KiB: the bit-round scan of the full-element path)
        big = b"[" + b",".join(b"%d" % i for i in range(20000)) + b"]"
        assert e.pfadd_ids_prefix(ids[:1], b"[0,1,2", [big[6:]]) == ref.pfadd(names[:1], [[big]])
        for nm in names:
            np.testing.assert_array_equal(e.hll_registers(nm), ref.regs[nm])
        with pytest.raises(RedisException, match="not held by a key"):
            e.pfadd_ids_prefix(np.array([1 << 20], dtype=np.uint32), pre, [b"1]"])
        # Bloom add / contains in prefix form
        assert e.bloom_try_init("pfx:bf", 50000, 0.01)
        size, k, _, _ = e.bloom_config("pfx:bf")
        bits = O.BitString()
        assert e.bloom_prefix("add", "pfx:bf", size, k, pre, [x[len(pre):] for x in els[:5000]]) == \
            bits.bloom_add(size, k, els[:5000])
        probe = els[2500:] + odd
        assert e.bloom_prefix("contains", "pfx:bf", size, k, b"", probe) == bits.bloom_contains(size, k, probe)
        assert e.bloom_prefix("contains", "pfx:bf", size, k, pre, [x[len(pre):] for x in els[2500:]]) == \
            bits.bloom_contains(size, k, els[2500:])
        assert e.get("pfx:bf") == bits.bytes()
    finally:
        e.close()
