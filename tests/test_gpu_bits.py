"""SETBIT / GETBIT by key name through the C ABI Java calls (sk_setbit / sk_getbit, M:RedissonBitSet.java:53-56,79-81,
202-228; RBatch runs, GpuSketchBatchService / SketchDispatch): every reply is the bit as batch order finds it, the
final strings equal the oracle's sequential SETBITs, and no library sort runs.

- replies, several keys, mixed values: the region partition with u64 records (k_sbv_part<u64> -> k_sbv_fine<u64> ->
  k_sbr_runs: each 32 KiB region's ops sorted by (bit, seq) in LDS);
- a region holding more ops than the LDS sort takes (a skewed batch): sorted in global memory by the same workgroup
  (LDS-sorted chunks + merge-path passes);
- SETBIT_VOID (no reply array) of one key and one value: the SETBIT_VOID kernels, the dense region path included.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits_ref(O, ops):
    """sequential oracle: {key: BitString}, replies"""
    ref, rep = {}, []
    for k, o, v in ops:
        rep.append(ref.setdefault(k, O.BitString()).setbit(int(o), int(v)))
    return ref, rep


def test_mixed_key_batch_with_replies_equals_oracle(engine, O):
    """An RBatch of SETBITs over 24 bitsets: sparse and dense keys, repeated bits with alternating values inside the
    batch (the replies depend on order), bits at region edges, a bad offset and a key of another type (each fails
    alone, reply 0, the call raises after applying the rest), then GETBITs of every key against the oracle."""
    from redisson_amd.engine import RedisException

    rng = np.random.default_rng(61)
    n = 300_000
    keys = [b"mb:%d" % k for k in rng.integers(0, 24, n)]
    width = {b"mb:%d" % k: (1 << (12 + (k % 12))) for k in range(24)}   # 4 Ki .. 8 Mi bits
    offs = np.array([rng.integers(0, width[k]) for k in keys], dtype=np.uint64)
    vals = rng.integers(0, 2, n).astype(np.uint8)
    hot = rng.integers(0, n, 40_000)                      # repeats of earlier ops' bits, any value
    src = rng.integers(0, n, len(hot))
    for h, s in zip(hot, src):
        keys[h], offs[h] = keys[s], offs[s]
    edge = rng.integers(0, n, 64)
    offs[edge[:32]] = (np.uint64(1) << np.uint64(18)) - np.uint64(1)   # last bit of region 0
    offs[edge[32:]] = np.uint64(1) << np.uint64(18)                    # first bit of region 1
    engine.pfadd([b"mb:hll"], [[b"x"]])
    keys[7] = b"mb:hll"                                   # WRONGTYPE
    offs[11] = np.uint64(1) << np.uint64(40)              # past max_bit_offset
    with pytest.raises(RedisException):
        engine.setbit(keys, offs, vals)
    good = [(k, o, v) for i, (k, o, v) in enumerate(zip(keys, offs, vals)) if i not in (7, 11)]
    ref, _ = _bits_ref(O, good)
    # the same batch without the two bad ops, on fresh keys: every reply
    keys2 = [k.replace(b"mb:", b"mc:") for k, _, _ in good]
    got = engine.setbit(keys2, [o for _, o, _ in good], [v for _, _, v in good])
    ref2, want = _bits_ref(O, [(k2, o, v) for k2, (_, o, v) in zip(keys2, good)])
    assert got == want
    for k, b in ref.items():
        assert engine.get(k) == b.bytes(), k
        assert engine.get(k.replace(b"mb:", b"mc:")) == b.bytes(), k
    q = rng.integers(0, 1 << 24, 50_000)
    qk = [b"mc:%d" % rng.integers(0, 26) for _ in q]     # mc:24, mc:25 missing -> 0
    assert engine.getbit(qk, q) == [ref2[k].getbit(int(o)) if k in ref2 else 0 for k, o in zip(qk, q)]
    one = rng.integers(0, 1 << 23, 20_000)               # one key: k_getbit_single
    assert engine.getbit([b"mc:11"] * len(one), one) == [ref2[b"mc:11"].getbit(int(o)) for o in one]


def test_skewed_region_sorted_in_global_memory(engine, O):
    """200 k ops with replies on one key, 60 % of them in one 32 KiB region and 5 % on a single bit with alternating
    values: that region holds ~50x the LDS sort's capacity (k_sbr_runs' merge-path passes); every reply and the
    final string equal the oracle's."""
    rng = np.random.default_rng(62)
    n = 200_000
    offs = rng.integers(0, 1 << 22, n).astype(np.uint64)
    hot = rng.random(n) < 0.6
    offs[hot] = (np.uint64(5) << np.uint64(18)) + rng.integers(0, 1 << 18, int(hot.sum())).astype(np.uint64)
    one = rng.random(n) < 0.05
    offs[one] = np.uint64((5 << 18) + 12345)
    vals = rng.integers(0, 2, n).astype(np.uint8)
    ref, want = _bits_ref(O, [(b"sk", o, v) for o, v in zip(offs, vals)])
    got = engine.setbit([b"sk"] * n, offs, vals)
    assert got == want
    assert engine.get(b"sk") == ref[b"sk"].bytes()


def test_setbit_void_by_name_takes_the_dense_kernels(engine):
    """SETBIT_VOID through sk_setbit (no reply array, one key, one value, host buffers): a dense 4 M-op batch on a
    2^27-bit string (the k_sbv_* region path) and a sparse one (per-op atomics) set exactly numpy's bits; a void batch
    of mixed values (order matters per bit) goes through the reply kernels and equals the sequential result."""
    rng = np.random.default_rng(63)
    nbits = 1 << 27
    offs = rng.integers(0, nbits, 4 << 20).astype(np.uint64)
    engine.setbit([b"v"] * len(offs), offs, np.ones(len(offs), np.uint8), want_old=False)
    want = np.zeros(nbits // 8, dtype=np.uint8)
    np.bitwise_or.at(want, (offs >> np.uint64(3)).astype(np.int64),
                     (np.uint8(1) << (np.uint8(7) - (offs & np.uint64(7)).astype(np.uint8))).astype(np.uint8))
    got = np.frombuffer(engine.get(b"v"), np.uint8)
    assert np.array_equal(got, want[:len(got)]) and len(got) == int(offs.max()) // 8 + 1
    sp = rng.integers(0, 1 << 30, 1000).astype(np.uint64)
    engine.setbit([b"vs"] * len(sp), sp, np.ones(len(sp), np.uint8), want_old=False)
    assert engine.bitcount(b"vs") == len(np.unique(sp))
    mo = rng.integers(0, 4096, 50_000).astype(np.uint64)
    mv = rng.integers(0, 2, len(mo)).astype(np.uint8)
    engine.setbit([b"vm"] * len(mo), mo, mv, want_old=False)
    last = {}
    for o, v in zip(mo, mv):
        last[int(o)] = int(v)
    assert engine.getbit([b"vm"] * 4096, list(range(4096))) == [last.get(i, 0) for i in range(4096)]


def test_device_setbit_with_values_and_replies(engine, O):
    """sk_setbit_values_dev / sk_setbit_dev with replies (the range-sharded RBitSet's owner apply) run the region
    kernels too: replies and bytes equal the oracle's."""
    rng = np.random.default_rng(64)
    n = 100_000
    offs = rng.integers(0, 1 << 21, n).astype(np.uint64)
    offs[n // 2:] = offs[:n // 2][rng.permutation(n // 2)]
    vals = rng.integers(0, 2, n).astype(np.uint8)
    ref, want = _bits_ref(O, [(b"dv", o, v) for o, v in zip(offs, vals)])
    out = engine.alloc(n)
    engine.setbit_values_dev(b"dv", n, engine.to_device(offs), engine.to_device(vals), out)
    assert out.download(np.uint8, n).tolist() == want
    assert engine.get(b"dv") == ref[b"dv"].bytes()
    ref1, want1 = _bits_ref(O, [(b"d1", o, 1) for o in offs])
    engine.setbit_dev(b"d1", n, engine.to_device(offs), 1, out)
    assert out.download(np.uint8, n).tolist() == want1
    assert engine.get(b"d1") == ref1[b"d1"].bytes()
