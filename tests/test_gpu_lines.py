"""GPU parity of the PFADD line schedule (k_pfl_*: group-committed RBatches applied sketch-major with the registers
in LDS) against the CPU oracle, bit-exact: replies of every command and every register.

The engine is opened with SK_PFL_MIN=1 and SK_PFL_RATIO=0 so that every device batch takes the line schedule,
whatever its size.
Cases: uniform tenants over several fine buckets and run tiles, registers carried over from an earlier batch,
one key receiving everything (fine buckets applied in chunks of runs), one element repeated past a chunk in one
run (the (slot, rho) -> min seq table), Zipf-skewed tenants, slab ids above the last fine bucket's start, and the
partition path and the line schedule agreeing on the same stream of batches."""
import os

import numpy as np
import pytest

from redisson_amd import gen_jackson_longs

pytestmark = pytest.mark.gpu


def _engine(pfl_min="1"):
    from redisson_amd import SketchEngine

    os.environ["SK_PFL_MIN"] = pfl_min
    os.environ["SK_PFL_RATIO"] = "0"   # every call of these tests takes the line schedule, whatever its size
    try:
        return SketchEngine(device=0, max_batch=1 << 23)
    finally:
        del os.environ["SK_PFL_MIN"]
        del os.environ["SK_PFL_RATIO"]


@pytest.fixture(scope="module")
def leng():
    e = _engine()
    yield e
    e.close()


def _run(e, O, names, kid, off, buf):
    """One device batch through the engine: its replies."""
    ids = e.hll_resolve(names)
    n = len(kid)
    d = [e.to_device(ids[kid].astype(np.uint32)), e.to_device(off), e.to_device(buf, pad=16), e.alloc(n)]
    e.pfadd_dev(n, d[0], d[1], d[2], int(off[-1]), d[3])
    got = d[3].download(np.uint8, n)
    for x in d:
        x.free()
    return got


def _oracle_from(O, regs0, kid, off, buf, nkeys):
    """The oracle's one-element PFADDs (or_pfadd_batch) continuing from registers regs0 (n_keys x 16384)."""
    from oracle import oracle as OO

    lib = OO.lib()
    regs = regs0.copy()
    exists = np.ones(nkeys, dtype=np.uint8)
    out = np.zeros(len(kid), dtype=np.uint8)
    counts = np.ones(len(kid), dtype=np.uint32)
    ids = np.ascontiguousarray(kid, dtype=np.uint32)
    lib.or_pfadd_batch(regs.ctypes.data, exists.ctypes.data, len(kid), ids.ctypes.data, counts.ctypes.data,
                       off.ctypes.data, buf.ctypes.data, 3, out.ctypes.data)
    return regs, out


def _check_regs(e, names, regs, which=None):
    for i in (range(len(names)) if which is None else which):
        np.testing.assert_array_equal(e.hll_registers(names[i]), regs[i], err_msg=names[i].decode())


def test_lines_uniform_two_batches(leng, O):
    """3000 tenants (6 fine buckets per coarse bucket, the last one partial), 2M + 1.5M elements with repeats:
    the second batch starts from the first batch's registers."""
    nkeys = 3000
    names = [b"ln:u:%d" % i for i in range(nkeys)]
    rng = np.random.default_rng(1)
    off, buf = gen_jackson_longs(0x5EED1001, 2_000_000)
    kid = rng.integers(0, nkeys, 2_000_000).astype(np.uint32)
    got = _run(leng, O, names, kid, off, buf)
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    assert np.array_equal(got, want)
    _check_regs(leng, names, regs)
    # second batch: half fresh elements, half repeats of the first batch's (replies 0 unless a new key)
    off2, buf2 = gen_jackson_longs(0x5EED1002, 750_000)
    els = [buf2[off2[i]:off2[i + 1]].tobytes() for i in range(750_000)]
    rep = rng.integers(0, 2_000_000, 750_000)
    els += [buf[off[i]:off[i + 1]].tobytes() for i in rep]
    kid2 = np.concatenate([rng.integers(0, nkeys, 750_000), kid[rep]]).astype(np.uint32)
    perm = rng.permutation(len(els))
    els = [els[i] for i in perm]
    kid2 = kid2[perm]
    o2, b2 = O.pack(els)
    got2 = _run(leng, O, names, kid2, o2, b2)
    regs2, want2 = _oracle_from(O, regs, kid2, o2, b2, nkeys)
    assert np.array_equal(got2, want2)
    _check_regs(leng, names, regs2)


def test_lines_single_key_chunks_and_big_run(leng, O):
    """C1-like: 3M elements into one key (each fine bucket applied in chunks of whole runs), then one element
    repeated 300k times among 100k others into another key (a run far past one chunk: the min-seq table)."""
    off, buf = gen_jackson_longs(0x5EED1003, 3_000_000)
    kid = np.zeros(3_000_000, dtype=np.uint32)
    got = _run(leng, O, [b"ln:c1"], kid, off, buf)
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, 1)
    assert np.array_equal(got, want)
    _check_regs(leng, [b"ln:c1"], regs)

    pool_off, pool_buf = gen_jackson_longs(0x5EED1004, 100_000)
    els = [pool_buf[pool_off[i]:pool_off[i + 1]].tobytes() for i in range(100_000)]
    els += [b"same-element"] * 300_000
    rng = np.random.default_rng(2)
    els = [els[i] for i in rng.permutation(len(els))]
    o2, b2 = O.pack(els)
    k2 = np.zeros(len(els), dtype=np.uint32)
    got2 = _run(leng, O, [b"ln:hot"], k2, o2, b2)
    regs2, want2 = O.HLLStore().pfadd_bulk(k2, o2, b2, 1)
    assert np.array_equal(got2, want2)
    _check_regs(leng, [b"ln:hot"], regs2)


def test_lines_zipf(leng, O):
    """Zipf(1.1) over 2000 tenants (SURVEY 8d C2 variant), 1.5M elements."""
    n, nkeys = 1_500_000, 2000
    off, buf = gen_jackson_longs(0x5EED1005, n)
    rng = np.random.default_rng(3)
    kid = (np.minimum(rng.zipf(1.1, n), nkeys) - 1).astype(np.uint32)
    names = [b"ln:z:%d" % i for i in range(nkeys)]
    got = _run(leng, O, names, kid, off, buf)
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    assert np.array_equal(got, want)
    hot = int(np.bincount(kid).argmax())
    _check_regs(leng, names, regs, sorted(set(np.unique(kid)[:300].tolist()) | {hot}))


def test_lines_ragged_and_small(leng, O):
    """Ragged element bytes (empty to 200 B), a batch below one hash block, and a batch whose tenants sit in
    one fine bucket of a store holding more slabs than the batch touches."""
    rng = np.random.default_rng(4)
    for n, nkeys in [(1000, 10), (70_000, 700)]:
        lens = rng.integers(0, 200, n)
        els = [rng.integers(0, 256, l, dtype=np.uint8).tobytes() for l in lens]
        off, buf = O.pack(els)
        names = [b"ln:r:%d:%d" % (n, i) for i in range(nkeys)]
        kid = rng.integers(0, nkeys, n).astype(np.uint32)
        got = _run(leng, O, names, kid, off, buf)
        regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
        assert np.array_equal(got, want)
        _check_regs(leng, names, regs)


def test_lines_agree_with_partition_path(O):
    """The same 4 batches of 1M through the partition path (one call per batch, the default below SK_PFL_MIN)
    and through the line schedule (one group-committed 4M call): identical replies and registers."""
    n, nkeys = 1 << 20, 5000
    names = [b"ln:a:%d" % i for i in range(nkeys)]
    rng = np.random.default_rng(5)
    off, buf = gen_jackson_longs(0x5EED1006, 4 * n)
    kid = rng.integers(0, nkeys, 4 * n).astype(np.uint32)
    res = []
    for mode in ("part", "line"):
        e = _engine("0" if mode == "part" else "1")
        try:
            ids = e.hll_resolve(names)
            d = [e.to_device(ids[kid]), e.to_device(off), e.to_device(buf, pad=16), e.alloc(4 * n)]
            if mode == "part":
                for h in range(4):
                    e.pfadd_dev(n, d[0].ptr + h * n * 4, d[1].ptr + h * n * 8, d[2], int(off[-1]), d[3].ptr + h * n)
            else:
                e.pfadd_dev(4 * n, d[0], d[1], d[2], int(off[-1]), d[3])
            regs = np.stack([e.hll_registers(nm) for nm in names])
            res.append((d[3].download(np.uint8, 4 * n), regs))
        finally:
            e.close()
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])
    regs, want = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    assert np.array_equal(res[1][0], want)
    assert np.array_equal(res[1][1], regs)


def test_lines_host_buffer_batches(leng, O):
    """Host-buffer PFADD (sk_pfadd by name, sk_pfadd_ids by slab id) of one-element commands goes through the line
    schedule too (SK_PFL_MIN=1 here): replies and registers equal the oracle's."""
    nkeys, n = 400, 60_000
    names = [b"ln:h:%d" % i for i in range(nkeys)]
    rng = np.random.default_rng(8)
    off, buf = gen_jackson_longs(0x5EED1008, 2 * n)
    els = [buf[off[i]:off[i + 1]].tobytes() for i in range(2 * n)]
    kid = rng.integers(0, nkeys, 2 * n).astype(np.uint32)
    ref = O.HLLStore()
    got = leng.pfadd([names[k] for k in kid[:n]], [[e] for e in els[:n]])
    assert got == ref.pfadd([names[k] for k in kid[:n]], [[e] for e in els[:n]])
    ids = leng.hll_resolve(names)
    got2 = leng.pfadd_ids(ids[kid[n:]], [[e] for e in els[n:]])
    assert got2 == ref.pfadd([names[k] for k in kid[n:]], [[e] for e in els[n:]])
    for nm in names:
        np.testing.assert_array_equal(leng.hll_registers(nm), ref.regs[nm])


def test_lines_reply_default_flips(leng, O):
    """The apply stores only replies that differ from the call's default (the previous call's majority reply):
    fresh elements (mostly 1s), the same elements again (all 0s), fresh again -- each call's replies equal the
    oracle's whichever default it ran with."""
    nkeys, n = 64, 400_000
    names = [b"ln:d:%d" % i for i in range(nkeys)]
    rng = np.random.default_rng(9)
    regs = np.zeros((nkeys, 16384), dtype=np.uint8)
    off, buf = gen_jackson_longs(0x5EED1009, n)
    kid = rng.integers(0, nkeys, n).astype(np.uint32)
    leng.hll_resolve(names)
    for seed, (o, b, k) in enumerate([(off, buf, kid), (off, buf, kid),
                                      (*gen_jackson_longs(0x5EED100A, n), kid[::-1].copy())]):
        got = _run(leng, O, names, k, o, b)
        regs, want = _oracle_from(O, regs, k, o, b, nkeys)
        assert np.array_equal(got, want), "call %d" % seed
        if seed == 1:
            assert not want.any()
    _check_regs(leng, names, regs)


def test_lines_dropped_ids_reply_zero_after_majority_one(leng, O):
    """a slab id the store never handed out is dropped by the region pass and replies 0, also when the
    call's default reply (the previous call's majority) is 1 -- the default fill runs before the region pass."""
    nkeys, n = 64, 400_000
    names = [b"ln:x:%d" % i for i in range(nkeys)]
    rng = np.random.default_rng(10)
    regs = np.zeros((nkeys, 16384), dtype=np.uint8)
    ids = leng.hll_resolve(names)
    for call, seed in enumerate((0x5EED100B, 0x5EED100C)):
        off, buf = gen_jackson_longs(seed, n)
        kid = rng.integers(0, nkeys, n).astype(np.uint32)
        dev_ids = ids[kid].astype(np.uint32)
        bad = np.zeros(n, dtype=bool)
        if call == 1:                                  # fresh elements again: the default is 1 from call 0
            bad[rng.choice(n, 5000, replace=False)] = True
            dev_ids[bad] = 0x00FFFFF0                  # a slab id far above every slab handed out
        d = [leng.to_device(dev_ids), leng.to_device(off), leng.to_device(buf, pad=16), leng.alloc(n)]
        leng.pfadd_dev(n, d[0], d[1], d[2], int(off[-1]), d[3])
        got = d[3].download(np.uint8, n)
        for x in d:
            x.free()
        keep = ~bad
        sub_off = np.concatenate([np.zeros(1, np.uint64), np.cumsum(np.diff(off)[keep], dtype=np.uint64)])
        sub_buf = np.concatenate([buf[off[i]:off[i + 1]] for i in np.flatnonzero(keep)] + [np.zeros(16, np.uint8)])
        regs, want = _oracle_from(O, regs, kid[keep], sub_off, sub_buf, nkeys)
        if call == 0:
            assert want.mean() > 0.5, "the first call must leave a majority of 1 replies"
        assert not got[bad].any(), "dropped ids must reply 0"
        assert np.array_equal(got[keep], want), "call %d" % call
    _check_regs(leng, names, regs)
