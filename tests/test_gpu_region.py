"""Bloom contains, region schedule (k_bloom_rc_hash + k_bloom_rc_probe) against the oracle.

Large contains batches take the region schedule (DESIGN.md "Bloom contains: region schedule"); these tests pin it
to the oracle's RBloomFilter.contains (M:RedissonBloomFilter.java:133-168, Q2: probes 0..k-2) for every k the
schedule takes (2..9), ragged batch sizes (partial hash blocks), filters whose string is shorter than m/8, and the
fallbacks (k > 9, small arrays) that must keep giving the same replies.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M = 1 << 20


def _engine(**kw):
    from redisson_amd import SketchEngine

    return SketchEngine(device=0, **kw)


def _p_for_k(k, n):
    """a false-positive probability whose tryInit(n, p) gives k hash functions"""
    from redisson_amd import bloom_optimal_bits, bloom_optimal_k

    for p in np.geomspace(0.5, 1e-6, 400):
        if bloom_optimal_k(n, bloom_optimal_bits(n, float(p))) == k:
            return float(p)
    raise AssertionError("no p for k=%d" % k)


def _contains_case(O, eng, name, n_exp, k, n_add, n_q, seed, rng):
    p = _p_for_k(k, n_exp)
    assert eng.bloom_try_init(name, n_exp, p)
    size, kk, _, _ = eng.bloom_config(name)
    assert kk == k
    if n_add:
        off, byt, tot = eng.gen_jackson_longs_dev(seed, n_add)
        d_out = eng.alloc(n_add)
        eng.bloom_add_dev(name, n_add, off, byt, tot, d_out)
        for x in (off, byt, d_out):
            x.free()
    bits, ln = O.bloom_add_gen(size, k, seed, 0, n_add)
    got = eng.get(name) or b""
    assert len(got) == ln
    assert np.array_equal(np.frombuffer(got, np.uint8), bits[:ln])
    idx = np.where(rng.random(n_q) < 0.5, rng.integers(0, max(n_add, 1), n_q, dtype=np.uint64),
                   rng.integers(1 << 40, 1 << 41, n_q, dtype=np.uint64)).astype(np.uint64)
    d_idx = eng.to_device(idx)
    off, byt, tot = eng.gen_jackson_longs_dev(seed, n_q, d_idx=d_idx)
    d_c = eng.alloc(n_q)
    eng.bloom_contains_dev(name, n_q, off, byt, tot, d_c)
    got_c = d_c.download(np.uint8, n_q)
    want = O.bloom_contains_gen(bits, ln, size, k, seed, idx)
    assert np.array_equal(got_c, want), "k=%d contains differs at %s" % (k, np.flatnonzero(got_c != want)[:8])
    if n_add:
        assert got_c[idx < n_add].all()
    for x in (d_idx, off, byt, d_c):
        x.free()
    return size


@pytest.mark.parametrize("k", [2, 3, 5, 7, 9, 10])
def test_region_contains_every_k(O, k):
    """3 M + 123 contains (region schedule for k <= 9, the one-per-thread kernel for k = 10) on a filter of
    >= 64 regions with 400 k adds: replies equal the oracle's, members all true."""
    eng = _engine(max_batch=4 * M)
    try:
        size = _contains_case(O, eng, "rc:k%d" % k, 40_000_000, k, 400_000, 3 * M + 123, 0x5EED7000 + k,
                              np.random.default_rng(k))
        assert size >= 64 << 20
    finally:
        eng.close()


def test_region_contains_forced_small_batches(O, monkeypatch):
    """With the schedule forced on every batch (SK_BLOOM_RC_MIN=1): batches of 1, 4095, 4096, 4097 and 70 k
    elements, and a filter whose string is far shorter than m/8 (3 adds), equal the oracle's replies."""
    monkeypatch.setenv("SK_BLOOM_RC_MIN", "1")
    eng = _engine(max_batch=4 * M)
    try:
        rng = np.random.default_rng(77)
        for i, nq in enumerate([1, 4095, 4096, 4097, 70_000]):
            _contains_case(O, eng, "rcf:%d" % i, 20_000_000, 7, 50_000, nq, 0x5EED7100 + i, rng)
        _contains_case(O, eng, "rcf:short", 20_000_000, 7, 3, 100_000, 0x5EED7200, rng)
    finally:
        eng.close()


def test_region_contains_pieces(O, monkeypatch):
    """A 40 M batch runs as a 32 M piece and an 8 M piece over the same scratch: replies equal the oracle's."""
    eng = _engine(max_batch=4 * M)
    try:
        _contains_case(O, eng, "rcp", 50_000_000, 7, 1_000_000, 40 * M + 5, 0x5EED7300, np.random.default_rng(9))
    finally:
        eng.close()


def test_region_contains_host_path(O):
    """The host-buffer entry point (sk_bloom_contains) takes the region schedule for a large batch too."""
    from oracle.oracle import gen_jackson_long

    eng = _engine(max_batch=4 * M)
    try:
        p = _p_for_k(7, 20_000_000)
        assert eng.bloom_try_init("rch", 20_000_000, p)
        size, k, _, _ = eng.bloom_config("rch")
        seed = 0x5EED7400
        off, byt, tot = eng.gen_jackson_longs_dev(seed, 100_000)
        d_out = eng.alloc(100_000)
        eng.bloom_add_dev("rch", 100_000, off, byt, tot, d_out)
        bits, ln = O.bloom_add_gen(size, k, seed, 0, 100_000)
        n = (2 << 20) + 17
        idx = np.random.default_rng(3).integers(0, 200_000, n, dtype=np.uint64)
        elems = [gen_jackson_long(seed, int(i)) for i in idx[:4096]]
        # the host call packs elements itself; repeat the 4096 distinct ones to reach the batch size
        reps = [elems[i % 4096] for i in range(n)]
        got = np.array(eng.bloom_contains("rch", size, k, reps), dtype=np.uint8)
        want = O.bloom_contains_gen(bits, ln, size, k, seed, np.array([idx[i % 4096] for i in range(n)], np.uint64))
        assert np.array_equal(got, want)
    finally:
        eng.close()
