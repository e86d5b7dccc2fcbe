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


# ------------------------------------------------------------------ Bloom add, region schedule
def _add_case(O, eng, name, n_exp, k, batches):
    """Adds `batches` (lists of byte elements) in order through sk_bloom_add; every reply and the whole string
    must equal the oracle's (one SETBIT per probe in (element, probe) order, M:RedissonBloomFilter.java:94-113)."""
    p = _p_for_k(k, n_exp)
    assert eng.bloom_try_init(name, n_exp, p)
    size, kk, _, _ = eng.bloom_config(name)
    assert kk == k
    ref = O.BitString(16)
    for b in batches:
        got = eng.bloom_add(name, size, k, b)
        want = ref.bloom_add(size, k, b)
        bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]  # no pytest diff of 10^5-element lists
        assert len(got) == len(want) and not bad, "k=%d add replies differ at %d places, first %s (got %s)" % (
            k, len(bad), bad[:8], [got[i] for i in bad[:8]])
    gb, wb = eng.get(name), ref.bytes()
    assert len(gb) == len(wb) and gb == wb, "bit string differs: %d vs %d bytes, first byte %s" % (
        len(gb), len(wb), next((i for i, (x, y) in enumerate(zip(gb, wb)) if x != y), None))
    return size


def _longs(a, b):
    return [b'["java.lang.Long",%d]' % i for i in range(a, b)]


@pytest.mark.parametrize("k", [1, 2, 3, 5, 7, 8, 9])
def test_region_add_every_k(O, k):
    """Two overlapping batches of 150 k adds (the second repeats half of the first, and repeats inside itself) on a
    filter of >= 8 regions: replies and the bit string equal the oracle's for every k the schedule takes (1..8)
    and for k = 9 (the sort path)."""
    eng = _engine(max_batch=4 * M)
    try:
        first = _longs(0, 150_000)
        second = _longs(75_000, 200_000) + _longs(190_000, 215_000)
        rng = np.random.default_rng(k)
        np.random.default_rng(k).shuffle(second)
        second = [second[i] if rng.random() < 0.9 else first[int(rng.integers(0, 150_000))] for i in range(len(second))]
        _add_case(O, eng, "ra:k%d" % k, 4_000_000, k, [first, second])
    finally:
        eng.close()


def test_region_add_windows_and_small_filters(O):
    """One-region filters (m < 2^20) filled far past one window per region (dense, hundreds of windows), a filter
    whose regions stay sparse (words set in place), and batches of 1, 2 and 2049 elements."""
    eng = _engine(max_batch=4 * M)
    try:
        _add_case(O, eng, "raw:one", 50_000, 7, [_longs(0, 120_000), _longs(100_000, 130_000)])
        _add_case(O, eng, "raw:sparse", 50_000_000, 5, [_longs(0, 3000), _longs(2000, 2500)])
        _add_case(O, eng, "raw:tiny", 1_000_000, 7, [_longs(5, 6), _longs(5, 7), _longs(0, 2049), _longs(7, 8)])
    finally:
        eng.close()


def test_region_add_repeated_element_takes_sort_path(O):
    """One element repeated 5000 times in a batch puts > RA_SEGMAX records of one block in one region: the piece
    goes to the sort path; replies (only the first copy answers true) and bits equal the oracle's either way."""
    eng = _engine(max_batch=4 * M)
    try:
        rep = [b'"same"'] * 5000 + _longs(0, 3000) + [b'"same"', b'"other"', b'"other"']
        _add_case(O, eng, "rar", 1_000_000, 7, [rep, _longs(2000, 4000)])
    finally:
        eng.close()


def test_region_add_device_pieces_match_gen(O, monkeypatch):
    """A 20 M device add runs as a 16 M piece and a 4 M piece (then a second add of 2 M old + 1 M new elements):
    the string and every reply equal the sequential oracle's."""
    eng = _engine(max_batch=4 * M)
    try:
        p = _p_for_k(7, 30_000_000)
        assert eng.bloom_try_init("rap", 30_000_000, p)
        size, k, _, _ = eng.bloom_config("rap")
        seed, n = 0x5EED7500, 20 * M + 3
        off, byt, tot = eng.gen_jackson_longs_dev(seed, n)
        d_out = eng.alloc(n)
        eng.bloom_add_dev("rap", n, off, byt, tot, d_out)
        bits, ln, want = O.bloom_add_gen_seq(size, k, seed, 0, n)
        got = eng.get("rap")
        assert len(got) == ln and np.array_equal(np.frombuffer(got, np.uint8), bits[:ln])
        rep = d_out.download(np.uint8, n)
        assert np.array_equal(rep, want), np.flatnonzero(rep != want)[:8]
        for x in (off, byt, d_out):
            x.free()
        # elements n-2M .. n+1M: the first 2 M are already in (only false positives of the sequential order differ)
        off, byt, tot = eng.gen_jackson_longs_dev(seed, 3 * M, first=n - 2 * M)
        d_out = eng.alloc(3 * M)
        eng.bloom_add_dev("rap", 3 * M, off, byt, tot, d_out)
        b2, ln2, w2 = O.bloom_add_gen_seq(size, k, seed, 0, n + M)
        got = eng.get("rap")
        assert len(got) == ln2 and np.array_equal(np.frombuffer(got, np.uint8), b2[:ln2])
        rep = d_out.download(np.uint8, 3 * M)
        assert not rep[:2 * M].any()
        assert np.array_equal(rep[2 * M:], w2[n:]), np.flatnonzero(rep[2 * M:] != w2[n:])[:8]
        for x in (off, byt, d_out):
            x.free()
    finally:
        eng.close()


def test_region_add_late_piece_falls_back_in_order(O):
    """A 9 M device add whose second piece (from element 8 M) holds one element 3000 times: piece 0 runs on the
    region schedule, the hash pass of piece 1 stops every later apply and the host redoes piece 1 on the sort path.
    Bits and every reply equal the sequential oracle's."""
    eng = _engine(max_batch=4 * M)
    try:
        p = _p_for_k(7, 20_000_000)
        assert eng.bloom_try_init("ral", 20_000_000, p)
        size, k, _, _ = eng.bloom_config("ral")
        seed, n = 0x5EED7600, 9 * M
        idx = np.arange(n, dtype=np.uint64)
        idx[8 * M + 1000:8 * M + 4000] = 42
        d_idx = eng.to_device(idx)
        off, byt, tot = eng.gen_jackson_longs_dev(seed, n, d_idx=d_idx)
        d_out = eng.alloc(n)
        eng.bloom_add_dev("ral", n, off, byt, tot, d_out)
        bits = np.zeros((size + 7) // 8 + 16, dtype=np.uint8)
        ln, want = O.bloom_add_idx_seq(bits, 0, size, k, seed, idx)
        got = eng.get("ral")
        assert len(got) == ln and np.array_equal(np.frombuffer(got, np.uint8), bits[:ln])
        rep = d_out.download(np.uint8, n)
        assert np.array_equal(rep, want), np.flatnonzero(rep != want)[:8]
        for x in (d_idx, off, byt, d_out):
            x.free()
    finally:
        eng.close()


def test_region_shared_prefix_mixed_elements(O, monkeypatch):
    """The hash blocks' shared-prefix path (sk_device.h bloom_hashes_pre): elements that match the block's 16-byte
    pattern with every length around the 33..63 window, elements differing in one byte of the pattern, and blocks
    whose first element is not a Jackson Long (the pattern is someone else's bytes) -- add replies, contains replies
    and the bit array equal the oracle's on the region schedule (forced for every batch size)."""
    monkeypatch.setenv("SK_BLOOM_RC_MIN", "1")
    monkeypatch.setenv("SK_BLOOM_RA_MIN", "1")
    rng = np.random.default_rng(77)
    pref = b'["java.lang.Long",'
    elems = []
    for i in range(30000):
        r = i % 6
        if r == 0:
            elems.append(b'["java.lang.Long",%d]' % int(rng.integers(-(1 << 63), 1 << 63)))
        elif r == 1:   # the pattern, then any length 16..80
            elems.append(pref[:16] + bytes(rng.integers(48, 58, int(rng.integers(0, 65)), dtype=np.uint8)))
        elif r == 2:   # one byte of the 16 differs
            e = bytearray(b'["java.lang.Long",%d]' % int(rng.integers(0, 1 << 62)))
            e[int(rng.integers(0, 16))] ^= 0x20
            elems.append(bytes(e))
        elif r == 3:   # random bytes, 0..90
            elems.append(rng.integers(0, 256, int(rng.integers(0, 91)), dtype=np.uint8).tobytes())
        elif r == 4:   # quoted strings (the String codec form)
            elems.append(b'"%s"' % (b"k" * int(rng.integers(0, 60))))
        else:
            elems.append(b'["java.lang.Long",%d]' % int(rng.integers(0, 1000)))
    order = rng.permutation(len(elems))
    elems = [elems[i] for i in order]
    eng = _engine()
    try:
        assert eng.bloom_try_init("pref", 40000, 0.01)
        size, k, _, _ = eng.bloom_config("pref")
        ref = O.BitString(16)
        half = len(elems) // 2
        assert eng.bloom_add("pref", size, k, elems[:half]) == ref.bloom_add(size, k, elems[:half])
        probe = elems[half // 2:] + [e + b"x" for e in elems[:2000]]
        assert eng.bloom_contains("pref", size, k, probe) == ref.bloom_contains(size, k, probe)
        assert eng.get("pref") == ref.bytes()
    finally:
        eng.close()
