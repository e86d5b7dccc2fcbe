"""Redis HLL strings byte for byte (sk_hll_exact_strings): GET of an HLL key returns what redis-server 3.2 holds.

redis-server keeps small HLLs sparse (hyperloglog.c hllSparseSet: the opcode covering a register is split, VAL
neighbours merged locally, promotion to dense past 3000 bytes or a register > 32) and keeps 8 bytes of cached
cardinality that PFADD marks stale, single-key PFCOUNT stores and PFMERGE marks stale.  The oracle
(oracle/sketch_oracle.c or_hllstr_*, HLLStrStore) replays every command in order; the engine decides every
register rise on the GPU (the apply kernel logs them) and replays only the rises into the string.  Sparse bytes
depend on the order registers rose, so the cases mix keys, repeat elements and cross the promotion size.
Parity of the sparse byte layout against a live redis-server is unpinned (no redis-server in the image); the
oracle restates hyperloglog.c.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine():
    from redisson_amd import SketchEngine

    eng = SketchEngine(device=0)
    eng.hll_exact_strings(True)
    return eng


def _elems(rng, n, space):
    return [b"e%d" % int(x) for x in rng.integers(0, space, n)]


def _check_all(eng, ref, keys):
    for k in keys:
        assert eng.get(k) == ref.get(k), k


def test_sparse_strings_follow_every_batch(O):
    """RBatch-style batches of PFADD over 24 keys, one and several elements per command, repeats across and inside
    batches: every reply and every key's GET bytes equal the oracle's after each batch."""
    eng = _engine()
    ref = O.HLLStrStore()
    try:
        rng = np.random.default_rng(1)
        keys = [b"hs:%d" % i for i in range(24)]
        for b in range(12):
            ks, es = [], []
            for _ in range(3000):
                ks.append(keys[int(rng.integers(0, len(keys)))])
                es.append(_elems(rng, int(rng.integers(1, 4)) if b % 3 else 1, 50000))
            got = eng.pfadd(ks, es)
            want = [bool(ref.pfadd(k, e)) for k, e in zip(ks, es)]
            assert got == want
            _check_all(eng, ref, keys)
            if b == 0:
                assert all(ref.get(k)[4] == 1 for k in keys)      # sparse after the first batch
        assert all(ref.get(k)[4] == 0 for k in keys)              # every key promoted on the way
    finally:
        eng.close()


def test_promotion_and_cached_cardinality(O):
    """One key grown element by element past the sparse limit (promotion to dense), with single-key PFCOUNTs that
    store the cached cardinality, PFADDs that leave it valid (no rise) or stale (a rise), and multi-key PFCOUNTs
    that leave it alone."""
    eng = _engine()
    ref = O.HLLStrStore()
    try:
        k, other = b"hp:k", b"hp:o"
        eng.pfadd([other], [[b"x", b"y"]])
        ref.pfadd(other, [b"x", b"y"])
        for i in range(0, 2600, 100):
            e = [b"p%d" % j for j in range(i, i + 100)]
            assert eng.pfadd([k], [e]) == [bool(ref.pfadd(k, e))]
            if i % 300 == 0:
                assert eng.pfcount([[k]]) == [ref.pfcount([k])]
            if i % 500 == 0:
                assert eng.pfcount([[k, other]]) == [ref.pfcount([k, other])]
            assert eng.pfadd([k], [[b"p%d" % i]]) == [bool(ref.pfadd(k, [b"p%d" % i]))]   # no rise: cache kept
            _check_all(eng, ref, [k, other])
        assert ref.get(k)[4] == 0, "grew past the sparse limit"
        assert eng.pfcount([[k]]) == [ref.pfcount([k])]
        _check_all(eng, ref, [k])
    finally:
        eng.close()


def test_pfmerge_destination_and_adopted_sparse_string(O):
    """PFMERGE makes its destination dense with a stale cache (new and existing destinations; sources untouched).
    A sparse string SET from the oracle is adopted with its own bytes and header, and later PFADDs continue from
    its opcodes as redis-server would."""
    eng = _engine()
    ref = O.HLLStrStore()
    try:
        rng = np.random.default_rng(3)
        srcs = [b"hm:%d" % i for i in range(4)]
        for s in srcs:
            e = _elems(rng, 60, 10**6)
            eng.pfadd([s], [e])
            ref.pfadd(s, e)
        eng.pfmerge(b"hm:new", srcs)
        ref.pfmerge(b"hm:new", srcs)
        eng.pfmerge(srcs[0], srcs[1:])
        ref.pfmerge(srcs[0], srcs[1:])
        _check_all(eng, ref, srcs + [b"hm:new"])
        assert eng.pfcount([[b"hm:new"]]) == [ref.pfcount([b"hm:new"])]
        _check_all(eng, ref, [b"hm:new"])
        # a sparse string written elsewhere, then more PFADDs on it
        donor = O.HLLStrStore()
        e0 = _elems(rng, 200, 10**6)
        donor.pfadd(b"d", e0)
        donor.pfcount([b"d"])                     # a valid cached cardinality in the header
        blob = donor.get(b"d")
        assert blob[4] == 1
        eng.set(b"hm:adopt", blob)
        ref.set(b"hm:adopt", blob)
        assert eng.pfcount([[b"hm:adopt"]]) == [ref.pfcount([b"hm:adopt"])]   # answered by the cached value
        e1 = _elems(rng, 300, 10**6)
        assert eng.pfadd([b"hm:adopt"] * len(e1), [[x] for x in e1]) == \
            [bool(ref.pfadd(b"hm:adopt", [x])) for x in e1]
        _check_all(eng, ref, [b"hm:adopt"])
    finally:
        eng.close()


def test_device_batches_and_mode_switch(O):
    """sk_pfadd_dev batches (generated Longs, one element per command over 500 tenants) keep the strings exact;
    the mode cannot change while HLL keys exist."""
    from oracle.oracle import gen_jackson_long
    from redisson_amd import RedisException

    eng = _engine()
    ref = O.HLLStrStore()
    try:
        keys = [b"hd:%d" % i for i in range(500)]
        ids = eng.hll_resolve(keys)
        for k in keys:       # the engine created them (PFADD's first command does in redis-server)
            ref.pfadd(k, [])
        rng = np.random.default_rng(5)
        seed, n, first = 0x5EED7700, 20000, 0
        for b in range(3):
            kid = rng.integers(0, len(keys), n)
            d_ids = eng.to_device(ids[kid].astype(np.uint32))
            off, byt, tot = eng.gen_jackson_longs_dev(seed, n, first=first)
            d_out = eng.alloc(n)
            eng.pfadd_dev(n, d_ids, off, byt, tot, d_out)
            got = d_out.download(np.uint8, n)
            want = [ref.pfadd(keys[int(t)], [gen_jackson_long(seed, first + i)]) for i, t in enumerate(kid)]
            assert got.tolist() == want
            for x in (d_ids, off, byt, d_out):
                x.free()
            first += n
        _check_all(eng, ref, keys)
        with pytest.raises(RedisException):
            eng.hll_exact_strings(False)
    finally:
        eng.close()
