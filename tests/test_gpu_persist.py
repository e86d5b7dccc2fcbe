"""Store persistence in redis-server's own formats (SURVEY 5 "Checkpoint / resume", 8(f) rank 1).

SAVE writes the whole store as an RDB file (RDB version 7, what redis-server 3.2 writes); a fresh context loads it
and every key comes back: HLL registers, PFCOUNTs, Bloom bit arrays and configs, bitset bytes -- checked against the
oracle, not against the saving context.  DUMP / RESTORE move single keys as redis-server's payloads; SCAN enumerates
the keys.  The payloads are also parsed here by an independent Python reader of the format (CRC64 pinned by its
check value), so the bytes the engine writes are the documented format, not only self-consistent.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M = 1 << 20


def _engine(**kw):
    from redisson_amd import SketchEngine

    return SketchEngine(device=0, **kw)


# ------------------------------------------------------------------ an independent reader of the payload format
def crc64(data: bytes, crc: int = 0) -> int:
    """redis crc64.c (Jones polynomial, reflected), bit by bit."""
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x95AC9329AC4BC9B5 if crc & 1 else 0)
    return crc


def test_crc64_check_value():
    assert crc64(b"123456789") == 0xE9C6D914C4B8D9CA


def _rdb_len(b: bytes, i: int):
    t = b[i] >> 6
    if t == 0:
        return b[i] & 0x3F, i + 1
    if t == 1:
        return ((b[i] & 0x3F) << 8) | b[i + 1], i + 2
    assert b[i] == 0x80, "32-bit length expected, got %#x" % b[i]
    return int.from_bytes(b[i + 1:i + 5], "big"), i + 5


def parse_payload(p: bytes):
    """(type, value): value = bytes for a string, [(field, value)] for a hash; checks version 7 and the CRC."""
    assert int.from_bytes(p[-10:-8], "little") == 7, "RDB version"
    assert int.from_bytes(p[-8:], "little") == crc64(p[:-8]), "CRC64"
    body, i = p[:-10], 1
    if p[0] == 0:
        n, i = _rdb_len(body, i)
        assert i + n == len(body)
        return 0, body[i:i + n]
    assert p[0] == 4
    nf, i = _rdb_len(body, i)
    out = []
    for _ in range(nf):
        a, i = _rdb_len(body, i)
        f, i = body[i:i + a], i + a
        b_, i = _rdb_len(body, i)
        out.append((f, body[i:i + b_]))
        i += b_
    assert i == len(body)
    return 4, out


# ------------------------------------------------------------------ single keys
def test_dump_restore_scan_every_type(O, tmp_path):
    """DUMP of an HLL (its GET bytes), a bit string, a Bloom config (Redisson's HMSET fields and order, :238-240);
    RESTORE into other names gives identical GET / registers / config; BUSYKEY without REPLACE; a corrupt payload is
    refused; the Redis documentation's DUMP example (an integer-encoded string, RDB 9) restores; SCAN returns every
    key once while keys are deleted between its calls."""
    from redisson_amd.engine import RedisException

    eng = _engine()
    try:
        elems = [b'["java.lang.Long",%d]' % (i * 7919) for i in range(5000)]
        eng.pfadd([b"h:%d" % (i % 7) for i in range(5000)], [[e] for e in elems])
        eng.setbit([b"bits"] * 3, [3, 5, 1 << 20], [1, 1, 1])
        assert eng.bloom_try_init(b"bf", 100, 0.03)
        eng.bloom_add(b"bf", 729, 5, elems[:50])
        p = eng.dump(b"h:3")
        t, v = parse_payload(p)
        assert t == 0 and v == eng.get(b"h:3") and v[:4] == b"HYLL"
        t, v = parse_payload(eng.dump(b"{bf}__config"))
        assert t == 4 and v == [(b"size", b"729"), (b"hashIterations", b"5"), (b"expectedInsertions", b"100"),
                                (b"falseProbability", b"0.03")]
        assert eng.dump(b"missing") is None
        for k, to in ((b"h:3", b"h:3:copy"), (b"bits", b"bits:copy"), (b"bf", b"bf:copy"),
                      (b"{bf}__config", b"{bf:copy}__config")):
            eng.restore(to, eng.dump(k))
            assert eng.dump(to) == eng.dump(k), k
        assert np.array_equal(eng.hll_registers(b"h:3:copy"), eng.hll_registers(b"h:3"))
        assert eng.pfcount([[b"h:3:copy"]]) == eng.pfcount([[b"h:3"]])
        assert eng.get(b"bits:copy") == eng.get(b"bits")
        assert eng.bloom_config(b"bf:copy")[:2] == (729, 5)
        with pytest.raises(RedisException, match="BUSYKEY"):
            eng.restore(b"bits", eng.dump(b"h:3"))
        eng.restore(b"bits", eng.dump(b"h:3"), replace=True)
        assert eng.get(b"bits") == eng.get(b"h:3")
        bad = bytearray(eng.dump(b"h:1"))
        bad[20] ^= 1
        with pytest.raises(RedisException, match="checksum"):
            eng.restore(b"bad", bytes(bad))
        eng.restore(b"mykey", b"\x00\xc0\n\t\x00\xbem\x06\x89Z(\x00\n")   # SET mykey 10; DUMP mykey (redis docs)
        assert eng.get(b"mykey") == b"10"
        # SCAN: every key once, in pieces, with other keys deleted between the calls
        want = {k for k, _ in eng.keys()}
        assert {b"h:0", b"bits", b"bf", b"{bf}__config", b"mykey", b"h:3:copy"} <= want
        seen, cur, first = [], 0, True
        while True:
            cur, part = eng.scan(cur, 3)
            seen += [k for k, _ in part]
            if first:
                eng.delete([b"mykey"] if b"mykey" not in seen else [b"bits:copy"])
                first = False
            if not cur:
                break
        assert len(seen) == len(set(seen))
        assert want - {b"mykey", b"bits:copy"} <= set(seen)
        types = dict(eng.keys())
        assert types[b"h:0"] == 1 and types[b"bf"] == 2 and types[b"{bf}__config"] == 3
    finally:
        eng.close()


def _hash_payload(fields):
    """a DUMP payload of a hash (RDB type 4, plain encoding) with a valid CRC64"""
    def ln(n):
        return bytes([n]) if n < 64 else bytes([0x40 | (n >> 8), n & 0xFF])
    body = bytes([4]) + ln(len(fields))
    for f, v in fields:
        body += ln(len(f)) + f + ln(len(v)) + v
    body += bytes([7, 0])
    return body + crc64(body).to_bytes(8, "little")


def test_restore_refuses_bad_bloom_configs_and_keeps_the_old_key(O):
    """a restored Bloom config must be one tryInit can make (1 <= size <= 4,294,967,294, hashIterations in
    int range: the probe kernels index in 32-bit words); RESTORE ... REPLACE that fails leaves the old key alone
    (redis-server decodes the object before it deletes the old key); DBSIZE counts every key; SCAN returns a key
    once across its change of type (a string adopted as an HLL on its first PFADD)."""
    from redisson_amd.engine import RedisException

    eng = _engine()
    try:
        assert eng.bloom_try_init(b"bf", 100, 0.03)
        eng.setbit([b"bits"], [9], [1])
        good = eng.dump(b"{bf}__config")
        assert parse_payload(_hash_payload([(b"size", b"729"), (b"hashIterations", b"5")]))[0] == 4
        eng.restore(b"{ok}__config", _hash_payload([(b"size", b"729"), (b"hashIterations", b"5")]))
        for size, k in ((b"4294967301", b"5"), (b"4294967295", b"5"), (b"0", b"5"), (b"729", b"4294967301"),
                        (b"729", b"0"), (b"-3", b"5")):
            with pytest.raises(RedisException, match="out of range"):
                eng.restore(b"{bad}__config", _hash_payload([(b"size", size), (b"hashIterations", k)]))
            with pytest.raises(RedisException, match="out of range"):
                eng.restore(b"bits", _hash_payload([(b"size", size), (b"hashIterations", k)]), replace=True)
            assert eng.get(b"bits") == b"\x00\x40", "a failed REPLACE deleted the old key"
        assert eng.dump(b"{bad}__config") is None and eng.dump(b"{bf}__config") == good
        n = eng.dbsize()
        assert n == len(eng.keys()) == 3   # {bf}__config, bits, {ok}__config
        # a string holding a dense HLL becomes an HLL on its first PFADD: its SCAN position holds
        eng.pfadd([b"h"], [[b"x"]])
        eng.set(b"s", eng.get(b"h"))
        eng.delete([b"h"])
        seen, cur, first = [], 0, True
        while True:
            cur, part = eng.scan(cur, 1)
            seen += [k for k, _ in part]
            if first:
                eng.pfadd([b"s"], [[b"y"]])   # adopted between SCAN calls
                first = False
            if not cur:
                break
        assert sorted(seen) == sorted(set(seen)) and b"s" in seen and len(seen) == eng.dbsize() == 4
        assert dict(eng.keys())[b"s"] == 1
    finally:
        eng.close()


def test_exact_mode_sparse_strings_survive_save_load(O, tmp_path):
    """Exact HLL strings (redis-server's sparse bytes, sk_hll_exact_strings): SAVE / load keeps every GET byte for
    byte and the registers; in the default mode a sparse string from a redis-server file stays a string until its
    first HLL command (GET unchanged), then counts like the oracle."""
    path = str(tmp_path / "exact.rdb")
    a = _engine()
    try:
        a.hll_exact_strings(True)
        keys = [b"s:%d" % (i % 40) for i in range(3000)]
        elems = [[b'"e%d"' % i] for i in range(3000)]
        a.pfadd(keys, elems)
        gets = {k: a.get(k) for k in set(keys)}
        assert any(g[4] == 1 for g in gets.values())       # some are sparse
        regs = {k: a.hll_registers(k) for k in set(keys)}
        assert a.save(path) == 40
    finally:
        a.close()
    b = _engine()
    try:
        b.hll_exact_strings(True)
        assert b.load(path) == 40
        for k, g in gets.items():
            assert b.get(k) == g, k
            assert np.array_equal(b.hll_registers(k), regs[k])
    finally:
        b.close()
    c = _engine()   # default mode
    try:
        c.load(path)
        ref = O.HLLStore()
        ref.pfadd(keys, elems)
        for k, g in gets.items():
            assert c.get(k) == g, k                       # still the stored string
        assert c.pfcount([[k] for k in sorted(gets)]) == [ref.count([k]) for k in sorted(gets)]
    finally:
        c.close()


# ------------------------------------------------------------------ the C2-sized store
def test_snapshot_c2_store_restores_into_fresh_context(O, tmp_path):
    """a C2-sized store -- 100 k tenant HLLs (16 M PFADDs), a C3 filter (tryInit(425 M, 0.008):
    534 MB, 32 M adds) and a 2^31-bit bitset (16 M SETBITs) -- saved, the context closed, loaded into a fresh one:
    every register, every PFCOUNT, the Bloom bit array and config, and the bitset bytes equal the oracle's."""
    T, N, seed = 100_000, 16 * M, 0x5EED5002
    path = str(tmp_path / "c2.rdb")
    names = ["tenant:%d:hll" % t for t in range(T)]
    kid = np.random.default_rng(52).integers(0, T, N).astype(np.uint32)
    nadd, bseed = 32 * M, 0x5EED5003
    boffs = np.random.default_rng(53).integers(0, 1 << 31, 16 * M, dtype=np.uint64)
    a = _engine(hll_capacity=T + 16, max_batch=4 * M, max_bit_offset=1 << 34)
    try:
        ids = a.hll_resolve(names)
        d_out = a.alloc(4 * M)
        for s in range(0, N, 4 * M):
            off, byt, tot = a.gen_jackson_longs_dev(seed, 4 * M, first=s)
            d_ids = a.to_device(ids[kid[s:s + 4 * M]])
            a.pfadd_dev(4 * M, d_ids, off, byt, tot, d_out)
            for x in (off, byt, d_ids):
                x.free()
        assert a.bloom_try_init("c3", 425_000_000, 0.008)
        size, k, _, _ = a.bloom_config("c3")
        for s in range(0, nadd, 4 * M):
            off, byt, tot = a.gen_jackson_longs_dev(bseed, 4 * M, first=s)
            a.bloom_add_dev("c3", 4 * M, off, byt, tot, d_out)
            off.free()
            byt.free()
        d = a.to_device(boffs)
        a.setbit_dev("bits31", len(boffs), d, 1)
        d.free()
        assert a.save(path) == T + 3
    finally:
        a.close()
    regs = np.zeros((T, 16384), dtype=np.uint8)
    O.pfadd_gen(regs, np.zeros(T, dtype=np.uint8), kid, seed, 0)
    bits, ln = O.bloom_add_gen(size, k, bseed, 0, nadd)
    bbuf = np.zeros((1 << 28) + 16, dtype=np.uint8)
    O.setbits(bbuf, boffs)
    bln = int(boffs.max() >> np.uint64(3)) + 1
    b = _engine(hll_capacity=T + 16, max_bit_offset=1 << 34)
    try:
        assert b.load(path) == T + 3
        assert len(b.keys()) == T + 3
        for t in range(T):
            r = b.hll_registers(names[t])
            if not np.array_equal(r, regs[t]):
                raise AssertionError("registers of %s differ at %s" % (names[t], np.flatnonzero(r != regs[t])[:8]))
        assert b.pfcount([[nm] for nm in names]) == [O.count_regs(regs[t], 1) for t in range(T)]
        assert b.bloom_config("c3") == (size, k, 425_000_000, 0.008)
        got = np.frombuffer(b.get("c3"), np.uint8)
        assert len(got) == ln and np.array_equal(got, bits[:ln])
        del got
        assert np.array_equal(np.frombuffer(b.get("bits31"), np.uint8), bbuf[:bln])
        # and the restored filter answers: members of the adds are all contained
        off, byt, tot = b.gen_jackson_longs_dev(bseed, 1 << 16, first=0)
        d_c = b.alloc(1 << 16)
        b.bloom_contains_dev("c3", 1 << 16, off, byt, tot, d_c)
        assert d_c.download(np.uint8, 1 << 16).all()
    finally:
        b.close()
