"""Pin the oracle before trusting it (CPU only).

No runnable reference exists here (no JVM, no redis-server, no OpenHFT jar:
SURVEY.md 8c), so each restated third-party algorithm is pinned to published
known answers, and the reference's own functional tests are re-expressed on
the oracle:

* MurmurHash64A -- SMHasher VerificationTest value 0x1F0D3804.
* XXH64 (OpenHFT xx_r39) -- python ``xxhash`` 3.8.1, every length 0..300.
* farmhashna::Hash64 (= OpenHFT farmUo for len <= 64) -- Guava
  FarmHashFingerprint64Test known answers for "test", "test"*8, "test"*64.
  farmUo for len > 64 is parity UNPINNED (no published vector available).
* CRC16-XMODEM -- check value crc16("123456789") = 0x31C3; calcSlot -- the
  CLUSTER KEYSLOT examples of the Redis cluster spec.
* Bloom sizing -- T:RedissonBloomFilterTest.java:12-16 (729 / 5).
* HLL -- T:RedissonHyperLogLogTest.java:10-38 (count 3, replies, merge 6).
"""
import numpy as np
import pytest


def test_murmur64a_smhasher_verification(O):
    assert O.lib().or_murmur64a_verification() == 0x1F0D3804


def test_xxh64_against_python_xxhash(O):
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(1)
    for n in range(0, 301):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.xxh64(b) == xxhash.xxh64_intdigest(b, 0), n
    assert O.xxh64(b"") == 0xEF46DB3751D8E999


def _s64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def test_farmhash_guava_known_answers(O):
    assert _s64(O.farmhash_na64(b"test")) == 8581389452482819506
    assert _s64(O.farmhash_na64(b"test" * 8)) == -4196240717365766262
    assert _s64(O.farmhash_na64(b"test" * 64)) == 3500507768004279527
    # farmUo == farmhashna for len <= 64
    for n in range(0, 65):
        b = bytes(range(n))
        assert O.farmhash_uo64(b) == O.farmhash_na64(b)


def test_crc16_and_calc_slot(O):
    assert O.crc16(b"123456789") == 0x31C3
    assert O.calc_slot("somekey") == 11058
    assert O.calc_slot("foo{hash_tag}") == 2515
    assert O.calc_slot("bar{hash_tag}") == 2515
    assert O.calc_slot("{}") == 0                # empty tag -> crc16("") = 0
    assert O.calc_slot("a}b{c") == -1            # Redisson: first '}' anywhere -> substring throws
    assert O.calc_slot("{user1000}.following") == O.calc_slot("user1000")


def test_bloom_sizing_reference(O):
    m = O.bloom_optimal_bits(100, 0.03)
    assert (m, O.bloom_optimal_k(100, m)) == (729, 5)
    m = O.bloom_optimal_bits(550000000, 0.03)
    assert (m, O.bloom_optimal_k(550000000, m)) == (4014142460, 5)
    m = O.bloom_optimal_bits(425000000, 0.008)   # C3
    assert (m, O.bloom_optimal_k(425000000, m)) == (4271038538, 7)


def test_hll_reference_cases(O):
    s = O.HLLStore()
    s.pfadd([b"log"] * 3, [[b"1"], [b"2"], [b"3"]])            # Integer -> "1"
    assert s.count([b"log"]) == 3
    q = lambda x: b'"' + x + b'"'
    assert s.pfadd([b"hll1"] * 4, [[q(b"foo")], [q(b"bar")], [q(b"zap")], [q(b"a")]]) == [True] * 4
    assert s.pfadd([b"hll2"] * 5, [[q(x)] for x in (b"a", b"b", b"c", b"foo", b"c")]) == [True] * 4 + [False]
    s.merge(b"hll3", [b"hll3", b"hll1", b"hll2"])
    assert s.count([b"hll3"]) == 6


def test_hll_patlen_versions(O):
    # both sentinel forms agree except when bits 14..62 are all zero
    rng = np.random.default_rng(2)
    for _ in range(2000):
        b = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        assert O.hll_patlen(b, 3) == O.hll_patlen(b, 5)


def test_hll_estimators_small_exact(O):
    s = O.HLLStore()
    for n in [0, 1, 7, 100, 1000]:
        k = b"n%d" % n
        s.pfadd([k], [[b"%d" % i for i in range(n)]])
        assert s.count([k]) == n if n <= 100 else abs(s.count([k]) - n) < 0.03 * n
    s5 = O.HLLStore(5)
    s5.pfadd([b"x"], [[b"%d" % i for i in range(7)]])
    assert s5.count([b"x"]) == 7


def test_dense_pack_roundtrip(O):
    rng = np.random.default_rng(3)
    regs = rng.integers(0, 64, 16384).astype(np.uint8)
    packed = O.dense_pack(regs)
    out = np.zeros(16384, dtype=np.uint8)
    O.lib().or_hll_dense_unpack(np.frombuffer(packed, dtype=np.uint8).ctypes.data, out.ctypes.data)
    np.testing.assert_array_equal(out, regs)


def test_bitops_reference_semantics(O):
    b = O.BitString()
    assert b.setbit(3, 1) == 0 and b.setbit(5, 1) == 0 and b.setbit(3, 1) == 1
    assert b.bytes() == bytes([0b00010100])
    assert O.bitop("NOT", [b.bytes()]) == bytes([0b11101011])     # RedissonBitSetTest.testNot
    assert O.bitop("AND", [b"\xff\x0f", None]) == b"\x00\x00"       # missing key = zeros, len = max
    assert O.bitop("OR", [None, None]) == b""


def test_hll_string_codec_round_trip(O):
    """Redis HLL strings (dense and the canonical sparse form) decode back to
    the registers; the sparse stream follows the opcode layout of hyperloglog.c."""
    rng = np.random.default_rng(5)
    for trial in range(6):
        regs = np.zeros(16384, dtype=np.uint8)
        m = [0, 1, 10, 500, 4000, 16384][trial]
        if m:
            regs[rng.integers(0, 16384, m)] = rng.integers(1, 33, m)
        for enc in ["dense", "sparse"]:
            s = O.hll_string(regs, enc)
            np.testing.assert_array_equal(O.hll_decode(s), regs)
    empty = O.hll_string(np.zeros(16384, dtype=np.uint8), "sparse")
    assert empty[16:] == bytes([0x7F, 0xFF]) and empty[4] == 1      # one XZERO covering 16384 registers
    one = np.zeros(16384, dtype=np.uint8)
    one[0] = 3
    assert O.hll_string(one, "sparse")[16:] == bytes([0x88, 0x7F, 0xFE])  # VAL(3,1) XZERO(16383)


def test_threaded_baseline_matches_oracle(O):
    """bench.py's whole-host CPU baseline (oracle_mt.c) gives the single-threaded oracle's registers and replies."""
    from redisson_amd import gen_jackson_longs

    n, nkeys = 60000, 97
    off, buf = gen_jackson_longs(0x5EED0777, n)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    buf = np.concatenate([np.asarray(buf, dtype=np.uint8), np.zeros(16, np.uint8)])
    kid = np.random.default_rng(5).integers(0, nkeys, n).astype(np.uint32)
    regs1, r1 = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    regs4, r4 = O.HLLStore().pfadd_bulk_mt(kid, off, buf, nkeys, 4)
    assert np.array_equal(regs1, regs4) and np.array_equal(r1, r4)
    bits = O.BitString()
    size, k = 200000, 5
    bits.bloom_add_raw(size, k, off[:20001], buf)
    c1 = bits.bloom_contains_raw(size, k, off, buf)
    c3 = bits.bloom_contains_raw_mt(size, k, off, buf, 3)
    assert np.array_equal(c1, c3) and c1[:20000].all() and not c1[20000:].all()


def test_full_size_checkers_agree_with_oracle(O):
    """The generator-driven checkers of tests/test_full_size.py (oracle_mt.c) equal the plain oracle on the
    elements the engine's host generator produces (sk_gen_jackson_longs: same SplitMix64 stream)."""
    from redisson_amd import gen_jackson_longs

    seed, n, nkeys = 0x5EED0888, 30000, 53
    off, buf = gen_jackson_longs(seed, n)
    els = [bytes(buf[off[i]:off[i + 1]]) for i in range(n)]
    assert [O.gen_jackson_long(seed, i) for i in (0, 1, 7, n - 1)] == [els[0], els[1], els[7], els[n - 1]]
    off = np.ascontiguousarray(off, dtype=np.uint64)
    kid = np.random.default_rng(9).integers(0, nkeys, n).astype(np.uint32)
    regs1, r1 = O.HLLStore().pfadd_bulk(kid, off, buf, nkeys)
    regs = np.zeros((nkeys, 16384), np.uint8)
    ex = np.zeros(nkeys, np.uint8)
    r, ones = O.pfadd_gen(regs, ex, kid[:10000], seed, 0)
    r2, ones2 = O.pfadd_gen(regs, ex, kid[10000:], seed, 10000)
    assert np.array_equal(regs, regs1) and np.array_equal(np.concatenate([r, r2]), r1)
    assert ones + ones2 == int(r1.sum())
    assert np.array_equal(O.hll_union_gen(n, seed), regs1.max(axis=0))
    size, k = 300007, 6
    bits = O.BitString()
    bits.bloom_add_raw(size, k, off[:12001], buf)
    g, ln = O.bloom_add_gen(size, k, seed, 0, 12000)
    assert ln == bits.len.value and bytes(g[:ln]) == bits.bytes() and not g[ln:].any()
    idx = np.arange(n, dtype=np.uint64)[::-1].copy()
    want = bits.bloom_contains(size, k, [els[i] for i in idx])
    assert O.bloom_contains_gen(g, ln, size, k, seed, idx).astype(bool).tolist() == want
    offs = np.random.default_rng(3).integers(0, 1 << 20, 5000).astype(np.uint64)
    b1 = O.BitString()
    for o in offs:
        b1.setbit(int(o), 1)
    b2 = np.zeros((1 << 17) + 16, np.uint8)
    O.setbits(b2, offs)
    assert bytes(b2[:b1.len.value]) == b1.bytes()
