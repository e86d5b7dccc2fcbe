"""The reference's own functional tests, re-expressed against the Redisson-shaped
API (which runs every command through the C ABI on the GPU).

T: = /root/reference/src/test/java/org/redisson/
"""
import pytest

from redisson_amd import IllegalStateException, JBitSet, JInteger, RedisException

pytestmark = pytest.mark.gpu


# ---- T:RedissonHyperLogLogTest.java ----------------------------------------
def test_hll_add(client):                                    # :10-17
    log = client.getHyperLogLog("log")
    log.add(JInteger(1))
    log.add(JInteger(2))
    log.add(JInteger(3))
    assert log.count() == 3


def test_hll_merge(client):                                  # :20-38
    hll1 = client.getHyperLogLog("hll1")
    assert hll1.add("foo")
    assert hll1.add("bar")
    assert hll1.add("zap")
    assert hll1.add("a")
    hll2 = client.getHyperLogLog("hll2")
    assert hll2.add("a")
    assert hll2.add("b")
    assert hll2.add("c")
    assert hll2.add("foo")
    assert not hll2.add("c")
    hll3 = client.getHyperLogLog("hll3")
    hll3.mergeWith("hll1", "hll2")
    assert hll3.count() == 6


def test_hll_count_with_and_addall_quirk(client):
    a = client.getHyperLogLog("cw:a")
    b = client.getHyperLogLog("cw:b")
    for i in range(100):
        a.add("x%d" % i)
        b.add("x%d" % (i + 50))
    assert a.countWith("cw:b") == client.getHyperLogLog("cw:a").countWith("cw:b")
    assert 140 <= a.countWith("cw:b") <= 160
    # Q1: addAll sends ONE element (the encoded Object[]), so count() == 1
    c = client.getHyperLogLog("cw:c")
    assert c.addAll(["p", "q", "r"])
    assert c.count() == 1


# ---- T:RedissonBloomFilterTest.java ----------------------------------------
def test_bloom_config(client):                               # :10-17
    f = client.getBloomFilter("filter")
    f.tryInit(100, 0.03)
    assert f.getExpectedInsertions() == 100
    assert f.getFalseProbability() == 0.03
    assert f.getHashIterations() == 5
    assert f.getSize() == 729


def test_bloom_init(client):                                 # :20-28
    f = client.getBloomFilter("filter2")
    assert f.tryInit(55000000, 0.03)
    assert not f.tryInit(55000001, 0.03)
    # Q6: the pipeline's HMSET runs after the failed EVAL assert, so the new
    # parameters replace the config (M:RedissonBloomFilter.java:231-248)
    assert f.getExpectedInsertions() == 55000001
    f.delete()
    assert f.tryInit(55000001, 0.03)


@pytest.mark.parametrize("op", ["getExpectedInsertions", "contains", "add"])
def test_bloom_not_initialized(client, op):                  # :30-49
    f = client.getBloomFilter("nofilter")
    with pytest.raises(IllegalStateException):
        if op == "getExpectedInsertions":
            f.getExpectedInsertions()
        else:
            getattr(f, op)("32")


def test_bloom(client):                                      # :52-66
    f = client.getBloomFilter("filter3")
    f.tryInit(550000000, 0.03)
    assert not f.contains("123")
    assert f.add("123")
    assert f.contains("123")
    assert not f.add("123")
    assert f.count() == 1
    assert not f.contains("hflgs;jl;ao1-32471320o31803-24")
    assert f.add("hflgs;jl;ao1-32471320o31803-24")
    assert f.contains("hflgs;jl;ao1-32471320o31803-24")
    assert f.count() == 2


# ---- T:RedissonBitSetTest.java ---------------------------------------------
def test_bitset_index_range(client):                         # :11-18
    bs = client.getBitSet("testbitset")
    top = 2147483647 * 2
    assert not bs.get(top)
    bs.set(top)
    assert bs.get(top)


def test_bitset_length(client):                              # :20-47
    bs = client.getBitSet("testbitset_len")
    bs.set(0, 5)
    bs.clear(0, 1)
    assert bs.length() == 5
    bs.clear()
    bs.set(28)
    bs.set(31)
    assert bs.length() == 32
    bs.clear()
    bs.set(3)
    bs.set(7)
    assert bs.length() == 8
    bs.clear()
    bs.set(3)
    bs.set(120)
    bs.set(121)
    assert bs.length() == 122
    bs.clear()
    bs.set(0)
    assert bs.length() == 1


def test_bitset_length_errors_on_empty(client):
    # Lua script: BITPOS -1 -> GETBIT -1 raises (reference behaviour)
    with pytest.raises(RedisException, match="bit offset"):
        client.getBitSet("never").length()


def test_bitset_clear(client):                               # :50-55
    bs = client.getBitSet("tb_clear")
    bs.set(0, 8)
    bs.clear(0, 3)
    assert str(bs) == "{3, 4, 5, 6, 7}"


def test_bitset_not(client):                                 # :58-64
    bs = client.getBitSet("tb_not")
    bs.set(3)
    bs.set(5)
    bs.not_()
    assert str(bs) == "{0, 1, 2, 4, 6, 7}"


def test_bitset_set(client):                                 # :67-80
    bs = client.getBitSet("tb_set")
    bs.set(3)
    bs.set(5)
    assert str(bs) == "{3, 5}"
    bs1 = JBitSet()
    bs1.set(1)
    bs1.set(10)
    bs.set(bs1)
    bs = client.getBitSet("tb_set")
    assert str(bs) == "{1, 10}"


def test_bitset_set_get(client):                             # :83-97
    bitset = client.getBitSet("tb_sg")
    assert bitset.cardinality() == 0
    assert bitset.size() == 0
    bitset.set(10, True)
    bitset.set(31, True)
    assert not bitset.get(0)
    assert bitset.get(31)
    assert bitset.get(10)
    assert bitset.cardinality() == 2
    assert bitset.size() == 32


def test_bitset_set_range(client):                           # :100-105
    bs = client.getBitSet("tb_range")
    bs.set(3, 10)
    assert bs.cardinality() == 7
    assert bs.size() == 16


def test_bitset_as_bitset(client):                           # :108-119
    bs = client.getBitSet("tb_as")
    bs.set(3, True)
    bs.set(41, True)
    assert bs.size() == 48
    b = bs.asBitSet()
    assert b.get(3)
    assert b.get(41)
    assert bs.cardinality() == 2


def test_bitset_and(client):                                 # :122-139
    bs1 = client.getBitSet("testbitset1")
    bs1.set(3, 5)
    assert bs1.cardinality() == 2
    assert bs1.size() == 8
    bs2 = client.getBitSet("testbitset2")
    bs2.set(4)
    bs2.set(10)
    bs1.and_(bs2.getName())
    assert not bs1.get(3)
    assert bs1.get(4)
    assert not bs1.get(5)
    assert bs2.get(10)
    assert bs1.cardinality() == 1
    assert bs1.size() == 16


# ---- T:RedissonBatchTest.java ----------------------------------------------
def test_batch_order_and_results(client):                    # :79-90, :116-148
    b = client.createBatch()
    futs = []
    for i in range(210):
        futs.append(b.getHyperLogLog("bt:%d" % (i % 7)).addAsync("e%d" % (i // 2)))
        futs.append(b.getBitSet("bt:bits").getAsync(i))
        b.getBitSet("bt:bits").setAsync(i, True)
        futs.append(b.getBitSet("bt:bits").getAsync(i))
    res = b.execute()
    assert len(res) == 210 * 4
    assert [f.get() for f in futs] == [r for j, r in enumerate(res) if j % 4 != 2]
    assert all(res[j] is True for j in range(3, len(res), 4))
    assert all(res[j] is False for j in range(1, len(res), 4))
    with pytest.raises(IllegalStateException):
        b.execute()
    assert client.createBatch().execute() is None
