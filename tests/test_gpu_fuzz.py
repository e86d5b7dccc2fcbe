"""Differential fuzzing: random interleavings of every command on the path,
through the C ABI on the GPU, against the CPU oracle's model of the keyspace.

Each step is a batch (the RBatch shape): PFADD with 0..4 elements per
command over a small key pool (many intra-batch collisions), PFCOUNT single
and multi-key (with missing keys), PFMERGE, SETBIT / GETBIT with replies,
range set/clear, BITOP, BITCOUNT / STRLEN / GET, DEL, Bloom add / contains.
Every reply is compared as it comes, and the whole state (HLL registers, bit
strings) every few steps and at the end."""
import numpy as np
import pytest

from redisson_amd import RedisException, gen_jackson_longs

pytestmark = pytest.mark.gpu

HLL_KEYS = [b"fz:h:%d" % i for i in range(8)]
BIT_KEYS = [b"fz:b:%d" % i for i in range(5)]


def _pool(seed, n):
    off, buf = gen_jackson_longs(seed, n)
    rng = np.random.default_rng(seed)
    out = [buf[off[i]:off[i + 1]].tobytes() for i in range(n)]
    out += [rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes() for _ in range(n // 4)]
    return out


class Model:
    def __init__(self, O):
        self.O = O
        self.hll = O.HLLStore()
        self.bits = {}

    def bitstr(self, k):
        if k not in self.bits:
            self.bits[k] = self.O.BitString()
        return self.bits[k]

    def bytes_of(self, k):
        return self.bits[k].bytes() if k in self.bits else None

    def set_bytes(self, k, data):
        if not data:
            self.bits.pop(k, None)
            return
        b = self.O.BitString(len(data) + 16)
        b.buf[: len(data)] = np.frombuffer(data, dtype=np.uint8)
        b.len.value = len(data)
        self.bits[k] = b


def _check_state(engine, m):
    for k in HLL_KEYS:
        if k in m.hll.regs:
            np.testing.assert_array_equal(engine.hll_registers(k), m.hll.regs[k], err_msg=str(k))
        else:
            assert engine.key_type(k) == 0, k
    for k in BIT_KEYS:
        assert engine.get(k) == m.bytes_of(k), k


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_random_command_interleavings(engine, O, seed):
    engine.flushall()
    rng = np.random.default_rng(1000 + seed)
    pool = _pool(0x5EED0A00 + seed, 6000)
    m = Model(O)
    bf = b"fz:bloom"
    assert engine.bloom_try_init(bf, 20000, 0.02)
    size, k, _, _ = engine.bloom_config(bf)
    bloom = O.BitString()
    for step in range(300):
        op = rng.choice(["pfadd", "pfadd", "pfcount", "pfmerge", "setbit", "getbit", "range", "bitop", "read",
                         "del", "bloom_add", "bloom_contains"])
        if op == "pfadd":
            n = int(rng.integers(1, 2500))
            keys = [HLL_KEYS[i] for i in rng.integers(0, len(HLL_KEYS), n)]
            elems = [[pool[j] for j in rng.integers(0, len(pool), int(rng.integers(0, 5)))] for _ in range(n)]
            assert engine.pfadd(keys, elems) == m.hll.pfadd(keys, elems), step
        elif op == "pfcount":
            cmds = []
            for _ in range(int(rng.integers(1, 12))):
                nk = int(rng.integers(1, 4))
                cmds.append([HLL_KEYS[i] for i in rng.integers(0, len(HLL_KEYS), nk)] +
                            ([b"fz:missing"] if rng.random() < 0.2 else []))
            assert engine.pfcount(cmds) == [m.hll.count(c) for c in cmds], step
        elif op == "pfmerge":
            dest = HLL_KEYS[int(rng.integers(0, len(HLL_KEYS)))]
            srcs = [HLL_KEYS[i] for i in rng.integers(0, len(HLL_KEYS), int(rng.integers(1, 4)))] + [b"fz:missing"]
            engine.pfmerge(dest, [dest] + srcs)
            m.hll.merge(dest, [dest] + srcs)
        elif op == "setbit":
            n = int(rng.integers(1, 3000))
            keys = [BIT_KEYS[i] for i in rng.integers(0, len(BIT_KEYS), n)]
            hi = 1 << int(rng.choice([10, 16, 20]))
            offs = [int(x) for x in rng.integers(0, hi, n)]
            vals = [int(x) for x in rng.integers(0, 2, n)]
            got = engine.setbit(keys, offs, vals)
            assert list(got) == [m.bitstr(kk).setbit(o, v) for kk, o, v in zip(keys, offs, vals)], step
        elif op == "getbit":
            n = int(rng.integers(1, 3000))
            keys = [BIT_KEYS[i] for i in rng.integers(0, len(BIT_KEYS), n)]
            offs = [int(x) for x in rng.integers(0, 1 << 17, n)]
            want = [m.bits[kk].getbit(o) if kk in m.bits else 0 for kk, o in zip(keys, offs)]
            assert list(engine.getbit(keys, offs)) == want, step
        elif op == "range":
            kk = BIT_KEYS[int(rng.integers(0, len(BIT_KEYS)))]
            a = int(rng.integers(0, 1 << 15))
            b = a + int(rng.integers(0, 5000))
            v = int(rng.integers(0, 2))
            engine.set_bit_range(kk, a, b, v)
            for i in range(a, b):
                m.bitstr(kk).setbit(i, v)
        elif op == "bitop":
            name = str(rng.choice(["AND", "OR", "XOR", "NOT"]))
            dest = BIT_KEYS[int(rng.integers(0, len(BIT_KEYS)))]
            srcs = [BIT_KEYS[i] for i in rng.integers(0, len(BIT_KEYS), 1 if name == "NOT" else int(rng.integers(1, 4)))]
            want = O.bitop(name, [m.bytes_of(s) for s in srcs])
            assert engine.bitop(name, dest, srcs) == len(want), step
            m.set_bytes(dest, want)
        elif op == "read":
            kk = BIT_KEYS[int(rng.integers(0, len(BIT_KEYS)))]
            data = m.bytes_of(kk)
            assert engine.get(kk) == data, step
            assert engine.strlen(kk) == (len(data) if data else 0), step
            assert engine.bitcount(kk) == (m.bits[kk].bitcount() if data else 0), step
        elif op == "del":
            kk = (HLL_KEYS + BIT_KEYS)[int(rng.integers(0, len(HLL_KEYS) + len(BIT_KEYS)))]
            existed = kk in m.hll.regs or kk in m.bits
            assert engine.delete([kk]) == int(existed), step
            m.hll.regs.pop(kk, None)
            m.bits.pop(kk, None)
        elif op == "bloom_add":
            els = [pool[j] for j in rng.integers(0, len(pool), int(rng.integers(1, 3000)))]
            assert engine.bloom_add(bf, size, k, els) == bloom.bloom_add(size, k, els), step
        else:
            els = [pool[j] for j in rng.integers(0, len(pool), int(rng.integers(1, 3000)))]
            assert engine.bloom_contains(bf, size, k, els) == bloom.bloom_contains(size, k, els), step
        if step % 20 == 19:
            _check_state(engine, m)
    _check_state(engine, m)
    assert engine.get(bf) == bloom.bytes()
    # type errors leave the state untouched
    engine.pfadd([b"fz:typed:h"], [[b"x"]])
    engine.setbit([b"fz:typed:b"], [1], [1])
    with pytest.raises(RedisException):
        engine.setbit([b"fz:typed:h"], [1], [1])
    with pytest.raises(RedisException, match="HyperLogLog"):
        engine.pfadd([b"fz:typed:b"], [[b"x"]])
    _check_state(engine, m)
