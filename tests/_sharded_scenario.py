"""Cross-GPU RBitSet / BITOP scenario shared by the multi-rank tests (redisson_amd/cluster.py).

`run_scenario(engine, rank, world, coll)` drives ShardedBitSet and keyed_bitop SPMD-style and returns what every
rank observed; `expected()` computes the same with the oracle in one process (the single redis-server the
reference talks to).  The CPU test runs it with an oracle-backed engine on gloo (world 2); the GPU tests with
SketchEngine contexts (RCCL at world 1, gloo between two processes sharing the GPU at world 2).
"""
import numpy as np

NBITS = 1 << 20
KEYS = [b"kb:%d" % i for i in range(6)]


def _offsets(seed, n):
    return np.random.default_rng(seed).integers(0, NBITS, n, dtype=np.uint64)


HKEYS = [b"hk:%d" % i for i in range(24)]
HN = [37 * i + 5 for i in range(24)]


def _hll_elems(i):
    return [b'["java.lang.Long",%d]' % (i * 100_003 + j) for j in range(HN[i])]


def run_scenario(engine, rank, world, coll):
    from redisson_amd.cluster import ShardedBitSet, keyed_bitop
    from redisson_amd import owner

    out = {}
    a = ShardedBitSet(engine, b"sb:a", NBITS, rank, world, coll)
    b = ShardedBitSet(engine, b"sb:b", NBITS, rank, world, coll)
    c = ShardedBitSet(engine, b"sb:c", NBITS, rank, world, coll)
    oa = _offsets(1, 3000)
    oa[0] = NBITS - 1                       # the last byte of the string

    def mine(x):                            # this rank's part of a batch: rank r submits the r-th slice
        return x[rank * len(x) // world:(rank + 1) * len(x) // world]

    def gathered(rep):                      # every rank's replies, in rank order (= the whole batch's order)
        return [int(v) for part in coll.allgather_bytes(np.asarray(rep, np.uint8).tobytes()) for v in part]

    out["set_a"] = gathered(a.set(mine(oa), 1))      # repeats inside the batch: second SETBIT of a bit replies 1
    out["set_b"] = gathered(b.set(mine(_offsets(2, 2000)[:1000]), 1))   # b ends early: shorter than a
    vals = (np.arange(500) % 3 == 0).astype(np.uint8)   # clear most of them, set every third again
    out["clear_a"] = gathered(a.set(mine(oa[:500]), mine(vals)))
    out["get_a"] = gathered(a.get(mine(np.concatenate([oa[:800], _offsets(3, 800)]))))
    try:
        a.set(mine(np.array([NBITS + 8 * 64 * world], dtype=np.uint64)) if rank == world - 1 else [], 1)
        out["range_err"] = False
    except Exception as e:                  # one rank's bad offset fails the call on every rank, none blocks
        out["range_err"] = "out of range" in str(e) or "failed" in str(e)
    out["range_err"] = all(x == b"1" for x in coll.allgather_bytes(b"1" if out["range_err"] else b"0"))
    out["card"] = [a.cardinality(), b.cardinality(), c.cardinality()]
    out["len"] = [a.length_bytes(), b.length_bytes(), c.length_bytes()]
    out["size"] = a.size()
    out["bytes_a"] = a.to_bytes()
    a2 = ShardedBitSet(engine, b"sb:a2", NBITS, rank, world, coll)
    a2.set(mine(oa[500:]), 1)
    a2.op("AND", [b])
    out["and"] = a2.to_bytes()
    a3 = ShardedBitSet(engine, b"sb:a3", NBITS, rank, world, coll)
    a3.set(mine(oa[500:]), 1)
    a3.op("OR", [b, c])                      # c is empty (missing on every rank)
    out["or"] = a3.to_bytes()
    a4 = ShardedBitSet(engine, b"sb:a4", NBITS, rank, world, coll)
    a4.set(mine(_offsets(2, 2000)[:1000]), 1)
    a4.op("XOR", [b])                        # equal strings: an all-zero result of b's length
    out["xor"] = a4.to_bytes()
    b.op("NOT")                              # shards before b's last byte are padded, then inverted
    out["not_b"] = b.to_bytes()
    out["card_not_b"] = b.cardinality()

    # whole keys on their owners: BITOP across GPUs by one all-gather + a local op
    for i, k in enumerate(KEYS[:5]):
        if owner(k, world) == rank:
            offs = _offsets(10 + i, 300 + 200 * i) % np.uint64(NBITS >> (i % 3))
            engine.setbit([k] * len(offs), offs, [1] * len(offs), want_old=False)
    res = {}
    for op, dest, srcs in (("OR", b"kd:or", KEYS[:5]), ("AND", b"kd:and", KEYS[:3]),
                           ("XOR", b"kd:xor", [KEYS[1], KEYS[4], KEYS[5]]), ("NOT", b"kd:not", [KEYS[2]])):
        n = keyed_bitop(engine, op, dest, srcs, rank, world, coll)
        val = engine.get(dest) if owner(dest, world) == rank else None
        res[op] = (n, val)
    out["keyed"] = res

    # a failure on one rank only (the owner of KEYS[0] cannot read its length) raises on every rank instead of
    # leaving the other ranks in the next collective (cluster.agree)
    class _FailOn:
        def __init__(self, e, key):
            self.e, self.key = e, key

        def __getattr__(self, a):
            return getattr(self.e, a)

        def strlen(self, k):
            if bytes(k) == self.key:
                raise RuntimeError("injected strlen failure")
            return self.e.strlen(k)

    try:
        keyed_bitop(_FailOn(engine, KEYS[0]), "OR", b"kd:fail", KEYS[:3], rank, world, coll)
        out["keyed_agree"] = False
    except Exception as e:  # noqa: BLE001 - both the failing rank and the others must raise
        out["keyed_agree"] = "injected" in str(e)
    out["keyed_after"] = keyed_bitop(engine, "OR", b"kd:or2", KEYS[:2], rank, world, coll)   # still in step

    # C4: HLLs sharded by calcSlot % world, each rank adding only the keys it owns; global countWith / PFMERGE by
    # local union + u8 MAX exchange, by key names and by a cached device slab-id set (GlobalKeySet)
    from redisson_amd.cluster import GlobalKeySet, global_count_with, global_merge
    for i, k in enumerate(HKEYS):
        if owner(k, world) == rank:
            engine.pfadd([k] * HN[i], [[e] for e in _hll_elems(i)])
    hk = HKEYS + [b"hk:absent"]
    out["count_with"] = global_count_with(engine, hk, rank, world, coll)
    ks = GlobalKeySet(engine, hk, rank, world)
    out["count_with_ids"] = [global_count_with(engine, ks, rank, world, coll) for _ in range(2)]
    resolves = ks.resolves
    extra = b"hk:late"                          # created after the set was resolved: the next call includes it
    if owner(extra, world) == rank:
        engine.pfadd([extra] * 50, [[b"late:%d" % j] for j in range(50)])
    ks2 = GlobalKeySet(engine, hk + [extra], rank, world)
    ks2.ids()
    if owner(extra, world) == rank:
        engine.pfadd([extra] * 50, [[b"late2:%d" % j] for j in range(50)])   # registers change, no new key
    out["count_with_late"] = global_count_with(engine, ks2, rank, world, coll)
    out["id_set_cached"] = resolves == 1 and ks2.resolves == 1
    global_merge(engine, b"hk:dest", ks, rank, world, coll)
    global_merge(engine, b"hk:dest", [HKEYS[0]], rank, world, coll)          # dest kept in the max
    out["merge_dest"] = engine.hll_registers(b"hk:dest") if owner(b"hk:dest", world) == rank else None

    # one Bloom filter served by every rank (replicas): adds on all, contains split and gathered
    from redisson_amd.cluster import ReplicatedBloom
    bf = ReplicatedBloom(engine, b"rb:c3", rank, world, coll)
    bf.try_init(20000, 0.01)
    adds = [b'["java.lang.Long",%d]' % i for i in range(3000)]
    out["bloom_add"] = [bool(x) for x in bf.add(adds[:2000])] + [bool(x) for x in bf.add(adds[1000:])]
    probe = [b'["java.lang.Long",%d]' % i for i in range(0, 6000, 3)]
    out["bloom_contains"] = [bool(x) for x in bf.contains(probe)]
    return out


def expected():
    """The same commands against one oracle store (what one redis-server holds)."""
    from oracle import oracle as O

    s = {}

    def bs(k):
        return s.setdefault(k, O.BitString(NBITS // 8 + 16))

    def setbits(k, offs, v):
        return [bs(k).setbit(int(o), v) for o in offs]

    out = {}
    oa = _offsets(1, 3000)
    oa[0] = NBITS - 1
    out["set_a"] = setbits(b"a", oa, 1)
    ob = _offsets(2, 2000)[:1000]
    out["set_b"] = setbits(b"b", ob, 1)
    vals = (np.arange(500) % 3 == 0).astype(np.uint8)
    out["clear_a"] = [bs(b"a").setbit(int(o), int(v)) for o, v in zip(oa[:500], vals)]
    out["range_err"] = True
    out["get_a"] = [bs(b"a").getbit(int(o)) for o in np.concatenate([oa[:800], _offsets(3, 800)])]
    out["card"] = [bs(b"a").bitcount(), bs(b"b").bitcount(), 0]
    out["len"] = [len(bs(b"a").bytes()), len(bs(b"b").bytes()), 0]
    out["size"] = len(bs(b"a").bytes()) * 8
    out["bytes_a"] = bs(b"a").bytes()
    setbits(b"a2", oa[500:], 1)
    out["and"] = O.bitop("AND", [bs(b"a2").bytes(), bs(b"b").bytes()])
    setbits(b"a3", oa[500:], 1)
    out["or"] = O.bitop("OR", [bs(b"a3").bytes(), bs(b"b").bytes(), None])
    setbits(b"a4", ob, 1)
    out["xor"] = O.bitop("XOR", [bs(b"a4").bytes(), bs(b"b").bytes()])
    nb = O.bitop("NOT", [bs(b"b").bytes()])
    out["not_b"] = nb
    out["card_not_b"] = int(np.unpackbits(np.frombuffer(nb, np.uint8)).sum())
    keys = {}
    for i, k in enumerate(KEYS[:5]):
        offs = _offsets(10 + i, 300 + 200 * i) % np.uint64(NBITS >> (i % 3))
        setbits(k, offs, 1)
        keys[k] = bs(k).bytes()
    res = {}
    for op, dest, srcs in (("OR", b"kd:or", KEYS[:5]), ("AND", b"kd:and", KEYS[:3]),
                           ("XOR", b"kd:xor", [KEYS[1], KEYS[4], KEYS[5]]), ("NOT", b"kd:not", [KEYS[2]])):
        v = O.bitop(op, [keys.get(k) for k in srcs])
        res[op] = (len(v), v if v else None)
    out["keyed"] = res
    out["keyed_agree"] = True
    out["keyed_after"] = len(O.bitop("OR", [keys.get(k) for k in KEYS[:2]]))
    h = O.HLLStore()
    for i, k in enumerate(HKEYS):
        h.pfadd([k] * HN[i], [[e] for e in _hll_elems(i)])
    union = np.maximum.reduce([h.regs[k] for k in HKEYS])
    out["count_with"] = O.count_regs(union, 2, 3)
    out["count_with_ids"] = [out["count_with"]] * 2
    h.pfadd([b"hk:late"] * 50, [[b"late:%d" % j] for j in range(50)])
    h.pfadd([b"hk:late"] * 50, [[b"late2:%d" % j] for j in range(50)])
    out["count_with_late"] = O.count_regs(np.maximum(union, h.regs[b"hk:late"]), 2, 3)
    out["id_set_cached"] = True
    out["merge_dest"] = union
    m = O.bloom_optimal_bits(20000, 0.01)
    kk = O.bloom_optimal_k(20000, m)
    b = O.BitString(16)
    adds = [b'["java.lang.Long",%d]' % i for i in range(3000)]
    out["bloom_add"] = [bool(x) for x in b.bloom_add(m, kk, adds[:2000])] + \
        [bool(x) for x in b.bloom_add(m, kk, adds[1000:])]
    out["bloom_contains"] = [bool(x) for x in b.bloom_contains(m, kk, [b'["java.lang.Long",%d]' % i
                                                                      for i in range(0, 6000, 3)])]
    return out


def check(got, want, rank, world):
    from redisson_amd import owner

    assert got["range_err"], "an out-of-range offset on one rank must fail the call on every rank"
    for k in ("set_a", "set_b", "clear_a", "get_a"):
        assert [int(x) for x in got[k]] == [int(x) for x in want[k]], k
    for k in ("card", "len", "size", "bytes_a", "and", "or", "xor", "not_b", "card_not_b", "bloom_add",
              "bloom_contains", "count_with", "count_with_ids", "count_with_late", "id_set_cached", "keyed_agree",
              "keyed_after"):
        assert got[k] == want[k], k
    if owner(b"hk:dest", world) == rank:
        np.testing.assert_array_equal(got["merge_dest"], want["merge_dest"])
    for op, (n, val) in want["keyed"].items():
        gn, gval = got["keyed"][op]
        assert gn == n, op
        dest = {"OR": b"kd:or", "AND": b"kd:and", "XOR": b"kd:xor", "NOT": b"kd:not"}[op]
        if owner(dest, world) == rank:
            assert gval == val, op


class HostBuf:
    """A 'device buffer' of the oracle engine: host bytes with the DeviceBuffer methods the protocols use."""

    def __init__(self, nbytes):
        self.a = np.zeros(nbytes, dtype=np.uint8)

    def upload(self, arr, offset=0):
        b = np.ascontiguousarray(arr).view(np.uint8).ravel()
        self.a[offset:offset + len(b)] = b

    def download(self, dtype=np.uint8, count=-1, offset=0):
        v = self.a[offset:].view(dtype)
        return (v if count < 0 else v[:count]).copy()

    def zero(self):
        self.a[:] = 0
        return self

    def free(self):
        pass

    def view(self, offset, nbytes=-1):
        v = HostBuf(0)
        v.a = self.a[offset:] if nbytes < 0 else self.a[offset:offset + nbytes]
        return v


class OracleBitEngine:
    """The engine methods the cluster protocols call, over oracle bit strings and HLLs (CPU tests only)."""

    def __init__(self):
        from oracle import oracle as O

        self.O = O
        self.s = {}
        self.h = O.HLLStore()
        self.epoch = 0
        self.slab = {}          # HLL key -> slab id (index into self.slabs)
        self.slabs = []

    def _bs(self, k):
        return self.s.setdefault(bytes(k), self.O.BitString(16))

    def key_type(self, k):
        return 2 if bytes(k) in self.s else (1 if bytes(k) in self.h.regs else 0)

    # -------- HLL (SketchEngine signatures)
    def _hll(self, k):
        k = bytes(k)
        if k not in self.slab:
            self.slab[k] = len(self.slabs)
            self.slabs.append(k)
            self.epoch += 1
        return k

    def pfadd(self, keys, elems):
        return self.h.pfadd([self._hll(k) for k in keys], elems)

    def hll_registers(self, k):
        return self.h.regs.get(bytes(k), np.zeros(16384, np.uint8)).copy()

    def hll_epoch(self):
        return self.epoch

    def hll_lookup(self, keys):
        if isinstance(keys, tuple):
            off, buf = keys
            keys = [buf[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)]
        return np.array([self.slab.get(bytes(k), 0xFFFFFFFF) for k in keys], dtype=np.uint32)

    def alloc(self, nbytes):
        return HostBuf(nbytes)

    def to_device(self, arr, pad=0):
        b = HostBuf(np.ascontiguousarray(arr).nbytes + pad)
        b.upload(arr)
        return b

    def d2d(self, dst, src, n):
        dst.a[:n] = src.a[:n]

    # -------- the range-sharded / replicated Bloom filter's device steps
    @staticmethod
    def _elems(n, d_off, d_bytes):
        off = d_off.download(np.uint64, n + 1)
        raw = d_bytes.a
        return [raw[int(off[i]):int(off[i + 1])].tobytes() for i in range(n)]

    def bloom_indexes_dev(self, n, d_off, d_bytes, size, k, nprobe, d_idx):
        if n and nprobe:
            idx = [self.O.bloom_indexes(e, k, size)[:nprobe] for e in self._elems(n, d_off, d_bytes)]
            d_idx.upload(np.asarray(idx, dtype=np.uint64).ravel())

    def reduce_groups_u8(self, n, group, take, invert, d_in, d_out):
        v = d_in.download(np.uint8, n * group).reshape(n, group)[:, :take] if group else np.zeros((n, 0), np.uint8)
        d_out.upload((v.all(axis=1) ^ bool(invert)).astype(np.uint8))

    def bloom_contains_dev(self, name, n, d_off, d_bytes, bytes_len, d_out):
        size, k, _, _ = self.bloom_config(name)
        d_out.upload(np.asarray(self.bloom_contains(name, size, k, self._elems(n, d_off, d_bytes)), np.uint8))

    def hll_union_dev(self, n, d_ids, d_out):
        ids = d_ids.download(np.uint32, n)
        u = np.zeros(16384, np.uint8)
        for i in ids:
            np.maximum(u, self.h.regs[self.slabs[int(i)]], out=u)
        d_out.upload(u)

    def hll_union_keys(self, keys, world, rank, d_out):
        from redisson_amd import owner
        if isinstance(keys, tuple):
            off, buf = keys
            keys = [buf[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)]
        u = np.zeros(16384, np.uint8)
        used = 0
        for k in keys:
            if owner(k, world) == rank and bytes(k) in self.h.regs:
                np.maximum(u, self.h.regs[bytes(k)], out=u)
                used += 1
        d_out.upload(u)
        return used

    def hll_count_registers_dev(self, d_regs):
        return self.O.count_regs(d_regs.download(np.uint8, 16384), 2, 3)

    def hll_merge_registers_dev(self, key, d_regs):
        k = self._hll(key)
        r = self.h.regs.setdefault(k, np.zeros(16384, np.uint8))
        np.maximum(r, d_regs.download(np.uint8, 16384), out=r)

    def setbit(self, keys, offsets, values, want_old=True):
        vals = np.broadcast_to(np.asarray(values, dtype=np.uint8), (len(keys),))
        old = [self._bs(k).setbit(int(o), int(v)) for k, o, v in zip(keys, offsets, vals)]
        return old if want_old else None

    def getbit(self, keys, offsets):
        return [self.s[bytes(k)].getbit(int(o)) if bytes(k) in self.s else 0 for k, o in zip(keys, offsets)]

    def strlen(self, k):
        return len(self.s[bytes(k)].bytes()) if bytes(k) in self.s else 0

    def bitcount(self, k):
        return self.s[bytes(k)].bitcount() if bytes(k) in self.s else 0

    def get(self, k):
        return self.s[bytes(k)].bytes() if bytes(k) in self.s else None

    def set(self, k, v):
        b = self.O.BitString(len(v) + 16)
        b.buf[:len(v)] = np.frombuffer(bytes(v), np.uint8)
        b.len.value = len(v)
        self.s[bytes(k)] = b

    def delete(self, keys):
        n = 0
        for k in keys:
            n += self.s.pop(bytes(k), None) is not None
        return n

    def bloom_try_init(self, name, n, p):
        m = self.O.bloom_optimal_bits(n, p)
        self.cfg = getattr(self, "cfg", {})
        fresh = bytes(name) not in self.cfg
        self.cfg[bytes(name)] = (m, self.O.bloom_optimal_k(n, m), n, p)
        return fresh

    def bloom_config(self, name):
        return self.cfg[bytes(name)]

    def bloom_add(self, name, size, k, elems):
        return self._bs(name).bloom_add(size, k, elems)

    def bloom_contains(self, name, size, k, elems):
        b = self.s.get(bytes(name))
        return b.bloom_contains(size, k, elems) if b else [False] * len(elems)

    def bitop(self, op, dest, srcs):
        v = self.O.bitop(op.upper(), [self.get(k) for k in srcs])
        if v:
            self.set(dest, v)
        else:
            self.s.pop(bytes(dest), None)
        return len(v)

    # -------- the device router's engine steps (sk_route_bits / sk_unroute_u8 / *_dev), over HostBufs
    def route_bits(self, n, d_offsets, d_values, shard_bits, world, d_send, d_send_values, d_dst):
        from redisson_amd.engine import RedisException
        offs = d_offsets.download(np.uint64, n) if n else np.zeros(0, np.uint64)
        sh = (offs // np.uint64(shard_bits)).astype(np.int64)
        if (sh >= world).any():
            raise RedisException("ERR bit offset is not an integer or out of range")
        order = np.argsort(sh, kind="stable")
        if n:
            d_send.upload(offs[order] - sh[order].astype(np.uint64) * np.uint64(shard_bits))
            if d_values is not None:
                d_send_values.upload(d_values.download(np.uint8, n)[order])
            pos = np.empty(n, dtype=np.uint32)
            pos[order] = np.arange(n, dtype=np.uint32)
            d_dst.upload(pos)
        return np.bincount(sh, minlength=world).astype(np.uint64)

    def unroute_u8(self, n, d_dst, d_rep, d_out):
        d_out.upload(d_rep.download(np.uint8, -1)[d_dst.download(np.uint32, n)])

    def setbit_dev(self, key, n, d_offsets, value, d_out_old=None):
        old = self.setbit([key] * n, d_offsets.download(np.uint64, n), [value] * n)
        if d_out_old is not None:
            d_out_old.upload(np.asarray(old, np.uint8))

    def setbit_values_dev(self, key, n, d_offsets, d_values, d_out_old=None):
        old = self.setbit([key] * n, d_offsets.download(np.uint64, n), d_values.download(np.uint8, n))
        if d_out_old is not None:
            d_out_old.upload(np.asarray(old, np.uint8))

    def getbit_dev(self, key, n, d_offsets, d_out):
        d_out.upload(np.asarray(self.getbit([key] * n, d_offsets.download(np.uint64, n)), np.uint8))


class HostDevCollective:
    """HostCollective plus the RCCL collective's device-buffer calls (alltoallv_dev, allgather_dev) through the
    buffers' download / upload and gloo, so the device protocols (ShardedBitSet's router, RangeShardedBloom,
    ReplicatedBloom.contains_dev) run on an OracleBitEngine on the CPU and on engine contexts sharing one GPU."""

    def __init__(self, dist):
        from redisson_amd.cluster import HostCollective
        self.h = HostCollective(dist)

    def __getattr__(self, a):
        return getattr(self.h, a)

    def alltoallv_dev(self, send, send_bytes, recv, recv_bytes):
        sb = np.asarray(send_bytes, dtype=np.int64)
        cut = np.concatenate([[0], np.cumsum(sb)])
        flat_send = send.download(np.uint8, int(cut[-1])) if cut[-1] else np.zeros(0, np.uint8)
        got = self.h.alltoallv_bytes([flat_send[cut[p]:cut[p + 1]].tobytes() for p in range(len(sb))])
        assert [len(g) for g in got] == [int(x) for x in recv_bytes], "alltoallv sizes disagree"
        flat = b"".join(got)
        if flat:
            recv.upload(np.frombuffer(flat, np.uint8))

    def allgather_dev(self, send, recv, nbytes):
        parts = self.h.allgather_bytes(send.download(np.uint8, nbytes).tobytes())
        recv.upload(np.frombuffer(b"".join(parts), np.uint8))


def run_route_mix(engine, rank, world, coll):
    """ranks calling the device router with different call shapes.  Rank r sets (r even) or clears (r odd)
    its slice of one offset list; then rank 0 asks for no replies while the others do; then rank 0 passes per-op
    values while the others pass one value.  Every rank's replies are gathered in rank order."""
    from redisson_amd.cluster import ShardedBitSet

    bs = ShardedBitSet(engine, b"sb:mix", NBITS, rank, world, coll)
    offs = _offsets(21, 2400)
    offs[:300] = offs[300:600]                    # bits touched by both ranks' slices
    mine = offs[rank * len(offs) // world:(rank + 1) * len(offs) // world]
    out = {}

    def run(value, d_values=None, want=True):
        n = len(mine)
        d_off, d_rep = engine.to_device(mine), engine.alloc(max(n, 1))
        dv = engine.to_device(d_values) if d_values is not None else None
        bs.set_dev(n, d_off, d_rep if want else None, value=value, d_values=dv)
        rep = d_rep.download(np.uint8, n) if want else np.zeros(0, np.uint8)
        for b in (d_off, d_rep, dv):
            if b is not None:
                b.free()
        return [int(v) for part in coll.allgather_bytes(rep.tobytes()) for v in part]

    out["mixed_values"] = run(1 if rank % 2 == 0 else 0)
    out["void_on_rank0"] = run(1, want=rank != 0)
    pv = (np.arange(len(mine)) % 2).astype(np.uint8)
    out["per_op_on_rank0"] = run(0, d_values=pv if rank == 0 else None)
    out["bytes"] = bs.to_bytes()
    try:
        if rank == 0:
            bs.get_dev(0, engine.alloc(8), engine.alloc(8))
        else:
            bs.set_dev(0, engine.alloc(8), engine.alloc(8))
        out["op_mismatch"] = False
    except Exception as e:  # noqa: BLE001 - every rank must raise
        out["op_mismatch"] = "different routed operations" in str(e)
    return out


def expected_route_mix(world):
    from oracle import oracle as O

    b = O.BitString(NBITS // 8 + 16)
    offs = _offsets(21, 2400)
    offs[:300] = offs[300:600]
    slices = [offs[r * len(offs) // world:(r + 1) * len(offs) // world] for r in range(world)]
    out = {"mixed_values": [], "void_on_rank0": [], "per_op_on_rank0": []}
    for r, s in enumerate(slices):                # owners apply in (submitting rank, position) order
        out["mixed_values"] += [b.setbit(int(o), 1 if r % 2 == 0 else 0) for o in s]
    for r, s in enumerate(slices):
        rep = [b.setbit(int(o), 1) for o in s]
        out["void_on_rank0"] += rep if r != 0 else []
    for r, s in enumerate(slices):
        vals = (np.arange(len(s)) % 2).astype(np.uint8) if r == 0 else np.zeros(len(s), np.uint8)
        out["per_op_on_rank0"] += [b.setbit(int(o), int(v)) for o, v in zip(s, vals)]
    out["bytes"] = b.bytes()
    out["op_mismatch"] = world > 1
    return out


BLOOM_ADDS = [b'["java.lang.Long",%d]' % (i * 7919) for i in range(3000)]
BLOOM_PROBE = [b'["java.lang.Long",%d]' % (i * 7919) for i in range(0, 6000, 3)] + [b'"x%d"' % i for i in range(500)]


def run_bloom_shard(engine, rank, world, coll):
    """one filter range-sharded over the ranks (RangeShardedBloom: adds and contains submitted on
    every rank, routed to the bits' owners) and one replicated filter answering a device batch (contains_dev)."""
    from redisson_amd.cluster import RangeShardedBloom, ReplicatedBloom
    from redisson_amd.engine import pack

    def mine(x):
        return x[rank * len(x) // world:(rank + 1) * len(x) // world]

    def gathered(rep):
        return [bool(v) for part in coll.allgather_bytes(np.asarray(rep, np.uint8).tobytes()) for v in part]

    out = {}
    rb = RangeShardedBloom(engine, b"rsb:c3", rank, world, coll)
    out["init"] = [rb.try_init(20000, 0.01), rb.try_init(20000, 0.01)]
    out["cfg"] = (rb.size, rb.k)
    out["add1"] = gathered(rb.add(mine(BLOOM_ADDS[:2000])))
    out["add2"] = gathered(rb.add(mine(BLOOM_ADDS[1000:])))   # repeats reply False
    out["contains"] = gathered(rb.contains(mine(BLOOM_PROBE)))
    out["empty"] = rb.contains([])                            # an empty batch on every rank
    out["bytes"] = rb.to_bytes()
    out["count"] = rb.count()
    # Q6: a re-init replaces the config and keeps the one global bit string -- bit i stays bit i, both
    # when the first shard layout still covers the new size and when a larger filter needs a wider layout
    out["reinit_small"] = rb.try_init(2000, 0.01)
    out["bytes_small"] = rb.to_bytes()
    out["reinit_big"] = rb.try_init(200000, 0.01)
    out["bytes_big"] = rb.to_bytes()
    out["cfg_big"] = (rb.size, rb.k)
    out["contains_big"] = gathered(rb.contains(mine(BLOOM_PROBE)))
    rp = ReplicatedBloom(engine, b"rpb:c3", rank, world, coll)
    rp.try_init(20000, 0.01)
    rp.add(BLOOM_ADDS[:1500])
    off, buf = pack(BLOOM_PROBE)
    d_off, d_bytes, d_out = engine.to_device(off), engine.to_device(buf, pad=16), engine.alloc(len(BLOOM_PROBE))
    rp.contains_dev(len(BLOOM_PROBE), d_off, d_bytes, int(off[-1]), d_out)
    out["rep_contains_dev"] = [bool(v) for v in d_out.download(np.uint8, len(BLOOM_PROBE))]
    for b in (d_off, d_bytes, d_out):
        b.free()
    return out


def expected_bloom_shard():
    from oracle import oracle as O

    m = O.bloom_optimal_bits(20000, 0.01)
    k = O.bloom_optimal_k(20000, m)
    b = O.BitString(16)
    out = {"init": [True, False], "cfg": (m, k)}
    out["add1"] = [bool(x) for x in b.bloom_add(m, k, BLOOM_ADDS[:2000])]
    out["add2"] = [bool(x) for x in b.bloom_add(m, k, BLOOM_ADDS[1000:])]
    out["contains"] = [bool(x) for x in b.bloom_contains(m, k, BLOOM_PROBE)]
    out["empty"] = []
    out["bytes"] = b.bytes()
    out["count"] = O.bloom_count(m, k, b.bitcount())
    out["reinit_small"], out["bytes_small"] = False, b.bytes()
    m2 = O.bloom_optimal_bits(200000, 0.01)
    k2 = O.bloom_optimal_k(200000, m2)
    out["reinit_big"], out["bytes_big"], out["cfg_big"] = False, b.bytes(), (m2, k2)
    out["contains_big"] = [bool(x) for x in b.bloom_contains(m2, k2, BLOOM_PROBE)]
    r = O.BitString(16)
    r.bloom_add(m, k, BLOOM_ADDS[:1500])
    out["rep_contains_dev"] = [bool(x) for x in r.bloom_contains(m, k, BLOOM_PROBE)]
    return out
