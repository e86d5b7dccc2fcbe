"""Group commit of concurrently executed RBatches (redisson_amd/coalesce.py BatchCoalescer).

CPU tests run the coalescer over an oracle-backed engine stand-in (pfadd / pfadd_status / pfcount / key_type, and the
slab-id path the coalescer takes: key_types, hll_resolve, pfadd_ids_status; a PFADD on a key of another type fails
that command alone).  Expected results
come from running the same batches one after another through the oracle, in the FIFO order they were submitted:
merged PFADD-only batches must give every batch exactly its sequential replies, a batch with another command runs
on its own, and a WRONGTYPE command fails only the batch that holds it."""
import threading

import numpy as np
import pytest

from redisson_amd import _native as N
from redisson_amd.engine import RedisException
from redisson_amd.redisson import Config, RBatch, Redisson


class OracleHLLEngine:
    def __init__(self, strings=()):
        from oracle import oracle as O

        self.ref = O.HLLStore()
        self.strings = set(strings)
        self.calls = 0

    def pfadd_status(self, keys, elems):
        self.calls += 1
        out = np.zeros(len(keys), dtype=np.uint8)
        st, msg = N.SK_OK, ""
        for i, (k, es) in enumerate(zip(keys, elems)):
            if k in self.strings:
                st, msg = N.SK_EWRONGTYPE, "WRONGTYPE Key is not a valid HyperLogLog string value."
                continue
            out[i] = self.ref.pfadd([k], [es])[0]
        return st, out, msg

    def pfadd(self, keys, elems):
        st, out, msg = self.pfadd_status(keys, elems)
        if st:
            raise RedisException(msg)
        return [bool(x) for x in out]

    def pfcount(self, cmds):
        return [self.ref.count(list(c)) for c in cmds]

    def key_type(self, k):
        return N.SK_TYPE_STRING if k in self.strings else (N.SK_TYPE_HLL if k in self.ref.regs else N.SK_TYPE_NONE)

    # the slab-id path the coalescer uses (sk_type_many, sk_hll_resolve, sk_pfadd_ids)
    def key_types(self, keys):
        return np.array([self.key_type(k) for k in keys], dtype=np.int32)

    def hll_resolve(self, keys, with_created=False):
        self.slabs = getattr(self, "slabs", [])
        ids, cr = [], []
        for k in keys:
            if k in self.strings:
                raise RedisException("WRONGTYPE Key is not a valid HyperLogLog string value.")
            cr.append(k not in self.ref.regs)
            if cr[-1]:
                self.ref.regs[k] = np.zeros(16384, dtype=np.uint8)
                self.slabs.append(k)
            ids.append(self.slabs.index(k) if k in self.slabs else self._adopt(k))
        ids = np.array(ids, dtype=np.uint32)
        return (ids, np.array(cr, dtype=np.uint8)) if with_created else ids

    def _adopt(self, k):
        self.slabs.append(k)
        return len(self.slabs) - 1

    def pfadd_ids_status(self, ids, elems):
        self.calls += 1
        keys = [self.slabs[int(i)] for i in ids]
        if any(k not in self.ref.regs for k in keys):
            return N.SK_ESTALE, np.zeros(len(keys), np.uint8), "stale"
        return N.SK_OK, np.array(self.ref.pfadd(keys, elems), dtype=np.uint8), ""


class FakeClient:
    """The Redisson executor (_run_batch) over the stand-in engine, with a batch coalescer."""

    def __init__(self, engine):
        from redisson_amd.coalesce import BatchCoalescer

        self.config = Config()
        self.engine = engine
        self.batch_coalescer = BatchCoalescer(self)

    _run_batch = Redisson._run_batch

    def createBatch(self):
        return RBatch(self)

    def close(self):
        self.batch_coalescer.close()


def _fill(batch, seed, n, nkeys, count_at=None):
    rng = np.random.default_rng(seed)
    for i in range(n):
        batch.getHyperLogLog("t:%d" % rng.integers(0, nkeys)).addAsync(int(rng.integers(0, 1 << 62)))
        if count_at is not None and i == count_at:
            batch.getHyperLogLog("t:0").countAsync()


def _sequential(batches_spec, strings=()):
    """Each batch executed on its own, in order, through the plain executor (no coalescer)."""
    eng = OracleHLLEngine(strings)

    class Plain:
        config = Config()
        engine = eng
        _run_batch = Redisson._run_batch

    out = []
    for spec in batches_spec:
        b = RBatch(Plain())
        spec(b)
        try:
            out.append(("ok", b.execute()))
        except RedisException as e:
            out.append(("err", str(e)))
    return out, eng


def _coalesced(batches_spec, strings=()):
    eng = OracleHLLEngine(strings)
    cl = FakeClient(eng)
    try:
        with cl.batch_coalescer.hold():
            futs = []
            for spec in batches_spec:
                b = cl.createBatch()
                spec(b)
                futs.append(b.executeAsync())
        out = []
        for f in futs:
            try:
                out.append(("ok", f.get(30)))
            except RedisException as e:
                out.append(("err", str(e)))
        return out, eng, cl.batch_coalescer.calls
    finally:
        cl.close()


def test_pfadd_batches_merge_into_one_call():
    specs = [lambda b, s=s: _fill(b, s, 300, 40) for s in range(12)]
    want, weng = _sequential(specs)
    got, geng, calls = _coalesced(specs)
    assert calls == 1 and geng.calls == 1
    assert got == want
    for k in weng.ref.regs:
        np.testing.assert_array_equal(geng.ref.regs[k], weng.ref.regs[k])


def test_other_command_splits_the_group():
    specs = [lambda b, s=s: _fill(b, s, 200, 10, count_at=(50 if s == 3 else None)) for s in range(7)]
    want, _ = _sequential(specs)
    got, geng, calls = _coalesced(specs)
    assert got == want
    assert calls == 2           # batches 0-2 merged, batch 3 alone (PFCOUNT), batches 4-6 merged


def test_wrongtype_fails_only_its_batch():
    def bad(b):
        _fill(b, 99, 50, 5)
        b.getHyperLogLog("str").addAsync(7)
        _fill(b, 98, 50, 5)

    specs = [lambda b, s=s: _fill(b, s, 100, 5) for s in range(3)] + [bad] + \
            [lambda b, s=s: _fill(b, s, 100, 5) for s in range(3, 6)]
    want, weng = _sequential(specs, strings={"str"})
    got, geng, calls = _coalesced(specs, strings={"str"})
    assert calls == 1
    assert [g[0] for g in got] == [w[0] for w in want] == ["ok"] * 3 + ["err"] + ["ok"] * 3
    assert [g for g in got if g[0] == "ok"] == [w for w in want if w[0] == "ok"]
    for k in weng.ref.regs:
        np.testing.assert_array_equal(geng.ref.regs[k], weng.ref.regs[k])


def test_group_error_fails_group_and_thread_survives():
    """An exception inside the group's engine call (packing / encoding) fails every future of the group; the
    completion thread keeps serving later batches."""

    class Exploding(OracleHLLEngine):
        def pfadd_ids_status(self, ids, elems):
            if any(self.slabs[int(i)] == "boom" for i in ids):
                raise TypeError("cannot encode element")
            return super().pfadd_ids_status(ids, elems)

    cl = FakeClient(Exploding())
    try:
        b1 = cl.createBatch()
        _fill(b1, 1, 20, 3)
        f_cmd = b1.getHyperLogLog("boom").addAsync(5)
        f1 = b1.executeAsync()
        with pytest.raises(TypeError):
            f1.get(30)
        assert f_cmd.isDone() and not f_cmd.isSuccess()
        b2 = cl.createBatch()
        _fill(b2, 2, 20, 3)
        assert len(b2.executeAsync().get(30)) == 20
    finally:
        cl.close()


def test_cached_ids_survive_and_recover_from_delete():
    """Groups after the first use cached slab handles (no name resolution); a key deleted between groups makes
    the cached handle stale: the coalescer drops its cache, resolves again, and the command that re-creates the
    key replies 1 (PFADD on a missing key creates it)."""
    eng = OracleHLLEngine()
    cl = FakeClient(eng)
    try:
        b = cl.createBatch()
        _fill(b, 7, 50, 4)
        b.executeAsync().get(30)
        n_slabs = len(eng.slabs)
        b = cl.createBatch()
        _fill(b, 8, 50, 4)
        b.executeAsync().get(30)
        assert len(eng.slabs) == n_slabs            # every key came from the cache
        del eng.ref.regs["t:1"]                     # DEL t:1 behind the coalescer's back
        b = cl.createBatch()
        f = b.getHyperLogLog("t:1").addAsync(12345)
        b.getHyperLogLog("t:1").addAsync(12345)
        b.executeAsync().get(30)
        assert f.get() is True and "t:1" in eng.ref.regs
    finally:
        cl.close()


def test_concurrent_threads_each_get_sequential_replies():
    """Threads execute batches concurrently; the coalescer linearizes them in FIFO order: replaying the batches in
    that order (the order the coalescer completed them in is not observable, so each batch is checked on its own
    keys, disjoint per thread)."""
    eng = OracleHLLEngine()
    cl = FakeClient(eng)
    res = {}
    try:
        def worker(t):
            outs = []
            for r in range(5):
                b = cl.createBatch()
                _fill_keys = np.random.default_rng(t * 100 + r)
                for i in range(200):
                    b.getHyperLogLog("th:%d:%d" % (t, _fill_keys.integers(0, 4))).addAsync(
                        int(_fill_keys.integers(0, 1 << 62)))
                outs.append(b.execute())
            res[t] = outs

        th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        cl.close()
    # per thread: its batches ran in its own order on its own keys, so its replies are the sequential ones
    for t in range(6):
        def spec_of(r, t=t):
            def spec(b):
                g = np.random.default_rng(t * 100 + r)
                for i in range(200):
                    b.getHyperLogLog("th:%d:%d" % (t, g.integers(0, 4))).addAsync(int(g.integers(0, 1 << 62)))
            return spec
        want, _ = _sequential([spec_of(r) for r in range(5)])
        assert [("ok", x) for x in res[t]] == want


@pytest.mark.gpu
def test_coalesced_batches_on_engine(O):
    """Redisson with Config(batch_coalesce=True) on the GPU: 20 held PFADD batches become one sk_pfadd call, with
    the oracle's sequential replies and registers."""
    cl = Redisson.create(Config(batch_coalesce=True))
    try:
        specs = [lambda b, s=s: _fill(b, s, 500, 30) for s in range(20)]
        want, weng = _sequential(specs)
        with cl.batch_coalescer.hold():
            futs = []
            for spec in specs:
                b = cl.createBatch()
                spec(b)
                futs.append(b.executeAsync())
        got = [("ok", f.get(60)) for f in futs]
        assert got == want
        assert cl.batch_coalescer.calls == 1
        for k, r in weng.ref.regs.items():
            np.testing.assert_array_equal(cl.engine.hll_registers(k), r)
    finally:
        cl.shutdown()

