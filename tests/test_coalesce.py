"""Group commit of concurrent RBloomFilter calls (redisson_amd/coalesce.py).

CPU tests drive the coalescer over an oracle-backed engine stand-in (the same bloom_add / bloom_contains
signature, config check included); the GPU test drives RBloomFilter with Config(bloom_coalesce=True) on the
engine.  Replies are checked against the oracle replaying the coalescer's own execution log (the FIFO order the
requests were linearized in), so concurrent adds are exact too.
"""
import threading

import numpy as np
import pytest

from redisson_amd.engine import RedisException

SIZE, K = 1 << 20, 7


class OracleBloomEngine:
    """bloom_add / bloom_contains over oracle bit strings, with the addConfigCheck of the engine."""

    def __init__(self):
        from oracle import oracle as O

        self.O = O
        self.bits = {}
        self.cfg = {}
        self.calls = 0

    def _check(self, name, size, k):
        if self.cfg.get(name, (SIZE, K)) != (size, k):
            raise RedisException("ERR Error running script: Bloom filter config has been changed")

    def bloom_add(self, name, size, k, elems):
        self._check(name, size, k)
        self.calls += 1
        return self.bits.setdefault(name, self.O.BitString(16)).bloom_add(size, k, elems)

    def bloom_contains(self, name, size, k, elems):
        self._check(name, size, k)
        self.calls += 1
        b = self.bits.get(name)
        return b.bloom_contains(size, k, elems) if b else [False] * len(elems)

    def bloom_prefix(self, op, name, size, k, prefix, suffixes):  # the prefix form: elements = prefix + suffix
        self.prefix_calls = getattr(self, "prefix_calls", 0) + 1
        elems = [prefix + x for x in suffixes]
        return (self.bloom_add if op == "add" else self.bloom_contains)(name, size, k, elems)


def _elem(t, i):
    return b'["java.lang.Long",%d]' % (t * 1_000_003 + i)


def _replay(log, size=SIZE, k=K):
    """The oracle over the logged runs in execution order: {request future: its replies}."""
    from oracle import oracle as O

    b = O.BitString(16)
    out = {}
    for kind, reqs in log:
        for elems, fut in reqs:
            out[id(fut)] = b.bloom_add(size, k, elems) if kind == "add" else b.bloom_contains(size, k, elems)
    return out, b


def test_held_requests_merge_into_one_call():
    from redisson_amd.coalesce import BloomCoalescer

    eng = OracleBloomEngine()
    co = BloomCoalescer(eng, record=True)
    try:
        futs = []
        with co.hold():
            for t in range(16):
                futs.append(co.submit(b"bf", "add", SIZE, K, [_elem(t, i) for i in range(50)]))
        got = [f.get(30) for f in futs]
        assert co.calls == 1 and eng.calls == 1 and co.requests == 16
        want, _ = _replay(co.log)
        assert [want[id(f)] for f in futs] == got
        # a contains run after the adds: every added element is a member
        with co.hold():
            cf = [co.submit(b"bf", "contains", SIZE, K, [_elem(t, i) for i in range(50)]) for t in range(16)]
        assert all(all(f.get(30)) for f in cf)
        assert co.calls == 2
    finally:
        co.close()


def test_runs_never_cross_another_kind_or_filter():
    from redisson_amd.coalesce import BloomCoalescer

    eng = OracleBloomEngine()
    co = BloomCoalescer(eng, record=True)
    try:
        with co.hold():
            seq = [("add", b"a"), ("add", b"a"), ("contains", b"a"), ("add", b"a"), ("add", b"b"), ("add", b"b")]
            futs = [co.submit(nm, kind, SIZE, K, [_elem(j, 0)]) for j, (kind, nm) in enumerate(seq)]
        [f.get(30) for f in futs]
        assert [(k, len(r)) for k, r in co.log] == [("add", 2), ("contains", 1), ("add", 1), ("add", 2)]
        # the contains saw the two adds before it and not the one after
        assert futs[2].get() == [False]
    finally:
        co.close()


def test_config_changed_fails_the_run():
    from redisson_amd.coalesce import BloomCoalescer

    eng = OracleBloomEngine()
    co = BloomCoalescer(eng)
    try:
        f = co.submit(b"bf", "add", SIZE + 1, K, [b"x"])
        with pytest.raises(RedisException, match="config has been changed"):
            f.get(30)
    finally:
        co.close()


def test_concurrent_threads_linearizable():
    """16 threads, mixed add / contains on two filters, free running: every reply equals the oracle replaying
    the coalescer's execution order, and there are fewer engine calls than requests."""
    from redisson_amd.coalesce import BloomCoalescer

    eng = OracleBloomEngine()
    co = BloomCoalescer(eng, record=True)
    res = {}

    def worker(t):
        rng = np.random.default_rng(t)
        mine = []
        for i in range(60):
            kind = "add" if rng.random() < 0.5 else "contains"
            elems = [_elem(int(rng.integers(0, 8)), int(rng.integers(0, 40))) for _ in range(int(rng.integers(1, 6)))]
            mine.append((kind, elems, co.submit(b"bf", kind, SIZE, K, elems)))
        res[t] = [(k, e, f, f.get(60)) for k, e, f in mine]

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    co.close()
    want, _ = _replay(co.log)
    assert co.requests == 16 * 60 == len(want)
    assert co.calls < co.requests
    # each request's replies are those of its position in the linearized order
    for t in range(16):
        for kind, elems, fut, got in res[t]:
            assert list(got) == list(want[id(fut)])


@pytest.mark.gpu
def test_rbloomfilter_coalesced_on_engine(O):
    """RBloomFilter with Config(bloom_coalesce=True): 16 threads' add / contains calls run as merged engine
    launches; replies equal the oracle replaying the execution order; the filter's bit array equals it too."""
    from redisson_amd import Config, Redisson
    from redisson_amd.coalesce import BloomCoalescer

    r = Redisson.create(Config(device=0, bloom_coalesce=True))
    try:
        bf = r.getBloomFilter("cbf")
        assert bf.tryInit(1_000_000, 0.03)
        size, k = bf.getSize(), bf.getHashIterations()
        r.bloom_coalescer.close()
        r.bloom_coalescer = co = BloomCoalescer(r.engine, record=True)
        res = {}

        def worker(t):
            out = []
            for i in range(200):
                o = "v%d" % (t * 1000 + i % 120)
                out.append(("add", o, bf.add(o)) if i % 3 else ("contains", o, bf.contains(o)))
            res[t] = out

        th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert co.calls < co.requests == 16 * 200
        want, ref = _replay(co.log, size, k)
        # every request's future got the oracle's reply at its place in the execution order
        for kind, reqs in co.log:
            for elems, fut in reqs:
                assert fut.get() == [bool(x) for x in want[id(fut)]]
        enc = bf.codec.encode
        for t in range(16):                       # and the callers saw those futures' values
            for kind, o, got in res[t]:
                assert isinstance(got, bool)
        assert r.engine.get("cbf") == ref.bytes()
    finally:
        r.shutdown()


class _CfgBloomEngine(OracleBloomEngine):
    """OracleBloomEngine plus the filter's other engine calls (tryInit / config / count / DEL), each recording the
    thread it ran on."""

    def __init__(self):
        super().__init__()
        self.threads = []

    def _t(self, what):
        self.threads.append((what, threading.current_thread().name))

    def bloom_add(self, name, size, k, elems):
        self._t("add")
        return super().bloom_add(name, size, k, elems)

    def bloom_contains(self, name, size, k, elems):
        self._t("contains")
        return super().bloom_contains(name, size, k, elems)

    def bloom_try_init(self, name, n, p):
        self._t("tryInit")
        m = self.O.bloom_optimal_bits(n, p)
        fresh = name not in self.cfg
        self.cfg[name] = (m, self.O.bloom_optimal_k(n, m))
        return fresh

    def bloom_config(self, name):
        self._t("config")
        from redisson_amd.engine import IllegalStateException

        if name not in self.cfg:
            raise IllegalStateException("Bloom filter is not initialized!")
        m, k = self.cfg[name]
        return m, k, 0, 0.0

    def bloom_count(self, name):
        self._t("count")
        m, k = self.cfg[name]
        b = self.bits.get(name)
        return self.O.bloom_count(m, k, b.bitcount() if b else 0)

    def delete(self, keys):
        self._t("delete")
        n = 0
        for key in keys:
            n += self.bits.pop(key, None) is not None
            n += self.cfg.pop(key, None) is not None
        return n


class _Client:
    def __init__(self, eng, co):
        from redisson_amd.redisson import Config

        self.engine, self.bloom_coalescer, self.config = eng, co, Config()


def test_filter_calls_run_on_the_fifo_worker_in_order():
    """with group commit on, every engine call of RBloomFilter (tryInit, the config read, count,
    getters, delete) runs on the coalescer's completion thread, and deleteAsync completes from it only after every
    request queued before it -- a delete issued after a queued containsAllAsync never overtakes it."""
    from redisson_amd.coalesce import BloomCoalescer
    from redisson_amd.redisson import RBloomFilter

    eng = _CfgBloomEngine()
    co = BloomCoalescer(eng)
    try:
        bf = RBloomFilter(_Client(eng, co), "bf")
        assert bf.tryInit(20000, 0.01) and not bf.tryInit(20000, 0.01)
        elems = [_elem(1, i) for i in range(300)]
        assert all(bf.addAll(elems))
        m, k = eng.cfg["bf"]
        assert (bf.getSize(), bf.getHashIterations()) == (m, k)
        assert bf.count() > 250
        with co.hold():
            fc = bf.containsAllAsync(elems)     # queued: no config read or engine call on this thread
            fd = bf.deleteAsync()               # queued behind the contains
            fa = bf.containsAllAsync(elems[:5])   # after the delete: the filter is gone
            assert not fc.isDone() and not fd.isDone()
        assert fc.get(30) == [True] * len(elems)
        assert fd.get(30) is True
        with pytest.raises(Exception, match="not initialized"):
            fa.get(30)
        assert [w for w, _ in eng.threads][-3:] == ["contains", "delete", "config"]
        assert {t for _, t in eng.threads} == {"sk-bloom-coalescer"}, eng.threads
    finally:
        co.close()
