"""Group commit of concurrent RBloomFilter calls.

The reference pays one pipeline round trip per element: every ``add`` / ``contains`` is its own
CommandBatchService with the config-check EVAL and k SETBIT / GETBIT (M:RedissonBloomFilter.java:94-100,
147-153), and RBatch has no Bloom filter (M:RedissonBatch.java).  On the GPU one element per launch would waste
the device, so concurrent calls are coalesced: callers (Netty event-loop threads in the Java executor) only
enqueue and get a future; one completion thread drains the queue in FIFO order, merges each maximal run of
requests for the same (filter, operation, size, k) into ONE engine call, splits the replies and completes the
futures.  A run never crosses a request of another kind or filter, so every caller sees the linearizable
result of the FIFO order (an add is never moved across a contains, or the reverse).  Replies inside a merged
add run are the engine's exact sequential replies of the concatenation, i.e. of the requests in FIFO order.

A request carries the (size, k) its caller read; the engine checks them against the stored config and fails
the run with "Bloom filter config has been changed" if they differ, which the caller's retry loop handles
exactly as RedissonBloomFilter does (:108-111, :162-166).
"""
from __future__ import annotations

import collections
import contextlib
import threading
from typing import List, Optional, Sequence

import numpy as np

from .redisson import Future


class WaitFuture(Future):
    """A Future another thread completes; get() blocks until it is done."""

    def __init__(self):
        super().__init__()
        self._ev = threading.Event()

    def _set(self, v):
        super()._set(v)
        self._ev.set()

    def _fail(self, e):
        super()._fail(e)
        self._ev.set()

    def get(self, timeout: Optional[float] = None):
        if not self._ev.wait(timeout):
            raise TimeoutError("Bloom request not completed")
        return super().get()

    getNow = Future.get
    sync = get


class _Req:
    __slots__ = ("name", "kind", "size", "k", "elems", "future", "fn")

    def __init__(self, name, kind, size, k, elems, fn=None):
        self.name, self.kind, self.size, self.k, self.elems, self.fn = name, kind, size, k, elems, fn
        self.future = WaitFuture()

    def key(self):
        # a task is a run of its own: it never merges, and nothing merges across it
        return (self.name, self.kind, self.size, self.k) if self.fn is None else self


class BloomCoalescer:
    """One completion thread per engine context; `submit` never blocks on the device."""

    def __init__(self, engine, max_batch: int = 1 << 22, record: bool = False):
        self.engine = engine
        self.max_batch = max_batch
        self._q: collections.deque = collections.deque()
        self._cv = threading.Condition()
        self._stop = False
        self._held = 0
        self.calls = 0                 # engine calls made (one per merged run)
        self.requests = 0              # requests completed
        # per run, in execution order: (kind, [(request elems, its future), ...]) -- replay tests only
        self.log: Optional[List] = [] if record else None
        self._t = threading.Thread(target=self._loop, name="sk-bloom-coalescer", daemon=True)
        self._t.start()

    def submit(self, name, kind: str, size: int, k: int, elems: Sequence[bytes]) -> WaitFuture:
        """An add / contains request.  size = 0: the filter's config is read on the completion thread right before
        the engine call (the non-blocking callers' form, which must not read it on their own thread)."""
        if kind not in ("add", "contains"):
            raise ValueError(kind)
        return self._enqueue(_Req(name, kind, int(size), int(k), list(elems)))

    def submit_task(self, fn) -> WaitFuture:
        """Any other engine call on a filter (tryInit, the config read, count, delete): run by the completion thread
        in its FIFO place, after every request queued before it, so it neither blocks the caller's thread on the
        device nor overtakes a queued add / contains."""
        return self._enqueue(_Req(None, "task", 0, 0, [], fn))

    def _enqueue(self, r: _Req) -> WaitFuture:
        with self._cv:
            if self._stop:
                raise RuntimeError("coalescer closed")
            self._q.append(r)
            self._cv.notify()
        return r.future

    @contextlib.contextmanager
    def hold(self):
        """Let requests queue up without draining (tests / explicit group commit)."""
        with self._cv:
            self._held += 1
        try:
            yield self
        finally:
            with self._cv:
                self._held -= 1
                self._cv.notify()

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._t.join()

    def _take_run(self) -> List[_Req]:
        head = self._q.popleft()
        run, n = [head], len(head.elems)
        key = head.key()
        while self._q and self._q[0].key() == key and n + len(self._q[0].elems) <= self.max_batch:
            r = self._q.popleft()
            run.append(r)
            n += len(r.elems)
        return run

    def _loop(self):
        while True:
            with self._cv:
                while not self._stop and (not self._q or self._held):
                    self._cv.wait()
                if not self._q:
                    return                      # stopped and drained
                run = self._take_run()
            self._execute(run)

    def _execute(self, run: List[_Req]):
        head = run[0]
        if head.fn is not None:
            try:
                v = head.fn()
            except Exception as e:  # noqa: BLE001 - the task's caller sees its error
                head.future._fail(e)
            else:
                head.future._set(v)
            if self.log is not None:
                self.log.append(("task", [([], head.future)]))
            self.calls += 1
            self.requests += 1
            return
        elems = [e for r in run for e in r.elems]
        fn = self.engine.bloom_add if head.kind == "add" else self.engine.bloom_contains
        try:
            from .engine import common_prefix

            size, k = head.size, head.k
            if size == 0:   # config read here, in FIFO order (submit's size = 0 form)
                size, k = self.engine.bloom_config(head.name)[:2]
            plen = common_prefix(elems) if elems else 0
            if plen >= 8:   # a shared codec prefix: prefix form, only the suffixes cross the host link
                res = self.engine.bloom_prefix(head.kind, head.name, size, k, bytes(elems[0])[:plen],
                                               [bytes(e)[plen:] for e in elems])
            else:
                res = fn(head.name, size, k, elems) if elems else []
        except Exception as e:  # noqa: BLE001 - every request of the run sees the engine's error
            for r in run:
                r.future._fail(e)
        else:
            p = 0
            for r in run:
                r.future._set(list(res[p:p + len(r.elems)]))
                p += len(r.elems)
            if self.log is not None:
                self.log.append((head.kind, [(r.elems, r.future) for r in run]))
        self.calls += 1
        self.requests += len(run)


# ---------------------------------------------------------------------------------------------------------------
# Group commit of concurrent RBatch executions (the C2 ingestion shape: many clients each executing an RBatch of
# PFADDs).  The reference sends every RBatch as its own pipeline (M:command/CommandBatchService.java:184-293) and
# redis-server applies the batches one after another.  Here a completion thread drains every queued batch in
# FIFO order and merges each maximal sequence of PFADD-only batches into ONE sk_pfadd call, so a device call
# carries tens of millions of commands and the engine applies them with its line schedule (registers streamed once
# per call, not once per element).  The concatenation keeps FIFO order, and PFADD replies depend only on order, so
# every batch gets exactly the replies it would get if the batches had run one after another in that order.
# A batch with any other command runs on its own, in its place in the FIFO order.

class _BatchReq:
    __slots__ = ("batch", "future")

    def __init__(self, batch):
        self.batch = batch
        self.future = WaitFuture()

    def pfadd_only(self) -> bool:
        return all(c[0][0] == "PFADD" and c[1] is None for c in self.batch._cmds)


class BatchCoalescer:
    """One completion thread per client; `submit(batch)` enqueues an RBatch and returns the future of its result
    list (or its error, as RBatch.execute would raise it)."""

    def __init__(self, client, max_cmds: int = 1 << 26):
        self.client = client
        self.engine = client.engine
        self.max_cmds = max_cmds
        self._q: collections.deque = collections.deque()
        self._cv = threading.Condition()
        self._stop = False
        self._held = 0
        self.calls = 0       # engine PFADD calls made for merged groups
        self.batches = 0     # batches completed
        self._ids = {}       # key -> slab handle (sk_hll_resolve), valid until the key is deleted / replaced
        self._created = set()
        self._t = threading.Thread(target=self._loop, name="sk-batch-coalescer", daemon=True)
        self._t.start()

    def submit(self, batch) -> WaitFuture:
        r = _BatchReq(batch)
        with self._cv:
            if self._stop:
                raise RuntimeError("coalescer closed")
            self._q.append(r)
            self._cv.notify()
        return r.future

    hold = BloomCoalescer.hold

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._t.join()

    def _take(self) -> List[_BatchReq]:
        head = self._q.popleft()
        group = [head]
        if head.pfadd_only():
            n = len(head.batch._cmds)
            while self._q and self._q[0].pfadd_only() and n + len(self._q[0].batch._cmds) <= self.max_cmds:
                r = self._q.popleft()
                group.append(r)
                n += len(r.batch._cmds)
        return group

    def _loop(self):
        while True:
            with self._cv:
                while not self._stop and (not self._q or self._held):
                    self._cv.wait()
                if not self._q:
                    return
                group = self._take()
            try:
                if len(group) == 1 and not group[0].pfadd_only():
                    self._run_one(group[0])
                else:
                    self._run_pfadd(group)
            except Exception as e:  # noqa: BLE001 - packing / encoding / type lookup failed: fail the whole group,
                # as BloomCoalescer._execute does; the completion thread lives on for the batches behind it
                for r in group:
                    r.batch._executed = True
                    for (_c, _fn, _post, f) in r.batch._cmds:
                        if not f.isDone():
                            f._fail(e)
                    if not r.future.isDone():
                        r.future._fail(e)
            self.batches += len(group)

    def _run_one(self, r: _BatchReq):
        try:
            r.future._set(r.batch._execute_now())
        except Exception as e:  # noqa: BLE001 - the batch's own error, as execute() raises it
            r.future._fail(e)

    def _resolve(self, keys) -> "tuple[dict, set]":
        """Slab handles of the group's distinct keys: from the coalescer's cache (the Java executor's per-tenant
        cache), else typed in ONE call and resolved (created) in one call.  A key holding a plain string is
        resolved on its own: it is adopted if it holds a valid HLL string, otherwise its commands fail (WRONGTYPE).
        Returns ({key: handle}, {key: error text of the keys whose commands fail}) and records created keys."""
        from . import _native as N
        from .engine import RedisException

        miss = [k for k in dict.fromkeys(keys) if k not in self._ids]
        bad = {}
        if miss:
            t = self.engine.key_types(miss)
            plain = [k for k, ty in zip(miss, t) if ty in (N.SK_TYPE_NONE, N.SK_TYPE_HLL)]
            if plain:
                h, cr = self.engine.hll_resolve(plain, with_created=True)
                for k, hk, c in zip(plain, h, cr):
                    self._ids[k] = int(hk)
                    if c:
                        self._created.add(k)
            for k, ty in zip(miss, t):
                if ty in (N.SK_TYPE_NONE, N.SK_TYPE_HLL):
                    continue
                try:
                    self._ids[k] = int(self.engine.hll_resolve([k])[0])
                except RedisException as e:
                    bad[k] = str(e)
        return self._ids, bad

    def _run_pfadd(self, group: List[_BatchReq]):
        """The group as ONE sk_pfadd_ids call over cached slab handles (names are resolved only on a cache miss);
        a stale cache (a key deleted or replaced since) is dropped and resolved again once."""
        from . import _native as N
        from .engine import RedisException

        cmds = [c for r in group for c in r.batch._cmds]
        keys = [c[0][1] for c in cmds]
        for attempt in range(2):
            self._created = set()
            ids, bad_msg = self._resolve(keys)
            ok = [i for i, k in enumerate(keys) if k not in bad_msg]
            out = np.zeros(len(keys), dtype=np.uint8)
            st, sub, msg = self.engine.pfadd_ids_status(np.array([ids[keys[i]] for i in ok], dtype=np.uint32),
                                                        [cmds[i][0][2] for i in ok]) if ok else (N.SK_OK, out[:0], "")
            if st == N.SK_ESTALE and attempt == 0:
                self._ids.clear()
                continue
            break
        self.calls += 1
        out[ok] = sub
        seen = set()
        for i in ok:                          # PFADD replies 1 on the command that created its key
            k = keys[i]
            if k in self._created and k not in seen:
                out[i] = 1
            seen.add(k)
        bad = set(bad_msg)
        if bad:
            msg = next(iter(bad_msg.values()))
        if st != N.SK_OK:                     # a device / capacity error fails every command of the group
            bad = set(keys)
        p = 0
        for r in group:
            r.batch._executed = True
            err, res = None, []
            for (c, fn, post, f) in r.batch._cmds:
                if c[1] in bad:
                    e = RedisException(msg)
                    f._fail(e)
                    err = e
                    res.append(None)
                else:
                    v = bool(out[p])
                    f._set(post(v) if post else v)
                    res.append(f._value)
                p += 1
            if err is not None:
                r.future._fail(err)
            else:
                r.future._set(res)
