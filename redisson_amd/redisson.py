"""Redisson-shaped host API over the GPU sketch engine.

Mirrors the reference's public interfaces for the hot path, same method names,
argument meaning and error behaviour (Python spelling: ``or_``/``and_``/
``not_`` because ``or``/``and``/``not`` are keywords):

* ``RHyperLogLog``  -- M:core/RHyperLogLog.java:20-32, impl M:RedissonHyperLogLog.java:66-97
* ``RBitSet``       -- M:core/RBitSet.java:25-63,     impl M:RedissonBitSet.java:53-268
* ``RBloomFilter``  -- M:core/RBloomFilter.java:27-60, impl M:RedissonBloomFilter.java
* ``RBatch``        -- M:core/RBatch.java, impl M:RedissonBatch.java / CommandBatchService

Every command becomes a call into the C ABI (what the Java JNI executor would
do in place of CommandAsyncService.async, M:command/CommandAsyncService.java:378).
Async methods return an already-completed ``Future`` (the engine call is
synchronous); RBatch queues commands and runs them in enqueue order on
``execute()``, grouping consecutive same-kind commands into one device batch.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional

from .codec import Codec, JsonJacksonCodec, params_bytes
from .engine import (IllegalArgumentException, IllegalStateException, RedisException, SketchEngine)


# ------------------------------------------------------------------ futures
class Future:
    def __init__(self):
        self._done = False
        self._value = None
        self._exc: Optional[BaseException] = None

    def _set(self, v):
        self._value, self._done = v, True

    def _fail(self, e):
        self._exc, self._done = e, True

    def isDone(self):
        return self._done

    def isSuccess(self):
        return self._done and self._exc is None

    def cause(self):
        return self._exc

    def get(self):
        if not self._done:
            raise IllegalStateException("batch not executed")
        if self._exc is not None:
            raise self._exc
        return self._value

    getNow = get
    sync = get


def _completed(fn: Callable[[], Any]) -> Future:
    f = Future()
    try:
        f._set(fn())
    except Exception as e:  # noqa: BLE001 - delivered through the future
        f._fail(e)
    return f


# ------------------------------------------------------------------ config
@dataclass
class Config:
    """Subset of org.redisson.Config that matters for this path."""

    device: int = 0
    redis_major: int = 3          # redis-server semantics to reproduce (reference CI: 3.2.0)
    max_bit_offset: int = 0       # 0 -> 2^32 (redis 3.2 string limit)
    hll_capacity: int = 0
    max_batch: int = 0
    codec: Codec = field(default_factory=JsonJacksonCodec)   # M:Config.java:68-70
    # group commit of concurrent RBloomFilter add/contains calls (redisson_amd/coalesce.py): callers only enqueue,
    # one completion thread merges FIFO runs into single engine calls
    bloom_coalesce: bool = False
    # group commit of concurrently executed RBatches (coalesce.BatchCoalescer): PFADD-only batches queued together
    # become one engine call (the line schedule at >= 4 M commands and >= 160 per HLL key), replies split back per batch
    batch_coalesce: bool = False


class JBitSet:
    """Minimal java.util.BitSet (toString "{3, 5}")."""

    def __init__(self, bits=()):
        self.bits = set(int(b) for b in bits)

    def set(self, i, value=True):
        (self.bits.add if value else self.bits.discard)(int(i))

    def get(self, i):
        return int(i) in self.bits

    def length(self):
        return max(self.bits) + 1 if self.bits else 0

    def cardinality(self):
        return len(self.bits)

    def __eq__(self, o):
        return isinstance(o, JBitSet) and o.bits == self.bits

    def __str__(self):
        return "{" + ", ".join(str(b) for b in sorted(self.bits)) + "}"

    __repr__ = __str__


def _to_byte_array_reverse(bs: JBitSet) -> bytes:
    # M:RedissonBitSet.java:164-173: new byte[bits.length()/8 + 1], MSB-first
    out = bytearray(bs.length() // 8 + 1)
    for i in bs.bits:
        out[i // 8] |= 1 << (7 - (i % 8))
    return bytes(out)


def _from_byte_array_reverse(b: bytes) -> JBitSet:
    # M:RedissonBitSet.java:152-161
    return JBitSet(i for i in range(len(b) * 8) if b[i // 8] & (1 << (7 - (i % 8))))


def _int32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


# ------------------------------------------------------------------ objects
class RObject:
    def __init__(self, client: "Redisson", name: str, codec: Optional[Codec] = None):
        self._c = client
        self._name = name
        self.codec = codec or client.config.codec

    def getName(self):
        return self._name

    @property
    def _e(self) -> SketchEngine:
        return self._c.engine

    def delete(self) -> bool:
        return self.deleteAsync().get()

    def deleteAsync(self) -> Future:
        return self._c._submit(("DEL", [self._name]), lambda: self._e.delete([self._name]) > 0)

    def isExists(self) -> bool:
        return self._e.key_type(self._name) != 0


class RHyperLogLog(RObject):
    def add(self, obj) -> bool:
        return self.addAsync(obj).get()

    def addAsync(self, obj) -> Future:
        # PFADD name e (RedisCommands.PFADD inParamIndex 2 -> codec-encoded), :66-68
        return self._c._submit(("PFADD", self._name, [self.codec.encode(obj)]))

    def addAll(self, objects) -> bool:
        return self.addAllAsync(objects).get()

    def addAllAsync(self, objects) -> Future:
        # Q1 (:70-76): params = [name, Object[]{name, e1..en}] -> ONE element,
        # the codec encoding of that Object[] (CommandEncoder :76-79)
        arr = [self._name] + list(objects)
        return self._c._submit(("PFADD", self._name, [self.codec.encode(arr)]))

    def count(self) -> int:
        return self.countAsync().get()

    def countAsync(self) -> Future:
        return self._c._submit(("PFCOUNT", [self._name]))

    def countWith(self, *other_log_names) -> int:
        return self.countWithAsync(*other_log_names).get()

    def countWithAsync(self, *other_log_names) -> Future:
        return self._c._submit(("PFCOUNT", [self._name] + list(other_log_names)))

    def mergeWith(self, *other_log_names) -> None:
        return self.mergeWithAsync(*other_log_names).get()

    def mergeWithAsync(self, *other_log_names) -> Future:
        # PFMERGE name name others...  (dest included in the max)
        return self._c._submit(("PFMERGE", self._name, [self._name] + list(other_log_names)))


class RBitSet(RObject):
    # ---- single bits
    def get(self, bitIndex: int) -> bool:
        return self.getAsync(bitIndex).get()

    def getAsync(self, bitIndex: int) -> Future:
        return self._c._submit(("GETBIT", self._name, int(bitIndex)))

    def set(self, *args):
        return self.setAsync(*args).get()

    def setAsync(self, *args) -> Future:
        if len(args) == 1 and isinstance(args[0], JBitSet):          # set(BitSet) :211-214
            data = _to_byte_array_reverse(args[0])
            return self._c._submit(("SET", self._name, data))
        if len(args) == 1:                                           # set(bitIndex)
            return self._c._submit(("SETBIT", self._name, int(args[0]), 1))
        if len(args) == 2 and isinstance(args[1], bool):             # set(bitIndex, value)
            return self._c._submit(("SETBIT", self._name, int(args[0]), 1 if args[1] else 0))
        if len(args) == 2:                                           # set(from, to) :222-228
            return self._range(int(args[0]), int(args[1]), 1)
        if len(args) == 3:                                           # set(from, to, value) :194-200
            return self._range(int(args[0]), int(args[1]), 1 if args[2] else 0)
        raise TypeError("set() arguments")

    def _range(self, frm: int, to: int, v: int) -> Future:
        # the reference: one SETBIT_VOID per bit in a new batch (M:RedissonBitSet.java:202-228);
        # here one range-fill kernel with the same final string and the same error
        return self._c._submit(("SETRANGE", self._name, frm, to, v))

    def clear(self, *args):
        return self.clearAsync(*args).get()

    def clearAsync(self, *args) -> Future:
        if not args:                                                 # DEL :250-253
            return self._c._submit(("DEL", [self._name]), lambda: (self._e.delete([self._name]), None)[1])
        if len(args) == 1:
            return self._c._submit(("SETBIT", self._name, int(args[0]), 0))
        return self._range(int(args[0]), int(args[1]), 0)

    # ---- whole string
    def toByteArray(self) -> bytes:
        return self.toByteArrayAsync().get()

    def toByteArrayAsync(self) -> Future:
        return _completed(lambda: self._e.get(self._name) or b"")

    def asBitSet(self) -> JBitSet:
        return _from_byte_array_reverse(self.toByteArray())

    def __str__(self):
        return str(self.asBitSet())

    def toString(self):
        return str(self)

    def cardinality(self) -> int:
        return self.cardinalityAsync().get()

    def cardinalityAsync(self) -> Future:
        return self._c._submit(("BITCOUNT", self._name))

    def size(self) -> int:
        return self.sizeAsync().get()

    def sizeAsync(self) -> Future:
        # STRLEN -> BitsSizeReplayConvertor: val.intValue() * 8 in int (Q3 overflow)
        return self._c._submit(("STRLEN", self._name), post=lambda v: _int32(_int32(v) * 8))

    def length(self) -> int:
        return self.lengthAsync().get()

    def lengthAsync(self) -> Future:
        return self._c._submit(("LENGTH", self._name))

    def _op(self, op: str, names) -> Future:
        # BITOP op name name others... :138-145
        return self._c._submit(("BITOP", op, self._name, [self._name] + list(names)))

    def or_(self, *names):
        return self._op("OR", names).get()

    def and_(self, *names):
        return self._op("AND", names).get()

    def xor(self, *names):
        return self._op("XOR", names).get()

    def not_(self):
        return self._op("NOT", ()).get()

    def orAsync(self, *names):
        return self._op("OR", names)

    def andAsync(self, *names):
        return self._op("AND", names)

    def xorAsync(self, *names):
        return self._op("XOR", names)

    def notAsync(self):
        return self._op("NOT", ())


class RBloomFilter(RObject):
    MAX_SIZE = 2 * 2147483647  # :52

    def __init__(self, client, name, codec=None):
        super().__init__(client, name, codec)
        self._size = 0
        self._k = 0

    def _co(self):
        return getattr(self._c, "bloom_coalescer", None)

    def _call(self, fn):
        """Every engine call of the filter: with group commit on, it runs on the coalescer's completion thread in
        FIFO order with the queued add / contains requests, never on the caller's thread."""
        co = self._co()
        return co.submit_task(fn).get() if co is not None else fn()

    def _read_config(self):
        size, k, _, _ = self._call(lambda: self._e.bloom_config(self._name))   # IllegalStateException if absent
        self._size, self._k = size, k

    def tryInit(self, expectedInsertions: int, falseProbability: float) -> bool:
        ok = self._call(lambda: self._e.bloom_try_init(self._name, int(expectedInsertions), float(falseProbability)))
        self._read_config()
        return ok

    def _run(self, fn, objs):
        elems = [self.codec.encode(o) for o in objs]
        co = self._co()
        while True:
            if self._size == 0:
                self._read_config()
            try:
                if co is not None:   # group commit: merged with concurrent callers' requests into one engine call
                    kind = "add" if fn == self._e.bloom_add else "contains"
                    return co.submit(self._name, kind, self._size, self._k, elems).get()
                return fn(self._name, self._size, self._k, elems)
            except RedisException as e:          # retry loop :108-111 / :162-166
                if "Bloom filter config has been changed" not in str(e):
                    raise
                self._read_config()

    def add(self, obj) -> bool:
        return self._run(self._e.bloom_add, [obj])[0]

    def contains(self, obj) -> bool:
        return self._run(self._e.bloom_contains, [obj])[0]

    # batched Bloom API (RBatch has no Bloom filter)
    def addAll(self, objs) -> List[bool]:
        return self._run(self._e.bloom_add, list(objs))

    def containsAll(self, objs) -> List[bool]:
        return self._run(self._e.bloom_contains, list(objs))

    def _async(self, kind, objs) -> Future:
        """Non-blocking form (the Java twin's containsAllAsync, for event-loop callers): with group commit on, the
        request carries no config and the completion thread reads it in FIFO order; the future completes from
        that thread."""
        elems = [self.codec.encode(o) for o in objs]
        co = self._co()
        if co is None:
            return _completed(lambda: self._run(self._e.bloom_add if kind == "add" else self._e.bloom_contains, objs))
        return co.submit(self._name, kind, 0, 0, elems)

    def addAllAsync(self, objs) -> Future:
        return self._async("add", list(objs))

    def containsAllAsync(self, objs) -> Future:
        return self._async("contains", list(objs))

    def count(self) -> int:
        return self._call(lambda: self._e.bloom_count(self._name))

    def _cfg(self, i):
        return self._call(lambda: self._e.bloom_config(self._name))[i]

    def getExpectedInsertions(self) -> int:
        return self._cfg(2)

    def getFalseProbability(self) -> float:
        return self._cfg(3)

    def getSize(self) -> int:
        return self._cfg(0)

    def getHashIterations(self) -> int:
        return self._cfg(1)

    def deleteAsync(self) -> Future:
        # DEL name {name}__config (:201-203); with group commit on, completed by the coalescer's thread after every
        # request queued before it
        cfg = "{" + self._name + "}__config"
        fn = lambda: self._e.delete([self._name, cfg]) > 0   # noqa: E731
        co = self._co()
        return co.submit_task(fn) if co is not None else _completed(fn)


# ------------------------------------------------------------------ batch
class RBatch:
    """RBatch: commands queued in enqueue order, results as a list in that order
    (M:command/CommandBatchService.java:142-182)."""

    def __init__(self, client: "Redisson"):
        self._c = client
        self._cmds: List[tuple] = []
        self._executed = False

    def _submit(self, cmd, fn=None, post=None) -> Future:
        f = Future()
        self._cmds.append((cmd, fn, post, f))
        return f

    # objects bound to this batch
    def getHyperLogLog(self, name, codec=None) -> RHyperLogLog:
        return RHyperLogLog(_BatchClient(self), name, codec)

    def getBitSet(self, name) -> RBitSet:
        return RBitSet(_BatchClient(self), name)

    def execute(self):
        if self._executed:
            raise IllegalStateException("Batch already executed!")
        if not self._cmds:
            return None           # newSucceededFuture(null) for an empty batch
        co = getattr(self._c, "batch_coalescer", None)
        if co is not None:        # group commit with concurrently executed batches (coalesce.BatchCoalescer)
            self._executed = True
            return co.submit(self).get()
        return self._execute_now()

    def _execute_now(self):
        self._executed = True
        self._c._run_batch(self._cmds)
        err = None
        out = []
        for (_, _, _, f) in self._cmds:
            if f._exc is not None:
                err = f._exc
            out.append(f._value)
        if err is not None:       # any error fails the whole batch (CommandDecoder :183-197)
            raise err
        return out

    def executeAsync(self) -> Future:
        co = getattr(self._c, "batch_coalescer", None)
        if co is None or not self._cmds or self._executed:
            return _completed(self.execute)
        self._executed = True
        return co.submit(self)    # completed by the coalescer's thread; the caller never waits on the device


class _BatchClient:
    """Client view whose _submit enqueues into a batch."""

    def __init__(self, batch: RBatch):
        self._batch = batch
        self.config = batch._c.config
        self.engine = batch._c.engine

    def _submit(self, cmd, fn=None, post=None):
        return self._batch._submit(cmd, fn, post)

    def createBatch(self):
        return self._batch._c.createBatch()


# ------------------------------------------------------------------ client
class Redisson:
    """Redisson.create(config) -> client (M:Redisson.java:160)."""

    def __init__(self, config: Config):
        self.config = config
        self.engine = SketchEngine(config.device, config.redis_major, config.max_bit_offset,
                                   config.hll_capacity, config.max_batch)
        self.bloom_coalescer = None
        if config.bloom_coalesce:
            from .coalesce import BloomCoalescer
            self.bloom_coalescer = BloomCoalescer(self.engine)
        self.batch_coalescer = None
        if config.batch_coalesce:
            from .coalesce import BatchCoalescer
            self.batch_coalescer = BatchCoalescer(self)

    @staticmethod
    def create(config: Optional[Config] = None) -> "Redisson":
        return Redisson(config or Config())

    def shutdown(self):
        if self.bloom_coalescer is not None:
            self.bloom_coalescer.close()
        if self.batch_coalescer is not None:
            self.batch_coalescer.close()
        self.engine.close()

    def getHyperLogLog(self, name, codec=None) -> RHyperLogLog:
        return RHyperLogLog(self, name, codec)

    def getBitSet(self, name) -> RBitSet:
        return RBitSet(self, name)

    def getBloomFilter(self, name, codec=None) -> RBloomFilter:
        return RBloomFilter(self, name, codec)

    def createBatch(self) -> RBatch:
        return RBatch(self)

    # single command = a batch of one
    def _submit(self, cmd, fn=None, post=None) -> Future:
        f = Future()
        self._run_batch([(cmd, fn, post, f)])
        return f

    # ---- the executor: consecutive same-kind commands -> one engine call
    def _run_batch(self, cmds):
        e = self.engine
        i = 0
        while i < len(cmds):
            kind = cmds[i][0][0]
            j = i + 1
            if kind in ("PFADD", "GETBIT", "SETBIT", "PFCOUNT"):
                while j < len(cmds) and cmds[j][0][0] == kind and cmds[j][1] is None:
                    j += 1
            run = cmds[i:j]
            try:
                if run[0][1] is not None:            # custom callable
                    results = [run[0][1]()]
                elif kind == "PFADD":
                    results = e.pfadd([c[0][1] for c in run], [c[0][2] for c in run])
                elif kind == "PFCOUNT":
                    results = e.pfcount([c[0][1] for c in run])
                elif kind == "PFMERGE":
                    results = [e.pfmerge(run[0][0][1], run[0][0][2])]
                elif kind == "GETBIT":
                    results = [bool(x) for x in e.getbit([c[0][1] for c in run], [c[0][2] for c in run])]
                elif kind == "SETBIT":
                    e.setbit([c[0][1] for c in run], [c[0][2] for c in run], [c[0][3] for c in run],
                             want_old=False)
                    results = [None] * len(run)      # SETBIT_VOID
                elif kind == "BITCOUNT":
                    results = [e.bitcount(run[0][0][1])]
                elif kind == "STRLEN":
                    results = [e.strlen(run[0][0][1])]
                elif kind == "LENGTH":
                    results = [e.bitset_length(run[0][0][1])]
                elif kind == "BITOP":
                    _, op, dest, srcs = run[0][0]
                    e.bitop(op, dest, srcs)
                    results = [None]
                elif kind == "SETRANGE":
                    _, name, frm, to, v = run[0][0]
                    e.set_bit_range(name, frm, to, v)
                    results = [None]
                elif kind == "SET":
                    e.set(run[0][0][1], run[0][0][2])
                    results = [None]
                elif kind == "DEL":
                    results = [e.delete(run[0][0][1]) > 0]
                else:
                    raise RedisException(f"ERR unknown command '{kind}'")
                for (c, fn, post, f), r in zip(run, results):
                    f._set(post(r) if post else r)
            except (RedisException, IllegalStateException, IllegalArgumentException) as ex:
                for (_, _, _, f) in run:
                    f._fail(ex)
            i = j
