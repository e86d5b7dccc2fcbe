"""SketchEngine: one GPU-resident sketch store (one C-ABI context per device).

Thin Python marshalling over libredisson_sketch.so: packs byte strings into
(offsets u64[n+1], bytes) arrays, calls the C ABI, maps status codes to the
exceptions Redisson raises (RedisException for server replies,
IllegalStateException / IllegalArgumentException for the Bloom filter's
client-side checks, M:RedissonBloomFilter.java:72-74,217,284).
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, List, Sequence

import numpy as np

from . import _native as N


class RedisException(Exception):
    """Error reply of a command (M:client/RedisException.java)."""


class IllegalStateException(RuntimeError):
    pass


class IllegalArgumentException(ValueError):
    pass


class DeviceUnavailable(RuntimeError):
    pass


def _addr(a) -> int:
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if isinstance(a, DeviceBuffer):
        return a.ptr
    return int(a)


class DeviceBuffer:
    """HBM allocation owned by an engine context (no torch: the engine links the
    system HIP runtime, and one process must not load two)."""

    def __init__(self, engine: "SketchEngine", nbytes: int):
        self.engine = engine
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        engine._check(engine.lib.sk_dev_alloc(engine.ctx, self.nbytes, ctypes.addressof(p)))
        self.ptr = p.value

    def upload(self, arr: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        self.engine._check(self.engine.lib.sk_h2d(self.engine.ctx, self.ptr + offset, a.ctypes.data, a.nbytes))
        return self

    def download(self, dtype=np.uint8, count: int = -1, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        if count < 0:
            count = (self.nbytes - offset) // dt.itemsize
        out = np.empty(count, dtype=dt)
        self.engine._check(self.engine.lib.sk_d2h(self.engine.ctx, out.ctypes.data, self.ptr + offset, out.nbytes))
        return out

    def zero(self):
        self.engine._check(self.engine.lib.sk_dev_memset(self.engine.ctx, self.ptr, 0, self.nbytes))
        return self

    def free(self):
        if self.ptr and self.engine.ctx:
            self.engine.lib.sk_dev_free(self.engine.ctx, self.ptr)
        self.ptr = 0

    def view(self, offset: int, nbytes: int = -1) -> "DeviceView":
        """Bytes [offset, offset + nbytes) of this allocation, without ownership (freeing a view is a no-op)."""
        return DeviceView(self.engine, self.ptr + offset, self.nbytes - offset if nbytes < 0 else nbytes)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceView(DeviceBuffer):
    """A range of an engine allocation (DeviceBuffer.view): the same upload / download / zero, no ownership."""

    def __init__(self, engine: "SketchEngine", ptr: int, nbytes: int):  # noqa: D107 - no allocation
        self.engine, self.ptr, self.nbytes = engine, int(ptr), int(nbytes)

    def free(self):
        self.ptr = 0

    def __del__(self):
        pass


def pack(items: Sequence[bytes]):
    """(off u64[n+1], bytes u8[total+16]) with 16 B zero padding."""
    n = len(items)
    off = np.zeros(n + 1, dtype=np.uint64)
    if n:
        lens = np.fromiter((len(x) for x in items), dtype=np.uint64, count=n)
        np.cumsum(lens, out=off[1:])
    blob = b"".join(items)
    buf = np.zeros(len(blob) + 16, dtype=np.uint8)
    if blob:
        buf[: len(blob)] = np.frombuffer(blob, dtype=np.uint8)
    return off, buf


def common_prefix(items: Sequence[bytes], cap: int = 255) -> int:
    """Length of the longest byte prefix every item shares (<= cap): the prefix form's shared part."""
    if not items:
        return 0
    first = bytes(items[0])[:cap]
    plen = len(first)
    for x in items[1:]:
        x = bytes(x)
        m = min(plen, len(x))
        j = 0
        while j < m and x[j] == first[j]:
            j += 1
        plen = j
        if plen == 0:
            break
    return plen


def pack_u32(items: Sequence[bytes]):
    """(u32 offsets[n+1], bytes + 16 B of padding): the suffix form of the prefix-form entry points."""
    lens = np.fromiter((len(x) for x in items), dtype=np.uint32, count=len(items))
    off = np.zeros(len(items) + 1, dtype=np.uint32)
    np.cumsum(lens, out=off[1:])
    buf = np.frombuffer(b"".join(bytes(x) for x in items) + b"\0" * 16, dtype=np.uint8)
    return off, buf


def _b(x) -> bytes:
    return x.encode("utf-8") if isinstance(x, str) else bytes(x)


class SketchEngine:
    def __init__(self, device: int = 0, redis_major: int = 3, max_bit_offset: int = 0,
                 hll_capacity: int = 0, max_batch: int = 0):
        self.lib = N.load()
        cfg = N.SkConfig(device, redis_major, max_bit_offset, hll_capacity, max_batch)
        h = ctypes.c_void_p()
        st = self.lib.sk_open(ctypes.byref(cfg), ctypes.byref(h))
        if st != N.SK_OK:
            raise DeviceUnavailable(f"sk_open(device={device}) failed with status {st}: no usable HIP device")
        self.ctx = h.value
        self.device = device
        self.redis_major = redis_major

    # ------------------------------------------------------------ plumbing
    def close(self):
        if self.ctx:
            self.lib.sk_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int):
        if st == N.SK_OK:
            return
        msg = (self.lib.sk_last_error(self.ctx) or b"").decode("utf-8", "replace")
        if st == N.SK_ENOTINIT:
            raise IllegalStateException(msg)
        if st == N.SK_ETOOBIG:
            raise IllegalArgumentException(msg)
        raise RedisException(msg or self.lib.sk_strerror(st).decode())

    @property
    def stream(self) -> int:
        return self.lib.sk_stream(self.ctx)

    def sync(self):
        self._check(self.lib.sk_sync(self.ctx))

    # ------------------------------------------------------------ device memory / timing / RCCL
    def host_alloc(self, nbytes: int) -> np.ndarray:
        """Pinned host memory (sk_host_alloc) as a u8 array; freed with host_free.  Inputs the caller builds in it are
        copied to the device at the link's rate with no staging (the JNI side's direct ByteBuffers)."""
        p = ctypes.c_void_p()
        self._check(self.lib.sk_host_alloc(self.ctx, int(nbytes), ctypes.addressof(p)))
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * max(int(nbytes), 1)).from_address(p.value))
        return arr[:nbytes]

    def host_free(self, arr: np.ndarray):
        self._check(self.lib.sk_host_free(self.ctx, arr.ctypes.data))

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def to_device(self, arr: np.ndarray, pad: int = 0) -> DeviceBuffer:
        a = np.ascontiguousarray(arr)
        return DeviceBuffer(self, a.nbytes + pad).zero().upload(a)

    def gen_jackson_longs_dev(self, seed: int, n: int, first: int = 0, d_idx=None):
        """Device-resident Jackson Long elements: (d_off u64[n+1], d_bytes, total_bytes)."""
        d_off = self.alloc((n + 1) * 8)
        d_bytes = self.alloc(n * 39 + 16).zero()
        self._check(self.lib.sk_gen_jackson_longs_dev(self.ctx, seed, _addr(d_idx), first, n, d_off.ptr,
                                                      d_bytes.ptr))
        total = int(d_off.download(np.uint64, 1, offset=n * 8)[0])
        return d_off, d_bytes, total

    def timer_record(self, slot: int):
        self._check(self.lib.sk_timer_record(self.ctx, slot))

    def timer_elapsed_ms(self, a: int, b: int) -> float:
        ms = ctypes.c_float()
        self._check(self.lib.sk_timer_elapsed(self.ctx, a, b, ctypes.addressof(ms)))
        return ms.value

    def hll_exact_strings(self, on: bool = True):
        """GET of an HLL returns redis-server's bytes (sparse writer + cached cardinality); set before any HLL key."""
        self._check(self.lib.sk_hll_exact_strings(self.ctx, int(on)))

    def set_async(self, on: bool = True):
        self._check(self.lib.sk_set_async(self.ctx, int(on)))

    def prof_enable(self, on: bool = True):
        self._check(self.lib.sk_prof_enable(self.ctx, int(on)))

    def ticket(self) -> int:
        """Completion ticket for everything enqueued so far (async mode)."""
        t = ctypes.c_uint64()
        self._check(self.lib.sk_ticket(self.ctx, ctypes.addressof(t)))
        return t.value

    def poll(self, ticket: int) -> bool:
        done = ctypes.c_int()
        self._check(self.lib.sk_poll(self.ctx, ticket, ctypes.addressof(done)))
        return bool(done.value)

    def wait(self, ticket: int):
        self._check(self.lib.sk_wait(self.ctx, ticket))

    def flushall(self):
        self._check(self.lib.sk_flushall(self.ctx))

    def prof_only(self, phase=None):
        """Time only `phase` while profiling is on (None: every phase)."""
        self._check(self.lib.sk_prof_only(self.ctx, phase.encode() if phase else None))

    def prof_reset(self):
        self._check(self.lib.sk_prof_reset(self.ctx))

    def prof_read(self, phase: str):
        n, ms = ctypes.c_uint64(), ctypes.c_double()
        self._check(self.lib.sk_prof_read(self.ctx, phase.encode(), ctypes.addressof(n), ctypes.addressof(ms)))
        return n.value, ms.value

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        st = N.load().sk_comm_unique_id(ctypes.addressof(buf))
        if st != N.SK_OK:
            raise RedisException("ncclGetUniqueId failed")
        return bytes(buf)

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        b = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.lib.sk_comm_init(self.ctx, nranks, rank, ctypes.addressof(b)))

    def allreduce_max_u8(self, buf: DeviceBuffer, n: int):
        self._check(self.lib.sk_allreduce_max_u8(self.ctx, _addr(buf), n))

    def allreduce_sum_u64(self, buf: DeviceBuffer, n: int):
        self._check(self.lib.sk_allreduce_sum_u64(self.ctx, _addr(buf), n))

    def allgather(self, send: DeviceBuffer, recv: DeviceBuffer, bytes_per_rank: int):
        self._check(self.lib.sk_allgather(self.ctx, _addr(send), _addr(recv), bytes_per_rank))

    # ------------------------------------------------------------ keys
    def key_type(self, key) -> int:
        k = _b(key)
        t = ctypes.c_int()
        self._check(self.lib.sk_type(self.ctx, k, len(k), ctypes.addressof(t)))
        return t.value

    def key_types(self, keys) -> np.ndarray:
        """key_type of many keys in one call (int32); keys: a sequence or a pack()."""
        off, buf = keys if isinstance(keys, tuple) else pack([_b(k) for k in keys])
        out = np.zeros(len(off) - 1, dtype=np.int32)
        self._check(self.lib.sk_type_many(self.ctx, len(out), _addr(off), _addr(buf), _addr(out)))
        return out

    def pfadd_ids_status(self, key_ids, elems: Sequence[Sequence[bytes]]):
        """sk_pfadd_ids without raising: (status, replies u8[n], error text).  One-element commands whose elements
        share a codec prefix of >= 8 bytes go in prefix form (sk_pfadd_ids_prefix: only the suffixes cross the host
        link), as the Java group commit does."""
        ids = np.ascontiguousarray(key_ids, dtype=np.uint32)
        n = len(ids)
        out = np.zeros(n, dtype=np.uint8)
        flat = [e[0] for e in elems] if all(len(e) == 1 for e in elems) else None
        plen = common_prefix(flat) if flat else 0
        if plen >= 8:
            soff, sbuf = pack_u32([bytes(x)[plen:] for x in flat])
            pre = np.frombuffer(bytes(flat[0])[:plen], dtype=np.uint8)
            st = self.lib.sk_pfadd_ids_prefix(self.ctx, n, _addr(ids), _addr(pre), plen, _addr(soff), _addr(sbuf),
                                              _addr(out))
            msg = (self.lib.sk_last_error(self.ctx) or b"").decode("utf-8", "replace") if st != N.SK_OK else ""
            return st, out, msg
        counts = np.fromiter((len(e) for e in elems), dtype=np.uint32, count=n)
        eoff, ebuf = pack([x for e in elems for x in e])
        st = self.lib.sk_pfadd_ids(self.ctx, n, _addr(ids), _addr(counts), _addr(eoff), _addr(ebuf), _addr(out))
        msg = (self.lib.sk_last_error(self.ctx) or b"").decode("utf-8", "replace") if st != N.SK_OK else ""
        return st, out, msg

    def delete(self, keys: Iterable) -> int:
        ks = [_b(k) for k in keys]
        off, buf = pack(ks)
        out = ctypes.c_uint64()
        self._check(self.lib.sk_del(self.ctx, len(ks), _addr(off), _addr(buf), ctypes.addressof(out)))
        return out.value

    def hll_lookup(self, keys: Sequence) -> np.ndarray:
        """Handles of existing HLL keys (0xFFFFFFFF: missing), creating nothing; keys: a sequence or a pack()."""
        off, buf = keys if isinstance(keys, tuple) else pack([_b(k) for k in keys])
        ids = np.zeros(len(off) - 1, dtype=np.uint32)
        self._check(self.lib.sk_hll_lookup(self.ctx, len(ids), _addr(off), _addr(buf), _addr(ids)))
        return ids

    def hll_resolve(self, keys: Sequence, with_created: bool = False):
        """Slab handles of HLL keys, creating empty HLLs for missing names; with_created: (handles, created u8[])."""
        ks = [_b(k) for k in keys]
        off, buf = pack(ks)
        ids = np.zeros(len(ks), dtype=np.uint32)
        cr = np.zeros(len(ks), dtype=np.uint8)
        self._check(self.lib.sk_hll_resolve(self.ctx, len(ks), _addr(off), _addr(buf), _addr(ids), _addr(cr)))
        return (ids, cr) if with_created else ids

    # ------------------------------------------------------------ HLL
    def pfadd(self, keys: Sequence, elems: Sequence[Sequence[bytes]]) -> List[bool]:
        """PFADD batch: command i = PFADD keys[i] *elems[i] (raw element bytes)."""
        st, out, _ = self.pfadd_status(keys, elems)
        self._check(st)
        return [bool(x) for x in out]

    def pfadd_status(self, keys: Sequence, elems: Sequence[Sequence[bytes]]):
        """sk_pfadd without raising: (status, replies u8[n], error text).  A command on a key of another type fails
        alone (pipeline semantics): the status reports it, the other commands' replies are valid."""
        n = len(keys)
        koff, kbuf = pack([_b(k) for k in keys])
        counts = np.fromiter((len(e) for e in elems), dtype=np.uint32, count=n)
        flat = [x for e in elems for x in e]
        eoff, ebuf = pack(flat)
        out = np.zeros(n, dtype=np.uint8)
        st = self.lib.sk_pfadd(self.ctx, n, _addr(koff), _addr(kbuf), _addr(counts), _addr(eoff), _addr(ebuf),
                               _addr(out))
        msg = (self.lib.sk_last_error(self.ctx) or b"").decode("utf-8", "replace") if st != N.SK_OK else ""
        return st, out, msg

    def pfadd_ids(self, key_ids, elems: Sequence[Sequence[bytes]]) -> List[bool]:
        """PFADD batch with keys pre-resolved by hll_resolve: command i = PFADD key_ids[i] *elems[i]."""
        ids = np.ascontiguousarray(key_ids, dtype=np.uint32)
        n = len(ids)
        counts = np.fromiter((len(e) for e in elems), dtype=np.uint32, count=n)
        eoff, ebuf = pack([x for e in elems for x in e])
        out = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.sk_pfadd_ids(self.ctx, n, _addr(ids), _addr(counts), _addr(eoff), _addr(ebuf),
                                          _addr(out)))
        return [bool(x) for x in out]

    def pfadd_ids_prefix(self, key_ids, prefix: bytes, suffixes: Sequence[bytes]) -> List[bool]:
        """One-element PFADDs by slab handle whose elements are prefix + suffixes[i] (sk_pfadd_ids_prefix)."""
        ids = np.ascontiguousarray(key_ids, dtype=np.uint32)
        soff, sbuf = pack_u32(suffixes)
        pre = np.frombuffer(bytes(prefix) or b"\0", dtype=np.uint8)
        out = np.zeros(len(ids), dtype=np.uint8)
        self._check(self.lib.sk_pfadd_ids_prefix(self.ctx, len(ids), _addr(ids), _addr(pre), len(prefix),
                                                 _addr(soff), _addr(sbuf), _addr(out)))
        return [bool(x) for x in out]

    def pfadd_dev(self, n: int, d_key_ids, d_elem_off, d_elem_bytes, bytes_len: int, d_out):
        self._check(self.lib.sk_pfadd_dev(self.ctx, n, _addr(d_key_ids), _addr(d_elem_off), _addr(d_elem_bytes),
                                          bytes_len, _addr(d_out)))

    def pfcount(self, cmds: Sequence[Sequence]) -> List[int]:
        """PFCOUNT batch: command i counts the union of keys cmds[i]."""
        nk = np.fromiter((len(c) for c in cmds), dtype=np.uint32, count=len(cmds))
        koff, kbuf = pack([_b(k) for c in cmds for k in c])
        out = np.zeros(len(cmds), dtype=np.int64)
        self._check(self.lib.sk_pfcount(self.ctx, len(cmds), _addr(nk), _addr(koff), _addr(kbuf), _addr(out)))
        return [int(x) for x in out]

    def pfcount_ids(self, key_ids) -> np.ndarray:
        """Per-key PFCOUNT of slab ids from hll_resolve (int64 array)."""
        ids = np.ascontiguousarray(key_ids, dtype=np.uint32)
        out = np.zeros(len(ids), dtype=np.int64)
        self._check(self.lib.sk_pfcount_ids(self.ctx, len(ids), _addr(ids), _addr(out)))
        return out

    def pfmerge(self, dest, srcs: Sequence):
        d = _b(dest)
        soff, sbuf = pack([_b(s) for s in srcs])
        self._check(self.lib.sk_pfmerge(self.ctx, d, len(d), len(srcs), _addr(soff), _addr(sbuf)))

    def hll_sum_dev(self, n: int, d_ids, d_out):
        """Per-key exact register sums (k_hll_sum): d_out u64[2n] = (sum 2^(40-r), zeros | (any r >= 40) << 32)."""
        self._check(self.lib.sk_hll_sum_dev(self.ctx, n, _addr(d_ids), _addr(d_out)))

    def hll_histogram_dev(self, n: int, d_ids, d_hist):
        self._check(self.lib.sk_hll_histogram_dev(self.ctx, n, _addr(d_ids), _addr(d_hist)))

    def hll_union_keys(self, keys, n_gpus: int, rank: int, d_out) -> int:
        """Register max of the existing HLLs among `keys` (a sequence, or a pack() result) owned by `rank` under
        calcSlot % n_gpus, into d_out (16384 B device); returns how many were merged."""
        off, buf = keys if isinstance(keys, tuple) else pack([_b(k) for k in keys])
        used = ctypes.c_uint32()
        n = len(off) - 1
        self._check(self.lib.sk_hll_union_keys(self.ctx, n, _addr(off), _addr(buf), n_gpus, rank, _addr(d_out),
                                               ctypes.addressof(used)))
        return int(used.value)

    def hll_count_registers_dev(self, d_regs) -> int:
        """PFCOUNT (multi-key / raw semantics) of 16384 registers in device memory."""
        v = ctypes.c_int64()
        self._check(self.lib.sk_hll_count_registers_dev(self.ctx, _addr(d_regs), ctypes.addressof(v)))
        return int(v.value)

    def hll_epoch(self) -> int:
        """HLL keyspace epoch: moves whenever an HLL key is created or removed (sk_hll_epoch)."""
        v = ctypes.c_uint64()
        self._check(self.lib.sk_hll_epoch(self.ctx, ctypes.addressof(v)))
        return int(v.value)

    def hll_union_dev(self, n: int, d_ids, d_out):
        self._check(self.lib.sk_hll_union_dev(self.ctx, n, _addr(d_ids), _addr(d_out)))

    def hll_merge_registers_dev(self, key, d_regs):
        k = _b(key)
        self._check(self.lib.sk_hll_merge_registers_dev(self.ctx, k, len(k), _addr(d_regs)))

    def hll_registers(self, key) -> np.ndarray:
        k = _b(key)
        out = np.zeros(16384, dtype=np.uint8)
        self._check(self.lib.sk_hll_registers(self.ctx, k, len(k), _addr(out)))
        return out

    def estimate_hist(self, hist64) -> int:
        h = np.ascontiguousarray(hist64, dtype=np.uint32)
        return int(self.lib.sk_hll_estimate_hist(_addr(h), self.redis_major))

    # ------------------------------------------------------------ bits
    def setbit(self, keys: Sequence, offsets: Sequence[int], values: Sequence[int], want_old: bool = True):
        n = len(keys)
        koff, kbuf = pack([_b(k) for k in keys])
        offs = np.asarray(offsets, dtype=np.uint64)
        vals = np.asarray(values, dtype=np.uint8)
        out = np.zeros(n, dtype=np.uint8) if want_old else None
        self._check(self.lib.sk_setbit(self.ctx, n, _addr(koff), _addr(kbuf), _addr(offs), _addr(vals),
                                       _addr(out)))
        return [int(x) for x in out] if want_old else None

    def getbit(self, keys: Sequence, offsets: Sequence[int]) -> List[int]:
        n = len(keys)
        koff, kbuf = pack([_b(k) for k in keys])
        offs = np.asarray(offsets, dtype=np.uint64)
        out = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.sk_getbit(self.ctx, n, _addr(koff), _addr(kbuf), _addr(offs), _addr(out)))
        return [int(x) for x in out]

    def setbit_packed(self, koff, kbuf, offsets, values, out=None):
        """sk_setbit over caller-packed key names (koff u64[n + 1] into kbuf) and host arrays, as the JNI shim passes
        them; out: u8[n] for the old bits, None for SETBIT_VOID."""
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        vals = np.ascontiguousarray(values, dtype=np.uint8)
        self._check(self.lib.sk_setbit(self.ctx, len(offs), _addr(koff), _addr(kbuf), _addr(offs), _addr(vals),
                                       _addr(out)))

    def getbit_packed(self, koff, kbuf, offsets, out):
        """sk_getbit over caller-packed key names and host arrays (out: u8[n])."""
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        self._check(self.lib.sk_getbit(self.ctx, len(offs), _addr(koff), _addr(kbuf), _addr(offs), _addr(out)))

    def setbit_dev(self, key, n: int, d_offsets, value: int, d_out_old=None):
        k = _b(key)
        self._check(self.lib.sk_setbit_dev(self.ctx, k, len(k), n, _addr(d_offsets), value, _addr(d_out_old)))

    def getbit_dev(self, key, n: int, d_offsets, d_out):
        k = _b(key)
        self._check(self.lib.sk_getbit_dev(self.ctx, k, len(k), n, _addr(d_offsets), _addr(d_out)))

    def setbit_values_dev(self, key, n: int, d_offsets, d_values, d_out_old=None):
        """SETBIT of a device batch with one value per op (u8); old bits in d_out_old if given."""
        k = _b(key)
        self._check(self.lib.sk_setbit_values_dev(self.ctx, k, len(k), n, _addr(d_offsets), _addr(d_values),
                                                  _addr(d_out_old)))

    def route_bits(self, n: int, d_offsets, d_values, shard_bits: int, world: int, d_send, d_send_values,
                   d_dst) -> np.ndarray:
        """Split a device batch of logical bit offsets by owner shard (sk_route_bits): ops per shard (u64)."""
        out = np.zeros(world, dtype=np.uint64)
        self._check(self.lib.sk_route_bits(self.ctx, n, _addr(d_offsets), _addr(d_values), int(shard_bits), world,
                                           _addr(d_send), _addr(d_send_values), _addr(d_dst), _addr(out)))
        return out

    def bloom_indexes_dev(self, n: int, d_off, d_bytes, size: int, k: int, nprobe: int, d_idx):
        """Probe bit indexes of n device elements, element-major u64[n * nprobe] (sk_bloom_indexes_dev)."""
        self._check(self.lib.sk_bloom_indexes_dev(self.ctx, n, _addr(d_off), _addr(d_bytes), int(size), int(k),
                                                  int(nprobe), _addr(d_idx)))

    def reduce_groups_u8(self, n: int, group: int, take: int, invert: bool, d_in, d_out):
        """d_out[i] = AND(d_in[i * group .. i * group + take)) ^ invert (sk_reduce_groups_u8)."""
        self._check(self.lib.sk_reduce_groups_u8(self.ctx, n, group, take, 1 if invert else 0, _addr(d_in),
                                                 _addr(d_out)))

    def d2d(self, d_dst, d_src, n: int):
        self._check(self.lib.sk_d2d(self.ctx, _addr(d_dst), _addr(d_src), n))

    def unroute_u8(self, n: int, d_dst, d_rep, d_out):
        self._check(self.lib.sk_unroute_u8(self.ctx, n, _addr(d_dst), _addr(d_rep), _addr(d_out)))

    def alltoallv(self, d_send, send_bytes, d_recv, recv_bytes):
        sb = np.ascontiguousarray(send_bytes, dtype=np.uint64)
        rb = np.ascontiguousarray(recv_bytes, dtype=np.uint64)
        self._check(self.lib.sk_alltoallv(self.ctx, _addr(d_send), _addr(sb), _addr(d_recv), _addr(rb)))

    def set_bit_range(self, key, frm: int, to: int, value: int):
        """RBitSet.set(from, to) / clear(from, to): bits [from, to) := value."""
        k = _b(key)
        self._check(self.lib.sk_set_bit_range(self.ctx, k, len(k), int(frm), int(to), int(value)))

    def bitcount(self, key) -> int:
        k = _b(key)
        out = ctypes.c_uint64()
        self._check(self.lib.sk_bitcount(self.ctx, k, len(k), ctypes.addressof(out)))
        return out.value

    def strlen(self, key) -> int:
        k = _b(key)
        out = ctypes.c_uint64()
        self._check(self.lib.sk_strlen(self.ctx, k, len(k), ctypes.addressof(out)))
        return out.value

    def bitop(self, op: str, dest, srcs: Sequence) -> int:
        d = _b(dest)
        soff, sbuf = pack([_b(s) for s in srcs])
        out = ctypes.c_uint64()
        self._check(self.lib.sk_bitop(self.ctx, N.SK_BITOP[op.upper()], d, len(d), len(srcs), _addr(soff),
                                      _addr(sbuf), ctypes.addressof(out)))
        return out.value

    def get(self, key):
        k = _b(key)
        ln = ctypes.c_int64()
        self._check(self.lib.sk_get(self.ctx, k, len(k), None, 0, ctypes.addressof(ln)))
        if ln.value < 0:
            return None
        buf = np.zeros(max(ln.value, 1), dtype=np.uint8)
        self._check(self.lib.sk_get(self.ctx, k, len(k), _addr(buf), ln.value, ctypes.addressof(ln)))
        return buf[: ln.value].tobytes()

    def set(self, key, value: bytes):
        k = _b(key)
        v = np.frombuffer(bytes(value) + b"\0", dtype=np.uint8)
        self._check(self.lib.sk_set(self.ctx, k, len(k), _addr(v), len(value)))

    # ------------------------------------------------------------ persistence (redis-server's DUMP / RDB formats)
    def scan(self, cursor: int = 0, count: int = 1000):
        """SCAN: (next cursor, [(key bytes, SK_TYPE_*)]); next cursor 0 = done."""
        cap = 1 << 20
        nxt, n = ctypes.c_uint64(), ctypes.c_uint32()
        off = np.zeros(count + 1, dtype=np.uint64)
        names = np.zeros(cap, dtype=np.uint8)
        types = np.zeros(max(count, 1), dtype=np.int32)
        self._check(self.lib.sk_scan(self.ctx, int(cursor), int(count), ctypes.addressof(nxt), ctypes.addressof(n),
                                     _addr(off), _addr(names), cap, _addr(types)))
        raw = names.tobytes()
        return nxt.value, [(raw[off[i]:off[i + 1]], int(types[i])) for i in range(n.value)]

    def dbsize(self) -> int:
        """DBSIZE: keys in the store (HLLs, strings, Bloom filter configs)."""
        n = ctypes.c_uint64()
        self._check(self.lib.sk_dbsize(self.ctx, ctypes.addressof(n)))
        return n.value

    def keys(self) -> List[tuple]:
        """Every (key, type) of the store, by a full SCAN."""
        out, cur = [], 0
        while True:
            cur, part = self.scan(cur, 4096)
            out += part
            if not cur:
                return out

    def dump(self, key):
        """DUMP key: redis-server's payload (type, value, RDB version, CRC64), or None."""
        k = _b(key)
        ln = ctypes.c_int64()
        self._check(self.lib.sk_dump(self.ctx, k, len(k), None, 0, ctypes.addressof(ln)))
        if ln.value < 0:
            return None
        buf = np.zeros(max(ln.value, 1), dtype=np.uint8)
        self._check(self.lib.sk_dump(self.ctx, k, len(k), _addr(buf), ln.value, ctypes.addressof(ln)))
        return buf[: ln.value].tobytes()

    def restore(self, key, payload: bytes, replace: bool = False):
        """RESTORE key 0 payload [REPLACE]."""
        k = _b(key)
        v = np.frombuffer(bytes(payload) + b"\0", dtype=np.uint8)
        self._check(self.lib.sk_restore(self.ctx, k, len(k), _addr(v), len(payload), int(replace)))

    def save(self, path, extra=()) -> int:
        """SAVE the whole store as an RDB file; extra: (key, DUMP payload) pairs written with it.  Keys written."""
        items = [bytes(x) for kv in extra for x in (_b(kv[0]), kv[1])]
        off, buf = pack(items) if items else (np.zeros(1, dtype=np.uint64), np.zeros(16, dtype=np.uint8))
        n = ctypes.c_uint64()
        self._check(self.lib.sk_save(self.ctx, os.fsencode(path), len(extra), _addr(off), _addr(buf),
                                     ctypes.addressof(n)))
        return n.value

    def load(self, path) -> int:
        """Load an RDB file (this store's SAVE or redis-server's dump.rdb of strings / hashes).  Keys read."""
        n = ctypes.c_uint64()
        self._check(self.lib.sk_load(self.ctx, os.fsencode(path), None, None, ctypes.addressof(n)))
        return n.value

    def get_dev(self, key, d_buf, cap: int) -> int:
        """Copy a bit string into device memory (<= cap bytes); its length, or -1 if the key does not exist."""
        k = _b(key)
        ln = ctypes.c_int64()
        self._check(self.lib.sk_get_dev(self.ctx, k, len(k), _addr(d_buf), int(cap), ctypes.addressof(ln)))
        return ln.value

    def set_dev(self, key, d_val, n: int):
        """SET key from n bytes of device memory."""
        k = _b(key)
        self._check(self.lib.sk_set_dev(self.ctx, k, len(k), _addr(d_val), int(n)))

    def bitset_length(self, key) -> int:
        k = _b(key)
        out = ctypes.c_int64()
        self._check(self.lib.sk_bitset_length(self.ctx, k, len(k), ctypes.addressof(out)))
        return out.value

    # ------------------------------------------------------------ Bloom
    def bloom_try_init(self, name, expected: int, fpp: float) -> bool:
        k = _b(name)
        ok = ctypes.c_int()
        self._check(self.lib.sk_bloom_try_init(self.ctx, k, len(k), expected, fpp, ctypes.addressof(ok)))
        return bool(ok.value)

    def bloom_config(self, name):
        k = _b(name)
        size, kk, exp, fpp = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_double()
        self._check(self.lib.sk_bloom_config(self.ctx, k, len(k), ctypes.addressof(size), ctypes.addressof(kk),
                                             ctypes.addressof(exp), ctypes.addressof(fpp)))
        return size.value, kk.value, exp.value, fpp.value

    def bloom_add(self, name, size: int, k: int, elems: Sequence[bytes]) -> List[bool]:
        nm = _b(name)
        off, buf = pack(list(elems))
        out = np.zeros(len(elems), dtype=np.uint8)
        self._check(self.lib.sk_bloom_add(self.ctx, nm, len(nm), size, k, len(elems), _addr(off), _addr(buf),
                                          _addr(out)))
        return [bool(x) for x in out]

    def bloom_contains(self, name, size: int, k: int, elems: Sequence[bytes]) -> List[bool]:
        nm = _b(name)
        off, buf = pack(list(elems))
        out = np.zeros(len(elems), dtype=np.uint8)
        self._check(self.lib.sk_bloom_contains(self.ctx, nm, len(nm), size, k, len(elems), _addr(off),
                                               _addr(buf), _addr(out)))
        return [bool(x) for x in out]

    def bloom_add_dev(self, name, n: int, d_off, d_bytes, bytes_len: int, d_out):
        nm = _b(name)
        self._check(self.lib.sk_bloom_add_dev(self.ctx, nm, len(nm), n, _addr(d_off), _addr(d_bytes), bytes_len,
                                              _addr(d_out)))

    def bloom_contains_dev(self, name, n: int, d_off, d_bytes, bytes_len: int, d_out):
        nm = _b(name)
        self._check(self.lib.sk_bloom_contains_dev(self.ctx, nm, len(nm), n, _addr(d_off), _addr(d_bytes),
                                                   bytes_len, _addr(d_out)))

    def bloom_prefix(self, op: str, name, size: int, k: int, prefix: bytes, suffixes: Sequence[bytes]) -> List[bool]:
        """add / contains of elements prefix + suffixes[i] (sk_bloom_add_prefix / sk_bloom_contains_prefix)."""
        nm = _b(name)
        soff, sbuf = pack_u32(suffixes)
        pre = np.frombuffer(bytes(prefix) or b"\0", dtype=np.uint8)
        out = np.zeros(len(suffixes), dtype=np.uint8)
        fn = self.lib.sk_bloom_add_prefix if op == "add" else self.lib.sk_bloom_contains_prefix
        self._check(fn(self.ctx, nm, len(nm), size, k, len(suffixes), _addr(pre), len(prefix), _addr(soff),
                       _addr(sbuf), _addr(out)))
        return [bool(x) for x in out]

    def bloom_count(self, name) -> int:
        nm = _b(name)
        out = ctypes.c_int32()
        self._check(self.lib.sk_bloom_count(self.ctx, nm, len(nm), ctypes.addressof(out)))
        return out.value


# ---------------------------------------------------------------- host-only
def device_count() -> int:
    return int(N.load().sk_device_count())


def calc_slot(key) -> int:
    k = _b(key)
    return int(N.load().sk_calc_slot(k, len(k)))


def crc16(data: bytes) -> int:
    return int(N.load().sk_crc16(bytes(data), len(data)))


def owner(key, n_gpus: int) -> int:
    k = _b(key)
    return int(N.load().sk_owner(k, len(k), n_gpus))


def owners(keys: Sequence, n_gpus: int) -> np.ndarray:
    """owner() of many keys in one call (int32; -1 where calcSlot throws); keys: a sequence or a pack()."""
    off, buf = keys if isinstance(keys, tuple) else pack([_b(k) for k in keys])
    out = np.zeros(len(off) - 1, dtype=np.int32)
    N.load().sk_owner_many(len(out), _addr(off), _addr(buf), n_gpus, _addr(out))
    return out


def bloom_optimal_bits(n: int, p: float) -> int:
    return int(N.load().sk_bloom_optimal_bits(n, p))


def bloom_optimal_k(n: int, m: int) -> int:
    return int(N.load().sk_bloom_optimal_k(n, m))


def gen_jackson_longs(seed: int, n: int):
    """(off u64[n+1], bytes u8[total+16]) of ["java.lang.Long",v] for SplitMix64(seed)."""
    lib = N.load()
    off = np.zeros(n + 1, dtype=np.uint64)
    lib.sk_gen_jackson_longs(seed, n, off.ctypes.data, None)
    buf = np.zeros(int(off[n]) + 16, dtype=np.uint8)
    lib.sk_gen_jackson_longs(seed, n, off.ctypes.data, buf.ctypes.data)
    return off, buf
