"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / CPU comparator.  The product
(redisson_amd, libredisson_sketch.so) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        sig = {
            "or_murmur64a": (c_uint64, [c_void_p, c_int64, c_uint64]),
            "or_murmur64a_verification": (c_uint32, []),
            "or_xxh64": (c_uint64, [c_void_p, c_uint64, c_uint64]),
            "or_farmhash_na64": (c_uint64, [c_void_p, c_uint64]),
            "or_farmhash_uo64": (c_uint64, [c_void_p, c_uint64]),
            "or_crc16": (c_uint32, [c_void_p, c_uint64]),
            "or_calc_slot": (c_int32, [c_void_p, c_uint64]),
            "or_hll_patlen": (c_int, [c_void_p, c_uint64, c_int, c_void_p]),
            "or_hll_add": (c_int, [c_void_p, c_void_p, c_uint64, c_int]),
            "or_pfadd_batch": (None, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                      c_void_p]),
            "or_hll_sum": (c_double, [c_void_p, c_int, c_void_p]),
            "or_hll_count": (c_uint64, [c_void_p, c_int, c_int]),
            "or_hll_histogram": (None, [c_void_p, c_void_p]),
            "or_hll_union": (None, [c_void_p, c_uint32, c_void_p]),
            "or_hll_dense_pack": (None, [c_void_p, c_void_p]),
            "or_hll_dense_unpack": (None, [c_void_p, c_void_p]),
            "or_bloom_optimal_bits": (c_int64, [c_int64, c_double]),
            "or_bloom_optimal_k": (c_int32, [c_int64, c_int64]),
            "or_bloom_indexes": (None, [c_void_p, c_uint64, c_int32, c_int64, c_void_p]),
            "or_bloom_count": (c_int32, [c_int64, c_int32, c_int64]),
            "or_bloom_add_batch": (None, [c_void_p, c_void_p, c_int64, c_int32, c_uint32, c_void_p, c_void_p,
                                          c_void_p]),
            "or_bloom_contains_batch": (None, [c_void_p, c_uint64, c_int64, c_int32, c_uint32, c_void_p, c_void_p,
                                               c_void_p]),
            "or_pfadd_owned_mt": (None, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                         c_int]),
            "or_bloom_contains_mt": (None, [c_void_p, c_uint64, c_int64, c_int32, c_uint32, c_void_p, c_void_p,
                                            c_void_p, c_int]),
            "or_gen_jackson_long": (c_uint32, [c_uint64, c_uint64, c_void_p]),
            "or_pfadd_gen_mt": (c_uint64, [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_int,
                                           c_void_p, c_int]),
            "or_hll_union_gen_mt": (None, [c_void_p, c_uint64, c_uint64, c_uint64, c_int, c_int]),
            "or_bloom_add_gen_mt": (c_uint64, [c_void_p, c_int64, c_int32, c_uint64, c_uint64, c_uint64, c_int]),
            "or_bloom_add_gen_seq": (c_uint64, [c_void_p, c_int64, c_int32, c_uint64, c_uint64, c_uint64, c_void_p]),
            "or_hllstr_new": (c_uint64, [c_void_p]),
            "or_hllstr_to_dense": (c_int, [c_void_p, c_void_p]),
            "or_hllstr_set": (c_int, [c_void_p, c_void_p, ctypes.c_long, ctypes.c_uint8]),
            "or_hllstr_pfadd": (c_int, [c_void_p, c_void_p, c_int, c_uint32, c_void_p, c_void_p, c_int]),
            "or_hllstr_registers": (c_int, [c_void_p, c_uint64, c_void_p]),
            "or_bloom_add_idx_seq": (c_uint64, [c_void_p, c_uint64, c_int64, c_int32, c_uint64, c_void_p, c_uint64,
                                                c_void_p]),
            "or_bloom_contains_gen_mt": (None, [c_void_p, c_uint64, c_int64, c_int32, c_uint64, c_void_p, c_uint64,
                                                c_void_p, c_int]),
            "or_setbits_mt": (None, [c_void_p, c_void_p, c_uint64, c_int]),
            "or_getbit": (c_int, [c_void_p, c_uint64, c_uint64]),
            "or_setbit": (c_int, [c_void_p, c_void_p, c_uint64, c_int]),
            "or_bitcount": (c_uint64, [c_void_p, c_uint64]),
            "or_bitop": (c_uint64, [c_int, c_void_p, c_void_p, c_void_p, c_uint32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if isinstance(a, np.ndarray) else a


def pack(items):
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        np.cumsum([len(x) for x in items], out=off[1:])
    blob = b"".join(items) + b"\0" * 16
    return off, np.frombuffer(blob, dtype=np.uint8).copy()


# ---- hashes ------------------------------------------------------------
def murmur64a(b: bytes, seed: int = 0xADC83B19) -> int:
    return lib().or_murmur64a(b, len(b), seed)


def xxh64(b: bytes) -> int:
    return lib().or_xxh64(b, len(b), 0)


def farmhash_na64(b: bytes) -> int:
    return lib().or_farmhash_na64(b, len(b))


def farmhash_uo64(b: bytes) -> int:
    return lib().or_farmhash_uo64(b, len(b))


def crc16(b: bytes) -> int:
    return lib().or_crc16(b, len(b))


def calc_slot(key) -> int:
    b = key.encode() if isinstance(key, str) else key
    return lib().or_calc_slot(b, len(b))


# ---- HLL -----------------------------------------------------------------
def hll_patlen(b: bytes, redis_major: int = 3):
    reg = c_int64()
    cnt = lib().or_hll_patlen(b, len(b), redis_major, ctypes.addressof(reg))
    return reg.value, cnt


class HLLStore:
    """Reference keyspace of HLLs (unpacked registers), redis semantics."""

    def __init__(self, redis_major: int = 3):
        self.m = redis_major
        self.regs = {}

    def pfadd(self, keys, elems):
        out = []
        for k, es in zip(keys, elems):
            created = k not in self.regs
            r = self.regs.setdefault(k, np.zeros(16384, dtype=np.uint8))
            ch = created
            for e in es:
                ch |= bool(lib().or_hll_add(r.ctypes.data, e, len(e), self.m))
            out.append(ch)
        return out

    def pfadd_bulk(self, key_ids: np.ndarray, off: np.ndarray, buf: np.ndarray, n_keys: int):
        """One element per command, key given by integer id (fast C loop)."""
        regs = np.zeros((n_keys, 16384), dtype=np.uint8)
        exists = np.zeros(n_keys, dtype=np.uint8)
        n = len(key_ids)
        counts = np.ones(n, dtype=np.uint32)
        out = np.zeros(n, dtype=np.uint8)
        ids = np.ascontiguousarray(key_ids, dtype=np.uint32)
        lib().or_pfadd_batch(regs.ctypes.data, exists.ctypes.data, n, ids.ctypes.data, counts.ctypes.data,
                             off.ctypes.data, buf.ctypes.data, self.m, out.ctypes.data)
        return regs, out

    def pfadd_bulk_mt(self, key_ids: np.ndarray, off: np.ndarray, buf: np.ndarray, n_keys: int, threads: int):
        """pfadd_bulk on `threads` host threads, each owning the keys id % threads (oracle_mt.c)."""
        regs = np.zeros((n_keys, 16384), dtype=np.uint8)
        exists = np.zeros(n_keys, dtype=np.uint8)
        n = len(key_ids)
        out = np.zeros(n, dtype=np.uint8)
        ids = np.ascontiguousarray(key_ids, dtype=np.uint32)
        lib().or_pfadd_owned_mt(regs.ctypes.data, exists.ctypes.data, n, ids.ctypes.data, off.ctypes.data,
                                buf.ctypes.data, self.m, out.ctypes.data, threads)
        return regs, out

    def count(self, keys):
        keys = [k for k in keys if k in self.regs]
        if len(keys) == 1 or (len(keys) == 0):
            r = self.regs[keys[0]] if keys else np.zeros(16384, dtype=np.uint8)
            return count_regs(r, 1, self.m)
        u = np.maximum.reduce([self.regs[k] for k in keys])
        return count_regs(u, 2, self.m)

    def merge(self, dest, srcs):
        arrs = [self.regs[k] for k in srcs if k in self.regs]
        d = self.regs.setdefault(dest, np.zeros(16384, dtype=np.uint8))
        for a in arrs:
            np.maximum(d, a, out=d)


class HLLStrStore:
    """Reference keyspace of HLL strings byte for byte as redis-server 3.2 keeps them (hyperloglog.c): keys start
    sparse (createHLLObject), PFADD runs hllSparseSet per element (promotion past 3000 bytes or a value > 32),
    the 8 cached-cardinality bytes follow PFADD (invalidate), single-key PFCOUNT (store) and PFMERGE
    (dest made dense, invalidated)."""

    CAP = 16 + 12288 + 64

    def __init__(self, redis_major: int = 3):
        self.m = redis_major
        self.s = {}

    def _new(self):
        b = np.zeros(self.CAP, dtype=np.uint8)
        n = c_uint64(lib().or_hllstr_new(b.ctypes.data))
        return [b, n]

    def pfadd(self, key, elems) -> int:
        created = key not in self.s
        if created:
            self.s[key] = self._new()
        b, n = self.s[key]
        off, buf = pack(list(elems))
        r = lib().or_hllstr_pfadd(b.ctypes.data, ctypes.addressof(n), int(created), len(elems), off.ctypes.data,
                                  buf.ctypes.data, self.m)
        assert r >= 0, "corrupted HLL"
        return r

    def registers(self, key) -> np.ndarray:
        regs = np.zeros(16384, dtype=np.uint8)
        if key in self.s:
            b, n = self.s[key]
            assert lib().or_hllstr_registers(b.ctypes.data, n.value, regs.ctypes.data) == 0
        return regs

    def pfcount(self, keys) -> int:
        if len(keys) == 1:
            k = keys[0]
            if k not in self.s:
                return 0
            b, n = self.s[k]
            if not (b[15] & 0x80):                      # valid cache
                return int.from_bytes(bytes(b[8:16]), "little")
            enc = 0 if b[4] == 1 else 1                  # sparse sum (exact) / dense sum order
            c = count_regs(self.registers(k), enc, self.m)
            b[8:16] = np.frombuffer(int(c).to_bytes(8, "little"), np.uint8)
            return c
        u = np.maximum.reduce([self.registers(k) for k in keys])
        return count_regs(u, 2, self.m)

    def pfmerge(self, dest, srcs):
        u = np.maximum.reduce([self.registers(k) for k in [dest] + list(srcs)])
        if dest not in self.s:
            self.s[dest] = self._new()
        b, n = self.s[dest]
        assert lib().or_hllstr_to_dense(b.ctypes.data, ctypes.addressof(n)) == 0
        b[16:16 + 12288] = np.frombuffer(dense_pack(u), np.uint8)
        b[15] |= 0x80

    def get(self, key):
        if key not in self.s:
            return None
        b, n = self.s[key]
        return b[:n.value].tobytes()

    def set(self, key, value: bytes):
        b = np.zeros(self.CAP, dtype=np.uint8)
        b[:len(value)] = np.frombuffer(value, np.uint8)
        self.s[key] = [b, c_uint64(len(value))]


def count_regs(regs: np.ndarray, encoding: int = 1, redis_major: int = 3) -> int:
    r = np.ascontiguousarray(regs, dtype=np.uint8)
    return lib().or_hll_count(r.ctypes.data, encoding, redis_major)


def hll_histogram(regs: np.ndarray) -> np.ndarray:
    h = np.zeros(64, dtype=np.uint32)
    r = np.ascontiguousarray(regs, dtype=np.uint8)
    lib().or_hll_histogram(r.ctypes.data, h.ctypes.data)
    return h


def dense_pack(regs: np.ndarray) -> bytes:
    out = np.zeros(12288, dtype=np.uint8)
    r = np.ascontiguousarray(regs, dtype=np.uint8)
    lib().or_hll_dense_pack(r.ctypes.data, out.ctypes.data)
    return out.tobytes()


def hll_string(regs: np.ndarray, encoding: str = "dense", card: int = None) -> bytes:
    """A Redis 3.2 HLL string (hyperloglog.c struct hllhdr + registers).

    dense: HLL_DENSE_SET_REGISTER packing; sparse: a canonical opcode stream
    (zero runs as XZERO when longer than 64, else ZERO; equal non-zero values
    as VAL runs of at most 4) -- one of the valid sparse forms redis-server
    reads (its own writer may split VAL runs differently, by update order).
    card: cached cardinality (valid) or None (the invalid flag, MSB of byte 15)."""
    hdr = bytearray(b"HYLL" + bytes([0 if encoding == "dense" else 1, 0, 0, 0]) + bytes(8))
    if card is None:
        hdr[15] = 0x80
    else:
        hdr[8:16] = int(card).to_bytes(8, "little")
    if encoding == "dense":
        return bytes(hdr) + dense_pack(regs)
    r = [int(x) for x in regs]
    assert max(r) <= 32, "sparse VAL opcodes hold values 1..32"
    out, i = bytearray(), 0
    while i < 16384:
        j = i
        while j < 16384 and r[j] == r[i]:
            j += 1
        run = j - i
        if r[i] == 0:
            while run:
                n = min(run, 16384)
                if n > 64:
                    out += bytes([0x40 | ((n - 1) >> 8), (n - 1) & 0xFF])
                else:
                    out.append(n - 1)
                run -= n
        else:
            while run:
                n = min(run, 4)
                out.append(0x80 | ((r[i] - 1) << 2) | (n - 1))
                run -= n
        i = j
    return bytes(hdr) + bytes(out)


def hll_decode(s: bytes):
    """Registers of a Redis HLL string (dense or sparse), or None if it is not one."""
    if len(s) < 16 or s[:4] != b"HYLL" or s[4] > 1:
        return None
    regs = np.zeros(16384, dtype=np.uint8)
    if s[4] == 0:
        if len(s) != 16 + 12288:
            return None
        bits = np.unpackbits(np.frombuffer(s[16:], dtype=np.uint8), bitorder="little").reshape(16384, 6)
        return (bits * (1 << np.arange(6))).sum(axis=1).astype(np.uint8)
    i, p = 0, 16
    while p < len(s):
        op = s[p]
        if op & 0xC0 == 0:
            run, val, p = (op & 0x3F) + 1, 0, p + 1
        elif op & 0xC0 == 0x40:
            run, val, p = (((op & 0x3F) << 8) | s[p + 1]) + 1, 0, p + 2
        else:
            run, val, p = (op & 3) + 1, ((op >> 2) & 31) + 1, p + 1
        if i + run > 16384:
            return None
        regs[i:i + run] = val
        i += run
    return regs if i == 16384 else None


# ---- Bloom ---------------------------------------------------------------
def bloom_optimal_bits(n, p):
    return lib().or_bloom_optimal_bits(n, p)


def bloom_optimal_k(n, m):
    return lib().or_bloom_optimal_k(n, m)


def bloom_indexes(b: bytes, k: int, size: int):
    out = np.zeros(k, dtype=np.int64)
    lib().or_bloom_indexes(b, len(b), k, size, out.ctypes.data)
    return [int(x) for x in out]


def bloom_count(size, k, bitcount):
    return lib().or_bloom_count(size, k, bitcount)


class BitString:
    """A redis string used as a bit array (MSB-first), growable."""

    def __init__(self, cap_bytes: int = 16):
        self.buf = np.zeros(max(cap_bytes, 16), dtype=np.uint8)
        self.len = c_uint64(0)

    def reserve(self, nbytes):
        if nbytes > len(self.buf):
            nb = np.zeros(max(nbytes, 2 * len(self.buf)), dtype=np.uint8)
            nb[: len(self.buf)] = self.buf
            self.buf = nb

    def setbit(self, off: int, val: int) -> int:
        self.reserve(off // 8 + 1)
        return lib().or_setbit(self.buf.ctypes.data, ctypes.addressof(self.len), off, val)

    def getbit(self, off: int) -> int:
        return lib().or_getbit(self.buf.ctypes.data, self.len.value, off)

    def bitcount(self) -> int:
        return lib().or_bitcount(self.buf.ctypes.data, self.len.value)

    def bytes(self) -> bytes:
        return self.buf[: self.len.value].tobytes()

    def bloom_add(self, size, k, elems):
        self.reserve((size + 7) // 8)
        off, buf = pack(list(elems))
        out = np.zeros(len(elems), dtype=np.uint8)
        lib().or_bloom_add_batch(self.buf.ctypes.data, ctypes.addressof(self.len), size, k, len(elems),
                                 off.ctypes.data, buf.ctypes.data, out.ctypes.data)
        return [bool(x) for x in out]

    def bloom_contains(self, size, k, elems):
        off, buf = pack(list(elems))
        out = np.zeros(len(elems), dtype=np.uint8)
        lib().or_bloom_contains_batch(self.buf.ctypes.data, self.len.value, size, k, len(elems),
                                      off.ctypes.data, buf.ctypes.data, out.ctypes.data)
        return [bool(x) for x in out]

    def bloom_contains_raw(self, size, k, off, buf):
        n = len(off) - 1
        out = np.zeros(n, dtype=np.uint8)
        lib().or_bloom_contains_batch(self.buf.ctypes.data, self.len.value, size, k, n,
                                      off.ctypes.data, buf.ctypes.data, out.ctypes.data)
        return out

    def bloom_contains_raw_mt(self, size, k, off, buf, threads):
        n = len(off) - 1
        out = np.zeros(n, dtype=np.uint8)
        lib().or_bloom_contains_mt(self.buf.ctypes.data, self.len.value, size, k, n, off.ctypes.data,
                                   buf.ctypes.data, out.ctypes.data, threads)
        return out

    def bloom_add_raw(self, size, k, off, buf):
        self.reserve((size + 7) // 8)
        n = len(off) - 1
        out = np.zeros(n, dtype=np.uint8)
        lib().or_bloom_add_batch(self.buf.ctypes.data, ctypes.addressof(self.len), size, k, n,
                                 off.ctypes.data, buf.ctypes.data, out.ctypes.data)
        return out


def bitop(op: str, srcs):
    """srcs: list of bytes or None (missing key) -> result bytes (b'' deletes)."""
    code = {"AND": 0, "OR": 1, "XOR": 2, "NOT": 3}[op]
    arrs = [np.frombuffer((s or b"") + b"\0", dtype=np.uint8) for s in srcs]
    lens = np.array([len(s or b"") for s in srcs], dtype=np.uint64)
    ptrs = (c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    dst = np.zeros(int(lens.max()) + 1 if len(lens) else 1, dtype=np.uint8)
    n = lib().or_bitop(code, dst.ctypes.data, ptrs, lens.ctypes.data, len(arrs))
    return dst[:n].tobytes()


# ---------------------------------------------------------------- full-size checkers (oracle_mt.c)
def threads() -> int:
    """Host threads for the threaded checkers: the box's CPU share (OMP_NUM_THREADS), else up to 16."""
    import os
    return int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)


def gen_jackson_long(seed: int, i: int) -> bytes:
    """Element i of the synthetic stream `seed`: SplitMix64 -> Jackson ["java.lang.Long",v] bytes."""
    b = ctypes.create_string_buffer(48)
    n = lib().or_gen_jackson_long(seed, i, b)
    return b.raw[:n]


def pfadd_gen(regs: np.ndarray, exists: np.ndarray, key_ids: np.ndarray, seed: int, first: int,
              redis_major: int = 3):
    """PFADD element first+c of stream `seed` into key key_ids[c], in order per key (threads own keys).
    regs: (n_keys, 16384) u8, exists: n_keys u8, both updated; returns (replies u8[n], number of 1s)."""
    ids = np.ascontiguousarray(key_ids, dtype=np.uint32)
    out = np.zeros(len(ids), dtype=np.uint8)
    ones = lib().or_pfadd_gen_mt(regs.ctypes.data, exists.ctypes.data, len(ids), ids.ctypes.data, seed, first,
                                 redis_major, out.ctypes.data, threads())
    return out, int(ones)


def hll_union_gen(n: int, seed: int, first: int = 0, redis_major: int = 3) -> np.ndarray:
    regs = np.zeros(16384, dtype=np.uint8)
    lib().or_hll_union_gen_mt(regs.ctypes.data, n, seed, first, redis_major, threads())
    return regs


def bloom_add_gen(size: int, k: int, seed: int, first: int, n: int):
    """(bit array u8[(size+7)/8], Redis string length) after adding elements first..first+n-1."""
    bits = np.zeros((size + 7) // 8 + 16, dtype=np.uint8)
    ln = lib().or_bloom_add_gen_mt(bits.ctypes.data, size, k, seed, first, n, threads())
    return bits, int(ln)


def bloom_add_gen_seq(size: int, k: int, seed: int, first: int, n: int):
    """(bit array, Redis string length, replies u8[n]) after adding elements first..first+n-1 in order."""
    bits = np.zeros((size + 7) // 8 + 16, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint8)
    ln = lib().or_bloom_add_gen_seq(bits.ctypes.data, size, k, seed, first, n, out.ctypes.data)
    return bits, int(ln), out


def bloom_add_idx_seq(bits: np.ndarray, strlen: int, size: int, k: int, seed: int, idx: np.ndarray):
    """Adds element numbers idx (in order, repeats allowed) to `bits` in place; (new string length, replies)."""
    ix = np.ascontiguousarray(idx, dtype=np.uint64)
    out = np.zeros(len(ix), dtype=np.uint8)
    ln = lib().or_bloom_add_idx_seq(bits.ctypes.data, strlen, size, k, seed, ix.ctypes.data, len(ix), out.ctypes.data)
    return int(ln), out


def bloom_contains_gen(bits: np.ndarray, strlen: int, size: int, k: int, seed: int, idx: np.ndarray) -> np.ndarray:
    ix = np.ascontiguousarray(idx, dtype=np.uint64)
    out = np.zeros(len(ix), dtype=np.uint8)
    lib().or_bloom_contains_gen_mt(bits.ctypes.data, strlen, size, k, seed, ix.ctypes.data, len(ix),
                                   out.ctypes.data, threads())
    return out


def setbits(buf: np.ndarray, offsets: np.ndarray):
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    lib().or_setbits_mt(buf.ctypes.data, o.ctypes.data, len(o), threads())
