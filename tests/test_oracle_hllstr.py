"""The oracle's restatement of redis-server 3.2's HLL string writer (oracle/sketch_oracle.c or_hllstr_*):
internal consistency with the register model, the opcode forms hyperloglog.c's comments spell out, order
dependence of VAL merging, and the promotion rules.  (No redis-server in the image: byte parity against a live
server is unpinned; these pin the restatement against hyperloglog.c's documented behaviour.)"""
import ctypes

import numpy as np


def _new(O):
    b = np.zeros(O.HLLStrStore.CAP, dtype=np.uint8)
    n = ctypes.c_uint64(O.lib().or_hllstr_new(b.ctypes.data))
    return b, n


def _set(O, b, n, idx, val):
    return O.lib().or_hllstr_set(b.ctypes.data, ctypes.addressof(n), idx, val)


def test_fresh_hll_string(O):
    b, n = _new(O)
    assert b[:n.value].tobytes() == b"HYLL\x01\x00\x00\x00" + bytes(8) + b"\x7f\xff"   # XZERO(16384), card 0 valid
    st = O.HLLStrStore()
    assert st.pfadd(b"k", []) == 1                                                  # created: updated
    assert st.get(b"k")[15] == 0x80                                                 # cache marked stale


def test_opcode_splits(O):
    b, n = _new(O)
    assert _set(O, b, n, 0, 3) == 1
    # VAL(3,1) XZERO(16383)
    assert b[16:n.value].tobytes() == bytes([0x80 | (2 << 2), 0x40 | (16382 >> 8), 16382 & 0xFF])
    assert _set(O, b, n, 100, 1) == 1
    # VAL(3,1) XZERO(99) VAL(1,1) XZERO(16283)
    assert b[16:n.value].tobytes() == bytes([0x88, 0x40, 98, 0x80, 0x40 | (16282 >> 8), 16282 & 0xFF])
    assert _set(O, b, n, 100, 1) == 0 and _set(O, b, n, 100, 0) == 0                  # not raised
    assert _set(O, b, n, 102, 1) == 1                                               # XZERO split into ZERO(1) VAL ZERO..
    assert b[16 + 3:16 + 6].tobytes() == bytes([0x80, 0x00, 0x80])


def test_val_merge_depends_on_order(O):
    """Five neighbours of one value: left to right they end VAL(v,4) VAL(v,1); the first one last gives
    VAL(v,1) VAL(v,4) -- the same registers, different bytes (why the writer replays rises in batch order)."""
    a, na = _new(O)
    for i in range(5):
        _set(O, a, na, 10 + i, 2)
    b, nb = _new(O)
    for i in [1, 2, 3, 4, 0]:
        _set(O, b, nb, 10 + i, 2)
    va, vb = a[16:na.value].tobytes(), b[16:nb.value].tobytes()
    assert va != vb
    assert bytes([0x87, 0x84]) in va and bytes([0x84, 0x87]) in vb                  # VAL(2,4) VAL(2,1) / reverse
    ra, rb = np.zeros(16384, np.uint8), np.zeros(16384, np.uint8)
    assert O.lib().or_hllstr_registers(a.ctypes.data, na.value, ra.ctypes.data) == 0
    assert O.lib().or_hllstr_registers(b.ctypes.data, nb.value, rb.ctypes.data) == 0
    assert np.array_equal(ra, rb)


def test_promotion_rules(O):
    b, n = _new(O)
    assert _set(O, b, n, 7, 33) == 1 and b[4] == 0                                 # a value past 32: dense
    regs = np.zeros(16384, np.uint8)
    O.lib().or_hllstr_registers(b.ctypes.data, n.value, regs.ctypes.data)
    assert regs[7] == 33 and regs.sum() == 33 and n.value == 16 + 12288
    b, n = _new(O)
    i = 0
    while b[4] == 1:                                                                # grow until past 3000 bytes
        before = n.value
        _set(O, b, n, i, 1 + (i % 3))
        i += 7
    assert before <= 3000 and n.value == 16 + 12288


def test_sparse_writer_matches_register_model(O):
    rng = np.random.default_rng(0)
    strs, regs = O.HLLStrStore(), O.HLLStore()
    keys = [b"m:%d" % i for i in range(30)]
    for _ in range(4000):
        k = keys[int(rng.integers(0, len(keys)))]
        e = [b"%d" % int(x) for x in rng.integers(0, 10**6, int(rng.integers(0, 3)))]
        assert strs.pfadd(k, e) == int(regs.pfadd([k], [e])[0])
    for k in keys:
        assert np.array_equal(strs.registers(k), regs.regs[k])
        assert strs.pfcount([k]) == regs.count([k])
