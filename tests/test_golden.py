"""Golden fixtures (tests/golden/golden_v1.json, made by make_golden.py from the
pinned oracle): the oracle must still reproduce them (CPU), and the GPU path
must reproduce them bit for bit (gpu)."""
import base64
import json
import os

import numpy as np
import pytest

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.json")))


def test_oracle_reproduces_hash_vectors(O):
    for h in G["hashes"]:
        b = bytes.fromhex(h["in"])
        assert "%016x" % O.murmur64a(b) == h["murmur64a"]
        assert "%016x" % O.xxh64(b) == h["xxh64"]
        assert "%016x" % O.farmhash_uo64(b) == h["farm_uo64"]
        assert O.hll_patlen(b, 3) == (h["reg"], h["rho3"])
        assert O.hll_patlen(b, 5) == (h["reg"], h["rho5"])


def test_oracle_reproduces_slots_and_bloom(O):
    for k, s in G["calc_slot"].items():
        assert O.calc_slot(k) == s
    for c in G["bloom_sizing"]:
        m = O.bloom_optimal_bits(c["n"], c["p"])
        assert (m, O.bloom_optimal_k(c["n"], m)) == (c["size"], c["k"])
        for e, idx in c["indexes"].items():
            assert O.bloom_indexes(e.encode(), c["k"], c["size"]) == idx


def test_oracle_reproduces_hll_and_bloom_state(O):
    h = G["hll"]
    st = O.HLLStore()
    keys = [k.encode() for k in h["keys"]]
    els = [e.encode() for e in h["elements"]]
    rep = st.pfadd(keys, [[e] for e in els])
    assert "".join("1" if r else "0" for r in rep) == h["replies"]
    for k, d in h["dense"].items():
        assert O.dense_pack(st.regs[k.encode()]) == base64.b64decode(d)
        assert O.count_regs(st.regs[k.encode()], 1, 3) == h["count_v3"][k]
        assert O.count_regs(st.regs[k.encode()], 1, 5) == h["count_v5"][k]


@pytest.mark.gpu
def test_gpu_reproduces_golden(engine):
    from redisson_amd import calc_slot

    for k, s in G["calc_slot"].items():
        assert calc_slot(k) == s
    h = G["hll"]
    keys = [("gold:" + k).encode() for k in h["keys"]]
    els = [e.encode() for e in h["elements"]]
    rep = engine.pfadd(keys, [[e] for e in els])
    assert "".join("1" if r else "0" for r in rep) == h["replies"]
    for k, d in h["dense"].items():
        raw = engine.get(b"gold:" + k.encode())
        assert raw[:4] == b"HYLL" and raw[16:] == base64.b64decode(d)
        assert engine.pfcount([[b"gold:" + k.encode()]]) == [h["count_v3"][k]]
    assert engine.pfcount([[b"gold:" + k.encode() for k in sorted(h["dense"])]]) == [h["union_v3"]]

    b = G["bloom"]
    assert engine.bloom_try_init("gold:bf", 2000, 0.01)
    size, k, _, _ = engine.bloom_config("gold:bf")
    assert (size, k) == (b["size"], b["k"])
    from tests.golden.make_golden import jlongs  # noqa: E402  (same seeded inputs)

    adds = jlongs(0x5EED0004, 2000)
    r = engine.bloom_add("gold:bf", size, k, adds)
    assert "".join("1" if x else "0" for x in r) == b["add_replies"]
    probes = adds[::4] + jlongs(0x5EED0005, 1000)
    r = engine.bloom_contains("gold:bf", size, k, probes)
    assert "".join("1" if x else "0" for x in r) == b["contains_replies"]
    assert engine.get("gold:bf") == base64.b64decode(b["bits"])
    assert engine.bloom_count("gold:bf") == b["count"]

    bo = G["bitop"]
    engine.set(b"gold:a", bytes.fromhex(bo["a"]))
    engine.set(b"gold:b", bytes.fromhex(bo["b"]))
    for op in ["AND", "OR", "XOR"]:
        engine.bitop(op, b"gold:r", [b"gold:a", b"gold:b", b"gold:none"])
        assert engine.get(b"gold:r").hex() == bo[op]
    engine.bitop("NOT", b"gold:r", [b"gold:a"])
    assert engine.get(b"gold:r").hex() == bo["NOT"]
