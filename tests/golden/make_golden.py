"""Regenerate tests/golden/golden_v1.json from the pinned CPU oracle.

The oracle is pinned first (tests/test_oracle_pins.py: SMHasher, python
xxhash, Guava FarmHash vectors, CRC16 check value, Redis cluster-spec slots,
the reference's own test expectations); these fixtures freeze its outputs on
seeded inputs so the GPU path and any later oracle change are checked against
the same bytes.  Run: python tests/golden/make_golden.py
"""
import base64
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402


def jlongs(seed, n):
    st, M, out = seed, (1 << 64) - 1, []
    for _ in range(n):
        st = (st + 0x9E3779B97F4A7C15) & M
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        v = z - (1 << 64) if z >> 63 else z
        out.append(b'["java.lang.Long",%d]' % v)
    return out


def main():
    rng = np.random.default_rng(20261015)
    inputs = [bytes(range(n)) for n in range(0, 130)]
    inputs += [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 300, 40)]
    inputs += jlongs(0x5EED0000, 30) + [b"1", b"2", b"3", b'"foo"', b'"123"', b'"hflgs;jl;ao1-32471320o31803-24"']
    hashes = []
    for b in inputs:
        r3, c3 = O.hll_patlen(b, 3)
        r5, c5 = O.hll_patlen(b, 5)
        hashes.append({"in": b.hex(), "murmur64a": "%016x" % O.murmur64a(b), "xxh64": "%016x" % O.xxh64(b),
                       "farm_uo64": "%016x" % O.farmhash_uo64(b), "reg": r3, "rho3": c3, "rho5": c5})
    assert all(h["reg"] == O.hll_patlen(bytes.fromhex(h["in"]), 5)[0] for h in hashes)

    keys = ["somekey", "foo{hash_tag}", "{user1000}.following", "tenant:42:hll", "{bf}__config", "a}b{c", "{}"]
    keys += ["tenant:%d:hll" % i for i in range(0, 100000, 997)]
    slots = {k: O.calc_slot(k) for k in keys}

    bloom = []
    for n, p in [(100, 0.03), (550000000, 0.03), (425000000, 0.008)]:
        m = O.bloom_optimal_bits(n, p)
        k = O.bloom_optimal_k(n, m)
        idx = {e.decode(): O.bloom_indexes(e, k, m) for e in [b'"123"', b'"hflgs;jl;ao1-32471320o31803-24"'] +
               jlongs(0x5EED0003, 5)}
        bloom.append({"n": n, "p": p, "size": m, "k": k, "indexes": idx})

    # HLL: 5000 Jackson Longs into 3 keys (+ 500 repeats), replies and registers
    els = jlongs(0x5EED0001, 5000)
    els += [els[i] for i in rng.integers(0, 5000, 500)]
    ks = [b"g:%d" % (i % 3) for i in range(len(els))]
    st = O.HLLStore()
    replies = st.pfadd(ks, [[e] for e in els])
    hll = {"elements_seed": "0x5EED0001", "n": 5000, "repeat_idx_seed": 20261015,
           "keys": [k.decode() for k in ks], "elements": [e.decode() for e in els],
           "replies": "".join("1" if r else "0" for r in replies),
           "dense": {k.decode(): base64.b64encode(O.dense_pack(st.regs[k])).decode() for k in sorted(set(ks))},
           "count_v3": {k.decode(): O.count_regs(st.regs[k], 1, 3) for k in sorted(set(ks))},
           "count_v5": {k.decode(): O.count_regs(st.regs[k], 1, 5) for k in sorted(set(ks))},
           "union_v3": O.count_regs(np.maximum.reduce([st.regs[k] for k in sorted(set(ks))]), 2, 3)}

    # Bloom add/contains on a small filter (tryInit(2000, 0.01))
    m = O.bloom_optimal_bits(2000, 0.01)
    k = O.bloom_optimal_k(2000, m)
    bs = O.BitString()
    adds = jlongs(0x5EED0004, 2000)
    add_r = bs.bloom_add(m, k, adds)
    probes = adds[::4] + jlongs(0x5EED0005, 1000)
    con_r = bs.bloom_contains(m, k, probes)
    bl = {"size": m, "k": k, "adds_seed": "0x5EED0004", "probes": "adds[::4] + 1000 of seed 0x5EED0005",
          "add_replies": "".join("1" if r else "0" for r in add_r),
          "contains_replies": "".join("1" if r else "0" for r in con_r),
          "bits": base64.b64encode(bs.bytes()).decode(), "bitcount": bs.bitcount(),
          "count": O.bloom_count(m, k, bs.bitcount())}

    a = rng.integers(0, 256, 300, dtype=np.uint8).tobytes()
    b = rng.integers(0, 256, 77, dtype=np.uint8).tobytes()
    bitop = {"a": a.hex(), "b": b.hex(), **{op: O.bitop(op, [a, b, None]).hex() for op in ["AND", "OR", "XOR"]},
             "NOT": O.bitop("NOT", [a]).hex()}

    out = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/sketch_oracle.c",
           "hashes": hashes, "calc_slot": slots, "bloom_sizing": bloom, "hll": hll, "bloom": bl, "bitop": bitop}
    with open(os.path.join(HERE, "golden_v1.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
