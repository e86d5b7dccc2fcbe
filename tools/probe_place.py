"""Dev: is the Bloom contains probe time a property of the filter's placement or of the process?

Fills NF copies of bench.py's C3 filter (each its own allocation, separated by padding buffers of different sizes)
and times the contains chain on each, several rounds, in one process.  Prints per filter: hash / probe ms.
usage (GPU box): python3 tools/probe_place.py [NF] [fill]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from redisson_amd import SketchEngine  # noqa: E402

# clocks or placement?  an MFMA-bound torch GEMM (clock-proportional) next to the contains numbers
import time  # noqa: E402

import torch  # noqa: E402

a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    a @ b
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    a @ b
torch.cuda.synchronize()
print("gemm %.1f TFLOP/s" % (20 * 2 * 8192 ** 3 / (time.perf_counter() - t0) / 1e12), flush=True)
del a, b

NF = int(sys.argv[1]) if len(sys.argv) > 1 else 4
FILL = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
CB = 64 << 20
eng = SketchEngine(device=0)
seed_b = 0x5EED0003
pads = []
names = []
chunk = 1 << 25
out = eng.alloc(chunk)
for f in range(NF):
    pads.append(eng.alloc((f * 37 + 3) << 20))   # shift the next allocation
    nm = "bf%d" % f
    eng.bloom_try_init(nm, 425_000_000, 0.008)
    size, k, _, _ = eng.bloom_config(nm)
    for s in range(0, FILL, chunk):
        n = min(chunk, FILL - s)
        a_off, a_bytes, a_tot = eng.gen_jackson_longs_dev(seed_b, n, first=s)
        eng.bloom_add_dev(nm, n, a_off, a_bytes, a_tot, out)
        eng.sync()
        a_off.free()
        a_bytes.free()
    names.append(nm)
    print("filled", nm, flush=True)
rng = np.random.default_rng(7)
member = rng.integers(0, FILL, CB, dtype=np.uint64)
fresh = rng.integers(1 << 39, 1 << 40, CB, dtype=np.uint64)
idx = np.where(rng.random(CB) < 0.5, member, fresh)
d_idx = eng.to_device(idx)
off, byt, tot = eng.gen_jackson_longs_dev(seed_b, CB, d_idx=d_idx)
d_out = eng.alloc(CB)
size, k, _, _ = eng.bloom_config(names[0])
for rnd in range(3):
    for nm in names:
        eng.prof_reset()
        eng.prof_enable(True)
        for _ in range(3):
            eng.bloom_contains_dev(nm, CB, off, byt, tot, d_out)
        eng.sync()
        eng.prof_enable(False)
        h = eng.prof_read("bloom_rc_hash")
        p = eng.prof_read("bloom_rc_probe")
        print("round %d %s hash %.3f probe %.3f ms per 64M" % (rnd, nm, h[1] / 3, p[1] / 3), flush=True)
eng.sync()

pad = eng.alloc(3 << 30)
off2, byt2, tot2 = eng.gen_jackson_longs_dev(seed_b, CB, d_idx=d_idx)
for inp, tag in (((off, byt, tot), "old inputs"), ((off2, byt2, tot2), "new inputs")):
    eng.prof_reset()
    eng.prof_enable(True)
    for _ in range(3):
        eng.bloom_contains_dev(names[0], CB, *inp, d_out)
    eng.sync()
    eng.prof_enable(False)
    print("%s hash %.3f probe %.3f" % (tag, eng.prof_read("bloom_rc_hash")[1] / 3, eng.prof_read("bloom_rc_probe")[1] / 3),
          flush=True)
eng.close()
