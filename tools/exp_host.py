"""Host-side enqueue times of the bench step in async mode (dev experiment; GPU box, repo root):
does any call block the host until earlier device work is done?"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redisson_amd import SketchEngine  # noqa: E402

B, T, STEPS = 1 << 20, 100000, 20
eng = SketchEngine(device=0, hll_capacity=T + 16, max_batch=1 << 23, max_bit_offset=1 << 34)
ids = eng.hll_resolve(["tenant:%d:hll" % t for t in range(T)])
rng = np.random.default_rng(7)
off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0002, STEPS * B)
d_ids = eng.to_device(ids[rng.integers(0, T, STEPS * B)].astype(np.uint32))
d_out = eng.alloc(B)
d_c = eng.alloc(B)
eng.bloom_try_init("bf", 425000000, 0.008)
coff, cbyt, ctot = eng.gen_jackson_longs_dev(0x5EED0003, STEPS * B)
eng.sync()
for prof in (False, True):
    eng.set_async(True)
    if prof:
        eng.prof_only("bloom_contains")
        eng.prof_reset()
        eng.prof_enable(True)
    t = []
    t0 = time.perf_counter()
    for s in range(STEPS):
        a = time.perf_counter()
        eng.pfadd_dev(B, d_ids.ptr + s * B * 4, off.ptr + s * B * 8, byt, tot, d_out)
        b = time.perf_counter()
        eng.bloom_contains_dev("bf", B, coff.ptr + s * B * 8, cbyt, ctot, d_c)
        c = time.perf_counter()
        t.append(((b - a) * 1e6, (c - b) * 1e6))
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    eng.prof_enable(False)
    eng.prof_only(None)
    eng.set_async(False)
    print("prof=%s enqueue %.1f us/step, total %.1f us/step; per call (pfadd, contains) us:" % (
        prof, (t1 - t0) / STEPS * 1e6, (t2 - t0) / STEPS * 1e6), [(round(x), round(y)) for x, y in t[:8]], flush=True)
