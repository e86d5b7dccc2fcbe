"""Per-launch PFADD partition-kernel times in sync vs async mode, with and
without Bloom contains beside it (dev experiment; GPU box, repo root)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redisson_amd import SketchEngine  # noqa: E402

B, T, STEPS = 1 << 20, 100000, 12
eng = SketchEngine(device=0, hll_capacity=T + 16, max_batch=1 << 23, max_bit_offset=1 << 34)
ids = eng.hll_resolve(["tenant:%d:hll" % t for t in range(T)])
rng = np.random.default_rng(7)
off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0002, 4 * STEPS * B)
d_ids = eng.to_device(ids[rng.integers(0, T, 4 * STEPS * B)].astype(np.uint32))
d_out = eng.alloc(B)
PH = ["pfp_hash", "pfp_apply", "pfp_reply"]


def run(label, mode_async, first, sync_each):
    eng.set_async(mode_async)
    per = []
    for s in range(first, first + STEPS):
        eng.prof_reset()
        eng.prof_enable(True)
        eng.pfadd_dev(B, d_ids.ptr + s * B * 4, off.ptr + s * B * 8, byt, tot, d_out)
        if sync_each:
            eng.sync()
        eng.prof_enable(False)
        per.append([round(eng.prof_read(p)[1] * 1e3, 1) for p in PH])
    eng.sync()
    eng.set_async(False)
    a = np.array(per)
    print(label, "per-step us [hash apply reply]:", per[:6], "median", np.median(a, axis=0).tolist(), flush=True)


run("sync ", False, 0, True)
run("async+sync", True, STEPS, True)
run("sync again", False, 2 * STEPS, True)
run("async", True, 3 * STEPS, False)
