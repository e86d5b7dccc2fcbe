#!/usr/bin/env python3
"""C5 RBatch runs through the C ABI the Java executors call (sk_setbit / sk_getbit by key name, host buffers): one
64 M-op SETBIT_VOID call (no reply array), one SETBIT call with replies, one GETBIT call, on a 2^34-bit RBitSet.  Run
under `rocprofv3 --kernel-trace --stats` to list the kernels these calls launch (dev tool, GPU box)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redisson_amd import SketchEngine  # noqa: E402

bits, m = 1 << 34, 1 << 26
eng = SketchEngine(device=0, max_bit_offset=bits)
key = b"bs5:0"
eng.setbit([key], [bits - 1], [1])
rng = np.random.default_rng(5)
offs = rng.integers(0, bits, m, dtype=np.uint64)
koff = np.arange(m + 1, dtype=np.uint64) * np.uint64(len(key))
kbuf = np.frombuffer(key * m + b"\0" * 16, dtype=np.uint8)
ones = np.ones(m, dtype=np.uint8)
rep = np.zeros(m, dtype=np.uint8)
for name, fn in (("setbit_void", lambda: eng.setbit_packed(koff, kbuf, offs, ones)),
                 ("setbit_replies", lambda: eng.setbit_packed(koff, kbuf, offs, ones, rep)),
                 ("getbit", lambda: eng.getbit_packed(koff, kbuf, offs, rep))):
    eng.sync()
    t0 = time.perf_counter()
    fn()
    eng.sync()
    dt = time.perf_counter() - t0
    print("%s: %d ops in %.1f ms host-timed = %.2f G ops/s" % (name, m, dt * 1e3, m / dt / 1e9), flush=True)
assert rep.all(), "every bit was set"
eng.close()
