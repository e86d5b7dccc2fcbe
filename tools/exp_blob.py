"""A/B timing of the long-element hash (k_ms_planes + k_ms_rounds) on the C1 Q1 element: device ms per run, 5 runs.
Usage: SK_LIB_PATH=<lib> python3 tools/exp_blob.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from redisson_amd import JsonJacksonCodec, JLong, SketchEngine  # noqa: E402

eng = SketchEngine(device=0)
vals = np.random.default_rng(1).integers(-(1 << 63), (1 << 63) - 1, 1 << 20, dtype=np.int64)
blob = JsonJacksonCodec().encode(["hll:c1q"] + [JLong(int(v)) for v in vals])
eng.pfadd([b"hll:c1q"], [[blob]])
ms = []
for _ in range(5):
    eng.prof_reset(); eng.prof_enable(True)
    eng.pfadd([b"hll:c1q"], [[blob]])
    eng.prof_enable(False)
    n, t = eng.prof_read("pfadd_long")
    ms.append(round(t / max(n, 1), 2))
print(json.dumps({"lib": os.environ.get("SK_LIB_PATH", "in-tree"), "bytes": len(blob), "ms": ms}))
eng.close()
