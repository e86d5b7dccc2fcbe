"""Dev: phase durations of the contains hash blocks (k_bloom_rc_hash<false>) from s_memtime stamps in a
-DSK_RC_STAMP=1 build (tools/build_variant.sh stamp "-DSK_RC_STAMP=1"; run with SK_LIB_PATH=redisson_amd/var_stamp.so).
Phases per block (thread 0): 0 entry -> 1 window 0 staged -> 2 rounds hashed -> 3 scan + segment table ->
4 records placed in LDS -> 5 chunk stores issued.  Prints means over the blocks of one 32 M piece, in cycles."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.getcwd())
from redisson_amd import SketchEngine  # noqa: E402
from redisson_amd import _native as N  # noqa: E402

lib = N.load()
lib.sk_rc_stamp_read.restype = ctypes.c_int
lib.sk_rc_stamp_read.argtypes = [ctypes.c_void_p]
M = 1 << 20
eng = SketchEngine(device=0, max_batch=32 * M)
assert eng.bloom_try_init("c3", 425_000_000, 0.008)
off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0003, 4 * M)
d_out = eng.alloc(32 * M)
eng.bloom_add_dev("c3", 4 * M, off, byt, tot, d_out)
off.free()
byt.free()
off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0004, 32 * M)
for _ in range(3):
    eng.bloom_contains_dev("c3", 32 * M, off, byt, tot, d_out)
buf = (ctypes.c_ulonglong * (8192 * 8))()
assert lib.sk_rc_stamp_read(ctypes.addressof(buf)) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8)[:, :6].astype(np.int64)
d = np.diff(t, axis=1)
names = ["window 0", "rounds", "scan + S", "placement", "chunk stores"]
print("blocks", len(t), "span %.0f cycles" % (t[:, 5].max() - t[:, 0].min()))
for k, nm in enumerate(names):
    print("%-14s mean %8.0f  p50 %8.0f  p90 %8.0f cycles" % (nm, d[:, k].mean(), np.median(d[:, k]),
                                                          np.percentile(d[:, k], 90)))
tot_b = t[:, 5] - t[:, 0]
print("block          mean %8.0f  p50 %8.0f  p90 %8.0f cycles" % (tot_b.mean(), np.median(tot_b), np.percentile(tot_b, 90)))
# gaps between consecutive blocks on one CU are not visible here (no CU id); the span / (blocks / 256) gives the
# per-CU period
print("per-CU period (span x 256 / blocks) %.0f cycles" % ((t[:, 5].max() - t[:, 0].min()) * 256 / len(t)))
eng.close()
