"""Bloom add phase times on the C3 filter (bloom_ra_hash / bloom_ra_apply, or the sort path with SK_BLOOM_RA_MIN=0)."""
import sys
import time

sys.path.insert(0, ".")
from redisson_amd import SketchEngine  # noqa: E402

eng = SketchEngine(device=0)
eng.bloom_try_init("c3", 425_000_000, 0.008)
size, k, _, _ = eng.bloom_config("c3")
CH = 32 << 20
total = int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 20
d_out = eng.alloc(CH)
bufs = []
for s in range(0, total, CH):
    bufs.append(eng.gen_jackson_longs_dev(0x5EED0003, CH, first=s))
eng.sync()
eng.prof_reset()
eng.prof_enable(True)
t0 = time.perf_counter()
for off, byt, tot in bufs:
    eng.bloom_add_dev("c3", CH, off, byt, tot, d_out)
eng.sync()
t = time.perf_counter() - t0
eng.prof_enable(False)
out = {"adds_per_s": total / t, "total": total, "k": k}
for ph in ("bloom_ra_hash", "bloom_ra_apply", "bloom_probes", "bloom_sort", "bloom_apply"):
    n, ms = eng.prof_read(ph)
    if n:
        out[ph] = (n, ms / n)
print(out)
