"""Mean FETCH_SIZE (x2, gfx950) and WRITE_SIZE per dispatch from tools/pmc_rw.sh output."""
import collections
import csv
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_rw"
agg = collections.defaultdict(lambda: [0.0, 0, 0.0, 0])
for sub, col in (("f", 0), ("w", 2)):
    for r in csv.DictReader(open(f"{base}/{sub}/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0][-34:]
        agg[k][col] += float(r["Counter_Value"]) * 1024 * (2 if sub == "f" else 1)   # counters in KiB
        agg[k][col + 1] += 1
for k, (f, nf, w, nw) in sorted(agg.items()):
    print(f"{k:36s} fetch {f / max(nf, 1) / 1e6:9.1f} MB  write {w / max(nw, 1) / 1e6:9.1f} MB  ({nf} dispatches)")
