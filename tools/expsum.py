"""Print the PFADD/contains breakdown of bench.py JSON lines (experiment summaries)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "no result", e)
        continue
    k, c = d["kernels"], d["chains"]
    print(f.split("/")[-1], "%.2f G/s" % (d["value"] / 1e9), "ms/step %.3f" % d["ms_per_step"],
          " ".join("%s %.1f/%.1f" % (n, v["ms_isolated"] * 1e3, v["ms_overlapped"] * 1e3) for n, v in k.items()),
          "| chains", " ".join("%s %.1f/%.1f" % (n, v["ms_isolated"] * 1e3, v["ms_overlapped"] * 1e3)
                               for n, v in c.items()))
