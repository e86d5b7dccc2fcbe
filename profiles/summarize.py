"""Summarize a rocprofv3 profile directory (profiles/run_profile.sh) into the
committed per-round files: kernel stats CSV copy + per-kernel PMC means.

PMC units: FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md
(HBM section): on gfx950 FETCH_SIZE = TCC_EA0_RDREQ x 64 B while the requests
are 128 B, i.e. it reads 1/2 of the bytes fetched -- the summary doubles it
(`fetch_bytes`, raw value kept as `fetch_bytes_raw`).  WRITE_SIZE is taken as
reported.  `traffic_bytes_per_launch` = fetch_bytes + write_bytes.
Usage: python profiles/summarize.py gpurun_out/prof_r01 r01 [--into DIR]
(--into: write the summary files into DIR instead of profiles/, for copying later)
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def main(src, tag, into=None):
    out = into or os.path.dirname(os.path.abspath(__file__))
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    # per-kernel dispatch durations from the trace: mean, the mean without each kernel's first dispatch (the bench's
    # warm-up call: cold TLBs / L2 after the setup), median -- the bench's own per-kernel timing skips its warm-up
    tr = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        durs = defaultdict(list)
        for r in csv.DictReader(open(tr)):
            nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
            durs[nm].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        steady = {}
        for nm, v in durs.items():
            d = [x[1] for x in sorted(v)]
            rest = d[1:] or d
            steady[nm] = {"dispatches": len(d), "mean_ns": sum(d) / len(d), "mean_ns_after_first": sum(rest) / len(rest),
                          "median_ns": sorted(d)[len(d) // 2], "first_ns": d[0]}
        json.dump({"source": src, "kernels": steady}, open(os.path.join(out, f"{tag}_kernel_steady.json"), "w"), indent=1)
    res = defaultdict(dict)
    for sub, ctr in [("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")]:
        acc = defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, sub, "run_counter_collection.csv"))):
            if r["Counter_Name"] != ctr:
                continue
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(
                (float(r["Counter_Value"]) * 1024, int(r["Grid_Size"])))
        for k, v in acc.items():
            res[k][ctr] = sum(x[0] for x in v) / len(v)
            res[k]["dispatches"] = len(v)
            res[k]["grid"] = max(x[1] for x in v)
    for k, d in res.items():
        d["fetch_bytes_raw"] = d.get("FETCH_SIZE", 0.0)
        d["fetch_bytes"] = 2 * d.get("FETCH_SIZE", 0.0)
        d["write_bytes"] = d.get("WRITE_SIZE", 0.0)
        d["traffic_bytes_per_launch"] = d["fetch_bytes"] + d["write_bytes"]
    keep = {k: v for k, v in res.items() if k.startswith("sk::")}
    json.dump({"source": src, "units": "bytes per dispatch (mean); fetch_bytes = 2 x FETCH_SIZE (gfx950)",
               "kernels": keep}, open(os.path.join(out, f"{tag}_pmc_summary.json"), "w"), indent=1)
    for k, v in sorted(keep.items()):
        print("%-28s n=%5d fetch=%12.0f write=%12.0f" % (k, v["dispatches"], v["fetch_bytes"], v["write_bytes"]))


if __name__ == "__main__":
    into = sys.argv[sys.argv.index("--into") + 1] if "--into" in sys.argv else None
    main(sys.argv[1], sys.argv[2], into)
