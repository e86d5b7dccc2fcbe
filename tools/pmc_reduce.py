"""Reduce rocprofv3 counter_collection CSVs to per-kernel mean counter values (dev tool).
usage: python tools/pmc_reduce.py DIR  -> DIR/pmc_means.json, raw CSVs removed"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        os.remove(f)
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    json.dump(out, open(os.path.join(d, "pmc_means.json"), "w"), indent=1)
    for k, cs in sorted(out.items()):
        if k.startswith("sk::"):
            print(k, {c: round(v) for c, v in cs.items()})


if __name__ == "__main__":
    main(sys.argv[1])
