#!/bin/bash
# Dev (GPU box, repo root): timing + memory-side request counts of tools/micro/packed_lines
set -o pipefail
O=$(pwd)/gpurun_out/${1:-plines}; mkdir -p $O; export TMPDIR=/tmp; B=$(pwd)/tools/micro/packed_lines
timeout -k 10 120 $B 100000 10 | tee $O/time.txt || exit 1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $O/rd -o run -- $B 100000 1 > /dev/null 2>&1 || { echo rd failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $O/wr -o run -- $B 100000 1 > /dev/null 2>&1 || { echo wr failed; exit 1; }
python3 - $O <<'PY'
import csv, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("rd", "wr"):
    for r in csv.DictReader(open(f"{O}/{sub}/run_counter_collection.csv")):
        acc[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = collections.defaultdict(list)
for (k, d), c in acc.items():
    rows[k].append({n: sum(v) for n, v in c.items()})
for k, lst in rows.items():
    print(k, len(lst))
    for x in lst:
        rd = x.get("TCC_EA0_RDREQ_32B_sum", 0) * 32 + x.get("TCC_EA0_RDREQ_64B_sum", 0) * 64 + x.get("TCC_EA0_RDREQ_128B_sum", 0) * 128
        print("   ", {n: int(v) for n, v in x.items()}, "read bytes %.3f GB" % (rd / 1e9))
PY
