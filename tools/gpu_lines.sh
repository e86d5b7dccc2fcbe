#!/bin/bash
# line-schedule parity + bench at group 16 / 1 + kernel trace
set -o pipefail
O=gpurun_out/${1:-lines}
mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for g in ${GROUPS_:-16 1}; do
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --group $g $BARGS > $O/bench_g$g.json 2> $O/bench_g$g.err || { tail $O/bench_g$g.err; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline $BARGS > $R/$O/prof_bench.json 2> $R/$O/prof.err || { tail $R/$O/prof.err; exit 1; }
cd $R
python - $O <<'PY'
import json, sys, glob, csv
O=sys.argv[1]
for f in sorted(glob.glob(O+"/bench_g*.json")):
    d=json.load(open(f))
    print(f, "value %.3e"%d["value"], "ms/step %.3f"%d["ms_per_step"], "hll/s %.3e"%d["hll_inserts_per_s"], "roof", d["roofline"]["kernel"], "%.3f"%d["roofline"]["frac"])
    print({k:(round(v["ms_isolated"],4), round(v["ms_overlapped"] or 0,4)) for k,v in d["kernels"].items()})
st=glob.glob(O+"/prof/**/*kernel_stats.csv", recursive=True)
for row in csv.DictReader(open(st[0])):
    print(row["Name"][:60], row["Calls"], "%.1f us"%(float(row["AverageNs"])/1e3), "%.1f%%"%float(row["Percentage"]))
PY
rm -f $O/prof/*/*kernel_trace.csv
