#!/bin/bash
# line schedule: parity + bench at several per-GPU tenant counts + Zipf group commit (dev tool)
set -o pipefail
O=gpurun_out/${1:-sh}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in ${TENANTS:-12500 50000 100000}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --tenants $t > $O/t$t.json 2> $O/t$t.err || { tail $O/t$t.err; exit 1; }
done
timeout -k 10 300 python bench_configs.py --configs ${CFGS:-c2zipf} > $O/cfg.jsonl 2> $O/cfg.err || { tail $O/cfg.err; exit 1; }
python - $O <<'PY'
import json, sys, glob
O = sys.argv[1]
for f in sorted(glob.glob(O + "/t*.json")):
    d = json.load(open(f))
    print(f, "value %.3e ms/step %.3f hll/s %.3e frac %.3f" % (d["value"], d["ms_per_step"], d["hll_inserts_per_s"], d["roofline"]["frac"]), {k: round(v["ms_isolated"], 4) for k, v in d["kernels"].items()})
for l in open(O + "/cfg.jsonl"):
    d = json.loads(l)
    print(d["metric"][:40], "%.3e" % d["value"], "group %.3e" % d.get("group_commit_inserts_per_s", 0))
PY
