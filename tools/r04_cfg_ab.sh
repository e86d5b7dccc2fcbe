#!/bin/bash
# Round-4 A/B of engine builds on bench_configs.py configs (dev tool, GPU box, repo root).
# usage: bash tools/r04_cfg_ab.sh TAG "base prev" "c4,c5"
set -o pipefail
T=$1; VARS=$2; CFG=${3:-c4,c5}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for v in $VARS; do
    if [ "$v" = base ]; then L=$R/redisson_amd/libredisson_sketch.so; else L=$R/redisson_amd/var_$v.so; fi
    SK_LIB_PATH=$L timeout -k 10 300 python3 -u bench_configs.py --configs $CFG > $O/$v.$rep.jsonl 2> $O/$v.$rep.err \
      || { echo "$v failed"; tail -5 $O/$v.$rep.err; exit 1; }
    python3 - $O/$v.$rep.jsonl $v <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if not l.startswith('{'): continue
    d=json.loads(l); r=d.get('roofline') or {}
    print('%-6s %-6s value %.4g %s  roofline %s %.0f GB/s frac %.3f %s' % (sys.argv[2], d['config']['workload'], d['value'], d['unit'],
          r.get('kernel'), r.get('achieved') or 0, r.get('frac') or 0, d.get('device_GBps', '')))
PY
  done
done
