#!/bin/bash
# A/B of engine env knobs on the headline bench (GPU box, repo root):
#   bash tools/ab_env.sh TAG "VAR=a" "VAR=b" ...   -> gpurun_out/TAG/<i>.json, one summary line each
set -o pipefail
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 240 python -u bench.py --steps 50 --no-cpu-baseline > $O/$i.json 2> $O/$i.err || { echo "run $i ($kv) failed"; tail -5 $O/$i.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/$i.json').read().strip().splitlines()[-1])
print('$kv', round(d['value']/1e9,3), 'G/s step_us', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['kernel_ms_per_launch'].items()}, 'iso', {k: round(v*1e3,1) for k,v in d['roofline_isolated']['kernel_ms_per_launch'].items()})"
done
