#!/bin/bash
# Dev (GPU box): bench_configs lines for several engine builds (base = the in-tree library, NAME = var_NAME.so)
# usage: bash tools/r06_ab_cfg.sh TAG "base bytew" "c1,c2zipf"
set -o pipefail
T=$1; VARS=$2; CF=${3:-c1,c2zipf}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for v in $VARS; do
    E=""  # "e_NAME=VALUE[+NAME2=VALUE2]": the base build with those environment settings
    if [ "$v" = base ]; then L=$R/redisson_amd/libredisson_sketch.so
    elif [ "${v#e_}" != "$v" ]; then L=$R/redisson_amd/libredisson_sketch.so; E=${v#e_}; E=${E//+/ }
    else L=$R/redisson_amd/var_$v.so; fi
    env $E SK_LIB_PATH=$L timeout -k 10 300 python3 -u bench_configs.py --configs $CF > $O/$v.$rep.jsonl 2> $O/$v.$rep.err || { echo "$v failed"; tail $O/$v.$rep.err; exit 1; }
    python3 - $O/$v.$rep.jsonl $v <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    d=json.loads(ln)
    print('%-8s %-40s %.3f G' % (sys.argv[2], d['metric'][:40], d['value']/1e9), {k: (round(v/1e9,2) if isinstance(v,(int,float)) and v > 1e6 else v) for k, v in d.items() if k.endswith('_per_s')})
PY
  done
done
