#!/bin/bash
# Dev: C1 (bench_configs.py --configs c1) for several engine builds, alternating twice.
# Usage on the box (repo root): bash tools/c1_ab.sh TAG "base v1 ..."
set -o pipefail
T=$1; VARS=$2
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for v in $VARS; do
    if [ "$v" = base ]; then L=$R/redisson_amd/libredisson_sketch.so; else L=$R/redisson_amd/var_$v.so; fi
    SK_LIB_PATH=$L timeout -k 10 300 python3 -u bench_configs.py --configs c1 > $O/$v.$rep.jsonl 2> $O/$v.$rep.err \
      || { echo "$v failed"; tail $O/$v.$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('%-6s' % sys.argv[2], 'gc %.2f G/s' % (d['group_commit_inserts_per_s']/1e9), {k: round(v, 4) for k, v in d['group_commit_kernel_ms'].items()})" $O/$v.$rep.jsonl $v
  done
done
