#!/bin/bash
# Dev: A/B of engine builds (redisson_amd/var_NAME.so, tools/build_variant.sh) on the bench, alternating twice.
# usage on the box: bash tools/gpu_ab.sh TAG "base a512 e_SK_PFL_PROBE=64 ..." [bench args]
set -o pipefail
T=$1; VARS=$2; BARGS=${3:-"--steps 5 --warmup 1 --no-cpu-baseline"}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for v in $VARS; do
    E=""  # a variant "e_NAME=VALUE" is the base build with that environment setting
    if [ "$v" = base ]; then L=$R/redisson_amd/libredisson_sketch.so
    elif [ "${v#e_}" != "$v" ]; then L=$R/redisson_amd/libredisson_sketch.so; E=${v#e_}
    else L=$R/redisson_amd/var_$v.so; fi
    env $E SK_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py $BARGS > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "$v failed"; tail $O/$v.$rep.err; exit 1; }
    python3 - $O/$v.$rep.json $v <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
k=d['kernels']
print('%-8s value %.3f G add %.2f G/s ' % (sys.argv[2], d['value']/1e9, (d.get('bloom_add_per_s') or 0)/1e9) + '  '.join('%s %.3f' % (n, v['ms_isolated']) for n, v in k.items()) + '  chain %.3f' % d['chains']['pfadd']['ms_isolated'])
PY
  done
done
