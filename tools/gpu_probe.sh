#!/bin/bash
# Dev: bench under several SK_PFL_PROBE ablation values (results not valid, timing only).
# Usage on the box: bash tools/gpu_probe.sh TAG "0 64 4 68" [bench args]
set -o pipefail
T=$1; PROBES=$2; BARGS=${3:-"--steps 5 --warmup 1 --no-cpu-baseline"}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
for p in $PROBES; do
  SK_PFL_PROBE=$p timeout -k 10 300 python3 -u bench.py $BARGS > $O/p$p.json 2> $O/p$p.err || { echo "probe $p failed"; tail $O/p$p.err; exit 1; }
  python3 - $O/p$p.json $p <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
k=d['kernels']
print('probe %-4s value %.3f G  ' % (sys.argv[2], d['value']/1e9) + '  '.join('%s %.3f' % (n, v['ms_isolated']) for n, v in k.items()))
PY
done
