#!/bin/bash
# A/B of env settings on the default bench, alternating runs on one box (dev tool)
# usage: bash tools/ab_env.sh TAG ROUNDS "ENV1" "ENV2" ...   (ENV "-" = none)
set -o pipefail
O=gpurun_out/$1; shift; N=$1; shift; mkdir -p $O
for r in $(seq 1 $N); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    if [ "$e" = "-" ]; then e=""; fi
    env $e timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --bloom-fill ${FILL:-1000000000} $BARGS > $O/r${r}_$i.json 2> $O/r${r}_$i.err || { tail $O/r${r}_$i.err; exit 1; }
  done
done
python - $O $N $# <<'PY'
import json,sys
O,N,M=sys.argv[1],int(sys.argv[2]),int(sys.argv[3])
for i in range(1,M+1):
    rows=[json.load(open(f"{O}/r{r}_{i}.json")) for r in range(1,N+1)]
    print(i, "value", ["%.3e"%d["value"] for d in rows], {k:[round(d["kernels"][k]["ms_isolated"],4) for d in rows] for k in rows[0]["kernels"]})
PY
