#!/bin/bash
# Dev: FETCH_SIZE / WRITE_SIZE (KiB per dispatch: x 2048 / x 1024 bytes, profiles/summarize.py) of the PFADD line-schedule kernels for several engine builds (var_NAME.so, base =
# the default build).  Usage on the box (repo root): bash tools/pmc_ab.sh TAG "base v1 v2" [kernel regex]
set -o pipefail
T=$1; VARS=$2; RX=${3:-k_pfl}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
SHORT="--steps 2 --warmup 1 --no-cpu-baseline"
for v in $VARS; do
  if [ "$v" = base ]; then L=$R/redisson_amd/libredisson_sketch.so; else L=$R/redisson_amd/var_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && SK_LIB_PATH=$L timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "$RX" --output-format csv \
      -d $O/$v.$c -o run -- python3 $R/bench.py $SHORT > $O/$v.$c.json 2> $O/$v.$c.err) || { echo "$v $c failed"; exit 1; }
    python3 tools/pmc_reduce.py $O/$v.$c > /dev/null || exit 1
  done
  python3 - $O $v <<'PY'
import json, sys
o, v = sys.argv[1], sys.argv[2]
f = json.load(open(f"{o}/{v}.FETCH_SIZE/pmc_means.json")); w = json.load(open(f"{o}/{v}.WRITE_SIZE/pmc_means.json"))
for k in sorted(f):
    if k.startswith("sk::"):
        print("%-8s %-16s fetch %.3f write %.3f GB" % (v, k[4:], 2048 * f[k]["FETCH_SIZE"] / 1e9, 1024 * w[k]["WRITE_SIZE"] / 1e9))
PY
done
