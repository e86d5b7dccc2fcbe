#!/bin/bash
# Round-4 dev: FETCH_SIZE and WRITE_SIZE (separate passes) of kernels matching $2 under environment settings.
# usage (GPU box, repo root): bash tools/r04_pmc_ab.sh TAG "regex" "-" "SK_PFL_PROBE=64" ...   ("-" = defaults)
set -o pipefail
T=$1; RE=$2; shift 2
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1)); [ "$e" = "-" ] && e=""
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$O/v$i/$( [ $c = FETCH_SIZE ] && echo f || echo w )
    env $e timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "$RE" --output-format csv -d $d -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/v$i.$c.json 2> $O/v$i.$c.err \
      || { echo "pass $i $c failed"; tail -3 $O/v$i.$c.err; exit 1; }
  done
  echo "== ${e:-defaults}"; python3 $R/tools/pmc_table.py $O/v$i
  rm -f $O/v$i/*/run_counter_collection.csv.bak
done
