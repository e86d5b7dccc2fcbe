#!/bin/bash
# One rocprofv3 PMC pass per counter group over a short bench run (dev tool).
# usage (GPU box, repo root): KRE="regex" BENCH_ARGS="..." bash tools/pmc_pass.sh TAG "C1 C2 ..." ["C1 C2 ..." ...]
set -o pipefail
T=$1; shift
R=$(pwd)
O=$R/gpurun_out/$T
KRE=${KRE:-"pfp|bloom"}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
    -d $O/pmc$i -o run -- python3 $R/bench.py $ARGS > $O/pmc$i.json 2> $O/pmc$i.err \
    || { echo "pass $i failed"; tail -5 $O/pmc$i.err; exit 1; }
done
python3 $R/tools/pmc_reduce.py $O && echo done
