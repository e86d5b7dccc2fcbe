#!/bin/bash
# Profile recipe (run on the GPU box from the repo root):
#   kernel trace + stats, then one PMC pass per TCC counter group (FETCH_SIZE, WRITE_SIZE),
#   then a clean bench line.  Usage: bash profiles/run_profile.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_${1:-r01}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
KSEL='sk::'
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KSEL" --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/bench_fetch.json 2> $OUT/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KSEL" --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/bench_write.json 2> $OUT/write.err
timeout -k 10 300 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
cd $R && python3 profiles/summarize.py $OUT ${1:-r01} --into $OUT/summary && rm -f $OUT/trace/run_kernel_trace.csv $OUT/pmc_*/run_counter_collection.csv
