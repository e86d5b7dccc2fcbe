#!/bin/bash
# Dev: GPU tests matching an expression, then a bench line (optional profile).  Usage on the box:
#   bash tools/gpu_run.sh TAG "pytest -k expr or test files" [bench args|-] [prof]
set -o pipefail
T=$1; TESTS=$2; BARGS=${3:-}; PROF=${4:-}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 \
    || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
if [ "$BARGS" != "-" ]; then
  timeout -k 10 300 python3 -u bench.py $BARGS > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
  python3 - $O/bench.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print('value %.3f G ms/step %.3f' % (d['value']/1e9, d['ms_per_step']))
for k,v in d['kernels'].items(): print('  %-16s %.3f  ovl %s' % (k, v['ms_isolated'], v['ms_overlapped'] and round(v['ms_overlapped'],3)))
for k,v in d['chains'].items(): print('  chain %-14s %.3f frac %.3f' % (k, v['ms_isolated'], v['s8d_frac_isolated']))
PY
fi
if [ -n "$PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { echo trace failed; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "sk::" --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch.json 2> $O/fetch.err || { echo fetch failed; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "sk::" --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/write.json 2> $O/write.err || { echo write failed; exit 1; }
  cd $R && python3 profiles/summarize.py $O $T --into $O/summary && rm -f $O/trace/run_kernel_trace.csv $O/pmc_*/run_counter_collection.csv
fi
echo done
