#!/bin/bash
# Dev: histogram kernel parity tests, then the C2 PFCOUNT histogram line for the default build and any var_NAME builds in VARS.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/hh; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "pfadd_dev_path or histogram or redis5" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ${VARS:-base}; do
  if [ "$v" = base ]; then L=$R/redisson_amd/libredisson_sketch.so; else L=$R/redisson_amd/var_$v.so; fi
  SK_LIB_PATH=$L timeout -k 10 300 python3 -u bench_configs.py --configs c2zipf > $O/$v.jsonl 2> $O/$v.err || { echo "$v failed"; tail $O/$v.err; exit 1; }
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if 'hll_hist' in d: print(sys.argv[2], 'hist', round(d['hll_hist']['avg_launch_ms'],3), 'ms frac', round(d['hll_hist']['frac'],3), 'sum frac', round(d['roofline']['frac'],3))
" $O/$v.jsonl $v
done
