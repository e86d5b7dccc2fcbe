# C4 union: union parity tests, then per-kernel times of the union tree (rocprof kernel trace + stats)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_distributed.py tests/test_gpu_persist.py -k "union or merge or count or pfmerge or save or dump or restore" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench_configs.py --configs c4 > $O/c4.jsonl 2> $O/c4.err || { echo trace failed; tail $O/c4.err; exit 1; }
cd $R && python3 - $O <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/trace/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'union' in r['Name'] or 'hll' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
PY
