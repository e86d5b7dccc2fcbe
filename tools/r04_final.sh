#!/bin/bash
# Round-4 record run at a final build (dev tool, GPU box, repo root): the whole -m gpu suite, smoke, the default
# bench line, a kernel-trace + stats pass and FETCH/WRITE PMC passes of a short bench, and every secondary config.
# Usage: bash tools/r04_final.sh TAG
set -o pipefail
T=${1:-r04f}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 \
  || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']/1e9,3), 'G', round(d['ms_per_step'],3), 'ms', 'frac', round(d['roofline']['frac'],3))" $O/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { echo trace failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "sk::" --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch.json 2> $O/fetch.err || { echo fetch failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "sk::" --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/write.json 2> $O/write.err || { echo write failed; exit 1; }
cd $R && python3 profiles/summarize.py $O $T --into $O/summary > /dev/null && rm -f $O/trace/run_kernel_trace.csv $O/pmc_*/run_counter_collection.csv
timeout -k 10 900 python3 -u bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { echo configs failed; tail -5 $O/configs.err; exit 1; }
if [ -n "$EXTRA" ]; then
  timeout -k 10 300 python3 -u bench.py --overlap --no-cpu-baseline > $O/bench_overlap.json 2> $O/bench_overlap.err || { echo overlap failed; exit 1; }
  timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --no-cpu-baseline > $O/bench_n2_shared_gpu.json 2> $O/bench_n2.err || { echo n2 failed; tail -5 $O/bench_n2.err; exit 1; }
fi
echo all done
