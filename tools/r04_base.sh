#!/bin/bash
# Round-4 baseline on the GPU box (dev tool): the default bench line and a kernel-trace + stats pass of a short
# bench.  Usage (repo root on the box): bash tools/r04_base.sh TAG
set -o pipefail
T=${1:-r04a}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']/1e9,3), 'G', round(d['ms_per_step'],3), 'ms', 'frac', round(d['roofline']['frac'],3), 'add', round((d.get('bloom_add_per_s') or 0)/1e9,2)); print({n: round(v['ms_isolated'],3) for n,v in d['kernels'].items()})" $O/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { echo trace failed; exit 1; }
rm -f $O/trace/run_kernel_trace.csv
echo all done
