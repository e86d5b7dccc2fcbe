#!/bin/bash
# Round-3 SQ counter passes (dev tool): LDS / VALU / wait / VMEM instruction counters on the bench's kernels and on
# the PFCOUNT / union kernels, plus a reply-store ablation bench.  Usage (repo root on the box): bash tools/r03_sq.sh TAG
set -o pipefail
T=${1:-r03sq}
R=$(pwd)
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
SHORT="--steps 3 --warmup 1 --no-cpu-baseline"
SK_PFL_PROBE=64 timeout -k 10 300 python3 -u bench.py $SHORT > $O/bench_norep.json 2> $O/bench_norep.err || { echo norep failed; tail -5 $O/bench_norep.err; exit 1; }
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 200 rocprofv3 --pmc $SQ1 --kernel-include-regex "sk::" --output-format csv -d $O/sq1 -o run -- \
  python3 $R/bench.py $SHORT > $O/sq1.json 2> $O/sq1.err || { echo sq1 failed; tail -5 $O/sq1.err; exit 1; }
SQ2="SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVES"
timeout -s KILL 200 rocprofv3 --pmc $SQ2 --kernel-include-regex "sk::" --output-format csv -d $O/sq2 -o run -- \
  python3 $R/bench.py $SHORT > $O/sq2.json 2> $O/sq2.err || { echo sq2 failed; tail -5 $O/sq2.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $SQ1 --kernel-include-regex "hll_hist|hll_sum|hll_union" --output-format csv -d $O/sq3 -o run -- \
  python3 $R/bench_configs.py --configs c2zipf,c4 > $O/sq3.json 2> $O/sq3.err || { echo sq3 failed; tail -5 $O/sq3.err; exit 1; }
cd $R && python3 tools/pmc_reduce.py $O/sq1 > /dev/null && python3 tools/pmc_reduce.py $O/sq2 > /dev/null && python3 tools/pmc_reduce.py $O/sq3 > /dev/null
echo done
