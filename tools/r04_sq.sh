#!/bin/bash
# Round-4 SQ counter pass (dev tool): VALU / LDS / VMEM instruction counts and wave-cycle split of the bench's kernels,
# with a kernel-trace pass for their durations.  Usage (repo root on the box): bash tools/r04_sq.sh TAG
set -o pipefail
T=${1:-r04sq}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
SHORT="--steps 3 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py $SHORT > $O/trace.json 2> $O/trace.err || { echo trace failed; exit 1; }
rm -f $O/trace/run_kernel_trace.csv
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 200 rocprofv3 --pmc $SQ1 --kernel-include-regex "sk::" --output-format csv -d $O/sq1 -o run -- \
  python3 $R/bench.py $SHORT > $O/sq1.json 2> $O/sq1.err || { echo sq1 failed; tail -5 $O/sq1.err; exit 1; }
SQ2="SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $SQ2 --kernel-include-regex "sk::" --output-format csv -d $O/sq2 -o run -- \
  python3 $R/bench.py $SHORT > $O/sq2.json 2> $O/sq2.err || { echo sq2 failed; tail -5 $O/sq2.err; exit 1; }
cd $R && python3 tools/pmc_reduce.py $O/sq1 > /dev/null && python3 tools/pmc_reduce.py $O/sq2 > /dev/null
rm -f $O/sq*/run_counter_collection.csv
echo done
