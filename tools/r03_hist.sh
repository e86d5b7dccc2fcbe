#!/bin/bash
# Round-3 counter passes on the PFCOUNT histogram kernel (dev tool): SQ wave-cycle split, LDS busy / conflicts,
# LDS atomic instructions and VALU, plus a kernel-trace for the durations.  Usage (box, repo root): bash tools/r03_hist.sh TAG
set -o pipefail
T=${1:-r03hist}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
RX="hll_hist|hll_sum"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$RX" --output-format csv -d $O/trace -o run -- \
  python3 $R/bench_configs.py --configs c2zipf > $O/trace.json 2> $O/trace.err || { echo trace failed; tail -5 $O/trace.err; exit 1; }
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 300 rocprofv3 --pmc $SQ1 --kernel-include-regex "$RX" --output-format csv -d $O/sq1 -o run -- \
  python3 $R/bench_configs.py --configs c2zipf > $O/sq1.json 2> $O/sq1.err || { echo sq1 failed; tail -5 $O/sq1.err; exit 1; }
L1="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_LDS_ATOMIC GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $L1 --kernel-include-regex "$RX" --output-format csv -d $O/lds1 -o run -- \
  python3 $R/bench_configs.py --configs c2zipf > $O/lds1.json 2> $O/lds1.err || { echo lds1 failed; tail -5 $O/lds1.err; exit 1; }
cd $R && python3 tools/pmc_reduce.py $O/sq1 > /dev/null && python3 tools/pmc_reduce.py $O/lds1 > /dev/null \
  && python3 profiles/sq_summary.py $O/sq1,$O/lds1 $T $(ls $O/trace/*kernel_stats.csv | head -1) && rm -f $O/*/run_counter_collection.csv $O/trace/run_kernel_trace.csv
echo done
