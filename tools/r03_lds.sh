#!/bin/bash
# Round-3 LDS / atomic counter passes (dev tool): LDS-array busy cycles, bank conflicts, LDS atomic instructions and
# L2 atomics on the bench's kernels, with GRBM_GUI_ACTIVE for the dispatch cycles.
# Usage (repo root on the box): bash tools/r03_lds.sh TAG
set -o pipefail
T=${1:-r03lds}
R=$(pwd)
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
SHORT="--steps 3 --warmup 1 --no-cpu-baseline"
cd /tmp
L1="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ATOMIC_RETURN SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $L1 --kernel-include-regex "sk::" --output-format csv -d $O/lds1 -o run -- \
  python3 $R/bench.py $SHORT > $O/lds1.json 2> $O/lds1.err || { echo lds1 failed; tail -5 $O/lds1.err; exit 1; }
L0="SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $L0 --kernel-include-regex "sk::" --output-format csv -d $O/lds0 -o run -- \
  python3 $R/bench.py $SHORT > $O/lds0.json 2> $O/lds0.err || { echo lds0 failed; tail -5 $O/lds0.err; exit 1; }
L2="TCC_ATOMIC TA_FLAT_ATOMIC_WAVEFRONTS TA_BUFFER_ATOMIC_WAVEFRONTS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $L2 --kernel-include-regex "sk::" --output-format csv -d $O/lds2 -o run -- \
  python3 $R/bench.py $SHORT > $O/lds2.json 2> $O/lds2.err || { echo lds2 failed; tail -5 $O/lds2.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $L1 --kernel-include-regex "hll_hist|hll_sum|hll_union" --output-format csv -d $O/lds3 -o run -- \
  python3 $R/bench_configs.py --configs c2zipf,c4 > $O/lds3.json 2> $O/lds3.err || { echo lds3 failed; tail -5 $O/lds3.err; exit 1; }
cd $R && python3 tools/pmc_reduce.py $O/lds0 > /dev/null && python3 tools/pmc_reduce.py $O/lds1 > /dev/null && python3 tools/pmc_reduce.py $O/lds2 > /dev/null && python3 tools/pmc_reduce.py $O/lds3 > /dev/null
echo done
