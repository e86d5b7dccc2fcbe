#!/bin/bash
# Round-4 dev run on the GPU box: selected GPU tests (TESTS, pytest -k expression or file list), then an A/B of the
# engine builds in VARS (tools/gpu_ab.sh) on the default bench.  Usage: TESTS="..." bash tools/r04_ab.sh TAG "base v1"
set -o pipefail
T=${1:-r04x}; VARS=${2:-base}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 \
    || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
bash tools/gpu_ab.sh $T "$VARS" "${BARGS:---steps 5 --warmup 1 --no-cpu-baseline}"
