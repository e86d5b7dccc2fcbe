#!/bin/bash
# Dev scratch: the last A/B command sent to the GPU box this round (parity of the variants, then tools/gpu_ab.sh).
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
SK_LIB_PATH=$PWD/redisson_amd/var_oneb.so timeout -k 10 600 $T tests/test_gpu_lines.py tests/test_full_size.py tests/test_gpu_fuzz.py -k "lines or c2 or fuzz" > $O/tests_oneb.log 2>&1 || { echo ONEB TESTS FAILED; tail -30 $O/tests_oneb.log; exit 1; }
tail -1 $O/tests_oneb.log
bash tools/gpu_ab.sh r03e "base oneb" "--steps 5 --warmup 1 --no-cpu-baseline" || exit 1
bash tools/gpu_ab.sh r03e2 "base oneb" "--steps 5 --warmup 1 --no-cpu-baseline" || exit 1
echo all done
