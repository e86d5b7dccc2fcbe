# the histogram tests (the slow path for registers >= 32 included)
set -o pipefail
O=gpurun_out/r06z2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "histogram" > $O/hist.log 2>&1 || { echo HIST FAILED; tail -30 $O/hist.log; exit 1; }
grep -c PASSED $O/hist.log
