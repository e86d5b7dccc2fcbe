# SETBIT with replies: record loads issued with the region loads (base) vs after them (head):
# the bit tests, then C5 (replies path host + device) A/B
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bits.py tests/test_gpu_parity.py tests/test_jni_drive.py -k "bit or setbit or getbit or jni" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r06_ab_cfg.sh r06x_ab "base head" "c5"
