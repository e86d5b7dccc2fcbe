set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lines.py tests/test_full_size.py tests/test_gpu_fuzz.py tests/test_gpu_hllstr.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r06e_ab "base u8 xord0 xord16"
