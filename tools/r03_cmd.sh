set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_lines.py tests/test_gpu_region.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SK_LIB_PATH=$PWD/redisson_amd/var_mark.so timeout -k 10 600 $T tests/test_gpu_lines.py tests/test_full_size.py -k "lines or c2" > $O/tests_mark.log 2>&1 || { echo MARK TESTS FAILED; tail -30 $O/tests_mark.log; exit 1; }
tail -1 $O/tests_mark.log
SK_LIB_PATH=$PWD/redisson_amd/var_own.so timeout -k 10 600 $T tests/test_gpu_region.py tests/test_full_size.py -k "region or c3" > $O/tests_own.log 2>&1 || { echo OWN TESTS FAILED; tail -30 $O/tests_own.log; exit 1; }
tail -1 $O/tests_own.log
bash tools/gpu_ab.sh r03d "base mark own" "--steps 5 --warmup 1 --no-cpu-baseline" || exit 1
echo all done
