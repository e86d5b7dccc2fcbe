set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lines.py tests/test_gpu_region.py tests/test_full_size.py tests/test_gpu_parity.py -k "lines or region or full or long" > gpurun_out/r03b/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03b/tests.log; exit 1; }
tail -2 gpurun_out/r03b/tests.log
bash tools/gpu_ab.sh r03b "base" "--steps 5 --warmup 1 --no-cpu-baseline --add-chunk 33554432"
