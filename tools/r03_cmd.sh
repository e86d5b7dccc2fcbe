set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lines.py tests/test_gpu_region.py tests/test_full_size.py tests/test_gpu_parity.py tests/test_distributed.py -k "lines or region or full or long or engine or rccl or route" > gpurun_out/r03a/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03a/tests.log; exit 1; }
tail -2 gpurun_out/r03a/tests.log
bash tools/gpu_ab.sh r03a "h0 base pf2 ra16" "--steps 5 --warmup 1 --no-cpu-baseline --add-chunk 33554432" || exit 1
bash tools/r03_lds.sh r03lds || exit 1
timeout -k 10 600 python3 -u bench_configs.py > gpurun_out/r03a/configs.jsonl 2> gpurun_out/r03a/configs.err || { echo configs failed; tail -5 gpurun_out/r03a/configs.err; exit 1; }
echo all done
