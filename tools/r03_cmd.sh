set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_gpu_lines.py tests/test_gpu_region.py tests/test_full_size.py tests/test_gpu_parity.py -k "lines or region or full or long" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SK_LIB_PATH=$PWD/redisson_amd/var_ra4k.so timeout -k 10 600 $T tests/test_gpu_region.py tests/test_full_size.py -k "region or c3" > $O/tests_ra4k.log 2>&1 || { echo RA4K TESTS FAILED; tail -30 $O/tests_ra4k.log; exit 1; }
tail -1 $O/tests_ra4k.log
SK_LIB_PATH=$PWD/redisson_amd/var_lf.so timeout -k 10 600 $T tests/test_gpu_lines.py > $O/tests_lf.log 2>&1 || { echo LF TESTS FAILED; tail -30 $O/tests_lf.log; exit 1; }
tail -1 $O/tests_lf.log
SK_LIB_PATH=$PWD/redisson_amd/var_r2.so timeout -k 10 600 $T tests/test_gpu_lines.py > $O/tests_r2.log 2>&1 || { echo R2 TESTS FAILED; tail -30 $O/tests_r2.log; exit 1; }
tail -1 $O/tests_r2.log
bash tools/gpu_ab.sh r03c "h0 base lf ra4k ra0 r2" "--steps 5 --warmup 1 --no-cpu-baseline --add-chunk 33554432" || exit 1
SK_HOST_TIMING=1 timeout -k 10 300 python3 -u bench_configs.py --configs host > $O/host.jsonl 2> $O/host.err || { echo host failed; tail -5 $O/host.err; exit 1; }
SK_STAGE=1 timeout -k 10 300 python3 -u bench_configs.py --configs host > $O/host_stage.jsonl 2> $O/host_stage.err || { echo host2 failed; tail -5 $O/host_stage.err; exit 1; }
echo all done
