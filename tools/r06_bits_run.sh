set -o pipefail
R=$(pwd); O=$R/gpurun_out/r06b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bits.py tests/test_jni_drive.py tests/test_gpu_persist.py tests/test_gpu_parity.py > $O/tests1.log 2>&1 || { echo T1 FAILED; tail -40 $O/tests1.log; exit 1; }
tail -1 $O/tests1.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5trace -o run -- python3 $R/tools/c5_host_trace.py > $O/c5trace.log 2>&1 || { echo trace failed; tail $O/c5trace.log; exit 1; }
cat $O/c5trace.log; rm -f $O/c5trace/run_kernel_trace.csv
cd $R && timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
