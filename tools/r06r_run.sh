# partition apply loading each register when it writes it (base) vs at gather time (early): parity, then A/B
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
SK_LIB_PATH=$(pwd)/redisson_amd/libredisson_sketch.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_full_size.py -k "pfadd or partition or golden or hll" > $O/tests_late.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests_late.log; exit 1; }
tail -1 $O/tests_late.log
bash tools/r06_ab_cfg.sh r06r_ab "base early" "c2u,c1,c2zipf"
for f in gpurun_out/r06r_ab/*.jsonl; do python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d['config']['workload']=='c2u': print(sys.argv[1], d['kernel_ms'], d['device_ms_per_call'])" $f; done
