# partition path with 2048-element hash blocks (two hash workgroups per CU, base) vs 4096 (epb4096): the PFADD
# parity tests of the new build (the whole gpu suite's PFADD files), then c2u / c1 / c2zipf A/B
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_full_size.py tests/test_gpu_persist.py tests/test_gpu_hllstr.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r06_ab_cfg.sh r06s_ab "base epb4096" "c2u,c1,c2zipf"
for f in gpurun_out/r06s_ab/*.jsonl; do python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d['config']['workload']=='c2u': print(sys.argv[1], d['kernel_ms'], d['device_ms_per_call'])" $f; done
