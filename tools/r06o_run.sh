# union: parity at the new build, then u16-pair running max (base) vs unpack-to-u8 (old) on c4 (+ c2zipf PFCOUNT)
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_full_size.py tests/test_distributed.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r06_ab_cfg.sh r06o_ab "base old" "c4"
for f in gpurun_out/r06o_ab/*.jsonl; do python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" $f; done
bash tools/r06_ab_cfg.sh r06o_lines "base e_SK_PFL_MIN=1+SK_PFL_RATIO=1" "c2u"
