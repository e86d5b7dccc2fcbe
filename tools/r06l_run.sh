# histogram counters: parity at the new build, then 16-bit packed (base) vs u32 (hh32) counters on c2zipf
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "hll or pfcount or union or count" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r06_ab_cfg.sh r06l_ab "base hh32" "c2zipf"
for f in gpurun_out/r06l_ab/*.jsonl; do python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1], d['hll_hist']['avg_launch_ms'], d['roofline']['avg_launch_ms'])" $f; done
