# PFCOUNT histograms: rows of the low 5 bits with a rare slow path for registers >= 32 (base) vs bins 2i / 2i + 1 in
# the halves (head): the histogram / PFCOUNT parity tests, then c2zipf A/B (hll_hist avg_launch_ms)
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_distributed.py -k "hll or pfcount or count or union or hist or golden" > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r06_ab_cfg.sh r06z_ab "base head" "c2zipf"
for f in gpurun_out/r06z_ab/*.jsonl; do python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[1], d['hll_hist']['avg_launch_ms'], d['roofline']['avg_launch_ms'])" $f; done
