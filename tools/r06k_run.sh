# PFADD parity + PFCOUNT at the new build, then the one-RBatch-per-call A/B (word-merged stores vs XORs)
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_full_size.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench_configs.py --configs c2zipf,c4 > $O/cfg.jsonl 2> $O/cfg.err || { echo cfg failed; tail $O/cfg.err; exit 1; }
python3 -c "
import json
for ln in open('$O/cfg.jsonl'):
    d=json.loads(ln); print(d['metric'][:50], round(d['value']/1e9,3), 'roof', round(d['roofline']['frac'],3), round(d['roofline']['avg_launch_ms'],4), d.get('hll_hist'))
"
bash tools/r06_ab_cfg.sh r06k_ab "base xor" "c2u,c1"
