# configs only (after a green test run): c2zipf (PFCOUNT sums / histograms) and c4 (union)
set -o pipefail
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python3 -u bench_configs.py --configs ${CFGS:-c2zipf,c4} > $O/cfg.jsonl 2> $O/cfg.err || { echo cfg failed; tail $O/cfg.err; exit 1; }
python3 -c "
import json
for ln in open('$O/cfg.jsonl'):
    d=json.loads(ln); print(d['metric'][:50], round(d['value']/1e9,3), 'roof', round(d['roofline']['frac'],3) if 'roofline' in d else None, round(d['roofline']['avg_launch_ms'],4) if 'roofline' in d else None, d.get('hll_hist'))
"
