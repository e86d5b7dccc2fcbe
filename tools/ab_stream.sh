#!/bin/bash
# A/B of the streaming PFCOUNT-histogram / union kernels through bench_configs (GPU box, repo root):
#   bash tools/ab_stream.sh "VAR=a" "VAR=b"   -> gpurun_out/ab_stream/<i>_<rep>.jsonl
set -o pipefail
O=gpurun_out/ab_stream; mkdir -p $O
for rep in 1 2; do i=0; for kv in "$@"; do i=$((i+1))
env $kv timeout -k 10 200 python -u bench_configs.py --configs c2zipf,c4 > $O/${i}_$rep.jsonl 2> $O/${i}_$rep.err || { tail $O/${i}_$rep.err; exit 1; }
python3 -c "
import json
for l in open('$O/${i}_$rep.jsonl'):
    d=json.loads(l); r=d.get('roofline',{}); print('$kv', d['metric'][:30], r.get('kernel'), round(r.get('achieved',0)), r.get('avg_launch_ms'))"
done; done
