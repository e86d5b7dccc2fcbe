#!/bin/bash
# Round-4 host-ingress A/B (dev tool, GPU box): bench_configs.py host under staging settings.
# usage: bash tools/r04_host.sh TAG "ENV1" "ENV2" ...   (ENV "-" = defaults)
set -o pipefail
T=$1; shift
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
i=0
for e in "$@"; do
  i=$((i+1))
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 400 python3 -u bench_configs.py --configs host > $O/h$i.jsonl 2> $O/h$i.err || { echo "run $i failed"; tail -5 $O/h$i.err; exit 1; }
  python3 - "$O/h$i.jsonl" "$e" <<'PY'
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print('%-40s pfadd_ids %.0f M/s (%.2f ms)  group %.0f M/s  pinned %.0f M/s  contains %.0f M/s  add %.0f M/s' % (sys.argv[2] or 'default',
  d['pfadd_ids_host_per_s']/1e6, d['pfadd_ids_ms_per_batch'], d['group_commit_ids_host_per_s']/1e6, d['group_commit_ids_pinned_per_s']/1e6,
  d['bloom_contains_host_per_s']/1e6, d['bloom_add_host_per_s']/1e6))
print('%-40s prefix form: pfadd_ids %.0f M/s (%.2f ms)  group %.0f M/s  pinned %.0f M/s  contains %.0f M/s' % ('',
  d['pfadd_ids_prefix_host_per_s']/1e6, d['pfadd_ids_prefix_ms_per_batch'], d['group_commit_prefix_host_per_s']/1e6,
  d['group_commit_prefix_pinned_per_s']/1e6, d['bloom_contains_prefix_host_per_s']/1e6))
PY
done
