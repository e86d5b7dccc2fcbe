set -o pipefail
mkdir -p gpurun_out/r03i
for cfg in "SK_STAGE=0" "SK_STAGE=1 SK_STAGE_THREADS=16" "SK_STAGE=1 SK_STAGE_THREADS=4"; do
  env $cfg SK_HOST_TIMING=1 timeout -k 10 300 python3 bench_configs.py --configs host > gpurun_out/r03i/h.json 2> gpurun_out/r03i/h.err || { echo fail; tail gpurun_out/r03i/h.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03i/h.json'))
print('$cfg', {k: round(v/1e6,1) if 'per_s' in k else v for k,v in d.items() if k in ('pfadd_ids_host_per_s','group_commit_ids_host_per_s','bloom_contains_host_per_s','pageable_h2d_GBps','pfadd_ids_ms_per_batch')})"
  grep "sk host pfadd" gpurun_out/r03i/h.err | tail -3
done
