#!/bin/bash
# Dev: line-schedule ablations on the bench (results discarded; SK_PFL_PROBE flags in sk_kernels.hip):
#   256 apply: run table only | 128 apply: lines + records loaded, nothing applied | 4 apply: no line loads/stores
#   64 apply: no reply stores | 2048 region: no record loads | 1024 region: no write-out
set -o pipefail
O=gpurun_out/${1:-r03abl}; mkdir -p $O
for f in 0 256 128 4 64 2048 1024; do
  SK_PFL_PROBE=$f timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/p$f.json 2> $O/p$f.err || { echo "probe $f failed"; tail -3 $O/p$f.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']; print('probe %5s' % sys.argv[2], ' '.join('%s %.3f' % (n, v['ms_isolated']) for n, v in k.items()))" $O/p$f.json $f
done
echo done
