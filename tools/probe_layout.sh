set -o pipefail
O=gpurun_out/${1:-probe}; shift; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
i=0
for a in "$@"; do
i=$((i+1))
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $a > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
done
python - $O $# <<'PY'
import json,sys
for i in range(1,int(sys.argv[2])+1):
    d=json.load(open(sys.argv[1]+"/b%d.json"%i))
    print(i, "value %.3e ms/step %.3f hll/s %.3e contains/s %.3e frac %.3f %s" % (d["value"], d["ms_per_step"], d["hll_inserts_per_s"], d["bloom_contains_per_s"], d["roofline"]["frac"], d["roofline"]["kernel"]))
    print({k:(round(v["ms_isolated"],4), round(v["ms_overlapped"] or 0,4)) for k,v in d["kernels"].items()})
PY
