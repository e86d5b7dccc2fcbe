set -o pipefail
O=gpurun_out/${1:-probe4}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --hll-batches 64 --contains-batch 67108864 > $O/g64.json 2> $O/g64.err || { tail $O/g64.err; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/g16.json 2> $O/g16.err || { tail $O/g16.err; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --group 1 > $O/g1.json 2> $O/g1.err || { tail $O/g1.err; exit 1; }
python - $O <<'PY'
import json,sys
for g in ("g64","g16","g1"):
    d=json.load(open(sys.argv[1]+"/%s.json"%g))
    print(g, "value %.3e ms/step %.3f hll/s %.3e contains/s %.3e frac %.3f %s" % (d["value"], d["ms_per_step"], d["hll_inserts_per_s"], d["bloom_contains_per_s"], d["roofline"]["frac"], d["roofline"]["kernel"]))
    print({k:(round(v["ms_isolated"],4), round(v["ms_overlapped"] or 0,4)) for k,v in d["kernels"].items()})
PY
