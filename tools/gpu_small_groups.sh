set -o pipefail
O=gpurun_out/small; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lines.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; tail -1 $O/t.log
for hb in 4 16; do for g in $hb 1; do
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --hll-batches $hb --group $g --contains-batch 4194304 --bloom-fill 100000000 > $O/h${hb}_g$g.json 2> $O/h${hb}_g$g.err || exit 1
python -c "import json;d=json.load(open('$O/h${hb}_g$g.json'));print('hb $hb g $g hll/s %.3e'%d['hll_inserts_per_s'], {k:round(v['ms_isolated'],3) for k,v in d['kernels'].items() if 'p' in k[:3]})"
done; done
