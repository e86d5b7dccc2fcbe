# the N = 2 bench path end to end (two ranks sharing the box's one GPU; says nothing about scaling)
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --no-cpu-baseline > $O/bench_n2_shared_gpu.json 2> $O/bench_n2.err || { echo n2 failed; tail -20 $O/bench_n2.err; exit 1; }
cat $O/bench_n2_shared_gpu.json | cut -c1-400
