set -e
mkdir -p gpurun_out/exp1
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 150 $B > gpurun_out/exp1/base.json 2>&1
SK_PFP_PIPE=0 timeout -k 10 150 $B > gpurun_out/exp1/nopipe.json 2>&1
SK_PFA_DLDS=65536 timeout -k 10 150 $B > gpurun_out/exp1/occ1.json 2>&1
SK_PFP_PIPE=0 SK_PFA_DLDS=65536 timeout -k 10 150 $B > gpurun_out/exp1/occ1_nopipe.json 2>&1
