# A/B: bench with the in-tree library and with abl/$1, alternating, $2 rounds each
mkdir -p gpurun_out/ab
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 240 python3 bench.py --no-cpu-baseline > gpurun_out/ab/new_$i.json 2>/dev/null || exit 1
  SK_LIB_PATH=$PWD/abl/$1 timeout -k 10 240 python3 bench.py --no-cpu-baseline > gpurun_out/ab/old_$i.json 2>/dev/null || exit 1
done
