# FETCH_SIZE and WRITE_SIZE (separate passes) for kernels matching $1 over a short bench run
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_rw
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$1" --output-format csv -d $O/f -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bf.json 2> $O/ef.txt && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$1" --output-format csv -d $O/w -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bw.json 2> $O/ew.txt
