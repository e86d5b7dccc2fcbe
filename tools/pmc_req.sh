#!/bin/bash
# Dev: memory-side request counts by size (TCC_EA0_RDREQ 32/64/128 B, TCC_EA0_WRREQ 64 B) of the bench's chain
# kernels for several engine builds, so read / write bytes are counted at each request's own size instead of
# FETCH_SIZE's fixed tally.  Usage on the box (repo root): bash tools/pmc_req.sh TAG "base v1" [kernel regex]
set -o pipefail
T=$1; VARS=$2; RX=${3:-k_pfl|k_bloom_rc|k_rc_}
R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
SHORT="--steps 2 --warmup 1 --no-cpu-baseline"
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
WR="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
for v in $VARS; do
  if [ "$v" = base ]; then L=$R/redisson_amd/libredisson_sketch.so; else L=$R/redisson_amd/var_$v.so; fi
  for p in rd wr; do
    if [ $p = rd ]; then C=$RD; else C=$WR; fi
    (cd /tmp && SK_LIB_PATH=$L timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv \
      -d $O/$v.$p -o run -- python3 $R/bench.py $SHORT > $O/$v.$p.json 2> $O/$v.$p.err) || { echo "$v $p failed"; exit 1; }
    python3 tools/pmc_reduce.py $O/$v.$p > /dev/null || exit 1
  done
  python3 tools/pmc_req_bytes.py $O $v || exit 1
done
