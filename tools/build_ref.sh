#!/bin/bash
# Dev: build the engine as it was at a git ref into redisson_amd/var_NAME.so (A/B baseline for tools/gpu_ab.sh).
# usage: bash tools/build_ref.sh NAME [REF=HEAD] ["-DFOO=1 ..."]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REF=${2:-HEAD}; DEFS=${3:-}
O=$R/build/ref_$NAME; rm -rf $O; mkdir -p $O/redisson_amd/csrc $O/include
for f in redisson_amd/csrc/sk_kernels.hip redisson_amd/csrc/sk_store.cpp redisson_amd/csrc/sk_device.h \
         redisson_amd/csrc/sk_internal.h redisson_amd/csrc/sk_hllstr.h redisson_amd/csrc/sk_rdb.h include/redisson_sketch.h; do
  git -C $R show $REF:$f > $O/$f
done
cd $O/redisson_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $DEFS -c sk_kernels.hip -o k.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $DEFS -c sk_store.cpp -o s.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/redisson_amd/var_$NAME.so k.o s.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built redisson_amd/var_$NAME.so from $REF
