#!/bin/bash
# Dev: build the engine with extra -D defines into redisson_amd/var_NAME.so (select with SK_LIB_PATH for A/B runs).
# usage: bash tools/build_variant.sh NAME "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/../redisson_amd/csrc"
O=../../build/var_$1; mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $2 -c sk_kernels.hip -o $O/k.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $2 -c sk_store.cpp -o $O/s.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../var_$1.so $O/k.o $O/s.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built ../var_$1.so
