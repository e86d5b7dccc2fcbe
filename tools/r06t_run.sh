# hash workgroups' bucket counts as u16 (LDS 81,472 -> 81,152 B for the line hash) and the partition path's block
# size as a parameter (4096 kept): the PFADD parity files, then the default bench and group-commit configs against
# the previous commit (head)
set -o pipefail
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_full_size.py tests/test_gpu_lines.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r06t_bench "base head"
bash tools/r06_ab_cfg.sh r06t_cfg "base head" "c1,c2zipf"
