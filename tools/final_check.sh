#!/bin/bash
# round-end check on the GPU box: full GPU suite, smoke, then the profile recipe (trace, PMC passes, clean bench)
set -o pipefail
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
bash profiles/run_profile.sh $T
