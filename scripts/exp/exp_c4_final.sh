#!/bin/bash
# Round 3: C4 targeted tests, then the 10M C4 stack (twice) at the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c4f; mkdir -p $O
stop() { echo "STOP after $1 (exit $2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c4_stack.py \
  -k "ruvector or producer or finish or edge or c4" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ge 1 ] && stop tests $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench_gnn.py --nodes 10000000 --no-cpu > $O/c4_$i.log 2>&1 || stop c4 $?
  grep -o '"ms_per_step": [0-9.]*' $O/c4_$i.log; grep -o '"kernel_ms_per_step": {[^}]*}' $O/c4_$i.log
done
