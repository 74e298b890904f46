#!/bin/bash
# Round 3: register-resident GRU finish + att row maxima from the edge kernel: bit-identity
# tests, the 10M C4 stack with the finish in registers (1) and the loop form (0), then the
# rocprofv3 kernel trace + PMC traffic of the default GraphSAGE bench (scripts/gpu_profile.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fin; mkdir -p $O
stop() { echo "STOP after $1 (exit $2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "finish_in_registers or producer_row_maxima or test_ruvector or edge" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ge 1 ] && stop tests $rc
for v in 1 0; do
  RVX_GNN_FINISH_REG=$v timeout -k 10 300 python -u bench_gnn.py --nodes 10000000 --no-cpu > $O/c4_$v.log 2>&1 || stop c4 $?
  echo "finish_reg=$v"; grep -o '"ms_per_step": [0-9.]*' $O/c4_$v.log; grep -o '"gnn_finish": [0-9.]*\|"gemm_row_scale": [0-9.]*' $O/c4_$v.log
done
bash scripts/gpu_profile.sh
