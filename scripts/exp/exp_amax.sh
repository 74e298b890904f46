#!/bin/bash
# Round 3: producer row maxima for the C4 layer GEMMs (RVX_GEMM_AMAX). New bit-identity
# test first, then the 10M C4 stack with and without, then the GPU suite, smoke and bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "STOP after $1 (exit $2)"; exit "$2"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "producer_row_maxima or ruvector_layer_wide" > gpurun_out/amax_tests.log 2>&1
rc=$?; tail -3 gpurun_out/amax_tests.log; [ $rc -ge 1 ] && stop amax_tests $rc
for v in 1 0 1; do
  RVX_GEMM_AMAX=$v timeout -k 10 300 python -u bench_gnn.py --nodes 10000000 --no-cpu > gpurun_out/c4_amax$v.log 2>&1
  rc=$?; echo "amax=$v"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4_amax$v.log; [ $rc -ge 2 ] && stop c4 $rc
done
[ "${FULL:-1}" = "1" ] || exit 0
bash scripts/gpu_check.sh
