#!/bin/bash
# Round 3: the layer's first gather chunk on a wider grid (RVX_AGG_FIRST_CAP) — interleaved
# 10M GraphSAGE runs, then the C4 stack under rocprofv3 (scripts/c4_profile.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fc; mkdir -p $O
stop() { echo "STOP after $1 (exit $2)"; exit "$2"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "gemm_helps_gather" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ge 1 ] && stop tests $rc
i=0
for v in 4 1 4 1 4 1; do
  i=$((i+1))
  RVX_AGG_FIRST_CAP=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/s${i}_$v.log 2>&1 || stop sage $?
  echo "first_cap=$v $(grep -o '"ms_per_step": [0-9.]*' $O/s${i}_$v.log)"
done
bash scripts/c4_profile.sh
