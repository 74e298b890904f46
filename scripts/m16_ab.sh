#!/bin/bash
# 16x16x32 MFMA form of the pipelined GraphSAGE GEMM (RVX_GEMM_M16) A/B at 10M x 768, interleaved,
# after its tests; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "m16 or wide_gemm_bits or helps_gather" > gpurun_out/m16_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/m16_tests.log; exit 1; }
tail -1 gpurun_out/m16_tests.log
B="python -u bench.py --steps 5 --warmup 2 --no-cpu --no-scan --no-c4 --no-hnsw --no-c3"
for rep in 1 2 3 4; do
  for v in 0 1; do
    RVX_GEMM_M16=$v timeout -k 10 300 $B > gpurun_out/m16_${v}_${rep}.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/m16_${v}_${rep}.log; exit 1; }
    python3 - "$v" "$rep" <<'PY'
import json, sys
j = json.loads([l for l in open(f"gpurun_out/m16_{sys.argv[1]}_{sys.argv[2]}.log") if l.startswith("{")][-1])
k = j["kernel_ms"]
print("m16", sys.argv[1], sys.argv[2], j["ms_per_step"], "agg", k.get("sage_aggregate"), "gemm", k.get("sage_gemm"),
      "norm", k.get("sage_normalize"), flush=True)
PY
  done
done
