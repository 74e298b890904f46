#!/bin/bash
# Last-layer normalisation placement A/B at 10M x 768 (bench.py sage legs): in line between the
# GEMMs (RVX_SAGE_NORM_AUX=0) vs on the gather stream behind the next gather (1), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "graphsage or sage" > gpurun_out/normaux_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/normaux_tests.log; exit 1; }
tail -1 gpurun_out/normaux_tests.log
B="python -u bench.py --steps 5 --warmup 2 --no-cpu --no-scan --no-c4 --no-hnsw --no-c3"
for rep in 1 2 3; do
  for v in 0 1; do
    RVX_SAGE_NORM_AUX=$v timeout -k 10 300 $B > gpurun_out/normaux_${v}_${rep}.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/normaux_${v}_${rep}.log; exit 1; }
    python3 - "$v" "$rep" <<'PY'
import json, sys
line = [l for l in open(f"gpurun_out/normaux_{sys.argv[1]}_{sys.argv[2]}.log") if l.startswith("{")][-1]
j = json.loads(line)
k = j["kernel_ms"]
print("norm_aux", sys.argv[1], sys.argv[2], "ms/step", j["ms_per_step"], "edges/s %.3fG" % (j["value"] / 1e9),
      "agg", k.get("sage_aggregate"), "gemm", k.get("sage_gemm"), "norm", k.get("sage_normalize"))
PY
  done
done
