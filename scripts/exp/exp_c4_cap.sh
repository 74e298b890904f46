#!/bin/bash
# C4 stack (2M x 768) with the standalone GEMMs on a persistent grid (RVX_GEMM_CAP=1: one
# block per CU taking tiles from the per-XCD queue) vs one block per tile (0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c4cap; mkdir -p $O
i=0
for v in ${ARMS:-1 0 1 0}; do
  i=$((i+1))
  RVX_GEMM_CAP=$v timeout -k 10 400 python -u bench_gnn.py --nodes 2000000 --steps 2 --warmup 1 --no-cpu > $O/r${i}_$v.log 2>&1 || exit 4
  python - $O/r${i}_$v.log $v <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["kernel_ms_per_step"]
        print("cap", sys.argv[2], "ms/step", d["ms_per_step"], "gemm", round(sum(v for a, v in k.items() if "gemm" in a), 1), {a: round(v, 1) for a, v in k.items() if "gemm" in a}, flush=True)
PY
done
