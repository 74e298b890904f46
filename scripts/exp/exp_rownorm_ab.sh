#!/bin/bash
# GraphSAGE 10M x 768: in-GEMM row normalisation (RVX_GEMM_ROWNORM=1) vs the separate pass (0), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rownorm; mkdir -p $O
i=0
for v in ${ARMS:-1 0 1 0 1 0}; do
  i=$((i+1))
  RVX_GEMM_ROWNORM=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/r${i}_$v.log 2>&1 || exit 4
  python - $O/r${i}_$v.log $v <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["roofline_kernels"]
        print("rownorm", sys.argv[2], "ms/step", d["ms_per_step"], "parity", d.get("parity"), {n: (v["avg_ms"], v["launches"]) for n, v in k.items()}, flush=True)
PY
done
