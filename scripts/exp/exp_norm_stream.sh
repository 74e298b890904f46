#!/bin/bash
# GraphSAGE 10M x 768: the row normalisation on a third stream (RVX_SAGE_NORM_STREAM=1, default)
# vs on the GEMM stream (0), alternating arms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/normstream; mkdir -p $O
i=0
for v in ${ARMS:-1 0 1 0 1 0}; do
  i=$((i+1))
  RVX_SAGE_NORM_STREAM=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/r${i}_$v.log 2>&1 || exit 4
  python - $O/r${i}_$v.log $v <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["roofline_kernels"]
        print("norm_stream", sys.argv[2], "ms/step", d["ms_per_step"], "parity", d.get("parity"), {n: (v["avg_ms"], v["launches"]) for n, v in k.items()}, flush=True)
PY
done
