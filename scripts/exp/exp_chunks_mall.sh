#!/bin/bash
# GraphSAGE 10M x 768 layer vs pipeline chunk count: small chunks keep each chunk's aggregate
# (and GEMM output) within the 256 MB Infinity Cache between producer and consumer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/chunks
i=0
for c in ${CHUNKS:-24 64 128 256}; do
  i=$((i+1))
  RVX_SAGE_CHUNKS=$c timeout -k 10 300 python -u bench.py --steps ${STEPS:-4} --warmup 2 --no-hnsw --no-scan --no-cpu > gpurun_out/chunks/r${i}_c$c.log 2>&1 || exit 4
  python - gpurun_out/chunks/r${i}_c$c.log $c <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["roofline_kernels"]
        print("chunks", sys.argv[2], "ms/step", d["ms_per_step"], {n: (v["avg_ms"], v["launches"]) for n, v in k.items()}, flush=True)
PY
done
