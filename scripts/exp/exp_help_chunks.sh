#!/bin/bash
# Round 3: GraphSAGE row-chunk count with the GEMM helping the gather (interleaved, 10M x 768).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hc; mkdir -p $O
i=0
for c in ${CH:-24 16 32 48 24 16 32 48}; do
  i=$((i+1))
  RVX_SAGE_CHUNKS=$c timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/c${i}_$c.log 2>&1 || exit 4
  echo "chunks=$c $(grep -o '"ms_per_step": [0-9.]*' $O/c${i}_$c.log)"
done
