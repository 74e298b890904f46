#!/bin/bash
# Overlapped 10M x 768 step: GEMM 256x192 8-wave (RVX_GEMM_WIDE=3) with the gather at one block
# per CU, vs the 128x192 4-wave GEMM (4: one GEMM wave per SIMD) with the gather at 2 or 1 blocks
# per CU (RVX_AGG_BLOCKS_PER_CU), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wide4; mkdir -p $O
i=0
for arm in ${ARMS:-3:1 4:2 4:1 3:1 4:2 4:1}; do
  i=$((i+1)); w=${arm%%:*}; c=${arm##*:}
  RVX_GEMM_WIDE=$w RVX_AGG_BLOCKS_PER_CU=$c timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/r${i}_${w}_${c}.log 2>&1 || exit 4
  python - $O/r${i}_${w}_${c}.log "wide=$w agg_cap=$c" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["roofline_kernels"]
        print(sys.argv[2], "ms/step", d["ms_per_step"], {n: (v["avg_ms"], v["launches"]) for n, v in k.items()}, flush=True)
PY
done
