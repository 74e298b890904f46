#!/bin/bash
# Interleaved A/B, 10M x 768 sage legs only: dense gather vs register-expanded row images.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python -u bench.py --steps 5 --warmup 2 --no-cpu --no-scan --no-c4 --no-hnsw --no-c3"
for rep in 1 2 3 4 5; do
  for v in dense reg; do
    case $v in dense) env="RVX_SAGE_IMAGE=0";; reg) env="RVX_SAGE_IMAGE=1 RVX_IMG_REG=1";; esac
    env $env timeout -k 10 300 $B > gpurun_out/img2_${v}_${rep}.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/img2_${v}_${rep}.log; exit 1; }
    python3 - "$v" "$rep" <<'PY'
import json, sys
j = json.loads([l for l in open(f"gpurun_out/img2_{sys.argv[1]}_{sys.argv[2]}.log") if l.startswith("{")][-1])
k = j["kernel_ms"]
print(sys.argv[1], sys.argv[2], j["ms_per_step"], k.get("sage_aggregate"), k.get("sage_aggregate_img"), k.get("sage_gemm"),
      k.get("rows_image_pack"), k.get("sage_normalize"), flush=True)
PY
  done
done
