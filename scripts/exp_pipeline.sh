#!/bin/bash
# Sweep of the layer pipeline knobs (chunks x gather grid cap) on the bench workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "8 1 4" "8 1 8" "8 2 8" "1 0 8" "4 1 8" "16 1 8"; do
  set -- $cfg; export RVX_AGG_UNROLL=$3
  RVX_SAGE_CHUNKS=$1 RVX_AGG_BLOCKS_PER_CU=$2 timeout -k 10 180 python bench.py --no-cpu --no-hnsw --steps 5 > gpurun_out/exp_$1_$2_$3.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "chunks=$1 agg_cap=$2 failed rc=$rc"; tail -5 gpurun_out/exp_$1_$2_$3.log; exit $rc; fi
  python3 - "$1" "$2" gpurun_out/exp_$1_$2_$3.log <<'PY'
import json, sys
l = json.loads([x for x in open(sys.argv[3]) if x.startswith("{")][-1])
k = l["kernel_ms"]; rk = l["roofline_kernels"]
print(f"chunks={sys.argv[1]} agg_cap={sys.argv[2]} unroll={__import__('os').environ['RVX_AGG_UNROLL']}: {l['ms_per_step']:.2f} ms/step  agg {rk['sage_aggregate']['achieved']:.0f} GB/s  gemm {rk['sage_gemm']['achieved']:.1f} TF  launches {rk['sage_gemm']['launches']}")
PY
done
