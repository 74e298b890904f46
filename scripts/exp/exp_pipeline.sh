#!/bin/bash
# Sweep of the layer pipeline knobs on the 1M x 768 bench workload:
# chunks, gather grid cap (blocks/CU, overlapped launches), gather rows in
# flight, GEMM register-prefetch depth.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${CFGS:-"8 1 8 1"}
IFS='|' read -ra LIST <<< "$CFGS"
for cfg in "${LIST[@]}"; do
  set -- $cfg
  tag="c$1_cap$2_u$3_d$4"
  tag="${tag}_nt${RVX_AGG_NT:-1}_x3${RVX_GEMM_X3:-1}"
  RVX_SAGE_CHUNKS=$1 RVX_AGG_BLOCKS_PER_CU=$2 RVX_AGG_UNROLL=$3 RVX_GEMM_DEPTH=$4 \
    timeout -k 10 300 python bench.py --nodes ${NODES:-1000000} --no-cpu --no-hnsw --steps 5 > gpurun_out/exp_$tag.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$tag failed rc=$rc"; tail -5 gpurun_out/exp_$tag.log; exit $rc; fi
  python3 - "$tag" gpurun_out/exp_$tag.log <<'PY'
import json, sys
l = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
rk = l["roofline_kernels"]
print(f"{sys.argv[1]}: {l['ms_per_step']:.2f} ms/step  agg {rk['sage_aggregate']['achieved']:.0f} GB/s  "
      f"gemm {rk['sage_gemm']['achieved']:.1f} TF  kernel_ms {l['kernel_ms']}")
PY
done
