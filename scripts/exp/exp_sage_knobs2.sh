#!/bin/bash
# GraphSAGE 10M x 768 pipeline knobs after the XCD-split GEMM (interleaved x2):
# default | GEMM 1 block/CU | gather 2 blocks/CU | 32 chunks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/knobs2; mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 5 --no-cpu --no-hnsw --no-scan > $O/$name.log 2>&1 || { echo "$name failed"; return 1; }
  python3 -c "import json;d=json.loads([l for l in open('$O/$name.log') if l.startswith('{\"metric')][0]);print('$name', round(d['value']/1e9,4), d['kernel_ms'])"
}
for rep in 1 2; do
  run def_$rep RVX_DUMMY=0 || exit 1
  run gemmcap1_$rep RVX_SAGE_GEMM_CAP=1 || exit 1
  run agg2_$rep RVX_AGG_BLOCKS_PER_CU=2 || exit 1
  run ch32_$rep RVX_SAGE_CHUNKS=32 || exit 1
done
