#!/bin/bash
# Round-2 re-tune of the GraphSAGE pipeline knobs with the queued GEMM: chunk
# count, GEMM blocks per CU, gather blocks per CU (interleaved repeats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/knobs
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu --no-hnsw --no-scan > gpurun_out/knobs/$name.json 2> gpurun_out/knobs/$name.err || { echo "$name failed"; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/knobs/$name.json')); print('$name', round(d['value']/1e9,4), d['kernel_ms'])"
}
for rep in 1 2; do
  run base_$rep RVX_SAGE_CHUNKS=24 || exit 1
  run ch16_$rep RVX_SAGE_CHUNKS=16 || exit 1
  run ch32_$rep RVX_SAGE_CHUNKS=32 || exit 1
  run gcap1_$rep RVX_SAGE_GEMM_CAP=1 || exit 1
  run agg2_$rep RVX_AGG_BLOCKS_PER_CU=2 || exit 1
  run gcap1agg2_$rep RVX_SAGE_GEMM_CAP=1 RVX_AGG_BLOCKS_PER_CU=2 || exit 1
done
