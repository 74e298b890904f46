#!/bin/bash
# Layer-GEMM tiling sweep on the serial 1M x 768 layer and the 10M pipeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wm in 4 8; do
  RVX_GEMM_WM=$wm RVX_SAGE_CHUNKS=1 timeout -k 10 200 python bench.py --nodes 1000000 --no-cpu --no-hnsw --steps 5 --warmup 2 > gpurun_out/tile_1m_wm$wm.json 2> gpurun_out/tile_1m_wm$wm.err || exit 1
  RVX_GEMM_WM=$wm timeout -k 10 300 python bench.py --no-cpu --no-hnsw > gpurun_out/tile_10m_wm$wm.json 2> gpurun_out/tile_10m_wm$wm.err || exit 1
done
echo done
