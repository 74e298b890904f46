#!/bin/bash
# A/B of the per-XCD GEMM tile queue (RVX_GEMM_QUEUE) on the 10M pipeline, then
# a FETCH_SIZE pass with the queue on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    RVX_GEMM_QUEUE=$v timeout -k 10 300 python bench.py --no-cpu --no-hnsw --no-scan > gpurun_out/q${v}_$i.json 2> gpurun_out/q${v}_$i.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/q${v}_$i.json')); print('queue=$v', d['value']/1e9, d['kernel_ms'])"
  done
done
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$ROOTDIR/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-hnsw --no-scan > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$ROOTDIR/gpurun_out/pmc_write" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-hnsw --no-scan > gpurun_out/pmc_write.log 2>&1 || exit 1
python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json gpurun_out/pmc_fetch.log
cat gpurun_out/pmc_traffic.json
