#!/bin/bash
# Dense vs ReLU-sparse packed gather (standalone timing + bit equality); zero fraction 0.5 and 0.3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 200 ./scripts/exp/sparse_gather_bench 2000000 0.5 > gpurun_out/r04_sparse_gather.log 2>&1 &&
timeout -k 10 200 ./scripts/exp/sparse_gather_bench 2000000 0.3 >> gpurun_out/r04_sparse_gather.log 2>&1
