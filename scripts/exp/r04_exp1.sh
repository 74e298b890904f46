#!/bin/bash
# round-4 experiments: ReLU-sparse gather (standalone) then K10 ablations on both MFMA shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
bash scripts/exp/exp_sparse_gather.sh && bash scripts/exp/exp_scan_ablate_m16.sh > gpurun_out/r04_scanab16.log 2>&1
