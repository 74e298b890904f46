#!/bin/bash
# SQ counters of the split-f16 GraphSAGE GEMM variants on the 1-chunk 1M x 768 layer:
# h2g (128x128), h2w (256x256, RVX_GEMM_WIDE=1), h2w8 (8 x 1 waves, 2), h2w5 (256x192
# software-pipelined, 5), h2p (pre-split A, RVX_GEMM_H2P=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-h2w h2g h2p}; do
  case $v in
    h2w) export RVX_GEMM_WIDE=1 RVX_GEMM_H2P=0 ;;
    h2w8) export RVX_GEMM_WIDE=2 RVX_GEMM_H2P=0 ;;
    h2w5) export RVX_GEMM_WIDE=5 RVX_GEMM_H2P=0 ;;
    h2g) export RVX_GEMM_WIDE=0 RVX_GEMM_H2P=0 ;;
    h2p) export RVX_GEMM_WIDE=0 RVX_GEMM_H2P=1 ;;
  esac
  bash scripts/gemm_counters.sh > gpurun_out/sq_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/sq_$v.log; exit 1; }
  rm -rf gpurun_out/sq_$v; mkdir -p gpurun_out/sq_$v
  mv gpurun_out/pmc_sq gpurun_out/pmc_sq2 gpurun_out/pmc_sq3 gpurun_out/kt_sq gpurun_out/sq_$v/
  python3 scripts/sq_summary.py gpurun_out/sq_$v gemm_nt_${v:0:3},k_aggregate_vec
done
