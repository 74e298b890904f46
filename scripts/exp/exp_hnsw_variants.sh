#!/bin/bash
# Same-box A/B of compile-time variants of the HNSW search (variants/librvx_<name>.so from
# scripts/exp/build_variant.sh) on one C3-shaped graph per run (scripts/exp/exp_hnsw_nst.py).
# usage: exp_hnsw_variants.sh name1 name2 ...   ("base" = the shipped build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/hv
cp ruvector_amd/librvx.so gpurun_out/hv/librvx_base.so
for v in "$@"; do
  if [ "$v" = base ]; then cp gpurun_out/hv/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_$v.so ruvector_amd/librvx.so; fi
  CONFIGS="" timeout -k 10 400 python -u scripts/exp/exp_hnsw_nst.py > gpurun_out/hv/$v.json 2> gpurun_out/hv/$v.err || { echo "$v failed"; break; }
  grep -E "build|ef " gpurun_out/hv/$v.err | sed "s/^/$v /"
done
cp gpurun_out/hv/librvx_base.so ruvector_amd/librvx.so
