#!/bin/bash
# Same-box A/B of two library builds on the 10M pipeline (interleaved runs).
# usage: exp_ab.sh <extra bench args...>; B side = ruvector_amd/librvx_ab.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for side in a b; do
    lib=ruvector_amd/librvx.so; [ $side = b ] && lib=ruvector_amd/librvx_ab.so
    RVX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-hnsw "$@" > gpurun_out/ab_${side}$i.json 2> gpurun_out/ab_${side}$i.err || exit 1
  done
done
echo done
