#!/bin/bash
# LDS-staged HNSW distances with one stage per wave (more waves per CU, no
# in-wave DMA overlap; variants/librvx_wd1.so) vs two, on C3 10M x 768.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wd
cp ruvector_amd/librvx.so gpurun_out/wd/librvx_base.so
for v in base wd1; do
  if [ "$v" = base ]; then cp gpurun_out/wd/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_$v.so ruvector_amd/librvx.so; fi
  timeout -k 10 500 python bench_c3.py --ef 100,800,3200 --no-cpu --check 0 > gpurun_out/wd/c3_$v.json 2> gpurun_out/wd/c3_$v.err || { echo "$v failed"; break; }
  grep -E "build|ef=" gpurun_out/wd/c3_$v.err | sed "s/^/$v /"
done
cp gpurun_out/wd/librvx_base.so ruvector_amd/librvx.so
