#!/bin/bash
# Overlapped gather issued at raised wave priority (RVX_AGG_PRIO builds,
# variants/librvx_p*.so) vs default, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prio
cp ruvector_amd/librvx.so gpurun_out/prio/librvx_base.so
for rep in 1 2; do
  for v in base p1 p3; do
    if [ "$v" = base ]; then cp gpurun_out/prio/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_$v.so ruvector_amd/librvx.so; fi
    timeout -k 10 200 python bench.py --no-cpu --no-hnsw --no-scan > gpurun_out/prio/${v}_$rep.json 2> gpurun_out/prio/${v}_$rep.err || { echo "$v failed"; break 2; }
    python3 -c "import json; d=json.load(open('gpurun_out/prio/${v}_$rep.json')); print('${v}_$rep', round(d['value']/1e9,4), d['kernel_ms'])"
  done
done
cp gpurun_out/prio/librvx_base.so ruvector_amd/librvx.so
