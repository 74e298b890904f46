#!/bin/bash
# K10 filter: full kernel vs the tile epilogue run only on each split's last
# tile (variants/librvx_ablate.so, -DRVX_ABLATE_EPI; results are wrong by
# design, only the time counts): how much of the filter is the k-loop.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ablate
cp ruvector_amd/librvx.so gpurun_out/ablate/librvx_base.so
for v in base ablate base ablate; do
  if [ "$v" = base ]; then cp gpurun_out/ablate/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_ablate.so ruvector_amd/librvx.so; fi
  timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > gpurun_out/ablate/$v.json 2>&1
  python3 -c "import json,re,sys;t=open('gpurun_out/ablate/$v.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};print('$v', d.get('mfma',{}).get('kernel_ms'))" || tail -c 300 gpurun_out/ablate/$v.json
done
cp gpurun_out/ablate/librvx_base.so ruvector_amd/librvx.so
