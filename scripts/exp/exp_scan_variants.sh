#!/bin/bash
# K10 filter ablations (build macros, same sources; timings only, results wrong
# by design): ab_epi = epilogue only on each split's last tile; ab_dma = that
# and no k-step DMA (MFMA + LDS reads + barriers on stale stages).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/scanvar; mkdir -p $O
cp ruvector_amd/librvx.so $O/librvx_base.so
for v in ${VARIANTS:-base ab_epi ab_dma}; do
  if [ "$v" = base ]; then cp $O/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_$v.so ruvector_amd/librvx.so; fi
  timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > $O/$v.json 2>&1
  python3 -c "import json;t=open('$O/$v.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};m=d.get('mfma',{});print('$v', m.get('qps'), m.get('kernel_ms',{}).get('scan_filter'), m.get('stats'), d.get('oracle_identical'))" || tail -c 300 $O/$v.json
done
cp $O/librvx_base.so ruvector_amd/librvx.so
