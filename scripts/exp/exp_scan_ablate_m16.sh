#!/bin/bash
# K10 filter ablations on both MFMA shapes (timings only; ab_* results are wrong by design):
# base, ab_epi (epilogue only on each split's last tile), ab_dma (that and no k-step DMA).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/scanab16; mkdir -p $O
for v in base ab_epi ab_dma; do
  for m in 1 0; do
    lib=ruvector_amd/librvx.so; [ "$v" = base ] || lib=variants/librvx_$v.so
    RVX_LIB=$lib RVX_SCAN_M16=$m timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > $O/${v}_m$m.json 2>&1 || exit 1
    python3 -c "import json;t=open('$O/${v}_m$m.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};m=d.get('mfma',{});print('$v m16=$m', m.get('qps'), m.get('kernel_ms',{}).get('scan_filter'), m.get('stats'))"
  done
done
