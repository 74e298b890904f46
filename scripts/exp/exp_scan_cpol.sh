#!/bin/bash
# K10 filter: cache policy of the LDS-DMA loads (rows / queries), interleaved repeats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/scancpol; mkdir -p $O
for v in base nt_rows nt_both sc_rows base nt_rows nt_both; do
  lib=ruvector_amd/librvx.so; [ "$v" = base ] || lib=variants/librvx_$v.so
  RVX_LIB=$lib timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > $O/$v.json 2>&1 || exit 1
  python3 -c "import json;t=open('$O/$v.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};m=d.get('mfma',{});print('$v', m.get('qps'), m.get('kernel_ms',{}).get('scan_filter'), m.get('stats'), d.get('oracle_identical'))"
done
