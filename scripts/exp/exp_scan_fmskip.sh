#!/bin/bash
# K10 filter: static s_setprio 1 for waves NW/2.. (variants/librvx_fmskip.so) vs default, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/scanfmskip; mkdir -p $O
for v in base fmskip base fmskip base fmskip; do
  lib=ruvector_amd/librvx.so; [ "$v" = base ] || lib=variants/librvx_$v.so
  RVX_LIB=$lib timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > $O/$v.json 2>&1 || exit 1
  python3 -c "import json;t=open('$O/$v.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};m=d.get('mfma',{});print('$v', m.get('qps'), m.get('kernel_ms',{}).get('scan_filter'), m.get('stats'), d.get('oracle_identical'))"
done
