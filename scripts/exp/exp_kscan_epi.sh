#!/bin/bash
# K10 filter at 10M x 768 / 10k queries: batched row-constant reads in the tile epilogue
# (current) vs the previous build (variants/librvx_kscan_old.so), interleaved; RVX_ALLOW_STALE
# lets the variant library load (its k_scan object is older than the sources).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/kscanepi; mkdir -p $O
cp ruvector_amd/librvx.so $O/librvx_new.so
for v in ${ARMS:-new old new old}; do
  cp $O/librvx_$v.so ruvector_amd/librvx.so 2>/dev/null || cp variants/librvx_kscan_old.so ruvector_amd/librvx.so
  RVX_ALLOW_STALE=1 timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > $O/$v.json 2>&1 || { cp $O/librvx_new.so ruvector_amd/librvx.so; exit 4; }
  python3 -c "import json;t=open('$O/$v.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};m=d.get('mfma',{});print('$v', m.get('qps'), m.get('kernel_ms',{}).get('scan_filter'), m.get('stats'), d.get('oracle_identical'))"
done
cp $O/librvx_new.so ruvector_amd/librvx.so
