#!/bin/bash
# K10 list insertion A/B at the bench_scan default (10M x 768, 10k queries, k 10):
# RVX_SCAN_GROUP 1 (16-lane group insertion) vs 0 (one lane per query), wide and narrow tiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/scangroup; mkdir -p $O
for w in 1 0; do for g in 1 0; do
  RVX_SCAN_WIDE=$w RVX_SCAN_GROUP=$g timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > $O/w${w}_g$g.json 2>&1 || exit 4
  python3 -c "import json;t=open('$O/w${w}_g$g.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};m=d.get('mfma',{});print('wide $w group $g', m.get('qps'), m.get('kernel_ms',{}).get('scan_filter'), m.get('stats'), d.get('oracle_identical'))"
done; done
