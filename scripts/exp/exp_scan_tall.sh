#!/bin/bash
# K10 tile shapes at 10M x 768 / 10k queries: 256 x 256 8-wave blocks (RVX_SCAN_WIDE=1, one per
# CU) vs 256 rows x 128 queries 4-wave blocks (2, two per CU, 2-stage ring), interleaved,
# after the tile-shape bit tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/scantall; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scan_mfma.py -k "tile_shapes or poincare_filter_matches" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for w in ${ARMS:-1 2 1 2}; do
  RVX_SCAN_WIDE=$w timeout -k 10 200 python bench_scan.py --no-valu --cpu-queries 0 > $O/w$w.json 2>&1 || exit 4
  python3 -c "import json;t=open('$O/w$w.json').read();i=t.rfind('{\"config\"');d=json.loads(t[i:]) if i>=0 else {};m=d.get('mfma',{});print('wide=$w', m.get('qps'), m.get('kernel_ms',{}).get('scan_filter'), m.get('stats'), d.get('oracle_identical'))"
done
