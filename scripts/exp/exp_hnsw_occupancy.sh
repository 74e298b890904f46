#!/bin/bash
# HNSW search occupancy variants (k_hnsw.hip built with RVX_ROW_BATCH /
# RVX_HNSW_WPE, variants/librvx_*.so; same sources, so the provenance hash
# matches): C1 sweep, 1M x 768 (per-lane distances) and 4M x 768 (LDS-staged).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/occ
cp ruvector_amd/librvx.so gpurun_out/occ/librvx_base.so
for v in base ${VARIANTS:-b8w4 b4w4 b4w5 b4w6}; do
  if [ "$v" = base ]; then cp gpurun_out/occ/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_$v.so ruvector_amd/librvx.so; fi
  timeout -k 10 120 python bench_hnsw.py --ef 300,600,800 > gpurun_out/occ/c1_$v.json 2> gpurun_out/occ/c1_$v.err || { echo "c1 $v failed"; break; }
  timeout -k 10 200 python bench_hnsw.py --n 1000000 --dim 768 --data normal --seed 5 --queries 4000 --ef 100,800,1600 > gpurun_out/occ/m1_$v.json 2> gpurun_out/occ/m1_$v.err || { echo "1m $v failed"; break; }
  timeout -k 10 300 python bench_hnsw.py --n 4000000 --dim 768 --data normal --seed 5 --queries 4000 --ef 100,800 > gpurun_out/occ/m4_$v.json 2> gpurun_out/occ/m4_$v.err || { echo "4m $v failed"; break; }
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
for t in ("c1", "m1", "m4"):
    d = json.load(open(f"gpurun_out/occ/{t}_{v}.json"))
    print(v, t, [(r["ef"], r["recall"], round(r["qps"])) for r in d["sweep"]], flush=True)
PY
done
cp gpurun_out/occ/librvx_base.so ruvector_amd/librvx.so
