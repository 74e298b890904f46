#!/bin/bash
# HNSW with M = 96 / 128 (layer-0 lists of 192 / 256): 100k x 768 recall curves (GPU side of
# scripts/hnsw_recall_curve.py, against the oracle's CPU build of the same corpus) and the
# 1M x 768 C3-distribution sweep (bench_hnsw.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hnswm; mkdir -p $O
set -o pipefail
for cfg in "96 600" "128 800"; do
  set -- $cfg
  timeout -k 10 200 python -u scripts/hnsw_recall_curve.py --side gpu --n 100000 --m $1 --efc $2 --ef 100,200,400,800,1600 > $O/curve_100k_m$1.json 2> $O/curve_100k_m$1.log || exit 4
done
for cfg in "96 600" "128 800"; do
  set -- $cfg
  timeout -k 10 500 python -u bench_hnsw.py --n 1000000 --dim 768 --queries 2000 --m $1 --ef-construction $2 --ef 400,800,1600,3200 --data normal > $O/c3_1m_m$1.log 2>&1 || exit 5
  tail -c 1500 $O/c3_1m_m$1.log
done
