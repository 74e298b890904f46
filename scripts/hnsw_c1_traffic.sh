#!/bin/bash
# Fabric bytes per C1 HNSW search launch (100k x 128 uniform, M 32, ef_c 200, 10k queries,
# ef 550 = the bench's recall-0.95 operating point): separate rocprofv3 --pmc passes for
# FETCH_SIZE and WRITE_SIZE (gfx950 FETCH correction, scripts/pmc_traffic.py)
# -> gpurun_out/pmc_traffic_hnsw_c1.json. The 51 MB table stays in L2 / Infinity Cache, so
# these are L2-miss bytes (Infinity-Cache hits included), an upper bound on HBM bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd); export TMPDIR=/tmp
O=gpurun_out/hnswpmc; mkdir -p $O
ARGS="--n 100000 --dim 128 --queries 10000 --m 32 --ef-construction 200 --ef 550"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$ROOTDIR/$O/fetch" -o run --output-format csv -- python3 bench_hnsw.py $ARGS > $O/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$ROOTDIR/$O/write" -o run --output-format csv -- python3 bench_hnsw.py $ARGS > $O/write.log 2>&1 || { echo "write failed"; tail -5 $O/write.log; exit 1; }
python3 scripts/pmc_traffic.py $O/fetch $O/write $O/pmc_raw.json
python3 - <<'PY'
import json
raw = json.load(open("gpurun_out/hnswpmc/pmc_raw.json"))
raw["config"] = {"n": 100_000, "d": 128, "nq": 10_000, "m": 32, "efc": 200, "ef": 550, "data": "uniform", "metric": "l2"}
json.dump(raw, open("gpurun_out/pmc_traffic_hnsw_c1.json", "w"), indent=1)
print({k: round(v["hbm_bytes_per_launch"] / 1e9, 3) for k, v in raw["kernels"].items()})
PY
