#!/bin/bash
# HBM bytes per K10 filter launch (10M x 768, 10k queries, k 10, L2): separate
# rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE, gfx950 FETCH correction
# (scripts/pmc_traffic.py) -> gpurun_out/pmc_traffic_scan.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd); export TMPDIR=/tmp
O=gpurun_out/scanpmc; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$ROOTDIR/$O/fetch" -o run --output-format csv -- python3 bench_scan.py --no-valu --cpu-queries 0 > $O/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$ROOTDIR/$O/write" -o run --output-format csv -- python3 bench_scan.py --no-valu --cpu-queries 0 > $O/write.log 2>&1 || { echo "write failed"; tail -5 $O/write.log; exit 1; }
python3 scripts/pmc_traffic.py $O/fetch $O/write $O/pmc_raw.json
python3 - <<'PY'
import json
raw = json.load(open("gpurun_out/scanpmc/pmc_raw.json"))
t = open("gpurun_out/scanpmc/fetch.log").read()
res = json.JSONDecoder().raw_decode(t[t.rfind('{"config"'):])[0]
launches = res["mfma"]["kernel_ms"]["launches"].get("scan_filter")
raw["config"] = {"workload": res["config"], "n": 10_000_000, "d": 768, "nq": 10_000, "k": 10, "metric": "l2",
                 "launches": launches}
json.dump(raw, open("gpurun_out/pmc_traffic_scan.json", "w"), indent=1)
print({k: round(v["hbm_bytes_per_launch"] / 1e9, 3) for k, v in raw["kernels"].items()})
PY
