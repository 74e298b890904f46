#!/bin/bash
# Round 4: bench with / without row images (per-layer gather tags)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in 1 0; do
  RVX_SAGE_IMAGE=$v timeout -k 10 300 python -u bench.py --no-scan --no-hnsw --no-c4 > gpurun_out/r04_image2_bench_$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import json, sys
for ln in open(f"gpurun_out/r04_image2_bench_{sys.argv[1]}.log"):
    if ln.startswith('{"metric"'):
        d = json.loads(ln)
        print("image", sys.argv[1], d["value"], d["ms_per_step"], d["kernel_ms"])
        for k, v in d["roofline_kernels"].items():
            print("   ", k, v.get("achieved"), v.get("avg_ms"), v.get("launches"))
PY
done
