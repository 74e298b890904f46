#!/bin/bash
# Round 4: row-image tests, then the bench with and without images (interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_row_image.py \
  "tests/test_gpu_parity.py::test_graphsage_gemm_helps_gather_bits" > gpurun_out/r04_image_pytest.log 2>&1 &&
for v in 1 0 1 0; do
  RVX_SAGE_IMAGE=$v timeout -k 10 300 python -u bench.py --no-scan --no-hnsw --no-c4 > gpurun_out/r04_image_bench_$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import json, sys
for ln in open(f"gpurun_out/r04_image_bench_{sys.argv[1]}.log"):
    if ln.startswith('{"metric"'):
        d = json.loads(ln)
        print("image", sys.argv[1], d["value"], d["ms_per_step"], d["kernel_ms"], d["config"].get("row_image"), d.get("parity", {}).get("ok"))
PY
done
