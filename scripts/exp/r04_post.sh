#!/bin/bash
# Round 4: dense/image gather kernels split — tests of the gather paths, two default bench runs,
# then the K10 filter's PMC traffic on the 16x16x32 tile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_row_image.py \
  "tests/test_gpu_parity.py::test_graphsage_gemm_helps_gather_bits" tests/test_gpu_shard_exchange.py > gpurun_out/r04p_pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-scan --no-hnsw --no-c4 --no-cpu > gpurun_out/r04p_bench_a.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-scan --no-hnsw --no-c4 --no-cpu > gpurun_out/r04p_bench_b.log 2>&1 &&
bash scripts/scan_traffic.sh > gpurun_out/r04p_scan_traffic.log 2>&1
