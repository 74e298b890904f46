#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_row_image.py > gpurun_out/r04_img3_pytest.log 2>&1 &&
VARIANTS="base img_noscan img_nowrite img_noexp base" bash scripts/exp/exp_img_variants.sh > gpurun_out/r04_img3_var.log 2>&1 &&
RVX_SAGE_IMAGE=0 timeout -k 10 300 python -u bench.py --no-scan --no-hnsw --no-c4 --no-cpu > gpurun_out/r04_img3_off.log 2>&1
