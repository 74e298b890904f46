# Round 4: K10 16x16x32 variant — bit-exactness tests then the interleaved 10M x 768 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scan_mfma.py > gpurun_out/r04_scan_m16_pytest.log 2>&1 &&
timeout -k 10 400 python -u scripts/exp/exp_scan_m16.py > gpurun_out/r04_scan_m16_ab.log 2>&1 &&
timeout -k 10 120 ./scripts/exp/mfma_shape_bench > gpurun_out/r04_mfma_shape.log 2>&1
