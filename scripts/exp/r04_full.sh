# Round 4: full GPU suite, smoke, then the default bench line (N=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r04_bench.log 2>&1 &&
timeout -k 10 120 ./scripts/exp/mfma_shape_bench > gpurun_out/r04_mfma_shape.log 2>&1
