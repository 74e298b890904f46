#!/bin/bash
# A/B of the fused full-width GraphSAGE GEMM (RVX_SAGE_FUSED) on the 10M x 768 bench layer,
# interleaved; GraphSAGE parity tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "graphsage or sage" > gpurun_out/sagef_tests.log 2>&1
rc=$?
tail -3 gpurun_out/sagef_tests.log
if [ $rc -gt 1 ] || grep -qiE "illegal memory|memory access fault" gpurun_out/sagef_tests.log; then exit 3; fi
for i in 1 2; do
  for f in 1 0; do
    RVX_SAGE_FUSED=$f timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-hnsw --no-scan --no-cpu > gpurun_out/sagef_b${f}_$i.log 2>&1 || exit 4
    echo "fused=$f run $i: $(grep -o '"value": [0-9.e+]*' gpurun_out/sagef_b${f}_$i.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sagef_b${f}_$i.log | head -1)"
  done
done
