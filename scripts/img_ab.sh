#!/bin/bash
# Row-image gather A/B at 10M x 768 (bench.py sage legs only): dense gather (default) vs the
# image gather with the expansion in registers (RVX_IMG_REG=1) and through LDS (0), interleaved.
# The bit-identity tests first; a failure or fault stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_row_image.py > gpurun_out/img_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/img_tests.log; exit 1; }
tail -1 gpurun_out/img_tests.log
B="python -u bench.py --steps 5 --warmup 2 --no-cpu --no-scan --no-c4 --no-hnsw --no-c3"
for rep in 1 2; do
  for v in dense reg lds; do
    case $v in
      dense) env="RVX_SAGE_IMAGE=0";;
      reg) env="RVX_SAGE_IMAGE=1 RVX_IMG_REG=1";;
      lds) env="RVX_SAGE_IMAGE=1 RVX_IMG_REG=0";;
    esac
    env $env timeout -k 10 300 $B > gpurun_out/img_ab_${v}_${rep}.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/img_ab_${v}_${rep}.log; exit 1; }
    python3 - "$v" "$rep" <<'PY'
import json, sys
line = [l for l in open(f"gpurun_out/img_ab_{sys.argv[1]}_{sys.argv[2]}.log") if l.startswith("{")][-1]
j = json.loads(line)
k = j["kernel_ms"]
print(sys.argv[1], sys.argv[2], "ms/step", j["ms_per_step"], "edges/s %.3fG" % (j["value"] / 1e9),
      "agg", k.get("sage_aggregate"), "agg_img", k.get("sage_aggregate_img"), "gemm", k.get("sage_gemm"),
      "parity", j.get("parity", {}).get("max_rel_err"))
PY
  done
done
