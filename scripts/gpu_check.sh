#!/bin/bash
# One GPU-box session: smoke, parity tests, bench. Each GPU step has its own
# time limit; a crash/abort/timeout (exit >= 124 or signal) ends the script.
# Plain test failures (exit 1) do not stop the later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_or_stop() {  # $1 = exit code, $2 = step name
  if [ "$1" -ge 2 ]; then echo "STOP after $2 (exit $1)"; exit "$1"; fi
}
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; ok_or_stop $rc smoke
echo "== pytest -m gpu"; timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; ok_or_stop $rc pytest
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  echo "== bench"; timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; tail -3 gpurun_out/bench.log; ok_or_stop $rc bench
fi
echo "== done"
