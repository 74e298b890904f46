#!/bin/bash
# Round 4 end: full GPU suite, smoke, default bench line, the same bench under rocprofv3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04f_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r04f_bench.log 2>&1 &&
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04f -o run -- python3 -u bench.py > gpurun_out/r04f_prof_bench.log 2>&1
