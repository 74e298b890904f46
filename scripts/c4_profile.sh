#!/bin/bash
# rocprofv3 kernel trace + stats of the C4 stack (RuvectorLayer x3 + attention head) at 10M x 768.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/gpurun_out/prof_c4" -o run --output-format csv -- python3 bench_gnn.py --nodes 10000000 --no-cpu > gpurun_out/prof_c4_bench.log 2>&1 || { echo "trace failed $?"; tail -20 gpurun_out/prof_c4_bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_c4_bench.log
find gpurun_out/prof_c4 -name "*kernel_stats*"
