#!/bin/bash
# rocprofv3 kernel-trace/stats of the bench, then separate --pmc passes for
# FETCH_SIZE and WRITE_SIZE (never combined with other trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
BA=${BENCH_ARGS:-}
echo "== kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/gpurun_out/prof" -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu --no-hnsw --no-scan $BA > gpurun_out/prof_bench.log 2>&1 || { echo "trace failed $?"; tail -20 gpurun_out/prof_bench.log; exit 1; }
tail -1 gpurun_out/prof_bench.log
echo "== pmc FETCH_SIZE"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$ROOTDIR/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-hnsw --no-scan $BA > gpurun_out/pmc_fetch.log 2>&1 || { echo "fetch failed $?"; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
echo "== pmc WRITE_SIZE"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$ROOTDIR/gpurun_out/pmc_write" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-hnsw --no-scan $BA > gpurun_out/pmc_write.log 2>&1 || { echo "write failed $?"; tail -20 gpurun_out/pmc_write.log; exit 1; }
python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json gpurun_out/pmc_fetch.log
find gpurun_out/prof -name "*stats*" | head
