#!/bin/bash
# Cache behaviour of the HNSW search kernel at d=768 (1M x 768 N(0,1), ef 400):
# L1 accesses / L2 requests / L2 hits+misses / HBM read requests per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--n 1000000 --dim 768 --data normal --seed 5 --queries 4000 --ef 400"
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d "$ROOTDIR/gpurun_out/pmc_h1" -o run --output-format csv -- python3 bench_hnsw.py $ARGS > gpurun_out/pmc_h1.log 2>&1 || { echo "h1 failed"; tail -5 gpurun_out/pmc_h1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum -d "$ROOTDIR/gpurun_out/pmc_h2" -o run --output-format csv -- python3 bench_hnsw.py $ARGS > gpurun_out/pmc_h2.log 2>&1 || { echo "h2 failed"; tail -5 gpurun_out/pmc_h2.log; exit 1; }
echo done
