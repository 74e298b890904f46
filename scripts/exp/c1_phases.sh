#!/bin/bash
# C1 (100k x 128, M 32, ef_c 200, 10k queries) search phases: the diagnostic build
# (variants/librvx_phases.so, -DRVX_HNSW_PHASES) swapped in for one bench_hnsw.py run at ef 550.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
cp ruvector_amd/librvx.so gpurun_out/librvx_base_c1.so
cp variants/librvx_phases.so ruvector_amd/librvx.so
timeout -k 10 300 python -u bench_hnsw.py --ef 550 > gpurun_out/c1_phases.json 2> gpurun_out/c1_phases.err
rc=$?
cp gpurun_out/librvx_base_c1.so ruvector_amd/librvx.so
grep "hnsw phases" gpurun_out/c1_phases.err | tail -2
exit $rc
