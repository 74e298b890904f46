#!/bin/bash
# C4 leg (bench_gnn.py, 10M x 768, 3 x RuvectorLayer + attention head) under rocprofv3:
# kernel trace + stats, then one --pmc pass for FETCH_SIZE and one for WRITE_SIZE (separate
# runs, MI355X_MICROARCH.md HBM section), reduced by scripts/pmc_traffic.py --c4 into
# profiles-ready JSON. Each GPU step has its own time limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
N=${C4_NODES:-10000000}
mkdir -p gpurun_out
run() {  # $1 tag, rest: rocprofv3 options
  local tag=$1; shift
  rm -rf "gpurun_out/c4_$tag"
  timeout -k 10 420 rocprofv3 "$@" -d "$ROOTDIR/gpurun_out/c4_$tag" -o run --output-format csv -- \
      python3 bench_gnn.py --nodes "$N" --no-cpu > "gpurun_out/c4_${tag}.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "c4 $tag failed rc=$rc"; tail -5 "gpurun_out/c4_${tag}.log"; exit 1; fi
  echo "c4 $tag ok: $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/c4_${tag}.log")"
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
python3 scripts/pmc_traffic.py --c4 gpurun_out/c4_fetch gpurun_out/c4_write gpurun_out/pmc_traffic_c4.json \
    gpurun_out/c4_fetch.log
find gpurun_out/c4_trace -name "*kernel_stats*" -exec cp {} gpurun_out/r05_c4_kernel_stats.csv \;
