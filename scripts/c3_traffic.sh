#!/bin/bash
# C3 leg (bench_c3.py: 10M x 768 HNSW M 32 / ef_c 200, ef sweep 100/400/1600, NeuralSearch) under
# rocprofv3: kernel trace + stats, then one --pmc pass for FETCH_SIZE and one for WRITE_SIZE
# (separate runs), reduced per ef by scripts/pmc_traffic.py --c3. A failure stops the script.
# C3_EFS overrides the ef list (the bench leg's 100,400,1600; 8192 and 12288 run R in HBM).
# C3_ARGS adds bench_c3.py options (e.g. "--n 2000000 --m 128 --efc 500") and C3_OUT names the
# reduced JSON (default gpurun_out/pmc_traffic_c3.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # $1 tag, rest: rocprofv3 options
  local tag=$1; shift
  rm -rf "gpurun_out/c3_$tag"
  timeout -k 10 540 rocprofv3 "$@" -d "$ROOTDIR/gpurun_out/c3_$tag" -o run --output-format csv -- \
      python3 -u bench_c3.py --ef "${C3_EFS:-100,400,1600}" --no-cpu --check 0 ${C3_ARGS:-} > "gpurun_out/c3_${tag}.json" 2> "gpurun_out/c3_${tag}.log"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "c3 $tag failed rc=$rc"; tail -5 "gpurun_out/c3_${tag}.log"; exit 1; fi
  echo "c3 $tag ok"
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
python3 scripts/pmc_traffic.py --c3 gpurun_out/c3_fetch gpurun_out/c3_write "${C3_OUT:-gpurun_out/pmc_traffic_c3.json}" \
    gpurun_out/c3_trace.json
find gpurun_out/c3_trace -name "*kernel_stats*" -exec cp {} gpurun_out/r05_c3_kernel_stats.csv \;
rm -rf gpurun_out/c3_fetch gpurun_out/c3_write
