#!/bin/bash
# SMU clock/power samples while the serial and the overlapped layer pipelines run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in 8 1; do
  RVX_SAGE_CHUNKS=$mode timeout -k 10 200 python3 bench.py --nodes 1000000 --no-cpu --no-hnsw --steps 400 --warmup 2 > gpurun_out/clk_run_$mode.log 2>&1 &
  pid=$!
  sleep 10
  for i in 1 2 3 4 5 6 7 8; do
    amd-smi metric -g 0 -c -p 2>/dev/null | grep -E "SOCKET_POWER|  CLK:" | head -3 >> gpurun_out/smi_$mode.txt
    echo "--" >> gpurun_out/smi_$mode.txt
    sleep 1
  done
  wait $pid || { echo "bench $mode failed"; exit 1; }
done
echo done
