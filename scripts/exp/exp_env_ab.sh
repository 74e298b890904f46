#!/bin/bash
# Same-box A/B of one environment switch on the 10M pipeline and the serial 1M layer.
# usage: exp_env_ab.sh VAR VALUE_A VALUE_B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
var=$1; va=$2; vb=$3
for i in 1 2; do
  for side in a b; do
    v=$va; [ $side = b ] && v=$vb
    env $var=$v timeout -k 10 300 python bench.py --no-cpu --no-hnsw > gpurun_out/env_${side}$i.json 2> gpurun_out/env_${side}$i.err || exit 1
  done
done
for side in a b; do
  v=$va; [ $side = b ] && v=$vb
  env $var=$v RVX_SAGE_CHUNKS=1 timeout -k 10 200 python bench.py --nodes 1000000 --no-cpu --no-hnsw > gpurun_out/env_s1m_${side}.json 2> gpurun_out/env_s1m_${side}.err || exit 1
done
echo done
