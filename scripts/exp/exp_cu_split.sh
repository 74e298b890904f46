#!/bin/bash
# GraphSAGE pipeline with the GEMM and the gather on disjoint CU halves
# (RVX_SAGE_CU_SPLIT 1/2, two mask patterns) vs shared CUs, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cus
for rep in 1 2; do
  for v in 0 1 2; do
    for cap in 2 3; do
      [ "$v" = 0 ] && [ "$cap" = 3 ] && continue
      RVX_SAGE_CU_SPLIT=$v RVX_AGG_BLOCKS_PER_CU=$([ "$v" = 0 ] && echo 1 || echo $cap) RVX_SAGE_GEMM_CAP=$([ "$v" = 0 ] && echo 2 || echo $cap) \
        timeout -k 10 200 python bench.py --no-cpu --no-hnsw --no-scan > gpurun_out/cus/s${v}c${cap}_$rep.json 2> gpurun_out/cus/s${v}c${cap}_$rep.err || { echo "s$v failed"; tail -3 gpurun_out/cus/s${v}c${cap}_$rep.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/cus/s${v}c${cap}_$rep.json')); print('split=$v cap=$cap rep=$rep', round(d['value']/1e9,4), d['kernel_ms'], d['parity']['max_rel_err'] if 'parity' in d else '')"
    done
  done
done
