#!/bin/bash
# Address-translation behaviour of the HNSW search at d=768 as the table grows
# (1M vs 4M rows, ef 400): UTCL1 requests / hits / misses per search launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in ${TLB_SIZES:-1000000 4000000}; do
  timeout -k 10 400 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum -d "$ROOTDIR/gpurun_out/pmc_tlb_$n" -o run --output-format csv -- python3 bench_hnsw.py --n $n --dim 768 --data normal --seed 5 --queries 4000 --ef 400 > gpurun_out/pmc_tlb_$n.log 2>&1 || { echo "tlb $n failed"; tail -5 gpurun_out/pmc_tlb_$n.log; exit 1; }
done
echo done
