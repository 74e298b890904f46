#!/bin/bash
# Occupancy of the HBM-R search with the LDS admission buffer (k_hnsw.hip RG): two distance stages
# (default) vs one (RVX_HNSW_RG_NST=1, 8 KB less LDS per wave) on the default build (170 VGPRs,
# 2 waves/SIMD) and on builds held to 3 waves/SIMD (variants/librvx_rgw3*.so, -DRVX_RG_WPE; c192:
# a 192-entry buffer). One GPU-built graph per arm (1M x 768, M 128, ef_c 500), ef 8192 / 12288.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/rgocc; mkdir -p $O
A="--n ${N:-1000000} --m 128 --efc 500 --ef 8192,12288 --queries ${Q:-2048} --reps 2 --forms 1"
timeout -k 10 400 python scripts/exp/rg_buf_ab.py $A > $O/default_nst2.log 2>&1 || exit 3
RVX_HNSW_RG_NST=1 timeout -k 10 400 python scripts/exp/rg_buf_ab.py $A > $O/default_nst1.log 2>&1 || exit 4
RVX_LIB=variants/librvx_rgw3.so RVX_HNSW_RG_NST=1 timeout -k 10 400 python scripts/exp/rg_buf_ab.py $A > $O/w3_nst1.log 2>&1 || exit 5
RVX_LIB=variants/librvx_rgw3c192.so RVX_HNSW_RG_NST=1 timeout -k 10 400 python scripts/exp/rg_buf_ab.py $A > $O/w3c192_nst1.log 2>&1 || exit 6
RVX_LIB=variants/librvx_rgw3.so timeout -k 10 400 python scripts/exp/rg_buf_ab.py $A > $O/w3_nst2.log 2>&1 || exit 7
for f in $O/*.log; do echo "== $f"; grep '^{"ef"' $f; done
