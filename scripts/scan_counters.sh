#!/bin/bash
# SQ counters of the MFMA-filtered exact scan (k_scan_filter) on 2M x 768 rows,
# 10k queries: issue/wait breakdown and MFMA busy (one --pmc pass per group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
O=gpurun_out/scan
mkdir -p $O
ARGS="--n 2000000 --no-valu --cpu-queries 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d "$ROOTDIR/$O/pmc_sq" -o run --output-format csv -- python3 bench_scan.py $ARGS > $O/pmc_sq.log 2>&1 || { echo "sq pass failed"; tail -5 $O/pmc_sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA -d "$ROOTDIR/$O/pmc_sq2" -o run --output-format csv -- python3 bench_scan.py $ARGS > $O/pmc_sq2.log 2>&1 || { echo "sq2 pass failed"; tail -5 $O/pmc_sq2.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS -d "$ROOTDIR/$O/pmc_sq3" -o run --output-format csv -- python3 bench_scan.py $ARGS > $O/pmc_sq3.log 2>&1 || { echo "sq3 pass failed"; tail -5 $O/pmc_sq3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOTDIR/$O/kt_sq" -o run --output-format csv -- python3 bench_scan.py $ARGS > $O/kt_sq.log 2>&1 || { echo "kt failed"; exit 1; }
python3 scripts/sq_summary.py $O k_scan_filter,k_rows_to_f16,k_scan_rerank
