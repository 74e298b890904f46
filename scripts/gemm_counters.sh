#!/bin/bash
# SQ counters of the layer kernels on the serial (1-chunk) 1M x 768 layer:
# issue/wait breakdown, MFMA busy, LDS conflicts (one --pmc pass, no tracing).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
RVX_SAGE_CHUNKS=1 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d "$ROOTDIR/gpurun_out/pmc_sq" -o run --output-format csv -- python3 bench.py --nodes 1000000 --no-cpu --no-hnsw --no-scan --steps 1 --warmup 1 > gpurun_out/pmc_sq.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/pmc_sq.log; exit 1; }
RVX_SAGE_CHUNKS=1 timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA -d "$ROOTDIR/gpurun_out/pmc_sq2" -o run --output-format csv -- python3 bench.py --nodes 1000000 --no-cpu --no-hnsw --no-scan --steps 1 --warmup 1 > gpurun_out/pmc_sq2.log 2>&1 || { echo "sq2 pass failed"; tail -5 gpurun_out/pmc_sq2.log; exit 1; }
RVX_SAGE_CHUNKS=1 timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS -d "$ROOTDIR/gpurun_out/pmc_sq3" -o run --output-format csv -- python3 bench.py --nodes 1000000 --no-cpu --no-hnsw --no-scan --steps 1 --warmup 1 > gpurun_out/pmc_sq3.log 2>&1 || { echo "sq3 pass failed"; tail -5 gpurun_out/pmc_sq3.log; exit 1; }
RVX_SAGE_CHUNKS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOTDIR/gpurun_out/kt_sq" -o run --output-format csv -- python3 bench.py --nodes 1000000 --no-cpu --no-hnsw --no-scan --steps 1 --warmup 1 > gpurun_out/kt_sq.log 2>&1 || { echo "kt failed"; exit 1; }
echo done
