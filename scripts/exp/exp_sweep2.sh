# Pipeline knobs after the split-f16 GEMM change (10M x 768 GraphSAGE, 5 timed steps each).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
run() {  # $1 = label, rest = env assignments
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-hnsw --no-scan > gpurun_out/sw_$label.log 2>&1 || { tail -5 gpurun_out/sw_$label.log; exit 1; }
  echo -n "$label: "; tail -1 gpurun_out/sw_$label.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6), 'Medges/s', d['ms_per_step'], 'ms', d['kernel_ms'])"
}
run base RVX_AGG_UNROLL=8
run cap1 RVX_AGG_BLOCKS_PER_CU=1
run cap2 RVX_AGG_BLOCKS_PER_CU=2
run c8 RVX_SAGE_CHUNKS=8
run c24 RVX_SAGE_CHUNKS=24
run u6 RVX_AGG_UNROLL=6
run base2 RVX_AGG_UNROLL=8
