# Gather knobs inside the 10M x 768 GraphSAGE pipeline (split-f16 GEMM).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
run() {  # $1 = label, rest = env assignments
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-hnsw > gpurun_out/bench_$label.log 2>&1 || { tail -5 gpurun_out/bench_$label.log; exit 1; }
  echo -n "$label: "; tail -1 gpurun_out/bench_$label.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6), 'Medges/s', d['ms_per_step'], 'ms', d['kernel_ms'], d['roofline_layer']['layer_ms'])"
}
run u4nt0 RVX_AGG_UNROLL=4 RVX_AGG_NT=0
run u4nt1 RVX_AGG_UNROLL=4 RVX_AGG_NT=1
run u8nt0 RVX_AGG_UNROLL=8 RVX_AGG_NT=0
run u8nt1 RVX_AGG_UNROLL=8 RVX_AGG_NT=1
run u4nt0_c32 RVX_AGG_UNROLL=4 RVX_AGG_NT=0 RVX_SAGE_CHUNKS=32
