# Interleaved repeats of the chunk-count / gather-cap candidates (10M x 768 GraphSAGE).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
run() {  # $1 = label, rest = env assignments
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-hnsw --no-scan > gpurun_out/sw_$label.log 2>&1 || { tail -5 gpurun_out/sw_$label.log; exit 1; }
  echo -n "$label: "; tail -1 gpurun_out/sw_$label.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6), 'Medges/s', d['ms_per_step'], 'ms')"
}
for rep in 1 2; do
  run base$rep RVX_SAGE_CHUNKS=16
  run c24_$rep RVX_SAGE_CHUNKS=24
  run c32_$rep RVX_SAGE_CHUNKS=32
  run c24cap1_$rep RVX_SAGE_CHUNKS=24 RVX_AGG_BLOCKS_PER_CU=1
  run c16cap1_$rep RVX_SAGE_CHUNKS=16 RVX_AGG_BLOCKS_PER_CU=1
done
