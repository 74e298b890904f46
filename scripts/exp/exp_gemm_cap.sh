# Interleaved repeats: persistent split-f16 GEMM grid (RVX_SAGE_GEMM_CAP blocks per CU) beside the gather, 10M x 768 GraphSAGE.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-hnsw --no-scan > gpurun_out/sw_$label.log 2>&1 || { tail -5 gpurun_out/sw_$label.log; exit 1; }
  echo -n "$label: "; tail -1 gpurun_out/sw_$label.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernel_ms',{})
print(round(d['value']/1e6), 'Medges/s', d['ms_per_step'], 'ms', {n: v for n, v in k.items() if 'gemm' in n or 'agg' in n})"
}
for rep in 1 2 3; do
  run cap0_$rep RVX_SAGE_GEMM_CAP=0
  run cap2_$rep RVX_SAGE_GEMM_CAP=2
done
