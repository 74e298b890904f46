# Pre-split split-f16 GEMM tile/ring configurations (RVX_GEMM_H2P_CFG) vs the in-GEMM split (h2g),
# standalone (1 chunk) and in the 24-chunk pipeline, 10M x 768 GraphSAGE.
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
for c in 0 1 2 3; do run c1_cfg$c RVX_GEMM_H2P_CFG=$c RVX_SAGE_CHUNKS=1; done
for rep in 1 2; do
  run h2g_$rep RVX_GEMM_H2P=0
  for c in 0 1 3; do run cfg${c}_$rep RVX_GEMM_H2P_CFG=$c; done
done
