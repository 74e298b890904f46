#!/bin/bash
# 256x256 split-f16 GEMM (RVX_GEMM_WIDE=1) vs the 128x128 h2g tile: standalone (one chunk)
# GraphSAGE GEMM kernel time, the overlapped 10M x 768 step, and the C4 stack at 2M.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/gwide; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d.get("roofline_kernels") or {}
        print(sys.argv[2], "ms/step", d["ms_per_step"], {n: (v["avg_ms"], v["launches"]) for n, v in k.items()} or d.get("kernel_ms_per_step"), flush=True)
PY
}
for w in ${SA_ARMS:-1 0}; do
  RVX_SAGE_CHUNKS=1 RVX_GEMM_WIDE=$w timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-hnsw --no-scan --no-cpu > $O/sa_$w.log 2>&1 || exit 4
  summ $O/sa_$w.log "standalone wide=$w"
done
for w in ${ARMS:-1 0 1 0}; do
  RVX_GEMM_WIDE=$w timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/pipe_$w.log 2>&1 || exit 5
  summ $O/pipe_$w.log "pipeline wide=$w"
done
for w in ${C4_ARMS:-1 0}; do
  RVX_GEMM_WIDE=$w timeout -k 10 400 python -u bench_gnn.py --nodes 2000000 --steps 2 --warmup 1 --no-cpu > $O/c4_$w.log 2>&1 || exit 6
  summ $O/c4_$w.log "c4-2M wide=$w"
done
