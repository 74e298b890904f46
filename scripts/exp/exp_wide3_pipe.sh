#!/bin/bash
# 256 x 192 split-f16 tile (RVX_GEMM_WIDE=3, 161 VGPRs: co-resident with a gather wave) in the
# overlapped 10M x 768 GraphSAGE step vs h2g (0), alternating; then the standalone GEMM.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wide3; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d.get("roofline_kernels") or {}
        print(sys.argv[2], "ms/step", d["ms_per_step"], {n: (v["avg_ms"], v["launches"]) for n, v in k.items()}, flush=True)
PY
}
i=0
for w in ${ARMS:-3 0 3 0 3 0}; do
  i=$((i+1))
  RVX_GEMM_WIDE=$w timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/p${i}_$w.log 2>&1 || exit 4
  summ $O/p${i}_$w.log "pipeline wide=$w"
done
for w in 3 2 0; do
  RVX_SAGE_CHUNKS=1 RVX_GEMM_WIDE=$w timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-hnsw --no-scan --no-cpu > $O/sa_$w.log 2>&1 || exit 5
  summ $O/sa_$w.log "standalone wide=$w"
done
