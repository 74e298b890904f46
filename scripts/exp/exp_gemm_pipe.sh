#!/bin/bash
# Software-pipelined 256x192 split-f16 GEMM (RVX_GEMM_WIDE=5) vs the standalone default
# (2: 256x256) and the 256x192 tile (3): bits (wide-GEMM parity tests), the standalone
# 10M x 768 GraphSAGE GEMM (one chunk) and the C4 stack at 2M. variants/librvx_ring6.so:
# the same kernel with a 6-slot B fragment ring (H2W_RING=6; default 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/gpipe; mkdir -p $O
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d.get("roofline_kernels") or {}
        km = d.get("kernel_ms_per_step") or {}
        g = {a: round(v, 1) for a, v in km.items() if "gemm" in a}
        print(sys.argv[2], "ms/step", d["ms_per_step"], {n: (v["avg_ms"], v["launches"]) for n, v in k.items()} or (round(sum(g.values()), 1), g), flush=True)
PY
}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "wide_gemm_bits" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for arm in ${SA_ARMS:-2 5 5r6 3 2 5}; do
  w=${arm%r6}; lib=""; [ "$arm" != "$w" ] && lib=variants/librvx_ring6.so
  RVX_LIB=$lib RVX_SAGE_CHUNKS=1 RVX_GEMM_WIDE=$w timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-hnsw --no-scan --no-cpu > $O/sa_$arm.log 2>&1 || exit 4
  summ $O/sa_$arm.log "standalone wide=$arm"
done
for arm in ${C4_ARMS:-2 5 2 5}; do
  RVX_GEMM_WIDE=$arm timeout -k 10 400 python -u bench_gnn.py --nodes 2000000 --steps 2 --warmup 1 --no-cpu > $O/c4_$arm.log 2>&1 || exit 6
  summ $O/c4_$arm.log "c4-2M wide=$arm"
done
