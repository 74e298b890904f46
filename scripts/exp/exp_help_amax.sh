#!/bin/bash
# Round 3: (1) producer row maxima for the C4 layer GEMMs (RVX_GEMM_AMAX) and (2) the GEMM of
# chunk c helping chunk c+1's gather (RVX_SAGE_HELP). Bit-identity tests first, then A/B on
# the 10M C4 stack and the 10M GraphSAGE bench, alternating arms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ha; mkdir -p $O
stop() { echo "STOP after $1 (exit $2)"; exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "producer_row_maxima or gemm_helps_gather or deferred_normalisation_stack or ruvector_layer_wide or graphsage_wide_gemm" \
  > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ge 1 ] && stop tests $rc
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d.get("roofline_kernels") or d.get("kernel_ms_per_step") or {}
        print(sys.argv[2], "ms/step", d["ms_per_step"], {n: (v.get("avg_ms"), v.get("launches")) if isinstance(v, dict) else v for n, v in k.items()}, flush=True)
PY
}
i=0
for h in ${SAGE_ARMS:-1 0 1 0 1 0}; do
  i=$((i+1))
  RVX_SAGE_HELP=$h timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/sage${i}_$h.log 2>&1 || stop sage $?
  summ $O/sage${i}_$h.log "sage help=$h"
done
i=0
for v in ${C4_ARMS:-1 0}; do
  i=$((i+1))
  RVX_GEMM_AMAX=$v timeout -k 10 300 python -u bench_gnn.py --nodes 10000000 --no-cpu > $O/c4_${i}_$v.log 2>&1 || stop c4 $?
  summ $O/c4_${i}_$v.log "c4 amax=$v"
done
