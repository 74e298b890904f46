#!/bin/bash
# K5 with four edges' rows loaded together (RVX_EDGE_BATCH=4) vs one at a time (1):
# bits test, then the C4 stack at 2M (edge kernel time per step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ebatch; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "edge_batch_bits or ruvector_layer or edge_attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for b in ${ARMS:-4 1 4 1}; do
  RVX_EDGE_BATCH=$b timeout -k 10 400 python -u bench_gnn.py --nodes ${NODES:-2000000} --steps 2 --warmup 1 --no-cpu > $O/c4_$b.log 2>&1 || exit 6
  python - $O/c4_$b.log $b <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["kernel_ms_per_step"]
        print("batch", sys.argv[2], "ms/step", d["ms_per_step"], "edge", round(k["gnn_edge_attention"], 1), "TB/s", d["roofline"]["gnn_edge_attention"]["achieved"], flush=True)
PY
done
