#!/bin/bash
# Unpipelined layer (one chunk): GEMM kernel time of the fused full-width GraphSAGE GEMM vs
# gemm_nt_h2 (+ normalize_rows), 10M x 768.
mkdir -p gpurun_out
for f in 1 0; do
  RVX_SAGE_CHUNKS=1 RVX_SAGE_FUSED=$f timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-hnsw --no-scan --no-cpu > gpurun_out/sagef_sa_$f.log 2>&1 || exit 4
  python - gpurun_out/sagef_sa_$f.log $f <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["roofline_kernels"]
        print("fused=" + sys.argv[2], "ms/step", d["ms_per_step"], {n: (v["avg_ms"], v["launches"]) for n, v in k.items()})
PY
done
