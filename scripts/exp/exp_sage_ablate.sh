#!/bin/bash
# GraphSAGE 10M x 768 step time without the normalise pass / without the aggregate store
# (variants/ built by scripts/build_sage_variants.sh; timings only, results wrong by design).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sageab; mkdir -p $O
cp ruvector_amd/librvx.so $O/librvx_base.so
for v in ${VARIANTS:-base nonorm noaggw both base}; do
  if [ "$v" = base ]; then cp $O/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_$v.so ruvector_amd/librvx.so; fi
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-hnsw --no-scan --no-cpu > $O/$v.log 2>&1 || { cp $O/librvx_base.so ruvector_amd/librvx.so; exit 4; }
  python - $O/$v.log $v <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        k = d["roofline_kernels"]
        print(sys.argv[2], "ms/step", d["ms_per_step"], {n: (v["avg_ms"], v["launches"]) for n, v in k.items()}, flush=True)
PY
done
cp $O/librvx_base.so ruvector_amd/librvx.so
