#!/bin/bash
# Imaged gather: U (rows in flight) and the LDS expansion's cost (timing-only variants)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/imgvar; mkdir -p $O
for v in ${VARIANTS:-base img_u4 img_noexp base}; do
  lib=ruvector_amd/librvx.so; [ "$v" = base ] || lib=variants/librvx_$v.so
  RVX_LIB=$lib timeout -k 10 300 python -u bench.py --no-scan --no-hnsw --no-c4 --no-cpu > $O/$v.log 2>&1 || exit 1
  python3 - $O/$v.log $v <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"metric"'):
        d = json.loads(ln); k = d["kernel_ms"]
        print(sys.argv[2], d["ms_per_step"], "dense", k.get("sage_aggregate"), "img", k.get("sage_aggregate_img"), "gemm", k.get("sage_gemm"), "pack", k.get("rows_image_pack"))
PY
done
