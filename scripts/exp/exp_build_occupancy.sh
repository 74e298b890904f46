#!/bin/bash
# HNSW builder occupancy variants (k_hnsw_build.hip with RVX_BUILD_WPE,
# variants/librvx_bw*.so; same sources, provenance hash matches): build time
# at C1 (100k x 128) and 1M x 768, and the exported graph's checksum (the
# register budget must not change the graph).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bocc
cp ruvector_amd/librvx.so gpurun_out/bocc/librvx_base.so
for v in base ${VARIANTS:-bw3 bw4}; do
  if [ "$v" = base ]; then cp gpurun_out/bocc/librvx_base.so ruvector_amd/librvx.so; else cp variants/librvx_$v.so ruvector_amd/librvx.so; fi
  timeout -k 10 300 python - "$v" <<'PY' || { echo "$v failed"; break; }
import hashlib, sys, time
import numpy as np
sys.path.insert(0, ".")
import ruvector_amd as rv
v = sys.argv[1]
for n, d, data in ((100_000, 128, "uniform"), (1_000_000, 768, "normal")):
    xb = rv.Buffer(n * d * 4)
    if data == "normal":
        xb.fill_normal(n * d, 5)
    else:
        xb.fill_uniform(n * d, 1, -1.0, 1.0)
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=32, ef_construction=200, ef_search=100), seed=5)
    rv.synchronize()
    t0 = time.perf_counter()
    rv._lib.call("rvx_index_add_batch_device", idx.handle, xb.handle, n, 0)
    rv.synchronize()
    dt = time.perf_counter() - t0
    g = idx.export_graph()
    h = hashlib.sha256(g["row_ptr0"].tobytes() + g["col0"].tobytes()).hexdigest()[:16]
    print(v, f"{n}x{d}", f"build {dt:.2f} s", "graph", h, flush=True)
PY
done
cp gpurun_out/bocc/librvx_base.so ruvector_amd/librvx.so
