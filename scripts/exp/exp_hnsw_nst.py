#!/usr/bin/env python3
"""A/B of the LDS-staged search's kernel settings (distance stages RVX_HNSW_NST, HBM-resident R
RVX_HNSW_RG and its stages RVX_HNSW_RG_NST) on one C3-shaped
graph: 10M x 768 N(0,1), HNSW M 32 ef_c 200 built once on the GPU, then each (ef, NST)
searched twice (the second timed); ids must match across NST (bit-identical search)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ruvector_amd as rv  # noqa: E402

n, d = int(os.environ.get("N", 10_000_000)), int(os.environ.get("D", 768))
efs = [int(e) for e in os.environ.get("EFS", "100,800,3200,8192,12288,16384").split(",")]
# ";"-separated environment settings, each "VAR=VAL,VAR=VAL" (empty: the defaults)
configs = os.environ.get("CONFIGS", ";RVX_HNSW_NST=2;RVX_HNSW_RG=1;RVX_HNSW_RG=1,RVX_HNSW_RG_NST=2").split(";")
KNOBS = ("RVX_HNSW_NST", "RVX_HNSW_RG", "RVX_HNSW_RG_NST", "RVX_HNSW_QG", "RVX_HNSW_RG_WAVES")
log = lambda s: print(s, file=sys.stderr, flush=True)  # noqa: E731
xb = rv.Buffer(n * d * 4)
xb.fill_normal(n * d, 5)
idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=32, ef_construction=200, ef_search=100), seed=5)
t0 = time.perf_counter()
rv._lib.call("rvx_index_add_batch_device", idx.handle, xb.handle, n, 0)
rv.synchronize()
log(f"build {time.perf_counter() - t0:.1f} s")
out = []
for ef in efs:
    nq = int(os.environ.get("NQ", 0)) or (4096 if ef <= 1000 else 1024)
    qb = rv.Buffer(nq * d * 4)
    qb.fill_normal(nq * d, 6)
    ids_b, dist_b = rv.Buffer(nq * 10 * 8), rv.Buffer(nq * 10 * 4)
    ref = None
    for cfg in configs:
        for kk in KNOBS:
            os.environ.pop(kk, None)
        for kv in filter(None, cfg.split(",")):
            kk, vv = kv.split("=")
            os.environ[kk] = vv
        rv._lib.call("rvx_index_search_device", idx.handle, qb.handle, nq, 10, ef, ids_b.handle, dist_b.handle)
        rv.synchronize()
        t0 = time.perf_counter()
        rv._lib.call("rvx_index_search_device", idx.handle, qb.handle, nq, 10, ef, ids_b.handle, dist_b.handle)
        rv.synchronize()
        dt = time.perf_counter() - t0
        got = ids_b.download(np.uint64, (nq, 10))
        same = True if ref is None else bool(np.array_equal(ref, got))
        ref = got if ref is None else ref
        st = rv.hnsw_last_search_stats()
        out.append({"ef": ef, "config": cfg, "qps": round(nq / dt, 1), "same_ids": same, "slots": st.get("slots")})
        log(f"ef {ef} [{cfg}]: {nq / dt:.0f} QPS same={same}")
print(json.dumps(out))
