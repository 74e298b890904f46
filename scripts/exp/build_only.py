#!/usr/bin/env python3
"""GPU HNSW build of N x 768 N(0,1) (M / ef_c from the environment) and nothing else: for
rocprofv3 kernel stats of the build's phases."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ruvector_amd as rv  # noqa: E402

n, d = int(os.environ.get("N", 4_000_000)), 768
m, efc = int(os.environ.get("M", 32)), int(os.environ.get("EFC", 200))
xb = rv.Buffer(n * d * 4)
xb.fill_normal(n * d, 5)
idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=m, ef_construction=efc, ef_search=100), seed=5)
rv.synchronize()
t0 = time.perf_counter()
rv._lib.call("rvx_index_add_batch_device", idx.handle, xb.handle, n, 0)
rv.synchronize()
print(f"N {n} M {m} ef_c {efc}: build {time.perf_counter() - t0:.1f} s", flush=True)
