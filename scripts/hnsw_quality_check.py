#!/usr/bin/env python3
"""Graph-quality check behind the C3 recall numbers: on N(0,1) 768-d data (the
C3 distribution), build the same index on the GPU (batched insert_slice rules)
and with the oracle's CPU hnsw_rs restatement (parallel insert), then compare
recall@10 of both graphs against the exact scan at the same ef. If the two
builds agree, the low C3 recall at 10M is a property of the data + the
reference's parameters (M=32, ef_c=200), not of the GPU builder.

Usage (GPU box): python scripts/hnsw_quality_check.py --n 50000 --d 768
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=50000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--nq", type=int, default=1000)
    p.add_argument("--m", type=int, default=32)
    p.add_argument("--efc", type=int, default=200)
    p.add_argument("--ef", default="100,200,400,800")
    p.add_argument("--threads", type=int, default=16)
    a = p.parse_args()
    import ruvector_amd as rv
    import oracle as O

    n, d, nq, k = a.n, a.d, a.nq, 10
    xb, qb = rv.Buffer(n * d * 4), rv.Buffer(nq * d * 4)
    xb.fill_normal(n * d, 5)
    qb.fill_normal(nq * d, 6)
    x = xb.download(np.float32, (n, d))
    q = qb.download(np.float32, (nq, d))
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=a.m, ef_construction=a.efc, ef_search=100),
                       seed=5)
    t0 = time.perf_counter()
    rv._lib.call("rvx_index_add_batch_device", idx.handle, xb.handle, n, 0)
    rv.synchronize()
    gpu_build = time.perf_counter() - t0
    ids_b, dist_b = rv.Buffer(nq * k * 8), rv.Buffer(nq * k * 4)
    rv._lib.call("rvx_index_brute_force_device", idx.handle, qb.handle, nq, k, ids_b.handle, dist_b.handle)
    gt = ids_b.download(np.uint64, (nq, k)).astype(np.int64)

    h = O.Hnsw(d, "l2", m=a.m, ef_construction=a.efc, seed=5)
    t0 = time.perf_counter()
    h.insert(x, threads=a.threads)
    cpu_build = time.perf_counter() - t0

    def rec(got):
        return float(np.mean([len(set(r.tolist()) & set(g.tolist())) / k for r, g in zip(gt, got)]))

    rows = []
    for ef in [int(e) for e in a.ef.split(",")]:
        r_gpu = rec(idx.search_array(q, k, ef)[0].astype(np.int64))
        r_cpu = rec(h.search(q, k, ef, threads=a.threads)[0])
        rows.append({"ef": ef, "recall_gpu_graph": round(r_gpu, 4), "recall_cpu_graph": round(r_cpu, 4)})
        print(f"ef={ef}: recall@10 GPU-built {r_gpu:.4f}  oracle CPU-built {r_cpu:.4f}", flush=True)
    print(json.dumps({"config": f"{n}x{d} N(0,1) seed 5, {nq} queries seed 6, M={a.m} ef_c={a.efc}, L2, k=10",
                      "gpu_build_s": round(gpu_build, 2), "cpu_build_s": round(cpu_build, 2),
                      "cpu_threads": a.threads, "sweep": rows}))


if __name__ == "__main__":
    main()
