#!/usr/bin/env python3
"""Recall-vs-N curve of the GPU batched HNSW build against the oracle's CPU
build (hnsw_rs insert rules restated in oracle/oracle.cpp, parallel insert),
on the C3 distribution (N(0,1), 768-d) at the same M / ef_c / ef sweep.

The two sides run on different machines, so each generates the corpus from the
same counter-based stream (k_data.hip k_fill_normal: splitmix64 Box-Muller,
seed 5 for rows, 6 for queries) and computes its own exact ground truth:

  --side cpu   (this container / any host): numpy restatement of the stream
               (f32 libm values may differ from the device's by an ulp; the
               curve is a property of the distribution, not of single values),
               oracle CPU build + oracle exact scan + oracle hnsw search.
  --side gpu   (GPU box): device stream, rvx batched build, rvx exact scan,
               rvx search.

Each side writes one JSON line {"side", "n", "d", "m", "efc", "sweep": [{ef,
recall}]}; scripts/hnsw_recall_compare.py (or DESIGN.md) puts them side by side.
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

_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x):
    x = x + _G
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def fill_normal_host(n, seed, block=1 << 24):
    """k_fill_normal (k_data.hip) on the host, in blocks to bound memory."""
    out = np.empty(n, np.float32)
    with np.errstate(over="ignore"):
        s0 = splitmix64(np.array([seed], np.uint64))[0]
        for b in range(0, n, block):
            i = np.arange(b, min(n, b + block), dtype=np.uint64)
            h1 = splitmix64(s0 + np.uint64(2) * i)
            h2 = splitmix64(s0 + np.uint64(2) * i + np.uint64(1))
            u1 = ((h1 >> np.uint64(40)).astype(np.uint32) + np.uint32(1)).astype(np.float32) * np.float32(2.0 ** -24)
            u2 = (h2 >> np.uint64(40)).astype(np.uint32).astype(np.float32) * np.float32(2.0 ** -24)
            out[b:b + i.size] = np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.283185307179586) * u2)
    return out


def recall(gt, got, k):
    return float(np.mean([len(set(r[:k].tolist()) & set(g[:k].tolist())) / k for r, g in zip(gt, got)]))


def run_cpu(a, efs, log):
    import oracle as O
    n, d, nq, k = a.n, a.d, a.nq, 10
    x = fill_normal_host(n * d, 5).reshape(n, d)
    q = fill_normal_host(nq * d, 6).reshape(nq, d)
    t0 = time.perf_counter()
    gt, _ = O.flat_search(x, q, k, "l2", threads=a.threads)
    log(f"cpu exact gt {time.perf_counter() - t0:.1f}s")
    h = O.Hnsw(d, "l2", m=a.m, ef_construction=a.efc, seed=5)
    t0 = time.perf_counter()
    h.insert(x, threads=a.threads)
    build = time.perf_counter() - t0
    log(f"cpu build {build:.1f}s")
    rows = []
    for ef in efs:
        t0 = time.perf_counter()
        ids = h.search(q, k, ef, threads=a.threads)[0]
        rows.append({"ef": ef, "recall": round(recall(gt, ids, k), 4), "s": round(time.perf_counter() - t0, 2)})
        log(str(rows[-1]))
    return {"build_s": round(build, 1), "threads": a.threads, "sweep": rows}


def run_gpu(a, efs, log):
    import ruvector_amd as rv
    n, d, nq, k = a.n, a.d, a.nq, 10
    xb, qb = rv.Buffer(n * d * 4), rv.Buffer(nq * d * 4)
    xb.fill_normal(n * d, 5)
    qb.fill_normal(nq * d, 6)
    q = qb.download(np.float32, (nq, d))
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=a.m, ef_construction=a.efc, ef_search=100),
                       seed=5)
    t0 = time.perf_counter()
    rv._lib.call("rvx_index_add_batch_device", idx.handle, xb.handle, n, 0)
    rv.synchronize()
    build = time.perf_counter() - t0
    log(f"gpu build {build:.1f}s")
    ids_b, dist_b = rv.Buffer(nq * k * 8), rv.Buffer(nq * k * 4)
    rv._lib.call("rvx_index_brute_force_device", idx.handle, qb.handle, nq, k, ids_b.handle, dist_b.handle)
    gt = ids_b.download(np.uint64, (nq, k)).astype(np.int64)
    rows = []
    for ef in efs:
        t0 = time.perf_counter()
        ids = idx.search_array(q, k, ef)[0].astype(np.int64)
        rows.append({"ef": ef, "recall": round(recall(gt, ids, k), 4), "s": round(time.perf_counter() - t0, 2)})
        log(str(rows[-1]))
    return {"build_s": round(build, 2), "sweep": rows}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--side", choices=("cpu", "gpu"), required=True)
    p.add_argument("--n", type=int, default=200_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--nq", type=int, default=1000)
    p.add_argument("--m", type=int, default=32)
    p.add_argument("--efc", type=int, default=200)
    p.add_argument("--ef", default="100,200,400,800,1600")
    p.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = p.parse_args()
    log = lambda s: print(s, file=sys.stderr, flush=True)  # noqa: E731
    efs = [int(e) for e in a.ef.split(",")]
    res = run_cpu(a, efs, log) if a.side == "cpu" else run_gpu(a, efs, log)
    res.update({"side": a.side, "n": a.n, "d": a.d, "nq": a.nq, "m": a.m, "efc": a.efc,
                "data": "N(0,1) k_fill_normal stream, rows seed 5, queries seed 6; L2, k=10"})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
