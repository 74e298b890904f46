#!/usr/bin/env python3
"""C3: 10M x 768 HNSW build + k=10 search + GNN re-rank on 1 GPU.

X 10,000,000 x 768 N(0,1) (seed 5, 30.7 GB resident in HBM), queries 10,000 N(0,1)
(seed 6); HNSW M=32, ef_c=200, L2, built on the GPU (hnsw_rs insert rules, batched).
Ground truth: the exact scan (distances in the reference's order, ties by id).
ef is swept; the reported search QPS is the fastest ef with recall@10 >= 0.95.

Re-rank: RuvectorQuery::default() for QueryMode::NeuralSearch (k 10, ef 50,
gnn_depth 2, T 1.0; query.rs:44-58) through ruvector_amd.NeuralSearch — HNSW
top-ef candidates -> 2 x RuvectorLayer(768, 768, heads 8).forward(query,
candidates, softmax weights) -> differentiable_search top-10 — timed for the
whole query batch with every input resident in HBM. A sample of queries is
re-checked against the oracle's per-query composition on the same candidates.

CPU baseline: the oracle's hnsw_rs search on the same graph (bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--queries", type=int, default=10_000)
    p.add_argument("--m", type=int, default=32)
    p.add_argument("--efc", type=int, default=200)
    p.add_argument("--ef", default="50,100,200,300,400,600")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--check", type=int, default=16, help="queries re-checked against the oracle re-rank")
    a = p.parse_args()

    import ruvector_amd as rv
    import bench_hnsw

    log = lambda s: print(s, file=sys.stderr, flush=True)  # noqa: E731
    n, d, nq, k = a.n, a.dim, a.queries, 10
    keep = {}
    t_all = time.perf_counter()
    out = bench_hnsw.run(n, d, nq, a.m, a.efc, [int(e) for e in a.ef.split(",")], k, "l2", seed_base=5,
                         cpu=not a.no_cpu, cpu_seconds=a.cpu_seconds, log=log, data="normal", keep=keep)
    out["config"] = (f"C3: {n} x {d} N(0,1) seed 5, {nq} queries seed 6, HNSW M={a.m} ef_c={a.efc}, L2, k={k}; "
                     f"re-rank RuvectorQuery::default NeuralSearch (ef 50, gnn_depth 2, T 1) with "
                     f"2 x RuvectorLayer({d},{d},h=8)")
    idx, xb, qb = keep["index"], keep["x"], keep["q"]

    layers = [rv.RuvectorLayer(d, d, 8, 0.0, seed=101 + i) for i in range(2)]
    ns = rv.NeuralSearch(idx, xb, n, d, layers)
    query = rv.RuvectorQuery(mode=rv.QueryMode.NeuralSearch)
    ns.run_device(qb, min(nq, 256), query)  # warm-up (scratch allocation)
    rv.synchronize()
    prof = rv.Profiler()
    with prof:
        t0 = time.perf_counter()
        cand, pos, w = ns.run_device(qb, nq, query)
        rv.synchronize()
        dt = time.perf_counter() - t0
    stages = {name: round(prof.query(name)[0], 2) for name in
              ("hnsw_search", "star_gather", "differentiable_search", "gnn_gemm_msg", "gnn_gemm_kv", "gnn_edge_attention",
               "gnn_finish")}
    ns_out = {"qps": round(nq / dt, 1), "ms": round(dt * 1e3, 2), "kernel_ms": stages,
              "query": "RuvectorQuery::default() NeuralSearch: k 10, ef 50, gnn_depth 2, T 1.0"}
    log(f"neural search {nq} queries: {dt * 1e3:.1f} ms -> {nq / dt:.0f} QPS; {stages}")

    if a.check > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle as O
        c = min(query.ef, n)
        s = min(a.check, nq)
        cids = cand.download(np.uint64, (nq, c))[:s].astype(np.int64)
        gp = pos.download(np.int64, (nq, k))[:s]
        q = qb.download(np.float32, (s, d))
        Ws = [O.RvlWeights(json.loads(l.to_json())) for l in layers]
        equal, werr = 0, 0.0
        gw = w.download(np.float32, (nq, k))[:s]
        for i in range(s):
            cv = np.stack([xb.download(np.float32, d, offset=int(j) * d * 4) for j in cids[i]])
            fi, fw = O.differentiable_search(q[i], cv, c, query.temperature)
            soft = np.empty(c, np.float32)
            soft[fi] = fw
            h = q[i]
            for W in Ws:
                h = O.rvl_forward_one(W, h, cv, soft)
            pi, pw = O.differentiable_search(h, cv, k, query.temperature)
            equal += int(np.array_equal(gp[i], pi))
            werr = max(werr, float(np.max(np.abs(gw[i] - pw)) / max(float(np.max(np.abs(pw))), 1e-30)))
        ns_out["oracle_check"] = {"queries": s, "positions_equal": equal, "max_rel_weight_err": werr}
        log(f"oracle re-rank check: {equal}/{s} equal, weight err {werr:.2e}")
    out["neural_search"] = ns_out
    out["total_s"] = round(time.perf_counter() - t_all, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
