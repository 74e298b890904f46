#!/usr/bin/env python3
"""C3 (BASELINE configs[2]): 10M x 768 HNSW build + k=10 search + GNN re-rank on 1 GPU.

X 10,000,000 x 768 N(0,1) (30.7 GB resident in HBM; `bench.py`'s c3 leg runs on its own
node table, seed 3; standalone seed 5), queries 10,000 N(0,1) (seed 6); HNSW M=32,
ef_c=200, L2, built on the GPU (hnsw_rs insert rules, batched). Ground truth: the exact
scan (distances in the reference's order, ties by id). ef is swept; the reported search
QPS is the fastest ef with recall@10 >= 0.95 (none on this data at M 32).

Re-rank: RuvectorQuery::default() for QueryMode::NeuralSearch (k 10, ef 50,
gnn_depth 2, T 1.0; query.rs:44-58) through ruvector_amd.NeuralSearch — HNSW
top-ef candidates -> 2 x RuvectorLayer(768, 768, heads 8).forward(query,
candidates, softmax weights) -> differentiable_search top-10 (search.rs:56-162) — timed
for the whole query batch with every input resident in HBM. A sample of queries is
re-checked against the oracle's per-query composition on the same candidates.

CPU baseline: the oracle's hnsw_rs search_filter on the same graph (bounded sample,
reference scalar distance order; ids compared with the GPU's).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def leg(xb, n, d, qb, nq, m=32, efc=200, efs=(100, 400, 1600), k=10, cpu=True, cpu_seconds=10.0, log=print, check=8,
        seed=5):
    """HNSW build over the HBM table xb [n][d], ef sweep with recall against the exact scan,
    NeuralSearch re-rank QPS, CPU baseline. Returns the report dict (the index is freed)."""
    import benchutil
    import ruvector_amd as rv
    out = {"config": f"C3: {n} x {d} N(0,1), {nq} queries N(0,1) seed 6, HNSW M={m} ef_c={efc}, L2, k={k}; re-rank "
                      f"RuvectorQuery::default NeuralSearch (ef 50, gnn_depth 2, T 1) with 2 x RuvectorLayer({d},{d},h=8)"}
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=m, ef_construction=efc, ef_search=100),
                       seed=seed)
    rv.synchronize()
    t0 = time.perf_counter()
    with benchutil.heartbeat(f"building {n}x{d}", log=log):
        rv._lib.call("rvx_index_add_batch_device", idx.handle, xb.handle, n, 0)
        rv.synchronize()
    out["build_s"] = round(time.perf_counter() - t0, 2)
    log(f"c3 build {n}x{d} M={m} ef_c={efc}: {out['build_s']} s")

    ids_b, dist_b = rv.Buffer(nq * k * 8), rv.Buffer(nq * k * 4)
    rv._lib.call("rvx_index_brute_force_device", idx.handle, qb.handle, nq, k, ids_b.handle, dist_b.handle)
    rv.synchronize()
    gt = ids_b.download(np.uint64, (nq, k))

    sweep = []
    prof = rv.Profiler()
    for ef in efs:
        rv._lib.call("rvx_index_search_device", idx.handle, qb.handle, nq, k, ef, ids_b.handle, dist_b.handle)
        rv.synchronize()
        with prof:
            t0 = time.perf_counter()
            rv._lib.call("rvx_index_search_device", idx.handle, qb.handle, nq, k, ef, ids_b.handle, dist_b.handle)
            rv.synchronize()
            dt = time.perf_counter() - t0
        ker_ms, launches = prof.query("hnsw_search")
        st = rv.hnsw_last_search_stats()
        # bytes = n_dist * d * 4 + n_expand * deg_cap * 4 (deg_cap = 2M on layer 0)
        alg_bytes = st["n_dist"] * d * 4 + st["n_expand"] * 2 * m * 4
        got = ids_b.download(np.uint64, (nq, k))
        rec = float(np.mean([len(set(a.tolist()) & set(b.tolist())) / k for a, b in zip(gt, got)]))
        ach = alg_bytes / (ker_ms * 1e-3) / 1e9 if ker_ms > 0 else None
        sweep.append({"ef": ef, "recall": round(rec, 4), "qps": round(nq / dt, 1), "kernel_ms": round(ker_ms, 3),
                      "dist_per_query": round(st["n_dist"] / nq, 1), "expand_per_query": round(st["n_expand"] / nq, 1),
                      "roofline": {"bound": "hbm", "achieved": round(ach, 1) if ach else None, "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                                   "rate_kind": RATE_KIND, "practical_ceiling_GBps": RANDOM_ROW_GBPS,
                                   "frac_of_practical": round(ach / RANDOM_ROW_GBPS, 4) if ach else None,
                                   "caveat": RATE_CAVEAT if ach and ach > 0.72 * HBM_PEAK_GBS else None,
                                   "traffic": None, "alg_bytes_per_launch": alg_bytes, "launches": launches}})
        log(f"c3 ef={ef}: recall@{k}={rec:.4f} qps={nq / dt:.0f} (kernel {ker_ms:.2f} ms, "
            f"{st['n_dist'] / nq:.0f} dist/query, {ach and round(ach)} GB/s algorithmic)")
    ok = [s for s in sweep if s["recall"] >= 0.95]
    best = max(ok, key=lambda s: s["qps"]) if ok else None
    out.update(sweep=sweep, qps_at_recall95=best["qps"] if best else None, ef_at_recall95=best["ef"] if best else None)
    out["c3_config"] = {"n": n, "d": d, "nq": nq, "m": m, "efc": efc}  # what profiles/pmc_traffic_c3.json matches
    attach_search_traffic(out, n, d, nq, m, efc)

    # NeuralSearch re-rank (query.rs:44-58, search.rs:56-162)
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
    log(f"c3 neural search {nq} queries: {dt * 1e3:.1f} ms -> {nq / dt:.0f} QPS")
    if check > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle as O
        c = min(query.ef, n)
        s = min(check, nq)
        cids = cand.download(np.uint64, (nq, c))[:s].astype(np.int64)
        gp = pos.download(np.int64, (nq, k))[:s]
        q = qb.download(np.float32, (s, d))
        Ws = [O.RvlWeights(json.loads(l.to_json())) for l in layers]
        equal, werr = 0, 0.0
        gw = w.download(np.float32, (nq, k))[:s]
        for i in range(s):
            cv = xb.gather_rows(n, d, cids[i])
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
        log(f"c3 oracle re-rank check: {equal}/{s} equal, weight err {werr:.2e}")
    out["neural_search"] = ns_out
    del ns, cand, pos, w

    if cpu:
        # at the sweep's highest-recall ef (the most CPU work per query, so the bounded sample
        # reaches its target time within the query set)
        top = max(sweep, key=lambda s_: (s_["recall"], s_["ef"]))
        out["cpu_baseline"], out["cpu_gpu_ids_equal"] = cpu_leg(idx, xb, qb, n, d, nq, k, top["ef"], cpu_seconds, log)
        out["cpu_baseline"]["gpu_qps_same_ef"] = top["qps"]
    del idx
    rv.release_scratch()
    return out


def cpu_leg(idx, xb, qb, n, d, nq, k, ef, cpu_seconds, log):
    """The oracle's search_filter (patches/hnsw_rs/src/hnsw.rs:1475-1589 restated, reference scalar
    distance order) on the GPU-built graph, a bounded query sample at the sweep's first ef;
    returns (cpu_baseline, ids equal to the GPU's on that sample)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from benchutil import host_threads
    threads, tinfo = host_threads()
    t0 = time.perf_counter()
    x = xb.download(np.float32, (n, d))
    h = O.Hnsw.from_graph(x, idx.export_graph(), "l2")
    del x
    setup = time.perf_counter() - t0
    q = qb.download(np.float32, (nq, d))
    m = min(nq, 64)
    t0 = time.perf_counter()
    h.search(q[:m], k, ef, threads=threads)
    dt = time.perf_counter() - t0
    m = int(min(nq, max(m, m * cpu_seconds / max(dt, 1e-3))))
    t0 = time.perf_counter()
    cids = h.search(q[:m], k, ef, threads=threads)[0]
    dt = time.perf_counter() - t0
    gpu = idx.search_array(q[:m], k, ef)[0].astype(np.int64)
    log(f"c3 cpu baseline: {m} queries in {dt:.1f} s ({m / dt:.0f} QPS; setup {setup:.0f} s)")
    return ({"value": round(m / dt, 1), "unit": "queries/s", "cores": threads, "kind": "port", "host": tinfo,
             "sample": f"hnsw_rs search_filter (hnsw.rs:1475-1589 restated, reference scalar distance order) on the "
                       f"GPU-built graph, {m} queries at ef {ef}, {threads} threads, {dt:.1f} s"},
            bool(np.array_equal(cids, gpu)))


# The search reads random rows; MI355X_MICROARCH.md:357 measures 5.7-5.8 TB/s for random 2,304-B
# rows of a table far past the Infinity Cache (6.29 TB/s for a float4 copy, :36). Rows that many
# in-flight queries share (the entry neighbourhood, hub rows) are served from the Infinity Cache,
# and FETCH_SIZE counts L2 misses including Infinity-Cache hits (:297), so neither the
# algorithmic rate nor the PMC bytes are pure HBM throughput.
RANDOM_ROW_GBPS = 5750.0
RATE_KIND = ("fabric: algorithmic row bytes (SURVEY.md §8d) / kernel time; rows shared by concurrent queries come "
             "from the Infinity Cache, so this bounds HBM bytes/s from above")
RATE_CAVEAT = ("above 0.72 of HBM peak = the guide's random-row gather ceiling (5.75 TB/s): part of these bytes are "
               "Infinity-Cache hits, so 'frac' is an upper bound on the HBM fraction, not HBM throughput")


def attach_search_traffic(out, n, d, nq, m, efc):
    """HBM bytes per search launch from the committed rocprofv3 --pmc passes of this leg
    (scripts/c3_traffic.sh -> profiles/pmc_traffic_c3.json), when the configuration matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic_c3.json")
    if not os.path.exists(path):
        return
    try:
        pmc = json.load(open(path))
    except ValueError:
        return
    cfg = pmc.get("config") or {}
    if any(cfg.get(kk) != v for kk, v in {"n": n, "d": d, "nq": nq, "m": m, "efc": efc}.items()):
        return
    per_ef = (pmc.get("kernels") or {}).get("hnsw_search_by_ef") or {}
    for s in out["sweep"]:
        ent = per_ef.get(str(s["ef"]))
        if ent:
            s["roofline"]["traffic"] = round(ent["hbm_bytes_per_launch"], 0)
            s["roofline"]["traffic_source"] = ("rocprofv3 --pmc FETCH_SIZE(x2, gfx950) + WRITE_SIZE, "
                                               "profiles/pmc_traffic_c3.json: L2-miss bytes, Infinity-Cache hits "
                                               "included (an upper bound on HBM bytes)")


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
    p.add_argument("--seed", type=int, default=5)
    a = p.parse_args()

    import ruvector_amd as rv
    log = lambda s: print(s, file=sys.stderr, flush=True)  # noqa: E731
    t_all = time.perf_counter()
    xb = rv.Buffer(a.n * a.dim * 4)
    xb.fill_normal(a.n * a.dim, a.seed)
    qb = rv.Buffer(a.queries * a.dim * 4)
    qb.fill_normal(a.queries * a.dim, 6)
    out = leg(xb, a.n, a.dim, qb, a.queries, a.m, a.efc, [int(e) for e in a.ef.split(",")], 10, cpu=not a.no_cpu,
              cpu_seconds=a.cpu_seconds, log=log, check=a.check, seed=a.seed)
    out["total_s"] = round(time.perf_counter() - t_all, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
