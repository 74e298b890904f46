#!/usr/bin/env python3
"""C5 benchmark: hyperbolic HNSW (Poincaré ball, c = 1) on one
GPU shard — the per-GPU unit of the 50M x 1024 / 8-GPU configuration.

Data (C5 generator): direction ~ N(0,1) normalised, radius 0.9 * U[0,1)
(seed 7 points, seed 8 queries), HyperbolicHnswConfig defaults (M=16, M0=32,
ef_c=200, ef_s=50). Build: GPU batched insert from HBM-resident vectors.
Ground truth: exact Poincaré scan (K8) on the GPU (bit-exact with the oracle's
scan order). Reports build time, recall@10 / QPS over an ef sweep, QPS at
recall >= 0.95, tangent-pruned search, and the oracle's CPU search on the same
graph (bounded sample) with an id-equality check.

--gpus N (one process per GPU: started here as child processes when no launcher set
WORLD_SIZE, else RANK / WORLD_SIZE / LOCAL_RANK from the launcher; `--transport host`
lets the ranks share one GPU): the C5 configuration itself,
node-range shards of --per-gpu points each (default 6.25M = 50M / 8; weak scaling,
so N = 8 is the full 50M x 1024 corpus), every rank generating exactly its rows of
the corpus on the GPU (rvx_fill_ball_rows). Each query batch runs
ShardedHyperbolicHnsw::search across the GPUs (shard.rs:354-373;
rvx_hyperbolic_sharded_search_device): rank 0's queries broadcast over RCCL, the
local shard searched (exact Poincaré scan, tangent-pruned search, graph search),
one all-gather of every rank's top-10 and the GPU merge. Ground truth = the exact
mode (global exact top-10). Reports QPS per mode, recall@10 against the exact
mode, the broadcast / all-gather / merge time, and the build time (max over ranks).
The exact mode is itself checked against the CPU at full scale: every rank streams its
shard through the oracle's Poincaré scan for `--cpu-queries` queries, the per-shard
top-10 lists are merged on rank 0 (shard.rs:354-373 order) and compared with the GPU's
ids and distances bit for bit.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def ball(n, d, seed, chunk=1 << 18):
    r = np.random.default_rng(seed)
    out = np.empty((n, d), np.float32)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        v = r.standard_normal((m, d), dtype=np.float32)
        v /= np.linalg.norm(v, axis=1, keepdims=True)
        out[s:s + m] = v * (0.9 * r.random((m, 1), dtype=np.float32))
    return out


def recall(gt, got):
    k = gt.shape[1]
    return float(np.mean([len(set(a.tolist()) & set(b.tolist())) / k for a, b in zip(gt, got)]))


F16_MFMA_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: dense f16/bf16 MFMA ~2.5 PF (spec)


def main_sharded(a):
    """C5 across GPUs: node-range shards + broadcast / all-gather / merge per query batch."""
    import ruvector_amd as rv
    from ruvector_amd.shard import comm_from_env
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rv.set_device(local % max(rv.device_count(), 1) if a.transport == "host" else local)
    comm = comm_from_env(a.transport)
    log = (lambda s: print(f"[rank {rank}] {s}", file=sys.stderr, flush=True))  # noqa: E731
    out = run_sharded(a.per_gpu, a.dim, a.queries, [int(e) for e in a.ef.split(",") if e], comm, rank, world,
                      cpu_queries=a.cpu_queries, cpu_seconds=0.0, log=log)
    if rank == 0:
        print(json.dumps(out), flush=True)


def run_sharded(n, d, nq, efs, comm, rank, world, cpu_queries=4, cpu_seconds=0.0, log=None, k=10):
    """One C5 measurement over `world` node-range shards of n points (weak scaling: world x n
    points in all; world 1 with comm None is the one-GPU shard). Every rank calls it; the
    returned dict is the same on every rank except for rank-0-only fields.

    * build: rvx_hyperbolic_insert_batch_device of this rank's rows (HyperbolicHnswConfig
      defaults, hnsw.rs:127-258), max over ranks; tangent cache (tangent.rs), max over ranks;
    * modes (ShardedHyperbolicHnsw::search, shard.rs:354-373): "exact" (K10 MFMA-filtered
      Poincaré scan + reference-order re-rank, the ground truth), "pruned"
      (search_with_pruning, hnsw.rs:450-490: tangent scan through K10, k x prune_factor
      candidates re-ranked by Poincaré distance) and the graph search at each ef in `efs`;
      QPS = nq / max-over-ranks wall time, recall@10 against the exact mode;
    * roofline of the exact mode's filter (MFMA: 2 nq n d f16 flops per rank) and of the
      pruned mode's candidate re-rank (HBM: 4 d B per evaluated candidate, §8d);
    * oracle check: the exact mode's ids and distances of the first `cpu_queries` queries equal
      the oracle's Poincaré scan over every shard, merged in shard.rs order (bit for bit);
      with cpu_seconds > 0 the number of checked queries grows until the oracle's scan takes
      about that long, and its rate is the CPU baseline (rank 0 of a one-rank run)."""
    import ruvector_amd as rv
    from ruvector_amd.shard import REDUCE_MAX

    import benchutil
    log = log or (lambda s: None)
    r0 = rank * n

    def barrier():
        rv.synchronize()
        if comm is not None:
            comm.barrier()

    def vmax(v):
        return comm.allreduce([v], REDUCE_MAX)[0] if comm is not None else v

    xb = rv.Buffer(n * d * 4)
    xb.fill_ball(n, d, 7, r0)  # this rank's rows of the (world x n)-point corpus
    qb = None
    if rank == 0:
        qb = rv.Buffer(nq * d * 4)
        qb.fill_ball(nq, d, 8, 0)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=7 + rank), dim=d)
    barrier()
    t0 = time.perf_counter()
    with benchutil.heartbeat(f"building shard {rank}: {n} x {d}", log=log):
        h.insert_device(xb, n, d)
        rv.synchronize()
    build_s = vmax(time.perf_counter() - t0)
    cpu_check = (oracle_scan_shard(cpu_queries, cpu_seconds, xb, n, d, r0, rank, world, comm, log)
                 if cpu_queries > 0 else None)
    del xb
    t0 = time.perf_counter()
    h.build_tangent_cache()
    rv.synchronize()
    cache_s = vmax(time.perf_counter() - t0)
    grp = rv.ShardedHyperbolicSearch(h, comm, r0)
    gid, dist = rv.Buffer(nq * k * 8), rv.Buffer(nq * k * 4)
    modes = [("exact", 0), ("pruned", 0)] + [("search", int(e)) for e in efs]
    out_modes, gt = {}, None
    roof = {}
    for mode, ef in modes:
        grp.search_device(qb, min(nq, 256), k, gid, dist, ef=ef, mode=mode)  # warm-up (scratch, code objects)
        barrier()
        prof = rv.Profiler()
        with prof:
            t0 = time.perf_counter()
            with benchutil.heartbeat(f"{mode} ef={ef}", log=log):
                grp.search_device(qb, nq, k, gid, dist, ef=ef, mode=mode)
                barrier()
            dt = vmax(time.perf_counter() - t0)
        kern = prof.summary()
        ids = gid.download(np.int64, (nq, k))
        if mode in ("exact", "pruned"):
            out_scan = rv.scan_last_stats()  # K10 filter vs exact-VALU queries of this rank's scan
        if mode == "exact":
            gt = ids
            if cpu_check is not None and rank == 0:
                m = cpu_check["ids"].shape[0]
                cpu_check["ids_equal"] = bool(np.array_equal(ids[:m], cpu_check["ids"]))
                cpu_check["distances_equal"] = bool(np.array_equal(dist.download(np.float32, (nq, k))[:m],
                                                                   cpu_check["dist"]))
        phases = {t: round(kern[t]["total_ms"], 2) for t in ("shard_bcast", "shard_allgather", "shard_merge")
                  if t in kern}
        key = mode if mode != "search" else f"search_ef{ef}"
        out_modes[key] = {"qps": round(nq / dt, 1), "recall_at_10": round(recall(gt, ids), 4),
                          "wall_ms": round(dt * 1e3, 1), "phase_ms_rank0": phases,
                          "kernel_ms_rank0": {t: round(v["total_ms"], 3) for t, v in kern.items()}}
        if mode in ("exact", "pruned"):
            out_modes[key]["scan_stats_rank0"] = out_scan
        filt = kern.get("scan_filter")
        if mode in ("exact", "pruned") and filt and filt["total_ms"] > 0:
            # K10 ranks every (query, row) pair with f16 MFMA over the d Poincaré (exact) or
            # tangent (pruned) coordinates: 2 nq n d flops on this rank's shard, plus the same
            # per query of the second filter launch (queries whose first lists proved nothing)
            nq2 = int((out_scan or {}).get("second_pass", 0))
            flops = 2.0 * (nq + nq2) * n * d
            tf = flops / (filt["total_ms"] * 1e-3) / 1e12
            roof[f"{mode}_scan_filter"] = {
                "bound": "mfma", "achieved": round(tf, 1), "peak": F16_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(tf / F16_MFMA_PEAK_TFS, 4), "ms_total": round(filt["total_ms"], 3),
                "launches": filt["launches"], "work_total": flops, "traffic": None,
                "work": f"2 n d flops per query: {nq} queries" + (f" + {nq2} in the second launch" if nq2 else "")}
        rr = kern.get("hyp_rerank")
        if mode == "pruned" and rr and rr["total_ms"] > 0:
            cand = k * h.config.prune_factor
            byts = float(nq) * cand * 4 * d  # §8d: 4 d B per evaluated point
            gbs = byts / (rr["total_ms"] * 1e-3) / 1e9
            roof["pruned_candidate_rerank"] = {
                "bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                "frac": round(gbs / 8000.0, 4), "avg_ms": round(rr["total_ms"] / rr["launches"], 3),
                "launches": rr["launches"], "work_per_launch": byts / rr["launches"], "traffic": None,
                "bytes": f"{cand} candidates x 4 d B per query"}
        log(f"{key}: {out_modes[key]['qps']} QPS, recall {out_modes[key]['recall_at_10']}")
    total = world * n
    res = {
        "metric": "C5 hyperbolic HNSW queries/s@recall, node-range sharded", "n_gpus": world,
        "scaling": "weak",
        "config": {"workload": f"configs[4] C5: {total} x {d} Poincaré ball (c=1), {world} node-range shard(s) of {n} "
                               f"(the 50M x 1024 corpus's per-GPU unit), {nq} queries, k={k}, "
                               "HyperbolicHnswConfig defaults (M=16, M0=32, ef_c=200, prune_factor 10)",
                   "points_total": total, "points_per_gpu": n, "dim": d, "queries": nq, "k": k},
        "build_s": round(build_s, 2), "build_points_per_s_per_gpu": round(n / build_s, 1),
        "tangent_cache_s": round(cache_s, 2), "modes": out_modes,
        "ground_truth": "exact mode: global exact Poincaré top-10 over every shard",
        "roofline": roof,
        "data": "synthetic (rvx_fill_ball_rows: direction N(0,1) normalised, radius 0.9 U[0,1); seed 7 points, 8 queries)"}
    if cpu_check is not None:
        res["exact_vs_oracle"] = {k2: v for k2, v in cpu_check.items() if k2 not in ("ids", "dist", "cpu_s_rank0")}
        if world == 1 and rank == 0:
            res["cpu_baseline"] = {
                "value": round(cpu_check["queries"] / cpu_check["cpu_s_rank0"], 3), "unit": "queries/s",
                "cores": cpu_check["threads"], "kind": "port",
                "sample": f"oracle exact Poincaré scan (poincare.rs:135-301 arithmetic, orc_hyp_scan_rows) of "
                          f"{cpu_check['queries']} queries over all {n} rows, {cpu_check['cpu_s_rank0']:.1f} s "
                          "(rows streamed from HBM in chunks; the copies are not timed)"}
    return res


def oracle_scan_shard(m, cpu_seconds, xb, n, d, r0, rank, world, comm, log, k=10):
    """Exact Poincaré top-10 of the first `m` queries over this rank's shard on the CPU
    (oracle/hyperbolic.cpp orc_hyp_scan_rows, rows streamed from HBM in chunks; only the
    oracle calls are timed), then every rank's lists merged on rank 0 in
    ShardedHyperbolicHnsw::search order (ascending distance, lower global id first on ties).
    cpu_seconds > 0 (one rank): m grows (up to 64 queries) until the scan takes about that
    long."""
    import ruvector_amd as rv
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from benchutil import host_threads
    threads, _ = host_threads()

    def scan(m):
        q = rv.Buffer(m * d * 4)
        q.fill_ball(m, d, 8, 0)  # the first m rows of the query batch
        qh = q.download(np.float32, (m, d))
        ids = dist = None
        cpu_s = 0.0
        chunk = 1 << 18
        for s0 in range(0, n, chunk):
            rows = min(chunk, n - s0)
            xs = xb.download(np.float32, (rows, d), offset=s0 * d * 4)
            t0 = time.perf_counter()
            ids, dist = O.hyp_scan_rows(xs, qh, k, id_base=r0 + s0, ids=ids, dist=dist, threads=threads)
            cpu_s += time.perf_counter() - t0
        return ids, dist, cpu_s

    ids, dist, cpu_s = scan(m)
    if cpu_seconds > 0 and world == 1 and cpu_s < 0.8 * cpu_seconds:
        m = int(min(64, max(m + 1, m * cpu_seconds / max(cpu_s, 1e-3))))
        ids, dist, cpu_s = scan(m)
    log(f"oracle exact scan of {m} queries over {n} rows: {cpu_s:.1f} s")
    if comm is not None:  # one-hot all-reduce sums move every rank's lists to every rank
        flat = np.zeros((world, m, k, 2))
        flat[rank, :, :, 0] = ids
        flat[rank, :, :, 1] = dist
        flat = np.asarray(comm.allreduce(flat.reshape(-1).tolist())).reshape(world, m, k, 2)
        parts = [(flat[p, :, :, 0].astype(np.int64), flat[p, :, :, 1].astype(np.float32)) for p in range(world)]
        from ruvector_amd.shard import merge_topk
        ids, dist = merge_topk(parts, k)
    return {"ids": ids, "dist": dist, "queries": m, "rows_per_rank": n, "cpu_s_rank0": round(cpu_s, 2),
            "threads": threads}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1_000_000)
    p.add_argument("--dim", type=int, default=1024)
    p.add_argument("--queries", type=int, default=10_000)
    p.add_argument("--ef", default="50,100,200,400,800")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--gpus", type=int, default=0, help="node-range-sharded C5 across GPUs (see module doc)")
    p.add_argument("--per-gpu", type=int, default=6_250_000, help="points per GPU shard with --gpus")
    p.add_argument("--transport", choices=("rccl", "host"), default="rccl")
    p.add_argument("--cpu-queries", type=int, default=4, help="with --gpus: queries checked against the oracle scan")
    a = p.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import benchutil  # N ranks as child processes, before any GPU call
        sys.exit(benchutil.spawn_ranks(a.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if a.gpus or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        if a.ef == "50,100,200,400,800":
            a.ef = "50,200"
        return main_sharded(a)
    import ruvector_amd as rv

    log = lambda s: print(s, file=sys.stderr, flush=True)  # noqa: E731
    n, d, nq, k = a.n, a.dim, a.queries, 10
    import benchutil
    with benchutil.heartbeat(f"generating {n} x {d}", log=log):
        x = ball(n, d, 7)
        q = ball(nq, d, 8)
        xb = rv.Buffer.from_numpy(x)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=7))
    rv.synchronize()
    t0 = time.perf_counter()
    with benchutil.heartbeat(f"building {n} x {d}", log=log):
        h.insert_device(xb, n, d)
        rv.synchronize()
    build_s = time.perf_counter() - t0
    log(f"build {n} x {d}: {build_s:.1f} s")
    del xb

    t0 = time.perf_counter()
    gt, gtd, _ = h.brute_force(q, k)
    gt_s = time.perf_counter() - t0
    log(f"exact Poincaré ground truth, {nq} queries: {gt_s:.2f} s")

    sweep = []
    prof = rv.Profiler()
    for ef in [int(e) for e in a.ef.split(",")]:
        h.search_batch(q[:256], k, ef)
        with prof:
            t0 = time.perf_counter()
            ids, dist, _ = h.search_batch(q, k, ef)
            dt = time.perf_counter() - t0
        ker, _ = prof.query("hnsw_search")
        rec = recall(gt, ids)
        sweep.append({"ef": ef, "recall": round(rec, 4), "qps": round(nq / dt, 1), "kernel_ms": round(ker, 2)})
        log(f"ef={ef}: recall@10 {rec:.4f}, {nq / dt:.0f} QPS (kernel {ker:.1f} ms)")
    ok = [s for s in sweep if s["recall"] >= 0.95]
    best = max(ok, key=lambda s: s["qps"]) if ok else None

    t0 = time.perf_counter()
    h.build_tangent_cache()
    rv.synchronize()
    cache_s = time.perf_counter() - t0
    h.search_with_pruning_batch(q[:256], k)
    t0 = time.perf_counter()
    pids, _, _ = h.search_with_pruning_batch(q, k)
    pdt = time.perf_counter() - t0
    pruned = {"tangent_cache_build_s": round(cache_s, 2), "recall": round(recall(gt, pids), 4),
              "qps": round(nq / pdt, 1), "candidates": k * h.config.prune_factor}
    log(f"pruned: {pruned}")

    out = {"config": f"C5 shard: {n} x {d} Poincaré ball (c=1), {nq} queries, M=16 M0=32 ef_c=200, k=10",
           "build_s": round(build_s, 2), "build_points_per_s": round(n / build_s, 1), "gt_s": round(gt_s, 2),
           "sweep": sweep, "qps_at_recall95": best["qps"] if best else None,
           "ef_at_recall95": best["ef"] if best else None, "search_with_pruning": pruned}

    if not a.no_cpu and best:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle as O
        g = h.export_graph()
        xs = np.stack([h.get_vector(i) for i in range(n)]) if n <= 200_000 else x  # projected == x inside the ball
        o = O.Hyp.from_graph(xs, g)
        threads = min(16, os.cpu_count() or 1)
        s = 64
        t0 = time.perf_counter()
        o.search(q[:s], k, best["ef"], threads=threads)
        dt = time.perf_counter() - t0
        s = int(min(nq, max(s, s * a.cpu_seconds / max(dt, 1e-3))))
        t0 = time.perf_counter()
        cids, _, _ = o.search(q[:s], k, best["ef"], threads=threads)
        dt = time.perf_counter() - t0
        gids, _, _ = h.search_batch(q[:s], k, best["ef"])
        out["cpu_baseline"] = {"value": round(s / dt, 1), "unit": "queries/s", "cores": threads, "kind": "port",
                               "sample": f"oracle HyperbolicHnsw::search on the same graph, {s} queries, ef={best['ef']}"}
        out["cpu_gpu_ids_equal_frac"] = float(np.mean(np.all(cids == gids, axis=1)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
