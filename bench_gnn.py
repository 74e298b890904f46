#!/usr/bin/env python3
"""C4 benchmark: multi-layer ruvector-gnn RuvectorLayer stack +
EdgeFeaturedAttention head over a graph, one process per GPU (node-range shards;
`--gpus N` starts the N ranks itself, or a launcher sets WORLD_SIZE — the processes
use no torch; rows exchanged over RCCL p2p, or the host socket transport).

Workload: N x 768 node table (N(0,1), seed 5); `--layers` x RuvectorLayer(768, 768,
heads=8, dropout=0, seeded init) (crates/ruvector-gnn/src/layer.rs:313-457), then
EdgeFeaturedAttention (node_dim 768, edge_dim 1, 8 heads, concat, slope 0.2;
crates/ruvector-attention/src/graph/edge_featured.rs:87-320). Graph (`--graph`):
  random  uniform random out-degree-32 CSR (seed 6), edge feature = weight U[0,1)
          (seed 7) — the default, shardable at any N;
  hnsw    the layer-0 CSR of an HNSW built on the GPU over the same table (M 32,
          ef_c 200, hnsw_rs rules; up to 64 neighbours per node in stored order) with
          edge feature = the stored HNSW edge distance, as §8(d) C4 names it
          (rvx_index_export_layer0; one GPU).

value = (edges x (layers + 1)) / wall time of one forward of the stack, inputs
resident in HBM. Per-kernel times are HIP events stamped by the dispatch
packets. CPU baseline: the oracle's RuvectorLayer restatement on a bounded
sample of layer-1 rows (16 threads), with a per-row parity check on the same rows.
bench.py runs the same leg (run()) at 10M x 768 on the random graph.
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
GEMM_PEAK_TFS = 2500.0 / 3  # split-f16 (3 f16 MFMA products per f32 FMA) ceiling, as in bench.py


def hnsw_layer0_graph(x, n, d, m=32, efc=200, log=None):
    """Build an HNSW over the n x d HBM table on the GPU and return (Graph with the
    layer-0 lists and their stored distances as edge weights, [E][1] edge-feature
    buffer, host (row_ptr, col, dist), build seconds)."""
    import ruvector_amd as rv
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=m, ef_construction=efc), seed=5)
    t0 = time.perf_counter()
    idx.add_device(x, n)
    rv.synchronize()
    build_s = time.perf_counter() - t0
    if log:
        log(f"HNSW over {n} x {d} (M {m}, ef_c {efc}): {build_s:.1f} s")
    rp, col, dist = idx.layer0()
    del idx
    g = rv.Graph.from_csr(rp, col, dist)
    ew = rv.Buffer.from_numpy(dist.reshape(-1, 1))
    return g, ew, (rp, col, dist), build_s


def run(n, d=768, deg=32, heads=8, nlayers=3, steps=2, warmup=1, comm=None, rank=0, world=1, graph="random",
        cpu=True, cpu_seconds=10.0, log=None):
    """One C4 measurement; returns the bench line (dict). Every rank calls it."""
    import ruvector_amd as rv
    from ruvector_amd.attention import EdgeFeaturedAttention, EdgeFeaturedConfig
    from ruvector_amd.shard import REDUCE_MAX, ShardPlan

    H = d
    plan = ShardPlan(n, world)
    r0, r1 = plan.rows(rank)
    n_loc = r1 - r0
    offsets = np.array([plan.rows(p)[0] for p in range(world)] + [n], dtype=np.int64)

    # node-range shards: every rank holds the whole-table buffers but reads and
    # writes only its own rows; its CSR rows (global column ids) and their slice
    # of the edge-weight stream are generated in place, so the sharded job is
    # the same graph as the 1-GPU one
    x = rv.Buffer(n * d * 4)
    x.fill_normal(n * d, 5)
    host_csr, hnsw_s = None, None
    if graph == "hnsw":
        if world > 1:
            raise ValueError("--graph hnsw runs on one GPU")
        g, ew, host_csr, hnsw_s = hnsw_layer0_graph(x, n, d, log=log)
        E = int(host_csr[0][-1])
        e_loc = E
    else:
        g = rv.Graph.random_shard(n, r0, n_loc, deg, 6, weight_seed=7)
        ew = g._keep[2]  # [E_local][1] edge features = the edge weights
        E = n * deg
        e_loc = n_loc * deg
    layers = [rv.RuvectorLayer(d, H, heads, 0.0, seed=100 + i) for i in range(nlayers)]
    head = EdgeFeaturedAttention(EdgeFeaturedConfig(node_dim=H, edge_dim=1, num_heads=heads))
    bufs = [rv.Buffer(n * H * 4) for _ in range(2)]
    out = rv.Buffer(n * H * 4)
    rv.synchronize()

    def step():
        src = x
        for i, layer in enumerate(layers):
            layer.forward_exchange(g, src, bufs[i % 2], offsets, comm)
            src = bufs[i % 2]
        head.forward_exchange(g, src, ew, out, offsets, comm)

    def barrier():
        rv.synchronize()
        if comm is not None:
            comm.barrier()

    for _ in range(warmup):
        step()
    barrier()
    prof = rv.Profiler()
    with prof:
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        rv.synchronize()
        t1 = time.perf_counter()
        barrier()
    dt = (t1 - t0) / steps
    kern = prof.summary()
    if comm is not None:
        dt = comm.allreduce([dt], REDUCE_MAX)[0]

    # algorithmic work per layer, this rank's rows and edges
    layer_flops = 2.0 * n_loc * (d * H + 11 * H * H)
    edge_bytes = e_loc * (3 * 4 * H + 8) + n_loc * (8 + 4 * H + 2 * 4 * H)
    gemm_ms = sum(v["total_ms"] for k, v in kern.items() if k.startswith("gnn_gemm")) / steps / nlayers
    edge_ms = kern.get("gnn_edge_attention", {"total_ms": 0})["total_ms"] / steps / nlayers
    roof = {
        "gnn_gemm (all dense layers of one RuvectorLayer)": {
            "bound": "mfma", "achieved": round(layer_flops / (gemm_ms / 1e3) / 1e12, 2), "peak": round(GEMM_PEAK_TFS, 1),
            "unit": "TFLOP/s", "frac": round(layer_flops / (gemm_ms / 1e3) / 1e12 / GEMM_PEAK_TFS, 4),
            "ms_per_layer": round(gemm_ms, 3), "work_per_layer": layer_flops, "traffic": None},
        "gnn_edge_attention": {
            "bound": "hbm", "achieved": round(edge_bytes / (edge_ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(edge_bytes / (edge_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "ms_per_layer": round(edge_ms, 3), "work_per_layer": edge_bytes, "traffic": None,
            "bytes": "per edge 3*4*H (k, v, m rows of the neighbour) + 8; per node 8 + 4H (q) + 2*4H (out, h)"},
    }
    attach_c4_traffic(roof, {"nodes": n, "edges": E, "layers": nlayers, "parallelism": f"node-range x{world}"})
    line = {
        "metric": "GNN-layer edges/sec (RuvectorLayer stack + graph-attention head)",
        "value": round(E * (nlayers + 1) / dt, 1), "unit": "edges/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "dtype": "f32", "gemm_dtype": "split-f16x3",
        "config": {"workload": f"configs[3] stack on {world} GPU(s): {n} x {d}, {nlayers} x RuvectorLayer(h={heads})"
                               " + EdgeFeaturedAttention(8 heads, edge_dim 1)", "nodes": n, "edges": E,
                   "graph": ("uniform random out-degree 32 CSR (seed 6), edge feature U[0,1) (seed 7)" if graph == "random"
                             else "layer 0 of a GPU-built HNSW (M 32, ef_c 200) over the table, edge feature = "
                                  "stored HNSW edge distance"),
                   "layers": nlayers, "parallelism": f"node-range x{world}",
                   "exchange": "per layer: M|K|V rows (RuvectorLayer), T rows (attention head), "
                               "chunked p2p rounds" if world > 1 else "none"},
        "data": "synthetic: X ~ N(0,1) seed 5" + ("; uniform random out-degree CSR seed 6; edge weights U[0,1) seed 7"
                                                   if graph == "random" else "; HNSW layer-0 graph built on the GPU"),
        "roofline": roof,
        "kernel_ms_per_step": {k: round(v["total_ms"] / steps, 3) for k, v in kern.items()},
    }
    if hnsw_s is not None:
        line["hnsw_build_s"] = round(hnsw_s, 2)
    if world > 1 and comm is not None:
        line["parity"] = multi_rank_check(x, g, layers[0], n, d, deg, offsets, comm, rank, world, bufs[1])
    if rank == 0 and world == 1 and cpu:
        # layer 1 is recomputed into bufs[1] (it holds layer 2 of the last step): at 10M x 768
        # the HBM has no room for another table beside the stack's scratch
        line["cpu_baseline"], line["parity"] = cpu_baseline(cpu_seconds, x, g, layers[0], n, d, deg, offsets,
                                                             host_csr, y1=bufs[1])
    del bufs, out, x, g, ew, layers, head
    rv.synchronize()
    return line


def attach_c4_traffic(roof, cfg):
    """HBM bytes per layer of the layer GEMMs and the edge kernel from the committed rocprofv3
    --pmc FETCH_SIZE / WRITE_SIZE passes of this leg (scripts/c4_traffic.sh ->
    profiles/pmc_traffic_c4.json, gfx950 FETCH correction), when the configuration matches:
    the profiled run's total bytes per tag over its forwards x layers."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic_c4.json")
    if not os.path.exists(path):
        return
    try:
        pmc = json.load(open(path))
    except ValueError:
        return
    pc = pmc.get("config") or {}
    if any(pc.get(k) != v for k, v in cfg.items()) or not pc.get("forwards"):
        return
    per = pc["forwards"] * cfg["layers"]
    for key, tag in (("gnn_gemm (all dense layers of one RuvectorLayer)", "gnn_gemm"),
                     ("gnn_edge_attention", "gnn_edge_attention")):
        ent = (pmc.get("kernels") or {}).get(tag)
        if ent and key in roof:
            roof[key]["traffic"] = round(ent["hbm_bytes_total"] / per, 0)
            roof[key]["traffic_source"] = ("rocprofv3 --pmc FETCH_SIZE(x2, gfx950) + WRITE_SIZE per layer, "
                                           "profiles/pmc_traffic_c4.json")


def multi_rank_check(x_buf, g, layer, n, d, deg, offsets, comm, rank, world, y1, rows=128):
    """Self-check of a multi-rank C4 run (after the timed steps): layer 1 runs once more across
    the M|K|V exchange into y1, and the LAST rank compares its first `rows` owned rows with the
    oracle's RuvectorLayer::forward (layer.rs:379-451) over the same graph; their neighbour
    rows' projections came from every other rank over the exchange. The errors reach every
    rank through one max all-reduce."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from bench import rel_errs
    from benchutil import host_threads
    from ruvector_amd.shard import REDUCE_MAX

    layer.forward_exchange(g, x_buf, y1, offsets, comm)
    last = world - 1
    a0 = int(offsets[last])
    rows = int(min(rows, int(offsets[last + 1]) - a0))
    errs = [0.0, 0.0]
    if rank == last and rows > 0:
        threads, _ = host_threads()
        W = O.RvlWeights(json.loads(layer.to_json()))
        rp, col = O.random_csr(n, deg, 6)
        ew = O.fill_uniform(n * deg, 7, 0.0, 1.0)
        nb = col[rp[a0]:rp[a0 + rows]].astype(np.int64)
        need = np.concatenate([np.arange(a0, a0 + rows, dtype=np.int64), nb])
        rp_sub = (rp[a0:a0 + rows + 1] - rp[a0]).astype(np.int64)
        col_sub = (rows + np.arange(nb.size)).astype(np.int32)
        ref = O.rvl_forward_graph(W, x_buf.gather_rows(n, d, need), rp_sub, col_sub, ew[rp[a0]:rp[a0 + rows]],
                                  rows=(0, rows), threads=threads)
        got = y1.gather_rows(n, layer.hidden_dim, np.arange(a0, a0 + rows))
        errs = list(rel_errs(got, ref))
    errs = comm.allreduce(errs, REDUCE_MAX)
    return {"ok": bool(errs[0] <= 1e-5 and errs[1] <= 1e-5), "tol": 1e-5, "max_rel_err": errs[0],
            "row_rel_l2_max": errs[1], "checked_rows": {"owner_rank": last, "rows": [a0, a0 + rows]},
            "input": "layer 1 across the M|K|V exchange (neighbour projections from every rank)",
            "metrics": "normwise max|gpu-ref|/max|ref| and per-row ||gpu_r-ref_r||/||ref_r|| (tests/parity.py)"}


def cpu_baseline(cpu_seconds, x_buf, g, layer, n, d, deg, offsets, host_csr=None, y1=None):
    """Oracle RuvectorLayer::forward on a bounded sample of layer-1 rows (the CPU
    baseline) and the per-row parity of the GPU's layer 1 on the same rows."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    import ruvector_amd as rv
    from bench import rel_errs
    from benchutil import host_threads

    threads, tinfo = host_threads()
    W = O.RvlWeights(json.loads(layer.to_json()))
    if host_csr is None:
        rp, col = O.random_csr(n, deg, 6)
        ew = O.fill_uniform(n * deg, 7, 0.0, 1.0)
    else:
        rp, col, ew = host_csr
    y1 = y1 if y1 is not None else rv.Buffer(n * layer.hidden_dim * 4)
    layer.forward_exchange(g, x_buf, y1, offsets)

    def inputs(r):
        # only the sample's rows and their neighbours leave HBM (before any timed region)
        nb = col[:rp[r]].astype(np.int64)
        need = np.concatenate([np.arange(r, dtype=np.int64), nb])
        return x_buf.gather_rows(n, d, need), (r + np.arange(nb.size)).astype(np.int32)

    def timed(r):
        h, cols = inputs(r)
        t0 = time.perf_counter()
        ref = O.rvl_forward_graph(W, h, rp[:r + 1], cols, ew[:rp[r]], rows=(0, r), threads=threads)
        return ref, time.perf_counter() - t0

    # calibrate on growing samples until one takes >= half the target, then time a sample
    # sized for the whole target (host copies of the rows are made before each timed call)
    rows, dt = 256, 0.0
    while True:
        _, dt = timed(rows)
        if dt >= 0.5 * cpu_seconds or rows >= n:
            break
        rows = int(min(n, max(2 * rows, rows * 0.6 * cpu_seconds / max(dt, 1e-3))))
    if dt < 0.8 * cpu_seconds and rows < n:
        rows = int(min(n, rows * cpu_seconds / max(dt, 1e-3)))
    ref, dt = timed(rows)
    got = y1.download(np.float32, (rows, layer.hidden_dim))
    del y1
    err, row_err = rel_errs(got, ref)
    edges = int(rp[rows])
    cpu = {"value": round(edges / dt, 1), "unit": "edges/s", "cores": threads, "kind": "port", "host": tinfo,
           "sample": f"oracle RuvectorLayer::forward per node (layer.rs:379-451 restated, {threads} threads) on rows "
                     f"0..{rows} of layer 1 ({edges} edges), {dt:.1f} s"}
    return cpu, {"rows": rows, "max_rel_err": err, "row_rel_l2_max": row_err, "tol": 1e-5,
                 "ok": err <= 1e-5 and row_err <= 1e-5,
                 "metrics": "normwise max|gpu-ref|/max|ref| and per-row ||gpu_r-ref_r||/||ref_r|| (tests/parity.py)"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nodes", type=int, default=2_000_000)
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--degree", type=int, default=32)
    p.add_argument("--heads", type=int, default=8)
    p.add_argument("--layers", type=int, default=3)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--graph", choices=("random", "hnsw"), default="random")
    p.add_argument("--gpus", type=int, default=1, help="ranks to start when no launcher set WORLD_SIZE")
    p.add_argument("--transport", choices=("rccl", "host"), default="rccl")
    a = p.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from benchutil import spawn_ranks  # N ranks as child processes, before any GPU call
        sys.exit(spawn_ranks(a.gpus, os.path.abspath(__file__), sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import ruvector_amd as rv
    from ruvector_amd.shard import comm_from_env

    rv.set_device(local % max(rv.device_count(), 1) if a.transport == "host" else local)
    comm = comm_from_env(a.transport)  # RCCL (TCP rendezvous for the id) or the host socket transport
    log = (lambda s: print(f"[rank {rank}] {s}", file=sys.stderr, flush=True))  # noqa: E731
    line = run(a.nodes, a.dim, a.degree, a.heads, a.layers, a.steps, a.warmup, comm, rank, world, a.graph,
               cpu=not a.no_cpu, cpu_seconds=a.cpu_seconds, log=log)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.barrier()


if __name__ == "__main__":
    main()
