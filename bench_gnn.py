#!/usr/bin/env python3
"""C4 benchmark: multi-layer ruvector-gnn RuvectorLayer stack +
EdgeFeaturedAttention head over a graph, one process per GPU (node-range shards,
launched with torch.distributed.run for N>1 — the processes use no torch; rows exchanged over RCCL p2p).

Workload: N x 768 node table (N(0,1), seed 5), uniform random out-degree-32
CSR (seed 6) with edge weights uniform [0,1) (seed 7) standing in for the HNSW
layer-0 graph; `--layers` x RuvectorLayer(768, 768, heads=8, dropout=0, seeded
init) (crates/ruvector-gnn/src/layer.rs:313-457), then EdgeFeaturedAttention
(node_dim 768, edge_dim 1 = the edge weight, 8 heads, concat, slope 0.2;
crates/ruvector-attention/src/graph/edge_featured.rs:87-320).

value = (edges x (layers + 1)) / wall time of one forward of the stack, inputs
resident in HBM. Per-kernel times are HIP events stamped by the dispatch
packets. CPU baseline: the oracle's RuvectorLayer restatement on a bounded
sample of layer-1 rows (16 threads), with a parity check on the same rows.
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
    from ruvector_amd.attention import EdgeFeaturedAttention, EdgeFeaturedConfig
    from ruvector_amd.shard import REDUCE_MAX, ShardPlan, comm_from_env

    rv.set_device(local % max(rv.device_count(), 1) if a.transport == "host" else local)
    n, d, deg, H = a.nodes, a.dim, a.degree, a.dim
    plan = ShardPlan(n, world)
    r0, r1 = plan.rows(rank)
    n_loc = r1 - r0
    offsets = np.array([plan.rows(p)[0] for p in range(world)] + [n], dtype=np.int64)
    comm = comm_from_env(a.transport)  # RCCL (TCP rendezvous for the id) or the host socket transport

    # node-range shards: every rank holds the whole-table buffers but reads and
    # writes only its own rows; its CSR rows (global column ids) and their slice
    # of the edge-weight stream are generated in place, so the sharded job is
    # the same graph as the 1-GPU one
    E = n * deg
    x = rv.Buffer(n * d * 4)
    x.fill_normal(n * d, 5)
    g = rv.Graph.random_shard(n, r0, n_loc, deg, 6, weight_seed=7)
    ew = g._keep[2]  # [E_local][1] edge features = the edge weights
    layers = [rv.RuvectorLayer(d, H, a.heads, 0.0, seed=100 + i) for i in range(a.layers)]
    head = EdgeFeaturedAttention(EdgeFeaturedConfig(node_dim=H, edge_dim=1, num_heads=a.heads))
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

    for _ in range(a.warmup):
        step()
    barrier()
    prof = rv.Profiler()
    with prof:
        barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        rv.synchronize()
        t1 = time.perf_counter()
        barrier()
    dt = (t1 - t0) / a.steps
    kern = prof.summary()
    if comm is not None:
        dt = comm.allreduce([dt], REDUCE_MAX)[0]
    n_own = n_loc  # per-launch work below is this rank's rows

    # algorithmic work per layer
    layer_flops = 2.0 * n_own * (d * H + 11 * H * H)
    edge_bytes = n_own * deg * (3 * 4 * H + 8) + n_own * (8 + 4 * H + 2 * 4 * H)
    gemm_ms = sum(v["total_ms"] for k, v in kern.items() if k.startswith("gnn_gemm")) / a.steps / a.layers
    edge_ms = kern.get("gnn_edge_attention", {"total_ms": 0})["total_ms"] / a.steps / a.layers
    roof = {
        "gnn_gemm (all dense layers of one RuvectorLayer)": {
            "bound": "mfma", "achieved": round(layer_flops / (gemm_ms / 1e3) / 1e12, 2), "peak": round(GEMM_PEAK_TFS, 1),
            "unit": "TFLOP/s", "frac": round(layer_flops / (gemm_ms / 1e3) / 1e12 / GEMM_PEAK_TFS, 4),
            "ms_per_layer": round(gemm_ms, 3)},
        "gnn_edge_attention": {
            "bound": "hbm", "achieved": round(edge_bytes / (edge_ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(edge_bytes / (edge_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "ms_per_layer": round(edge_ms, 3)},
    }
    line = {
        "metric": "GNN-layer edges/sec (RuvectorLayer stack + graph-attention head)",
        "value": round(E * (a.layers + 1) / dt, 1), "unit": "edges/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "scaling": "strong", "dtype": "f32",
        "config": {"workload": f"configs[3] stack on {world} GPU(s): {n} x {d}, {a.layers} x RuvectorLayer(h={a.heads})"
                               " + EdgeFeaturedAttention(8 heads, edge_dim 1)", "nodes": n, "degree": deg,
                   "edges": E, "layers": a.layers, "parallelism": f"node-range x{world}",
                   "exchange": "per layer: M|K|V rows (RuvectorLayer), T rows (attention head), "
                               "one grouped RCCL p2p round each" if world > 1 else "none"},
        "data": "synthetic: X ~ N(0,1) seed 5; uniform random out-degree CSR seed 6; edge weights U[0,1) seed 7",
        "roofline": roof,
        "kernel_ms_per_step": {k: round(v["total_ms"] / a.steps, 3) for k, v in kern.items()},
    }
    if rank == 0 and world == 1 and not a.no_cpu:
        line["cpu_baseline"], line["parity"] = cpu_baseline(a, x, g, ew, layers[0], n, d, deg, offsets)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.barrier()


def cpu_baseline(a, x_buf, g, ew_buf, layer, n, d, deg, offsets):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    import ruvector_amd as rv

    threads = min(16, os.cpu_count() or 1)
    W = O.RvlWeights(json.loads(layer.to_json()))
    x = x_buf.download(np.float32, (n, d))
    rp, col = O.random_csr(n, deg, 6)
    ew = O.fill_uniform(n * deg, 7, 0.0, 1.0)
    y1 = rv.Buffer(n * layer.hidden_dim * 4)
    layer.forward_exchange(g, x_buf, y1, offsets)
    rows = 64
    t0 = time.perf_counter()
    O.rvl_forward_graph(W, x, rp, col, ew, rows=(0, rows), threads=threads)
    dt = time.perf_counter() - t0
    rows = int(min(n, max(rows, rows * a.cpu_seconds / max(dt, 1e-3))))
    t0 = time.perf_counter()
    ref = O.rvl_forward_graph(W, x, rp, col, ew, rows=(0, rows), threads=threads)
    dt = time.perf_counter() - t0
    got = y1.download(np.float32, (rows, layer.hidden_dim))
    from bench import rel_errs
    err, row_err = rel_errs(got, ref)
    cpu = {"value": round(rows * deg / dt, 1), "unit": "edges/s", "cores": threads, "kind": "port",
           "sample": f"oracle RuvectorLayer::forward per node (layer.rs:379-451 restated, {threads} threads) on rows "
                     f"0..{rows} of layer 1, {dt:.1f} s"}
    return cpu, {"rows": rows, "max_rel_err": err, "row_rel_l2_max": row_err, "tol": 1e-5,
                 "ok": err <= 1e-5 and row_err <= 1e-5,
                 "metrics": "normwise max|gpu-ref|/max|ref| and per-row ||gpu_r-ref_r||/||ref_r|| (tests/parity.py)"}


if __name__ == "__main__":
    main()
