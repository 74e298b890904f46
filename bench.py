#!/usr/bin/env python3
"""Headline benchmark: GNN-layer edges/s of the MI355X GNN-learned-index path.

Workload (BASELINE.json configs[1], per GPU): 1M x 768 node table, uniform
random out-degree-32 CSR, 2-layer ruvector-gnn GraphSAGE-mean forward
(crates/ruvector-postgres/src/gnn/graphsage.rs:118-187) with the reference's
deterministic weights. A step = one full 2-layer forward over every node.
Multi-GPU (one process per GPU, torch.distributed.run): node-range shards of
1M rows per GPU (weak scaling); before each layer the node table is
all-gathered over RCCL/xGMI (the halo of a random graph is the whole graph).

value = (edges x layers over all ranks) / max-over-ranks wall time of K steps,
inputs resident in HBM. Per-kernel device time comes from HIP events on the
library stream (rvx profiler); the CPU baseline is the oracle (the reference
algorithm restated in C++) timed on a bounded sample of rows on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GNN-layer edges/sec + HNSW queries/sec@recall95, 10M×768, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (dense spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--nodes", type=int, default=1_000_000, help="nodes per GPU")
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--degree", type=int, default=32)
    p.add_argument("--layers", type=int, default=2)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu", action="store_true")
    return p.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # host-side only: barrier, id broadcast, max
        dist.init_process_group("gloo")

    import ruvector_amd as rv
    from ruvector_amd.shard import RcclComm, ShardPlan

    rv.set_device(local)
    n_loc, d, deg, layers = a.nodes, a.dim, a.degree, a.layers
    n_tot = n_loc * world
    plan = ShardPlan(n_tot, world)
    r0, r1 = plan.rows(rank)

    comm = None
    if world > 1:
        uid = [RcclComm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = RcclComm(world, rank, uid[0])

    # ---- inputs resident in HBM
    x_loc = rv.Buffer(n_loc * d * 4)
    x_loc.fill_normal(n_loc * d, 3 + rank)
    x_full = rv.Buffer(n_tot * d * 4) if world > 1 else x_loc
    h_loc = [rv.Buffer(n_loc * d * 4) for _ in range(2)]
    h_full = rv.Buffer(n_tot * d * 4) if world > 1 else None
    g = rv.Graph.random_shard(n_tot, r0, n_loc, deg, 4)
    sage = [rv.GraphSAGELayer(d, d, num_samples=deg) for _ in range(layers)]
    rv.synchronize()

    def step():
        src_full, src_loc = x_full, x_loc
        for li, layer in enumerate(sage):
            if world > 1:
                comm.allgather(src_loc, n_loc * d, src_full)
                tbl, off = src_full, r0
            else:
                tbl, off = src_loc, 0
            out = h_loc[li % 2]
            rv._lib.call("rvx_sage_forward_shard_device", layer._h, g.handle, tbl.handle, off, out.handle)
            src_loc = out
            src_full = h_full

    def barrier():
        rv.synchronize()
        if dist is not None:
            dist.barrier()

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
    elapsed = t1 - t0
    kern = prof.summary()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    edges_per_step = n_tot * deg * layers
    value = edges_per_step * a.steps / elapsed

    # ---- roofline of the kernels on the path (HIP events, same stream)
    def rl(name, unit, work_per_launch, peak, bound):
        if name not in kern or kern[name]["launches"] == 0:
            return None
        avg_s = kern[name]["total_ms"] / kern[name]["launches"] / 1e3
        ach = work_per_launch / avg_s / (1e9 if unit == "GB/s" else 1e12)
        return {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
                "traffic": None, "avg_ms": round(avg_s * 1e3, 4), "launches": kern[name]["launches"],
                "work_per_launch": work_per_launch}

    agg_bytes = n_loc * deg * (4 * d + 4) + n_loc * (8 + 4 * d)
    gemm_flops = 2.0 * n_loc * d * (2 * d)
    rls = {"sage_aggregate": rl("sage_aggregate", "GB/s", agg_bytes, HBM_PEAK_GBS, "hbm"),
           "sage_gemm": rl("sage_gemm", "TFLOP/s", gemm_flops, FP32_MFMA_PEAK_TFS, "mfma"),
           "sage_normalize": rl("sage_normalize", "GB/s", 2 * n_loc * d * 4, HBM_PEAK_GBS, "hbm")}
    if comm is not None and "rccl_allgather" in kern:
        rls["rccl_allgather"] = rl("rccl_allgather", "GB/s", (world - 1) * n_loc * d * 4, 7 * 153.0, "xgmi")
    dom = max((k for k in rls if rls[k]), key=lambda k: kern[k]["total_ms"])
    attach_pmc_traffic(rls, {"nodes_per_gpu": n_loc, "dim": d, "degree": deg, "layers": layers})

    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: X ~ N(0,1) Box-Muller on device (seed 3+rank); uniform random out-degree CSR (seed 4); "
                "GraphSAGE deterministic init (graphsage.rs:56-78)",
        "config": {"workload": "configs[1]: 1M x 768 2-layer ruvector-gnn GraphSAGE-mean forward per GPU; "
                               "node-range shards + RCCL all-gather halo for N>1",
                   "nodes_per_gpu": n_loc, "nodes_total": n_tot, "dim": d, "degree": deg, "layers": layers,
                   "edges_per_step": edges_per_step, "parallelism": f"node-range x{world}"},
        "roofline": dict(rls[dom], kernel=dom),
        "roofline_kernels": {k: v for k, v in rls.items() if v},
        "kernel_ms": {k: round(v["total_ms"] / max(v["launches"], 1), 4) for k, v in kern.items()},
    }

    if rank == 0 and world == 1 and not a.no_cpu:
        line["cpu_baseline"], line["parity"] = cpu_baseline(a, x_loc, g, h_loc[0], sage, n_loc, d, deg)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def attach_pmc_traffic(rls, cfg):
    """HBM bytes per launch from the committed rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE
    passes of this same workload (profiles/pmc_traffic_latest.json, gfx950 FETCH
    correction applied by scripts/pmc_traffic.py); left null when the profile was
    taken on a different configuration."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic_latest.json")
    if not os.path.exists(path):
        return
    try:
        pmc = json.load(open(path))
    except ValueError:
        return
    pc = pmc.get("config") or {}
    if any(pc.get(k) != v for k, v in cfg.items()):
        return
    for tag, r in rls.items():
        ent = pmc.get("kernels", {}).get(tag)
        if r is not None and ent and r["unit"] == "GB/s":
            r["traffic"] = round(ent["hbm_bytes_per_launch"], 0)
            r["traffic_source"] = "rocprofv3 --pmc FETCH_SIZE(x2, gfx950) + WRITE_SIZE, profiles/pmc_traffic_latest.json"
        elif r is not None and ent:
            r["traffic"] = round(ent["hbm_bytes_per_launch"], 0)
            r["traffic_source"] = "rocprofv3 --pmc (HBM bytes per launch; MFMA-bound kernel)"


def cpu_baseline(a, x_buf, g, h1_buf, sage, n, d, deg):
    """Oracle (reference algorithm, C++) on a bounded sample of layer-1 rows."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    import ruvector_amd as rv

    threads = min(16, os.cpu_count() or 1)
    x = x_buf.download(np.float32, (n, d))
    rp, col = O.random_csr(n, deg, 4)
    wn, ws = O.sage_init(d, d, 0), O.sage_init(d, d, 1000)
    # layer-1 GPU output for the whole graph (single forward, outside the timed region)
    rv._lib.call("rvx_sage_forward_shard_device", sage[0]._h, g.handle, x_buf.handle, 0, h1_buf.handle)
    rows = 2048
    t0 = time.perf_counter()
    O.sage_forward(x, rp, col, wn, ws, rows=(0, rows), threads=threads)
    dt = time.perf_counter() - t0
    rows = int(min(n, max(rows, rows * a.cpu_seconds / max(dt, 1e-3))))
    t0 = time.perf_counter()
    ref = O.sage_forward(x, rp, col, wn, ws, rows=(0, rows), threads=threads)
    dt = time.perf_counter() - t0
    got = h1_buf.download(np.float32, (rows, d))
    err = float(np.max(np.abs(got.astype(np.float64) - ref)) / max(float(np.max(np.abs(ref))), 1e-30))
    cpu = {"value": round(rows * deg / dt, 1), "unit": "edges/s", "cores": threads, "kind": "port",
           "sample": f"oracle GraphSAGE-mean layer 1 (graphsage.rs:118-187 restated, AVX2, {threads} threads) on "
                     f"rows 0..{rows} of the same 1M x 768 graph, {dt:.1f} s"}
    parity = {"rows": rows, "max_rel_err": err, "tol": 1e-5, "ok": err <= 1e-5}
    return cpu, parity


if __name__ == "__main__":
    main()
