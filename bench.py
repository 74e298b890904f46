#!/usr/bin/env python3
"""Headline benchmark: GNN-layer edges/s (+ HNSW queries/s@recall95) of the
MI355X GNN-learned-index path.

Workload (BASELINE.json metric "10M x 768, 1/2/4/8 MI355X"; the configs[1]
layer stack at configs[2]/[3] scale): a 10M x 768 node table, uniform random
out-degree-32 CSR, 2-layer ruvector-gnn GraphSAGE-mean forward
(crates/ruvector-postgres/src/gnn/graphsage.rs:118-187) with the reference's
deterministic weights. A step = one full 2-layer forward over every node.

Multi-GPU (one process per GPU: `--gpus N` starts the N ranks itself as child
processes, or a launcher such as torch.distributed.run does and sets WORLD_SIZE;
the processes use no torch: RCCL id over a TCP rendezvous, barriers and the
max-over-ranks clock as RCCL all-reduces; `--transport host` moves the same
exchange rounds through host memory and stdlib sockets so N ranks can share one
GPU): the 10M nodes are split into contiguous node-id ranges (strong scaling).
At N > 1 the run checks itself: every rank's copy of the exchanged layer-1 table
must have the same checksum, and the last rank's rows are compared with the
oracle (layer 1 on rank 0 from its exchanged copy, layer 2 on the last rank). The input node table is
resident on every GPU; each layer writes its owned rows of the next table and
ships them to every peer over RCCL p2p (xGMI) chunk by chunk while the
remaining chunks compute (rvx_sage_forward_exchange); the last layer's rows
stay local. value = (edges x layers) / max-over-ranks wall time of K steps.

Per-kernel device time comes from HIP events stamped by the dispatch packets
(rvx profiler); the CPU baseline is the oracle (the reference algorithm
restated in C++) timed on a bounded sample of rows on rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GNN-layer edges/sec + HNSW queries/sec@recall95, 10M\u00d7768, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (dense spec)
BF16_MFMA_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (spec)
# The layer GEMM runs as split-f16 MFMA (gemm_f32.hip gemm_nt_h2g): operands
# scaled by powers of two and split into two f16 parts, 3 f16 partial products
# per f32 product accumulated in f32 (f16 MFMA = the bf16 rate), so its ceiling
# in f32-equivalent FLOP/s is the f16/bf16 peak / 3. RVX_GEMM_H2=0 selects the
# split-bf16 GEMM (6 products, peak / 6); RVX_GEMM_X3=0 too, the FP32 MFMA
# kernel (ceiling 157.3 TF).
GEMM_H2 = os.environ.get("RVX_GEMM_H2", "1") != "0"
GEMM_X3 = os.environ.get("RVX_GEMM_X3", "1") != "0"
GEMM_PEAK_TFS = (BF16_MFMA_PEAK_TFS / 3 if GEMM_H2 else
                 BF16_MFMA_PEAK_TFS / 6 if GEMM_X3 else FP32_MFMA_PEAK_TFS)
GEMM_DESC = ("split-f16 MFMA (per-row/column power-of-two operand scaling, two f16 parts per f32 operand, 3 partial "
             "products a2b1+a1b2+a1b1, f32 accumulate; <= 2^-21 relative error per product), peak = 2.5 PF f16 / 3"
             if GEMM_H2 else
             "split-bf16 MFMA (exact 3-way bf16 split of each f32 operand, 6 partial products, f32 accumulate; "
             "f32 GEMM to within 2^-23 per product), peak = 2.5 PF bf16 / 6" if GEMM_X3 else
             "FP32 MFMA v_mfma_f32_32x32x2_f32")
XGMI_PEAK_GBS = 7 * 153.0    # 7 xGMI links x ~153 GB/s per direction per GPU
PIPELINE = ("row chunks x48 (>=786432 rows), gather (1 block/CU, rows from a per-chunk counter) on aux stream "
            "overlapping the GEMM (persistent 256x192 tiles, 1 block/CU) of the previous chunk, whose blocks take "
            "rows of that gather once their tiles are done (RVX_SAGE_HELP=1): sage_aggregate's duration is the "
            "chunk's gather completion and sage_gemm's includes the gather rows it took, so its TFLOP/s understates "
            "the GEMM")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--nodes", type=int, default=10_000_000, help="total nodes (split over GPUs)")
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--degree", type=int, default=32)
    p.add_argument("--layers", type=int, default=2)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-hnsw", action="store_true", help="skip the HNSW queries/s@recall95 leg")
    p.add_argument("--no-scan", action="store_true", help="skip the 10M x 768 exact-scan queries/s leg")
    p.add_argument("--no-c4", action="store_true", help="skip the C4 leg (3 x RuvectorLayer + graph-attention head)")
    p.add_argument("--no-c3", action="store_true", help="skip the C3 leg (HNSW build + search + GNN re-rank on the table)")
    p.add_argument("--c3-ef", default="100,400,1600", help="C3 leg: ef sweep")
    p.add_argument("--c4-nodes", type=int, default=0, help="C4 leg nodes (default: --nodes)")
    p.add_argument("--no-c5", action="store_true", help="skip the C5 leg (hyperbolic HNSW, node-range sharded)")
    p.add_argument("--c5-per-gpu", type=int, default=6_250_000,
                   help="C5 leg points per GPU shard (6.25M = the 50M x 1024 corpus over 8 GPUs; weak scaling)")
    p.add_argument("--transport", choices=("rccl", "host"), default="rccl",
                   help="N>1 exchange: RCCL over xGMI, or host memory + stdlib sockets (ranks may share a GPU)")
    p.add_argument("--check-rows", type=int, default=8192, help="N>1: oracle-checked rows of the last rank")
    p.add_argument("--force-comm", action="store_true",
                   help="N=1: build the RCCL communicator anyway and run every exchange round through it "
                        "(RVX_COMM_SELF_P2P=1: grouped send/recv to the rank itself), so the RCCL barriers, "
                        "clock all-reduce and p2p rounds run on a one-GPU box")
    return p.parse_args()


_STAGE = ["start"]


def _progress(stage):
    """Name the leg that runs now; a daemon thread prints it to stderr every minute so a
    supervisor watching the output sees a long leg (the C3 build, the C4 stack) alive."""
    _STAGE[0] = stage
    print(f"[bench] {stage}", file=sys.stderr, flush=True)


def _start_progress_thread():
    import threading
    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(60.0)
            print(f"[bench] ... {_STAGE[0]} ({time.perf_counter() - t0:.0f} s)", file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here, before anything touches the GPU
        from benchutil import spawn_ranks
        sys.exit(spawn_ranks(a.gpus, os.path.abspath(__file__), sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rank == 0:
        _start_progress_thread()
    import ruvector_amd as rv
    from ruvector_amd.shard import REDUCE_MAX, ShardPlan, comm_from_env, comm_traffic

    # host transport: ranks may outnumber the GPUs and share them
    rv.set_device(local % max(rv.device_count(), 1) if a.transport == "host" else local)
    n_tot, d, deg, layers = a.nodes, a.dim, a.degree, a.layers
    plan = ShardPlan(n_tot, world)
    r0, r1 = plan.rows(rank)
    n_loc = r1 - r0
    offsets = np.array([plan.rows(p)[0] for p in range(world)] + [n_tot], dtype=np.int64)
    off_ptr = offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))

    # RCCL communicator: id over a stdlib TCP rendezvous, barriers and the
    # max-over-ranks clock as RCCL all-reduces (no other collective library);
    # or the host-staged socket transport
    comm = comm_from_env(a.transport)
    forced = False
    if comm is None and a.force_comm:
        from ruvector_amd.shard import RcclComm, rendezvous_unique_id
        os.environ["RVX_COMM_SELF_P2P"] = "1"
        comm = RcclComm(1, 0, rendezvous_unique_id(0, 1, RcclComm.unique_id))
        forced = True

    # ---- inputs resident in HBM: the node table (same on every GPU), this
    # rank's CSR rows (global column ids), two full tables for layer outputs
    x = rv.Buffer(n_tot * d * 4)
    x.fill_normal(n_tot * d, 3)
    tables = [rv.Buffer(n_tot * d * 4) for _ in range(min(layers, 2))]
    # Layer l's L2 normalisation is carried into layer l+1 (rvx_sage_forward_exchange2:
    # the unnormalised rows and 1/|y| per row, exchanged together) instead of a pass that
    # re-reads and re-writes the table; the last layer normalises in place. RVX_SAGE_DEFER=0
    # runs every layer with its own pass.
    defer = layers > 1 and os.environ.get("RVX_SAGE_DEFER", "1") != "0"
    invs = [rv.Buffer(n_tot * 4) for _ in range(2)] if defer else None
    # RVX_SAGE_IMAGE=1 (opt-in): layer l (< last) also writes a ReLU-sparse image of its output
    # rows (rvx_row_image_pack: a 3 KiB slot of the values other than +0.0 per row), from which
    # layer l+1's overlapped gather reads its neighbour rows — same terms, same order, same bits,
    # 46% fewer bytes; beside the GEMM the expansion through LDS costs what the bytes save
    # (DESIGN.md §4.3), so the default gathers from the dense table.
    use_img = layers > 1 and 512 < d <= 768 and d % 4 == 0 and os.environ.get("RVX_SAGE_IMAGE", "0") == "1"
    imgs = [rv.row_image(n_tot, d) for _ in range(min(layers - 1, 2))] if use_img else None
    g = rv.Graph.random_shard(n_tot, r0, n_loc, deg, 4)
    sage = [rv.GraphSAGELayer(d, d, num_samples=deg) for _ in range(layers)]
    rv.synchronize()

    def step():
        src = x
        for li, layer in enumerate(sage):
            dst = tables[li % 2]
            xm = invs[(li - 1) % 2].handle if defer and li > 0 else None
            yi = invs[li % 2].handle if defer and li < layers - 1 else None
            xi = imgs[(li - 1) % 2].handle if use_img and li > 0 else None
            yimg = imgs[li % 2].handle if use_img and li < layers - 1 else None
            rv._lib.call("rvx_sage_forward_exchange3", layer._h, g.handle, src.handle, xm, xi, dst.handle, yi, yimg,
                         off_ptr, comm._h if comm else None, int(li < layers - 1))
            src = dst

    def barrier():
        rv.synchronize()
        if comm is not None:
            comm.barrier()

    _progress("graphsage headline")
    for _ in range(a.warmup):
        step()
    barrier()
    prof = rv.Profiler()
    traffic0 = comm_traffic(comm) if comm is not None else (0, 0)
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
    traffic = tuple(v - v0 for v, v0 in zip(comm_traffic(comm), traffic0)) if comm is not None else (0, 0)
    if comm is not None:
        elapsed = comm.allreduce([elapsed], REDUCE_MAX)[0]

    edges_per_step = n_tot * deg * layers
    value = edges_per_step * a.steps / elapsed

    # ---- roofline of the kernels on the path. Layers run as a row-chunked
    # two-stream pipeline (gather of chunk c+1 overlaps the GEMM of chunk c),
    # so a kernel launches several times per layer; work per launch = work per
    # step x steps / launches (this rank's rows).
    def rl(name, unit, work_per_step, peak, bound):
        if name not in kern or kern[name]["launches"] == 0:
            return None
        work_per_launch = work_per_step * a.steps / kern[name]["launches"]
        avg_s = kern[name]["total_ms"] / kern[name]["launches"] / 1e3
        ach = work_per_launch / avg_s / (1e9 if unit == "GB/s" else 1e12)
        return {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
                "traffic": None, "avg_ms": round(avg_s * 1e3, 4), "launches": kern[name]["launches"],
                "work_per_launch": work_per_launch}

    agg_bytes = n_loc * deg * (4 * d + 4) + n_loc * (8 + 4 * d)   # per layer, dense neighbour rows
    gemm_flops = 2.0 * n_loc * d * (2 * d)
    norm_bytes = 2 * n_loc * d * 4
    norm_layers = 1 if defer else layers  # carried normalisation: only the last layer runs the pass
    agg_total, img_info, pack_bytes = agg_bytes * layers, None, 0
    if use_img:
        # layers >= 2 read imaged neighbour rows: per edge the record the gather loads (16-B
        # granules of header + values; the dense row where the slot holds none) + column id +
        # count; the image's mean over every row of the table (the graph is uniform random)
        nnz = imgs[0].download(np.uint16, (n_tot,), offset=n_tot * 3072).astype(np.int64)
        rec = np.where(nnz <= 736, (128 + 4 * nnz + 15) // 16 * 16, 4 * d)
        rec_mean = float(rec.mean())
        agg_img = n_loc * deg * (rec_mean + 4 + 2) + n_loc * (8 + 4 * d)
        agg_total = agg_bytes + agg_img * (layers - 1)
        pack_bytes = n_tot * (4 * d + rec_mean + 2) * (layers - 1)  # every row imaged where it lands
        img_info = {"mean_nnz": round(float(nnz.mean()), 1), "rows_in_slots": round(float((nnz <= 736).mean()), 4),
                    "mean_record_bytes": round(rec_mean, 1), "dense_row_bytes": 4 * d,
                    "gather_bytes_per_layer": {"dense": agg_bytes, "imaged": round(agg_img)}}
    rls = {"sage_aggregate": rl("sage_aggregate", "GB/s", agg_bytes * (1 if use_img else layers), HBM_PEAK_GBS, "hbm"),
           "sage_gemm": rl("sage_gemm", "TFLOP/s", gemm_flops * layers, GEMM_PEAK_TFS, "mfma"),
           "sage_normalize": rl("sage_normalize", "GB/s", norm_bytes * norm_layers, HBM_PEAK_GBS, "hbm")}
    if use_img:  # layers >= 2 gather from the image (their own tag)
        rls["sage_aggregate_img"] = rl("sage_aggregate_img", "GB/s", agg_img * (layers - 1), HBM_PEAK_GBS, "hbm")
        rls["rows_image_pack"] = rl("rows_image_pack", "GB/s", pack_bytes, HBM_PEAK_GBS, "hbm")
    if comm is not None:
        rls["halo_exchange"] = rl("halo_exchange", "GB/s", (n_tot - n_loc) * d * 4 * (layers - 1), XGMI_PEAK_GBS,
                                  "xgmi")
    dom = max((k for k in rls if rls[k] and k != "halo_exchange"), key=lambda k: kern[k]["total_ms"])
    pmc_cfg = {"nodes_total": n_tot, "dim": d, "degree": deg, "layers": layers,
               "parallelism": f"node-range x{world}", "pipeline": PIPELINE}
    if use_img:
        pmc_cfg["row_image"] = True  # profiles of the dense-gather pipeline do not apply
    attach_pmc_traffic(rls, pmc_cfg)
    # whole-layer floor: HBM and MFMA work overlap, so a layer cannot beat the
    # larger of the two floors
    layer_ms = elapsed / a.steps / layers * 1e3
    hbm_floor = (agg_total / layers + norm_bytes * norm_layers / layers) / (HBM_PEAK_GBS * 1e9) * 1e3
    mfma_floor = gemm_flops / (GEMM_PEAK_TFS * 1e12) * 1e3
    layer_rl = {"layer_ms": round(layer_ms, 3), "hbm_floor_ms": round(hbm_floor, 3),
                "mfma_floor_ms": round(mfma_floor, 3), "frac": round(max(hbm_floor, mfma_floor) / layer_ms, 4)}

    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "gemm_dtype": "split-f16x3" if GEMM_H2 else "split-bf16x6" if GEMM_X3 else "fp32",
        "gemm": GEMM_DESC,
        "data": "synthetic: X ~ N(0,1) Box-Muller on device (seed 3); uniform random out-degree CSR (seed 4); "
                "GraphSAGE deterministic init (graphsage.rs:56-78)",
        "config": {"workload": "10M x 768 2-layer ruvector-gnn GraphSAGE-mean forward (configs[1] layers at the "
                               "metric's 10M scale); node-range shards + chunked RCCL p2p halo exchange for N>1",
                   "nodes_total": n_tot, "nodes_per_gpu": n_loc, "dim": d, "degree": deg, "layers": layers,
                   "edges_per_step": edges_per_step, "parallelism": f"node-range x{world}",
                   "pipeline": PIPELINE,
                   "normalisation": ("layer l's L2 normalisation carried into layer l+1 as 1/|y| per row "
                                     "(rvx_sage_forward_exchange2); the last layer normalises in place")
                   if defer else "every layer normalises in place",
                   "row_image": (dict(img_info, note="layer l+1 gathers layer l's ReLU-sparse rows from a packed "
                                      "image (rvx_sage_forward_exchange3; same bits as the dense gather)")
                                 if use_img else "off")},
        "roofline": dict(rls[dom], kernel=dom),
        "roofline_kernels": {k: v for k, v in rls.items() if v},
        "roofline_layer": layer_rl,
        "kernel_ms": {k: round(v["total_ms"] / max(v["launches"], 1), 4) for k, v in kern.items()},
    }

    if comm is not None:
        line["comm"] = {"transport": a.transport, "forced": forced,
                        "self_p2p_rounds": kern.get("halo_exchange", {}).get("launches", 0) if forced else 0}
        if forced:  # the compact records' RCCL round trip + unpack, checked word for word (rvx_comm_selfcheck)
            from ruvector_amd.shard import comm_selfcheck
            rows_chk, bad = comm_selfcheck(comm)
            line["comm"]["record_selfcheck"] = {"rows": rows_chk, "mismatched_words": bad}
        line["multi_gpu"] = exchange_report(a, kern, comm, world, rank, offsets, d, layers, traffic)
        line["multi_gpu"]["transport"] = ("rccl (p2p over xGMI)" if a.transport == "rccl" else
                                          "host-staged (host memory + stdlib TCP sockets)")
        line["parity"] = multi_rank_check(a, comm, rank, world, offsets, x, tables, invs, n_tot, d, deg, layers)
    if rank == 0 and world == 1 and not a.no_cpu:
        _progress("graphsage cpu baseline + parity")
        line["cpu_baseline"], line["parity"] = cpu_baseline(a, x, g, tables, n_tot, d, deg, layers, invs)
    if world == 1:
        line["gemm_paths"] = gemm_alternatives(g, x, tables[0], off_ptr, d, deg)
    del tables, g, invs
    if not a.no_scan:
        _progress("exact scan leg")
        line["exact_scan"] = scan_leg(a, x, n_tot, d, rank, world, comm)
        rv.release_scratch()
    if not a.no_c3:
        _progress("c3 leg (HNSW build, search, re-rank)")
        line["c3"] = c3_leg(a, x, n_tot, d, rank, world, comm)
    del x
    rv.release_scratch()  # the C4 leg needs ~235 GB of the 288 GB at 10M x 768
    if not a.no_c4:
        _progress("c4 leg")
        line["c4"] = c4_leg(a, comm, rank, world)
        rv.release_scratch()
    if not a.no_c5:
        _progress("c5 leg (hyperbolic HNSW shards: build, exact + pruned search)")
        line["c5"] = c5_leg(a, comm, rank, world)
        rv.release_scratch()
    if not a.no_hnsw:
        _progress("c1 hnsw leg")
        line["hnsw"] = hnsw_leg(a, rank, world, comm)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.barrier()


def multi_rank_check(a, comm, rank, world, offsets, x, tables, invs, n_tot, d, deg, layers):
    """Self-check of a multi-rank run (after the timed steps, on the last step's tables):
    * agreement: every rank's copy of the exchanged layer-1 table (and its 1/|y| column
      when the normalisation is carried) has the same 64-bit checksum (device kernel);
    * layer 1: rank 0 compares `check_rows` rows owned by the LAST rank, as they arrived
      over the exchange, with the oracle (per-row and normwise, tests/parity.py metrics);
    * layer 2: the last rank compares the same rows of its own output, computed from its
      exchanged layer-1 table.
    Inputs: x rows gathered from HBM; the CSR rows from the oracle's own generator."""
    from ruvector_amd.shard import REDUCE_MAX, REDUCE_MIN
    if layers < 2:
        return {"ok": None, "note": "one layer: nothing is exchanged"}
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from benchutil import host_threads

    cs = [tables[0].checksum(n_tot * d * 4)] + ([invs[0].checksum(n_tot * 4)] if invs else [])
    halves = [float(v) for c in cs for v in (c & 0xFFFFFFFF, c >> 32)]
    agree = comm.allreduce(halves, REDUCE_MAX) == comm.allreduce(halves, REDUCE_MIN)

    last = world - 1
    a0 = int(offsets[last])
    rows = int(min(a.check_rows, int(offsets[last + 1]) - a0))
    errs = [0.0, 0.0, 0.0, 0.0]
    if rank in (0, last) and rows > 0:
        threads, _ = host_threads()
        rp, col = O.random_csr(n_tot, deg, 4)
        wn, ws = O.sage_init(d, d, 0), O.sage_init(d, d, 1000)
        nb = col[rp[a0]:rp[a0 + rows]].astype(np.int64)
        need = np.concatenate([np.arange(a0, a0 + rows, dtype=np.int64), nb])
        rp_sub = (rp[a0:a0 + rows + 1] - rp[a0]).astype(np.int64)
        col_sub = (rows + np.arange(nb.size)).astype(np.int32)
        inv = invs[0].download(np.float32, (n_tot,)) if invs else None

        def layer1_rows(ids):
            r = tables[0].gather_rows(n_tot, d, ids)
            return (r * inv[ids][:, None]).astype(np.float32) if inv is not None and layers > 1 else r

        if rank == 0:  # layer 1 of the last rank's rows, as rank 0 received them
            ref = O.sage_forward(x.gather_rows(n_tot, d, need), rp_sub, col_sub, wn, ws, rows=(0, rows),
                                 threads=threads)
            errs[0], errs[1] = rel_errs(layer1_rows(np.arange(a0, a0 + rows)), ref)
        if rank == last and layers > 1:  # layer 2 of its own rows from its exchanged layer-1 table
            ref = O.sage_forward(layer1_rows(need), rp_sub, col_sub, wn, ws, rows=(0, rows), threads=threads)
            got = tables[1 % len(tables)].gather_rows(n_tot, d, np.arange(a0, a0 + rows))
            errs[2], errs[3] = rel_errs(got, ref)
    errs = comm.allreduce(errs, REDUCE_MAX)
    worst = max(errs)
    return {"ok": bool(agree and worst <= 1e-5), "tol": 1e-5, "max_rel_err": max(errs[0], errs[2]),
            "row_rel_l2_max": max(errs[1], errs[3]),
            "tables_agree": bool(agree), "table_checksums": [f"{c:016x}" for c in cs],
            "checked_rows": {"owner_rank": last, "rows": [a0, a0 + rows]},
            "per_layer": [{"layer": 1, "checked_on_rank": 0, "max_rel_err": errs[0], "row_rel_l2_max": errs[1],
                           "input": "x (HBM); rows received over the exchange"},
                          {"layer": 2, "checked_on_rank": last, "max_rel_err": errs[2], "row_rel_l2_max": errs[3],
                           "input": "the last rank's exchanged layer-1 table"}],
            "metrics": "max_rel_err = max|gpu-ref| / max|ref|; row_rel_l2_max = max over rows of "
                       "||gpu_r-ref_r||_2 / ||ref_r||_2 (tests/parity.py); tables_agree: every rank's "
                       "exchanged layer-1 table (and 1/|y|) has the same checksum"}


def exchange_report(a, kern, comm, world, rank, offsets, d, layers, traffic):
    """Per-rank view of the halo exchange (the 8-GPU bottleneck candidate): bytes each rank
    handed to / took from the transport per exchanged layer over the timed steps, as the
    library counted them (rvx_comm_traffic: the compact row records, their counts, 1/|y| and
    the dense rows of records past the slot), beside the dense-row bytes; the transfer
    stream's exchange time and the exposed tail the compute stream waits for (rvx profiler
    tag exchange_wait: from the last chunk's compute to the last round's arrival), per layer,
    for every rank."""
    exchanged = max(layers - 1, 0)
    n_loc = int(offsets[rank + 1] - offsets[rank])
    n_tot = int(offsets[-1])

    def per_rank(v):  # every rank's value, via one RCCL sum of a one-hot vector
        vec = [0.0] * world
        vec[rank] = float(v)
        return comm.allreduce(vec)

    def ms_per_layer(tag):
        k = kern.get(tag)
        return (k["total_ms"] / a.steps / max(exchanged, 1)) if k else 0.0

    wait = per_rank(ms_per_layer("exchange_wait"))
    xfer = per_rank(ms_per_layer("halo_exchange"))
    per_layer = max(a.steps * exchanged, 1)
    sent = per_rank(traffic[0] / per_layer)
    recv = per_rank(traffic[1] / per_layer)
    dense_sent = [int(offsets[p + 1] - offsets[p]) * (d * 4 + 4) * (world - 1) for p in range(world)]
    return {"exchanged_layers_per_step": exchanged,
            "bytes_sent_per_layer": [int(v) for v in sent],
            "bytes_recv_per_layer": [int(v) for v in recv],
            "dense_bytes_sent_per_layer": dense_sent,
            "sent_vs_dense": [round(s_ / max(d_, 1), 4) for s_, d_ in zip(sent, dense_sent)],
            "format": ("compact ReLU-sparse row records (bitmap + values other than +0.0, back to back within a "
                       "per-round byte budget agreed from chunk 0, expanded bit for bit on arrival; rows past the "
                       "budget sent dense after the rounds)"
                       if os.environ.get("RVX_XCHG_IMAGE", "1") != "0" and 512 < d <= 768 and d % 4 == 0
                       else "dense rows"),
            "exchange_ms_per_layer": [round(v, 3) for v in xfer],
            "exchange_wait_ms_per_layer": [round(v, 3) for v in wait],
            "note": "exchange_ms: transfer-stream time of the chunked RCCL p2p rounds (overlapped with compute); "
                    "exchange_wait: the part the compute stream waited for after its last chunk"}


def c4_leg(a, comm, rank, world):
    """configs[3] at the metric's scale: 3 x RuvectorLayer(768, h 8) + EdgeFeaturedAttention
    (8 heads, edge_dim 1) over the --nodes x 768 table and a uniform random out-degree-32
    graph with U[0,1) edge features (bench_gnn.run; `bench_gnn.py --graph hnsw` runs it on
    a GPU-built HNSW layer-0 graph), node-range sharded at N > 1 with the M|K|V and T rows
    exchanged per layer. 1 warm-up + 2 timed forwards; roofline of the layer GEMMs and
    the edge kernel; CPU baseline and per-row parity of layer 1 on rank 0 at N = 1."""
    import bench_gnn
    n = a.c4_nodes or a.nodes
    return bench_gnn.run(n, a.dim, a.degree, 8, 3, steps=2, warmup=1, comm=comm, rank=rank, world=world,
                         graph="random", cpu=(rank == 0 and world == 1 and not a.no_cpu), cpu_seconds=8.0)


def c5_leg(a, comm, rank, world):
    """configs[4] (C5): the 50M x 1024 hyperbolic-HNSW corpus as node-range shards of
    --c5-per-gpu points per GPU (6.25M = 50M / 8, so N = 8 is the full configuration and N = 1
    its per-GPU unit; weak scaling). Per shard the GPU builds HyperbolicHnsw (defaults,
    hnsw.rs:127-258) and its tangent cache; every query batch runs ShardedHyperbolicHnsw::search
    (shard.rs:354-373: rank 0's 10k queries broadcast, each shard searched, per-rank top-10
    all-gathered and merged on the GPU) in the exact mode (K10 Poincaré scan, the ground truth)
    and the tangent-pruned mode (search_with_pruning, hnsw.rs:450-490). The graph-search mode is
    left out: on this data the reference's graph rules give a non-navigable graph (recall@10
    0.002 at 6.25M, DESIGN.md §6 C5 note); the pruned mode (recall 0.85) is reported beside the
    exact one, which is as fast since the band pass (round 6). value = exact
    queries/s (recall 1.0) over the whole corpus; the exact mode's ids and distances are checked
    bit for bit against the oracle's scan of a query sample over every shard, whose rate on rank 0
    at N = 1 is the CPU baseline."""
    import bench_hyperbolic
    res = bench_hyperbolic.run_sharded(
        a.c5_per_gpu, 1024, 10_000, [], comm, rank, world, cpu_queries=4,
        cpu_seconds=(6.0 if rank == 0 and world == 1 and not a.no_cpu else 0.0),
        log=(lambda s: print(f"[bench] c5: {s}", file=sys.stderr, flush=True)) if rank == 0 else None)
    res["value"] = res["modes"]["exact"]["qps"]
    res["unit"] = "queries/s (exact Poincaré top-10 over every shard, recall 1.0; pruned mode beside it)"
    ex = res["roofline"].get("exact_scan_filter")
    if ex:
        res["roofline_dominant"] = dict(ex, kernel="scan_filter (exact mode)")
    return res


def c3_leg(a, x, n, d, rank, world, comm):
    """configs[2] on the bench's resident table: GPU HNSW build (M 32, ef_c 200), k=10 ef sweep
    with recall against the exact scan, NeuralSearch re-rank (RuvectorQuery defaults,
    query.rs:44-58) QPS with an oracle check, and the oracle's search_filter on the same graph
    as the CPU baseline (rank 0, N = 1). Replicas at N > 1: each rank builds and searches its
    own copy; the job rates are summed."""
    import bench_c3
    import ruvector_amd as rv
    nq = 10_000
    qb = rv.Buffer(nq * d * 4)
    qb.fill_normal(nq * d, 6)
    res = bench_c3.leg(x, n, d, qb, nq, 32, 200, [int(e) for e in a.c3_ef.split(",")], 10,
                       cpu=(rank == 0 and world == 1 and not a.no_cpu), cpu_seconds=8.0,
                       log=(lambda s: print(f"[bench] {s}", file=sys.stderr, flush=True)) if rank == 0 else
                       (lambda s: None), check=8 if rank == 0 else 0, seed=5)
    qps = res["neural_search"]["qps"]
    if comm is not None:
        qps = comm.allreduce([qps])[0]
    res["value"] = round(qps, 1)
    res["unit"] = "queries/s (NeuralSearch re-rank: HNSW ef 50 candidates + 2 GNN layers + differentiable_search; " \
                  "replicas summed over GPUs)"
    return res


def hnsw_leg(a, rank, world, comm):
    """Second half of the metric: HNSW queries/s at recall@10 >= 0.95 on
    BASELINE configs[0] (C1: 100k x 128, M=32, ef_c=200, 10k queries). The index
    is a replica per GPU (search does not shard), built on the GPU; each rank
    answers its own 10k queries, so the job rate is the sum over ranks."""
    import bench_hnsw
    # ef grid fine enough around the 0.95 crossing (C1: between ef 400 and 600)
    res = bench_hnsw.run(100_000, 128, 10_000, 32, 200, [300, 400, 450, 500, 550, 600, 800], 10, "l2",
                         cpu=(rank == 0 and world == 1 and not a.no_cpu), log=lambda s: None)
    qps = res["qps_at_recall95"] or 0.0
    if comm is not None:
        from ruvector_amd.shard import REDUCE_MIN
        res["per_gpu_min_qps"] = comm.allreduce([qps], REDUCE_MIN)[0]
        qps = comm.allreduce([qps])[0]
    res["value"] = round(qps, 1)
    res["unit"] = "queries/s (recall@10 >= 0.95, replicas summed over GPUs)"
    attach_hnsw_traffic(res)
    return res


def attach_hnsw_traffic(res):
    """C1's 51 MB table stays resident in L2 / the Infinity Cache, so `alg_GBps` (SURVEY.md
    §8d bytes / kernel time) is not an HBM rate. The committed rocprofv3 --pmc passes of the
    same search (scripts/hnsw_c1_traffic.sh -> profiles/pmc_traffic_hnsw_c1.json) give the
    bytes that left L2 per launch (Infinity-Cache hits included, so an upper bound on HBM
    bytes); the HBM fraction is capped by those bytes over the kernel time."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic_hnsw_c1.json")
    row = next((s for s in res.get("sweep", []) if s["ef"] == 550), None)
    if row is None or not os.path.exists(path):
        return
    try:
        pmc = json.load(open(path))
    except ValueError:
        return
    ent = pmc.get("kernels", {}).get("hnsw_search")
    if not ent or (pmc.get("config") or {}).get("ef") != 550 or not row.get("kernel_ms"):
        return
    fab = ent["hbm_bytes_per_launch"]
    rate = fab / (row["kernel_ms"] * 1e-3) / 1e9
    res["traffic_ef550"] = {
        "fabric_bytes_per_launch": round(fab, 0), "fabric_bytes_per_query": round(fab / 10_000, 1),
        "algorithmic_GBps": row["alg_GBps"], "fabric_GBps": round(rate, 1), "hbm_frac_upper_bound": round(rate / 8000.0, 4),
        "source": "rocprofv3 --pmc FETCH_SIZE(x2, gfx950) + WRITE_SIZE, profiles/pmc_traffic_hnsw_c1.json",
        "caveat": "51 MB table resident in L2 / Infinity Cache: the algorithmic rate is served on die, "
                  "FETCH counts L2 misses including Infinity-Cache hits, so HBM traffic is at most these bytes"}


def scan_leg(a, x, n, d, rank, world, comm):
    """Queries/s at recall@10 >= 0.95 on the metric's 10M x 768 table itself: on N(0,1)
    768-d rows the reference's HNSW parameters (M=32, ef_c=200) do not reach recall 0.95
    at 10M (profiles/r01_c3_10m.json; the GPU-built graph's recall equals the oracle
    CPU build's, profiles/r01_hnsw_quality_50k_768.log), so the 10M figure is the exact
    FlatIndex::search (flat.rs:36-76) over the bench's resident node table: recall 1.0,
    results identical to the reference-order scan (k_scan.hip MFMA filter + exact
    re-rank). 10k queries N(0,1) seed 6, k=10, L2; each rank answers its own batch on
    its replica of the table, so the job rate is the sum over ranks."""
    import bench_scan
    res = bench_scan.run(n, d, 10_000, 10, "l2", cpu_queries=(16 if rank == 0 and world == 1 and not a.no_cpu else 0),
                         valu=False, log=lambda s: None, xb=x, x_seed=3)
    qps = res["mfma"]["qps"]
    if comm is not None:
        qps = comm.allreduce([qps])[0]
    res["value"] = round(qps, 1)
    res["unit"] = "queries/s (recall@10 = 1.0, exact; replicas summed over GPUs)"
    # HBM bytes per filter launch from the committed PMC passes of this workload
    # (scripts/scan_traffic.sh -> profiles/pmc_traffic_scan.json), when they match
    path = os.path.join(ROOT, "profiles", "pmc_traffic_scan.json")
    rl = res.get("roofline")
    if rl is not None and os.path.exists(path):
        try:
            pmc = json.load(open(path))
        except ValueError:
            pmc = {}
        want = {"n": n, "d": d, "nq": 10_000, "k": 10, "metric": "l2",
                "launches": res["mfma"]["kernel_ms"].get("launches", {}).get("scan_filter")}
        ent = pmc.get("kernels", {}).get("scan_filter")
        if ent and all((pmc.get("config") or {}).get(k) == v for k, v in want.items()):
            rl["traffic"] = round(ent["hbm_bytes_per_launch"], 0)
            rl["traffic_source"] = "rocprofv3 --pmc FETCH_SIZE(x2, gfx950) + WRITE_SIZE, profiles/pmc_traffic_scan.json"
    return res


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
        pair = pmc.get("kernels", {}).get("sage_chunk_gather_gemm")
        if tag == "sage_aggregate" and r is not None and pair:
            # the chunk's gather rows are split between the gather kernel and the helping GEMM
            r["traffic"] = round(pair["hbm_bytes_per_launch"], 0)
            r["traffic_gather_kernel_only"] = round(ent["hbm_bytes_per_launch"], 0) if ent else None
            r["traffic_source"] = ("rocprofv3 --pmc FETCH_SIZE(x2, gfx950) + WRITE_SIZE, profiles/pmc_traffic_latest.json: "
                                   "gather kernel + the GEMM kernel that took part of its rows, per chunk (includes "
                                   "the GEMM's own A / W / y bytes)")
        elif r is not None and ent and r["unit"] == "GB/s":
            r["traffic"] = round(ent["hbm_bytes_per_launch"], 0)
            r["traffic_source"] = "rocprofv3 --pmc FETCH_SIZE(x2, gfx950) + WRITE_SIZE, profiles/pmc_traffic_latest.json"
        elif r is not None and ent:
            r["traffic"] = round(ent["hbm_bytes_per_launch"], 0)
            r["traffic_source"] = "rocprofv3 --pmc (HBM bytes per launch; MFMA-bound kernel)"


def gemm_alternatives(g, x, y, off_ptr, d, deg):
    """One GraphSAGE layer (layer 1 of the bench, same graph and input) with each GEMM
    path, to put the default split-f16x3 timing beside the split-bf16 (exact 3-way
    bf16 split, 6 products) and FP32-MFMA ones: ms per layer, averaged over 2 runs
    after one warm-up. Default path first so the three numbers come from one box state."""
    import ruvector_amd as rv
    layer = rv.GraphSAGELayer(d, d, num_samples=deg)
    out = {}
    for name, env in (("split-f16x3", {}), ("split-bf16x6", {"RVX_GEMM_H2": "0"}),
                      ("fp32-mfma", {"RVX_GEMM_H2": "0", "RVX_GEMM_X3": "0"})):
        old = {k: os.environ.get(k) for k in ("RVX_GEMM_H2", "RVX_GEMM_X3")}
        os.environ.update(env)
        try:
            ts = []
            for i in range(3):
                rv.synchronize()
                t0 = time.perf_counter()
                rv._lib.call("rvx_sage_forward_exchange", layer._h, g.handle, x.handle, y.handle, off_ptr, None, 0)
                rv.synchronize()
                if i:
                    ts.append(time.perf_counter() - t0)
            out[name] = {"layer_ms": round(sum(ts) / len(ts) * 1e3, 2)}
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    return out


def cpu_baseline(a, x_buf, g, tables, n, d, deg, layers, invs=None):
    """Oracle (reference algorithm, C++) on a bounded sample of layer-1 rows, plus
    per-layer parity of every layer: tables[i] holds the GPU's layer-(i+1) output of
    the last timed step; layer i+1 > 1 is checked on rows 0..8191 from the GPU's own
    layer-i rows (gathered from HBM), so each layer is compared on its actual input.
    The reference's GraphSAGE (graphsage.rs:105-115 linear_transform) is plain Rust
    loops with sequential f32 sums, so the scalar-order oracle is its CPU speed."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    from benchutil import host_threads

    threads, tinfo = host_threads()
    x = x_buf.download(np.float32, (n, d))
    rp, col = O.random_csr(n, deg, 4)
    wn, ws = O.sage_init(d, d, 0), O.sage_init(d, d, 1000)
    rows = 2048
    t0 = time.perf_counter()
    O.sage_forward(x, rp, col, wn, ws, rows=(0, rows), threads=threads)
    dt = time.perf_counter() - t0
    rows = int(min(n, max(rows, rows * a.cpu_seconds / max(dt, 1e-3))))
    t0 = time.perf_counter()
    ref = O.sage_forward(x, rp, col, wn, ws, rows=(0, rows), threads=threads)
    dt = time.perf_counter() - t0
    del x
    # deferred normalisation: layer l's table holds unnormalised rows, invs[l] their 1/|y|
    inv = [b.download(np.float32, (n,)) for b in invs] if invs else None

    def rows_of(li, ids):
        r = tables[li % 2].gather_rows(n, d, ids)
        if inv is not None and li < layers - 1:
            r = (r * inv[li % 2][ids][:, None]).astype(np.float32)
        return r

    got = rows_of(0, np.arange(rows))
    err, row_err = rel_errs(got, ref)
    del got, ref
    cpu = {"value": round(rows * deg / dt, 1), "unit": "edges/s", "cores": threads, "kind": "port", "host": tinfo,
           "sample": f"oracle GraphSAGE-mean layer 1 (graphsage.rs:118-187 restated in the reference's scalar order, "
                     f"{threads} threads) on rows 0..{rows} of the same {n} x {d} graph, {dt:.1f} s"}
    per_layer = [{"layer": 1, "rows": rows, "max_rel_err": err, "row_rel_l2_max": row_err, "input": "x"}]
    r2 = min(n, 8192)
    for li in range(1, layers):
        need = np.unique(np.concatenate([np.arange(r2), col[:rp[r2]]]))
        h = rows_of(li - 1, need)
        ref = O.sage_forward(h, rp[:r2 + 1], np.searchsorted(need, col[:rp[r2]]).astype(np.int32), wn, ws,
                             rows=(0, r2), threads=threads)
        got = rows_of(li, np.arange(r2))
        e, re_ = rel_errs(got, ref)
        per_layer.append({"layer": li + 1, "rows": r2, "max_rel_err": e, "row_rel_l2_max": re_,
                          "input": f"GPU layer-{li} rows"})
    worst = max(p["max_rel_err"] for p in per_layer)
    worst_row = max(p["row_rel_l2_max"] for p in per_layer)
    parity = {"rows": rows, "max_rel_err": worst, "row_rel_l2_max": worst_row, "tol": 1e-5,
              "ok": worst <= 1e-5 and worst_row <= 1e-5, "per_layer": per_layer,
              "metrics": "max_rel_err = max|gpu-ref| / max|ref| over the rows; row_rel_l2_max = max over rows of "
                         "||gpu_r-ref_r||_2 / ||ref_r||_2 (tests/parity.py)"}
    return cpu, parity


def rel_errs(got, ref):
    """(normwise, per-row) relative error of got vs ref, as tests/parity.py."""
    g, r = got.astype(np.float64), np.asarray(ref, np.float64)
    normwise = float(np.max(np.abs(g - r)) / max(float(np.max(np.abs(r))), 1e-30))
    nb = np.linalg.norm(r, axis=1)
    per_row = np.linalg.norm(g - r, axis=1) / np.where(nb > 0, nb, max(float(nb.max()), 1e-30))
    return normwise, float(per_row.max())


if __name__ == "__main__":
    main()
