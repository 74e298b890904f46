"""One rank of tests/test_gpu_shard_exchange.py (not collected by pytest).

Runs the three C++ node-range exchange entry points with world > 1 — all ranks
share GPU 0 over the host-staged transport (rvx_comm_init_host; RCCL refuses
two ranks on one device) — and compares with the 1-process forward:

  * rvx_sage_forward_exchange, 2 layers: after layer 1 EVERY row of the table
    (owned rows + the rows received from each peer, round by round) must equal
    the unsharded layer bit for bit; layer 2's owned rows likewise;
  * rvx_gnn_forward_exchange (RuvectorLayer, M|K|V exchange): owned rows;
  * rvx_edge_attention_forward_exchange (T exchange): owned rows.

usage: shard_exchange_worker.py WORLD RANK PORT OUT_JSON OFFSETS(comma-separated) [CHUNKS]
(CHUNKS: RVX_SAGE_CHUNKS for the GraphSAGE pipeline, default 3; the plan takes that many
rounds when the largest shard holds >= CHUNKS x 16384 rows)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    world, rank, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    offsets = np.array([int(v) for v in sys.argv[5].split(",")], np.int64)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # several exchange rounds at test size (>= CHUNKS x 16384 rows in the largest shard)
    os.environ["RVX_SAGE_CHUNKS"] = sys.argv[6] if len(sys.argv) > 6 else "3"
    import ctypes as C

    import torch.distributed as dist

    import oracle as O
    import ruvector_amd as rv
    from ruvector_amd.attention import EdgeFeaturedAttention, EdgeFeaturedConfig
    from host_comm import HostComm
    from ruvector_amd.shard import PLAN_SAGE, exchange_plan

    from datetime import timedelta
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=90))
    res = {"rank": rank}
    try:
        rv.set_device(0)
        comm = HostComm(world, rank)
        N = int(offsets[-1])
        o0, o1 = int(offsets[rank]), int(offsets[rank + 1])
        off_p = offsets.ctypes.data_as(C.POINTER(C.c_int64))
        one = np.array([0, N], np.int64)
        one_p = one.ctypes.data_as(C.POINTER(C.c_int64))
        res["rounds"] = len(exchange_plan(PLAN_SAGE, offsets))

        # ---- GraphSAGE (chunked rounds overlapped with the layer pipeline)
        d, deg = 32, 6
        x = O.fill_uniform(N * d, 81).reshape(N, d)
        rp, col = O.random_csr(N, deg, 82)
        g_full = rv.Graph.from_csr(rp, col)
        g_loc = rv.Graph.shard_from_csr(rp[o0:o1 + 1] - rp[o0], col[rp[o0]:rp[o1]], N)
        layer = rv.GraphSAGELayer(d, d, num_samples=deg)
        xb = rv.Buffer.from_numpy(x)
        y1, y2, r1, r2 = (rv.Buffer(N * d * 4) for _ in range(4))
        for b in (y1, y2):
            b.upload(np.full((N, d), np.nan, np.float32))  # unreceived rows would stay NaN
        call = rv._lib.call
        prof = rv.Profiler()
        with prof:
            call("rvx_sage_forward_exchange", layer._h, g_loc.handle, xb.handle, y1.handle, off_p, comm._h, 1)
            rv.synchronize()
        res["prof_tags"] = {t: prof.query(t)[1] for t in ("halo_exchange", "exchange_wait")}
        call("rvx_sage_forward_exchange", layer._h, g_loc.handle, y1.handle, y2.handle, off_p, comm._h, 0)
        call("rvx_sage_forward_exchange", layer._h, g_full.handle, xb.handle, r1.handle, one_p, None, 0)
        call("rvx_sage_forward_exchange", layer._h, g_full.handle, r1.handle, r2.handle, one_p, None, 0)
        a1, b1 = y1.download(np.float32, (N, d)), r1.download(np.float32, (N, d))
        a2, b2 = y2.download(np.float32, (N, d)), r2.download(np.float32, (N, d))
        res["sage_layer1_all_rows_equal"] = bool(np.array_equal(a1, b1))
        res["sage_layer1_halo_rows"] = int(N - (o1 - o0))
        res["sage_layer2_owned_equal"] = bool(np.array_equal(a2[o0:o1], b2[o0:o1]))
        # (an empty shard checks the rows of its lower neighbour's range instead)
        c0 = o0 if o1 > o0 else int(offsets[np.flatnonzero(np.diff(offsets))[0]])
        ref = O.sage_forward(x, rp, col, O.sage_init(d, d, 0), O.sage_init(d, d, 1000), rows=(c0, 500))
        res["sage_layer1_vs_oracle"] = float(np.max(np.abs(a1[c0:c0 + len(ref)] - ref)) / np.max(np.abs(ref)))
        # the same two layers with the normalisation deferred across the exchange
        # (rvx_sage_forward_exchange2: unnormalised rows + 1/|y| exchanged together)
        iv = rv.Buffer(N * 4)
        y1d, y2d = rv.Buffer(N * d * 4), rv.Buffer(N * d * 4)
        y1d.upload(np.full((N, d), np.nan, np.float32))
        call("rvx_sage_forward_exchange2", layer._h, g_loc.handle, xb.handle, None, y1d.handle, iv.handle, off_p,
             comm._h, 1)
        call("rvx_sage_forward_exchange2", layer._h, g_loc.handle, y1d.handle, iv.handle, y2d.handle, None, off_p,
             comm._h, 0)
        inv = iv.download(np.float32, (N,))
        a1d = y1d.download(np.float32, (N, d)).astype(np.float64) * inv[:, None]
        a2d = y2d.download(np.float32, (N, d))
        def row_rel(u, v):
            if len(v) == 0:  # an empty shard owns no rows
                return 0.0
            v = np.asarray(v, np.float64)
            nb = np.linalg.norm(v, axis=1)
            return float(np.max(np.linalg.norm(np.asarray(u, np.float64) - v, axis=1) / np.where(nb > 0, nb, 1.0)))
        res["sage_deferred_layer1_row_rel"] = row_rel(a1d, b1)
        res["sage_deferred_layer2_row_rel"] = row_rel(a2d[o0:o1], b2[o0:o1])
        # ranks that decide differently: rank 1 takes the split-bf16 GEMM, which cannot carry
        # the factors, so it normalises in place and ships 1.0 for its rows; the others
        # defer. The collective sequences must still match (no hang) and every row agree.
        if rank == 1:
            os.environ["RVX_GEMM_H2"] = "0"
        y1d.upload(np.full((N, d), np.nan, np.float32))
        iv.upload(np.full(N, np.nan, np.float32))
        call("rvx_sage_forward_exchange2", layer._h, g_loc.handle, xb.handle, None, y1d.handle, iv.handle, off_p,
             comm._h, 1)
        # read layer 1 now: a rank that cannot take the factors in layer 2 rescales its
        # input table in place (x_rowmul materialised), as documented for exchange2
        inv = iv.download(np.float32, (N,))
        a1d = y1d.download(np.float32, (N, d)).astype(np.float64) * inv[:, None]
        call("rvx_sage_forward_exchange2", layer._h, g_loc.handle, y1d.handle, iv.handle, y2d.handle, None, off_p,
             comm._h, 0)
        os.environ.pop("RVX_GEMM_H2", None)
        lo1, hi1 = int(offsets[1]), int(offsets[2])
        res["sage_mixed_defer_rank1_factors_one"] = bool(np.all(inv[lo1:hi1] == 1.0))
        a2d = y2d.download(np.float32, (N, d))
        # expected tables: rank 1's layer-1 rows from the split-bf16 path, the others from the
        # default path; layer 2 over that table with the owner's GEMM path (one process)
        os.environ["RVX_GEMM_H2"] = "0"
        call("rvx_sage_forward_exchange", layer._h, g_full.handle, xb.handle, r1.handle, one_p, None, 0)
        os.environ.pop("RVX_GEMM_H2", None)
        e1 = b1.copy()
        e1[lo1:hi1] = r1.download(np.float32, (N, d))[lo1:hi1]
        r1.upload(e1)
        if rank == 1:
            os.environ["RVX_GEMM_H2"] = "0"
        call("rvx_sage_forward_exchange", layer._h, g_full.handle, r1.handle, r2.handle, one_p, None, 0)
        os.environ.pop("RVX_GEMM_H2", None)
        e2 = r2.download(np.float32, (N, d))
        res["sage_mixed_defer_layer1_row_rel"] = row_rel(a1d, e1)
        res["sage_mixed_defer_layer2_row_rel"] = row_rel(a2d[o0:o1], e2[o0:o1])

        # ---- ReLU-sparse row images across the exchange (rvx_sage_forward_exchange3): every
        # rank images its own layer-1 rows and the rows it receives; layer 2 gathers from the
        # image. Same bits as the image-free stack; the image counts match the table.
        dI = 768
        xI = rv.Buffer.from_numpy(O.fill_uniform(N * dI, 86).reshape(N, dI) - 0.5)
        layI = [rv.GraphSAGELayer(dI, dI, num_samples=deg) for _ in range(2)]
        ivI = rv.Buffer(N * 4)
        outs = []
        for use_img in (False, True):
            img = rv.row_image(N, dI) if use_img else None
            h = img.handle if img else None
            t1, t2 = rv.Buffer(N * dI * 4), rv.Buffer(N * dI * 4)
            call("rvx_sage_forward_exchange3", layI[0]._h, g_loc.handle, xI.handle, None, None, t1.handle,
                 ivI.handle, h, off_p, comm._h, 1)
            call("rvx_sage_forward_exchange3", layI[1]._h, g_loc.handle, t1.handle, ivI.handle, h, t2.handle,
                 None, None, off_p, comm._h, 0)
            outs.append((t1.download(np.float32, (N, dI)), t2.download(np.float32, (N, dI))[o0:o1]))
            if img is not None:
                nnz = img.download(np.uint16, (N,), offset=N * 3072).astype(np.int64)
                res["image_nnz_all_rows_match"] = bool(np.array_equal(
                    nnz, (outs[-1][0].view(np.uint32) != 0).sum(axis=1)))
                res["image_rows_in_slots"] = float((nnz <= 736).mean())
            del t1, t2, img
        res["image_layer1_all_rows_equal"] = bool(np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32)))
        res["image_layer2_owned_equal"] = bool(np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32)))
        del outs

        # ---- compact exchange records (kernels.hpp rows_xchg_pack/unpack): rows travel as
        # bitmap + values other than +0.0 in a fixed slot and are expanded on arrival; rows
        # past the slot travel dense after the rounds. Every row of layer 1 (owned and
        # received) and layer 2's owned rows bit-identical to one process, for the dense
        # exchange (RVX_XCHG_IMAGE=0), the default (slot sized from chunk 0), a slot about half
        # the rows overflow and one every row overflows.
        from ruvector_amd.shard import comm_traffic
        q1, q2 = rv.Buffer(N * dI * 4), rv.Buffer(N * dI * 4)
        refI = [rv.GraphSAGELayer(dI, dI, num_samples=deg) for _ in range(2)]
        call("rvx_sage_forward_exchange3", refI[0]._h, g_full.handle, xI.handle, None, None, q1.handle, ivI.handle,
             None, one_p, None, 0)
        call("rvx_sage_forward_exchange3", refI[1]._h, g_full.handle, q1.handle, ivI.handle, None, q2.handle, None,
             None, one_p, None, 0)
        e1, e2 = q1.download(np.float32, (N, dI)).view(np.uint32), q2.download(np.float32, (N, dI)).view(np.uint32)
        nz = (e1 != 0).sum(axis=1)
        res["xchg_row_nnz_mean"] = float(nz.mean())
        rec = {}
        rec_mean = float(np.where(nz <= 736, (128 + 4 * nz + 15) // 16 * 16, 4 * dI).mean())
        res["xchg_record_bytes_mean"] = rec_mean
        for name, env in (("dense", {"RVX_XCHG_IMAGE": "0"}), ("default", {}),
                          ("half", {"RVX_XCHG_ROW_BYTES": str(int(rec_mean / 2))}), ("all", {"RVX_XCHG_ROW_BYTES": "16"})):
            os.environ.update(env)
            ls = [rv.GraphSAGELayer(dI, dI, num_samples=deg) for _ in range(2)]
            img = rv.row_image(N, dI) if name == "half" else None
            t1, t2 = rv.Buffer(N * dI * 4), rv.Buffer(N * dI * 4)
            t1.upload(np.full((N, dI), np.nan, np.float32))
            s0 = comm_traffic(comm)[0]
            call("rvx_sage_forward_exchange3", ls[0]._h, g_loc.handle, xI.handle, None, None, t1.handle, ivI.handle,
                 img.handle if img else None, off_p, comm._h, 1)
            rv.synchronize()
            sent = comm_traffic(comm)[0] - s0
            call("rvx_sage_forward_exchange3", ls[1]._h, g_loc.handle, t1.handle, ivI.handle,
                 img.handle if img else None, t2.handle, None, None, off_p, comm._h, 0)
            a1 = t1.download(np.float32, (N, dI)).view(np.uint32)
            a2 = t2.download(np.float32, (N, dI)).view(np.uint32)
            r = {"sent": int(sent), "layer1_all_rows_equal": bool(np.array_equal(a1, e1)),
                 "layer2_owned_equal": bool(np.array_equal(a2[o0:o1], e2[o0:o1]))}
            if img is not None:  # rows past the budget are imaged again after their dense pass
                inz = img.download(np.uint16, (N,), offset=N * 3072).astype(np.int64)
                r["image_counts_ok"] = bool(np.array_equal(inz, nz))
            rec[name] = r
            for k in env:
                os.environ.pop(k)
            del t1, t2, img, ls
        res["xchg"] = rec
        del xI, q1, q2

        # ---- RuvectorLayer (M|K|V exchange) and the attention head (T exchange)
        n2 = int(offsets[-1])
        H, heads, deg2 = 64, 4, 5
        xg = O.fill_uniform(n2 * H, 83).reshape(n2, H)
        rp2, col2 = O.random_csr(n2, deg2, 84)
        ew = O.fill_uniform(len(col2), 85, 0.0, 1.0)
        gf = rv.Graph.from_csr(rp2, col2, ew)
        gl = rv.Graph.shard_from_csr(rp2[o0:o1 + 1] - rp2[o0], col2[rp2[o0]:rp2[o1]], n2, ew[rp2[o0]:rp2[o1]])
        rl = rv.RuvectorLayer(H, H, heads, 0.0, seed=7)
        xgb = rv.Buffer.from_numpy(xg)
        ys, yr = rv.Buffer(n2 * H * 4), rv.Buffer(n2 * H * 4)
        # M|K|V exchange (RVX_GNN_FOLD=0, default) and the folded M-only
        # exchange (forced on for the 1-process reference too)
        for mode, key in (("0", "gnn_owned_equal"), ("2", "gnn_fold_owned_equal")):
            os.environ["RVX_GNN_FOLD"] = mode
            rl.forward_exchange(gl, xgb, ys, offsets, comm)
            rl.forward_graph_device(xgb, gf, yr)
            res[key] = bool(np.array_equal(ys.download(np.float32, (n2, H))[o0:o1],
                                           yr.download(np.float32, (n2, H))[o0:o1]))
        os.environ.pop("RVX_GNN_FOLD")
        W = O.RvlWeights(json.loads(rl.to_json()))
        if o1 > o0:
            ref = O.rvl_forward_graph(W, xg, rp2, col2, ew, rows=(o0, min(o1 - o0, 300)))
            got = ys.download(np.float32, (n2, H))[o0:o0 + len(ref)]
            res["gnn_fold_vs_oracle"] = float(np.max(np.abs(got - ref)) / np.max(np.abs(ref)))
        else:  # an empty shard owns no rows to check
            res["gnn_fold_vs_oracle"] = 0.0
        att = EdgeFeaturedAttention(EdgeFeaturedConfig(node_dim=H, edge_dim=1, num_heads=heads))
        efl, eff = rv.Buffer.from_numpy(ew[rp2[o0]:rp2[o1]].copy()), rv.Buffer.from_numpy(ew)
        zs, zr = rv.Buffer(n2 * H * 4), rv.Buffer(n2 * H * 4)
        att.forward_exchange(gl, yr, efl, zs, offsets, comm)
        att.forward_graph_device(yr, gf, eff, zr)
        res["efa_owned_equal"] = bool(np.array_equal(zs.download(np.float32, (n2, H))[o0:o1],
                                                     zr.download(np.float32, (n2, H))[o0:o1]))
        rv.synchronize()
    except Exception as e:  # reported to the test, not swallowed
        import traceback
        res["error"] = f"{e!r}\n{traceback.format_exc()}"
    finally:
        with open(out, "w") as f:
            json.dump(res, f)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
