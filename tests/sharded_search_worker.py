"""One rank of tests/test_gpu_sharded_search.py (not collected by pytest).

Node-range-sharded index search across processes (SURVEY.md §8e option 2,
ShardedHyperbolicHnsw::search, crates/ruvector-hyperbolic-hnsw/src/shard.rs:354-373):
all ranks share GPU 0 over the host-staged transport (rvx_comm_init_host), rank r
holds global ids [offsets[r], offsets[r+1]). Each rank loads the ORACLE-built graph
of its shard, runs rvx_hyperbolic_sharded_search / rvx_index_sharded_search (query
broadcast from rank 0, local search, all-gather of per-rank top-k, GPU merge) and
compares its merged result with the merge of the per-shard oracle searches.

usage: sharded_search_worker.py WORLD RANK PORT OUT_JSON OFFSETS(comma-separated) DIM
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def ball_points(n, d, seed, rmax=0.9):
    r = np.random.default_rng(seed)
    v = r.standard_normal((n, d)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return (v * (rmax * r.random((n, 1)))).astype(np.float32)


def merge(parts, k):
    """shard.rs:354-373 over per-shard (global id, distance) lists: by distance,
    ties in shard order (stable), -1 padding last, first k."""
    ids = np.concatenate([p[0] for p in parts], axis=1)
    d = np.concatenate([p[1] for p in parts], axis=1).astype(np.float64)
    d = np.where(ids < 0, np.inf, d)
    order = np.argsort(d, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(ids, order, 1), np.take_along_axis(d, order, 1)


def close(a, b, tol=0.0):  # bit-exact distances by default (glibc-identical device libm)
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    fin = np.isfinite(b)
    return bool(np.array_equal(np.isfinite(a), fin) and
                np.all(np.abs(a[fin] - b[fin]) <= tol * np.maximum(np.abs(b[fin]), 1e-30)))


def main():
    world, rank, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    offsets = [int(v) for v in sys.argv[5].split(",")]
    d = int(sys.argv[6])
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from datetime import timedelta

    import torch.distributed as dist

    import oracle as O
    import ruvector_amd as rv
    from host_comm import HostComm

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=90))
    res = {"rank": rank}
    try:
        rv.set_device(0)
        comm = HostComm(world, rank)
        N = offsets[-1]
        o0, o1 = offsets[rank], offsets[rank + 1]
        x = ball_points(N, d, 61)
        q = ball_points(48, d, 62)
        nq = q.shape[0]
        qa = q if rank == 0 else nq  # only rank 0's queries are read

        # ---- HyperbolicHnsw shards (oracle-built graphs on every shard)
        orc = []
        for s in range(world):
            o = O.Hyp(d, seed=5 + s)
            o.insert(x[offsets[s]:offsets[s + 1]])
            orc.append(o)
        h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=5 + rank), dim=d)
        h.insert_batch(x[o0:o1])
        h.load_graph(orc[rank].export())
        grp = rv.ShardedHyperbolicSearch(h, comm, o0)
        checks = {}
        expect = {}
        for k, ef in ((10, 0), (5, 100), (1, 0)):
            gid, lid, gd, cnt = grp.search_batch(qa, k, ef)
            parts = []
            for s, o in enumerate(orc):
                oi, od, _ = o.search(q, k, ef)
                parts.append((np.where(oi >= 0, oi + offsets[s], -1), od))
            ei, ed = merge(parts, k)
            owner = np.searchsorted(offsets, np.maximum(ei, 0), side="right") - 1
            el = np.where(ei >= 0, ei - np.asarray(offsets)[owner], -1)
            expect[(k, ef)] = ei
            checks[f"search_k{k}_ef{ef}"] = bool(
                np.array_equal(gid, ei) and np.array_equal(lid, el) and close(gd, ed) and
                np.array_equal(cnt, (ei >= 0).sum(1)))
        # exact scans (mode 1) and the reference result shape on one query
        gid, lid, gd, cnt = grp.search_batch(qa, 10, 0, "exact")
        parts = [(np.where(oi >= 0, oi + offsets[s], -1), od)
                 for s, o in enumerate(orc) for oi, od in [o.brute_force(q, 10)]]
        ei, ed = merge(parts, 10)
        checks["exact_k10"] = bool(np.array_equal(gid, ei) and close(gd, ed))
        expect_exact = (gid.copy(), gd.copy())
        one = grp.search(q[3] if rank == 0 else None, 10)  # shard.search = graph search (hnsw.rs:427)
        e10 = expect[(10, 0)]
        checks["shape"] = all(g == int(e10[3, j]) and r.id == g - offsets[int(np.searchsorted(offsets, g, "right")) - 1]
                              for j, (g, r) in enumerate(one)) and len(one) == int((e10[3] >= 0).sum())
        # search_with_pruning (mode 2) after building every shard's tangent cache
        h.build_tangent_cache()
        for o in orc:
            o.build_tangent_cache()
        gid, lid, gd, cnt = grp.search_batch(qa, 10, 0, "pruned")
        parts = [(np.where(oi >= 0, oi + offsets[s], -1), od)
                 for s, o in enumerate(orc) for oi, od in [o.search_with_pruning(q, 10)]]
        ei, ed = merge(parts, 10)
        rec = np.mean([len(set(a.tolist()) & set(b.tolist())) / 10 for a, b in zip(ei, gid)])
        res["pruned_recall_vs_oracle"] = float(rec)
        checks["pruned_sorted"] = bool(np.all(np.diff(gd, axis=1) >= 0))
        # every shard's centroid and tangent coordinates equal the oracle's bits
        checks["pruned_exact"] = bool(np.array_equal(gid, ei) and close(gd, ed))
        # k * prune_factor is unbounded (hnsw.rs:469-470): 200 tangent candidates per shard
        gid, lid, gd, cnt = grp.search_batch(qa, 20, 0, "pruned")
        parts = [(np.where(oi >= 0, oi + offsets[s], -1), od)
                 for s, o in enumerate(orc) for oi, od in [o.search_with_pruning(q, 20)]]
        ei, ed = merge(parts, 20)
        checks["pruned_k20_exact"] = bool(np.array_equal(gid, ei) and close(gd, ed))
        # a precondition that fails on some shards only (rank 1's shard uses the Euclidean
        # metric, which search_with_pruning does not serve) fails on EVERY rank instead of
        # leaving the passing ranks waiting in a collective, and so do arguments that differ
        # between ranks; the group stays usable afterwards
        def fails(*args, group=None):
            try:
                (group or grp).search_batch(*args)
                return False
            except rv.RvxError:
                return True
        hx = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=9, metric="euclidean" if rank == 1 else "poincare"),
                               dim=d)
        hx.insert_batch(x[o0:o0 + min(50, o1 - o0)])
        hx.build_tangent_cache()
        checks["one_shard_failure_fails_all"] = fails(qa, 10, 0, "pruned",
                                                      group=rv.ShardedHyperbolicSearch(hx, comm, o0))
        checks["arg_mismatch_fails_all"] = fails(qa, 10 if rank == 0 else 9, 0, "exact")
        checks["rank0_without_queries_fails_all"] = fails(nq, 10, 0, "exact")
        gid2, _, gd2, _ = grp.search_batch(qa, 10, 0, "exact")
        checks["usable_after_failures"] = bool(np.array_equal(gid2[:, :10], expect_exact[0]) and
                                               np.array_equal(gd2[:, :10], expect_exact[1]))
        # nq = 0 is a no-op on every rank
        e = grp.search_batch(np.zeros((0, d), np.float32) if rank == 0 else 0, 10)
        checks["empty"] = e[0].shape == (0, 10)

        # ---- VectorIndex shards: FlatIndex (exact) and HnswIndex on oracle graphs
        keys = np.arange(o0, o1, dtype=np.uint64)
        fl = rv.FlatIndex(d, rv.DistanceMetric.Euclidean)
        fl.add_array(x[o0:o1], keys)
        ids, dd, cnt = fl.sharded_search_array(comm, qa, 10)
        ri, rd = O.flat_search(x, q, 10)
        checks["flat_exact"] = bool(np.array_equal(ids.astype(np.int64), ri) and np.array_equal(dd, rd))
        # a real hit at +inf (the 3e19 rows of ranks > 0 overflow the squared
        # distance) orders before every rank's empty slots (gid -1), so the first `count`
        # merged slots are real hits in rank order
        fz = rv.FlatIndex(d, rv.DistanceMetric.Euclidean)
        fz.add_array(np.full((1, d), 3e19 if rank > 0 else 0.0, np.float32), np.array([1000 + rank], np.uint64))
        kz = 4
        zi, zd, zc = fz.sharded_search_array(comm, qa, kz)
        m = min(kz, world)
        checks["inf_hits_before_empty_slots"] = bool(
            np.all(zc == m) and np.array_equal(zi[:, :m].astype(np.int64), np.tile(1000 + np.arange(m), (nq, 1))) and
            np.all(np.isfinite(zd[:, 0])) and np.all(np.isinf(zd[:, 1:m])))
        horc = []
        for s in range(world):
            o = O.Hnsw(d, "l2", m=8, ef_construction=64, seed=3 + s)
            o.insert(x[offsets[s]:offsets[s + 1]], threads=1)
            horc.append(o)
        hi = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=8, ef_construction=64, ef_search=40),
                          seed=3 + rank)
        hi.add_array(x[o0:o1], keys)
        hi.load_graph(horc[rank].export())
        for k, ef in ((10, 40), (3, 20)):
            ids, dd, cnt = hi.sharded_search_array(comm, qa, k, ef)
            parts = [(np.where(oi >= 0, oi + offsets[s], -1), od)
                     for s, o in enumerate(horc) for oi, od, _ in [o.search(q, k, ef)]]
            ei, ed = merge(parts, k)
            got = np.where(np.arange(k)[None, :] < cnt[:, None], ids.astype(np.int64), -1)
            checks[f"hnsw_index_k{k}"] = bool(np.array_equal(got, ei) and close(dd, ed, 0.0))
        res["checks"] = checks
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
