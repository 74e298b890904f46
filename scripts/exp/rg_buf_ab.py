#!/usr/bin/env python3
"""A/B of the HBM-resident-R search (k_hnsw.hip RG): admissions buffered in LDS and flushed into
the HBM array (RVX_HNSW_RG_BUF=1, default) against one merge into the HBM array per admission
batch (0), interleaved on one GPU-built graph; ids and distances must be identical.
usage: python scripts/exp/rg_buf_ab.py --n 2000000 --m 128 --efc 500 --ef 8192,12288 --queries 4096"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=2_000_000)
    p.add_argument("--d", type=int, default=768)
    p.add_argument("--m", type=int, default=128)
    p.add_argument("--efc", type=int, default=500)
    p.add_argument("--ef", default="8192,12288")
    p.add_argument("--queries", type=int, default=4096)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--forms", default="1,0", help="RVX_HNSW_RG_BUF settings to run")
    p.add_argument("--arms", default="", help="instead of --forms: arms 'name:VAR=v,VAR=v;name2:...' (env read per call)")
    a = p.parse_args()
    import ruvector_amd as rv
    from benchutil import heartbeat
    n, d, nq, k = a.n, a.d, a.queries, 10
    xb = rv.Buffer(n * d * 4)
    xb.fill_normal(n * d, 3)
    qb = rv.Buffer(nq * d * 4)
    qb.fill_normal(nq * d, 6)
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=a.m, ef_construction=a.efc, ef_search=100))
    t0 = time.perf_counter()
    with heartbeat(f"build {n} x {d} M {a.m} ef_c {a.efc}", every=30.0):
        idx.add_device(xb, n, 0)
        rv.synchronize()
    print(f"build {time.perf_counter() - t0:.1f} s", flush=True)
    ids_b, dist_b = rv.Buffer(nq * k * 8), rv.Buffer(nq * k * 4)
    gt_b, gtd_b = rv.Buffer(nq * k * 8), rv.Buffer(nq * k * 4)
    rv._lib.call("rvx_index_brute_force_device", idx.handle, qb.handle, nq, k, gt_b.handle, gtd_b.handle)
    gt = gt_b.download(np.uint64, (nq, k))
    out = {"config": vars(a), "runs": []}
    for ef in [int(e) for e in a.ef.split(",")]:
        ref = None
        for rep in range(a.reps):
            arms = ([(f"buf{b}", {"RVX_HNSW_RG_BUF": b}) for b in a.forms.split(",")] if not a.arms else
                    [(x.split(":")[0], dict(kv.split("=") for kv in x.split(":")[1].split(",") if kv))
                     for x in a.arms.split(";")])
            for buf, env in arms:
                saved = {kk: os.environ.get(kk) for kk in env}
                os.environ.update(env)
                rv._lib.call("rvx_index_search_device", idx.handle, qb.handle, min(nq, 256), k, ef, ids_b.handle,
                             dist_b.handle)
                rv.synchronize()
                prof = rv.Profiler()
                with prof, heartbeat(f"ef {ef} buf {buf}", every=30.0):
                    t0 = time.perf_counter()
                    rv._lib.call("rvx_index_search_device", idx.handle, qb.handle, nq, k, ef, ids_b.handle,
                                 dist_b.handle)
                    rv.synchronize()
                    dt = time.perf_counter() - t0
                st = rv.hnsw_last_search_stats()
                got = (ids_b.download(np.uint64, (nq, k)), dist_b.download(np.float32, (nq, k)))
                if ref is None:
                    ref = got
                same = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1].view(np.uint32),
                                                                             ref[1].view(np.uint32)))
                rec = float(np.mean([len(set(x.tolist()) & set(y.tolist())) / k for x, y in zip(gt, got[0])]))
                for kk, vv in saved.items():
                    if vv is None:
                        os.environ.pop(kk, None)
                    else:
                        os.environ[kk] = vv
                row = {"ef": ef, "buf": buf, "rep": rep, "qps": round(nq / dt, 1), "kernel_ms": round(prof.query("hnsw_search")[0], 2),
                       "recall": round(rec, 4), "same_as_first": same, "r_in_hbm": st["r_in_hbm"], "stages": st["stages"],
                       "dist_per_query": round(st["n_dist"] / nq, 1), "expand_per_query": round(st["n_expand"] / nq, 1)}
                out["runs"].append(row)
                print(json.dumps(row), flush=True)
    os.environ.pop("RVX_HNSW_RG_BUF", None)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
