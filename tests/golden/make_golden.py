#!/usr/bin/env python3
"""Generate the small golden fixtures in tests/golden/ from the CPU oracle.

The reference's Rust cannot run here (no cargo/rustc; its prebuilt addons may
not be run), so these vectors come from the oracle restatement,
whose own pinning is the reference's known-answer tests
(tests/test_oracle_known_answers.py). They freeze the oracle's outputs so any
later drift of either side is caught. Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle as O  # noqa: E402


def layer_json(in_dim, hidden, heads, dropout, seed):
    rng = np.random.default_rng(seed)

    def lin(i, o):
        w = rng.normal(0, np.sqrt(2 / (i + o)), o * i).astype(np.float32)
        b = rng.normal(0, 0.01, o).astype(np.float32)
        return {"weights": {"v": 1, "dim": [o, i], "data": [float(v) for v in w]},
                "bias": {"v": 1, "dim": [o], "data": [float(v) for v in b]}}
    return {"w_msg": lin(in_dim, hidden), "w_agg": lin(hidden, hidden),
            "w_update": {k: lin(hidden, hidden) for k in ("w_z", "u_z", "w_r", "u_r", "w_h", "u_h")},
            "attention": {"num_heads": heads, "head_dim": hidden // heads,
                          **{k: lin(hidden, hidden) for k in ("q_linear", "k_linear", "v_linear", "out_linear")}},
            "norm": {"gamma": {"v": 1, "dim": [hidden], "data": [1.0] * hidden},
                     "beta": {"v": 1, "dim": [hidden], "data": [0.0] * hidden}, "eps": 1e-5},
            "dropout": dropout}


def main():
    out = {}
    # distances (distance.rs fallback order)
    q = O.fill_uniform(5 * 13, 101).reshape(5, 13)
    x = O.fill_uniform(7 * 13, 102).reshape(7, 13)
    dist = {m: O.distance_matrix(q, x, m) for m in ("l2", "cosine", "dot", "l1")}
    np.savez(os.path.join(HERE, "distances.npz"), q=q, x=x, **dist)

    # flat search with a tombstone
    base = O.fill_uniform(400 * 24, 103).reshape(400, 24)
    qs = O.fill_uniform(9 * 24, 104).reshape(9, 24)
    deleted = np.zeros(400, np.uint8)
    deleted[[3, 77, 250]] = 1
    ids, d = O.flat_search(base, qs, 10, "l2", deleted=deleted)
    np.savez(os.path.join(HERE, "flat.npz"), base=base, q=qs, deleted=deleted, ids=ids, dist=d)

    # GraphSAGE mean / maxpool, 1 layer, with an isolated node
    n, f = 40, 12
    xs = O.fill_uniform(n * f, 105).reshape(n, f)
    edges = [(int(a), int(b)) for a, b in np.random.default_rng(5).integers(0, n - 1, (160, 2))]
    rp, col, _ = O.build_csr(n, edges)
    wn, ws = O.sage_init(f, 10, 0), O.sage_init(f, 10, 1000)
    np.savez(os.path.join(HERE, "sage.npz"), x=xs, edges=np.array(edges, np.int64), rp=rp, col=col,
             mean=O.sage_forward(xs, rp, col, wn, ws, 0), maxpool=O.sage_forward(xs, rp, col, wn, ws, 1))

    # RuvectorLayer (layer.rs) per-node cases from a serde JSON layer
    js = layer_json(4, 8, 2, 0.1, 7)
    json.dump(js, open(os.path.join(HERE, "rvl_layer_4_8_2.json"), "w"))
    W = O.RvlWeights(js)
    node = np.array([1.0, 2.0, 3.0, 4.0], np.float32)
    nbrs = np.array([[0.5, 1.0, 1.5, 2.0], [2.0, 3.0, 4.0, 5.0]], np.float32)
    cases = {"two_nbrs": O.rvl_forward_one(W, node, nbrs, [0.3, 0.7]),
             "no_nbrs": O.rvl_forward_one(W, node, [], []),
             "no_weights": O.rvl_forward_one(W, node, nbrs, []),
             "zero_weights": O.rvl_forward_one(W, node, nbrs, [0.0, 0.0])}
    np.savez(os.path.join(HERE, "rvl.npz"), node=node, nbrs=nbrs, **cases)

    # HNSW: fixed graph + exact search results (hnsw_rs search_filter semantics)
    hv = O.fill_uniform(300 * 16, 106).reshape(300, 16)
    h = O.Hnsw(16, "l2", m=8, ef_construction=40, seed=11)
    h.insert(hv, threads=1)
    g = h.export()
    hq = O.fill_uniform(20 * 16, 107).reshape(20, 16)
    ids, d, cnt = h.search(hq, 10, 32)
    gz = {"vecs": hv, "q": hq, "ids": ids, "dist": d, "cnt": cnt, "n": g["n"], "max_level": g["max_level"],
          "entry": g["entry"], "levels": g["levels"], "row_ptr0": g["row_ptr0"], "col0": g["col0"]}
    for l in range(g["max_level"]):
        gz[f"up_ids_{l + 1}"] = g["upper_ids"][l]
        gz[f"up_rp_{l + 1}"] = g["upper_row_ptr"][l]
        gz[f"up_col_{l + 1}"] = g["upper_col"][l]
    np.savez(os.path.join(HERE, "hnsw.npz"), **gz)

    # differentiable_search, EdgeFeaturedAttention, Poincaré
    dq = O.fill_uniform(32, 108)
    dc = O.fill_uniform(12 * 32, 109).reshape(12, 32)
    di, dw = O.differentiable_search(dq, dc, 5, 0.5)
    ef_q = O.fill_uniform(16, 110)
    ef_k = O.fill_uniform(6 * 16, 111).reshape(6, 16)
    ef_v = O.fill_uniform(6 * 16, 112).reshape(6, 16)
    ef_e = O.fill_uniform(6 * 4, 113).reshape(6, 4)
    efa = O.efa_compute(16, 4, 2, ef_q, ef_k, ef_v, ef_e)
    pu = (O.fill_uniform(6 * 8, 114).reshape(6, 8) * 0.3).astype(np.float32)
    pd = np.array([[O.poincare_distance(a, b) for b in pu] for a in pu], np.float32)
    np.savez(os.path.join(HERE, "misc.npz"), dq=dq, dc=dc, di=di, dw=dw, ef_q=ef_q, ef_k=ef_k, ef_v=ef_v, ef_e=ef_e,
             efa=efa, pu=pu, pd=pd)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
