"""Committed golden fixtures (tests/golden/, made by make_golden.py from the
oracle): the oracle must still reproduce them bit for bit (CPU), and the HIP
path must match them (GPU; bit-exact for distances/top-k/HNSW, 1e-5 relative
for embeddings)."""
import json
import os

import numpy as np
import pytest

import oracle as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def graph_of(z):
    L = int(z["max_level"])
    return {"n": int(z["n"]), "max_level": L, "entry": int(z["entry"]), "levels": z["levels"],
            "row_ptr0": z["row_ptr0"], "col0": z["col0"],
            "upper_ids": [z[f"up_ids_{l}"] for l in range(1, L + 1)],
            "upper_row_ptr": [z[f"up_rp_{l}"] for l in range(1, L + 1)],
            "upper_col": [z[f"up_col_{l}"] for l in range(1, L + 1)]}


# ------------------------------------------------------------------ oracle is stable
def test_oracle_reproduces_distances():
    z = load("distances.npz")
    for m in ("l2", "cosine", "dot", "l1"):
        assert np.array_equal(O.distance_matrix(z["q"], z["x"], m), z[m])


def test_oracle_reproduces_flat():
    z = load("flat.npz")
    ids, d = O.flat_search(z["base"], z["q"], 10, "l2", deleted=z["deleted"])
    assert np.array_equal(ids, z["ids"]) and np.array_equal(d, z["dist"])


def test_oracle_reproduces_sage():
    z = load("sage.npz")
    f = z["x"].shape[1]
    wn, ws = O.sage_init(f, 10, 0), O.sage_init(f, 10, 1000)
    assert np.array_equal(O.sage_forward(z["x"], z["rp"], z["col"], wn, ws, 0), z["mean"])
    assert np.array_equal(O.sage_forward(z["x"], z["rp"], z["col"], wn, ws, 1), z["maxpool"])


def test_oracle_reproduces_rvl():
    z = load("rvl.npz")
    W = O.RvlWeights(json.load(open(os.path.join(G, "rvl_layer_4_8_2.json"))))
    assert np.array_equal(O.rvl_forward_one(W, z["node"], z["nbrs"], [0.3, 0.7]), z["two_nbrs"])
    assert np.array_equal(O.rvl_forward_one(W, z["node"], [], []), z["no_nbrs"])
    assert np.array_equal(O.rvl_forward_one(W, z["node"], z["nbrs"], []), z["no_weights"])
    assert np.array_equal(O.rvl_forward_one(W, z["node"], z["nbrs"], [0.0, 0.0]), z["zero_weights"])


def test_oracle_reproduces_hnsw_search_on_fixed_graph():
    z = load("hnsw.npz")
    h = O.Hnsw.from_graph(z["vecs"], graph_of(z), "l2")
    ids, d, cnt = h.search(z["q"], 10, 32)
    assert np.array_equal(ids, z["ids"]) and np.array_equal(d, z["dist"]) and np.array_equal(cnt, z["cnt"])


def test_oracle_reproduces_misc():
    z = load("misc.npz")
    di, dw = O.differentiable_search(z["dq"], z["dc"], 5, 0.5)
    assert np.array_equal(di, z["di"]) and np.array_equal(dw, z["dw"])
    assert np.array_equal(O.efa_compute(16, 4, 2, z["ef_q"], z["ef_k"], z["ef_v"], z["ef_e"]), z["efa"])


# ------------------------------------------------------------------ HIP path vs fixtures
@pytest.mark.gpu
def test_gpu_matches_golden():
    import ruvector_amd as rv
    z = load("distances.npz")
    for m, e in (("l2", rv.DistanceMetric.Euclidean), ("cosine", rv.DistanceMetric.Cosine),
                 ("dot", rv.DistanceMetric.DotProduct), ("l1", rv.DistanceMetric.Manhattan)):
        assert np.array_equal(rv.distance_matrix(z["q"], z["x"], e), z[m])

    z = load("flat.npz")
    idx = rv.FlatIndex(24, rv.DistanceMetric.Euclidean)
    idx.add_array(z["base"], np.arange(400, dtype=np.uint64))
    for r in np.nonzero(z["deleted"])[0]:
        idx._ids[str(int(r))] = int(r)
        assert idx.remove(str(int(r)))
    ids, d, _ = idx.search_array(z["q"], 10)
    assert np.array_equal(ids.astype(np.int64), z["ids"]) and np.array_equal(d, z["dist"])

    z = load("sage.npz")
    g = rv.Graph.from_edges(len(z["x"]), z["edges"])
    for agg in ("mean", "maxpool"):
        y = rv.GraphSAGELayer(12, 10, num_samples=64, aggregator=agg).forward_graph(z["x"], g)
        ref = z[agg]
        assert float(np.max(np.abs(y - ref)) / np.max(np.abs(ref))) <= 1e-5

    z = load("rvl.npz")
    layer = rv.RuvectorLayer.from_json(open(os.path.join(G, "rvl_layer_4_8_2.json")).read())
    for key, w, nb in (("two_nbrs", [0.3, 0.7], z["nbrs"]), ("no_nbrs", [], []), ("no_weights", [], z["nbrs"]),
                       ("zero_weights", [0.0, 0.0], z["nbrs"])):
        y = layer.forward(z["node"], list(nb), w)
        assert float(np.max(np.abs(y - z[key])) / np.max(np.abs(z[key]))) <= 1e-5, key

    z = load("hnsw.npz")
    hi = rv.HnswIndex(16, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=8, ef_construction=40, ef_search=32))
    hi.add_array(z["vecs"], np.arange(300, dtype=np.uint64))
    hi.load_graph(graph_of(z))
    ids, d, cnt = hi.search_array(z["q"], 10, 32)
    assert np.array_equal(ids.astype(np.int64), z["ids"]) and np.array_equal(d, z["dist"])
    assert np.array_equal(cnt, z["cnt"])
