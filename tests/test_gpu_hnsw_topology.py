"""C2 and C4 on the topology SURVEY.md §8(d) names for them (VERDICT r3 "next" 3): the
layer-0 CSR of an HNSW built on the GPU (M 32, ef_c 200: lists of up to 64 neighbours
in stored order; patches/hnsw_rs/src/hnsw.rs:1149-1196), exported with
rvx_index_export_layer0, edge feature = the stored HNSW edge distance.

* export: every edge's stored distance equals the reference-order L2 of its endpoints
  (the oracle's distance()), row_ptr is monotone and lists hold <= 2M entries;
* C2: 2-layer GraphSAGE-mean (num_samples 32, so lists longer than 32 go through the
  sample_neighbors path; crates/ruvector-postgres/src/gnn/graphsage.rs:92-187);
* C4: 3 x RuvectorLayer(768, h 8) with the distances as edge weights
  (crates/ruvector-gnn/src/layer.rs:379-418), then EdgeFeaturedAttention with the
  distance as the 1-d edge feature (crates/ruvector-attention/src/graph/edge_featured.rs:196-258).
Every layer is compared with the oracle on a row sample, each on its actual input (the
GPU's previous layer), per row and normwise within 1e-5 (tests/parity.py)."""
import json

import numpy as np
import pytest

import oracle as O
from parity import assert_close

rv = pytest.importorskip("ruvector_amd")
from ruvector_amd.attention import EdgeFeaturedAttention, EdgeFeaturedConfig  # noqa: E402

pytestmark = pytest.mark.gpu
N, D = 100_000, 768


@pytest.fixture(scope="module")
def hnsw_graph():
    x = np.random.default_rng(5).standard_normal((N, D), dtype=np.float32)
    xb = rv.Buffer.from_numpy(x)
    idx = rv.HnswIndex(D, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=32, ef_construction=200), seed=5)
    idx.add_device(xb, N)
    rp, col, dist = idx.layer0()
    return x, xb, rp, col, dist


def _sub(rp, col, rows):
    """CSR of rows [0, rows) whose neighbours are renumbered rows + edge position, and the
    global ids to gather in that order (self rows first)."""
    nb = col[:rp[rows]].astype(np.int64)
    need = np.concatenate([np.arange(rows, dtype=np.int64), nb])
    return rp[:rows + 1].copy(), (rows + np.arange(nb.size)).astype(np.int32), need


def test_layer0_export_is_the_hnsw_graph(hnsw_graph):
    x, _, rp, col, dist = hnsw_graph
    assert rp.shape == (N + 1,) and rp[0] == 0 and np.all(np.diff(rp) >= 0) and np.all(np.diff(rp) <= 64)
    assert rp[-1] == col.size == dist.size and col.min() >= 0 and col.max() < N
    assert np.mean(np.diff(rp)) > 16  # a real HNSW layer 0, not a sparse stand-in
    for i in (0, 1, 777, N // 2, N - 1):
        for p in range(rp[i], rp[i + 1]):
            assert dist[p] == O.distance(x[i], x[col[p]], "l2")


def test_graphsage_two_layers_on_hnsw_layer0(hnsw_graph):
    x, xb, rp, col, _ = hnsw_graph
    g = rv.Graph.from_csr(rp, col)
    wn, ws = O.sage_init(D, D, 0), O.sage_init(D, D, 1000)
    l1, l2 = rv.GraphSAGELayer(D, D, num_samples=32), rv.GraphSAGELayer(D, D, num_samples=32)
    h1 = rv.Buffer(N * D * 4)
    h2 = rv.Buffer(N * D * 4)
    l1.forward_device(xb, g, h1)
    l2.forward_device(h1, g, h2)
    rows = 2048
    assert np.any(np.diff(rp)[:rows] > 32)  # the sampled path is exercised
    ref1 = O.sage_forward(x, rp, col, wn, ws, rows=(0, rows), threads=16, num_samples=32)
    assert_close(h1.download(np.float32, (rows, D)), ref1)
    srp, scol, need = _sub(rp, col, rows)
    ref2 = O.sage_forward(h1.gather_rows(N, D, need), srp, scol, wn, ws, rows=(0, rows), threads=16, num_samples=32)
    assert_close(h2.download(np.float32, (rows, D)), ref2)


def test_c4_stack_on_hnsw_layer0_with_distance_features(hnsw_graph):
    x, xb, rp, col, dist = hnsw_graph
    g = rv.Graph.from_csr(rp, col, dist)
    eb = rv.Buffer.from_numpy(dist.reshape(-1, 1))
    layers = [rv.RuvectorLayer(D, D, 8, 0.0, seed=100 + i) for i in range(3)]
    head = EdgeFeaturedAttention(EdgeFeaturedConfig(node_dim=D, edge_dim=1, num_heads=8))
    bufs = [rv.Buffer(N * D * 4) for _ in range(3)]
    out = rv.Buffer(N * D * 4)
    src = xb
    for layer, b in zip(layers, bufs):
        layer.forward_graph_device(src, g, b)
        src = b
    head.forward_graph_device(src, g, eb, out)
    rows = 192
    srp, scol, need = _sub(rp, col, rows)
    sew = dist[:rp[rows]]
    inputs = [xb] + bufs[:2]
    for i, (layer, inp, b) in enumerate(zip(layers, inputs, bufs)):
        W = O.RvlWeights(json.loads(layer.to_json()))
        ref = O.rvl_forward_graph(W, inp.gather_rows(N, D, need), srp, scol, sew, rows=(0, rows), threads=16)
        assert_close(b.download(np.float32, (rows, D)), ref), f"layer {i + 1}"
    h3 = bufs[2]
    ref = np.stack([O.efa_compute(D, 1, 8, h3.gather_rows(N, D, [i])[0], h3.gather_rows(N, D, col[rp[i]:rp[i + 1]]),
                                  h3.gather_rows(N, D, col[rp[i]:rp[i + 1]]), dist[rp[i]:rp[i + 1]].reshape(-1, 1))
                    for i in range(rows)])
    assert_close(out.download(np.float32, (rows, D)), ref)
