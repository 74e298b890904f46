"""C4 stack parity (BASELINE configs[3]): 3 x RuvectorLayer(768, 768,
heads 8, dropout 0) then EdgeFeaturedAttention(node_dim 768, edge_dim 1, heads 8,
concat) over one CSR graph, compared as a STACK with the oracle's composition
(crates/ruvector-gnn/src/layer.rs:379-451 per node, three times, then
crates/ruvector-attention/src/graph/edge_featured.rs:196-258 per node with
keys = values = the layer-3 rows of the neighbours and the edge weight as the
1-d edge feature). Isolated rows take the reference's deg-0 paths
(LayerNorm(w_msg x), layer.rs:385-389; zero attention output).

Tolerance (north star 1e-5 relative), per layer and for the head: normwise
(1e-5 of max|ref| over the compared rows) and per row (||gpu_r - ref_r||_2 /
||ref_r||_2, tests/parity.py).
"""
import json

import numpy as np
import pytest

import oracle as O
from parity import row_rel_err

rv = pytest.importorskip("ruvector_amd")
from ruvector_amd.attention import EdgeFeaturedAttention, EdgeFeaturedConfig  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-5


def rel_err(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(float(np.max(np.abs(b))), 1e-30))


def _graph(n, deg, isolated, seed):
    rp, col = O.random_csr(n, deg, seed)
    keep = np.ones(n, bool)
    keep[isolated] = False
    rp2 = np.concatenate([[0], np.cumsum(np.where(keep, deg, 0))]).astype(np.int64)
    col2 = np.concatenate([col[i * deg:(i + 1) * deg] for i in range(n) if keep[i]]).astype(np.int32)
    return rp2, col2


@pytest.mark.parametrize("entry", ["graph", "exchange"])
def test_c4_stack_matches_oracle(entry):
    n, d, heads, deg = 640, 768, 8, 8
    isolated = [0, 5, 131, 257, 400, 639]
    rp, col = _graph(n, deg, isolated, 71)
    ew = O.fill_uniform(len(col), 72, 0.0, 1.0)
    x = O.fill_uniform(n * d, 73, -2.0, 2.0).reshape(n, d)
    g = rv.Graph.from_csr(rp, col, ew)
    layers = [rv.RuvectorLayer(d, d, heads, 0.0, seed=100 + i) for i in range(3)]
    ws = [O.RvlWeights(json.loads(l.to_json())) for l in layers]
    head = EdgeFeaturedAttention(EdgeFeaturedConfig(node_dim=d, edge_dim=1, num_heads=heads))

    xb = rv.Buffer.from_numpy(x)
    eb = rv.Buffer.from_numpy(ew)
    bufs = [rv.Buffer(n * d * 4) for _ in range(3)]
    out = rv.Buffer(n * d * 4)
    src = xb
    for i, l in enumerate(layers):
        if entry == "graph":
            l.forward_graph_device(src, g, bufs[i])
        else:
            l.forward_exchange(g, src, bufs[i], [0, n])
        src = bufs[i]
    if entry == "graph":
        head.forward_graph_device(src, g, eb, out)
    else:
        head.forward_exchange(g, src, eb, out, [0, n])
    got = [b.download(np.float32, (n, d)) for b in bufs]
    y = out.download(np.float32, (n, d))

    # oracle composition, layer by layer on every row (each layer's input is the
    # oracle's previous layer, so errors compound exactly as in the stack)
    h = x
    for i, W in enumerate(ws):
        h = O.rvl_forward_graph(W, h, rp, col, ew, threads=16)
        e = rel_err(got[i], h)
        assert e <= TOL, f"layer {i + 1}: relative error {e:.3e}"
        e = row_rel_err(got[i], h)
        assert e <= TOL, f"layer {i + 1}: per-row relative error {e:.3e}"
    rows = sorted(set(range(0, n, 2)) | set(isolated))
    ref = np.stack([O.efa_compute(d, 1, heads, h[i], h[col[rp[i]:rp[i + 1]]], h[col[rp[i]:rp[i + 1]]],
                                  ew[rp[i]:rp[i + 1]].reshape(-1, 1)) for i in rows])
    e = rel_err(y[rows], ref)
    assert e <= TOL, f"attention head: relative error {e:.3e}"
    e = row_rel_err(y[rows], ref)
    assert e <= TOL, f"attention head: per-row relative error {e:.3e}"
    assert len(rows) >= 256
    assert np.all(y[isolated] == 0.0) and np.all(ref[[rows.index(i) for i in isolated]] == 0.0)
