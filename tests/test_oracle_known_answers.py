"""Pin the CPU oracle against the reference's own known-answer tests.

Each test re-encodes a #[test] of the reference (file:line cited) and runs it
on the oracle restatement (oracle/oracle.cpp). These are the golden checks the
reference holds for this path; the committed fixtures under
tests/golden/ are checked in test_golden.py.
"""
import math

import numpy as np
import pytest

import oracle as O


# ---- crates/ruvector-core/src/distance.rs:113-166 -------------------------
def test_euclidean_distance():
    assert abs(O.distance([1, 2, 3], [4, 5, 6], "l2") - 5.196) < 0.01


def test_cosine_distance():
    assert O.distance([1, 2, 3], [1, 2, 3], "cosine") < 0.01
    assert O.distance([1, 0, 0], [-1, 0, 0], "cosine") > 1.5


def test_dot_product_distance():
    assert abs(O.distance([1, 2, 3], [4, 5, 6], "dot") + 32.0) < 0.01


def test_manhattan_distance():
    assert abs(O.distance([1, 2, 3], [4, 5, 6], "l1") - 9.0) < 0.01


def test_l2_is_sequential_f32_order():
    # the fallback sums (x-y)^2 left to right in f32 (distance.rs:37-41)
    rng = np.random.default_rng(0)
    a, b = rng.standard_normal(257).astype(np.float32), rng.standard_normal(257).astype(np.float32)
    s = np.float32(0)
    for x, y in zip(a, b):
        t = np.float32(x - y)
        s = np.float32(s + np.float32(t * t))
    assert O.distance(a, b, "l2") == np.float32(np.sqrt(s))


# ---- crates/ruvector-postgres/src/gnn/aggregators.rs:134-180 --------------
def _rows(msgs):
    # node 0 receives messages from nodes 1..len (aggregate over one CSR row)
    x = np.zeros((len(msgs) + 1, len(msgs[0])), np.float32)
    x[1:] = msgs
    rp = np.array([0, len(msgs)] + [len(msgs)] * len(msgs), np.int64)
    col = np.arange(1, len(msgs) + 1, dtype=np.int32)
    return x, rp, col


def test_sum_aggregate():
    x, rp, col = _rows([[1, 2], [3, 4], [5, 6]])
    assert O.aggregate(x, rp, col, "sum")[0].tolist() == [9.0, 12.0]


def test_mean_aggregate():
    x, rp, col = _rows([[1, 2], [3, 4], [5, 6]])
    assert O.aggregate(x, rp, col, "mean")[0].tolist() == [3.0, 4.0]


def test_max_aggregate():
    x, rp, col = _rows([[1, 6], [5, 2], [3, 4]])
    assert O.aggregate(x, rp, col, "max")[0].tolist() == [5.0, 6.0]


def test_weighted_aggregate():
    x, rp, col = _rows([[1, 2], [3, 4]])
    assert O.aggregate(x, rp, col, "sum", w=[2.0, 0.5])[0].tolist() == [3.5, 6.0]


# ---- message_passing.rs:199-232 -------------------------------------------
def test_build_adjacency_list():
    rp, col, _ = O.build_csr(3, [(0, 1), (1, 2), (2, 0)])
    adj = [col[rp[i]:rp[i + 1]].tolist() for i in range(3)]
    assert adj == [[2], [0], [1]]


def test_build_adjacency_drops_out_of_range_and_keeps_edge_order():
    rp, col, _ = O.build_csr(3, [(2, 0), (7, 0), (1, 0), (0, 5), (0, 0)])
    assert col[rp[0]:rp[1]].tolist() == [2, 1, 0]


def test_gcn_disconnected_node_keeps_features():
    x = np.array([[1.0], [2.0], [3.0]], np.float32)
    rp, col, _ = O.build_csr(3, [(0, 1)])
    w = O.sage_init(1, 1, 0)
    y = O.gcn_forward(x, rp, col, w, bias=np.zeros(1, np.float32))
    assert y[2, 0] == 3.0  # propagate returns the original features, then ReLU


# ---- graphsage.rs:251-294 --------------------------------------------------
def test_graphsage_forward_shape_and_normalization():
    wn, ws = O.sage_init(2, 2, 0), O.sage_init(2, 2, 1000)
    x = np.array([[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]], np.float32)
    rp, col, _ = O.build_csr(3, [(0, 1), (1, 2), (2, 0)])
    y = O.sage_forward(x, rp, col, wn, ws)
    assert y.shape == (3, 2)
    for row in y:
        n = math.sqrt(float(np.sum(row.astype(np.float64) ** 2)))
        assert abs(n - 1.0) < 1e-5 or n == 0.0


def test_graphsage_deterministic_init_formula():
    w = O.sage_init(3, 4, 1000)
    scale = np.float32(math.sqrt(np.float32(2.0) / np.float32(7.0)))
    i, j = 2, 3
    val = np.float32(np.fmod(np.float32(i * 4 + j + 1000) * np.float32(0.01), np.float32(1.0)))
    assert w[i, j] == np.float32((val - np.float32(0.5)) * scale)


# ---- crates/ruvector-gnn/src/search.rs:168-225 -----------------------------
def test_cosine_similarity():
    assert abs(O.cosine_similarity([1, 0, 0], [1, 0, 0]) - 1.0) < 1e-6
    assert abs(O.cosine_similarity([1, 0, 0], [0, 1, 0])) < 1e-6


def test_differentiable_search():
    idx, w = O.differentiable_search([1, 0, 0], [[1, 0, 0], [0.9, 0.1, 0], [0, 1, 0]], 2, 1.0)
    assert len(idx) == 2 and len(w) == 2
    assert idx[0] == 0
    assert float(np.sum(w)) <= 1.0 + 1e-6


# ---- crates/ruvector-gnn/src/layer.rs:459-546 -------------------------------
def _layer_json(in_dim, hidden, heads, dropout, seed=0):
    rng = np.random.default_rng(seed)

    def lin(i, o):
        return {"weights": {"v": 1, "dim": [o, i], "data": rng.normal(0, math.sqrt(2 / (i + o)), o * i).tolist()},
                "bias": {"v": 1, "dim": [o], "data": [0.0] * o}}
    return {"w_msg": lin(in_dim, hidden), "w_agg": lin(hidden, hidden),
            "w_update": {k: lin(hidden, hidden) for k in ("w_z", "u_z", "w_r", "u_r", "w_h", "u_h")},
            "attention": {"num_heads": heads, "head_dim": hidden // heads,
                          **{k: lin(hidden, hidden) for k in ("q_linear", "k_linear", "v_linear", "out_linear")}},
            "norm": {"gamma": {"v": 1, "dim": [hidden], "data": [1.0] * hidden},
                     "beta": {"v": 1, "dim": [hidden], "data": [0.0] * hidden}, "eps": 1e-5},
            "dropout": dropout}


def test_ruvector_layer_output_len():
    W = O.RvlWeights(_layer_json(4, 8, 2, 0.1))
    out = O.rvl_forward_one(W, [1, 2, 3, 4], [[0.5, 1, 1.5, 2], [2, 3, 4, 5]], [0.3, 0.7])
    assert out.shape == (8,) and np.all(np.isfinite(out))


def test_ruvector_layer_no_neighbors_is_layernorm():
    W = O.RvlWeights(_layer_json(4, 8, 2, 0.1))
    out = O.rvl_forward_one(W, [1, 2, 3, 4], [], [])
    assert out.shape == (8,)
    assert abs(float(np.mean(out))) < 1e-5  # LayerNorm test (layer.rs:471-480)


# ---- crates/ruvector-gnn/src/search.rs:227-245 (test_hierarchical_forward) ----
def test_hierarchical_forward_len():
    W = O.RvlWeights(_layer_json(2, 2, 1, 0.0))
    out = O.hierarchical_forward([1.0, 0.0], [[[1.0, 0.0], [0.0, 1.0]]], [W])
    assert out.shape == (2,) and np.all(np.isfinite(out))


def test_hierarchical_forward_walk_rules():
    """search.rs:109-111: no levels or no layers -> the query itself; :121-123 an empty
    level skips its paired layer; zip bounds the walk by the shorter list; one level
    equals the composition differentiable_search -> combine -> forward by hand."""
    W1, W2 = O.RvlWeights(_layer_json(4, 6, 2, 0.0, 1)), O.RvlWeights(_layer_json(6, 4, 2, 0.0, 2))
    q = np.array([0.3, -1.0, 0.5, 2.0], np.float32)
    emb1 = O.fill_uniform(7 * 4, 3).reshape(7, 4)
    emb2 = O.fill_uniform(3 * 6, 4).reshape(3, 6)
    assert np.array_equal(O.hierarchical_forward(q, [], [W1]), q)
    assert np.array_equal(O.hierarchical_forward(q, [emb1], []), q)
    one = O.hierarchical_forward(q, [emb1], [W1])
    idx, w = O.differentiable_search(q, emb1, 5, 1.0)
    agg = np.zeros(4, np.float32)
    for i, wt in zip(idx, w):
        agg = (agg + np.float32(wt) * emb1[i]).astype(np.float32)
    comb = ((q + agg) / np.float32(2.0)).astype(np.float32)
    assert np.array_equal(one, O.rvl_forward_one(W1, comb, emb1[idx], w))
    assert np.array_equal(O.hierarchical_forward(q, [emb1, emb2], [W1]), one)  # zip stops at 1
    two = O.hierarchical_forward(q, [emb1, emb2], [W1, W2])
    assert two.shape == (4,)
    # empty first level: W1 skipped, level 2 (dim 6) cannot pair with a dim-4 query
    skip = O.hierarchical_forward(q, [np.zeros((0, 4), np.float32), emb1], [W2, W1])
    assert np.array_equal(skip, one)


# ---- crates/ruvector-attention/src/graph/edge_featured.rs:327-393 ----------
def test_edge_featured_attention_len():
    out = O.efa_compute(64, 16, 4, [0.5] * 64, [[0.3] * 64] * 10, [[1.0] * 64] * 10, [[0.2] * 16] * 10)
    assert out.shape == (64,)
    # identical values: every head averages ones
    assert np.allclose(out, np.float32(O.efa_compute(64, 16, 4, [0.5] * 64, [[0.3] * 64] * 10, [[1.0] * 64] * 10,
                                                     [[0.2] * 16] * 10)))


def test_edge_featured_without_edges_and_leaky_relu():
    assert O.efa_compute(32, 8, 2, [0.5] * 32, [[0.3] * 32] * 5, [[1.0] * 32] * 5).shape == (32,)
    assert O.efa_compute(16, 4, 1, [-1.0] * 16, [[-0.5] * 16] * 3, [[1.0] * 16] * 3).shape == (16,)


def test_edge_featured_lcg_init_first_value():
    wn, *_ = O.efa_init(4, 1, 1)
    seed = (42 * 6364136223846793005 + 1) % (1 << 64)
    r = np.float32(np.float32(seed) / np.float32(2.0 ** 64)) - np.float32(0.5)
    node_scale = np.float32(math.sqrt(np.float32(2.0) / np.float32(4 + 4)))
    assert wn[0] == np.float32(np.float32(r * np.float32(2.0)) * node_scale)


# ---- crates/ruvector-attention/src/graph/dual_space.rs:296-411 --------------
def test_dual_space_reference_cases():
    # test_dual_space_basic, test_euclidean_dominant, test_hyperbolic_dominant
    assert O.dsa_compute(64, [0.1] * 64, [[0.1] * 64] * 10, [[1.0] * 64] * 10).shape == (64,)
    assert O.dsa_compute(32, [0.5] * 32, [[0.3] * 32] * 5, [[1.0] * 32] * 5, euclidean_weight=1.0,
                         hyperbolic_weight=0.0).shape == (32,)
    assert O.dsa_compute(32, [0.1] * 32, [[0.1] * 32] * 5, [[1.0] * 32] * 5, curvature=0.5, euclidean_weight=0.0,
                         hyperbolic_weight=1.0).shape == (32,)
    # empty keys: the reference's Err(InvalidConfig("Empty keys"))
    assert O.dsa_compute(16, [0.5] * 16, [], []) is None


def test_dual_space_temperature_and_identical_keys():
    # test_temperature_scaling: both compute; identical keys -> uniform weights, so the
    # pre-projection output is the values' mean and value_dim != dim skips the projection
    k2 = [[0.8] * 16, [0.2] * 16]
    v2 = [[1.0] * 16, [0.0] * 16]
    lo = O.dsa_compute(16, [0.5] * 16, k2, v2, temperature=0.5)
    hi = O.dsa_compute(16, [0.5] * 16, k2, v2, temperature=2.0)
    assert lo.shape == hi.shape == (16,) and np.all(np.isfinite(lo)) and np.all(np.isfinite(hi))
    vals = [[1.0, 2.0, 3.0], [3.0, 4.0, 5.0]]
    out = O.dsa_compute(8, [0.2] * 8, [[0.3] * 8] * 2, vals)
    assert np.allclose(out, [2.0, 3.0, 4.0], atol=1e-6)


def test_dual_space_lcg_init():
    we, wh, wo = O.dsa_init(4)
    w_scale = np.float32(math.sqrt(np.float32(2.0) / np.float32(8)))
    seed = 42
    vals = []
    for _ in range(3 * 16):
        seed = (seed * 6364136223846793005 + 1) % (1 << 64)
        r = np.float32(np.float32(seed) / np.float32(2.0 ** 64)) - np.float32(0.5)
        vals.append(np.float32(np.float32(r * np.float32(2.0)) * w_scale))
    assert np.array_equal(np.concatenate([we, wh, wo]), np.array(vals, np.float32))


# ---- crates/ruvector-hyperbolic-hnsw/tests/math_tests.rs:84-130 ------------
def test_poincare_metric_properties():
    rng = np.random.default_rng(1)
    pts = rng.uniform(-0.3, 0.3, (6, 8)).astype(np.float32)
    for a in pts:
        assert O.poincare_distance(a, a) < 1e-3  # identity (fast_acosh small-delta branch)
        for b in pts:
            assert abs(O.poincare_distance(a, b) - O.poincare_distance(b, a)) < 1e-6  # symmetry
            for c in pts:
                assert O.poincare_distance(a, c) <= O.poincare_distance(a, b) + O.poincare_distance(b, c) + 1e-5


def test_poincare_from_origin_is_2_atanh():
    x = np.array([0.3, 0.4, 0.0, 0.0], np.float32)  # |x| = 0.5
    assert abs(O.poincare_distance(np.zeros(4, np.float32), x) - 2 * math.atanh(0.5)) < 1e-5


# ---- crates/ruvector-core/tests/hnsw_integration_test.rs -------------------
def _unit_vectors(n, d, seed):
    v = O.fill_uniform(n * d, seed).reshape(n, d)
    nrm = np.sqrt(np.sum(v * v, axis=1, dtype=np.float32)).astype(np.float32)
    return (v / nrm[:, None]).astype(np.float32)


def _recall(gt, got):
    return np.mean([len(set(g.tolist()) & set(r.tolist())) / len(g) for g, r in zip(gt, got)])


def test_hnsw_100_vectors_recall():  # :57-118, m=16 ef_c=100 ef_s=200, >= 0.90
    x = _unit_vectors(100, 128, 12345)
    h = O.Hnsw(128, "cosine", m=16, ef_construction=100, seed=3)
    h.insert(x, threads=1)
    q = x[::10]
    ids, _, _ = h.search(q, 10, 200)
    gt, _ = O.flat_search(x, q, 10, "cosine")
    assert _recall(gt, ids) >= 0.90


def test_hnsw_1000_vectors_recall():  # :122-185, m=32 ef_c=200 ef_s=200, >= 0.95
    x = _unit_vectors(1000, 128, 42)
    h = O.Hnsw(128, "cosine", m=32, ef_construction=200, seed=4)
    h.insert(x, threads=4)
    q = x[::50]
    ids, _, _ = h.search(q, 10, 200)
    gt, _ = O.flat_search(x, q, 10, "cosine")
    assert _recall(gt, ids) >= 0.95


def test_hnsw_export_roundtrip_same_results():
    x = _unit_vectors(600, 32, 7)
    h = O.Hnsw(32, "l2", m=8, ef_construction=64, seed=5)
    h.insert(x, threads=4)
    g = h.export()
    assert g["row_ptr0"][-1] == len(g["col0"])
    h2 = O.Hnsw.from_graph(x, g, "l2")
    q = _unit_vectors(40, 32, 8)
    a = h.search(q, 10, 50)
    b = h2.search(q, 10, 50)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_hnsw_results_sorted():  # property_tests.rs:308-331
    x = _unit_vectors(300, 16, 9)
    h = O.Hnsw(16, "l2", m=8, ef_construction=50, seed=6)
    h.insert(x, threads=2)
    _, d, cnt = h.search(_unit_vectors(20, 16, 10), 10, 40)
    for row, c in zip(d, cnt):
        assert np.all(np.diff(row[:c]) >= 0)


# ---------------------------------------------------------------- HyperbolicHnsw
# crates/ruvector-hyperbolic-hnsw/tests/math_tests.rs, restated on the oracle
def _grid20():
    return [[0.1 * (i % 5), 0.05 * (i / 5)] for i in range(20)]


def test_hyp_insert_and_search_sorted():  # math_tests.rs:308-331
    h = O.Hyp(2)
    h.insert(np.array(_grid20(), np.float32))
    assert len(h) == 20
    ids, d, cnt = h.search([0.25, 0.125], 5)
    assert cnt[0] == 5 and np.all(np.diff(d[0]) >= 0)


def test_hyp_nearest_is_origin():  # math_tests.rs:334-354
    h = O.Hyp(2)
    h.insert(np.array([[0.0, 0.0], [0.5, 0.0], [0.0, 0.5], [0.3, 0.3]], np.float32))
    ids, _, _ = h.search([0.05, 0.05], 1)
    assert ids[0, 0] == 0


def test_hyp_edge_cases():  # math_tests.rs:357-375, 464-495
    h = O.Hyp(2)
    ids, _, cnt = h.search([0.1, 0.2], 5)
    assert cnt[0] == 0 and np.all(ids == -1)
    h.insert(np.array([[0.3, 0.2]], np.float32))
    ids, _, cnt = h.search([0.1, 0.2], 5)
    assert cnt[0] == 1 and ids[0, 0] == 0
    h3 = O.Hyp(2)
    h3.insert(np.array([[0.1 * i, 0.1] for i in range(3)], np.float32))
    assert h3.search([0.15, 0.1], 10)[2][0] == 3
    h2 = O.Hyp(2)
    h2.insert(np.array([[0.1, 0.2], [0.3, 0.1]], np.float32))
    h2.set_curvature(2.0)
    assert h2.search([0.2, 0.15], 2)[2][0] == 2


def test_hyp_search_performance_case():  # math_tests.rs:498-530
    h = O.Hyp(2)
    h.insert(np.array([[0.05 * (i % 10), 0.05 * (i // 10)] for i in range(100)], np.float32))
    for _ in range(10):
        assert h.search([0.25, 0.25], 10)[2][0] == 10


def test_hyp_frechet_mean_and_tangent_cache():  # math_tests.rs:219-305
    one = O.Hyp(2)
    one.insert(np.array([[0.3, 0.2]], np.float32))
    one.build_tangent_cache()
    assert np.allclose(one.centroid(), [0.3, 0.2], atol=1e-4)
    sym = O.Hyp(2)
    sym.insert(np.array([[0.3, 0.0], [-0.3, 0.0]], np.float32))
    sym.build_tangent_cache()
    assert np.linalg.norm(sym.centroid()) < 0.1
    tc = O.Hyp(3)
    tc.insert(np.array([[0.1, 0.2, 0.1], [-0.1, 0.15, 0.05], [0.2, -0.1, 0.1]], np.float32))
    tc.build_tangent_cache()
    assert np.linalg.norm(tc.centroid()) < 1.0 - 1e-5
    # tangent_distance_ordering: with one candidate kept, the tangent nearest is the hyperbolic nearest
    to = O.Hyp(2, prune_factor=1)
    to.insert(np.array([[0.1, 0.1], [0.2, 0.1], [0.5, 0.3]], np.float32))
    to.build_tangent_cache()
    ids, _ = to.search_with_pruning([0.12, 0.11], 1)
    exact, _ = to.brute_force([0.12, 0.11], 1)
    assert ids[0, 0] == exact[0, 0]
