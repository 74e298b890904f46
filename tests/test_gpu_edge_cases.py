"""Edge cases of the reference API on the GPU path: empty indexes, k larger
than the index, a single stored vector, one-node graphs, dimension mismatches
(crates/ruvector-core/src/index/flat.rs:36-76, index/hnsw.rs:240-260,
hnsw.rs:472-486 test_dimension_mismatch; graphsage.rs:150-152 empty
neighbourhoods). Results are compared with the oracle where it has an answer."""
import numpy as np
import pytest

import oracle as O

rv = pytest.importorskip("ruvector_amd")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["flat", "hnsw"])
def test_search_on_empty_index_returns_nothing(kind):
    idx = (rv.FlatIndex(8, rv.DistanceMetric.Euclidean) if kind == "flat" else
           rv.HnswIndex(8, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=8, ef_construction=20, ef_search=10)))
    assert len(idx) == 0
    assert idx.search([0.0] * 8, 5) == []


@pytest.mark.parametrize("kind", ["flat", "hnsw"])
def test_k_larger_than_index(kind):
    n, d = 7, 16
    x = O.fill_uniform(n * d, 3).reshape(n, d)
    idx = (rv.FlatIndex(d, rv.DistanceMetric.Euclidean) if kind == "flat" else
           rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=4, ef_construction=16, ef_search=16)))
    idx.add_batch([(f"v{i}", x[i]) for i in range(n)])
    q = O.fill_uniform(d, 4)
    got = idx.search(q, 50)
    if kind == "flat":  # every stored vector, nearest first
        assert len(got) == n
        ids, dist = O.flat_search(x, q[None, :], n, "l2")
        ids, dist = ids[0], dist[0]
    else:  # hnsw_rs returns what the layer-0 search reached: the oracle's search of the same graph
        ids, dist, cnt = O.Hnsw.from_graph(x, idx.export_graph(), "l2").search(q[None, :], 50, 50)
        ids, dist = ids[0][:cnt[0]], dist[0][:cnt[0]]
    assert [r.id for r in got] == [f"v{i}" for i in ids]
    assert np.array_equal(np.array([r.score for r in got], np.float32), dist)


def test_single_vector_hnsw():
    idx = rv.HnswIndex(4, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=4, ef_construction=8, ef_search=8))
    idx.add_batch([("only", [1.0, 2.0, 3.0, 4.0])])
    got = idx.search([1.0, 2.0, 3.0, 4.5], 3)
    assert [r.id for r in got] == ["only"] and got[0].score == pytest.approx(0.5)


def test_dimension_mismatch_is_an_error():
    idx = rv.HnswIndex(3, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=4, ef_construction=8, ef_search=8))
    with pytest.raises(rv.RuvectorError):
        idx.add_batch([("a", [1.0, 2.0])])
    idx.add_batch([("a", [1.0, 2.0, 3.0])])
    with pytest.raises(rv.RuvectorError):
        idx.search([1.0, 2.0], 1)


def test_graphsage_single_isolated_node_and_all_isolated_graph():
    for n, d in ((1, 8), (5, 32)):
        x = O.fill_uniform(n * d, 9).reshape(n, d)
        rp = np.zeros(n + 1, np.int64)
        col = np.zeros(0, np.int32)
        g = rv.Graph.from_csr(rp, col)
        layer = rv.GraphSAGELayer(d, d, num_samples=4)
        y = layer.forward_graph(x, g)
        ref = O.sage_forward(x, rp, col, O.sage_init(d, d, 0), O.sage_init(d, d, 1000))
        assert np.max(np.abs(y - ref)) <= 1e-5 * max(1.0, float(np.max(np.abs(ref))))


def test_exact_scan_k_equals_n_and_duplicate_rows():
    # all rows identical: distances tie everywhere, ids ascend (ties by id)
    n, d = 300, 32
    x = np.tile(O.fill_uniform(d, 11), (n, 1)).astype(np.float32)
    idx = rv.FlatIndex(d, rv.DistanceMetric.Euclidean)
    idx.add_array(x, np.arange(n, dtype=np.uint64))
    q = O.fill_uniform(4 * d, 12).reshape(4, d)
    ids, dist, _ = idx.search_array(q, 16)
    rids, rd = O.flat_search(x, q, 16, "l2")
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)
    assert np.array_equal(rids[0], np.arange(16))


def test_hnsw_visited_bitmap_respects_the_hbm_budget(monkeypatch):
    """The per-slot visited bitmaps are only taken when min(nq, 1024) slots fit the
    budget (min(16 GiB, 1/4 of free HBM)); a small budget (forced here) selects the
    tagged hash, with the same results (the bitmap ignored free HBM)."""
    n, d = 200_000, 32
    x = O.fill_uniform(n * d, 91).reshape(n, d)
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=8, ef_construction=40, ef_search=40))
    idx.add_array(x, np.arange(n, dtype=np.uint64))
    q = O.fill_uniform(2000 * d, 92).reshape(2000, d)
    ids_a, dist_a, cnt_a = idx.search_array(q, 10, 64)
    st = rv.core.hnsw_last_search_stats()
    assert st["visited_bitmap"] and st["slots"] == 2000
    monkeypatch.setenv("RVX_HNSW_BITMAP_BUDGET_MB", "1")  # 25 KB per slot at 200k nodes -> 41 slots < 1024
    ids_b, dist_b, cnt_b = idx.search_array(q, 10, 64)
    st = rv.core.hnsw_last_search_stats()
    assert not st["visited_bitmap"]
    assert np.array_equal(ids_a, ids_b) and np.array_equal(dist_a, dist_b) and np.array_equal(cnt_a, cnt_b)
