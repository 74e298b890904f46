"""The drop-in boundary takes every k and ef the reference takes.

Reference behaviour: FlatIndex::search sorts every (id, distance) pair and truncates to
any k (crates/ruvector-core/src/index/flat.rs:63-64); hnsw_rs searches with
ef = max(ef_arg, k) and no cap (patches/hnsw_rs/src/hnsw.rs:1519, :913-1055);
search_with_pruning keeps k * prune_factor tangent candidates, unbounded
(crates/ruvector-hyperbolic-hnsw/src/hnsw.rs:469-470). The fused scans keep lists of
at most 128 entries and one wave's LDS holds R up to ~19k entries, so beyond those the
library takes the any-k scan (whole distance rows + radix select, k_select.hip) and the
HBM-resident R of the HNSW kernels (RG). Bar: ids and distances array_equal to the oracle.
"""
import numpy as np
import pytest

import oracle as O

rv = pytest.importorskip("ruvector_amd")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c1_like():
    n, d = 100_000, 128
    x = O.fill_uniform(n * d, 201).reshape(n, d)
    q = O.fill_uniform(40 * d, 202).reshape(40, d)
    return x, q


def test_flat_k1000_on_100k_x_128(c1_like):
    x, q = c1_like
    idx = rv.FlatIndex(128, rv.DistanceMetric.Euclidean)
    idx.add_array(x, np.arange(x.shape[0], dtype=np.uint64))
    ids, dist, cnt = idx.search_array(q, 1000)
    rids, rd = O.flat_search(x, q, 1000, "l2")
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)
    assert np.all(cnt == 1000)
    assert rv.scan_last_stats()["valu"] == q.shape[0]  # the any-k path answered


@pytest.mark.parametrize("metric", ["l2", "cosine", "dot", "l1"])
def test_any_k_metrics_deletions_and_batches(monkeypatch, metric):
    # several query batches (1 MB of distance rows per batch), tombstoned rows, k past
    # the live row count (empty slots), and duplicate rows (exact distance ties by id)
    monkeypatch.setenv("RVX_SCAN_WIDE_BUDGET_MB", "1")
    n, d, nq = 3000, 64, 70
    x = O.fill_uniform(n * d, 203).reshape(n, d)
    x[100:140] = x[0]  # 41 identical rows
    q = np.ascontiguousarray(np.concatenate([x[:3], O.fill_uniform((nq - 3) * d, 204).reshape(nq - 3, d)]))
    m = {"l2": rv.DistanceMetric.Euclidean, "cosine": rv.DistanceMetric.Cosine, "dot": rv.DistanceMetric.DotProduct,
         "l1": rv.DistanceMetric.Manhattan}[metric]
    idx = rv.FlatIndex(d, m)
    idx.add_batch([(str(i), x[i]) for i in range(n)])  # keys 0..n-1 in insertion order
    dead = np.arange(7, n, 13)
    for i in dead:
        assert idx.remove(str(int(i)))
    live = np.ones(n, bool)
    live[dead] = False
    for k in (129, 700, n):
        ids, dist, cnt = idx.search_array(q, k)
        rids, rd = O.flat_search(x, q, k, metric, deleted=(~live).astype(np.uint8))
        got = np.where(np.arange(k)[None, :] < cnt[:, None], ids.astype(np.int64), -1)
        assert np.array_equal(got, rids), (metric, k)
        assert np.array_equal(dist.view(np.uint32), rd.view(np.uint32)), (metric, k)
        assert np.all(cnt == min(k, int(live.sum())))


def test_any_k_large_rocprim_sort():
    # k > 8192 takes the segmented radix sort instead of the LDS bitonic sort
    n, d, k = 30_000, 32, 20_000
    x = O.fill_uniform(n * d, 205).reshape(n, d)
    q = O.fill_uniform(5 * d, 206).reshape(5, d)
    idx = rv.FlatIndex(d, rv.DistanceMetric.Euclidean)
    idx.add_array(x, np.arange(n, dtype=np.uint64))
    ids, dist, cnt = idx.search_array(q, k)
    rids, rd = O.flat_search(x, q, k, "l2")
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)


def test_vectordb_search_k200():
    # VectorDB.search(k=200): the flat configuration against the oracle, and the default
    # HNSW one (ef = max(ef_search, k) = 200) returning 200 results
    n, d = 5000, 48
    x = O.fill_uniform(n * d, 207).reshape(n, d)
    rids, rd = O.flat_search(x, x[17:18], 200, "l2")
    for hnsw in (None, rv.HnswConfig()):
        db = rv.VectorDB(rv.DbOptions(dimensions=d, distance_metric=rv.DistanceMetric.Euclidean, hnsw_config=hnsw))
        db.insert_batch([rv.VectorEntry(id=str(i), vector=x[i].tolist()) for i in range(n)])
        res = db.search(rv.SearchQuery(vector=x[17].tolist(), k=200))
        assert len(res) == 200
        if hnsw is None:
            assert [int(r.id) for r in res] == rids[0].tolist()
            assert np.array_equal(np.array([r.score for r in res], np.float32), rd[0])
        else:
            assert len(set(int(r.id) for r in res) & set(rids[0].tolist())) >= 180


def _hnsw_pair(n, d, m, efc, seed):
    x = O.fill_uniform(n * d, seed).reshape(n, d)
    h = O.Hnsw(d, "l2", m=m, ef_construction=efc, seed=3)
    h.insert(x)
    idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=m, ef_construction=efc, ef_search=100))
    idx.add_array(x, np.arange(n, dtype=np.uint64))
    idx.load_graph(h.export())
    return x, h, idx


@pytest.fixture(scope="module")
def wide_graph():
    return _hnsw_pair(30_000, 32, 8, 40, 208)


@pytest.mark.parametrize("k,ef,rg,bitmap", [(10, 16384, "0", "1"), (300, 16384, "0", "1"), (10, 25000, "0", "1"),
                                            (50, 2000, "1", "1"), (10, 70000, "0", "0")])
def test_hnsw_ef_past_8192_bit_exact(monkeypatch, wide_graph, k, ef, rg, bitmap):
    # ef 16384: R in one wave's LDS (one wave per CU); ef 25000: past the LDS, R in HBM;
    # rg 1 forces the HBM-resident R at an ef the LDS would hold; ef 70000 on the visited HASH
    # (bitmap 0): past the old 2^24-entry table cap (ef x 4 x 64 > 2^24), the table is
    # sized by the graph (2n slots: never more than half full) and its slots by bytes
    monkeypatch.setenv("RVX_HNSW_RG", rg)
    monkeypatch.setenv("RVX_HNSW_BITMAP", bitmap)
    x, h, idx = wide_graph
    q = O.fill_uniform(12 * 32, 209).reshape(12, 32)
    if ef > 30000:
        q = q[:4]
    ids, dist, cnt = idx.search_array(q, k, ef)
    rids, rd, rc = h.search(q, k, ef)
    assert np.array_equal(cnt, rc)
    assert np.array_equal(ids.astype(np.int64)[:, :k], rids)
    assert np.array_equal(dist, rd)


@pytest.mark.parametrize("ef,k", [(2000, 300), (6000, 10)])
def test_hnsw_hbm_r_buffer_and_merge_forms_bit_exact(monkeypatch, wide_graph, ef, k):
    # R in HBM (forced): admissions buffered in LDS and flushed into the HBM array (default,
    # RVX_HNSW_RG_BUF=1; many flushes at these ef on a 30k-node graph) and the one-merge-per-batch
    # form (0) give the oracle's ids and distances
    monkeypatch.setenv("RVX_HNSW_RG", "1")
    x, h, idx = wide_graph
    q = O.fill_uniform(24 * 32, 215).reshape(24, 32)
    rids, rd, rc = h.search(q, k, ef)
    for buf in ("1", "0"):
        monkeypatch.setenv("RVX_HNSW_RG_BUF", buf)
        ids, dist, cnt = idx.search_array(q, k, ef)
        assert rv.hnsw_last_search_stats()["r_in_hbm"]
        assert np.array_equal(cnt, rc), buf
        assert np.array_equal(ids.astype(np.int64)[:, :k], rids), buf
        assert np.array_equal(dist, rd), buf


@pytest.fixture(scope="module")
def long_list_graph():
    return _hnsw_pair(6000, 32, 48, 100, 217)  # layer-0 lists of up to 96 > one 64-lane slice


@pytest.mark.parametrize("rg", ["0", "1"])
def test_hnsw_whole_list_fresh_batches_bit_exact(monkeypatch, long_list_graph, rg):
    # a whole layer-0 list claimed first and its fresh neighbours admitted in batches of 64
    # (RVX_HNSW_COLLECT=1, default) or slice by slice (0): the oracle's ids and distances, with R
    # in LDS and in HBM
    monkeypatch.setenv("RVX_HNSW_RG", rg)
    x, h, idx = long_list_graph
    q = O.fill_uniform(40 * 32, 218).reshape(40, 32)
    for k, ef in ((10, 200), (50, 1500)):
        rids, rd, rc = h.search(q, k, ef)
        for col in ("1", "0"):
            monkeypatch.setenv("RVX_HNSW_COLLECT", col)
            ids, dist, cnt = idx.search_array(q, k, ef)
            assert np.array_equal(cnt, rc), (col, k, ef)
            assert np.array_equal(ids.astype(np.int64)[:, :k], rids), (col, k, ef)
            assert np.array_equal(dist, rd), (col, k, ef)


def test_hnsw_build_whole_list_batches_same_graph(monkeypatch):
    # the builder's layer searches with whole lists claimed first and fresh neighbours batched
    # (RVX_HNSW_COLLECT=1) build the same graph as slice by slice (0): layer-0 lists of up to 96
    n, d = 5000, 32
    x = O.fill_uniform(n * d, 219).reshape(n, d)
    graphs = []
    for col in ("1", "0"):
        monkeypatch.setenv("RVX_HNSW_COLLECT", col)
        idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=48, ef_construction=120, ef_search=50),
                           seed=5)
        idx.add_array(x, np.arange(n, dtype=np.uint64))
        graphs.append(idx.export_graph())
    assert int(np.max(np.diff(np.asarray(graphs[0]["row_ptr0"])))) > 64
    for key in ("levels", "row_ptr0", "col0"):
        assert np.array_equal(np.asarray(graphs[0][key]), np.asarray(graphs[1][key])), key


def test_flat_k_past_n_many_queries_small_budget(monkeypatch):
    # k > n over many queries — the wide scan's batches budget the whole per-query
    # footprint (row, selection histogram, min(k, n) keys) and select_topk sizes its keys by
    # min(k, n); a small budget forces many batches. Equal to the oracle, padding included.
    monkeypatch.setenv("RVX_SCAN_WIDE_BUDGET_MB", "8")
    n, d, nq, k = 200, 16, 20_000, 300
    x = O.fill_uniform(n * d, 213).reshape(n, d)
    q = O.fill_uniform(nq * d, 214).reshape(nq, d)
    idx = rv.FlatIndex(d, rv.DistanceMetric.Euclidean)
    idx.add_array(x, np.arange(n, dtype=np.uint64))
    ids, dist, cnt = idx.search_array(q, k)
    rids, rd = O.flat_search(x, q, k, "l2")
    assert np.all(cnt == n)
    got = np.where(np.arange(k)[None, :] < cnt[:, None], ids.astype(np.int64), -1)
    assert np.array_equal(got, rids) and np.array_equal(dist.view(np.uint32), rd.view(np.uint32))


@pytest.mark.parametrize("coop", ["0", "2"])
def test_hnsw_build_with_hbm_r_same_graph(monkeypatch, coop):
    # the builder's layer searches with R in HBM build the same graph as with R in LDS
    # (per-lane and LDS-staged distances)
    n, d = 6000, 64
    x = O.fill_uniform(n * d, 210).reshape(n, d)
    monkeypatch.setenv("RVX_HNSW_COOP", coop)
    graphs = []
    for rg in ("0", "1"):
        monkeypatch.setenv("RVX_HNSW_RG", rg)
        idx = rv.HnswIndex(d, rv.DistanceMetric.Euclidean, rv.HnswConfig(m=8, ef_construction=64, ef_search=50),
                           seed=5)
        idx.add_array(x, np.arange(n, dtype=np.uint64))
        graphs.append(idx.export_graph())
    for key in ("levels", "row_ptr0", "col0"):
        assert np.array_equal(np.asarray(graphs[0][key]), np.asarray(graphs[1][key])), key


def ball_points(n, d, seed, rmax=0.9):
    r = np.random.default_rng(seed)
    v = r.standard_normal((n, d)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return (v * (rmax * r.random((n, 1)))).astype(np.float32)


def test_pruned_k50_and_exact_k200_hyperbolic():
    # k * prune_factor = 500 tangent candidates (was capped at 128); exact Poincaré k 200
    n, d = 8000, 64
    x = ball_points(n, d, 211)
    q = ball_points(30, d, 212)
    o = O.Hyp(d, seed=13)
    o.insert(x)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=13))
    h.insert_batch(x)
    h.build_tangent_cache()
    o.build_tangent_cache()
    ids, dist, cnt = h.search_with_pruning_batch(q, 50)
    rids, rd = o.search_with_pruning(q, 50)
    assert np.array_equal(ids, rids) and np.array_equal(dist, rd)
    assert np.all(cnt == 50)
    ids, dist, _ = h.brute_force(q, 200)
    rids, rd = o.brute_force(q, 200)
    assert np.array_equal(ids, rids) and np.array_equal(dist, rd)
