"""MFMA-filtered exact scan (k_scan.hip k_scan_filter + k_scan_rerank).

The filter ranks rows with f16 MFMA dot products and recomputes the reference
distance (distance.rs:34-42, :52-63, :77-78 scalar order) only for rows that can
still be in the top-k, so FlatIndex::search / brute force results must be
bit-identical to the oracle's flat scan (flat.rs:36-76, ties by id) and to the
exact VALU scan — ids AND distances. RVX_SCAN_MFMA=2 forces the path at test
sizes; RVX_SCAN_MFMA_CHUNK_ROWS forces several conversion chunks.
"""
import numpy as np
import pytest

import oracle as O

rv = pytest.importorskip("ruvector_amd")
pytestmark = pytest.mark.gpu

METRICS = [(rv.DistanceMetric.Euclidean, "l2"), (rv.DistanceMetric.Cosine, "cosine"),
           (rv.DistanceMetric.DotProduct, "dot")]


def flat(x, metric):
    idx = rv.FlatIndex(x.shape[1], metric)
    idx.add_array(x, np.arange(len(x), dtype=np.uint64))
    return idx


def normal(n, d, seed):
    b = rv.Buffer(n * d * 4)
    b.fill_normal(n * d, seed)
    return b.download(np.float32, (n, d))


@pytest.mark.parametrize("metric,name", METRICS)
@pytest.mark.parametrize("k", [1, 10, 16])
def test_forced_filter_bit_exact(monkeypatch, metric, name, k):
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    n, d, nq = 20011, 64, 300
    x = O.fill_uniform(n * d, 41).reshape(n, d)
    q = O.fill_uniform(nq * d, 42).reshape(nq, d)
    ids, dist = flat(x, metric).brute_force_array(q, k)
    st = rv.scan_last_stats()
    assert st["mfma"] == nq and st["fallback"] == 0, st
    rids, rd = O.flat_search(x, q, k, name)
    assert np.array_equal(ids.astype(np.int64), rids)
    assert np.array_equal(dist, rd)


@pytest.mark.parametrize("wide", ["0", "1", "2", "3"])
@pytest.mark.parametrize("metric,name", METRICS)
@pytest.mark.parametrize("d", [32, 96, 256, 768])
def test_tile_shapes_bit_exact(monkeypatch, wide, metric, name, d):
    """Every filter tile shape (128^2, 256^2 and 256 rows x 128 queries, RVX_SCAN_WIDE) at depths that take
    the ring's unrolled k-loop (d/32 a multiple of 3), the generic one, and d < 64
    (fills two tiles ahead); ragged row and query counts."""
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_WIDE", wide)
    n, nq = 9001, 300
    x = normal(n, d, 50 + d)
    q = normal(nq, d, 51 + d)
    ids, dist = flat(x, metric).brute_force_array(q, 10)
    st = rv.scan_last_stats()
    # a query whose split list fills below its k-th value + 2 eps cannot be proven
    # complete and is re-run on the VALU scan (cosine's eps window is wide at this n)
    assert st["mfma"] == nq and st["fallback"] <= 3, st
    rids, rd = O.flat_search(x, q, 10, name)
    assert np.array_equal(ids.astype(np.int64), rids)
    assert np.array_equal(dist, rd)


@pytest.mark.parametrize("metric,name", METRICS)
def test_chunked_conversion_and_flat_search(monkeypatch, metric, name):
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_MFMA_CHUNK_ROWS", "2048")  # 6 chunks, ragged last one
    n, d, nq = 11000, 128, 257
    x = normal(n, d, 5)
    q = normal(nq, d, 6)
    ids, dist, _ = flat(x, metric).search_array(q, 10)
    assert rv.scan_last_stats()["mfma"] == nq
    rids, rd = O.flat_search(x, q, 10, name)
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)


def test_removed_rows_are_skipped(monkeypatch):
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    n, d = 6000, 32
    x = O.fill_uniform(n * d, 7).reshape(n, d)
    idx = rv.FlatIndex(d, rv.DistanceMetric.Euclidean)
    idx.add_batch([(f"v{i}", x[i]) for i in range(n)])
    gone = list(range(0, n, 3))
    for i in gone:
        assert idx.remove(f"v{i}")
    q = x[:200]
    ids, dist, _ = idx.search_array(q, 10)
    deleted = np.zeros(n, np.uint8)
    deleted[gone] = 1
    rids, rd = O.flat_search(x, q, 10, "l2", deleted=deleted)
    assert rv.scan_last_stats()["mfma"] == 200
    assert np.array_equal(dist, rd)
    # FlatIndex ids are its internal keys; map the oracle rows through the same order
    assert np.array_equal(ids.astype(np.int64), rids)


@pytest.mark.parametrize("band,cap", [("1", None), ("1", "8"), ("0", None)])
def test_duplicates_fall_back_and_stay_exact(monkeypatch, band, cap):
    # 40 copies of every base row: a split's list fills with equal values, so
    # completeness cannot be proven from the lists; those queries take the band pass
    # (every row within the proven bound, k_scan_band) or, band off or past its
    # capacity (RVX_SCAN_BAND_CAP), the exact VALU scan — the same bits every way
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_BAND", band)
    if cap:
        monkeypatch.setenv("RVX_SCAN_BAND_CAP", cap)
    d = 32
    base = O.fill_uniform(150 * d, 9).reshape(150, d)
    x = np.repeat(base, 40, axis=0)
    q = O.fill_uniform(260 * d, 10).reshape(260, d)
    for metric, name in METRICS:
        ids, dist = flat(x, metric).brute_force_array(q, 12)
        st = rv.scan_last_stats()
        assert st["mfma"] == 260, st
        assert st["second_pass"] >= st["band"] > 0 if band == "1" else st["band"] == 0, st
        if band == "1" and not cap:
            assert st["fallback"] == 0, st  # 40-row ties fit a band
        else:
            assert st["fallback"] > 0 and st["second_pass"] >= st["fallback"], st
        rids, rd = O.flat_search(x, q, 12, name)
        assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)


def test_unbounded_inputs_take_the_valu_scan(monkeypatch):
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    n, d = 3000, 32
    x = O.fill_uniform(n * d, 11).reshape(n, d)
    x[17, 3] = 3.0e30  # beyond the filter's 2^60 bound
    q = O.fill_uniform(300 * d, 12).reshape(300, d)
    ids, dist = flat(x, rv.DistanceMetric.Euclidean).brute_force_array(q, 10)
    st = rv.scan_last_stats()
    assert st["valu"] == 300, st
    rids, rd = O.flat_search(x, q, 10, "l2")
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)


@pytest.mark.parametrize("metric", [rv.DistanceMetric.Euclidean, rv.DistanceMetric.Cosine])
def test_auto_mode_matches_valu_scan_at_768(monkeypatch, metric):
    # auto mode takes the filter from 256 queries x 65536 rows; compare with the
    # VALU kernel on the same device data (both exact), C3's dimension
    n, d, nq = 70000, 768, 300
    x = normal(n, d, 13)
    q = normal(nq, d, 14)
    idx = flat(x, metric)
    monkeypatch.setenv("RVX_SCAN_MFMA", "1")
    ids, dist = idx.brute_force_array(q, 10)
    assert rv.scan_last_stats()["mfma"] == nq
    monkeypatch.setenv("RVX_SCAN_MFMA", "0")
    vids, vdist = idx.brute_force_array(q, 10)
    assert rv.scan_last_stats()["valu"] == nq
    assert np.array_equal(ids, vids) and np.array_equal(dist, vdist)


@pytest.mark.parametrize("metric,name", METRICS)
def test_shared_bound_across_chunks_with_planted_ties(monkeypatch, metric, name):
    """Splits share a per-query rejection bound (k-th listed value + 2 eps, min over
    splits and chunks). Plant, in the LAST conversion chunk, exact copies of each
    query's k-th nearest row from the first chunk: they tie with the k-th value and
    must still reach the rerank after earlier chunks tightened the bound."""
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_MFMA_CHUNK_ROWS", "4096")
    n, d, nq, k = 16384, 96, 260, 10
    x = normal(n, d, 61)
    q = normal(nq, d, 62)
    first = x[:4096]
    rids0, _ = O.flat_search(first, q[:64], k, name)
    for i in range(64):  # one planted tie per query for the first 64 queries
        x[n - 1 - i] = first[rids0[i, k - 1]]
    ids, dist = flat(x, metric).brute_force_array(q, k)
    assert rv.scan_last_stats()["mfma"] == nq
    rids, rd = O.flat_search(x, q, k, name)
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)


# ---- k > 16 (FKP-long lists, no shared bound) and the per-row-bound metrics ----
@pytest.mark.parametrize("metric,name", METRICS)
@pytest.mark.parametrize("k", [17, 64, 128])
def test_large_k_bit_exact(monkeypatch, metric, name, k):
    """k beyond one split's list: the rerank proves completeness from the union of the
    splits' lists (or re-runs the query on the VALU scan); results as the oracle."""
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    n, d, nq = 30011, 64, 260
    x = normal(n, d, 71)
    q = normal(nq, d, 72)
    ids, dist = flat(x, metric).brute_force_array(q, k)
    st = rv.scan_last_stats()
    assert st["mfma"] == nq, st
    rids, rd = O.flat_search(x, q, k, name)
    assert np.array_equal(ids.astype(np.int64), rids) and np.array_equal(dist, rd)


def ball_points(n, d, seed, rmax=0.9):
    r = np.random.default_rng(seed)
    v = r.standard_normal((n, d)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    return (v * (rmax * r.random((n, 1)))).astype(np.float32)


@pytest.mark.parametrize("d,wide", [(1024, "1"), (1024, "3"), (768, "1"), (768, "2"), (768, "3"), (128, "0"), (64, "1")])
@pytest.mark.parametrize("k", [10, 100])
def test_poincare_filter_matches_valu_and_oracle(monkeypatch, d, wide, k):
    """HyperbolicHnsw exact scan through the MFMA filter with per-row bounds
    (k_rows_to_f16_pr / k_scan_rerank_pr): ids and distances identical to the VALU
    Poincaré scan (K8) and to the oracle's exact scan on the C5 generator."""
    n, nq = 70_000 if d >= 768 else 30_000, 300
    x = ball_points(n, d, 80 + d)
    q = ball_points(nq, d, 81 + d)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=1, ef_construction=16, max_connections=4,
                                                  max_connections_0=8), dim=d)
    h.insert_batch(x)
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_WIDE", wide)
    ids, dist, _ = h.brute_force(q, k)
    st = rv.scan_last_stats()
    assert st["mfma"] == nq and st["fallback"] <= nq // 50, st
    monkeypatch.setenv("RVX_SCAN_MFMA", "0")
    vids, vdist, _ = h.brute_force(q, k)
    assert rv.scan_last_stats()["valu"] == nq
    assert np.array_equal(ids, vids) and np.array_equal(dist, vdist)
    o = O.Hyp.from_graph(x, h.export_graph())  # every point lies inside the ball: stored == x
    rids, rd = o.brute_force(q[:40], k)
    assert np.array_equal(ids[:40], rids) and np.array_equal(dist[:40], rd)


def test_poincare_filter_chunks_deletions_free_and_edge_rows(monkeypatch):
    """Several conversion chunks; rows on the ball's edge (lambda ~ 1e-5, the bound's
    relative width > 2^-6) send the whole call to the VALU scan."""
    d, n, nq = 128, 20_000, 260
    x = ball_points(n, d, 90)
    q = ball_points(nq, d, 91)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=2, ef_construction=16, max_connections=4,
                                                  max_connections_0=8), dim=d)
    h.insert_batch(x)
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_MFMA_CHUNK_ROWS", "4096")
    ids, dist, _ = h.brute_force(q, 10)
    assert rv.scan_last_stats()["mfma"] == nq
    monkeypatch.setenv("RVX_SCAN_MFMA", "0")
    vids, vdist, _ = h.brute_force(q, 10)
    assert np.array_equal(ids, vids) and np.array_equal(dist, vdist)
    edge = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=2, ef_construction=16, max_connections=4,
                                                     max_connections_0=8), dim=d)
    y = x.copy()
    y[5] *= 50.0  # projected onto the ball's edge
    edge.insert_batch(y)
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    ids, dist, _ = edge.brute_force(q, 10)
    assert rv.scan_last_stats()["valu"] == nq
    monkeypatch.setenv("RVX_SCAN_MFMA", "0")
    vids, vdist, _ = edge.brute_force(q, 10)
    assert np.array_equal(ids, vids) and np.array_equal(dist, vdist)


@pytest.mark.parametrize("d", [1024, 256])
def test_tangent_pruned_scan_through_the_filter(monkeypatch, d):
    """search_with_pruning's tangent scan (k * prune_factor = 100 candidates by
    tangent_distance_squared) through the MFMA filter gives the same candidates, hence
    the same results, as the VALU scan."""
    n, nq = 70_000, 300
    x = ball_points(n, d, 95)
    q = ball_points(nq, d, 96)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=3, ef_construction=16, max_connections=4,
                                                  max_connections_0=8), dim=d)
    h.insert_batch(x)
    h.build_tangent_cache()
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    ids, dist, _ = h.search_with_pruning_batch(q, 10)
    st = rv.scan_last_stats()
    assert st["mfma"] == nq and st["fallback"] <= nq // 50, st
    monkeypatch.setenv("RVX_SCAN_MFMA", "0")
    vids, vdist, _ = h.search_with_pruning_batch(q, 10)
    assert np.array_equal(ids, vids) and np.array_equal(dist, vdist)


@pytest.mark.parametrize("second", ["1", "0"])
def test_poincare_second_pass_same_bits(monkeypatch, second):
    """Queries whose first-pass lists cannot prove completeness run the filter again with the most
    splits the re-rank holds (RVX_SCAN_SECOND, default on) before any VALU fallback: the exact
    Poincaré top-k is the oracle's bit for bit either way (C5-shaped ball data, d 256)."""
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_SECOND", second)
    n, d, nq, k = 20000, 256, 300, 10
    r = np.random.default_rng(216)
    x = r.standard_normal((n, d)).astype(np.float32)
    x = (x / np.linalg.norm(x, axis=1, keepdims=True) * (0.9 * r.random((n, 1)))).astype(np.float32)
    q = r.standard_normal((nq, d)).astype(np.float32)
    q = (q / np.linalg.norm(q, axis=1, keepdims=True) * (0.9 * r.random((nq, 1)))).astype(np.float32)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=3), dim=d)
    h.insert_batch(x)
    ids, dist, _ = h.brute_force(q, k)
    st = rv.scan_last_stats()
    assert st["mfma"] == nq, st
    if second == "0":
        assert st["second_pass"] == 0, st
    rids, rd = O.hyp_scan_rows(x, q, k, threads=8)  # the oracle's exact Poincaré scan (poincare.rs order)
    assert np.array_equal(np.asarray(ids, np.int64), rids) and np.array_equal(dist, rd)


@pytest.mark.parametrize("band", ["1", "0"])
def test_poincare_band_pass_duplicates(monkeypatch, band):
    """Ball rows repeated 40 times: the exact Poincaré scan (and the tangent-pruned scan's squared
    L2) cannot prove completeness from FKP-long lists; the band pass (RVX_SCAN_BAND, default on)
    resolves the queries from every row within the bound, RVX_SCAN_BAND=0 sends them to the VALU
    scan: ids and distances are the oracle's (poincare.rs order) either way."""
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    monkeypatch.setenv("RVX_SCAN_BAND", band)
    d, k = 64, 10
    base = ball_points(500, d, 301)
    x = np.repeat(base, 40, axis=0)
    q = ball_points(300, d, 302)
    h = rv.HyperbolicHnsw(rv.HyperbolicHnswConfig(seed=4, ef_construction=16, max_connections=4,
                                                  max_connections_0=8), dim=d)
    h.insert_batch(x)
    ids, dist, _ = h.brute_force(q, k)
    st = rv.scan_last_stats()
    assert st["mfma"] == 300, st
    if band == "1":
        assert st["band"] > 0 and st["fallback"] == 0, st
    else:
        assert st["band"] == 0 and st["fallback"] > 0, st
    rids, rd = O.hyp_scan_rows(x, q, k, threads=8)
    assert np.array_equal(np.asarray(ids, np.int64), rids) and np.array_equal(dist, rd)
    h.build_tangent_cache()
    pids, pdist, _ = h.search_with_pruning_batch(q, k)
    monkeypatch.setenv("RVX_SCAN_MFMA", "0")
    vids, vdist, _ = h.search_with_pruning_batch(q, k)
    assert np.array_equal(pids, vids) and np.array_equal(pdist, vdist)


@pytest.mark.parametrize("metric,name", METRICS)
def test_band_pass_skips_removed_rows(monkeypatch, metric, name):
    """Duplicate-heavy rows (the lists cannot settle the queries, the band pass does) with every
    third row removed: the band kernel must skip the removed rows exactly as the lists do
    (NaN row factor), results equal to the oracle's scan over the live rows."""
    monkeypatch.setenv("RVX_SCAN_MFMA", "2")
    n_base, d = 200, 64
    base = O.fill_uniform(n_base * d, 231).reshape(n_base, d)
    x = np.repeat(base, 30, axis=0)
    n = len(x)
    idx = rv.FlatIndex(d, metric)
    idx.add_batch([(f"v{i}", x[i]) for i in range(n)])
    gone = list(range(0, n, 3))
    for i in gone:
        assert idx.remove(f"v{i}")
    q = O.fill_uniform(300 * d, 232).reshape(300, d)
    ids, dist, _ = idx.search_array(q, 10)
    st = rv.scan_last_stats()
    assert st["mfma"] == 300 and st["band"] > 0 and st["fallback"] == 0, st
    deleted = np.zeros(n, np.uint8)
    deleted[gone] = 1
    rids, rd = O.flat_search(x, q, 10, name, deleted=deleted)
    assert np.array_equal(dist, rd)
    assert np.array_equal(ids.astype(np.int64), rids)
