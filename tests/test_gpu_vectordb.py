"""VectorDB facade (crates/ruvector-core/src/vector_db.rs, types.rs) on the GPU indexes.

Checks the reference's semantics: HNSW iff hnsw_config is set (vector_db.rs:81-98);
search() ignores SearchQuery.ef_search and uses the configured one
(vector_db.rs:171-173 -> index/hnsw.rs:331-334); enrichment + metadata filter
(vector_db.rs:175-193); "vec_<n>" ids and DimensionMismatch (storage_memory.rs).
"""
import numpy as np
import pytest

import oracle as O

rv = pytest.importorskip("ruvector_amd")
from ruvector_amd.vector_db import DbOptions, SearchQuery, VectorDB, VectorEntry  # noqa: E402

pytestmark = pytest.mark.gpu


def test_index_kind_follows_hnsw_config():
    assert isinstance(VectorDB(DbOptions(dimensions=8)).index, rv.HnswIndex)
    assert isinstance(VectorDB(DbOptions(dimensions=8, hnsw_config=None)).index, rv.FlatIndex)
    d = DbOptions()
    assert (d.dimensions, d.distance_metric, d.hnsw_config.m, d.hnsw_config.ef_search) == \
        (384, rv.DistanceMetric.Cosine, 32, 100)


def test_search_ignores_query_ef_search():
    n, d = 3000, 32
    x = O.fill_uniform(n * d, 21).reshape(n, d)
    q = O.fill_uniform(40 * d, 22).reshape(40, d)
    cfg = rv.HnswConfig(m=4, ef_construction=16, ef_search=10)
    db = VectorDB(DbOptions(dimensions=d, distance_metric=rv.DistanceMetric.Euclidean, hnsw_config=cfg))
    ids = db.insert_batch([VectorEntry(vector=v) for v in x])
    assert ids[:3] == ["vec_0", "vec_1", "vec_2"] and len(db) == n
    differs = 0
    for qi in q:
        a = db.search(SearchQuery(vector=qi, k=10, ef_search=400))
        b = db.search(SearchQuery(vector=qi, k=10, ef_search=None))
        c = db.index.search_with_ef(qi, 10, cfg.ef_search)
        wide = db.index.search_with_ef(qi, 10, 400)
        assert [r.id for r in a] == [r.id for r in b] == [r.id for r in c]
        assert [r.score for r in a] == [r.score for r in c]
        differs += [r.id for r in a] != [r.id for r in wide]
    assert differs > 0, "test data must make ef 10 and ef 400 disagree for the check to mean anything"


def test_flat_search_enrichment_and_filter():
    n, d = 500, 16
    x = O.fill_uniform(n * d, 31).reshape(n, d)
    db = VectorDB(DbOptions(dimensions=d, distance_metric=rv.DistanceMetric.Euclidean, hnsw_config=None))
    ents = [VectorEntry(vector=x[i], id=f"doc{i}", metadata={"parity": i % 2, "tag": "t"} if i % 5 else None)
            for i in range(n)]
    assert db.insert_batch(ents)[7] == "doc7"
    q = O.fill_uniform(d, 32)
    res = db.search(SearchQuery(vector=q, k=20))
    rids, rd = O.flat_search(x, q[None], 20, "l2")
    assert [r.id for r in res] == [f"doc{i}" for i in rids[0]]
    assert np.array_equal(np.array([r.score for r in res], np.float32), rd[0])
    for r in res:
        assert np.array_equal(np.asarray(r.vector, np.float32), x[int(r.id[3:])])
        assert (r.metadata is None) == (int(r.id[3:]) % 5 == 0)
    flt = db.search(SearchQuery(vector=q, k=20, filter={"parity": 1}))
    assert [r.id for r in flt] == [r.id for r in res if r.metadata is not None and r.metadata["parity"] == 1]
    assert db.search(SearchQuery(vector=q, k=20, filter={"missing": 1})) == []
    # get / delete / len
    e = db.get("doc3")
    assert e.id == "doc3" and e.metadata == {"parity": 1, "tag": "t"}
    assert db.delete("doc3") and not db.delete("doc3") and db.get("doc3") is None and len(db) == n - 1
    assert "doc3" not in [r.id for r in db.search(SearchQuery(vector=x[3], k=5))]
    # re-insert overwrites: one row per id in the flat index
    db.insert(VectorEntry(vector=x[3], id="doc4"))
    top = db.search(SearchQuery(vector=x[3], k=3))
    assert top[0].id == "doc4" and top[0].score == 0.0 and [r.id for r in top].count("doc4") == 1


def test_dimension_mismatch():
    db = VectorDB(DbOptions(dimensions=4, hnsw_config=None))
    with pytest.raises(rv.RuvectorError) as e:
        db.insert(VectorEntry(vector=[1.0, 2.0, 3.0]))
    assert e.value.kind == "DimensionMismatch" and len(db) == 0
    db.insert(VectorEntry(vector=[1.0, 0.0, 0.0, 0.0]))
    with pytest.raises(rv.RuvectorError):
        db.search(SearchQuery(vector=[1.0, 0.0], k=1))


@pytest.mark.parametrize("hnsw", [True, False])
def test_failed_batch_leaves_earlier_rows_alone(hnsw):
    """storage.rs:168-206 (default redb build): a failing batch commits nothing; rows
    stored before it stay stored and indexed, and the valid entries go in together."""
    opts = DbOptions(dimensions=4) if hnsw else DbOptions(dimensions=4, hnsw_config=None)
    db = VectorDB(opts)
    db.insert(VectorEntry(vector=[0.0, 0.0, 0.0, 1.0], id="before"))
    batch = [VectorEntry(vector=[1.0, 2.0, 3.0, 4.0], id="a"), VectorEntry(vector=[1.0, 2.0, 3.0]),
             VectorEntry(vector=[9.0, 9.0, 9.0, 9.0], id="d")]
    with pytest.raises(rv.RuvectorError):
        db.insert_batch(batch)
    assert db.keys() == ["before"] and db.index.len() == 1
    ids = db.insert_batch([b for b in batch if len(b.vector) == 4])
    assert ids == ["a", "d"] and len(db) == 3 and db.index.len() == 3
    assert db.search(SearchQuery(vector=[9.0, 9.0, 9.0, 9.0], k=1))[0].id == "d"
