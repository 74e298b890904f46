"""VectorDB storage semantics that need no device (crates/ruvector-core/src/
storage_memory.rs:68-99, vector_db.rs:154-168): a batch with an entry of the wrong
dimension stores the entries before it, raises DimensionMismatch, and indexes none
of them (VectorDB::insert_batch returns before index.add_batch)."""
import pytest

rv = pytest.importorskip("ruvector_amd")
from ruvector_amd.vector_db import DbOptions, VectorDB, VectorEntry  # noqa: E402


@pytest.mark.parametrize("hnsw", [True, False])
def test_mixed_batch_partial_store_like_the_reference(hnsw):
    opts = DbOptions(dimensions=4) if hnsw else DbOptions(dimensions=4, hnsw_config=None)
    db = VectorDB(opts)
    batch = [VectorEntry(vector=[1.0, 2.0, 3.0, 4.0], id="a"),
             VectorEntry(vector=[0.5, 0.5, 0.5, 0.5]),  # generated id vec_0
             VectorEntry(vector=[1.0, 2.0, 3.0]),         # wrong dimension: stops here
             VectorEntry(vector=[9.0, 9.0, 9.0, 9.0], id="d")]
    with pytest.raises(rv.RuvectorError) as e:
        db.insert_batch(batch)
    assert "DimensionMismatch" in str(e.value)
    assert len(db) == 2 and sorted(db.keys()) == ["a", "vec_0"]
    assert db.get("a").vector == [1.0, 2.0, 3.0, 4.0] and db.get("d") is None
    assert db.index.len() == 0  # stored, never indexed
