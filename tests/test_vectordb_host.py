"""VectorDB storage semantics that need no device (crates/ruvector-core/src/storage.rs:168-206,
vector_db.rs:154-168, default features incl. "storage" = redb, Cargo.toml:89): a batch with
an entry of the wrong dimension is one uncommitted write transaction — it raises
DimensionMismatch and stores and indexes none of its entries."""
import pytest

rv = pytest.importorskip("ruvector_amd")
from ruvector_amd.vector_db import DbOptions, VectorDB, VectorEntry  # noqa: E402


@pytest.mark.parametrize("hnsw", [True, False])
def test_mixed_batch_stores_nothing_like_the_default_build(hnsw):
    opts = DbOptions(dimensions=4) if hnsw else DbOptions(dimensions=4, hnsw_config=None)
    db = VectorDB(opts)
    batch = [VectorEntry(vector=[1.0, 2.0, 3.0, 4.0], id="a"),
             VectorEntry(vector=[0.5, 0.5, 0.5, 0.5]),  # generated id
             VectorEntry(vector=[1.0, 2.0, 3.0]),         # wrong dimension: the transaction never commits
             VectorEntry(vector=[9.0, 9.0, 9.0, 9.0], id="d")]
    with pytest.raises(rv.RuvectorError) as e:
        db.insert_batch(batch)
    assert "DimensionMismatch" in str(e.value)
    assert len(db) == 0 and db.keys() == []
    assert db.get("a") is None and db.get("d") is None
    assert db.index.len() == 0
