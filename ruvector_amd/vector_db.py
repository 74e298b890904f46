"""VectorDB — ruvector-core's query facade (crates/ruvector-core/src/vector_db.rs:22-235,
types.rs:11-126) over the rvx indexes.

Semantics kept from the reference:
  * the index is HnswIndex iff `DbOptions.hnsw_config` is set, FlatIndex otherwise
    (vector_db.rs:81-98);
  * `search(SearchQuery)` runs `index.search(vector, k)`, i.e. HnswIndex searches with
    the CONFIGURED `hnsw_config.ef_search` (index/hnsw.rs:331-334) —
    `SearchQuery.ef_search` is ignored, as in the reference (vector_db.rs:171-173);
  * results are enriched with the stored vector and metadata (vector_db.rs:175-181), then
    the metadata filter keeps results whose metadata holds every (key, value) pair
    (vector_db.rs:184-193); a result without metadata is dropped by any filter;
  * entries without an id get "vec_<n>" from a counter (storage_memory.rs:33-36);
    a vector of the wrong length is DimensionMismatch{expected, actual};
  * re-inserting an id overwrites the stored entry; FlatIndex keeps one row per id
    (its DashMap insert overwrites, index/flat.rs), HnswIndex keeps the old point in the
    graph under the same id (index/hnsw.rs:263-287 only re-points id_to_idx).

Storage is the in-memory backend (storage_memory.rs, the reference's non-`storage`
build): redb persistence and quantization are outside the hot path, so
`storage_path` and `quantization` are accepted and recorded but unused.

Thread model: the reference wraps the index in Arc<RwLock<..>> (vector_db.rs:22-26);
here one lock serialises writers against readers, and searches share it.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import _lib as L
from .core import DistanceMetric, FlatIndex, HnswConfig, HnswIndex, RuvectorError, SearchResult

_DEFAULT = object()


@dataclass
class VectorEntry:
    """VectorEntry (types.rs:23-31)."""
    vector: Sequence[float]
    id: Optional[str] = None
    metadata: Optional[Dict[str, Any]] = None


@dataclass
class SearchQuery:
    """SearchQuery (types.rs:34-44). `ef_search` is carried but not used by
    VectorDB.search, exactly as in the reference (vector_db.rs:171-173)."""
    vector: Sequence[float]
    k: int = 10
    filter: Optional[Dict[str, Any]] = None
    ef_search: Optional[int] = None


@dataclass
class DbOptions:
    """DbOptions (types.rs:59-71) with DbOptions::default (types.rs:117-126)."""
    dimensions: int = 384
    distance_metric: DistanceMetric = DistanceMetric.Cosine
    storage_path: str = "./ruvector.db"
    hnsw_config: Optional[HnswConfig] = field(default_factory=HnswConfig)
    quantization: Optional[str] = "Scalar"


class VectorDB:
    """VectorDB::new (vector_db.rs:36-126) with in-memory storage."""

    def __init__(self, options: Optional[DbOptions] = None, seed: int = 0):
        self.options = options or DbOptions()
        o = self.options
        if o.hnsw_config is not None:
            self._index = HnswIndex(o.dimensions, o.distance_metric, o.hnsw_config, seed=seed)
        else:
            self._index = FlatIndex(o.dimensions, o.distance_metric)
        self._vectors: Dict[str, np.ndarray] = {}
        self._metadata: Dict[str, Dict[str, Any]] = {}
        self._counter = 0
        self._lock = threading.RLock()

    @classmethod
    def with_dimensions(cls, dimensions: int) -> "VectorDB":
        """VectorDB::with_dimensions (vector_db.rs:129-135)."""
        return cls(DbOptions(dimensions=dimensions))

    @property
    def index(self):
        return self._index

    # ---- storage (storage_memory.rs) ------------------------------------------------
    def _check_dim(self, v: np.ndarray) -> None:
        if v.size != self.options.dimensions:
            raise RuvectorError(1, f"DimensionMismatch expected {self.options.dimensions} actual {v.size}")

    def _store(self, entries: Sequence[VectorEntry]) -> List[str]:
        """VectorStorage::insert_batch of the reference's default build (features
        "storage" = redb, ruvector-core Cargo.toml:89; storage.rs:168-206): the batch is
        one write transaction, and an entry of the wrong dimension returns
        DimensionMismatch before the commit — nothing of the batch is stored (and, as
        VectorDB::insert_batch returns before index.add_batch, vector_db.rs:154-165,
        nothing is indexed). The memory-only build (storage_memory.rs:68-99) would keep
        the entries before the bad one; this mirrors the default."""
        vecs = [L.f32c(e.vector).reshape(-1) for e in entries]
        for v in vecs:
            self._check_dim(v)
        ids = []
        for e, v in zip(entries, vecs):
            if e.id is not None:
                vid = e.id
            else:
                vid = f"vec_{self._counter}"
                self._counter += 1
            self._vectors[vid] = v.copy()
            if e.metadata is not None:
                self._metadata[vid] = dict(e.metadata)
            ids.append(vid)
        return ids

    def _index_add(self, ids: Sequence[str], vecs: Sequence[np.ndarray]) -> None:
        idx = self._index
        keys = np.empty(len(ids), np.uint64)
        for i, vid in enumerate(ids):
            old = idx._ids.get(vid)
            if old is not None and isinstance(idx, FlatIndex):
                idx.remove(vid)  # FlatIndex: one row per id
            k = idx._next
            idx._next += 1
            idx._ids[vid] = k  # HnswIndex: the old point keeps its name (idx_to_id) too
            idx._names[k] = vid
            keys[i] = k
        idx.add_array(np.stack(vecs), keys)

    # ---- VectorDB API ----------------------------------------------------------------
    def insert(self, entry: VectorEntry) -> str:
        """VectorDB::insert (vector_db.rs:138-146)."""
        return self.insert_batch([entry])[0]

    def insert_batch(self, entries: Sequence[VectorEntry]) -> List[str]:
        """VectorDB::insert_batch (vector_db.rs:154-168)."""
        with self._lock:
            if not entries:
                return []
            ids = self._store(entries)
            self._index_add(ids, [self._vectors[i] for i in ids])
            return ids

    def search(self, query: SearchQuery) -> List[SearchResult]:
        """VectorDB::search (vector_db.rs:166-195): index.search(vector, k) — the
        configured ef_search, never query.ef_search — then enrich and filter."""
        with self._lock:
            results = self._index.search(query.vector, int(query.k))
            for r in results:
                v = self._vectors.get(r.id)
                if v is not None:
                    r.vector = v.tolist()
                    r.metadata = dict(self._metadata[r.id]) if r.id in self._metadata else None
            if query.filter is not None:
                results = [r for r in results if r.metadata is not None and
                           all(key in r.metadata and r.metadata[key] == val for key, val in query.filter.items())]
            return results

    def search_batch(self, queries: np.ndarray, k: int):
        """Batched form of search without enrichment: (ids [nq][k] as str, scores [nq][k]),
        one GPU launch for the whole batch (same ef as search)."""
        with self._lock:
            ef = self.options.hnsw_config.ef_search if self.options.hnsw_config is not None else 0
            ids, dist, cnt = self._index.search_array(queries, int(k), ef)
            names = self._index._names
            out = [[names[int(ids[q, s])] for s in range(int(cnt[q])) if ids[q, s] != np.uint64(2**64 - 1)]
                   for q in range(ids.shape[0])]
            return out, dist

    def delete(self, vid: str) -> bool:
        """VectorDB::delete (vector_db.rs:198-207)."""
        with self._lock:
            if vid not in self._vectors:
                return False
            del self._vectors[vid]
            self._metadata.pop(vid, None)
            self._index.remove(vid)
            return True

    def get(self, vid: str) -> Optional[VectorEntry]:
        """VectorDB::get (vector_db.rs:210-212)."""
        with self._lock:
            v = self._vectors.get(vid)
            if v is None:
                return None
            md = self._metadata.get(vid)
            return VectorEntry(vector=v.tolist(), id=vid, metadata=dict(md) if md is not None else None)

    def len(self) -> int:
        return len(self._vectors)

    def __len__(self) -> int:
        return len(self._vectors)

    def is_empty(self) -> bool:
        return len(self._vectors) == 0

    def keys(self) -> List[str]:
        return list(self._vectors)
