"""RuvectorQuery (crates/ruvector-gnn/src/query.rs) and its GNN-enhanced search on the GPU.

The reference defines the query configuration (mode, k, ef, gnn_depth,
temperature; defaults query.rs:44-58) and the pieces — HNSW search,
RuvectorLayer::forward(node, neighbours, edge_weights) (layer.rs:379-423) and
differentiable_search (search.rs:56-94) — but no batched executor. NeuralSearch
composes them for a whole query batch resident in HBM:

  1. cand = HNSW top-`ef` of each query (index.search_device, k = ef)
  2. w    = softmax(cos(q, cand) / T) in candidate order (differentiable_search's weights)
  3. h    = q; gnn_depth times: h = RuvectorLayer::forward(h, cand, w)
  4. (pos, weight) = differentiable_search(h, cand, k, T); result ids = cand[pos]

Every step is a device call; only the final [nq][k] ids/weights come back.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .device import Buffer
from .gnn import GnnError, RuvectorLayer, differentiable_search_device

EMPTY = np.uint64(0xFFFFFFFFFFFFFFFF)


class QueryMode(enum.Enum):
    """QueryMode (query.rs:9-19)."""
    VectorSearch = 0
    NeuralSearch = 1
    SubgraphExtraction = 2
    DifferentiableSearch = 3


@dataclass
class RuvectorQuery:
    """RuvectorQuery (query.rs:22-58); defaults as Default::default()."""
    vector: Optional[Sequence[float]] = None
    text: Optional[str] = None
    node_id: Optional[int] = None
    mode: QueryMode = QueryMode.VectorSearch
    k: int = 10
    ef: int = 50
    gnn_depth: int = 2
    temperature: float = 1.0
    return_attention: bool = False

    @classmethod
    def vector_search(cls, vector, k: int) -> "RuvectorQuery":
        return cls(vector=vector, mode=QueryMode.VectorSearch, k=k)

    @classmethod
    def neural_search(cls, vector, k: int, gnn_depth: int) -> "RuvectorQuery":
        return cls(vector=vector, mode=QueryMode.NeuralSearch, k=k, gnn_depth=gnn_depth)

    @classmethod
    def subgraph_search(cls, vector, k: int) -> "RuvectorQuery":
        return cls(vector=vector, mode=QueryMode.SubgraphExtraction, k=k)

    @classmethod
    def differentiable_search(cls, vector, k: int, temperature: float) -> "RuvectorQuery":
        return cls(vector=vector, mode=QueryMode.DifferentiableSearch, k=k, temperature=temperature)


class NeuralSearch:
    """Batched QueryMode::NeuralSearch over an HNSW index whose vectors are `table`
    (row i = id i, as after index.add_device(table, n, 0)).

    layers[i] runs at depth i; every layer must map dim -> dim (the re-embedded
    query is compared with the raw candidates by cosine similarity).
    """

    def __init__(self, index, table: Buffer, table_rows: int, dim: int, layers: Sequence[RuvectorLayer]):
        for l in layers:
            if l.input_dim != dim or l.hidden_dim != dim:
                raise GnnError(1, f"layer {l.input_dim}->{l.hidden_dim} does not map dim {dim} to itself")
        self.index, self.table, self.rows, self.dim, self.layers = index, table, int(table_rows), int(dim), list(layers)
        self._bufs = {}

    def _buf(self, name: str, nbytes: int) -> Buffer:
        b = self._bufs.get(name)
        if b is None or b.nbytes < nbytes:
            b = Buffer(nbytes)
            self._bufs[name] = b
        return b

    def run_device(self, q: Buffer, nq: int, query: RuvectorQuery) -> Tuple[Buffer, Buffer, Buffer]:
        """Device buffers (cand ids [nq][ef] u64, positions [nq][k] i64, weights [nq][k] f32)."""
        if query.gnn_depth > len(self.layers):
            raise GnnError(1, f"gnn_depth {query.gnn_depth} > {len(self.layers)} layers")
        c = min(int(query.ef), self.rows)
        k, d, T = int(query.k), self.dim, float(query.temperature)
        if c <= 0:
            raise GnnError(1, "empty index")
        cand = self._buf("cand", nq * c * 8)
        dist = self._buf("dist", nq * c * 4)
        self.index.search_device(q, nq, c, max(c, int(query.ef)), cand, dist)
        soft = self._buf("soft", nq * c * 4)
        differentiable_search_device(q, nq, self.table, self.rows, cand, c, d, 0, T, soft=soft)
        h = q
        for i in range(query.gnn_depth):
            out = self._buf(f"h{i & 1}", nq * d * 4)
            self.layers[i].forward_star_device(h, nq, self.table, self.rows, cand, c, soft, out)
            h = out
        pos = self._buf("pos", nq * max(k, 1) * 8)
        w = self._buf("w", nq * max(k, 1) * 4)
        differentiable_search_device(h, nq, self.table, self.rows, cand, c, d, k, T, idx=pos, w=w)
        return cand, pos, w

    def search(self, queries: np.ndarray, query: Optional[RuvectorQuery] = None) -> Tuple[np.ndarray, np.ndarray]:
        """Host convenience: ids [nq][k] u64 (EMPTY padded) and weights [nq][k]."""
        query = query or RuvectorQuery(mode=QueryMode.NeuralSearch)
        qa = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, self.dim)
        nq = qa.shape[0]
        qb = Buffer.from_numpy(qa)
        cand, pos, w = self.run_device(qb, nq, query)
        c, k = min(int(query.ef), self.rows), int(query.k)
        cids = cand.download(np.uint64, (nq, c))
        p = pos.download(np.int64, (nq, k))
        ww = w.download(np.float32, (nq, k))
        ids = np.full((nq, k), EMPTY, np.uint64)
        ok = p >= 0
        ids[ok] = cids[np.nonzero(ok)[0], p[ok]]
        return ids, ww
