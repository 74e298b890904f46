"""HyperbolicHnsw on the GPU: the Python mirror of
crates/ruvector-hyperbolic-hnsw/src/hnsw.rs:127-528 (and shard.rs:354-373).

Vectors are projected into the Poincaré ball on insert; ids are insertion
order; search / search_with_pruning / build_tangent_cache / set_curvature keep
the reference's semantics (include/rvx/rvx.h, rvx_hyperbolic_*). Batch forms
take numpy arrays or HBM Buffers.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .core import export_graph_handle, load_graph_handle
from .device import Buffer


class HyperbolicError(L.RvxError):
    """HyperbolicError (crates/ruvector-hyperbolic-hnsw/src/error.rs)."""


def _check(name, *args):
    try:
        L.call(name, *args)
    except L.RvxError as e:
        raise HyperbolicError(e.code, str(e).split(": ", 1)[-1]) from None


@dataclass
class HyperbolicHnswConfig:
    """HyperbolicHnswConfig (hnsw.rs:36-72). metric: "poincare" (default) or "euclidean"
    (DistanceMetric::Euclidean: sqrt of fused_norms' chunked |a-b|^2, hnsw.rs:182-185)."""
    max_connections: int = 16
    max_connections_0: int = 32
    ef_construction: int = 200
    ef_search: int = 50
    level_mult: float = 1.0 / math.log(16.0)
    curvature: float = 1.0
    prune_factor: int = 10
    use_tangent_pruning: bool = True
    seed: int = 0
    metric: str = "poincare"


@dataclass(frozen=True)
class SearchResult:
    id: int
    distance: float


class HyperbolicHnsw:
    """HyperbolicHnsw (hnsw.rs:127-528). The dimension is fixed by the first insert."""

    def __init__(self, config: Optional[HyperbolicHnswConfig] = None, dim: Optional[int] = None):
        self.config = config or HyperbolicHnswConfig()
        self._h = None
        self._dim = None
        if dim is not None:
            self._create(dim)

    @classmethod
    def default_config(cls) -> "HyperbolicHnsw":
        return cls()

    def _create(self, dim: int) -> None:
        c = self.config
        cfg = L.HyperbolicConfig(dim=int(dim), max_connections=c.max_connections,
                                 max_connections_0=c.max_connections_0, ef_construction=c.ef_construction,
                                 ef_search=c.ef_search, level_mult=c.level_mult, curvature=c.curvature,
                                 prune_factor=c.prune_factor, seed=c.seed,
                                 metric=L.METRIC_HYP_L2 if c.metric == "euclidean" else L.METRIC_POINCARE)
        h = C.c_void_p()
        _check("rvx_hyperbolic_create", C.byref(cfg), C.byref(h))
        self._h, self._dim = h, int(dim)

    # ---- size ------------------------------------------------------------
    def __len__(self) -> int:
        if self._h is None:
            return 0
        n = C.c_int64()
        _check("rvx_hyperbolic_len", self._h, C.byref(n))
        return n.value

    def is_empty(self) -> bool:
        return len(self) == 0

    def dim(self) -> Optional[int]:
        return self._dim if len(self) else None

    # ---- insert ----------------------------------------------------------
    def insert(self, vector: Sequence[float]) -> int:
        return int(self.insert_batch(np.asarray(vector, np.float32).reshape(1, -1))[0])

    def insert_batch(self, vectors) -> List[int]:
        v = L.f32c(vectors)
        if v.ndim == 1:
            v = v.reshape(1, -1)
        if self._h is None:
            self._create(v.shape[1])
        if v.shape[1] != self._dim:
            raise HyperbolicError(1, f"expected dimension {self._dim}, got {v.shape[1]}")
        first = C.c_int64()
        _check("rvx_hyperbolic_insert_batch", self._h, L.fptr(v), v.shape[0], C.byref(first))
        return list(range(first.value, first.value + v.shape[0]))

    def insert_device(self, vectors: Buffer, n: int, dim: int) -> int:
        """n rows of an HBM buffer [n][dim]; returns the first new id."""
        if self._h is None:
            self._create(dim)
        first = C.c_int64()
        _check("rvx_hyperbolic_insert_batch_device", self._h, vectors.handle, int(n), C.byref(first))
        return first.value

    # ---- search ----------------------------------------------------------
    def _batch(self, fn, q, k, *extra):
        q = L.f32c(q).reshape(-1, self._dim)
        nq = q.shape[0]
        ids = np.empty((nq, k), np.int64)
        d = np.empty((nq, k), np.float32)
        cnt = np.empty(nq, np.int32)
        if fn == "rvx_hyperbolic_brute_force":
            _check(fn, self._h, L.fptr(q), nq, k, L.i64ptr(ids), L.fptr(d))
            cnt[:] = (ids >= 0).sum(1)
        elif fn == "rvx_hyperbolic_search":
            _check(fn, self._h, L.fptr(q), nq, k, int(extra[0]), L.i64ptr(ids), L.fptr(d), L.i32ptr(cnt))
        else:
            _check(fn, self._h, L.fptr(q), nq, k, L.i64ptr(ids), L.fptr(d), L.i32ptr(cnt))
        return ids, d, cnt

    @staticmethod
    def _results(ids, d, cnt) -> List[SearchResult]:
        return [SearchResult(int(ids[0, s]), float(d[0, s])) for s in range(int(cnt[0]))]

    def search(self, query: Sequence[float], k: int) -> List[SearchResult]:
        if self.is_empty():
            return []
        return self._results(*self._batch("rvx_hyperbolic_search", query, k, 0))

    def search_batch(self, queries, k: int, ef: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        return self._batch("rvx_hyperbolic_search", queries, k, ef)

    def search_with_pruning(self, query: Sequence[float], k: int) -> List[SearchResult]:
        if self.is_empty():
            return []
        if not self.config.use_tangent_pruning:
            return self.search(query, k)
        return self._results(*self._batch("rvx_hyperbolic_search_with_pruning", query, k))

    def search_with_pruning_batch(self, queries, k: int):
        return self._batch("rvx_hyperbolic_search_with_pruning", queries, k)

    def brute_force(self, queries, k: int):
        """Exact scan by the index distance (ground truth, k <= 128)."""
        return self._batch("rvx_hyperbolic_brute_force", queries, k)

    def search_device(self, queries: Buffer, nq: int, k: int, ids: Buffer, dist: Buffer, ef: int = 0,
                      mode: int = 0) -> None:
        """HBM-resident queries/outputs (ids int64 [nq][k]); mode 0 search, 1 exact, 2 pruned."""
        _check("rvx_hyperbolic_search_device", self._h, queries.handle, int(nq), int(k), int(ef), int(mode),
               ids.handle, dist.handle)

    # ---- tangent cache / curvature ---------------------------------------
    def build_tangent_cache(self) -> None:
        if self._h is not None:
            _check("rvx_hyperbolic_build_tangent_cache", self._h)

    def tangent_centroid(self) -> np.ndarray:
        out = np.empty(self._dim, np.float32)
        _check("rvx_hyperbolic_tangent_centroid", self._h, L.fptr(out))
        return out

    def set_curvature(self, curvature: float) -> None:
        if curvature <= 0.0:
            raise HyperbolicError(2, f"invalid curvature {curvature}")
        self.config.curvature = float(curvature)
        if self._h is not None:
            _check("rvx_hyperbolic_set_curvature", self._h, float(curvature))

    def get_vector(self, id: int) -> Optional[np.ndarray]:
        if id < 0 or id >= len(self):
            return None
        out = np.empty(self._dim, np.float32)
        _check("rvx_hyperbolic_get_vector", self._h, int(id), L.fptr(out))
        return out

    def vectors(self) -> List[np.ndarray]:
        return [self.get_vector(i) for i in range(len(self))]

    # ---- graph interchange (rvx_hnsw_graph layout) -------------------------
    def _index(self):
        ix = C.c_void_p()
        _check("rvx_hyperbolic_index", self._h, C.byref(ix))
        return ix

    def export_graph(self) -> dict:
        return export_graph_handle(self._index())

    def load_graph(self, graph: dict) -> None:
        load_graph_handle(self._index(), graph)

    def __del__(self):
        try:
            if self._h is not None:
                L.call("rvx_hyperbolic_destroy", self._h)
                self._h = None
        except Exception:
            pass


def merge_shard_results(per_shard: Sequence[Tuple[np.ndarray, np.ndarray]], k: int) -> Tuple[np.ndarray, np.ndarray]:
    """ShardedHyperbolicHnsw::search merge (shard.rs:354-373): concatenate the
    shards' (global id, distance) lists, sort by distance (stable in shard
    order, -1 padding last), truncate to k."""
    ids = np.concatenate([p[0] for p in per_shard], axis=1)
    d = np.concatenate([p[1] for p in per_shard], axis=1)
    d = np.where(ids < 0, np.inf, d)
    order = np.argsort(d, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(ids, order, 1), np.take_along_axis(d, order, 1)


@dataclass
class ShardedHyperbolicHnsw:
    """ShardedHyperbolicHnsw (shard.rs:220-373) over node-range shards: shard s
    holds global ids [offsets[s], offsets[s+1]); search scatters the queries to
    every shard and merges. Each shard is a HyperbolicHnsw on this process's
    device; across GPUs, one process per shard and the same merge."""
    curvature: float = 1.0
    config: HyperbolicHnswConfig = field(default_factory=HyperbolicHnswConfig)
    shards: List[HyperbolicHnsw] = field(default_factory=list)
    offsets: List[int] = field(default_factory=lambda: [0])

    def add_shard(self, vectors) -> int:
        cfg = HyperbolicHnswConfig(**{**self.config.__dict__, "curvature": self.curvature})
        s = HyperbolicHnsw(cfg)
        s.insert_batch(vectors)
        self.shards.append(s)
        self.offsets.append(self.offsets[-1] + len(s))
        return len(self.shards) - 1

    def __len__(self) -> int:
        return self.offsets[-1]

    def num_shards(self) -> int:
        return len(self.shards)

    def search_batch(self, queries, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """(global ids, distances) [nq][k] of the merged search (-1 / inf past the end)."""
        parts = []
        for s, base in zip(self.shards, self.offsets):
            ids, d, _ = s.search_batch(queries, k)
            parts.append((np.where(ids >= 0, ids + base, -1), d))
        return merge_shard_results(parts, k)

    def search(self, query, k: int) -> List[Tuple[int, SearchResult]]:
        """Vec<(global_id, SearchResult{id: local_id, distance})> (shard.rs:354-373)."""
        ids, d = self.search_batch(np.asarray(query, np.float32).reshape(1, -1), k)
        out = []
        for g, x in zip(ids[0], d[0]):
            if g < 0:
                continue
            s = int(np.searchsorted(self.offsets, g, side="right")) - 1
            out.append((int(g), SearchResult(int(g) - self.offsets[s], float(x))))
        return out


SEARCH_MODES = {"search": 0, "exact": 1, "pruned": 2}


class ShardedHyperbolicSearch:
    """ShardedHyperbolicHnsw::search (shard.rs:354-373) with one node-range shard per
    process / GPU (SURVEY.md §8e option 2): this process's HyperbolicHnsw holds global
    ids [id_base, id_base + len). search_batch broadcasts rank 0's queries, searches
    every shard, all-gathers each rank's top-k over `comm` (RcclComm over xGMI, or any
    communicator handle of librvx; None = one process) and merges on the GPU
    (rvx_hyperbolic_sharded_search). mode: "search" (what shard.search runs,
    hnsw.rs:427), "exact" or "pruned" (search_with_pruning, hnsw.rs:450)."""

    def __init__(self, shard: HyperbolicHnsw, comm=None, id_base: int = 0):
        if shard._h is None:
            raise HyperbolicError(2, "the shard needs a dimension (create it with dim= or insert first)")
        self.shard, self.comm, self.id_base = shard, comm, int(id_base)

    @property
    def rank(self) -> int:
        return 0 if self.comm is None else int(self.comm.rank)

    def search_batch(self, queries, k: int, ef: int = 0, mode: str = "search"):
        """queries [nq][dim] (read on rank 0; other ranks pass nq or an array of that
        shape). Returns (global ids, local ids, distances, counts), same on every rank."""
        d = self.shard._dim
        if isinstance(queries, (int, np.integer)):
            nq, q = int(queries), None
        else:
            q = L.f32c(queries).reshape(-1, d)
            nq = q.shape[0]
        # rank 0 without queries is reported by the library on every rank (a Python-side
        # raise on one rank would leave the others waiting in the collective)
        gid = np.empty((nq, k), np.int64)
        lid = np.empty((nq, k), np.int64)
        dist = np.empty((nq, k), np.float32)
        cnt = np.empty(nq, np.int32)
        _check("rvx_hyperbolic_sharded_search", self.shard._h, self.comm._h if self.comm is not None else None,
               self.id_base, L.fptr(q) if q is not None else None, nq, int(k), int(ef), SEARCH_MODES[mode],
               L.i64ptr(gid), L.i64ptr(lid), L.fptr(dist), L.i32ptr(cnt))
        return gid, lid, dist, cnt

    def search(self, query, k: int) -> List[Tuple[int, SearchResult]]:
        """Vec<(global_id, SearchResult{id: local_id, distance})>, as shard.rs:354-373."""
        q = None if query is None else np.asarray(query, np.float32).reshape(1, -1)
        gid, lid, dist, cnt = self.search_batch(q if q is not None else 1, k)
        return [(int(gid[0, s]), SearchResult(int(lid[0, s]), float(dist[0, s]))) for s in range(int(cnt[0]))]

    def search_device(self, queries: Optional[Buffer], nq: int, k: int, gid: Buffer, dist: Buffer,
                      lid: Optional[Buffer] = None, ef: int = 0, mode: str = "search") -> None:
        """HBM-resident form: queries on rank 0, outputs (int64 ids) on every rank."""
        _check("rvx_hyperbolic_sharded_search_device", self.shard._h,
               self.comm._h if self.comm is not None else None, self.id_base,
               queries.handle if queries is not None else None, int(nq), int(k), int(ef), SEARCH_MODES[mode],
               gid.handle, lid.handle if lid is not None else None, dist.handle)


class DualSpaceIndex:
    """DualSpaceIndex (crates/ruvector-hyperbolic-hnsw/src/hnsw.rs:536-605): a Poincaré
    HyperbolicHnsw (primary) and a Euclidean-metric twin over the same inserted vectors,
    searched for 2k each and fused by reciprocal rank: score(id) = w / (rank_h + 1) +
    (1 - w) / (rank_e + 1) in f32, highest first, then the top k re-scored with the
    Poincaré distance of the raw query to the stored vector. Ties in the fused score
    are ordered by first appearance (hyperbolic ranks, then Euclidean-only ids); the
    reference leaves them in HashMap order."""

    def __init__(self, curvature: float, fusion_weight: float, seed: int = 0):
        self.hyperbolic = HyperbolicHnsw(HyperbolicHnswConfig(curvature=curvature, seed=seed))
        self.euclidean = HyperbolicHnsw(HyperbolicHnswConfig(metric="euclidean", seed=seed))
        self.fusion_weight = float(np.float32(min(max(fusion_weight, 0.0), 1.0)))

    def insert(self, vector: Sequence[float]) -> int:
        self.euclidean.insert(vector)
        return self.hyperbolic.insert(vector)

    def insert_batch(self, vectors) -> List[int]:
        self.euclidean.insert_batch(vectors)
        return self.hyperbolic.insert_batch(vectors)

    def __len__(self) -> int:
        return len(self.hyperbolic)

    def search(self, query: Sequence[float], k: int) -> List[SearchResult]:
        q = np.asarray(query, np.float32).reshape(-1)
        hyp = self.hyperbolic.search(q, k * 2)
        euc = self.euclidean.search(q, k * 2)
        w = np.float32(self.fusion_weight)
        scores = {}
        for rank, r in enumerate(hyp):
            scores[r.id] = np.float32(scores.get(r.id, np.float32(0.0)) + w * (np.float32(1.0) / np.float32(rank + 1)))
        for rank, r in enumerate(euc):
            scores[r.id] = np.float32(scores.get(r.id, np.float32(0.0)) +
                                      (np.float32(1.0) - w) * (np.float32(1.0) / np.float32(rank + 1)))
        top = sorted(scores.items(), key=lambda t: -t[1])[:k]
        if not top:
            return []
        vecs = np.stack([self.hyperbolic.get_vector(i) for i, _ in top]).astype(np.float32)
        dist = np.empty((1, len(top)), np.float32)
        _check("rvx_distance_matrix", L.METRIC_POINCARE, L.fptr(q), 1, L.fptr(vecs), len(top), q.size,
               float(self.hyperbolic.config.curvature), L.fptr(dist))
        return [SearchResult(int(i), float(dd)) for (i, _), dd in zip(top, dist[0])]
