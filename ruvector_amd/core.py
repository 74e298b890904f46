"""ruvector-core's index/query API over HBM.

DistanceMetric / HnswConfig / SearchResult   crates/ruvector-core/src/types.rs:10-126
distance / batch_distances                   crates/ruvector-core/src/distance.rs:9-107
VectorIndex (FlatIndex, HnswIndex)           crates/ruvector-core/src/index.rs:11-36,
                                             index/flat.rs, index/hnsw.rs

Vector ids are strings in the reference (VectorId = String); here the index
stores dense u64 keys and this module keeps the String <-> u64 map, as
HnswIndex's id_to_idx / idx_to_id DashMaps do (index/hnsw.rs:38-44).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from enum import Enum
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .device import Buffer


class RuvectorError(L.RvxError):
    pass


def _check(name, *args):
    try:
        L.call(name, *args)
    except L.RvxError as e:
        raise RuvectorError(e.code, str(e).split(": ", 1)[-1]) from None


class DistanceMetric(Enum):
    Euclidean = L.METRIC_L2
    Cosine = L.METRIC_COSINE
    DotProduct = L.METRIC_DOT
    Manhattan = L.METRIC_L1


@dataclass
class HnswConfig:
    """HnswConfig::default (types.rs:87-96)."""
    m: int = 32
    ef_construction: int = 200
    ef_search: int = 100
    max_elements: int = 10_000_000


@dataclass
class SearchResult:
    id: str
    score: float
    vector: Optional[List[float]] = None
    metadata: Optional[dict] = None


def distance_matrix(queries, vectors, metric: DistanceMetric = DistanceMetric.Euclidean) -> np.ndarray:
    q = L.f32c(queries)
    x = L.f32c(vectors)
    if q.ndim == 1:
        q = q[None]
    if x.ndim == 1:
        x = x[None]
    if q.shape[1] != x.shape[1]:
        raise RuvectorError(1, f"DimensionMismatch expected {q.shape[1]} actual {x.shape[1]}")
    out = np.empty((q.shape[0], x.shape[0]), np.float32)
    _check("rvx_distance_matrix", metric.value, L.fptr(q), q.shape[0], L.fptr(x), x.shape[0], q.shape[1], 1.0,
           L.fptr(out))
    return out


def distance(a, b, metric: DistanceMetric) -> float:
    """distance (distance.rs:9-23), errors on dimension mismatch."""
    a, b = L.f32c(a).reshape(-1), L.f32c(b).reshape(-1)
    if a.size != b.size:
        raise RuvectorError(1, f"DimensionMismatch expected {a.size} actual {b.size}")
    return float(distance_matrix(a[None], b[None], metric)[0, 0])


def batch_distances(query, vectors, metric: DistanceMetric) -> List[float]:
    """batch_distances (distance.rs:89-107)."""
    return [float(v) for v in distance_matrix(L.f32c(query)[None], vectors, metric)[0]]


class _Index:
    kind = L.INDEX_FLAT

    def __init__(self, dimensions: int, metric: DistanceMetric, config: Optional[HnswConfig] = None, seed: int = 0):
        cfg = config or HnswConfig()
        c = L.IndexConfig(kind=self.kind, dim=dimensions, metric=metric.value, m=cfg.m,
                          ef_construction=cfg.ef_construction, ef_search=cfg.ef_search,
                          max_elements=cfg.max_elements, curvature=1.0, seed=seed)
        h = C.c_void_p()
        _check("rvx_index_create", C.byref(c), C.byref(h))
        self._h = h
        self.dimensions, self.metric, self.config = dimensions, metric, cfg
        self._ids: Dict[str, int] = {}
        self._names: Dict[int, str] = {}
        self._next = 0

    @property
    def handle(self):
        return self._h

    def _key(self, vid: str) -> int:
        if vid in self._ids:
            raise RuvectorError(2, f"duplicate id {vid}")
        k = self._next
        self._next += 1
        self._ids[vid] = k
        self._names[k] = vid
        return k

    def add(self, vid: str, vector: Sequence[float]) -> None:
        self.add_batch([(vid, vector)])

    def add_batch(self, entries: Sequence[Tuple[str, Sequence[float]]]) -> None:
        if not entries:
            return
        vecs = [L.f32c(v).reshape(-1) for _, v in entries]
        for v in vecs:
            if v.size != self.dimensions:
                raise RuvectorError(1, f"DimensionMismatch expected {self.dimensions} actual {v.size}")
        keys = np.array([self._key(vid) for vid, _ in entries], dtype=np.uint64)
        self.add_array(np.stack(vecs), keys)

    def add_array(self, vectors: np.ndarray, keys: np.ndarray) -> None:
        """Bulk insert rows with explicit u64 keys (no String ids)."""
        v = L.f32c(vectors)
        k = np.ascontiguousarray(keys, dtype=np.uint64)
        for kk in k:
            self._names.setdefault(int(kk), str(int(kk)))
        self._next = max(self._next, int(k.max()) + 1 if len(k) else 0)
        _check("rvx_index_add_batch", self._h, L.fptr(v), L.u64ptr(k), len(k))

    def remove(self, vid: str) -> bool:
        key = self._ids.get(vid)
        if key is None:
            return False
        r = C.c_int32(0)
        _check("rvx_index_remove", self._h, key, C.byref(r))
        if r.value:
            del self._ids[vid]
        return bool(r.value)

    def __len__(self) -> int:
        n = C.c_int64(0)
        _check("rvx_index_len", self._h, C.byref(n))
        return n.value

    def len(self) -> int:
        return len(self)

    def is_empty(self) -> bool:
        return len(self) == 0

    def search_array(self, queries: np.ndarray, k: int, ef: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Batched search: (ids u64 [nq][k], distances [nq][k], counts [nq])."""
        q = L.f32c(queries)
        if q.ndim == 1:
            q = q[None]
        if q.shape[1] != self.dimensions:
            raise RuvectorError(1, f"DimensionMismatch expected {self.dimensions} actual {q.shape[1]}")
        nq = q.shape[0]
        ids = np.empty((nq, k), np.uint64)
        dist = np.empty((nq, k), np.float32)
        cnt = np.empty(nq, np.int32)
        _check("rvx_index_search", self._h, L.fptr(q), nq, int(k), int(ef), L.u64ptr(ids), L.fptr(dist),
               cnt.ctypes.data_as(L.PI32))
        return ids, dist, cnt

    # ---- HBM-resident forms (rvx_buffer in, rvx_buffer out; no host staging)
    def add_device(self, vectors, n: int, first_id: int = 0) -> None:
        """Insert n rows of a device buffer with ids first_id .. first_id+n-1 (GPU HNSW build)."""
        _check("rvx_index_add_batch_device", self._h, vectors.handle, int(n), int(first_id))
        self._next = max(self._next, int(first_id) + int(n))

    def search_device(self, q, nq: int, k: int, ef: int, ids, dist) -> None:
        """ids [nq][k] u64 (all-ones = empty slot), dist [nq][k] f32, written in HBM."""
        _check("rvx_index_search_device", self._h, q.handle, int(nq), int(k), int(ef), ids.handle, dist.handle)

    def brute_force_device(self, q, nq: int, k: int, ids, dist) -> None:
        """Exact scan (ties by id) into device buffers."""
        _check("rvx_index_brute_force_device", self._h, q.handle, int(nq), int(k), ids.handle, dist.handle)

    def sharded_search_array(self, comm, queries, k: int, ef: int = 0, exact: bool = False):
        """Node-range-sharded search across processes (rvx_index_sharded_search): this
        index is one rank's shard of `comm` (None = one process); rank 0's queries are
        broadcast (other ranks may pass nq), per-rank top-k all-gathered and merged by
        distance on the GPU. Returns (ids u64, distances, counts), same on every rank."""
        if isinstance(queries, (int, np.integer)):
            nq, q = int(queries), None
        else:
            q = L.f32c(queries).reshape(-1, self.dimensions)
            nq = q.shape[0]
        ids = np.empty((nq, k), np.uint64)
        d = np.empty((nq, k), np.float32)
        cnt = np.empty(nq, np.int32)
        _check("rvx_index_sharded_search", self._h, comm._h if comm is not None else None,
               L.fptr(q) if q is not None else None, nq, int(k), int(ef), int(bool(exact)), L.u64ptr(ids),
               L.fptr(d), L.i32ptr(cnt))
        return ids, d, cnt

    def brute_force_array(self, queries: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        q = L.f32c(queries)
        if q.ndim == 1:
            q = q[None]
        nq = q.shape[0]
        ids = np.empty((nq, k), np.uint64)
        dist = np.empty((nq, k), np.float32)
        _check("rvx_index_brute_force", self._h, L.fptr(q), nq, int(k), L.u64ptr(ids), L.fptr(dist))
        return ids, dist

    def search(self, query: Sequence[float], k: int) -> List[SearchResult]:
        """VectorIndex::search (index.rs:25)."""
        ids, dist, cnt = self.search_array(L.f32c(query).reshape(1, -1), k)
        out = []
        for s in range(int(cnt[0]) if self.kind == L.INDEX_HNSW else k):
            if ids[0, s] == np.uint64(0xFFFFFFFFFFFFFFFF):
                break
            name = self._names.get(int(ids[0, s]), str(int(ids[0, s])))
            out.append(SearchResult(id=name, score=float(dist[0, s])))
        return out

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_index_destroy", self._h)
                self._h = None
        except Exception:
            pass


def hnsw_last_search_stats() -> dict:
    """Work of the most recent HNSW search launch: distance evaluations, layer-0 expansions, queries."""
    a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
    _check("rvx_hnsw_last_search_stats", C.byref(a), C.byref(b), C.byref(c))
    v, sl = C.c_int32(), C.c_int32()
    _check("rvx_hnsw_last_search_visited", C.byref(v), C.byref(sl))
    rg, st, ov = C.c_int32(), C.c_int32(), C.c_int32()
    _check("rvx_hnsw_last_search_form", C.byref(rg), C.byref(st), C.byref(ov))
    return {"n_dist": a.value, "n_expand": b.value, "nq": c.value, "visited_bitmap": bool(v.value),
            "slots": sl.value, "r_in_hbm": bool(rg.value), "stages": st.value, "visited_overflow": bool(ov.value)}


def scan_last_stats() -> dict:
    """Path of the most recent exact scan: MFMA-filtered queries, exact-VALU queries, filter fallbacks."""
    a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
    _check("rvx_scan_last_stats", C.byref(a), C.byref(b), C.byref(c))
    s2 = C.c_int64()
    _check("rvx_scan_last_second_pass", C.byref(s2))
    bd = C.c_int64()
    _check("rvx_scan_last_band", C.byref(bd))
    return {"mfma": a.value, "valu": b.value, "fallback": c.value, "second_pass": s2.value, "band": bd.value}


class FlatIndex(_Index):
    """FlatIndex (index/flat.rs): exact scan, results sorted by distance."""
    kind = L.INDEX_FLAT


class HnswIndex(_Index):
    """HnswIndex (index/hnsw.rs) searching a loaded HNSW graph on the GPU."""
    kind = L.INDEX_HNSW

    def search_with_ef(self, query, k: int, ef_search: int) -> List[SearchResult]:
        ids, dist, cnt = self.search_array(L.f32c(query).reshape(1, -1), k, ef_search)
        return [SearchResult(id=self._names.get(int(ids[0, s]), str(int(ids[0, s]))), score=float(dist[0, s]))
                for s in range(int(cnt[0]))]

    def load_graph(self, graph: dict) -> None:
        """Install a fixed HNSW graph (rvx_hnsw_graph layout; see oracle export)."""
        load_graph_handle(self._h, graph)

    def export_graph(self) -> dict:
        """The searchable graph in the rvx_hnsw_graph layout (same dict as load_graph takes)."""
        return export_graph_handle(self._h)

    # ---- persistence
    def export_rows(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """All stored rows in insertion order: (vectors [n][d], u64 keys, tombstones)."""
        total = C.c_int64(0)
        _check("rvx_index_export_rows", self._h, 0, 0, None, None, None, C.byref(total))
        n = total.value
        vecs = np.empty((max(n, 1), self.dimensions), np.float32)
        keys = np.empty(max(n, 1), np.uint64)
        dead = np.empty(max(n, 1), np.uint8)
        _check("rvx_index_export_rows", self._h, 0, n, L.fptr(vecs), L.u64ptr(keys),
               dead.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(total))
        return vecs[:n], keys[:n], dead[:n]

    def serialize(self) -> bytes:
        """HnswIndex::serialize (index/hnsw.rs:136-169): bincode HnswState of the live vectors."""
        from .formats import HnswState, METRIC_VARIANTS
        vecs, keys, dead = self.export_rows()
        st = HnswState(next_idx=self._next, m=self.config.m, ef_construction=self.config.ef_construction,
                       ef_search=self.config.ef_search, max_elements=self.config.max_elements,
                       dimensions=self.dimensions, metric=METRIC_VARIANTS[self.metric.value])
        for v, k, d in zip(vecs, keys, dead):
            if d:
                continue
            name = self._names.get(int(k), str(int(k)))
            st.vectors.append((name, v))
            st.id_to_idx.append((name, int(k)))
            st.idx_to_id.append((int(k), name))
        return st.encode()

    @classmethod
    def deserialize(cls, data: bytes, seed: int = 0) -> "HnswIndex":
        """HnswIndex::deserialize (index/hnsw.rs:171-226): rebuild by inserting every vector
        (here in ascending idx order, on the GPU builder)."""
        from .formats import HnswState, METRIC_VARIANTS
        st = HnswState.decode(data)
        cfg = HnswConfig(m=st.m, ef_construction=st.ef_construction, ef_search=st.ef_search,
                         max_elements=st.max_elements)
        ix = cls(st.dimensions, DistanceMetric(METRIC_VARIANTS.index(st.metric)), cfg, seed=seed)
        by_name = {vid: vec for vid, vec in st.vectors}
        order = sorted((idx, vid) for idx, vid in st.idx_to_id if vid in by_name)
        if order:
            keys = np.array([idx for idx, _ in order], np.uint64)
            ix.add_array(np.stack([by_name[vid] for _, vid in order]), keys)
            for idx, vid in order:
                ix._ids[vid] = idx
                ix._names[idx] = vid
        ix._next = max(ix._next, st.next_idx)
        return ix

    def file_dump(self, directory: str, basename: str) -> None:
        """Hnsw::file_dump (patches/hnsw_rs/src/hnswio.rs): `<basename>.hnsw.graph` + `.hnsw.data`."""
        _check("rvx_index_file_dump", self._h, directory.encode(), basename.encode())

    @classmethod
    def file_load(cls, directory: str, basename: str, metric: Optional[DistanceMetric] = None,
                  ef_search: int = 100) -> "HnswIndex":
        """HnswIo::load_hnsw: the dumped graph and vectors become the GPU-searchable index."""
        h = C.c_void_p()
        _check("rvx_index_file_load", directory.encode(), basename.encode(), -1 if metric is None else metric.value,
               int(ef_search), 0, C.byref(h))
        from .formats import describe_dump
        ds = describe_dump(directory, basename)
        ix = cls.__new__(cls)
        ix._h = h
        ix.dimensions = ds["dimension"]
        cfg_metric = metric
        if cfg_metric is None:
            name = ds["distname"]
            cfg_metric = next(m for m, suf in ((DistanceMetric.Euclidean, "DistL2"), (DistanceMetric.Cosine, "DistCosine"),
                                                (DistanceMetric.DotProduct, "DistDot"),
                                                (DistanceMetric.Manhattan, "DistL1")) if name.endswith(suf))
        ix.metric = cfg_metric
        ix.config = HnswConfig(m=ds["max_nb_connection"], ef_construction=ds["ef"], ef_search=ef_search,
                               max_elements=max(ds["nb_point"], 1))
        _, keys, _ = ix.export_rows()
        ix._ids, ix._names = {}, {int(k): str(int(k)) for k in keys}
        ix._next = int(keys.max()) + 1 if len(keys) else 0
        return ix

    def layer0(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Layer-0 adjacency (row_ptr, col, edge distance) for the GNN."""
        n, e = C.c_int64(), C.c_int64()
        _check("rvx_index_layer0_size", self._h, C.byref(n), C.byref(e))
        rp = np.empty(n.value + 1, np.int64)
        col = np.empty(max(e.value, 1), np.int32)
        dist = np.empty(max(e.value, 1), np.float32)
        _check("rvx_index_export_layer0", self._h, L.i64ptr(rp), L.i32ptr(col), L.fptr(dist))
        return rp, col[:e.value], dist[:e.value]


def load_graph_handle(handle, graph: dict) -> None:
    """Install a fixed HNSW graph (rvx_hnsw_graph layout; see oracle export) on an rvx_index handle."""
    n = int(graph["n"])
    max_level = int(graph["max_level"])
    levels = np.ascontiguousarray(graph["levels"], dtype=np.uint8)
    rp0 = np.ascontiguousarray(graph["row_ptr0"], dtype=np.int64)
    col0 = np.ascontiguousarray(graph["col0"], dtype=np.int32)
    ucount = np.zeros(17, np.int64)
    ids_l, rp_l, col_l = [], [], []
    for l in range(1, max_level + 1):
        ids_l.append(np.ascontiguousarray(graph["upper_ids"][l - 1], dtype=np.int32))
        rp_l.append(np.ascontiguousarray(graph["upper_row_ptr"][l - 1], dtype=np.int64))
        col_l.append(np.ascontiguousarray(graph["upper_col"][l - 1], dtype=np.int32))
        ucount[l] = len(ids_l[-1])
    dummy32 = np.zeros(1, np.int32)
    dummy64 = np.zeros(1, np.int64)
    P32 = C.POINTER(C.c_int32)
    P64 = C.POINTER(C.c_int64)
    ids_arr = (P32 * 17)(*([dummy32.ctypes.data_as(P32)] + [a.ctypes.data_as(P32) for a in ids_l] +
                           [dummy32.ctypes.data_as(P32)] * (16 - max_level)))
    rp_arr = (P64 * 17)(*([dummy64.ctypes.data_as(P64)] + [a.ctypes.data_as(P64) for a in rp_l] +
                          [dummy64.ctypes.data_as(P64)] * (16 - max_level)))
    col_arr = (P32 * 17)(*([dummy32.ctypes.data_as(P32)] + [a.ctypes.data_as(P32) for a in col_l] +
                           [dummy32.ctypes.data_as(P32)] * (16 - max_level)))
    g = L.HnswGraph(n=n, max_level=max_level, entry_point=int(graph["entry"]),
                    levels=levels.ctypes.data_as(C.POINTER(C.c_uint8)), row_ptr0=L.i64ptr(rp0),
                    col0=L.i32ptr(col0), upper_count=L.i64ptr(ucount),
                    upper_ids=C.cast(ids_arr, C.POINTER(P32)), upper_row_ptr=C.cast(rp_arr, C.POINTER(P64)),
                    upper_col=C.cast(col_arr, C.POINTER(P32)))
    _check("rvx_index_load_graph", handle, C.byref(g))

def export_graph_handle(handle) -> dict:
    """The searchable graph of an rvx_index handle in the rvx_hnsw_graph layout."""
    n, ml, ent, e0 = C.c_int64(), C.c_int32(), C.c_int64(), C.c_int64()
    uc = np.zeros(17, np.int64)
    ue = np.zeros(17, np.int64)
    _check("rvx_index_graph_sizes", handle, C.byref(n), C.byref(ml), C.byref(ent), C.byref(e0), L.i64ptr(uc),
           L.i64ptr(ue))
    N, Lm = n.value, ml.value
    levels = np.empty(max(N, 1), np.uint8)
    rp0 = np.empty(N + 1, np.int64)
    col0 = np.empty(max(e0.value, 1), np.int32)
    ids = np.empty(max(int(uc.sum()), 1), np.int32)
    rps = np.empty(max(int((uc[1:Lm + 1] + 1).sum()), 1), np.int64)
    cols = np.empty(max(int(ue.sum()), 1), np.int32)
    _check("rvx_index_export_graph", handle, levels.ctypes.data_as(C.POINTER(C.c_uint8)), L.i64ptr(rp0),
           L.i32ptr(col0), L.i32ptr(ids), L.i64ptr(rps), L.i32ptr(cols))
    g = {"n": N, "max_level": Lm, "entry": ent.value, "levels": levels[:N], "row_ptr0": rp0,
         "col0": col0[:e0.value], "upper_ids": [], "upper_row_ptr": [], "upper_col": []}
    oi = orp = oc = 0
    for l in range(1, Lm + 1):
        c = int(uc[l])
        g["upper_ids"].append(ids[oi:oi + c].copy())
        rp = rps[orp:orp + c + 1].copy()
        g["upper_row_ptr"].append(rp)
        g["upper_col"].append(cols[oc:oc + int(rp[-1])].copy())
        oi, orp, oc = oi + c, orp + c + 1, oc + int(rp[-1])
    return g
