"""GNN layers on HNSW topology — the ruvector-gnn / ruvector-postgres gnn API.

RuvectorLayer       crates/ruvector-gnn/src/layer.rs:313-457
differentiable_search / hierarchical_forward   crates/ruvector-gnn/src/search.rs:56-162
GraphSAGELayer      crates/ruvector-postgres/src/gnn/graphsage.rs:25-196
GCNLayer            crates/ruvector-postgres/src/gnn/gcn.rs:12-149
aggregate           crates/ruvector-postgres/src/gnn/aggregators.rs:35-101

Per-node calls keep the reference signatures; the *_graph methods run every
node of a CSR graph in one batched pass of HIP kernels (the drop-in hot path).
"""
from __future__ import annotations

import ctypes as C
import json
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .device import Buffer
from .graph import Graph


class GnnError(L.RvxError):
    pass


def _check(name, *args):
    try:
        L.call(name, *args)
    except L.RvxError as e:
        raise GnnError(e.code, str(e).split(": ", 1)[-1]) from None


class RuvectorLayer:
    """RuvectorLayer::new(input_dim, hidden_dim, heads, dropout) (layer.rs:347-368).

    Weights come from a seeded stream (`seed`); the reference draws them from
    thread_rng, so use from_json() to run a reference layer's exact weights.
    """

    def __init__(self, input_dim: int, hidden_dim: int, heads: int, dropout: float, seed: int = 0, _handle=None):
        if _handle is None:
            h = C.c_void_p()
            _check("rvx_gnn_layer_create", int(input_dim), int(hidden_dim), int(heads), float(dropout), int(seed),
                   C.byref(h))
            _handle = h
        self._h = _handle
        a, b, c, d = C.c_int32(), C.c_int32(), C.c_int32(), C.c_float()
        L.call("rvx_gnn_layer_dims", self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d))
        self.input_dim, self.hidden_dim, self.heads, self.dropout = a.value, b.value, c.value, d.value

    @classmethod
    def from_json(cls, text: str) -> "RuvectorLayer":
        h = C.c_void_p()
        _check("rvx_gnn_layer_from_json", text.encode(), C.byref(h))
        return cls(0, 0, 0, 0.0, _handle=h)

    def to_json(self) -> str:
        n = C.c_size_t(0)
        L.call("rvx_gnn_layer_to_json", self._h, None, C.byref(n))
        buf = C.create_string_buffer(n.value)
        L.call("rvx_gnn_layer_to_json", self._h, buf, C.byref(n))
        return buf.value.decode()

    def forward(self, node_embedding: Sequence[float], neighbor_embeddings: Sequence[Sequence[float]],
                edge_weights: Sequence[float]) -> np.ndarray:
        """RuvectorLayer::forward (layer.rs:379-418) for one node."""
        node = L.f32c(node_embedding).reshape(-1)
        nb = [L.f32c(n).reshape(-1) for n in neighbor_embeddings]
        deg = len(nb)
        for v in [node] + nb:
            if v.size != self.input_dim:
                raise GnnError(1, f"expected input_dim {self.input_dim}, got {v.size}")
        nbrs = np.ascontiguousarray(np.stack(nb)) if deg else np.zeros((1, self.input_dim), np.float32)
        w = L.f32c(edge_weights).reshape(-1) if len(edge_weights) else np.zeros(1, np.float32)
        out = np.empty(self.hidden_dim, np.float32)
        _check("rvx_gnn_forward_one", self._h, L.fptr(node), L.fptr(nbrs), deg, L.fptr(w), len(edge_weights),
               L.fptr(out))
        return out

    def forward_graph(self, x: np.ndarray, graph: Graph) -> np.ndarray:
        """Every node of `graph` through forward(x_i, x[adj(i)], w[adj(i)])."""
        x = L.f32c(x)
        y = np.empty((graph.num_nodes, self.hidden_dim), np.float32)
        _check("rvx_gnn_forward_graph", self._h, graph.handle, L.fptr(x), graph.num_nodes, L.fptr(y))
        return y

    def forward_graph_device(self, x: Buffer, graph: Graph, y: Buffer) -> None:
        _check("rvx_gnn_forward_graph_device", self._h, graph.handle, x.handle, y.handle)

    def forward_exchange(self, local_graph: Graph, x_full: Buffer, y_full: Buffer, offsets, comm=None) -> None:
        """Node-range-sharded forward (rvx_gnn_forward_exchange): this rank's rows of
        y_full from its rows of x_full; M|K|V rows travel to the peers over RCCL."""
        off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
        _check("rvx_gnn_forward_exchange", self._h, local_graph.handle, x_full.handle, y_full.handle,
               off.ctypes.data_as(C.POINTER(C.c_int64)), comm._h if comm is not None else None)

    def forward_star_device(self, nodes: Buffer, nq: int, table: Buffer, table_rows: int, cand_ids: Buffer, c: int,
                            weights: Optional[Buffer], out: Buffer) -> None:
        """forward(nodes[i], table[cand_ids[i]], weights[i]) for i < nq, all resident in HBM
        (ids outside [0, table_rows) are absent neighbours; weights None -> no edge weights)."""
        _check("rvx_gnn_forward_star_device", self._h, nodes.handle, int(nq), table.handle, int(table_rows),
               cand_ids.handle, int(c), weights.handle if weights is not None else None, out.handle)

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_gnn_layer_destroy", self._h)
                self._h = None
        except Exception:
            pass


class GraphSAGELayer:
    """GraphSAGELayer::with_aggregator (graphsage.rs:49-89); aggregator 'mean'|'maxpool'|'lstm'."""

    _AGG = {"mean": L.SAGE_MEAN, "maxpool": L.SAGE_MAXPOOL, "lstm": L.SAGE_LSTM}

    def __init__(self, in_features: int, out_features: int, num_samples: int, aggregator: str = "mean",
                 normalize: bool = True, neighbor_weights=None, self_weights=None):
        self.in_features, self.out_features, self.num_samples = in_features, out_features, num_samples
        self.aggregator, self.normalize = aggregator, normalize
        wn = None if neighbor_weights is None else L.f32c(neighbor_weights).reshape(in_features, out_features)
        ws = None if self_weights is None else L.f32c(self_weights).reshape(in_features, out_features)
        h = C.c_void_p()
        _check("rvx_sage_layer_create", in_features, out_features, num_samples, self._AGG[aggregator],
               1 if normalize else 0, L.fptr(wn) if wn is not None else None,
               L.fptr(ws) if ws is not None else None, C.byref(h))
        self._h = h

    def sample_neighbors(self, neighbors: Sequence[int], k: int) -> list:
        """GraphSAGELayer::sample_neighbors (graphsage.rs:92-102): the list itself when
        len <= k, else the prefix [..k] left by StdRng::seed_from_u64(42) partial_shuffle."""
        nb = list(neighbors)
        if len(nb) <= k:
            return nb
        pos = np.empty(k, np.int32)
        _check("rvx_sage_sample_positions", len(nb), k, pos.ctypes.data_as(L.PI32))
        return [nb[p] for p in pos]

    def forward(self, node_features, edge_index: Sequence[Tuple[int, int]]) -> np.ndarray:
        """GraphSAGELayer::forward(node_features, edge_index) (graphsage.rs:190-196)."""
        x = L.f32c(node_features)
        g = Graph.from_edges(len(x), edge_index)
        return self.forward_graph(x, g)

    def forward_graph(self, x: np.ndarray, graph: Graph) -> np.ndarray:
        x = L.f32c(x)
        y = np.empty((graph.num_nodes, self.out_features), np.float32)
        _check("rvx_sage_forward", self._h, graph.handle, L.fptr(x), graph.num_nodes, L.fptr(y))
        return y

    def forward_device(self, x: Buffer, graph: Graph, y: Buffer) -> None:
        _check("rvx_sage_forward_device", self._h, graph.handle, x.handle, y.handle)

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_sage_layer_destroy", self._h)
                self._h = None
        except Exception:
            pass


def row_image_bytes(n: int, dim: int) -> int:
    """Size of a ReLU-sparse row image of an n x dim table (rvx_row_image_bytes; rvx.h)."""
    b = C.c_int64()
    _check("rvx_row_image_bytes", int(n), int(dim), C.byref(b))
    return b.value


_IMG_SLOT = 3072  # bytes per row slot of a row image (kernels.hpp IMG_SLOT)


def row_image(n: int, dim: int) -> Buffer:
    """A row-image buffer for n rows of dim (see rvx_sage_forward_exchange3). Every row's
    count starts at 0xFFFF (> IMG_CAP: "no slot, read the dense row"), so a row that is
    never packed falls back to the dense table instead of decoding an unwritten slot."""
    b = Buffer(row_image_bytes(n, dim))
    if n > 0:
        b.upload(np.full(int(n), 0xFFFF, np.uint16), offset=int(n) * _IMG_SLOT)
    return b


def pack_row_image(x: Buffer, n_total: int, dim: int, image: Buffer, r0: int = 0, rows: Optional[int] = None) -> None:
    """Rows [r0, r0 + rows) of the n_total x dim table x into the image (rvx_row_image_pack)."""
    rows = n_total - r0 if rows is None else rows
    _check("rvx_row_image_pack", x.handle, int(n_total), int(r0), int(rows), int(dim), image.handle)


class GCNLayer:
    """GCNLayer::new_with_normalize (gcn.rs:24-53)."""

    def __init__(self, in_features: int, out_features: int, normalize: bool = True, weights=None, bias=None):
        self.in_features, self.out_features = in_features, out_features
        w = None if weights is None else L.f32c(weights).reshape(in_features, out_features)
        b = None if bias is None else L.f32c(bias).reshape(out_features)
        h = C.c_void_p()
        _check("rvx_gcn_layer_create", in_features, out_features, 1 if normalize else 0,
               L.fptr(w) if w is not None else None, L.fptr(b) if b is not None else None, C.byref(h))
        self._h = h

    def forward(self, node_features, edge_index, edge_weights: Optional[Sequence[float]] = None) -> np.ndarray:
        """GCNLayer::forward (gcn.rs:93-112)."""
        x = L.f32c(node_features)
        g = Graph.from_edges(len(x), edge_index, edge_weights)
        y = np.empty((g.num_nodes, self.out_features), np.float32)
        _check("rvx_gcn_forward", self._h, g.handle, 1 if edge_weights is not None else 0, L.fptr(x), g.num_nodes,
               L.fptr(y))
        return y

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_gcn_layer_destroy", self._h)
                self._h = None
        except Exception:
            pass


def aggregate(x: Buffer, graph: Graph, dim: int, method: str, out: Buffer, weighted: bool = False,
              keep_isolated: bool = False) -> None:
    """sum/mean/max aggregation over CSR rows (aggregators.rs:35-101), on device buffers."""
    m = {"sum": L.AGG_SUM, "mean": L.AGG_MEAN, "avg": L.AGG_MEAN, "max": L.AGG_MAX}[method.lower()]
    L.call("rvx_aggregate_device", graph.handle, m, 1 if weighted else 0, 1 if keep_isolated else 0, x.handle,
           int(dim), out.handle)


def differentiable_search_batch(queries: np.ndarray, candidates: np.ndarray, k: int,
                                temperature: float) -> Tuple[np.ndarray, np.ndarray]:
    """differentiable_search for nq queries at once: queries [nq][d], candidates [nq][c][d].
    Returns (indices [nq][min(k,c)], weights); see search.rs:56-94."""
    q = L.f32c(queries)
    cand = L.f32c(candidates)
    nq, c, d = cand.shape
    kk = min(k, c)
    idx = np.empty((nq, k), np.int64)
    w = np.empty((nq, k), np.float32)
    if nq and k:
        _check("rvx_differentiable_search_batch", L.fptr(q), nq, L.fptr(cand), c, d, k, float(temperature),
               L.i64ptr(idx), L.fptr(w))
    return idx[:, :kk], w[:, :kk]


def differentiable_search_device(q: Buffer, nq: int, table: Buffer, table_rows: int, cand_ids: Buffer, c: int,
                                 d: int, k: int, temperature: float, idx: Optional[Buffer] = None,
                                 w: Optional[Buffer] = None, soft: Optional[Buffer] = None) -> None:
    """differentiable_search (search.rs:56-94) for nq queries whose candidates are table rows
    cand_ids[i] (all valid): idx [nq][k] int64 positions in the candidate list, w [nq][k],
    soft (optional) [nq][c] the softmax weights in candidate order."""
    _check("rvx_differentiable_search_device", q.handle, int(nq), table.handle, int(table_rows), cand_ids.handle,
           int(c), int(d), int(k), float(temperature), idx.handle if idx is not None else None,
           w.handle if w is not None else None, soft.handle if soft is not None else None)


def differentiable_search(query, candidate_embeddings, k: int, temperature: float) -> Tuple[List[int], List[float]]:
    """differentiable_search (search.rs:56-94)."""
    if len(candidate_embeddings) == 0:
        return [], []
    cand = L.f32c(candidate_embeddings)[None]
    idx, w = differentiable_search_batch(L.f32c(query)[None], cand, k, temperature)
    return [int(i) for i in idx[0]], [float(x) for x in w[0]]


def hierarchical_forward_device(q: Buffer, nq: int, dim: int, levels: Sequence[Tuple[Buffer, int]],
                                gnn_layers: Sequence[RuvectorLayer], out: Buffer) -> int:
    """hierarchical_forward (search.rs:105-162) for nq queries resident in HBM:
    levels[s] = (buffer, rows) of level s's embeddings. Returns the output dim."""
    nl, nv = len(gnn_layers), len(levels)
    lay = (C.c_void_p * max(nl, 1))(*[l._h.value if isinstance(l._h, C.c_void_p) else l._h for l in gnn_layers])
    lev = (C.c_void_p * max(nv, 1))(*[b.handle.value if isinstance(b.handle, C.c_void_p) else b.handle
                                      for b, _ in levels])
    rows = np.ascontiguousarray([int(r) for _, r in levels] or [0], dtype=np.int64)
    od = C.c_int32(0)
    _check("rvx_hierarchical_forward_device", lay, nl, lev, L.i64ptr(rows), nv, q.handle, int(nq), int(dim),
           out.handle, C.byref(od))
    return od.value


def hierarchical_forward_batch(queries: np.ndarray, layer_embeddings: Sequence[np.ndarray],
                               gnn_layers: Sequence[RuvectorLayer]) -> np.ndarray:
    """hierarchical_forward for a batch of queries [nq][d] over shared layer embeddings
    (one device pass per level; see rvx_hierarchical_forward_device)."""
    q = L.f32c(queries)
    if q.ndim == 1:
        q = q[None]
    nq, d = q.shape
    levels, keep, dd = [], [], d
    for s, emb in enumerate(layer_embeddings[:len(gnn_layers)]):
        e = L.f32c(emb).reshape(len(emb), -1) if len(emb) else np.zeros((0, dd), np.float32)
        if len(e) and e.shape[1] != dd:
            raise GnnError(1, f"level {s} embeddings have dim {e.shape[1]}, expected {dd}")
        b = Buffer.from_numpy(e)
        keep.append(b)
        levels.append((b, len(e)))
        if len(e):
            dd = gnn_layers[s].hidden_dim
    out_dim = max([d] + [l.hidden_dim for l in gnn_layers])
    qb, ob = Buffer.from_numpy(q), Buffer(max(nq * out_dim * 4, 4))
    od = hierarchical_forward_device(qb, nq, d, levels, gnn_layers, ob)
    return ob.download(np.float32, (nq, od))


def hierarchical_forward(query, layer_embeddings: Sequence[Sequence[Sequence[float]]],
                         gnn_layers: Sequence[RuvectorLayer]) -> np.ndarray:
    """hierarchical_forward (search.rs:105-162) for one query (the reference signature)."""
    cur = L.f32c(query).reshape(-1)
    if len(layer_embeddings) == 0 or len(gnn_layers) == 0:
        return cur
    return hierarchical_forward_batch(cur[None], layer_embeddings, gnn_layers)[0]
