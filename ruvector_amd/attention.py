"""Graph-attention head: EdgeFeaturedAttention
(crates/ruvector-attention/src/graph/edge_featured.rs:11-320)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib as L
from .device import Buffer
from .graph import Graph


class AttentionError(L.RvxError):
    pass


def _check(name, *args):
    try:
        L.call(name, *args)
    except L.RvxError as e:
        raise AttentionError(e.code, str(e).split(": ", 1)[-1]) from None


@dataclass
class EdgeFeaturedConfig:
    """EdgeFeaturedConfig::default (edge_featured.rs:22-33)."""
    node_dim: int = 256
    edge_dim: int = 64
    num_heads: int = 4
    dropout: float = 0.0
    concat_heads: bool = True
    add_self_loops: bool = True
    negative_slope: float = 0.2

    def head_dim(self) -> int:
        return self.node_dim // self.num_heads


class EdgeFeaturedAttention:
    """EdgeFeaturedAttention::new (deterministic LCG init, seed 42, edge_featured.rs:98-141)."""

    def __init__(self, config: EdgeFeaturedConfig):
        self.config = config
        c = L.EdgeAttentionConfig(node_dim=config.node_dim, edge_dim=config.edge_dim, num_heads=config.num_heads,
                                  dropout=config.dropout, concat_heads=1 if config.concat_heads else 0,
                                  add_self_loops=1 if config.add_self_loops else 0,
                                  negative_slope=config.negative_slope)
        h = C.c_void_p()
        _check("rvx_edge_attention_create", C.byref(c), C.byref(h))
        self._h = h
        d = C.c_int32()
        L.call("rvx_edge_attention_dim", self._h, C.byref(d))
        self.out_dim = d.value

    def edge_dim(self) -> int:
        return self.config.edge_dim

    def num_heads(self) -> int:
        return self.config.num_heads

    def _run(self, query, keys, values, edges) -> np.ndarray:
        q = L.f32c(query).reshape(-1)
        if q.size != self.config.node_dim:
            raise AttentionError(1, f"DimensionMismatch expected {self.config.node_dim} actual {q.size}")
        n = len(keys)
        if len(values) != n:
            raise AttentionError(2, "keys and values must have the same length")
        k = L.f32c(keys).reshape(n, -1) if n else np.zeros((1, self.config.node_dim), np.float32)
        v = L.f32c(values).reshape(n, -1) if n else np.zeros((1, self.config.node_dim), np.float32)
        e = None
        if edges is not None:
            if len(edges) != n:
                raise AttentionError(2, "Keys and edges must have same length")
            e = L.f32c(edges).reshape(n, -1) if n and self.config.edge_dim else np.zeros((1, 1), np.float32)
        out = np.empty(max(self.out_dim, 1), np.float32)
        _check("rvx_edge_attention_compute", self._h, L.fptr(q), L.fptr(k), L.fptr(v),
               L.fptr(e) if e is not None else None, n, L.fptr(out))
        return out[:self.out_dim]

    def compute(self, query, keys: Sequence, values: Sequence) -> np.ndarray:
        """Attention::compute with zero edge features (edge_featured.rs:267-288)."""
        return self._run(query, keys, values, None)

    def compute_with_edges(self, query, keys: Sequence, values: Sequence, edges: Sequence) -> np.ndarray:
        """compute_with_edges (edge_featured.rs:196-258)."""
        return self._run(query, keys, values, edges)

    def forward_graph_device(self, x: Buffer, graph: Graph, edge_features: Optional[Buffer], y: Buffer) -> None:
        """Every node as query, its CSR neighbours as keys = values."""
        _check("rvx_edge_attention_forward_graph_device", self._h, graph.handle, x.handle,
               edge_features.handle if edge_features is not None else None, y.handle)

    def forward_exchange(self, local_graph: Graph, x_full: Buffer, edge_features: Optional[Buffer], y_full: Buffer,
                         offsets, comm=None) -> None:
        """Node-range-sharded forward_graph_device (rvx_edge_attention_forward_exchange):
        this rank's rows of y_full; the transformed rows travel to the peers over RCCL."""
        off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
        _check("rvx_edge_attention_forward_exchange", self._h, local_graph.handle, x_full.handle,
               edge_features.handle if edge_features is not None else None, y_full.handle,
               off.ctypes.data_as(C.POINTER(C.c_int64)), comm._h if comm is not None else None)

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_edge_attention_destroy", self._h)
                self._h = None
        except Exception:
            pass


@dataclass
class DualSpaceConfig:
    """DualSpaceConfig (crates/ruvector-attention/src/graph/dual_space.rs:30-50)."""
    dim: int = 256
    curvature: float = 1.0
    euclidean_weight: float = 0.5
    hyperbolic_weight: float = 0.5
    temperature: float = 1.0


class DualSpaceAttention:
    """DualSpaceAttention::new (dual_space.rs:107-131: LCG seed 42 weights)."""

    def __init__(self, config: DualSpaceConfig):
        self.config = config
        c = L.DualAttentionConfig(dim=config.dim, curvature=config.curvature,
                                  euclidean_weight=config.euclidean_weight,
                                  hyperbolic_weight=config.hyperbolic_weight, temperature=config.temperature)
        h = C.c_void_p()
        _check("rvx_dual_attention_create", C.byref(c), C.byref(h))
        self._h = h

    def dim(self) -> int:
        return self.config.dim

    def compute(self, query, keys: Sequence, values: Sequence) -> np.ndarray:
        """Attention::compute (dual_space.rs:207-268)."""
        q = L.f32c(query).reshape(-1)
        if q.size != self.config.dim:
            raise AttentionError(1, f"DimensionMismatch expected {self.config.dim} actual {q.size}")
        n = len(keys)
        if n == 0:
            raise AttentionError(2, "Empty keys")
        k = L.f32c(keys).reshape(n, -1)
        v = L.f32c(values).reshape(len(values), -1)
        vd = v.shape[1]
        out = np.empty(vd, np.float32)
        _check("rvx_dual_attention_compute", self._h, L.fptr(q), L.fptr(k), L.fptr(v), n, vd, L.fptr(out))
        return out

    def compute_with_mask(self, query, keys: Sequence, values: Sequence, mask=None) -> np.ndarray:
        """compute_with_mask (dual_space.rs:271-291): keep the masked-in keys/values."""
        if mask is None:
            return self.compute(query, keys, values)
        keep = [i for i, m in enumerate(mask) if m]
        return self.compute(query, [keys[i] for i in keep], [values[i] for i in keep])

    def forward_graph_device(self, x: Buffer, graph: Graph, y: Buffer) -> None:
        """Every node as query, its CSR neighbours as keys = values."""
        _check("rvx_dual_attention_forward_graph_device", self._h, graph.handle, x.handle, y.handle)

    def __del__(self):
        try:
            if self._h:
                L.call("rvx_dual_attention_destroy", self._h)
                self._h = None
        except Exception:
            pass
