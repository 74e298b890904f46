"""CSR graph handle (destination-major, neighbours in edge order).

Mirrors build_adjacency_list (crates/ruvector-postgres/src/gnn/message_passing.rs:34-50):
row i lists the sources j of the edges (j -> i) in edge order; edges with an
out-of-range endpoint are dropped.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .device import Buffer


class Graph:
    def __init__(self, handle, keep=()):
        self._h = handle
        self._keep = keep  # device buffers a device-built graph references
        n, e, md = C.c_int64(0), C.c_int64(0), C.c_int32(0)
        L.call("rvx_graph_info", self._h, C.byref(n), C.byref(e), C.byref(md))
        self.num_nodes, self.num_edges, self.max_degree = n.value, e.value, md.value

    @property
    def handle(self):
        return self._h

    @classmethod
    def from_edges(cls, num_nodes: int, edge_index: Sequence[Tuple[int, int]],
                   edge_weights: Optional[Sequence[float]] = None) -> "Graph":
        ei = np.asarray(edge_index, dtype=np.int64).reshape(-1, 2)
        src, dst = np.ascontiguousarray(ei[:, 0]), np.ascontiguousarray(ei[:, 1])
        w = None if edge_weights is None else L.f32c(edge_weights)
        if w is not None and len(w) < len(src):  # propagate_weighted: missing weights are 1.0
            w = np.concatenate([w, np.ones(len(src) - len(w), np.float32)])
        h = C.c_void_p()
        L.call("rvx_graph_from_edges", int(num_nodes), L.i64ptr(src), L.i64ptr(dst), len(src),
               L.fptr(w) if w is not None else None, C.byref(h))
        return cls(h)

    @classmethod
    def from_csr(cls, row_ptr, col, edge_weights=None) -> "Graph":
        rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
        cl = np.ascontiguousarray(col, dtype=np.int32)
        w = None if edge_weights is None else L.f32c(edge_weights)
        h = C.c_void_p()
        L.call("rvx_graph_from_csr", len(rp) - 1, L.i64ptr(rp), L.i32ptr(cl), L.fptr(w) if w is not None else None,
               C.byref(h))
        return cls(h)

    @classmethod
    def shard_from_csr(cls, row_ptr, col, num_nodes_total: int, edge_weights=None) -> "Graph":
        """A node-range shard: CSR rows of this rank's destination nodes whose column
        ids are GLOBAL node ids in [0, num_nodes_total) (the *_forward_exchange layout)."""
        rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
        cl = np.ascontiguousarray(col, dtype=np.int32)
        if cl.size and (int(cl.min()) < 0 or int(cl.max()) >= num_nodes_total):
            raise L.RvxError(3, "column index out of range")
        rpb, clb = Buffer.from_numpy(rp), Buffer.from_numpy(cl if cl.size else np.zeros(1, np.int32))
        wb = None if edge_weights is None else Buffer.from_numpy(L.f32c(edge_weights))
        h = C.c_void_p()
        L.call("rvx_graph_from_device_csr", len(rp) - 1, int(rp[-1]), rpb.handle, clb.handle,
               wb.handle if wb is not None else None, C.byref(h))
        return cls(h, keep=(rpb, clb) if wb is None else (rpb, clb, wb))

    @classmethod
    def random(cls, num_nodes: int, degree: int, seed: int, weight_seed: Optional[int] = None) -> "Graph":
        """Uniform random out-degree CSR generated on the device;
        with weight_seed, edge weights uniform [0, 1) from the same generator."""
        rp = Buffer((num_nodes + 1) * 8)
        col = Buffer(max(num_nodes * degree * 4, 4))
        L.call("rvx_random_csr", int(num_nodes), int(degree), int(seed), rp.handle, col.handle)
        w = None
        if weight_seed is not None:
            w = Buffer(max(num_nodes * degree * 4, 4))
            w.fill_uniform(num_nodes * degree, weight_seed, 0.0, 1.0)
        h = C.c_void_p()
        L.call("rvx_graph_from_device_csr", int(num_nodes), int(num_nodes * degree), rp.handle, col.handle,
               w.handle if w is not None else None, C.byref(h))
        return cls(h, keep=(rp, col) if w is None else (rp, col, w))

    @classmethod
    def random_shard(cls, num_nodes_total: int, row_begin: int, num_rows: int, degree: int, seed: int,
                     weight_seed: Optional[int] = None) -> "Graph":
        """Rows [row_begin, row_begin+num_rows) of Graph.random(num_nodes_total, ...), global column ids
        (with weight_seed, the same rows' slice of the global edge-weight stream)."""
        rp = Buffer((num_rows + 1) * 8)
        col = Buffer(max(num_rows * degree * 4, 4))
        L.call("rvx_random_csr_shard", int(num_nodes_total), int(row_begin), int(num_rows), int(degree), int(seed),
               rp.handle, col.handle)
        w = None
        if weight_seed is not None:
            w = Buffer(max(num_rows * degree * 4, 4))
            w.fill_uniform_at(num_rows * degree, weight_seed, row_begin * degree, 0.0, 1.0)
        h = C.c_void_p()
        L.call("rvx_graph_from_device_csr", int(num_rows), int(num_rows * degree), rp.handle, col.handle,
               w.handle if w is not None else None, C.byref(h))
        return cls(h, keep=(rp, col) if w is None else (rp, col, w))

    def destroy(self):
        if self._h:
            L.call("rvx_graph_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
