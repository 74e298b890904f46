"""Interchange formats of the reference around the hot path.

* ``HnswState`` — ruvector-core's ``HnswIndex::serialize`` / ``deserialize``
  payload (crates/ruvector-core/src/index/hnsw.rs:47-64,136-226): bincode 2.0.1
  ``config::standard()`` (little-endian, variable-length integers) of
  ``{vectors: Vec<(String, Vec<f32>)>, id_to_idx: Vec<(String, usize)>,
  idx_to_id: Vec<(usize, String)>, next_idx: usize, config: {m, ef_construction,
  ef_search, max_elements}, dimensions: usize, metric: enum}``. The graph is not
  part of it: ``deserialize`` rebuilds the index by inserting the vectors.
* hnsw_rs dump files (``.hnsw.graph`` / ``.hnsw.data``,
  patches/hnsw_rs/src/hnswio.rs) — read/written natively by librvx
  (``rvx_index_file_dump`` / ``rvx_index_file_load`` / ``rvx_hnswio_describe``).
* Node-feature files — MmapManager's raw ``[n][d]`` f32 table
  (crates/ruvector-gnn/src/mmap.rs:147-218) and FeatureStorage's cold-tier file
  (crates/ruvector-gnn/src/cold_tier.rs:17-151), streamed into / out of HBM by
  librvx (``rvx_feature_file_*``).
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

from . import _lib as L
from .device import Buffer

RAW, COLD_TIER = 0, 1

# SerializableDistanceMetric variant order (index/hnsw.rs:66-72)
METRIC_VARIANTS = ("Euclidean", "Cosine", "DotProduct", "Manhattan")


# ---------------------------------------------------------------- bincode 2 (standard config)
def enc_varint(v: int) -> bytes:
    """bincode 2 varint: < 251 one byte; 251/252/253/254 + u16/u32/u64/u128 LE."""
    if v < 0:
        raise ValueError("unsigned varint")
    if v < 251:
        return bytes([v])
    if v < 1 << 16:
        return b"\xfb" + struct.pack("<H", v)
    if v < 1 << 32:
        return b"\xfc" + struct.pack("<I", v)
    if v < 1 << 64:
        return b"\xfd" + struct.pack("<Q", v)
    return b"\xfe" + v.to_bytes(16, "little")


class _Reader:
    def __init__(self, data: bytes):
        self.b, self.i = memoryview(data), 0

    def take(self, n: int) -> bytes:
        if self.i + n > len(self.b):
            raise L.RvxError(9, "Serialization: unexpected end of bincode data")
        out = bytes(self.b[self.i:self.i + n])
        self.i += n
        return out

    def varint(self) -> int:
        t = self.take(1)[0]
        if t < 251:
            return t
        width = {251: 2, 252: 4, 253: 8, 254: 16}.get(t)
        if width is None:
            raise L.RvxError(9, f"Serialization: invalid varint tag {t}")
        return int.from_bytes(self.take(width), "little")

    def string(self) -> str:
        return self.take(self.varint()).decode("utf-8")

    def f32_vec(self) -> np.ndarray:
        n = self.varint()
        return np.frombuffer(self.take(4 * n), dtype="<f4").astype(np.float32)


@dataclass
class HnswState:
    """ruvector-core's serialisable HNSW index state (index/hnsw.rs:47-64)."""
    vectors: List[Tuple[str, np.ndarray]] = field(default_factory=list)
    id_to_idx: List[Tuple[str, int]] = field(default_factory=list)
    idx_to_id: List[Tuple[int, str]] = field(default_factory=list)
    next_idx: int = 0
    m: int = 32
    ef_construction: int = 200
    ef_search: int = 100
    max_elements: int = 10_000_000
    dimensions: int = 0
    metric: str = "Euclidean"

    def encode(self) -> bytes:
        out = bytearray()
        out += enc_varint(len(self.vectors))
        for vid, vec in self.vectors:
            s = vid.encode("utf-8")
            v = np.ascontiguousarray(vec, dtype="<f4")
            out += enc_varint(len(s)) + s + enc_varint(v.size) + v.tobytes()
        out += enc_varint(len(self.id_to_idx))
        for vid, idx in self.id_to_idx:
            s = vid.encode("utf-8")
            out += enc_varint(len(s)) + s + enc_varint(int(idx))
        out += enc_varint(len(self.idx_to_id))
        for idx, vid in self.idx_to_id:
            s = vid.encode("utf-8")
            out += enc_varint(int(idx)) + enc_varint(len(s)) + s
        out += enc_varint(self.next_idx)
        for v in (self.m, self.ef_construction, self.ef_search, self.max_elements, self.dimensions):
            out += enc_varint(int(v))
        out += enc_varint(METRIC_VARIANTS.index(self.metric))
        return bytes(out)

    @classmethod
    def decode(cls, data: bytes) -> "HnswState":
        r = _Reader(data)
        st = cls()
        st.vectors = [(r.string(), r.f32_vec()) for _ in range(r.varint())]
        st.id_to_idx = [(r.string(), r.varint()) for _ in range(r.varint())]
        st.idx_to_id = [(r.varint(), r.string()) for _ in range(r.varint())]
        st.next_idx = r.varint()
        st.m, st.ef_construction, st.ef_search, st.max_elements, st.dimensions = (r.varint() for _ in range(5))
        v = r.varint()
        if v >= len(METRIC_VARIANTS):
            raise L.RvxError(9, f"Serialization: unknown metric variant {v}")
        st.metric = METRIC_VARIANTS[v]
        return st


# ---------------------------------------------------------------- hnsw_rs dump description
def describe_dump(directory: str, basename: str) -> dict:
    """load_description (hnswio.rs:937-1040) of `<directory>/<basename>.hnsw.graph` (host only)."""
    d = L.HnswioDescription()
    L.call("rvx_hnswio_describe", directory.encode(), basename.encode(), C.byref(d))
    return {"format_version": d.format_version, "dump_mode": d.dump_mode, "max_nb_connection": d.max_nb_connection,
            "nb_layer": d.nb_layer, "level_scale": d.level_scale, "ef": d.ef_construction,
            "nb_point": d.nb_point, "dimension": d.dimension, "distname": d.distname.decode(),
            "t_name": d.t_name.decode()}


# ---------------------------------------------------------------- node-feature files
def feature_file_info(path: str, layout: int = RAW, dim: int = 0) -> dict:
    """Rows / dim / per-row block bytes of a raw (dim required) or cold-tier feature file."""
    rows, d, blk = C.c_int64(), C.c_int64(), C.c_int64()
    L.call("rvx_feature_file_info", path.encode(), int(layout), int(dim), C.byref(rows), C.byref(d), C.byref(blk))
    return {"rows": rows.value, "dim": d.value, "block_size": blk.value}


def load_features(path: str, layout: int = RAW, dim: int = 0, row0: int = 0, rows: int = -1,
                  out: Buffer = None, out_row0: int = 0) -> Buffer:
    """Stream rows [row0, row0+rows) of a feature file into an HBM buffer ([rows][dim] f32)."""
    info = feature_file_info(path, layout, dim)
    n = info["rows"] - row0 if rows < 0 else rows
    if out is None:
        out = Buffer(max(n, 1) * info["dim"] * 4)
    L.call("rvx_feature_file_load", path.encode(), int(layout), int(info["dim"]), int(row0), int(n), out.handle,
           int(out_row0))
    return out


def store_features(buf: Buffer, path: str, rows: int, dim: int, layout: int = RAW, page_size: int = 0) -> None:
    """Write [rows][dim] f32 from HBM as a raw (MmapManager) or cold-tier (FeatureStorage) file."""
    L.call("rvx_feature_file_store", path.encode(), int(layout), buf.handle, int(dim), int(rows), int(page_size))
