"""HBM-resident buffers, device selection and the event profiler of librvx."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def release_scratch() -> None:
    """Free librvx's per-device scratch pool (kept between calls for reuse)."""
    L.call("rvx_scratch_release")


def device_count() -> int:
    n = C.c_int32(0)
    L.call("rvx_device_count", C.byref(n))
    return n.value


def set_device(dev: int) -> None:
    L.call("rvx_set_device", dev)


def synchronize() -> None:
    L.call("rvx_synchronize")


def device_info() -> dict:
    cus, hbm = C.c_int32(0), C.c_int64(0)
    arch = C.create_string_buffer(64)
    L.call("rvx_device_info", C.byref(cus), C.byref(hbm), arch, 64)
    return {"num_cus": cus.value, "hbm_bytes": hbm.value, "arch": arch.value.decode()}


class Buffer:
    """A device allocation owned by librvx (row-major f32/i32/i64 data)."""

    def __init__(self, nbytes: int):
        h = C.c_void_p()
        L.call("rvx_buffer_alloc", int(nbytes), C.byref(h))
        self._h = h
        self.nbytes = int(nbytes)

    @property
    def handle(self):
        return self._h

    @classmethod
    def from_numpy(cls, a: np.ndarray) -> "Buffer":
        a = np.ascontiguousarray(a)
        b = cls(max(a.nbytes, 1))
        if a.nbytes:
            L.call("rvx_buffer_upload", b._h, a.ctypes.data_as(C.c_void_p), a.nbytes, 0)
        return b

    def upload(self, a: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(a)
        L.call("rvx_buffer_upload", self._h, a.ctypes.data_as(C.c_void_p), a.nbytes, offset)

    def gather_rows(self, rows: int, dim: int, ids) -> np.ndarray:
        """Rows `ids` of this buffer viewed as a [rows][dim] f32 table (device gather)."""
        ids = np.ascontiguousarray(ids, dtype=np.int64).reshape(-1)
        out = np.empty((ids.size, dim), np.float32)
        if ids.size:
            L.call("rvx_buffer_gather_rows_f32", self._h, int(rows), int(dim), ids.ctypes.data_as(C.c_void_p),
                   ids.size, out.ctypes.data_as(C.c_void_p))
        return out

    def download(self, dtype, shape, offset: int = 0) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        if out.nbytes:
            L.call("rvx_buffer_download", self._h, out.ctypes.data_as(C.c_void_p), out.nbytes, offset)
        return out

    def zero(self) -> None:
        L.call("rvx_buffer_zero", self._h)

    def checksum(self, nbytes: int = None, offset: int = 0) -> int:
        """Position-keyed 64-bit checksum of bytes [offset, offset + nbytes) (device kernel)."""
        out = C.c_uint64(0)
        L.call("rvx_buffer_checksum", self._h, int(offset), int(self.nbytes - offset if nbytes is None else nbytes),
               C.byref(out))
        return int(out.value)

    def fill_uniform(self, n: int, seed: int, lo: float = -1.0, hi: float = 1.0) -> None:
        L.call("rvx_fill_uniform", self._h, int(n), int(seed), float(lo), float(hi))

    def fill_uniform_at(self, n: int, seed: int, first: int, lo: float = -1.0, hi: float = 1.0) -> None:
        """Elements [first, first+n) of the fill_uniform(seed) stream."""
        L.call("rvx_fill_uniform_at", self._h, int(n), int(seed), int(first), float(lo), float(hi))

    def fill_normal(self, n: int, seed: int) -> None:
        L.call("rvx_fill_normal", self._h, int(n), int(seed))

    def fill_ball(self, rows: int, dim: int, seed: int, first_row: int = 0, rmax: float = 0.9) -> None:
        """Rows [first_row, first_row+rows) of the C5 corpus (rvx_fill_ball_rows)."""
        L.call("rvx_fill_ball_rows", self._h, int(rows), int(dim), int(seed), int(first_row), float(rmax))

    def normalize_rows(self, rows: int, dim: int) -> None:
        L.call("rvx_normalize_rows", self._h, int(rows), int(dim))

    def free(self) -> None:
        if self._h:
            L.call("rvx_buffer_free", self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Profiler:
    """Per-kernel device time from HIP events recorded on the library stream."""

    def __enter__(self):
        L.call("rvx_profile_reset")
        L.call("rvx_profile_enable", 1)
        return self

    def __exit__(self, *exc):
        L.call("rvx_profile_enable", 0)

    @staticmethod
    def names() -> list:
        buf = C.create_string_buffer(1 << 16)
        L.call("rvx_profile_names", buf, 1 << 16)
        s = buf.value.decode()
        return [x for x in s.split(",") if x]

    @staticmethod
    def query(name: str) -> tuple:
        ms, n = C.c_double(0.0), C.c_int64(0)
        L.call("rvx_profile_query", name.encode(), C.byref(ms), C.byref(n))
        return ms.value, n.value

    def summary(self) -> dict:
        return {n: dict(zip(("total_ms", "launches"), self.query(n))) for n in self.names()}
