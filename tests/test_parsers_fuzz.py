"""Caller-supplied files and text through librvx's host parsers, truncated and corrupted
(VERDICT r3 hygiene): the hnsw_rs dump reader (rvx_hnswio_describe, rvx_index_file_load;
patches/hnsw_rs/src/hnswio.rs:48-67 description, :937-1040, :1221-1290 point graph), the
feature-file headers (rvx_feature_file_info; mmap.rs:147-218, cold_tier.rs:45-101) and the
RuvectorLayer JSON reader (rvx_gnn_layer_from_json; crates/ruvector-gnn/src/layer.rs:313-333).

Every variant must come back as an RvxError (or, for a structurally valid input, a
device error on a machine without a GPU) — never a crash. The same tests run under
AddressSanitizer + UBSan in tests/test_asan.py (`make asan`), which turns any
out-of-bounds access or undefined arithmetic on these paths into a failure."""
import os
import struct

import numpy as np
import pytest

import hnswrs_io as H
import oracle as O
from ruvector_amd import RvxError
from ruvector_amd import _lib as L
from ruvector_amd import formats as F

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _variants(blob, seed, flips=48):
    """Truncations at many lengths and single-byte / multi-byte corruptions of `blob`."""
    out = [blob[:k] for k in sorted({0, 1, 3, 4, 5, 8, 16, len(blob) // 3, len(blob) // 2, len(blob) - 1})]
    r = np.random.default_rng(seed)
    for _ in range(flips):
        b = bytearray(blob)
        for _ in range(int(r.integers(1, 4))):
            i = int(r.integers(0, len(b)))
            b[i] = int(r.integers(0, 256))
        out.append(bytes(b))
    for i in range(0, min(len(blob), 64), 4):  # header words to extreme values
        for v in (b"\xff\xff\xff\xff", b"\x00\x00\x00\x80"):
            b = bytearray(blob)
            b[i:i + 4] = v
            out.append(bytes(b))
    return out


@pytest.fixture(scope="module")
def dump(tmp_path_factory):
    n, d = 120, 8
    x = O.fill_uniform(n * d, 3).reshape(n, d)
    h = O.Hnsw(d, "l2", m=4, ef_construction=20, seed=3)
    h.insert(x, threads=2)
    base = str(tmp_path_factory.mktemp("dump") / "idx")
    H.write_dump(base, h.export(), x, np.arange(n, dtype=np.uint64), 4, 20)
    return open(base + ".hnsw.graph", "rb").read(), open(base + ".hnsw.data", "rb").read()


def _load(dirname, name):
    import ctypes as C
    h = C.c_void_p()
    try:
        L.call("rvx_index_file_load", dirname.encode(), name.encode(), -1, 0, 0, C.byref(h))
    finally:
        if h.value:
            L.call("rvx_index_destroy", h)


def test_hnsw_dump_reader_rejects_damaged_files(dump, tmp_path):
    graph, data = dump
    cases = [(g, data) for g in _variants(graph, 1)] + [(graph, dd) for dd in _variants(data, 2, flips=24)]
    for i, (g, dd) in enumerate(cases):
        name = f"v{i}"
        (tmp_path / f"{name}.hnsw.graph").write_bytes(g)
        (tmp_path / f"{name}.hnsw.data").write_bytes(dd)
        try:
            F.describe_dump(str(tmp_path), name)
        except RvxError:
            pass
        try:
            _load(str(tmp_path), name)
        except RvxError:
            pass  # serialization error, or a device error once the files parse (no GPU here)


def test_feature_file_headers_reject_damaged_files(tmp_path):
    d, n = 6, 5
    x = np.arange(n * d, dtype=np.float32).reshape(n, d)
    cold = struct.pack("<QQQ", d, n, 64) + b"".join(r.tobytes() + b"\0" * (64 - 4 * d) for r in x)
    bad_headers = [struct.pack("<QQQ", 2**63 - 1, n, 64), struct.pack("<QQQ", d, 2**63, 64),
                   struct.pack("<QQQ", d, n, 2**64 - 1), struct.pack("<QQQ", 2**62, 1, 2**62),
                   struct.pack("<QQQ", d, n, 0), struct.pack("<QQQ", 0, n, 64), struct.pack("<QQQ", d, 10**6, 64)]
    blobs = _variants(cold, 3) + [h + cold[24:] for h in bad_headers]
    for i, blob in enumerate(blobs):
        p = tmp_path / f"f{i}.cold"
        p.write_bytes(blob)
        try:
            info = F.feature_file_info(str(p), F.COLD_TIER)
            assert info["rows"] * info["block_size"] <= len(blob) - 24  # what it accepts fits the file
        except RvxError:
            pass
    raw = tmp_path / "raw.bin"
    x.tofile(str(raw))
    for dim in (0, -1, 2**62, 2**31 + 1):
        with pytest.raises(RvxError):
            F.feature_file_info(str(raw), F.RAW, dim)


def test_layer_json_reader_rejects_damaged_text():
    text = open(os.path.join(GOLDEN, "rvl_layer_4_8_2.json")).read()
    blob = text.encode()
    extra = [b"", b"{", b"[", b'{"w_msg":', b'{"a":1e999999}', b'{"a":"\\u12"}', b"[" * 5000 + b"]" * 5000,
             b'{"w_msg":{"weight":{"v":1,"dim":[4294967296,4294967296],"data":[1]}}}',
             b'{"w_msg":{"weight":{"v":1,"dim":[-1,2],"data":[]}}}', b'"\\', b"nul", b"-", b"1e", b"\x00"]
    import ctypes as C
    for v in _variants(blob, 4, flips=64) + extra:
        h = C.c_void_p()
        try:
            L.call("rvx_gnn_layer_from_json", v, C.byref(h))
        except RvxError:
            continue
        if h.value:
            L.call("rvx_gnn_layer_destroy", h)
