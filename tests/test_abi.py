"""The C-ABI library loads and exports every symbol include/rvx/rvx.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rvx", "rvx.h")
LIB = os.path.join(ROOT, "ruvector_amd", "librvx.so")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rvx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for must in ("rvx_index_search", "rvx_index_load_graph", "rvx_gnn_forward_one", "rvx_gnn_layer_from_json",
                 "rvx_sage_forward_device", "rvx_edge_attention_compute", "rvx_comm_allgather_f32"):
        assert must in syms
    assert len(syms) > 50


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build librvx.so first"
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"declared but not exported: {missing}"


def test_python_bindings_cover_the_header():
    from ruvector_amd import _lib
    assert set(declared_symbols()) == set(_lib.SIGNATURES), \
        set(declared_symbols()) ^ set(_lib.SIGNATURES)


def test_version_and_errors_without_gpu():
    from ruvector_amd import _lib
    lib = _lib.load()
    assert lib.rvx_version().startswith(b"rvx")
    # an invalid argument fails with a status code and a message, without touching a device
    cfg = _lib.IndexConfig(kind=7, dim=4, metric=0)
    h = ctypes.c_void_p()
    st = lib.rvx_index_create(ctypes.byref(cfg), ctypes.byref(h))
    assert st == 2 and "kind" in _lib.last_error()


def test_graft_entry_exposes_build_and_smoke():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ge", os.path.join(ROOT, "__graft_entry__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert callable(m.build) and callable(m.smoke)


def test_library_built_from_shipped_sources():
    """Binary provenance: rvx_version() carries the sha256 of the sources the
    library was built from (Makefile SRC_HASH); it must equal the hash of the
    tree's csrc + header, so a stale prebuilt librvx.so cannot run unnoticed."""
    from ruvector_amd import _lib
    lib = _lib.load()
    assert _lib.built_hash(lib) == _lib.source_hash()
    assert len(_lib.source_hash()) == 16


def test_row_image_sizes_without_gpu():
    """rvx_row_image_bytes (host only): a 3 KiB slot and a u16 count per row, for
    512 < dim <= 768 with dim % 4 == 0; anything else is refused with a status."""
    import ruvector_amd as rv
    assert rv.row_image_bytes(0, 768) == 16
    assert rv.row_image_bytes(10, 768) == 10 * (3072 + 2) + 16
    assert rv.row_image_bytes(7, 516) == 7 * (3072 + 2) + 16
    for n, d in ((10, 512), (10, 772), (10, 770), (-1, 768)):
        with pytest.raises(rv.RvxError):
            rv.row_image_bytes(n, d)
