"""ctypes binding of librvx.so — the C ABI declared in include/rvx/rvx.h.

The product path of this package always runs through this library (HIP
kernels on gfx950). If the shared object is missing, importing a compute API
raises immediately; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RVX_LIB: load another in-tree build (A/B kernel experiments); default librvx.so
LIB_PATH = os.environ.get("RVX_LIB") or os.path.join(_HERE, "librvx.so")

COMM_ID_BYTES = 128

# status codes (rvx.h)
OK = 0
STATUS_NAMES = {
    1: "DimensionMismatch", 2: "InvalidParameter", 3: "IndexError", 4: "LayerConfig", 5: "InvalidShape",
    6: "DeviceError", 7: "OutOfMemory", 8: "Unsupported", 9: "Serialization", 10: "CommError", 11: "NotFound",
}

METRIC_L2, METRIC_COSINE, METRIC_DOT, METRIC_L1, METRIC_POINCARE, METRIC_HYP_L2 = 0, 1, 2, 3, 4, 5
INDEX_FLAT, INDEX_HNSW = 0, 1
AGG_SUM, AGG_MEAN, AGG_MAX = 0, 1, 2
SAGE_MEAN, SAGE_MAXPOOL, SAGE_LSTM = 0, 1, 2


class RvxError(RuntimeError):
    """A failed rvx call. `code` is the rvx_status, `kind` its reference error name."""

    def __init__(self, code: int, msg: str):
        self.code = code
        self.kind = STATUS_NAMES.get(code, f"status{code}")
        super().__init__(f"{self.kind}: {msg}")


class IndexConfig(C.Structure):
    _fields_ = [("kind", C.c_int32), ("dim", C.c_int32), ("metric", C.c_int32), ("m", C.c_int32),
                ("ef_construction", C.c_int32), ("ef_search", C.c_int32), ("max_elements", C.c_int64),
                ("curvature", C.c_float), ("seed", C.c_uint64)]


class EdgeAttentionConfig(C.Structure):
    _fields_ = [("node_dim", C.c_int32), ("edge_dim", C.c_int32), ("num_heads", C.c_int32), ("dropout", C.c_float),
                ("concat_heads", C.c_int32), ("add_self_loops", C.c_int32), ("negative_slope", C.c_float)]


class DualAttentionConfig(C.Structure):
    _fields_ = [("dim", C.c_int32), ("curvature", C.c_float), ("euclidean_weight", C.c_float),
                ("hyperbolic_weight", C.c_float), ("temperature", C.c_float)]


class HyperbolicConfig(C.Structure):
    _fields_ = [("dim", C.c_int32), ("max_connections", C.c_int32), ("max_connections_0", C.c_int32),
                ("ef_construction", C.c_int32), ("ef_search", C.c_int32), ("level_mult", C.c_float),
                ("curvature", C.c_float), ("prune_factor", C.c_int32), ("seed", C.c_uint64),
                ("metric", C.c_int32)]


class HnswGraph(C.Structure):
    _fields_ = [("n", C.c_int64), ("max_level", C.c_int32), ("entry_point", C.c_int64),
                ("levels", C.POINTER(C.c_uint8)), ("row_ptr0", C.POINTER(C.c_int64)),
                ("col0", C.POINTER(C.c_int32)), ("upper_count", C.POINTER(C.c_int64)),
                ("upper_ids", C.POINTER(C.POINTER(C.c_int32))), ("upper_row_ptr", C.POINTER(C.POINTER(C.c_int64))),
                ("upper_col", C.POINTER(C.POINTER(C.c_int32)))]


class HnswioDescription(C.Structure):
    _fields_ = [("format_version", C.c_int32), ("dump_mode", C.c_int32), ("max_nb_connection", C.c_int32),
                ("nb_layer", C.c_int32), ("level_scale", C.c_double), ("ef_construction", C.c_int64),
                ("nb_point", C.c_int64), ("dimension", C.c_int64), ("distname", C.c_char * 257),
                ("t_name", C.c_char * 257)]


P = C.c_void_p
I32, I64, U64, F32, SZ = C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_size_t
PI32, PI64, PU64, PF32 = C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_uint64), C.POINTER(C.c_float)
PP = C.POINTER(C.c_void_p)

# name -> (restype, argtypes). restype None = rvx_status checked.
SIGNATURES = {
    "rvx_last_error": (I32, [C.c_char_p, SZ]),
    "rvx_version": (C.c_char_p, []),
    "rvx_device_count": (None, [PI32]),
    "rvx_set_device": (None, [I32]),
    "rvx_get_device": (None, [PI32]),
    "rvx_synchronize": (None, []),
    "rvx_scratch_release": (None, []),
    "rvx_device_info": (None, [PI32, PI64, C.c_char_p, SZ]),
    "rvx_buffer_alloc": (None, [I64, PP]),
    "rvx_buffer_free": (None, [P]),
    "rvx_buffer_bytes": (I64, [P]),
    "rvx_buffer_device_ptr": (P, [P]),
    "rvx_buffer_upload": (None, [P, P, I64, I64]),
    "rvx_buffer_download": (None, [P, P, I64, I64]),
    "rvx_buffer_gather_rows_f32": (None, [P, I64, I32, P, I64, P]),
    "rvx_buffer_zero": (None, [P]),
    "rvx_fill_uniform": (None, [P, I64, U64, F32, F32]),
    "rvx_fill_uniform_at": (None, [P, I64, U64, I64, F32, F32]),
    "rvx_fill_ball_rows": (None, [P, I64, I32, U64, I64, F32]),
    "rvx_fill_normal": (None, [P, I64, U64]),
    "rvx_normalize_rows": (None, [P, I64, I32]),
    "rvx_random_csr": (None, [I64, I32, U64, P, P]),
    "rvx_random_csr_shard": (None, [I64, I64, I64, I32, U64, P, P]),
    "rvx_graph_from_edges": (None, [I64, PI64, PI64, I64, PF32, PP]),
    "rvx_graph_from_csr": (None, [I64, PI64, PI32, PF32, PP]),
    "rvx_graph_from_device_csr": (None, [I64, I64, P, P, P, PP]),
    "rvx_graph_info": (None, [P, PI64, PI64, PI32]),
    "rvx_graph_destroy": (None, [P]),
    "rvx_aggregate_device": (None, [P, I32, I32, I32, P, I32, P]),
    "rvx_sage_layer_create": (None, [I32, I32, I32, I32, I32, PF32, PF32, PP]),
    "rvx_sage_layer_destroy": (None, [P]),
    "rvx_sage_sample_positions": (None, [I32, I32, PI32]),
    "rvx_sage_forward": (None, [P, P, PF32, I64, PF32]),
    "rvx_sage_forward_device": (None, [P, P, P, P]),
    "rvx_sage_forward_shard_device": (None, [P, P, P, I64, P]),
    "rvx_sage_forward_exchange": (None, [P, P, P, P, PI64, P, I32]),
    "rvx_sage_forward_exchange2": (None, [P, P, P, P, P, P, PI64, P, I32]),
    "rvx_sage_forward_exchange3": (None, [P, P, P, P, P, P, P, P, PI64, P, I32]),
    "rvx_row_image_bytes": (None, [I64, I32, PI64]),
    "rvx_row_image_pack": (None, [P, I64, I64, I64, I32, P]),
    "rvx_gcn_layer_create": (None, [I32, I32, I32, PF32, PF32, PP]),
    "rvx_gcn_layer_destroy": (None, [P]),
    "rvx_gcn_forward": (None, [P, P, I32, PF32, I64, PF32]),
    "rvx_gnn_layer_create": (None, [I32, I32, I32, F32, U64, PP]),
    "rvx_gnn_layer_from_json": (None, [C.c_char_p, PP]),
    "rvx_gnn_layer_to_json": (None, [P, C.c_char_p, C.POINTER(SZ)]),
    "rvx_gnn_layer_dims": (None, [P, PI32, PI32, PI32, PF32]),
    "rvx_gnn_layer_destroy": (None, [P]),
    "rvx_gnn_forward_one": (None, [P, PF32, PF32, I32, PF32, I32, PF32]),
    "rvx_gnn_forward_graph": (None, [P, P, PF32, I64, PF32]),
    "rvx_gnn_forward_graph_device": (None, [P, P, P, P]),
    "rvx_gnn_forward_exchange": (None, [P, P, P, P, PI64, P]),
    "rvx_differentiable_search_batch": (None, [PF32, I64, PF32, I32, I32, I32, F32, PI64, PF32]),
    "rvx_gnn_forward_star_device": (None, [P, P, I64, P, I64, P, I32, P, P]),
    "rvx_hierarchical_forward_device": (None, [P, I32, P, P, I32, P, I64, I32, P, P]),
    "rvx_hnsw_last_search_stats": (None, [PI64, PI64, PI64]),
    "rvx_scan_last_stats": (None, [PI64, PI64, PI64]),
    "rvx_differentiable_search_device": (None, [P, I64, P, I64, P, I32, I32, I32, F32, P, P, P]),
    "rvx_edge_attention_create": (None, [C.POINTER(EdgeAttentionConfig), PP]),
    "rvx_edge_attention_destroy": (None, [P]),
    "rvx_edge_attention_dim": (None, [P, PI32]),
    "rvx_edge_attention_compute": (None, [P, PF32, PF32, PF32, PF32, I32, PF32]),
    "rvx_edge_attention_forward_graph_device": (None, [P, P, P, P, P]),
    "rvx_edge_attention_forward_exchange": (None, [P, P, P, P, P, PI64, P]),
    "rvx_dual_attention_create": (None, [C.POINTER(DualAttentionConfig), PP]),
    "rvx_dual_attention_destroy": (None, [P]),
    "rvx_dual_attention_compute": (None, [P, PF32, PF32, PF32, I32, I32, PF32]),
    "rvx_dual_attention_forward_graph_device": (None, [P, P, P, P]),
    "rvx_index_create": (None, [C.POINTER(IndexConfig), PP]),
    "rvx_index_destroy": (None, [P]),
    "rvx_index_add_batch": (None, [P, PF32, PU64, I64]),
    "rvx_index_add_batch_device": (None, [P, P, I64, U64]),
    "rvx_index_len": (None, [P, PI64]),
    "rvx_index_remove": (None, [P, U64, PI32]),
    "rvx_index_search": (None, [P, PF32, I64, I32, I32, PU64, PF32, PI32]),
    "rvx_index_search_device": (None, [P, P, I64, I32, I32, P, P]),
    "rvx_index_brute_force": (None, [P, PF32, I64, I32, PU64, PF32]),
    "rvx_index_brute_force_device": (None, [P, P, I64, I32, P, P]),
    "rvx_hnsw_last_search_visited": (None, [PI32, PI32]),
    "rvx_hnsw_last_search_form": (None, [PI32, PI32, PI32]),
    "rvx_scan_last_second_pass": (None, [PI64]),
    "rvx_scan_last_band": (None, [PI64]),
    "rvx_index_sharded_search": (None, [P, P, PF32, I64, I32, I32, I32, PU64, PF32, PI32]),
    "rvx_index_sharded_search_device": (None, [P, P, P, I64, I32, I32, I32, P, P]),
    "rvx_index_load_graph": (None, [P, C.POINTER(HnswGraph)]),
    "rvx_hyperbolic_default_config": (C.c_void_p, [C.POINTER(HyperbolicConfig)]),  # void
    "rvx_hyperbolic_create": (None, [C.POINTER(HyperbolicConfig), PP]),
    "rvx_hyperbolic_destroy": (None, [P]),
    "rvx_hyperbolic_index": (None, [P, PP]),
    "rvx_hyperbolic_insert_batch": (None, [P, PF32, I64, PI64]),
    "rvx_hyperbolic_insert_batch_device": (None, [P, P, I64, PI64]),
    "rvx_hyperbolic_len": (None, [P, PI64]),
    "rvx_hyperbolic_search": (None, [P, PF32, I64, I32, I32, PI64, PF32, PI32]),
    "rvx_hyperbolic_search_with_pruning": (None, [P, PF32, I64, I32, PI64, PF32, PI32]),
    "rvx_hyperbolic_brute_force": (None, [P, PF32, I64, I32, PI64, PF32]),
    "rvx_hyperbolic_search_device": (None, [P, P, I64, I32, I32, I32, P, P]),
    "rvx_hyperbolic_sharded_search": (None, [P, P, I64, PF32, I64, I32, I32, I32, PI64, PI64, PF32, PI32]),
    "rvx_hyperbolic_sharded_search_device": (None, [P, P, I64, P, I64, I32, I32, I32, P, P, P]),
    "rvx_hyperbolic_build_tangent_cache": (None, [P]),
    "rvx_hyperbolic_tangent_centroid": (None, [P, PF32]),
    "rvx_hyperbolic_get_vector": (None, [P, I64, PF32]),
    "rvx_hyperbolic_set_curvature": (None, [P, F32]),
    "rvx_index_graph_sizes": (None, [P, PI64, PI32, PI64, PI64, PI64, PI64]),
    "rvx_index_export_graph": (None, [P, C.POINTER(C.c_uint8), PI64, PI32, PI32, PI64, PI32]),
    "rvx_index_layer0_size": (None, [P, PI64, PI64]),
    "rvx_index_export_layer0": (None, [P, PI64, PI32, PF32]),
    "rvx_hnswio_describe": (None, [C.c_char_p, C.c_char_p, P]),
    "rvx_index_file_dump": (None, [P, C.c_char_p, C.c_char_p]),
    "rvx_index_file_load": (None, [C.c_char_p, C.c_char_p, I32, I32, U64, PP]),
    "rvx_index_export_rows": (None, [P, I64, I64, PF32, PU64, C.POINTER(C.c_uint8), PI64]),
    "rvx_feature_file_info": (None, [C.c_char_p, I32, I64, PI64, PI64, PI64]),
    "rvx_feature_file_load": (None, [C.c_char_p, I32, I64, I64, I64, P, I64]),
    "rvx_feature_file_store": (None, [C.c_char_p, I32, P, I64, I64, I64]),
    "rvx_distance_matrix": (None, [I32, PF32, I64, PF32, I64, I32, F32, PF32]),
    "rvx_selftest_libm": (None, [I32, U64, U64, I64, PF32]),
    "rvx_buffer_checksum": (None, [P, I64, I64, C.POINTER(C.c_uint64)]),
    "rvx_profile_enable": (None, [I32]),
    "rvx_profile_reset": (None, []),
    "rvx_profile_query": (None, [C.c_char_p, C.POINTER(C.c_double), PI64]),
    "rvx_profile_names": (None, [C.c_char_p, SZ]),
    "rvx_comm_unique_id": (None, [C.POINTER(C.c_uint8)]),
    "rvx_comm_init_host": (None, [I32, I32, P, P, P]),
    "rvx_exchange_plan": (None, [I32, P, I32, P, P, P]),
    "rvx_comm_init": (None, [C.POINTER(C.c_uint8), I32, I32, PP]),
    "rvx_comm_destroy": (None, [P]),
    "rvx_comm_allgather_f32": (None, [P, P, I64, P]),
    "rvx_comm_allreduce_max_f64": (None, [P, C.POINTER(C.c_double)]),
    "rvx_comm_allreduce_f64": (None, [P, C.POINTER(C.c_double), I32, I32]),
    "rvx_comm_traffic": (None, [P, PI64, PI64]),
    "rvx_comm_selfcheck": (None, [P, PI64, PI64]),
}

_lib = None
_lock = threading.Lock()


CSRC_DIR = os.path.join(_HERE, "csrc")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "rvx", "rvx.h")


def source_hash() -> str:
    """sha256 (first 16 hex digits) over the library's sources, the same files
    and order as the Makefile's SRC_HASH: sorted paths of csrc/*.cpp, *.hip,
    *.hpp and include/rvx/rvx.h, contents concatenated."""
    import hashlib
    names = [f"ruvector_amd/csrc/{f}" for f in os.listdir(CSRC_DIR)
             if f.endswith((".cpp", ".hip", ".hpp"))] + ["include/rvx/rvx.h"]
    root = os.path.dirname(_HERE)
    h = hashlib.sha256()
    for rel in sorted(names):
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def built_hash(lib) -> str:
    v = lib.rvx_version().decode()
    return v.rsplit(" src ", 1)[-1] if " src " in v else "unknown"


def load() -> C.CDLL:
    """Load librvx.so (raises loudly if it was not built, or if it was built
    from other sources than the ones shipped beside it)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
        lib = C.CDLL(LIB_PATH)
        lib.rvx_version.restype = C.c_char_p
        lib.rvx_version.argtypes = []
        if (not os.environ.get("RVX_LIB") and os.environ.get("RVX_ALLOW_STALE") != "1"
                and os.path.isdir(CSRC_DIR)):
            want, got = source_hash(), built_hash(lib)
            if want != got:
                raise ImportError(
                    f"{LIB_PATH} was built from sources {got}, the tree holds {want}: rebuild it "
                    "(python -c 'import __graft_entry__ as g; g.build()').")
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = I32 if res is None else res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    lib = load()
    buf = C.create_string_buffer(4096)
    lib.rvx_last_error(buf, 4096)
    return buf.value.decode(errors="replace")


def call(name: str, *args):
    """Call a status-returning rvx function, raising RvxError on failure."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != OK:
        raise RvxError(st, last_error())
    return st


def fptr(a: np.ndarray):
    return a.ctypes.data_as(PF32)


def i64ptr(a: np.ndarray):
    return a.ctypes.data_as(PI64)


def i32ptr(a: np.ndarray):
    return a.ctypes.data_as(PI32)


def u64ptr(a: np.ndarray):
    return a.ctypes.data_as(PU64)


def f32c(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)
