"""ruvector_amd — MI355X-native GNN-learned-index hot path of ruvector.

Every compute call goes through librvx.so (hand-written HIP kernels for
gfx950, C ABI in include/rvx/rvx.h). Importing the package loads the library
and fails loudly if it is missing; there is no CPU fallback.
"""
from . import _lib

_lib.load()

from ._lib import RvxError  # noqa: E402
from .device import Buffer, Profiler, device_count, device_info, release_scratch, set_device, synchronize  # noqa: E402
from .graph import Graph  # noqa: E402
from .core import (DistanceMetric, FlatIndex, HnswConfig, HnswIndex, RuvectorError, SearchResult,  # noqa: E402
                   batch_distances, distance, distance_matrix, hnsw_last_search_stats, scan_last_stats)
from .gnn import (GCNLayer, GnnError, GraphSAGELayer, RuvectorLayer, aggregate, differentiable_search,
                  differentiable_search_device,  # noqa: E402
                  differentiable_search_batch, hierarchical_forward, hierarchical_forward_batch,
                  hierarchical_forward_device, pack_row_image, row_image, row_image_bytes)
from .attention import DualSpaceAttention, DualSpaceConfig, EdgeFeaturedAttention, EdgeFeaturedConfig  # noqa: E402
from .hyperbolic import (DualSpaceIndex, HyperbolicError, HyperbolicHnsw, HyperbolicHnswConfig,  # noqa: E402
                         ShardedHyperbolicHnsw, ShardedHyperbolicSearch)

from .query import NeuralSearch, QueryMode, RuvectorQuery  # noqa: E402
from .vector_db import DbOptions, SearchQuery, VectorDB, VectorEntry  # noqa: E402

__all__ = [
    "RvxError", "Buffer", "Profiler", "device_count", "device_info", "release_scratch", "set_device", "synchronize", "Graph",
    "DistanceMetric", "FlatIndex", "HnswConfig", "HnswIndex", "RuvectorError", "SearchResult", "batch_distances",
    "distance", "distance_matrix", "GCNLayer", "GnnError", "GraphSAGELayer", "RuvectorLayer", "aggregate",
    "differentiable_search", "differentiable_search_batch", "hierarchical_forward", "EdgeFeaturedAttention",
    "DualSpaceAttention", "DualSpaceConfig",
    "EdgeFeaturedConfig", "HyperbolicError", "HyperbolicHnsw", "HyperbolicHnswConfig", "ShardedHyperbolicHnsw", "ShardedHyperbolicSearch",
    "DualSpaceIndex",
    "NeuralSearch", "QueryMode", "RuvectorQuery", "DbOptions", "SearchQuery", "VectorDB", "VectorEntry", "differentiable_search_device", "hnsw_last_search_stats", "scan_last_stats",
    "pack_row_image", "row_image", "row_image_bytes",
]
__version__ = "0.1.0"
