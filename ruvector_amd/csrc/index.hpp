// index.hpp — the rvx_index handle (VectorIndex over HBM) and its HNSW graph state.
#pragma once
#include <shared_mutex>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "hnsw.hpp"
#include "hnsw_build.hpp"

namespace rvx {

// Host copy of a searchable graph in the rvx_hnsw_graph layout.
struct HostGraph {
    int64_t n = 0;
    int max_level = 0;
    int64_t entry = 0;
    std::vector<uint8_t> levels;
    std::vector<int64_t> rp0;
    std::vector<int32_t> col0;
    std::vector<float> dist0;                 // distance of each layer-0 edge (owner, neighbour)
    std::vector<std::vector<int32_t>> up_ids;  // [max_level+1], index 0 unused
    std::vector<std::vector<int64_t>> up_rp;
    std::vector<std::vector<int32_t>> up_col;
};

}  // namespace rvx

struct rvx_index {
    rvx_index_config cfg{};
    int64_t n = 0, cap = 0;
    rvx::DevMem vecs;     // [cap][dim]
    rvx::DevMem norms;    // [cap] (cosine)
    rvx::DevMem ids_dev;  // [cap] u64 user ids
    rvx::DevMem deleted;  // [cap] u8 tombstones
    std::vector<uint64_t> ids;
    std::vector<uint8_t> deleted_h;
    std::unordered_map<uint64_t, int64_t> id_to_row;
    int64_t live = 0;

    // searchable HNSW graph (CSR, loaded or converted from the build state)
    bool has_graph = false;
    int64_t graph_n = 0;
    rvx::HnswDev g;
    rvx::DevMem rp0, col0, up_ids, up_rp, up_col;
    rvx::HostGraph hg;

    // GPU build state (fixed-capacity lists, k_hnsw_build.hip)
    bool build_valid = true;  // false once a foreign graph was loaded
    int64_t bn_cap = 0, bu_cap = 0, n_upper = 0;
    std::vector<uint8_t> h_level;
    std::vector<int64_t> h_up_base;
    rvx::DevMem b_level, b_up_base, b_nb0, b_nbd0, b_cnt0, b_nbu, b_nbud, b_cntu, b_rev_head;
    int entry = -1, entry_level = -1;
    unsigned level_mask = 0;

    // HyperbolicHnsw mode (crates/ruvector-hyperbolic-hnsw/src/hnsw.rs): Poincaré
    // metric with curvature `curv`, M0 lists at layer 0, level = floor(-ln r * level_mult)
    bool hyper = false;
    int m0 = 0;
    float level_mult = 0.0f, curv = 1.0f;
    // TangentCache (tangent.rs:24-40): Fréchet-mean centroid + log-map coordinates
    bool tan_valid = false;
    rvx::DevMem tan_centroid, tan_coords, tan_norms;

    mutable std::shared_mutex mu;
};

namespace rvx {
// Insert rows [first, first+count) of the index into the HNSW graph on the GPU.
void hnsw_insert_range(rvx_index* ix, int64_t first, int64_t count);
// Make `hg` the searchable graph (uploads the CSR).
void hnsw_install(rvx_index* ix, HostGraph&& hg);
// hnsw_rs level of point i (seeded LayerGenerator::generate, hnsw.rs:358-369).
int hnsw_level(uint64_t seed, int m, int max_layer, int64_t i);
// HyperbolicHnsw::random_level (hyperbolic hnsw.rs:186-189) from the same seeded stream.
int hyper_level(uint64_t seed, float level_mult, int64_t i);

// index plumbing shared by the VectorIndex and HyperbolicHnsw entry points (api_index.cpp)
void index_append_rows(rvx_index* ix, const float* rows, const uint64_t* ids, int64_t cnt, bool rows_on_device);
void index_search_rows(const rvx_index* ix, const float* q, int64_t nq, int k, int ef, float* dd, int64_t* di,
                       int32_t* dn, bool exact);
void index_load_graph(rvx_index* ix, const rvx_hnsw_graph* hg);
}  // namespace rvx
