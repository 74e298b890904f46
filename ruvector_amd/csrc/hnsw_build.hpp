// hnsw_build.hpp — mutable fixed-capacity HNSW graph for the GPU builder (k_hnsw_build.hip).
#pragma once
#include <cstdint>

namespace rvx {

struct BuildGraph {
    int64_t n_cap = 0;     // capacity of the layer-0 arrays; upper list keys start here
    int M = 0, C0 = 0;     // capacity M above layer 0, C0 at layer 0 (2M for hnsw_rs, M0 for HyperbolicHnsw)
    int max_layer = 0;     // min(16, dim) as ruvector-core wires it (index/hnsw.rs:102-108); 16 hyperbolic
    const uint8_t* level = nullptr;   // [n_cap]
    int* nb0 = nullptr;               // [n_cap][C0]
    float* nbd0 = nullptr;            // [n_cap][C0] distance to the owner
    int* cnt0 = nullptr;              // [n_cap]
    const int64_t* up_base = nullptr; // [n_cap] first upper list of p (layer 1), -1 at level 0
    int* nbu = nullptr;               // [U][M]
    float* nbud = nullptr;            // [U][M]
    int* cntu = nullptr;              // [U]
};

struct BuildScratch {
    int* rev_head = nullptr;  // [n_cap + U] chain heads of reverse edges, -1 when idle
};

// hyper != 0: HyperbolicHnsw::insert rules (hnsw.rs:192-251): the closest
// max_conn of the ef_c search (no heuristic), reverse edge into the neighbour's
// list at the CURRENT level, pruned to its max_conn closest.
void build_insert_batch(const BuildGraph& G, int metric, const float* x, const float* xnorm, int d,
                        int64_t batch_begin, int batch_n, int entry, int entry_level, unsigned nonempty_mask, int ef_c,
                        BuildScratch& s, float curv = 1.0f, int hyper = 0);

}  // namespace rvx
