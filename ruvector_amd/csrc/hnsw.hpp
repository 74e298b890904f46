// hnsw.hpp — device-side HNSW graph view and the search launcher (k_hnsw.hip).
#pragma once
#include <cstdint>

namespace rvx {

// ef is unbounded in the reference (ef = max(ef_arg, k), hnsw.rs:1519); here R lives in
// one wave's LDS up to ~19k entries (d 768) and in HBM beyond, so the only limit is the
// int32 index range of the R row.
constexpr int HNSW_MAX_EF = (1 << 30);
constexpr int HNSW_MAX_LEVEL = 16;  // NB_LAYER_MAX (patches/hnsw_rs/src/hnsw.rs:41)

// Layer 0 is a CSR over all n points; layer l>=1 is a CSR over the sorted ids
// of the points whose level is >= l. Offsets index the packed upper arrays.
struct HnswDev {
    int64_t n = 0;
    int max_level = 0;
    int64_t entry = 0;
    int max_deg = 0;  // longest layer-0 list (sizes the hashed visited set)
    const int64_t* rp0 = nullptr;
    const int* col0 = nullptr;
    const int* up_ids = nullptr;
    const int64_t* up_rp = nullptr;
    const int* up_col = nullptr;
    int64_t up_count[HNSW_MAX_LEVEL + 1] = {};
    int64_t up_ids_off[HNSW_MAX_LEVEL + 1] = {};
    int64_t up_rp_off[HNSW_MAX_LEVEL + 1] = {};
    int64_t up_col_off[HNSW_MAX_LEVEL + 1] = {};
};

// hyper != 0: HyperbolicHnsw::search semantics (iterated greedy upper descent,
// layer-0 stop also needs |R| >= ef); curv: Poincaré curvature.
void hnsw_search(const HnswDev& g, int metric, const float* x, const float* xnorm, int d, const float* q,
                 const float* qnorm, int64_t nq, int k, int ef, float* out_d, int64_t* out_i, int32_t* out_n,
                 const char* tag, float curv = 1.0f, int hyper = 0);

// Wave-cooperative (LDS-staged) distances: metric not Poincaré, d % 32 == 0, and
// (RVX_HNSW_COOP=1, default) a table of >= RVX_HNSW_COOP_MIN_MB (4096) bytes, where
// per-lane row reads outgrow the per-CU translation cache; 2 forces, 0 disables.
bool hnsw_coop(int metric, int d, int64_t rows);

// Work tallies of the most recent hnsw_search launch (SURVEY.md §8d C1/C3:
// bytes = n_dist * d * 4 + n_expand * deg_cap * 4 per launch).
struct SearchStats {
    int64_t n_dist = 0, n_expand = 0, nq = 0;
    int32_t visited_bitmap = 0, slots = 0;  // visited-set form and search slots of the launch
    int32_t visited_overflow = 0;           // a query's visited hash table filled (nodes were skipped)
    int32_t r_in_hbm = 0, stages = 0;       // kernel form: R in HBM, LDS distance stages (0 per-lane)
};
extern SearchStats g_search_stats;
// The last search's device tallies (n_dist, n_expand) into g_search_stats (waits for the search).
void hnsw_search_stats_settle();
// settle, then fail (RVX_ERR_INDEX) if the last search's visited hash overflowed; host-returning
// entry points call it after their own wait, so it costs no extra synchronisation
void hnsw_search_check();

}  // namespace rvx
