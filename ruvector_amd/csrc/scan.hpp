// scan.hpp — exact distance scan / top-k launchers (k_scan.hip).
#pragma once
#include <cstdint>

namespace rvx {

// Longest per-query list of the fused top-k scans (K1, K10); larger k take the any-k path
// (the distance rows of a query batch, then select_topk).
constexpr int SCAN_MAX_K = 128;
// Internal metric id (not in rvx.h): squared L2 as a sequential f32 sum without the
// square root, TangentCache::tangent_distance_squared (crates/ruvector-hyperbolic-
// hnsw/src/tangent.rs:105-117), the ranking of search_with_pruning's tangent scan.
constexpr int METRIC_L2SQ = 16;

// Path of the most recent scan_topk call (rvx_scan_last_stats).
struct ScanStats {
    int64_t mfma_queries = 0, valu_queries = 0, fallback_queries = 0;
    int64_t second_pass_queries = 0;  // unsure after the first filter, run again with the most splits
    int64_t band_queries = 0;         // still unsure: every row within the proven bound (k_scan_band)
};
ScanStats& last_scan_stats();

// Sequential-order row norms sqrt(sum x*x) (distance.rs:56-57), one per row.
void row_norms(const float* x, int64_t n, int d, float* out);
// Top-k (ascending (distance, id)) of every query against rows [0, n) of x, any k >= 1.
// Output ids are row + id_offset; rows with deleted[row] != 0 are skipped.
// Poincaré (HyperbolicHnsw::distance with curvature curv): qnorm/xnorm are
// squared norms from row_norm_sq.
void scan_topk(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
               const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
               const char* tag, float curv = 1.0f);
// Exact top-k of each of nseg rows of distances D[seg][0..len) (row stride ld), any k:
// ascending (distance, position), NaN entries excluded, -0.0 tied with +0.0; out ids =
// idmap[seg][pos] (idmap [nseg][len]) or pos + id_offset; empty slots (+inf, INT64_MAX);
// out_n (nullable) = min(k, valid entries). k_select.hip.
void select_topk(const float* D, int64_t nseg, int64_t len, int64_t ld, int k, const int64_t* idmap, int64_t id_offset,
                 float* out_d, int64_t* out_i, int32_t* out_n);
// Squared norms in poincare.rs norm_squared's chunked order, one per row.
void row_norm_sq(const float* x, int64_t n, int d, float* out);
// out[i][j] = distance(q_i, x_j) in the reference scalar order.
void distance_matrix(int metric, const float* q, const float* qn, int64_t nq, const float* x, const float* xn, int64_t n,
                     int d, float* out);

// out[p] = distance(x[owner(p)], x[col[p]]) for every CSR edge p (wave per row).
void edge_distances(int metric, const float* x, const float* xnorm, const int64_t* rp, const int32_t* col, int64_t n,
                    int d, float* out);
// Merge per-chunk ascending top-k lists part_[d|i] [nq][nchunks*k] into out [nq][k].
void merge_topk(const float* part_d, const int64_t* part_i, int64_t nq, int nchunks, int k, float* out_d,
                int64_t* out_i);
// Poincaré ball distance matrix (poincare.rs:227-255), curvature c.
void poincare_matrix(const float* q, int64_t nq, const float* x, int64_t n, int d, float c, float* out);

}  // namespace rvx
