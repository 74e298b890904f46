// k_hyper.hip — the Poincaré-ball kernels of HyperbolicHnsw beyond graph
// search (crates/ruvector-hyperbolic-hnsw/src/{hnsw.rs,tangent.rs,poincare.rs}):
//   project_rows      project_to_ball of inserted vectors / queries (hnsw.rs:195, :409)
//   poincare_topk     exact top-k with HyperbolicHnsw::distance (ground truth, K8) on
//                     the tiled scan of k_scan.hip
//   log_map_rows      TangentCache coordinates log_c(x) (tangent.rs:57-62)
//   frechet_grad      sum_i w log_mean(p_i) for frechet_mean's gradient step (poincare.rs:463-538)
//   rerank            search_with_pruning phase 2: exact distance of the tangent
//                     candidates, stable ascending sort, first k (hnsw.rs:471-482)
// Every per-point distance / map is one thread's sequential chain in the
// reference order (poincare_dev.hpp); HBM reads of a row are per-thread
// streams, which is fine for these O(N d) passes that run once per build or
// for ground truth.
#include "common.hpp"
#include "graph.hpp"
#include "hyper.hpp"
#include "poincare_dev.hpp"
#include "scan.hpp"

namespace rvx {
namespace {

__global__ void k_project_rows(float* x, int64_t n, int d, float c) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    pdev::project_inplace(x + r * d, d, c, pdev::EPS);
}

// out[r] = log_centroid(x[r]) with -centroid and |centroid|^2 precomputed.
__global__ void k_log_map_rows(const float* x, int64_t n, int d, const float* negp, float np_sq, float c, float* out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    pdev::log_map_negp(x + r * d, negp, np_sq, d, c, out + r * d);
}

// Column sums of w * rows[i][j]: blockIdx.y takes a contiguous run of rows
// (index order inside the run), then the runs are added in order —
// deterministic for a given n.
__global__ void k_col_sum_part(const float* rows, int64_t n, int d, float w, int64_t run, float* part) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d) return;
    const int64_t i0 = (int64_t)blockIdx.y * run, i1 = min<int64_t>(n, i0 + run);
    float s = 0.0f;
    for (int64_t i = i0; i < i1; ++i) s = s + w * rows[i * d + j];
    part[(int64_t)blockIdx.y * d + j] = s;
}
__global__ void k_col_sum_final(const float* part, int runs, int d, float* out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d) return;
    float s = 0.0f;
    for (int r = 0; r < runs; ++r) s = s + part[(int64_t)r * d + j];
    out[j] = s;
}

// one wave per query: exact distances of its candidates (ids from the tangent
// scan, ascending tangent order), then the first k by (distance, position)
__global__ __launch_bounds__(64) void k_rerank(const float* q, int64_t nq, const float* x, int d, float c,
                                              const int64_t* cand, int nc, int k, float* out_d, int64_t* out_i,
                                              int32_t* out_n) {
    __shared__ float cd[SCAN_MAX_K];
    const int lane = threadIdx.x;
    const int64_t qi = blockIdx.x;
    if (qi >= nq) return;
    const float* qv = q + qi * d;
    const int64_t* ci = cand + qi * nc;
    int valid = 0;
    for (int s = lane; s < nc; s += 64) {
        const int64_t id = ci[s];
        cd[s] = (id >= 0 && id != INT64_MAX) ? pdev::hyp_dist(qv, x + id * d, d, c) : INFINITY;
    }
    for (int s = 0; s < nc; ++s) valid += (ci[s] >= 0 && ci[s] != INT64_MAX) ? 1 : 0;
    __syncthreads();
    const int take = min(k, valid);
    float last_d = -INFINITY;
    int last_p = -1;
    for (int s = 0; s < k; ++s) {
        float bd = INFINITY;
        int bp = INT_MAX;
        if (s < take) {
            for (int p = lane; p < nc; p += 64) {
                const float dd = cd[p];
                const bool after = dd > last_d || (dd == last_d && p > last_p);
                if (after && (dd < bd || (dd == bd && p < bp))) { bd = dd; bp = p; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const float od = __shfl_xor(bd, o);
                const int op = __shfl_xor(bp, o);
                if (od < bd || (od == bd && op < bp)) { bd = od; bp = op; }
            }
        }
        if (lane == 0) {
            out_d[qi * k + s] = s < take ? bd : INFINITY;
            out_i[qi * k + s] = s < take ? ci[bp] : (int64_t)-1;
        }
        last_d = bd;
        last_p = bp;
    }
    if (lane == 0 && out_n) out_n[qi] = take;
}

}  // namespace

void project_rows(float* x, int64_t n, int d, float c) {
    if (n <= 0) return;
    RVX_LAUNCH("hyp_project", k_project_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, x, n, d, c);
}

void poincare_topk(const float* q, int64_t nq, const float* x, int64_t n, int d, float c, int k, float* out_d,
                   int64_t* out_i) {
    if (nq <= 0) return;
    // the exact scan (k_scan.hip) with the Poincaré metric: the MFMA filter with
    // per-row bounds and a reference-order rerank for query batches (K10), else the
    // tiled VALU scan with |q-x|^2 per pair in fused_norms' chunked order and the
    // squared norms computed there (K8); identical results either way
    scan_topk(RVX_METRIC_POINCARE, q, nullptr, nq, x, nullptr, nullptr, n, d, k, 0, out_d, out_i, "hyp_brute_force", c);
}

void log_map_rows(const float* x, int64_t n, int d, const float* negp_dev, float np_sq, float c, float* out) {
    if (n <= 0) return;
    RVX_LAUNCH("hyp_log_map", k_log_map_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, x, n, d, negp_dev, np_sq,
               c, out);
}

void col_sum(const float* rows, int64_t n, int d, float w, float* out) {
    if (n <= 0 || d <= 0) return;
    const int runs = (int)std::min<int64_t>(1024, std::max<int64_t>(1, n / 256));
    const int64_t run = (n + runs - 1) / runs;
    float* part = scratch_f32("hyp_colsum_part", (int64_t)runs * d);
    RVX_LAUNCH("hyp_col_sum", k_col_sum_part, dim3((unsigned)((d + 255) / 256), (unsigned)runs), dim3(256), 0, rows, n, d,
               w, run, part);
    RVX_LAUNCH("hyp_col_sum", k_col_sum_final, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, part, runs, d, out);
}

void rerank(const float* q, int64_t nq, const float* x, int d, float c, const int64_t* cand, int nc, int k,
            float* out_d, int64_t* out_i, int32_t* out_n) {
    if (nq <= 0) return;
    RVX_REQUIRE(nc >= 1 && nc <= SCAN_MAX_K, RVX_ERR_INVALID_PARAMETER, "candidate count out of range");
    RVX_LAUNCH("hyp_rerank", k_rerank, dim3((unsigned)nq), dim3(64), 0, q, nq, x, d, c, cand, nc, k, out_d, out_i,
               out_n);
}

}  // namespace rvx
