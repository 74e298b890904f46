// k_hyper.hip — the Poincaré-ball kernels of HyperbolicHnsw beyond graph
// search (crates/ruvector-hyperbolic-hnsw/src/{hnsw.rs,tangent.rs,poincare.rs}):
//   project_rows      project_to_ball of inserted vectors / queries (hnsw.rs:195, :409)
//   poincare_topk     exact top-k with HyperbolicHnsw::distance (ground truth, K8) on
//                     the tiled scan of k_scan.hip
//   log_map_rows      TangentCache coordinates log_c(x) (tangent.rs:57-62)
//   col_chain         frechet_mean's point-major sums sum_i w x_i and sum_i w log_mean(p_i)
//                     in the reference's f32 order (poincare.rs:463-538)
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

// acc[j] = (((acc[j] + w*rows[0][j]) + w*rows[1][j]) + ...): the reference's point-major
// f32 accumulation, `mean[i] += weight * val` and `grad[i] += weight * val` over the
// points in order (frechet_mean, poincare.rs:501-506, :519-525) — one sequential chain
// per dimension, continued across calls through acc. A block owns CH_DIMS dimensions:
// its 256 threads stage CH_ROWS rows of them (the products w*x, rounded as the reference
// rounds them) into LDS, transposed so a chain lane reads four consecutive rows of its
// dimension with one ds_read_b128; lanes 0..3 of wave 0 run the chains of tile t while
// every thread's loads of tile t+1 are in flight (two LDS buffers, one barrier per tile).
// Blocks of one XCD (block id mod 8) take adjacent dimension groups, so a row's cache
// line is fetched from HBM once per XCD.
constexpr int CH_DIMS = 4;
constexpr int CH_ROWS = 1024;
constexpr int CH_PER_THREAD = CH_ROWS / 256;

template <bool VEC>
__device__ __forceinline__ void chain_load(const float* rows, int64_t n, int d, int j0, float w, int64_t r0, int t,
                                           float (&v)[CH_PER_THREAD][CH_DIMS]) {
#pragma unroll
    for (int u = 0; u < CH_PER_THREAD; ++u) {
        const int64_t r = r0 + t + 256 * u;
        if (r < n) {
            const float* p = rows + r * d + j0;
            if constexpr (VEC) {
                const float4 q = *reinterpret_cast<const float4*>(p);
                v[u][0] = q.x; v[u][1] = q.y; v[u][2] = q.z; v[u][3] = q.w;
            } else {
#pragma unroll
                for (int c = 0; c < CH_DIMS; ++c) v[u][c] = (j0 + c < d) ? p[c] : 0.0f;
            }
        } else {
#pragma unroll
            for (int c = 0; c < CH_DIMS; ++c) v[u][c] = 0.0f;
        }
    }
#pragma unroll
    for (int u = 0; u < CH_PER_THREAD; ++u)
#pragma unroll
        for (int c = 0; c < CH_DIMS; ++c) v[u][c] = w * v[u][c];
}

template <bool VEC>
__global__ __launch_bounds__(256) void k_col_chain(const float* rows, int64_t n, int d, float w, float* acc) {
    __shared__ float4 st[2][CH_DIMS][CH_ROWS / 4];  // [buffer][dim][row / 4]: 32 KB
    const int groups = (d + CH_DIMS - 1) / CH_DIMS;
    const int per_xcd = (groups + 7) / 8;
    const int g = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (g >= groups) return;  // uniform over the block, before any barrier
    const int j0 = g * CH_DIMS;
    const int t = threadIdx.x;
    const bool chain = t < CH_DIMS && j0 + t < d;
    float s = chain ? acc[j0 + t] : 0.0f;
    const int64_t tiles = (n + CH_ROWS - 1) / CH_ROWS;
    float v[CH_PER_THREAD][CH_DIMS];
    chain_load<VEC>(rows, n, d, j0, w, 0, t, v);
    for (int64_t k = 0; k < tiles; ++k) {
        float* buf = reinterpret_cast<float*>(st[k & 1]);
#pragma unroll
        for (int u = 0; u < CH_PER_THREAD; ++u)
#pragma unroll
            for (int c = 0; c < CH_DIMS; ++c) buf[c * CH_ROWS + t + 256 * u] = v[u][c];
        __syncthreads();
        if (k + 1 < tiles) chain_load<VEC>(rows, n, d, j0, w, (k + 1) * CH_ROWS, t, v);
        if (chain) {
            const int cnt = (int)min<int64_t>(CH_ROWS, n - k * CH_ROWS);
            const float4* col = st[k & 1][t];
            int i = 0;
            for (; i + 4 <= cnt; i += 4) {
                const float4 q = col[i / 4];
                s = s + q.x;
                s = s + q.y;
                s = s + q.z;
                s = s + q.w;
            }
            const float* tail = reinterpret_cast<const float*>(col);
            for (; i < cnt; ++i) s = s + tail[i];
        }
        // the next iteration writes the other buffer; the one after writes this one
        // only after the next barrier, which every chain lane reaches after its reads
    }
    if (chain) acc[j0 + t] = s;
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

// k * prune_factor > SCAN_MAX_K: every candidate's exact distance (NaN for an empty
// candidate slot), then select_topk by (distance, position) — the stable sort of
// hnsw.rs:481 over the ascending tangent order.
__global__ void k_rerank_dist(const float* q, int64_t nq, const float* x, int d, float c, const int64_t* cand, int nc,
                              float* out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nq * nc) return;
    const int64_t qi = t / nc;
    const int64_t id = cand[t];
    out[t] = (id >= 0 && id != INT64_MAX) ? pdev::hyp_dist(q + qi * d, x + id * d, d, c) : __builtin_nanf("");
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

void col_chain(const float* rows, int64_t n, int d, float w, float* acc) {
    if (n <= 0 || d <= 0) return;
    const int groups = (d + CH_DIMS - 1) / CH_DIMS;
    const unsigned blocks = (unsigned)(8 * ((groups + 7) / 8));
    const bool vec = d % 4 == 0 && ((uintptr_t)rows & 15) == 0;
    if (vec)
        RVX_LAUNCH("hyp_col_chain", k_col_chain<true>, dim3(blocks), dim3(256), 0, rows, n, d, w, acc);
    else
        RVX_LAUNCH("hyp_col_chain", k_col_chain<false>, dim3(blocks), dim3(256), 0, rows, n, d, w, acc);
}

void rerank(const float* q, int64_t nq, const float* x, int d, float c, const int64_t* cand, int nc, int k,
            float* out_d, int64_t* out_i, int32_t* out_n) {
    if (nq <= 0) return;
    RVX_REQUIRE(nc >= 1, RVX_ERR_INVALID_PARAMETER, "candidate count out of range");
    if (nc > SCAN_MAX_K) {
        // query batches whose distances and selection footprint (row, histogram, min(k, nc) keys)
        // stay within 4 GiB, as the wide scan batches its rows
        const int64_t keys = std::min<int64_t>(k, nc);
        const int64_t per_query = (int64_t)nc * 4 + 2048 * 4 + 64 + keys * (keys > 8192 ? 16 : 8);
        const int64_t nqb = std::max<int64_t>(1, std::min<int64_t>(nq, ((int64_t)4 << 30) / per_query));
        float* dist = scratch_f32("hyp_rerank_d", nqb * (int64_t)nc);
        for (int64_t q0 = 0; q0 < nq; q0 += nqb) {
            const int64_t nb = std::min(nqb, nq - q0);
            RVX_LAUNCH("hyp_rerank", k_rerank_dist, dim3((unsigned)((nb * nc + 255) / 256)), dim3(256), 0, q + q0 * d,
                       nb, x, d, c, cand + q0 * nc, nc, dist);
            select_topk(dist, nb, nc, nc, k, cand + q0 * nc, 0, out_d + q0 * k, out_i + q0 * k,
                        out_n ? out_n + q0 : nullptr);
        }
        return;
    }
    RVX_LAUNCH("hyp_rerank", k_rerank, dim3((unsigned)nq), dim3(64), 0, q, nq, x, d, c, cand, nc, k, out_d, out_i,
               out_n);
}

}  // namespace rvx
