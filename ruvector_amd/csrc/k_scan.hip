// k_scan.hip — batched distance scan with fused top-k (FlatIndex / ground truth).
//
// Replaces FlatIndex::search (crates/ruvector-core/src/index/flat.rs:36-76) and
// batch_distances (crates/ruvector-core/src/distance.rs:89-107). Every (query,
// base row) distance is accumulated by ONE lane, sequentially over the
// dimension, without FMA contraction — the exact arithmetic of the reference's
// scalar distance functions (distance.rs:34-42, :52-63, :77-78, :85):
//   L2      sqrt( sum_k (x_k - y_k)*(x_k - y_k) )
//   cosine  1 - dot/(|x|*|y|)  (1.0 if a norm <= 1e-8), norms precomputed per row
//   dot     -sum_k x_k*y_k
//   L1      sum_k |x_k - y_k|
// so distances are bit-identical to the reference fallback and the top-k ids
// are bit-exact (ties ordered by id; the reference leaves ties unordered).
//
// Tiling: a 256-thread block owns 32 queries x 128 base rows per step; each
// lane keeps 4 queries x 4 rows = 16 independent sequential accumulators.
// Operand chunks of 32 dims are staged through LDS (144-B padded rows, lane
// reads with ds_read_b128 are conflict free). Base rows stream once per
// 32-query tile (24 flop/B). Per-query running top-k lives in LDS; candidates
// that beat the current k-th distance are appended to a per-query buffer and
// merged by one lane per query after each row tile.
#include <cfloat>

#include "common.hpp"
#include "kernels.hpp"
#include "graph.hpp"
#include "poincare_dev.hpp"
#include "scan.hpp"

namespace rvx {
namespace {

constexpr int TQ = 32, TR = 128, BKD = 32, ROWF = BKD + 4;

template <int METRIC>
__device__ __forceinline__ float pair_step(float acc, float q, float x) {
    if (METRIC == RVX_METRIC_L2) { const float d = q - x; return acc + d * d; }
    if (METRIC == RVX_METRIC_L1) return acc + fabsf(q - x);
    return acc + q * x;  // cosine / dot
}

template <int METRIC>
__device__ __forceinline__ float pair_finish(float acc, float qn, float xn, float curv = 1.0f) {
    // Poincaré: acc = |q-x|^2 in fused_norms' chunked order, qn/xn = squared
    // norms in the same order (norm_squared == fused_norms' own norm sums)
    if (METRIC == RVX_METRIC_POINCARE) return pdev::from_norms(acc, qn, xn, curv);
    if (METRIC == RVX_METRIC_L2) return sqrtf(acc);
    if (METRIC == RVX_METRIC_DOT) return -acc;
    if (METRIC == RVX_METRIC_COSINE) return (qn > 1e-8f && xn > 1e-8f) ? 1.0f - acc / (qn * xn) : 1.0f;
    return acc;
}

__device__ __forceinline__ bool better(float d, int64_t id, float bd, int64_t bid) {
    return d < bd || (d == bd && id < bid);
}

struct ScanArgs {
    const float* q; const float* x; const float* qnorm; const float* xnorm;
    int64_t nq, n; int d; int k;
    int64_t rows_per_chunk; int nchunks;
    float* part_d; int64_t* part_i;  // [nq][nchunks][k]
    int64_t id_offset;               // added to row index
    const uint8_t* deleted;          // optional tombstones [n]
    float curv;                      // Poincaré curvature
};

template <int METRIC>
__global__ __launch_bounds__(256) void k_scan_topk(ScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    float* qs = reinterpret_cast<float*>(lds_raw);                // [TQ][ROWF]
    float* xs = qs + TQ * ROWF;                                   // [TR][ROWF]
    float* best_d = xs + TR * ROWF;                               // [TQ][k]
    int64_t* best_i = reinterpret_cast<int64_t*>(best_d + TQ * a.k);  // [TQ][k]
    float* cand_d = reinterpret_cast<float*>(best_i + TQ * a.k);      // [TQ][TR]
    int32_t* cand_r = reinterpret_cast<int32_t*>(cand_d + TQ * TR);   // [TQ][TR]
    int32_t* cand_n = cand_r + TQ * TR;                               // [TQ]
    float* thr = reinterpret_cast<float*>(cand_n + TQ);               // [TQ]
    int32_t* filled = reinterpret_cast<int32_t*>(thr + TQ);           // [TQ]

    const int tid = threadIdx.x;
    const int tq = tid >> 5, tr = tid & 31;
    const int64_t q0 = (int64_t)blockIdx.x * TQ;
    const int chunk = blockIdx.y;
    const int64_t r_beg = (int64_t)chunk * a.rows_per_chunk;
    const int64_t r_end = min(a.n, r_beg + a.rows_per_chunk);
    const int K = a.k;

    for (int i = tid; i < TQ * K; i += 256) { best_d[i] = INFINITY; best_i[i] = INT64_MAX; }
    if (tid < TQ) { cand_n[tid] = 0; thr[tid] = INFINITY; filled[tid] = 0; }

    float qn[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t qi = q0 + tq + 8 * i;
        qn[i] = ((METRIC == RVX_METRIC_COSINE || METRIC == RVX_METRIC_POINCARE) && qi < a.nq) ? a.qnorm[qi] : 0.0f;
    }
    __syncthreads();

    for (int64_t rt = r_beg; rt < r_end; rt += TR) {
        float acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = 0.0f;

        for (int k0 = 0; k0 < a.d; k0 += BKD) {
            // stage queries: 32 rows x 32 floats = 256 float4 -> one per thread
            {
                const int row = tid >> 3, c = (tid & 7) * 4;
                const int64_t qi = q0 + row;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (qi < a.nq && k0 + c < a.d) v = *reinterpret_cast<const float4*>(a.q + qi * a.d + k0 + c);
                *reinterpret_cast<float4*>(qs + row * ROWF + c) = v;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {  // base rows: 128 x 32 floats = 1024 float4
                const int f = tid + 256 * i;
                const int row = f >> 3, c = (f & 7) * 4;
                const int64_t ri = rt + row;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (ri < r_end && k0 + c < a.d) v = *reinterpret_cast<const float4*>(a.x + ri * a.d + k0 + c);
                *reinterpret_cast<float4*>(xs + row * ROWF + c) = v;
            }
            __syncthreads();
            const int kc = min(BKD, a.d - k0);
            if (kc == BKD) {
#pragma unroll
                for (int kk = 0; kk < BKD; kk += 4) {
                    float4 qv[4], xv[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) qv[i] = *reinterpret_cast<const float4*>(qs + (tq + 8 * i) * ROWF + kk);
#pragma unroll
                    for (int j = 0; j < 4; ++j) xv[j] = *reinterpret_cast<const float4*>(xs + (tr + 32 * j) * ROWF + kk);
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if constexpr (METRIC == RVX_METRIC_POINCARE) {  // one 4-wide chunk of fused_norms
                                const float d0 = qv[i].x - xv[j].x, d1 = qv[i].y - xv[j].y;
                                const float d2 = qv[i].z - xv[j].z, d3 = qv[i].w - xv[j].w;
                                acc[i][j] = acc[i][j] + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
                            } else {
                                acc[i][j] = pair_step<METRIC>(acc[i][j], qv[i].x, xv[j].x);
                                acc[i][j] = pair_step<METRIC>(acc[i][j], qv[i].y, xv[j].y);
                                acc[i][j] = pair_step<METRIC>(acc[i][j], qv[i].z, xv[j].z);
                                acc[i][j] = pair_step<METRIC>(acc[i][j], qv[i].w, xv[j].w);
                            }
                        }
                }
            } else if (METRIC == RVX_METRIC_POINCARE) {  // tail tile: whole chunks, then a sequential remainder
                int kk = 0;
                for (; kk + 4 <= kc; kk += 4) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float* qp = qs + (tq + 8 * i) * ROWF + kk;
                            const float* xp = xs + (tr + 32 * j) * ROWF + kk;
                            const float d0 = qp[0] - xp[0], d1 = qp[1] - xp[1], d2 = qp[2] - xp[2], d3 = qp[3] - xp[3];
                            acc[i][j] = acc[i][j] + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
                        }
                }
                for (; kk < kc; ++kk) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            acc[i][j] = pair_step<RVX_METRIC_L2>(acc[i][j], qs[(tq + 8 * i) * ROWF + kk], xs[(tr + 32 * j) * ROWF + kk]);
                }
            } else {
                for (int kk = 0; kk < kc; ++kk) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            acc[i][j] = pair_step<METRIC>(acc[i][j], qs[(tq + 8 * i) * ROWF + kk], xs[(tr + 32 * j) * ROWF + kk]);
                }
            }
            __syncthreads();
        }

        // candidates that beat the running k-th distance of their query
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ql = tq + 8 * i;
            if (q0 + ql >= a.nq) continue;
            const float t = thr[ql];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t ri = rt + tr + 32 * j;
                if (ri >= r_end) continue;
                if (a.deleted && a.deleted[ri]) continue;
                const float xn = (METRIC == RVX_METRIC_COSINE || METRIC == RVX_METRIC_POINCARE) ? a.xnorm[ri] : 0.0f;
                const float dist = pair_finish<METRIC>(acc[i][j], qn[i], xn, a.curv);
                if (dist <= t) {  // ties at the threshold are resolved by id in the merge
                    const int slot = atomicAdd(&cand_n[ql], 1);
                    cand_d[ql * TR + slot] = dist;
                    cand_r[ql * TR + slot] = tr + 32 * j;
                }
            }
        }
        __syncthreads();
        if (tid < TQ) {  // one lane per query: insertion into the sorted top-k
            const int ql = tid;
            const int nc = cand_n[ql];
            float* bd = best_d + ql * K;
            int64_t* bi = best_i + ql * K;
            int fill = filled[ql];
            for (int c = 0; c < nc; ++c) {
                const float dd = cand_d[ql * TR + c];
                const int64_t id = rt + cand_r[ql * TR + c] + a.id_offset;
                if (fill == K && !better(dd, id, bd[K - 1], bi[K - 1])) continue;
                int p = (fill < K) ? fill : K - 1;
                while (p > 0 && better(dd, id, bd[p - 1], bi[p - 1])) { bd[p] = bd[p - 1]; bi[p] = bi[p - 1]; --p; }
                bd[p] = dd; bi[p] = id;
                if (fill < K) ++fill;
            }
            filled[ql] = fill;
            cand_n[ql] = 0;
            thr[ql] = (fill == K) ? bd[K - 1] : INFINITY;
        }
        __syncthreads();
    }

    for (int i = tid; i < TQ * K; i += 256) {
        const int ql = i / K, s = i % K;
        const int64_t qi = q0 + ql;
        if (qi >= a.nq) continue;
        const int64_t o = (qi * a.nchunks + chunk) * (int64_t)K + s;
        a.part_d[o] = best_d[i];
        a.part_i[o] = best_i[i];
    }
}

// One wave per query: k rounds of wave-wide (dist,id) argmin over the
// nchunks*k partial candidates.
__global__ __launch_bounds__(256) void k_merge_topk(const float* part_d, const int64_t* part_i, int64_t nq, int nchunks,
                                                   int k, float* out_d, int64_t* out_i) {
    const int lane = threadIdx.x & 63;
    const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= nq) return;
    const int total = nchunks * k;
    const float* pd = part_d + qi * total;
    const int64_t* pi = part_i + qi * total;
    float last_d = -INFINITY;
    int64_t last_i = INT64_MIN;
    for (int s = 0; s < k; ++s) {
        float bd = INFINITY;
        int64_t bi = INT64_MAX;
        for (int c = lane; c < total; c += 64) {
            const float d = pd[c];
            const int64_t id = pi[c];
            // strictly after the previous pick in (d, id) order
            const bool after = (d > last_d) || (d == last_d && id > last_i);
            if (after && better(d, id, bd, bi)) { bd = d; bi = id; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float od = __shfl_xor(bd, o);
            const int64_t oi = __shfl_xor(bi, o);
            if (better(od, oi, bd, bi)) { bd = od; bi = oi; }
        }
        if (lane == 0) { out_d[qi * k + s] = bd; out_i[qi * k + s] = bi; }
        last_d = bd;
        last_i = bi;
    }
}

// Sequential norms sqrt(sum x*x) in the reference order (distance.rs:56-57).
__global__ void k_row_norms(const float* x, int64_t n, int d, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* r = x + i * d;
    float s = 0.0f;
    for (int k = 0; k < d; ++k) s = s + r[k] * r[k];
    out[i] = sqrtf(s);
}

template <int METRIC>
__global__ void k_dist_matrix(const float* q, int64_t nq, const float* x, int64_t n, int d, const float* qn,
                              const float* xn, float* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nq * n) return;
    const int64_t i = idx / n, j = idx % n;
    float acc = 0.0f;
    for (int k = 0; k < d; ++k) acc = pair_step<METRIC>(acc, q[i * d + k], x[j * d + k]);
    out[idx] = pair_finish<METRIC>(acc, METRIC == RVX_METRIC_COSINE ? qn[i] : 0.f,
                                   METRIC == RVX_METRIC_COSINE ? xn[j] : 0.f);
}

template <int METRIC>
__global__ __launch_bounds__(256) void k_edge_dist(const float* x, const float* xn, const int64_t* rp, const int32_t* col,
                                                  int64_t n, int d, float* out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const float* a = x + row * d;
    for (int64_t p = rp[row] + lane; p < rp[row + 1]; p += 64) {
        const int64_t j = col[p];
        const float* b = x + j * d;
        float acc = 0.0f;
        for (int k = 0; k < d; ++k) acc = pair_step<METRIC>(acc, a[k], b[k]);
        out[p] = pair_finish<METRIC>(acc, METRIC == RVX_METRIC_COSINE ? xn[row] : 0.f,
                                     METRIC == RVX_METRIC_COSINE ? xn[j] : 0.f);
    }
}

size_t scan_lds_bytes(int k) {
    return (size_t)(TQ + TR) * ROWF * 4 + (size_t)TQ * k * 12 + (size_t)TQ * TR * 8 + TQ * 12;
}

}  // namespace

void row_norms(const float* x, int64_t n, int d, float* out) {
    if (n <= 0) return;
    ProfScope ps("row_norms");
    hipLaunchKernelGGL(k_row_norms, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream(), x, n, d, out);
    RVX_HIP(hipGetLastError());
}

__global__ void k_row_norm_sq(const float* x, int64_t n, int d, float* out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) out[r] = pdev::norm_sq(x + r * d, d);
}

void row_norm_sq(const float* x, int64_t n, int d, float* out) {
    if (n <= 0) return;
    RVX_LAUNCH("row_norm_sq", k_row_norm_sq, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, x, n, d, out);
}

void scan_topk(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
               const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
               const char* tag, float curv) {
    RVX_REQUIRE(k >= 1 && k <= SCAN_MAX_K, RVX_ERR_INVALID_PARAMETER,
                "k must be in [1, " + std::to_string(SCAN_MAX_K) + "]");
    RVX_REQUIRE(d % 4 == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)x & 15) == 0, RVX_ERR_UNSUPPORTED,
                "scan needs dim % 4 == 0 and 16-B aligned rows");
    if (nq <= 0) return;
    const int64_t qtiles = (nq + TQ - 1) / TQ;
    int64_t nchunks = (2048 + qtiles - 1) / qtiles;
    const int64_t max_chunks = std::max<int64_t>(1, (n + TR - 1) / TR);
    nchunks = std::min(std::max<int64_t>(nchunks, 1), std::min<int64_t>(max_chunks, 65535));
    int64_t rows_per_chunk = (n + nchunks - 1) / nchunks;
    rows_per_chunk = ((rows_per_chunk + TR - 1) / TR) * TR;
    nchunks = std::max<int64_t>(1, (n + rows_per_chunk - 1) / rows_per_chunk);

    float* part_d = (float*)scratch_bytes("scan_part_d", nq * nchunks * k * 4);
    int64_t* part_i = (int64_t*)scratch_bytes("scan_part_i", nq * nchunks * k * 8);
    ScanArgs a{q, x, qnorm, xnorm, nq, n, d, k, rows_per_chunk, (int)nchunks, part_d, part_i, id_offset, deleted, curv};
    const size_t lds = scan_lds_bytes(k);
    static bool attr_done = false;
    if (!attr_done) {
        hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_COSINE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_DOT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_L1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_POINCARE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    const dim3 grid((unsigned)qtiles, (unsigned)nchunks);
    const char* t = tag ? tag : "scan_topk";
    switch (metric) {
        case RVX_METRIC_L2: RVX_LAUNCH(t, k_scan_topk<RVX_METRIC_L2>, grid, dim3(256), lds, a); break;
        case RVX_METRIC_COSINE: RVX_LAUNCH(t, k_scan_topk<RVX_METRIC_COSINE>, grid, dim3(256), lds, a); break;
        case RVX_METRIC_DOT: RVX_LAUNCH(t, k_scan_topk<RVX_METRIC_DOT>, grid, dim3(256), lds, a); break;
        case RVX_METRIC_L1: RVX_LAUNCH(t, k_scan_topk<RVX_METRIC_L1>, grid, dim3(256), lds, a); break;
        case RVX_METRIC_POINCARE: RVX_LAUNCH(t, k_scan_topk<RVX_METRIC_POINCARE>, grid, dim3(256), lds, a); break;
        default: fail(RVX_ERR_UNSUPPORTED, "metric not supported by the flat scan");
    }
    RVX_LAUNCH("scan_merge", k_merge_topk, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, part_d, part_i, nq,
               (int)nchunks, k, out_d, out_i);
}

void merge_topk(const float* part_d, const int64_t* part_i, int64_t nq, int nchunks, int k, float* out_d,
                int64_t* out_i) {
    if (nq <= 0) return;
    RVX_LAUNCH("scan_merge", k_merge_topk, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, part_d, part_i, nq, nchunks, k,
               out_d, out_i);
}

void edge_distances(int metric, const float* x, const float* xn, const int64_t* rp, const int32_t* col, int64_t n,
                    int d, float* out) {
    if (n <= 0) return;
    const dim3 grid((unsigned)((n + 3) / 4));
    ProfScope ps("edge_distances");
    switch (metric) {
        case RVX_METRIC_L2: hipLaunchKernelGGL(k_edge_dist<RVX_METRIC_L2>, grid, dim3(256), 0, stream(), x, xn, rp, col, n, d, out); break;
        case RVX_METRIC_COSINE: hipLaunchKernelGGL(k_edge_dist<RVX_METRIC_COSINE>, grid, dim3(256), 0, stream(), x, xn, rp, col, n, d, out); break;
        case RVX_METRIC_DOT: hipLaunchKernelGGL(k_edge_dist<RVX_METRIC_DOT>, grid, dim3(256), 0, stream(), x, xn, rp, col, n, d, out); break;
        case RVX_METRIC_L1: hipLaunchKernelGGL(k_edge_dist<RVX_METRIC_L1>, grid, dim3(256), 0, stream(), x, xn, rp, col, n, d, out); break;
        default: fail(RVX_ERR_UNSUPPORTED, "metric not supported");
    }
    RVX_HIP(hipGetLastError());
}

void distance_matrix(int metric, const float* q, const float* qn, int64_t nq, const float* x, const float* xn, int64_t n,
                     int d, float* out) {
    const int64_t total = nq * n;
    if (total <= 0) return;
    const dim3 grid((unsigned)((total + 255) / 256));
    ProfScope ps("distance_matrix");
    switch (metric) {
        case RVX_METRIC_L2: hipLaunchKernelGGL(k_dist_matrix<RVX_METRIC_L2>, grid, dim3(256), 0, stream(), q, nq, x, n, d, qn, xn, out); break;
        case RVX_METRIC_COSINE: hipLaunchKernelGGL(k_dist_matrix<RVX_METRIC_COSINE>, grid, dim3(256), 0, stream(), q, nq, x, n, d, qn, xn, out); break;
        case RVX_METRIC_DOT: hipLaunchKernelGGL(k_dist_matrix<RVX_METRIC_DOT>, grid, dim3(256), 0, stream(), q, nq, x, n, d, qn, xn, out); break;
        case RVX_METRIC_L1: hipLaunchKernelGGL(k_dist_matrix<RVX_METRIC_L1>, grid, dim3(256), 0, stream(), q, nq, x, n, d, qn, xn, out); break;
        default: fail(RVX_ERR_UNSUPPORTED, "metric not supported");
    }
    RVX_HIP(hipGetLastError());
}

}  // namespace rvx
