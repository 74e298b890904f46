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
#include <type_traits>
#ifdef RVX_SCAN_CLOCK
#include <algorithm>
#include <cstdio>
#include <vector>
#endif

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
    if (METRIC == RVX_METRIC_L2 || METRIC == METRIC_L2SQ) { const float d = q - x; return acc + d * d; }
    if (METRIC == RVX_METRIC_L1) return acc + fabsf(q - x);
    return acc + q * x;  // cosine / dot
}

template <int METRIC>
__device__ __forceinline__ float pair_finish(float acc, float qn, float xn, float curv = 1.0f) {
    // Poincaré: acc = |q-x|^2 in fused_norms' chunked order, qn/xn = squared
    // norms in the same order (norm_squared == fused_norms' own norm sums)
    if (METRIC == RVX_METRIC_POINCARE) return pdev::from_norms(acc, qn, xn, curv);
    if (METRIC == RVX_METRIC_HYP_L2) return sqrtf(acc);  // fused_norms' chunked |q-x|^2
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
    float* full;                     // FULL: distances [nq][full_ld] (deleted rows NaN)
    int64_t full_ld;
};

// FULL = false: the fused top-k (k <= SCAN_MAX_K). FULL = true: the same tiles write every
// (query, row) distance to a.full for the any-k selection (k_select.hip).
template <int METRIC, bool FULL = false>
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
                            if constexpr (METRIC == RVX_METRIC_POINCARE || METRIC == RVX_METRIC_HYP_L2) {  // one 4-wide chunk of fused_norms
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
            } else if (METRIC == RVX_METRIC_POINCARE || METRIC == RVX_METRIC_HYP_L2) {  // tail tile: whole chunks, then a sequential remainder
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

        if constexpr (FULL) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t qi = q0 + tq + 8 * i;
                if (qi >= a.nq) continue;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t ri = rt + tr + 32 * j;
                    if (ri >= r_end) continue;
                    const float xn = (METRIC == RVX_METRIC_COSINE || METRIC == RVX_METRIC_POINCARE) ? a.xnorm[ri] : 0.0f;
                    const float dist = (a.deleted && a.deleted[ri]) ? __builtin_nanf("")
                                                                    : pair_finish<METRIC>(acc[i][j], qn[i], xn, a.curv);
                    a.full[qi * a.full_ld + ri] = dist;
                }
            }
            continue;  // uniform: FULL is a template parameter
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

    if constexpr (FULL) return;
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

// ---------------------------------------------------------------------------
// MFMA-filtered exact scan (L2 / cosine / dot, large query batches).
//
// The scan above is VALU-bound (three exact f32 ops per dimension per pair).
// For a batch of queries the (query, row) dot products are a GEMM, so this
// path ranks rows with f16 MFMA and computes REFERENCE distances only for the
// few rows that can still be in the top-k:
//   1. rows and queries are scaled by a power of two (exact) so the row max
//      lands in [2^14, 2^15) and rounded to f16 (k_rows_to_f16);
//   2. k_scan_filter: v_mfma_f32_32x32x16_f16 dot products over 256 x 256 (or
//      128 x 128) row x query tiles, the approximate value v (L2: |x|^2 - 2 x.q,
//      squared units shifted by |q|^2; cosine / dot as the reference forms), a
//      running per-(query, row split) list of the FKP smallest v in LDS, and a
//      per-query bound shared by all splits (k-th listed value + 2 eps, min over
//      splits) above which no value is admitted;
//   3. k_scan_rerank (one wave per query): D = k-th smallest v + 2 eps_q, where
//      eps_q bounds |v - reference value| for every row (f16 rounding 2^-11 per
//      operand, f32 accumulation, the reference's own f32 sum; 2x slack). Every
//      row whose reference value is <= the k-th reference value has v <= D, so
//      the candidates {v <= D} hold the exact top-k unless a split's list was
//      full below D (then the query is re-run on the exact VALU scan). The
//      candidates' distances are recomputed with the reference arithmetic
//      (pair_step / pair_finish, same bits as k_scan_topk) and the top-k is
//      taken in (distance, id) order: results are identical to k_scan_topk.
// Inputs that are non-finite or outside 2^+-60 (where the scaled products could
// leave f32 range) send the whole call to the VALU scan.
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifndef RVX_SCAN_FKP
#define RVX_SCAN_FKP 16
#define RVX_SCAN_FCB 8
#define RVX_SCAN_NSTAGE 3
#endif
constexpr int FK = 32;                      // K per stage
constexpr int FKP = RVX_SCAN_FKP;           // list length per (query, split)
constexpr int FCB = RVX_SCAN_FCB;           // candidate slots per query per merge round
constexpr int F_NSTAGE = RVX_SCAN_NSTAGE;   // LDS-DMA ring: F_NSTAGE - 1 k-steps in flight across the barrier
// Tile shapes. Waves 2 (rows) x WQ (queries); each wave FM x 2 accumulators of
// 32 x 32 (rows x queries). Each wave DMAs RP row pieces and QP query pieces (16
// rows x 64 B each) per k-step.
//   1 (wide): 256 x 256, 8 waves, one block per CU (149 KB LDS) — half the L2->LDS
//         bytes per MFMA; taken for d >= 512 (10M x 768: 78.6 -> 64.3 ms per launch)
//   0: 128 x 128, 4 waves, two blocks per CU (74.5 KB) — shorter tile
//         epilogues for short rows (100k x 128: 3.8 vs 5.7 ms)
//   2 (tall): 256 rows x 128 queries, 4 waves of the wide tile's 128 x 64 shape, a
//         2-stage ring, two blocks per CU (79.5 KB): each block's tile epilogue and
//         barriers can run beside the other block's MFMAs (opt-in, RVX_SCAN_WIDE=2)
//   3 (wide, 16x16x32): the wide tile with v_mfma_f32_16x16x32_f16 — the same cycles per
//         flop and LDS bytes, 8 x 4 accumulators of 16 x 16 per wave; the chip holds a
//         higher clock under the smaller MFMA shape (MI355X_MICROARCH.md, DVFS item 7)
template <int C>
struct FCfg {
    static constexpr bool M16 = C == 3;
    static constexpr int WQ = (C == 1 || C == 3) ? 4 : 2, FM = C == 0 ? 2 : 4;
    static constexpr int THREADS = 64 * 2 * WQ, NW = THREADS / 64;
    static constexpr int FQ = 64 * WQ, FR = 64 * FM;
    static constexpr int NST = C == 2 ? 2 : F_NSTAGE;  // LDS-DMA ring stages
    static constexpr int RP = FR / 16 / NW, QP = FQ / 16 / NW;  // DMA pieces per wave and k-step
    static constexpr int STAGE = (FR + FQ) * FK * 2;  // f16 rows then f16 queries, 64 B per row
    // + row constants (float4) and per-query {Qs, P} of the per-row-bound metrics
    // + per-query shared bound B_q and eps_q (group insertion, RVX_SCAN_GROUP_INSERT)
    static constexpr int LDS = NST * STAGE + FQ * FKP * 8 + FQ * FCB * 8 + FQ * 12 + 16 + FR * 16 + FQ * 8 + FQ * 8;
    static constexpr int BLOCKS = (C == 1 || C == 3) ? 1 : 2;
    static_assert(RP * 16 * NW == FR && QP * 16 * NW == FQ && RP >= QP, "DMA pieces cover the stage");
    static_assert(BLOCKS * LDS <= 160 * 1024, "resident blocks fit the CU's LDS");
};
constexpr int F_MAXE = 32;                  // rerank: list entries per lane (nsplit_total * FKP <= 64 * F_MAXE)

struct FilterArgs {
    // per-row constants {1/scale (NaN for a deleted row), |x|^2 (L2, dot) or the
    // reference norm (cosine)}; xh / xc are chunk rows indexed from row0
    const _Float16* xh; const float2* xc;
    const _Float16* qh; const float2* qc;
    int64_t nq, row0, row_end; int d;
    int64_t rows_per_split; int split0, qtiles, nsplit_total;
    float* part_v; int32_t* part_r;  // [nq][nsplit_total][FKP]
    // shared rejection bound per query (order-encoded float, see below), the
    // result count k and max_x |x|^2 over ALL rows (for eps, as the rerank)
    unsigned* gbound; int k; const unsigned* xsq_max_bits;
    // per-row-bound metrics (Poincaré, squared L2): row factors {R, C, S, N} and beta
    const float4* xc4; float beta;
    // diagnostic build only (-DRVX_SCAN_CLOCK): per block {delta s_memtime, delta s_memrealtime}
    // over the block's life; null and unused in the real kernel
    unsigned long long* clk;
};

// Order-preserving float <-> uint (atomicMin over possibly negative values).
__device__ __forceinline__ unsigned ord_enc(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_dec(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
// Smallest float above f (f itself for +INF / NaN): v < next_up(B) <=> v <= B.
__device__ __forceinline__ float next_up(float f) {
    if (!(f < INFINITY)) return f;
    if (f == 0.0f) return __uint_as_float(1u);
    const unsigned u = __float_as_uint(f);
    return __uint_as_float((u & 0x80000000u) ? u - 1u : u + 1u);
}

// eps_q: bound on |v - reference value| for every row (f16 rounding 2^-11 per
// operand, f32 accumulation, the reference's own f32 sum; 2x slack), shared by
// the filter's rejection bound and the rerank so both compute the same bits.
template <int METRIC>
__device__ __forceinline__ float filter_eps(float qs, float xs_max) {
    if (METRIC == RVX_METRIC_COSINE) return 0x1p-8f + 0x1p-12f;
    const float qx = sqrtf(qs) * sqrtf(xs_max);
    return (METRIC == RVX_METRIC_L2) ? 0x1p-8f * qx + 0x1p-12f * (qs + xs_max) : (0x1p-8f + 0x1p-12f) * qx;
}

// The filter ranks by v = C_row + (acc * R_row) * Q_query, one multiply and one
// FMA per (row, query) value (acc * R and the product with Q only move powers of
// two for L2 / dot, so the only rounding is the FMA's):
//   L2      R = 1/t_x, C = |x|^2, Q = -2/t_q      v = |x|^2 - 2 x.q (|q|^2 left out:
//           a per-query shift, so lists, thresholds and the rerank's D = v_k + 2 eps
//           stay consistent in the shifted units)
//   dot     R = 1/t_x, C = 0,     Q = -1/t_q      v = -x.q
//   cosine  R = 1/(t_x |x|), C = 1, Q = -1/(t_q |q|)   v = 1 - x.q/(|x||q|); a norm
//           <= 1e-8 zeroes its factor (v = 1, distance.rs:58-62)
// A deleted row (1/t_x = NaN) and a padding query (1/t_q = NaN) give v = NaN.
template <int METRIC>
__device__ __forceinline__ float2 row_factors(float2 pre) {  // {R, C} from {1/t_x, |x|^2 or |x|}
    if (METRIC == RVX_METRIC_L2) return pre;
    if (METRIC == RVX_METRIC_DOT) return make_float2(pre.x, 0.0f);
    return make_float2(pre.y > 1e-8f ? pre.x / pre.y : 0.0f * pre.x, 1.0f);
}
template <int METRIC>
__device__ __forceinline__ float query_factor(float qinv, float qn) {
    if (METRIC == RVX_METRIC_L2) return -2.0f * qinv;
    if (METRIC == RVX_METRIC_DOT) return -qinv;
    return qn > 1e-8f ? -(qinv / qn) : 0.0f * qinv;
}

__device__ __forceinline__ bool lt_vr(float v, int r, float bv, int br) { return v < bv || (v == bv && r < br); }

template <int METRIC, int CFG, bool GROUP>
__global__ __launch_bounds__(FCfg<CFG>::THREADS, FCfg<CFG>::BLOCKS) void k_scan_filter(FilterArgs a) {
    using Cf = FCfg<CFG>;
    constexpr int FQ = Cf::FQ, FR = Cf::FR, F_STAGE = Cf::STAGE, F_FM = Cf::FM, F_THREADS = Cf::THREADS;
    constexpr int NST = Cf::NST, RP = Cf::RP, QP = Cf::QP, PCS = RP + QP;
    // accumulator geometry: AM x AN tiles of TT x TT per wave, AE values per lane each
    constexpr bool M16 = Cf::M16;
    constexpr int AM = M16 ? 2 * F_FM : F_FM, AN = M16 ? 4 : 2, AE = M16 ? 4 : 16, TT = M16 ? 16 : 32;
    using AccT = typename std::conditional<M16, f32x4v, f32x16>::type;
    using OffT = typename std::conditional<M16, uint32_t, uint64_t>::type;
    // per-row bounds (Poincaré, squared L2; see rows_to_f16_pr): the lists rank lower bounds
    constexpr bool PRB = METRIC == RVX_METRIC_POINCARE || METRIC == METRIC_L2SQ;
    extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
    float* best_v = reinterpret_cast<float*>(fsm + NST * F_STAGE);  // [FQ][FKP] ascending (v, row)
    int32_t* best_r = reinterpret_cast<int32_t*>(best_v + FQ * FKP);
    float* cand_v = reinterpret_cast<float*>(best_r + FQ * FKP);  // [FQ][FCB]
    int32_t* cand_r = reinterpret_cast<int32_t*>(cand_v + FQ * FCB);
    int32_t* cand_n = cand_r + FQ * FCB;                            // [FQ]
    float* thr = reinterpret_cast<float*>(cand_n + FQ);             // [FQ] list's FKP-th v (INF until full)
    int32_t* fillc = reinterpret_cast<int32_t*>(thr + FQ);          // [FQ]
    int32_t* ovf = fillc + FQ;  // [0..1] candidate-slot overflow per round, [2..3] tile vote per tile parity

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef RVX_SCAN_CLOCK  // MI355X_MICROARCH.md DVFS item 6: clock = d(s_memtime) / d(s_memrealtime) x 100 MHz
    const unsigned long long clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef RVX_SCAN_PRIO  // experiment: static priority for the second-dispatched half of the waves
    if (wave >= Cf::NW / 2) __builtin_amdgcn_s_setprio(1);
#endif
    const int lr = lane & 31, lh = lane >> 5, wm = wave & 1, wn = wave >> 1;
    const int lc = lane & 15, lg = lane >> 4;  // 16x16x32 lane roles: query / row-group
    const int lq = M16 ? lc : lr;              // the lane's query column inside an accumulator tile
    // consecutive blocks share a row split (and, 8 at a time, an XCD's L2)
    const int qt = (int)(blockIdx.x % (unsigned)a.qtiles);
    const int sl = (int)(blockIdx.x / (unsigned)a.qtiles);
    const int64_t q0 = (int64_t)qt * FQ;
    const int64_t r_beg = a.row0 + (int64_t)sl * a.rows_per_split;
    const int64_t r_end = min(a.row_end, r_beg + a.rows_per_split);

    float2* rowc = reinterpret_cast<float2*>(ovf + 4);              // [FR] current tile's row constants
    float4* rowc4 = reinterpret_cast<float4*>(ovf + 4);             // [FR] (per-row-bound metrics)
    float2* qfac = reinterpret_cast<float2*>(rowc4 + FR);           // [FQ] {Qs, P} (per-row-bound metrics)
    float* gbl = reinterpret_cast<float*>(qfac + FQ);               // [FQ] B_q as this block knows it
    float* gepsl = gbl + FQ;                                        // [FQ] eps_q

    for (int i = tid; i < FQ * FKP; i += F_THREADS) { best_v[i] = INFINITY; best_r[i] = -1; }
    if (tid < FQ) { cand_n[tid] = 0; thr[tid] = INFINITY; fillc[tid] = 0; }
    if (tid < 4) ovf[tid] = 0;

    float qf_[AN];  // query factor Q
    bool qv_[AN];
#pragma unroll
    for (int fn = 0; fn < AN; ++fn) {
        const int64_t qg = q0 + wn * 64 + fn * TT + lq;
        qv_[fn] = qg < a.nq;
        const int64_t qc = min(qg, a.nq - 1);
        const float2 c = a.qc[qc];
        if constexpr (PRB) qf_[fn] = -2.0f * (qv_[fn] ? c.x : __builtin_nanf(""));
        else qf_[fn] = query_factor<METRIC>(qv_[fn] ? c.x : __builtin_nanf(""), c.y);  // padding query: NaN
    }
    if constexpr (PRB) {
        // L = S*|q|^2*(1-beta) + (acc*R)*Q + C + N*P, P = -1.5 2^-9 |q| (the f16 term of the bound)
        if (tid < FQ) {
            const float2 c = a.qc[min<int64_t>(q0 + tid, a.nq - 1)];
            qfac[tid] = make_float2(c.y * (1.0f - a.beta), -0x1.8p-9f * sqrtf(c.y));
        }
    }
    // Shared rejection bound (lanes tid < FQ, one query each). A split's list
    // holding k entries proves v_k <= its k-th value, so B_q = min over splits
    // of (k-th value + 2 eps_q) is >= the rerank's D = v_k + 2 eps_q (same
    // arithmetic, rounding is monotone): a value above B_q is never a
    // candidate. Blocks publish with atomicMin and re-read B_q once per tile,
    // so every split stops admitting what the others have already beaten.
    const int64_t gq_idx = min<int64_t>(q0 + tid, a.nq - 1);
    const bool gq_own = tid < FQ && q0 + tid < a.nq;
    float geps = 0.0f, gb = INFINITY;
    unsigned graw = 0xFF800000u;  // last B_q read (ord_enc(+INF)); folded into gb at the next epilogue
    if (gq_own) {
        geps = filter_eps<METRIC>(a.qc[gq_idx].y, __uint_as_float(*a.xsq_max_bits));
        gb = ord_dec(__hip_atomic_load(a.gbound + gq_idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    if (tid < FQ) {  // LDS copies for the group insertion (whichever lanes insert a query's offers)
        gbl[tid] = gb;
        gepsl[tid] = geps;
    }

    // LDS-DMA fill: 1 KB pieces of 16 rows x 64 B; lane -> (row, 16-B chunk)
    // with the chunk XOR-swizzled by (row >> 2) & 3 on the source address, so
    // the fragment reads below are bank-conflict free.
    // swizzle of a row's four 16-B chunks by g = (row >> 2) & 3: g for the 32x32x16 reads;
    // (4 - g) & 3 for the 16x16x32 reads (lane (lc, lg) reads row lc, chunk lg), which keeps
    // each of ds_read_b128's four 16-lane bank groups on 16 distinct 4-bank quads
    auto swz = [](int g) { return M16 ? ((4 - g) & 3) : g; };
    int prow[RP], pchunk[RP], qrow[QP], qchunk[QP];
#pragma unroll
    for (int j = 0; j < RP; ++j) {
        prow[j] = 16 * (RP * wave + j) + (lane >> 2);
        pchunk[j] = (lane & 3) ^ swz((prow[j] >> 2) & 3);
    }
#pragma unroll
    for (int j = 0; j < QP; ++j) {
        qrow[j] = 16 * (QP * wave + j) + (lane >> 2);
        qchunk[j] = (lane & 3) ^ swz((qrow[j] >> 2) & 3);
    }
    const int nk = a.d / FK;
    const int64_t ntile = r_end > r_beg ? (r_end - r_beg + FR - 1) / FR : 0;
    const int64_t iters = ntile * nk;
    // DMA sources as a wave-uniform base plus 32-bit per-lane offsets (rows past
    // the end clamp to the last row), so a k-step's fill is address-add free:
    // SGPR base + k, VGPR offset (the tile offsets change once per tile)
    const char* qbase = reinterpret_cast<const char*>(a.qh + q0 * a.d);
    uint32_t qoff[QP];
#pragma unroll
    for (int j = 0; j < QP; ++j)
        qoff[j] = (uint32_t)(((int64_t)min<int64_t>(qrow[j], a.nq - 1 - q0) * a.d + qchunk[j] * 8) * 2);
    struct TileSrc { const char* base; uint32_t off[RP]; };
    auto tile_src = [&](int64_t t) {  // t = first row of a tile in [r_beg, r_end)
        TileSrc ts;
        ts.base = reinterpret_cast<const char*>(a.xh + (t - a.row0) * a.d);
#pragma unroll
        for (int j = 0; j < RP; ++j)
            ts.off[j] = (uint32_t)(((int64_t)min<int64_t>(prow[j], r_end - 1 - t) * a.d + pchunk[j] * 8) * 2);
        return ts;
    };
    // DMA piece j of a k-step: rows and queries alternate while both last, then rows
#ifndef RVX_SCAN_ROW_CPOL
#define RVX_SCAN_ROW_CPOL 0
#define RVX_SCAN_QRY_CPOL 0
#endif
    auto dma_piece = [&](const TileSrc& ts, int k0, unsigned char* dst, int j) {
        const bool qry = j < 2 * QP && (j & 1);
        const int h = j < 2 * QP ? j >> 1 : j - QP;
        if (qry)
            __builtin_amdgcn_global_load_lds((const void*)(qbase + k0 * 2 + qoff[h]),
                                             (__attribute__((address_space(3))) void*)(dst + FR * 64 +
                                                                                      (QP * wave + h) * 1024),
                                             16, 0, RVX_SCAN_QRY_CPOL);
        else
            __builtin_amdgcn_global_load_lds((const void*)(ts.base + k0 * 2 + ts.off[h]),
                                             (__attribute__((address_space(3))) void*)(dst + (RP * wave + h) * 1024),
                                             16, 0, RVX_SCAN_ROW_CPOL);
    };
    auto fill = [&](const TileSrc& ts, int k0, unsigned char* dst) {
#pragma unroll
        for (int j = 0; j < PCS; ++j) dma_piece(ts, k0, dst, j);
    };
    constexpr int WROWS = 32 * F_FM;  // rows per wave
    // LDS read offsets of fragment 0 per k-half; the XOR swizzle depends on
    // (row >> 2) & 3 = (lr >> 2) & 3 only (fragment rows differ by multiples of
    // 32), so fragment f sits f * 2 KiB further: an immediate offset, not a VGPR
    int a_rd[2], b_rd[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        if constexpr (M16) {  // one K = 32 step: row lc, chunk lg (fragments 16 rows = 1 KiB apart)
            const int sw = (lg ^ swz((lc >> 2) & 3)) << 4;
            a_rd[ks] = (wm * WROWS + lc) * 64 + sw;
            b_rd[ks] = FR * 64 + (wn * 64 + lc) * 64 + sw;
        } else {
            const int sw = ((2 * ks + lh) ^ ((lr >> 2) & 3)) << 4;
            a_rd[ks] = (wm * WROWS + lr) * 64 + sw;
            b_rd[ks] = FR * 64 + (wn * 64 + lr) * 64 + sw;
        }
    }

    AccT acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int e = 0; e < AE; ++e) acc[i][j][e] = 0.0f;

    // Tile epilogue. The accumulators are overwritten in place by the
    // approximate values v; invalid rows (past the split, deleted: 1/scale =
    // NaN) and padding queries (Q = NaN) give v = NaN, which no threshold test
    // admits. When no value of the tile is below its query's list threshold
    // (the common case once the lists are full) the tile costs its values, a
    // running min and one block-wide vote. Otherwise every value below the
    // threshold is offered: one compare whose lane mask is the uniform branch
    // condition; offered values are marked in a per-lane bit mask; slots per
    // query per round are bounded (FCB), so rounds repeat with the tightened
    // thresholds until no offer overflowed (thresholds only fall, so a
    // rejection is final and needs no mark).
    auto epilogue = [&](int64_t rt, float4 pre) {
        if (tid < FQ) {  // B_q read at the end of the last tile: its wait lands on the drain below
            gb = fminf(gbl[tid], ord_dec(graw));
            gbl[tid] = gb;
            thr[tid] = fminf(thr[tid], next_up(gb));  // admit v <= B_q
        }
        if (tid < FR) {
            if constexpr (PRB) rowc4[tid] = pre;
            else rowc[tid] = row_factors<METRIC>(make_float2(pre.x, pre.y));
        }
        __syncthreads();
        float vmin[AN];
#pragma unroll
        for (int fn = 0; fn < AN; ++fn) vmin[fn] = INFINITY;
        if constexpr (PRB && M16) {
            float2 qsp[AN];
#pragma unroll
            for (int fn = 0; fn < AN; ++fn) qsp[fn] = qfac[wn * 64 + fn * TT + lq];
            // the lane's 4 values of a 16 x 16 tile are 4 consecutive rows: four float4 reads
#pragma unroll
            for (int fm = 0; fm < AM; ++fm) {
                float4 cr[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) cr[w] = rowc4[wm * WROWS + fm * 16 + 4 * lg + w];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float4 c = cr[e];
#pragma unroll
                    for (int fn = 0; fn < AN; ++fn) {
                        const float v = __builtin_fmaf(
                            c.w, qsp[fn].y,
                            __builtin_fmaf(c.z, qsp[fn].x, __builtin_fmaf(acc[fm][fn][e] * c.x, qf_[fn], c.y)));
                        acc[fm][fn][e] = v;
                        vmin[fn] = fminf(vmin[fn], v);
                    }
                }
            }
        } else if constexpr (PRB) {
            float2 qsp[2];
#pragma unroll
            for (int fn = 0; fn < 2; ++fn) qsp[fn] = qfac[wn * 64 + fn * 32 + lr];
            // rows (e & 3) of a run are consecutive: four float4 reads issued together per run
#pragma unroll
            for (int fm = 0; fm < F_FM; ++fm)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float4 cr[4];
#pragma unroll
                    for (int w = 0; w < 4; ++w) cr[w] = rowc4[wm * WROWS + fm * 32 + w + 8 * g + 4 * lh];
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const int e = 4 * g + w;
                        const float4 c = cr[w];
#pragma unroll
                        for (int fn = 0; fn < 2; ++fn) {
                            const float v = __builtin_fmaf(
                                c.w, qsp[fn].y,
                                __builtin_fmaf(c.z, qsp[fn].x, __builtin_fmaf(acc[fm][fn][e] * c.x, qf_[fn], c.y)));
                            acc[fm][fn][e] = v;
                            vmin[fn] = fminf(vmin[fn], v);
                        }
                    }
                }
        } else if constexpr (M16) {
            // 4 consecutive rows per lane and tile: two float4 reads (two rows' {R, C} each)
            const float4* rc4 = reinterpret_cast<const float4*>(rowc);
#pragma unroll
            for (int fm = 0; fm < AM; ++fm) {
                const int rbase = (wm * WROWS + fm * 16 + 4 * lg) >> 1;
                const float4 cc[2] = {rc4[rbase], rc4[rbase + 1]};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float4 q = cc[e >> 1];
                    const float2 c = (e & 1) ? make_float2(q.z, q.w) : make_float2(q.x, q.y);
#pragma unroll
                    for (int fn = 0; fn < AN; ++fn) {
                        const float v = __builtin_fmaf(acc[fm][fn][e] * c.x, qf_[fn], c.y);
                        acc[fm][fn][e] = v;
                        vmin[fn] = fminf(vmin[fn], v);
                    }
                }
            }
        } else {
            // the 16 rows of a 32-row block that one lane holds are 4 runs of 4 consecutive
            // rows: 8 ds_read_b128 (two rows' {C, R} each) issued together per block, instead
            // of 16 dependent 8-byte reads the compiler waited on one by one
            const float4* rc4 = reinterpret_cast<const float4*>(rowc);
#pragma unroll
            for (int fm = 0; fm < F_FM; ++fm) {
                const int rbase = (wm * WROWS + fm * 32 + 4 * lh) >> 1;  // even row: a float4 holds rows 2i, 2i+1
                float4 cc[8];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    cc[2 * g] = rc4[rbase + 4 * g];
                    cc[2 * g + 1] = rc4[rbase + 4 * g + 1];
                }
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const float4 q = cc[2 * (e >> 2) + ((e & 3) >> 1)];
                    const float2 c = (e & 1) ? make_float2(q.z, q.w) : make_float2(q.x, q.y);
#pragma unroll
                    for (int fn = 0; fn < 2; ++fn) {
                        const float v = __builtin_fmaf(acc[fm][fn][e] * c.x, qf_[fn], c.y);
                        acc[fm][fn][e] = v;
                        vmin[fn] = fminf(vmin[fn], v);  // NaN-ignoring: an all-NaN lane stays NaN
                    }
                }
            }
        }
        // Fast path: no value of the tile is below its query's threshold -> one
        // compare per query, no offers (with 256 queries per tile most tiles still
        // admit something).
        bool any = false;
#pragma unroll
        for (int fn = 0; fn < AN; ++fn) any = any || vmin[fn] < thr[wn * 64 + fn * TT + lq];
        // block vote: one flag per tile parity, one LDS barrier (no VMEM drain)
        const int vp = 2 + (int)(((rt - r_beg) / FR) & 1);
        if (__ballot(any) && lane == 0) ovf[vp] = 1;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const bool slow = ovf[vp] != 0;
        if (tid == 0) ovf[vp ^ 1] = 0;  // every wave has read the other parity's flag (last tile)
        if (!slow) return;
#ifdef RVX_COUNT_SLOW
        if (tid == 0) atomicAdd((unsigned*)a.xsq_max_bits + 2, 1u);
#endif
        static_assert(AM * AE <= 8 * (int)sizeof(OffT), "offered-value mask holds one bit per (fm, e)");
        OffT offered[AN];  // per fn: values already handed to the list
#pragma unroll
        for (int fn = 0; fn < AN; ++fn) offered[fn] = 0;
        for (int round = 0;; ++round) {
#pragma unroll
            for (int fn = 0; fn < AN; ++fn) {
                const int ql = wn * 64 + fn * TT + lq;
                const float t = thr[ql];
                if (!__ballot(vmin[fn] < t)) continue;  // none of the wave's queries has a value below its threshold
#pragma unroll
                for (int fm = 0; fm < AM; ++fm) {
#ifdef RVX_SCAN_FMSKIP  // experiment: one wave vote per accumulator tile before its per-value votes
                    {
                        bool anyf = false;
#pragma unroll
                        for (int e = 0; e < AE; ++e)
                            anyf = anyf || (acc[fm][fn][e] < t && !(offered[fn] & ((OffT)1 << (fm * AE + e))));
                        if (!__ballot(anyf)) continue;
                    }
#endif
#pragma unroll
                    for (int e = 0; e < AE; ++e) {
                        const float v = acc[fm][fn][e];
                        const OffT bit = (OffT)1 << (fm * AE + e);
                        const bool pass = v < t && !(offered[fn] & bit);
                        if (!__ballot(pass)) continue;
                        if (!pass) continue;
                        const int slot = atomicAdd(&cand_n[ql], 1);
                        if (slot < FCB) {
                            cand_v[ql * FCB + slot] = v;
                            cand_r[ql * FCB + slot] = (int32_t)(rt + wm * WROWS + fm * TT +
                                                                (M16 ? 4 * lg + e : (e & 3) + 8 * (e >> 2) + 4 * lh));
                            offered[fn] |= bit;
                        } else {
                            ovf[round & 1] = 1;
                        }
                    }
                }
            }
            __syncthreads();
            // Insertion of this round's offers into the sorted lists (a query with no
            // offer keeps its list, threshold and published bound). A 16-lane group
            // holds one query's list in registers, lane j = slot j: per offer one
            // ballot gives its rank, one shuffle shifts the tail — no dependent LDS
            // round trips; the groups of all waves take the queries in turn.
            if constexpr (!GROUP) {
            if (tid < FQ && cand_n[tid] != 0) {  // one lane per query, serial insertion (round 2 form)
                const int ql = tid;
                const int nc = min(cand_n[ql], FCB);
                float* bv = best_v + ql * FKP;
                int32_t* br = best_r + ql * FKP;
                int fill_n = fillc[ql];
                for (int c = 0; c < nc; ++c) {
                    const float v = cand_v[ql * FCB + c];
                    const int32_t r = cand_r[ql * FCB + c];
                    if (fill_n == FKP && !lt_vr(v, r, bv[FKP - 1], br[FKP - 1])) continue;
                    int p = fill_n < FKP ? fill_n : FKP - 1;
                    while (p > 0 && lt_vr(v, r, bv[p - 1], br[p - 1])) { bv[p] = bv[p - 1]; br[p] = br[p - 1]; --p; }
                    bv[p] = v;
                    br[p] = r;
                    if (fill_n < FKP) ++fill_n;
                }
                fillc[ql] = fill_n;
                cand_n[ql] = 0;
                float gbq = gbl[ql];
                if (!PRB && gq_own && fill_n >= a.k) {
                    const float ub = bv[a.k - 1] + 2.0f * gepsl[ql];
                    if (ub < gbq) {
                        gbq = ub;
                        gbl[ql] = ub;
                        atomicMin(a.gbound + gq_idx, ord_enc(ub));
                    }
                }
                thr[ql] = fminf(fill_n == FKP ? bv[FKP - 1] : INFINITY, next_up(gbq));
            }
            } else {
            static_assert(FKP == 16, "group insertion: one lane per list slot");
            const int grp = lane >> 4, gl = lane & 15;
#pragma unroll 1
            for (int ql = wave * 4 + grp; ql < FQ; ql += F_THREADS / 16) {
                const int nc = min(cand_n[ql], FCB);
                if (nc == 0) continue;
                float bvj = best_v[ql * FKP + gl];
                int32_t brj = best_r[ql * FKP + gl];
                int fill_n = fillc[ql];
#pragma unroll 1
                for (int c = 0; c < nc; ++c) {
                    const float v = cand_v[ql * FCB + c];
                    const int32_t r = cand_r[ql * FCB + c];
                    const bool less = gl < fill_n && lt_vr(bvj, brj, v, r);
                    const int pos = __popcll((__ballot(less) >> (16 * grp)) & 0xFFFFull);
                    // slot j-1 -> j inside each 16-lane row (DPP row_shr:1)
                    const float upv = __int_as_float(
                        __builtin_amdgcn_update_dpp(__float_as_int(bvj), __float_as_int(bvj), 0x111, 0xF, 0xF, false));
                    const int32_t upr = __builtin_amdgcn_update_dpp(brj, brj, 0x111, 0xF, 0xF, false);
                    if (pos < FKP) {  // group-uniform
                        if (gl == pos) { bvj = v; brj = r; }
                        else if (gl > pos) { bvj = upv; brj = upr; }
                        fill_n = min(fill_n + 1, FKP);
                    }
                }
                best_v[ql * FKP + gl] = bvj;
                best_r[ql * FKP + gl] = brj;
                if (gl == 0) {  // the group's own writes are ordered before these reads (one wave)
                    const float vk = best_v[ql * FKP + (a.k < FKP ? a.k : FKP) - 1];
                    const float vlast = best_v[ql * FKP + FKP - 1];
                    fillc[ql] = fill_n;
                    cand_n[ql] = 0;
                    float gbq = gbl[ql];
                    if (!PRB && q0 + ql < a.nq && fill_n >= a.k) {
                        const float ub = vk + 2.0f * gepsl[ql];
                        if (ub < gbq) {
                            gbq = ub;
                            gbl[ql] = ub;
                            atomicMin(a.gbound + q0 + ql, ord_enc(ub));
                        }
                    }
                    thr[ql] = fminf(fill_n == FKP ? vlast : INFINITY, next_up(gbq));
                }
            }
            }
            if (tid == 0) ovf[(round + 1) & 1] = 0;
            __syncthreads();
            if (!ovf[round & 1]) break;
        }
    };

    // Ring of F_NSTAGE stages: step it reads stage it % F_NSTAGE while the DMA
    // of the next F_NSTAGE-1 steps is in flight. Each wave issues 4 DMAs per
    // step, so vmcnt(4 * later) retires its share of step it; the raw barrier
    // then publishes every wave's share (barriers do not drain VMEM;
    // __syncthreads would). Tiles are the outer loop and k-steps the inner one
    // (unrolled by F_NSTAGE when nk is a multiple of it, so ring stages and LDS
    // read offsets are constants): per-tile work stays out of the k-loop. The
    // tile epilogue's own barriers drain the ring once per 128-row tile.
    __syncthreads();  // list init visible before the first epilogue
    TileSrc cur_src = tile_src(r_beg);
    TileSrc nxt_src = cur_src;
#pragma unroll
    for (int f = 0; f < NST - 1; ++f)
        if (f < iters) fill(f < nk ? cur_src : tile_src(r_beg + (f / nk) * FR), (f % nk) * FK, fsm + f * F_STAGE);

    // One k-step: global step it, ring stage st. Every step issues one DMA group
    // (k-step it + F_NSTAGE - 1 into the stage read in step it - 1; the last
    // F_NSTAGE - 1 steps re-read the tile's first k-slice into a stage nobody
    // reads again), so the groups in flight beyond the one a step waits for are
    // a per-block constant. The group's four 1-KiB pieces are issued between
    // the step's first MFMAs rather than ahead of them: both waves of a SIMD
    // leave the barrier together, and a piece issued beside a running MFMA
    // overlaps it instead of idling the matrix core.
    const int64_t later_c = min((int64_t)NST - 2, iters - 1);
    auto kstep = [&](int64_t it, int64_t rt, int kt, int st) {
        static_assert(PCS == 4 || PCS == 6, "vmcnt immediates below");
        if constexpr (PCS == 4) {
            if (later_c >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (later_c == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (later_c >= 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else if (later_c == 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int fk = kt + NST - 1;
        const int fst = st == 0 ? NST - 1 : st - 1;
        TileSrc fs = cur_src;
        int fk0 = 0;
        if (it + NST - 1 < iters) {
            if (fk < nk) fk0 = fk * FK;
            else if (fk < 2 * nk) { fs = nxt_src; fk0 = (fk - nk) * FK; }
            else { fs = tile_src(rt + (fk / nk) * FR); fk0 = (fk % nk) * FK; }  // d < 64
        }
        unsigned char* fdst = fsm + fst * F_STAGE;
        auto piece = [&](int j) {  // j: 0 rows/0, 1 queries/0, 2 rows/1, 3 queries/1 (then rows)
#ifdef RVX_ABLATE_DMA
            return;
#endif
            dma_piece(fs, fk0, fdst, j);
        };
        const unsigned char* cur = fsm + st * F_STAGE;
        if constexpr (M16) {
            // one K = 32 step of 16x16x32 MFMAs: B fragments of the wave's 4 query tiles,
            // then the 8 row tiles in two halves (4 A fragments live at a time); DMA piece j
            // follows MFMA j * 32 / PCS, as in the 32x32 form
            h16x8 bf[AN];
#pragma unroll
            for (int f = 0; f < AN; ++f)
                bf[f] = __builtin_bit_cast(h16x8, *reinterpret_cast<const u32x4*>(cur + b_rd[0] + f * 1024));
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                h16x8 af[AM / 2];
#pragma unroll
                for (int f = 0; f < AM / 2; ++f)
                    af[f] = __builtin_bit_cast(h16x8,
                                               *reinterpret_cast<const u32x4*>(cur + a_rd[0] + (half * AM / 2 + f) * 1024));
#pragma unroll
                for (int f = 0; f < AM / 2; ++f)
#pragma unroll
                    for (int fn = 0; fn < AN; ++fn) {
                        const int fm = half * AM / 2 + f;
                        acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[f], bf[fn], acc[fm][fn], 0, 0, 0);
                        constexpr int PS16 = AM * AN / PCS;
                        const int m = fm * AN + fn;
                        if (m % PS16 == 0 && m / PS16 < PCS) {
                            __builtin_amdgcn_sched_barrier(0);
                            piece(m / PS16);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
            }
        } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            h16x8 af[F_FM], bf[2];
#pragma unroll
            for (int f = 0; f < F_FM; ++f)
                af[f] = __builtin_bit_cast(h16x8, *reinterpret_cast<const u32x4*>(cur + a_rd[ks] + f * 2048));
#pragma unroll
            for (int f = 0; f < 2; ++f)
                bf[f] = __builtin_bit_cast(h16x8, *reinterpret_cast<const u32x4*>(cur + b_rd[ks] + f * 2048));
#pragma unroll
            for (int fm = 0; fm < F_FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < 2; ++fn) {
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
                    constexpr int PS = 2 * F_FM / PCS > 1 ? 2 * F_FM / PCS : 1;
                    const int m = 2 * fm + fn;  // piece j follows MFMA j * PS of the step
                    if (ks == 0 && m % PS == 0 && m / PS < PCS) {
                        __builtin_amdgcn_sched_barrier(0);
                        piece(m / PS);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
        }
        }
    };

    const bool unrolled = nk % NST == 0;  // every tile starts on ring stage 0
    int st = 0;
    int64_t it = 0;
    for (int64_t rt = r_beg; rt < r_end; rt += FR) {
        // the tile's row constants, consumed by its epilogue
        float4 pre;
        if constexpr (PRB) {
            pre = (tid < FR && rt + tid < r_end) ? a.xc4[rt + tid - a.row0] : make_float4(NAN, 0.0f, 0.0f, 0.0f);
        } else {
            const float2 p2 = (tid < FR && rt + tid < r_end) ? a.xc[rt + tid - a.row0] : make_float2(NAN, 0.0f);
            pre = make_float4(p2.x, p2.y, 0.0f, 0.0f);
        }
        if (rt + FR < r_end) nxt_src = tile_src(rt + FR);
        if (unrolled) {
            for (int kt = 0; kt < nk; kt += NST, it += NST)
#pragma unroll
                for (int u = 0; u < NST; ++u) kstep(it + u, rt, kt + u, u);
        } else {
            for (int kt = 0; kt < nk; ++kt, ++it) {
                kstep(it, rt, kt, st);
                st = st == NST - 1 ? 0 : st + 1;
            }
        }
#ifdef RVX_ABLATE_EPI
        if (rt + FR >= r_end)
#endif
        epilogue(rt, pre);
        if (gq_own) graw = __hip_atomic_load(a.gbound + gq_idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j)
#pragma unroll
                for (int e = 0; e < AE; ++e) acc[i][j][e] = 0.0f;
        cur_src = nxt_src;
    }
    __syncthreads();

    for (int i = tid; i < FQ * FKP; i += F_THREADS) {
        const int64_t qg = q0 + i / FKP;
        if (qg >= a.nq) continue;
        const int64_t o = (qg * a.nsplit_total + a.split0 + sl) * FKP + (i % FKP);
        a.part_v[o] = best_v[i];
        a.part_r[o] = best_r[i];
    }
#ifdef RVX_SCAN_CLOCK
    if (tid == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        a.clk[2 * blockIdx.x] = t1 - clk_t0;
        a.clk[2 * blockIdx.x + 1] = r1 - clk_r0;
    }
#endif
}

struct RerankArgs {
    const float* q; const float* qnorm; const float2* qc;
    const float* x; const float* xnorm;
    int64_t nq; int d, k, nsplit_total;
    const float* part_v; const int32_t* part_r;
    const unsigned* xsq_max_bits;  // max_x |x|^2 (float bits)
    int64_t id_offset;
    float* out_d; int64_t* out_i; int32_t* unsure;
    float* uthr;  // [nq] (nullable): an unsure query's proven bound D, for the band pass
};

template <int METRIC>
__global__ __launch_bounds__(256) void k_scan_rerank(RerankArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= a.nq) return;
    const int total = a.nsplit_total * FKP;
    const float* pv = a.part_v + qi * total;
    const int32_t* pr = a.part_r + qi * total;
    float v[F_MAXE];
    int32_t r[F_MAXE];
#pragma unroll
    for (int j = 0; j < F_MAXE; ++j) {
        const int c = lane + 64 * j;
        const bool ok = c < total && pr[c] >= 0;
        v[j] = ok ? pv[c] : INFINITY;
        r[j] = ok ? pr[c] : INT32_MAX;
    }
    // k-th smallest approximate value (rows are distinct across lists)
    float lv = -INFINITY, vk = INFINITY;
    int32_t lrow = INT32_MIN;
    for (int s = 0; s < a.k; ++s) {
        float bv = INFINITY;
        int32_t brr = INT32_MAX;
#pragma unroll
        for (int j = 0; j < F_MAXE; ++j) {
            const bool after = v[j] > lv || (v[j] == lv && r[j] > lrow);
            if (after && lt_vr(v[j], r[j], bv, brr)) { bv = v[j]; brr = r[j]; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o);
            const int32_t orr = __shfl_xor(brr, o);
            if (lt_vr(ov, orr, bv, brr)) { bv = ov; brr = orr; }
        }
        lv = bv;
        lrow = brr;
        vk = bv;
    }
    const float eps = filter_eps<METRIC>(a.qc[qi].y, __uint_as_float(*a.xsq_max_bits));
    const float D = vk + 2.0f * eps;  // INF when fewer than k rows exist
    // a full list whose last entry is <= D may have dropped a needed row
    bool unsure = false;
    for (int s = lane; s < a.nsplit_total; s += 64) {
        const int c = s * FKP + FKP - 1;
        if (pr[c] >= 0 && pv[c] <= D) unsure = true;
    }
    if (__any(unsure)) {
        if (lane == 0) {
            a.unsure[qi] = 1;
            atomicAdd(a.unsure - 2, 1);  // flags[2]: how many queries need the VALU scan
            if (a.uthr) a.uthr[qi] = D;
        }
        return;
    }
    // reference distances of the candidates (one lane each, sequential order)
    const float* qrow = a.q + qi * a.d;
    const float qn = (METRIC == RVX_METRIC_COSINE) ? a.qnorm[qi] : 0.0f;
    float ex[F_MAXE];
#pragma unroll
    for (int j = 0; j < F_MAXE; ++j) {
        ex[j] = INFINITY;
        if (r[j] == INT32_MAX || !(v[j] <= D)) continue;
        const float* xr = a.x + (int64_t)r[j] * a.d;
        float acc = 0.0f;
        for (int kk = 0; kk < a.d; kk += 4) {
            const float4 qv = *reinterpret_cast<const float4*>(qrow + kk);
            const float4 xv = *reinterpret_cast<const float4*>(xr + kk);
            acc = pair_step<METRIC>(acc, qv.x, xv.x);
            acc = pair_step<METRIC>(acc, qv.y, xv.y);
            acc = pair_step<METRIC>(acc, qv.z, xv.z);
            acc = pair_step<METRIC>(acc, qv.w, xv.w);
        }
        ex[j] = pair_finish<METRIC>(acc, qn, (METRIC == RVX_METRIC_COSINE) ? a.xnorm[r[j]] : 0.0f);
    }
    float ld = -INFINITY;
    int64_t li = INT64_MIN;
    for (int s = 0; s < a.k; ++s) {
        float bd = INFINITY;
        int64_t bi = INT64_MAX;
#pragma unroll
        for (int j = 0; j < F_MAXE; ++j) {
            const int64_t id = r[j] == INT32_MAX ? INT64_MAX : (int64_t)r[j] + a.id_offset;
            if (ex[j] == INFINITY && id == INT64_MAX) continue;
            const bool after = ex[j] > ld || (ex[j] == ld && id > li);
            if (after && better(ex[j], id, bd, bi)) { bd = ex[j]; bi = id; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float od = __shfl_xor(bd, o);
            const int64_t oi = __shfl_xor(bi, o);
            if (better(od, oi, bd, bi)) { bd = od; bi = oi; }
        }
        if (lane == 0) { a.out_d[qi * a.k + s] = bd; a.out_i[qi * a.k + s] = bi; }
        ld = bd;
        li = bi;
    }
}

// ---------------------------------------------------------------------------
// Per-row bounds (Poincaré distance and the tangent scan's squared L2).
//
// The global eps above bounds |v - reference| with max_x |x| for every row. That
// is tight for rows of similar norm (10M x 768 N(0,1)) but not for the C5 data,
// where the nearest rows (small radius, or the tangent coordinates of such
// points) are far shorter than the longest row, and for the Poincaré distance
// the ranking quantity carries a per-row factor. Here every (row, query) value
// is a LOWER bound L of the reference's own ranking quantity T, with the row's
// own norm in the bound:
//   |x.q - x^.q^/(t_x t_q)| <= 2^-10 |x||q| (f16 rounding) + f32 accumulation
//   |T_sum - |q-x|^2| <= (d+2) 2^-24 (|q|^2+|x|^2)  (the reference's f32 sum, and
//                                                    the |x|^2 / |q|^2 estimates)
//   E = 1.5 2^-9 |q||x| + beta (|q|^2+|x|^2),  beta = 2^-12 max(1, d/1024)
//   (v = |x|^2 - 2 x.q carries twice the dot's 1.06 2^-10 |x||q|: 1.4x slack; beta 1.3x)
//   squared L2 (tangent_distance_squared): T = sum (q-x)^2 in [|q|^2+v-E, |q|^2+v+E],
//     v = |x|^2 - 2 x.q from the MFMA dot
//   Poincaré: arg - 1 = 2c |q-x|^2 / (lambda_q lambda_x) with lambda_q fixed per query,
//     so the ranking is T = s_x |q-x|^2, s_x = 1/max(1 - c|x|^2, 1e-5), known to
//     relative delta_s = (c 2^-13 |x|^2 + 2^-22) / lambda_x (the reference's |x|^2
//     sum and the subtraction), widened by rho = 2^-13 for the reference's own
//     rounding of arg and fast_acosh (at most a few ulp, and the 8e-6 relative jump
//     at its delta = 1e-4 branch): T in [s_lo (|q|^2+v-E), s_hi (|q|^2+v+E)].
// Rows whose delta_s exceeds 2^-6 (points on the ball's edge) send the call to
// the VALU scan. Next to distance 0 the Poincaré distance is quantised by the f32
// rounding of arg = 1 + (2c/lambda_q) T (ties broken by id), so the rerank widens Uk by
// 2^-22 (1/2c + Uk) there. L = s_lo (|q|^2 (1-beta) + |x|^2 (1-beta) - 2 x.q - 1.5 2^-9|q||x|)
// is one multiply and three FMAs per value from row factors {R = s_lo/t_x,
// C = s_lo |x|^2 (1-beta), S = s_lo, N = s_lo |x|} and query factors {Q = -2/t_q,
// Qs = |q|^2 (1-beta), P = -1.5 2^-9 |q|}. The rerank rebuilds each listed row's
// upper bound U = s_hi (L/s_lo + 2.0625 E) (the 1/32 covers the f32 rounding of L),
// takes Uk = k-th smallest U, and computes the reference distance of every listed
// row with L <= Uk; a split whose full list ends at or below Uk may have dropped a
// needed row and the query goes to the VALU scan.
__global__ __launch_bounds__(256) void k_rows_to_f16_pr(const float* __restrict__ x, int64_t n, int d,
                                                       _Float16* __restrict__ xh, float4* __restrict__ rc4,
                                                       float4* __restrict__ rb, const uint8_t* __restrict__ deleted,
                                                       float c, float beta, int32_t* bad) {
    typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    bool run_ok = true;
    for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += nwaves) {
        const float* xr = x + row * d;
        float m = 0.0f, s = 0.0f;
        bool fin = true;
        for (int k = 4 * lane; k < d; k += 256) {
            const float4 v = *reinterpret_cast<const float4*>(xr + k);
            fin = fin && __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z) &&
                  __builtin_isfinite(v.w);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            m = fmaxf(m, __shfl_xor(m, o));
            s += __shfl_xor(s, o);
        }
        fin = !__any(!fin);
        const float t = h2_scale_dev(m);
        for (int k = 4 * lane; k < d; k += 256) {
            const float4 v = *reinterpret_cast<const float4*>(xr + k);
            h16x4 h = {(_Float16)(v.x * t), (_Float16)(v.y * t), (_Float16)(v.z * t), (_Float16)(v.w * t)};
            *reinterpret_cast<h16x4*>(xh + row * d + k) = h;
        }
        float s_lo = 1.0f, s_hi = 1.0f;
        bool ok = true;
        if (c > 0.0f) {  // Poincaré: s_x = 1 / max(1 - c|x|^2, EPS)
            const float lam = fmaxf(1.0f - c * s, pdev::EPS);
            const float ds = (c * s * 0x1p-13f + 0x1p-22f) / lam;
            ok = ds <= 0x1p-6f;
            const float sx = 1.0f / lam;
            s_lo = sx * (1.0f - ds) * (1.0f - 0x1p-13f);
            s_hi = sx * (1.0f + ds) * (1.0f + 0x1p-13f);
        }
        const float nrm = sqrtf(s);
        if (lane == 0) {
            const bool del = deleted && deleted[row];
            rc4[row] = make_float4(del ? NAN : s_lo / t, s_lo * s * (1.0f - beta), s_lo, s_lo * nrm);
            rb[row] = make_float4(s_lo, s_hi, s, nrm);
        }
        run_ok = run_ok && ok && fin && __builtin_isfinite(s) && (m == 0.0f || (ilogbf(m) >= -60 && ilogbf(m) <= 60));
    }
    if (lane == 0 && !run_ok) atomicOr(bad, 1);
}

struct RerankPrArgs {
    const float* q; const float2* qc;  // queries and {1/t_q, |q|^2}
    const float* x; const float4* rb;  // rows and {s_lo, s_hi, |x|^2, |x|} of every row
    int64_t nq; int d, k, nsplit_total;
    const float* part_v; const int32_t* part_r;
    float beta, curv;
    int64_t id_offset;
    float* out_d; int64_t* out_i; int32_t* unsure;
    float* uthr;  // [nq] (nullable): an unsure query's proven bound thr, for the band pass
};

// one wave per query: Uk, candidates, reference distances, top-k by (distance, id)
template <int METRIC>
__global__ __launch_bounds__(256) void k_scan_rerank_pr(RerankPrArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (qi >= a.nq) return;
    const int total = a.nsplit_total * FKP;
    const float* pv = a.part_v + qi * total;
    const int32_t* pr = a.part_r + qi * total;
    const float q2 = a.qc[qi].y, qn = sqrtf(q2);
    float l[F_MAXE], u[F_MAXE];
    int32_t r[F_MAXE];
#pragma unroll
    for (int j = 0; j < F_MAXE; ++j) {
        const int c = lane + 64 * j;
        const bool ok = c < total && pr[c] >= 0;
        l[j] = ok ? pv[c] : INFINITY;
        r[j] = ok ? pr[c] : INT32_MAX;
        u[j] = INFINITY;
        if (ok) {
            const float4 b = a.rb[r[j]];
            const float e = 0x1.8p-9f * qn * b.w + a.beta * (q2 + b.z);
            u[j] = b.y * (l[j] / b.x + 2.0625f * e);
        }
    }
    // k-th smallest upper bound (rows are distinct across lists)
    float lu = -INFINITY, uk = INFINITY;
    int32_t lrow = INT32_MIN;
    for (int s = 0; s < a.k; ++s) {
        float bu = INFINITY;
        int32_t brr = INT32_MAX;
#pragma unroll
        for (int j = 0; j < F_MAXE; ++j) {
            const bool after = u[j] > lu || (u[j] == lu && r[j] > lrow);
            if (after && lt_vr(u[j], r[j], bu, brr)) { bu = u[j]; brr = r[j]; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ou = __shfl_xor(bu, o);
            const int32_t orr = __shfl_xor(brr, o);
            if (lt_vr(ou, orr, bu, brr)) { bu = ou; brr = orr; }
        }
        lu = bu;
        lrow = brr;
        uk = bu;
    }
    // Poincaré: arg = 1 + (2c/lambda_q) T is rounded to f32 next to 1, so rows whose T
    // differ by less than ~ulp(arg) lambda_q / 2c share one distance (all T below
    // 2^-24 lambda_q / 2c give distance 0) and are ordered by id: a row ties with the
    // k-th while its T exceeds Uk by up to 2^-23 (lambda_q / 2c + T) (both roundings
    // and the division's); 2x slack.
    const float thr = (METRIC == RVX_METRIC_POINCARE) ? uk + 0x1p-22f * (0.5f / a.curv + fabsf(uk)) : uk;
    bool unsure = false;
    for (int s = lane; s < a.nsplit_total; s += 64) {
        const int c = s * FKP + FKP - 1;
        if (pr[c] >= 0 && pv[c] <= thr) unsure = true;
    }
    if (__any(unsure)) {
        if (lane == 0) {
            a.unsure[qi] = 1;
            atomicAdd(a.unsure - 2, 1);
            if (a.uthr) a.uthr[qi] = thr;
        }
        return;
    }
    const float* qrow = a.q + qi * a.d;
    float ex[F_MAXE];
#pragma unroll
    for (int j = 0; j < F_MAXE; ++j) {
        ex[j] = INFINITY;
        if (r[j] == INT32_MAX || !(l[j] <= thr)) continue;
        const float* xr = a.x + (int64_t)r[j] * a.d;
        if constexpr (METRIC == RVX_METRIC_POINCARE) {  // fused_norms chunk order, then from_norms (as K8)
            float ds = 0.0f, nu = 0.0f, nv = 0.0f;
            for (int kk = 0; kk < a.d; kk += 4) {
                const float4 qv = *reinterpret_cast<const float4*>(qrow + kk);
                const float4 xv = *reinterpret_cast<const float4*>(xr + kk);
                const float d0 = qv.x - xv.x, d1 = qv.y - xv.y, d2 = qv.z - xv.z, d3 = qv.w - xv.w;
                ds = ds + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
                nu = nu + (((qv.x * qv.x + qv.y * qv.y) + qv.z * qv.z) + qv.w * qv.w);
                nv = nv + (((xv.x * xv.x + xv.y * xv.y) + xv.z * xv.z) + xv.w * xv.w);
            }
            ex[j] = pdev::from_norms(ds, nu, nv, a.curv);
        } else {  // tangent_distance_squared: sequential sum of (q - x)^2
            float acc = 0.0f;
            for (int kk = 0; kk < a.d; kk += 4) {
                const float4 qv = *reinterpret_cast<const float4*>(qrow + kk);
                const float4 xv = *reinterpret_cast<const float4*>(xr + kk);
                acc = pair_step<METRIC_L2SQ>(acc, qv.x, xv.x);
                acc = pair_step<METRIC_L2SQ>(acc, qv.y, xv.y);
                acc = pair_step<METRIC_L2SQ>(acc, qv.z, xv.z);
                acc = pair_step<METRIC_L2SQ>(acc, qv.w, xv.w);
            }
            ex[j] = acc;
        }
    }
    float ld = -INFINITY;
    int64_t li = INT64_MIN;
    for (int s = 0; s < a.k; ++s) {
        float bd = INFINITY;
        int64_t bi = INT64_MAX;
#pragma unroll
        for (int j = 0; j < F_MAXE; ++j) {
            const int64_t id = r[j] == INT32_MAX ? INT64_MAX : (int64_t)r[j] + a.id_offset;
            if (ex[j] == INFINITY && id == INT64_MAX) continue;
            const bool after = ex[j] > ld || (ex[j] == ld && id > li);
            if (after && better(ex[j], id, bd, bi)) { bd = ex[j]; bi = id; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float od = __shfl_xor(bd, o);
            const int64_t oi = __shfl_xor(bi, o);
            if (better(od, oi, bd, bi)) { bd = od; bi = oi; }
        }
        if (lane == 0) { a.out_d[qi * a.k + s] = bd; a.out_i[qi * a.k + s] = bi; }
        ld = bd;
        li = bi;
    }
}

// ---------------------------------------------------------------------------
// Band pass: queries still unsure after the list passes (a split's FKP-long list
// filled at or below the query's bound). The rerank proved a bound thr_q that every
// row of the query's true top-k meets with its filter value (D = v_k + 2 eps; for the
// per-row-bound metrics the tie-widened Uk, see k_scan_rerank_pr), and a lane's value
// below meets the same error bound in any f32 summation order. So the band kernel
// streams the f16 image once per 64 queries and appends EVERY row whose value is
// <= thr_q — no list, nothing dropped — and the band rerank takes the reference
// distances of exactly those rows: the same candidates' superset argument as the
// lists, hence the same top-k bits as the VALU scan. A band longer than its capacity
// sends the query on to the VALU scan. One wave: 32 rows x 64 queries per tile, the
// f16 fragments straight from global memory (a row's 2 KB is read once per 64
// queries; the query image stays in L2).
struct BandArgs {
    const _Float16* xh; const float2* xc; const float4* xc4;  // the whole table's f16 image and row factors
    const _Float16* qh; const float2* qc;                      // band queries' f16 image and {1/t_q, |q|^2 or |q|}
    int64_t nq, n; int d;
    float beta;
    const float* thr;  // [nq]
    int32_t* cnt;      // [nq] band length (may exceed cap)
    int32_t* cand;     // [nq][cap] rows
    int cap;
};

template <int METRIC>
__global__ __launch_bounds__(256) void k_scan_band(BandArgs a) {
    constexpr bool PRB = METRIC == RVX_METRIC_POINCARE || METRIC == METRIC_L2SQ;
    const int lane = threadIdx.x & 63, lr = lane & 31, lh = lane >> 5;
    const int64_t q0 = (int64_t)blockIdx.y * 64;
    float qf[2], qs[2], qp[2], th[2];
    int64_t qg[2];
#pragma unroll
    for (int fn = 0; fn < 2; ++fn) {
        qg[fn] = q0 + fn * 32 + lr;
        const int64_t qc = min(qg[fn], a.nq - 1);
        const float2 c = a.qc[qc];
        if constexpr (PRB) {
            qf[fn] = -2.0f * c.x;
            qs[fn] = c.y * (1.0f - a.beta);
            qp[fn] = -0x1.8p-9f * sqrtf(c.y);
        } else {
            qf[fn] = query_factor<METRIC>(c.x, c.y);
            qs[fn] = qp[fn] = 0.0f;
        }
        th[fn] = qg[fn] < a.nq ? a.thr[qc] : -INFINITY;  // padding query: nothing passes
    }
    const _Float16* qb0 = a.qh + min(q0 + lr, a.nq - 1) * a.d + 8 * lh;
    const _Float16* qb1 = a.qh + min(q0 + 32 + lr, a.nq - 1) * a.d + 8 * lh;
    const int64_t ntiles = (a.n + 31) / 32;
    const int64_t wstride = (int64_t)gridDim.x * 4;
    for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < ntiles; t += wstride) {
        const int64_t r0 = t * 32;
        const _Float16* xb = a.xh + min(r0 + lr, a.n - 1) * a.d + 8 * lh;
        f32x16 acc0, acc1;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc0[e] = acc1[e] = 0.0f;
#pragma unroll 4
        for (int k0 = 0; k0 < a.d; k0 += 16) {
            const h16x8 av = *reinterpret_cast<const h16x8*>(xb + k0);
            const h16x8 b0 = *reinterpret_cast<const h16x8*>(qb0 + k0);
            const h16x8 b1 = *reinterpret_cast<const h16x8*>(qb1 + k0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, b1, acc1, 0, 0, 0);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t row = r0 + (e & 3) + 8 * (e >> 2) + 4 * lh;
            if (row >= a.n) continue;
            float v[2];
            if constexpr (PRB) {
                const float4 c = a.xc4[row];
                v[0] = __builtin_fmaf(c.w, qp[0], __builtin_fmaf(c.z, qs[0], __builtin_fmaf(acc0[e] * c.x, qf[0], c.y)));
                v[1] = __builtin_fmaf(c.w, qp[1], __builtin_fmaf(c.z, qs[1], __builtin_fmaf(acc1[e] * c.x, qf[1], c.y)));
            } else {
                const float2 f = row_factors<METRIC>(a.xc[row]);
                v[0] = __builtin_fmaf(acc0[e] * f.x, qf[0], f.y);
                v[1] = __builtin_fmaf(acc1[e] * f.x, qf[1], f.y);
            }
#pragma unroll
            for (int fn = 0; fn < 2; ++fn)
                if (v[fn] <= th[fn]) {  // NaN (deleted row) never passes
                    const int pos = atomicAdd(a.cnt + qg[fn], 1);
                    if (pos < a.cap) a.cand[qg[fn] * a.cap + pos] = (int32_t)row;
                }
        }
    }
}

struct BandRerankArgs {
    const float* q; const float* qnorm;  // band queries [nq][d]; reference norms (cosine)
    const float* x; const float* xnorm;  // rows; reference norms (cosine)
    const int32_t* cnt; const int32_t* cand; int cap;
    float* dist;  // [nq][cap] scratch
    int64_t nq; int d, k; float curv;
    int64_t id_offset;
    float* out_d; int64_t* out_i;  // [nq][k]
};

// one block per band query: the reference distance of every band row (the rerank's
// arithmetic), then k rounds of a block-wide (distance, id) minimum
template <int METRIC>
__global__ __launch_bounds__(256) void k_scan_band_rerank(BandRerankArgs a) {
    const int64_t qi = blockIdx.x;
    const int m = a.cnt[qi];
    if (m > a.cap) return;  // the VALU scan owns this query
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float* qrow = a.q + qi * a.d;
    const int32_t* cr = a.cand + qi * a.cap;
    float* dr = a.dist + qi * a.cap;
    for (int c = tid; c < m; c += 256) {
        const float* xr = a.x + (int64_t)cr[c] * a.d;
        float ex;
        if constexpr (METRIC == RVX_METRIC_POINCARE) {  // fused_norms chunk order, then from_norms (as K8)
            float ds = 0.0f, nu = 0.0f, nv = 0.0f;
            for (int kk = 0; kk < a.d; kk += 4) {
                const float4 qv = *reinterpret_cast<const float4*>(qrow + kk);
                const float4 xv = *reinterpret_cast<const float4*>(xr + kk);
                const float d0 = qv.x - xv.x, d1 = qv.y - xv.y, d2 = qv.z - xv.z, d3 = qv.w - xv.w;
                ds = ds + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
                nu = nu + (((qv.x * qv.x + qv.y * qv.y) + qv.z * qv.z) + qv.w * qv.w);
                nv = nv + (((xv.x * xv.x + xv.y * xv.y) + xv.z * xv.z) + xv.w * xv.w);
            }
            ex = pdev::from_norms(ds, nu, nv, a.curv);
        } else {  // sequential sum in the reference order (tangent_distance_squared: no finish)
            float acc = 0.0f;
            for (int kk = 0; kk < a.d; kk += 4) {
                const float4 qv = *reinterpret_cast<const float4*>(qrow + kk);
                const float4 xv = *reinterpret_cast<const float4*>(xr + kk);
                acc = pair_step<METRIC>(acc, qv.x, xv.x);
                acc = pair_step<METRIC>(acc, qv.y, xv.y);
                acc = pair_step<METRIC>(acc, qv.z, xv.z);
                acc = pair_step<METRIC>(acc, qv.w, xv.w);
            }
            if constexpr (METRIC == METRIC_L2SQ) ex = acc;
            else ex = pair_finish<METRIC>(acc, METRIC == RVX_METRIC_COSINE ? a.qnorm[qi] : 0.0f,
                                          METRIC == RVX_METRIC_COSINE ? a.xnorm[cr[c]] : 0.0f);
        }
        dr[c] = ex;
    }
    __syncthreads();
    __shared__ float sd[4];
    __shared__ int64_t si[4];
    float ld = -INFINITY;
    int64_t li = INT64_MIN;
    for (int s = 0; s < a.k; ++s) {
        float bd = INFINITY;
        int64_t bi = INT64_MAX;
        for (int c = tid; c < m; c += 256) {
            const float dv = dr[c];
            const int64_t id = (int64_t)cr[c] + a.id_offset;
            const bool after = dv > ld || (dv == ld && id > li);
            if (after && better(dv, id, bd, bi)) { bd = dv; bi = id; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float od = __shfl_xor(bd, o);
            const int64_t oi = __shfl_xor(bi, o);
            if (better(od, oi, bd, bi)) { bd = od; bi = oi; }
        }
        if (lane == 0) { sd[wave] = bd; si[wave] = bi; }
        __syncthreads();
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (better(sd[w], si[w], bd, bi)) { bd = sd[w]; bi = si[w]; }
        __syncthreads();  // every wave has read sd / si before the next round writes them
        if (tid == 0) { a.out_d[qi * a.k + s] = bd; a.out_i[qi * a.k + s] = bi; }
        ld = bd;
        li = bi;
    }
}

// Waves stride over rows: power-of-two scale t (row max in [2^14, 2^15)),
// f16(x*t), and the row constants {1/t, or NaN for a deleted row; cnorm[row]
// when given (cosine) else sum x^2 (any order; only the filter uses it)}, the
// running max of sum x^2 (one atomic per wave), and a flag for rows the filter
// cannot bound (non-finite, |x| beyond 2^+-60).
__global__ __launch_bounds__(256) void k_rows_to_f16(const float* __restrict__ x, int64_t n, int d,
                                                    _Float16* __restrict__ xh, float2* __restrict__ rc,
                                                    const float* __restrict__ cnorm, const uint8_t* __restrict__ deleted,
                                                    unsigned* max_sq_bits, int32_t* bad) {
    typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    float run_max = 0.0f;
    bool run_ok = true;
    for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += nwaves) {
        const float* xr = x + row * d;
        float m = 0.0f, s = 0.0f;
        bool fin = true;
        for (int k = 4 * lane; k < d; k += 256) {
            const float4 v = *reinterpret_cast<const float4*>(xr + k);
            fin = fin && __builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z) &&
                  __builtin_isfinite(v.w);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
            s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            m = fmaxf(m, __shfl_xor(m, o));
            s += __shfl_xor(s, o);
        }
        fin = !__any(!fin);
        const float t = h2_scale_dev(m);
        for (int k = 4 * lane; k < d; k += 256) {
            const float4 v = *reinterpret_cast<const float4*>(xr + k);
            h16x4 h = {(_Float16)(v.x * t), (_Float16)(v.y * t), (_Float16)(v.z * t), (_Float16)(v.w * t)};
            *reinterpret_cast<h16x4*>(xh + row * d + k) = h;
        }
        if (lane == 0) {
            const bool del = deleted && deleted[row];
            rc[row] = make_float2(del ? NAN : 1.0f / t, cnorm ? cnorm[row] : s);
        }
        run_ok = run_ok && fin && __builtin_isfinite(s) && (m == 0.0f || (ilogbf(m) >= -60 && ilogbf(m) <= 60));
        run_max = fmaxf(run_max, s);
    }
    if (lane == 0) {
        if (!run_ok) atomicOr(bad, 1);
        if (max_sq_bits && run_max > 0.0f) atomicMax(max_sq_bits, __float_as_uint(run_max));
    }
}

// max over rows of sum x^2 (wave per row, any order), into max_sq_bits
__global__ __launch_bounds__(256) void k_row_sq_max(const float* __restrict__ x, int64_t n, int d,
                                                   unsigned* max_sq_bits) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    float run_max = 0.0f;
    for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += nwaves) {
        const float* xr = x + row * d;
        float s = 0.0f;
        for (int k = 4 * lane; k < d; k += 256) {
            const float4 v = *reinterpret_cast<const float4*>(xr + k);
            s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        run_max = fmaxf(run_max, s);
    }
    if (lane == 0 && run_max > 0.0f) atomicMax(max_sq_bits, __float_as_uint(run_max));
}

void row_sq_max(const float* x, int64_t n, int d, unsigned* max_bits) {
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, 4096));
    RVX_LAUNCH("scan_f16", k_row_sq_max, dim3((unsigned)blocks), dim3(256), 0, x, n, d, max_bits);
}

void rows_to_f16(const float* x, int64_t n, int d, _Float16* xh, float2* rc, const float* cnorm,
                 const uint8_t* deleted, unsigned* max_bits, int32_t* bad) {
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, 4096));
    RVX_LAUNCH("scan_f16", k_rows_to_f16, dim3((unsigned)blocks), dim3(256), 0, x, n, d, xh, rc, cnorm, deleted,
               max_bits, bad);
}

__global__ void k_gather_rows(const float* src, const int32_t* idx, int64_t cnt, int d, float* dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt * d) return;
    dst[i] = src[(int64_t)idx[i / d] * d + i % d];
}

__global__ void k_scatter_topk(const float* sd, const int64_t* si, const int32_t* idx, int64_t cnt, int k, float* dd,
                               int64_t* di) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt * k) return;
    const int64_t q = idx[i / k];
    dd[q * k + i % k] = sd[i];
    di[q * k + i % k] = si[i];
}

void scan_topk_valu(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
                    const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
                    const char* tag, float curv);
void scan_topk_wide(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
                    const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
                    float curv);

// Returns false (nothing written) when the call should take the VALU scan.
bool scan_topk_mfma(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
                    const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
                    float curv) {
    const int mode = env_int("RVX_SCAN_MFMA", 1);  // 0 off, 1 auto, 2 force (tests); read per call
    if (mode == 0) return false;
    const bool prb = metric == RVX_METRIC_POINCARE || metric == METRIC_L2SQ;  // per-row bounds
    if (metric != RVX_METRIC_L2 && metric != RVX_METRIC_COSINE && metric != RVX_METRIC_DOT && !prb) return false;
    if (metric == RVX_METRIC_POINCARE && !(curv > 0.0f)) return false;
    // tile shape: RVX_SCAN_WIDE 0/1/2 forces it (tests, A/B), else 256^2 for d >= 512
    const int wide_env = env_int("RVX_SCAN_WIDE", -1);
    // the wide tile runs on 16x16x32 MFMAs (cfg 3) unless RVX_SCAN_M16=0: same cycles per
    // flop, the chip holds a higher clock (10M x 768 / 10k: filter 156-161 vs 175-177 ms,
    // identical results; profiles/r04_scan_m16_ab.log); RVX_SCAN_WIDE forces any form
    const int cfg = wide_env >= 0 && wide_env <= 3 ? wide_env
                    : d >= 512                     ? (env_int("RVX_SCAN_M16", 1) ? 3 : 1)
                                                   : 0;
    const int FR = cfg == 1 ? FCfg<1>::FR : cfg == 2 ? FCfg<2>::FR : cfg == 3 ? FCfg<3>::FR : FCfg<0>::FR;
    const int FQ = cfg == 1 ? FCfg<1>::FQ : cfg == 2 ? FCfg<2>::FQ : cfg == 3 ? FCfg<3>::FQ : FCfg<0>::FQ;
    const int F_LDS = cfg == 1 ? FCfg<1>::LDS : cfg == 2 ? FCfg<2>::LDS : cfg == 3 ? FCfg<3>::LDS : FCfg<0>::LDS;
    const int F_THREADS =
        cfg == 1 ? FCfg<1>::THREADS : cfg == 2 ? FCfg<2>::THREADS : cfg == 3 ? FCfg<3>::THREADS : FCfg<0>::THREADS;
    const int F_BLOCKS =
        cfg == 1 ? FCfg<1>::BLOCKS : cfg == 2 ? FCfg<2>::BLOCKS : cfg == 3 ? FCfg<3>::BLOCKS : FCfg<0>::BLOCKS;
    // k > FKP: the lists stay FKP long (no single split proves a k-th value, so the
    // shared bound is off) and the rerank's completeness test decides per query
    if (d % FK != 0 || k > SCAN_MAX_K || n >= ((int64_t)1 << 31) - FR || nq <= 0 || n <= 0) return false;
    if (metric == RVX_METRIC_COSINE && (!qnorm || !xnorm)) return false;
    if (mode == 1 && (nq < 256 || n < 65536)) return false;
    // rows converted per chunk: the f16 image of the whole table when it fits
    // min(16 GiB, a quarter of free HBM) — one filter launch, no max|x|^2
    // pre-pass (10M x 768: 50.3k -> 52.3k QPS) — else chunks of that size
    // (at least 1 GiB; RVX_SCAN_MFMA_CHUNK_ROWS overrides, tests)
    int64_t chunk_rows = env_int("RVX_SCAN_MFMA_CHUNK_ROWS", 0);
    if (chunk_rows <= 0) {
        size_t free_b = 0, total_b = 0;
        RVX_HIP(hipMemGetInfo(&free_b, &total_b));
        const int64_t budget =
            std::max<int64_t>((int64_t)1 << 30, std::min<int64_t>((int64_t)16 << 30, (int64_t)(free_b / 4)));
        chunk_rows = budget / ((int64_t)d * 2);
    }
    chunk_rows = chunk_rows >= n ? (n + FR - 1) / FR * FR : std::max<int64_t>(FR, chunk_rows / FR * FR);
    const int64_t nchunks = (n + chunk_rows - 1) / chunk_rows;
    const int64_t qtiles = (nq + FQ - 1) / FQ;
    const int64_t max_splits = 64 * F_MAXE / FKP;  // rerank capacity
    if (nchunks > max_splits || qtiles > 65535) return false;
    // splits per chunk: a block streams one split's tiles for one query tile, and
    // resident blocks run in waves (one per CU for the 256^2 tile, two for 128^2).
    // Time ~ waves(s) x (tiles per split + warm-up), the warm-up being the early
    // tiles of a split whose still-empty lists admit most values (~8 tiles'
    // worth): 10M x 768 / 10k queries takes 32 splits per chunk (1280 blocks =
    // 5 full waves, not 640 = 2.5), 100k x 128 takes 6 (one wave).
    const int64_t slots = (int64_t)device().num_cus * F_BLOCKS;
    const int64_t tiles = (chunk_rows + FR - 1) / FR;
    const int64_t s_max = std::max<int64_t>(1, std::min<int64_t>(max_splits / nchunks, tiles / 8));
    int64_t s_c = 1;
    double best_t = 1e300;
    for (int64_t s = 1; s <= s_max; ++s) {
        const int64_t waves = (qtiles * s + slots - 1) / slots;
        const double t = (double)waves * ((double)tiles / (double)s + 8.0);
        if (t < best_t * (1.0 - 1e-9)) { best_t = t; s_c = s; }
    }
    // k beyond one list: as many splits as the rerank holds (down to 2 tiles per
    // split), so the candidates spread over many FKP-long lists and few queries
    // find a list full inside their window (C5 tangent scan: k * prune_factor = 100)
    if (k > FKP) s_c = std::max<int64_t>(s_c, std::min<int64_t>(max_splits / nchunks, std::max<int64_t>(1, tiles / 2)));
    int64_t rows_per_split = ((chunk_rows + s_c - 1) / s_c + FR - 1) / FR * FR;
    s_c = (chunk_rows + rows_per_split - 1) / rows_per_split;
    const int nsplit_total = (int)(nchunks * s_c);

    _Float16* qh = (_Float16*)scratch_bytes("mscan_qh", nq * d * 2);
    float2* qc = (float2*)scratch_bytes("mscan_qc", nq * 8);
    _Float16* xh = (_Float16*)scratch_bytes("mscan_xh", chunk_rows * d * 2);
    float2* xc = (float2*)scratch_bytes("mscan_xc", chunk_rows * 8);
    float* part_v = scratch_f32("mscan_part_v", nq * nsplit_total * FKP);
    int32_t* part_r = (int32_t*)scratch_bytes("mscan_part_r", nq * nsplit_total * FKP * 4);
    int32_t* flags = (int32_t*)scratch_bytes("mscan_flags", 16 + nq * 4);  // [0] bad, [1] max |x|^2 bits, [2] unsure count, [4..] unsure
    unsigned* max_bits = (unsigned*)(flags + 1);
    int32_t* unsure = flags + 4;
    RVX_HIP(hipMemsetAsync(flags, 0, (size_t)(16 + nq * 4), stream()));
    unsigned* gbound = (unsigned*)scratch_bytes("mscan_gbound", nq * 4);
    RVX_HIP(hipMemsetD32Async((hipDeviceptr_t)gbound, 0xFF800000u, (size_t)nq, stream()));  // ord_enc(+INF)
    float4* xc4 = prb ? (float4*)scratch_bytes("mscan_xc4", chunk_rows * 16) : nullptr;
    float4* rb = prb ? (float4*)scratch_bytes("mscan_rb", n * 16) : nullptr;
    const float beta = 0x1p-12f * std::max(1.0f, (float)d / 1024.0f);

    static bool attr = false;
    if (!attr) {
#define RVX_FILTER_ATTR(M, W) \
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_filter<M, W, false>, hipFuncAttributeMaxDynamicSharedMemorySize, FCfg<W>::LDS)); \
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_filter<M, W, true>, hipFuncAttributeMaxDynamicSharedMemorySize, FCfg<W>::LDS))
        RVX_FILTER_ATTR(RVX_METRIC_L2, 1); RVX_FILTER_ATTR(RVX_METRIC_COSINE, 1); RVX_FILTER_ATTR(RVX_METRIC_DOT, 1);
        RVX_FILTER_ATTR(RVX_METRIC_L2, 0); RVX_FILTER_ATTR(RVX_METRIC_COSINE, 0); RVX_FILTER_ATTR(RVX_METRIC_DOT, 0);
        RVX_FILTER_ATTR(RVX_METRIC_POINCARE, 1); RVX_FILTER_ATTR(METRIC_L2SQ, 1);
        RVX_FILTER_ATTR(RVX_METRIC_POINCARE, 0); RVX_FILTER_ATTR(METRIC_L2SQ, 0);
        RVX_FILTER_ATTR(RVX_METRIC_L2, 2); RVX_FILTER_ATTR(RVX_METRIC_COSINE, 2); RVX_FILTER_ATTR(RVX_METRIC_DOT, 2);
        RVX_FILTER_ATTR(RVX_METRIC_POINCARE, 2); RVX_FILTER_ATTR(METRIC_L2SQ, 2);
        RVX_FILTER_ATTR(RVX_METRIC_L2, 3); RVX_FILTER_ATTR(RVX_METRIC_COSINE, 3); RVX_FILTER_ATTR(RVX_METRIC_DOT, 3);
        RVX_FILTER_ATTR(RVX_METRIC_POINCARE, 3); RVX_FILTER_ATTR(METRIC_L2SQ, 3);
#undef RVX_FILTER_ATTR
        attr = true;
    }
    const bool cos = metric == RVX_METRIC_COSINE;
    // list insertion: one lane per query (0, default) or 16-lane groups with one list
    // slot per lane (1, opt-in: spills ~100 B/lane in the 256-register wide tile and ran
    // 225 vs 173 ms at 10M x 768 / 10k, scripts/exp_scan_group.sh); read per call
    const bool group = env_int("RVX_SCAN_GROUP", 0) != 0;
    auto launch_filter = [&](FilterArgs& fa, dim3 grid) {
        const dim3 blk((unsigned)F_THREADS);
#define RVX_FILTER_LAUNCH(C)                                                                                          \
    switch (metric) {                                                                                                 \
        case RVX_METRIC_L2: if (group) RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_L2, C, true>), grid, blk, F_LDS, fa); else RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_L2, C, false>), grid, blk, F_LDS, fa); break; \
        case RVX_METRIC_COSINE: if (group) RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_COSINE, C, true>), grid, blk, F_LDS, fa); else RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_COSINE, C, false>), grid, blk, F_LDS, fa); break; \
        case RVX_METRIC_POINCARE: if (group) RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_POINCARE, C, true>), grid, blk, F_LDS, fa); else RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_POINCARE, C, false>), grid, blk, F_LDS, fa); break; \
        case METRIC_L2SQ: if (group) RVX_LAUNCH("scan_filter", (k_scan_filter<METRIC_L2SQ, C, true>), grid, blk, F_LDS, fa); else RVX_LAUNCH("scan_filter", (k_scan_filter<METRIC_L2SQ, C, false>), grid, blk, F_LDS, fa); break; \
        default: if (group) RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_DOT, C, true>), grid, blk, F_LDS, fa); else RVX_LAUNCH("scan_filter", (k_scan_filter<RVX_METRIC_DOT, C, false>), grid, blk, F_LDS, fa); break; \
    }
#ifdef RVX_SCAN_CLOCK
        fa.clk = (unsigned long long*)scratch_bytes("scan_clk", (int64_t)grid.x * 16);
#endif
        if (cfg == 1) { RVX_FILTER_LAUNCH(1) }
        else if (cfg == 2) { RVX_FILTER_LAUNCH(2) }
        else if (cfg == 3) { RVX_FILTER_LAUNCH(3) }
        else { RVX_FILTER_LAUNCH(0) }
#undef RVX_FILTER_LAUNCH
#ifdef RVX_SCAN_CLOCK
        {  // median over blocks of each block's own clock; printed per launch (diagnostic build)
            std::vector<unsigned long long> h((size_t)grid.x * 2);
            RVX_HIP(hipMemcpyAsync(h.data(), fa.clk, h.size() * 8, hipMemcpyDeviceToHost, stream()));
            sync();
            std::vector<double> ghz;
            double life = 0.0;
            for (unsigned b = 0; b < grid.x; ++b)
                if (h[2 * b + 1] > 0) {
                    ghz.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);
                    life += (double)h[2 * b + 1] * 10e-9;
                }
            std::sort(ghz.begin(), ghz.end());
            static int launch = 0;
            if (!ghz.empty())
                std::fprintf(stderr, "[scan clock] launch %d cfg %d: median %.3f GHz (p10 %.3f, p90 %.3f) over %zu blocks, "
                             "mean block life %.2f ms\n", launch, cfg, ghz[ghz.size() / 2], ghz[ghz.size() / 10],
                             ghz[ghz.size() * 9 / 10], ghz.size(), life / (double)ghz.size() * 1e3);
            ++launch;
        }
#endif
    };
    // the reference-order rerank of nqq queries' lists (qq rows, their norms and f16 constants)
    auto launch_rerank = [&](const float* qq, const float* qqn, const float2* qqc, int64_t nqq, int nsplit,
                             float* pv, int32_t* pr, float* od, int64_t* oi, int32_t* uns, float* ut) {
        const dim3 rg((unsigned)((nqq + 3) / 4));
        if (prb) {
            RerankPrArgs rp{qq, qqc, x, rb, nqq, d, k, nsplit, pv, pr, beta, curv, id_offset, od, oi, uns, ut};
            if (metric == RVX_METRIC_POINCARE) RVX_LAUNCH("scan_rerank", k_scan_rerank_pr<RVX_METRIC_POINCARE>, rg, dim3(256), 0, rp);
            else RVX_LAUNCH("scan_rerank", k_scan_rerank_pr<METRIC_L2SQ>, rg, dim3(256), 0, rp);
            return;
        }
        RerankArgs ra{qq, qqn, qqc, x, xnorm, nqq, d, k, nsplit, pv, pr, max_bits, id_offset, od, oi, uns, ut};
        switch (metric) {
            case RVX_METRIC_L2: RVX_LAUNCH("scan_rerank", k_scan_rerank<RVX_METRIC_L2>, rg, dim3(256), 0, ra); break;
            case RVX_METRIC_COSINE: RVX_LAUNCH("scan_rerank", k_scan_rerank<RVX_METRIC_COSINE>, rg, dim3(256), 0, ra); break;
            default: RVX_LAUNCH("scan_rerank", k_scan_rerank<RVX_METRIC_DOT>, rg, dim3(256), 0, ra); break;
        }
    };
    rows_to_f16(q, nq, d, qh, qc, cos ? qnorm : nullptr, nullptr, nullptr, flags);
    // the filter's shared bound needs eps from max |x|^2 over every row before
    // the first chunk's filter (cosine: eps is a constant)
    if (nchunks > 1 && !cos && !prb) row_sq_max(x, n, d, max_bits);
    for (int64_t c = 0; c < nchunks; ++c) {
        const int64_t c0 = c * chunk_rows, c1 = std::min(n, c0 + chunk_rows);
        if (prb) {
            const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((c1 - c0 + 3) / 4, 4096));
            RVX_LAUNCH("scan_f16", k_rows_to_f16_pr, dim3((unsigned)blocks), dim3(256), 0, x + c0 * d, c1 - c0, d, xh, xc4,
                       rb + c0, deleted ? deleted + c0 : nullptr, metric == RVX_METRIC_POINCARE ? curv : 0.0f, beta,
                       flags);
        } else {
            rows_to_f16(x + c0 * d, c1 - c0, d, xh, xc, cos ? xnorm + c0 : nullptr, deleted ? deleted + c0 : nullptr,
                        max_bits, flags);
        }
        FilterArgs fa{xh, xc, qh, qc, nq, c0, c1, d, rows_per_split, (int)(c * s_c), (int)qtiles, nsplit_total,
                      part_v, part_r, gbound, k, max_bits, xc4, beta};
        launch_filter(fa, dim3((unsigned)(qtiles * s_c)));
    }
    // the bound each unsure query proved (one conversion chunk: for the band pass)
    const bool band = nchunks == 1 && env_int("RVX_SCAN_BAND", 1) != 0;
    float* uthr = band ? scratch_f32("mscan_uthr", nq) : nullptr;
    launch_rerank(q, qnorm, qc, nq, nsplit_total, part_v, part_r, out_d, out_i, unsure, uthr);
    // flags[0] bad input, flags[2] unsure-query count: 16 B through a pinned
    // host word; the per-query flags come down only when some query is unsure
    static int32_t* hflags = nullptr;
    if (!hflags) RVX_HIP(hipHostMalloc((void**)&hflags, 16, hipHostMallocDefault));
    RVX_HIP(hipMemcpyAsync(hflags, flags, 16, hipMemcpyDeviceToHost, stream()));
    sync();
#ifdef RVX_COUNT_SLOW
    {
        int32_t hf[4];
        RVX_HIP(hipMemcpy(hf, flags, 16, hipMemcpyDeviceToHost));
        fprintf(stderr, "[scan] slow-path tiles %u (block-tiles %lld)\n", (unsigned)hf[3],
                (long long)(qtiles * ((n + FR - 1) / FR)));
    }
#endif
    if (hflags[0]) return false;  // unbounded inputs: the VALU scan owns the whole call
    std::vector<int32_t> redo;
    if (hflags[2] > 0) {
        std::vector<int32_t> h(nq);
        RVX_HIP(hipMemcpyAsync(h.data(), unsure, (size_t)(nq * 4), hipMemcpyDeviceToHost, stream()));
        sync();
        for (int64_t i = 0; i < nq; ++i)
            if (h[i]) redo.push_back((int32_t)i);
    }
    last_scan_stats().mfma_queries += nq;
    if (redo.empty()) return true;
    // where each query left in redo has its bound: thr_src[thr_idx[i]]
    const float* thr_src = uthr;
    std::vector<int32_t> thr_idx = redo;
    // Second pass (one conversion chunk: the f16 image of every row is still in scratch): the
    // queries whose lists could not prove completeness run the filter again on their own with as
    // many splits as the rerank holds — each FKP-long list then covers fewer rows, so far fewer
    // lists fill below the threshold — before the rest take the exact VALU scan over every row.
    // C5's 6.25M x 1024 Poincaré scan: ~0.6% of 10k queries were unsure with 32 splits, and their
    // VALU scan took 61 of 221 ms; their second filter streams the f16 image once. Results are the
    // same bits either way (the rerank is the reference arithmetic); RVX_SCAN_SECOND=0 skips it.
    if (nchunks == 1 && env_int("RVX_SCAN_SECOND", 1) != 0) {
        const int64_t s2 = std::max<int64_t>(1, std::min<int64_t>(max_splits, (tiles + 1) / 2));
        const int64_t rps2 = ((n + s2 - 1) / s2 + FR - 1) / FR * FR;
        const int nsplit2 = (int)((n + rps2 - 1) / rps2);
        if (nsplit2 > nsplit_total) {
            const int64_t c2 = (int64_t)redo.size();
            const int64_t qtiles2 = (c2 + FQ - 1) / FQ;
            int32_t* didx2 = (int32_t*)scratch_bytes("mscan2_idx", c2 * 4);
            RVX_HIP(hipMemcpyAsync(didx2, redo.data(), (size_t)c2 * 4, hipMemcpyHostToDevice, stream()));
            float* q2 = scratch_f32("mscan2_q", c2 * d);
            float* q2n = cos ? scratch_f32("mscan2_qn", c2) : nullptr;
            RVX_LAUNCH("scan_gather", k_gather_rows, dim3((unsigned)((c2 * d + 255) / 256)), dim3(256), 0, q, didx2, c2, d,
                       q2);
            if (q2n)
                RVX_LAUNCH("scan_gather", k_gather_rows, dim3((unsigned)((c2 + 255) / 256)), dim3(256), 0, qnorm, didx2, c2,
                           1, q2n);
            _Float16* qh2 = (_Float16*)scratch_bytes("mscan2_qh", c2 * d * 2);
            float2* qc2 = (float2*)scratch_bytes("mscan2_qc", c2 * 8);
            int32_t* flags2 = (int32_t*)scratch_bytes("mscan2_flags", 16 + c2 * 4);
            RVX_HIP(hipMemsetAsync(flags2, 0, (size_t)(16 + c2 * 4), stream()));
            unsigned* gbound2 = (unsigned*)scratch_bytes("mscan2_gbound", c2 * 4);
            RVX_HIP(hipMemsetD32Async((hipDeviceptr_t)gbound2, 0xFF800000u, (size_t)c2, stream()));
            float* pv2 = scratch_f32("mscan2_part_v", c2 * nsplit2 * FKP);
            int32_t* pr2 = (int32_t*)scratch_bytes("mscan2_part_r", c2 * nsplit2 * FKP * 4);
            float* rd2 = scratch_f32("mscan2_d", c2 * k);
            float* uthr2 = band ? scratch_f32("mscan2_uthr", c2) : nullptr;
            int64_t* ri2 = (int64_t*)scratch_bytes("mscan2_i", c2 * k * 8);
            rows_to_f16(q2, c2, d, qh2, qc2, q2n, nullptr, nullptr, flags2);
            FilterArgs fa2{xh, xc, qh2, qc2, c2, 0, n, d, rps2, 0, (int)qtiles2, nsplit2, pv2, pr2, gbound2, k, max_bits,
                           xc4, beta};
            launch_filter(fa2, dim3((unsigned)(qtiles2 * nsplit2)));
            launch_rerank(q2, q2n, qc2, c2, nsplit2, pv2, pr2, rd2, ri2, flags2 + 4, uthr2);
            RVX_LAUNCH("scan_gather", k_scatter_topk, dim3((unsigned)((c2 * k + 255) / 256)), dim3(256), 0, rd2, ri2,
                       didx2, c2, k, out_d, out_i);
            RVX_HIP(hipMemcpyAsync(hflags, flags2, 16, hipMemcpyDeviceToHost, stream()));
            sync();
            last_scan_stats().second_pass_queries += c2;
            std::vector<int32_t> still, still_i;
            if (hflags[2] > 0) {
                std::vector<int32_t> h(c2);
                RVX_HIP(hipMemcpyAsync(h.data(), flags2 + 4, (size_t)(c2 * 4), hipMemcpyDeviceToHost, stream()));
                sync();
                for (int64_t i = 0; i < c2; ++i)
                    if (h[i]) {
                        still.push_back(redo[i]);
                        still_i.push_back((int32_t)i);
                    }
            }
            redo.swap(still);
            thr_idx.swap(still_i);
            thr_src = uthr2;
            if (redo.empty()) return true;
        }
    }
    // Band pass (k_scan_band): the queries still unsure take every row whose value is within
    // their proven bound, and the reference distances of those rows (C5's 6.25M x 1024 exact
    // Poincaré scan: 52 of 10k queries left after the second pass, whose VALU scan took 60 of
    // 233 ms). Same bits as the VALU scan; a band past its capacity still goes there.
    // RVX_SCAN_BAND=0 skips it, RVX_SCAN_BAND_CAP caps rows per query (tests).
    if (band) {
        const int64_t nb = (int64_t)redo.size();
        const int64_t cap_env = env_int("RVX_SCAN_BAND_CAP", 65536);
        // rows per query: 64k by default, fewer when many queries are unsure (the row ids and
        // their distances stay within ~1 GiB up to 2M band queries)
        const int cap = (int)std::max<int64_t>(
            1, std::min<int64_t>(cap_env, std::max<int64_t>(64, ((int64_t)1 << 30) / (8 * nb))));
        int32_t* bidx = (int32_t*)scratch_bytes("mscanb_idx", nb * 4);
        int32_t* btix = (int32_t*)scratch_bytes("mscanb_tidx", nb * 4);
        RVX_HIP(hipMemcpyAsync(bidx, redo.data(), (size_t)nb * 4, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(btix, thr_idx.data(), (size_t)nb * 4, hipMemcpyHostToDevice, stream()));
        float* bthr = scratch_f32("mscanb_thr", nb);
        RVX_LAUNCH("scan_gather", k_gather_rows, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, thr_src, btix, nb, 1,
                   bthr);
        float* bq = scratch_f32("mscanb_q", nb * d);
        RVX_LAUNCH("scan_gather", k_gather_rows, dim3((unsigned)((nb * d + 255) / 256)), dim3(256), 0, q, bidx, nb, d,
                   bq);
        float* bqn = nullptr;
        if (cos) {
            bqn = scratch_f32("mscanb_qn", nb);
            RVX_LAUNCH("scan_gather", k_gather_rows, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, qnorm, bidx, nb,
                       1, bqn);
        }
        _Float16* bqh = (_Float16*)scratch_bytes("mscanb_qh", nb * d * 2);
        float2* bqc = (float2*)scratch_bytes("mscanb_qc", nb * 8);
        int32_t* bcnt = (int32_t*)scratch_bytes("mscanb_cnt", 16 + nb * 4);  // [0..3] the conversion's bad flag
        RVX_HIP(hipMemsetAsync(bcnt, 0, (size_t)(16 + nb * 4), stream()));
        rows_to_f16(bq, nb, d, bqh, bqc, bqn, nullptr, nullptr, bcnt);
        int32_t* bcand = (int32_t*)scratch_bytes("mscanb_cand", nb * cap * 4);
        float* bdist = scratch_f32("mscanb_dist", nb * cap);
        float* bd = scratch_f32("mscanb_d", nb * k);
        int64_t* bi = (int64_t*)scratch_bytes("mscanb_i", nb * k * 8);
        BandArgs ba{xh, xc, xc4, bqh, bqc, nb, n, d, beta, bthr, bcnt + 4, bcand, cap};
        const int64_t wtiles = (n + 31) / 32;
        const dim3 bg((unsigned)std::max<int64_t>(1, std::min<int64_t>((wtiles + 3) / 4, 2048)), (unsigned)((nb + 63) / 64));
        BandRerankArgs br{bq, bqn, x, xnorm, bcnt + 4, bcand, cap, bdist, nb, d, k, curv, id_offset, bd, bi};
        switch (metric) {
#define RVX_BAND(M)                                                                                       RVX_LAUNCH("scan_band", k_scan_band<M>, bg, dim3(256), 0, ba);                                        RVX_LAUNCH("scan_band", k_scan_band_rerank<M>, dim3((unsigned)nb), dim3(256), 0, br);                 break;
            case RVX_METRIC_L2: RVX_BAND(RVX_METRIC_L2)
            case RVX_METRIC_COSINE: RVX_BAND(RVX_METRIC_COSINE)
            case RVX_METRIC_POINCARE: RVX_BAND(RVX_METRIC_POINCARE)
            case METRIC_L2SQ: RVX_BAND(METRIC_L2SQ)
            default: RVX_BAND(RVX_METRIC_DOT)
#undef RVX_BAND
        }
        RVX_LAUNCH("scan_gather", k_scatter_topk, dim3((unsigned)((nb * k + 255) / 256)), dim3(256), 0, bd, bi, bidx, nb,
                   k, out_d, out_i);
        std::vector<int32_t> h((size_t)nb);
        RVX_HIP(hipMemcpyAsync(h.data(), bcnt + 4, (size_t)nb * 4, hipMemcpyDeviceToHost, stream()));
        sync();
        last_scan_stats().band_queries += nb;
        std::vector<int32_t> still;
        for (int64_t i = 0; i < nb; ++i)
            if (h[(size_t)i] > cap) still.push_back(redo[(size_t)i]);  // band past capacity
        redo.swap(still);
        if (redo.empty()) return true;
    }
    last_scan_stats().fallback_queries += (int64_t)redo.size();
    // queries whose lists could not prove completeness: exact VALU scan
    const int64_t cnt = (int64_t)redo.size();
    int32_t* didx = (int32_t*)scratch_bytes("mscan_redo_idx", cnt * 4);
    RVX_HIP(hipMemcpyAsync(didx, redo.data(), (size_t)cnt * 4, hipMemcpyHostToDevice, stream()));
    float* rq = scratch_f32("mscan_redo_q", cnt * d);
    const bool pc = metric == RVX_METRIC_POINCARE;
    float* rqn = (metric == RVX_METRIC_COSINE || pc) ? scratch_f32("mscan_redo_qn", cnt) : nullptr;
    float* rd = scratch_f32("mscan_redo_d", cnt * k);
    int64_t* ri = (int64_t*)scratch_bytes("mscan_redo_i", cnt * k * 8);
    RVX_LAUNCH("scan_gather", k_gather_rows, dim3((unsigned)((cnt * d + 255) / 256)), dim3(256), 0, q, didx, cnt, d, rq);
    if (rqn && !pc)
        RVX_LAUNCH("scan_gather", k_gather_rows, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, qnorm, didx, cnt, 1,
                   rqn);
    const float* xn = xnorm;
    if (pc) {  // the VALU Poincaré scan takes squared norms in norm_squared's chunk order
        row_norm_sq(rq, cnt, d, rqn);
        if (!xn) {
            float* t = scratch_f32("mscan_redo_xn", n);
            row_norm_sq(x, n, d, t);
            xn = t;
        }
    }
    scan_topk_valu(metric, rq, rqn, cnt, x, xn, deleted, n, d, k, id_offset, rd, ri, "scan_fallback", curv);
    RVX_LAUNCH("scan_gather", k_scatter_topk, dim3((unsigned)((cnt * k + 255) / 256)), dim3(256), 0, rd, ri, didx, cnt,
               k, out_d, out_i);
    return true;
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

// The same per-row chain (norm_squared's order: one running sum over groups of four) with the
// rows staged through LDS 32 floats at a time: a thread per row reading its own 4 KB row walks
// addresses 4 KB apart across the wave (1 TB/s at 6.25M x 1024, 25 ms); here each 128-B row
// segment is one coalesced load and the chain reads LDS (odd row stride: no bank conflicts).
constexpr int RNS_CH = 32;
__global__ __launch_bounds__(256) void k_row_norm_sq_lds(const float* __restrict__ x, int64_t n, int d,
                                                          float* __restrict__ out) {
    __shared__ float tile[256 * (RNS_CH + 1)];
    const int tid = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * 256;
    const int rows = (int)min<int64_t>(256, n - r0);
    float s = 0.0f;
    for (int c0 = 0; c0 < d; c0 += RNS_CH) {
#pragma unroll
        for (int k = 0; k < RNS_CH / 4; ++k) {  // 256 rows x 8 float4: 8 lanes per 128-B row segment
            const int f = k * 256 + tid, r = f / (RNS_CH / 4), c4 = f % (RNS_CH / 4);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r < rows) v = *reinterpret_cast<const float4*>(x + (r0 + r) * d + c0 + 4 * c4);
            float* t = tile + r * (RNS_CH + 1) + 4 * c4;
            t[0] = v.x; t[1] = v.y; t[2] = v.z; t[3] = v.w;
        }
        __syncthreads();
        const float* t = tile + tid * (RNS_CH + 1);
#pragma unroll
        for (int i = 0; i < RNS_CH; i += 4)
            s = s + (((t[i] * t[i] + t[i + 1] * t[i + 1]) + t[i + 2] * t[i + 2]) + t[i + 3] * t[i + 3]);
        __syncthreads();
    }
    if (tid < rows) out[r0 + tid] = s;
}

void row_norm_sq(const float* x, int64_t n, int d, float* out) {
    if (n <= 0) return;
    if (d % RNS_CH == 0 && ((uintptr_t)x & 15) == 0)
        RVX_LAUNCH("row_norm_sq", k_row_norm_sq_lds, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, x, n, d, out);
    else
        RVX_LAUNCH("row_norm_sq", k_row_norm_sq, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, x, n, d, out);
}

ScanStats& last_scan_stats() {
    static ScanStats s;
    return s;
}

void scan_topk(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
               const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
               const char* tag, float curv) {
    RVX_REQUIRE(k >= 1, RVX_ERR_INVALID_PARAMETER, "k must be >= 1");
    RVX_REQUIRE(d % 4 == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)x & 15) == 0, RVX_ERR_UNSUPPORTED,
                "scan needs dim % 4 == 0 and 16-B aligned rows");
    if (nq <= 0) return;
    last_scan_stats() = ScanStats{};
    if (n <= 0) {  // no rows: every slot empty (distance +inf, row -1)
        RVX_HIP(hipMemsetD32Async((hipDeviceptr_t)out_d, 0x7F800000u, (size_t)(nq * k), stream()));
        RVX_HIP(hipMemsetAsync(out_i, 0xFF, (size_t)(nq * k * 8), stream()));
        return;
    }
    if (k <= SCAN_MAX_K &&
        scan_topk_mfma(metric, q, qnorm, nq, x, xnorm, deleted, n, d, k, id_offset, out_d, out_i, curv))
        return;
    if (metric == RVX_METRIC_POINCARE && (!qnorm || !xnorm)) {  // squared norms for the VALU scan (K8)
        float* qn = scratch_f32("scan_pc_qn", nq);
        float* xn = scratch_f32("scan_pc_xn", n);
        row_norm_sq(q, nq, d, qn);
        row_norm_sq(x, n, d, xn);
        qnorm = qn;
        xnorm = xn;
    }
    if (k > SCAN_MAX_K) {
        scan_topk_wide(metric, q, qnorm, nq, x, xnorm, deleted, n, d, k, id_offset, out_d, out_i, curv);
        return;
    }
    scan_topk_valu(metric, q, qnorm, nq, x, xnorm, deleted, n, d, k, id_offset, out_d, out_i, tag, curv);
}

namespace {
// k > SCAN_MAX_K (flat.rs:63-64 sorts every pair and truncates to any k): K1's tiles write
// the whole distance rows of a query batch (reference scalar order, the same arithmetic as
// the fused top-k), and select_topk takes the first k by (distance, id) from them. Batches
// of queries so that a query's whole footprint — its distance row, the selection's histogram
// and state, and its min(k, n) keys (twice past the LDS sort) — fits min(4 GiB, 1/8 of the free
// HBM) per batch (the histograms and keys were outside the budget).
void scan_topk_wide(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
                    const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
                    float curv) {
    RVX_REQUIRE(n < ((int64_t)1 << 32), RVX_ERR_INVALID_PARAMETER, "k > 128 scans take up to 2^32 rows");
    last_scan_stats().valu_queries += nq;
    size_t fr = 0, tot = 0;
    RVX_HIP(hipMemGetInfo(&fr, &tot));
    int64_t budget = std::min<int64_t>((int64_t)4 << 30, std::max<int64_t>((int64_t)256 << 20, (int64_t)(fr / 8)));
    const int64_t cap_mb = env_int("RVX_SCAN_WIDE_BUDGET_MB", 0);  // tests force several batches
    if (cap_mb > 0) budget = cap_mb << 20;
    const int64_t keys = std::min<int64_t>(k, n);
    const int64_t per_query = n * 4 + 2048 * 4 + 64 + keys * (keys > 8192 ? 16 : 8);
    const int64_t nqb = std::max<int64_t>(1, std::min<int64_t>(nq, budget / per_query));
    float* D = scratch_f32("scan_wide_d", nqb * n);
    for (int64_t q0 = 0; q0 < nq; q0 += nqb) {
        const int64_t nb = std::min(nqb, nq - q0);
        const int64_t qtiles = (nb + TQ - 1) / TQ;
        int64_t nchunks = std::min<int64_t>(std::max<int64_t>(1, (2048 + qtiles - 1) / qtiles),
                                            std::min<int64_t>(std::max<int64_t>(1, (n + TR - 1) / TR), 65535));
        int64_t rows_per_chunk = ((n + nchunks - 1) / nchunks + TR - 1) / TR * TR;
        nchunks = std::max<int64_t>(1, (n + rows_per_chunk - 1) / rows_per_chunk);
        const float* qn = qnorm ? qnorm + q0 : nullptr;
        ScanArgs a{q + q0 * d, x, qn, xnorm, nb, n, d, 0, rows_per_chunk, (int)nchunks, nullptr, nullptr, id_offset,
                   deleted, curv, D, n};
        const dim3 grid((unsigned)qtiles, (unsigned)nchunks);
        const size_t lds = scan_lds_bytes(0);
        switch (metric) {
            case RVX_METRIC_L2: RVX_LAUNCH("scan_wide", (k_scan_topk<RVX_METRIC_L2, true>), grid, dim3(256), lds, a); break;
            case RVX_METRIC_COSINE: RVX_LAUNCH("scan_wide", (k_scan_topk<RVX_METRIC_COSINE, true>), grid, dim3(256), lds, a); break;
            case RVX_METRIC_DOT: RVX_LAUNCH("scan_wide", (k_scan_topk<RVX_METRIC_DOT, true>), grid, dim3(256), lds, a); break;
            case RVX_METRIC_L1: RVX_LAUNCH("scan_wide", (k_scan_topk<RVX_METRIC_L1, true>), grid, dim3(256), lds, a); break;
            case RVX_METRIC_POINCARE: RVX_LAUNCH("scan_wide", (k_scan_topk<RVX_METRIC_POINCARE, true>), grid, dim3(256), lds, a); break;
            case RVX_METRIC_HYP_L2: RVX_LAUNCH("scan_wide", (k_scan_topk<RVX_METRIC_HYP_L2, true>), grid, dim3(256), lds, a); break;
            case METRIC_L2SQ: RVX_LAUNCH("scan_wide", (k_scan_topk<METRIC_L2SQ, true>), grid, dim3(256), lds, a); break;
            default: fail(RVX_ERR_UNSUPPORTED, "metric not supported by the flat scan");
        }
        select_topk(D, nb, n, n, k, nullptr, id_offset, out_d + q0 * k, out_i + q0 * k, nullptr);
    }
}

void scan_topk_valu(int metric, const float* q, const float* qnorm, int64_t nq, const float* x, const float* xnorm,
                    const uint8_t* deleted, int64_t n, int d, int k, int64_t id_offset, float* out_d, int64_t* out_i,
                    const char* tag, float curv) {
    if (nq <= 0) return;
    last_scan_stats().valu_queries += nq;
    const int64_t qtiles = (nq + TQ - 1) / TQ;
    int64_t nchunks = (2048 + qtiles - 1) / qtiles;
    const int64_t max_chunks = std::max<int64_t>(1, (n + TR - 1) / TR);
    nchunks = std::min(std::max<int64_t>(nchunks, 1), std::min<int64_t>(max_chunks, 65535));
    int64_t rows_per_chunk = (n + nchunks - 1) / nchunks;
    rows_per_chunk = ((rows_per_chunk + TR - 1) / TR) * TR;
    nchunks = std::max<int64_t>(1, (n + rows_per_chunk - 1) / rows_per_chunk);

    float* part_d = (float*)scratch_bytes("scan_part_d", nq * nchunks * k * 4);
    int64_t* part_i = (int64_t*)scratch_bytes("scan_part_i", nq * nchunks * k * 8);
    ScanArgs a{q, x, qnorm, xnorm, nq, n, d, k, rows_per_chunk, (int)nchunks, part_d, part_i, id_offset, deleted, curv,
               nullptr, 0};
    const size_t lds = scan_lds_bytes(k);
    static bool attr_done = false;
    if (!attr_done) {
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_COSINE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_DOT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_L1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_POINCARE>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_topk<RVX_METRIC_HYP_L2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        RVX_HIP(hipFuncSetAttribute((const void*)k_scan_topk<METRIC_L2SQ>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
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
        case RVX_METRIC_HYP_L2: RVX_LAUNCH(t, k_scan_topk<RVX_METRIC_HYP_L2>, grid, dim3(256), lds, a); break;
        case METRIC_L2SQ: RVX_LAUNCH(t, k_scan_topk<METRIC_L2SQ>, grid, dim3(256), lds, a); break;
        default: fail(RVX_ERR_UNSUPPORTED, "metric not supported by the flat scan");
    }
    RVX_LAUNCH("scan_merge", k_merge_topk, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, part_d, part_i, nq,
               (int)nchunks, k, out_d, out_i);
}
}  // namespace

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
