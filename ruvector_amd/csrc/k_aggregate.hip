// k_aggregate.hip — CSR neighbour-gather + message-aggregate (HBM-bound).
//
// Replaces the per-node aggregation loops of the reference:
//   sum_aggregate / mean_aggregate / max_aggregate
//     (crates/ruvector-postgres/src/gnn/aggregators.rs:35-92)
//   GCN message x*w + sum + 1/sqrt(deg) (gcn.rs:116-137)
// One 64-lane wave owns one destination row; every lane owns float4 column
// slices (col = 4*lane + 256*j), so each gathered neighbour row is read with
// fully coalesced 1-KiB wave instructions. Neighbour ids of a row are loaded
// 64 at a time (one per lane) and broadcast with v_readlane, so the row base
// is wave-uniform. Four neighbour rows are kept in flight before they are
// accumulated — in CSR (= reference edge) order, so every output element is
// the same sequential f32 sum as the reference's `result[i] += val` loop:
// sum/mean/max are bit-exact.
//
// Algorithmic traffic per destination row i: deg_i*(4*dim + 4[+4 weight]) bytes
// of gathers + 8 (row_ptr) + 4*dim written.
#include "common.hpp"
#include "graph.hpp"
#include "kernels.hpp"

namespace rvx {
namespace {

constexpr int ROWS_PER_BLOCK = 4;  // 4 waves

template <int AGG>
__device__ __forceinline__ float4 agg_op(float4 a, float4 v) {
    if (AGG == AGG_MAX) return make_float4(fmaxf(a.x, v.x), fmaxf(a.y, v.y), fmaxf(a.z, v.z), fmaxf(a.w, v.w));
    return make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
}
__device__ __forceinline__ float4 scale4(float4 v, float w) { return make_float4(v.x * w, v.y * w, v.z * w, v.w * w); }

// NV = float4 slots per lane (dim <= 256*NV; dim % 4 == 0).
template <int NV, int AGG, bool W>
__global__ __launch_bounds__(256) void k_aggregate_vec(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                      const float* __restrict__ wts, int64_t n,
                                                      const float* __restrict__ x, int dim, int empty_fill,
                                                      int post_scale, float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= n) return;
    const int64_t beg = rp[row], end = rp[row + 1];
    const int cnt_total = (int)(end - beg);

    const float init = (AGG == AGG_MAX) ? -INFINITY : 0.0f;
    float4 acc[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = make_float4(init, init, init, init);
    bool active[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) active[j] = (4 * lane + 256 * j) < dim;

    for (int64_t e0 = beg; e0 < end; e0 += 64) {
        const int cnt = (int)min<int64_t>(64, end - e0);
        const int my_c = lane < cnt ? col[e0 + lane] : 0;
        const float my_w = (W && lane < cnt) ? wts[e0 + lane] : 1.0f;
        int t = 0;
        for (; t + 4 <= cnt; t += 4) {
            float4 v[4][NV];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = __builtin_amdgcn_readlane(my_c, t + u);
                const float* src = x + (int64_t)c * dim + 4 * lane;
#pragma unroll
                for (int j = 0; j < NV; ++j)
                    v[u][j] = active[j] ? *reinterpret_cast<const float4*>(src + 256 * j) : make_float4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float wu = 1.0f;
                if (W) wu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_w), t + u));
#pragma unroll
                for (int j = 0; j < NV; ++j) acc[j] = agg_op<AGG>(acc[j], W ? scale4(v[u][j], wu) : v[u][j]);
            }
        }
        for (; t < cnt; ++t) {
            const int c = __builtin_amdgcn_readlane(my_c, t);
            const float* src = x + (int64_t)c * dim + 4 * lane;
            float wu = 1.0f;
            if (W) wu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_w), t));
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                float4 v = active[j] ? *reinterpret_cast<const float4*>(src + 256 * j) : make_float4(0, 0, 0, 0);
                acc[j] = agg_op<AGG>(acc[j], W ? scale4(v, wu) : v);
            }
        }
    }

    float* dst = out + row * dim + 4 * lane;
    if (cnt_total == 0) {
        const float* self = x + row * dim + 4 * lane;
#pragma unroll
        for (int j = 0; j < NV; ++j)
            if (active[j])
                *reinterpret_cast<float4*>(dst + 256 * j) =
                    empty_fill == 1 ? *reinterpret_cast<const float4*>(self + 256 * j) : make_float4(0, 0, 0, 0);
        return;
    }
    if (AGG == AGG_MEAN) {
        const float cntf = (float)cnt_total;  // mean_aggregate: x / count (aggregators.rs:64-67)
#pragma unroll
        for (int j = 0; j < NV; ++j)
            acc[j] = make_float4(acc[j].x / cntf, acc[j].y / cntf, acc[j].z / cntf, acc[j].w / cntf);
    }
    if (post_scale == 1) {  // GCN: aggregated *= 1/sqrt(degree) (gcn.rs:127-134)
        const float nrm = 1.0f / sqrtf((float)cnt_total);
#pragma unroll
        for (int j = 0; j < NV; ++j) acc[j] = scale4(acc[j], nrm);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
        if (active[j]) *reinterpret_cast<float4*>(dst + 256 * j) = acc[j];
}

// Any dim: one wave per row, scalar columns; same sequential order.
template <int AGG, bool W>
__global__ __launch_bounds__(256) void k_aggregate_scalar(const int64_t* rp, const int32_t* col, const float* wts,
                                                         int64_t n, const float* x, int dim, int empty_fill,
                                                         int post_scale, float* out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    if (row >= n) return;
    const int64_t beg = rp[row], end = rp[row + 1];
    const int cnt_total = (int)(end - beg);
    for (int c0 = lane; c0 < dim; c0 += 64) {
        float acc = (AGG == AGG_MAX) ? -INFINITY : 0.0f;
        for (int64_t e = beg; e < end; ++e) {
            float v = x[(int64_t)col[e] * dim + c0];
            if (W) v = v * wts[e];
            acc = (AGG == AGG_MAX) ? fmaxf(acc, v) : acc + v;
        }
        if (cnt_total == 0) acc = empty_fill == 1 ? x[row * dim + c0] : 0.0f;
        else {
            if (AGG == AGG_MEAN) acc = acc / (float)cnt_total;
            if (post_scale == 1) acc = acc * (1.0f / sqrtf((float)cnt_total));
        }
        out[row * dim + c0] = acc;
    }
}

template <int AGG, bool W>
void launch_agg(const char* t, const int64_t* rp, const int32_t* col, const float* w, int64_t n, const float* x, int dim,
                int empty_fill, int post_scale, float* out) {
    const dim3 grid((unsigned)((n + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK)), block(256);
    const bool vec = (dim % 4 == 0) && (((uintptr_t)x & 15) == 0) && (((uintptr_t)out & 15) == 0);
    if (vec && dim <= 256)
        RVX_LAUNCH(t, (k_aggregate_vec<1, AGG, W>), grid, block, 0, rp, col, w, n, x, dim, empty_fill, post_scale, out);
    else if (vec && dim <= 512)
        RVX_LAUNCH(t, (k_aggregate_vec<2, AGG, W>), grid, block, 0, rp, col, w, n, x, dim, empty_fill, post_scale, out);
    else if (vec && dim <= 768)
        RVX_LAUNCH(t, (k_aggregate_vec<3, AGG, W>), grid, block, 0, rp, col, w, n, x, dim, empty_fill, post_scale, out);
    else if (vec && dim <= 1024)
        RVX_LAUNCH(t, (k_aggregate_vec<4, AGG, W>), grid, block, 0, rp, col, w, n, x, dim, empty_fill, post_scale, out);
    else
        RVX_LAUNCH(t, (k_aggregate_scalar<AGG, W>), grid, block, 0, rp, col, w, n, x, dim, empty_fill, post_scale, out);
}

}  // namespace

void aggregate_rows(const int64_t* row_ptr, const int32_t* col, const float* w, int64_t n, const float* x, int dim,
                    int agg, int empty_fill, int post_scale, float* out, const char* tag) {
    if (n <= 0) return;
    RVX_REQUIRE(n / ROWS_PER_BLOCK < ((int64_t)1 << 31), RVX_ERR_INVALID_SHAPE, "graph too large for one launch");
    const char* t = tag ? tag : "aggregate";
    const bool W = w != nullptr;
    switch (agg) {
        case AGG_SUM: W ? launch_agg<AGG_SUM, true>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out)
                        : launch_agg<AGG_SUM, false>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out); break;
        case AGG_MEAN: W ? launch_agg<AGG_MEAN, true>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out)
                         : launch_agg<AGG_MEAN, false>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out); break;
        case AGG_MAX: W ? launch_agg<AGG_MAX, true>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out)
                        : launch_agg<AGG_MAX, false>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out); break;
        default: fail(RVX_ERR_INVALID_PARAMETER, "unknown aggregator");
    }
}

}  // namespace rvx
