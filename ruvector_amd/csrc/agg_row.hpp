// agg_row.hpp — the per-destination-row body of the vector CSR gather (k_aggregate.hip),
// shared by the gather kernels and by the split-f16 GEMM that helps finish the next row
// chunk's gather (gemm_f32.hip, AggHelp): one definition, so a row's aggregate is the same
// arithmetic whichever kernel computes it (-ffp-contract=off: no implicit FMA either way).
#pragma once
#include "common.hpp"
#include "graph.hpp"
#include "kernels.hpp"

namespace rvx {
namespace aggrow {

template <int AGG>
__device__ __forceinline__ float4 agg_op(float4 a, float4 v) {
    if (AGG == AGG_MAX) return make_float4(fmaxf(a.x, v.x), fmaxf(a.y, v.y), fmaxf(a.z, v.z), fmaxf(a.w, v.w));
    return make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
}
__device__ __forceinline__ float4 scale4(float4 v, float w) { return make_float4(v.x * w, v.y * w, v.z * w, v.w * w); }

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// v*t as f16 hi = rn(v*t) at p[0..3] and lo = rn(v*t - hi) at p[pstride..]
__device__ __forceinline__ void split_store4(float4 v, float t, _Float16* p, int64_t pstride) {
    const float x[4] = {v.x * t, v.y * t, v.z * t, v.w * t};
    f16x4 hi, lo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        hi[i] = (_Float16)x[i];
        lo[i] = (_Float16)(x[i] - (float)hi[i]);
    }
    *reinterpret_cast<f16x4*>(p) = hi;
    *reinterpret_cast<f16x4*>(p + pstride) = lo;
}
// Gathered rows are touched once per edge at random, so they never hit in L2
// on a large table; NT loads keep them from evicting the working set of a
// GEMM running beside the gather.
template <bool NT>
__device__ __forceinline__ float4 ld_row4(const float* p) {
    if (NT) {
        const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    }
    return *reinterpret_cast<const float4*>(p);
}

// One wave computes destination row `row` (see k_aggregate_vec for the arguments).
template <int NV, int AGG, bool W, int U, bool NT>
__device__ __forceinline__ void agg_vec_row(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                            const float* __restrict__ wts, const float* __restrict__ x, int dim,
                                            int empty_fill, int post_scale, float* __restrict__ out,
                                            const float* __restrict__ self_x, float* __restrict__ row_scale,
                                            _Float16* __restrict__ planes, int64_t pstride,
                                            const float* __restrict__ row_mul, const float* __restrict__ self_mul,
                                            int64_t row, int lane) {
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
        // deferred normalisation: one multiplier per gathered row (wave-uniform id)
        const float my_m = (row_mul && lane < cnt) ? row_mul[my_c] : 1.0f;
        for (; t + U <= cnt; t += U) {
            float4 v[U][NV];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = __builtin_amdgcn_readlane(my_c, t + u);
                const float* src = x + (int64_t)c * dim + 4 * lane;
#pragma unroll
                for (int j = 0; j < NV; ++j)
                    v[u][j] = active[j] ? ld_row4<NT>(src + 256 * j) : make_float4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float wu = 1.0f;
                if (W) wu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_w), t + u));
                if (row_mul) {
                    const float mu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_m), t + u));
#pragma unroll
                    for (int j = 0; j < NV; ++j) v[u][j] = scale4(v[u][j], mu);
                }
#pragma unroll
                for (int j = 0; j < NV; ++j) acc[j] = agg_op<AGG>(acc[j], W ? scale4(v[u][j], wu) : v[u][j]);
            }
        }
        for (; t < cnt; ++t) {
            const int c = __builtin_amdgcn_readlane(my_c, t);
            const float* src = x + (int64_t)c * dim + 4 * lane;
            float wu = 1.0f;
            if (W) wu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_w), t));
            const float mu = row_mul ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_m), t)) : 1.0f;
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                float4 v = active[j] ? ld_row4<NT>(src + 256 * j) : make_float4(0, 0, 0, 0);
                if (row_mul) v = scale4(v, mu);
                acc[j] = agg_op<AGG>(acc[j], W ? scale4(v, wu) : v);
            }
        }
    }

    float* dst = out + row * dim + 4 * lane;
    if (cnt_total > 0) {
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
    }
    if (row_scale) {  // split-f16 GEMM operand scale over this row's aggregate and self rows
        float m = 0.0f;
        const float* sp = self_x + row * dim + 4 * lane;
        const float smul = self_mul ? self_mul[row] : 1.0f;
        float4 sv[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j)
            if (active[j]) {
                float4 v = *reinterpret_cast<const float4*>(sp + 256 * j);
                if (self_mul) v = scale4(v, smul);
                sv[j] = v;
                m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
                if (cnt_total > 0)
                    m = fmaxf(m, fmaxf(fmaxf(fabsf(acc[j].x), fabsf(acc[j].y)), fmaxf(fabsf(acc[j].z), fabsf(acc[j].w))));
            }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        const float t = h2_scale_dev(m);
        if (lane == 0) row_scale[row] = t;
        if (planes) {
            // the GEMM operand itself: [aggregate | self] * t split into two f16
            // planes, rounding exactly as the in-GEMM split (split_h2_pair)
            _Float16* p0 = planes + row * 2 * dim + 4 * lane;
#pragma unroll
            for (int j = 0; j < NV; ++j)
                if (active[j]) {
                    const float4 a = cnt_total > 0 ? acc[j] : make_float4(0, 0, 0, 0);
                    split_store4(a, t, p0 + 256 * j, pstride);
                    split_store4(sv[j], t, p0 + dim + 256 * j, pstride);
                }
            return;
        }
    }
    if (cnt_total == 0) {
        const float* self = x + row * dim + 4 * lane;
#pragma unroll
        for (int j = 0; j < NV; ++j)
            if (active[j])
                *reinterpret_cast<float4*>(dst + 256 * j) =
                    empty_fill == 1 ? *reinterpret_cast<const float4*>(self + 256 * j) : make_float4(0, 0, 0, 0);
        return;
    }
#ifdef RVX_AB_NO_AGG_WRITE  // timing-only ablation build (scripts/exp_sage_ablate.sh): results wrong
    if (NT && acc[0].x == 12345.0f)
#endif
#pragma unroll
    for (int j = 0; j < NV; ++j)
        if (active[j]) *reinterpret_cast<float4*>(dst + 256 * j) = acc[j];
}

// Dynamic form of the overlapped GraphSAGE gather (AggHelp): every wave takes destination
// rows from the chunk's counter until it passes n. Used by the chunk's own gather kernel and
// by the previous chunk's GEMM blocks once their tiles are done.
template <int NV, int AGG>
__device__ __forceinline__ void agg_help_rows(const AggHelp& h, int lane) {
    for (;;) {
        int64_t row = 0;
        if (lane == 0) row = (int64_t)atomicAdd(h.counter, 1u);
        row = __builtin_amdgcn_readfirstlane((int)row);
        if (row >= h.n) return;
        agg_vec_row<NV, AGG, false, 8, true>(h.rp, h.col, nullptr, h.x, h.dim, 0, 0, h.out, h.self_x, h.row_scale,
                                            nullptr, 0, h.row_mul, h.self_mul, row, lane);
    }
}
template <int NV>
__device__ __forceinline__ void agg_help_run_nv(const AggHelp& h, int lane) {
    if (h.agg == AGG_MEAN) agg_help_rows<NV, AGG_MEAN>(h, lane);
    else if (h.agg == AGG_SUM) agg_help_rows<NV, AGG_SUM>(h, lane);
    else agg_help_rows<NV, AGG_MAX>(h, lane);
}
__device__ __forceinline__ void agg_help_run(const AggHelp& h) {
    const int lane = threadIdx.x & 63;
    if (h.dim > 512) agg_help_run_nv<3>(h, lane);
    else if (h.dim > 256) agg_help_run_nv<2>(h, lane);
    else agg_help_run_nv<1>(h, lane);
}

}  // namespace aggrow
}  // namespace rvx
