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

template <int NV, int AGG>
__device__ __forceinline__ void agg_row_finish(float4 (&acc)[NV], const bool (&active)[NV], int cnt_total,
                                               const float* __restrict__ x, int dim, int empty_fill, int post_scale,
                                               float* __restrict__ out, const float* __restrict__ self_x,
                                               float* __restrict__ row_scale, _Float16* __restrict__ planes,
                                               int64_t pstride, const float* __restrict__ self_mul, int64_t row,
                                               int lane);

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

    agg_row_finish<NV, AGG>(acc, active, cnt_total, x, dim, empty_fill, post_scale, out, self_x, row_scale, planes,
                            pstride, self_mul, row, lane);
}

// The end of a destination row: mean / GCN scale, the split-f16 operand scale (and planes) over
// [aggregate | self], the store (or the empty-row fill). Shared by the dense and image gathers.
template <int NV, int AGG>
__device__ __forceinline__ void agg_row_finish(float4 (&acc)[NV], const bool (&active)[NV], int cnt_total,
                                               const float* __restrict__ x, int dim, int empty_fill, int post_scale,
                                               float* __restrict__ out, const float* __restrict__ self_x,
                                               float* __restrict__ row_scale, _Float16* __restrict__ planes,
                                               int64_t pstride, const float* __restrict__ self_mul, int64_t row,
                                               int lane) {
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

// ---- ReLU-sparse row image (RowImage, kernels.hpp) ----
// inclusive wave64 prefix sum in VALU: DPP row shifts 1/2/4/8, then row broadcasts 15 / 31
__device__ __forceinline__ unsigned img_wave_scan(unsigned x) {
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
// header bits of this lane (12: block j's 4 columns at bits 4j..4j+3) -> the packed position of
// the lane's first value in each block (values are stored block by block, lane by lane); also
// the row's total count
__device__ __forceinline__ void img_positions(unsigned h, int (&p)[3], unsigned& total) {
    const unsigned c = __popc(h & 15u) | (__popc((h >> 4) & 15u) << 10) | (__popc((h >> 8) & 15u) << 20);
    const unsigned s = img_wave_scan(c);
    const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)s, 63);
    const unsigned ex = s - c;
    const int b1 = (int)(tot & 1023u), b2 = b1 + (int)((tot >> 10) & 1023u);
    p[0] = (int)(ex & 1023u);
    p[1] = b1 + (int)((ex >> 10) & 1023u);
    p[2] = b2 + (int)(ex >> 20);
    total = (unsigned)b2 + (tot >> 20);
}
// a value is kept unless its bits are those of +0.0 (so -0.0 and NaN travel as they are)
__device__ __forceinline__ unsigned img_nz(float v) { return __float_as_uint(v) != 0u; }

// Image gather of one destination row (mean / sum, no edge weights, NV == 3): the same terms,
// order and arithmetic as agg_vec_row<3, AGG, false, 8, true>, so the same bits. Per group of 8
// neighbour rows, three 16-B loads per lane and row — from the row's slot (lanes past the
// record re-read its last 16 B: only the record's bytes are fetched) when nnz <= IMG_CAP, else
// from the dense row — then, two rows at a time, each imaged record passes through one of the
// wave's two 3 KiB LDS windows (ds_write_b128 per KiB it spans) and each lane reads its header
// bits and its values (12 ds_read_b32 at the packed positions).
template <int AGG>
__device__ __forceinline__ void agg_img_row(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                            const float* __restrict__ x, int dim,
                                            const unsigned char* __restrict__ slots,
                                            const uint16_t* __restrict__ nnz, float* __restrict__ out,
                                            const float* __restrict__ self_x, float* __restrict__ row_scale,
                                            const float* __restrict__ row_mul, const float* __restrict__ self_mul,
                                            int64_t row, int lane, unsigned char* win) {
#ifndef RVX_IMG_U
#define RVX_IMG_U 8
#endif
    constexpr int NV = 3, U = RVX_IMG_U;
    const int64_t beg = rp[row], end = rp[row + 1];
    const int cnt_total = (int)(end - beg);
    float4 acc[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    bool active[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) active[j] = (4 * lane + 256 * j) < dim;
    const int dlast = (dim - 4) * 4;  // byte offset of the row's last float4 (inactive lanes re-read it)
    int doff[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) doff[j] = active[j] ? (4 * lane + 256 * j) * 4 : dlast;

    for (int64_t e0 = beg; e0 < end; e0 += 64) {
        const int cnt = (int)min<int64_t>(64, end - e0);
        const int my_c = lane < cnt ? col[e0 + lane] : 0;
        const float my_m = (row_mul && lane < cnt) ? row_mul[my_c] : 1.0f;
        const int my_n = lane < cnt ? (int)nnz[my_c] : 0;
        for (int t = 0; t < cnt; t += U) {
            float4 v[U][NV];
            bool img[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int tu = min(t + u, cnt - 1);  // a short group re-reads its last row (not accumulated)
                const int c = __builtin_amdgcn_readlane(my_c, tu);
                const int nz = __builtin_amdgcn_readlane(my_n, tu);
                img[u] = nz <= IMG_CAP;
                const char* base;
                int o[NV];
                if (img[u]) {
                    base = reinterpret_cast<const char*>(slots + (int64_t)c * IMG_SLOT);
                    const int last = ((128 + 4 * nz - 1) & ~15);
                    o[0] = min(16 * lane, last);
                    o[1] = min(1024 + 16 * lane, last);
                    o[2] = min(2048 + 16 * lane, last);
                } else {
                    base = reinterpret_cast<const char*>(x + (int64_t)c * dim);
#pragma unroll
                    for (int j = 0; j < NV; ++j) o[j] = doff[j];
                }
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    const f32x4 w = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(base + o[j]));
                    v[u][j] = make_float4(w.x, w.y, w.z, w.w);
                }
            }
            // rows in pairs through the wave's two windows: both records in, both expanded, then
            // accumulated in edge order (the LDS round trips of the pair overlap)
#pragma unroll
            for (int u = 0; u < U; u += 2) {
                if (t + u >= cnt) break;
#pragma unroll
                for (int b = 0; b < 2; ++b) {
#ifdef RVX_IMG_NOEXP  // timing-only ablation: imaged rows accumulated unexpanded (wrong values)
                    continue;
#endif
                    if (t + u + b >= cnt || !img[u + b]) continue;
                    const int rec = 128 + 4 * __builtin_amdgcn_readlane(my_n, t + u + b);
                    f32x4* wv = reinterpret_cast<f32x4*>(win + b * IMG_SLOT);
#ifdef RVX_IMG_NOWRITE  // timing-only ablation (wrong values)
                    continue;
#endif
                    wv[lane] = f32x4{v[u + b][0].x, v[u + b][0].y, v[u + b][0].z, v[u + b][0].w};
                    if (rec > 1024) wv[64 + lane] = f32x4{v[u + b][1].x, v[u + b][1].y, v[u + b][1].z, v[u + b][1].w};
                    if (rec > 2048) wv[128 + lane] = f32x4{v[u + b][2].x, v[u + b][2].y, v[u + b][2].z, v[u + b][2].w};
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
                for (int b = 0; b < 2; ++b) {
#ifdef RVX_IMG_NOEXP
                    continue;
#endif
                    if (t + u + b >= cnt || !img[u + b]) continue;
                    const unsigned char* wb = win + b * IMG_SLOT;
                    const unsigned h = reinterpret_cast<const uint16_t*>(wb)[lane];
                    const float* wf = reinterpret_cast<const float*>(wb + 128);
                    int p[3];
                    unsigned tot;
#ifdef RVX_IMG_NOSCAN  // timing-only ablation (wrong values)
                    p[0] = 4 * lane; p[1] = 256 + 4 * lane; p[2] = 480 + 4 * lane; tot = 0;
#else
                    img_positions(h, p, tot);
#endif
#pragma unroll
                    for (int j = 0; j < NV; ++j) {
                        // the lane's values of block j are consecutive from p[j]: four 4-B reads
                        // at p[j]..p[j]+3 (two ds_read2_b32; the window has slack past its end),
                        // then value k is the one of rank popc(bits below k), or +0.0
                        const unsigned nib = (h >> (4 * j)) & 15u;
                        const float w0 = wf[p[j]], w1 = wf[p[j] + 1], w2 = wf[p[j] + 2], w3 = wf[p[j] + 3];
                        const bool b0 = nib & 1u, b1 = nib & 2u, b2 = nib & 4u, b3 = nib & 8u;
                        const int r2 = (int)b0 + (int)b1, r3 = r2 + (int)b2;
                        const float e0 = b0 ? w0 : 0.0f;
                        const float e1 = b1 ? (b0 ? w1 : w0) : 0.0f;
                        const float e2 = b2 ? (r2 == 0 ? w0 : r2 == 1 ? w1 : w2) : 0.0f;
                        const float e3 = b3 ? (r3 == 0 ? w0 : r3 == 1 ? w1 : r3 == 2 ? w2 : w3) : 0.0f;
                        v[u + b][j] = make_float4(e0, e1, e2, e3);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // reads done before the next pair's writes
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    if (t + u + b >= cnt) break;
                    if (row_mul) {
                        const float mu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_m), t + u + b));
#pragma unroll
                        for (int j = 0; j < NV; ++j) v[u + b][j] = scale4(v[u + b][j], mu);
                    }
#pragma unroll
                    for (int j = 0; j < NV; ++j) acc[j] = agg_op<AGG>(acc[j], v[u + b][j]);
                }
            }
        }
    }
    agg_row_finish<NV, AGG>(acc, active, cnt_total, x, dim, 0, 0, out, self_x, row_scale, nullptr, 0, self_mul, row,
                            lane);
}

// Image gather of one destination row with the expansion in registers (AggHelp::img_reg):
// the same terms, order and arithmetic as agg_vec_row<3, AGG, false, 8, true>, so the same
// bits, without the LDS round trip of agg_img_row. Per group of U neighbour rows: each
// lane loads its u16 header word of every imaged row (128 B per row), the DPP scan turns
// it into the packed positions of the lane's three blocks, and the lane loads its values
// of block j straight from the record as one 16-B load at 128 + 4 p[j] (4-B aligned;
// bytes past the lane's own values belong to the next lane or the next slot and are not
// used), then expands them with the header bits. Two dependent round trips per group, so
// the next group's headers are issued before this group's values are consumed.
template <int AGG>
__device__ __forceinline__ void agg_img_row_reg(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                const float* __restrict__ x, int dim,
                                                const unsigned char* __restrict__ slots,
                                                const uint16_t* __restrict__ nnz, float* __restrict__ out,
                                                const float* __restrict__ self_x, float* __restrict__ row_scale,
                                                const float* __restrict__ row_mul, const float* __restrict__ self_mul,
                                                int64_t row, int lane) {
#ifndef RVX_IMGR_U
#define RVX_IMGR_U 8
#endif
    constexpr int NV = 3, U = RVX_IMGR_U;
    const int64_t beg = rp[row], end = rp[row + 1];
    const int cnt_total = (int)(end - beg);
    float4 acc[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    bool active[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) active[j] = (4 * lane + 256 * j) < dim;
    const int dlast = (dim - 4) * 4;  // byte offset of the row's last float4 (inactive lanes re-read it)
    int doff[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) doff[j] = active[j] ? (4 * lane + 256 * j) * 4 : dlast;

    for (int64_t e0 = beg; e0 < end; e0 += 64) {
        const int cnt = (int)min<int64_t>(64, end - e0);
        const int my_c = lane < cnt ? col[e0 + lane] : 0;
        const float my_m = (row_mul && lane < cnt) ? row_mul[my_c] : 1.0f;
        const int my_n = lane < cnt ? (int)nnz[my_c] : 0;
        unsigned hh[U];
        auto load_hdr = [&](int t, unsigned (&h)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int tu = min(t + u, cnt - 1);
                const int c = __builtin_amdgcn_readlane(my_c, tu);
                const int nz = __builtin_amdgcn_readlane(my_n, tu);
                h[u] = nz <= IMG_CAP
                           ? (unsigned)__builtin_nontemporal_load(
                                 reinterpret_cast<const uint16_t*>(slots + (int64_t)c * IMG_SLOT) + lane)
                           : 0u;
            }
        };
        load_hdr(0, hh);
        for (int t = 0; t < cnt; t += U) {
            float4 v[U][NV];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int tu = min(t + u, cnt - 1);  // a short group re-reads its last row (not accumulated)
                const int c = __builtin_amdgcn_readlane(my_c, tu);
                const int nz = __builtin_amdgcn_readlane(my_n, tu);
                const char* base;
                int o[NV];
                if (nz <= IMG_CAP) {
                    int p[3];
                    unsigned tot;
                    img_positions(hh[u], p, tot);
                    base = reinterpret_cast<const char*>(slots + (int64_t)c * IMG_SLOT + 128);
#pragma unroll
                    for (int j = 0; j < NV; ++j) o[j] = 4 * p[j];
                } else {
                    base = reinterpret_cast<const char*>(x + (int64_t)c * dim);
#pragma unroll
                    for (int j = 0; j < NV; ++j) o[j] = doff[j];
                }
#pragma unroll
                for (int j = 0; j < NV; ++j) {
                    f32x4 w;
                    __builtin_memcpy(&w, base + o[j], 16);  // 4-B aligned: unaligned-access mode
                    v[u][j] = make_float4(w.x, w.y, w.z, w.w);
                }
            }
            unsigned hn[U];
            if (t + U < cnt) load_hdr(t + U, hn);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (t + u >= cnt) break;
                const int nz = __builtin_amdgcn_readlane(my_n, t + u);
                if (nz <= IMG_CAP) {
#pragma unroll
                    for (int j = 0; j < NV; ++j) {
                        const unsigned nib = (hh[u] >> (4 * j)) & 15u;
                        const float w0 = v[u][j].x, w1 = v[u][j].y, w2 = v[u][j].z, w3 = v[u][j].w;
                        const bool b0 = nib & 1u, b1 = nib & 2u, b2 = nib & 4u, b3 = nib & 8u;
                        const int r2 = (int)b0 + (int)b1, r3 = r2 + (int)b2;
                        const float x0 = b0 ? w0 : 0.0f;
                        const float x1 = b1 ? (b0 ? w1 : w0) : 0.0f;
                        const float x2 = b2 ? (r2 == 0 ? w0 : r2 == 1 ? w1 : w2) : 0.0f;
                        const float x3 = b3 ? (r3 == 0 ? w0 : r3 == 1 ? w1 : r3 == 2 ? w2 : w3) : 0.0f;
                        v[u][j] = make_float4(x0, x1, x2, x3);
                    }
                }
                if (row_mul) {
                    const float mu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_m), t + u));
#pragma unroll
                    for (int j = 0; j < NV; ++j) v[u][j] = scale4(v[u][j], mu);
                }
#pragma unroll
                for (int j = 0; j < NV; ++j) acc[j] = agg_op<AGG>(acc[j], v[u][j]);
            }
            if (t + U < cnt) {
#pragma unroll
                for (int u = 0; u < U; ++u) hh[u] = hn[u];
            }
        }
    }
    agg_row_finish<NV, AGG>(acc, active, cnt_total, x, dim, 0, 0, out, self_x, row_scale, nullptr, 0, self_mul, row,
                            lane);
}

// Dynamic form of the overlapped GraphSAGE gather (AggHelp): every wave takes destination
// rows from the chunk's counter until it passes n. Used by the chunk's own gather kernel and
// by the previous chunk's GEMM blocks once their tiles are done. `win`: this wave's two
// IMG_SLOT LDS windows for the image path.
template <int NV, int AGG, bool IMG>
__device__ __forceinline__ void agg_help_rows(const AggHelp& h, int lane, unsigned char* win) {
    const bool use_img = IMG && NV == 3 && AGG != AGG_MAX && h.img_slots != nullptr;
    for (;;) {
        int64_t row = 0;
        if (lane == 0) row = (int64_t)atomicAdd(h.counter, 1u);
        row = __builtin_amdgcn_readfirstlane((int)row);
        if (row >= h.n) return;
        if constexpr (IMG && NV == 3 && AGG != AGG_MAX) {
            if (use_img) {
                if (h.img_reg)
                    agg_img_row_reg<AGG>(h.rp, h.col, h.x, h.dim, h.img_slots, h.img_nnz, h.out, h.self_x,
                                         h.row_scale, h.row_mul, h.self_mul, row, lane);
                else
                    agg_img_row<AGG>(h.rp, h.col, h.x, h.dim, h.img_slots, h.img_nnz, h.out, h.self_x, h.row_scale,
                                     h.row_mul, h.self_mul, row, lane, win);
                continue;
            }
        }
        agg_vec_row<NV, AGG, false, 8, true>(h.rp, h.col, nullptr, h.x, h.dim, 0, 0, h.out, h.self_x, h.row_scale,
                                            nullptr, 0, h.row_mul, h.self_mul, row, lane);
    }
}
template <int NV, bool IMG>
__device__ __forceinline__ void agg_help_run_nv(const AggHelp& h, int lane, unsigned char* win) {
    if (h.agg == AGG_MEAN) agg_help_rows<NV, AGG_MEAN, IMG>(h, lane, win);
    else if (h.agg == AGG_SUM) agg_help_rows<NV, AGG_SUM, IMG>(h, lane, win);
    else agg_help_rows<NV, AGG_MAX, IMG>(h, lane, win);
}
// IMG: the image path is compiled in (h.img_slots may then be set); lds: IMG_WIN bytes per
// wave of the block (wave w uses lds + w * IMG_WIN), unused without IMG
template <bool IMG>
__device__ __forceinline__ void agg_help_run(const AggHelp& h, unsigned char* lds) {
    const int lane = threadIdx.x & 63;
    unsigned char* win = lds + (threadIdx.x >> 6) * IMG_WIN;
    if (h.dim > 512) agg_help_run_nv<3, IMG>(h, lane, win);
    else if (h.dim > 256) agg_help_run_nv<2, IMG>(h, lane, win);
    else agg_help_run_nv<1, IMG>(h, lane, win);
}

}  // namespace aggrow
}  // namespace rvx
