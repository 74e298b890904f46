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
#include "agg_row.hpp"

#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

namespace rvx {
namespace {

constexpr int ROWS_PER_BLOCK = 4;  // 4 waves

using namespace aggrow;

// NV = float4 slots per lane (dim <= 256*NV; dim % 4 == 0); U = neighbour
// rows in flight per wave (more when the grid is capped to few waves per CU).
template <int NV, int AGG, bool W, int U = 4, bool NT = false>
__global__ __launch_bounds__(256) void k_aggregate_vec(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                      const float* __restrict__ wts, int64_t n,
                                                      const float* __restrict__ x, int dim, int empty_fill,
                                                      int post_scale, float* __restrict__ out,
                                                      const float* __restrict__ self_x, float* __restrict__ row_scale,
                                                      _Float16* __restrict__ planes, int64_t pstride,
                                                      const float* __restrict__ row_mul,
                                                      const float* __restrict__ self_mul) {
    const int lane = threadIdx.x & 63;
#ifndef RVX_AGG_PRIO
#define RVX_AGG_PRIO 0
#endif
    // overlapped launches: optionally issue ahead of the GEMM waves on the same SIMD
    if constexpr (NT && RVX_AGG_PRIO > 0) __builtin_amdgcn_s_setprio(RVX_AGG_PRIO);
    // grid-stride over rows: the grid may be capped (persistent) so the gather
    // leaves CU slots to a concurrently running GEMM
    for (int64_t row = (int64_t)blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6); row < n;
         row += (int64_t)gridDim.x * ROWS_PER_BLOCK) {
    aggrow::agg_vec_row<NV, AGG, W, U, NT>(rp, col, wts, x, dim, empty_fill, post_scale, out, self_x, row_scale, planes,
                                           pstride, row_mul, self_mul, row, lane);
    }
}

// Overlapped GraphSAGE gather (beside the GEMM, one block per CU) for rows of exactly
// 256 NV floats: k_aggregate_vec's groups of U neighbour rows, with the latencies between
// destination rows taken off the chain — the next row's CSR bounds and first 64 column ids
// load while this row's neighbours stream, and this row's self row (operand scale) loads
// with its first group (k_aggregate_vec waits for rp, then col, then the neighbours, then
// the self row: four dependent round trips per destination row). Straight-line loads (no
// per-load conditions, which would make the compiler wait for every load). Same
// accumulation order (CSR order) and arithmetic as k_aggregate_vec: bit-identical outputs.
// rows per group: eight at NV <= 3 (d 768: <= 176 VGPRs, so one wave fits on a SIMD beside
// two waves of the 168-VGPR GEMM, 512 per SIMD)
#define ROLL_U(NV) ((NV) <= 3 ? 8 : 4)
template <int NV, int AGG, int U>
__global__ __launch_bounds__(256) void k_aggregate_roll(const int64_t* __restrict__ rp, const int32_t* __restrict__ col,
                                                       int64_t n, const float* __restrict__ x, int dim,
                                                       float* __restrict__ out, const float* __restrict__ self_x,
                                                       float* __restrict__ row_scale, const float* __restrict__ row_mul,
                                                       const float* __restrict__ self_mul) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * ROWS_PER_BLOCK;
    int64_t row = (int64_t)blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    int64_t beg = 0, end = 0;
    int c_lane = 0;
    if (row < n) {
        beg = rp[row];
        end = rp[row + 1];
        c_lane = lane < min<int64_t>(64, end - beg) ? col[beg + lane] : 0;
    }
    auto load_row_from = [&](float4 (&v)[NV], const float* base) {
        const float* src = base + 4 * lane;
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = ld_row4<true>(src + 256 * j);
    };
    auto load_row = [&](float4 (&v)[NV], int c) { load_row_from(v, x + (int64_t)c * dim); };
    while (row < n) {
        const int cnt_total = (int)(end - beg);
        const int64_t nxt = row + stride;
        int64_t nbeg = 0, nend = 0;
        if (nxt < n) {
            nbeg = rp[nxt];
            nend = rp[nxt + 1];
        }
        float4 sv[NV];  // this row's self row (operand scale), in flight with the neighbours
        if (row_scale) load_row_from(sv, self_x + row * dim);
        const float init = (AGG == AGG_MAX) ? -INFINITY : 0.0f;
        float4 acc[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) acc[j] = make_float4(init, init, init, init);
        int ncl = 0;
        bool ncl_done = false;
        for (int64_t e0 = beg; e0 < end; e0 += 64) {
            const int cnt = (int)min<int64_t>(64, end - e0);
            const int my_c = e0 == beg ? c_lane : (lane < cnt ? col[e0 + lane] : 0);
            const float my_m = (row_mul && lane < cnt) ? row_mul[my_c] : 1.0f;
            auto take = [&](float4 (&v)[NV], int idx) {
                if (row_mul) {
                    const float mu = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_m), idx));
#pragma unroll
                    for (int j = 0; j < NV; ++j) v[j] = scale4(v[j], mu);
                }
#pragma unroll
                for (int j = 0; j < NV; ++j) acc[j] = agg_op<AGG>(acc[j], v[j]);
            };
            const int groups = cnt / U;
            for (int gi = 0; gi < groups; ++gi) {
                float4 v[U][NV];
#pragma unroll
                for (int u = 0; u < U; ++u) load_row(v[u], __builtin_amdgcn_readlane(my_c, gi * U + u));
                if (!ncl_done && nxt < n) {  // next row's ids, behind this row's first loads
                    ncl = lane < min<int64_t>(64, nend - nbeg) ? col[nbeg + lane] : 0;
                    ncl_done = true;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) take(v[u], gi * U + u);
            }
            for (int t = groups * U; t < cnt; ++t) {  // the last cnt % U rows, one at a time
                float4 v[NV];
                load_row(v, __builtin_amdgcn_readlane(my_c, t));
                take(v, t);
            }
        }
        if (!ncl_done && nxt < n) ncl = lane < min<int64_t>(64, nend - nbeg) ? col[nbeg + lane] : 0;

        if (cnt_total > 0 && AGG == AGG_MEAN) {
            const float cntf = (float)cnt_total;  // mean_aggregate: x / count (aggregators.rs:64-67)
#pragma unroll
            for (int j = 0; j < NV; ++j)
                acc[j] = make_float4(acc[j].x / cntf, acc[j].y / cntf, acc[j].z / cntf, acc[j].w / cntf);
        }
        if (row_scale) {  // split-f16 GEMM operand scale over this row's aggregate and self rows
            float m = 0.0f;
            const float smul = self_mul ? self_mul[row] : 1.0f;
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                float4 v = sv[j];
                if (self_mul) v = scale4(v, smul);
                m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
                if (cnt_total > 0)
                    m = fmaxf(m, fmaxf(fmaxf(fabsf(acc[j].x), fabsf(acc[j].y)), fmaxf(fabsf(acc[j].z), fabsf(acc[j].w))));
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
            if (lane == 0) row_scale[row] = h2_scale_dev(m);
        }
        float* dst = out + row * dim + 4 * lane;
#pragma unroll
        for (int j = 0; j < NV; ++j)
            *reinterpret_cast<float4*>(dst + 256 * j) = cnt_total > 0 ? acc[j] : make_float4(0, 0, 0, 0);
        row = nxt;
        beg = nbeg;
        end = nend;
        c_lane = ncl;
    }
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
                int empty_fill, int post_scale, float* out, int cap_per_cu, bool deep, bool nt, const float* self_x,
                float* row_scale, _Float16* planes, int64_t pstride, const float* row_mul, const float* self_mul) {
    int64_t blocks = (n + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
    if (cap_per_cu > 0) blocks = std::min<int64_t>(blocks, (int64_t)cap_per_cu * active_cus());
    const dim3 grid((unsigned)blocks), block(256);
    const bool vec = (dim % 4 == 0) && (((uintptr_t)x & 15) == 0) && (((uintptr_t)out & 15) == 0);
    RVX_REQUIRE(!planes || (vec && row_scale && self_x && empty_fill == 0), RVX_ERR_INVALID_SHAPE,
                "planes need the vector gather with zero-filled empty rows");
    RVX_REQUIRE(!row_mul || (vec && empty_fill == 0), RVX_ERR_INVALID_SHAPE,
                "row multipliers need the vector gather with zero-filled empty rows");
    // opt-in (RVX_AGG_ROLL=1, read per call; tests cover both): the overlapped gather with the
    // next row's CSR data and the self row prefetched (k_aggregate_roll). Same bits; beside the
    // 256 x 192 GEMM it slowed the GEMM more than it saved (401-427 vs 410 ms/step,
    // scripts/exp_roll_ab.sh)
    const bool roll = deep && nt && !W && empty_fill == 0 && post_scale == 0 && !planes && (!row_scale || self_x) &&
                      dim % 256 == 0 && env_int("RVX_AGG_ROLL", 0);
#define RVX_AGG_VEC(NV)                                                                                          \
    do {                                                                                                         \
        if (roll)                                                                                                \
            RVX_LAUNCH(t, (k_aggregate_roll<NV, AGG, ROLL_U(NV)>), grid, block, 0, rp, col, n, x, dim, out,      \
                       self_x, row_scale, row_mul, self_mul);                                                    \
        else if (deep && nt)                                                                                     \
            RVX_LAUNCH(t, (k_aggregate_vec<NV, AGG, W, 8, true>), grid, block, 0, rp, col, w, n, x, dim,         \
                       empty_fill, post_scale, out, self_x, row_scale, planes, pstride, row_mul, self_mul);                         \
        else if (deep)                                                                                           \
            RVX_LAUNCH(t, (k_aggregate_vec<NV, AGG, W, 8>), grid, block, 0, rp, col, w, n, x, dim, empty_fill,   \
                       post_scale, out, self_x, row_scale, planes, pstride, row_mul, self_mul);                                     \
        else                                                                                                     \
            RVX_LAUNCH(t, (k_aggregate_vec<NV, AGG, W, 4>), grid, block, 0, rp, col, w, n, x, dim, empty_fill,   \
                       post_scale, out, self_x, row_scale, planes, pstride, row_mul, self_mul);                                     \
    } while (0)
    if (vec && dim <= 256) RVX_AGG_VEC(1);
    else if (vec && dim <= 512) RVX_AGG_VEC(2);
    else if (vec && dim <= 768) RVX_AGG_VEC(3);
    else if (vec && dim <= 1024) RVX_AGG_VEC(4);
    else {
        RVX_REQUIRE(!row_scale, RVX_ERR_INVALID_SHAPE, "row_scale needs the vector gather (dim % 4 == 0, <= 1024)");
        RVX_LAUNCH(t, (k_aggregate_scalar<AGG, W>), grid, block, 0, rp, col, w, n, x, dim, empty_fill, post_scale, out);
    }
#undef RVX_AGG_VEC
}

}  // namespace

// Overlapped launches (beside a GEMM) keep 8 neighbour rows in flight per wave
// and use NT loads; RVX_AGG_BLOCKS_PER_CU caps the grid to a persistent one.
// With the split-bf16 GEMM the uncapped grid gave the shortest 10M x 768 layer
// (552 vs 578 ms/step for 1 block/CU at 16 chunks, scripts/exp_pipeline.sh).
int g_agg_overlap_cap = env_int("RVX_AGG_BLOCKS_PER_CU", 1);
int g_agg_overlap_unroll = env_int("RVX_AGG_UNROLL", 8);
int g_agg_nt = env_int("RVX_AGG_NT", 1);

void aggregate_rows(const int64_t* row_ptr, const int32_t* col, const float* w, int64_t n, const float* x, int dim,
                    int agg, int empty_fill, int post_scale, float* out, const char* tag, bool overlapped,
                    const float* self_x, float* row_scale, _Float16* planes, int64_t plane_stride,
                    const float* row_mul, const float* self_mul) {
    if (n <= 0) return;
    static const int standalone_deep = env_int("RVX_AGG_STANDALONE_DEEP", 0);  // experiment knob
    const int cap = overlapped ? g_agg_overlap_cap : 0;
    const bool deep = (overlapped || standalone_deep) && g_agg_overlap_unroll >= 8;
    const bool nt = (overlapped || standalone_deep) && g_agg_nt;
    RVX_REQUIRE(n / ROWS_PER_BLOCK < ((int64_t)1 << 31), RVX_ERR_INVALID_SHAPE, "graph too large for one launch");
    const char* t = tag ? tag : "aggregate";
    const bool W = w != nullptr;
    switch (agg) {
        case AGG_SUM: W ? launch_agg<AGG_SUM, true>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out, cap, deep, nt, self_x, row_scale, planes, plane_stride, row_mul, self_mul)
                        : launch_agg<AGG_SUM, false>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out, cap, deep, nt, self_x, row_scale, planes, plane_stride, row_mul, self_mul); break;
        case AGG_MEAN: W ? launch_agg<AGG_MEAN, true>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out, cap, deep, nt, self_x, row_scale, planes, plane_stride, row_mul, self_mul)
                         : launch_agg<AGG_MEAN, false>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out, cap, deep, nt, self_x, row_scale, planes, plane_stride, row_mul, self_mul); break;
        case AGG_MAX: W ? launch_agg<AGG_MAX, true>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out, cap, deep, nt, self_x, row_scale, planes, plane_stride, row_mul, self_mul)
                        : launch_agg<AGG_MAX, false>(t, row_ptr, col, w, n, x, dim, empty_fill, post_scale, out, cap, deep, nt, self_x, row_scale, planes, plane_stride, row_mul, self_mul); break;
        default: fail(RVX_ERR_INVALID_PARAMETER, "unknown aggregator");
    }
}

namespace {
// IMG: with the row-image path (and its LDS windows, ROWS_PER_BLOCK * IMG_WIN of dynamic LDS);
// the dense form keeps its registers and no LDS (4 waves per SIMD for the layer's first chunk)
template <bool IMG>
__global__ __launch_bounds__(256) void k_aggregate_help(AggHelp h) {
    extern __shared__ __attribute__((aligned(16))) unsigned char win[];
    aggrow::agg_help_run<IMG>(h, win);
}

// One wave per row: header bits, packed positions (agg_row.hpp), the record assembled in the
// wave's LDS window (scattered 4-B LDS stores), then written out as whole 16-B chunks
// (coalesced); nnz for every row (rows above IMG_CAP keep no slot: readers take the dense row).
// ids (nullable): row i is ids[i] instead of r0 + i.
__global__ __launch_bounds__(256) void k_rows_image_pack(const float* __restrict__ x, int64_t r0, int64_t rows,
                                                         int dim, unsigned char* __restrict__ slots,
                                                         uint16_t* __restrict__ nnz, const int64_t* __restrict__ ids) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) f32x4 win[ROWS_PER_BLOCK][IMG_SLOT / 16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * ROWS_PER_BLOCK + w;
    if (i >= rows) return;
    const int64_t r = ids ? ids[i] : r0 + i;
    const float* src = x + r * dim;
    float4 v[3];
    unsigned h = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = 4 * lane + 256 * j < dim;
        v[j] = act ? *reinterpret_cast<const float4*>(src + 4 * lane + 256 * j) : make_float4(0, 0, 0, 0);
        const unsigned nib = aggrow::img_nz(v[j].x) | (aggrow::img_nz(v[j].y) << 1) | (aggrow::img_nz(v[j].z) << 2) |
                             (aggrow::img_nz(v[j].w) << 3);
        h |= (act ? nib : 0u) << (4 * j);
    }
    int p[3];
    unsigned tot;
    aggrow::img_positions(h, p, tot);
    if (lane == 0) nnz[r] = (uint16_t)tot;
    if (tot > (unsigned)IMG_CAP) return;
    unsigned char* wb = reinterpret_cast<unsigned char*>(win[w]);
    reinterpret_cast<uint16_t*>(wb)[lane] = (uint16_t)h;
    float* vals = reinterpret_cast<float*>(wb + 128);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
        int q = p[j];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if ((h >> (4 * j + k)) & 1u) vals[q++] = e[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int chunks = (128 + 4 * (int)tot + 15) / 16;
    f32x4* dst = reinterpret_cast<f32x4*>(slots + r * IMG_SLOT);
    for (int c = lane; c < chunks; c += 64) dst[c] = win[w][c];
}

// ---- compact exchange records (rvx_sage_forward_exchange3 at world > 1) ----
// A round's block of rows travels as the rows' image records (header + kept values, as
// k_rows_image_pack, 16-B rounded) back to back within a byte budget agreed in advance, and
// their counts. Record i sits at the exclusive prefix sum of the record sizes before it
// (rec_bytes of the counts), which sender and receiver compute alike from the counts; a
// row whose record ends past the budget, or has more than IMG_CAP kept values (its dense
// row is smaller), is an overflow row and travels dense after the rounds.
__device__ __forceinline__ uint64_t rec_bytes(unsigned t) {
    return t > (unsigned)IMG_CAP ? 0ull : (uint64_t)((128 + 4 * t + 15) / 16 * 16);
}
struct RecBytes {
    __device__ uint64_t operator()(uint32_t t) const { return rec_bytes(t); }
};

// counts (values other than +0.0) of rows r0 + i into cnt[i]; with acc: acc[0] += record
// bytes (dense bytes for a row past IMG_CAP), acc[1] += rows (the budget estimate of chunk 0)
__global__ __launch_bounds__(256) void k_rows_rec_count(const float* __restrict__ x, int64_t r0, int64_t rows, int dim,
                                                        uint32_t* __restrict__ cnt, unsigned long long* __restrict__ acc) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * ROWS_PER_BLOCK + w;
    if (i >= rows) return;
    const float* src = x + (r0 + i) * dim;
    int t = 0;
    for (int c = lane; c < dim; c += 64) t += aggrow::img_nz(src[c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (lane == 0) {
        cnt[i] = (uint32_t)t;
        if (acc) {
            const unsigned long long rb = rec_bytes((unsigned)t);
            atomicAdd(&acc[0], rb ? rb : (unsigned long long)(4 * dim));
            atomicAdd(&acc[1], 1ull);
        }
    }
}

// Row r0 + i's record at xs + off[i] when it fits the budget, else its global id appended to
// ovf_ids.
__global__ __launch_bounds__(256) void k_rows_xchg_pack(const float* __restrict__ x, int64_t r0, int64_t rows, int dim,
                                                        unsigned char* __restrict__ xs, uint64_t budget,
                                                        const uint32_t* __restrict__ cnt, const uint64_t* __restrict__ off,
                                                        int64_t* __restrict__ ovf_ids,
                                                        unsigned long long* __restrict__ ovf_n) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) f32x4 win[ROWS_PER_BLOCK][IMG_SLOT / 16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * ROWS_PER_BLOCK + w;
    if (i >= rows) return;
    const int64_t r = r0 + i;
    const uint64_t rb = rec_bytes(cnt[i]);
    if (rb == 0 || off[i] + rb > budget) {
        if (lane == 0) ovf_ids[atomicAdd(ovf_n, 1ull)] = r;
        return;
    }
    const float* src = x + r * dim;
    float4 v[3];
    unsigned h = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = 4 * lane + 256 * j < dim;
        v[j] = act ? *reinterpret_cast<const float4*>(src + 4 * lane + 256 * j) : make_float4(0, 0, 0, 0);
        const unsigned nib = aggrow::img_nz(v[j].x) | (aggrow::img_nz(v[j].y) << 1) | (aggrow::img_nz(v[j].z) << 2) |
                             (aggrow::img_nz(v[j].w) << 3);
        h |= (act ? nib : 0u) << (4 * j);
    }
    int p[3];
    unsigned tot;
    aggrow::img_positions(h, p, tot);
    unsigned char* wb = reinterpret_cast<unsigned char*>(win[w]);
    reinterpret_cast<uint16_t*>(wb)[lane] = (uint16_t)h;
    float* vals = reinterpret_cast<float*>(wb + 128);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
        int q = p[j];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if ((h >> (4 * j + k)) & 1u) vals[q++] = e[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int chunks = (int)(rb / 16);
    f32x4* dst = reinterpret_cast<f32x4*>(xs + off[i]);
    for (int c = lane; c < chunks; c += 64) dst[c] = win[w][c];
}

// The receiving side: record i back into the dense row r0 + i of x — every kept value's bits,
// +0.0 elsewhere, so the row equals the sender's — and, with an image, into that row's image
// slot. Overflow rows are left to the dense pass, which images them again (their image
// count is set past IMG_CAP meanwhile).
__global__ __launch_bounds__(256) void k_rows_xchg_unpack(float* __restrict__ x, int64_t r0, int64_t rows, int dim,
                                                          const unsigned char* __restrict__ xs, uint64_t budget,
                                                          const uint32_t* __restrict__ cnt,
                                                          const uint64_t* __restrict__ off,
                                                          unsigned char* __restrict__ slots,
                                                          uint16_t* __restrict__ nnz) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) f32x4 win[ROWS_PER_BLOCK][IMG_SLOT / 16 + 1];  // + slack for wf[p + 3]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * ROWS_PER_BLOCK + w;
    if (i >= rows) return;
    const int64_t r = r0 + i;
    const unsigned tot = cnt[i];
    const uint64_t rb = rec_bytes(tot);
    if (rb == 0 || off[i] + rb > budget) {
        if (nnz && lane == 0) nnz[r] = (uint16_t)(IMG_CAP + 1);
        return;
    }
    const int chunks = (int)(rb / 16);
    const f32x4* src = reinterpret_cast<const f32x4*>(xs + off[i]);
    for (int c = lane; c < chunks; c += 64) win[w][c] = src[c];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const unsigned char* wb = reinterpret_cast<const unsigned char*>(win[w]);
    const unsigned h = reinterpret_cast<const uint16_t*>(wb)[lane];
    int p[3];
    unsigned t2;
    aggrow::img_positions(h, p, t2);
    const float* wf = reinterpret_cast<const float*>(wb + 128);
    float* dst = x + r * dim;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (4 * lane + 256 * j >= dim) continue;
        const unsigned nib = (h >> (4 * j)) & 15u;
        const float w0 = wf[p[j]], w1 = wf[p[j] + 1], w2 = wf[p[j] + 2], w3 = wf[p[j] + 3];
        const bool b0 = nib & 1u, b1 = nib & 2u, b2 = nib & 4u, b3 = nib & 8u;
        const int q2 = (int)b0 + (int)b1, q3 = q2 + (int)b2;
        float4 e;
        e.x = b0 ? w0 : 0.0f;
        e.y = b1 ? (b0 ? w1 : w0) : 0.0f;
        e.z = b2 ? (q2 == 0 ? w0 : q2 == 1 ? w1 : w2) : 0.0f;
        e.w = b3 ? (q3 == 0 ? w0 : q3 == 1 ? w1 : q3 == 2 ? w2 : w3) : 0.0f;
        *reinterpret_cast<float4*>(dst + 4 * lane + 256 * j) = e;
    }
    if (slots) {
        f32x4* sd = reinterpret_cast<f32x4*>(slots + r * IMG_SLOT);
        for (int c = lane; c < chunks; c += 64) sd[c] = win[w][c];
        if (lane == 0) nnz[r] = (uint16_t)tot;
    }
}

// Dense rows by global id: gather (ids -> rows[cnt][dim]) or scatter (rows -> x[ids]); one
// block per row.
__global__ __launch_bounds__(192) void k_rows_by_id(float* __restrict__ x, int dim, const int64_t* __restrict__ ids,
                                                    float* __restrict__ rows, int scatter) {
    const int64_t i = blockIdx.x;
    const int64_t r = ids[i];
    for (int c = threadIdx.x; c < dim; c += blockDim.x) {
        if (scatter) x[r * dim + c] = rows[i * dim + c];
        else rows[i * dim + c] = x[r * dim + c];
    }
}
}  // namespace

void rows_rec_count(const float* x, int64_t r0, int64_t rows, int dim, uint32_t* cnt, unsigned long long* acc) {
    if (rows <= 0) return;
    RVX_LAUNCH("rows_rec_count", k_rows_rec_count, dim3((unsigned)((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK)),
               dim3(256), 0, x, r0, rows, dim, cnt, acc);
}

size_t rec_offsets_temp_bytes(int64_t rows) {
    size_t bytes = 0;
    rocprim::transform_iterator<const uint32_t*, RecBytes, uint64_t> in(nullptr, RecBytes());
    RVX_HIP(rocprim::exclusive_scan(nullptr, bytes, in, (uint64_t*)nullptr, (uint64_t)0,
                                    (size_t)std::max<int64_t>(rows, 1), rocprim::plus<uint64_t>(), stream()));
    return bytes;
}

void rec_offsets(const uint32_t* cnt, int64_t rows, uint64_t* off, void* temp, size_t temp_bytes) {
    if (rows <= 0) return;
    rocprim::transform_iterator<const uint32_t*, RecBytes, uint64_t> in(cnt, RecBytes());
    size_t bytes = temp_bytes;
    RVX_HIP(rocprim::exclusive_scan(temp, bytes, in, off, (uint64_t)0, (size_t)rows, rocprim::plus<uint64_t>(),
                                    stream()));
}

void rows_xchg_pack(const float* x, int64_t r0, int64_t rows, int dim, unsigned char* xs, uint64_t budget,
                    const uint32_t* cnt, const uint64_t* off, int64_t* ovf_ids, unsigned long long* ovf_n) {
    if (rows <= 0) return;
    RVX_REQUIRE(row_image_ok(dim) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)xs & 15) == 0, RVX_ERR_INVALID_SHAPE,
                "exchange records: bad arguments");
    RVX_LAUNCH("rows_xchg_pack", k_rows_xchg_pack, dim3((unsigned)((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK)),
               dim3(256), 0, x, r0, rows, dim, xs, budget, cnt, off, ovf_ids, ovf_n);
}

void rows_xchg_unpack(float* x, int64_t r0, int64_t rows, int dim, const unsigned char* xs, uint64_t budget,
                      const uint32_t* cnt, const uint64_t* off, const RowImage& img) {
    if (rows <= 0) return;
    RVX_REQUIRE(row_image_ok(dim) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)xs & 15) == 0, RVX_ERR_INVALID_SHAPE,
                "exchange records: bad arguments");
    RVX_LAUNCH("rows_xchg_unpack", k_rows_xchg_unpack, dim3((unsigned)((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK)),
               dim3(256), 0, x, r0, rows, dim, xs, budget, cnt, off, img.slots, img.nnz);
}

void rows_by_id(float* x, int dim, const int64_t* ids, int64_t cnt, float* rows, bool scatter) {
    if (cnt <= 0) return;
    RVX_LAUNCH("rows_by_id", k_rows_by_id, dim3((unsigned)cnt), dim3(192), 0, x, dim, ids, rows, scatter ? 1 : 0);
}

bool row_image_ok(int dim) { return dim > 512 && dim <= 768 && dim % 4 == 0; }

void rows_image_pack(const float* x, int64_t r0, int64_t rows, int dim, const RowImage& img) {
    if (rows <= 0) return;
    RVX_REQUIRE(img && row_image_ok(dim) && ((uintptr_t)x & 15) == 0, RVX_ERR_INVALID_SHAPE, "row image: bad arguments");
    RVX_LAUNCH("rows_image_pack", k_rows_image_pack, dim3((unsigned)((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK)),
               dim3(256), 0, x, r0, rows, dim, img.slots, img.nnz, (const int64_t*)nullptr);
}

void rows_image_pack_ids(const float* x, const int64_t* ids, int64_t cnt, int dim, const RowImage& img) {
    if (cnt <= 0) return;
    RVX_REQUIRE(img && row_image_ok(dim) && ((uintptr_t)x & 15) == 0, RVX_ERR_INVALID_SHAPE, "row image: bad arguments");
    RVX_LAUNCH("rows_image_pack", k_rows_image_pack, dim3((unsigned)((cnt + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK)),
               dim3(256), 0, x, (int64_t)0, cnt, dim, img.slots, img.nnz, ids);
}

bool agg_help_ok(int dim, const float* x, const float* out, const float* self_x) {
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    return env_int("RVX_SAGE_HELP", 1) && g_agg_overlap_unroll >= 8 && g_agg_nt && !env_int("RVX_AGG_ROLL", 0) &&
           dim > 0 && dim % 4 == 0 && dim <= 768 && al(x) && al(out) && self_x && al(self_x);
}

void aggregate_rows_help(const AggHelp& h, const char* tag, int blocks_per_cu) {
    if (h.n <= 0) return;
    RVX_REQUIRE(h.counter && h.agg >= AGG_SUM && h.agg <= AGG_MAX && h.dim % 4 == 0 && h.dim <= 768,
                RVX_ERR_INVALID_SHAPE, "dynamic gather: bad arguments");
    const int cap = blocks_per_cu > 0 ? blocks_per_cu : std::max(1, g_agg_overlap_cap);
    const int64_t blocks = std::min<int64_t>((h.n + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK,
                                             (int64_t)cap * active_cus());
    if (h.img_slots)
        RVX_LAUNCH(tag ? tag : "aggregate", k_aggregate_help<true>, dim3((unsigned)blocks), dim3(256),
                   h.img_reg ? 0 : ROWS_PER_BLOCK * IMG_WIN, h);  // register expansion: no LDS windows
    else
        RVX_LAUNCH(tag ? tag : "aggregate", k_aggregate_help<false>, dim3((unsigned)blocks), dim3(256), 0, h);
}

}  // namespace rvx
