// k_gnn.hip — the per-edge and per-node kernels of RuvectorLayer::forward,
// batched over a whole graph (crates/ruvector-gnn/src/layer.rs:379-451).
//
// The dense Linear layers run as MFMA GEMMs (gemm_f32.hip). What is left is
// per destination node i with CSR neighbours j (edge order):
//   K5 edge kernel (one wave per node):
//     score_hj = (q_ih · k_jh) / sqrt(head_dim)        (layer.rs:184-193)
//     a_hj = exp(s - max) / max(sum exp, 1e-10)         (layer.rs:196-199)
//     att_i[h] = sum_j a_hj v_jh                        (layer.rs:202-207)
//     wagg_i = sum_j w^_j m_j, w^ = w/sum(w) or 1/len   (layer.rs:421-445)
//   gate kernel  r ⊙ h                                  (layer.rs:265)
//   finish kernel (1-z)⊙h + z⊙h~, ×(1-dropout), LayerNorm (layer.rs:270-274, 448-451, 68-81)
// Every per-neighbour sum runs in CSR order, one sequential f32 chain per
// output element, like the reference loops. The q·k dot uses a lane tree.
//
// Traffic per edge: 3*H floats (k_j, v_j, m_j rows) + 4 B index (+4 B weight).
#include "common.hpp"
#include "gnn.hpp"
#include "kernels.hpp"

namespace rvx {
namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Weighted-aggregate normaliser for row [beg,end): mode 0 none, 1 raw weights,
// 2 pre-normalised weights.
__device__ __forceinline__ float row_weight_sum(const float* w, int64_t beg, int64_t end) {
    float s = 0.0f;
    for (int64_t e = beg; e < end; ++e) s = s + w[e];  // weights.iter().sum()
    return s;
}
__device__ __forceinline__ float norm_weight(int mode, const float* w, int64_t e, float wsum, int deg) {
    if (mode == 1) return wsum > 0.0f ? w[e] / wsum : 1.0f / (float)deg;
    return w[e];
}

// Fast path: H = 64*CPL, lane owns columns [lane*CPL, lane*CPL+CPL), a head is
// G = head_dim/CPL consecutive lanes (G a power of two). B edges' rows are loaded
// together before their arithmetic (B = 1: one edge at a time); each edge's dot and every
// running sum keep the same operations in the same order, so B does not change the bits.
template <int CPL, int B>
__global__ __launch_bounds__(256) void k_edge_attn_grouped(EdgeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int H = a.H, G = a.G;
    const int head = (lane * CPL) / a.hd;
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    const int deg = (int)(end - beg);
    float* scores = a.scores - a.rp[0] * a.heads;  // chunk-relative edge slots
    const int c0 = lane * CPL;
    float att[CPL], agg[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) { att[c] = 0.0f; agg[c] = 0.0f; }
    if (deg == 0) {
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
            *reinterpret_cast<float4*>(a.att + i * H + c0 + c) = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(a.wagg + i * H + c0 + c) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (a.att_amax && lane < ROWSUMSQ_SLOTS) a.att_amax[i * ROWSUMSQ_SLOTS + lane] = 0.0f;
        return;
    }
    float q[CPL];
#pragma unroll
    for (int c = 0; c < CPL; c += 4) {
        const float4 v = ld4(a.q + i * a.ldq + c0 + c);
        q[c] = v.x; q[c + 1] = v.y; q[c + 2] = v.z; q[c + 3] = v.w;
    }
    const float scale = sqrtf((float)a.hd);
    float mx = -INFINITY;
    // pass 1: scores
    auto score_of = [&](int64_t e, const float4 (&kv)[CPL / 4]) {
        float p = 0.0f;
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
            const float4 v = kv[c / 4];
            p = p + q[c] * v.x; p = p + q[c + 1] * v.y; p = p + q[c + 2] * v.z; p = p + q[c + 3] * v.w;
        }
        for (int o = 1; o < G; o <<= 1) p += __shfl_xor(p, o);
        const float s = p / scale;
        mx = fmaxf(mx, s);
        if ((lane & (G - 1)) == 0) scores[e * a.heads + head] = s;
    };
    int64_t e = beg;
    for (; e + B <= end; e += B) {
        float4 kv[B][CPL / 4];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const float* kr = a.k + (int64_t)a.col[e + b] * a.ldkv + c0;
#pragma unroll
            for (int c = 0; c < CPL; c += 4) kv[b][c / 4] = ld4(kr + c);
        }
#pragma unroll
        for (int b = 0; b < B; ++b) score_of(e + b, kv[b]);
    }
    for (; e < end; ++e) {
        float4 kv[CPL / 4];
        const float* kr = a.k + (int64_t)a.col[e] * a.ldkv + c0;
#pragma unroll
        for (int c = 0; c < CPL; c += 4) kv[c / 4] = ld4(kr + c);
        score_of(e, kv);
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    // pass 2: sum of exp in neighbour order
    float sum = 0.0f;
    for (int64_t e2 = beg; e2 < end; ++e2) sum = sum + expf(scores[e2 * a.heads + head] - mx);
    sum = fmaxf(sum, 1e-10f);
    float wsum = 0.0f;
    if (a.wmode == 1) wsum = row_weight_sum(a.w, beg, end);
    // pass 3: weighted sums of values and messages
    const bool msg = a.wmode != 0;
    auto accumulate = [&](int64_t e3, const float4 (&vv)[CPL / 4], const float4 (&mv)[CPL / 4]) {
        const float wt = expf(scores[e3 * a.heads + head] - mx) / sum;
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
            const float4 v = vv[c / 4];
            att[c] = att[c] + wt * v.x; att[c + 1] = att[c + 1] + wt * v.y;
            att[c + 2] = att[c + 2] + wt * v.z; att[c + 3] = att[c + 3] + wt * v.w;
        }
        if (msg) {
            const float ww = norm_weight(a.wmode, a.w, e3, wsum, deg);
#pragma unroll
            for (int c = 0; c < CPL; c += 4) {
                const float4 v = mv[c / 4];
                agg[c] = agg[c] + ww * v.x; agg[c + 1] = agg[c + 1] + ww * v.y;
                agg[c + 2] = agg[c + 2] + ww * v.z; agg[c + 3] = agg[c + 3] + ww * v.w;
            }
        }
    };
    auto load_vm = [&](int64_t e3, float4 (&vv)[CPL / 4], float4 (&mv)[CPL / 4]) {
        const int j = a.col[e3];
        const float* vr = a.v + (int64_t)j * a.ldkv + c0;
        const float* mr = a.m + (int64_t)j * H + c0;
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
            vv[c / 4] = ld4(vr + c);
            mv[c / 4] = msg ? ld4(mr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    e = beg;
    for (; e + B <= end; e += B) {
        float4 vv[B][CPL / 4], mv[B][CPL / 4];
#pragma unroll
        for (int b = 0; b < B; ++b) load_vm(e + b, vv[b], mv[b]);
#pragma unroll
        for (int b = 0; b < B; ++b) accumulate(e + b, vv[b], mv[b]);
    }
    for (; e < end; ++e) {
        float4 vv[CPL / 4], mv[CPL / 4];
        load_vm(e, vv, mv);
        accumulate(e, vv, mv);
    }
#pragma unroll
    for (int c = 0; c < CPL; c += 4) {
        *reinterpret_cast<float4*>(a.att + i * H + c0 + c) = make_float4(att[c], att[c + 1], att[c + 2], att[c + 3]);
        *reinterpret_cast<float4*>(a.wagg + i * H + c0 + c) = make_float4(agg[c], agg[c + 1], agg[c + 2], agg[c + 3]);
    }
    if (a.att_amax) {  // the out GEMM's split-f16 row scale, without a pass over att
        float mx2 = 0.0f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) mx2 = fmaxf(mx2, fabsf(att[c]));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx2 = fmaxf(mx2, __shfl_xor(mx2, o));
        if (lane < ROWSUMSQ_SLOTS) a.att_amax[i * ROWSUMSQ_SLOTS + lane] = lane == 0 ? mx2 : 0.0f;
    }
}

// Any H / heads: one wave per node. Scores: one lane per neighbour, a fully
// sequential dot over the head (the reference order); sums: lanes over columns.
__global__ __launch_bounds__(256) void k_edge_attn_generic(EdgeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int H = a.H, hd = a.hd, heads = a.heads;
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    const int deg = (int)(end - beg);
    float* scores = a.scores - a.rp[0] * heads;  // chunk-relative edge slots
    const float* qi = a.q + i * a.ldq;
    const float scale = sqrtf((float)hd);
    for (int64_t e = beg + lane; e < end; e += 64) {
        const float* kr = a.k + (int64_t)a.col[e] * a.ldkv;
        for (int h = 0; h < heads; ++h) {
            float p = 0.0f;
            for (int c = 0; c < hd; ++c) p = p + qi[h * hd + c] * kr[h * hd + c];
            scores[e * heads + h] = p / scale;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    float wsum = 0.0f;
    if (a.wmode == 1 && deg > 0) wsum = row_weight_sum(a.w, beg, end);
    for (int c = lane; c < H; c += 64) {
        const int h = c / hd;
        float mx = -INFINITY;
        for (int64_t e = beg; e < end; ++e) mx = fmaxf(mx, scores[e * heads + h]);
        float sum = 0.0f;
        for (int64_t e = beg; e < end; ++e) sum = sum + expf(scores[e * heads + h] - mx);
        sum = fmaxf(sum, 1e-10f);
        float at = 0.0f, ag = 0.0f;
        for (int64_t e = beg; e < end; ++e) {
            const int j = a.col[e];
            const float wt = expf(scores[e * heads + h] - mx) / sum;
            at = at + wt * a.v[(int64_t)j * a.ldkv + c];
            if (a.wmode != 0) ag = ag + norm_weight(a.wmode, a.w, e, wsum, deg) * a.m[(int64_t)j * H + c];
        }
        a.att[i * H + c] = at;
        a.wagg[i * H + c] = ag;
    }
}

// Folded attention (gnn.hpp EdgeFoldArgs), one wave per destination: lane owns
// columns [lane*CPL, lane*CPL+CPL) of every head's qt / u rows and of m_j, so
// an edge reads one H-float row. Scores: per head a lane partial over its
// columns + a full-wave tree; softmax per head in edge order (one lane per
// head: max, exp, sum, e/sum as layer.rs:196-199); u_h and the weighted
// message aggregate in edge order.
constexpr int FOLD_MAXH = 8;

template <int CPL>
__device__ __forceinline__ void ld_cols(const float* p, float (&v)[CPL]) {
    if constexpr (CPL % 4 == 0) {
#pragma unroll
        for (int c = 0; c < CPL; c += 4) {
            const float4 t = ld4(p + c);
            v[c] = t.x; v[c + 1] = t.y; v[c + 2] = t.z; v[c + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int c = 0; c < CPL; ++c) v[c] = p[c];
    }
}
template <int CPL>
__device__ __forceinline__ void st_cols(float* p, const float (&v)[CPL]) {
    if constexpr (CPL % 4 == 0) {
#pragma unroll
        for (int c = 0; c < CPL; c += 4) *reinterpret_cast<float4*>(p + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
    } else {
#pragma unroll
        for (int c = 0; c < CPL; ++c) p[c] = v[c];
    }
}
__device__ __forceinline__ float wave_sum(float p) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
    return p;
}

template <int CPL>
__global__ __launch_bounds__(256) void k_edge_attn_fold(EdgeFoldArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int H = a.H, heads = a.heads, hd = a.hd;
    const int c0 = lane * CPL;
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    const int deg = (int)(end - beg);
    float* scores = a.scores - a.rp[0] * heads;  // chunk-relative edge slots
    float* urow = a.u + i * (int64_t)heads * H + c0;
    float zero[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) zero[c] = 0.0f;
    if (deg == 0) {
        for (int h = 0; h < heads; ++h) st_cols<CPL>(urow + (int64_t)h * H, zero);
        st_cols<CPL>(a.wagg + i * H + c0, zero);
        return;
    }
    // q_h · b_k,h per head (the key bias folded out of the edge loop)
    float cb[FOLD_MAXH];
    {
        float qv[CPL], bv[CPL];
        ld_cols<CPL>(a.q + i * H + c0, qv);
        ld_cols<CPL>(a.bk + c0, bv);
#pragma unroll
        for (int h = 0; h < FOLD_MAXH; ++h) {
            float p = 0.0f;
            if (h < heads) {
#pragma unroll
                for (int c = 0; c < CPL; ++c) p = ((c0 + c) / hd == h) ? p + qv[c] * bv[c] : p;
                p = wave_sum(p);
            }
            cb[h] = p;
        }
    }
    const float scale = sqrtf((float)hd);
    float mx[FOLD_MAXH];
    {
        float qt[FOLD_MAXH][CPL];
#pragma unroll
        for (int h = 0; h < FOLD_MAXH; ++h) {
            if (h < heads) ld_cols<CPL>(a.qt + i * (int64_t)heads * H + (int64_t)h * H + c0, qt[h]);
            mx[h] = -INFINITY;
        }
        // pass 1: scores
        for (int64_t e = beg; e < end; ++e) {
            float mv[CPL];
            ld_cols<CPL>(a.m + (int64_t)a.col[e] * H + c0, mv);
#pragma unroll
            for (int h = 0; h < FOLD_MAXH; ++h) {
                if (h >= heads) continue;
                float p = 0.0f;
#pragma unroll
                for (int c = 0; c < CPL; ++c) p = p + qt[h][c] * mv[c];
                const float s = (wave_sum(p) + cb[h]) / scale;
                mx[h] = fmaxf(mx[h], s);
                if (lane == h) scores[e * heads + h] = s;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    // pass 2: lane h < heads runs head h's softmax in edge order
    if (lane < heads) {
        float m_h = mx[0];
#pragma unroll
        for (int h = 1; h < FOLD_MAXH; ++h)
            if (lane == h) m_h = mx[h];
        float sum = 0.0f;
        for (int64_t e = beg; e < end; ++e) {
            const float ex = expf(scores[e * heads + lane] - m_h);
            scores[e * heads + lane] = ex;
            sum = sum + ex;
        }
        sum = fmaxf(sum, 1e-10f);
        for (int64_t e = beg; e < end; ++e) scores[e * heads + lane] = scores[e * heads + lane] / sum;
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    // pass 3: u_h = sum_j a_jh m_j and the weighted message aggregate
    float u[FOLD_MAXH][CPL], agg[CPL];
#pragma unroll
    for (int h = 0; h < FOLD_MAXH; ++h)
#pragma unroll
        for (int c = 0; c < CPL; ++c) u[h][c] = 0.0f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) agg[c] = 0.0f;
    float wsum = 0.0f;
    if (a.wmode == 1) wsum = row_weight_sum(a.w, beg, end);
    for (int64_t e = beg; e < end; ++e) {
        float mv[CPL];
        ld_cols<CPL>(a.m + (int64_t)a.col[e] * H + c0, mv);
#pragma unroll
        for (int h = 0; h < FOLD_MAXH; ++h) {
            if (h >= heads) continue;
            const float wt = scores[e * heads + h];
#pragma unroll
            for (int c = 0; c < CPL; ++c) u[h][c] = u[h][c] + wt * mv[c];
        }
        if (a.wmode != 0) {
            const float ww = norm_weight(a.wmode, a.w, e, wsum, deg);
#pragma unroll
            for (int c = 0; c < CPL; ++c) agg[c] = agg[c] + ww * mv[c];
        }
    }
#pragma unroll
    for (int h = 0; h < FOLD_MAXH; ++h)
        if (h < heads) st_cols<CPL>(urow + (int64_t)h * H, u[h]);
    st_cols<CPL>(a.wagg + i * H + c0, agg);
}

__global__ void k_mul(const float* r, int64_t ldr, const float* h, float* out, int64_t n, int H) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n * H) return;
    const int64_t i = idx / H;
    const int c = (int)(idx % H);
    out[idx] = r[i * ldr + c] * h[idx];
}

// The same products one wave per row, also writing the row's max |out| (slot 0 of
// ROWSUMSQ_SLOTS, the others 0) for the next split-f16 GEMM's row scale.
__global__ __launch_bounds__(256) void k_mul_amax(const float* __restrict__ r, int64_t ldr, const float* __restrict__ h,
                                                 float* __restrict__ out, int64_t n, int H, float* __restrict__ amax) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    float m = 0.0f;
    for (int c = 4 * lane; c < H; c += 256) {
        const float4 a = *reinterpret_cast<const float4*>(r + i * ldr + c);
        const float4 b = *reinterpret_cast<const float4*>(h + i * (int64_t)H + c);
        const float4 o = make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
        *reinterpret_cast<float4*>(out + i * (int64_t)H + c) = o;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane < ROWSUMSQ_SLOTS) amax[i * ROWSUMSQ_SLOTS + lane] = lane == 0 ? m : 0.0f;
}

// (1-z)⊙h + z⊙h~, ×(1-dropout), LayerNorm; deg==0 rows: LayerNorm(m_i).
__global__ __launch_bounds__(256) void k_gru_finish(FinishArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int H = a.H;
    const bool iso = a.rp[i + 1] == a.rp[i];
    float* y = a.y + i * H;
    float s = 0.0f;
    for (int c = lane; c < H; c += 64) {
        float v;
        const float h = a.m[i * H + c];
        if (iso) v = h;
        else {
            const float z = a.zr[i * 2 * (int64_t)H + c];
            const float t1 = (1.0f - z) * h;
            const float t2 = z * a.ht[i * H + c];
            v = (t1 + t2) * a.keep;
        }
        y[c] = v;
        s += v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s / (float)H;
    float var = 0.0f;
    for (int c = lane; c < H; c += 64) { const float d = y[c] - mean; var += d * d; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) var += __shfl_xor(var, o);
    var = var / (float)H;
    const float den = sqrtf(var + a.eps);
    for (int c = lane; c < H; c += 64) y[c] = a.gamma[c] * ((y[c] - mean) / den) + a.beta[c];
}

// k_gru_finish with the row in registers (H = 64 NJ): element c = lane + 64 j as above, the
// three loads of every element issued before any arithmetic, the sums in the same j order and
// the same xor trees, y written once — the same bits as k_gru_finish.
template <int NJ>
__global__ __launch_bounds__(256) void k_gru_finish_reg(FinishArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    constexpr int H = 64 * NJ;
    const bool iso = a.rp[i + 1] == a.rp[i];
    const float* __restrict__ mr = a.m + i * H;
    const float* __restrict__ zr = a.zr + i * 2 * (int64_t)H;
    const float* __restrict__ hr = a.ht + i * H;
    float v[NJ];
    float s = 0.0f;
    if (iso) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) v[j] = mr[lane + 64 * j];
    } else {
        float hm[NJ], z[NJ], ht[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            hm[j] = mr[lane + 64 * j];
            z[j] = zr[lane + 64 * j];
            ht[j] = hr[lane + 64 * j];
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const float t1 = (1.0f - z[j]) * hm[j];
            const float t2 = z[j] * ht[j];
            v[j] = (t1 + t2) * a.keep;
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) s += v[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s / (float)H;
    float var = 0.0f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) { const float d = v[j] - mean; var += d * d; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) var += __shfl_xor(var, o);
    var = var / (float)H;
    const float den = sqrtf(var + a.eps);
    float* y = a.y + i * H;
#pragma unroll
    for (int j = 0; j < NJ; ++j) y[lane + 64 * j] = a.gamma[lane + 64 * j] * ((v[j] - mean) / den) + a.beta[lane + 64 * j];
}

}  // namespace

void edge_attention(const EdgeArgs& a) {
    if (a.n <= 0) return;
    const dim3 grid((unsigned)((a.n + 3) / 4)), block(256);
    const char* t = "gnn_edge_attention";
    const bool aligned = (((uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v | (uintptr_t)a.m | (uintptr_t)a.att |
                           (uintptr_t)a.wagg) & 15) == 0 && a.ldq % 4 == 0 && a.ldkv % 4 == 0;
    // RVX_EDGE_BATCH: edges whose rows are loaded together (1 or 4; same bits). 4 costs
    // occupancy (159 vs 80 VGPRs at CPL 12) and lost: 356-365 vs 330-337 ms of edge kernel per
    // 2M C4 step (scripts/exp_edge_batch.sh), so 1 stays the default.
    const bool b4 = env_int("RVX_EDGE_BATCH", 1) == 4;
    const bool grp = aligned && a.H % 64 == 0 && a.G > 0;
    if (grp && a.H / 64 == 4) RVX_LAUNCH(t, (b4 ? k_edge_attn_grouped<4, 4> : k_edge_attn_grouped<4, 1>), grid, block, 0, a);
    else if (grp && a.H / 64 == 8) RVX_LAUNCH(t, (b4 ? k_edge_attn_grouped<8, 4> : k_edge_attn_grouped<8, 1>), grid, block, 0, a);
    else if (grp && a.H / 64 == 12) RVX_LAUNCH(t, (b4 ? k_edge_attn_grouped<12, 4> : k_edge_attn_grouped<12, 1>), grid, block, 0, a);
    else if (grp && a.H / 64 == 16) RVX_LAUNCH(t, (b4 ? k_edge_attn_grouped<16, 4> : k_edge_attn_grouped<16, 1>), grid, block, 0, a);
    else {
        RVX_LAUNCH(t, k_edge_attn_generic, grid, block, 0, a);
        if (a.att_amax) row_absmax_pass(a.att, a.H, a.n, a.H, a.att_amax);
    }
}

bool edge_fold_ok(int H, int heads) {
    if (H % 64 != 0 || heads <= 0 || heads > FOLD_MAXH || H % heads != 0) return false;
    const int cpl = H / 64;
    return cpl == 1 || cpl == 2 || cpl == 4 || cpl == 8 || cpl == 12 || cpl == 16;
}

void edge_attention_fold(const EdgeFoldArgs& a) {
    if (a.n <= 0) return;
    RVX_REQUIRE(edge_fold_ok(a.H, a.heads), RVX_ERR_UNSUPPORTED, "folded attention needs H % 64 == 0, heads <= 8");
    const bool aligned = (((uintptr_t)a.q | (uintptr_t)a.qt | (uintptr_t)a.m | (uintptr_t)a.u | (uintptr_t)a.wagg |
                           (uintptr_t)a.bk) & 15) == 0;
    const int cpl = a.H / 64;
    RVX_REQUIRE(aligned || cpl % 4 != 0, RVX_ERR_INVALID_PARAMETER, "folded attention operands must be 16-B aligned");
    const dim3 grid((unsigned)((a.n + 3) / 4)), block(256);
    const char* t = "gnn_edge_attention";
    switch (cpl) {
        case 1: RVX_LAUNCH(t, k_edge_attn_fold<1>, grid, block, 0, a); break;
        case 2: RVX_LAUNCH(t, k_edge_attn_fold<2>, grid, block, 0, a); break;
        case 4: RVX_LAUNCH(t, k_edge_attn_fold<4>, grid, block, 0, a); break;
        case 8: RVX_LAUNCH(t, k_edge_attn_fold<8>, grid, block, 0, a); break;
        case 12: RVX_LAUNCH(t, k_edge_attn_fold<12>, grid, block, 0, a); break;
        default: RVX_LAUNCH(t, k_edge_attn_fold<16>, grid, block, 0, a); break;
    }
}

int edge_group_lanes(int H, int heads) {
    if (H % 64 != 0 || heads <= 0 || H % heads != 0) return 0;
    const int cpl = H / 64, hd = H / heads;
    if (cpl % 4 != 0 || hd % cpl != 0) return 0;
    const int g = hd / cpl;
    if (g > 64 || (g & (g - 1)) != 0) return 0;
    if (cpl != 4 && cpl != 8 && cpl != 12 && cpl != 16) return 0;
    return g;
}

void mul_rows(const float* r, int64_t ldr, const float* h, float* out, int64_t n, int H, float* amax) {
    const int64_t total = n * H;
    if (total <= 0) return;
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (amax && H % 4 == 0 && ldr % 4 == 0 && al(r) && al(h) && al(out)) {
        RVX_LAUNCH("gnn_gate_mul", k_mul_amax, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, r, ldr, h, out, n, H, amax);
        return;
    }
    RVX_LAUNCH("gnn_gate_mul", k_mul, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, r, ldr, h, out, n, H);
    if (amax) row_absmax_pass(out, H, n, H, amax);
}

void gru_finish(const FinishArgs& a) {
    if (a.n <= 0) return;
    const dim3 grid((unsigned)((a.n + 3) / 4)), block(256);
    // registers-resident row for H = 64 NJ (RVX_GNN_FINISH_REG=0 restores the loop form; same bits)
    const int nj = a.H % 64 == 0 && env_int("RVX_GNN_FINISH_REG", 1) ? a.H / 64 : 0;
    switch (nj) {
        case 1: RVX_LAUNCH("gnn_finish", k_gru_finish_reg<1>, grid, block, 0, a); return;
        case 2: RVX_LAUNCH("gnn_finish", k_gru_finish_reg<2>, grid, block, 0, a); return;
        case 4: RVX_LAUNCH("gnn_finish", k_gru_finish_reg<4>, grid, block, 0, a); return;
        case 8: RVX_LAUNCH("gnn_finish", k_gru_finish_reg<8>, grid, block, 0, a); return;
        case 12: RVX_LAUNCH("gnn_finish", k_gru_finish_reg<12>, grid, block, 0, a); return;
        case 16: RVX_LAUNCH("gnn_finish", k_gru_finish_reg<16>, grid, block, 0, a); return;
        default: break;
    }
    RVX_LAUNCH("gnn_finish", k_gru_finish, grid, block, 0, a);
}

namespace {

__global__ __launch_bounds__(256) void k_star_gather(const float* nodes, int64_t nq, const float* table, int64_t trows,
                                                     const int64_t* ids, int c, int d, float* dst) {
    const int64_t rows = (nodes ? nq : 0) + nq * c;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t base = nodes ? nq : 0;
    const float* src = nullptr;
    if (nodes && r < nq) src = nodes + r * d;
    else {
        const int64_t id = ids[r - base];
        if (id >= 0 && id < trows) src = table + id * d;
    }
    float* o = dst + r * d;
    if (!src) {
        for (int i = lane; i < d; i += 64) o[i] = 0.0f;
        return;
    }
    if ((d & 3) == 0 && (((uintptr_t)src | (uintptr_t)o) & 15) == 0) {
        for (int i = lane; i < d / 4; i += 64)
            reinterpret_cast<float4*>(o)[i] = reinterpret_cast<const float4*>(src)[i];
    } else {
        for (int i = lane; i < d; i += 64) o[i] = src[i];
    }
}

__global__ void k_star_degrees(const int64_t* ids, int64_t nq, int c, int64_t trows, int32_t* deg) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    int n = 0;
    for (int j = 0; j < c; ++j) {
        const int64_t id = ids[i * c + j];
        n += (id >= 0 && id < trows);
    }
    deg[i] = n;
}

__global__ void k_star_csr(const int64_t* ids, const float* w, int64_t nq, int c, int64_t trows, const int64_t* rp,
                           int32_t* col, float* wn) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    int64_t e = rp[i];
    const int deg = (int)(rp[i + 1] - rp[i]);
    float sum = 0.0f;
    if (w)
        for (int j = 0; j < c; ++j) {
            const int64_t id = ids[i * c + j];
            if (id >= 0 && id < trows) sum = sum + w[i * c + j];
        }
    for (int j = 0; j < c; ++j) {
        const int64_t id = ids[i * c + j];
        if (!(id >= 0 && id < trows)) continue;
        col[e] = (int32_t)(nq + i * c + j);
        if (w) wn[e] = sum > 0.0f ? w[i * c + j] / sum : 1.0f / (float)deg;
        ++e;
    }
}

}  // namespace

void star_gather(const float* nodes, int64_t nq, const float* table, int64_t trows, const int64_t* ids, int c, int d,
                 float* dst) {
    const int64_t rows = (nodes ? nq : 0) + nq * c;
    if (rows <= 0) return;
    RVX_LAUNCH("star_gather", k_star_gather, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, nodes, nq, table, trows,
               ids, c, d, dst);
}

void star_degrees(const int64_t* ids, int64_t nq, int c, int64_t trows, int32_t* deg) {
    if (nq <= 0) return;
    RVX_LAUNCH("star_csr", k_star_degrees, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, ids, nq, c, trows, deg);
}

void star_csr(const int64_t* ids, const float* w, int64_t nq, int c, int64_t trows, const int64_t* rp, int32_t* col,
              float* wn) {
    if (nq <= 0) return;
    RVX_LAUNCH("star_csr", k_star_csr, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, ids, w, nq, c, trows, rp, col,
               wn);
}

}  // namespace rvx
