// k_attn.hip — graph-attention head (EdgeFeaturedAttention) and the batched
// differentiable_search re-rank.
//
// EdgeFeaturedAttention::compute_with_edges
// (crates/ruvector-attention/src/graph/edge_featured.rs:196-258), per destination
// node with transformed rows T = X W_node^T precomputed by one MFMA GEMM:
//   score_hj = LeakyReLU( sum_c  tq[c]*a_src[c] + tk_j[c]*a_dst[c] + te_j[c]*a_edge[c] )
//     as ONE interleaved f32 chain over c (edge_featured.rs:177-183), te = W_edge e_ij
//   w_h = stable_softmax(score_h) (crates/ruvector-attention/src/utils.rs:11-54)
//   out_h[c] = sum_j w_hj tv_j[c] ; concat or mean over heads.
// Scores: one lane per edge, sequential over (head, c) in the reference order.
// Sums: lanes over output columns, sequential over neighbours.
//
// differentiable_search (crates/ruvector-gnn/src/search.rs:56-94): one wave per
// query, one lane per candidate: f32 dot + f64 norms (search.rs:4-26), softmax
// with temperature, stable descending sort, top-k.
#include "attn.hpp"
#include "common.hpp"

namespace rvx {
namespace {

// The score of edge (i, j) in head h is LeakyReLU of
//   sum_c tq_i[c] a_src[c] + tk_j[c] a_dst[c] + te_ij[c] a_edge[c],  c over the head,
// which the reference accumulates as one interleaved chain (edge_featured.rs:177-183).
// It is evaluated here as three separately summed parts: per-node head dots
// sq_i[h] = tq_i . a_src and sk_j[h] = tk_j . a_dst (one pass over T), and the
// edge term sum_k e_ij[k] u[h][k] with u = W_edge^T a_edge folded once per call
// — O(E heads) instead of O(E heads hd), reassociating one f32 sum (the 1e-5
// bar of the north star covers it; tests/test_gpu_parity.py).
__global__ void k_efa_row_dots(const float* __restrict__ t, int64_t ld, int64_t rows, int heads, int hd,
                               const float* __restrict__ av, float* __restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * heads) return;
    const int64_t r = idx / heads;
    const int h = (int)(idx % heads);
    const float* tr = t + r * ld + (int64_t)h * hd;
    const float* ar = av + (int64_t)h * hd;
    float s = 0.0f;
    for (int c = 0; c < hd; ++c) s = s + tr[c] * ar[c];
    out[idx] = s;
}

__global__ void k_efa_edge_u(const float* __restrict__ w_edge, const float* __restrict__ a_edge, int heads, int hd,
                             int ed, float* __restrict__ u) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= heads * ed) return;
    const int h = idx / ed, kk = idx % ed;
    float s = 0.0f;
    for (int c = 0; c < hd; ++c) s = s + w_edge[(int64_t)(h * hd + c) * ed + kk] * a_edge[h * hd + c];
    u[idx] = s;
}

__global__ __launch_bounds__(256) void k_edge_feat_scores(EfaArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int heads = a.heads, ed = a.edge_dim;
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    for (int64_t e = beg + lane; e < end; e += 64) {
        const int64_t j = a.col[e];
        const float* ef = a.edges ? a.edges + e * (int64_t)ed : nullptr;
        for (int h = 0; h < heads; ++h) {
            float te = 0.0f;
            if (ef)
                for (int kk = 0; kk < ed; ++kk) te = te + ef[kk] * a.u[h * ed + kk];
            const float score = (a.sq[i * heads + h] + a.sk[j * heads + h]) + te;
            a.scores[e * heads + h] = score < 0.0f ? a.slope * score : score;
        }
    }
}

// Scores and their stable_softmax in one pass (one wave per destination node): the lanes
// take the node's (edge, head) scores in storage order (coalesced stores, neighbour head dots
// read as runs), keep them in LDS, one lane per head runs the softmax's max / sequential sum /
// normalisation in edge order exactly as k_edge_feat_softmax, and the lanes store the weights.
// Same expressions, same order, same bits as the two-kernel form (RVX_EFA_FUSED=0); a node
// with more than EFA_LCAP (edge, head) scores writes raw scores for k_edge_feat_softmax.
constexpr int EFA_LCAP = 2048;
__global__ __launch_bounds__(256) void k_edge_feat_scores_sm(EfaArgs a) {
    __shared__ float sbuf[4][EFA_LCAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 4 + w;
    if (i >= a.n) return;
    const int heads = a.heads, ed = a.edge_dim;
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    const int64_t cnt = end - beg, tot = cnt * heads;
    const bool fused = tot <= EFA_LCAP;
    float* sb = sbuf[w];
    for (int64_t t = lane; t < tot; t += 64) {
        const int64_t e = beg + t / heads;
        const int h = (int)(t % heads);
        const int64_t j = a.col[e];
        float te = 0.0f;
        if (a.edges) {
            const float* ef = a.edges + e * (int64_t)ed;
            for (int kk = 0; kk < ed; ++kk) te = te + ef[kk] * a.u[h * ed + kk];
        }
        const float score = (a.sq[i * heads + h] + a.sk[j * heads + h]) + te;
        const float v = score < 0.0f ? a.slope * score : score;
        if (fused) sb[t] = v;
        else a.scores[beg * heads + t] = v;
    }
    if (!fused || cnt == 0) return;
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    for (int h = lane; h < heads; h += 64) {
        float mx = -INFINITY;
        for (int64_t e = 0; e < cnt; ++e) {
            const float v = sb[e * heads + h];
            if (isfinite(v)) mx = fmaxf(mx, v);
        }
        if (!isfinite(mx)) {
            for (int64_t e = 0; e < cnt; ++e) sb[e * heads + h] = 1.0f / (float)cnt;
            continue;
        }
        float sum = 0.0f;
        for (int64_t e = 0; e < cnt; ++e) {
            const float v = sb[e * heads + h];
            sum = sum + (isfinite(v) ? expf(v - mx) : 0.0f);
        }
        if (sum <= 1e-10f || !isfinite(sum)) {
            for (int64_t e = 0; e < cnt; ++e) sb[e * heads + h] = 1.0f / (float)cnt;
            continue;
        }
        const float inv = 1.0f / sum;
        for (int64_t e = 0; e < cnt; ++e) {
            const float v = sb[e * heads + h];
            sb[e * heads + h] = (isfinite(v) ? expf(v - mx) : 0.0f) * inv;
        }
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    for (int64_t t = lane; t < tot; t += 64) a.scores[beg * heads + t] = sb[t];
}

// stable_softmax per (node, head), in place over the score scratch. SKIP: nodes the fused
// kernel above already normalised (at most EFA_LCAP scores) are left alone.
template <bool SKIP>
__global__ void k_edge_feat_softmax(EfaArgs a) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n * a.heads) return;
    const int64_t i = t / a.heads;
    const int h = (int)(t % a.heads);
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    const int64_t cnt = end - beg;
    if (cnt == 0) return;
    if (SKIP && cnt * a.heads <= EFA_LCAP) return;
    float mx = -INFINITY;
    for (int64_t e = beg; e < end; ++e) {
        const float v = a.scores[e * a.heads + h];
        if (isfinite(v)) mx = fmaxf(mx, v);
    }
    if (!isfinite(mx)) {
        for (int64_t e = beg; e < end; ++e) a.scores[e * a.heads + h] = 1.0f / (float)cnt;
        return;
    }
    float sum = 0.0f;
    for (int64_t e = beg; e < end; ++e) {
        const float v = a.scores[e * a.heads + h];
        sum = sum + (isfinite(v) ? expf(v - mx) : 0.0f);
    }
    if (sum <= 1e-10f || !isfinite(sum)) {
        for (int64_t e = beg; e < end; ++e) a.scores[e * a.heads + h] = 1.0f / (float)cnt;
        return;
    }
    const float inv = 1.0f / sum;
    for (int64_t e = beg; e < end; ++e) {
        const float v = a.scores[e * a.heads + h];
        a.scores[e * a.heads + h] = (isfinite(v) ? expf(v - mx) : 0.0f) * inv;
    }
}

__global__ __launch_bounds__(256) void k_edge_feat_out(EfaArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int heads = a.heads, hd = a.hd, D = heads * hd;
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    if (a.concat) {
        for (int c = lane; c < D; c += 64) {
            const int h = c / hd;
            float acc = 0.0f;
            for (int64_t e = beg; e < end; ++e)
                acc = acc + a.scores[e * heads + h] * a.tv[(int64_t)a.col[e] * a.ldv + c];
            a.out[i * (int64_t)D + c] = acc;
        }
    } else {
        for (int c = lane; c < hd; c += 64) {
            float o = 0.0f;
            for (int h = 0; h < heads; ++h) {
                float acc = 0.0f;
                for (int64_t e = beg; e < end; ++e)
                    acc = acc + a.scores[e * heads + h] * a.tv[(int64_t)a.col[e] * a.ldv + h * hd + c];
                o = o + acc / (float)heads;
            }
            a.out[i * (int64_t)hd + c] = o;
        }
    }
}

// k_edge_feat_out's concat form with float4 rows: lane l of the node's wave owns columns
// 4(l + 64 v) .. +3 (v < NV), all in one head (hd % 4 == 0), and U edges' rows are in
// flight at once. Per column the sum is the same chain — edges ascending, product then
// add, from 0 — so the output bits equal the scalar kernel's.
template <int NV>
__global__ __launch_bounds__(256) void k_edge_feat_out_vec(EfaArgs a) {
    constexpr int U = NV <= 2 ? 8 : 4;
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int heads = a.heads, hd = a.hd, D4 = heads * hd / 4;
    const int64_t ldv4 = a.ldv / 4;
    const float4* __restrict__ tv4 = reinterpret_cast<const float4*>(a.tv);
    const int64_t beg = a.rp[i], end = a.rp[i + 1];
    int hv[NV];
    bool ok[NV];
    float4 acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c4 = lane + 64 * v;
        ok[v] = c4 < D4;
        hv[v] = ok[v] ? 4 * c4 / hd : 0;
        acc[v] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    auto add = [](float4& s, float w, const float4& t) {
        s.x = s.x + w * t.x;
        s.y = s.y + w * t.y;
        s.z = s.z + w * t.z;
        s.w = s.w + w * t.w;
    };
    int64_t e = beg;
    for (; e + U <= end; e += U) {
        float4 t[U][NV];
        float w[U][NV];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = a.col[e + u];
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (ok[v]) {
                    t[u][v] = tv4[j * ldv4 + lane + 64 * v];
                    w[u][v] = a.scores[(e + u) * heads + hv[v]];
                }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (ok[v]) add(acc[v], w[u][v], t[u][v]);
    }
    for (; e < end; ++e) {
        const int64_t j = a.col[e];
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (ok[v]) add(acc[v], a.scores[e * heads + hv[v]], tv4[j * ldv4 + lane + 64 * v]);
    }
    float4* o4 = reinterpret_cast<float4*>(a.out) + i * (int64_t)D4;
#pragma unroll
    for (int v = 0; v < NV; ++v)
        if (ok[v]) o4[lane + 64 * v] = acc[v];
}

// k_efa_row_dots with the rows staged through LDS: a block takes 8 rows (coalesced float4
// copies), then lane (row, head) runs the same sequential chain over its head's hd values.
__global__ __launch_bounds__(256) void k_efa_row_dots_lds(const float* __restrict__ t, int64_t ld, int64_t rows,
                                                          int heads, int hd, const float* __restrict__ av,
                                                          float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float rs[];  // [8][D + 1]
    const int D = heads * hd, D4 = D / 4, st = D + 4;
    const int64_t r0 = (int64_t)blockIdx.x * 8;
    for (int idx = threadIdx.x; idx < 8 * D4; idx += blockDim.x) {
        const int rr = idx / D4, c4 = idx % D4;
        if (r0 + rr < rows)
            *reinterpret_cast<float4*>(rs + rr * st + 4 * c4) =
                reinterpret_cast<const float4*>(t + (r0 + rr) * ld)[c4];
    }
    __syncthreads();
    for (int p = threadIdx.x; p < 8 * heads; p += blockDim.x) {
        const int rr = p / heads, h = p % heads;
        if (r0 + rr >= rows) continue;
        const float* tr = rs + rr * st + h * hd;
        const float* ar = av + (int64_t)h * hd;
        float s = 0.0f;
        for (int c = 0; c < hd; ++c) s = s + tr[c] * ar[c];
        out[(r0 + rr) * heads + h] = s;
    }
}

// ---- differentiable_search -------------------------------------------------
// One wave per query. cand rows of query qi start at cand + qi * cand_q_stride
// (stride C*d: per-query candidate lists; 0: one table shared by every query,
// hierarchical_forward's layer embeddings). Lanes split the candidates for the
// similarities, the max (order-free), the exps and the divisions; the softmax
// denominator is summed by lane 0 in candidate order (search.rs:41 `.sum()`),
// so every weight is the reference's value. The top-k (stable descending sort,
// search.rs:80-88) is k rounds of a wave arg-max under (weight desc, index asc).
__device__ __forceinline__ bool ds_better(float w, int j, float bw, int bj) {
    return bj < 0 || w > bw || (w == bw && j < bj);
}

__global__ __launch_bounds__(64) void k_diff_search(const float* q, int64_t nq, const float* cand,
                                                    int64_t cand_q_stride, int C, int d, int k, float temperature,
                                                    float* sims, int64_t* out_idx, float* out_w, float* soft) {
    const int lane = threadIdx.x;
    const int64_t qi = blockIdx.x;
    if (qi >= nq) return;
    const float* qv = q + qi * d;
    const float* cq = cand + qi * cand_q_stride;
    float* s = sims + qi * C;
    // rows as float4 when they allow it: the same sequential sums, a quarter of the loads
    const bool v4 = (d & 3) == 0 && ((uintptr_t)qv & 15) == 0 && ((uintptr_t)cq & 15) == 0;
    double qn2 = 0.0;
    if (v4) {
        for (int c = 0; c < d; c += 4) {
            const float4 a = *reinterpret_cast<const float4*>(qv + c);
            qn2 = qn2 + (double)a.x * (double)a.x; qn2 = qn2 + (double)a.y * (double)a.y;
            qn2 = qn2 + (double)a.z * (double)a.z; qn2 = qn2 + (double)a.w * (double)a.w;
        }
    } else {
        for (int c = 0; c < d; ++c) qn2 = qn2 + (double)qv[c] * (double)qv[c];
    }
    const float na = (float)sqrt(qn2);
    float mx = -INFINITY;
    for (int j = lane; j < C; j += 64) {
        const float* cv = cq + (int64_t)j * d;
        float dot = 0.0f;
        double n2 = 0.0;
        if (v4) {
            for (int c = 0; c < d; c += 4) {
                const float4 a = *reinterpret_cast<const float4*>(qv + c);
                const float4 b = *reinterpret_cast<const float4*>(cv + c);
                dot = dot + a.x * b.x; n2 = n2 + (double)b.x * (double)b.x;
                dot = dot + a.y * b.y; n2 = n2 + (double)b.y * (double)b.y;
                dot = dot + a.z * b.z; n2 = n2 + (double)b.z * (double)b.z;
                dot = dot + a.w * b.w; n2 = n2 + (double)b.w * (double)b.w;
            }
        } else {
            for (int c = 0; c < d; ++c) {
                dot = dot + qv[c] * cv[c];
                n2 = n2 + (double)cv[c] * (double)cv[c];
            }
        }
        const float nb = (float)sqrt(n2);
        const float sim = (na == 0.0f || nb == 0.0f) ? 0.0f : dot / (na * nb);
        s[j] = sim;
        mx = fmaxf(mx, sim);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    // softmax with temperature (search.rs:29-44)
    for (int j = lane; j < C; j += 64) s[j] = expf((s[j] - mx) / temperature);
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    float sum = 0.0f;
    if (lane == 0) {
        for (int j = 0; j < C; ++j) sum = sum + s[j];
        sum = fmaxf(sum, 1e-10f);
    }
    sum = __shfl(sum, 0);
    for (int j = lane; j < C; j += 64) {
        const float w = s[j] / sum;
        s[j] = w;
        if (soft) soft[qi * C + j] = w;
    }
    if (k == 0) return;
    // stable sort by weight descending (ties keep index order), take k; NaN
    // weights (no order in partial_cmp) are never taken
    const int kk = min(k, C);
    for (int t = 0; t < k; ++t) {
        int bj = -1;
        float bw = 0.0f;
        if (t < kk)
            for (int j = lane; j < C; j += 64) {
                const float w = s[j];
                if (w != w || w == -INFINITY) continue;  // NaN or consumed
                if (ds_better(w, j, bw, bj)) { bj = j; bw = w; }
            }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int oj = __shfl_xor(bj, o);
            const float ow = __shfl_xor(bw, o);
            if (oj >= 0 && ds_better(ow, oj, bw, bj)) { bj = oj; bw = ow; }
        }
        if (lane == 0) {
            out_idx[qi * k + t] = bj;
            out_w[qi * k + t] = bj < 0 ? 0.0f : bw;
        }
        if (bj >= 0 && (bj & 63) == lane) s[bj] = -INFINITY;  // consumed (owner lane rereads it)
    }
}

// hierarchical_forward's combine (search.rs:132-148): agg = sum_t w_t * row(idx_t)
// accumulated in top-k order from 0, combined = (cur + agg) / 2. Lanes over
// columns, one block per query.
__global__ __launch_bounds__(256) void k_hier_combine(const float* cur, int64_t nq, const float* table, int d,
                                                      const int64_t* idx, const float* w, int k, float* comb) {
    const int64_t qi = blockIdx.x;
    if (qi >= nq) return;
    for (int c = threadIdx.x; c < d; c += blockDim.x) {
        float agg = 0.0f;
        for (int t = 0; t < k; ++t) {
            const int64_t j = idx[qi * k + t];
            if (j < 0) continue;
            const float p = w[qi * k + t] * table[j * d + c];
            agg = agg + p;
        }
        comb[qi * d + c] = (cur[qi * d + c] + agg) / 2.0f;
    }
}

}  // namespace

void edge_feat_attention(const EfaArgs& a) {
    if (a.n <= 0) return;
    const int64_t nq = a.n * a.heads, nkh = a.nk * a.heads;
    const int D = a.heads * a.hd;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    // row dots through LDS when rows are float4-aligned and 8 of them fit 64 KB (<= 2040 columns)
    auto row_dots = [&](const float* t, int64_t ld, int64_t rows, const float* av, float* out) {
        if (rows <= 0) return;
        if (D % 4 == 0 && ld % 4 == 0 && al16(t) && D <= 2040 && env_int("RVX_EFA_VEC", 1)) {
            const size_t lds = (size_t)8 * (D + 4) * sizeof(float);
            RVX_LAUNCH("efa_node_dots", k_efa_row_dots_lds, dim3((unsigned)((rows + 7) / 8)), dim3(256), lds, t, ld,
                       rows, a.heads, a.hd, av, out);
        } else {
            RVX_LAUNCH("efa_node_dots", k_efa_row_dots, dim3((unsigned)((rows * a.heads + 255) / 256)), dim3(256), 0, t,
                       ld, rows, a.heads, a.hd, av, out);
        }
    };
    row_dots(a.tq, a.ldq, a.n, a.a_src, a.sq);
    if (nkh > 0) row_dots(a.tk, a.ldk, a.nk, a.a_dst, a.sk);
    if (a.edges && a.edge_dim > 0) {
        const int nu = a.heads * a.edge_dim;
        RVX_LAUNCH("efa_node_dots", k_efa_edge_u, dim3((unsigned)((nu + 255) / 256)), dim3(256), 0, a.w_edge, a.a_edge,
                   a.heads, a.hd, a.edge_dim, a.u);
    }
    // scores + softmax fused (RVX_EFA_FUSED=1, default; read per call): the second kernel then only
    // takes nodes past EFA_LCAP scores
    if (env_int("RVX_EFA_FUSED", 1)) {
        RVX_LAUNCH("efa_scores", k_edge_feat_scores_sm, dim3((unsigned)((a.n + 3) / 4)), dim3(256), 0, a);
        RVX_LAUNCH("efa_softmax", k_edge_feat_softmax<true>, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, a);
    } else {
        RVX_LAUNCH("efa_scores", k_edge_feat_scores, dim3((unsigned)((a.n + 3) / 4)), dim3(256), 0, a);
        RVX_LAUNCH("efa_softmax", k_edge_feat_softmax<false>, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, a);
    }
    const bool vec = a.concat && a.hd % 4 == 0 && a.ldv % 4 == 0 && al16(a.tv) && al16(a.out) && D <= 1024 &&
                     env_int("RVX_EFA_VEC", 1);
    const dim3 og((unsigned)((a.n + 3) / 4)), ob(256);
    if (vec && D <= 256) RVX_LAUNCH("efa_out", k_edge_feat_out_vec<1>, og, ob, 0, a);
    else if (vec && D <= 512) RVX_LAUNCH("efa_out", k_edge_feat_out_vec<2>, og, ob, 0, a);
    else if (vec && D <= 768) RVX_LAUNCH("efa_out", k_edge_feat_out_vec<3>, og, ob, 0, a);
    else if (vec) RVX_LAUNCH("efa_out", k_edge_feat_out_vec<4>, og, ob, 0, a);
    else RVX_LAUNCH("efa_out", k_edge_feat_out, og, ob, 0, a);
}

void differentiable_search(const float* q, int64_t nq, const float* cand, int C, int d, int k, float temperature,
                           float* sims, int64_t* out_idx, float* out_w, float* soft, bool shared_table) {
    if (nq <= 0) return;
    RVX_LAUNCH("differentiable_search", k_diff_search, dim3((unsigned)nq), dim3(64), 0, q, nq, cand,
               shared_table ? (int64_t)0 : (int64_t)C * d, C, d, k, temperature, sims, out_idx, out_w, soft);
}

void hier_combine(const float* cur, int64_t nq, const float* table, int d, const int64_t* idx, const float* w, int k,
                  float* comb) {
    if (nq <= 0) return;
    RVX_LAUNCH("hier_combine", k_hier_combine, dim3((unsigned)nq), dim3(256), 0, cur, nq, table, d, idx, w, k, comb);
}


namespace {
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// One wave per row: |row|, project_to_ball in place, |row|^2 after.
__global__ __launch_bounds__(256) void k_dsa_ball(float* __restrict__ t, int64_t rows, int dim, float curvature,
                                                 float* __restrict__ nh) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    float* x = t + r * dim;
    float s = 0.0f;
    for (int k = lane; k < dim; k += 64) s += x[k] * x[k];
    s = wave_sum(s);
    const float c = fabsf(curvature);
    const float norm_x = sqrtf(s);
    const float max_norm = (1.0f / sqrtf(c)) - 1e-5f;
    if (norm_x >= max_norm) {
        const float sc = max_norm / fmaxf(norm_x, 1e-7f);
        float s2 = 0.0f;
        for (int k = lane; k < dim; k += 64) {
            const float v = sc * x[k];
            x[k] = v;
            s2 += v * v;
        }
        s = wave_sum(s2);
    }
    if (lane == 0) nh[r] = s;
}

// One wave per destination row: per-edge combined score (Euclidean dot * scale and
// -poincare_dist, dual_space.rs:14-27, 160-168, 231-244; every lane holds it after
// the wave reductions), stable_softmax (utils.rs:11-54) folded into one pass as a
// running max with rescaled sums (non-finite scores weigh 0; no finite score ->
// uniform weights), and the weighted sum of the value rows. value_dim <= 1024.
constexpr int DSA_VPL = 16;  // value elements per lane
__global__ __launch_bounds__(256) void k_dsa_rows(DsaArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int64_t b = a.rp[i], e = a.rp[i + 1];
    float* o = a.out + i * a.value_dim;
    const float* teq = a.te_q + i * a.dim;
    const float* thq = a.th_q + i * a.dim;
    const float nq = a.nh_q[i];
    const float c = fabsf(a.curvature);
    float acc[DSA_VPL], plain[DSA_VPL];
#pragma unroll
    for (int t = 0; t < DSA_VPL; ++t) { acc[t] = 0.0f; plain[t] = 0.0f; }
    float m = -INFINITY, sum = 0.0f;
    for (int64_t p = b; p < e; ++p) {
        const int64_t j = a.col[p];
        const float* tek = a.te_k + j * a.dim;
        const float* thk = a.th_k + j * a.dim;
        float dot = 0.0f, diff = 0.0f;
        for (int k = lane; k < a.dim; k += 64) {
            dot += teq[k] * tek[k];
            const float d = thq[k] - thk[k];
            diff += d * d;
        }
        dot = wave_sum(dot);
        diff = wave_sum(diff);
        const float denom = fmaxf(1.0f - c * nq, 1e-7f) * fmaxf(1.0f - c * a.nh_k[j], 1e-7f);
        const float arg = 1.0f + 2.0f * c * diff / denom;
        const float hyp = -((1.0f / sqrtf(c)) * acoshf(fmaxf(arg, 1.0f)));
        const float s = (a.euclidean_weight * (dot * a.scale) + a.hyperbolic_weight * hyp) / a.temperature;
        const float* vr = a.val + j * a.ldv;
        float w = 0.0f, r = 1.0f;
        if (__builtin_isfinite(s)) {
            if (s > m) { r = (m == -INFINITY) ? 0.0f : expf(m - s); m = s; w = 1.0f; }
            else w = expf(s - m);
        }
        sum = sum * r + w;
#pragma unroll
        for (int t = 0; t < DSA_VPL; ++t) {
            const int k = lane + 64 * t;
            if (k < a.value_dim) {
                const float v = vr[k];
                acc[t] = acc[t] * r + w * v;
                plain[t] = plain[t] + v;
            }
        }
    }
    const int64_t deg = e - b;
    const bool uniform = m == -INFINITY || sum <= 1e-10f || !__builtin_isfinite(sum);
#pragma unroll
    for (int t = 0; t < DSA_VPL; ++t) {
        const int k = lane + 64 * t;
        if (k < a.value_dim) o[k] = deg == 0 ? 0.0f : uniform ? plain[t] * (1.0f / (float)deg) : acc[t] / sum;
    }
}
}  // namespace

void dsa_project_rows(float* t, int64_t rows, int dim, float curvature, float* nh) {
    if (rows <= 0) return;
    RVX_LAUNCH("dsa_ball", k_dsa_ball, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, t, rows, dim, curvature, nh);
}

void dual_space_attention(const DsaArgs& a) {
    if (a.n <= 0) return;
    RVX_LAUNCH("dsa_rows", k_dsa_rows, dim3((unsigned)((a.n + 3) / 4)), dim3(256), 0, a);
}

}  // namespace rvx
