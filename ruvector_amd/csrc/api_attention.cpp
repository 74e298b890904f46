// api_attention.cpp — EdgeFeaturedAttention (crates/ruvector-attention/src/graph/edge_featured.rs)
// and the batched differentiable_search (crates/ruvector-gnn/src/search.rs:56-94).
#include <cmath>

#include "attn.hpp"
#include "comm.hpp"
#include "gnn.hpp"
#include "graph.hpp"
#include "kernels.hpp"

using namespace rvx;

struct rvx_edge_attention {
    rvx_edge_attention_config cfg{};
    int hd = 0, D = 0;
    std::vector<float> w_node, w_edge, a_src, a_dst, a_edge;
    DevMem d_wnode, d_wedge, d_asrc, d_adst, d_aedge;
    DevMem d_wnode_x3;  // exact 3-way bf16 split of W_node (split-bf16 MFMA GEMM)
};

struct rvx_dual_attention {
    rvx_dual_attention_config cfg{};
    std::vector<float> w_euc, w_hyp, w_out;  // [dim][dim] = [out][in]
    DevMem d_w[3], d_x3[3];                  // f32 and exact 3-way bf16 splits (split-bf16 GEMM)
};

namespace {

void upload_vec(DevMem& d, const std::vector<float>& v) {
    d.reset((int64_t)std::max<size_t>(v.size(), 1) * 4);
    d.upload(v.data(), (int64_t)v.size() * 4);
}

// One destination row per query row q of `tq`, neighbours given by rp/col.
void run_efa(const rvx_edge_attention* a, int64_t n, const int64_t* rp, const int32_t* col, int64_t E, const float* tq,
             int64_t nk, const float* tk, const float* tv, const float* edges, float* out) {
    EfaArgs ea;
    ea.n = n; ea.heads = a->cfg.num_heads; ea.hd = a->hd; ea.edge_dim = a->cfg.edge_dim;
    ea.concat = a->cfg.concat_heads ? 1 : 0; ea.slope = a->cfg.negative_slope;
    ea.rp = rp; ea.col = col;
    ea.tq = tq; ea.ldq = a->D; ea.tk = tk; ea.ldk = a->D; ea.tv = tv; ea.ldv = a->D;
    ea.edges = (a->cfg.edge_dim > 0) ? edges : nullptr;
    ea.w_edge = a->d_wedge.as<float>();
    ea.a_src = a->d_asrc.as<float>(); ea.a_dst = a->d_adst.as<float>(); ea.a_edge = a->d_aedge.as<float>();
    ea.scores = scratch_f32("efa_scores", std::max<int64_t>(E, 1) * a->cfg.num_heads);
    ea.out = out;
    ea.nk = nk;
    ea.sq = scratch_f32("efa_sq", std::max<int64_t>(n, 1) * a->cfg.num_heads);
    ea.sk = scratch_f32("efa_sk", std::max<int64_t>(nk, 1) * a->cfg.num_heads);
    ea.u = scratch_f32("efa_u", (int64_t)a->cfg.num_heads * std::max(a->cfg.edge_dim, 1));
    edge_feat_attention(ea);
}

void transform(const rvx_edge_attention* a, const float* x, int64_t rows, float* t, const char* tag) {
    // transform_node for every head at once: T = X W_node^T, W_node [heads*hd][node_dim]
    gemm_nt(rows, a->D,
            GemmOperand{x, a->cfg.node_dim, a->d_wnode.as<float>(), a->cfg.node_dim, a->cfg.node_dim,
                        a->d_wnode_x3.as<uint16_t>(), (int64_t)a->D * a->cfg.node_dim},
            nullptr, GemmEpilogue(), t, a->D, tag);
}

// C = X · W^T for one of the three DualSpaceAttention matrices (0 euc, 1 hyp, 2 out).
void dsa_gemm(const rvx_dual_attention* a, int w, const float* x, int64_t rows, float* c, const char* tag) {
    const int d = a->cfg.dim;
    gemm_nt(rows, d, GemmOperand{x, d, a->d_w[w].as<float>(), d, d, a->d_x3[w].as<uint16_t>(), (int64_t)d * d},
            nullptr, GemmEpilogue(), c, d, tag);
}

// te = x W_euc^T, th = project_to_ball(x W_hyp^T), nh = |th|^2 for `rows` rows.
void dsa_transform(const rvx_dual_attention* a, const float* x, int64_t rows, float* te, float* th, float* nh) {
    dsa_gemm(a, 0, x, rows, te, "dsa_transform");
    dsa_gemm(a, 1, x, rows, th, "dsa_transform");
    dsa_project_rows(th, rows, a->cfg.dim, a->cfg.curvature, nh);
}

DsaArgs dsa_args(const rvx_dual_attention* a) {
    DsaArgs da;
    da.dim = a->cfg.dim;
    da.curvature = a->cfg.curvature;
    da.euclidean_weight = a->cfg.euclidean_weight;
    da.hyperbolic_weight = a->cfg.hyperbolic_weight;
    da.temperature = a->cfg.temperature;
    da.scale = 1.0f / std::sqrt((float)a->cfg.dim);  // DualSpaceAttention::new (dual_space.rs:109)
    return da;
}

}  // namespace

extern "C" {

rvx_status rvx_dual_attention_create(const rvx_dual_attention_config* cfg, rvx_dual_attention** out) {
    return guard([&] {
        RVX_REQUIRE(cfg && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(cfg->dim > 0 && cfg->dim <= 1024, RVX_ERR_INVALID_PARAMETER, "dim must be in [1, 1024]");
        auto a = std::make_unique<rvx_dual_attention>();
        a->cfg = *cfg;
        const int64_t d = cfg->dim;
        // DualSpaceAttention::new (dual_space.rs:107-131): one LCG stream, seed 42
        const float w_scale = std::sqrt(2.0f / (float)(d + d));
        uint64_t seed = 42;
        auto rnd = [&]() {
            seed = seed * 6364136223846793005ull + 1ull;
            return ((float)seed / (float)UINT64_MAX - 0.5f) * 2.0f * w_scale;
        };
        for (auto* w : {&a->w_euc, &a->w_hyp, &a->w_out}) {
            w->resize(d * d);
            for (auto& v : *w) v = rnd();
        }
        const std::vector<float>* ws[3] = {&a->w_euc, &a->w_hyp, &a->w_out};
        for (int i = 0; i < 3; ++i) {
            upload_vec(a->d_w[i], *ws[i]);
            a->d_x3[i].reset(std::max<int64_t>(d * d, 1) * 6);
            split_x3(a->d_w[i].as<float>(), d * d, a->d_x3[i].as<uint16_t>());
        }
        sync();
        *out = a.release();
    });
}

rvx_status rvx_dual_attention_destroy(rvx_dual_attention* a) {
    return guard([&] { delete a; });
}

rvx_status rvx_dual_attention_compute(const rvx_dual_attention* a, const float* query, const float* keys,
                                      const float* values, int32_t n, int32_t value_dim, float* out) {
    return guard([&] {
        RVX_REQUIRE(a && query && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(n > 0, RVX_ERR_INVALID_PARAMETER, "Empty keys");  // dual_space.rs:213-215
        RVX_REQUIRE(keys && values && value_dim > 0 && value_dim <= 1024, RVX_ERR_INVALID_PARAMETER,
                    "bad keys/values");
        ComputeLock cl;
        const int64_t d = a->cfg.dim;
        float* dq = scratch_f32("dsa1_q", d);
        float* dk = scratch_f32("dsa1_k", n * d);
        float* dv = scratch_f32("dsa1_v", (int64_t)n * value_dim);
        float* teq = scratch_f32("dsa1_teq", d);
        float* thq = scratch_f32("dsa1_thq", d);
        float* tek = scratch_f32("dsa1_tek", n * d);
        float* thk = scratch_f32("dsa1_thk", n * d);
        float* nh = scratch_f32("dsa1_nh", n + 1);
        float* o1 = scratch_f32("dsa1_o1", std::max<int64_t>(value_dim, d));
        float* o2 = scratch_f32("dsa1_o2", d);
        auto* rp = (int64_t*)scratch_bytes("dsa1_rp", 16);
        auto* col = (int32_t*)scratch_bytes("dsa1_col", (int64_t)n * 4);
        std::vector<int64_t> hrp{0, n};
        std::vector<int32_t> hcol(n);
        for (int j = 0; j < n; ++j) hcol[j] = j;
        RVX_HIP(hipMemcpyAsync(dq, query, (size_t)d * 4, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(dk, keys, (size_t)(n * d * 4), hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(dv, values, (size_t)n * value_dim * 4, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(rp, hrp.data(), 16, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(col, hcol.data(), (size_t)n * 4, hipMemcpyHostToDevice, stream()));
        dsa_transform(a, dq, 1, teq, thq, nh + n);
        dsa_transform(a, dk, n, tek, thk, nh);
        DsaArgs da = dsa_args(a);
        da.n = 1; da.value_dim = value_dim; da.rp = rp; da.col = col;
        da.te_q = teq; da.th_q = thq; da.nh_q = nh + n;
        da.te_k = tek; da.th_k = thk; da.nh_k = nh;
        da.val = dv; da.ldv = value_dim; da.out = o1;
        dual_space_attention(da);
        const bool proj = value_dim == a->cfg.dim;  // dual_space.rs:263-267
        if (proj) dsa_gemm(a, 2, o1, 1, o2, "dsa_out");
        RVX_HIP(hipMemcpyAsync(out, proj ? o2 : o1, (size_t)value_dim * 4, hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_dual_attention_forward_graph_device(const rvx_dual_attention* a, const rvx_graph* g,
                                                   const rvx_buffer* x, rvx_buffer* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(a && x && y, RVX_ERR_INVALID_PARAMETER, "null argument");
        const int64_t d = a->cfg.dim, n = g->n;
        RVX_REQUIRE(x->mem.bytes >= n * d * 4 && y->mem.bytes >= n * d * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "x / y smaller than n*dim");
        ComputeLock cl;
        float* te = scratch_f32("dsa_te", n * d);
        float* th = scratch_f32("dsa_th", n * d);
        float* nh = scratch_f32("dsa_nh", std::max<int64_t>(n, 1));
        float* o1 = scratch_f32("dsa_o1", n * d);
        dsa_transform(a, x->mem.as<float>(), n, te, th, nh);
        DsaArgs da = dsa_args(a);
        da.n = n; da.value_dim = (int)d; da.rp = g->row_ptr; da.col = g->col;
        da.te_q = te; da.th_q = th; da.nh_q = nh;
        da.te_k = te; da.th_k = th; da.nh_k = nh;
        da.val = x->mem.as<float>(); da.ldv = d; da.out = o1;
        dual_space_attention(da);
        dsa_gemm(a, 2, o1, n, y->mem.as<float>(), "dsa_out");
    });
}

rvx_status rvx_edge_attention_create(const rvx_edge_attention_config* cfg, rvx_edge_attention** out) {
    return guard([&] {
        RVX_REQUIRE(cfg && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(cfg->node_dim > 0 && cfg->num_heads > 0 && cfg->edge_dim >= 0, RVX_ERR_INVALID_PARAMETER,
                    "bad EdgeFeaturedConfig");
        RVX_REQUIRE(cfg->node_dim / cfg->num_heads > 0, RVX_ERR_INVALID_PARAMETER, "num_heads > node_dim");
        auto a = std::make_unique<rvx_edge_attention>();
        a->cfg = *cfg;
        const int hd = cfg->node_dim / cfg->num_heads;  // EdgeFeaturedConfig::head_dim
        a->hd = hd;
        a->D = hd * cfg->num_heads;
        // EdgeFeaturedAttention::new (edge_featured.rs:98-141): LCG seed 42.
        const float node_scale = std::sqrt(2.0f / (float)(cfg->node_dim + hd));
        const float edge_scale = std::sqrt(2.0f / (float)(cfg->edge_dim + hd));
        const float attn_scale = std::sqrt(1.0f / (float)hd);
        uint64_t seed = 42;
        auto rnd = [&]() {
            seed = seed * 6364136223846793005ull + 1ull;
            return (float)seed / (float)UINT64_MAX - 0.5f;
        };
        const int64_t H = cfg->num_heads;
        a->w_node.resize(H * hd * cfg->node_dim);
        for (auto& v : a->w_node) v = rnd() * 2.0f * node_scale;
        a->w_edge.resize(H * hd * cfg->edge_dim);
        for (auto& v : a->w_edge) v = rnd() * 2.0f * edge_scale;
        a->a_src.resize(H * hd);
        for (auto& v : a->a_src) v = rnd() * 2.0f * attn_scale;
        a->a_dst.resize(H * hd);
        for (auto& v : a->a_dst) v = rnd() * 2.0f * attn_scale;
        a->a_edge.resize(H * hd);
        for (auto& v : a->a_edge) v = rnd() * 2.0f * attn_scale;
        upload_vec(a->d_wnode, a->w_node);
        a->d_wnode_x3.reset(std::max<int64_t>((int64_t)a->w_node.size(), 1) * 6);
        split_x3(a->d_wnode.as<float>(), (int64_t)a->w_node.size(), a->d_wnode_x3.as<uint16_t>());
        sync();
        upload_vec(a->d_wedge, a->w_edge);
        upload_vec(a->d_asrc, a->a_src);
        upload_vec(a->d_adst, a->a_dst);
        upload_vec(a->d_aedge, a->a_edge);
        *out = a.release();
    });
}

rvx_status rvx_edge_attention_destroy(rvx_edge_attention* a) {
    return guard([&] { delete a; });
}

rvx_status rvx_edge_attention_dim(const rvx_edge_attention* a, int32_t* out_dim) {
    return guard([&] {
        RVX_REQUIRE(a && out_dim, RVX_ERR_INVALID_PARAMETER, "null argument");
        *out_dim = a->cfg.concat_heads ? a->D : a->hd;
    });
}

rvx_status rvx_edge_attention_compute(const rvx_edge_attention* a, const float* query, const float* keys,
                                      const float* values, const float* edges, int32_t n, float* out) {
    return guard([&] {
        RVX_REQUIRE(a && query && out && n >= 0, RVX_ERR_INVALID_PARAMETER, "bad arguments");
        // Attention::compute rejects empty keys (edge_featured.rs:273-275).
        RVX_REQUIRE(edges != nullptr || n > 0, RVX_ERR_INVALID_PARAMETER, "Empty keys");
        RVX_REQUIRE(n == 0 || (keys && values), RVX_ERR_INVALID_PARAMETER, "null keys/values");
        ComputeLock cl;
        const int nd = a->cfg.node_dim, D = a->D;
        const int64_t nn = std::max(n, 1);
        float* dq = scratch_f32("efa1_q", nd);
        float* dk = scratch_f32("efa1_k", nn * nd);
        float* dv = scratch_f32("efa1_v", nn * nd);
        float* tq = scratch_f32("efa1_tq", D);
        float* tk = scratch_f32("efa1_tk", nn * D);
        float* tv = scratch_f32("efa1_tv", nn * D);
        float* de = scratch_f32("efa1_e", nn * std::max(a->cfg.edge_dim, 1));
        float* dout = scratch_f32("efa1_out", D);
        auto* rp = (int64_t*)scratch_bytes("efa1_rp", 16);
        auto* col = (int32_t*)scratch_bytes("efa1_col", nn * 4);
        std::vector<int64_t> hrp{0, n};
        std::vector<int32_t> hcol(nn);
        for (int j = 0; j < n; ++j) hcol[j] = j;
        RVX_HIP(hipMemcpyAsync(dq, query, (size_t)nd * 4, hipMemcpyHostToDevice, stream()));
        if (n) {
            RVX_HIP(hipMemcpyAsync(dk, keys, (size_t)n * nd * 4, hipMemcpyHostToDevice, stream()));
            RVX_HIP(hipMemcpyAsync(dv, values, (size_t)n * nd * 4, hipMemcpyHostToDevice, stream()));
            if (edges && a->cfg.edge_dim > 0)
                RVX_HIP(hipMemcpyAsync(de, edges, (size_t)n * a->cfg.edge_dim * 4, hipMemcpyHostToDevice, stream()));
        }
        RVX_HIP(hipMemcpyAsync(rp, hrp.data(), 16, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(col, hcol.data(), (size_t)nn * 4, hipMemcpyHostToDevice, stream()));
        transform(a, dq, 1, tq, "efa_transform");
        if (n) {
            transform(a, dk, n, tk, "efa_transform");
            transform(a, dv, n, tv, "efa_transform");
        }
        run_efa(a, 1, rp, col, n, tq, n, tk, tv, (edges && a->cfg.edge_dim > 0) ? de : nullptr, dout);
        const int od = a->cfg.concat_heads ? D : a->hd;
        RVX_HIP(hipMemcpyAsync(out, dout, (size_t)od * 4, hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_edge_attention_forward_graph_device(const rvx_edge_attention* a, const rvx_graph* g, const rvx_buffer* x,
                                                   const rvx_buffer* ef, rvx_buffer* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(a && x && y, RVX_ERR_INVALID_PARAMETER, "null argument");
        const int nd = a->cfg.node_dim;
        const int od = a->cfg.concat_heads ? a->D : a->hd;
        RVX_REQUIRE(x->mem.bytes >= g->n * nd * 4, RVX_ERR_DIMENSION_MISMATCH, "x smaller than n*node_dim");
        RVX_REQUIRE(y->mem.bytes >= g->n * od * 4, RVX_ERR_DIMENSION_MISMATCH, "y smaller than n*out_dim");
        RVX_REQUIRE(!ef || ef->mem.bytes >= g->e * a->cfg.edge_dim * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "edge features smaller than E*edge_dim");
        ComputeLock cl;
        float* t = scratch_f32("efa_t", g->n * (int64_t)a->D);
        transform(a, x->mem.as<float>(), g->n, t, "efa_transform");
        run_efa(a, g->n, g->row_ptr, g->col, g->e, t, g->n, t, t, ef ? ef->mem.as<float>() : nullptr, y->mem.as<float>());
    });
}

rvx_status rvx_edge_attention_forward_exchange(const rvx_edge_attention* a, const rvx_graph* g,
                                               const rvx_buffer* x_full, const rvx_buffer* ef, rvx_buffer* y_full,
                                               const int64_t* offsets, rvx_comm* comm) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(a && x_full && y_full && offsets, RVX_ERR_INVALID_PARAMETER, "null argument");
        const int world = comm_size(comm), me = comm_rank(comm);
        for (int p = 0; p < world; ++p)
            RVX_REQUIRE(offsets[p] >= 0 && offsets[p] <= offsets[p + 1], RVX_ERR_INVALID_PARAMETER,
                        "offsets must be non-decreasing");
        RVX_REQUIRE(offsets[me + 1] - offsets[me] == g->n, RVX_ERR_DIMENSION_MISMATCH,
                    "graph rows differ from this rank's shard");
        const int64_t N = offsets[world], o = offsets[me], D = a->D;
        const int nd = a->cfg.node_dim;
        const int od = a->cfg.concat_heads ? a->D : a->hd;
        RVX_REQUIRE(x_full->mem.bytes >= N * nd * 4, RVX_ERR_DIMENSION_MISMATCH, "x_full smaller than N*node_dim");
        RVX_REQUIRE(y_full->mem.bytes >= N * od * 4, RVX_ERR_DIMENSION_MISMATCH, "y_full smaller than N*out_dim");
        RVX_REQUIRE(!ef || ef->mem.bytes >= g->e * a->cfg.edge_dim * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "edge features smaller than E*edge_dim");
        ComputeLock cl;
        // owned rows of T = x W_node^T into the whole table, every rank's rows to
        // every peer, then the per-edge scores/softmax/aggregate on owned rows
        // (queries T[o..o+n), keys = values = all of T by global column id)
        // (the transform in row chunks, each chunk's rows exchanged while the
        // next chunk transforms: produce_and_exchange)
        float* t = scratch_f32("efa_t", N * D);
        const float* xf = x_full->mem.as<float>();
        produce_and_exchange(comm, offsets, {{t, D}}, [&](int64_t r0, int64_t rows) {
            transform(a, xf + r0 * nd, rows, t + r0 * D, "efa_transform");
        });
        run_efa(a, g->n, g->row_ptr, g->col, g->e, t + o * D, N, t, t, ef ? ef->mem.as<float>() : nullptr,
                y_full->mem.as<float>() + o * od);
    });
}

rvx_status rvx_differentiable_search_batch(const float* q, int64_t nq, const float* cand, int32_t c, int32_t d, int32_t k,
                                           float temperature, int64_t* idx, float* w) {
    return guard([&] {
        RVX_REQUIRE(nq >= 0 && c >= 0 && d > 0 && k >= 0, RVX_ERR_INVALID_PARAMETER, "bad sizes");
        if (nq == 0 || k == 0) return;
        RVX_REQUIRE(q && idx && w && (c == 0 || cand), RVX_ERR_INVALID_PARAMETER, "null argument");
        if (c == 0) {  // empty candidates -> empty result (search.rs:62-64)
            for (int64_t i = 0; i < nq * k; ++i) { idx[i] = -1; w[i] = 0.0f; }
            return;
        }
        ComputeLock cl;
        float* dq = scratch_f32("ds_q", nq * d);
        float* dc = scratch_f32("ds_c", nq * c * (int64_t)d);
        float* ds = scratch_f32("ds_s", nq * c);
        auto* di = (int64_t*)scratch_bytes("ds_i", nq * k * 8);
        float* dw = scratch_f32("ds_w", nq * k);
        RVX_HIP(hipMemcpyAsync(dq, q, (size_t)(nq * d * 4), hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(dc, cand, (size_t)(nq * c * (int64_t)d * 4), hipMemcpyHostToDevice, stream()));
        differentiable_search(dq, nq, dc, c, d, k, temperature, ds, di, dw);
        RVX_HIP(hipMemcpyAsync(idx, di, (size_t)(nq * k * 8), hipMemcpyDeviceToHost, stream()));
        RVX_HIP(hipMemcpyAsync(w, dw, (size_t)(nq * k * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_differentiable_search_device(const rvx_buffer* q, int64_t nq, const rvx_buffer* table, int64_t table_rows,
                                            const rvx_buffer* cand_ids, int32_t c, int32_t d, int32_t k,
                                            float temperature, rvx_buffer* idx, rvx_buffer* w, rvx_buffer* soft) {
    return guard([&] {
        RVX_REQUIRE(nq >= 0 && c > 0 && d > 0 && k >= 0 && table_rows >= 0, RVX_ERR_INVALID_PARAMETER, "bad sizes");
        if (nq == 0) return;
        RVX_REQUIRE(q && table && cand_ids, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(k == 0 || (idx && w), RVX_ERR_INVALID_PARAMETER, "null outputs");
        RVX_REQUIRE(q->mem.bytes >= nq * (int64_t)d * 4, RVX_ERR_DIMENSION_MISMATCH, "q smaller than nq*d");
        RVX_REQUIRE(table->mem.bytes >= table_rows * (int64_t)d * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "table smaller than table_rows*d");
        RVX_REQUIRE(cand_ids->mem.bytes >= nq * (int64_t)c * 8, RVX_ERR_DIMENSION_MISMATCH, "cand_ids smaller than nq*c");
        RVX_REQUIRE(k == 0 || (idx->mem.bytes >= nq * (int64_t)k * 8 && w->mem.bytes >= nq * (int64_t)k * 4),
                    RVX_ERR_DIMENSION_MISMATCH, "outputs smaller than nq*k");
        RVX_REQUIRE(!soft || soft->mem.bytes >= nq * (int64_t)c * 4, RVX_ERR_DIMENSION_MISMATCH, "soft smaller than nq*c");
        ComputeLock cl;
        const int64_t* ids = cand_ids->mem.as<int64_t>();
        // every slot must name a table row: the reference's candidate list has no holes
        auto* deg = (int32_t*)scratch_bytes("dsd_deg", nq * 4);
        star_degrees(ids, nq, c, table_rows, deg);
        std::vector<int32_t> hdeg(nq);
        RVX_HIP(hipMemcpyAsync(hdeg.data(), deg, (size_t)nq * 4, hipMemcpyDeviceToHost, stream()));
        sync();
        for (int64_t i = 0; i < nq; ++i)
            RVX_REQUIRE(hdeg[i] == c, RVX_ERR_INVALID_PARAMETER, "candidate id outside the table");
        float* dc = scratch_f32("dsd_c", nq * (int64_t)c * d);
        float* ds = scratch_f32("dsd_s", nq * (int64_t)c);
        star_gather(nullptr, nq, table->mem.as<float>(), table_rows, ids, c, d, dc);
        differentiable_search(q->mem.as<float>(), nq, dc, c, d, k, temperature, ds, k ? idx->mem.as<int64_t>() : nullptr,
                              k ? w->mem.as<float>() : nullptr, soft ? soft->mem.as<float>() : nullptr);
    });
}

}  // extern "C"
