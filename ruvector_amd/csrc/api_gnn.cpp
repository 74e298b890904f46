// api_gnn.cpp — RuvectorLayer (crates/ruvector-gnn/src/layer.rs:313-457) and
// differentiable_search (crates/ruvector-gnn/src/search.rs:4-94) over HBM.
//
// Batched forward of every node of a graph (node = x_i, neighbours = its CSR
// row in edge order, edge_weights = the row's edge weights):
//   M    = X W_msg^T + b_msg                              GEMM   (layer.rs:392-396)
//   QKV  = M [W_q;W_k;W_v]^T + [b_q;b_k;b_v]              GEMM   (layer.rs:135-137)
//   ATT, WAGG = edge kernel                               K5     (layer.rs:139-207, 421-445)
//   COMB = ATT W_o^T + b_o + WAGG                         GEMM   (layer.rs:159, 407)
//   AGG  = COMB W_agg^T + b_agg                           GEMM   (layer.rs:408)
//   ZR   = sigmoid(AGG [W_z;W_r]^T + M [U_z;U_r]^T + b)   GEMM   (layer.rs:257-262)
//   RH   = R ⊙ M ;  HT = tanh(AGG W_h^T + RH U_h^T + b)  GEMM   (layer.rs:265-267)
//   Y    = LayerNorm((1-Z)⊙M + Z⊙HT) × (1-dropout))        finish (layer.rs:270-274, 414-417)
// Nodes without neighbours get LayerNorm(M_i) (layer.rs:385-389).
// K/V are computed once per node instead of once per (destination, neighbour)
// pair as the reference does; the values are the same Linear outputs.
#include <cmath>
#include <cstring>

#include "attn.hpp"
#include "comm.hpp"
#include "gnn.hpp"
#include "graph.hpp"
#include "json.hpp"
#include "kernels.hpp"

using namespace rvx;

namespace {

struct HostLinear {
    int out = 0, in = 0;
    std::vector<float> w;  // [out][in]
    std::vector<float> b;  // [out]
};

uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Linear::new (layer.rs:21-34): weights ~ N(0, sqrt(2/(in+out))), bias 0. The
// reference uses thread_rng; here a seeded counter stream.
HostLinear make_linear(int in, int out, uint64_t seed) {
    HostLinear l;
    l.in = in; l.out = out;
    l.w.resize((size_t)in * out);
    l.b.assign(out, 0.0f);
    const double scale = std::sqrt(2.0f / (float)(in + out));
    const uint64_t s0 = sm64(seed);
    for (size_t i = 0; i < l.w.size(); ++i) {
        const double u1 = ((double)(sm64(s0 + 2 * i) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
        const double u2 = (double)(sm64(s0 + 2 * i + 1) >> 11) * (1.0 / 9007199254740992.0);
        l.w[i] = (float)(scale * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2));
    }
    return l;
}

}  // namespace

namespace rvx {
// A [rows][cols] weight on the device: f32, its split_x3 planes (split-bf16
// GEMM) and its split-f16 planes with per-output-row inverse scales (gemm_auto
// -> gemm_nt_h2). A weight paired with another in a dual GEMM shares that
// one's column scales (joint_h2).
struct DevWeight {
    DevMem w, x3, h2, inv;
    const float* inv_ptr = nullptr;
    int64_t rows = 0, cols = 0;
    void upload(const std::vector<float>& v, int64_t r, int64_t c) {
        rows = r; cols = c;
        w.reset(std::max<int64_t>(r * c, 1) * 4);
        w.upload(v.data(), r * c * 4);
        x3.reset(std::max<int64_t>(r * c, 1) * 6);
        split_x3(w.as<float>(), r * c, x3.as<uint16_t>());
        h2.reset(std::max<int64_t>(r * c, 1) * 4);
        inv.reset(std::max<int64_t>(r, 1) * 4);
        split_h2_rows(w.as<float>(), nullptr, (int)r, (int)c, h2.as<_Float16>(), nullptr, inv.as<float>());
        inv_ptr = inv.as<float>();
    }
    // operand C = A · W[row_off : row_off+n]^T with A [M][cols] (lda)
    GemmOperand op(const float* A, int64_t lda, int64_t row_off = 0) const {
        GemmOperand o{A, lda, w.as<float>() + row_off * cols, cols, (int)cols,
                      x3.as<uint16_t>() + row_off * cols, rows * cols};
        o.Bh = h2.as<_Float16>() + row_off * cols;
        o.Bh_plane = rows * cols;
        o.b_inv = inv_ptr + row_off;
        return o;
    }
};

// Re-split a dual GEMM's two weights (same shape) with one scale per output row.
void joint_h2(DevWeight& a, DevWeight& b) {
    split_h2_rows(a.w.as<float>(), b.w.as<float>(), (int)a.rows, (int)a.cols, a.h2.as<_Float16>(),
                  b.h2.as<_Float16>(), a.inv.as<float>());
    b.inv_ptr = a.inv.as<float>();
}
}  // namespace rvx

struct rvx_layer {
    int in = 0, H = 0, heads = 0, hd = 0;
    float dropout = 0.0f;
    HostLinear w_msg, w_agg, w_z, u_z, w_r, u_r, w_h, u_h, q, k, v, o;
    std::vector<float> gamma, beta;
    float eps = 1e-5f;
    // device: weights [out][in] (the GEMM's K-contiguous B) with their exact
    // 3-way bf16 splits for the split-bf16 MFMA GEMM; biases and norm f32
    DevWeight d_wmsg, d_wqkv, d_wo, d_wagg, d_wzr, d_uzr, d_wh, d_uh;
    DevWeight d_wkT;  // folded attention: per head W_k,h^T as [heads][H][hd] (rows heads*H, cols hd)
    DevMem d_bmsg, d_bqkv, d_bo, d_bagg, d_bwzr, d_buzr, d_bwh, d_buh, d_gamma, d_beta;
};

namespace {

void upload(DevMem& d, const std::vector<float>& v) {
    d.reset((int64_t)std::max<size_t>(v.size(), 1) * 4);
    d.upload(v.data(), (int64_t)v.size() * 4);
}
std::vector<float> cat(std::initializer_list<const std::vector<float>*> parts) {
    std::vector<float> r;
    for (auto* p : parts) r.insert(r.end(), p->begin(), p->end());
    return r;
}

void validate(const rvx_layer* l) {
    RVX_REQUIRE(l->dropout >= 0.0f && l->dropout <= 1.0f, RVX_ERR_LAYER_CONFIG,
                "Dropout must be between 0.0 and 1.0");
    RVX_REQUIRE(l->heads > 0 && l->H % l->heads == 0, RVX_ERR_LAYER_CONFIG,
                "Embedding dimension must be divisible by number of heads");
    auto chk = [&](const HostLinear& x, int out, int in, const char* name) {
        RVX_REQUIRE(x.out == out && x.in == in && (int64_t)x.w.size() == (int64_t)out * in && (int)x.b.size() == out,
                    RVX_ERR_INVALID_SHAPE, std::string("bad shape for ") + name);
    };
    chk(l->w_msg, l->H, l->in, "w_msg");
    for (auto* p : {&l->w_agg, &l->w_z, &l->u_z, &l->w_r, &l->u_r, &l->w_h, &l->u_h, &l->q, &l->k, &l->v, &l->o})
        chk(*p, l->H, l->H, "hidden linear");
    RVX_REQUIRE((int)l->gamma.size() == l->H && (int)l->beta.size() == l->H, RVX_ERR_INVALID_SHAPE, "bad norm shape");
}

void upload_layer(rvx_layer* l) {
    const int64_t H = l->H;
    l->d_wmsg.upload(l->w_msg.w, H, l->in); upload(l->d_bmsg, l->w_msg.b);
    l->d_wqkv.upload(cat({&l->q.w, &l->k.w, &l->v.w}), 3 * H, H); upload(l->d_bqkv, cat({&l->q.b, &l->k.b, &l->v.b}));
    {
        const int64_t hd = l->hd, heads = l->heads;
        std::vector<float> wkt((size_t)(H * H));
        for (int64_t h = 0; h < heads; ++h)
            for (int64_t c = 0; c < H; ++c)
                for (int64_t d = 0; d < hd; ++d) wkt[(size_t)((h * H + c) * hd + d)] = l->k.w[(size_t)((h * hd + d) * H + c)];
        l->d_wkT.upload(wkt, heads * H, hd);
    }
    l->d_wo.upload(l->o.w, H, H); upload(l->d_bo, l->o.b);
    l->d_wagg.upload(l->w_agg.w, H, H); upload(l->d_bagg, l->w_agg.b);
    l->d_wzr.upload(cat({&l->w_z.w, &l->w_r.w}), 2 * H, H); l->d_uzr.upload(cat({&l->u_z.w, &l->u_r.w}), 2 * H, H);
    upload(l->d_bwzr, cat({&l->w_z.b, &l->w_r.b})); upload(l->d_buzr, cat({&l->u_z.b, &l->u_r.b}));
    l->d_wh.upload(l->w_h.w, H, H); l->d_uh.upload(l->u_h.w, H, H);
    joint_h2(l->d_wzr, l->d_uzr);
    joint_h2(l->d_wh, l->d_uh);
    upload(l->d_bwh, l->w_h.b); upload(l->d_buh, l->u_h.b);
    upload(l->d_gamma, l->gamma); upload(l->d_beta, l->beta);
    sync();
}

// ---- serde JSON ------------------------------------------------------------
std::vector<float> arr_data(const json::Value* a, std::vector<int64_t>& dim) {
    RVX_REQUIRE(a && a->kind == json::Value::Object, RVX_ERR_SERIALIZATION, "expected ndarray object");
    const json::Value* d = a->get("dim");
    const json::Value* data = a->get("data");
    RVX_REQUIRE(d && d->kind == json::Value::Array && data && data->kind == json::Value::Array, RVX_ERR_SERIALIZATION,
                "ndarray needs dim and data");
    dim.clear();
    // dims are untrusted numbers: integral, in [0, 2^31), and their product bounded by
    // the data actually present before any arithmetic that could overflow
    int64_t total = 1;
    for (auto& x : d->arr) {
        RVX_REQUIRE(x.kind == json::Value::Number && x.num >= 0.0 && x.num < 2147483648.0 && x.num == std::floor(x.num),
                    RVX_ERR_SERIALIZATION, "ndarray dim must be a non-negative integer");
        const int64_t e = (int64_t)x.num;
        dim.push_back(e);
        RVX_REQUIRE(e == 0 || total <= (int64_t)data->arr.size() / e, RVX_ERR_SERIALIZATION,
                    "ndarray data length != prod(dim)");
        total *= e;
    }
    RVX_REQUIRE((int64_t)data->arr.size() == total, RVX_ERR_SERIALIZATION, "ndarray data length != prod(dim)");
    std::vector<float> v(total);
    for (int64_t i = 0; i < total; ++i)
        v[i] = data->arr[i].kind == json::Value::Number ? (float)data->arr[i].num : NAN;
    return v;
}
HostLinear linear_from(const json::Value* o, const char* name) {
    RVX_REQUIRE(o && o->kind == json::Value::Object, RVX_ERR_SERIALIZATION, std::string("missing ") + name);
    HostLinear l;
    std::vector<int64_t> dw, db;
    l.w = arr_data(o->get("weights"), dw);
    l.b = arr_data(o->get("bias"), db);
    RVX_REQUIRE(dw.size() == 2 && db.size() == 1, RVX_ERR_SERIALIZATION, std::string("bad dims for ") + name);
    l.out = (int)dw[0]; l.in = (int)dw[1];
    return l;
}
void put_arr(std::string& s, const std::vector<float>& v, std::initializer_list<int64_t> dim) {
    s += "{\"v\":1,\"dim\":[";
    bool first = true;
    for (auto d : dim) { if (!first) s += ","; s += std::to_string(d); first = false; }
    s += "],\"data\":[";
    for (size_t i = 0; i < v.size(); ++i) { if (i) s += ","; json::put_f32(s, v[i]); }
    s += "]}";
}
void put_linear(std::string& s, const HostLinear& l) {
    s += "{\"weights\":"; put_arr(s, l.w, {l.out, l.in});
    s += ",\"bias\":"; put_arr(s, l.b, {l.out});
    s += "}";
}

// ---- batched forward ---------------------------------------------------------
// wmode: 0 no weights, 1 raw per-edge weights (graph), 2 pre-normalised.
// rp/col/w: the CSR of destination rows 0..n-1 (global edge indices); x/y
// [n][in] / [n][H]; max_deg bounds the per-chunk edge count.
//
// Phase 1 (whole table, neighbours read it): M = w_msg(x) [n][H] and
// K|V = M·[W_k;W_v]^T [n][2H]. Phase 2 (row chunks of CHUNK rows, everything
// row-local): Q, edge attention + weighted message aggregate, COMB = out(att)
// + wagg, AGG = w_agg(COMB), z|r, r⊙h, h~, GRU blend + dropout + LayerNorm.
// Peak scratch = 3 n H + CHUNK (6 H + max_deg heads) floats — a 10M x 768
// layer fits beside its input and output in HBM.
//
// n_out (< 0: n): phase 2 runs for rows [0, n_out) only — the star form, whose
// rows past n_out are neighbour-only (they feed phase 1's M and K|V); rp and y
// then need only n_out + 1 / n_out rows.
// Folded attention (gnn.hpp EdgeFoldArgs): K|V are never formed, the edges
// read M alone and a sharded layer exchanges H columns per row instead of 3H
// (SURVEY.md §8e). RVX_GNN_FOLD: 0 (default) off, 1 the multi-rank exchange
// path, 2 every batched forward. Opt-in: on one GPU at 2M x 768 / 8 heads the
// folded layer is 1.5x slower (edge kernel 2 x 120 -> 220 ms per layer: eight
// full-wave score reductions per edge and M read twice; the eight K = 96 qt
// GEMMs 51 ms), which the 3x smaller exchange (7/8 x N x 2H x 4 B less per
// GPU and layer) only repays on a slow or contended interconnect. Read per call.
bool use_fold(const rvx_layer* l, bool exchange_multi) {
    const int mode = env_int("RVX_GNN_FOLD", 0);
    if (!edge_fold_ok(l->H, l->heads)) return false;
    return mode == 2 || (mode == 1 && exchange_multi);
}

// Phase 1 for `rows` rows: M = w_msg(x) and (KV non-null) K|V = M·[W_k;W_v]^T.
// Mamax (nullable): M's per-row max |m| slots (GemmEpilogue::row_absmax), so the GEMMs
// reading M (K|V here, Q and z|r in phase 2) take their split-f16 row scales from it
// instead of a pass over M (RVX_GEMM_AMAX=0 restores the passes; same scales, same bits).
void phase1_dev(const rvx_layer* l, int64_t rows, const float* x, float* M, float* KV, float* Mamax) {
    const int64_t H = l->H;
    GemmEpilogue ep;
    ep.bias0 = l->d_bmsg.as<float>();
    ep.row_absmax = Mamax;
    gemm_auto(rows, (int)H, l->d_wmsg.op(x, l->in), nullptr, ep, M, H, "gnn_gemm_msg");
    if (!KV) return;
    ep = GemmEpilogue();
    ep.bias0 = l->d_bqkv.as<float>() + H;
    GemmOperand a = l->d_wqkv.op(M, H, H);
    a.amax = Mamax;
    gemm_auto(rows, (int)(2 * H), a, nullptr, ep, KV, 2 * H, "gnn_gemm_kv");
}

// Phase 2 for destination rows [0, rows_out) of rp: neighbours index the whole
// M / KV tables (global ids), the destination rows themselves are rows
// self_off + r of them; y receives rows_out rows.
// KV == nullptr: folded attention (qt / u tables of heads*H floats per row, so
// the row chunk is capped at 128k rows).
void phase2_dev(const rvx_layer* l, int64_t rows_out, const int64_t* rp, const int32_t* col, int64_t max_deg,
                const float* w, int wmode, const float* M, const float* KV, int64_t self_off, float* y,
                const float* Mamax) {
    const int64_t H = l->H, heads = l->heads, hd = l->hd;
    const bool fold = KV == nullptr;
    int64_t CHUNK = std::max<int64_t>(4096, env_int("RVX_GNN_CHUNK_ROWS", 1 << 20));  // read per call
    if (fold) CHUNK = std::min<int64_t>(CHUNK, 1 << 17);
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(rows_out, CHUNK));
    float* QT = fold ? scratch_f32("rvl_qt", chunk * heads * H) : nullptr;
    float* U = fold ? scratch_f32("rvl_u", chunk * heads * H) : nullptr;
    float* Q = scratch_f32("rvl_q", chunk * H);
    float* S1 = scratch_f32("rvl_s1", chunk * 2 * H);
    float* S2 = scratch_f32("rvl_s2", chunk * H);
    float* S3 = scratch_f32("rvl_s3", chunk * H);
    float* S4 = scratch_f32("rvl_s4", chunk * H);
    float* scores = scratch_f32("rvl_scores", std::max<int64_t>(chunk * max_deg, 1) * l->heads);
    // per-row max |a| slots of the chunk's GEMM operands (COMB, AGG, r ⊙ h), written by
    // their producers: the consumers' split-f16 row scales without a pass over the rows
    const bool amx = Mamax && env_int("RVX_GEMM_AMAX", 1);
    float* S4amax = amx ? scratch_f32("rvl_s4_amax", chunk * ROWSUMSQ_SLOTS) : nullptr;
    float* S2amax = amx ? scratch_f32("rvl_s2_amax", chunk * ROWSUMSQ_SLOTS) : nullptr;
    float* S3amax = amx ? scratch_f32("rvl_s3_amax", chunk * ROWSUMSQ_SLOTS) : nullptr;
    GemmEpilogue ep;
    for (int64_t r0 = 0; r0 < rows_out; r0 += chunk) {
        const int64_t rows = std::min(chunk, rows_out - r0);
        const float* Mc = M + (self_off + r0) * H;
        const float* Mcamax = amx ? Mamax + (self_off + r0) * ROWSUMSQ_SLOTS : nullptr;
        ep = GemmEpilogue();
        ep.bias0 = l->d_bqkv.as<float>();
        GemmOperand qa = l->d_wqkv.op(Mc, H, 0);
        qa.amax = Mcamax;
        gemm_auto(rows, (int)H, qa, nullptr, ep, Q, H, "gnn_gemm_q");

        if (fold) {
            // qt_h = W_k,h^T q_h (one GEMM per head), edges over m_j, att_h = W_v,h u_h + b_v,h
            for (int64_t h = 0; h < heads; ++h)
                gemm_auto(rows, (int)H, l->d_wkT.op(Q + h * hd, H, h * H), nullptr, GemmEpilogue(), QT + h * H,
                          heads * H, "gnn_gemm_qt");
            EdgeFoldArgs fa;
            fa.n = rows; fa.H = (int)H; fa.heads = (int)heads; fa.hd = (int)hd;
            fa.rp = rp + r0; fa.col = col; fa.w = w; fa.wmode = w ? wmode : 0;
            fa.q = Q; fa.bk = l->d_bqkv.as<float>() + H; fa.qt = QT; fa.m = M;
            fa.scores = scores; fa.u = U; fa.wagg = S3;
            edge_attention_fold(fa);
            for (int64_t h = 0; h < heads; ++h) {
                ep = GemmEpilogue();
                ep.bias0 = l->d_bqkv.as<float>() + 2 * H + h * hd;
                gemm_auto(rows, (int)hd, l->d_wqkv.op(U + h * H, heads * H, 2 * H + h * hd), nullptr, ep, S2 + h * hd, H,
                          "gnn_gemm_att");
            }
        } else {
            EdgeArgs ea;
            ea.n = rows; ea.H = (int)H; ea.heads = l->heads; ea.hd = l->hd; ea.G = edge_group_lanes((int)H, l->heads);
            ea.rp = rp + r0; ea.col = col; ea.w = w; ea.wmode = w ? wmode : 0;
            ea.q = Q; ea.ldq = H; ea.k = KV; ea.v = KV + H; ea.ldkv = 2 * H; ea.m = M;
            ea.scores = scores; ea.att = S2; ea.wagg = S3;
            ea.att_amax = S2amax;  // att's row maxima for the out GEMM (S2amax is rewritten by AGG below)
            edge_attention(ea);
        }

        ep = GemmEpilogue();
        ep.bias0 = l->d_bo.as<float>();
        ep.addend = S3; ep.ld_addend = H;
        ep.row_absmax = S4amax;
        GemmOperand oa = l->d_wo.op(S2, H);
        oa.amax = fold ? nullptr : S2amax;
        gemm_auto(rows, (int)H, oa, nullptr, ep, S4, H, "gnn_gemm_out");  // COMB
        ep = GemmEpilogue();
        ep.bias0 = l->d_bagg.as<float>();
        ep.row_absmax = S2amax;
        GemmOperand aa = l->d_wagg.op(S4, H);
        aa.amax = S4amax;
        gemm_auto(rows, (int)H, aa, nullptr, ep, S2, H, "gnn_gemm_agg");  // AGG
        ep = GemmEpilogue();
        ep.epi = GEMM_EPI_SIGMOID; ep.bias0 = l->d_bwzr.as<float>(); ep.bias1 = l->d_buzr.as<float>();
        GemmOperand zr_a = l->d_wzr.op(S2, H), zr_b = l->d_uzr.op(Mc, H);
        zr_a.amax = S2amax; zr_b.amax = Mcamax;
        // RH = r ⊙ h. Opt-in (RVX_GNN_GATE_EPI=1, read per call; tests cover both): from the
        // z|r GEMM's epilogue (r never stored; the same product as mul_rows). It needs the 4-wave
        // 128 x 192 tile (registers), whose z|r GEMM is 10% slower than the 256 x 256 default:
        // 10M C4 step 3.67 / 3.69 vs 3.65 / 3.75 s (zr 522 vs 473 ms + gate 49 ms; a wash)
        const bool gate_epi = amx && env_int("RVX_GNN_GATE_EPI", 0);
        if (gate_epi) {
            ep.row_absmax = S3amax;
            ep.gate_h = Mc; ep.ld_gate_h = H; ep.gate_out = S3; ep.ld_gate_out = H; ep.gate_col0 = (int)H;
        }
        gemm_auto(rows, (int)(2 * H), zr_a, &zr_b, ep, S1, 2 * H, "gnn_gemm_zr");
        if (!gate_epi) mul_rows(S1 + H, 2 * H, Mc, S3, rows, (int)H, S3amax);
        ep = GemmEpilogue();
        ep.epi = GEMM_EPI_TANH; ep.bias0 = l->d_bwh.as<float>(); ep.bias1 = l->d_buh.as<float>();
        GemmOperand h_a = l->d_wh.op(S2, H), h_b = l->d_uh.op(S3, H);
        h_a.amax = S2amax; h_b.amax = S3amax;
        gemm_auto(rows, (int)H, h_a, &h_b, ep, S4, H, "gnn_gemm_h");  // HT

        FinishArgs fa;
        fa.n = rows; fa.H = (int)H; fa.rp = rp + r0; fa.m = Mc; fa.zr = S1; fa.ht = S4;
        fa.gamma = l->d_gamma.as<float>(); fa.beta = l->d_beta.as<float>(); fa.eps = l->eps;
        fa.keep = 1.0f - l->dropout;
        fa.y = y + r0 * H;
        gru_finish(fa);
    }
}

void forward_dev(const rvx_layer* l, int64_t n, const int64_t* rp, const int32_t* col, int64_t max_deg,
                 const float* w, int wmode, const float* x, float* y, int64_t n_out = -1) {
    const int64_t H = l->H;
    const int64_t rows_out = n_out < 0 ? n : std::min(n_out, n);
    float* M = scratch_f32("rvl_m", n * H);
    float* KV = use_fold(l, false) ? nullptr : scratch_f32("rvl_kv", n * 2 * H);
    float* Mamax = env_int("RVX_GEMM_AMAX", 1) ? scratch_f32("rvl_m_amax", n * ROWSUMSQ_SLOTS) : nullptr;
    phase1_dev(l, n, x, M, KV, Mamax);
    phase2_dev(l, rows_out, rp, col, max_deg, w, wmode, M, KV, 0, y, Mamax);
}

// RuvectorLayer::forward(nodes[i], table[ids[i*c .. i*c+c)], weights[i*c ..]) for
// every i < nq (ids outside [0, trows) are absent neighbours; weights nullable =
// empty edge-weight slice): one star graph over [nodes | gathered rows].
void star_forward(const rvx_layer* l, const float* nodes, int64_t nq, const float* table, int64_t table_rows,
                  const int64_t* ids, int c, const float* weights, float* out) {
    const int64_t in = l->in;
    const int64_t n = nq + nq * (int64_t)c;
    RVX_REQUIRE(n < ((int64_t)1 << 31), RVX_ERR_INVALID_SHAPE, "star table exceeds int32 neighbour ids");
    float* T = scratch_f32("rvs_t", n * in);
    auto* deg = (int32_t*)scratch_bytes("rvs_deg", nq * 4);
    auto* drp = (int64_t*)scratch_bytes("rvs_rp", (nq + 1) * 8);
    auto* dcol = (int32_t*)scratch_bytes("rvs_col", std::max<int64_t>(nq * c, 1) * 4);
    float* dw = weights ? scratch_f32("rvs_w", std::max<int64_t>(nq * c, 1)) : nullptr;
    star_gather(nodes, nq, table, table_rows, ids, c, (int)in, T);
    // row_ptr: prefix sum of the per-node valid-candidate counts on the host
    star_degrees(ids, nq, c, table_rows, deg);
    std::vector<int32_t> hdeg(nq);
    std::vector<int64_t> hrp(nq + 1, 0);
    RVX_HIP(hipMemcpyAsync(hdeg.data(), deg, (size_t)nq * 4, hipMemcpyDeviceToHost, stream()));
    sync();
    int64_t max_deg = 0;
    for (int64_t i = 0; i < nq; ++i) {
        hrp[i + 1] = hrp[i] + hdeg[i];
        max_deg = std::max<int64_t>(max_deg, hdeg[i]);
    }
    RVX_HIP(hipMemcpyAsync(drp, hrp.data(), (size_t)(nq + 1) * 8, hipMemcpyHostToDevice, stream()));
    star_csr(ids, weights, nq, c, table_rows, drp, dcol, dw);
    // weights absent -> aggregate_messages returns zeros (layer.rs:427-429): wmode 0
    forward_dev(l, n, drp, dcol, max_deg, dw, weights ? 2 : 0, T, out, nq);
    sync();  // hrp / hdeg are host temporaries
}

}  // namespace

extern "C" {

rvx_status rvx_gnn_layer_create(int32_t in, int32_t hidden, int32_t heads, float dropout, uint64_t seed,
                                rvx_layer** out) {
    return guard([&] {
        RVX_REQUIRE(out && in > 0 && hidden > 0, RVX_ERR_LAYER_CONFIG, "dimensions must be positive");
        RVX_REQUIRE(dropout >= 0.0f && dropout <= 1.0f, RVX_ERR_LAYER_CONFIG,
                    "Dropout must be between 0.0 and 1.0, got " + std::to_string(dropout));
        RVX_REQUIRE(heads > 0 && hidden % heads == 0, RVX_ERR_LAYER_CONFIG,
                    "Embedding dimension (" + std::to_string(hidden) + ") must be divisible by number of heads (" +
                        std::to_string(heads) + ")");
        auto l = std::make_unique<rvx_layer>();
        l->in = in; l->H = hidden; l->heads = heads; l->hd = hidden / heads; l->dropout = dropout;
        uint64_t s = seed * 1315423911ull;
        l->w_msg = make_linear(in, hidden, s + 1);
        l->w_agg = make_linear(hidden, hidden, s + 2);
        l->w_z = make_linear(hidden, hidden, s + 3); l->u_z = make_linear(hidden, hidden, s + 4);
        l->w_r = make_linear(hidden, hidden, s + 5); l->u_r = make_linear(hidden, hidden, s + 6);
        l->w_h = make_linear(hidden, hidden, s + 7); l->u_h = make_linear(hidden, hidden, s + 8);
        l->q = make_linear(hidden, hidden, s + 9); l->k = make_linear(hidden, hidden, s + 10);
        l->v = make_linear(hidden, hidden, s + 11); l->o = make_linear(hidden, hidden, s + 12);
        l->gamma.assign(hidden, 1.0f); l->beta.assign(hidden, 0.0f); l->eps = 1e-5f;
        validate(l.get());
        upload_layer(l.get());
        *out = l.release();
    });
}

rvx_status rvx_gnn_layer_from_json(const char* text, rvx_layer** out) {
    return guard([&] {
        RVX_REQUIRE(text && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        json::Value root;
        std::string err;
        RVX_REQUIRE(json::parse(text, root, err), RVX_ERR_SERIALIZATION, "Deserialization error: " + err);
        RVX_REQUIRE(root.kind == json::Value::Object, RVX_ERR_SERIALIZATION, "expected a JSON object");
        auto l = std::make_unique<rvx_layer>();
        l->w_msg = linear_from(root.get("w_msg"), "w_msg");
        l->w_agg = linear_from(root.get("w_agg"), "w_agg");
        const json::Value* up = root.get("w_update");
        RVX_REQUIRE(up, RVX_ERR_SERIALIZATION, "missing w_update");
        l->w_z = linear_from(up->get("w_z"), "w_z"); l->u_z = linear_from(up->get("u_z"), "u_z");
        l->w_r = linear_from(up->get("w_r"), "w_r"); l->u_r = linear_from(up->get("u_r"), "u_r");
        l->w_h = linear_from(up->get("w_h"), "w_h"); l->u_h = linear_from(up->get("u_h"), "u_h");
        const json::Value* at = root.get("attention");
        RVX_REQUIRE(at && at->get("num_heads") && at->get("head_dim"), RVX_ERR_SERIALIZATION, "missing attention");
        auto small_int = [](const json::Value* v, const char* what) {  // untrusted: check before the cast
            RVX_REQUIRE(v->kind == json::Value::Number && v->num >= 0.0 && v->num <= 65536.0 && v->num == std::floor(v->num),
                        RVX_ERR_SERIALIZATION, std::string(what) + " must be an integer in [0, 65536]");
            return (int)v->num;
        };
        l->heads = small_int(at->get("num_heads"), "num_heads");
        l->hd = small_int(at->get("head_dim"), "head_dim");
        l->q = linear_from(at->get("q_linear"), "q_linear"); l->k = linear_from(at->get("k_linear"), "k_linear");
        l->v = linear_from(at->get("v_linear"), "v_linear"); l->o = linear_from(at->get("out_linear"), "out_linear");
        const json::Value* nm = root.get("norm");
        RVX_REQUIRE(nm && nm->get("eps"), RVX_ERR_SERIALIZATION, "missing norm");
        std::vector<int64_t> dg, db;
        l->gamma = arr_data(nm->get("gamma"), dg);
        l->beta = arr_data(nm->get("beta"), db);
        l->eps = (float)nm->get("eps")->num;
        const json::Value* dr = root.get("dropout");
        RVX_REQUIRE(dr && dr->kind == json::Value::Number, RVX_ERR_SERIALIZATION, "missing dropout");
        l->dropout = (float)dr->num;
        l->in = l->w_msg.in;
        l->H = l->w_msg.out;
        RVX_REQUIRE((int64_t)l->heads * l->hd == l->H, RVX_ERR_SERIALIZATION, "num_heads*head_dim != hidden_dim");
        validate(l.get());
        upload_layer(l.get());
        *out = l.release();
    });
}

rvx_status rvx_gnn_layer_to_json(const rvx_layer* l, char* buf, size_t* len) {
    return guard([&] {
        RVX_REQUIRE(l && len, RVX_ERR_INVALID_PARAMETER, "null argument");
        std::string s;
        s.reserve((size_t)(12 * (int64_t)l->H * l->H + l->H * l->in) * 12);
        s += "{\"w_msg\":"; put_linear(s, l->w_msg);
        s += ",\"w_agg\":"; put_linear(s, l->w_agg);
        s += ",\"w_update\":{\"w_z\":"; put_linear(s, l->w_z);
        s += ",\"u_z\":"; put_linear(s, l->u_z);
        s += ",\"w_r\":"; put_linear(s, l->w_r);
        s += ",\"u_r\":"; put_linear(s, l->u_r);
        s += ",\"w_h\":"; put_linear(s, l->w_h);
        s += ",\"u_h\":"; put_linear(s, l->u_h);
        s += "},\"attention\":{\"num_heads\":" + std::to_string(l->heads) + ",\"head_dim\":" + std::to_string(l->hd);
        s += ",\"q_linear\":"; put_linear(s, l->q);
        s += ",\"k_linear\":"; put_linear(s, l->k);
        s += ",\"v_linear\":"; put_linear(s, l->v);
        s += ",\"out_linear\":"; put_linear(s, l->o);
        s += "},\"norm\":{\"gamma\":"; put_arr(s, l->gamma, {l->H});
        s += ",\"beta\":"; put_arr(s, l->beta, {l->H});
        s += ",\"eps\":"; json::put_f32(s, l->eps);
        s += "},\"dropout\":"; json::put_f32(s, l->dropout);
        s += "}";
        const size_t need = s.size() + 1;
        const size_t have = *len;
        *len = need;
        if (buf && have >= need) std::memcpy(buf, s.c_str(), need);
        else RVX_REQUIRE(buf == nullptr, RVX_ERR_INVALID_PARAMETER, "buffer too small");
    });
}

rvx_status rvx_gnn_layer_dims(const rvx_layer* l, int32_t* in, int32_t* hidden, int32_t* heads, float* dropout) {
    return guard([&] {
        RVX_REQUIRE(l, RVX_ERR_INVALID_PARAMETER, "null layer");
        if (in) *in = l->in;
        if (hidden) *hidden = l->H;
        if (heads) *heads = l->heads;
        if (dropout) *dropout = l->dropout;
    });
}

rvx_status rvx_gnn_layer_destroy(rvx_layer* l) {
    return guard([&] { delete l; });
}

rvx_status rvx_gnn_forward_one(const rvx_layer* l, const float* node, const float* nbrs, int32_t deg, const float* w,
                               int32_t nw, float* out) {
    return guard([&] {
        RVX_REQUIRE(l && node && out && deg >= 0 && nw >= 0, RVX_ERR_INVALID_PARAMETER, "bad arguments");
        RVX_REQUIRE(deg == 0 || nbrs, RVX_ERR_INVALID_PARAMETER, "null neighbours");
        RVX_REQUIRE(nw == 0 || w, RVX_ERR_INVALID_PARAMETER, "null weights");
        ComputeLock cl;
        const int64_t n = 1 + (int64_t)deg;
        // Row 0 = the node, its neighbours rows 1..deg; other rows are unused.
        std::vector<int64_t> rp(n + 1, deg);
        rp[0] = 0;
        std::vector<int32_t> col(std::max(deg, 1));
        for (int j = 0; j < deg; ++j) col[j] = j + 1;
        // aggregate_messages weights (layer.rs:421-445): empty -> zeros; the sum
        // runs over every given weight; zip() truncates to min(deg, nw).
        std::vector<float> wn(std::max(deg, 1), 0.0f);
        int wmode = 0;
        if (nw > 0 && deg > 0) {
            wmode = 2;
            float sum = 0.0f;
            for (int j = 0; j < nw; ++j) sum = sum + w[j];
            for (int j = 0; j < std::min(deg, nw); ++j) wn[j] = sum > 0.0f ? w[j] / sum : 1.0f / (float)nw;
        }
        float* dx = scratch_f32("rvl1_x", n * l->in);
        float* dy = scratch_f32("rvl1_y", n * l->H);
        auto* drp = (int64_t*)scratch_bytes("rvl1_rp", (n + 1) * 8);
        auto* dcol = (int32_t*)scratch_bytes("rvl1_col", (int64_t)col.size() * 4);
        float* dw = scratch_f32("rvl1_w", (int64_t)wn.size());
        RVX_HIP(hipMemcpyAsync(dx, node, (size_t)l->in * 4, hipMemcpyHostToDevice, stream()));
        if (deg)
            RVX_HIP(hipMemcpyAsync(dx + l->in, nbrs, (size_t)deg * l->in * 4, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(drp, rp.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(dcol, col.data(), col.size() * 4, hipMemcpyHostToDevice, stream()));
        RVX_HIP(hipMemcpyAsync(dw, wn.data(), wn.size() * 4, hipMemcpyHostToDevice, stream()));
        // rows 1..deg are neighbour-only: phase 2 runs for row 0 alone
        forward_dev(l, n, drp, dcol, deg, dw, wmode, dx, dy, 1);
        RVX_HIP(hipMemcpyAsync(out, dy, (size_t)l->H * 4, hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

rvx_status rvx_gnn_forward_star_device(const rvx_layer* l, const rvx_buffer* nodes, int64_t nq, const rvx_buffer* table,
                                       int64_t table_rows, const rvx_buffer* cand_ids, int32_t c,
                                       const rvx_buffer* weights, rvx_buffer* out) {
    return guard([&] {
        RVX_REQUIRE(l && nodes && table && cand_ids && out, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(nq >= 0 && c >= 0 && table_rows >= 0, RVX_ERR_INVALID_PARAMETER, "bad sizes");
        if (nq == 0) return;
        const int64_t in = l->in, H = l->H;
        RVX_REQUIRE(nodes->mem.bytes >= nq * in * 4, RVX_ERR_DIMENSION_MISMATCH, "nodes smaller than nq*input_dim");
        RVX_REQUIRE(table->mem.bytes >= table_rows * in * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "table smaller than table_rows*input_dim");
        RVX_REQUIRE(cand_ids->mem.bytes >= nq * (int64_t)c * 8, RVX_ERR_DIMENSION_MISMATCH, "cand_ids smaller than nq*c");
        RVX_REQUIRE(!weights || weights->mem.bytes >= nq * (int64_t)c * 4, RVX_ERR_DIMENSION_MISMATCH,
                    "weights smaller than nq*c");
        RVX_REQUIRE(out->mem.bytes >= nq * H * 4, RVX_ERR_DIMENSION_MISMATCH, "out smaller than nq*hidden_dim");
        ComputeLock cl;
        star_forward(l, nodes->mem.as<float>(), nq, table->mem.as<float>(), table_rows, cand_ids->mem.as<int64_t>(), c,
                     weights ? weights->mem.as<float>() : nullptr, out->mem.as<float>());
    });
}

rvx_status rvx_hierarchical_forward_device(const rvx_layer* const* layers, int32_t n_layers,
                                           const rvx_buffer* const* levels, const int64_t* level_rows,
                                           int32_t n_levels, const rvx_buffer* q, int64_t nq, int32_t dim,
                                           rvx_buffer* out, int32_t* out_dim) {
    return guard([&] {
        RVX_REQUIRE(q && out && out_dim && nq >= 0 && dim > 0 && n_layers >= 0 && n_levels >= 0,
                    RVX_ERR_INVALID_PARAMETER, "bad arguments");
        RVX_REQUIRE((n_layers == 0 || layers) && (n_levels == 0 || (levels && level_rows)), RVX_ERR_INVALID_PARAMETER,
                    "null layer or level arrays");
        RVX_REQUIRE(q->mem.bytes >= nq * (int64_t)dim * 4, RVX_ERR_DIMENSION_MISMATCH, "q smaller than nq*dim");
        // zip(layer_embeddings, gnn_layers) (search.rs:117-119): the shorter list bounds the walk
        const int steps = std::min(n_layers, n_levels);
        int64_t d = dim, dmax = dim;
        for (int s = 0; s < steps; ++s) {
            RVX_REQUIRE(layers[s], RVX_ERR_INVALID_PARAMETER, "null layer");
            RVX_REQUIRE(level_rows[s] >= 0 && level_rows[s] < ((int64_t)1 << 31), RVX_ERR_INVALID_PARAMETER,
                        "bad level size");
            if (level_rows[s] == 0) continue;  // empty level: skipped (search.rs:121-123)
            RVX_REQUIRE(levels[s], RVX_ERR_INVALID_PARAMETER, "null level buffer");
            // cosine_similarity asserts equal lengths (search.rs:5); Linear needs input_dim
            RVX_REQUIRE(layers[s]->in == d, RVX_ERR_DIMENSION_MISMATCH,
                        "layer " + std::to_string(s) + " input_dim " + std::to_string(layers[s]->in) +
                            " != embedding dim " + std::to_string(d));
            RVX_REQUIRE(levels[s]->mem.bytes >= level_rows[s] * d * 4, RVX_ERR_DIMENSION_MISMATCH,
                        "level buffer smaller than rows*dim");
            d = layers[s]->H;
            dmax = std::max(dmax, d);
        }
        RVX_REQUIRE(out->mem.bytes >= nq * d * 4, RVX_ERR_DIMENSION_MISMATCH, "out smaller than nq*out_dim");
        *out_dim = (int32_t)d;
        if (nq == 0) return;
        ComputeLock cl;
        float* cur_buf[2] = {scratch_f32("hier_a", nq * dmax), scratch_f32("hier_b", nq * dmax)};
        float* comb = scratch_f32("hier_comb", nq * dmax);
        const float* cur = q->mem.as<float>();
        int ping = 0;
        d = dim;
        for (int s = 0; s < steps; ++s) {
            const int64_t C = level_rows[s];
            if (C == 0) continue;
            const int k = (int)std::min<int64_t>(5, C);  // 5.min(embeddings.len()) (search.rs:128)
            const float* table = levels[s]->mem.as<float>();
            float* sims = scratch_f32("hier_sims", nq * C);
            auto* idx = (int64_t*)scratch_bytes("hier_idx", nq * k * 8);
            float* w = scratch_f32("hier_w", nq * k);
            differentiable_search(cur, nq, table, (int)C, (int)d, k, 1.0f, sims, idx, w, nullptr, true);
            hier_combine(cur, nq, table, (int)d, idx, w, k, comb);
            float* nxt = cur_buf[ping];
            ping ^= 1;
            star_forward(layers[s], comb, nq, table, C, idx, k, w, nxt);
            cur = nxt;
            d = layers[s]->H;
        }
        RVX_HIP(hipMemcpyAsync(out->mem.p, cur, (size_t)(nq * d * 4), hipMemcpyDeviceToDevice, stream()));
    });
}

rvx_status rvx_gnn_forward_graph_device(const rvx_layer* l, const rvx_graph* g, const rvx_buffer* x, rvx_buffer* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x && y, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(x->mem.bytes >= g->n * l->in * 4, RVX_ERR_DIMENSION_MISMATCH, "x smaller than n*input_dim");
        RVX_REQUIRE(y->mem.bytes >= g->n * l->H * 4, RVX_ERR_DIMENSION_MISMATCH, "y smaller than n*hidden_dim");
        ComputeLock cl;
        forward_dev(l, g->n, g->row_ptr, g->col, g->max_deg, g->w, 1, x->mem.as<float>(), y->mem.as<float>());
    });
}

rvx_status rvx_gnn_forward_exchange(const rvx_layer* l, const rvx_graph* g, const rvx_buffer* x_full,
                                    rvx_buffer* y_full, const int64_t* offsets, rvx_comm* comm) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x_full && y_full && offsets, RVX_ERR_INVALID_PARAMETER, "null argument");
        const int world = comm_size(comm), me = comm_rank(comm);
        for (int p = 0; p < world; ++p)
            RVX_REQUIRE(offsets[p] >= 0 && offsets[p] <= offsets[p + 1], RVX_ERR_INVALID_PARAMETER,
                        "offsets must be non-decreasing");
        RVX_REQUIRE(offsets[me + 1] - offsets[me] == g->n, RVX_ERR_DIMENSION_MISMATCH,
                    "graph rows differ from this rank's shard");
        const int64_t N = offsets[world], o = offsets[me], H = l->H;
        RVX_REQUIRE(x_full->mem.bytes >= N * l->in * 4, RVX_ERR_DIMENSION_MISMATCH, "x_full smaller than N*input_dim");
        RVX_REQUIRE(y_full->mem.bytes >= N * H * 4, RVX_ERR_DIMENSION_MISMATCH, "y_full smaller than N*hidden_dim");
        ComputeLock cl;
        // phase 1 on the owned rows, straight into the whole-table M (and,
        // unfolded, K|V), every rank's rows to every peer, then phase 2 on owned
        // rows. Folded (RVX_GNN_FOLD=1/2) only M travels: H columns per row, not 3H.
        // Phase 1 runs in row chunks; each chunk's rows travel on the transfer
        // stream while the next chunk's GEMMs run (produce_and_exchange).
        const bool fold = use_fold(l, world > 1);
        float* M = scratch_f32("rvl_m", N * H);
        float* KV = fold ? nullptr : scratch_f32("rvl_kv", N * 2 * H);
        std::vector<TableRef> tables{{M, H}};
        if (KV) tables.push_back({KV, 2 * H});
        const float* x = x_full->mem.as<float>();
        // row maxima of M for the owned rows only (phase 2 reads no peer row through a GEMM)
        float* Mamax = env_int("RVX_GEMM_AMAX", 1) ? scratch_f32("rvl_m_amax", N * ROWSUMSQ_SLOTS) : nullptr;
        produce_and_exchange(comm, offsets, tables, [&](int64_t r0, int64_t rows) {
            phase1_dev(l, rows, x + r0 * l->in, M + r0 * H, KV ? KV + r0 * 2 * H : nullptr,
                       Mamax ? Mamax + r0 * ROWSUMSQ_SLOTS : nullptr);
        });
        phase2_dev(l, g->n, g->row_ptr, g->col, g->max_deg, g->w, 1, M, KV, o, y_full->mem.as<float>() + o * H,
                   Mamax);
    });
}

rvx_status rvx_gnn_forward_graph(const rvx_layer* l, const rvx_graph* g, const float* x, int64_t n, float* y) {
    return guard([&] {
        check_graph(g);
        RVX_REQUIRE(l && x && y, RVX_ERR_INVALID_PARAMETER, "null argument");
        RVX_REQUIRE(n == g->n, RVX_ERR_DIMENSION_MISMATCH, "feature rows != graph nodes");
        ComputeLock cl;
        float* dx = scratch_f32("rvlg_x", n * l->in);
        float* dy = scratch_f32("rvlg_y", n * l->H);
        RVX_HIP(hipMemcpyAsync(dx, x, (size_t)(n * l->in * 4), hipMemcpyHostToDevice, stream()));
        forward_dev(l, n, g->row_ptr, g->col, g->max_deg, g->w, 1, dx, dy);
        RVX_HIP(hipMemcpyAsync(y, dy, (size_t)(n * l->H * 4), hipMemcpyDeviceToHost, stream()));
        sync();
    });
}

}  // extern "C"
