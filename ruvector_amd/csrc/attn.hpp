// attn.hpp — launch arguments of the graph-attention and re-rank kernels (k_attn.hip).
#pragma once
#include <cstdint>

namespace rvx {

struct EfaArgs {
    int64_t n = 0;               // destination rows
    int heads = 0, hd = 0, edge_dim = 0;
    int concat = 1;
    float slope = 0.2f;
    const int64_t* rp = nullptr;
    const int32_t* col = nullptr;
    const float* tq = nullptr; int64_t ldq = 0;  // transformed query rows [n][heads*hd]
    const float* tk = nullptr; int64_t ldk = 0;  // transformed key rows (by col)
    const float* tv = nullptr; int64_t ldv = 0;  // transformed value rows (by col)
    const float* edges = nullptr;                // [E][edge_dim] or null (zero features)
    const float* w_edge = nullptr;               // [heads*hd][edge_dim]
    const float* a_src = nullptr;
    const float* a_dst = nullptr;
    const float* a_edge = nullptr;               // [heads*hd]
    float* scores = nullptr;                     // [E][heads] scratch
    float* out = nullptr;                        // [n][concat ? heads*hd : hd]
    int64_t nk = 0;                              // rows of tk
    float* sq = nullptr;                         // [n][heads]  scratch: tq . a_src per head
    float* sk = nullptr;                         // [nk][heads] scratch: tk . a_dst per head
    float* u = nullptr;                          // [heads][edge_dim] scratch: W_edge^T a_edge per head
};

void edge_feat_attention(const EfaArgs& a);

// DualSpaceAttention (crates/ruvector-attention/src/graph/dual_space.rs) over CSR
// rows: query-side rows i (te_q / th_q / nh_q), key rows by col (te_k / th_k /
// nh_k), values by col. te = x W_euclidean^T, th = project_to_ball(x W_hyperbolic^T),
// nh = |th|^2. Isolated rows produce zeros.
struct DsaArgs {
    int64_t n = 0;
    int dim = 0, value_dim = 0;
    const int64_t* rp = nullptr;
    const int32_t* col = nullptr;
    const float* te_q = nullptr; const float* th_q = nullptr; const float* nh_q = nullptr;
    const float* te_k = nullptr; const float* th_k = nullptr; const float* nh_k = nullptr;
    const float* val = nullptr; int64_t ldv = 0;
    float curvature = 1.0f, euclidean_weight = 0.5f, hyperbolic_weight = 0.5f, temperature = 1.0f, scale = 1.0f;
    float* out = nullptr;     // [n][value_dim], value_dim <= 1024
};
void dual_space_attention(const DsaArgs& a);
// project_to_ball (ruvector-attention hyperbolic/poincare.rs:121-132, eps 1e-5) of every
// row in place, nh[r] = |row r|^2 after projection.
void dsa_project_rows(float* t, int64_t rows, int dim, float curvature, float* nh);
// differentiable_search (search.rs:56-94) for nq queries: candidates of query i
// are cand[i*C .. i*C+C) rows, or all C rows of one shared table (shared_table).
// out_idx/out_w [nq][k] (idx -1 past min(k, C)); soft (nullable) [nq][C].
void differentiable_search(const float* q, int64_t nq, const float* cand, int C, int d, int k, float temperature,
                           float* sims, int64_t* out_idx, float* out_w, float* soft = nullptr,
                           bool shared_table = false);
// hierarchical_forward's combine step (search.rs:132-148): comb = (cur + sum_t w_t table[idx_t]) / 2.
void hier_combine(const float* cur, int64_t nq, const float* table, int d, const int64_t* idx, const float* w, int k,
                  float* comb);

}  // namespace rvx
