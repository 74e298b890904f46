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
void differentiable_search(const float* q, int64_t nq, const float* cand, int C, int d, int k, float temperature,
                           float* sims, int64_t* out_idx, float* out_w, float* soft = nullptr);

}  // namespace rvx
