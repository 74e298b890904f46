// gnn.hpp — launch arguments of the RuvectorLayer kernels (k_gnn.hip).
#pragma once
#include <cstdint>

namespace rvx {

// Destination rows i = 0..n-1 of a row chunk: rp points at the chunk's first
// row_ptr entry (edge indices stay global, so col / w are the whole graph's);
// q, att, wagg are chunk-local; k, v, m are whole node tables indexed by the
// global neighbour id. scores holds the chunk's edges from rp[0] on.
struct EdgeArgs {
    int64_t n = 0;
    int H = 0, heads = 0, hd = 0, G = 0;  // G = lanes per head of the grouped kernel (0 = generic)
    const int64_t* rp = nullptr;
    const int32_t* col = nullptr;
    const float* w = nullptr;  // per-edge weights (wmode 1: raw, 2: pre-normalised)
    int wmode = 0;
    const float* q = nullptr; int64_t ldq = 0;   // [n][ldq]
    const float* k = nullptr;                    // [N][ldkv]
    const float* v = nullptr;                    // [N][ldkv]
    int64_t ldkv = 0;
    const float* m = nullptr;    // [N][H]   messages w_msg(x)
    float* scores = nullptr;     // [chunk edges][heads] scratch
    float* att = nullptr;        // [n][H]   concat of head outputs
    float* wagg = nullptr;       // [n][H]   weighted message aggregate
    float* att_amax = nullptr;   // optional [n][ROWSUMSQ_SLOTS]: max |att| per row (slot 0, others 0)
};

struct FinishArgs {
    int64_t n = 0;
    int H = 0;
    const int64_t* rp = nullptr;
    const float* m = nullptr;   // [n][H]  (GRU hidden = node message)
    const float* zr = nullptr;  // [n][2H] (z | r)
    const float* ht = nullptr;  // [n][H]
    const float* gamma = nullptr;
    const float* beta = nullptr;
    float eps = 1e-5f;
    float keep = 1.0f;          // 1 - dropout
    float* y = nullptr;         // [n][H]
};

void edge_attention(const EdgeArgs& a);

// Folded attention (RuvectorLayer exchanging M only): with
// k_j = W_k m_j + b_k and v_j = W_v m_j + b_v, per destination i and head h
//   score_ij,h = (qt_i,h · m_j + q_i,h · b_k,h) / sqrt(hd),  qt_i,h = W_k,h^T q_i,h
//   u_i,h      = sum_j a_ij,h m_j            (att_i,h = W_v,h u_i,h + b_v,h)
// so the edges read m_j alone. qt: [n][heads][H]; u: [n][heads][H].
struct EdgeFoldArgs {
    int64_t n = 0;
    int H = 0, heads = 0, hd = 0;
    const int64_t* rp = nullptr;
    const int32_t* col = nullptr;
    const float* w = nullptr;
    int wmode = 0;
    const float* q = nullptr;    // [n][H]  (for q_h · b_k,h)
    const float* bk = nullptr;   // [H]
    const float* qt = nullptr;   // [n][heads][H]
    const float* m = nullptr;    // [N][H]
    float* scores = nullptr;     // [chunk edges][heads] scratch
    float* u = nullptr;          // [n][heads][H]
    float* wagg = nullptr;       // [n][H]
};
bool edge_fold_ok(int H, int heads);
void edge_attention_fold(const EdgeFoldArgs& a);
int edge_group_lanes(int H, int heads);  // 0 when the grouped kernel does not apply
// out = r ⊙ h per row; amax (optional): the rows' max |out| as GemmOperand::amax slots
void mul_rows(const float* r, int64_t ldr, const float* h, float* out, int64_t n, int H, float* amax = nullptr);
void gru_finish(const FinishArgs& a);

// Star tables for batched per-node calls (RuvectorLayer::forward(node,
// neighbours, weights) and differentiable_search over candidate lists):
// dst rows [0, nq) = nodes (skipped when nodes == nullptr), rows nq + i*c + j =
// table[ids[i*c + j]] (zeros for an id outside [0, trows)).
void star_gather(const float* nodes, int64_t nq, const float* table, int64_t trows, const int64_t* ids, int c, int d,
                 float* dst);
// Valid-candidate count per node (ids in [0, trows)).
void star_degrees(const int64_t* ids, int64_t nq, int c, int64_t trows, int32_t* deg);
// CSR over the star table from host-summed row_ptr: col = nq + i*c + j for each
// valid slot in order; w (nullable) -> aggregate_messages-normalised weights
// (layer.rs:421-445: w / sum over the node's weights, 1/deg when sum <= 0).
void star_csr(const int64_t* ids, const float* w, int64_t nq, int c, int64_t trows, const int64_t* rp, int32_t* col,
              float* wn);

}  // namespace rvx
