// kernels.hpp — internal launch wrappers shared by the C-ABI translation units.
// All launches go to rvx::stream() and are tagged for the event profiler.
#pragma once
#include <cstdint>

namespace rvx {

// ---- GEMM (gemm_f32.hip) ------------------------------------------------
enum { GEMM_EPI_STORE = 0, GEMM_EPI_RELU = 1, GEMM_EPI_SIGMOID = 2, GEMM_EPI_TANH = 3 };
struct GemmOperand {
    const float* A; int64_t lda;  // A [M][K]
    const float* B; int64_t ldb;  // B [N][K]  (C = A · B^T)
    int K;
    // optional exact 3-way bf16 split of B (split_x3): planes of [N][ldb]
    // uint16 at Bx3 + p*Bx3_plane; selects the split-bf16 MFMA kernel
    const uint16_t* Bx3 = nullptr;
    int64_t Bx3_plane = 0;
};
// Epilogue: C = epi(alpha * acc + bias0 + bias1 + addend[row][col])
struct GemmEpilogue {
    int epi = GEMM_EPI_STORE;
    float alpha = 1.0f;
    const float* bias0 = nullptr;
    const float* bias1 = nullptr;
    const float* addend = nullptr;
    int64_t ld_addend = 0;
};
// C[M][N] = epilogue(A0·B0^T [+ A1·B1^T])
void gemm_nt(int64_t M, int N, const GemmOperand& s0, const GemmOperand* s1, const GemmEpilogue& ep, float* C,
             int64_t ldc, const char* tag);

// dst[p*n + i] = bf16 part p of src[i] (exact split src = p0 + p1 + p2)
void split_x3(const float* src, int64_t n, uint16_t* dst);

// ---- data generators (k_data.hip) ---------------------------------------
void fill_uniform(float* p, int64_t n, uint64_t seed, float lo, float hi);
void fill_normal(float* p, int64_t n, uint64_t seed);
void normalize_rows(float* p, int64_t rows, int dim, bool divide_only_if_positive, const char* tag);
void random_csr(int64_t n, int deg, uint64_t seed, int64_t* row_ptr, int32_t* col);
void random_csr_shard(int64_t n_total, int64_t row_begin, int64_t n_rows, int deg, uint64_t seed, int64_t* row_ptr,
                      int32_t* col);
void transpose(const float* in, int64_t rows, int64_t cols, float* out);  // out[c][r] = in[r][c]

// ---- gather / aggregate (k_aggregate.hip) -------------------------------
enum { AGG_SUM = 0, AGG_MEAN = 1, AGG_MAX = 2 };
// out[i] = agg over CSR row i of (w_e * x[col_e]) ; empty row -> `empty_fill`
// (0 = zeros, 1 = copy x[i], 2 = -inf for max). post_scale: 0 none, 1 = ×1/sqrt(deg) (GCN).
void aggregate_rows(const int64_t* row_ptr, const int32_t* col, const float* w, int64_t n, const float* x,
                    int dim, int agg, int empty_fill, int post_scale, float* out, const char* tag,
                    bool overlapped = false);  // true: runs beside a GEMM (capped grid)

}  // namespace rvx
