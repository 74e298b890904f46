// hyper.hpp — launchers of the HyperbolicHnsw kernels (k_hyper.hip).
#pragma once
#include <cstdint>

namespace rvx {

// project_to_ball of every row of x [n][d] in place (eps = poincare EPS)
void project_rows(float* x, int64_t n, int d, float c);
// exact top-k (k <= 128) of every query by HyperbolicHnsw::distance, ascending (distance, row)
void poincare_topk(const float* q, int64_t nq, const float* x, int64_t n, int d, float c, int k, float* out_d,
                   int64_t* out_i);
// out[r] = log_p(x[r]) given -p (device) and |p|^2
void log_map_rows(const float* x, int64_t n, int d, const float* negp_dev, float np_sq, float c, float* out);
// acc[j] = acc[j] + w*rows[0][j] + w*rows[1][j] + ... left to right, each product and
// sum rounded to f32 (frechet_mean's point-major accumulation); acc is device memory
void col_chain(const float* rows, int64_t n, int d, float w, float* acc);
// exact Poincaré re-rank of nc candidates per query (ids, -1 = none), first k ascending
void rerank(const float* q, int64_t nq, const float* x, int d, float c, const int64_t* cand, int nc, int k,
            float* out_d, int64_t* out_i, int32_t* out_n);

// out[i] = f(bits(start + i * stride)), f = 0 logf, 1 log1pf, 2 expm1f, 3 tanhf,
// 4 Rust atanh (libm_f32.hpp restatements; k_poincare.hip)
void libm_eval(int fn, uint64_t start, uint64_t stride, int64_t count, float* out);

}  // namespace rvx
