// poincare_dev.hpp — Poincaré-ball math of crates/ruvector-hyperbolic-hnsw/src/poincare.rs
// in the reference's accumulation order, usable on host and device.
//
// Every reduction follows the reference's 4-wide unrolled loops: per chunk the
// four products are summed left to right, ((a0*a0 + a1*a1) + a2*a2) + a3*a3, and
// that is added to the running sum; the remainder is sequential
// (norm_squared :77-103, dot :112-131, fused_norms :135-168, mobius_add :310-356).
// Transcendentals are the glibc restatements of libm_f32.hpp (Rust's f32::ln,
// f32::tanh and std's f32::atanh formula), so host and device return the reference's
// bits; sqrtf and the f32 arithmetic are correctly rounded IEEE operations.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "libm_f32.hpp"

namespace rvx {
namespace pdev {

constexpr float EPS = 1e-5f;  // poincare.rs EPS

__host__ __device__ inline float norm_sq(const float* x, int d) {
    float s = 0.0f;
    int i = 0;
    for (; i + 4 <= d; i += 4) s = s + (((x[i] * x[i] + x[i + 1] * x[i + 1]) + x[i + 2] * x[i + 2]) + x[i + 3] * x[i + 3]);
    for (; i < d; ++i) s = s + x[i] * x[i];
    return s;
}

// (|u-v|^2, |u|^2, |v|^2) in one pass (fused_norms)
__host__ __device__ inline void fused3(const float* u, const float* v, int d, float& ds, float& nu, float& nv) {
    ds = 0.0f; nu = 0.0f; nv = 0.0f;
    int i = 0;
    for (; i + 4 <= d; i += 4) {
        const float u0 = u[i], u1 = u[i + 1], u2 = u[i + 2], u3 = u[i + 3];
        const float v0 = v[i], v1 = v[i + 1], v2 = v[i + 2], v3 = v[i + 3];
        const float d0 = u0 - v0, d1 = u1 - v1, d2 = u2 - v2, d3 = u3 - v3;
        ds = ds + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
        nu = nu + (((u0 * u0 + u1 * u1) + u2 * u2) + u3 * u3);
        nv = nv + (((v0 * v0 + v1 * v1) + v2 * v2) + v3 * v3);
    }
    for (; i < d; ++i) {
        const float ui = u[i], vi = v[i], di = ui - vi;
        ds = ds + di * di;
        nu = nu + ui * ui;
        nv = nv + vi * vi;
    }
}

__host__ __device__ inline float fast_acosh(float x) {  // poincare.rs:259-276
    if (x <= 1.0f) return 0.0f;
    const float delta = x - 1.0f;
    if (delta < 1e-4f) return sqrtf(2.0f * delta);
    if (x < 1e6f) return glibc::logf(x + sqrtf(x * x - 1.0f));
    return glibc::logf(2.0f * x);
}

// poincare_distance_from_norms (:238-255); c is used as given
__host__ __device__ inline float from_norms(float diff_sq, float nu, float nv, float c) {
    const float sqrt_c = sqrtf(c);
    const float lu = fmaxf(1.0f - c * nu, EPS);
    const float lv = fmaxf(1.0f - c * nv, EPS);
    const float arg = 1.0f + (2.0f * c * diff_sq) / (lu * lv);
    if (arg <= 1.0f) return 0.0f;
    return (1.0f / sqrt_c) * fast_acosh(arg);
}

// HyperbolicHnsw::distance for the Poincaré metric (hnsw.rs:173-180): fused
// norms + from_norms with the index curvature as configured
__host__ __device__ inline float hyp_dist(const float* a, const float* b, int d, float c) {
    float ds, na, nb;
    fused3(a, b, d, ds, na, nb);
    return from_norms(ds, na, nb, c);
}

// HyperbolicHnsw::distance for DistanceMetric::Euclidean (hnsw.rs:182-185):
// sqrt of fused_norms' chunked |a-b|^2
__host__ __device__ inline float hyp_l2(const float* a, const float* b, int d) {
    float ds, na, nb;
    fused3(a, b, d, ds, na, nb);
    return sqrtf(ds);
}

// project_to_ball_inplace (:189-203)
__host__ __device__ inline void project_inplace(float* x, int d, float c, float eps) {
    c = fmaxf(fabsf(c), EPS);
    const float ns = norm_sq(x, d);
    const float max_norm = (1.0f / sqrtf(c)) - eps;
    if (ns >= max_norm * max_norm && ns >= eps * eps) {
        const float scale = max_norm / sqrtf(ns);
        for (int i = 0; i < d; ++i) x[i] = x[i] * scale;
    }
}

// mobius_add (:310-356): out = x (+)_c y, projected back into the ball
__host__ __device__ inline void mobius_add(const float* x, const float* y, int d, float c, float* out) {
    c = fmaxf(fabsf(c), EPS);
    float nx = 0.0f, ny = 0.0f, dxy = 0.0f;
    int i = 0;
    for (; i + 4 <= d; i += 4) {
        const float x0 = x[i], x1 = x[i + 1], x2 = x[i + 2], x3 = x[i + 3];
        const float y0 = y[i], y1 = y[i + 1], y2 = y[i + 2], y3 = y[i + 3];
        nx = nx + (((x0 * x0 + x1 * x1) + x2 * x2) + x3 * x3);
        ny = ny + (((y0 * y0 + y1 * y1) + y2 * y2) + y3 * y3);
        dxy = dxy + (((x0 * y0 + x1 * y1) + x2 * y2) + x3 * y3);
    }
    for (; i < d; ++i) {
        nx = nx + x[i] * x[i];
        ny = ny + y[i] * y[i];
        dxy = dxy + x[i] * y[i];
    }
    const float coef_x = (1.0f + 2.0f * c * dxy) + c * ny;
    const float coef_y = 1.0f - c * nx;
    const float denom = fmaxf((1.0f + 2.0f * c * dxy) + c * c * nx * ny, EPS);
    const float inv = 1.0f / denom;
    for (int j = 0; j < d; ++j) out[j] = (coef_x * x[j] + coef_y * y[j]) * inv;
    project_inplace(out, d, c, EPS);
}

// log_map (:431-451): out = log_p(y); tmp holds d floats of scratch
__host__ __device__ inline void log_map(const float* y, const float* p, int d, float c, float* out, float* tmp) {
    c = fmaxf(fabsf(c), EPS);
    const float sqrt_c = sqrtf(c);
    for (int i = 0; i < d; ++i) tmp[i] = -p[i];
    mobius_add(tmp, y, d, c, out);  // diff = -p (+) y
    const float norm_diff = sqrtf(norm_sq(out, d));
    if (norm_diff < EPS) {
        for (int i = 0; i < d; ++i) out[i] = 0.0f;
        return;
    }
    const float lambda_p = 2.0f / fmaxf(1.0f - c * norm_sq(p, d), EPS);
    const float arg = fminf(sqrt_c * norm_diff, 1.0f - EPS);
    const float coef = (2.0f / (sqrt_c * lambda_p)) * glibc::rust_atanhf(arg) / norm_diff;
    for (int i = 0; i < d; ++i) out[i] = coef * out[i];
}

// log_map with -p and |p|^2 precomputed (the same y -> log_p(y) for a fixed p)
__host__ __device__ inline void log_map_negp(const float* y, const float* negp, float np_sq, int d, float c, float* out) {
    c = fmaxf(fabsf(c), EPS);
    const float sqrt_c = sqrtf(c);
    mobius_add(negp, y, d, c, out);
    const float norm_diff = sqrtf(norm_sq(out, d));
    if (norm_diff < EPS) {
        for (int i = 0; i < d; ++i) out[i] = 0.0f;
        return;
    }
    const float lambda_p = 2.0f / fmaxf(1.0f - c * np_sq, EPS);
    const float arg = fminf(sqrt_c * norm_diff, 1.0f - EPS);
    const float coef = (2.0f / (sqrt_c * lambda_p)) * glibc::rust_atanhf(arg) / norm_diff;
    for (int i = 0; i < d; ++i) out[i] = coef * out[i];
}

// exp_map (:407-428): out = exp_p(v); tmp holds d floats of scratch
__host__ __device__ inline void exp_map(const float* v, const float* p, int d, float c, float* out, float* tmp) {
    c = fmaxf(fabsf(c), EPS);
    const float sqrt_c = sqrtf(c);
    const float lambda_p = 2.0f / fmaxf(1.0f - c * norm_sq(p, d), EPS);
    const float norm_v = sqrtf(norm_sq(v, d));
    if (norm_v < EPS) {
        for (int i = 0; i < d; ++i) out[i] = p[i];
        return;
    }
    const float scaled = sqrt_c * lambda_p * norm_v / 2.0f;
    const float coef = glibc::tanhf(scaled) / (sqrt_c * norm_v);
    for (int i = 0; i < d; ++i) tmp[i] = coef * v[i];
    mobius_add(p, tmp, d, c, out);
}

}  // namespace pdev
}  // namespace rvx
