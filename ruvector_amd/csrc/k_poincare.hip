// k_poincare.hip — Poincaré-ball distance (crates/ruvector-hyperbolic-hnsw/src/poincare.rs).
//
// fused_norms (poincare.rs:135-168): one pass accumulating |u-v|^2, |u|^2, |v|^2
// in 4-wide chunks, each chunk's a0*a0+a1*a1+a2*a2+a3*a3 summed left to right and
// then added to its accumulator, remainder sequential; then
// poincare_distance_from_norms (:238-255) with fast_acosh (:259-276).
// The three sums follow the reference order exactly; logf/sqrtf come from the
// device math library (<=1 ulp from glibc), so distances agree to ~1e-6 rel.
#include "common.hpp"
#include "scan.hpp"

namespace rvx {
namespace {

constexpr float PEPS = 1e-5f;  // poincare.rs EPS

__device__ __forceinline__ float fast_acosh(float x) {
    if (x <= 1.0f) return 0.0f;
    const float delta = x - 1.0f;
    if (delta < 1e-4f) return sqrtf(2.0f * delta);
    if (x < 1e6f) return logf(x + sqrtf(x * x - 1.0f));
    return logf(2.0f * x);
}

__device__ __forceinline__ float from_norms(float diff_sq, float nu, float nv, float c) {
    const float sqrt_c = sqrtf(c);
    const float lu = fmaxf(1.0f - c * nu, PEPS);
    const float lv = fmaxf(1.0f - c * nv, PEPS);
    const float num = 2.0f * c * diff_sq;
    const float den = lu * lv;
    const float arg = 1.0f + num / den;
    if (arg <= 1.0f) return 0.0f;
    return (1.0f / sqrt_c) * fast_acosh(arg);
}

__global__ void k_poincare_matrix(const float* q, int64_t nq, const float* x, int64_t n, int d, float c, float* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nq * n) return;
    const float* u = q + (idx / n) * d;
    const float* v = x + (idx % n) * d;
    float ds = 0.0f, nu = 0.0f, nv = 0.0f;
    const int chunks = d / 4;
    int i = 0;
    for (int ch = 0; ch < chunks; ++ch, i += 4) {
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
    out[idx] = from_norms(ds, nu, nv, c);
}

}  // namespace

void poincare_matrix(const float* q, int64_t nq, const float* x, int64_t n, int d, float c, float* out) {
    const int64_t total = nq * n;
    if (total <= 0) return;
    c = fmaxf(fabsf(c), PEPS);  // poincare_distance: c.abs().max(EPS) (poincare.rs:228)
    ProfScope ps("poincare_matrix");
    hipLaunchKernelGGL(k_poincare_matrix, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream(), q, nq, x, n, d,
                       c, out);
    RVX_HIP(hipGetLastError());
}

}  // namespace rvx
