// k_poincare.hip — Poincaré-ball distance (crates/ruvector-hyperbolic-hnsw/src/poincare.rs).
//
// fused_norms (poincare.rs:135-168): one pass accumulating |u-v|^2, |u|^2, |v|^2
// in 4-wide chunks, each chunk's a0*a0+a1*a1+a2*a2+a3*a3 summed left to right and
// then added to its accumulator, remainder sequential; then
// poincare_distance_from_norms (:238-255) with fast_acosh (:259-276).
// The three sums follow the reference order exactly; fast_acosh's logf is the
// glibc restatement of libm_f32.hpp and sqrtf is correctly rounded, so every
// distance equals the reference's bit for bit.
#include "common.hpp"
#include "hyper.hpp"
#include "poincare_dev.hpp"
#include "scan.hpp"

namespace rvx {
namespace {

constexpr float PEPS = pdev::EPS;

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
    out[idx] = pdev::from_norms(ds, nu, nv, c);
}

// rvx_selftest_libm: out[i] = f(bits(start + i * stride)) for the libm_f32.hpp
// restatements, so tests can compare the device's bits with the host's glibc
__global__ void k_libm_eval(int fn, uint64_t start, uint64_t stride, int64_t count, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float x = glibc::u2f((uint32_t)(start + (uint64_t)i * stride));
    float y;
    switch (fn) {
        case 0: y = glibc::logf(x); break;
        case 1: y = glibc::log1pf(x); break;
        case 2: y = glibc::expm1f(x); break;
        case 3: y = glibc::tanhf(x); break;
        default: y = glibc::rust_atanhf(x); break;
    }
    out[i] = y;
}

}  // namespace

void libm_eval(int fn, uint64_t start, uint64_t stride, int64_t count, float* out) {
    if (count <= 0) return;
    RVX_LAUNCH("libm_eval", k_libm_eval, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, fn, start, stride, count,
               out);
}

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
