// libm_check.cpp — TEST INFRASTRUCTURE: compares the product's glibc restatements
// (ruvector_amd/csrc/libm_f32.hpp) with the host's glibc libm, which is what the
// reference's f32::ln / ln_1p / tanh call on x86-64 Linux. Host-compiled restatements
// (dev == nullptr) or device outputs copied back (dev != nullptr) are checked input
// by input: x = bits(start + i * stride), i < count, NaN equal to NaN.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../ruvector_amd/csrc/libm_f32.hpp"

namespace {

float ref_fn(int fn, float x) {
    switch (fn) {
        case 0: return ::logf(x);
        case 1: return ::log1pf(x);
        case 2: return ::expm1f(x);
        case 3: return ::tanhf(x);
        default: return 0.5f * ::log1pf((2.0f * x) / (1.0f - x));  // Rust std f32::atanh
    }
}

float restated(int fn, float x) {
    switch (fn) {
        case 0: return rvx::glibc::logf(x);
        case 1: return rvx::glibc::log1pf(x);
        case 2: return rvx::glibc::expm1f(x);
        case 3: return rvx::glibc::tanhf(x);
        default: return rvx::glibc::rust_atanhf(x);
    }
}

bool same(float a, float b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    uint32_t ua, ub;
    std::memcpy(&ua, &a, 4);
    std::memcpy(&ub, &b, 4);
    return ua == ub;
}

}  // namespace

extern "C" int64_t orc_libm_check(int32_t fn, uint64_t start, uint64_t stride, uint64_t count, const float* dev,
                                  int32_t threads, uint32_t* first_bad) {
    if (threads < 1) threads = 1;
    std::vector<int64_t> bad((size_t)threads, 0);
    std::vector<uint64_t> first((size_t)threads, UINT64_MAX);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            const uint64_t lo = count * (uint64_t)t / (uint64_t)threads, hi = count * (uint64_t)(t + 1) / (uint64_t)threads;
            for (uint64_t i = lo; i < hi; ++i) {
                const uint32_t u = (uint32_t)(start + i * stride);
                float x;
                std::memcpy(&x, &u, 4);
                const float got = dev ? dev[i] : restated(fn, x);
                if (!same(got, ref_fn(fn, x))) {
                    if (first[(size_t)t] == UINT64_MAX) first[(size_t)t] = u;
                    ++bad[(size_t)t];
                }
            }
        });
    for (auto& t : ts) t.join();
    int64_t total = 0;
    uint64_t f = UINT64_MAX;
    for (int t = 0; t < threads; ++t) {
        total += bad[(size_t)t];
        if (f == UINT64_MAX) f = first[(size_t)t];
    }
    if (first_bad) *first_bad = f == UINT64_MAX ? 0u : (uint32_t)f;
    return total;
}
