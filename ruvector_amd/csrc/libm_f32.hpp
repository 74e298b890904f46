// libm_f32.hpp — the f32 transcendental functions the reference's Poincaré path calls,
// restated so that device and host return the bits glibc returns.
//
// The reference is Rust on x86-64 Linux: f32::ln lowers to libm `logf`, f32::ln_1p to
// `log1pf`, f32::tanh to `tanhf` (std's cmath), and f32::atanh is std's own formula
// 0.5 * ln_1p(2x / (1 - x)) (library/std/src/f32.rs). The image's libm is glibc 2.35:
//   logf    sysdeps/ieee754/flt-32/e_logf.c + e_logf_data.c (table-driven, double
//           evaluation; the x86-64 FMA ifunc variant contracts the polynomial — both
//           forms give identical f32 results, verified exhaustively)
//   log1pf  sysdeps/ieee754/flt-32/s_log1pf.c (fdlibm)
//   expm1f  sysdeps/ieee754/flt-32/s_expm1f.c (fdlibm)
//   tanhf   sysdeps/ieee754/flt-32/s_tanhf.c  (fdlibm, through expm1f)
// Each restatement equals the host glibc function on all 2^32 inputs (NaN payloads
// aside): oracle/libm_check.cpp runs that comparison on the CPU (tests/test_libm.py),
// and tests/test_gpu_libm.py compares the device evaluations (rvx_selftest_libm) of
// every input with glibc.
//
// Used where a reported value or a ranking must match the reference bit for bit:
// fast_acosh (poincare.rs:259-276), log_map (:431-451, atanh) and exp_map (:407-428,
// tanh). Every float operation here is a single IEEE operation (the library builds with
// -ffp-contract=off); the double FMAs in logf are explicit.
//
// Notices of the restated algorithms, tables and constants:
//
//   logf (glibc sysdeps/ieee754/flt-32/e_logf.c, e_logf_data.c) comes from Arm's
//   optimized-routines:
//     Copyright (c) 2017-2018, Arm Limited.
//     (upstream licence: MIT, later Apache-2.0 WITH LLVM-exception; distributed in
//     glibc under the GNU Lesser General Public License 2.1 or later)
//
//   log1pf, expm1f, tanhf (glibc sysdeps/ieee754/flt-32/s_log1pf.c, s_expm1f.c,
//   s_tanhf.c) are fdlibm's float conversions:
//     Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//     Developed at SunPro, a Sun Microsystems, Inc. business.
//     Permission to use, copy, modify, and distribute this software is freely granted,
//     provided that this notice is preserved.
//   (float conversions by Ian Lance Taylor, Cygnus Support)
#pragma once
#include <cmath>
#include <cstdint>

// The library compiles this header as HIP (host + device); the CPU check
// (oracle/libm_check.cpp, g++) includes it as plain C++.
#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define RVX_LIBM_FN __host__ __device__ inline
#else
#define RVX_LIBM_FN inline
#endif

namespace rvx {
namespace glibc {

RVX_LIBM_FN uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
RVX_LIBM_FN float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// e_logf_data.c: LOGF_TABLE_BITS 4, {invc, logc} per subinterval, ln2, log1p poly
struct LogfEntry {
    double invc, logc;
};
RVX_LIBM_FN LogfEntry logf_tab(int i) {
    switch (i) {
        case 0: return {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2};
        case 1: return {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2};
        case 2: return {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2};
        case 3: return {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3};
        case 4: return {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3};
        case 5: return {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3};
        case 6: return {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4};
        case 7: return {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4};
        case 8: return {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5};
        case 9: return {0x1p+0, 0x0p+0};
        case 10: return {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5};
        case 11: return {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4};
        case 12: return {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3};
        case 13: return {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3};
        case 14: return {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2};
        default: return {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2};
    }
}

RVX_LIBM_FN float logf(float x) {
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -INFINITY;                             // log(+-0)
        if (ix == 0x7f800000u) return x;                               // log(inf)
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return NAN;  // x < 0 or NaN
        ix = f2u(x * 0x1p23f);                                         // subnormal: normalise
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;  // OFF
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const LogfEntry t = logf_tab(i);
    const double z = (double)u2f(iz);
    constexpr double Ln2 = 0x1.62e42fefa39efp-1;
    constexpr double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    const double r = fma(z, t.invc, -1.0);
    const double y0 = fma((double)k, Ln2, t.logc);
    const double r2 = r * r;
    double y = fma(A1, r, A2);
    y = fma(A0, r2, y);
    y = fma(y, r2, y0 + r);
    return (float)y;
}

RVX_LIBM_FN float log1pf(float x) {
    constexpr float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    constexpr float Lp1 = 6.6666668653e-01f, Lp2 = 4.0000000596e-01f, Lp3 = 2.8571429849e-01f,
                    Lp4 = 2.2222198546e-01f, Lp5 = 1.8183572590e-01f, Lp6 = 1.5313838422e-01f,
                    Lp7 = 1.4798198640e-01f;
    float f = 0.0f, c = 0.0f, u;
    int32_t hu = 0;
    const int32_t hx = (int32_t)f2u(x);
    const int32_t ax = hx & 0x7fffffff;
    int32_t k = 1;
    if (hx < 0x3ed413d7) {  // x < 0.41422
        if (ax >= 0x3f800000) return x == -1.0f ? -INFINITY : NAN;
        if (ax < 0x31000000) {  // |x| < 2^-29
            if (ax < 0x24800000) return x;
            return x - x * x * 0.5f;
        }
        if (hx > 0 || hx <= (int32_t)0xbe95f61f) {  // -0.2929 < x < 0.41422
            k = 0;
            f = x;
            hu = 1;
        }
    } else if (hx >= 0x7f800000) {
        return x + x;
    }
    if (k != 0) {
        if (hx < 0x5a000000) {
            u = 1.0f + x;
            hu = (int32_t)f2u(u);
            k = (hu >> 23) - 127;
            c = (k > 0) ? 1.0f - (u - x) : x - (u - 1.0f);  // correction term
            c /= u;
        } else {
            u = x;
            hu = (int32_t)f2u(u);
            k = (hu >> 23) - 127;
            c = 0.0f;
        }
        hu &= 0x007fffff;
        if (hu < 0x3504f7) {
            u = u2f((uint32_t)hu | 0x3f800000u);
        } else {
            k += 1;
            u = u2f((uint32_t)hu | 0x3f000000u);
            hu = (0x00800000 - hu) >> 2;
        }
        f = u - 1.0f;
    }
    const float hfsq = 0.5f * f * f;
    if (hu == 0) {  // |f| < 2^-20
        if (f == 0.0f) {
            if (k == 0) return 0.0f;
            c += (float)k * ln2_lo;
            return (float)k * ln2_hi + c;
        }
        const float R = hfsq * (1.0f - 0.66666666666666666f * f);
        if (k == 0) return f - R;
        return (float)k * ln2_hi - ((R - ((float)k * ln2_lo + c)) - f);
    }
    const float s = f / (2.0f + f);
    const float z = s * s;
    const float R = z * (Lp1 + z * (Lp2 + z * (Lp3 + z * (Lp4 + z * (Lp5 + z * (Lp6 + z * Lp7))))));
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return (float)k * ln2_hi - ((hfsq - (s * (hfsq + R) + ((float)k * ln2_lo + c))) - f);
}

RVX_LIBM_FN float expm1f(float x) {
    constexpr float huge = 1.0e+30f, tiny = 1.0e-30f, o_threshold = 8.8721679688e+01f;
    constexpr float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f, invln2 = 1.4426950216e+00f;
    constexpr float Q1 = -3.3333335072e-02f, Q2 = 1.5873016091e-03f, Q3 = -7.9365076090e-05f,
                    Q4 = 4.0082177293e-06f, Q5 = -2.0109921195e-07f;
    float y, hi, lo, c = 0.0f, t, e;
    int32_t k;
    uint32_t hx = f2u(x);
    const uint32_t xsb = hx & 0x80000000u;
    hx &= 0x7fffffffu;
    if (hx >= 0x4195b844u) {  // |x| >= 27 ln2
        if (hx >= 0x42b17218u) {
            if (hx > 0x7f800000u) return x + x;
            if (hx == 0x7f800000u) return xsb == 0 ? x : -1.0f;
            if (x > o_threshold) return huge * huge;
        }
        if (xsb != 0) return tiny - 1.0f;
    }
    if (hx > 0x3eb17218u) {  // |x| > 0.5 ln2
        if (hx < 0x3F851592u) {
            if (xsb == 0) { hi = x - ln2_hi; lo = ln2_lo; k = 1; }
            else { hi = x + ln2_hi; lo = -ln2_lo; k = -1; }
        } else {
            k = (int32_t)(invln2 * x + (xsb == 0 ? 0.5f : -0.5f));
            t = (float)k;
            hi = x - t * ln2_hi;
            lo = t * ln2_lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (hx < 0x33000000u) {  // |x| < 2^-25
        t = huge + x;
        return x - (t - (huge + x));
    } else {
        k = 0;
    }
    const float hfx = 0.5f * x;
    const float hxs = x * hfx;
    const float r1 = 1.0f + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
    t = 3.0f - r1 * hfx;
    e = hxs * ((r1 - t) / (6.0f - x * t));
    if (k == 0) return x - (x * e - hxs);
    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5f * (x - e) - 0.5f;
    if (k == 1) {
        if (x < -0.25f) return -2.0f * (e - (x + 0.5f));
        return 1.0f + 2.0f * (x - e);
    }
    if (k <= -2 || k > 56) {
        y = 1.0f - (e - x);
        if (k == 128) y = y * 2.0f * 0x1p127f;
        else y = u2f(f2u(y) + ((uint32_t)k << 23));
        return y - 1.0f;
    }
    if (k < 23) {
        t = u2f(0x3f800000u - (0x1000000u >> k));  // 1 - 2^-k
        y = t - (e - x);
    } else {
        t = u2f((uint32_t)((0x7f - k) << 23));  // 2^-k
        y = x - (e + t);
        y += 1.0f;
    }
    return u2f(f2u(y) + ((uint32_t)k << 23));
}

RVX_LIBM_FN float tanhf(float x) {
    const int32_t jx = (int32_t)f2u(x);
    const int32_t ix = jx & 0x7fffffff;
    if (ix >= 0x7f800000) return jx >= 0 ? 1.0f / x + 1.0f : 1.0f / x - 1.0f;
    float z;
    if (ix < 0x41b00000) {  // |x| < 22
        if (ix == 0) return x;
        if (ix < 0x24000000) return x * (1.0f + x);  // |x| < 2^-55
        if (ix >= 0x3f800000) {
            const float t = expm1f(2.0f * fabsf(x));
            z = 1.0f - 2.0f / (t + 2.0f);
        } else {
            const float t = expm1f(-2.0f * fabsf(x));
            z = -t / (t + 2.0f);
        }
    } else {
        z = 1.0f - 1.0e-30f;
    }
    return jx >= 0 ? z : -z;
}

// Rust std f32::atanh: 0.5 * ((2.0 * self) / (1.0 - self)).ln_1p()
RVX_LIBM_FN float rust_atanhf(float x) { return 0.5f * log1pf((2.0f * x) / (1.0f - x)); }

}  // namespace glibc
}  // namespace rvx
