// spec_pow.h — powf(SpecularTerm, Ns) of raytracing.cpp:226, evaluated in double with a short
// log2/exp2 pair and rounded once to float. The library pow(double) spends ~30 extra VGPRs and a
// double-double log on accuracy a float result never sees; this form is ~4e-14 relative, so its
// float rounding equals the correctly rounded powf except within ~1e-6 of a rounding midpoint
// (one float ulp there; colour-only, as glibc powf itself is not correctly rounded everywhere).
// Header-only and host-callable so tests/cxx/spec_pow_check.cpp checks the same code on the CPU.
#ifndef RT_SPEC_POW_H_
#define RT_SPEC_POW_H_

#include <cmath>
#include <cstdint>
#include <cstring>

#include "spec_pow_tab.h"

#ifndef RT_SPEC_POW_TABLE
#define RT_SPEC_POW_TABLE 0   // 1: table-driven log2/exp2 (r05, measured 1-2% slower: profiles/r05zh_ab_spec_table.txt)
#endif

#if defined(__HIP__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

namespace rt {

// A coefficient materialised in scalar registers where it is used: without this the compiler
// hoists every loop-invariant double constant of the polynomials into a VGPR pair (~40 VGPRs
// held across the whole traversal loop of the chain kernel).
RT_HD inline double sconst(double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(c));
#endif
    return c;
}

RT_HD inline float spec_pow(float xf, float yf) {
    if (yf == 0.0f || xf == 1.0f) return 1.0f;                       // pow(x, ±0) = pow(1, y) = 1
    if (xf != xf || yf != yf) return xf + yf;                         // NaN
    // negative bases (SpecularTerm is std::max(.., 0), so only -0 reaches here): C99 pow's sign. The
    // exponent's integer/odd tests (an fmod loop) run only for a negative base.
    float sgn = 1.0f;
    if (std::signbit(xf)) {
        const bool y_int = std::fabs(yf) >= 16777216.0f || yf == std::trunc(yf);
        const bool y_odd = std::fabs(yf) < 16777216.0f && y_int && std::fmod(yf, 2.0f) != 0.0f;
        if (xf != 0.0f && !y_int) return NAN;
        if (y_odd) sgn = -1.0f;
    }
    xf = std::fabs(xf);
    if (xf == 1.0f) return sgn;
    const double y = static_cast<double>(yf);
    if (xf == 0.0f) return sgn * (y > 0 ? 0.0f : INFINITY);
#if RT_SPEC_POW_TABLE
    // Table-driven (r05): log2(x) = e + logc + log1p(r) / ln 2 with m = x 2^-e in [1, 2), r = m invc - 1
    // (one fma, |r| <= 2^-7, degree 7: truncation < 3e-17); exp2(t) = 2^n T[j] e^u, t = n + j/64 + g,
    // u = g ln 2, |u| <= 0.0055, degree 5 (truncation < 4e-17). About half the double instructions of
    // the atanh / degree-14 form below, and no double division; ~1e-15 relative before the float rounding.
    int e;
    const float mf = std::frexp(xf, &e) * 2.0f;                        // [1, 2), exact
    e -= 1;
    uint32_t mb;
    std::memcpy(&mb, &mf, sizeof(mb));
    const int i = static_cast<int>((mb >> 17) & 63u);
    const double r = std::fma(static_cast<double>(mf), kSpecLogTab[i][0], -1.0);
    double p = sconst(1.0 / 7);
    p = std::fma(p, r, sconst(-1.0 / 6)); p = std::fma(p, r, sconst(1.0 / 5)); p = std::fma(p, r, sconst(-1.0 / 4));
    p = std::fma(p, r, sconst(1.0 / 3));  p = std::fma(p, r, -0.5);            p = std::fma(p, r, 1.0);
    double t = y * std::fma(p * r, sconst(1.4426950408889634074), static_cast<double>(e) + kSpecLogTab[i][1]);
    if (t != t) return NAN;   // (not reached: NaN inputs returned above)
    if (t < -1100.0) t = -1100.0;                                     // 0 after rounding either way
    if (t > 1100.0) t = 1100.0;                                       // inf
    const double k = std::rint(t * 64.0);
    const int ki = static_cast<int>(k);
    const double u = (t - k * (1.0 / 64)) * sconst(0.69314718055994530942);   // t - k/64 exact
    double q = sconst(1.0 / 120);
    q = std::fma(q, u, sconst(1.0 / 24)); q = std::fma(q, u, sconst(1.0 / 6)); q = std::fma(q, u, 0.5);
    q = std::fma(q, u, 1.0);
    q = std::fma(q * u, kSpecExpTab[ki & 63], kSpecExpTab[ki & 63]);          // T (1 + u q)
    return sgn * static_cast<float>(std::ldexp(q, ki >> 6));          // (arithmetic shift: floor(k / 64))
#else
    // log2(x) = e + ln(m) / ln 2, m in [sqrt(1/2), sqrt(2)), ln(m) = 2 atanh(s), s = (m-1)/(m+1)
    int e;
    double m = std::frexp(static_cast<double>(xf), &e);
    if (m < 0.70710678118654752440) { m *= 2.0; e -= 1; }
    const double s = (m - 1.0) / (m + 1.0), z = s * s;                // |s| <= 0.1716, z <= 0.0295
    double p = sconst(1.0 / 23);
    p = std::fma(p, z, sconst(1.0 / 21)); p = std::fma(p, z, sconst(1.0 / 19)); p = std::fma(p, z, sconst(1.0 / 17));
    p = std::fma(p, z, sconst(1.0 / 15)); p = std::fma(p, z, sconst(1.0 / 13)); p = std::fma(p, z, sconst(1.0 / 11));
    p = std::fma(p, z, sconst(1.0 / 9));  p = std::fma(p, z, sconst(1.0 / 7));  p = std::fma(p, z, sconst(1.0 / 5));
    p = std::fma(p, z, sconst(1.0 / 3));  p = std::fma(p, z, 1.0);
    const double ln_m = 2.0 * s * p;
    double t = y * std::fma(ln_m, sconst(1.4426950408889634074), static_cast<double>(e));
    if (t != t) return NAN;   // (not reached: NaN inputs returned above)
    if (t < -1100.0) t = -1100.0;                                     // 0 after rounding either way
    if (t > 1100.0) t = 1100.0;                                       // inf
    // exp2(t) = 2^n e^g, n = rint(t), g = (t - n) ln 2 in [-0.347, 0.347]: Taylor to degree 14
    const double n = std::rint(t);
    const double g = (t - n) * sconst(0.69314718055994530942);
    double q = sconst(1.0 / 87178291200.0);                                   // 1/14!
    q = std::fma(q, g, sconst(1.0 / 6227020800.0)); q = std::fma(q, g, sconst(1.0 / 479001600.0));
    q = std::fma(q, g, sconst(1.0 / 39916800.0));   q = std::fma(q, g, sconst(1.0 / 3628800.0));
    q = std::fma(q, g, sconst(1.0 / 362880.0));     q = std::fma(q, g, sconst(1.0 / 40320.0));
    q = std::fma(q, g, sconst(1.0 / 5040.0));       q = std::fma(q, g, sconst(1.0 / 720.0));
    q = std::fma(q, g, sconst(1.0 / 120.0));        q = std::fma(q, g, sconst(1.0 / 24.0));
    q = std::fma(q, g, sconst(1.0 / 6.0));          q = std::fma(q, g, 0.5);
    q = std::fma(q, g, 1.0);                q = std::fma(q, g, 1.0);
    return sgn * static_cast<float>(std::ldexp(q, static_cast<int>(n)));
#endif
}

}  // namespace rt

#endif  // RT_SPEC_POW_H_
