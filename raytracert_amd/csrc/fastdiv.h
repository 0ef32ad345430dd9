// fastdiv.h — unsigned division by a run-time invariant divisor as a multiply-high and shifts
// (Granlund & Montgomery 1994, the round-up variant with a 33-bit multiplier folded into one
// 32-bit mulhi + add): exact for every 32-bit numerator. The kernels divide sample and tile
// indices by the frame's tile geometry; with the magic numbers precomputed on the host, a
// division is 5 integer VALU operations on scalar constants instead of a per-launch reciprocal
// setup the compiler keeps (and spills) in vector registers.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

namespace rt {

struct UDiv {
    uint32_t m;     // 2^32 * (2^l - d) / d + 1, l = ceil(log2 d); 0 for d == 1
    uint32_t sh1;   // 1; 0 for d == 1
    uint32_t sh2;   // l - 1; 0 for d == 1
    uint32_t d;
};

inline UDiv make_udiv(uint32_t d) {
    UDiv u{0, 0, 0, d};
    if (d <= 1) return u;
    uint32_t l = 0;
    while ((uint64_t(1) << l) < d) ++l;
    u.m = static_cast<uint32_t>(((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1);
    u.sh1 = 1;
    u.sh2 = l - 1;
    return u;
}

RT_HD inline uint32_t udiv(uint32_t n, const UDiv &u) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t t = __umulhi(n, u.m);
#else
    const uint32_t t = static_cast<uint32_t>((static_cast<uint64_t>(n) * u.m) >> 32);
#endif
    return (t + ((n - t) >> u.sh1)) >> u.sh2;
}

RT_HD inline uint32_t umod(uint32_t n, const UDiv &u) { return n - udiv(n, u) * u.d; }

}  // namespace rt
