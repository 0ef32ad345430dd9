// Host twin of the kernels' specular powf (raytracert_amd/csrc/spec_pow.h): the same code, built
// with g++ -ffp-contract=off, against (float)pow(double) — the correctly rounded powf up to
// double's own error — and glibc powf, the reference's function (raytracing.cpp:226).
// Prints: samples, mismatches vs (float)pow(double), max |ulp| there, mismatches vs powf for
// spec_pow and for (float)pow(double), then the special cases as hex bits.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "spec_pow.h"

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    const int per_y = argc > 1 ? std::atoi(argv[1]) : 200000;
    std::mt19937_64 r(1);
    std::uniform_real_distribution<float> ux(0.0f, 1.0000002f);
    const float ys[] = {1, 2, 3, 5, 7.7f, 10, 20, 32, 50, 64, 96, 100, 128, 200, 256, 500, 1000, 1e4f, 0.5f, 0.1f, -1, -3.5f};
    long long n = 0, mis = 0, mis_g = 0, mis_dg = 0, maxulp = 0;
    for (float y : ys)
        for (int i = 0; i < per_y; ++i) {
            float x = ux(r);
            if (i % 7 == 0) x = std::ldexp(ux(r), -static_cast<int>(r() % 140));   // small and subnormal bases
            const float a = rt::spec_pow(x, y), b = static_cast<float>(std::pow(static_cast<double>(x), static_cast<double>(y)));
            const float c = powf(x, y);
            ++n;
            if (bits(a) != bits(b)) {
                ++mis;
                const long long d = std::llabs(static_cast<long long>(bits(a)) - static_cast<long long>(bits(b)));
                if (d > maxulp) maxulp = d;
            }
            mis_g += bits(a) != bits(c);
            mis_dg += bits(b) != bits(c);
        }
    std::printf("%lld %lld %lld %lld %lld\n", n, mis, maxulp, mis_g, mis_dg);
    const float xs[] = {0.0f, -0.0f, 1.0f, 0.5f, NAN, 1e-45f, 0.999999f};
    const float yv[] = {0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e30f};
    for (float x : xs)
        for (float y : yv) std::printf("%08x %08x\n", bits(rt::spec_pow(x, y)), bits(powf(x, y)));
    return 0;
}
