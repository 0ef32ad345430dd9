// Host check of raytracert_amd/csrc/fastdiv.h (built with g++ by tests/test_fastdiv.py): udiv/umod
// against '/' and '%' for every divisor up to 4096 and sampled larger ones, on edge numerators
// (0, 1, d-1, d, d+1, multiples, 2^31-1, 2^32-1) and random ones. Prints "ok <checks>".
#include <cstdio>
#include <random>
#include <vector>

#include "fastdiv.h"

int main() {
    std::mt19937_64 rng(7);
    unsigned long long checks = 0;
    auto check = [&](uint32_t n, uint32_t d, const rt::UDiv &u) {
        ++checks;
        if (rt::udiv(n, u) != n / d || rt::umod(n, u) != n % d) {
            std::printf("fail n=%u d=%u got %u %u\n", n, d, rt::udiv(n, u), rt::umod(n, u));
            return false;
        }
        return true;
    };
    std::vector<uint32_t> ds;
    for (uint32_t d = 1; d <= 4096; ++d) ds.push_back(d);
    for (int i = 0; i < 4000; ++i) ds.push_back(static_cast<uint32_t>(rng() >> (32 + rng() % 32)) | 1u);
    for (uint32_t d : {65535u, 65536u, 65537u, 1u << 30, (1u << 31) - 1, 1u << 31, 0xFFFFFFFFu}) ds.push_back(d);
    for (uint32_t d : ds) {
        if (d == 0) continue;
        const rt::UDiv u = rt::make_udiv(d);
        const uint32_t edge[] = {0u, 1u, d - 1, d, d + 1, 2 * d, 2 * d - 1, 3 * d + 1, 0x7FFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFEu};
        for (uint32_t n : edge)
            if (!check(n, d, u)) return 1;
        for (int k = 0; k < 200; ++k)
            if (!check(static_cast<uint32_t>(rng()), d, u) || !check(static_cast<uint32_t>(rng() >> 40), d, u)) return 1;
    }
    std::printf("ok %llu\n", checks);
    return 0;
}
