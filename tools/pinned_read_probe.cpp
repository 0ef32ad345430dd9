// How fast the host reads memory from rt_host_alloc (hipHostMalloc) against ordinary pageable memory:
// the drop-in answers the 'r' loop's calls from a frame's records in pinned memory (36 B per call).
// Build: g++ -O2 -std=c++17 -Iinclude tools/pinned_read_probe.cpp -Lraytracert_amd -lrtamd -Wl,-rpath,$PWD/raytracert_amd
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "raytracert.h"

static double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static double read_ms(const float *p, size_t n, float &sink) {
    double best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
        const double t0 = now_s();
        float acc = 0;
        for (size_t i = 0; i < n; i += 9) acc += p[i] + p[i + 6];   // the fields a cached call reads, record by record
        sink += acc;
        best = std::min(best, (now_s() - t0) * 1e3);
    }
    return best;
}

int main() {
    const size_t n = 9ull * 1920 * 1080;   // floats of a C4 frame's records
    float sink = 0;
    void *pin = nullptr;
    if (rt_host_alloc(n * sizeof(float), &pin) != RT_OK) { std::printf("rt_host_alloc failed: %s\n", rt_last_error_string()); return 1; }
    std::memset(pin, 1, n * sizeof(float));
    std::vector<float> page(n, 1.0f);
    const double tp = read_ms(static_cast<const float *>(pin), n, sink), tq = read_ms(page.data(), n, sink);
    const double t0 = now_s();
    std::memcpy(page.data(), pin, n * sizeof(float));
    const double tc = (now_s() - t0) * 1e3;
    std::printf("records %zu MB: pinned read %.3f ms (%.1f GB/s), pageable read %.3f ms (%.1f GB/s), pinned->pageable memcpy %.3f ms (sink %g)\n",
                n * 4 >> 20, tp, n * 4 / tp / 1e6, tq, n * 4 / tq / 1e6, tc, sink);
    rt_host_free(pin);
    return 0;
}
