// The drop-in's cached performRayTracing path alone, on the CPU (no GPU, no scene): a host-only build
// whose frame cache is filled with the 'r' loop's own rays (loop_ray) and stand-in colours, then the
// literal main.cpp:355-395 loop timed against the same loop with a trace that only reads its arguments
// (the host floor). The difference over the loop's calls is what each cached call costs the host.
// Build: g++ -std=c++17 -O2 -ffp-contract=off -Iinclude tools/dropin_cache_bench.cpp -Lraytracert_amd -lrtamd
//        -Wl,-rpath,$PWD/raytracert_amd -o tools/bin/dropin_cache_bench
// Run:   tools/bin/dropin_cache_bench [W H pf reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "raytracert_dropin.hpp"

Vec3Df MyCameraPosition(0, 0, 4);
std::vector<Vec3Df> MyLightPositions;
Mesh MyMesh;
unsigned int WindowSize_X = 500;
unsigned int WindowSize_Y = 500;
unsigned int RayTracingResolutionX = 500;
unsigned int RayTracingResolutionY = 500;

static float g_c[8][3];
void produceRay(int x, int y, Vec3Df &o, Vec3Df &d) {   // the default camera's corner rays (rt_default_corners)
    const int i = (x == 0 ? 0 : 2) + (y == 0 ? 0 : 1);
    o = Vec3Df(g_c[2 * i][0], g_c[2 * i][1], g_c[2 * i][2]);
    d = Vec3Df(g_c[2 * i + 1][0], g_c[2 * i + 1][1], g_c[2 * i + 1][2]);
}

static double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static Vec3Df floor_trace(const Vec3Df &o, const Vec3Df &d) { return Vec3Df(o[0] * 1e-9f, d[1] * 1e-9f, 0.5f); }

template <bool kCached>
static double loop_ms(Vec3Df &acc) {
    Vec3Df origin00, dest00, origin01, dest01, origin10, dest10, origin11, dest11, origin, dest;
    produceRay(0, 0, origin00, dest00);
    produceRay(0, WindowSize_Y - 1, origin01, dest01);
    produceRay(WindowSize_X - 1, 0, origin10, dest10);
    produceRay(WindowSize_X - 1, WindowSize_Y - 1, origin11, dest11);
    if (kCached) rtamd_dropin::frame_cache().next = 0;
    const double t0 = now_s();
    float divX = (WindowSize_X * pixelfactorX - 1);
    float divY = (WindowSize_Y * pixelfactorY - 1);
    int raysPerPixel = (pixelfactorX * pixelfactorY);
    for (unsigned int y = 0; y < WindowSize_Y; ++y)
        for (unsigned int x = 0; x < WindowSize_X; ++x) {
            Vec3Df rgb = Vec3Df(0, 0, 0);
            for (int subx = 0; subx < (int)pixelfactorX; subx++)
                for (int suby = 0; suby < (int)pixelfactorY; suby++) {
                    float xscale = 1.0f - (float(x) * pixelfactorX + subx) / divX;
                    float yscale = 1.0f - (float(y) * pixelfactorY + suby) / divY;
                    origin = yscale * (xscale * origin00 + (1 - xscale) * origin10) +
                             (1 - yscale) * (xscale * origin01 + (1 - xscale) * origin11);
                    dest = yscale * (xscale * dest00 + (1 - xscale) * dest10) +
                           (1 - yscale) * (xscale * dest01 + (1 - xscale) * dest11);
                    rgb += kCached ? performRayTracing(origin, dest) : floor_trace(origin, dest);
                }
            acc += rgb / raysPerPixel;
        }
    return 1e3 * (now_s() - t0);
}

int main(int argc, char **argv) {
    if (argc > 2) { WindowSize_X = unsigned(std::atoi(argv[1])); WindowSize_Y = unsigned(std::atoi(argv[2])); }
    if (argc > 3) pixelfactorX = pixelfactorY = unsigned(std::atoi(argv[3]));
    const int reps = argc > 4 ? std::atoi(argv[4]) : 5;
    if (rt_default_corners(int32_t(WindowSize_X), int32_t(WindowSize_Y), g_c) != RT_OK) return 3;
    MyLightPositions.push_back(MyCameraPosition);
    // the frame cache as start_frame leaves it after a device frame trace of the loop's own rays
    rtamd_dropin::FrameCache &fc = rtamd_dropin::frame_cache();
    const size_t spp = size_t(pixelfactorX) * pixelfactorY, n = size_t(WindowSize_X) * WindowSize_Y * spp;
    // (pinned memory on a GPU host, as the drop-in makes it; plain memory where no device is visible)
    std::vector<float> plain;
    int32_t ndev = 0;
    if (rt_device_count(&ndev) == RT_OK && ndev > 0) {
        rtamd_dropin::ensure_records(fc.rec, fc.rec_cap, 9 * n);
    } else {
        plain.resize(9 * n);
        fc.rec = plain.data();
        fc.rec_cap = plain.size();
    }
    Vec3Df c[8];
    for (int i = 0; i < 8; ++i) c[i] = Vec3Df(g_c[i][0], g_c[i][1], g_c[i][2]);
    const float divX = (WindowSize_X * pixelfactorX - 1), divY = (WindowSize_Y * pixelfactorY - 1);
    for (size_t s = 0; s < n; ++s) {
        const size_t pix = s / spp, sub = s % spp;
        Vec3Df o, d;
        rtamd_dropin::loop_ray(unsigned(pix % WindowSize_X), unsigned(pix / WindowSize_X), int(sub / pixelfactorY),
                               int(sub % pixelfactorY), divX, divY, c, o, d);
        float *r = fc.rec + 9 * s;
        for (int k = 0; k < 3; ++k) { r[k] = o[k]; r[3 + k] = d[k]; r[6 + k] = 0.25f; }
    }
    fc.state = rtamd_dropin::TraceState::now();
    fc.n = n;
    Vec3Df acc(0, 0, 0);
    double best_c = 1e9, best_f = 1e9;
    for (int r = 0; r < reps; ++r) {
        best_f = std::min(best_f, loop_ms<false>(acc));
        best_c = std::min(best_c, loop_ms<true>(acc));
        if (fc.next != n) { std::printf("cache missed at call %zu of %zu\n", fc.next, n); return 1; }
    }
    if (!plain.empty()) { fc.rec = nullptr; fc.rec_cap = 0; }   // (not the drop-in's to free)
    std::printf("{\"pinned\": %s, \"calls\": %zu, \"cached_loop_ms\": %.3f, \"host_floor_ms\": %.3f, \"ns_per_cached_call\": %.2f, \"checksum\": %g}\n", plain.empty() ? "true" : "false", n,
                best_c, best_f, (best_c - best_f) * 1e6 / double(n), acc[0] + acc[1] + acc[2]);
    return 0;
}
