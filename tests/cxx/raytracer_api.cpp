// Exercises include/raytracert.hpp the way the reference's main.cpp / raytracing.cpp use the
// tracer interface; tests/test_cxx_api.py compiles it with g++ and checks its output against the
// Python binding and the oracle.
//   raytracer_api host <obj>            loader + getMaterial + error path (no GPU)
//   raytracer_api gpu <obj> <out.ppm>   render, performRayTracing (single and batched), trace(lvl),
//                                       intersectMesh, debugTrace
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "raytracert.hpp"

using rtamd::Vec3Df;

static unsigned bits(float f) { unsigned u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const bool gpu = std::strcmp(argv[1], "gpu") == 0;
    rtamd::RayTracer rt(gpu ? 0 : RT_HOST_ONLY);
    try {
        rtamd::RayTracer bad(RT_HOST_ONLY);
        bad.init("/nonexistent/model.obj");
        std::printf("error_path none\n");
    } catch (const rtamd::Error &e) {
        std::printf("error_path %d\n", e.code());
    }
    rt.init(argv[2]);
    std::printf("lights %zu %g %g %g\n", rt.MyLightPositions.size(), rt.MyLightPositions[0][0], rt.MyLightPositions[0][1],
                rt.MyLightPositions[0][2]);
    for (int t : {0, 1}) {
        const rtamd::Material m = rt.getMaterial(t);
        std::printf("material %d Kd %08x %08x %08x Ks %08x Ns %08x Tr %08x illum %d has %d%d%d%d%d%d%d\n", t, bits(m.Kd()[0]),
                    bits(m.Kd()[1]), bits(m.Kd()[2]), bits(m.Ks()[0]), bits(m.Ns()), bits(m.Tr()), m.illum(), m.has_Kd(),
                    m.has_Ka(), m.has_Ks(), m.has_Ns(), m.has_Ni(), m.has_illum(), m.has_Tr());
    }
    if (!gpu) return 0;
    rt.WindowSize_X = 96;
    rt.WindowSize_Y = 64;
    rt.pixelfactorX = rt.pixelfactorY = 1;
    rt.max_lvl = 3;
    rt.MyLightPositions.push_back(Vec3Df(1.5f, 1.5f, 4.0f));
    uint64_t rays[3] = {0, 0, 0};
    const std::vector<unsigned char> img = rt.render(nullptr, rays);
    rt.writeImage(argc > 3 ? argv[3] : "cxx.ppm", img);
    std::printf("rays %llu %llu %llu\n", (unsigned long long)rays[0], (unsigned long long)rays[1], (unsigned long long)rays[2]);
    float c[8][3];
    rtamd::check(rt_default_corners(96, 64, c));
    std::vector<Vec3Df> os, ds;
    for (int i = 0; i < 16; ++i) {
        const float a = (i % 4 + 0.5f) / 4, b = (i / 4 + 0.5f) / 4;
        Vec3Df o, d;
        for (int k = 0; k < 3; ++k) {
            o[k] = (c[0][k] * a + c[4][k] * (1 - a)) * b + (c[2][k] * a + c[6][k] * (1 - a)) * (1 - b);
            d[k] = (c[1][k] * a + c[5][k] * (1 - a)) * b + (c[3][k] * a + c[7][k] * (1 - a)) * (1 - b);
        }
        os.push_back(o);
        ds.push_back(d);
    }
    const std::vector<Vec3Df> batch = rt.performRayTracing(os, ds);
    for (size_t i = 0; i < os.size(); ++i) {
        const Vec3Df one = rt.performRayTracing(os[i], ds[i]);
        const Vec3Df deep = rt.trace(os[i], ds[i], rt.max_lvl);   // no recursion left
        Vec3Df I;
        const int idx = rt.intersectMesh(os[i], ds[i], &I);
        Vec3Df col;
        const std::vector<rt_debug_bounce> chain = rt.debugTrace(os[i], ds[i], &col);
        std::printf("ray %zu o %08x %08x %08x d %08x %08x %08x rgb %08x %08x %08x single_eq %d local %08x %08x %08x idx %d "
                    "I %08x %08x %08x chain %zu dbg_eq %d\n",
                    i, bits(os[i][0]), bits(os[i][1]), bits(os[i][2]), bits(ds[i][0]), bits(ds[i][1]), bits(ds[i][2]),
                    bits(batch[i][0]), bits(batch[i][1]), bits(batch[i][2]), one == batch[i], bits(deep[0]), bits(deep[1]),
                    bits(deep[2]), idx, bits(I[0]), bits(I[1]), bits(I[2]), chain.size(), col == batch[i]);
    }
    return 0;
}
