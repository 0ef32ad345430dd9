// A host program written against the reference tracer's interface (CG_Project/raytracing.h and
// the globals of main.cpp) that compiles unchanged against include/raytracert_dropin.hpp: it
// defines the globals the way main.cpp:17-18,130-141 does, produces the four corner rays, runs
// the 'r' key's per-sub-sample loop (main.cpp:355-395: corner blend, rgb += performRayTracing,
// rgb / raysPerPixel, RGBValue clamp, Image::writeImage's truncation) and, for comparison, the
// one-call renderImage(). tests/test_cxx_dropin.py builds it with g++ and checks its output
// against the oracle.
//   dropin_frame host <obj>                                  loader, MyMesh, normals, getMaterial
//   dropin_frame gpu <obj> W H pf max_lvl loop.ppm fast.ppm   both frames; prints equality + rays
#include <cstdio>
#include <cstring>
#include <vector>

#include "raytracert_dropin.hpp"

// ---- what the host's main.cpp defines (main.cpp:17-18,130,137-141) ----
Vec3Df MyCameraPosition(0.0f, 0.0f, 4.0f);
std::vector<Vec3Df> MyLightPositions;
Mesh MyMesh;
unsigned int WindowSize_X = 500;
unsigned int WindowSize_Y = 500;
unsigned int RayTracingResolutionX = 500;
unsigned int RayTracingResolutionY = 500;

// produceRay for the default view without GL (rt_default_corners restates GLU's unproject)
static float g_corners[8][3];
static void produceRay(int x_I, int y_I, Vec3Df *origin, Vec3Df *dest) {
    const int cx = x_I == 0 ? 0 : 1, cy = y_I == 0 ? 0 : 1;   // corner pixels only
    const int k = 2 * (2 * cx + cy);                           // origin00, origin01, origin10, origin11
    *origin = Vec3Df(g_corners[k][0], g_corners[k][1], g_corners[k][2]);
    *dest = Vec3Df(g_corners[k + 1][0], g_corners[k + 1][1], g_corners[k + 1][2]);
}

// RGBValue's clamp (main.cpp:21-42) and Image::writeImage's bytes (main.cpp:102-128)
static float clamp01(float v) {
    if (v > 1) v = 1.0f;
    if (v < 0) v = 0.0f;
    return v;
}
static bool writePPM(const char *path, unsigned w, unsigned h, const std::vector<float> &img) {
    FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%i %i\n255\n", static_cast<int>(w), static_cast<int>(h));
    std::vector<unsigned char> bytes(img.size());
    for (size_t i = 0; i < img.size(); ++i) bytes[i] = static_cast<unsigned char>(img[i] * 255.0f);
    const bool ok = std::fwrite(bytes.data(), bytes.size(), 1, f) == 1;
    std::fclose(f);
    return ok;
}

static unsigned bits(float f) { unsigned u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const bool gpu = std::strcmp(argv[1], "gpu") == 0;
    RayTracerDevice = gpu ? 0 : RT_HOST_ONLY;
    init(argv[2]);
    std::printf("mesh %zu %zu %zu %zu lights %zu normals %zu\n", MyMesh.vertices.size(), MyMesh.triangles.size(),
                MyMesh.triangleMaterials.size(), MyMesh.materials.size(), MyLightPositions.size(), normals.size());
    unsigned long long hv = 1469598103934665603ull, hn = hv, ht = hv;
    for (const Vertex &v : MyMesh.vertices)
        for (int k = 0; k < 3; ++k) hv = (hv ^ bits(v.p[k])) * 1099511628211ull;
    for (const Vec3Df &n : normals)
        for (int k = 0; k < 3; ++k) hn = (hn ^ bits(n[k])) * 1099511628211ull;
    for (size_t i = 0; i < MyMesh.triangles.size(); ++i) {
        for (int k = 0; k < 3; ++k) ht = (ht ^ MyMesh.triangles[i].v[k]) * 1099511628211ull;
        ht = (ht ^ MyMesh.triangleMaterials[i]) * 1099511628211ull;
    }
    std::printf("digest %016llx %016llx %016llx\n", hv, hn, ht);
    for (int t : {0, static_cast<int>(MyMesh.triangles.size()) - 1}) {
        const Material m = getMaterial(t);
        std::printf("material %d %08x %08x %08x %08x %08x %08x %d %d%d%d%d%d\n", t, bits(m.Kd()[0]), bits(m.Kd()[1]),
                    bits(m.Kd()[2]), bits(m.Ks()[0]), bits(m.Ns()), bits(m.Tr()), m.illum(), m.has_Kd(), m.has_Ka(),
                    m.has_Ks(), m.has_Ns(), m.has_Tr());
    }
    if (!gpu) return 0;
    if (argc < 9) return 2;
    WindowSize_X = static_cast<unsigned>(std::atoi(argv[3]));
    WindowSize_Y = static_cast<unsigned>(std::atoi(argv[4]));
    pixelfactorX = pixelfactorY = static_cast<unsigned>(std::atoi(argv[5]));
    max_lvl = std::atoi(argv[6]);
    MyLightPositions.push_back(Vec3Df(1.5f, 1.5f, 4.0f));
    if (rt_default_corners(static_cast<int32_t>(WindowSize_X), static_cast<int32_t>(WindowSize_Y), g_corners) != RT_OK)
        return 3;

    // ---- the 'r' key, one performRayTracing per sub-sample ----
    std::vector<float> image(3u * WindowSize_X * WindowSize_Y);
    Vec3Df origin00, dest00, origin01, dest01, origin10, dest10, origin11, dest11, origin, dest;
    produceRay(0, 0, &origin00, &dest00);
    produceRay(0, WindowSize_Y - 1, &origin01, &dest01);
    produceRay(WindowSize_X - 1, 0, &origin10, &dest10);
    produceRay(WindowSize_X - 1, WindowSize_Y - 1, &origin11, &dest11);
    float divX = (WindowSize_X * pixelfactorX - 1);
    float divY = (WindowSize_Y * pixelfactorY - 1);
    int raysPerPixel = (pixelfactorX * pixelfactorY);
    for (unsigned int y = 0; y < WindowSize_Y; ++y) {
        for (unsigned int x = 0; x < WindowSize_X; ++x) {
            Vec3Df rgb = Vec3Df(0, 0, 0);
            for (int subx = 0; subx < static_cast<int>(pixelfactorX); subx++) {
                for (int suby = 0; suby < static_cast<int>(pixelfactorY); suby++) {
                    float xscale = 1.0f - (float(x) * pixelfactorX + subx) / divX;
                    float yscale = 1.0f - (float(y) * pixelfactorY + suby) / divY;
                    origin = yscale * (xscale * origin00 + (1 - xscale) * origin10) +
                             (1 - yscale) * (xscale * origin01 + (1 - xscale) * origin11);
                    dest = yscale * (xscale * dest00 + (1 - xscale) * dest10) +
                           (1 - yscale) * (xscale * dest01 + (1 - xscale) * dest11);
                    rgb += performRayTracing(origin, dest);
                }
            }
            rgb = rgb / raysPerPixel;
            const size_t o = 3u * (WindowSize_X * y + x);
            for (int k = 0; k < 3; ++k) image[o + k] = clamp01(rgb[k]);
        }
    }
    // ---- the same frame in one call ----
    uint64_t rays[3] = {0, 0, 0};
    const std::vector<float> fast =
        renderImage(origin00, dest00, origin01, dest01, origin10, dest10, origin11, dest11, rays);
    size_t same_bits = 0;
    for (size_t i = 0; i < image.size(); ++i) same_bits += bits(image[i]) == bits(fast[i]);
    std::printf("frames %zu %zu rays %llu %llu %llu\n", same_bits, image.size(), (unsigned long long)rays[0],
                (unsigned long long)rays[1], (unsigned long long)rays[2]);
    // a few single-ray entry points of the interface
    Vec3Df I;
    const int idx = intersectMesh(origin00 * 0.5f + origin11 * 0.5f, dest00 * 0.5f + dest11 * 0.5f, &I);
    Vec3Df R[2] = {origin00 * 0.5f + origin11 * 0.5f, dest00 * 0.5f + dest11 * 0.5f};
    Vec3Df T[3] = {MyMesh.vertices[MyMesh.triangles[idx < 0 ? 0 : idx].v[0]].p,
                   MyMesh.vertices[MyMesh.triangles[idx < 0 ? 0 : idx].v[1]].p,
                   MyMesh.vertices[MyMesh.triangles[idx < 0 ? 0 : idx].v[2]].p};
    Vec3Df I2;
    const bool hit = rayIntersectTriangle(R, T, &I2);
    std::printf("centre %d %08x %08x %08x tri_hit %d same_point %d\n", idx, bits(I[0]), bits(I[1]), bits(I[2]), hit ? 1 : 0,
                hit && I == I2 ? 1 : 0);
    return writePPM(argv[7], WindowSize_X, WindowSize_Y, image) && writePPM(argv[8], WindowSize_X, WindowSize_Y, fast) ? 0 : 4;
}
