// A host written fresh against the reference tracer's interface, the way CG_Project/main.cpp uses
// it, compiled with g++ against include/ only (raytracert_dropin.hpp in place of raytracing.h +
// mesh.h) and linked with librtamd. It makes every reference-API call main.cpp makes:
//   MyMesh.draw() (main.cpp:179) and yourDebugDraw() (:186) from the preview's draw function,
//   init(argv[1]) (:258), produceRay in both overloads (defined here, :300-325, without GL),
//   the 'r' key (:340-411): four produceRay corners, the per-sub-sample loop with performRayTracing,
//   rgb / raysPerPixel, RGBValue's clamp, Image::writeImage's truncation,
//   'L' / 'l' (:334-339) and yourKeyboardFunc(key, x, y) (:417) for every key.
// The keys come from the command line, so tests/test_cxx_dropin.py can replay a session and check
// each frame and each 'd' colour against the oracle with the same toggles.
//   dropin_main host <obj>                                    loader, MyMesh, normals, getMaterial
//   dropin_main keys <obj> W H <prefix> <key> [<key> ...]     a key session; 'r' writes <prefix>N.ppm
// A key is one character; 'd@X,Y' is 'd' with the mouse at (X, Y); 'R' renders through the one-call
// renderImage() for comparison; 'T' times the 'r' loop, 'H' the same loop with no trace at all (the
// host floor), 'P:N' N single performRayTracing calls on rays the frame cache has never seen.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#ifdef RTAMD_REFCOMPAT   // main.cpp:13-14 unchanged, include/refcompat on the include path
#include "raytracing.h"
#include "mesh.h"
#else
#include "raytracert_dropin.hpp"
#endif

// ---- the globals main.cpp defines (main.cpp:17-18,130,137-141) ----
Vec3Df MyCameraPosition;
std::vector<Vec3Df> MyLightPositions;
Mesh MyMesh;
unsigned int WindowSize_X = 500;
unsigned int WindowSize_Y = 500;
unsigned int RayTracingResolutionX = 500;
unsigned int RayTracingResolutionY = 500;

// ---- RGBValue and Image (main.cpp:21-128) ----
class RGBValue {
  public:
    RGBValue(float rI = 0, float gI = 0, float bI = 0) : r(rI), b(bI), g(gI) {
        if (r > 1) r = 1.0;
        if (g > 1) g = 1.0;
        if (b > 1) b = 1.0;
        if (r < 0) r = 0.0;
        if (g < 0) g = 0.0;
        if (b < 0) b = 0.0;
    }
    float operator[](int i) const { return i == 1 ? g : i == 2 ? b : r; }
    float r, b, g;
};

class Image {
  public:
    Image(int width, int height) : _width(width), _height(height) { _image.resize(3 * _width * _height); }
    void setPixel(int i, int j, const RGBValue &rgb) {
        for (int k = 0; k < 3; ++k) _image[3 * (_width * j + i) + k] = rgb[k];
    }
    bool writeImage(const char *filename) {
        FILE *file = std::fopen(filename, "wb");
        if (!file) return false;
        std::fprintf(file, "P6\n%i %i\n255\n", _width, _height);
        std::vector<unsigned char> imageC(_image.size());
        for (unsigned int i = 0; i < _image.size(); ++i) imageC[i] = (unsigned char)(_image[i] * 255.0f);
        const bool ok = std::fwrite(&imageC[0], _width * _height * 3, 1, file) == 1;
        std::fclose(file);
        return ok;
    }
    std::vector<float> _image;
    int _width, _height;
};

// ---- produceRay without GL: the default view's corner rays (rt_default_corners restates
// gluPerspective + gluUnProject for main.cpp's pose), blended bilinearly for other pixels ----
static float g_c[8][3];
void produceRay(int x_I, int y_I, Vec3Df *origin, Vec3Df *dest) {
    const float fx = WindowSize_X > 1 ? float(x_I) / float(WindowSize_X - 1) : 0.0f;
    const float fy = WindowSize_Y > 1 ? float(y_I) / float(WindowSize_Y - 1) : 0.0f;
    for (int k = 0; k < 3; ++k) {   // corners exact at the four corner pixels
        origin->p[k] = (1 - fx) * ((1 - fy) * g_c[0][k] + fy * g_c[2][k]) + fx * ((1 - fy) * g_c[4][k] + fy * g_c[6][k]);
        dest->p[k] = (1 - fx) * ((1 - fy) * g_c[1][k] + fy * g_c[3][k]) + fx * ((1 - fy) * g_c[5][k] + fy * g_c[7][k]);
    }
    if (fx == 0 || fx == 1)
        if (fy == 0 || fy == 1) {
            const int k = 2 * (2 * (fx == 1) + (fy == 1));
            *origin = Vec3Df(g_c[k]);   // Vec3D(T*), implicit as Vec3D.h:70
            *dest = Vec3Df(g_c[k + 1]);
        }
}
void produceRay(int x_I, int y_I, Vec3Df &origin, Vec3Df &dest) { produceRay(x_I, y_I, &origin, &dest); }

// ---- the preview's draw (main.cpp:169-187) ----
static void dessiner() {
    MyMesh.draw();
    yourDebugDraw();
}

static int g_frame = 0;
static std::string g_prefix;

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- the 'r' key (main.cpp:340-411) ----
static void render_r(bool timed) {
    const double t0 = now_s();
    Image result(WindowSize_X, WindowSize_Y);
    Vec3Df origin00, dest00;
    Vec3Df origin01, dest01;
    Vec3Df origin10, dest10;
    Vec3Df origin11, dest11;
    Vec3Df origin, dest;
    produceRay(0, 0, &origin00, &dest00);
    produceRay(0, WindowSize_Y - 1, &origin01, &dest01);
    produceRay(WindowSize_X - 1, 0, &origin10, &dest10);
    produceRay(WindowSize_X - 1, WindowSize_Y - 1, &origin11, &dest11);
    float divX = (WindowSize_X * pixelfactorX - 1);
    float divY = (WindowSize_Y * pixelfactorY - 1);
    int raysPerPixel = (pixelfactorX * pixelfactorY);
    double tc0 = 0, tc1 = 0;   // (the frame's first call, which traces the whole frame: timed apart)
    for (unsigned int y = 0; y < WindowSize_Y; ++y) {
        for (unsigned int x = 0; x < WindowSize_X; ++x) {
            Vec3Df rgb = Vec3Df(0, 0, 0);
            for (int subx = 0; subx < (int)pixelfactorX; subx++) {
                for (int suby = 0; suby < (int)pixelfactorY; suby++) {
                    float xscale = 1.0f - (float(x) * pixelfactorX + subx) / divX;
                    float yscale = 1.0f - (float(y) * pixelfactorY + suby) / divY;
                    origin = yscale * (xscale * origin00 + (1 - xscale) * origin10) +
                             (1 - yscale) * (xscale * origin01 + (1 - xscale) * origin11);
                    dest = yscale * (xscale * dest00 + (1 - xscale) * dest10) +
                           (1 - yscale) * (xscale * dest01 + (1 - xscale) * dest11);
                    if (y == 0 && x == 0 && subx == 0 && suby == 0) {
                        tc0 = now_s();
                        rgb += performRayTracing(origin, dest);
                        tc1 = now_s();
                    } else {
                        rgb += performRayTracing(origin, dest);
                    }
                }
            }
            rgb = rgb / raysPerPixel;
            result.setPixel(x, y, RGBValue(rgb[0], rgb[1], rgb[2]));
        }
    }
    const double t1 = now_s();
    const std::string path = g_prefix + std::to_string(g_frame++) + ".ppm";
    result.writeImage(path.c_str());
    std::printf("frame %s pf %u %u flags %d%d%d%d%d%d lights %zu ms %.3f first_call_ms %.3f\n", path.c_str(), pixelfactorX,
                pixelfactorY, Ambient, Diffuse, Specular, Reflection, Shadows, Refraction, MyLightPositions.size(),
                timed ? 1e3 * (t1 - t0) : 0.0, timed ? 1e3 * (tc1 - tc0) : 0.0);
}

// The host floor of the 'r' loop: the same loop with performRayTracing replaced by a function that
// only reads its arguments (no GPU, no cache lookup): what the unchanged loop costs by itself.
static Vec3Df host_only_trace(const Vec3Df &o, const Vec3Df &d) { return Vec3Df(o[0] * 1e-9f, d[1] * 1e-9f, 0.5f); }
static void render_host_floor() {
    const double t0 = now_s();
    Vec3Df origin00, dest00, origin01, dest01, origin10, dest10, origin11, dest11, origin, dest;
    produceRay(0, 0, &origin00, &dest00);
    produceRay(0, WindowSize_Y - 1, &origin01, &dest01);
    produceRay(WindowSize_X - 1, 0, &origin10, &dest10);
    produceRay(WindowSize_X - 1, WindowSize_Y - 1, &origin11, &dest11);
    float divX = (WindowSize_X * pixelfactorX - 1);
    float divY = (WindowSize_Y * pixelfactorY - 1);
    int raysPerPixel = (pixelfactorX * pixelfactorY);
    Vec3Df acc(0, 0, 0);
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
                    rgb += host_only_trace(origin, dest);
                }
            acc += rgb / raysPerPixel;
        }
    std::printf("hostfloor %u x %u pf %u ms %.3f (checksum %g)\n", WindowSize_X, WindowSize_Y, pixelfactorX,
                1e3 * (now_s() - t0), acc[0] + acc[1] + acc[2]);
}

// the same frame through renderImage (one call), written like the loop's Image
static void render_one_call() {
    Vec3Df c[8];
    produceRay(0, 0, &c[0], &c[1]);
    produceRay(0, WindowSize_Y - 1, &c[2], &c[3]);
    produceRay(WindowSize_X - 1, 0, &c[4], &c[5]);
    produceRay(WindowSize_X - 1, WindowSize_Y - 1, &c[6], &c[7]);
    const double t0 = now_s();
    uint64_t rays[3] = {0, 0, 0};
    Image result(WindowSize_X, WindowSize_Y);
    result._image = renderImage(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], rays);
    const double t1 = now_s();
    const std::string path = g_prefix + std::to_string(g_frame++) + ".ppm";
    result.writeImage(path.c_str());
    std::printf("frame %s pf %u %u renderImage ms %.3f rays %llu %llu %llu\n", path.c_str(), pixelfactorX, pixelfactorY,
                1e3 * (t1 - t0), (unsigned long long)rays[0], (unsigned long long)rays[1], (unsigned long long)rays[2]);
}

// ---- keyboard (main.cpp:328-418), with a getCameraPosition stand-in for 'L' / 'l' ----
static Vec3Df getCameraPosition() { return Vec3Df(0.0f, 0.0f, 4.0f); }
static void keyboard(unsigned char key, int x, int y) {
    std::printf("key %d pressed at %d,%d\n", key, x, y);
    std::fflush(stdout);
    switch (key) {
        case 'L': MyLightPositions.push_back(getCameraPosition()); break;
        case 'l': MyLightPositions[MyLightPositions.size() - 1] = getCameraPosition(); break;
        case 'r': render_r(false); break;
    }
    yourKeyboardFunc(key, x, y);
}

static unsigned bits(float f) { unsigned u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const bool host = std::strcmp(argv[1], "host") == 0;
    RayTracerDevice = host ? RT_HOST_ONLY : 0;
    MyCameraPosition = getCameraPosition();
    init(argv[2]);   // main.cpp:258
    if (host) {
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
        // Vec3D API surface (Vec3D.h): getTwoOrthogonals, toString, swap
        Vec3Df a(0.25f, -2.0f, 1.0f), u, v;
        a.getTwoOrthogonals(u, v);
        char buf[64];
        Vec3Df b(1, 2, 3);
        swap(a, b);
        std::printf("vec %g %g %s\n", Vec3Df::dotProduct(b, u), Vec3Df::dotProduct(b, v), a.toString(buf, sizeof buf));
        // Mesh::texcoords and Triangle::t (mesh.cpp:199-209, 263-316)
        unsigned long long htc = 1469598103934665603ull, htt = htc;
        for (const Vec3Df &t : MyMesh.texcoords)
            for (int k = 0; k < 3; ++k) htc = (htc ^ bits(t[k])) * 1099511628211ull;
        for (const Triangle &t : MyMesh.triangles)
            for (int k = 0; k < 3; ++k) htt = (htt ^ t.t[k]) * 1099511628211ull;
        std::printf("texcoords %zu %016llx %016llx\n", MyMesh.texcoords.size(), htc, htt);
        // Mesh::loadMtl as a separate call (argv[3]): into an empty mesh with an empty index
        if (argc > 3) {
            Mesh m;
            std::map<std::string, unsigned int> index;
            const bool ok = m.loadMtl(argv[3], index);
            std::printf("loadmtl %d %zu", ok ? 1 : 0, m.materials.size());
            for (const auto &kv : index) std::printf(" %s=%u", kv.first.c_str(), kv.second);
            std::printf("\n");
            for (const Material &mm : m.materials)
                std::printf("mtl %s %08x %08x %08x %08x %d\n", mm.name().c_str(), bits(mm.Kd()[0]), bits(mm.Ka()[1]),
                            bits(mm.Tr()), bits(mm.Ns()), mm.has_Ks());
        }
        dessiner();
        return 0;
    }
    if (argc < 6) return 2;
    WindowSize_X = static_cast<unsigned>(std::atoi(argv[3]));
    WindowSize_Y = static_cast<unsigned>(std::atoi(argv[4]));
    g_prefix = argv[5];
    if (rt_default_corners(static_cast<int32_t>(WindowSize_X), static_cast<int32_t>(WindowSize_Y), g_c) != RT_OK) return 3;
    for (int i = 6; i < argc; ++i) {
        const char *k = argv[i];
        if (k[0] == 'd' && k[1] == '@') {   // 'd' with the mouse at (X, Y): print the ray it shoots
            int x = 0, y = 0;
            std::sscanf(k + 2, "%d,%d", &x, &y);
            Vec3Df o, d;
            produceRay(x, y, o, d);
            std::printf("dray %08x %08x %08x %08x %08x %08x\n", bits(o[0]), bits(o[1]), bits(o[2]), bits(d[0]), bits(d[1]),
                        bits(d[2]));
            const size_t before = rtamd_dropin::debug_origins.size();
            keyboard('d', x, y);
            for (size_t j = before; j < rtamd_dropin::debug_origins.size(); ++j) {   // what 'd' recorded
                const Vec3Df &a = rtamd_dropin::debug_origins[j], &h = rtamd_dropin::debug_hits[j];
                std::printf("dpair %08x %08x %08x %08x %08x %08x\n", bits(a[0]), bits(a[1]), bits(a[2]), bits(h[0]), bits(h[1]),
                            bits(h[2]));
            }
        } else if (k[0] == 'R') {
            render_one_call();
        } else if (k[0] == 'T') {
            render_r(true);
            std::printf("cache host_ray_frames %zu device_frames %zu\n", rtamd_dropin::frame_cache().host_ray_frames,
                        rtamd_dropin::frame_cache().device_frames);
        } else if (k[0] == 'H') {
            render_host_floor();
        } else if (k[0] == 'M' && k[1] == ':') {   // max_lvl (raytracing.cpp:29) set by the host, e.g. a BASELINE config
            max_lvl = std::atoi(k + 2);
        } else if (k[0] == 'A' && k[1] == ':') {   // a light at a given position (as 'L' appends the camera's)
            float x = 0, y = 0, z = 0;
            std::sscanf(k + 2, "%f,%f,%f", &x, &y, &z);
            MyLightPositions.push_back(Vec3Df(x, y, z));
        } else if (k[0] == 'V' && k[1] == ':') {   // after a frame: N of its cached records against the per-call path
            // (the loop's own ray for the record, made by this translation unit as the loop makes it, and
            // trace(origin, dest, 0): one rt_trace_rays of that ray)
            const int n = std::atoi(k + 2);
            const rtamd_dropin::FrameCache &fc = rtamd_dropin::frame_cache();
            Vec3Df c[8];
            produceRay(0, 0, c[0], c[1]);
            produceRay(0, WindowSize_Y - 1, c[2], c[3]);
            produceRay(WindowSize_X - 1, 0, c[4], c[5]);
            produceRay(WindowSize_X - 1, WindowSize_Y - 1, c[6], c[7]);
            const float divX = (WindowSize_X * pixelfactorX - 1), divY = (WindowSize_Y * pixelfactorY - 1);
            const size_t spp = size_t(pixelfactorX) * pixelfactorY;
            int ray_diff = 0, rgb_diff = 0;
            for (int j = 0; j < n && fc.n > 0; ++j) {
                const size_t s = (fc.n - 1) * size_t(j) / size_t(n > 1 ? n - 1 : 1), pix = s / spp, sub = s % spp;
                const unsigned x = unsigned(pix % WindowSize_X), y = unsigned(pix / WindowSize_X);
                const int subx = int(sub / pixelfactorY), suby = int(sub % pixelfactorY);
                float xscale = 1.0f - (float(x) * pixelfactorX + subx) / divX;   // main.cpp:380-386, as render_r
                float yscale = 1.0f - (float(y) * pixelfactorY + suby) / divY;
                Vec3Df origin = yscale * (xscale * c[0] + (1 - xscale) * c[4]) + (1 - yscale) * (xscale * c[2] + (1 - xscale) * c[6]);
                Vec3Df dest = yscale * (xscale * c[1] + (1 - xscale) * c[5]) + (1 - yscale) * (xscale * c[3] + (1 - xscale) * c[7]);
                const float *r = fc.rec + 9 * s;
                ray_diff += std::memcmp(r, origin.p, 12) != 0 || std::memcmp(r + 3, dest.p, 12) != 0;
                const Vec3Df t = trace(origin, dest, 0);
                rgb_diff += std::memcmp(r + 6, t.p, 12) != 0;
            }
            std::printf("verify %d records ray_diff %d rgb_diff %d host_rays %d\n", n, ray_diff, rgb_diff, fc.host_rays ? 1 : 0);
        } else if (k[0] == 'P' && k[1] == ':') {   // single calls off the frame cache (rays of no frame)
            const int n = std::atoi(k + 2);
            Vec3Df o00, d00, o11, d11, acc;
            produceRay(0, 0, o00, d00);
            produceRay(WindowSize_X - 1, WindowSize_Y - 1, o11, d11);
            const double t0 = now_s();
            for (int j = 0; j < n; ++j) {
                const float t = (j + 0.5f) / n;
                acc += performRayTracing(o00 * (1 - t) + o11 * t, d00 * (1 - t) + d11 * t);
            }
            std::printf("single %d calls us_per_call %.2f sum %g\n", n, 1e6 * (now_s() - t0) / n, acc[0] + acc[1] + acc[2]);
        } else {
            keyboard(static_cast<unsigned char>(k[0]), 0, 0);
        }
        dessiner();
    }
    return 0;
}
