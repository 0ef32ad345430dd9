/* raytracert.hpp — C++ host layer over librtamd.so (include/raytracert.h) with the names and
 * argument meaning of the reference's tracer interface (CG_Project/raytracing.h), so a host that
 * calls init / performRayTracing / trace / getMaterial keeps its code and gets the MI355X path.
 *
 *   reference (CG_Project/)                      here (namespace rtamd)
 *   extern Mesh MyMesh; normals (raytracing.h:8)  RayTracer holds the scene (rt_scene)
 *   MyLightPositions, MyCameraPosition,           RayTracer members of the same names
 *   WindowSize_X/Y, pixelfactorX/Y, max_lvl,
 *   Ambient ... Refraction (raytracing.cpp:15-29)
 *   void init(char*)              :19, .cpp:42-73  RayTracer::init — load OBJ/MTL, face normals,
 *                                                  light 0 = the camera position
 *   Material getMaterial(int)     :27, .cpp:373    RayTracer::getMaterial
 *   Vec3Df trace(o, d, lvl)       :30, .cpp:381    RayTracer::trace (max_lvl - lvl levels left)
 *   Vec3Df performRayTracing(o,d) :33, .cpp:410    RayTracer::performRayTracing (+ a batched form)
 *   intersectMesh (.cpp:161-192)                   RayTracer::intersectMesh
 *   key 'd' debug shot (.cpp:493-510)              RayTracer::debugTrace
 *   key 'r' frame loop (main.cpp:340-411)          RayTracer::render (+ writeImage)
 *
 * Vec3Df is layout-compatible with the reference's Vec3D<float> (three floats, Vec3D.h:272,291)
 * and Material exposes the accessors of mesh.h:10-125. Failures throw rtamd::Error with
 * rt_last_error_string() (the reference has no error path: a missing OBJ crashes, mesh.cpp:329).
 * Header-only; link with -lrtamd. */
#ifndef RAYTRACERT_HPP_
#define RAYTRACERT_HPP_

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "raytracert.h"

namespace rtamd {

class Error : public std::runtime_error {
  public:
    Error(int code, const std::string &what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

  private:
    int code_;
};

inline void check(int rc) {
    if (rc != RT_OK) throw Error(rc, rt_last_error_string());
}

struct Vec3Df {
    float p[3];
    Vec3Df() : p{0.0f, 0.0f, 0.0f} {}
    Vec3Df(float x, float y, float z) : p{x, y, z} {}
    float &operator[](int i) { return p[i]; }
    const float &operator[](int i) const { return p[i]; }
    Vec3Df operator+(const Vec3Df &o) const { return Vec3Df(p[0] + o.p[0], p[1] + o.p[1], p[2] + o.p[2]); }
    Vec3Df operator-(const Vec3Df &o) const { return Vec3Df(p[0] - o.p[0], p[1] - o.p[1], p[2] - o.p[2]); }
    Vec3Df operator*(float f) const { return Vec3Df(p[0] * f, p[1] * f, p[2] * f); }
    bool operator==(const Vec3Df &o) const { return p[0] == o.p[0] && p[1] == o.p[1] && p[2] == o.p[2]; }
    static float dotProduct(const Vec3Df &a, const Vec3Df &b) { return a.p[0] * b.p[0] + a.p[1] * b.p[1] + a.p[2] * b.p[2]; }
};
static_assert(sizeof(Vec3Df) == 12, "Vec3Df must be three packed floats");
static_assert(sizeof(Vec3Df) == sizeof(rt_vec3), "Vec3Df and rt_vec3 share the layout");

// Material with the accessor names of the reference (mesh.h:10-125)
class Material {
  public:
    Material() : m_{} {}
    explicit Material(const rt_material &m) : m_(m) {}
    Vec3Df Kd() const { return Vec3Df(m_.Kd[0], m_.Kd[1], m_.Kd[2]); }
    Vec3Df Ka() const { return Vec3Df(m_.Ka[0], m_.Ka[1], m_.Ka[2]); }
    Vec3Df Ks() const { return Vec3Df(m_.Ks[0], m_.Ks[1], m_.Ks[2]); }
    float Ns() const { return m_.Ns; }
    float Ni() const { return m_.Ni; }
    float Tr() const { return m_.Tr; }
    int illum() const { return m_.illum; }
    bool has_Kd() const { return (m_.flags & RT_HAS_KD) != 0; }
    bool has_Ka() const { return (m_.flags & RT_HAS_KA) != 0; }
    bool has_Ks() const { return (m_.flags & RT_HAS_KS) != 0; }
    bool has_Ns() const { return (m_.flags & RT_HAS_NS) != 0; }
    bool has_Ni() const { return (m_.flags & RT_HAS_NI) != 0; }
    bool has_illum() const { return (m_.flags & RT_HAS_ILLUM) != 0; }
    bool has_Tr() const { return (m_.flags & RT_HAS_TR) != 0; }
    bool is_valid() const { return has_Kd() || has_Ka() || has_Ks() || has_Tr(); }   // mesh.h:55-56
    const rt_material &raw() const { return m_; }

  private:
    rt_material m_;
};

class RayTracer {
  public:
    // the reference's globals (raytracing.h:8-16, raytracing.cpp:15-29, main.cpp:130-138)
    std::vector<Vec3Df> MyLightPositions;
    Vec3Df MyCameraPosition{0.0f, 0.0f, 4.0f};
    unsigned int WindowSize_X = 800, WindowSize_Y = 800;
    unsigned int pixelfactorX = 3, pixelfactorY = 3;
    int max_lvl = 10;
    bool Ambient = true, Diffuse = true, Reflection = true, Shadows = true, Specular = true, Refraction = true;

    // device: a HIP device index, or RT_HOST_ONLY (loader and getMaterial only)
    explicit RayTracer(int device = 0) : device_(device) {}
    ~RayTracer() { rt_scene_destroy(scene_); }
    RayTracer(const RayTracer &) = delete;
    RayTracer &operator=(const RayTracer &) = delete;

    // init(char*), raytracing.cpp:42-73: loadMesh + calculateNormals, then light 0 = camera
    void init(const char *fileName) {
        rt_scene_destroy(scene_);
        scene_ = nullptr;
        check(rt_scene_load_obj(fileName ? fileName : "cube.obj", device_, &scene_));
        MyLightPositions.push_back(MyCameraPosition);
    }

    // getMaterial(int), raytracing.cpp:373-376
    Material getMaterial(int index) const {
        rt_material m;
        check(rt_get_material(scene_, index, &m));
        return Material(m);
    }

    // intersectMesh, raytracing.cpp:161-192: closest triangle index or -1, point in *intersectOut
    int intersectMesh(const Vec3Df &origin, const Vec3Df &dest, Vec3Df *intersectOut) const {
        int32_t idx = -1;
        Vec3Df I;
        check(rt_intersect_mesh(scene_, origin.p, dest.p, 1, &idx, I.p));
        if (intersectOut) *intersectOut = I;
        return idx;
    }

    // trace(origin, dest, lvl), raytracing.cpp:381-406: the chain below level lvl of max_lvl
    // (every level test is lvl < max_lvl with unit steps, so it is the max_lvl - lvl chain)
    Vec3Df trace(const Vec3Df &origin, const Vec3Df &dest, int lvl) {
        rt_params p = params();
        p.max_lvl = lvl >= max_lvl ? 0 : max_lvl - lvl;
        Vec3Df c;
        check(rt_trace_rays(scene_, &p, origin.p, dest.p, 1, c.p, nullptr));
        return c;
    }

    // performRayTracing, raytracing.cpp:410-416 (= trace(origin, dest, 0))
    Vec3Df performRayTracing(const Vec3Df &origin, const Vec3Df &dest) { return trace(origin, dest, 0); }

    // the same for many rays at once (the form the GPU wants)
    std::vector<Vec3Df> performRayTracing(const std::vector<Vec3Df> &origins, const std::vector<Vec3Df> &dests) {
        if (origins.size() != dests.size()) throw Error(RT_E_ARG, "origins/dests size mismatch");
        std::vector<Vec3Df> out(origins.size());
        rt_params p = params();
        check(rt_trace_rays(scene_, &p, origins.empty() ? nullptr : origins[0].p, dests.empty() ? nullptr : dests[0].p,
                            static_cast<int32_t>(origins.size()), out.empty() ? nullptr : out[0].p, nullptr));
        return out;
    }

    // the debug key 'd' (raytracing.cpp:493-510): every trace() of the ray's chain, and its colour
    std::vector<rt_debug_bounce> debugTrace(const Vec3Df &origin, const Vec3Df &dest, Vec3Df *color = nullptr) {
        std::vector<rt_debug_bounce> b(static_cast<size_t>(max_lvl) * 2 + 2);
        int32_t n = 0;
        Vec3Df c;
        rt_params p = params();
        check(rt_debug_trace(scene_, &p, origin.p, dest.p, b.data(), static_cast<int32_t>(b.size()), &n, c.p));
        b.resize(static_cast<size_t>(n) < b.size() ? static_cast<size_t>(n) : b.size());
        if (color) *color = c;
        return b;
    }

    // the 'r' key (main.cpp:340-411): WindowSize_X x WindowSize_Y bytes as Image::writeImage
    // writes them. corners = the four produceRay results origin00, dest00, origin01, dest01,
    // origin10, dest10, origin11, dest11 (main.cpp:355-358); nullptr: the default view.
    std::vector<unsigned char> render(const Vec3Df *corners = nullptr, uint64_t rays[3] = nullptr) {
        rt_params p = params();
        if (corners) {
            for (int i = 0; i < 8; ++i)
                for (int k = 0; k < 3; ++k) p.corners[i][k] = corners[i][k];
        } else {
            check(rt_default_corners(p.width, p.height, p.corners));
        }
        std::vector<unsigned char> img(3u * WindowSize_X * WindowSize_Y);
        check(rt_render_tile(scene_, &p, 0, 0, p.width, p.height, img.data(), nullptr, rays));
        return img;
    }

    // Image::writeImage (main.cpp:106-128)
    void writeImage(const char *filename, const std::vector<unsigned char> &rgb) const {
        check(rt_write_ppm(filename, static_cast<int32_t>(WindowSize_X), static_cast<int32_t>(WindowSize_Y), rgb.data()));
    }

    rt_scene *scene() const { return scene_; }

    rt_params params() const {
        rt_params p{};
        p.width = static_cast<int32_t>(WindowSize_X);
        p.height = static_cast<int32_t>(WindowSize_Y);
        p.pfx = static_cast<int32_t>(pixelfactorX);
        p.pfy = static_cast<int32_t>(pixelfactorY);
        p.max_lvl = max_lvl;
        p.flags = (Ambient ? RT_AMBIENT : 0u) | (Diffuse ? RT_DIFFUSE : 0u) | (Specular ? RT_SPECULAR : 0u) |
                  (Reflection ? RT_REFLECTION : 0u) | (Shadows ? RT_SHADOWS : 0u) | (Refraction ? RT_REFRACTION : 0u);
        // any number of lights (the reference's list is an unbounded vector): the first RT_MAX_LIGHTS
        // inline, and the whole list through light_list (Vec3Df is three packed floats), read during the call
        p.n_lights = static_cast<int32_t>(MyLightPositions.size());
        for (size_t i = 0; i < MyLightPositions.size() && i < RT_MAX_LIGHTS; ++i)
            for (int k = 0; k < 3; ++k) p.lights[i][k] = MyLightPositions[i][k];
        if (MyLightPositions.size() > RT_MAX_LIGHTS) p.light_list = MyLightPositions[0].p;
        for (int k = 0; k < 3; ++k) p.camera_pos[k] = MyCameraPosition[k];
        return p;
    }

  private:
    int device_;
    rt_scene *scene_ = nullptr;
};

}  // namespace rtamd

#endif  // RAYTRACERT_HPP_
