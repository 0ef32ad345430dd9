/* raytracert_dropin.hpp — source-level drop-in for the reference tracer's headers over librtamd.so.
 *
 * The reference's render path is declared in CG_Project/raytracing.h (globals and functions), with
 * its types in Vec3D.h, Vertex.h and mesh.h, and defined in raytracing.cpp + mesh.cpp. A host
 * (the reference's main.cpp) switches by editing its two includes, main.cpp:13-14,
 *     #include "raytracing.h"  +  #include "mesh.h"      ->      #include "raytracert_dropin.hpp"
 * (or, with no edit at all, by putting include/refcompat/ first on its include path: its
 * raytracing.h, mesh.h, Vec3D.h and Vertex.h forward to this header), and by dropping
 * raytracing.cpp and mesh.cpp from its build. Every reference-API call main.cpp makes then compiles
 * and links against include/ + librtamd: MyMesh.draw() (main.cpp:179), yourDebugDraw() (:186),
 * init() (:258), produceRay (defined by main.cpp, :300-325), the 'r' loop's performRayTracing per
 * sub-sample and Vec3Df arithmetic (:355-395), yourKeyboardFunc() (:417). tests/cxx/dropin_main.cpp
 * is such a host, written fresh against the reference interface.
 *
 *   reference                                   here
 *   template Vec3D<T>, Vec3Df (Vec3D.h)         Vec3D<T> with the same members, operators and operation order
 *   Vertex (Vertex.h), Triangle, Material,      the same members and accessors; Mesh::loadMesh loads
 *   Mesh (mesh.h:10-201)                        through librtamd (mesh.cpp semantics); draw/drawSmooth
 *                                               draw with GL when the host defines RTAMD_DROPIN_GL
 *   globals of raytracing.h:8-16                declared extern here, defined by the host's main.cpp
 *                                               as before (MyMesh, MyLightPositions, ...)
 *   globals of raytracing.cpp:15-36             defined here (inline): Ambient..Refraction, WireFrame,
 *                                               pixelfactorX/Y, max_lvl, normals (the debug-ray lists
 *                                               and DebugMode live in namespace rtamd_dropin)
 *   init, calculateNormals, getMaterial,        same signatures and meaning; the ray functions run
 *   trace, performRayTracing, intersectMesh,    on the GPU scene built from MyMesh (uploadMesh())
 *   rayIntersectTriangle, isNullVector,
 *   yourDebugDraw, yourKeyboardFunc             the keys of raytracing.cpp:453-553 ('d' through
 *                                               rt_debug_trace)
 *
 * performRayTracing and the 'r' loop: a call whose (origin, dest) is the first sub-sample of the
 * loop main.cpp:369-388 runs for the current corner rays (produceRay) makes the header trace every
 * sub-sample of that frame in one GPU call (rt_trace_frame_samples: the device makes the loop's rays
 * with the loop's own binary32 expressions and returns, per sub-sample in the loop's order, the ray and
 * its colour into pinned memory); the loop's later calls are answered from it while each (origin,
 * dest) equals the next record's ray bit for bit and every parameter the trace reads is unchanged, and
 * any other call is traced on its own. The colours are those of the per-call path either way (each
 * is the trace of the very ray the call passed; tests/test_cxx_dropin.py checks both against the
 * oracle); the unchanged loop just stops paying one GPU round trip per sub-sample
 * (RTAMD_DROPIN_NO_FRAME_CACHE turns it off).
 *
 * Extra: RayTracerDevice (the GPU init() binds; RT_HOST_ONLY = loader only), uploadMesh() (re-upload
 * MyMesh after editing it), renderImage() (the 'r' loop in one call, Image::_image's floats),
 * performRayTracing over vectors (batched). Failures throw rtamd_dropin::Error (the reference has no
 * error path). Mesh::texcoords and Triangle::t are loaded as mesh.cpp loads them
 * (RT_LOAD_TEXCOORDS) and Mesh::loadMtl is a separate call too (rt_load_mtl), though the render
 * path reads neither. Not provided (never called by main.cpp, no effect on the image): the dead
 * box/rectangle intersectors and getTeller (declared, never defined by the reference), and
 * trace()'s DebugMode records of 'r' frames (every ray of a frame; they only feed the debug draw).
 * Header-only; C++17; -lrtamd.
 */
#ifndef RAYTRACERT_DROPIN_HPP_
#define RAYTRACERT_DROPIN_HPP_

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "raytracert.h"

// ---- Vec3D (Vec3D.h): component-wise operators; dot = (a0*b0 + a1*b1) + a2*b2 ----------------
template <typename T>
class Vec3D {
  public:
    T p[3];
    Vec3D() { p[0] = p[1] = p[2] = T(); }
    Vec3D(T x, T y, T z) { p[0] = x; p[1] = y; p[2] = z; }
    Vec3D(const Vec3D &o) { p[0] = o.p[0]; p[1] = o.p[1]; p[2] = o.p[2]; }
    Vec3D(T *q) { p[0] = q[0]; p[1] = q[1]; p[2] = q[2]; }   // implicit, as Vec3D.h:70
    T &operator[](int i) { return p[i]; }
    const T &operator[](int i) const { return p[i]; }
    Vec3D &operator=(const Vec3D &o) { p[0] = o.p[0]; p[1] = o.p[1]; p[2] = o.p[2]; return *this; }
    Vec3D &operator+=(const Vec3D &o) { for (int k = 0; k < 3; ++k) p[k] += o.p[k]; return *this; }
    Vec3D &operator-=(const Vec3D &o) { for (int k = 0; k < 3; ++k) p[k] -= o.p[k]; return *this; }
    Vec3D &operator*=(const Vec3D &o) { for (int k = 0; k < 3; ++k) p[k] *= o.p[k]; return *this; }
    Vec3D &operator*=(T s) { for (int k = 0; k < 3; ++k) p[k] *= s; return *this; }
    Vec3D &operator/=(const Vec3D &o) { for (int k = 0; k < 3; ++k) p[k] /= o.p[k]; return *this; }
    Vec3D &operator/=(T s) { for (int k = 0; k < 3; ++k) p[k] /= s; return *this; }
    Vec3D &init(T x, T y, T z) { p[0] = x; p[1] = y; p[2] = z; return *this; }
    T getSquaredLength() const { return dotProduct(*this, *this); }
    T getLength() const { return static_cast<T>(std::sqrt(getSquaredLength())); }
    // scales by the rounded reciprocal of the length (not a division per component)
    T normalize() {
        const T len = getLength();
        if (len == 0.0f) return 0;
        const T inv = 1.0f / len;
        p[0] *= inv; p[1] *= inv; p[2] *= inv;
        return len;
    }
    void fromTo(const Vec3D &a, const Vec3D &b) { for (int k = 0; k < 3; ++k) p[k] = b.p[k] - a.p[k]; }
    float transProduct(const Vec3D &v) const { return p[0] * v[0] + p[1] * v[1] + p[2] * v[2]; }
    // two vectors orthogonal to this one (Vec3D.h:160-173): u from the smaller components, v = this x u
    void getTwoOrthogonals(Vec3D &u, Vec3D &v) const {
        if (std::fabs(p[0]) < std::fabs(p[1])) {
            if (std::fabs(p[0]) < std::fabs(p[2])) u = Vec3D(0, -p[2], p[1]);
            else u = Vec3D(-p[1], p[0], 0);
        } else {
            if (std::fabs(p[1]) < std::fabs(p[2])) u = Vec3D(p[2], 0, -p[0]);
            else u = Vec3D(-p[1], p[0], 0);
        }
        v = crossProduct(*this, u);
    }
    Vec3D projectOn(const Vec3D &N, const Vec3D &P) const { return *this - N * dotProduct(*this - P, N); }
    // (length, angle with z, angle of the x-y projection with x) and back (Vec3D.h:212-243)
    static Vec3D cartesianToPolar(const Vec3D &v) {
        Vec3D polar;
        polar[0] = v.getLength();
        const T rxy = static_cast<T>(std::sqrt(v[0] * v[0] + v[1] * v[1]));
        if (v[2] > 0.0f) polar[1] = static_cast<T>(std::atan(rxy / v[2]));
        else if (v[2] < 0.0f) polar[1] = static_cast<T>(std::atan(rxy / v[2]) + M_PI);
        else polar[1] = static_cast<T>(M_PI * 0.5f);
        if (v[0] > 0.0f) polar[2] = static_cast<T>(std::atan(v[1] / v[0]));
        else if (v[0] < 0.0f) polar[2] = static_cast<T>(std::atan(v[1] / v[0]) + M_PI);
        else if (v[1] > 0) polar[2] = static_cast<T>(M_PI * 0.5f);
        else polar[2] = static_cast<T>(-M_PI * 0.5);
        return polar;
    }
    static Vec3D polarToCartesian(const Vec3D &v) {
        return Vec3D(v[0] * static_cast<T>(std::sin(v[1])) * static_cast<T>(std::cos(v[2])),
                     v[0] * static_cast<T>(std::sin(v[1])) * static_cast<T>(std::sin(v[2])), v[0] * static_cast<T>(std::cos(v[1])));
    }
    // this point in the frame (pos; u, v, n) (Vec3D.h:249-254)
    Vec3D transformIn(const Vec3D &pos, const Vec3D &n, const Vec3D &u, const Vec3D &v) const {
        const Vec3D q = *this - pos;
        return Vec3D(u[0] * q[0] + u[1] * q[1] + u[2] * q[2], v[0] * q[0] + v[1] * q[1] + v[2] * q[2],
                     n[0] * q[0] + n[1] * q[1] + n[2] * q[2]);
    }
    // "(x, y, z)" into buffer (the 'd' key prints it, raytracing.cpp:508-509). The reference's body is
    // commented out (Vec3D.h:257), so it prints whatever the stack buffer held; this writes the text its
    // comment intends.
    char *toString(char *buffer, size_t size) const {
        if (buffer && size) std::snprintf(buffer, size, "(%f, %f, %f)", static_cast<double>(p[0]), static_cast<double>(p[1]),
                                          static_cast<double>(p[2]));
        return buffer;
    }
    T *pointer() { return p; }
    const T *pointer() const { return p; }
    static Vec3D segment(const Vec3D &a, const Vec3D &b) { return Vec3D(b[0] - a[0], b[1] - a[1], b[2] - a[2]); }
    static Vec3D crossProduct(const Vec3D &a, const Vec3D &b) {
        return Vec3D(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
    }
    static T dotProduct(const Vec3D &a, const Vec3D &b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
    static T squaredDistance(const Vec3D &a, const Vec3D &b) { return (a - b).getSquaredLength(); }
    static T distance(const Vec3D &a, const Vec3D &b) { return (a - b).getLength(); }
    static Vec3D interpolate(const Vec3D &u, const Vec3D &v, T alpha) { return u * (1.0f - alpha) + v * alpha; }
    static Vec3D projectOntoVector(const Vec3D &v1, const Vec3D &v2) { return v2 * dotProduct(v1, v2); }
};

template <class T> const Vec3D<T> operator*(const Vec3D<T> &a, float f) { return Vec3D<T>(a[0] * f, a[1] * f, a[2] * f); }
template <class T> const Vec3D<T> operator*(float f, const Vec3D<T> &a) { return Vec3D<T>(a[0] * f, a[1] * f, a[2] * f); }
template <class T> const Vec3D<T> operator*(const Vec3D<T> &a, const Vec3D<T> &b) {
    return Vec3D<T>(a[0] * b[0], a[1] * b[1], a[2] * b[2]);
}
template <class T> const Vec3D<T> operator+(const Vec3D<T> &a, const Vec3D<T> &b) {
    return Vec3D<T>(a[0] + b[0], a[1] + b[1], a[2] + b[2]);
}
template <class T> const Vec3D<T> operator-(const Vec3D<T> &a, const Vec3D<T> &b) {
    return Vec3D<T>(a[0] - b[0], a[1] - b[1], a[2] - b[2]);
}
template <class T> const Vec3D<T> operator-(const Vec3D<T> &a) { return Vec3D<T>(-a[0], -a[1], -a[2]); }
template <class T> const Vec3D<T> operator/(const Vec3D<T> &a, float d) { return Vec3D<T>(a[0] / d, a[1] / d, a[2] / d); }
template <class T> bool operator==(const Vec3D<T> &a, const Vec3D<T> &b) { return a[0] == b[0] && a[1] == b[1] && a[2] == b[2]; }
template <class T> bool operator!=(const Vec3D<T> &a, const Vec3D<T> &b) { return !(a == b); }
template <class T> bool operator<(const Vec3D<T> &a, const Vec3D<T> &b) { return a[0] < b[0] && a[1] < b[1] && a[2] < b[2]; }
template <class T> bool operator>=(const Vec3D<T> &a, const Vec3D<T> &b) { return a[0] >= b[0] || a[1] >= b[1] || a[2] >= b[2]; }
template <class T> std::ostream &operator<<(std::ostream &o, const Vec3D<T> &v) { return o << v[0] << " " << v[1] << " " << v[2]; }
template <class T> std::istream &operator>>(std::istream &i, Vec3D<T> &v) { return i >> v[0] >> v[1] >> v[2]; }
template <class T> void swap(Vec3D<T> &a, Vec3D<T> &b) { const Vec3D<T> t = a; a = b; b = t; }   // Vec3D.h:275

typedef Vec3D<float> Vec3Df;
typedef Vec3D<double> Vec3Dd;
typedef Vec3D<int> Vec3Di;
static_assert(sizeof(Vec3Df) == sizeof(rt_vec3), "Vec3Df is three packed floats, as rt_vec3");

// ---- Vertex, Triangle, Material, Mesh (Vertex.h, mesh.h) --------------------------------------
class Vertex {
  public:
    Vertex() {}
    Vertex(const Vec3Df &pos) : p(pos) {}
    Vertex(const Vec3Df &pos, const Vec3Df &nrm) : p(pos), n(nrm) {}
    Vec3Df p;   // position
    Vec3Df n;   // vertex normal (Mesh::computeVertexNormals)
};

class Triangle {
  public:
    Triangle() { v[0] = v[1] = v[2] = 0; t[0] = t[1] = t[2] = 0; }
    Triangle(unsigned v0, unsigned t0, unsigned v1, unsigned t1, unsigned v2, unsigned t2) {
        v[0] = v0; v[1] = v1; v[2] = v2;
        t[0] = t0; t[1] = t1; t[2] = t2;
    }
    Triangle(const Triangle &o) = default;
    // mesh.h:150-158 as written: assignment copies the vertex indices into t too (the copy
    // constructor, which loadMesh's push_back uses, copies t)
    Triangle &operator=(const Triangle &o) {
        v[0] = o.v[0]; v[1] = o.v[1]; v[2] = o.v[2];
        t[0] = o.v[0]; t[1] = o.v[1]; t[2] = o.v[2];
        return *this;
    }
    unsigned int v[3];   // vertex indices
    unsigned int t[3];   // texture-coordinate indices (Mesh::texcoords)
};

class Material {
  public:
    Material() { cleanup(); }
    void cleanup() { flags_ = 0; name_ = "empty"; }   // resets the flags only, as mesh.h:43-53
    bool is_valid() const { return has(RT_HAS_KD) || has(RT_HAS_KA) || has(RT_HAS_KS) || has(RT_HAS_TR); }
    bool has_Kd() const { return has(RT_HAS_KD); }
    bool has_Ka() const { return has(RT_HAS_KA); }
    bool has_Ks() const { return has(RT_HAS_KS); }
    bool has_Ns() const { return has(RT_HAS_NS); }
    bool has_Ni() const { return has(RT_HAS_NI); }
    bool has_illum() const { return has(RT_HAS_ILLUM); }
    bool has_Tr() const { return has(RT_HAS_TR); }
    void set_Kd(float r, float g, float b) { Kd_ = Vec3Df(r, g, b); flags_ |= RT_HAS_KD; }
    void set_Ka(float r, float g, float b) { Ka_ = Vec3Df(r, g, b); flags_ |= RT_HAS_KA; }
    void set_Ks(float r, float g, float b) { Ks_ = Vec3Df(r, g, b); flags_ |= RT_HAS_KS; }
    void set_Ns(float r) { Ns_ = r; flags_ |= RT_HAS_NS; }
    void set_Ni(float r) { Ni_ = r; flags_ |= RT_HAS_NI; }
    void set_illum(int r) { illum_ = r; flags_ |= RT_HAS_ILLUM; }
    void set_Tr(float t) { Tr_ = t; flags_ |= RT_HAS_TR; }
    void set_textureName(const std::string &s) { textureName_ = s; }
    void set_name(const std::string &s) { name_ = s; }
    const Vec3Df &Kd() const { return Kd_; }
    const Vec3Df &Ka() const { return Ka_; }
    const Vec3Df &Ks() const { return Ks_; }
    float Ni() const { return Ni_; }
    float Ns() const { return Ns_; }
    int illum() const { return illum_; }
    float Tr() const { return Tr_; }
    const std::string &textureName() const { return textureName_; }
    const std::string &name() const { return name_; }
    // conversions to and from the C-ABI's plain material
    static Material from_rt(const rt_material &m) {
        Material o;
        o.Kd_ = Vec3Df(m.Kd[0], m.Kd[1], m.Kd[2]);
        o.Ka_ = Vec3Df(m.Ka[0], m.Ka[1], m.Ka[2]);
        o.Ks_ = Vec3Df(m.Ks[0], m.Ks[1], m.Ks[2]);
        o.Ns_ = m.Ns; o.Ni_ = m.Ni; o.Tr_ = m.Tr; o.illum_ = m.illum; o.flags_ = m.flags;
        o.name_.clear();
        return o;
    }
    rt_material to_rt() const {
        rt_material m{};
        for (int k = 0; k < 3; ++k) { m.Kd[k] = Kd_[k]; m.Ka[k] = Ka_[k]; m.Ks[k] = Ks_[k]; }
        m.Ns = Ns_; m.Ni = Ni_; m.Tr = Tr_; m.illum = illum_; m.flags = flags_;
        return m;
    }

  private:
    bool has(uint32_t f) const { return (flags_ & f) != 0; }
    // never-set values read 0 (the reference reads uninitialised memory there)
    Vec3Df Kd_, Ka_, Ks_;
    float Ns_ = 0, Ni_ = 0, Tr_ = 0;
    int illum_ = 0;
    uint32_t flags_ = 0;
    std::string name_, textureName_;
};

namespace rtamd_dropin {
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
}  // namespace rtamd_dropin

class Mesh {
  public:
    Mesh() {}
    Mesh(const std::vector<Vertex> &v, const std::vector<Triangle> &t) : vertices(v), triangles(t) {}
    // Mesh::loadMesh (mesh.cpp:95-331, with loadMtl :334-460): through librtamd's loader, which
    // keeps the reference's parse semantics; false when the file cannot be read (the reference
    // crashes there, mesh.cpp:329)
    bool loadMesh(const char *filename, bool /*randomizeTriangulation: disabled in the reference too*/) {
        rt_scene *s = nullptr;
        if (rt_scene_load_obj_ex(filename, RT_HOST_ONLY, RT_LOAD_SEQUENTIAL | RT_LOAD_TEXCOORDS, &s) != RT_OK) return false;
        int32_t nv = 0, nt = 0, nm = 0;
        rt_scene_info(s, &nv, &nt, &nm);
        std::vector<float> xyz(3 * static_cast<size_t>(nv));
        std::vector<uint32_t> tv(3 * static_cast<size_t>(nt));
        std::vector<rt_material> mats(static_cast<size_t>(nm));
        triangleMaterials.assign(static_cast<size_t>(nt), 0u);
        rt_scene_export(s, xyz.data(), tv.data(), triangleMaterials.data(), mats.data(), nullptr);
        int32_t ntc = 0;
        rt_scene_texcoords(s, &ntc, nullptr, nullptr);
        std::vector<float> tc(3 * static_cast<size_t>(ntc));
        std::vector<uint32_t> tt(3 * static_cast<size_t>(nt));
        rt_scene_texcoords(s, &ntc, tc.data(), tt.data());
        rt_scene_destroy(s);
        vertices.assign(static_cast<size_t>(nv), Vertex());
        for (int32_t i = 0; i < nv; ++i) vertices[i].p = Vec3Df(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
        triangles.assign(static_cast<size_t>(nt), Triangle());
        for (int32_t i = 0; i < nt; ++i)
            for (int k = 0; k < 3; ++k) {
                triangles[i].v[k] = tv[3 * i + k];
                triangles[i].t[k] = tt[3 * i + k];
            }
        materials.clear();
        for (const rt_material &m : mats) materials.push_back(Material::from_rt(m));
        texcoords.assign(static_cast<size_t>(ntc), Vec3Df());
        for (int32_t i = 0; i < ntc; ++i) texcoords[i] = Vec3Df(tc[3 * i], tc[3 * i + 1], tc[3 * i + 2]);
        return true;
    }
    // Mesh::loadMtl (mesh.cpp:334-460): appends each block of the file whose name materialIndex does
    // not hold yet and indexes it; false (with the reference's warning) if the file cannot be read
    bool loadMtl(const char *filename, std::map<std::string, unsigned int> &materialIndex) {
        int32_t n = 0;
        if (rt_load_mtl(filename, &n, nullptr, 0, nullptr, 0) != RT_OK) {
            std::printf("  Warning! Material file '%s' not found!\n", filename);
            return false;
        }
        std::vector<rt_material> mats(static_cast<size_t>(n));
        size_t cap = 1;
        for (int32_t i = 0; i < n; ++i) cap += 256;   // (a name is at most one 256-byte line)
        std::vector<char> names(cap);
        if (rt_load_mtl(filename, &n, mats.data(), n, names.data(), names.size()) != RT_OK) return false;
        const char *nm = names.data();
        for (int32_t i = 0; i < n; ++i) {
            const std::string key(nm);
            nm += key.size() + 1;
            if (materialIndex.find(key) != materialIndex.end()) continue;
            Material m = Material::from_rt(mats[static_cast<size_t>(i)]);
            m.set_name(key);
            materials.push_back(m);
            materialIndex[key] = static_cast<unsigned int>(materials.size() - 1);
        }
        return true;
    }
    // Mesh::computeVertexNormals (mesh.cpp:28-47): the sum of the adjacent face normals, normalised
    // (the GL preview's smooth shading; the render path does not read it)
    void computeVertexNormals() {
        for (Vertex &v : vertices) v.n = Vec3Df(0, 0, 0);
        for (const Triangle &t : triangles) {
            Vec3Df n = Vec3Df::crossProduct(vertices[t.v[1]].p - vertices[t.v[0]].p, vertices[t.v[2]].p - vertices[t.v[0]].p);
            n.normalize();
            for (int j = 0; j < 3; ++j) vertices[t.v[j]].n += n;
        }
        for (Vertex &v : vertices) v.n.normalize();
    }
    // the GL preview (mesh.cpp:53-90): flat (face normals) and smooth (vertex normals) shading, the
    // triangle's Kd as colour. Immediate-mode GL when the host includes GL and defines
    // RTAMD_DROPIN_GL; otherwise nothing (the render path never draws).
    void draw() const {
#ifdef RTAMD_DROPIN_GL
        glBegin(GL_TRIANGLES);
        for (size_t i = 0; i < triangles.size(); ++i) {
            glColor3fv(materials.at(triangleMaterials.at(i)).Kd().pointer());
            const Triangle &t = triangles[i];
            Vec3Df n = Vec3Df::crossProduct(vertices[t.v[1]].p - vertices[t.v[0]].p, vertices[t.v[2]].p - vertices[t.v[0]].p);
            n.normalize();
            glNormal3f(n[0], n[1], n[2]);
            for (int v = 0; v < 3; ++v) glVertex3fv(vertices[t.v[v]].p.pointer());
        }
        glEnd();
#endif
    }
    void drawSmooth() const {
#ifdef RTAMD_DROPIN_GL
        glBegin(GL_TRIANGLES);
        for (size_t i = 0; i < triangles.size(); ++i) {
            glColor3fv(materials[triangleMaterials[i]].Kd().pointer());
            for (int v = 0; v < 3; ++v) {
                glNormal3fv(vertices[triangles[i].v[v]].n.pointer());
                glVertex3fv(vertices[triangles[i].v[v]].p.pointer());
            }
        }
        glEnd();
#endif
    }
    std::vector<Vertex> vertices;
    std::vector<Vec3Df> texcoords;
    std::vector<Triangle> triangles;
    std::vector<unsigned int> triangleMaterials;
    std::vector<Material> materials;
};

// ---- globals ------------------------------------------------------------------------------------
// raytracing.h:8-16 — defined by the host (main.cpp:17-18,130,137-141), as with the reference
extern Mesh MyMesh;
extern std::vector<Vec3Df> MyLightPositions;
extern Vec3Df MyCameraPosition;
extern unsigned int WindowSize_X;
extern unsigned int WindowSize_Y;
extern unsigned int RayTracingResolutionX;
extern unsigned int RayTracingResolutionY;
// raytracing.cpp:15-36 — defined here (the reference defines them in raytracing.cpp)
inline bool Ambient = true;
inline bool Diffuse = true;
inline bool Reflection = true;
inline bool Shadows = true;
inline bool Specular = true;
inline bool Refraction = true;
inline bool WireFrame = false;
inline unsigned int pixelfactorX = 3;
inline unsigned int pixelfactorY = 3;
inline int max_lvl = 10;
inline std::vector<Vec3Df> normals;   // per-triangle normals (calculateNormals)
// the GPU init() binds (a HIP device index), or RT_HOST_ONLY: loader and getMaterial only
inline int RayTracerDevice = 0;

// raytracing.h:24 — "defined elsewhere" (main.cpp:322-325, over gluUnProject). Weak here: the 'r'
// loop's frame cache and the 'd' key call it when the host defines it, and a host that never
// does still links.
void produceRay(int x_I, int y_I, Vec3Df &origin, Vec3Df &dest) __attribute__((weak));

namespace rtamd_dropin {
inline rt_scene *&scene() {
    static rt_scene *s = nullptr;
    return s;
}
inline uint64_t &scene_generation() {   // bumped by every uploadMesh()
    static uint64_t g = 0;
    return g;
}
// the ray debugger's state (raytracing.cpp:35-37: `o`, `d`, DebugMode; kept out of the global
// namespace, where one-letter globals would collide with a host's names)
inline bool DebugMode = false;
inline std::vector<Vec3Df> debug_origins, debug_hits;
inline rt_scene *need_scene() {
    if (!scene()) throw Error(RT_E_ARG, "no GPU scene: call init() (with RayTracerDevice a device index) first");
    return scene();
}
// Everything the reference reads from globals during a trace.
inline rt_params params(int levels_left) {
    rt_params p{};
    p.width = static_cast<int32_t>(WindowSize_X);
    p.height = static_cast<int32_t>(WindowSize_Y);
    p.pfx = static_cast<int32_t>(pixelfactorX);
    p.pfy = static_cast<int32_t>(pixelfactorY);
    p.max_lvl = levels_left;
    p.flags = (Ambient ? RT_AMBIENT : 0u) | (Diffuse ? RT_DIFFUSE : 0u) | (Specular ? RT_SPECULAR : 0u) |
              (Reflection ? RT_REFLECTION : 0u) | (Shadows ? RT_SHADOWS : 0u) | (Refraction ? RT_REFRACTION : 0u);
    // any number of lights, as the reference's unbounded list ('L' appends one, main.cpp:334-336): the
    // first RT_MAX_LIGHTS inline, the whole list through light_list (Vec3Df is three packed floats; read
    // during the call that takes these params)
    p.n_lights = static_cast<int32_t>(MyLightPositions.size());
    for (size_t i = 0; i < MyLightPositions.size() && i < RT_MAX_LIGHTS; ++i)
        for (int k = 0; k < 3; ++k) p.lights[i][k] = MyLightPositions[i][k];
    if (MyLightPositions.size() > RT_MAX_LIGHTS) p.light_list = MyLightPositions[0].p;
    for (int k = 0; k < 3; ++k) p.camera_pos[k] = MyCameraPosition[k];
    p.seed = RT_DEFAULT_SEED;
    return p;
}
}  // namespace rtamd_dropin

// (Re)build the GPU scene from MyMesh: call after editing MyMesh by hand. init() calls it.
inline void uploadMesh() {
    rt_scene_destroy(rtamd_dropin::scene());
    rtamd_dropin::scene() = nullptr;
    ++rtamd_dropin::scene_generation();
    if (RayTracerDevice == RT_HOST_ONLY) return;
    std::vector<float> xyz;
    xyz.reserve(3 * MyMesh.vertices.size());
    for (const Vertex &v : MyMesh.vertices) { xyz.push_back(v.p[0]); xyz.push_back(v.p[1]); xyz.push_back(v.p[2]); }
    std::vector<uint32_t> tv;
    tv.reserve(3 * MyMesh.triangles.size());
    for (const Triangle &t : MyMesh.triangles) { tv.push_back(t.v[0]); tv.push_back(t.v[1]); tv.push_back(t.v[2]); }
    std::vector<rt_material> mats;
    for (const Material &m : MyMesh.materials) mats.push_back(m.to_rt());
    rtamd_dropin::check(rt_scene_create(xyz.data(), static_cast<int32_t>(MyMesh.vertices.size()), tv.data(),
                                        MyMesh.triangleMaterials.data(), static_cast<int32_t>(MyMesh.triangles.size()),
                                        mats.data(), static_cast<int32_t>(mats.size()), RayTracerDevice,
                                        &rtamd_dropin::scene()));
}

// calculateNormals (raytracing.cpp:78-86): one normal per triangle into `normals` (appended, as
// the reference's push_back); on a GPU scene these are the device-computed normals it renders with
inline void calculateNormals() {
    const size_t nt = MyMesh.triangles.size();
    std::vector<float> n(3 * nt);
    rt_scene *s = rtamd_dropin::scene();
    bool own = false;
    if (!s) {   // host only: the loader's normals of MyMesh
        std::vector<float> xyz;
        for (const Vertex &v : MyMesh.vertices) { xyz.push_back(v.p[0]); xyz.push_back(v.p[1]); xyz.push_back(v.p[2]); }
        std::vector<uint32_t> tv;
        for (const Triangle &t : MyMesh.triangles) { tv.push_back(t.v[0]); tv.push_back(t.v[1]); tv.push_back(t.v[2]); }
        std::vector<rt_material> mats(1);
        mats[0].flags = RT_HAS_KD;
        std::vector<uint32_t> tm(nt, 0u);
        rtamd_dropin::check(rt_scene_create(xyz.data(), static_cast<int32_t>(MyMesh.vertices.size()), tv.data(), tm.data(),
                                            static_cast<int32_t>(nt), mats.data(), 1, RT_HOST_ONLY, &s));
        own = true;
    }
    const int rc = rt_scene_export(s, nullptr, nullptr, nullptr, nullptr, n.data());
    if (own) rt_scene_destroy(s);
    rtamd_dropin::check(rc);
    for (size_t i = 0; i < nt; ++i) normals.push_back(Vec3Df(n[3 * i], n[3 * i + 1], n[3 * i + 2]));
}

namespace rtamd_dropin {
// Pinned records for one 'r' frame's sub-samples (FrameCache::rec), grown when the frame grows.
inline void ensure_records(float *&rec, size_t &cap, size_t floats) {
    if (floats <= cap) return;
    rt_host_free(rec);
    rec = nullptr;
    cap = 0;
    void *m = nullptr;
    check(rt_host_alloc(floats * sizeof(float), &m));
    rec = static_cast<float *>(m);
    cap = floats;
}
inline void reserve_frame();
}  // namespace rtamd_dropin

// init(char*), raytracing.cpp:42-73
inline void init(char *fileName) {
    const char *path = fileName ? fileName : "cube.obj";
    if (!MyMesh.loadMesh(path, true)) throw rtamd_dropin::Error(RT_E_IO, std::string("cannot load '") + path + "'");
    MyMesh.computeVertexNormals();
    uploadMesh();
    calculateNormals();
    MyLightPositions.push_back(MyCameraPosition);   // light 0 = the camera position (:72)
    rtamd_dropin::reserve_frame();
}

// isNullVector (raytracing.cpp:92-94)
inline bool isNullVector(Vec3Df v) { return v[0] == 0 && v[1] == 0 && v[2] == 0; }

// rayIntersectTriangle (raytracing.cpp:99-154), on the GPU bound by RayTracerDevice
inline bool rayIntersectTriangle(Vec3Df R[], Vec3Df T[], Vec3Df *intersectOut) {
    float r[6] = {R[0][0], R[0][1], R[0][2], R[1][0], R[1][1], R[1][2]};
    float t[9];
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) t[3 * i + k] = T[i][k];
    uint8_t hit = 0;
    float I[3];
    rtamd_dropin::check(rt_ray_intersect_triangle(RayTracerDevice, r, t, 1, &hit, I));
    if (hit && intersectOut) *intersectOut = Vec3Df(I[0], I[1], I[2]);
    return hit != 0;
}

// intersectMesh (raytracing.cpp:161-192): closest triangle or -1; the point, or (0,0,0)
inline int intersectMesh(Vec3Df origin, Vec3Df dest, Vec3Df *intersectOut) {
    int32_t idx = -1;
    float I[3] = {0, 0, 0};
    rtamd_dropin::check(rt_intersect_mesh(rtamd_dropin::need_scene(), origin.p, dest.p, 1, &idx, I));
    if (intersectOut) *intersectOut = Vec3Df(I[0], I[1], I[2]);
    return idx;
}

// getMaterial (raytracing.cpp:373-376)
inline Material getMaterial(int index) { return MyMesh.materials[MyMesh.triangleMaterials[index]]; }

// trace (raytracing.cpp:381-406): every level test is `lvl < max_lvl` with unit steps, so trace
// at lvl is the chain with max_lvl - lvl levels left
inline Vec3Df trace(const Vec3Df &origin, const Vec3Df &dest, int lvl) {
    const rt_params p = rtamd_dropin::params(lvl >= max_lvl ? 0 : max_lvl - lvl);
    Vec3Df c;
    rtamd_dropin::check(rt_trace_rays(rtamd_dropin::need_scene(), &p, origin.p, dest.p, 1, c.p, nullptr));
    return c;
}

namespace rtamd_dropin {
// Everything a trace reads besides the ray: the globals of raytracing.cpp/main.cpp and the scene.
struct TraceState {
    rt_scene *scene = nullptr;
    uint64_t gen = 0;
    bool amb = false, dif = false, refl = false, sha = false, spec = false, refr = false;
    unsigned pfx = 0, pfy = 0, w = 0, h = 0;
    int lvl = 0;
    std::vector<Vec3Df> lights;
    Vec3Df cam;
    static TraceState now() {
        TraceState t;
        t.scene = rtamd_dropin::scene(); t.gen = scene_generation();
        t.amb = Ambient; t.dif = Diffuse; t.refl = Reflection; t.sha = Shadows; t.spec = Specular; t.refr = Refraction;
        t.pfx = pixelfactorX; t.pfy = pixelfactorY; t.w = WindowSize_X; t.h = WindowSize_Y;
        t.lvl = max_lvl; t.lights = MyLightPositions; t.cam = MyCameraPosition;
        return t;
    }
    bool operator==(const TraceState &o) const {   // (bitwise on the floats)
        if (scene != o.scene || gen != o.gen || amb != o.amb || dif != o.dif || refl != o.refl || sha != o.sha ||
            spec != o.spec || refr != o.refr || pfx != o.pfx || pfy != o.pfy || w != o.w || h != o.h || lvl != o.lvl ||
            lights.size() != o.lights.size() || std::memcmp(cam.p, o.cam.p, sizeof cam.p) != 0)
            return false;
        return lights.empty() || std::memcmp(lights.data(), o.lights.data(), sizeof(Vec3Df) * lights.size()) == 0;
    }
    // The same test against the live globals, without copying them: every comparison folded into one
    // word (no branch per global: this runs once per performRayTracing call of the 'r' loop).
    bool matches_globals() const {
        uint32_t x = static_cast<uint32_t>(scene != rtamd_dropin::scene()) | static_cast<uint32_t>(gen != scene_generation()) |
                     static_cast<uint32_t>(amb != Ambient) | static_cast<uint32_t>(dif != Diffuse) |
                     static_cast<uint32_t>(refl != Reflection) | static_cast<uint32_t>(sha != Shadows) |
                     static_cast<uint32_t>(spec != Specular) | static_cast<uint32_t>(refr != Refraction) |
                     (pfx ^ pixelfactorX) | (pfy ^ pixelfactorY) | (w ^ WindowSize_X) | (h ^ WindowSize_Y) |
                     static_cast<uint32_t>(lvl ^ max_lvl) | diff3(cam.p, MyCameraPosition.p);
        const Vec3Df *a = lights.data(), *b = MyLightPositions.data();
        const size_t nl = lights.size();
        if (x != 0 || nl != MyLightPositions.size()) return false;
        for (size_t i = 0; i < nl; ++i) x |= diff3(a[i].p, b[i].p);
        return x == 0;
    }
    // the bits of one float, loaded as a 32-bit word (no copy through a stack array: an 8-byte load
    // of two floats just stored one by one misses store forwarding, ~15 cycles a time on x86)
    static uint32_t bits(const float *f) {
        uint32_t u;
        std::memcpy(&u, f, 4);
        return u;
    }
    static uint32_t diff3(const float *a, const float *b) {   // 0 when the three floats are the same bits
        return (bits(a) ^ bits(b)) | (bits(a + 1) ^ bits(b + 1)) | (bits(a + 2) ^ bits(b + 2));
    }
    static bool same_bits3(const float *a, const float *b) { return diff3(a, b) == 0; }
};

inline bool same_bits(const Vec3Df &a, const Vec3Df &b) { return std::memcmp(a.p, b.p, sizeof a.p) == 0; }

// The 'r' loop's sub-sample ray (main.cpp:380-386), with the loop's own expressions and types.
inline void loop_ray(unsigned x, unsigned y, int subx, int suby, float divX, float divY, const Vec3Df *c, Vec3Df &origin,
                     Vec3Df &dest) {
    float xscale = 1.0f - (float(x) * pixelfactorX + subx) / divX;
    float yscale = 1.0f - (float(y) * pixelfactorY + suby) / divY;
    origin = yscale * (xscale * c[0] + (1 - xscale) * c[4]) + (1 - yscale) * (xscale * c[2] + (1 - xscale) * c[6]);
    dest = yscale * (xscale * c[1] + (1 - xscale) * c[5]) + (1 - yscale) * (xscale * c[3] + (1 - xscale) * c[7]);
}

// One 'r' frame's sub-samples, traced on the device in one call (rt_trace_frame_samples with
// RT_SAMPLES_RAY_RGB): per call of the loop, in its order, the ray the device made for it with the
// loop's own expressions and that ray's colour. Call `next` is answered from record `next` when its
// (origin, dest) equals the record's ray bit for bit: the colour is then exactly trace() of the
// call's own ray, whatever compiler flags the host loop was built with (a host whose floats differ
// just misses and takes the per-call path).
struct FrameCache {
    TraceState state;
    size_t n = 0, next = 0;   // records in the frame; the next call's record
    float *rec = nullptr;     // 9 floats per sub-sample: origin, dest, rgb (pinned host memory)
    size_t rec_cap = 0;
    size_t host_ray_frames = 0;   // frames whose records hold host-made rays (the host rounds differently)
    size_t device_frames = 0;     // frame traces made on the device (rt_trace_frame_samples)
    bool host_rays = false;       // this frame's records are host-made
    Vec3Df c[8];                  // this frame's corner rays (produceRay) and divisors
    float divX = 0, divY = 0;
    ~FrameCache() { rt_host_free(rec); }
    bool matches(const Vec3Df &o, const Vec3Df &d) const {   // the call's ray is record `next`'s, bit for bit
        const float *r = rec + 9 * next;
        return (TraceState::diff3(o.p, r) | TraceState::diff3(d.p, r + 3)) == 0;
    }
    Vec3Df take() {
        const float *c = rec + 9 * next++ + 6;
        return Vec3Df(c[0], c[1], c[2]);
    }
};
inline FrameCache &frame_cache() {
    static FrameCache c;
    return c;
}

// If (origin, dest) is the first sub-sample of the 'r' loop for the current corner rays (produceRay),
// trace every sub-sample of that frame in one GPU call into the cache and return true.
// The host's loop rounds differently from the device (e.g. built with FMA contraction: GCC's default
// -ffp-contract=fast on an FMA target): make every sub-sample's ray of the cached frame with loop_ray,
// compiled into this translation unit with the host's own flags like its loop, and trace exactly those
// in one call (records from `next` on are then the loop's own rays and their colours).
// Records `from` .. n - 1 only: the records before `from` were answered already (resume_frame).
inline void trace_host_rays(FrameCache &fc, size_t from = 0) {
    const size_t n = fc.n, m = n > from ? n - from : 0;
    const size_t spp = static_cast<size_t>(pixelfactorX) * pixelfactorY;
    std::vector<float> o(3 * m), d(3 * m), rgb(3 * m);
    for (size_t k = 0; k < m; ++k) {   // record from + k: pixel (from + k) / spp, sub-sample (subx, suby) in loop order
        const size_t s = from + k, pix = s / spp, sub = s % spp;
        Vec3Df ro, rd;
        loop_ray(static_cast<unsigned>(pix % WindowSize_X), static_cast<unsigned>(pix / WindowSize_X),
                 static_cast<int>(sub / pixelfactorY), static_cast<int>(sub % pixelfactorY), fc.divX, fc.divY, fc.c, ro, rd);
        std::memcpy(&o[3 * k], ro.p, 12);
        std::memcpy(&d[3 * k], rd.p, 12);
    }
    if (m > 0) {
        const rt_params p = params(max_lvl);
        check(rt_trace_rays(scene(), &p, o.data(), d.data(), static_cast<int32_t>(m), rgb.data(), nullptr));
    }
    for (size_t k = 0; k < m; ++k) {
        float *r = fc.rec + 9 * (from + k);
        std::memcpy(r, &o[3 * k], 12);
        std::memcpy(r + 3, &d[3 * k], 12);
        std::memcpy(r + 6, &rgb[3 * k], 12);
    }
    fc.host_rays = true;
    ++fc.host_ray_frames;
}

inline bool start_frame(const Vec3Df &origin, const Vec3Df &dest) {
    if (!produceRay || WindowSize_X == 0 || WindowSize_Y == 0 || pixelfactorX == 0 || pixelfactorY == 0 || !scene())
        return false;
    Vec3Df c[8];   // origin00, dest00, origin01, dest01, origin10, dest10, origin11, dest11 (main.cpp:355-358)
    produceRay(0, 0, c[0], c[1]);
    produceRay(0, WindowSize_Y - 1, c[2], c[3]);
    produceRay(WindowSize_X - 1, 0, c[4], c[5]);
    produceRay(WindowSize_X - 1, WindowSize_Y - 1, c[6], c[7]);
    float divX = (WindowSize_X * pixelfactorX - 1);
    float divY = (WindowSize_Y * pixelfactorY - 1);
    Vec3Df o0, d0;
    loop_ray(0, 0, 0, 0, divX, divY, c, o0, d0);
    if (!same_bits(o0, origin) || !same_bits(dest, d0)) return false;
    FrameCache &fc = frame_cache();
    const size_t n = static_cast<size_t>(WindowSize_X) * WindowSize_Y * pixelfactorX * pixelfactorY;
    // The previous frame needed the host's own rays (the host rounds its loop differently from the
    // device) and nothing it depends on has changed since: this frame's rays are the host's too, so the
    // device's frame trace would be thrown away: trace the host's rays directly.
    bool same_view = fc.host_rays && fc.n == n && same_bits(Vec3Df(divX, divY, 0), Vec3Df(fc.divX, fc.divY, 0)) &&
                     fc.state.matches_globals();
    for (int i = 0; i < 8 && same_view; ++i) same_view = same_bits(c[i], fc.c[i]);
    fc.n = fc.next = 0;
    ensure_records(fc.rec, fc.rec_cap, 9 * n);
    if (same_view) {
        fc.n = n;
        trace_host_rays(fc);
        return fc.matches(origin, dest);
    }
    rt_params p = params(max_lvl);
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 3; ++k) p.corners[i][k] = c[i][k];
    check(rt_trace_frame_samples(scene(), &p, RT_SAMPLES_RAY_RGB, fc.rec, fc.rec_cap, nullptr));
    ++fc.device_frames;
    fc.state = TraceState::now();
    fc.n = n;
    fc.host_rays = false;
    for (int i = 0; i < 8; ++i) fc.c[i] = c[i];
    fc.divX = divX;
    fc.divY = divY;
    if (fc.matches(origin, dest)) return true;   // the device's first ray is the loop's
    trace_host_rays(fc);
    return fc.matches(origin, dest);
}

// A call the cached frame did not answer, in the middle of a frame: if its ray is the host's own loop
// ray for record `next` (the host rounds differently from the device from some sub-sample on), the
// frame's records are remade from host rays once, and the call and the rest of the loop hit them.
inline bool resume_frame(const Vec3Df &origin, const Vec3Df &dest) {
    FrameCache &fc = frame_cache();
    if (fc.host_rays || fc.next == 0 || fc.next >= fc.n || !fc.state.matches_globals()) return false;
    const size_t spp = static_cast<size_t>(pixelfactorX) * pixelfactorY, pix = fc.next / spp, sub = fc.next % spp;
    Vec3Df o, d;
    loop_ray(static_cast<unsigned>(pix % WindowSize_X), static_cast<unsigned>(pix / WindowSize_X),
             static_cast<int>(sub / pixelfactorY), static_cast<int>(sub % pixelfactorY), fc.divX, fc.divY, fc.c, o, d);
    if (!same_bits(o, origin) || !same_bits(d, dest)) return false;
    trace_host_rays(fc, fc.next);   // (the records before `next` were answered already)
    return fc.matches(origin, dest);
}

// The buffers of the first 'r' frame, made in init() (the reference's init loads the mesh; its first
// 'r' press then pays only the trace): the render workspace and sample staging of a frame of the
// current window and pixel factors (rt_scene_reserve) and the pinned records of its sub-samples.
inline void reserve_frame() {
    if (!scene() || WindowSize_X == 0 || WindowSize_Y == 0 || pixelfactorX == 0 || pixelfactorY == 0) return;
    const rt_params p = params(max_lvl);
    check(rt_scene_reserve(scene(), &p, 16, 16, RT_SAMPLES_RAY_RGB));
    FrameCache &fc = frame_cache();
    ensure_records(fc.rec, fc.rec_cap, 9 * static_cast<size_t>(WindowSize_X) * WindowSize_Y * pixelfactorX * pixelfactorY);
}
}  // namespace rtamd_dropin

// performRayTracing (raytracing.cpp:410-416). The sub-samples of an 'r' loop come from the frame
// cache (see the top of this file); any other ray is traced on its own. Same colours either way.
namespace rtamd_dropin {
// performRayTracing's path for a call the frame cache does not answer (out of line: the cached
// path below stays small enough to inline into the host's loop)
__attribute__((noinline)) inline Vec3Df perform_uncached(const Vec3Df &origin, const Vec3Df &dest) {
#ifndef RTAMD_DROPIN_NO_FRAME_CACHE
    if (start_frame(origin, dest) || resume_frame(origin, dest)) return frame_cache().take();
#endif
    return trace(origin, dest, 0);
}
}  // namespace rtamd_dropin

inline Vec3Df performRayTracing(const Vec3Df &origin, const Vec3Df &dest) {
#ifndef RTAMD_DROPIN_NO_FRAME_CACHE
    rtamd_dropin::FrameCache &fc = rtamd_dropin::frame_cache();
    if (__builtin_expect(fc.next < fc.n && fc.matches(origin, dest) && fc.state.matches_globals(), 1)) return fc.take();
#endif
    return rtamd_dropin::perform_uncached(origin, dest);
}

// the same for many rays in one GPU call
inline std::vector<Vec3Df> performRayTracing(const std::vector<Vec3Df> &origins, const std::vector<Vec3Df> &dests) {
    if (origins.size() != dests.size()) throw rtamd_dropin::Error(RT_E_ARG, "origins/dests size mismatch");
    std::vector<Vec3Df> out(origins.size());
    if (origins.empty()) return out;
    const rt_params p = rtamd_dropin::params(max_lvl);
    rtamd_dropin::check(rt_trace_rays(rtamd_dropin::need_scene(), &p, origins[0].p, dests[0].p,
                                      static_cast<int32_t>(origins.size()), out[0].p, nullptr));
    return out;
}

// The 'r' key's loop (main.cpp:355-395) in one call: for the four corner rays produceRay gives,
// the clamped RGB floats of every pixel, row-major from the top row, i.e. Image::_image after
// the loop's setPixel(x, y, RGBValue(rgb)) calls. rays (may be NULL): queries per kind.
inline std::vector<float> renderImage(const Vec3Df &origin00, const Vec3Df &dest00, const Vec3Df &origin01,
                                      const Vec3Df &dest01, const Vec3Df &origin10, const Vec3Df &dest10,
                                      const Vec3Df &origin11, const Vec3Df &dest11, uint64_t rays[3] = nullptr) {
    rt_params p = rtamd_dropin::params(max_lvl);
    const Vec3Df *c[8] = {&origin00, &dest00, &origin01, &dest01, &origin10, &dest10, &origin11, &dest11};
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 3; ++k) p.corners[i][k] = (*c[i])[k];
    std::vector<float> img(3u * WindowSize_X * WindowSize_Y);
    rtamd_dropin::check(rt_render_tile(rtamd_dropin::need_scene(), &p, 0, 0, p.width, p.height, nullptr, img.data(), rays));
    return img;
}

// yourDebugDraw (raytracing.cpp:434-451): the debug rays (origin red -> hit green) and light 0 as
// a point, with GL when the host defines RTAMD_DROPIN_GL; otherwise nothing (no effect on the image).
inline void yourDebugDraw() {
#ifdef RTAMD_DROPIN_GL
    glPushAttrib(GL_ALL_ATTRIB_BITS);
    glDisable(GL_LIGHTING);
    glBegin(GL_LINES);
    for (size_t i = 0; i < rtamd_dropin::debug_origins.size(); ++i) {
        glColor3f(1, 0, 0);
        glVertex3fv(rtamd_dropin::debug_origins[i].pointer());
        glColor3f(0, 1, 0);
        glVertex3fv(rtamd_dropin::debug_hits[i].pointer());
    }
    glEnd();
    glPointSize(10);
    glBegin(GL_POINTS);
    if (!MyLightPositions.empty()) glVertex3fv(MyLightPositions[0].pointer());
    glEnd();
    glPopAttrib();
#endif
}

// yourKeyboardFunc (raytracing.cpp:453-553): '1'-'6' toggle Ambient, Diffuse, Specular, Reflection,
// Shadows, Refraction; '+'/'-' step both pixel factors (clamped at 1); '0' toggles the ray debugger;
// 'd' (debugger on) shoots the ray through the mouse position (produceRay), records (origin, first
// hit) and, as trace() does in DebugMode, (origin, hit) of every trace() call of the chain that hit,
// and prints the ray's colour, through rt_debug_trace (the per-bounce records of trace()). (trace()'s
// DebugMode records of 'r' frames, every ray of the frame, are not kept: they only feed the debug draw.)
// 'c' clears the recorded rays; 'w' toggles wire frame. Then the settings, as the reference prints them.
inline void yourKeyboardFunc(char key, int x, int y) {
    using rtamd_dropin::DebugMode;
    switch (key) {
        case '1': Ambient = !Ambient; break;
        case '2': Diffuse = !Diffuse; break;
        case '3': Specular = !Specular; break;
        case '4': Reflection = !Reflection; break;
        case '5': Shadows = !Shadows; break;
        case '6': Refraction = !Refraction; break;
        case '+':
            pixelfactorX++;
            pixelfactorY++;
            break;
        case '-':
            pixelfactorX--;
            pixelfactorY--;
            if (pixelfactorX < 1) pixelfactorX = 1;
            if (pixelfactorY < 1) pixelfactorY = 1;
            break;
        case '0':
            DebugMode = !DebugMode;
            std::cout << "Debug Mode:\n 0 to enable / disable debug mode\n d to shoot & draw a ray trace.\n c to clear ray trace history.\n";
            break;
        case 'd':
            if (DebugMode && produceRay) {
                Vec3Df origin, dest;
                produceRay(x, y, origin, dest);
                const rt_params p = rtamd_dropin::params(max_lvl);
                // every trace() call of the chain, in call order (at most two per level: reflection, refraction)
                std::vector<rt_debug_bounce> b(static_cast<size_t>(max_lvl > 0 ? max_lvl : 0) * 2 + 2);
                int32_t nb = 0;
                Vec3Df color;
                rtamd_dropin::check(rt_debug_trace(rtamd_dropin::need_scene(), &p, origin.p, dest.p, b.data(),
                                                   static_cast<int32_t>(b.size()), &nb, color.p));
                if (static_cast<size_t>(nb) > b.size()) {   // (a deeper chain than the estimate: fetch it whole)
                    b.resize(static_cast<size_t>(nb));
                    rtamd_dropin::check(rt_debug_trace(rtamd_dropin::need_scene(), &p, origin.p, dest.p, b.data(), nb, &nb,
                                                       color.p));
                }
                // intersectMesh's point (raytracing.cpp:498-502): the first bounce's hit, (0,0,0) on a miss;
                // then, as trace() does in DebugMode (:398-401), (origin, hit) of every call that hit
                rtamd_dropin::debug_origins.push_back(origin);
                rtamd_dropin::debug_hits.push_back(nb > 0 && b[0].triangle >= 0 ? Vec3Df(b[0].hit[0], b[0].hit[1], b[0].hit[2])
                                                                               : Vec3Df(0, 0, 0));
                for (int32_t i = 0; i < nb; ++i) {
                    if (b[i].triangle < 0) continue;
                    rtamd_dropin::debug_origins.push_back(Vec3Df(b[i].origin[0], b[i].origin[1], b[i].origin[2]));
                    rtamd_dropin::debug_hits.push_back(Vec3Df(b[i].hit[0], b[i].hit[1], b[i].hit[2]));
                }
                char buffer[128];
                std::cout << "Ray trace color = " << color.toString(buffer, sizeof(buffer)) << std::endl;
            }
            return;
        case 'c':
            rtamd_dropin::debug_origins.clear();
            rtamd_dropin::debug_hits.clear();
            std::cout << "Ray trace history cleared\n";
            return;
        case 'w':
            WireFrame = !WireFrame;
#ifdef RTAMD_DROPIN_GL
            glPolygonMode(GL_FRONT_AND_BACK, WireFrame ? GL_LINE : GL_FILL);
#endif
            std::cout << (WireFrame ? "WireFrame enabled\n" : "WireFrame disabled\n");
            break;
        default: break;
    }
    std::cout << std::endl << "------SETTINGS------" << std::endl
              << "Ammbient " << (Ambient ? "ON" : "OFF") << std::endl
              << "Diffuse " << (Diffuse ? "ON" : "OFF") << std::endl
              << "Specular " << (Specular ? "ON" : "OFF") << std::endl
              << "Reflection " << (Reflection ? "ON" : "OFF") << std::endl
              << "Shadow " << (Shadows ? "ON" : "OFF") << std::endl
              << "Refraction " << (Refraction ? "ON" : "OFF") << std::endl
              << "pixelfactorX = " << pixelfactorX << std::endl
              << "pixelfactorY = " << pixelfactorY << std::endl
              << "DebugMode " << (DebugMode ? "ON" : "OFF") << std::endl
              << "WireFrame " << (WireFrame ? "ON" : "OFF") << std::endl
              << "--------------------" << std::endl;
    std::cout << " pressed! The mouse was in location " << x << "," << y << "!" << std::endl;
}

#endif  // RAYTRACERT_DROPIN_HPP_
