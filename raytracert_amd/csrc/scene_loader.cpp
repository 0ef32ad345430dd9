// scene_loader.cpp — OBJ/MTL loading with the semantics of the reference's Mesh::loadMesh and
// Mesh::loadMtl (CG_Project/mesh.cpp:95-460), face normals as calculateNormals
// (raytracing.cpp:78-86), and the device record builders.
//
// Semantics kept on purpose (they decide triangle order, material indices and colours):
//  * lines are read in 256-byte fgets chunks (LINE_LEN, mesh.cpp:22): longer lines split;
//  * OBJ lines starting with '#' or whitespace are skipped (mesh.cpp:154);
//  * `v` uses sscanf "%f %f %f" into x,y,z that persist across lines (mesh.cpp:121,195);
//  * `f` tokenises on '/', ' ', '\r', '\n' (mesh.cpp:218-288), n-gons become the fan
//    (0,i+1,i+2) (mesh.cpp:293-316); faces with <3 vertices are dropped;
//  * `mtllib` appends to the OBJ's directory prefix in place (mesh.cpp:157-178);
//  * MTL: a material is committed on a blank/whitespace-led line or at EOF when one of
//    Kd/Ka/Ks/Tr is set and the name is new (mesh.cpp:363-377,445-453); cleanup() clears only the
//    is-set flags, so unset values are inherited from the previous block (mesh.h:43-53);
//    `d` and `Tr` both set Tr without inversion (mesh.cpp:434-443).
// Reference UB given a defined meaning (identically in oracle/rt_oracle.c): never-set
// Ns/Ni/Tr/illum read 0; unknown or missing usemtl -> default material 0; faces referencing
// non-existent vertices are dropped.
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "rt_internal.h"

namespace rt {

struct MtlIndex {
    std::unordered_map<std::string, int> by_name;   // std::map<string,uint> materialIndex
    int find(const std::string &k) const {
        auto it = by_name.find(k);
        return it == by_name.end() ? -1 : it->second;
    }
};

namespace {

constexpr int kLineLen = 256;   // mesh.cpp:22

constexpr uint32_t kValidMask = RT_HAS_KD | RT_HAS_KA | RT_HAS_KS | RT_HAS_TR;  // is_valid(), mesh.h:55-56


// Mesh::loadMtl, mesh.cpp:334-460: every block it would commit, in order (the name filter is the caller's)
bool parse_mtl_file(const std::string &filename, std::vector<HostMaterial> &blocks) {
    FILE *in = std::fopen(filename.c_str(), "r");
    if (!in) return false;
    char line[kLineLen];
    std::string key;
    HostMaterial mat;            // zeroed: never-set values read 0
    float f1 = 0, f2 = 0, f3 = 0;
    bool indef = false;
    auto commit = [&]() {
        HostMaterial m = mat;
        m.name = key;
        blocks.push_back(m);
    };
    std::memset(line, 0, kLineLen);
    while (!std::feof(in)) {
        if (!std::fgets(line, kLineLen, in)) { /* line stays zeroed */ }
        if (line[0] == '#') { std::memset(line, 0, kLineLen); continue; }
        if (std::isspace(static_cast<unsigned char>(line[0])) || line[0] == '\0') {
            if (indef && !key.empty() && (mat.flags & kValidMask)) {
                commit();
                mat.flags = 0;   // cleanup()
            }
            if (line[0] == '\0') break;
        } else if (std::strncmp(line, "newmtl ", 7) == 0) {
            char *p0 = line + 6;
            while (std::isspace(static_cast<unsigned char>(*++p0))) {}
            char *p1 = p0;
            while (*p1 && !std::isspace(static_cast<unsigned char>(*p1))) ++p1;
            key.assign(p0, p1);
            indef = true;
        } else if (std::strncmp(line, "Kd ", 3) == 0) {
            std::sscanf(line, "Kd %f %f %f", &f1, &f2, &f3);
            mat.Kd[0] = f1; mat.Kd[1] = f2; mat.Kd[2] = f3; mat.flags |= RT_HAS_KD;
        } else if (std::strncmp(line, "Ka ", 3) == 0) {
            std::sscanf(line, "Ka %f %f %f", &f1, &f2, &f3);
            mat.Ka[0] = f1; mat.Ka[1] = f2; mat.Ka[2] = f3; mat.flags |= RT_HAS_KA;
        } else if (std::strncmp(line, "Ks ", 3) == 0) {
            std::sscanf(line, "Ks %f %f %f", &f1, &f2, &f3);
            mat.Ks[0] = f1; mat.Ks[1] = f2; mat.Ks[2] = f3; mat.flags |= RT_HAS_KS;
        } else if (std::strncmp(line, "Ns ", 3) == 0) {
            std::sscanf(line, "Ns %f", &f1); mat.Ns = f1; mat.flags |= RT_HAS_NS;
        } else if (std::strncmp(line, "Ni ", 3) == 0) {
            std::sscanf(line, "Ni %f", &f1); mat.Ni = f1; mat.flags |= RT_HAS_NI;
        } else if (std::strncmp(line, "illum ", 6) == 0) {
            int illum = -1;
            std::sscanf(line, "illum %i", &illum); mat.illum = illum; mat.flags |= RT_HAS_ILLUM;
        } else if (std::strncmp(line, "map_Kd ", 7) == 0) {
            // texture name: stored by the reference, never used by the tracer
        } else if (std::strncmp(line, "Tr ", 3) == 0) {
            std::sscanf(line, "Tr %f", &f1); mat.Tr = f1; mat.flags |= RT_HAS_TR;
        } else if (std::strncmp(line, "d ", 2) == 0) {
            std::sscanf(line, "d %f", &f1); mat.Tr = f1; mat.flags |= RT_HAS_TR;
        }
        if (std::feof(in) && indef && (mat.flags & kValidMask) && !key.empty()) commit();
        std::memset(line, 0, kLineLen);
    }
    std::fclose(in);
    return true;
}

// Mesh::loadMtl into the scene: the blocks whose name is not yet indexed (materialIndex.find(key) == end)
void load_mtl(const std::string &filename, HostScene &s, MtlIndex &index) {
    std::vector<HostMaterial> blocks;
    if (!parse_mtl_file(filename, blocks)) {
        std::fprintf(stderr, "  Warning! Material file '%s' not found!\n", filename.c_str());
        return;
    }
    for (const HostMaterial &m : blocks) {
        if (index.find(m.name) >= 0) continue;
        s.mats.push_back(m);
        index.by_name[m.name] = static_cast<int>(s.mats.size()) - 1;
    }
}

}  // namespace

bool parse_mtl(const std::string &filename, std::vector<HostMaterial> &blocks) { return parse_mtl_file(filename, blocks); }

// The OBJ reader's material state (mesh.cpp:108-117 default material, :157-178 mtllib, :180-193
// usemtl), shared by the sequential and the parallel parser so both replay it identically.
ObjControlState::ObjControlState(const char *path, HostScene &scene) : s(scene), index(new MtlIndex) {
    HostMaterial def;   // defaultMat, mesh.cpp:108-117
    def.Kd[0] = def.Kd[1] = def.Kd[2] = 0.5f;
    def.Ks[0] = def.Ks[1] = def.Ks[2] = 0.5f;
    def.Ns = 96.7f;
    def.illum = 2;
    def.flags = RT_HAS_KD | RT_HAS_KA | RT_HAS_KS | RT_HAS_NS | RT_HAS_ILLUM;
    def.name = "StandardMaterialInitFromTriMesh";
    s.mats.push_back(def);
    std::string real(path);
    for (char &c : real) if (c == '\\') c = '/';
    const size_t slash = real.rfind('/');
    if (slash != std::string::npos) prefix = real.substr(0, slash + 1);
}

ObjControlState::~ObjControlState() { delete index; }

void ObjControlState::mtllib(char *line) {
    char *p0 = line + 6;
    while (std::isspace(static_cast<unsigned char>(*++p0))) {}
    size_t i = 0;
    while (p0[i] && !(static_cast<signed char>(p0[i]) < 32)) ++i;
    prefix.append(p0, i);      // path_.append(...) mutates the prefix (mesh.cpp:173-175)
    load_mtl(prefix, s, *index);
}

void ObjControlState::usemtl(char *line) {
    char *p0 = line + 6;
    while (std::isspace(static_cast<unsigned char>(*++p0))) {}
    char *p1 = p0;
    while (*p1 && !std::isspace(static_cast<unsigned char>(*p1))) ++p1;
    matname.assign(p0, p1);
    if (index->find(matname) < 0) {
        std::fprintf(stderr, "Warning! Material '%s' not defined in material file. Taking default!\n", matname.c_str());
        matname.clear();
    }
}

int ObjControlState::current_material() const {
    const int m = matname.empty() ? -1 : index->find(matname);
    return m < 0 ? 0 : m;
}

// Drop triangles referencing non-existent vertices (reference: out-of-bounds read), then the
// face normals.
void finish_obj(HostScene &s) {
    const uint32_t nv = static_cast<uint32_t>(s.verts.size() / 3);
    size_t k = 0;
    for (size_t i = 0; i < s.tri_mat.size(); ++i) {
        if (s.tris[3 * i] < nv && s.tris[3 * i + 1] < nv && s.tris[3 * i + 2] < nv) {
            s.tris[3 * k] = s.tris[3 * i]; s.tris[3 * k + 1] = s.tris[3 * i + 1]; s.tris[3 * k + 2] = s.tris[3 * i + 2];
            s.tri_mat[k] = s.tri_mat[i];
            if (s.has_texcoords)
                for (int j = 0; j < 3; ++j) s.tri_t[3 * k + j] = s.tri_t[3 * i + j];
            ++k;
        }
    }
    s.tris.resize(3 * k);
    s.tri_mat.resize(k);
    if (s.has_texcoords) s.tri_t.resize(3 * k);
    compute_face_normals(s);
}

int load_obj(const char *path, HostScene &s, std::string &err, bool texcoords) {
    s = HostScene();
    s.has_texcoords = texcoords;
    FILE *in = std::fopen(path, "r");
    if (!in) {
        err = std::string("cannot open OBJ file '") + path + "'";
        return RT_E_IO;
    }
    ObjControlState cs(path, s);
    char line[kLineLen];
    float x = 0, y = 0, z = 0;
    std::vector<int> vh, th;   // vhandles, texhandles (mesh.cpp:218-288)
    vh.reserve(64);
    th.reserve(64);
    std::memset(line, 0, kLineLen);
    while (!std::feof(in) && std::fgets(line, kLineLen, in)) {
        const char c0 = line[0];
        if (c0 == '#' || std::isspace(static_cast<unsigned char>(c0)) || c0 == '\0') {
            std::memset(line, 0, kLineLen);
            continue;
        }
        if (c0 == 'v' && line[1] == ' ') {
            std::sscanf(line, "v %f %f %f", &x, &y, &z);
            s.verts.push_back(x); s.verts.push_back(y); s.verts.push_back(z);
        } else if (texcoords && std::strncmp(line, "vt ", 3) == 0) {   // mesh.cpp:199-209: 2D, z = 0
            float t[3] = {0, 0, 0};
            std::sscanf(line, "vt %f %f", &t[0], &t[1]);
            s.texcoords.push_back(t[0]); s.texcoords.push_back(t[1]); s.texcoords.push_back(t[2]);
        } else if (c0 == 'f' && line[1] == ' ') {
            int component = 0;
            bool endOfVertex = false;
            char *p0, *p1 = line + 2;
            vh.clear();
            th.clear();
            while (*p1 == ' ') ++p1;
            while (p1) {
                p0 = p1;
                while (*p1 != '/' && *p1 != '\r' && *p1 != '\n' && *p1 != ' ' && *p1 != '\0') ++p1;
                if (*p1 != '/') endOfVertex = true;
                if (*p1 != '\0') { *p1 = '\0'; ++p1; }
                if (*p1 == '\0' || *p1 == '\n') p1 = nullptr;
                if (*p0 != '\0' && component == 0) vh.push_back(std::atoi(p0) - 1);
                if (*p0 != '\0' && component == 1 && texcoords) th.push_back(std::atoi(p0) - 1);
                ++component;
                if (endOfVertex) { component = 0; endOfVertex = false; }
            }
            const int m = cs.current_material();
            bool bad = false;
            for (int v : vh) bad |= (v < 0);
            if (texcoords && th.size() != vh.size()) th.resize(vh.size(), 0);   // mesh.cpp:290-291
            if (!bad) {
                if (vh.size() > 3) {
                    for (size_t i = 0; i + 2 < vh.size(); ++i) {
                        s.tris.push_back(uint32_t(vh[0])); s.tris.push_back(uint32_t(vh[i + 1]));
                        s.tris.push_back(uint32_t(vh[i + 2])); s.tri_mat.push_back(uint32_t(m));
                        if (texcoords) {
                            s.tri_t.push_back(uint32_t(th[0])); s.tri_t.push_back(uint32_t(th[i + 1]));
                            s.tri_t.push_back(uint32_t(th[i + 2]));
                        }
                    }
                } else if (vh.size() == 3) {
                    s.tris.push_back(uint32_t(vh[0])); s.tris.push_back(uint32_t(vh[1]));
                    s.tris.push_back(uint32_t(vh[2])); s.tri_mat.push_back(uint32_t(m));
                    if (texcoords) {
                        s.tri_t.push_back(uint32_t(th[0])); s.tri_t.push_back(uint32_t(th[1]));
                        s.tri_t.push_back(uint32_t(th[2]));
                    }
                }
            }
        } else if (std::strncmp(line, "mtllib ", 7) == 0) {
            cs.mtllib(line);
        } else if (std::strncmp(line, "usemtl ", 7) == 0) {
            cs.usemtl(line);
        }
        // `vn`, `o`, `g`, `s` (and `vt` without RT_LOAD_TEXCOORDS): not used by the tracer
        std::memset(line, 0, kLineLen);
    }
    std::fclose(in);
    finish_obj(s);
    return RT_OK;
}

// binary32 helpers with the Vec3D.h operation order (no contraction: built with -ffp-contract=off)
static inline void sub3(const float *a, const float *b, float *o) { o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2]; }
static inline float dot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void cross3(const float *a, const float *b, float *o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

void compute_face_normals(HostScene &s) {
    const size_t nt = s.tri_mat.size();
    s.normals.assign(3 * nt, 0.0f);
    for (size_t i = 0; i < nt; ++i) {
        const float *v0 = &s.verts[3 * s.tris[3 * i]];
        const float *v1 = &s.verts[3 * s.tris[3 * i + 1]];
        const float *v2 = &s.verts[3 * s.tris[3 * i + 2]];
        float e01[3], e02[3], n[3];
        sub3(v1, v0, e01);
        sub3(v2, v0, e02);
        cross3(e01, e02, n);
        float len = std::sqrt(dot3(n, n));     // Vec3D::normalize, Vec3D.h:142-151
        if (len != 0.0f) {
            float rez = 1.0f / len;
            n[0] *= rez; n[1] *= rez; n[2] *= rez;
        }
        s.normals[3 * i] = n[0]; s.normals[3 * i + 1] = n[1]; s.normals[3 * i + 2] = n[2];
    }
}

void build_tri_records(const HostScene &s, std::vector<TriRec> &out) {
    const size_t nt = s.tri_mat.size();
    out.resize(nt);
    for (size_t i = 0; i < nt; ++i) {
        const float *T0 = &s.verts[3 * s.tris[3 * i]];
        const float *T1 = &s.verts[3 * s.tris[3 * i + 1]];
        const float *T2 = &s.verts[3 * s.tris[3 * i + 2]];
        TriRec &r = out[i];
        float u[3], v[3], n[3];
        sub3(T1, T0, u);                        // raytracing.cpp:106
        sub3(T2, T0, v);                        // :107
        cross3(u, v, n);                        // :108
        const float uu = dot3(u, u);            // :134
        const float uv = dot3(u, v);            // :135
        const float vv = dot3(v, v);            // :136
        const float D = uv * uv - uu * vv;      // :140
        for (int k = 0; k < 3; ++k) { r.t0[k] = T0[k]; r.u[k] = u[k]; r.v[k] = v[k]; r.n[k] = n[k]; }
        r.uu = uu; r.uv = uv; r.vv = vv; r.D = D;
    }
}

void build_dev_materials(const HostScene &s, std::vector<DevMaterial> &out) {
    out.resize(s.mats.size());
    for (size_t i = 0; i < s.mats.size(); ++i) {
        const HostMaterial &m = s.mats[i];
        DevMaterial &d = out[i];
        for (int k = 0; k < 3; ++k) { d.Kd[k] = m.Kd[k]; d.Ka[k] = m.Ka[k]; d.Ks[k] = m.Ks[k]; }
        d.Ns = m.Ns; d.Ni = m.Ni; d.Tr = m.Tr; d.flags = m.flags;
        volatile float two = 2.0f;               // call glibc powf, as refraction() does
        float nr = 1 / m.Ni;                     // raytracing.cpp:301
        d.powf_nr2 = std::pow(nr, static_cast<float>(two));
        d.powf_ni2 = std::pow(m.Ni, static_cast<float>(two));
        d.transparent = ((m.flags & RT_HAS_TR) && m.Tr < 1.0f) ? 1u : 0u;
    }
}

}  // namespace rt
