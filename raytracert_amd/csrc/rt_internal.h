// rt_internal.h — host-side scene model and device-side record layouts shared by the loader,
// the render driver (rt_capi.cpp) and the kernels (rt_kernels.hip).
#pragma once

#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "raytracert_tune.h"   // (includes raytracert.h)

namespace rt {

// ---- host scene (Mesh, mesh.h:172-201, plus the face normals of raytracing.cpp:33) ---------
struct HostMaterial {
    float Kd[3] = {0, 0, 0}, Ka[3] = {0, 0, 0}, Ks[3] = {0, 0, 0};
    float Ns = 0, Ni = 0, Tr = 0;
    int32_t illum = 0;
    uint32_t flags = 0;
    std::string name;
};

struct HostScene {
    std::vector<float> verts;        // 3 per vertex
    std::vector<uint32_t> tris;      // 3 per triangle
    std::vector<uint32_t> tri_mat;   // per triangle
    std::vector<HostMaterial> mats;  // index 0 = default material (mesh.cpp:108-117)
    std::vector<float> normals;      // 3 per triangle (calculateNormals, raytracing.cpp:78-86)
    // Mesh::texcoords and Triangle::t (mesh.cpp:199-209, 263-268, 290-316), kept only when the scene
    // is loaded with RT_LOAD_TEXCOORDS (the tracer never reads them)
    bool has_texcoords = false;
    std::vector<float> texcoords;    // 3 per `vt` line (x, y, 0)
    std::vector<uint32_t> tri_t;     // 3 per triangle
};

// OBJ/MTL loader with Mesh::loadMesh / loadMtl semantics (mesh.cpp:95-460).
// Returns RT_OK or RT_E_IO; warnings go to stderr like the reference's printf.
int load_obj(const char *path, HostScene &out, std::string &err, bool texcoords = false);
// Mesh::loadMtl's parse (mesh.cpp:334-460) without the name filter: every block the reference
// would commit (name and material, in file order, unset values inherited from the previous block);
// loadMtl keeps the first block of each name not already indexed. false if the file cannot be opened.
bool parse_mtl(const std::string &filename, std::vector<HostMaterial> &blocks);
// calculateNormals (raytracing.cpp:78-86), binary32 without contraction.
void compute_face_normals(HostScene &s);

// ---- device layouts -----------------------------------------------------------------------
// One triangle = 4 x float4 = 64 B, every ray-independent quantity of rayIntersectTriangle
// (raytracing.cpp:106-108,134-136,140) hoisted; hoisting is bit-exact (same ops, same order).
//   q0 = {T0.x, T0.y, T0.z, uu}   q1 = {u.x, u.y, u.z, uv}
//   q2 = {v.x,  v.y,  v.z,  vv}   q3 = {n.x, n.y, n.z, D}
struct alignas(16) TriRec {
    float t0[3]; float uu;
    float u[3];  float uv;
    float v[3];  float vv;
    float n[3];  float D;
};
static_assert(sizeof(TriRec) == 64, "TriRec must be 64 bytes");
// The device copy of a record when the kernels divide by the reciprocal slot (tri_rcp_records):
// D replaced by RN(1/D) for normal |D| in [2^-30, 2^30], else NaN (those lanes divide by the
// recomputed D). The host's own copy (BVH build, validation) keeps D.
inline TriRec tri_rcp_slot(TriRec r) {
    const float a = std::fabs(r.D);
    r.D = (std::isnormal(r.D) && a >= 0x1p-30f && a <= 0x1p30f) ? 1.0f / r.D : NAN;
    return r;
}

struct alignas(16) DevMaterial {
    float Kd[3]; float Ns;
    float Ka[3]; float Ni;
    float Ks[3]; float Tr;
    uint32_t flags;
    float powf_nr2;      // glibc powf(1/Ni, 2)  (raytracing.cpp:302), precomputed on the host
    float powf_ni2;      // glibc powf(Ni, 2)    (raytracing.cpp:316)
    uint32_t transparent; // has_Tr && Tr < 1 (raytracing.cpp:254)
};
static_assert(sizeof(DevMaterial) == 64, "DevMaterial must be 64 bytes");

// ---- BVH (bvh.cpp) -------------------------------------------------------------------------
constexpr int kMaxBvhDepth = 40;                 // builder bound = GPU traversal stack depth
constexpr uint32_t kBvhLeafBit = 0x80000000u;    // child ref: leaf | count << 21 | first
constexpr int kBvhCountShift = 21;
constexpr uint32_t kBvhCountMask = 0x3FFu;
constexpr int32_t kBvhEmpty = static_cast<int32_t>(kBvhLeafBit);   // a leaf with no triangles
constexpr int kTopLevels4 = 4;                   // four-wide levels stored first, breadth-first (<= 85 nodes)
constexpr int kMaxTopNodes = 85;                 // RT_TUNE_TOP_NODES bound (LDS copy of the node array's prefix)

// Two children per node, both boxes stored in the parent (64 B).
struct alignas(16) BvhNode {
    float lo0[3], hi0[3];
    float lo1[3], hi1[3];
    int32_t c0, c1;
    int32_t pad[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must be 64 bytes");

// Four children per node (64 B): child boxes quantised to 8 bits per bound in the node's frame.
// Bound k of child c decodes as origin[k] + q * 2^ex[k] in float (the product is exact, so the
// device's fmaf gives the same value); the builder picks q so the decoded box contains the child's
// float box, so the exactness argument of the two-wide tree carries over unchanged.
struct alignas(16) Bvh4Node {
    float origin[3];
    int8_t ex[3];
    uint8_t n_children;
    uint32_t qlo[3];      // byte c of qlo[k] = child c's lower bound on axis k
    uint32_t qhi[3];
    int32_t child[4];     // inner node index, leaf ref (kBvhLeafBit | count << 21 | first) or kBvhEmpty
    uint32_t pad[2];
};
static_assert(sizeof(Bvh4Node) == 64, "Bvh4Node must be 64 bytes");

// The same four-wide node with float child boxes, the layout the kernels traverse: per axis k the
// four children's lower bounds (lo[k][c]) and upper bounds (hi[k][c]) as float4 rows, so a lane
// loads the near and far rows its ray direction needs by address (row k or 3 + k) and each slab
// plane of each child costs one FMA; the boxes are the children's padded acceptance-box unions
// themselves (no quantisation). Empty slots hold an inverted box (lo = +inf, hi = -inf).
struct alignas(16) Bvh4F {
    float lo[3][4];
    float hi[3][4];
    int32_t child[4];     // inner node index, leaf ref (kBvhLeafBit | count << 21 | first) or kBvhEmpty
    int32_t pad[4];
};
static_assert(sizeof(Bvh4F) == 128, "Bvh4F must be 128 bytes");

struct HostBvh {
    std::vector<BvhNode> nodes;       // nodes[0] is the root
    std::vector<Bvh4Node> nodes4;     // the same tree collapsed to four-wide nodes; nodes4[0] is the root
    std::vector<Bvh4F> nodes4f;       // nodes4 with float child boxes (same topology and order): what kernels read
    int depth4 = 0;                   // inner levels of the four-wide tree
    std::vector<uint32_t> leaf_tris;  // original triangle index of each leaf slot
    std::vector<uint32_t> always;     // ill-conditioned triangles every query tests
    size_t n_never = 0;               // n == 0: never accepted, never tested
    int depth = 0;
    float scene_m1 = 0;               // max |x|+|y|+|z| over vertices
};

bool acceptance_box(const TriRec &T, const float *v0, const float *v1, const float *v2, float lo[3], float hi[3],
                    bool *never);
int build_bvh(const HostScene &s, const std::vector<TriRec> &recs, HostBvh &out);
float bvh4_decode(float origin, int ex, uint32_t q);
uint64_t bvh_digest(const HostBvh &h);
int validate_bvh(const HostScene &s, const std::vector<TriRec> &recs, const HostBvh &h, std::string &err);

// OBJ reader material state shared by the sequential and the parallel parser (scene_loader.cpp).
struct MtlIndex;
class ObjControlState {
  public:
    ObjControlState(const char *path, HostScene &s);
    ~ObjControlState();
    ObjControlState(const ObjControlState &) = delete;
    ObjControlState &operator=(const ObjControlState &) = delete;
    void mtllib(char *line);    // an "mtllib ..." chunk
    void usemtl(char *line);    // a "usemtl ..." chunk
    int current_material() const;

  private:
    HostScene &s;
    MtlIndex *index;
    std::string prefix, matname;
};
void finish_obj(HostScene &s);
// Parallel parser, same result as load_obj (obj_parallel.cpp); threads <= 0: up to 16.
int load_obj_parallel(const char *path, HostScene &s, std::string &err, int threads);

void build_tri_records(const HostScene &s, std::vector<TriRec> &out);
void build_dev_materials(const HostScene &s, std::vector<DevMaterial> &out);

// glibc powf(x, 2) differs from the correctly rounded x*x exactly on the inputs listed in this
// table (|x| < 2, sorted bit patterns of |x|); on each of them glibc returns the next float up.
const uint32_t *powf2_tie_table(size_t *n);

// Error slot of the C-ABI (rt_last_error_string) for the library's other translation units, and
// the device a scene is bound to (RT_HOST_ONLY for host-only scenes).
int set_error(int code, const std::string &msg);
int guard_failure() noexcept;   // inside a catch handler of a C entry: the exception as an RT_E_* code
int scene_device(const rt_scene *s);

}  // namespace rt
