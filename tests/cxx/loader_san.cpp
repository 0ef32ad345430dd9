// Host-code sanitizer driver (ASan + UBSan; tests/sanitize.mk): the library's two OBJ/MTL loaders
// (scene_loader.cpp, the line-by-line restatement of mesh.cpp:95-460; obj_parallel.cpp, the
// parallel parser), its BVH builder (bvh.cpp) and the oracle (oracle/rt_oracle.c: loader, and a
// small brute-force render) run on each OBJ given. The reference's own loader has real UB
// (unknown usemtl names, missing usemtl, out-of-range indices: mesh.cpp:149-151,308,320,329);
// the restatements give it defined meaning, and this run checks they stay free of memory errors
// and UB on adversarial files. Also checks the parallel loader against the sequential one.
//   loader_san <obj>...     exit 0 and "ok <n>" per file; a sanitizer report aborts
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt_internal.h"
extern "C" {
#include "rt_oracle.h"
}

using namespace rt;

static bool same_bits(const std::vector<float> &a, const std::vector<float> &b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i) {
        if (a[i] != a[i] && b[i] != b[i]) continue;   // any NaN matches any NaN
        if (std::memcmp(&a[i], &b[i], 4) != 0) return false;
    }
    return true;
}

int main(int argc, char **argv) {
    int bad = 0;
    for (int f = 1; f < argc; ++f) {
        const char *path = argv[f];
        HostScene seq;
        std::string err;
        if (load_obj(path, seq, err) != RT_OK) { std::printf("unreadable %s\n", path); continue; }
        for (int threads : {1, 3, 16}) {
            HostScene par;
            if (load_obj_parallel(path, par, err, threads) != RT_OK) { std::printf("parallel failed %s\n", path); bad = 1; continue; }
            if (par.tris != seq.tris || par.tri_mat != seq.tri_mat || !same_bits(par.verts, seq.verts) ||
                !same_bits(par.normals, seq.normals) || par.mats.size() != seq.mats.size()) {
                std::printf("mismatch %s threads %d\n", path, threads);
                bad = 1;
            }
        }
        std::vector<TriRec> recs;
        build_tri_records(seq, recs);
        std::vector<DevMaterial> dm;
        build_dev_materials(seq, dm);
        HostBvh bvh;
        if (!recs.empty()) {
            if (build_bvh(seq, recs, bvh) != RT_OK) { std::printf("bvh failed %s\n", path); bad = 1; }
            else if (validate_bvh(seq, recs, bvh, err) != RT_OK) { std::printf("bvh invalid %s: %s\n", path, err.c_str()); bad = 1; }
        }
        ora_scene *o = nullptr;
        if (ora_load_obj(path, &o) != 0) { std::printf("oracle unreadable %s\n", path); bad = 1; continue; }
        int32_t nv = 0, nt = 0, nm = 0;
        ora_counts(o, &nv, &nt, &nm);
        if (static_cast<size_t>(nt) != seq.tri_mat.size() || static_cast<size_t>(nv) * 3 != seq.verts.size()) {
            std::printf("oracle counts differ %s\n", path);
            bad = 1;
        }
        ora_params p;
        std::memset(&p, 0, sizeof(p));
        p.width = 12; p.height = 9; p.pfx = p.pfy = 2; p.max_lvl = 3; p.flags = ORA_ALL_FEATURES; p.n_lights = 2;
        p.lights[0][2] = 4.0f; p.lights[1][0] = 1.5f; p.lights[1][1] = 1.5f; p.lights[1][2] = 4.0f;
        p.camera_pos[2] = 4.0f;
        ora_default_corners(p.width, p.height, p.corners);
        std::vector<uint8_t> u8(12 * 9 * 3);
        uint64_t counts[3] = {0, 0, 0};
        ora_render(o, &p, 0, 0, 12, 9, nullptr, u8.data(), 2, counts);
        ora_free(o);
        std::printf("ok %s %zu %llu\n", path, seq.tri_mat.size(), static_cast<unsigned long long>(counts[0] + counts[1] + counts[2]));
    }
    return bad;
}
