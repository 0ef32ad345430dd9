// obj_parallel.cpp — parallel OBJ parser with exactly the result of the sequential restatement
// load_obj (scene_loader.cpp, itself Mesh::loadMesh, CG_Project/mesh.cpp:95-331) — SURVEY.md §8
// row f2.
//
// How the sequential semantics survive the split:
//  * The file is read whole and cut into segments at line starts. fgets(line, 256) chunks restart
//    at every newline, so each segment yields exactly the chunks the sequential reader sees there
//    (lines longer than 255 characters split the same way).
//  * Each chunk goes through the same classification and face tokenisation as load_obj. `v`
//    lines: a strict decimal token grammar is converted exactly (Clinger's fast path when the
//    digits fit in 24 bits and the power of ten is exact in binary32, strtof otherwise); any other
//    spelling falls back to the same sscanf call. The number of assigned components is kept, and
//    the values sscanf would have left from the previous `v` line (x, y, z persist, mesh.cpp:121)
//    are filled in order after the merge.
//  * `mtllib` / `usemtl` are recorded with the number of faces the segment had produced at that
//    point and replayed in file order after the parse (load_mtl runs then, so materials, indices
//    and warnings come out exactly as in the sequential pass).
//  * Face indices are absolute (atoi - 1), so per-segment face lists concatenate unchanged.
// tests/test_loader.py compares the two loaders field by field on every reference OBJ and on
// adversarial files (long lines, partial `v` lines, odd number spellings, usemtl before mtllib).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rt_internal.h"

namespace rt {
namespace {

constexpr int kLineLen = 256;   // mesh.cpp:22

struct Control {
    bool mtllib;            // else usemtl
    std::string arg;        // the raw chunk text after the keyword (parsed at replay)
    size_t faces_before;    // triangles this segment had produced before the line
};

struct Segment {
    std::vector<float> v;        // x, y, z per `v` line
    std::vector<uint8_t> vn;     // components sscanf assigned (0..3)
    std::vector<uint32_t> tris;  // 3 per triangle (absolute, unchecked)
    std::vector<Control> ctl;
};

inline bool is_space(char c) { return std::isspace(static_cast<unsigned char>(c)) != 0; }

const float kPow10[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};   // all exact

// One %f conversion of a strict decimal token at p (after optional whitespace). Returns the
// pointer past the token, or nullptr when the spelling is outside the grammar
// [+-]?digits[.digits]?([eE][+-]?digits)? followed by whitespace or the end of the string; then
// the caller lets sscanf decide.
const char *parse_decimal(const char *p, float *out) {
    while (is_space(*p)) ++p;
    const char *start = p;
    bool neg = false;
    if (*p == '+' || *p == '-') { neg = (*p == '-'); ++p; }
    uint64_t mant = 0;
    int frac = 0, nd = 0;
    bool any = false;
    while (*p >= '0' && *p <= '9') {
        any = true;
        if (mant || *p != '0') { if (nd < 19) { mant = mant * 10 + uint64_t(*p - '0'); ++nd; } else return nullptr; }
        ++p;
    }
    if (*p == '.') {
        ++p;
        while (*p >= '0' && *p <= '9') {
            any = true;
            if (mant || *p != '0') { if (nd < 19) { mant = mant * 10 + uint64_t(*p - '0'); ++nd; } else return nullptr; }
            ++frac; ++p;
        }
    }
    if (!any) return nullptr;
    int e10 = 0;
    if (*p == 'e' || *p == 'E') {
        const char *q = p + 1;
        bool eneg = false;
        if (*q == '+' || *q == '-') { eneg = (*q == '-'); ++q; }
        if (!(*q >= '0' && *q <= '9')) return nullptr;   // "1e" / "1e+": scanf's pushback rules, not ours
        int ev = 0;
        while (*q >= '0' && *q <= '9') { if (ev < 100000) ev = ev * 10 + (*q - '0'); ++q; }
        e10 = eneg ? -ev : ev;
        p = q;
    }
    if (*p != '\0' && !is_space(*p)) return nullptr;
    const int e = e10 - frac;
    float v;
    if (mant < (uint64_t(1) << 24) && e >= -10 && e <= 10) {
        // Clinger: both operands exact in binary32, one correctly rounded operation
        const float m = static_cast<float>(mant);
        v = e >= 0 ? m * kPow10[e] : m / kPow10[-e];
    } else {
        char tmp[kLineLen];
        const size_t n = static_cast<size_t>(p - start);
        if (n >= sizeof tmp) return nullptr;
        std::memcpy(tmp, start, n);
        tmp[n] = '\0';
        v = std::strtof(tmp, nullptr);   // glibc: correctly rounded, as scanf's %f
        *out = v;
        return p;
    }
    *out = neg ? -v : v;
    return p;
}

// The `v` line: the values sscanf("v %f %f %f") assigns and how many.
void parse_vertex(const char *line, float xyz[3], uint8_t *n) {
    const char *p = line + 1;   // after 'v'; "%f" skips the whitespace the format's ' ' matches
    int k = 0;
    for (; k < 3; ++k) {
        const char *q = parse_decimal(p, &xyz[k]);
        if (!q) break;
        p = q;
    }
    if (k == 3) { *n = 3; return; }
    // outside the fast grammar: the sequential loader's own call decides (assigned prefix)
    float a = 0, b = 0, c = 0;
    const int r = std::sscanf(line, "v %f %f %f", &a, &b, &c);
    const int m = r < 0 ? 0 : r;
    xyz[0] = a; xyz[1] = b; xyz[2] = c;
    *n = static_cast<uint8_t>(m);
}

// Face tokenisation of load_obj (mesh.cpp:218-316) on a private copy of the chunk.
void parse_face(char *line, std::vector<int> &vh, std::vector<uint32_t> &tris) {
    int component = 0;
    bool endOfVertex = false;
    char *p0, *p1 = line + 2;
    vh.clear();
    while (*p1 == ' ') ++p1;
    while (p1) {
        p0 = p1;
        while (*p1 != '/' && *p1 != '\r' && *p1 != '\n' && *p1 != ' ' && *p1 != '\0') ++p1;
        if (*p1 != '/') endOfVertex = true;
        if (*p1 != '\0') { *p1 = '\0'; ++p1; }
        if (*p1 == '\0' || *p1 == '\n') p1 = nullptr;
        if (*p0 != '\0' && component == 0) vh.push_back(std::atoi(p0) - 1);
        ++component;
        if (endOfVertex) { component = 0; endOfVertex = false; }
    }
    for (int v : vh)
        if (v < 0) return;
    if (vh.size() > 3) {
        for (size_t i = 0; i + 2 < vh.size(); ++i) {
            tris.push_back(uint32_t(vh[0])); tris.push_back(uint32_t(vh[i + 1])); tris.push_back(uint32_t(vh[i + 2]));
        }
    } else if (vh.size() == 3) {
        tris.push_back(uint32_t(vh[0])); tris.push_back(uint32_t(vh[1])); tris.push_back(uint32_t(vh[2]));
    }
}

// All fgets chunks of [a, b) (a at a line start).
void parse_segment(const char *buf, size_t a, size_t b, Segment &sg) {
    char line[kLineLen];
    std::vector<int> vh;
    vh.reserve(64);
    size_t pos = a;
    while (pos < b) {
        const size_t lim = std::min(b, pos + (kLineLen - 1));
        const void *nl = std::memchr(buf + pos, '\n', lim - pos);
        const size_t end = nl ? static_cast<size_t>(static_cast<const char *>(nl) - buf) + 1 : lim;
        const size_t len = end - pos;
        std::memcpy(line, buf + pos, len);
        line[len] = '\0';
        pos = end;
        const char c0 = line[0];
        if (c0 == '#' || is_space(c0) || c0 == '\0') continue;
        if (c0 == 'v' && line[1] == ' ') {
            float xyz[3] = {0, 0, 0};
            uint8_t n = 0;
            parse_vertex(line, xyz, &n);
            sg.v.insert(sg.v.end(), xyz, xyz + 3);
            sg.vn.push_back(n);
        } else if (c0 == 'f' && line[1] == ' ') {
            parse_face(line, vh, sg.tris);
        } else if (std::strncmp(line, "mtllib ", 7) == 0) {
            sg.ctl.push_back(Control{true, std::string(line), sg.tris.size() / 3});
        } else if (std::strncmp(line, "usemtl ", 7) == 0) {
            sg.ctl.push_back(Control{false, std::string(line), sg.tris.size() / 3});
        }
    }
}

}  // namespace

int load_obj_parallel(const char *path, HostScene &s, std::string &err, int threads) {
    s = HostScene();
    FILE *in = std::fopen(path, "rb");
    if (!in) {
        err = std::string("cannot open OBJ file '") + path + "'";
        return RT_E_IO;
    }
    std::vector<char> buf;
    {
        std::fseek(in, 0, SEEK_END);
        const long sz = std::ftell(in);
        std::fseek(in, 0, SEEK_SET);
        if (sz < 0) { std::fclose(in); err = "cannot size OBJ file"; return RT_E_IO; }
        buf.resize(static_cast<size_t>(sz) + 1);
        const size_t got = std::fread(buf.data(), 1, static_cast<size_t>(sz), in);
        buf.resize(got);
    }
    std::fclose(in);
    const size_t size = buf.size();

    // segments at line starts, ~equal bytes
    if (threads <= 0) {   // auto: up to 16 threads, about 1 MiB of text each at least
        threads = static_cast<int>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
        threads = static_cast<int>(std::max<size_t>(1, std::min<size_t>(threads, size / (1 << 20) + 1)));
    }
    threads = std::min(threads, 256);
    std::vector<size_t> cut{0};
    for (int t = 1; t < threads; ++t) {
        size_t p = size * static_cast<size_t>(t) / static_cast<size_t>(threads);
        p = std::max(p, cut.back());
        const void *nl = p < size ? std::memchr(buf.data() + p, '\n', size - p) : nullptr;
        cut.push_back(nl ? static_cast<size_t>(static_cast<const char *>(nl) - buf.data()) + 1 : size);
    }
    cut.push_back(size);
    const int ns = static_cast<int>(cut.size()) - 1;
    std::vector<Segment> seg(ns);
    {
        std::vector<std::thread> pool;
        for (int t = 1; t < ns; ++t) pool.emplace_back(parse_segment, buf.data(), cut[t], cut[t + 1], std::ref(seg[t]));
        if (ns > 0) parse_segment(buf.data(), cut[0], cut[1], seg[0]);
        for (auto &th : pool) th.join();
    }

    // vertices in file order; components sscanf left unassigned keep the previous line's values
    size_t nv = 0, ntri = 0;
    for (const Segment &sg : seg) { nv += sg.vn.size(); ntri += sg.tris.size() / 3; }
    s.verts.resize(3 * nv);
    {
        float run[3] = {0, 0, 0};   // x, y, z start at 0 (load_obj)
        size_t o = 0;
        for (const Segment &sg : seg) {
            for (size_t i = 0; i < sg.vn.size(); ++i, ++o) {
                const uint8_t n = sg.vn[i];
                for (int k = 0; k < 3; ++k) {
                    if (k < n) run[k] = sg.v[3 * i + k];
                    s.verts[3 * o + k] = run[k];
                }
            }
        }
    }

    // materials and face materials: replay mtllib / usemtl in file order
    s.tris.reserve(3 * ntri);
    s.tri_mat.reserve(ntri);
    ObjControlState cs(path, s);
    for (const Segment &sg : seg) {
        size_t done = 0;
        auto emit = [&](size_t upto) {
            for (; done < upto; ++done) {
                s.tris.push_back(sg.tris[3 * done]);
                s.tris.push_back(sg.tris[3 * done + 1]);
                s.tris.push_back(sg.tris[3 * done + 2]);
                s.tri_mat.push_back(static_cast<uint32_t>(cs.current_material()));
            }
        };
        for (const Control &c : sg.ctl) {
            emit(c.faces_before);
            std::vector<char> line(c.arg.begin(), c.arg.end());
            line.push_back('\0');
            if (c.mtllib) cs.mtllib(line.data());
            else cs.usemtl(line.data());
        }
        emit(sg.tris.size() / 3);
    }
    finish_obj(s);
    return RT_OK;
}

}  // namespace rt
