// bvh.cpp — parity-preserving BVH over the triangle records (the reference's own
// intended acceleration, CG_Project/raytracing.cpp:167-172).
//
// Exactness argument. intersectMesh (raytracing.cpp:161-192) returns the lexicographic minimum of
// (distance, index) over every triangle that rayIntersectTriangle accepts with distance < FLT_MAX.
// That minimum does not depend on the order triangles are visited, so a traversal that (1) runs
// the identical per-triangle test on every triangle it visits and (2) never skips a triangle that
// could be accepted with a (distance, index) not larger than the current best returns the same
// index and the same hit point bit for bit. (2) needs conservative boxes:
//
//  * Acceptance region. rayIntersectTriangle computes s, t from w = I - T0 with rounding, so an I
//    slightly outside the triangle can be accepted. With c = |D| / (uu*vv) (sin^2 of the angle at
//    T0) and eps = 2^-24, first-order error analysis of wu, wv (4 eps |w||u|, 4 eps |w||v|), of
//    the products and difference in s's numerator, of uv, vv, D as rounded per-triangle values
//    (D relative error <= 8 eps / c) and of the final division and s+t, bounds the in-plane
//    SPATIAL displacement that any of the three tests can absorb by K eps |w| with
//    K = 36/c + 18/c^1.5 + 2/sqrt(c). A point at distance d outside the triangle has |w| <= 2L + d
//    (L = longest of |u|, |v|), so it can only be accepted if d <= 2 K eps L / (1 - K eps). The
//    box is the triangle's bounding box widened by 4x that bound, taken in the plane (axis k:
//    times sqrt(1 - n_k^2), r04), plus 1e-7 L.
//  * Off-plane. I = o + r*dir with r = a/b rounded; whatever the error in r, I stays on the ray, and
//    its distance from the plane is at most ~6 eps (|o - T0| + |I - o|). The kernel adds
//    pad_ray = 64 eps (|o|_1 + M_1) to every box at traversal time (M_1 = max |x|+|y|+|z| of the
//    vertices), which also covers the rounding of I itself.
//  * Triangles with D == 0 or non-finite (then s, t are NaN/inf and the reference accepts almost
//    anything), or with K eps > kMaxDelta = 0.2 (angle at T0 below ~1 degree; up to there the
//    first-order bound's second-order terms, ~(K eps)^2, stay far inside the factor-4 pad), are not put in the tree:
//    every query tests them first (the "always" list). Triangles with n == 0 are rejected by
//    isNullVector and never tested.
//  * Box tests and the distance cull use relative slack (1e-5) far above their rounding error.
//
// tests/test_bvh.py checks the acceptance claim directly against the oracle's arithmetic, and
// tests/test_gpu_parity.py checks BVH results against brute force bit for bit.
#include <algorithm>
#include <array>
#include <atomic>
#include <thread>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "rt_internal.h"

namespace rt {
namespace {

constexpr double kEps = 5.9604644775390625e-08;   // 2^-24
#ifndef RT_BVH_MAX_KE
#define RT_BVH_MAX_KE 0.2
#endif
// K*eps bound for a tree triangle (pad <= 2 L): angle at T0 >~ 1 degree. 0.5 (pad <= 8 L, >~ 0.75
// degree; its neglected terms still inside the factor-4 pad, tests/test_bvh.py) moved 13 of the car
// model's 30 always-tested slivers into the tree: ref_default 0.249 -> 0.235 ms but C2 0.079 ->
// 0.087 ms (their big boxes lengthen the car region's walks; profiles/r04_ab_max_ke.txt).
constexpr double kMaxDelta = RT_BVH_MAX_KE;
constexpr int kBins = 16;
#ifndef RT_BVH_MAX_LEAF
#define RT_BVH_MAX_LEAF 2   // measured: 2 beats 4 by ~4% (C4 and the 1M-triangle grid), 8 loses 15%
#endif
#ifndef RT_BVH_TRAV_COST
#define RT_BVH_TRAV_COST 1.0
#endif
#ifndef RT_BVH_INPLANE_PAD
#define RT_BVH_INPLANE_PAD 1   // the acceptance pad in the triangle's plane only (0: on every axis, r03)
#endif
constexpr int kMaxLeaf = RT_BVH_MAX_LEAF;
constexpr double kTravCost = RT_BVH_TRAV_COST;   // SAH: node traversal relative to one triangle test

struct Box {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const Box &b) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
    }
    void grow(const float *p) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
    }
    bool empty() const { return lo[0] > hi[0]; }
    double area() const {
        if (empty()) return 0.0;
        const double dx = double(hi[0]) - lo[0], dy = double(hi[1]) - lo[1], dz = double(hi[2]) - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct BuildPrim {
    Box box;
    float centroid[3];
    uint32_t tri;
};

struct BuildNode {
    Box box;
    int left = -1, right = -1;   // children (build indices) for inner nodes
    int first = 0, count = 0;    // prim range for leaves
};

// Round a float outward by one ulp-scale step (boxes must contain the exact double bounds).
inline float down(double v) { float f = static_cast<float>(v); return (static_cast<double>(f) > v) ? std::nextafter(f, -FLT_MAX) : f; }
inline float up(double v) { float f = static_cast<float>(v); return (static_cast<double>(f) < v) ? std::nextafter(f, FLT_MAX) : f; }

struct Builder {
    std::vector<BuildPrim> &prims;
    std::vector<BuildNode> nodes;
    int max_depth = 0;

    explicit Builder(std::vector<BuildPrim> &p) : prims(p) {}

    // One node over prims[first, first + count): its box, and either a leaf (returns -1) or the
    // binned-SAH split position with the range partitioned around it (returns mid).
    int threads = 1;   // > 1: the scans over one node's prims are split (top of the tree only)

    // Apply fn(begin, end, part) over [first, first + count) in `parts` contiguous parts.
    template <typename F>
    void split_scan(int first, int count, int parts, F &&fn) {
        if (parts <= 1) { fn(first, first + count, 0); return; }
        std::vector<std::thread> pool;
        for (int t = 1; t < parts; ++t)
            pool.emplace_back([&, t]() { fn(first + int(int64_t(count) * t / parts), first + int(int64_t(count) * (t + 1) / parts), t); });
        fn(first, first + int(int64_t(count) / parts), 0);
        for (auto &th : pool) th.join();
    }

    int make_node(int first, int count, int depth, int &id) {
        // min/max boxes and bin counts are order-independent, so splitting the scans changes nothing
        const int parts = (threads > 1 && count >= (1 << 17)) ? threads : 1;
        BuildNode n;
        Box cb;
        {
            std::vector<Box> pb(parts), pc(parts);
            split_scan(first, count, parts, [&](int a, int e, int t) {
                for (int i = a; i < e; ++i) { pb[t].grow(prims[i].box); pc[t].grow(prims[i].centroid); }
            });
            for (int t = 0; t < parts; ++t) { n.box.grow(pb[t]); cb.grow(pc[t]); }
        }
        id = static_cast<int>(nodes.size());
        nodes.push_back(n);
        max_depth = std::max(max_depth, depth);
        if (count <= kMaxLeaf || depth >= kMaxBvhDepth - 1) {
            nodes[id].first = first;
            nodes[id].count = count;
            return -1;
        }
        int best_axis = -1, best_split = -1;
        double best_cost = static_cast<double>(count) * n.box.area();   // cost of a leaf (intersection-only SAH)
        for (int axis = 0; axis < 3; ++axis) {
            const double lo = cb.lo[axis], ext = double(cb.hi[axis]) - lo;
            if (!(ext > 0)) continue;
            Box bb[kBins];
            int bc[kBins] = {0};
            {
                std::vector<std::array<Box, kBins>> pbb(parts);
                std::vector<std::array<int, kBins>> pbc(parts);
                split_scan(first, count, parts, [&](int a, int e, int t) {
                    pbc[t].fill(0);
                    for (int i = a; i < e; ++i) {
                        int b = static_cast<int>((prims[i].centroid[axis] - lo) / ext * kBins);
                        b = std::min(std::max(b, 0), kBins - 1);
                        pbb[t][b].grow(prims[i].box);
                        pbc[t][b]++;
                    }
                });
                for (int t = 0; t < parts; ++t)
                    for (int b = 0; b < kBins; ++b) { bb[b].grow(pbb[t][b]); bc[b] += pbc[t][b]; }
            }
            Box left[kBins];
            int lc[kBins];
            Box acc;
            int c = 0;
            for (int b = 0; b < kBins; ++b) { acc.grow(bb[b]); c += bc[b]; left[b] = acc; lc[b] = c; }
            acc = Box();
            c = 0;
            for (int b = kBins - 1; b > 0; --b) {
                acc.grow(bb[b]); c += bc[b];
                const int nl = lc[b - 1];
                if (nl == 0 || c == 0) continue;
                const double cost = kTravCost * n.box.area() + nl * left[b - 1].area() + c * acc.area();
                if (cost < best_cost) { best_cost = cost; best_axis = axis; best_split = b; }
            }
        }
        int mid;
        if (best_axis < 0) {
            if (count <= 2 * kMaxLeaf) {   // no useful split: small leaf
                nodes[id].first = first;
                nodes[id].count = count;
                return -1;
            }
            // degenerate centroids: median split on the widest box axis
            int axis = 0;
            for (int k = 1; k < 3; ++k)
                if (double(n.box.hi[k]) - n.box.lo[k] > double(n.box.hi[axis]) - n.box.lo[axis]) axis = k;
            mid = first + count / 2;
            std::nth_element(prims.begin() + first, prims.begin() + mid, prims.begin() + first + count,
                             [axis](const BuildPrim &a, const BuildPrim &b) { return a.centroid[axis] < b.centroid[axis]; });
        } else {
            const double lo = cb.lo[best_axis], ext = double(cb.hi[best_axis]) - lo;
            auto it = std::partition(prims.begin() + first, prims.begin() + first + count, [&](const BuildPrim &p) {
                int b = static_cast<int>((p.centroid[best_axis] - lo) / ext * kBins);
                b = std::min(std::max(b, 0), kBins - 1);
                return b < best_split;
            });
            mid = static_cast<int>(it - prims.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        return mid;
    }

    int build(int first, int count, int depth) {
        int id;
        const int mid = make_node(first, count, depth, id);
        if (mid < 0) return id;
        const int l = build(first, mid - first, depth + 1);
        const int r = build(mid, first + count - mid, depth + 1);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }

    // The same tree, built by `threads` threads: the top levels are split here until there are
    // about four subtrees per thread, then each subtree is built by its own Builder over its
    // disjoint prim range and spliced in. Every node makes the decision the sequential build
    // makes on the same range, so the flattened tree is identical.
    void build_parallel(int count, int threads) {
        struct Task { int first, count, depth, parent; bool right; };
        std::vector<Task> todo, frontier{Task{0, count, 0, -1, false}};
        this->threads = threads;
        const int grain = std::max(4096, count / (4 * std::max(threads, 1)));
        while (!frontier.empty()) {
            const Task t = frontier.back();
            frontier.pop_back();
            if (t.count <= grain) { todo.push_back(t); continue; }
            int id;
            const int mid = make_node(t.first, t.count, t.depth, id);
            if (t.parent >= 0) (t.right ? nodes[t.parent].right : nodes[t.parent].left) = id;
            if (mid < 0) continue;
            frontier.push_back(Task{mid, t.first + t.count - mid, t.depth + 1, id, true});
            frontier.push_back(Task{t.first, mid - t.first, t.depth + 1, id, false});
        }
        std::vector<Builder> sub;
        sub.reserve(todo.size());
        for (size_t i = 0; i < todo.size(); ++i) sub.emplace_back(prims);
        std::vector<int> root(todo.size(), -1);
        std::atomic<size_t> next{0};
        auto worker = [&]() {
            for (size_t i; (i = next.fetch_add(1)) < todo.size();) root[i] = sub[i].build(todo[i].first, todo[i].count, todo[i].depth);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < threads; ++t) pool.emplace_back(worker);
        worker();
        for (auto &th : pool) th.join();
        for (size_t i = 0; i < todo.size(); ++i) {
            const int off = static_cast<int>(nodes.size());
            for (BuildNode n : sub[i].nodes) {
                if (n.left >= 0) { n.left += off; n.right += off; }
                nodes.push_back(n);
            }
            const int r = root[i] + off;
            if (todo[i].parent >= 0) (todo[i].right ? nodes[todo[i].parent].right : nodes[todo[i].parent].left) = r;
            max_depth = std::max(max_depth, sub[i].max_depth);
        }
    }
};


int32_t leaf_ref(const BuildNode &bn) {
    return static_cast<int32_t>(kBvhLeafBit | (static_cast<uint32_t>(bn.count) << kBvhCountShift) | static_cast<uint32_t>(bn.first));
}

// Quantise axis k of up to four child boxes in the frame [L, H]: the smallest exponent for which
// every decoded bound lands on the outside of the float bound it replaces.
bool quantize_axis(float L, float H, const Box *boxes, int nc, int k, Bvh4Node &g) {
    const double ext = double(H) - double(L);
    int e = -126;
    if (ext > 0) e = std::max(-126, static_cast<int>(std::ceil(std::log2(ext / 255.0))) - 1);
    for (; e <= 100; ++e) {
        if (bvh4_decode(L, e, 255) < H) continue;
        const double scale = std::ldexp(1.0, e);
        uint32_t lo = 0, hi = 0;
        bool ok = true;
        for (int c = 0; c < nc && ok; ++c) {
            const float cl = boxes[c].lo[k], ch = boxes[c].hi[k];
            int ql = static_cast<int>(std::min(255.0, std::max(0.0, std::floor((double(cl) - L) / scale))));
            while (ql > 0 && bvh4_decode(L, e, ql) > cl) --ql;
            int qh = static_cast<int>(std::min(255.0, std::max(0.0, std::ceil((double(ch) - L) / scale))));
            while (qh < 255 && bvh4_decode(L, e, qh) < ch) ++qh;
            ok = bvh4_decode(L, e, ql) <= cl && bvh4_decode(L, e, qh) >= ch;
            lo |= static_cast<uint32_t>(ql) << (8 * c);
            hi |= static_cast<uint32_t>(qh) << (8 * c);
        }
        if (!ok) continue;
        g.ex[k] = static_cast<int8_t>(e);
        g.qlo[k] = lo;
        g.qhi[k] = hi;
        return true;
    }
    return false;
}

bool make_node4(const Box *boxes, const int32_t *refs, int nc, Bvh4Node &g) {
    g = Bvh4Node{};
    Box u;
    for (int c = 0; c < nc; ++c) u.grow(boxes[c]);
    g.n_children = static_cast<uint8_t>(nc);
    for (int c = 0; c < 4; ++c) g.child[c] = c < nc ? refs[c] : kBvhEmpty;
    for (int k = 0; k < 3; ++k) {
        g.origin[k] = nc ? u.lo[k] : 0.0f;
        if (nc == 0) continue;
        if (!quantize_axis(u.lo[k], u.hi[k], boxes, nc, k, g)) return false;
    }
    // empty slots get an inverted box (lo byte 255, hi byte 0 on every axis): the slab test
    // rejects it whatever the ray's direction (and if rounding ever let one through, its ref is an
    // empty leaf, which tests nothing), so the kernel needs no per-child empty check
    for (int c = nc; c < 4; ++c)
        for (int k = 0; k < 3; ++k) {
            g.qlo[k] |= 0xFFu << (8 * c);
            g.qhi[k] &= ~(0xFFu << (8 * c));
        }
    return true;
}

Bvh4F make_node4f(const Box *boxes, const int32_t *refs, int nc) {
    Bvh4F g{};
    for (int c = 0; c < 4; ++c) {
        g.child[c] = c < nc ? refs[c] : kBvhEmpty;
        for (int k = 0; k < 3; ++k) {
            g.lo[k][c] = c < nc ? boxes[c].lo[k] : INFINITY;   // empty: inverted, rejected by any slab test
            g.hi[k][c] = c < nc ? boxes[c].hi[k] : -INFINITY;
        }
    }
    return g;
}

// Collapse the binary build tree into four-wide nodes: repeatedly open the largest-area inner
// child until a node has four children (the usual SAH-driven collapse), depth-first order.
struct Collapser {
    const Builder &b;
    std::vector<Bvh4Node> &out;
    std::vector<Bvh4F> &outf;
    int depth = 0;
    bool ok = true;
    int run(int n, int level) {
        std::vector<int> ch{b.nodes[n].left, b.nodes[n].right};
        while (ch.size() < 4) {
            int best = -1;
            double best_area = -1;
            for (size_t i = 0; i < ch.size(); ++i) {
                const BuildNode &c = b.nodes[ch[i]];
                if (c.left >= 0 && c.box.area() > best_area) { best_area = c.box.area(); best = static_cast<int>(i); }
            }
            if (best < 0) break;
            const int x = ch[best];
            ch[best] = b.nodes[x].left;
            ch.insert(ch.begin() + best + 1, b.nodes[x].right);
        }
        const int id = static_cast<int>(out.size());
        out.emplace_back();
        outf.emplace_back();
        depth = std::max(depth, level);
        Box boxes[4];
        int32_t refs[4];
        const int nc = static_cast<int>(ch.size());
        for (int c = 0; c < nc; ++c) {
            const BuildNode &cn = b.nodes[ch[c]];
            boxes[c] = cn.box;
            refs[c] = cn.left >= 0 ? run(ch[c], level + 1) : leaf_ref(cn);
        }
        Bvh4Node g;
        ok = ok && make_node4(boxes, refs, nc, g);
        out[id] = g;
        outf[id] = make_node4f(boxes, refs, nc);
        return id;
    }
};

// Renumber the four-wide nodes so the top `levels` levels come first in breadth-first order
// (the root stays 0); deeper nodes keep their depth-first order. Kernels keep a prefix of the
// node array (the levels every query visits) together, at the start of the array.
void top_levels_first(std::vector<Bvh4Node> &nodes, std::vector<Bvh4F> &nodesf, int levels) {
    const size_t n = nodes.size();
    if (n <= 1) return;
    std::vector<int> order{0}, lvl{0};
    std::vector<char> top(n, 0);
    top[0] = 1;
    for (size_t head = 0; head < order.size(); ++head) {
        if (lvl[head] + 1 >= levels) continue;
        const Bvh4Node &g = nodes[order[head]];
        for (int c = 0; c < 4; ++c) {
            const int32_t r = g.child[c];
            if (r < 0 || top[r]) continue;   // leaf, empty slot
            top[r] = 1;
            order.push_back(r);
            lvl.push_back(lvl[head] + 1);
        }
    }
    for (size_t i = 0; i < n; ++i)
        if (!top[i]) order.push_back(static_cast<int>(i));
    std::vector<int32_t> id(n);
    for (size_t k = 0; k < n; ++k) id[order[k]] = static_cast<int32_t>(k);
    std::vector<Bvh4Node> out(n);
    std::vector<Bvh4F> outf(n);
    for (size_t k = 0; k < n; ++k) {
        out[k] = nodes[order[k]];
        outf[k] = nodesf[order[k]];
        for (int c = 0; c < 4; ++c)
            if (out[k].child[c] >= 0) outf[k].child[c] = out[k].child[c] = id[out[k].child[c]];
    }
    nodes.swap(out);
    nodesf.swap(outf);
}

}  // namespace

float bvh4_decode(float origin, int ex, uint32_t q) {
    return origin + static_cast<float>(q) * std::ldexp(1.0f, ex);   // q * 2^ex is exact
}

// Padded acceptance box of one record; returns false if the triangle must be tested by every
// query (ill-conditioned), and sets *never if it can never be accepted (n == 0).
bool acceptance_box(const TriRec &T, const float *v0, const float *v1, const float *v2, float lo[3], float hi[3],
                    bool *never) {
    *never = (T.n[0] == 0 && T.n[1] == 0 && T.n[2] == 0);
    if (*never) return true;
    const double uu = T.uu, vv = T.vv, D = T.D;
    if (!std::isfinite(D) || D == 0.0 || !std::isfinite(uu) || !std::isfinite(vv) || !(uu > 0) || !(vv > 0)) return false;
    const double c = std::fabs(D) / (uu * vv);
    const double L = std::sqrt(std::max(uu, vv));
    if (!std::isfinite(c) || !std::isfinite(L) || c <= 0) return false;
    const double K = 36.0 / c + 18.0 / (c * std::sqrt(c)) + 2.0 / std::sqrt(c);
    const double ke = K * kEps;
    if (!(ke <= kMaxDelta)) return false;
    const double pad = 4.0 * 2.0 * ke * L / (1.0 - ke);
    // The displacement is in the plane (the off-plane part is the per-ray pad's): along axis k a
    // disc of radius pad in the plane reaches pad * sqrt(1 - n_k^2). The normal is the double cross
    // product of the exact float edges (error ~1e-16 / sin(angle) <= ~1e-14 here); the 1e-12 under
    // the root keeps every axis >= 1e-6 of the pad, far above that.
    double e1[3], e2[3], nd[3];
    for (int k = 0; k < 3; ++k) {
        e1[k] = double(v1[k]) - double(v0[k]);
        e2[k] = double(v2[k]) - double(v0[k]);
    }
    nd[0] = e1[1] * e2[2] - e1[2] * e2[1];
    nd[1] = e1[2] * e2[0] - e1[0] * e2[2];
    nd[2] = e1[0] * e2[1] - e1[1] * e2[0];
    const double n2 = nd[0] * nd[0] + nd[1] * nd[1] + nd[2] * nd[2];
    for (int k = 0; k < 3; ++k) {
        const double along = !RT_BVH_INPLANE_PAD ? 1.0 : n2 > 0 ? std::min(1.0, std::sqrt(std::max(0.0, 1.0 - nd[k] * nd[k] / n2) + 1e-12)) : 1.0;
        const double pk = pad * along + 1e-7 * L;
        const double mn = std::min({double(v0[k]), double(v1[k]), double(v2[k])});
        const double mx = std::max({double(v0[k]), double(v1[k]), double(v2[k])});
        lo[k] = down(mn - pk);
        hi[k] = up(mx + pk);
    }
    return true;
}

int build_bvh(const HostScene &s, const std::vector<TriRec> &recs, HostBvh &out) {
    out = HostBvh();
    const size_t nt = recs.size();
    std::vector<BuildPrim> prims;
    Builder b(prims);
    int threads = static_cast<int>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
    if (const char *e = std::getenv("RTAMD_BVH_THREADS")) threads = std::max(1, std::atoi(e));   // diagnostics / tests
    double m1 = 0;
    for (size_t i = 0; i < s.verts.size() / 3; ++i)
        m1 = std::max(m1, std::fabs(double(s.verts[3 * i])) + std::fabs(double(s.verts[3 * i + 1])) + std::fabs(double(s.verts[3 * i + 2])));
    out.scene_m1 = static_cast<float>(m1 * (1 + 1e-6));
    // acceptance boxes in parallel, then the lists in triangle order
    std::vector<BuildPrim> all(nt);
    std::vector<uint8_t> kind(nt);   // 0 tree, 1 always list, 2 never accepted
    b.split_scan(0, static_cast<int>(nt), nt >= 65536 ? threads : 1, [&](int a, int e, int) {
        for (int i = a; i < e; ++i) {
            const float *v0 = &s.verts[3 * s.tris[3 * i]];
            const float *v1 = &s.verts[3 * s.tris[3 * i + 1]];
            const float *v2 = &s.verts[3 * s.tris[3 * i + 2]];
            BuildPrim &p = all[i];
            bool never = false;
            if (!acceptance_box(recs[i], v0, v1, v2, p.box.lo, p.box.hi, &never)) { kind[i] = 1; continue; }
            if (never) { kind[i] = 2; continue; }
            kind[i] = 0;
            for (int k = 0; k < 3; ++k) p.centroid[k] = 0.5f * (p.box.lo[k] + p.box.hi[k]);
            p.tri = static_cast<uint32_t>(i);
        }
    });
    prims.reserve(nt);
    for (size_t i = 0; i < nt; ++i) {
        if (kind[i] == 0) prims.push_back(all[i]);
        else if (kind[i] == 1) out.always.push_back(static_cast<uint32_t>(i));
        else out.n_never++;
    }
    std::vector<BuildPrim>().swap(all);
    const int np = static_cast<int>(b.prims.size());
    if (np == 0) {
        BvhNode root{};
        for (int k = 0; k < 3; ++k) { root.lo0[k] = root.lo1[k] = FLT_MAX; root.hi0[k] = root.hi1[k] = -FLT_MAX; }
        root.c0 = root.c1 = kBvhEmpty;
        out.nodes.push_back(root);
        out.depth = 1;
        out.nodes4.emplace_back();
        make_node4(nullptr, nullptr, 0, out.nodes4[0]);
        out.nodes4f.push_back(make_node4f(nullptr, nullptr, 0));
        out.depth4 = 1;
        return RT_OK;
    }
    if (np > 65536 && threads > 1) b.build_parallel(np, threads);
    else b.build(0, np, 0);
    out.depth = b.max_depth + 1;
    // leaf order
    out.leaf_tris.resize(np);
    for (int i = 0; i < np; ++i) out.leaf_tris[i] = b.prims[i].tri;
    // flatten: GPU node = an inner build node, holding both children's boxes
    std::vector<int> gpu_id(b.nodes.size(), -1);
    std::vector<int> order;
    order.reserve(b.nodes.size());
    // DFS order (left child right after parent) for locality
    std::vector<int> st{0};
    while (!st.empty()) {
        const int n = st.back();
        st.pop_back();
        if (b.nodes[n].left < 0) continue;   // leaves are not GPU nodes
        gpu_id[n] = static_cast<int>(order.size());
        order.push_back(n);
        st.push_back(b.nodes[n].right);
        st.push_back(b.nodes[n].left);
    }
    auto ref_of = [&](int n) -> int32_t { return b.nodes[n].left >= 0 ? gpu_id[n] : leaf_ref(b.nodes[n]); };
    if (np >= (1 << kBvhCountShift)) return RT_E_ARG;   // leaf first-index field overflow
    for (const BuildNode &bn : b.nodes)
        if (bn.left < 0 && static_cast<uint32_t>(bn.count) > kBvhCountMask) return RT_E_ARG;   // leaf too large
    // four-wide tree
    if (b.nodes[0].left < 0) {
        const int32_t r = leaf_ref(b.nodes[0]);
        out.nodes4.emplace_back();
        if (!make_node4(&b.nodes[0].box, &r, 1, out.nodes4[0])) return RT_E_ARG;
        out.nodes4f.push_back(make_node4f(&b.nodes[0].box, &r, 1));
        out.depth4 = 1;
    } else {
        Collapser c{b, out.nodes4, out.nodes4f};
        c.run(0, 1);
        if (!c.ok) return RT_E_ARG;   // a box no 8-bit grid can bound (coordinates near FLT_MAX)
        out.depth4 = c.depth;
        top_levels_first(out.nodes4, out.nodes4f, kTopLevels4);
    }
    if (b.nodes[0].left < 0) {   // the whole tree is one leaf: wrap it in a root with an empty sibling
        BvhNode root{};
        for (int k = 0; k < 3; ++k) {
            root.lo0[k] = b.nodes[0].box.lo[k]; root.hi0[k] = b.nodes[0].box.hi[k];
            root.lo1[k] = FLT_MAX; root.hi1[k] = -FLT_MAX;
        }
        root.c0 = ref_of(0);
        root.c1 = kBvhEmpty;
        out.nodes.push_back(root);
        out.depth = std::max(out.depth, 2);
        return RT_OK;
    }
    out.nodes.resize(order.size());
    for (size_t i = 0; i < order.size(); ++i) {
        const BuildNode &bn = b.nodes[order[i]];
        BvhNode &g = out.nodes[i];
        const BuildNode &L = b.nodes[bn.left], &R = b.nodes[bn.right];
        for (int k = 0; k < 3; ++k) { g.lo0[k] = L.box.lo[k]; g.hi0[k] = L.box.hi[k]; g.lo1[k] = R.box.lo[k]; g.hi1[k] = R.box.hi[k]; }
        g.c0 = ref_of(bn.left);
        g.c1 = ref_of(bn.right);
    }
    return RT_OK;
}

namespace {
// The float four-wide nodes (what the kernels read): the same topology as the quantised ones, and
// every child box contains everything below it (its child boxes, its leaf triangles' padded
// acceptance boxes); empty slots are inverted boxes.
int validate_bvh4f(const HostScene &s, const std::vector<TriRec> &recs, const HostBvh &h, std::string &err) {
    if (h.nodes4f.size() != h.nodes4.size()) { err = "4-wide float: node count differs"; return RT_E_PARSE; }
    struct Item { int32_t ref; float lo[3], hi[3]; };
    std::vector<Item> st{Item{0, {-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}}};
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        if (it.ref == kBvhEmpty) continue;
        if (static_cast<uint32_t>(it.ref) & kBvhLeafBit) {
            const uint32_t u = static_cast<uint32_t>(it.ref);
            const uint32_t cnt = (u >> kBvhCountShift) & kBvhCountMask, first = u & ((1u << kBvhCountShift) - 1);
            for (uint32_t i = first; i < first + cnt; ++i) {
                const uint32_t t = h.leaf_tris[i];
                float lo[3], hi[3];
                bool never;
                acceptance_box(recs[t], &s.verts[3 * s.tris[3 * t]], &s.verts[3 * s.tris[3 * t + 1]],
                               &s.verts[3 * s.tris[3 * t + 2]], lo, hi, &never);
                for (int k = 0; k < 3; ++k)
                    if (lo[k] < it.lo[k] || hi[k] > it.hi[k]) { err = "4-wide float: triangle box outside its leaf box"; return RT_E_PARSE; }
            }
            continue;
        }
        if (it.ref < 0 || static_cast<size_t>(it.ref) >= h.nodes4f.size()) { err = "4-wide float: bad node ref"; return RT_E_PARSE; }
        const Bvh4F &g = h.nodes4f[it.ref];
        const Bvh4Node &q = h.nodes4[it.ref];
        for (int c = 0; c < 4; ++c) {
            if (g.child[c] != q.child[c]) { err = "4-wide float: child refs differ from the quantised node"; return RT_E_PARSE; }
            Item ch{g.child[c], {}, {}};
            for (int k = 0; k < 3; ++k) {
                ch.lo[k] = g.lo[k][c];
                ch.hi[k] = g.hi[k][c];
                if (c >= q.n_children) {
                    if (!(ch.lo[k] == INFINITY && ch.hi[k] == -INFINITY)) { err = "4-wide float: empty slot not inverted"; return RT_E_PARSE; }
                } else if (ch.lo[k] < it.lo[k] || ch.hi[k] > it.hi[k]) {
                    err = "4-wide float: child box outside its parent's";
                    return RT_E_PARSE;
                }
            }
            if (c < q.n_children) st.push_back(ch);
        }
    }
    return RT_OK;
}

// The four-wide tree: decoded child boxes contain everything below them (nested boxes and padded
// triangle boxes), every tree triangle in exactly one leaf, every node reached once, the stack
// bound 3 * depth4 holds.
int validate_bvh4(const HostScene &s, const std::vector<TriRec> &recs, const HostBvh &h, std::string &err) {
    if (h.nodes4.empty()) { err = "no four-wide tree"; return RT_E_PARSE; }
    std::vector<int> seen(recs.size(), 0);
    std::vector<char> is_always(recs.size(), 0);
    for (uint32_t t : h.always) is_always[t] = 1;
    std::vector<int> node_seen(h.nodes4.size(), 0);
    struct Item { int32_t ref; float lo[3], hi[3]; int depth; };
    std::vector<Item> st{Item{0, {-FLT_MAX, -FLT_MAX, -FLT_MAX}, {FLT_MAX, FLT_MAX, FLT_MAX}, 0}};
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        if (it.ref == kBvhEmpty) continue;
        if (static_cast<uint32_t>(it.ref) & kBvhLeafBit) {
            const uint32_t u = static_cast<uint32_t>(it.ref);
            const uint32_t cnt = (u >> kBvhCountShift) & kBvhCountMask, first = u & ((1u << kBvhCountShift) - 1);
            for (uint32_t i = first; i < first + cnt; ++i) {
                const uint32_t t = h.leaf_tris[i];
                seen[t]++;
                float lo[3], hi[3];
                bool never;
                acceptance_box(recs[t], &s.verts[3 * s.tris[3 * t]], &s.verts[3 * s.tris[3 * t + 1]],
                               &s.verts[3 * s.tris[3 * t + 2]], lo, hi, &never);
                for (int k = 0; k < 3; ++k)
                    if (lo[k] < it.lo[k] || hi[k] > it.hi[k]) { err = "4-wide: triangle box outside its leaf box"; return RT_E_PARSE; }
            }
            continue;
        }
        if (it.ref < 0 || static_cast<size_t>(it.ref) >= h.nodes4.size()) { err = "4-wide: bad node ref"; return RT_E_PARSE; }
        if (node_seen[it.ref]++) { err = "4-wide: node reached twice"; return RT_E_PARSE; }
        if (it.depth + 1 > h.depth4) { err = "4-wide: depth bound exceeded"; return RT_E_PARSE; }
        const Bvh4Node &g = h.nodes4[it.ref];
        for (int c = 0; c < 4; ++c) {
            Item ch{g.child[c], {}, {}, it.depth + 1};
            if (c >= g.n_children) {
                if (g.child[c] != kBvhEmpty) { err = "4-wide: child past n_children"; return RT_E_PARSE; }
                continue;
            }
            for (int k = 0; k < 3; ++k) {
                ch.lo[k] = bvh4_decode(g.origin[k], g.ex[k], (g.qlo[k] >> (8 * c)) & 0xFF);
                ch.hi[k] = bvh4_decode(g.origin[k], g.ex[k], (g.qhi[k] >> (8 * c)) & 0xFF);
                if (ch.lo[k] < it.lo[k] || ch.hi[k] > it.hi[k]) {
                    // a quantised child may stick out of its quantised parent; what matters is that
                    // it contains its own content, checked below it. Clip for the nesting check.
                    ch.lo[k] = std::max(ch.lo[k], it.lo[k]);
                    ch.hi[k] = std::min(ch.hi[k], it.hi[k]);
                }
            }
            st.push_back(ch);
        }
    }
    for (size_t t = 0; t < recs.size(); ++t) {
        const TriRec &T = recs[t];
        const bool is_never = (T.n[0] == 0 && T.n[1] == 0 && T.n[2] == 0);
        if (seen[t] != ((is_never || is_always[t]) ? 0 : 1)) { err = "4-wide: triangle not covered exactly once"; return RT_E_PARSE; }
    }
    for (int v : node_seen)
        if (!v) { err = "4-wide: unreachable node"; return RT_E_PARSE; }
    return RT_OK;
}
}  // namespace

// Structural check used by tests: every tree triangle in exactly one leaf, every leaf's padded
// triangle boxes inside its parent's stored child box, every node reachable, depth bound kept.
int validate_bvh(const HostScene &s, const std::vector<TriRec> &recs, const HostBvh &h, std::string &err) {
    const size_t nt = recs.size();
    std::vector<int> seen(nt, 0);
    for (uint32_t t : h.always) seen[t]++;
    struct Item { int32_t ref; float lo[3], hi[3]; int depth; };
    std::vector<Item> st;
    const BvhNode &root = h.nodes[0];
    Item a{root.c0, {root.lo0[0], root.lo0[1], root.lo0[2]}, {root.hi0[0], root.hi0[1], root.hi0[2]}, 1};
    Item b{root.c1, {root.lo1[0], root.lo1[1], root.lo1[2]}, {root.hi1[0], root.hi1[1], root.hi1[2]}, 1};
    st.push_back(a);
    st.push_back(b);
    size_t inner_seen = 1;
    int max_stack = 0;
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        if (it.ref == kBvhEmpty) continue;
        if (it.depth > kMaxBvhDepth) { err = "depth bound exceeded"; return RT_E_PARSE; }
        if (static_cast<uint32_t>(it.ref) & kBvhLeafBit) {
            const uint32_t u = static_cast<uint32_t>(it.ref);
            const uint32_t cnt = (u >> kBvhCountShift) & kBvhCountMask, first = u & ((1u << kBvhCountShift) - 1);
            for (uint32_t i = first; i < first + cnt; ++i) {
                const uint32_t t = h.leaf_tris[i];
                seen[t]++;
                float lo[3], hi[3];
                bool never;
                acceptance_box(recs[t], &s.verts[3 * s.tris[3 * t]], &s.verts[3 * s.tris[3 * t + 1]],
                               &s.verts[3 * s.tris[3 * t + 2]], lo, hi, &never);
                for (int k = 0; k < 3; ++k)
                    if (lo[k] < it.lo[k] || hi[k] > it.hi[k]) { err = "triangle box outside its leaf box"; return RT_E_PARSE; }
            }
            continue;
        }
        const BvhNode &n = h.nodes[it.ref];
        inner_seen++;
        for (int k = 0; k < 3; ++k) {
            if (n.lo0[k] < it.lo[k] || n.hi0[k] > it.hi[k] || n.lo1[k] < it.lo[k] || n.hi1[k] > it.hi[k]) {
                err = "child box outside parent box"; return RT_E_PARSE;
            }
        }
        st.push_back(Item{n.c0, {n.lo0[0], n.lo0[1], n.lo0[2]}, {n.hi0[0], n.hi0[1], n.hi0[2]}, it.depth + 1});
        st.push_back(Item{n.c1, {n.lo1[0], n.lo1[1], n.lo1[2]}, {n.hi1[0], n.hi1[1], n.hi1[2]}, it.depth + 1});
        max_stack = std::max(max_stack, static_cast<int>(st.size()));
    }
    size_t never = 0;
    for (size_t t = 0; t < nt; ++t) {
        const TriRec &T = recs[t];
        const bool is_never = (T.n[0] == 0 && T.n[1] == 0 && T.n[2] == 0);
        if (is_never) { never++; if (seen[t]) { err = "degenerate triangle in tree"; return RT_E_PARSE; } continue; }
        if (seen[t] != 1) { err = "triangle not covered exactly once"; return RT_E_PARSE; }
    }
    if (inner_seen != h.nodes.size()) { err = "unreachable nodes"; return RT_E_PARSE; }
    if (never != h.n_never) { err = "degenerate count mismatch"; return RT_E_PARSE; }
    const int rc = validate_bvh4(s, recs, h, err);
    return rc ? rc : validate_bvh4f(s, recs, h, err);
}

uint64_t bvh_digest(const HostBvh &h) {
    uint64_t x = 1469598103934665603ull;   // FNV-1a over the arrays the device receives
    auto mix = [&](const void *p, size_t n) {
        const unsigned char *c = static_cast<const unsigned char *>(p);
        for (size_t i = 0; i < n; ++i) { x ^= c[i]; x *= 1099511628211ull; }
    };
    mix(h.nodes.data(), h.nodes.size() * sizeof(BvhNode));
    mix(h.nodes4.data(), h.nodes4.size() * sizeof(Bvh4Node));
    mix(h.nodes4f.data(), h.nodes4f.size() * sizeof(Bvh4F));
    mix(h.leaf_tris.data(), h.leaf_tris.size() * sizeof(uint32_t));
    mix(h.always.data(), h.always.size() * sizeof(uint32_t));
    return x;
}

}  // namespace rt
