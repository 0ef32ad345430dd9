// rt_kernels.hip — gfx950 kernels of the render path.
//
// Wavefront structure (one launch per stage, queues compacted with one atomic per block chunk):
//   gen_primary  -> main queue Q0 (one query per sub-sample; main.cpp:369-388)
//   per chain step k = 0..max_lvl:
//     closest_hit(Q_k)            intersectMesh, raytracing.cpp:161-192   <- the hot kernel
//     [shadow_gen +] shadow_hit   isShadow, raytracing.cpp:241-261 (any-hit when no material is
//                                 transparent, closest-hit + material test otherwise)
//     shade(Q_k) -> Q_{k+1}       shade/diffuse/specular/reflection/refraction, :194-368
//   frame        fold the chain back to front (trace() returns are consumed innermost first),
//                AA average, RGBValue clamp, (unsigned char)(v*255) (main.cpp:24-42,389-393,117)
//
// Numerics: compiled with -ffp-contract=off; HIP's f32 '/' and sqrtf are correctly rounded on
// gfx950 and f32 denormals are on, as on x86 SSE. Every expression keeps the reference's
// operand order (Vec3D.h dot = (a0*b0 + a1*b1) + a2*b2). acosf and powf(x,2) of refraction()
// are replaced by bit-exact equivalents of glibc (threshold / tie table, see below).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <type_traits>

#include "rt_kernels.h"
#include "spec_pow.h"

namespace rt {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ int as_int(float f) { return __float_as_int(f); }
__device__ __forceinline__ float as_float(int i) { return __int_as_float(i); }

struct V3 { float x, y, z; };
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 scale(V3 a, float f) { return mk(a.x * f, a.y * f, a.z * f); }   // Vec3D.h:12-18
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }  // Vec3D.h:20-22
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } // Vec3D.h:192-194
__device__ __forceinline__ void normalize(V3 &a) {                                                 // Vec3D.h:142-151
    float len = sqrtf(dot(a, a));
    if (len == 0.0f) return;
    float rez = 1.0f / len;
    a.x *= rez; a.y *= rez; a.z *= rez;
}
__device__ __forceinline__ float max_std(float a, float b) { return (a < b) ? b : a; }            // std::max
__device__ __forceinline__ V3 ld3(const float4 &v) { return mk(v.x, v.y, v.z); }

// Light l (MyLightPositions[l], raytracing.h:9): the first RT_MAX_LIGHTS ride in the kernel arguments,
// the rest (an unbounded list, as the reference's std::vector) come from the device copy light_ext.
// kExt false: the chain launch, which runs only with <= RT_MAX_LIGHTS lights (kChainMaxLights), reads
// the kernel arguments alone (r04: the per-lane l < RT_MAX_LIGHTS select cost C5 1.7%, C4 0.8%).
template <bool kExt = true>
__device__ __forceinline__ V3 light_at(const float (&inl)[RT_MAX_LIGHTS][3], const float *ext, int l) {
    if (!kExt || l < RT_MAX_LIGHTS) return mk(inl[l][0], inl[l][1], inl[l][2]);
    return mk(ext[3 * l], ext[3 * l + 1], ext[3 * l + 2]);
}
// (The chain launch serves up to kChainMaxLights = RT_MAX_LIGHTS lights, the ones in its arguments;
// with more, up to RT_LIGHTS_LIMIT, the render runs the per-step kernels, whose verdicts are bytes
// per (query, light) in the workspace: rt_capi.cpp run_chain.)

// acosf(check) in (0, 2] for check < 0 (raytracing.cpp:296-298): glibc's acosf crosses 2.0
// exactly once on [-1, 0), at -0x1.aa226cp-2 (acosf of it is 2.0f); verified exhaustively by
// tests/test_numerics.py::test_acos_threshold against this platform's libm.
constexpr float kAcosLe2Threshold = -0x1.aa226cp-2f;

// glibc powf(x, 2) (raytracing.cpp:302,316): x*x, moved one ulp where glibc differs (table from
// gen_powf2_ties.c; bit 31 = down). |x| >= 2 is outside the table and returns x*x.
__device__ float glibc_powf2(float x, const uint32_t *ties, int n) {
    float r = x * x;
    uint32_t ax = static_cast<uint32_t>(as_int(x)) & 0x7fffffffu;
    if (ax >= 0x40000000u || n <= 0) return r;
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if ((ties[mid] & 0x7fffffffu) < ax) lo = mid + 1; else hi = mid;
    }
    if (lo < n && (ties[lo] & 0x7fffffffu) == ax) {
        uint32_t rb = static_cast<uint32_t>(as_int(r));
        rb = (ties[lo] >> 31) ? rb - 1u : rb + 1u;
        r = as_float(static_cast<int>(rb));
    }
    return r;
}

// powf(SpecularTerm, Ns) (raytracing.cpp:226): spec_pow.h, double log2/exp2 rounded once; agrees
// with glibc powf except where glibc itself is not correctly rounded (colour-only, <= 1 LSB).
__device__ __forceinline__ float spec_powf(float x, float y) { return spec_pow(x, y); }

// popcount(m & lanes below this lane): the lane's rank among the lanes of m below it (v_mbcnt_lo/hi:
// two instructions, no 64-bit lane mask to make or keep live)
__device__ __forceinline__ int rank_below(unsigned long long m) {
    return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
}

// Block-wide reservation in an output queue for kPer coalesced rounds of items: round k covers
// items base + k*BLOCK + threadIdx.x, so reads and writes stay coalesced and the output keeps
// input order. One atomicAdd per block chunk: a single counter word takes only ~88 atomics/us
// (MI355X_MICROARCH.md, dequeue row), so queues are never appended per wave. Returns, for each
// round, this thread's output slot (or -1). Every thread of the block must call it (barriers).
template <int BLOCK, int PER>
__device__ __forceinline__ void block_reserve_rounds(const bool (&valid)[PER], int32_t *counter, int (&pos)[PER]) {
    constexpr int NW = BLOCK / 64;
    __shared__ int s_c[PER * NW + 1];
    const int lane = __lane_id(), wid = threadIdx.x >> 6;
    unsigned long long m[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        m[k] = __ballot(valid[k]);
        if (lane == 0) s_c[k * NW + wid] = __popcll(m[k]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int i = 0; i < PER * NW; ++i) { const int c = s_c[i]; s_c[i] = acc; acc += c; }
        s_c[PER * NW] = acc ? atomicAdd(counter, acc) : 0;
    }
    __syncthreads();
    const int base = s_c[PER * NW];
#pragma unroll
    for (int k = 0; k < PER; ++k)
        pos[k] = valid[k] ? base + s_c[k * NW + wid] + rank_below(m[k]) : -1;
    __syncthreads();
}

constexpr int kPer = 8;           // items per thread in the chunked queue kernels
constexpr int kMaxGrid = 2048;    // resident-size grids for grid-stride kernels (256 CUs x 8)

// ---------------------------------------------------------------------------------------------
// Closest hit: rayIntersectTriangle (raytracing.cpp:99-154) over every triangle in index order,
// strict '<' on the distance (:183) so ties keep the lowest index. One lane = one query; the
// triangle loop is wave-uniform, so each 64-byte record is fetched with scalar loads and the VALU
// reads it from SGPRs (no VGPR/LDS copy).
// ---------------------------------------------------------------------------------------------
// Forces every SGPR of a scalar-loaded record to be resident (s_waitcnt) at this point, and
// keeps later loads below it, so the next record's s_load overlaps this record's arithmetic.
__device__ __forceinline__ void sgpr_fence(const TriRec &T) {
    asm volatile("" ::"s"(T.t0[0]), "s"(T.t0[1]), "s"(T.t0[2]), "s"(T.uu), "s"(T.u[0]), "s"(T.u[1]), "s"(T.u[2]),
                 "s"(T.uv), "s"(T.v[0]), "s"(T.v[1]), "s"(T.v[2]), "s"(T.vv), "s"(T.n[0]), "s"(T.n[1]), "s"(T.n[2]),
                 "s"(T.D)
                 : "memory");
}

// One rayIntersectTriangle + intersectMesh update (raytracing.cpp:106-154, :180-187). In index
// order the update is the reference's strict '<' (:183); out of order (kLex, the BVH) it is the
// equivalent lexicographic (distance, index) minimum.
// kSignFirst: reject r = a / b < 0 from the signs of a and b before the division (exact: with
// |a| > 2^-100 |b| the quotient cannot round to -0, the one negative-signed value :125 lets through),
// so a wave whose lanes all face away from the plane skips the correctly rounded division.
// kStages (the brute-force roofline's counting pass only): stg[k] += 1 for each stage the test reaches
// (kTestStageFlops: 0 the plane terms, 1 the division, 2 the in-plane coordinates and s, 3 t, 4 the
// distance), so the work a launch performed is counted, not a union path every test is assumed to take.
#ifndef RT_TRI_RCP
#define RT_TRI_RCP 0   // 1: measured no faster (profiles/r05zi_ab_tri_rcp.txt)
#endif
// The s and t divisions by D (:144, :148) from the record's reciprocal slot (RT_TRI_RCP, r05): the
// uploaded records carry rD = RN(1/D) in D's place (NaN where |D| is outside [2^-30, 2^30] or D is
// not normal; tri_rcp_slot) and D is recomputed from uu, uv, vv as the loader computes it (:140, the
// same bits). With q = RN(n rD) in [2^-30, 2^30] every intermediate is normal, the residual
// fma(-q, D, n) is exact and q + r rD rounds to the correctly rounded n / D (Markstein's correction;
// tools/markstein_gpu.hip checks all 2^46 significand pairs); elsewhere (rD NaN, n near 0 or huge)
// the lane divides. Five instructions instead of ~11 for both divisions of a test that reaches them.
__device__ __forceinline__ float div_by_rec(float n, float D, float rD) {
    const float q = n * rD;
    if (__builtin_expect(fabsf(q) >= 0x1p-30f && fabsf(q) <= 0x1p30f, 1)) return fmaf(fmaf(-q, D, n), rD, q);
    return n / D;
}

constexpr int kTestStages = 5;
constexpr int kTestStageFlops[kTestStages] = {14, 1, 23, 5, 9};
template <bool kAnyHit, bool kLex = false, bool kSignFirst = false, bool kStages = false>
__device__ __forceinline__ void test_triangle(const TriRec &T, int t, V3 o, V3 dir, float &best, int &bidx, V3 &bI,
                                              bool &done, unsigned *stg = nullptr) {
    if (kAnyHit && done) return;
    if (kStages) ++stg[0];
    const V3 w0 = mk(o.x - T.t0[0], o.y - T.t0[1], o.z - T.t0[2]);
    const float b = T.n[0] * dir.x + T.n[1] * dir.y + T.n[2] * dir.z;          // :113
    const float a = -(T.n[0] * w0.x + T.n[1] * w0.y + T.n[2] * w0.z);          // :114
    if (fabsf(b) < 0.00001f) return;                                            // :115
    if (kSignFirst && (a < 0.0f) != (b < 0.0f) && fabsf(a) > fabsf(b) * 0x1p-100f) return;   // r < 0 (:125)
    if (kStages) ++stg[1];
    const float r = a / b;                                                      // :124
    if (r < 0) return;                                                          // :125
    if (kStages) ++stg[2];
    const V3 I = mk(o.x + dir.x * r, o.y + dir.y * r, o.z + dir.z * r);         // :130
    const V3 w = mk(I.x - T.t0[0], I.y - T.t0[1], I.z - T.t0[2]);               // :137
    const float wu = w.x * T.u[0] + w.y * T.u[1] + w.z * T.u[2];                 // :138
    const float wv = w.x * T.v[0] + w.y * T.v[1] + w.z * T.v[2];                 // :139
#if RT_TRI_RCP
    const float D = T.uv * T.uv - T.uu * T.vv;                                  // :140 (T.D holds rD)
    const float s = div_by_rec(T.uv * wv - T.vv * wu, D, T.D);                  // :144
#else
    const float s = (T.uv * wv - T.vv * wu) / T.D;                              // :144
#endif
    if (s < 0 || s > 1) return;                                                 // :145
    if (kStages) ++stg[3];
#if RT_TRI_RCP
    const float tt = div_by_rec(T.uv * wu - T.uu * wv, D, T.D);                 // :148
#else
    const float tt = (T.uv * wu - T.uu * wv) / T.D;                             // :148
#endif
    if (tt < 0 || (s + tt) > 1) return;                                         // :149
    if (kStages) ++stg[4];
    const V3 e = sub(o, I);                                                     // distance, Vec3D.h:199-202
    const float dist = sqrtf(dot(e, e));
    if (dist < best || (kLex && dist == best && t < bidx)) {                  // :183
        best = dist; bidx = t; bI = I;
        if (kAnyHit) done = true;
    }
}

// A leaf record of the BVH: the 64-B TriRec in leaf order. (A 48-B {T0, u, v, n} record with
// uu/uv/vv/D recomputed per test cut the leaf array by a quarter and measured no faster: the walk
// is not bound by bytes)
__device__ __forceinline__ TriRec leaf_rec(const DevScene &sc, int i) { return sc.leaf_recs[i]; }

// Scalar-load pipeline: records A and B alternate; each is fenced (s_waitcnt) before the next
// record's s_load is issued, so one load is always in flight behind the arithmetic.
template <bool kAnyHit>
__device__ __forceinline__ void closest_hit_loop(const TriRec *__restrict__ tris, int nt, V3 o, V3 dir, bool active,
                                                 int &bidx, V3 &bI) {
    float best = FLT_MAX;
    bool done = !active;
    if (nt <= 0) return;
    TriRec A = tris[0];
    int t = 0;
    for (; t + 1 < nt; t += 2) {
        if (kAnyHit && (t & 15) == 0 && __all(done)) return;
        sgpr_fence(A);
        const TriRec B = tris[t + 1];
        test_triangle<kAnyHit>(A, t, o, dir, best, bidx, bI, done);
        sgpr_fence(B);
        A = tris[min(t + 2, nt - 1)];
        test_triangle<kAnyHit>(B, t + 1, o, dir, best, bidx, bI, done);
    }
    if (t < nt) {
        sgpr_fence(A);
        test_triangle<kAnyHit>(A, t, o, dir, best, bidx, bI, done);
    }
}

// ---------------------------------------------------------------------------------------------
// BVH traversal (bvh.cpp states the exactness argument). One lane = one query; per-lane stack of
// child refs in LDS ([depth][lane], conflict-free); nearer child first; a child is skipped when
// its padded box misses the ray or (closest-hit) when even its entry point is farther than the
// current best. Leaves run test_triangle on the leaf-ordered records with the original index.
// ---------------------------------------------------------------------------------------------
#ifndef RT_BVH_BLOCK
#define RT_BVH_BLOCK 256   // threads per block of the BVH and chain kernels (r02h: 256 vs 128 measured C4 0.44 vs
                           // 0.48 ms, C3 0.250 vs 0.259, C5 8.75 vs 8.91; C2 0.178 vs 0.171; 64: C4 0.61 ms)
#endif
constexpr int kBvhBlock = RT_BVH_BLOCK;
// Any-hit walks visit the wanted children unsorted (measured 8% faster shadows than sorted).
// The per-step BVH kernels are built for 7 waves per SIMD (<= 72 VGPRs, no spills): measured a few
// percent faster than the unconstrained ~80 VGPRs (6 waves); 8 waves spills and is not.

struct RayBox { V3 o, inv; float pad, dlen; };

// Per-lane traversal stack: the first `cap` entries in LDS ([entry][lane], conflict-free), deeper
// entries in a global overflow area ([entry - cap][global lane], coalesced). Trees deeper than
// the LDS part are rare, so a small LDS part keeps occupancy high at no cost in the common case.
struct LaneStack {
    int32_t *lds;       // [entry][width lanes]
    int32_t *ovf;
    int cap, stride, gl, width;
    __device__ __forceinline__ void push(int &sp, int32_t v) const {
        if (sp < cap) lds[sp * width + static_cast<int>(threadIdx.x)] = v;
        else ovf[static_cast<size_t>(sp - cap) * stride + gl] = v;
        ++sp;
    }
    __device__ __forceinline__ int32_t at(int k) const {   // entry k of this lane's stack
        int32_t v = lds[min(k, cap - 1) * width + static_cast<int>(threadIdx.x)];
        if (k >= cap) v = ovf[static_cast<size_t>(k - cap) * stride + gl];
        return v;
    }
    __device__ __forceinline__ int32_t pop(int &sp) const {
        --sp;
        // the LDS read is unconditional so the two reads stay a ds_read and a global load (a
        // select between the two pointers would become a slower flat load)
        int32_t v = lds[min(sp, cap - 1) * width + static_cast<int>(threadIdx.x)];
        if (sp >= cap) v = ovf[static_cast<size_t>(sp - cap) * stride + gl];
        return v;
    }
    // The entry below sp if sp > base, else none (sp unchanged). When every active lane's entry is
    // in LDS (a wave-uniform test) it is one ds_read; else pop's two reads, which the compiler
    // merges into a flat load through a pointer select (r04: the walk's postponement and leaf-loop
    // pops used that flat form every time).
    __device__ __forceinline__ int32_t pop_or(int &sp, int base, int32_t none) const {
        if (__all(sp <= cap)) {
            const int32_t v = lds[max(sp - 1, 0) * width + static_cast<int>(threadIdx.x)];
            const int32_t r = sp > base ? v : none;
            sp = max(sp - 1, base);
            return r;
        }
        return sp > base ? pop(sp) : none;
    }
};

// Dynamic LDS of the per-lane BVH kernels: [lds_stack entries][block lanes] of stack.
template <int B = kBvhBlock>
__device__ __forceinline__ LaneStack lane_stack(const DevScene &sc, int32_t *lds) {
    LaneStack st;
    st.lds = lds;
    st.width = B;
    st.ovf = sc.stack_ovf;
    st.cap = sc.lds_stack;
    st.stride = static_cast<int>(gridDim.x) * B;
    st.gl = static_cast<int>(blockIdx.x) * B + static_cast<int>(threadIdx.x);
    return st;
}

// A four-wide node's rows for this ray (Bvh4F): the near and far bound rows of each axis (the
// lower bounds are the near plane when the ray's direction component is positive, the upper bounds
// when it is negative; Ray4::rows holds the byte offsets) and the child refs, as global loads from
// the node array's base plus a 32-bit per-lane offset, so the first row's FMAs start while the
// others are in flight. (An LDS copy of the top levels, read through flat loads with 64-bit row
// addresses, measured 2% slower on C4 and 18% on C5: profiles/r03_ab_float_nodes.txt.)
struct Node4Rows { float4 n[3], f[3]; int4 ref; };
__device__ __forceinline__ Node4Rows load_node4(const Bvh4F *__restrict__ nodes4, int32_t ref, const uint32_t (&rows)[6]) {
    Node4Rows r;
    // global loads from the node array's base (wave-uniform) plus a 32-bit per-lane byte offset
    const char *__restrict__ base = reinterpret_cast<const char *>(nodes4);
    const uint32_t o = static_cast<uint32_t>(ref) * static_cast<uint32_t>(sizeof(Bvh4F));
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        r.n[k] = *reinterpret_cast<const float4 *>(base + (o + rows[k]));
        r.f[k] = *reinterpret_cast<const float4 *>(base + (o + rows[3 + k]));
    }
    r.ref = *reinterpret_cast<const int4 *>(base + (o + static_cast<uint32_t>(offsetof(Bvh4F, child))));
    return r;
}

__device__ __forceinline__ bool box_hit(const RayBox &R, float lx, float ly, float lz, float hx, float hy, float hz,
                                        float &tentry) {
    const float ax = (lx - R.pad - R.o.x) * R.inv.x, bx = (hx + R.pad - R.o.x) * R.inv.x;
    const float ay = (ly - R.pad - R.o.y) * R.inv.y, by = (hy + R.pad - R.o.y) * R.inv.y;
    const float az = (lz - R.pad - R.o.z) * R.inv.z, bz = (hz + R.pad - R.o.z) * R.inv.z;
    const float tmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
    const float tmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    tentry = tmin;
    return tmin <= tmax * 1.00001f;
}

// The always list (ill-conditioned triangles, bvh.cpp): every query tests them. Their records are
// gathered contiguously (always_recs) and streamed like the brute-force loop: wave-uniform,
// two records alternating so one load is in flight behind the arithmetic.
#ifndef RT_LEAF_SIGN
#define RT_LEAF_SIGN 0     // the same in the walks' leaf loops
#endif
#ifndef RT_ALWAYS_SIGN
#define RT_ALWAYS_SIGN 1   // the always-tested list (uniform records, coherent rays) rejects r < 0 by signs first
#endif
template <bool kAnyHit>
__device__ __forceinline__ void test_always(const DevScene &sc, V3 o, V3 dir, float &best, int &bidx, V3 &bI,
                                            bool &done) {
    const int n = sc.n_always;
    if (n <= 0) return;
    const TriRec *__restrict__ recs = sc.always_recs;
    TriRec A = recs[0];
    int i = 0;
    for (; i + 1 < n; i += 2) {
        if (kAnyHit && (i & 15) == 0 && __all(done)) return;
        sgpr_fence(A);
        const TriRec B = recs[i + 1];
        test_triangle<kAnyHit, true, RT_ALWAYS_SIGN>(A, static_cast<int>(sc.always[i]), o, dir, best, bidx, bI, done);
        sgpr_fence(B);
        A = recs[min(i + 2, n - 1)];
        test_triangle<kAnyHit, true, RT_ALWAYS_SIGN>(B, static_cast<int>(sc.always[i + 1]), o, dir, best, bidx, bI, done);
    }
    if (i < n) {
        sgpr_fence(A);
        test_triangle<kAnyHit, true, RT_ALWAYS_SIGN>(A, static_cast<int>(sc.always[i]), o, dir, best, bidx, bI, done);
    }
}

// A leaf's records in leaf order. The original index (ties, result) is read only when a test
// reaches the comparison with the current best.
// (Skipping the divisions when their outcome is decided by signs or approximate quotients was
// measured slower: the extra branches and registers cost more than the divisions they save.)
#ifndef RT_LEAF_PAIRS
#define RT_LEAF_PAIRS 0   // measured neutral on C4 (0.88 vs 0.89 ms), costs VGPRs
#endif
template <bool kAnyHit>
__device__ __forceinline__ void test_leaf(const DevScene &sc, int first, int cnt, V3 o, V3 dir, float &best, int &bidx,
                                          V3 &bI, bool &done) {
    if (RT_LEAF_PAIRS) {
        // Two records per round, both loads in flight before either test (the second load repeats
        // the last record when the count is odd; its test is skipped). The lexicographic minimum
        // does not depend on the order of the tests.
        for (int k = 0; k < cnt; k += 2) {
            const int k1 = min(k + 1, cnt - 1);
            const TriRec A = leaf_rec(sc, first + k);
            const TriRec B = leaf_rec(sc, first + k1);
            test_triangle<kAnyHit, true>(A, static_cast<int>(sc.leaf_idx[first + k]), o, dir, best, bidx, bI, done);
            if (k1 != k) test_triangle<kAnyHit, true>(B, static_cast<int>(sc.leaf_idx[first + k1]), o, dir, best, bidx, bI, done);
        }
        return;
    }
    for (int k = 0; k < cnt; ++k) {
        const TriRec T = leaf_rec(sc, first + k);
        test_triangle<kAnyHit, true>(T, static_cast<int>(sc.leaf_idx[first + k]), o, dir, best, bidx, bI, done);
    }
}

template <bool kAnyHit>
__device__ __forceinline__ void bvh_query(const DevScene &sc, V3 o, V3 dir, bool active, int &bidx, V3 &bI,
                                          const LaneStack &stack, unsigned &tests, unsigned &visits) {
    float best = FLT_MAX;
    bool done = !active;
    test_always<kAnyHit>(sc, o, dir, best, bidx, bI, done);
    if (!active || (kAnyHit && done)) return;
    RayBox R;
    R.o = o;
    R.inv = mk(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
    R.pad = 64.0f * 5.9604645e-08f * (fabsf(o.x) + fabsf(o.y) + fabsf(o.z) + sc.scene_m1);
    R.dlen = sqrtf(dot(dir, dir));
    int sp = 0;
    int32_t ref = 0;
    while (true) {
        if (ref >= 0) {
            ++visits;
            const float4 *np = reinterpret_cast<const float4 *>(sc.nodes + ref);
            const float4 q0 = np[0], q1 = np[1], q2 = np[2], q3 = np[3];
            float t0, t1;
            bool h0 = box_hit(R, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, t0);
            bool h1 = box_hit(R, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, t1);
            if (!kAnyHit) {   // distance cull: no accepted point of the child is nearer than its entry
                h0 = h0 && (t0 * R.dlen - R.pad) * 0.99999f <= best;
                h1 = h1 && (t1 * R.dlen - R.pad) * 0.99999f <= best;
            }
            const int32_t c0 = __float_as_int(q3.x), c1 = __float_as_int(q3.y);
            if (h0 && h1) {
                const bool first0 = t0 <= t1;
                stack.push(sp, first0 ? c1 : c0);
                ref = first0 ? c0 : c1;
            } else if (h0) {
                ref = c0;
            } else if (h1) {
                ref = c1;
            } else {
                if (sp == 0) break;
                ref = stack.pop(sp);
            }
        } else {
            const uint32_t u = static_cast<uint32_t>(ref);
            const int cnt = static_cast<int>((u >> kBvhCountShift) & kBvhCountMask);
            const int first = static_cast<int>(u & ((1u << kBvhCountShift) - 1u));
            test_leaf<kAnyHit>(sc, first, cnt, o, dir, best, bidx, bI, done);
            tests += static_cast<unsigned>(cnt);
            if (kAnyHit && done) break;
            if (sp == 0) break;
            ref = stack.pop(sp);
        }
    }
}

// Four-wide traversal (bvh.cpp, Bvh4F): the same cull and leaf logic as bvh_query; the hit
// children are sorted by entry distance, the nearest is visited next and the others are pushed
// farthest first.
__device__ __forceinline__ void cswap(float &ta, int32_t &ra, float &tb, int32_t &rb) {
    const bool sw = tb < ta;
    const float t = sw ? tb : ta;
    const int32_t r = sw ? rb : ra;
    tb = sw ? ta : tb;
    rb = sw ? ra : rb;
    ta = t;
    ra = r;
}

// ---------------------------------------------------------------------------------------------
// "While-while" four-wide traversal (Aila & Laine 2009's speculative form): a lane that reaches a
// leaf postpones it and keeps visiting nodes until every lane of the wave holds a leaf (or has
// finished), then the wave tests leaves together, one triangle per iteration with the leaf ref as
// the cursor. Only the interleaving of node visits and leaf tests differs from a plain walk, so the
// lexicographic minimum and the any-hit verdict are the same. (Measured against the plain loop:
// C4 frame 0.88 -> 0.81 ms; the cursor another 2%; any speculation slack or a second postponed
// leaf was slower. DESIGN.md §7 records the variants that were measured and removed.)
// ---------------------------------------------------------------------------------------------
constexpr int32_t kDoneRef = kBvhEmpty;   // "no ref": a count-0 leaf is never a wanted child

// Per-ray traversal constants. A child's slab plane is
//   t = fma(b, inv, (-/+pad - o) * inv)
// for the plane's float bound b (Bvh4F), instead of (b -/+ pad - o) * inv: the same value up to a few
// ulps of (|o| + pad) * |inv| and of |t|, inside the pad (64 ulps of |o| + the scene's extent) and the
// 1e-5 relative slack of the te <= tx test.
//
// The six planes of two children are one v_pk_fma_f32 each (r04): a row's float4 is two register
// pairs, and op_sel / op_sel_hi broadcast one half of a per-ray pair to both elements, so the
// per-ray constants live in five pairs with no splat copies. Per element the packed FMA is the
// same IEEE fused multiply-add as v_fma_f32 (same rounding and denormal mode), so every slab
// parameter has the bits of the scalar form.
#ifndef RT_PK_BOX
#define RT_PK_BOX 0   // measured: VALU -5% but C4 +1-2% (profiles/r04_ab_pk_box.txt); kept for the record
#endif
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk_fma_xy(f2 a, f2 s) {          // a * s.x + s.y, both elements
    f2 d;
    asm("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "v"(s));
    return d;
}
__device__ __forceinline__ f2 pk_fma_x_x(f2 a, f2 s, f2 t) {   // a * s.x + t.x
    f2 d;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(s), "v"(t));
    return d;
}
__device__ __forceinline__ f2 pk_fma_x_y(f2 a, f2 s, f2 t) {   // a * s.x + t.y
    f2 d;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "v"(s), "v"(t));
    return d;
}
struct Ray4 {
    f2 ax, ay, az;   // per axis (inv, (+/-pad - o) * inv of the near plane)
    f2 fxy;          // (+/-pad - o) * inv of the far planes x, y
    f2 fzc;          // (far plane z, tcull)
    float inv_dlen;  // an upper bound of 1.00001 / |dir|
    uint32_t rows[6];   // byte offsets in a Bvh4F of the near rows (x, y, z), then the far rows
};

// tcull for the current best: no child whose entry parameter exceeds it can hold a hit at
// distance <= best ((t |dir| - pad)(1 - 1e-5) > best). inv_dlen is a reciprocal rounded up by 1e-4,
// which only raises tcull (visits no fewer nodes than the division form).
__device__ __forceinline__ float cull_param(const Ray4 &R, float best, float pad) {
    return (best * 1.00002f + pad) * R.inv_dlen;
}

#ifndef RT_LIM_ASM
#define RT_LIM_ASM 0   // min(tx (1 + 1e-5), tcull) as v_min_f32 in asm: compiled fminf re-canonicalises tcull each visit
#endif
#ifndef RT_ALWAYS_SORT
#define RT_ALWAYS_SORT 0   // closest-hit: sort every node's keys (no nh count, no one-child branch)
#endif
#ifndef RT_ANY_ORDER
#define RT_ANY_ORDER 0   // any-hit child order: 0 index order, 1 nearest entry first, 2 farthest first
#endif
#ifndef RT_TX_SLACK
#define RT_TX_SLACK 1   // the 1e-5 relative slack of te <= tx (0: A/B measurement only)
#endif
template <bool kAnyHit>
__device__ __forceinline__ float node_lim(float tx, float tcull) {
    const float txs = RT_TX_SLACK ? tx * 1.00001f : tx;
    if (kAnyHit) return txs;
    if (RT_LIM_ASM) {
        float lim;
        asm("v_min_f32 %0, %1, %2" : "=v"(lim) : "v"(txs), "v"(tcull));
        return lim;
    }
    return fminf(txs, tcull);
}

// One node visit: the wanted children by entry distance, the far ones pushed; returns the next ref
// (the nearest wanted child, else the stack top, else kDoneRef). Entries [base, sp) are this walk's.
template <bool kAnyHit>
__device__ __forceinline__ int32_t node4_next(const Ray4 &R, const Node4Rows &nd, const LaneStack &stack, int &sp,
                                              int base = 0) {
    // te <= tx (1 + 1e-5) and, closest-hit, te <= tcull, as one compare against their minimum.
    // te is finite for every non-empty child (bounds and inv are finite and |b inv| < 2^120, so no
    // FMA overflows; an empty slot's +inf/-inf bounds give te = +inf > tx = -inf), so a wanted
    // child's key is below INFINITY, which marks the others
    // (against two compares and an integer min of te: C4 0.418 -> 0.415 ms, C5 6.75 -> 6.71, C3
    // 0.254 -> 0.247; profiles/r03_ab_node_lim.txt)
    const float tcull = R.fzc.y;
    int32_t rc[4] = {nd.ref.x, nd.ref.y, nd.ref.z, nd.ref.w};
    float tc[4];
#if RT_PK_BOX
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // children 2h, 2h + 1
        const f2 nx = h ? f2{nd.n[0].z, nd.n[0].w} : f2{nd.n[0].x, nd.n[0].y};
        const f2 ny = h ? f2{nd.n[1].z, nd.n[1].w} : f2{nd.n[1].x, nd.n[1].y};
        const f2 nz = h ? f2{nd.n[2].z, nd.n[2].w} : f2{nd.n[2].x, nd.n[2].y};
        const f2 fx = h ? f2{nd.f[0].z, nd.f[0].w} : f2{nd.f[0].x, nd.f[0].y};
        const f2 fy = h ? f2{nd.f[1].z, nd.f[1].w} : f2{nd.f[1].x, nd.f[1].y};
        const f2 fz = h ? f2{nd.f[2].z, nd.f[2].w} : f2{nd.f[2].x, nd.f[2].y};
        const f2 a = pk_fma_xy(nx, R.ax), b = pk_fma_xy(ny, R.ay), c = pk_fma_xy(nz, R.az);
        const f2 d = pk_fma_x_x(fx, R.ax, R.fxy), e = pk_fma_x_y(fy, R.ay, R.fxy), f = pk_fma_x_x(fz, R.az, R.fzc);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // max(tnx, tny, tnz, 0) and min(tfx, tfy, tfz) as v_max3/v_min3 on the packed results
            // (compiled fmaxf/fminf would first canonicalise each asm output: no NaN reaches here)
            float te, tx;
            asm("v_max3_f32 %0, %1, %2, %3\n\tv_max_f32 %0, 0, %0" : "=&v"(te) : "v"(j ? a.y : a.x), "v"(j ? b.y : b.x), "v"(j ? c.y : c.x));
            asm("v_min3_f32 %0, %1, %2, %3" : "=v"(tx) : "v"(j ? d.y : d.x), "v"(j ? e.y : e.x), "v"(j ? f.y : f.x));
            tc[2 * h + j] = te <= node_lim<kAnyHit>(tx, tcull) ? te : INFINITY;
        }
    }
#else
    {
        const float nx[4] = {nd.n[0].x, nd.n[0].y, nd.n[0].z, nd.n[0].w}, fx[4] = {nd.f[0].x, nd.f[0].y, nd.f[0].z, nd.f[0].w};
        const float ny[4] = {nd.n[1].x, nd.n[1].y, nd.n[1].z, nd.n[1].w}, fy[4] = {nd.f[1].x, nd.f[1].y, nd.f[1].z, nd.f[1].w};
        const float nz[4] = {nd.n[2].x, nd.n[2].y, nd.n[2].z, nd.n[2].w}, fz[4] = {nd.f[2].x, nd.f[2].y, nd.f[2].z, nd.f[2].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float tnx = fmaf(nx[k], R.ax.x, R.ax.y), tfx = fmaf(fx[k], R.ax.x, R.fxy.x);
            const float tny = fmaf(ny[k], R.ay.x, R.ay.y), tfy = fmaf(fy[k], R.ay.x, R.fxy.y);
            const float tnz = fmaf(nz[k], R.az.x, R.az.y), tfz = fmaf(fz[k], R.az.x, R.fzc.x);
            const float te = fmaxf(fmaxf(fmaxf(tnx, tny), tnz), 0.0f);
            const float tx = fminf(fminf(tfx, tfy), tfz);
            tc[k] = te <= node_lim<kAnyHit>(tx, tcull) ? te : INFINITY;
        }
    }
#endif
    if (!kAnyHit) {
        // Sorted, branch-free pushes: the wanted children after the first go to the stack with
        // unconditional LDS writes when every lane's stack has room (slots past the new top are
        // scratch); pops the same way. Misses are INFINITY and sort last.
        const int lane = static_cast<int>(threadIdx.x);
        if (RT_ALWAYS_SORT) {
            cswap(tc[0], rc[0], tc[1], rc[1]);
            cswap(tc[2], rc[2], tc[3], rc[3]);
            cswap(tc[0], rc[0], tc[2], rc[2]);
            cswap(tc[1], rc[1], tc[3], rc[3]);
            cswap(tc[1], rc[1], tc[2], rc[2]);
            // the wanted children are a prefix of the sorted keys
            const bool w1 = tc[1] != INFINITY, w2 = tc[2] != INFINITY, w3 = tc[3] != INFINITY;
            if (__all(sp + 3 <= stack.cap)) {
                stack.lds[sp * stack.width + lane] = w3 ? rc[3] : w2 ? rc[2] : rc[1];
                stack.lds[(sp + 1) * stack.width + lane] = w3 ? rc[2] : rc[1];
                stack.lds[(sp + 2) * stack.width + lane] = rc[1];
                sp += static_cast<int>(w1) + static_cast<int>(w2) + static_cast<int>(w3);
            } else {
                if (w3) stack.push(sp, rc[3]);
                if (w2) stack.push(sp, rc[2]);
                if (w1) stack.push(sp, rc[1]);
            }
            if (tc[0] != INFINITY) return rc[0];
            return stack.pop_or(sp, base, kDoneRef);
        }
        const int nh = (tc[0] != INFINITY) + (tc[1] != INFINITY) + (tc[2] != INFINITY) + (tc[3] != INFINITY);
        if (nh > 1) {   // (the 5-exchange network costs ~25 VALU; nodes with one child or none skip it)
            cswap(tc[0], rc[0], tc[1], rc[1]);
            cswap(tc[2], rc[2], tc[3], rc[3]);
            cswap(tc[0], rc[0], tc[2], rc[2]);
            cswap(tc[1], rc[1], tc[3], rc[3]);
            cswap(tc[1], rc[1], tc[2], rc[2]);
        } else {
            rc[0] = tc[0] != INFINITY ? rc[0] : tc[1] != INFINITY ? rc[1] : tc[2] != INFINITY ? rc[2] : rc[3];
        }
        if (__all(sp + 3 <= stack.cap)) {
            stack.lds[sp * stack.width + lane] = nh == 4 ? rc[3] : nh == 3 ? rc[2] : rc[1];
            stack.lds[(sp + 1) * stack.width + lane] = nh == 4 ? rc[2] : rc[1];
            stack.lds[(sp + 2) * stack.width + lane] = rc[1];
            sp += max(nh - 1, 0);
        } else {
            if (tc[3] != INFINITY) stack.push(sp, rc[3]);
            if (tc[2] != INFINITY) stack.push(sp, rc[2]);
            if (tc[1] != INFINITY) stack.push(sp, rc[1]);
        }
        if (nh > 0) return rc[0];
        return stack.pop_or(sp, base, kDoneRef);
    }
    // any-hit: any order finds the same verdict; visit the first wanted child, push the others
#if RT_ANY_ORDER
    {   // visit the nearest (1) or farthest (2) wanted child first, push the others
        int kb = -1;
        float tb = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (tc[k] != INFINITY && (kb < 0 || (RT_ANY_ORDER == 1 ? tc[k] < tb : tc[k] > tb))) { kb = k; tb = tc[k]; }
#pragma unroll
        for (int k = 3; k >= 0; --k)
            if (tc[k] != INFINITY && k != kb) stack.push(sp, rc[k]);
        if (kb >= 0) return rc[kb];
        return stack.pop_or(sp, base, kDoneRef);
    }
#endif
    int32_t nxt = kDoneRef;
    bool have = false;
#pragma unroll
    for (int k = 3; k >= 0; --k) {
        if (tc[k] != INFINITY) {
            if (have) stack.push(sp, nxt);
            nxt = rc[k];
            have = true;
        }
    }
    if (have) return nxt;
    return stack.pop_or(sp, base, kDoneRef);
}

// The per-ray traversal constants of the four-wide walk (pad = the kernel's off-plane pad).
// v_rcp_f32 (1 ulp) for the slab reciprocals: every plane of every node uses the same inv, and a
// 1-ulp change of one axis' scale moves its slab parameters by 2^-23 relative, inside the 1e-5
// slack of the te <= tx test and the tcull bound. inv is clamped to |inv| <= 2^100 (dir
// components of 0 or below 2^-100): with the scene below 1e6 in magnitude (dev_view falls back to
// the binary tree otherwise) no slab distance can be NaN (an empty slot's infinite bound gives
// +/-inf, rejected), and a clamped axis only narrows a slab where no hit can exist (|n.dir| >= 1e-5
// needs |dir| >= 2.5e-18 there).
__device__ __forceinline__ void ray4_setup(const DevScene &sc, V3 o, V3 dir, Ray4 &R, float &pad) {
    V3 inv = mk(__builtin_amdgcn_rcpf(dir.x), __builtin_amdgcn_rcpf(dir.y), __builtin_amdgcn_rcpf(dir.z));
    constexpr float kInvMax = 0x1p100f;
    if (!(fabsf(inv.x) <= kInvMax)) inv.x = copysignf(kInvMax, dir.x);
    if (!(fabsf(inv.y) <= kInvMax)) inv.y = copysignf(kInvMax, dir.y);
    if (!(fabsf(inv.z) <= kInvMax)) inv.z = copysignf(kInvMax, dir.z);
    pad = 64.0f * 5.9604645e-08f * (fabsf(o.x) + fabsf(o.y) + fabsf(o.z) + sc.scene_m1);
    // 1.00001 / |dir| with v_rsq_f32 (1 ulp) rounded up by 1e-4: never below the division form
    R.inv_dlen = __builtin_amdgcn_rsqf(dot(dir, dir)) * 1.00011f;
    const bool nx = inv.x < 0, ny = inv.y < 0, nz = inv.z < 0;
    const float pnx = nx ? pad : -pad, pny = ny ? pad : -pad, pnz = nz ? pad : -pad;   // near = lo - pad / hi + pad
    R.ax = f2{inv.x, (pnx - o.x) * inv.x};
    R.ay = f2{inv.y, (pny - o.y) * inv.y};
    R.az = f2{inv.z, (pnz - o.z) * inv.z};
    R.fxy = f2{(-pnx - o.x) * inv.x, (-pny - o.y) * inv.y};
    R.fzc = f2{(-pnz - o.z) * inv.z, INFINITY};   // tcull
    constexpr uint32_t kLo = offsetof(Bvh4F, lo), kHi = offsetof(Bvh4F, hi), kRow = sizeof(float4);
    R.rows[0] = (nx ? kHi : kLo); R.rows[1] = (ny ? kHi : kLo) + kRow; R.rows[2] = (nz ? kHi : kLo) + 2 * kRow;
    R.rows[3] = (nx ? kLo : kHi); R.rows[4] = (ny ? kLo : kHi) + kRow; R.rows[5] = (nz ? kLo : kHi) + 2 * kRow;
}

#ifndef RT_POP_FAST
#define RT_POP_FAST 1   // the walks' own pops (postponement, leaf loop) through LaneStack::pop_or
#endif
__device__ __forceinline__ int32_t walk_pop(const LaneStack &stack, int &sp, int base) {
    if (RT_POP_FAST) return stack.pop_or(sp, base, kDoneRef);
    return sp > base ? stack.pop(sp) : kDoneRef;
}

template <bool kAnyHit>
__device__ __forceinline__ void bvh4_query_ww(const DevScene &sc, V3 o, V3 dir, bool active, int &bidx, V3 &bI,
                                              const LaneStack &stack, unsigned &tests, unsigned &visits) {
    float best = FLT_MAX;
    bool done = !active;
    test_always<kAnyHit>(sc, o, dir, best, bidx, bI, done);
    if (!active || (kAnyHit && done)) return;
    Ray4 R;
    float pad;
    ray4_setup(sc, o, dir, R, pad);
    int sp = 0;
    int32_t node = 0;          // inner node to visit, a leaf ref, or kDoneRef
    int32_t leaf = kDoneRef;   // the postponed leaf
    while (true) {
        while (node >= 0) {
            ++visits;
            node = node4_next<kAnyHit>(R, load_node4(sc.nodes4f, node, R.rows), stack, sp);
            if (node < 0 && node != kDoneRef && leaf == kDoneRef) {   // postpone it, keep walking
                leaf = node;
                node = walk_pop(stack, sp, 0);
            }
            if (__all(leaf != kDoneRef)) break;   // every lane still walking holds a leaf
        }
        while (leaf != kDoneRef) {
            const uint32_t u = static_cast<uint32_t>(leaf);
            const int cnt = static_cast<int>((u >> kBvhCountShift) & kBvhCountMask);
            const int first = static_cast<int>(u & ((1u << kBvhCountShift) - 1u));
            // one triangle per iteration: the ref is the cursor (first + 1, count - 1), so a lane
            // whose leaf ends goes on to its next leaf while the others test their next triangle
            const TriRec T = leaf_rec(sc, first);
            test_triangle<kAnyHit, true, RT_LEAF_SIGN>(T, static_cast<int>(sc.leaf_idx[first]), o, dir, best, bidx, bI, done);
            ++tests;
            if (kAnyHit && done) { node = kDoneRef; break; }
            if (cnt > 1) {
                leaf = static_cast<int32_t>(u + 1u - (1u << kBvhCountShift));
                continue;
            }
            if (!kAnyHit && best < FLT_MAX) R.fzc.y = cull_param(R, best, pad);
            leaf = kDoneRef;
            if (node < 0 && node != kDoneRef) {
                leaf = node;
                node = walk_pop(stack, sp, 0);
            }
        }
        if (node == kDoneRef) break;
    }
}
// ---------------------------------------------------------------------------------------------
// While-while walk with in-wave work stealing (RT_TUNE_WAVE_STEAL, chain launch): a lane whose own query is finished
// takes the bottom entry of another lane's traversal stack (a subtree that lane would visit later)
// together with that lane's ray, walks it with the same node and triangle arithmetic, and folds
// what it finds into the ray owner's (distance, index) key in LDS. Exactness: every subtree is
// walked by exactly one lane; a helper culls with its own best, which starts at the donor's best
// (an upper bound of the final minimum), so no triangle that could beat the final minimum is
// skipped; the result is the lexicographic minimum of all keys. The owner takes its own hit point
// when its own key wins, else re-runs test_triangle on the winning record (the same arithmetic on
// the same record and ray, so the same bits). Any-hit: any key is a hit; the owner stops walking
// once a helper has published one. Only placement changes, never results.
// ---------------------------------------------------------------------------------------------
#ifndef RT_STEAL_WPE
#define RT_STEAL_WPE 4   // waves per EU of the stealing chain kernel (5 spilled ~100 VGPRs in r03; r04, with the
                         // arguments read per batch, 88 B per lane and still slower on C2: profiles/r04_ab_steal_wpe.txt)
#endif
#ifndef RT_STEAL_MIN_IDLE
#define RT_STEAL_MIN_IDLE 8   // steal only when at least this many lanes of the wave are idle
#endif
// (how many of the longest batches run as half or quarter waves: RT_TUNE_STEAL_HALF / _QUARTER)
#ifndef RT_STEAL_SPLIT_DIV
#define RT_STEAL_SPLIT_DIV 32   // ... and at most this fraction (1 / DIV) of them
#endif
#ifndef RT_STEAL_TOP
#define RT_STEAL_TOP 1        // 1: a donor gives its nearest pending subtree (top of stack); 0: its farthest
#endif
constexpr unsigned long long kNoKey = ~0ull;
__device__ __forceinline__ unsigned long long hit_key(float best, int bidx) {
    return (static_cast<unsigned long long>(__float_as_uint(best)) << 32) | static_cast<uint32_t>(bidx);
}

template <bool kAnyHit>
__device__ __forceinline__ void bvh4_query_steal(const DevScene &sc, V3 o, V3 dir, bool active, int &bidx, V3 &bI,
                                                 const LaneStack &stack, unsigned &tests, unsigned &visits) {
    __shared__ unsigned long long s_key[kBvhBlock];   // per lane: its ray's best key (own walk and helpers)
    __shared__ float s_hit[3 * kBvhBlock];            // per lane: the hit point of that key
    __shared__ int32_t s_xfer[2 * kBvhBlock];         // per wave: [pair rank] donor lane | owner << 8, stolen ref
    const int tid = static_cast<int>(threadIdx.x), lane = __lane_id(), wb = tid & ~63;   // this wave's slots
    float best = FLT_MAX;
    bool done = !active;
    test_always<kAnyHit>(sc, o, dir, best, bidx, bI, done);
    s_key[tid] = kNoKey;
    // o, dir: the ray this lane walks (its own, later the rays it helps with)
    Ray4 R;
    float pad;
    ray4_setup(sc, o, dir, R, pad);
    int sp = 0, base = 0;
    int32_t node = (active && !(kAnyHit && done)) ? 0 : kDoneRef;
    int32_t leaf = kDoneRef;
    int owner = active ? tid : -1;   // the slot this walk reports to (its own, or the helped lane's); -1: idle
    int pidx = -1;                   // bidx as last published or adopted: a different bidx is a new find
    __builtin_amdgcn_wave_barrier();
    while (true) {
        // new finds go to the ray's slot: the key first, then (second pass) the hit point of the
        // winning key (equal keys: the same triangle and ray, so the same point)
        const bool pub = owner >= 0 && bidx != pidx;
        const unsigned long long k = hit_key(best, bidx);
        if (pub) atomicMin(&s_key[owner], k);
        __builtin_amdgcn_wave_barrier();
        if (pub && s_key[owner] == k) {
            s_hit[3 * owner] = bI.x; s_hit[3 * owner + 1] = bI.y; s_hit[3 * owner + 2] = bI.z;
        }
        if (pub) pidx = bidx;
        if (owner >= 0) {   // a better key from another walk of the same ray: cull with it
            const unsigned long long sk = s_key[owner];
            if (sk < hit_key(best, bidx)) {
                if (kAnyHit) { node = kDoneRef; leaf = kDoneRef; }   // any hit ends every walk of the ray
                best = __uint_as_float(static_cast<uint32_t>(sk >> 32));
                bidx = static_cast<int>(static_cast<uint32_t>(sk));
                pidx = bidx;
                if (!kAnyHit) R.fzc.y = cull_param(R, best, pad);
            }
        }
        if (node == kDoneRef && leaf == kDoneRef) { owner = -1; sp = base; }   // (an abandoned any-hit walk's stack too)
        __builtin_amdgcn_wave_barrier();
        const uint64_t act = __ballot(1), idle = __ballot(owner < 0);
        if (idle == act) break;
        const uint64_t donors = __ballot(owner >= 0 && sp - base >= 1);
        if (__popcll(idle) >= RT_STEAL_MIN_IDLE && donors) {
            const int np = min(__popcll(idle), __popcll(donors));
            const int ir = rank_below(idle), dr = rank_below(donors);
            if (((donors >> lane) & 1ull) && dr < np) {
                s_xfer[wb + 2 * dr] = lane | (owner << 8);
                if (RT_STEAL_TOP) {   // the top entry: the nearest subtree still pending
                    --sp;
                    s_xfer[wb + 2 * dr + 1] = stack.at(sp);
                } else {              // the bottom entry: the farthest
                    s_xfer[wb + 2 * dr + 1] = stack.at(base);
                    ++base;
                }
            }
            __builtin_amdgcn_wave_barrier();
            const bool helper = ((idle >> lane) & 1ull) && ir < np;
            int src = lane, xo = -1, ref = kDoneRef;
            if (helper) {
                const int v = s_xfer[wb + 2 * ir];
                src = v & 0xFF;
                xo = v >> 8;
                ref = s_xfer[wb + 2 * ir + 1];
            }
            __builtin_amdgcn_wave_barrier();
            const V3 ho = mk(__shfl(o.x, src), __shfl(o.y, src), __shfl(o.z, src));
            const V3 hd = mk(__shfl(dir.x, src), __shfl(dir.y, src), __shfl(dir.z, src));
            const float hb = __shfl(best, src);
            const int hi = __shfl(bidx, src);
            if (helper) {
                o = ho; dir = hd;
                best = hb; bidx = hi; pidx = hi;   // the donor's best bounds the final minimum: cull with it
                ray4_setup(sc, o, dir, R, pad);
                if (!kAnyHit && best < FLT_MAX) R.fzc.y = cull_param(R, best, pad);
                done = false;
                sp = 0; base = 0;
                node = ref;
                if (node < 0) { leaf = node; node = kDoneRef; }   // a leaf ref
                owner = xo;
            }
        }
        while (node >= 0) {
            ++visits;
            node = node4_next<kAnyHit>(R, load_node4(sc.nodes4f, node, R.rows), stack, sp, base);
            if (node < 0 && node != kDoneRef && leaf == kDoneRef) {   // postpone it, keep walking
                leaf = node;
                node = walk_pop(stack, sp, base);
            }
            if (__all(leaf != kDoneRef)) break;
        }
        while (leaf != kDoneRef) {
            const uint32_t u = static_cast<uint32_t>(leaf);
            const int cnt = static_cast<int>((u >> kBvhCountShift) & kBvhCountMask);
            const int first = static_cast<int>(u & ((1u << kBvhCountShift) - 1u));
            const TriRec T = leaf_rec(sc, first);
            test_triangle<kAnyHit, true, RT_LEAF_SIGN>(T, static_cast<int>(sc.leaf_idx[first]), o, dir, best, bidx, bI, done);
            ++tests;
            if (kAnyHit && done) { node = kDoneRef; leaf = kDoneRef; break; }
            if (cnt > 1) {
                leaf = static_cast<int32_t>(u + 1u - (1u << kBvhCountShift));
                continue;
            }
            if (!kAnyHit && best < FLT_MAX) R.fzc.y = cull_param(R, best, pad);
            leaf = kDoneRef;
            if (node < 0 && node != kDoneRef) {
                leaf = node;
                node = walk_pop(stack, sp, base);
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    const unsigned long long k = s_key[tid];
    bidx = -1;
    bI = mk(0, 0, 0);   // no hit: the callers' initial point (every call site starts from (0, 0, 0))
    if (active && k != kNoKey) {
        bidx = static_cast<int>(static_cast<uint32_t>(k));
        bI = mk(s_hit[3 * tid], s_hit[3 * tid + 1], s_hit[3 * tid + 2]);
    }
}

// ---------------------------------------------------------------------------------------------
// Quad walk (RT_TUNE_QUAD_WALK, the quarter tier of ordered launches, r05): four lanes per ray. The
// four lanes of a quad hold the same ray, its stack and its chain; lane q of the quad tests child q
// of each four-wide node (one box, not four), the quad ranks the four entry distances with DPP lane
// exchanges, the nearest wanted child is visited next and the others are pushed by their own lanes;
// a leaf's triangles are tested side by side (lane q: triangle q, q + 4, ...). A node visit is then
// ~60 wave-instructions instead of ~130, so a ray's walk, bound by the dependent issue and load
// latency of its visits, shortens: this is for the longest batches of the order (the frame's
// critical path), whose every lane carries three reflections. Exactness: the node test per child is
// the per-lane walk's (the same te/tx/tcull arithmetic), the cull bound is the quad's least accepted
// distance (a hit of this ray), every triangle of every visited leaf is tested by one lane, and the
// result is the lexicographic (distance, index) minimum over the quad's lanes: the same minimum as
// any other order of the same tests. Every DPP exchange below runs with all four lanes of each
// active quad active (the quad's control flow is uniform: all its values are the same).
// ---------------------------------------------------------------------------------------------
constexpr int kQuadSamples = kWaveBatch / 4;   // samples (quads) per wave in the quad walk
__device__ __forceinline__ int dpp_qx1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false); }   // lane ^ 1
__device__ __forceinline__ int dpp_qx2(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false); }   // lane ^ 2
__device__ __forceinline__ int dpp_qx3(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x1B, 0xF, 0xF, false); }   // lane ^ 3
__device__ __forceinline__ float quad_min(float x) {
    x = fminf(x, as_float(dpp_qx1(as_int(x))));
    return fminf(x, as_float(dpp_qx2(as_int(x))));
}
__device__ __forceinline__ bool quad_any(bool b) {
    int v = static_cast<int>(b);
    v |= dpp_qx1(v);
    v |= dpp_qx2(v);
    return v != 0;
}
// The lexicographic (distance, index) minimum over the quad, with its point, in every lane. A lane
// without a hit holds (FLT_MAX, -1): any hit is below FLT_MAX (test_triangle accepts dist < best).
__device__ __forceinline__ void quad_lex_min(float &best, int &bidx, V3 &bI) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const float ob = as_float(r ? dpp_qx2(as_int(best)) : dpp_qx1(as_int(best)));
        const int oi = r ? dpp_qx2(bidx) : dpp_qx1(bidx);
        const float ox = as_float(r ? dpp_qx2(as_int(bI.x)) : dpp_qx1(as_int(bI.x)));
        const float oy = as_float(r ? dpp_qx2(as_int(bI.y)) : dpp_qx1(as_int(bI.y)));
        const float oz = as_float(r ? dpp_qx2(as_int(bI.z)) : dpp_qx1(as_int(bI.z)));
        const bool take = ob < best || (ob == best && static_cast<uint32_t>(oi) < static_cast<uint32_t>(bidx));
        best = take ? ob : best;
        bidx = take ? oi : bidx;
        bI = take ? mk(ox, oy, oz) : bI;
    }
}

// A quad's traversal stack: its wave's 16 x 64 words of the block's lane stacks (LaneStack rows
// [entry][lane], this wave's 64 columns) seen as 64 entries x 16 quads; deeper entries in the global
// overflow area at the quad's first lane ([entry - cap][grid lane], inside the per-lane area).
struct QuadStack {
    int32_t *lds;   // this wave's first column of row 0
    int32_t *ovf;
    int cap, stride, gl0, slot;
    __device__ __forceinline__ int32_t *at_lds(int e) const { return lds + (e >> 2) * kBvhBlock + ((e & 3) << 4) + slot; }
    __device__ __forceinline__ void put(int e, int32_t v) const {
        if (e < cap) *at_lds(e) = v;
        else ovf[static_cast<size_t>(e - cap) * stride + gl0] = v;
    }
    __device__ __forceinline__ int32_t get(int e) const {
        int32_t v = *at_lds(min(e, cap - 1));
        if (e >= cap) v = ovf[static_cast<size_t>(e - cap) * stride + gl0];
        return v;
    }
};
__device__ __forceinline__ QuadStack quad_stack(const DevScene &sc, int32_t *lds, int lane) {
    QuadStack st;
    const int wbase = static_cast<int>(threadIdx.x) & ~63;
    st.lds = lds + wbase;
    st.ovf = sc.stack_ovf;
    st.cap = 4 * sc.lds_stack;
    st.stride = static_cast<int>(gridDim.x) * kBvhBlock;
    st.gl0 = static_cast<int>(blockIdx.x) * kBvhBlock + wbase + (lane & ~3);
    st.slot = lane >> 2;
    return st;
}

// One node visit of the quad walk: returns the next ref (the nearest wanted child, else the stack
// top, else kDoneRef) in every lane of the quad. q = this lane's child slot, qshift = the quad's
// first lane (its bits in a ballot).
template <bool kAnyHit>
__device__ __forceinline__ int32_t node4_next_quad(const Ray4 &R, const Bvh4F *__restrict__ nodes4, int32_t node, const QuadStack &st,
                                                   int &sp, int q, int qshift) {
    const char *__restrict__ base = reinterpret_cast<const char *>(nodes4);
    const uint32_t o = static_cast<uint32_t>(node) * static_cast<uint32_t>(sizeof(Bvh4F)) + 4u * static_cast<uint32_t>(q);
    const float nx = *reinterpret_cast<const float *>(base + (o + R.rows[0]));
    const float ny = *reinterpret_cast<const float *>(base + (o + R.rows[1]));
    const float nz = *reinterpret_cast<const float *>(base + (o + R.rows[2]));
    const float fx = *reinterpret_cast<const float *>(base + (o + R.rows[3]));
    const float fy = *reinterpret_cast<const float *>(base + (o + R.rows[4]));
    const float fz = *reinterpret_cast<const float *>(base + (o + R.rows[5]));
    const int32_t ref = *reinterpret_cast<const int32_t *>(base + (o + static_cast<uint32_t>(offsetof(Bvh4F, child))));
    const float tnx = fmaf(nx, R.ax.x, R.ax.y), tfx = fmaf(fx, R.ax.x, R.fxy.x);
    const float tny = fmaf(ny, R.ay.x, R.ay.y), tfy = fmaf(fy, R.ay.x, R.fxy.y);
    const float tnz = fmaf(nz, R.az.x, R.az.y), tfz = fmaf(fz, R.az.x, R.fzc.x);
    const float te = fmaxf(fmaxf(fmaxf(tnx, tny), tnz), 0.0f);
    const float tx = fminf(fminf(tfx, tfy), tfz);
    const bool want = te <= node_lim<kAnyHit>(tx, R.fzc.y);   // (the per-lane walk's test for this child)
    // rank among the quad by entry distance: te >= 0, so its bits order as the floats; the two low
    // bits (the slot) break ties and make the keys distinct (traversal order only); misses sort last
    const uint32_t key = want ? ((static_cast<uint32_t>(as_int(te)) & ~3u) | static_cast<uint32_t>(q)) : (0xFFFFFFFCu | static_cast<uint32_t>(q));
    const uint32_t k1 = static_cast<uint32_t>(dpp_qx1(static_cast<int>(key)));
    const uint32_t k2 = static_cast<uint32_t>(dpp_qx2(static_cast<int>(key)));
    const uint32_t k3 = static_cast<uint32_t>(dpp_qx3(static_cast<int>(key)));
    const int rank = static_cast<int>(k1 < key) + static_cast<int>(k2 < key) + static_cast<int>(k3 < key);
    const int nh = __popc(static_cast<uint32_t>(__ballot(want) >> qshift) & 0xFu);
    int32_t r0 = rank == 0 ? ref : 0;   // the nearest child's ref, to every lane of the quad
    r0 += dpp_qx1(r0);
    r0 += dpp_qx2(r0);
    if (want && rank > 0) st.put(sp + nh - 1 - rank, ref);   // farthest deepest: rank 1 ends on top
    sp += max(nh - 1, 0);
    if (nh > 0) return r0;
    if (sp <= 0) return kDoneRef;
    return st.get(--sp);
}

// The always-tested list split over the quad's lanes (lane q: entries q, q + 4, ...).
template <bool kAnyHit>
__device__ __forceinline__ void test_always_quad(const DevScene &sc, V3 o, V3 dir, float &best, int &bidx, V3 &bI, bool &done, int q) {
    for (int i = q; i < sc.n_always; i += 4)
        test_triangle<kAnyHit, true, RT_ALWAYS_SIGN>(sc.always_recs[i], static_cast<int>(sc.always[i]), o, dir, best, bidx, bI, done);
}

template <bool kAnyHit>
__device__ __forceinline__ void bvh4_query_quad(const DevScene &sc, V3 o, V3 dir, bool active, int &bidx, V3 &bI,
                                                const QuadStack &st, unsigned &tests, unsigned &visits, int q, int qshift) {
    float best = FLT_MAX;
    bool done = !active;
    test_always_quad<kAnyHit>(sc, o, dir, best, bidx, bI, done, q);
    if (active && !(kAnyHit && quad_any(done))) {
        Ray4 R;
        float pad;
        ray4_setup(sc, o, dir, R, pad);
        if (!kAnyHit) {
            const float qb = quad_min(best);
            if (qb < FLT_MAX) R.fzc.y = cull_param(R, qb, pad);
        }
        int sp = 0;
        int32_t node = 0, leaf = kDoneRef;
        while (true) {
            while (node >= 0) {
                if (q == 0) ++visits;
                node = node4_next_quad<kAnyHit>(R, sc.nodes4f, node, st, sp, q, qshift);
                if (node < 0 && node != kDoneRef && leaf == kDoneRef) {   // postpone the leaf, keep walking
                    leaf = node;
                    node = sp > 0 ? st.get(--sp) : kDoneRef;
                }
                if (__all(leaf != kDoneRef)) break;   // every quad still walking holds a leaf
            }
            while (leaf != kDoneRef) {   // one leaf per iteration: its triangles side by side
                const uint32_t u = static_cast<uint32_t>(leaf);
                const int cnt = static_cast<int>((u >> kBvhCountShift) & kBvhCountMask);
                const int first = static_cast<int>(u & ((1u << kBvhCountShift) - 1u));
                for (int k = q; k < cnt; k += 4) {
                    test_triangle<kAnyHit, true, RT_LEAF_SIGN>(leaf_rec(sc, first + k), static_cast<int>(sc.leaf_idx[first + k]), o, dir,
                                                               best, bidx, bI, done);
                    ++tests;
                }
                if (kAnyHit) {
                    if (quad_any(done)) { node = kDoneRef; leaf = kDoneRef; break; }
                } else {
                    const float qb = quad_min(best);
                    if (qb < FLT_MAX) R.fzc.y = cull_param(R, qb, pad);
                }
                leaf = kDoneRef;
                if (node < 0 && node != kDoneRef) {
                    leaf = node;
                    node = sp > 0 ? st.get(--sp) : kDoneRef;
                }
            }
            if (node == kDoneRef) break;
        }
    }
    quad_lex_min(best, bidx, bI);
    if (bidx < 0) bI = mk(0, 0, 0);
}


// The closest-hit / any-hit query of the tree kernels: W = 4 the four-wide while-while walk (or,
// kSteal, its in-wave stealing form), W = 2 the binary tree (scenes above 1e6 in magnitude).
template <bool kAnyHit, int W, bool kSteal = false>
__device__ __forceinline__ void bvh_query_w(const DevScene &sc, V3 o, V3 dir, bool active, int &bidx, V3 &bI,
                                            const LaneStack &stack, unsigned &tests, unsigned &visits) {
    if (W == 4 && kSteal) bvh4_query_steal<kAnyHit>(sc, o, dir, active, bidx, bI, stack, tests, visits);
    else if (W == 4) bvh4_query_ww<kAnyHit>(sc, o, dir, active, bidx, bI, stack, tests, visits);
    else bvh_query<kAnyHit>(sc, o, dir, active, bidx, bI, stack, tests, visits);
}

// XCD-aware work split (cdna_hip_programming.md T1): blocks are dealt round-robin over the 8 XCDs,
// so blocks b and b+8 share an XCD's L2. Queues are in screen order (tiles row-major, children
// after their parents), so giving each XCD one contiguous eighth of the queue keeps the part of
// the scene it touches small enough to stay in its 4 MB L2. Placement only changes speed.
constexpr int kXcds = 8;
constexpr int kWave = 64;
struct Segment { int begin, end, step, start; };
__device__ __forceinline__ Segment xcd_segment(int n, int block_dim, bool split) {
    const int nseg = split ? min(kXcds, static_cast<int>(gridDim.x)) : 1;   // every segment gets >= 1 block
    const int xcd = blockIdx.x % nseg;
    const int per_xcd_blocks = (static_cast<int>(gridDim.x) - 1 - xcd) / nseg + 1;   // blocks with this residue
    const int local = blockIdx.x / nseg;
    // (whole 64-query chunks: every wave's range starts on a multiple of 64, so a wave's query indices
    // j0 .. j0 + 63 share j0 >> 6 in every distribution, which the chain kernel reads as a scalar)
    const int chunk = ((n + nseg - 1) / nseg + kWave - 1) & ~(kWave - 1);
    Segment g;
    g.begin = min(n, xcd * chunk);
    g.end = min(n, g.begin + chunk);
    g.step = per_xcd_blocks * block_dim;
    g.start = g.begin + local * block_dim;
    return g;
}

// Per-kernel work counters (DevScene::work, kWorkFields per kind): ray-triangle tests, node
// visits, the sum over wave tasks (64 queries side by side) of the largest per-lane visit count,
// the largest visit count of any query, the number of wave tasks, the sum of per-task largest
// test counts. visits / (64 * wave-max sum) is the SIMD efficiency of the traversal loop. Only
// the kCount instantiations of the BVH kernels (RT_PROFILE_WORK) carry it.
template <bool kOn>
struct WorkTally {
    unsigned tests = 0, visits = 0, vmax = 0;
    unsigned long long wave_vmax = 0, wave_tmax = 0, tasks = 0;
    unsigned t0 = 0, v0 = 0;
    __device__ __forceinline__ void begin() { if (kOn) { t0 = tests; v0 = visits; } }
    __device__ __forceinline__ void end() {
        if (!kOn) return;
        unsigned dv = visits - v0, dt = tests - t0;
        vmax = max(vmax, dv);
        for (int off = 32; off > 0; off >>= 1) {
            dv = max(dv, static_cast<unsigned>(__shfl_xor(static_cast<int>(dv), off)));
            dt = max(dt, static_cast<unsigned>(__shfl_xor(static_cast<int>(dt), off)));
        }
        wave_vmax += dv;
        wave_tmax += dt;
        ++tasks;
    }
    __device__ __forceinline__ void flush(unsigned long long *work) {
        if (!kOn || !work) return;
        unsigned long long a = tests, b = visits;
        unsigned m = vmax;
        for (int off = 32; off > 0; off >>= 1) {
            a += __shfl_xor(a, off);
            b += __shfl_xor(b, off);
            m = max(m, static_cast<unsigned>(__shfl_xor(static_cast<int>(m), off)));
        }
        if (__lane_id() == 0) {
            atomicAdd(&work[0], a);
            atomicAdd(&work[1], b);
            atomicAdd(&work[2], wave_vmax);
            atomicMax(&work[3], static_cast<unsigned long long>(m));
            atomicAdd(&work[4], tasks);
            atomicAdd(&work[5], wave_tmax);
        }
    }
};

// Query distribution for the BVH kernels. split 0: resident grid-stride over the queue. split 1:
// each XCD's blocks stride over one contiguous eighth. split 2: the queue is cut into eight
// segments with one counter each; a wave takes 64 queries at a time from its own XCD's segment
// (screen-ordered, so the XCD's L2 holds a compact part of the scene) and, once that is empty,
// from the others in turn, so no XCD idles while another has work. Every wave leaves after it has
// seen all eight segments empty. Placement only changes speed, never results.
struct QueryCursor {
    int n, split, k = 0, base, step, end, glog;
    int32_t *wq;
    __device__ __forceinline__ QueryCursor(int n_, int split_, int32_t *wq_, int glog_ = 0) : n(n_), split(split_), glog(glog_), wq(wq_) {
        if ((split == 2 || split == 3 || split == 4) && wq) return;
        const Segment seg = xcd_segment(n, kBvhBlock, split == 1);
        base = seg.start - seg.step;
        step = seg.step;
        end = seg.end;
    }
    // Next query index for this lane (may be >= end: inactive lane); false once the wave is done.
    __device__ __forceinline__ bool next(int &j) {
        if (split == 4 && wq) {   // as 3, but every wave's first chunk is static (its own slot in its XCD's
            // sequence) and only later ones come from the counter, which then counts from the XCD's wave
            // count: a launch's waves do not queue on eight counter words to get their first chunk
            const int nx = min(kXcds, static_cast<int>(gridDim.x));   // (grids of fewer blocks: fewer sequences)
            const int g = blockIdx.x % nx;
            const int wpb = static_cast<int>(blockDim.x) / kWave;
            int c;
            if (k == 0) {   // (the wave's index in its block, as a scalar: the task index stays in SGPRs)
                c = static_cast<int>(blockIdx.x / nx) * wpb + __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
                k = 1;
            } else {
                const int nblk = (static_cast<int>(gridDim.x) - 1 - g) / nx + 1;   // blocks of this sequence
                int a = 0;
                if (__lane_id() == 0) a = atomicAdd(&wq[g * kWqStride], 1);
                c = nblk * wpb + __builtin_amdgcn_readfirstlane(__shfl(a, 0));   // (a scalar: the wave's task)
            }
            const int b = ((((c >> glog) * nx + g) << glog) + (c & ((1 << glog) - 1))) * kWave;
            end = n;
            if (b < n) { j = b + __lane_id(); return true; }
            return false;
        }
        if (split == 3 && wq) {   // 64-query chunks dealt round-robin to the XCDs (in groups of 2^glog consecutive
            const int nx = min(kXcds, static_cast<int>(gridDim.x));   // chunks), taken dynamically within each
            const int g = blockIdx.x % nx;
            int c = 0;
            if (__lane_id() == 0) c = atomicAdd(&wq[g * kWqStride], 1);
            c = __builtin_amdgcn_readfirstlane(__shfl(c, 0));
            const int b = ((((c >> glog) * nx + g) << glog) + (c & ((1 << glog) - 1))) * kWave;
            end = n;
            if (b < n) { j = b + __lane_id(); return true; }
            return false;
        }
        if (split == 2 && wq) {
            const int home = blockIdx.x % kXcds;
            const int chunk = (n + kXcds - 1) / kXcds;
            while (k < kXcds) {
                const int g = (home + k) % kXcds;
                const int begin = min(n, g * chunk);
                end = min(n, begin + chunk);
                int b = 0;
                if (__lane_id() == 0) b = atomicAdd(&wq[g * kWqStride], kWave);
                b = begin + __builtin_amdgcn_readfirstlane(__shfl(b, 0));
                if (b < end) { j = b + __lane_id(); return true; }
                ++k;
            }
            return false;
        }
        base += step;
        j = base + static_cast<int>(threadIdx.x);
        return base < end;
    }
};

template <typename F>
__device__ __forceinline__ void drive_queries(int n, int split, int32_t *__restrict__ wq, F &&body, int glog = 0) {
    QueryCursor c(n, split, wq, glog);
    int j;
    while (c.next(j)) body(j, c.end);
}

template <int W, bool kCount>
__global__ __launch_bounds__(kBvhBlock) __attribute__((amdgpu_waves_per_eu(7))) void k_bvh_closest_hit(const DevScene sc, const float4 *__restrict__ q_org,
                                                               const float4 *__restrict__ q_dst,
                                                               const int32_t *__restrict__ q_count,
                                                               int32_t *__restrict__ hit_idx, float4 *__restrict__ hit_I,
                                                               int32_t *__restrict__ wq) {
    extern __shared__ int32_t lds_stack[];
    const LaneStack stack = lane_stack(sc, lds_stack);
    WorkTally<kCount> wt;
    drive_queries(*q_count, sc.xcd_split, wq, [&](int j, int end) {
        bool active = j < end;
        V3 o = mk(0, 0, 0), dir = mk(0, 0, 0);
        if (active) {
            const float4 qo = q_org[j], qd = q_dst[j];
            active = as_int(qd.w) >= 0;
            o = mk(qo.x, qo.y, qo.z);
            dir = mk(qd.x - qo.x, qd.y - qo.y, qd.z - qo.z);
        }
        int bidx = -1;
        V3 bI = mk(0, 0, 0);
        wt.begin();
        bvh_query_w<false, W>(sc, o, dir, active, bidx, bI, stack, wt.tests, wt.visits);
        wt.end();
        if (j < end) {
            hit_idx[j] = bidx;
            hit_I[j] = make_float4(bI.x, bI.y, bI.z, 0.0f);
        }
    });
    wt.flush(sc.work);
}

// Shadow query j of a ShadowSource: ray and output slot; false if the pair is inactive.
__device__ __forceinline__ bool shadow_query(const ShadowSource &src, int j, int end, V3 &o, V3 &dir, int &slot) {
    if (j >= end) return false;
    if (src.virt) {
        const int L = src.n_lights;
        const int k = j / L, l = j - k * L;
        if (src.hit_idx[k] < 0) return false;
        const float4 I = src.hit_I[k];
        o = mk(I.x + 0.1f, I.y + 0.1f, I.z + 0.1f);                                    // :248
        const V3 Lp = light_at(src.lights, src.light_ext, l);
        dir = mk(Lp.x - o.x, Lp.y - o.y, Lp.z - o.z);
        slot = j;
        return true;
    }
    const float4 qo = src.sq_org[j], qd = src.sq_dst[j];
    o = mk(qo.x, qo.y, qo.z);
    dir = mk(qd.x - qo.x, qd.y - qo.y, qd.z - qo.z);
    slot = as_int(qo.w);
    return true;
}

__device__ __forceinline__ int shadow_total(const ShadowSource &src) {
    return src.virt ? *src.count * src.n_lights : *src.count;
}

// Virtual sources: the block's active pairs, one atomic per block (ray statistics).
__device__ __forceinline__ void add_pair_count(const ShadowSource &src, unsigned mine) {
    if (!src.virt) return;
    __shared__ unsigned s_pairs;
    if (threadIdx.x == 0) s_pairs = 0;
    __syncthreads();
    unsigned long long c = mine;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if (__lane_id() == 0 && c) atomicAdd(&s_pairs, static_cast<unsigned>(c));
    __syncthreads();
    if (threadIdx.x == 0 && s_pairs) atomicAdd(src.pair_count, static_cast<int32_t>(s_pairs));
}

template <bool kAnyHit, int W, bool kCount>
__global__ __launch_bounds__(kBvhBlock) __attribute__((amdgpu_waves_per_eu(7))) void k_bvh_shadow_hit(const DevScene sc, const ShadowSource src,
                                                              uint8_t *__restrict__ shadow, int32_t *__restrict__ wq) {
    extern __shared__ int32_t lds_stack[];
    const LaneStack stack = lane_stack(sc, lds_stack);
    WorkTally<kCount> wt;
    unsigned pairs = 0;
    drive_queries(shadow_total(src), sc.xcd_split, wq, [&](int j, int end) {
        V3 o = mk(0, 0, 0), dir = mk(0, 0, 0);
        int slot = 0;
        const bool active = shadow_query(src, j, end, o, dir, slot);
        pairs += active;
        int bidx = -1;
        V3 bI = mk(0, 0, 0);
        wt.begin();
        bvh_query_w<kAnyHit, W>(sc, o, dir, active, bidx, bI, stack, wt.tests, wt.visits);
        wt.end();
        if (active) {
            uint8_t sh = 0;
            if (bidx >= 0) sh = sc.mats[sc.tri_mat[bidx]].transparent ? 0 : 1;   // :253-257
            shadow[slot] = sh;
        }
    });
    wt.flush(sc.work ? sc.work + kWorkFields : nullptr);
    add_pair_count(src, pairs);
}

template <int W, bool kCount>
__global__ __launch_bounds__(kBvhBlock) void k_bvh_intersect_only(const DevScene sc, const float4 *__restrict__ q_org,
                                                                  const float4 *__restrict__ q_dst, int n,
                                                                  int32_t *__restrict__ idx, float4 *__restrict__ I) {
    extern __shared__ int32_t lds_stack[];
    const LaneStack stack = lane_stack(sc, lds_stack);
    WorkTally<kCount> wt;
    drive_queries(n, 0, nullptr, [&](int j, int end) {
        const bool active = j < end;
        V3 o = mk(0, 0, 0), dir = mk(0, 0, 0);
        if (active) {
            const float4 qo = q_org[j], qd = q_dst[j];
            o = mk(qo.x, qo.y, qo.z);
            dir = mk(qd.x - qo.x, qd.y - qo.y, qd.z - qo.z);
        }
        int bidx = -1;
        V3 bI = mk(0, 0, 0);
        wt.begin();
        bvh_query_w<false, W>(sc, o, dir, active, bidx, bI, stack, wt.tests, wt.visits);
        wt.end();
        if (active) { idx[j] = bidx; I[j] = make_float4(bI.x, bI.y, bI.z, 0.0f); }
    });
    wt.flush(sc.work);
}

__global__ __launch_bounds__(kBlock) void k_closest_hit(const TriRec *__restrict__ tris, int nt,
                                                        const float4 *__restrict__ q_org,
                                                        const float4 *__restrict__ q_dst,
                                                        const int32_t *__restrict__ q_count,
                                                        int32_t *__restrict__ hit_idx, float4 *__restrict__ hit_I) {
    const int n = *q_count;
    const int base = blockIdx.x * kBlock;
    if (base >= n) return;
    const int j = base + threadIdx.x;
    bool active = j < n;
    V3 o = mk(0, 0, 0), dir = mk(0, 0, 0);
    if (active) {
        const float4 qo = q_org[j], qd = q_dst[j];
        active = as_int(qd.w) >= 0;                                                 // lvl -1: outside the frame
        o = mk(qo.x, qo.y, qo.z);
        dir = mk(qd.x - qo.x, qd.y - qo.y, qd.z - qo.z);                          // :111
    }
    int bidx = -1;
    V3 bI = mk(0, 0, 0);
    closest_hit_loop<false>(tris, nt, o, dir, active, bidx, bI);
    if (j < n) {
        hit_idx[j] = bidx;
        hit_I[j] = make_float4(bI.x, bI.y, bI.z, 0.0f);
    }
}

// The brute-force closest hit's counting pass (RT_PROFILE_WORK): the same tests, one triangle per
// iteration, with the stages each test reaches summed per kind into diag words [0, kTestStages) of
// the work area (rt_diag_read). Results are written as k_closest_hit writes them.
__global__ __launch_bounds__(kBlock) void k_closest_hit_stages(const TriRec *__restrict__ tris, int nt,
                                                               const float4 *__restrict__ q_org, const float4 *__restrict__ q_dst,
                                                               const int32_t *__restrict__ q_count, int32_t *__restrict__ hit_idx,
                                                               float4 *__restrict__ hit_I, unsigned long long *__restrict__ diag) {
    const int n = *q_count;
    const int j = blockIdx.x * kBlock + threadIdx.x;
    unsigned stg[kTestStages] = {};
    if (j < n) {
        const float4 qo = q_org[j], qd = q_dst[j];
        if (as_int(qd.w) >= 0) {
            const V3 o = mk(qo.x, qo.y, qo.z), dir = mk(qd.x - qo.x, qd.y - qo.y, qd.z - qo.z);
            float best = FLT_MAX;
            int bidx = -1;
            V3 bI = mk(0, 0, 0);
            bool done = false;
            for (int t = 0; t < nt; ++t) test_triangle<false, false, false, true>(tris[t], t, o, dir, best, bidx, bI, done, stg);
            hit_idx[j] = bidx;
            hit_I[j] = make_float4(bI.x, bI.y, bI.z, 0.0f);
        } else {
            hit_idx[j] = -1;
            hit_I[j] = make_float4(0, 0, 0, 0);
        }
    }
    for (int k = 0; k < kTestStages; ++k) {
        unsigned long long c = stg[k];
        for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
        if (__lane_id() == 0 && c) atomicAdd(&diag[k], c);
    }
}

// Shadow queries (isShadow, raytracing.cpp:241-261). With no transparent material the verdict
// is "some triangle is hit at a distance < FLT_MAX", so lanes stop at their first such hit and
// the wave leaves the loop once every lane has one.
template <bool kAnyHit>
__global__ __launch_bounds__(kBlock) void k_shadow_hit(const TriRec *__restrict__ tris, int nt,
                                                       const uint32_t *__restrict__ tri_mat,
                                                       const DevMaterial *__restrict__ mats, const ShadowSource src,
                                                       uint8_t *__restrict__ shadow) {
    const int n = shadow_total(src);
    const int base = blockIdx.x * kBlock;
    if (base >= n) return;
    const int j = base + threadIdx.x;
    V3 o = mk(0, 0, 0), dir = mk(0, 0, 0);
    int slot = 0;
    const bool active = shadow_query(src, j, n, o, dir, slot);
    int bidx = -1;
    V3 bI = mk(0, 0, 0);
    if (__any(active)) closest_hit_loop<kAnyHit>(tris, nt, o, dir, active, bidx, bI);
    if (active) {
        uint8_t sh = 0;
        if (bidx >= 0) sh = mats[tri_mat[bidx]].transparent ? 0 : 1;               // :253-257
        shadow[slot] = sh;
    }
    add_pair_count(src, active ? 1u : 0u);
}

__global__ __launch_bounds__(kBlock) void k_intersect_only(const TriRec *__restrict__ tris, int nt,
                                                           const float4 *__restrict__ q_org,
                                                           const float4 *__restrict__ q_dst, int n,
                                                           int32_t *__restrict__ idx, float4 *__restrict__ I) {
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (blockIdx.x * kBlock >= n) return;
    const bool active = j < n;
    V3 o = mk(0, 0, 0), dir = mk(0, 0, 0);
    if (active) {
        const float4 qo = q_org[j], qd = q_dst[j];
        o = mk(qo.x, qo.y, qo.z);
        dir = mk(qd.x - qo.x, qd.y - qo.y, qd.z - qo.z);
    }
    int bidx = -1;
    V3 bI = mk(0, 0, 0);
    closest_hit_loop<false>(tris, nt, o, dir, active, bidx, bI);
    if (active) { idx[j] = bidx; I[j] = make_float4(bI.x, bI.y, bI.z, 0.0f); }
}

// ---------------------------------------------------------------------------------------------
// Sample generation: main.cpp:377-386 for every sub-sample of the batch's tiles.
// ---------------------------------------------------------------------------------------------
// (Indices are below 2^31: batches are capped at 2^30 samples and tile ids at 2^30, rt_capi.cpp.)
// The even bits of v packed into its low half (Morton decode of one coordinate).
__device__ __forceinline__ uint32_t compact_bits(uint32_t v) {
    v &= 0x55555555u;
    v = (v | (v >> 1)) & 0x33333333u;
    v = (v | (v >> 2)) & 0x0F0F0F0Fu;
    v = (v | (v >> 4)) & 0x00FF00FFu;
    return (v | (v >> 8)) & 0x0000FFFFu;
}

// Pixel pix of a batch (tile-major: tile tl = pix / (tw th), then the tile's pixels in g.pix_order):
// its frame position and its slot in the tile-major shard layout, where a tile is always row-major
// (rt_assemble_tiles_device's layout, whatever order the samples take).
__device__ __forceinline__ bool decode_pixel(const FrameGeom &g, int64_t pix64, int &x, int &y, uint32_t &slot) {
    const uint32_t pix = static_cast<uint32_t>(pix64);
    const uint32_t tl = udiv(pix, g.div_tpx);
    const uint32_t p = pix - tl * g.div_tpx.d;
    const uint32_t tid = umod(static_cast<uint32_t>(g.first) + (static_cast<uint32_t>(g.tile0) + tl) * static_cast<uint32_t>(g.stride),
                              g.div_tiles);
    const uint32_t ty = udiv(tid, g.div_tx), tx = tid - ty * g.div_tx.d;
    uint32_t py, pxl;
    if (g.pix_order) { pxl = compact_bits(p); py = compact_bits(p >> 1); }   // Morton (tw = th = 2^k)
    else { py = udiv(p, g.div_tw); pxl = p - py * g.div_tw.d; }
    slot = tl * g.div_tpx.d + py * g.div_tw.d + pxl;
    x = g.ox + static_cast<int>(tx) * g.tw + static_cast<int>(pxl);
    y = g.oy + static_cast<int>(ty) * g.th + static_cast<int>(py);
    return x < g.width && y < g.height && x < g.ox + g.cw && y < g.oy + g.ch && x >= 0 && y >= 0;
}

// The primary queue is dense: query s is sample s, so no compaction (and no atomics) at all;
// samples outside the frame or the clip rectangle are marked inactive with lvl = -1.
// MurmurHash3 32-bit finaliser (the RT_STOCHASTIC jitter hash; oracle/rt_oracle.c has the same)
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// Sample s of a batch (main.cpp:355-395 for one sub-sample): its pixel, its output index px (the
// tile-major shard slot or the row-major index in the clip rectangle) and its primary ray; false for
// samples outside the frame or the clip rectangle (origin and dest then (0,0,0)).
// cs: the corner rays (g.corners, or a multi-frame launch's frame's: primary_sample_view)
__device__ __forceinline__ bool primary_sample_view(const FrameGeom &g, const float (*cs)[3], int64_t s, V3 &origin, V3 &dest,
                                                    int64_t &px, int &sub) {
    const int spp = g.pfx * g.pfy;
    const int64_t pix = udiv(static_cast<uint32_t>(s), g.div_spp);
    sub = static_cast<int>(s - pix * spp);
    const int subx = static_cast<int>(udiv(static_cast<uint32_t>(sub), g.div_pfy));
    const int suby = sub - subx * g.pfy;   // subx outer, suby inner (:377-378)
    int x, y;
    uint32_t slot;
    const bool valid = decode_pixel(g, pix, x, y, slot);
    px = g.out_mode == 0 ? static_cast<int64_t>(g.tile0) * g.tw * g.th + slot
                         : static_cast<int64_t>(y - g.oy) * g.cw + (x - g.ox);
    origin = mk(0, 0, 0);
    dest = mk(0, 0, 0);
    if (valid) {
        float fx = static_cast<float>(subx), fy = static_cast<float>(suby);
        if (g.stochastic) {   // RT_STOCHASTIC (include/raytracert.h): jitter inside the grid cell
            const uint32_t key = (static_cast<uint32_t>(y) * static_cast<uint32_t>(g.width) + static_cast<uint32_t>(x)) *
                                     static_cast<uint32_t>(spp) + static_cast<uint32_t>(sub);
            const uint32_t h1 = fmix32(key ^ fmix32(g.seed));
            const uint32_t h2 = fmix32(h1 + 0x9E3779B9u);
            fx = fx + static_cast<float>(h1 >> 8) * 0x1p-24f;
            fy = fy + static_cast<float>(h2 >> 8) * 0x1p-24f;
        }
        const float xscale = 1.0f - (static_cast<float>(static_cast<unsigned>(x)) * static_cast<float>(static_cast<unsigned>(g.pfx)) + fx) / g.divX;  // :380
        const float yscale = 1.0f - (static_cast<float>(static_cast<unsigned>(y)) * static_cast<float>(static_cast<unsigned>(g.pfy)) + fy) / g.divY;  // :381
        const V3 o00 = mk(cs[0][0], cs[0][1], cs[0][2]);
        const V3 d00 = mk(cs[1][0], cs[1][1], cs[1][2]);
        const V3 o01 = mk(cs[2][0], cs[2][1], cs[2][2]);
        const V3 d01 = mk(cs[3][0], cs[3][1], cs[3][2]);
        const V3 o10 = mk(cs[4][0], cs[4][1], cs[4][2]);
        const V3 d10 = mk(cs[5][0], cs[5][1], cs[5][2]);
        const V3 o11 = mk(cs[6][0], cs[6][1], cs[6][2]);
        const V3 d11 = mk(cs[7][0], cs[7][1], cs[7][2]);
        const float ix = 1 - xscale, iy = 1 - yscale;
        origin = add(scale(add(scale(o00, xscale), scale(o10, ix)), yscale),
                     scale(add(scale(o01, xscale), scale(o11, ix)), iy));                     // :383-384
        dest = add(scale(add(scale(d00, xscale), scale(d10, ix)), yscale),
                   scale(add(scale(d01, xscale), scale(d11, ix)), iy));                       // :385-386
    }
    return valid;
}
__device__ __forceinline__ bool primary_sample(const FrameGeom &g, int64_t s, V3 &origin, V3 &dest, int64_t &px, int &sub) {
    return primary_sample_view(g, g.corners, s, origin, dest, px, sub);
}

// Also resets the batch's queue counters and work-queue slots (counter 0 = the queue's size), so
// no separate fills precede the batch. resets_only (the fused chain launch follows, which makes
// each primary ray in its lane with primary_sample and writes the pixels itself): nothing else.
__global__ __launch_bounds__(kBlock) void k_gen_primary(const FrameGeom g, DevWork w, int resets_only, float *__restrict__ samples) {
    const int spp = g.pfx * g.pfy;
    const int64_t n = static_cast<int64_t>(g.ntiles) * g.tw * g.th * spp;
    const int64_t s = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (s < 2 * kMaxStepsCounters) w.counters[s] = s == 0 ? static_cast<int32_t>(n) : 0;
    if (s < 2 * static_cast<int64_t>(w.steps) * kWqSlot) w.wq[s] = 0;
    if (s >= n || resets_only) return;
    V3 origin, dest;
    int64_t px;
    int sub;
    const bool valid = primary_sample(g, s, origin, dest, px, sub);
    if (samples && valid) {   // out_mode 2 records with rays (rt_trace_frame_samples, RT_SAMPLES_RAY_RGB)
        float *r = samples + static_cast<int64_t>(g.sample_stride) * (px * g.pfx * g.pfy + sub);
        r[0] = origin.x; r[1] = origin.y; r[2] = origin.z; r[3] = dest.x; r[4] = dest.y; r[5] = dest.z;
    }
    w.depth[s] = 0;
    w.q_org[0][s] = make_float4(origin.x, origin.y, origin.z, as_float(static_cast<int>(s)));
    w.q_dst[0][s] = make_float4(dest.x, dest.y, dest.z, as_float(valid ? 0 : -1));
}

__global__ __launch_bounds__(kBlock) void k_gen_rays(const float4 *__restrict__ org, const float4 *__restrict__ dst,
                                                     int32_t n, DevWork w) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= n) return;
    if (s == 0) w.counters[0] = n;
    const float4 o = org[s], d = dst[s];
    w.q_org[0][s] = make_float4(o.x, o.y, o.z, as_float(s));
    w.q_dst[0][s] = make_float4(d.x, d.y, d.z, as_float(0));
    w.depth[s] = 0;
}

// ---------------------------------------------------------------------------------------------
// Shadow query generation: for each hit query and each light, origin = I + (0.1,0.1,0.1)
// (raytracing.cpp:246), destination = light position (:248).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_shadow_gen(const ShadeParams p, DevWork w) {
    const int L = p.n_lights;
    const int total = w.counters[p.step] * L;                  // (query, light) pairs
    for (int base = blockIdx.x * kBlock * kPer; base < total; base += gridDim.x * kBlock * kPer) {
        bool valid[kPer];
        int pos[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int slot = base + k * kBlock + threadIdx.x;
            valid[k] = slot < total && w.hit_idx[slot / L] >= 0;
        }
        block_reserve_rounds<kBlock, kPer>(valid, &w.counters[kMaxStepsCounters + p.step], pos);
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (!valid[k]) continue;
            const int slot = base + k * kBlock + threadIdx.x;
            const int j = slot / L, l = slot - j * L;
            const float4 I = w.hit_I[j];
            w.sq_org[pos[k]] = make_float4(I.x + 0.1f, I.y + 0.1f, I.z + 0.1f, as_float(slot));
            const V3 Lp = light_at(p.lights, p.light_ext, l);
            w.sq_dst[pos[k]] = make_float4(Lp.x, Lp.y, Lp.z, 0.0f);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// shade (raytracing.cpp:335-368) for one hit, plus the secondary ray it spawns.
// ---------------------------------------------------------------------------------------------
struct Secondary {
    uint32_t state;     // kChildNone / kChildTrace / kChildZero
    V3 coef;
    V3 org, dst;
    int lvl;
    V3 local;           // this step's local colour (shade's sum before the child's term)
    uint32_t code;      // in-lane chain records: state | coefficient kind << 2 | material << 3
};

// In-lane chain (the fused chain launch): a step's record is written only when the step has a
// child, as 16 B {local colour, code}, where the code names the child's coefficient by the hit
// material (kind 0: Ks, reflection and the acos branch of refraction; kind 1: (1 - Tr) broadcast,
// transmission: raytracing.cpp:298-328,361-363), so the fold re-derives the same floats; the
// chain's last step stays in registers and the lane folds its chain itself. (Against 32-B records
// of every step: bytes written past L2 265 -> 104 MB per C4 launch, time unchanged.)
constexpr uint32_t kCoefTr = 4u;

// A chain record store. RT_CHAIN_SC1 (A/B build): written through past L2 (sc1), so the records,
// read back once when the chain is folded, do not evict scene lines from the XCD's L2.
#ifndef RT_CHAIN_SC1
#define RT_CHAIN_SC1 1   // measured ~1.5% faster C4 frame (0.520 vs 0.528 ms)
#endif
// The asm form exists on gfx94x/gfx950 only (this library is built for gfx950); the compiler does
// not count the asm store in its vmcnt bookkeeping, which only makes its later waits stricter
// (vector memory operations complete in order), and the s_nop covers the store-data hazard.
__device__ __forceinline__ void store_chain(float4 *p, float4 v) {
#if defined(__gfx942__) || defined(__gfx950__)
    constexpr bool kSc1Asm = RT_CHAIN_SC1;
#else
    constexpr bool kSc1Asm = false;
#endif
    if (kSc1Asm) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 x = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
    } else {
        *p = v;
    }
}

// In-lane chain records of steps < RT_LDS_RECORDS live in LDS ([step][block lane], 16 B each: 12 KB per
// 256-lane block for 3 steps) instead of HBM: each is written and read back only by its own lane, so
// no synchronisation is needed; deeper steps (max_lvl > 3) use w.chain_local as before.
#ifndef RT_LDS_RECORDS
#define RT_LDS_RECORDS 3
#endif
__device__ __forceinline__ float4 *lds_records() {
    __shared__ float4 s_rec[(RT_LDS_RECORDS > 0 ? RT_LDS_RECORDS : 1) * kBvhBlock];
    return s_rec;
}
__device__ __forceinline__ void put_record(const DevWork &w, int step, int sample, float4 v) {
    if (RT_LDS_RECORDS > 0 && step < RT_LDS_RECORDS) lds_records()[step * kBvhBlock + static_cast<int>(threadIdx.x)] = v;
    else store_chain(&w.chain_local[static_cast<int64_t>(step) * w.rec_cap + sample], v);
}
__device__ __forceinline__ float4 get_record(const DevWork &w, int step, int sample) {
    if (RT_LDS_RECORDS > 0 && step < RT_LDS_RECORDS) return lds_records()[step * kBvhBlock + static_cast<int>(threadIdx.x)];
    return w.chain_local[static_cast<int64_t>(step) * w.rec_cap + sample];
}

// reflection (raytracing.cpp:277-285) + addOffset (:266-271): the traced ray of level `lvl`.
__device__ __forceinline__ void reflection_ray(V3 ray, V3 p, V3 normal, V3 &point, V3 &dest) {
    normalize(ray);
    const V3 R = sub(ray, scale(normal, 2.0f * dot(normal, ray)));
    point = p;
    dest = add(p, R);
    V3 v = sub(dest, point);
    normalize(v);
    v = scale(v, 0.01f);
    point = add(point, v);
}

__device__ __forceinline__ void offset_point(V3 &point, V3 dest) {   // addOffset
    V3 v = sub(dest, point);
    normalize(v);
    v = scale(v, 0.01f);
    point = add(point, v);
}

// shade (raytracing.cpp:335-368) for a hit of the chain step `step`: writes the step's chain
// record (local colour and child state, the child's coefficient, the depth when the chain ends)
// and returns the secondary ray, if any. ray = dest - origin of the traced ray (:393);
// is_shadowed(l) is isShadow's verdict for light l.
#ifndef RT_HOIST_VIEW
#define RT_HOIST_VIEW 1   // r04 one frame per launch: C4 equal, C5 6.85 -> 6.89 ms (profiles/r04_ab_hoist_view.txt);
                          // r05 multi-frame launches (VALU-bound): C4 0.3398 -> 0.3395, C5 6.637 -> 6.589 ms
                          // (profiles/r05o_ab_shade.txt)
#endif
#ifndef RT_HOIST_LNORM
#define RT_HOIST_LNORM 1   // diffuse's normalize(light position) from ShadeParams::lnorm (made on the host)
#endif
#ifndef RT_PAIR_CLOSEST
#define RT_PAIR_CLOSEST 1  // paired shadow helpers also in the closest-hit-shadow instantiations (scenes with transparency)
#endif
#ifndef RT_NORMAL_TABLE
#define RT_NORMAL_TABLE 0  // the hit normal's normalize() states from DevScene::ntab (k_normal_table). Measured
                           // (multi-frame launches): C5 (4 lights) 6.594 -> 6.566 ms, C4 (2 lights) 0.3400 ->
                           // 0.3410 ms (profiles/r05p_ab_normal_table.txt): the table's loads cost about what the
                           // normalisations did at 2 lights; off for the C4 headline
#endif
template <bool kInLane = false, bool kExtLights = true, typename Shadowed>
__device__ __forceinline__ Secondary shade_hit(const DevScene &sc, const ShadeParams &p, const DevWork &w, int step,
                                               int sample, V3 ray, int lvl, int idx, V3 P,
                                               Shadowed &&is_shadowed) {
    Secondary sec;
    sec.state = kChildNone;
    sec.org = mk(0, 0, 0);
    sec.dst = mk(0, 0, 0);
    sec.lvl = -1;
    const int64_t ci = static_cast<int64_t>(step) * w.rec_cap + sample, cc = static_cast<int64_t>(step) * w.cap + sample;
    const float4 nw = sc.normals[idx];
    V3 normal = ld3(nw);                                             // :394 (copy, mutated below)
    // normal.normalize() (:199, :213): from the face's tabled states when it has them (k_normal_table)
    const bool tabled = RT_NORMAL_TABLE && nw.w != 0.0f;
    int nstate = 0;
    auto renormalize = [&]() {
        if (tabled) { nstate ^= 1; normal = ld3(sc.ntab[2 * static_cast<int64_t>(idx) + (nstate ? 0 : 1)]); }
        else normalize(normal);
    };
    const uint32_t mi = sc.tri_mat[idx];
    const DevMaterial m = sc.mats[mi];                               // :396
    uint32_t kind = 0;
    const V3 Kd = mk(m.Kd[0], m.Kd[1], m.Kd[2]);
    const V3 Ka = mk(m.Ka[0], m.Ka[1], m.Ka[2]);
    const V3 Ks = mk(m.Ks[0], m.Ks[1], m.Ks[2]);
    const uint32_t f = p.flags;
    V3 color = mk(0, 0, 0);                                          // :336
    if ((f & RT_AMBIENT) && (m.flags & RT_HAS_KA)) color = add(color, Ka);   // :337-340
    // specular's view vector (:213-215) depends on neither the light nor the normal: the same bits for
    // every light, so RT_HOIST_VIEW 1 makes it once per hit (default 0: per light, as the loop is
    // written; holding it across the light loop measured slower)
    const bool spec_on = (f & RT_SPECULAR) && (m.flags & RT_HAS_KS) && (m.flags & RT_HAS_NS);
    V3 Vh = mk(0, 0, 0);
    if (RT_HOIST_VIEW && spec_on && p.n_lights > 0) {
        Vh = sub(mk(p.cam[0], p.cam[1], p.cam[2]), P);
        normalize(Vh);
    }
    for (int l = 0; l < p.n_lights; ++l) {                           // :342
        const V3 L = light_at<kExtLights>(p.lights, p.light_ext, l);
        const bool shadowed = (f & RT_SHADOWS) ? is_shadowed(l) : false;
        if (shadowed) continue;
        if ((f & RT_DIFFUSE) && (m.flags & RT_HAS_KD)) {             // diffuseOnly :197-205
            V3 diffuse = mk(0, 0, 0);
            renormalize();
            V3 lp = L;
            if (RT_HOIST_LNORM && (!kExtLights || l < RT_MAX_LIGHTS)) lp = mk(p.lnorm[l][0], p.lnorm[l][1], p.lnorm[l][2]);
            else normalize(lp);
            diffuse = add(diffuse, scale(Kd, max_std(dot(normal, lp), 0.0f)));
            color = add(color, scale(diffuse, m.Tr));                // :349
        }
        if (spec_on) {                                               // :210-232
            V3 spec = mk(0, 0, 0);
            V3 Vv = Vh;
            if (!RT_HOIST_VIEW) Vv = sub(mk(p.cam[0], p.cam[1], p.cam[2]), P);
            renormalize();
            if (!RT_HOIST_VIEW) normalize(Vv);
            V3 Lv = sub(L, P);
            normalize(Lv);
            V3 H = add(Vv, Lv);
            normalize(H);
            float st = max_std(dot(H, normal), 0.0f);
            st = spec_powf(st, m.Ns);
            spec = add(spec, scale(Ks, st));
            color = add(color, scale(spec, m.Tr));                   // :353
        }
    }
    if ((f & RT_REFRACTION) && (m.Tr < 1) && lvl < p.max_lvl) {     // :357-359 -> refraction :290-330
        const int rl = lvl + 1;
        V3 r = ray;
        normalize(r);
        const float check = dot(r, normal);
        sec.state = kChildZero;
        if (check < 0) {
            if (check >= kAcosLe2Threshold) {                        // 0 < acosf(check) <= 2
                sec.state = kChildTrace; sec.coef = Ks; sec.lvl = rl + 1;
                reflection_ray(r, P, normal, sec.org, sec.dst);
            } else {
                const float nr = 1 / m.Ni;
                const float root = 1 - m.powf_nr2 * (1 - glibc_powf2(dot(normal, r), sc.ties, sc.n_ties));
                if (root >= 0.0f) {
                    const float rt = sqrtf(root);
                    const V3 T = sub(scale(sub(r, scale(normal, dot(normal, r))), nr), scale(normal, rt));
                    sec.org = P;
                    sec.dst = add(P, T);
                    offset_point(sec.org, sec.dst);
                    sec.state = kChildTrace; sec.lvl = rl + 1;
                    const float c = 1 - m.Tr;
                    sec.coef = mk(c, c, c);
                    kind = kCoefTr;
                }
            }
        } else {
            const float nr = m.Ni;
            const V3 nn = neg(normal);
            const float root = 1 - m.powf_ni2 * (1 - glibc_powf2(dot(nn, r), sc.ties, sc.n_ties));
            if (root >= 0.0f) {
                const float rt = sqrtf(root);
                const V3 T = sub(scale(sub(r, scale(nn, dot(nn, r))), nr), scale(nn, rt));
                sec.org = P;
                sec.dst = add(P, T);
                offset_point(sec.org, sec.dst);
                sec.state = kChildTrace; sec.lvl = rl + 1;
                const float c = 1 - m.Tr;
                sec.coef = mk(c, c, c);
                kind = kCoefTr;
            }
        }
    } else if ((f & RT_REFLECTION) && lvl < p.max_lvl) {            // :361-363
        sec.state = kChildTrace; sec.coef = Ks; sec.lvl = lvl + 1;
        reflection_ray(ray, P, normal, sec.org, sec.dst);
    }
    sec.local = color;
    sec.code = sec.state | kind | (mi << 3);
    if (kInLane) {   // the caller keeps the chain (records of the steps with a child only)
        if (sec.state == kChildTrace) put_record(w, step, sample, make_float4(color.x, color.y, color.z, as_float(static_cast<int>(sec.code))));
        return sec;
    }
    store_chain(&w.chain_local[ci], make_float4(color.x, color.y, color.z, as_float(static_cast<int>(sec.state))));
    if (sec.state == kChildTrace) store_chain(&w.chain_coef[cc], make_float4(sec.coef.x, sec.coef.y, sec.coef.z, 0.0f));
    else w.depth[sample] = static_cast<uint8_t>(step + 1);
    return sec;
}

// The in-lane fold: the last step's colour c (its state applied) through the stored records of the
// steps first..last-1 back to front, c_k = local_k + coef_k * c_{k+1} (fold_chain's arithmetic).
__device__ __forceinline__ V3 fold_inlane(const DevScene &sc, const DevWork &w, int first, int last, int sample, V3 c) {
    for (int k = last - 1; k >= first; --k) {
        const float4 L = get_record(w, k, sample);
        const uint32_t code = static_cast<uint32_t>(as_int(L.w));
        const DevMaterial &m = sc.mats[code >> 3];
        V3 K;
        if (code & kCoefTr) { const float t = 1 - m.Tr; K = mk(t, t, t); }
        else K = mk(m.Ks[0], m.Ks[1], m.Ks[2]);
        c = add(mk(L.x, L.y, L.z), mul(K, c));
    }
    return c;
}

// trace() miss (:389-391): black, and the chain ends at this step.
__device__ __forceinline__ void shade_miss(const DevWork &w, int step, int sample) {
    store_chain(&w.chain_local[static_cast<int64_t>(step) * w.rec_cap + sample], make_float4(0, 0, 0, as_float(kChildNone)));
    w.depth[sample] = static_cast<uint8_t>(step + 1);
}

// One thread per query of the step's queue; the secondary rays go straight into the next
// step's queue, compacted with one atomic per 1,024-query block round (a single counter word
// takes only ~88 atomics/us, so per-wave appends are too slow).
constexpr int kShadeBlock = 1024;
__global__ __launch_bounds__(kShadeBlock) void k_shade(const DevScene sc, const ShadeParams p, DevWork w) {
    const int n = w.counters[p.step];
    const int nb = (p.step + 1) & 1;
    for (int base = blockIdx.x * kShadeBlock; base < n; base += gridDim.x * kShadeBlock) {   // uniform per block
        const int j = base + static_cast<int>(threadIdx.x);
        Secondary sec;
        sec.state = kChildNone;
        int sample = 0;
        const float4 qo = j < n ? w.q_org[p.step & 1][j] : make_float4(0, 0, 0, 0);
        const float4 qd = j < n ? w.q_dst[p.step & 1][j] : make_float4(0, 0, 0, as_float(-1));
        const int lvl = as_int(qd.w);
        if (lvl >= 0) {                                                   // inactive (outside frame) otherwise
            sample = as_int(qo.w);
            int idx = w.hit_idx[j];
            if (idx >= sc.nt) {                   // never expected: flag it for the host, do not fault
                w.counters[kErrorSlot] = 1;
                idx = -1;
            }
            if (idx < 0) {
                shade_miss(w, p.step, sample);
            } else {
                sec = shade_hit(sc, p, w, p.step, sample, sub(mk(qd.x, qd.y, qd.z), mk(qo.x, qo.y, qo.z)), lvl, idx,
                                ld3(w.hit_I[j]), [&](int l) { return w.shadow[j * p.n_lights + l] != 0; });
            }
        }
        bool spawn[1] = {sec.state == kChildTrace};
        int pos[1];
        block_reserve_rounds<kShadeBlock, 1>(spawn, &w.counters[p.step + 1], pos);
        if (spawn[0]) {
            w.q_org[nb][pos[0]] = make_float4(sec.org.x, sec.org.y, sec.org.z, as_float(sample));
            w.q_dst[nb][pos[0]] = make_float4(sec.dst.x, sec.dst.y, sec.dst.z, as_float(sec.lvl));
        }
    }
}

// Fold one sample's chain back to front: c_k = local_k + coef_k * c_{k+1} (the order in which
// shade() adds the value returned by the recursive trace(), raytracing.cpp:359,363).
__device__ __forceinline__ V3 fold_chain(const DevWork &w, int64_t s) {
    V3 c = mk(0, 0, 0);
    const int d = w.depth[s];
    for (int k = d - 1; k >= 0; --k) {
        const float4 L = w.chain_local[static_cast<int64_t>(k) * w.rec_cap + s];
        const uint32_t st = static_cast<uint32_t>(as_int(L.w));
        if (st == kChildTrace) {
            const float4 K = w.chain_coef[static_cast<int64_t>(k) * w.cap + s];
            c = add(mk(L.x, L.y, L.z), mul(mk(K.x, K.y, K.z), c));
        } else if (st == kChildZero) {
            c = add(mk(L.x, L.y, L.z), mk(0.0f, 0.0f, 0.0f));
        } else {
            c = mk(L.x, L.y, L.z);
        }
    }
    return c;
}

// RGBValue clamp (main.cpp:29-41) and the (unsigned char)(v*255) quantisation (main.cpp:117;
// NaN -> 0) of one pixel's averaged colour, at element offset o.
__device__ __forceinline__ void store_pixel(V3 rgb, int64_t o, uint8_t *__restrict__ out_u8, float *__restrict__ out_f32) {
    float c[3] = {rgb.x, rgb.y, rgb.z};
    for (int k = 0; k < 3; ++k) {
        float v = c[k];
        if (v > 1) v = 1.0f;
        if (v < 0) v = 0.0f;
        if (out_f32) out_f32[o + k] = v;
        if (out_u8) {
            const float q = v * 255.0f;
            out_u8[o + k] = (q == q) ? static_cast<uint8_t>(static_cast<int>(q)) : 0;
        }
    }
}

constexpr int kChainSteps = 256;   // max_lvl <= 254
#ifndef RT_MULTI_WPE
#define RT_MULTI_WPE RT_CHAIN_WPE   // the multi-frame instantiation's (A/B: its launches are VALU-bound)
#endif
#ifndef RT_CHAIN_WPE
#define RT_CHAIN_WPE 5   // r02, with in-lane chains: 5 (0.493-0.499 ms) vs 6 (0.533, more spills) vs 4 (0.51);
                         // r01, before them: 6 (80 VGPRs, 36 B spill) beat 5 (92, none) and 7
#endif

// One chain step of one sample (trace, raytracing.cpp:381-406): the closest-hit query, isShadow
// per light (:241-261), shade (:335-368). Returns the secondary ray (state kChildTrace) or the end
// of the chain. Shadow-ray statistics are counted per block in s_sh.
// Shadow helpers (split waves of the fused launch, RT_TUNE_SHADOW_HELPERS): with roles > 1 (wave-
// uniform) lane o < plen owns a sample and lanes o + r plen (r = 1 .. roles - 1) are its helpers:
// they take the owner's hit by lane shuffles and walk lights r, r + roles, ... while the owner walks
// lights 0, roles, ...; the owner ORs their verdicts into its mask and shades. Each light's walk is
// the same walk on the same ray whichever lane runs it, so the mask is the same bits.
// RT_LDS_PARK (A/B build): the step's values that only shading needs (the ray, lvl, the sample) wait
// in LDS ([word][lane] beside the traversal stack) while the walks run, so they hold no VGPRs there.
#ifndef RT_LDS_PARK
#define RT_LDS_PARK 0
#endif
// RT_OPAQUE_ARGS 1 (default, r04): the chain kernel reads its frame geometry, shading parameters,
// scene and workspace per wave batch through the kernel-argument pointer instead of holding them from
// its start: 232 SGPRs had spilled into four VGPRs' lanes and pushed 48 B per lane into scratch;
// now 72 and 24 B. C4 0.361 -> 0.348 ms per frame, C5 6.86 -> 6.68 ms, VALU -5.7%, WRITE_SIZE
// 116 -> 72 MB per launch (profiles/r04_ab_opaque_args.txt). 0: the arguments as the compiler places them.
// 2: the launch's scalar arguments (outputs, first step, split tiers) too: within the spread
// (profiles/r04_ab_opaque_args2.txt).
#ifndef RT_OPAQUE_ARGS
#define RT_OPAQUE_ARGS 1
#endif

constexpr int kParkWords = 8;   // words per lane of the park area: ray xyz, lvl, sample, pixel (k_chain)
struct Park {
    float *base;   // [kParkWords][kBvhBlock] in LDS, or null
    __device__ __forceinline__ void put(int k, float v) const { base[k * kBvhBlock + static_cast<int>(threadIdx.x)] = v; }
    __device__ __forceinline__ float get(int k) const { return base[k * kBvhBlock + static_cast<int>(threadIdx.x)]; }
};

template <bool kAnyHit, int W, bool kCount, bool kInLane = false, bool kSteal = false>
__device__ __forceinline__ Secondary chain_step(const DevScene &sc, const ShadeParams &p, const DevWork &w, int step,
                                                int sample, V3 org, V3 dst, int lvl, const LaneStack &stack, int *s_sh,
                                                WorkTally<kCount> &wc, WorkTally<kCount> &ws, bool live = true,
                                                bool pair = false, Park park = Park{nullptr}) {
    // kPair (the fused in-lane launch): every lane of the wave calls this at every step of its batch,
    // live or not (live: this lane's chain traces a ray at this step); with `pair`, once the closest
    // hits are known the lanes without a hit (chain ended, missed, or no sample) help the lanes with
    // one walk their shadow rays: with nh hit lanes and nd = 64 - nh others, each hit lane gets
    // G = min(L - 1, nd / nh) helpers (the same G for all, so the shadow phase is uniform), the group
    // walking lights role, role + G + 1, ... Each (hit, light) verdict is still one walk of the same
    // ray, so the mask, and every colour, is the one the owner alone would have made.
    constexpr bool kPair = kInLane && !kSteal && (kAnyHit || RT_PAIR_CLOSEST);
    Secondary none;
    none.state = kChildNone;
    none.local = mk(0, 0, 0);   // trace() miss: black (:389-391)
    int bidx = -1;
    V3 bI = mk(0, 0, 0);
    V3 ray = sub(dst, org);
    if (RT_LDS_PARK && park.base) {
        park.put(0, ray.x); park.put(1, ray.y); park.put(2, ray.z);
        park.put(3, as_float(lvl)); park.put(4, as_float(sample));
    }
    bvh_query_w<false, W, kSteal>(sc, org, ray, live, bidx, bI, stack, wc.tests, wc.visits);
    if (bidx >= sc.nt) { w.counters[kErrorSlot] = 1; bidx = -1; }
    const bool hit = live && bidx >= 0;
    if (!kPair && !hit) {
        if (!kInLane && live) shade_miss(w, step, sample);
        return none;
    }
    uint32_t mask = 0;   // isShadow per light (:241-261)
    const bool shadows = (p.flags & RT_SHADOWS) && p.n_lights > 0;
    if (shadows) {
        const int lane = __lane_id();
        int role = 0, G = 0, nh = 0, rk = 0, at_helper = 0;
        if (kPair && pair) {
            const unsigned long long hm = __ballot(hit);
            nh = __popcll(hm);
            G = nh ? min(p.n_lights - 1, (kWave - nh) / nh) : 0;   // (wave-uniform)
            if (G > 0) {
                rk = rank_below(hit ? hm : ~hm);   // rank among the hit (other) lanes
                // lane k receives the hit lane of rank k and the other lane of rank k (lane 63 takes the
                // unused writes: with G > 0 fewer than 64 lanes are of either kind); every lane runs the
                // permutes, which read nothing from a masked lane
                const int at_owner = __builtin_amdgcn_ds_permute(4 * (hit ? rk : kWave - 1), lane);
                at_helper = __builtin_amdgcn_ds_permute(4 * (hit ? kWave - 1 : rk), lane);
                const int owner = __builtin_amdgcn_ds_bpermute(4 * (rk % nh), at_owner);
                const bool helps = !hit && rk < G * nh;
                if (helps) role = 1 + rk / nh;
                const int src = helps ? owner : lane;   // helpers take their owner's hit
                bidx = __shfl(bidx, src);
                bI = mk(__shfl(bI.x, src), __shfl(bI.y, src), __shfl(bI.z, src));
            }
        }
        if (hit || role > 0) {
            if (role == 0) atomicAdd(&s_sh[step], p.n_lights);
            const V3 so = mk(bI.x + 0.1f, bI.y + 0.1f, bI.z + 0.1f);                // :248
            for (int l = role; l < p.n_lights; l += G + 1) {
                int sidx = -1;
                V3 sI = mk(0, 0, 0);
                const V3 Lp = light_at<false>(p.lights, p.light_ext, l);   // (the chain launch: <= RT_MAX_LIGHTS)
                const V3 sd = mk(Lp.x - so.x, Lp.y - so.y, Lp.z - so.z);
                bvh_query_w<kAnyHit, W, kSteal>(sc, so, sd, true, sidx, sI, stack, ws.tests, ws.visits);
                if (sidx >= 0 && !sc.mats[sc.tri_mat[sidx]].transparent) mask |= 1u << l;   // :253-257
            }
        }
        for (int r = 0; r < G; ++r) {   // an owner's helpers' verdicts (ranks rk, rk + nh, ... among the others)
            const int hl = __builtin_amdgcn_ds_bpermute(4 * min(rk + r * nh, kWave - 1), at_helper);
            const uint32_t m = static_cast<uint32_t>(__shfl(static_cast<int>(mask), hl));
            if (hit) mask |= m;
        }
    }
    if (!hit) return none;   // (a helper's or an idle lane's return value is not used)
    if (RT_LDS_PARK && park.base) {
        ray = mk(park.get(0), park.get(1), park.get(2));
        lvl = as_int(park.get(3));
        sample = as_int(park.get(4));
    }
    return shade_hit<kInLane, false>(sc, p, w, step, sample, ray, lvl, bidx, bI, [&](int l) { return ((mask >> l) & 1u) != 0; });
}

// chain_step for a quad (the quad walk): the four lanes hold the same sample and ray and run the same
// shading (each writes the same chain record); the closest-hit and every light's shadow query are
// quad walks. Ray statistics and work counts come from lane q == 0 (tests from the lane that ran each).
template <bool kAnyHit, bool kCount>
__device__ __forceinline__ Secondary chain_step_quad(const DevScene &sc, const ShadeParams &p, const DevWork &w, int step, int sample,
                                                     V3 org, V3 dst, int lvl, const QuadStack &st, int *s_sh, WorkTally<kCount> &wc,
                                                     WorkTally<kCount> &ws, int q, int qshift) {
    Secondary none;
    none.state = kChildNone;
    none.local = mk(0, 0, 0);   // trace() miss: black (:389-391)
    int bidx = -1;
    V3 bI = mk(0, 0, 0);
    const V3 ray = sub(dst, org);
    bvh4_query_quad<false>(sc, org, ray, true, bidx, bI, st, wc.tests, wc.visits, q, qshift);
    if (bidx >= sc.nt) { w.counters[kErrorSlot] = 1; bidx = -1; }
    if (bidx < 0) return none;
    uint32_t mask = 0;   // isShadow per light (:241-261)
    if ((p.flags & RT_SHADOWS) && p.n_lights > 0) {
        if (q == 0) atomicAdd(&s_sh[step], p.n_lights);
        const V3 so = mk(bI.x + 0.1f, bI.y + 0.1f, bI.z + 0.1f);                // :248
        for (int l = 0; l < p.n_lights; ++l) {
            int sidx = -1;
            V3 sI = mk(0, 0, 0);
            const V3 Lp = light_at<false>(p.lights, p.light_ext, l);
            const V3 sd = mk(Lp.x - so.x, Lp.y - so.y, Lp.z - so.z);
            bvh4_query_quad<kAnyHit>(sc, so, sd, true, sidx, sI, st, ws.tests, ws.visits, q, qshift);
            if (sidx >= 0 && !sc.mats[sc.tri_mat[sidx]].transparent) mask |= 1u << l;   // :253-257
        }
    }
    return shade_hit<true, false>(sc, p, w, step, sample, ray, lvl, bidx, bI, [&](int l) { return ((mask >> l) & 1u) != 0; });
}

// The chain launch: steps first..max_lvl of every query, each lane carrying its own ray through
// closest-hit, its shadow rays and shade until its chain ends. With no launch boundary between
// steps, a lane's next step does not wait for the slowest wave of the current one, which is what
// the thin last steps of a per-step wavefront spend their time on. The per-ray arithmetic is the
// per-step kernels' own (the same functions). Query counts per step (ray statistics) are summed per
// block in LDS and added to the step counters once at the end.
//
// Batches. The launch walks wave-sized batches: batch b is lanes 0..63 of one wave. kInLane (the
// fused frame launch, from step 0): batch b holds samples [b * spb, b * spb + spb) with spb =
// floor(64 / spp) * spp, so a pixel's spp sub-samples sit in adjacent lanes of one wave (pf 3: 7
// pixels x 9 sub-samples in 63 lanes); each lane makes its primary ray (main.cpp:377-386), folds its
// chain back to front in the lane (c_k = local_k + coef_k * c_{k+1}, the order in which trace()
// results are added, raytracing.cpp:359,363), and the wave sums a pixel's sub-samples with lane
// shuffles in k_frame's order and writes the pixel. Otherwise (a tail from step first > 0, or
// rt_trace_rays) batch b is queries [64 b, 64 b + 64) of the step's queue and the chain records
// go to HBM for k_frame / k_fold_rays.
// Batch order (ordered): virtual wave vb of the grid-stride walk takes batch w.batch_order[...];
// every wave records its batch's duration in w.batch_cost, from which launch_order_batches
// prepares the next launch's order (longest first, so the deep reflection chains of a frame start
// at once instead of trailing it). split (ordered stealing launches) = s2 | s4 << 16: the first s4
// batches of the order run as four waves of 16 lanes each, the next s2 as two waves of 32, so the
// other lanes of each are free to steal subtrees of the long walks from the start: virtual wave
// vb < 4 s4 is quarter vb & 3 of batch order[vb >> 2]; then vb - 4 s4 < 2 s2 is half (vb - 4 s4) & 1
// of batch order[s4 + ((vb - 4 s4) >> 1)]; later ones batch order[vb - 3 s4 - s2]. The host only
// splits when a part holds whole pixels (launch_chain). Placement never changes results.
// One part of a quarter-tier batch as a quad walk (RT_TUNE_QUAD_WALK): samples j0 .. j0 + n - 1, sample
// j0 + lane / 4 on the four lanes of a quad, each lane making the same primary ray, chain and fold;
// then the part's whole pixels are summed in sub-sample order across quads (k_frame's arithmetic) and
// written by the pixel's first quad's lane 0. n <= kQuadSamples (the host enables the tier only then).
template <bool kAnyHit, bool kCount>
__device__ __forceinline__ void quad_batch(const DevScene &sc, const ShadeParams &p, const DevWork &w, const FrameGeom &g,
                                           const float (*cs)[3], int32_t *lds_stack,
                                           int *s_q, int *s_sh, WorkTally<kCount> &wc, WorkTally<kCount> &ws, uint8_t *out_u8,
                                           float *out_f32, int spp, int j0, int n, int nq) {
    // (the lane-derived values are recomputed per part, behind an empty asm: hoisted to the kernel's
    // start, they stayed live through the per-lane path of the other batches and spilled there)
    int lane = __lane_id();
    asm volatile("" : "+v"(lane));
    const int sl = lane >> 2, q = lane & 3, qshift = lane & ~3;
    const QuadStack st = quad_stack(sc, lds_stack, lane);
    const int j = j0 + sl;
    V3 rgb = mk(0, 0, 0);
    int px = -1;
    if (sl < n && j < nq) {
        V3 org, dst;
        int64_t pxi = 0;
        int sub = 0;
        if (!primary_sample_view(g, cs, j, org, dst, pxi, sub)) {
            if (g.out_mode == 0 && out_u8 && sub == 0 && q == 0) { out_u8[3 * pxi] = 0; out_u8[3 * pxi + 1] = 0; out_u8[3 * pxi + 2] = 0; }
        } else {
            px = g.out_mode == 2 ? static_cast<int>(pxi) * spp + sub : static_cast<int>(pxi);
            if (g.out_mode == 2 && g.sample_stride == 9 && q == 0) {   // the record's ray (RT_SAMPLES_RAY_RGB)
                float *r = out_f32 + 9 * static_cast<int64_t>(px);
                r[0] = org.x; r[1] = org.y; r[2] = org.z; r[3] = dst.x; r[4] = dst.y; r[5] = dst.z;
            }
            int lvl = 0;
            for (int step = 0; step < kChainSteps; ++step) {
                if (step > 0 && q == 0) atomicAdd(&s_q[step], 1);
                const Secondary sec = chain_step_quad<kAnyHit, kCount>(sc, p, w, step, j, org, dst, lvl, st, s_sh, wc, ws, q, qshift);
                if (sec.state != kChildTrace) {   // the chain ends here: fold it (fold_chain's arithmetic)
                    rgb = fold_inlane(sc, w, 0, step, j, sec.state == kChildZero ? add(sec.local, mk(0.0f, 0.0f, 0.0f)) : sec.local);
                    break;
                }
                org = sec.org;
                dst = sec.dst;
                lvl = sec.lvl;
            }
        }
    }
    if (g.out_mode == 2) {   // every sub-sample's own colour (rt_trace_frame_samples)
        if (px >= 0 && q == 0) {
            float *o = out_f32 + static_cast<int64_t>(g.sample_stride) * px + (g.sample_stride - 3);
            o[0] = rgb.x; o[1] = rgb.y; o[2] = rgb.z;
        }
        return;
    }
    const int pix_sl = sl - sl % spp;   // the pixel's first sub-sample's quad
    V3 acc = mk(0, 0, 0);
    for (int sub = 0; sub < spp; ++sub) {   // summed in sub-sample order (main.cpp:377-391)
        const int src = min(pix_sl + sub, kQuadSamples - 1) * 4;
        acc = add(acc, mk(__shfl(rgb.x, src), __shfl(rgb.y, src), __shfl(rgb.z, src)));
    }
    const float div = static_cast<float>(spp);
    acc = mk(acc.x / div, acc.y / div, acc.z / div);   // operator/, Vec3D.h:36-38
    if (sl == pix_sl && q == 0 && px >= 0) store_pixel(acc, 3 * static_cast<int64_t>(px), out_u8, out_f32);
}

// k_chain's explicit arguments as laid out in the kernel-argument segment (in order, each at its
// natural alignment, as the members of a struct), for RT_OPAQUE_ARGS. The layout is a property of
// the kernel's signature, so it is checked once per kernel instantiation rather than per launch:
// probe_chain_kernargs launches k_chain_kernarg_probe, a kernel with k_chain's exact parameter list,
// which compares every argument with the ChainKernargs member at its place (chain_kernarg_mismatch)
// and reports a bit per argument.
#ifndef RT_KARGS_PERTURB
#define RT_KARGS_PERTURB 0   // test build only (librtamd_kargperturb.so): a layout the probe must reject
#endif
struct ChainKernargs {
    DevScene sc;
    ShadeParams p;
    DevWork w;
#if RT_KARGS_PERTURB
    int perturb;
#endif
    int first, ordered;
    uint8_t *out_u8;
    float *out_f32;
    int fuse_spp, spb, nbatch;
    FrameGeom g;
    int split, split8;
    FrameSet fs;
};
// the kernel-argument segment is at most 4 KB (the scene, the shading parameters with 16 lights, the
// workspace, the frame geometry and the multi-frame set are 2,032 B now): growth past it fails here
static_assert(sizeof(ChainKernargs) <= 4096, "k_chain's arguments exceed the 4 KB kernel-argument segment");

// Bit k set: argument k of k_chain is not where ChainKernargs places it. The probe launch fills each
// by-value structure with a word pattern (word i of argument k = kKargTag[k] + i, padding included,
// probe_chain_kernargs), so every word the struct view reads is checked against the bytes the
// runtime packed for that argument; the scalars and pointers are compared with the formal values
// (distinct sentinels). Bit 31 marks that the probe ran. (Taking the formals' addresses instead made
// the compiler copy them into 736 B of scratch per lane.)
constexpr uint32_t kKargTagScene = 0xA0000000u, kKargTagShade = 0xB0000000u, kKargTagWork = 0xC0000000u,
                   kKargTagGeom = 0xD0000000u, kKargTagFrames = 0xE0000000u;
template <typename T>
__device__ __forceinline__ uint32_t karg_words_differ(const __attribute__((address_space(4))) T *m, uint32_t tag) {
    const __attribute__((address_space(4))) uint32_t *u = (const __attribute__((address_space(4))) uint32_t *)m;
    uint32_t bad = 0;
    for (uint32_t i = 0; i < sizeof(T) / 4; ++i) bad |= static_cast<uint32_t>(u[i] != tag + i);
    return bad;
}
__device__ __forceinline__ uint32_t chain_kernarg_mismatch(int first, int ordered, uint8_t *out_u8, float *out_f32, int fuse_spp,
                                                           int spb, int nbatch, int split, int split8) {
    typedef const __attribute__((address_space(4))) ChainKernargs *KargPtr;
    const KargPtr ka = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t bad = 0x80000000u;
    bad |= karg_words_differ(&ka->sc, kKargTagScene) << 0;
    bad |= karg_words_differ(&ka->p, kKargTagShade) << 1;
    bad |= karg_words_differ(&ka->w, kKargTagWork) << 2;
    bad |= static_cast<uint32_t>(ka->first != first) << 3;
    bad |= static_cast<uint32_t>(ka->ordered != ordered) << 4;
    bad |= static_cast<uint32_t>(ka->out_u8 != out_u8) << 5;
    bad |= static_cast<uint32_t>(ka->out_f32 != out_f32) << 6;
    bad |= static_cast<uint32_t>(ka->fuse_spp != fuse_spp) << 7;
    bad |= static_cast<uint32_t>(ka->spb != spb) << 8;
    bad |= static_cast<uint32_t>(ka->nbatch != nbatch) << 9;
    bad |= karg_words_differ(&ka->g, kKargTagGeom) << 10;
    bad |= static_cast<uint32_t>(ka->split != split) << 11;
    bad |= static_cast<uint32_t>(ka->split8 != split8) << 12;
    bad |= karg_words_differ(&ka->fs, kKargTagFrames) << 13;
    return bad;
}
template <int W, bool kAnyHit, bool kCount, bool kInLane = false, bool kSteal = false, bool kQuad = false, bool kMulti = false>
__global__ __launch_bounds__(kBvhBlock) __attribute__((amdgpu_waves_per_eu(kSteal ? RT_STEAL_WPE : kMulti ? RT_MULTI_WPE : RT_CHAIN_WPE))) void k_chain(
    const DevScene sc, const ShadeParams p, DevWork w, int first, int ordered, uint8_t *__restrict__ out_u8,
    float *__restrict__ out_f32, int fuse_spp, int spb, int nbatch, const FrameGeom g, int split, int split8, const FrameSet fs) {
    extern __shared__ int32_t lds_stack[];
    __shared__ int s_q[kChainSteps], s_sh[kChainSteps];
#if RT_LDS_PARK
    __shared__ float s_park[kParkWords * kBvhBlock];
    const Park park{s_park};
#else
    const Park park{nullptr};
#endif
    for (int i = threadIdx.x; i < kChainSteps; i += kBvhBlock) { s_q[i] = 0; s_sh[i] = 0; }
#if RT_OPAQUE_ARGS
    {   // a per-launch spot check of six fields besides the load-time probe (k_chain_kernarg_probe checks
        // every word): a mismatch sets the error slot and ends the launch. (A NaN corner is not one.
        // Without this block the compiler allocates the kernel's registers differently: 28 instead of
        // 24 B of spill per lane.)
        typedef const __attribute__((address_space(4))) ChainKernargs *KargPtr;
        const KargPtr ka = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
        if (ka->g.width != g.width || ka->p.n_lights != p.n_lights || ka->nbatch != nbatch || ka->split8 != split8 ||
            ka->p.max_lvl != p.max_lvl || (ka->g.corners[7][2] != g.corners[7][2] && g.corners[7][2] == g.corners[7][2])) {
            if (threadIdx.x == 0) w.counters[kErrorSlot] = 1;
            return;
        }
    }
#endif
    __syncthreads();
    const LaneStack stack = lane_stack(sc, lds_stack);
    WorkTally<kCount> wc, ws;   // closest-hit and shadow work (totals only: lanes diverge here)
    const int nq = kInLane ? static_cast<int>(static_cast<int64_t>(g.ntiles) * g.tw * g.th * g.pfx * g.pfy)
                           : w.counters[first];
    if (kInLane && w.counters_next) {   // k_gen_primary's resets, for the next launch (Pipe::cnt_buf)
        const int i0 = blockIdx.x * kBvhBlock + threadIdx.x;   // (this launch's counters: already zero)
        for (int i = i0; i < 2 * kMaxStepsCounters; i += gridDim.x * kBvhBlock) w.counters_next[i] = 0;
        if (i0 == 0) w.counters[0] = nq;
    }
    if (!kInLane) nbatch = (nq + kWave - 1) / kWave;   // (spb = 64)
    const int s2 = split & 0xFFFF, s4 = split >> 16, extra = 7 * split8 + 3 * s4 + s2;
    const int lane = __lane_id();
    const int spp = kInLane ? fuse_spp : 1, ppb = spb / spp;   // sample lanes per pixel, pixels per batch
    // pixel base lane of this lane's sample (fused launches): the first lane of its spp-lane group
    // distribution 4 (fused launches): wave tasks dealt round-robin to the XCDs and taken one at a
    // time from per-XCD counters in the (self-reset) counter buffer by a resident grid, so no wave
    // slot waits for the other waves of its block to retire; in batch order when ordered
    const bool dyn = kInLane && sc.chain_split == 4;
    // a multi-frame launch (FrameSet): task t is frame t % nfr's task t / nfr
    // (its own instantiation, kMulti: the frame bookkeeping moved the default kernel's spill 32 -> 44 B)
    const int nfr = (kInLane && kMulti) ? max(1, fs.count) : 1;
    drive_queries((nbatch + extra) * kWave * nfr, dyn ? 4 : (sc.chain_split & 3), dyn ? &w.counters[kWaveQueueSlot] : w.wq + (2 * first) * kWqSlot,
                  [&](int j0, int vend) {
#if RT_OPAQUE_ARGS
        // the frame geometry, shading parameters, scene and workspace are read from the kernel
        // arguments through a pointer the compiler cannot follow across batches, so their scalar
        // loads stay in the batch loop instead of being hoisted to the kernel's start and held
        // (spilled into VGPR lanes, and those VGPRs into scratch) for its whole life
        typedef const __attribute__((address_space(4))) ChainKernargs *KargPtr;
        KargPtr ka = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ka));
        const FrameGeom &gl = *(const FrameGeom *)&ka->g;
        const ShadeParams &pl = *(const ShadeParams *)&ka->p;
        const DevScene &scb = *(const DevScene *)&ka->sc;
        const DevWork &wb = *(const DevWork *)&ka->w;
#if RT_OPAQUE_ARGS >= 2
        uint8_t *const out_u8 = ka->out_u8;
        float *const out_f32 = ka->out_f32;
        const int first = ka->first, ordered = ka->ordered, fuse_spp = kInLane ? ka->fuse_spp : 0, spb = kInLane ? ka->spb : kWave;
        const int split8 = ka->split8, s2 = ka->split & 0xFFFF, s4 = ka->split >> 16, extra = 7 * split8 + 3 * s4 + s2;
        const int spp = kInLane ? fuse_spp : 1, ppb = spb / spp;
#endif
#else
        const FrameGeom &gl = g;
        const ShadeParams &pl = p;
        const DevScene &scb = sc;
        const DevWork &wb = w;
#endif
        // this wave's virtual batch: wave-uniform in every distribution (xcd_segment hands out whole
        // 64-query chunks), so it and everything derived from it (frame, batch, split tier, part, the
        // order's entry) live in scalar registers
        const int vball = __builtin_amdgcn_readfirstlane(j0 >> 6);
        const int fr = nfr > 1 ? vball % nfr : 0, vb = nfr > 1 ? vball / nfr : vball;   // (its frame, its batch in it)
        // the frame's outputs, read where they are written (held from the batch's start, they stayed live
        // through the chain and spilled), and its corner rays
#if RT_OPAQUE_ARGS
        auto frame_out = [&](auto which) {
            KargPtr kb = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
            asm volatile("" : "+s"(kb));
            return which(nfr > 1, kb->fs.out_u8[fr], kb->fs.out_f32[fr], kb->out_u8, kb->out_f32);
        };
        const float(*const fcs)[3] = (const float(*)[3]) & ka->fs.corners[fr][0];
#else
        auto frame_out = [&](auto which) { return which(nfr > 1, fs.out_u8[fr], fs.out_f32[fr], out_u8, out_f32); };
        const float(*const fcs)[3] = fs.corners[fr];
#endif
        auto o8f = [&]() { return frame_out([](bool m, uint8_t *a, float *, uint8_t *c, float *) { return m ? a : c; }); };
        auto of32f = [&]() { return frame_out([](bool m, uint8_t *, float *b, uint8_t *, float *d) { return m ? b : d; }); };
        // split tiers of the order: 8 parts, then 4, then 2; part = which part of batch order[ob]
        int ob = vb - (ordered ? extra : 0), nparts = 1, part = 0;
        if (ordered) {
            const int v4 = vb - 8 * split8, v2 = v4 - 4 * s4;
            if (vb < 8 * split8) { nparts = 8; ob = vb >> 3; part = vb & 7; }
            else if (v4 < 4 * s4) { nparts = 4; ob = split8 + (v4 >> 2); part = v4 & 3; }
            else if (v2 < 2 * s2) { nparts = 2; ob = split8 + s4 + (v2 >> 1); part = v2 & 1; }
        }
        if (ordered) {   // the longest batches (and their parts) issue first on their SIMD
            if (ob < scb.prio_batches) __builtin_amdgcn_s_setprio(3);
            else __builtin_amdgcn_s_setprio(0);
        }
        const int plen = ((ppb + nparts - 1) / nparts) * spp;   // whole pixels per part
        const bool wave_on = (vball << 6) < vend;
        // the batch of this wave task: a scalar load of the order (written by other launches only; read
        // through a vector load its value was held in a VGPR across the batch and spilled)
        const int pb = (ordered && wave_on)
                           ? ((const __attribute__((address_space(4))) int32_t *)reinterpret_cast<uintptr_t>(wb.batch_order))[ob] : vb;
        const int lane_off = nparts > 1 ? part * plen + lane : (j0 & (kWave - 1));
        // (unordered, the XCD-segment distributions hand out unaligned ranges: the lane's own bound)
        const bool lane_on = (ordered ? wave_on : j0 < vend) && (nparts == 1 || lane < plen) && lane_off < spb;
        const int j = pb * spb + lane_off;   // this lane's sample (kInLane) or queue entry
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        V3 rgb = mk(0, 0, 0);   // fused pixels: this lane's folded chain and its pixel (valid samples)
        int px = -1;   // (out_mode 2: the sample's output slot, pixel x spp + sub-sample)
        // shadow helpers (RT_TUNE_SHADOW_HELPERS): at every step the lanes without a closest hit (a split
        // wave's lanes past the part's samples, chains that ended or missed) walk shadow rays for the
        // lanes with one (chain_step's kPair)
        // the quad walk (RT_TUNE_QUAD_WALK): a quarter-tier part's samples on four lanes each
        // (its own instantiation, kQuad: compiled into the default kernel the quad path's registers moved the
        // per-lane path's allocation from 24 to 92 B of spill per lane)
        const bool quad = kQuad && kInLane && !kSteal && W == 4 && nparts == 4 && scb.quad_walk && plen <= kQuadSamples;
        if (quad) {
            if (wave_on)
                quad_batch<kAnyHit, kCount>(scb, pl, wb, gl, nfr > 1 ? fcs : gl.corners, lds_stack, s_q, s_sh, wc, ws, o8f(), of32f(),
                                            fuse_spp, pb * spb + part * plen, min(plen, spb - part * plen), nq);
        } else {
        constexpr bool kPair = kInLane && !kSteal && (kAnyHit || RT_PAIR_CLOSEST);   // (every lane stays in the step loop, chain_step)
        const bool pair = kPair && scb.shadow_helpers && (pl.flags & RT_SHADOWS) && pl.n_lights > 1;
        [&]() {
        bool own = lane_on && j < nq;
        V3 org = mk(0, 0, 0), dst = mk(0, 0, 0);
        int lvl = 0, sample = 0;
        if (kInLane) {   // sample j: its primary ray, as k_gen_primary makes it
            int64_t pxi = 0;
            int sub = 0;
            if (own && !(nfr > 1 ? primary_sample_view(gl, fcs, j, org, dst, pxi, sub) : primary_sample(gl, j, org, dst, pxi, sub))) {
                uint8_t *const o8 = o8f();
                if (gl.out_mode == 0 && o8 && sub == 0) { o8[3 * pxi] = 0; o8[3 * pxi + 1] = 0; o8[3 * pxi + 2] = 0; }
                own = false;
            }
            own = own && lane_on;
            if (!kPair && !own) return;
            if (own) px = gl.out_mode == 2 ? static_cast<int>(pxi) * fuse_spp + sub : static_cast<int>(pxi);
            if (own && gl.out_mode == 2 && gl.sample_stride == 9) {   // the record's ray (RT_SAMPLES_RAY_RGB)
                float *r = of32f() + 9 * static_cast<int64_t>(px);
                r[0] = org.x; r[1] = org.y; r[2] = org.z; r[3] = dst.x; r[4] = dst.y; r[5] = dst.z;
            }
            lvl = 0;
            // (a multi-frame launch: frame fr's chain records past the LDS ones at j + fr x nq; the host sized
            // the workspace for nfr x nq samples, rt_capi.cpp frames_workspace_cap)
            sample = nfr > 1 ? j + fr * nq : j;
        } else {
            if (!own) return;
            const float4 qo = wb.q_org[first & 1][j], qd = wb.q_dst[first & 1][j];
            lvl = as_int(qd.w);
            if (lvl < 0) return;
            sample = as_int(qo.w);
            org = mk(qo.x, qo.y, qo.z);
            dst = mk(qd.x, qd.y, qd.z);
        }
        bool live = own;   // (kPair: lanes stay after their chain ends, as helpers; the loop ends with the wave's last chain)
        for (int step = first; step < kChainSteps; ++step) {
            if (kPair && !__any(live)) break;
            if (live && step > first) atomicAdd(&s_q[step], 1);
            const Secondary sec = chain_step<kAnyHit, W, kCount, kInLane, kSteal>(scb, pl, wb, step, sample, org, dst, lvl, stack,
                                                                                  s_sh, wc, ws, live, pair, park);
            if (!live) continue;
            if (sec.state != kChildTrace) {
                if (kInLane)   // the chain ends here: fold it in the lane (fold_chain's arithmetic)
                    rgb = fold_inlane(scb, wb, first, step, sample,
                                      sec.state == kChildZero ? add(sec.local, mk(0.0f, 0.0f, 0.0f)) : sec.local);
                live = false;
                if (!kPair) break;
                continue;
            }
            org = sec.org;
            dst = sec.dst;
            lvl = sec.lvl;
        }
        }();
        if (kInLane && gl.out_mode == 2) {   // every sub-sample's own colour (rt_trace_frame_samples)
            if (px >= 0) {
                float *o = of32f() + static_cast<int64_t>(gl.sample_stride) * px + (gl.sample_stride - 3);
                o[0] = rgb.x; o[1] = rgb.y; o[2] = rgb.z;
            }
        } else if (kInLane) {   // k_frame's arithmetic: a pixel's fuse_spp sub-samples sit in adjacent lanes
            // (the pixel's first lane and the divisor made here from the argument, not at the kernel's start:
            // held across the batch they were spilled to scratch and reloaded per batch)
#if RT_OPAQUE_ARGS
            KargPtr kf = (KargPtr)__builtin_amdgcn_kernarg_segment_ptr();
            asm volatile("" : "+s"(kf));
            const int fuse_spp = kf->fuse_spp;
#endif
            const int pix_lane = (fuse_spp & (fuse_spp - 1)) == 0 ? (lane & ~(fuse_spp - 1)) : lane - lane % fuse_spp;
            V3 acc = mk(0, 0, 0);
            for (int sub = 0; sub < fuse_spp; ++sub)   // summed in sub-sample order (main.cpp:377-391)
                acc = add(acc, mk(__shfl(rgb.x, pix_lane + sub), __shfl(rgb.y, pix_lane + sub), __shfl(rgb.z, pix_lane + sub)));
            const float div = static_cast<float>(fuse_spp);
            acc = mk(acc.x / div, acc.y / div, acc.z / div);   // operator/, Vec3D.h:36-38
            if (lane == pix_lane && px >= 0) store_pixel(acc, 3 * static_cast<int64_t>(px), o8f(), of32f());
        }
        }
        // the batch's lifetime (a split batch: its parts' lifetimes, the last to finish stored), with
        // bit 31 set for a split batch (kCostSplit): the sort counts it double, so a batch that ran
        // faster because it was split (or helped) stays at the head of the order instead of
        // dropping out of the split tier and back in on every re-sort
        if (lane == 0 && wave_on && wb.batch_cost) {   // (null: a launch with no pipeline order, rt_trace_rays)
            const uint32_t d = static_cast<uint32_t>(min(__builtin_amdgcn_s_memrealtime() - t0, 0x7FFFFFFFull));
            wb.batch_cost[pb] = nparts > 1 ? (d | kCostSplit) : d;
        }
    }, dyn ? sc.dyn_group_log2 : 0);
    wc.flush(sc.work);
    ws.flush(sc.work ? sc.work + kWorkFields : nullptr);
    __syncthreads();
    for (int i = threadIdx.x; i < kChainSteps; i += kBvhBlock) {
        if (s_q[i]) atomicAdd(&w.counters[i], s_q[i]);
        if (s_sh[i]) atomicAdd(&w.counters[kMaxStepsCounters + i], s_sh[i]);
    }
}

// Cold-launch cost estimate (RT_TUNE_COLD_ESTIMATE): a launch over batches with no measured order
// (a new view's first frame) is dispatched in screen order, so the deep chains of a hit-dense
// region start late and trail the launch (C4: 0.73 vs 0.43 ms ordered). This pre-pass traces one
// primary ray per wave batch (the batch's middle sample, closest hit, the same walk the chain uses)
// and scores the batch: the walk's node visits + triangle tests, times (1 + lights) when it hits
// (the shadow walks), times (1 + min(max_lvl, 3)) more when the hit material reflects or refracts
// (the chain continues). launch_order_batches sorts the scores like measured durations. Placement
// only: the chain launch that follows still traces every sample itself.
template <int W>
__global__ __launch_bounds__(kBvhBlock) void k_estimate(const DevScene sc, const ShadeParams p, const FrameGeom g, int spb,
                                                        int nbatch, uint32_t *__restrict__ score) {
    extern __shared__ int32_t lds_stack[];
    const LaneStack stack = lane_stack(sc, lds_stack);
    const int b = static_cast<int>(blockIdx.x) * kBvhBlock + static_cast<int>(threadIdx.x);
    const int nq = static_cast<int>(static_cast<int64_t>(g.ntiles) * g.tw * g.th * g.pfx * g.pfy);
    V3 org = mk(0, 0, 0), dst = mk(0, 0, 0);
    bool active = false;
    if (b < nbatch) {
        const int first = b * spb, n = min(spb, nq - first);
        int64_t pxi;
        int sub;
        active = primary_sample(g, first + n / 2, org, dst, pxi, sub);
    }
    unsigned tests = 0, visits = 0;
    int bidx = -1;
    V3 bI = mk(0, 0, 0);
    bvh_query_w<false, W>(sc, org, sub(dst, org), active, bidx, bI, stack, tests, visits);
    if (b >= nbatch) return;
    uint32_t s = 1 + tests + visits;
    if (bidx >= 0 && bidx < sc.nt) {
        s *= 1 + static_cast<uint32_t>(((p.flags & RT_SHADOWS) ? p.n_lights : 0));
        const DevMaterial &m = sc.mats[sc.tri_mat[bidx]];
        const bool refl = (p.flags & RT_REFLECTION) && (m.Ks[0] != 0 || m.Ks[1] != 0 || m.Ks[2] != 0);
        const bool refr = (p.flags & RT_REFRACTION) && m.Tr < 1;
        if (p.max_lvl > 0 && (refl || refr)) s *= 1 + static_cast<uint32_t>(min(p.max_lvl, 3));
    }
    score[b] = s;
}

// Center-out cold order (RT_TUNE_COLD_ESTIMATE 2): no walk at all; a batch scores by the distance of
// its middle pixel from the frame's centre (score 2^30 / (1 + d^2 / 64), pixels), so the sort starts
// the frame from the middle outward, where a view's subject and its long reflection chains usually
// are. Placement only, like the walk estimate.
__global__ __launch_bounds__(kBlock) void k_estimate_center(const FrameGeom g, int spb, int nbatch, uint32_t *__restrict__ score) {
    const int b = static_cast<int>(blockIdx.x) * kBlock + static_cast<int>(threadIdx.x);
    if (b >= nbatch) return;
    const int64_t nq = static_cast<int64_t>(g.ntiles) * g.tw * g.th * g.pfx * g.pfy;
    const int64_t first = static_cast<int64_t>(b) * spb, n = min(static_cast<int64_t>(spb), nq - first);
    const uint32_t pix = udiv(static_cast<uint32_t>(first + n / 2), g.div_spp);
    int x, y;
    uint32_t slot;
    decode_pixel(g, pix, x, y, slot);
    const float dx = static_cast<float>(x) + 0.5f - 0.5f * static_cast<float>(g.width);
    const float dy = static_cast<float>(y) + 0.5f - 0.5f * static_cast<float>(g.height);
    score[b] = static_cast<uint32_t>(1073741824.0f / (1.0f + (dx * dx + dy * dy) * (1.0f / 64.0f)));
}


// Frame: per pixel, sum sub-samples (subx outer, suby inner), divide by pf^2 (main.cpp:391),
// clamp (RGBValue, main.cpp:29-41), quantise with truncation (main.cpp:117; NaN -> 0).
__global__ __launch_bounds__(kBlock) void k_frame(const FrameGeom g, DevWork w, uint8_t *__restrict__ out_u8,
                                                  float *__restrict__ out_f32) {
    const int64_t npix = static_cast<int64_t>(g.ntiles) * g.tw * g.th;
    const int64_t pix = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (pix >= npix) return;
    int x, y;
    uint32_t slot;
    const bool valid = decode_pixel(g, pix, x, y, slot);
    const int spp = g.pfx * g.pfy;
    int64_t o;
    if (g.out_mode == 0) o = 3 * (static_cast<int64_t>(g.tile0) * g.tw * g.th + slot);
    else o = 3 * (static_cast<int64_t>(y - g.oy) * g.cw + (x - g.ox));
    if (!valid) {
        if (g.out_mode == 0 && out_u8) { out_u8[o] = 0; out_u8[o + 1] = 0; out_u8[o + 2] = 0; }
        return;
    }
    if (g.out_mode == 2) {   // every sub-sample's own colour, unclamped (rt_trace_frame_samples)
        for (int sub = 0; sub < spp; ++sub) {
            const V3 c = fold_chain(w, pix * spp + sub);
            float *q = out_f32 + static_cast<int64_t>(g.sample_stride) * (o / 3 * spp + sub) + (g.sample_stride - 3);
            q[0] = c.x; q[1] = c.y; q[2] = c.z;
        }
        return;
    }
    V3 rgb = mk(0, 0, 0);
    for (int sub = 0; sub < spp; ++sub) rgb = add(rgb, fold_chain(w, pix * spp + sub));
    const float div = static_cast<float>(spp);
    rgb = mk(rgb.x / div, rgb.y / div, rgb.z / div);                 // operator/, Vec3D.h:36-38
    store_pixel(rgb, o, out_u8, out_f32);
}

__global__ __launch_bounds__(kBlock) void k_fold_rays(DevWork w, int32_t n, float *__restrict__ rgb) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= n) return;
    const V3 c = fold_chain(w, s);
    rgb[3 * s] = c.x; rgb[3 * s + 1] = c.y; rgb[3 * s + 2] = c.z;
}

// Counting sort of the batches by duration, longest first: bucket = 4 x log2(ticks) plus the two
// bits below the leading one (quarter-octave buckets); within a bucket the order is arbitrary.
// (An order within eight screen bands, one per XCD, for L2 locality measured 40% slower: the bands'
// unequal costs leave XCDs idle. DESIGN.md §7.)
constexpr int kOrderBlock = 256;
__device__ __forceinline__ int order_bucket(uint32_t c) {
    if (c & kCostSplit) c = min((c & ~kCostSplit) * 2u, ~kCostSplit);   // a split batch counts double
    if (c < 4) return kOrderBuckets - 1;
    const int e = 31 - __clz(c);
    const int k = 4 * e + static_cast<int>((c >> (e - 2)) & 3u);
    return kOrderBuckets - 1 - min(k, kOrderBuckets - 1);   // descending duration
}

__global__ __launch_bounds__(kOrderBlock) void k_order_hist(const uint32_t *__restrict__ cost, int n, int32_t *hist) {
    __shared__ int h[kOrderBuckets];
    for (int i = threadIdx.x; i < kOrderBuckets; i += kOrderBlock) h[i] = 0;
    __syncthreads();
    for (int i = blockIdx.x * kOrderBlock + threadIdx.x; i < n; i += gridDim.x * kOrderBlock)
        atomicAdd(&h[order_bucket(cost[i])], 1);
    __syncthreads();
    for (int i = threadIdx.x; i < kOrderBuckets; i += kOrderBlock)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

__global__ __launch_bounds__(kOrderBuckets) void k_order_scan(int32_t *hist) {
    __shared__ int h[kOrderBuckets];
    h[threadIdx.x] = hist[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int i = 0; i < kOrderBuckets; ++i) { const int c = h[i]; h[i] = acc; acc += c; }
    }
    __syncthreads();
    hist[threadIdx.x] = h[threadIdx.x];   // bucket offsets; the scatter advances them
}

__global__ __launch_bounds__(kOrderBlock) void k_order_scatter(const uint32_t *__restrict__ cost, int n, int32_t *offs,
                                                            int32_t *__restrict__ order) {
    __shared__ int h[kOrderBuckets], base[kOrderBuckets];
    for (int i0 = blockIdx.x * kOrderBlock; i0 < n; i0 += gridDim.x * kOrderBlock) {   // block-uniform
        for (int i = threadIdx.x; i < kOrderBuckets; i += kOrderBlock) h[i] = 0;
        __syncthreads();
        const int i = i0 + static_cast<int>(threadIdx.x);
        int b = 0, r = 0;
        if (i < n) {
            b = order_bucket(cost[i]);
            r = atomicAdd(&h[b], 1);
        }
        __syncthreads();
        for (int k = threadIdx.x; k < kOrderBuckets; k += kOrderBlock)
            if (h[k]) base[k] = atomicAdd(&offs[k], h[k]);
        __syncthreads();
        if (i < n && base[b] + r < n) order[base[b] + r] = i;   // (counts are from the histogram pass: in range)
        __syncthreads();
    }
}


// calculateNormals (raytracing.cpp:78-86) on the device, one lane per triangle:
// normalize(crossProduct(v1 - v0, v2 - v0)) with Vec3D's operation order (Vec3D.h:142-151,185-191),
// so each normal is bit-identical to the host loader's (scene_loader.cpp compute_face_normals).
__global__ __launch_bounds__(kBlock) void k_face_normals(const float *__restrict__ xyz, const uint32_t *__restrict__ tri_v,
                                                         int32_t nt, float4 *__restrict__ normals) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= nt) return;
    const uint32_t ia = tri_v[3 * i], ib = tri_v[3 * i + 1], ic = tri_v[3 * i + 2];
    const V3 p0 = mk(xyz[3 * ia], xyz[3 * ia + 1], xyz[3 * ia + 2]);
    const V3 e01 = sub(mk(xyz[3 * ib], xyz[3 * ib + 1], xyz[3 * ib + 2]), p0);
    const V3 e02 = sub(mk(xyz[3 * ic], xyz[3 * ic + 1], xyz[3 * ic + 2]), p0);
    V3 n = mk(e01.y * e02.z - e01.z * e02.y, e01.z * e02.x - e01.x * e02.z, e01.x * e02.y - e01.y * e02.x);
    normalize(n);
    normals[i] = make_float4(n.x, n.y, n.z, 0.0f);
}

// shade() normalises the hit's normal in place once per diffuse and once per specular term of every lit
// light (diffuseOnly / blinnPhongSpecularOnly, raytracing.cpp:199,213): the k-th state of a face's normal
// is N^k(n). Where N(N(N(n))) == N(n) bit for bit (the states alternate from the first on: nearly every
// face), the two states are tabled once here with the kernels' own normalize, and shading picks state k
// by its parity instead of normalising again (w = 1 marks the face; otherwise shading normalises).
__global__ __launch_bounds__(kBlock) void k_normal_table(float4 *__restrict__ normals, float4 *__restrict__ ntab, int32_t nt) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= nt) return;
    const float4 n0 = normals[i];
    V3 n1 = mk(n0.x, n0.y, n0.z);
    normalize(n1);
    V3 n2 = n1;
    normalize(n2);
    V3 n3 = n2;
    normalize(n3);
    const bool ok = as_int(n3.x) == as_int(n1.x) && as_int(n3.y) == as_int(n1.y) && as_int(n3.z) == as_int(n1.z);
    ntab[2 * i] = make_float4(n1.x, n1.y, n1.z, 0.0f);
    ntab[2 * i + 1] = make_float4(n2.x, n2.y, n2.z, 0.0f);
    normals[i] = make_float4(n0.x, n0.y, n0.z, ok ? 1.0f : 0.0f);
}

// rayIntersectTriangle (raytracing.cpp:99-154) for n independent (ray, triangle) pairs, every
// step in the reference's order; unlike intersectMesh's use of it there is no distance compare, so
// a hit whose point is NaN or infinite is still reported, as the reference returns true for it.
// hit[i] = 1 and I[i] = the point, or 0 and (0,0,0).
__global__ __launch_bounds__(kBlock) void k_ray_triangle_pairs(const float *__restrict__ R, const float *__restrict__ T,
                                                               int32_t n, uint8_t *__restrict__ hit, float *__restrict__ I) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= n) return;
    const float *r = R + 6 * i, *t = T + 9 * i;
    V3 out = mk(0, 0, 0);
    uint8_t h = 0;
    do {
        const V3 T0 = mk(t[0], t[1], t[2]);
        const V3 u = sub(mk(t[3], t[4], t[5]), T0), v = sub(mk(t[6], t[7], t[8]), T0);            // :106-107
        const V3 nn = mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);      // :108
        if (nn.x == 0 && nn.y == 0 && nn.z == 0) break;                                             // :109
        const V3 o = mk(r[0], r[1], r[2]);
        const V3 dir = sub(mk(r[3], r[4], r[5]), o);                                                // :111
        const V3 w0 = sub(o, T0);                                                                   // :112
        const float b = dot(nn, dir);                                                               // :113
        const float a = -dot(nn, w0);                                                               // :114
        if (fabsf(b) < 0.00001f) break;                                                             // :115
        const float rr = a / b;                                                                     // :124
        if (rr < 0) break;                                                                          // :125
        const V3 Ip = add(o, scale(dir, rr));                                                       // :130
        const float uu = dot(u, u), uv = dot(u, v), vv = dot(v, v);                                 // :134-136
        const V3 w = sub(Ip, T0);                                                                   // :137
        const float wu = dot(w, u), wv = dot(w, v);                                                 // :138-139
        const float D = uv * uv - uu * vv;                                                          // :140
        const float ss = (uv * wv - vv * wu) / D;                                                   // :144
        if (ss < 0 || ss > 1) break;
        const float tt = (uv * wu - uu * wv) / D;                                                   // :148
        if (tt < 0 || (ss + tt) > 1) break;
        out = Ip;
        h = 1;
    } while (false);
    hit[i] = h;
    I[3 * i] = out.x; I[3 * i + 1] = out.y; I[3 * i + 2] = out.z;
}

// Un-permute of gathered tile shards (multi-GPU frame): gathered = [rank][nslots]
// tiles of tw x th x 3 bytes, the slots slot0 .. slot0 + nslots - 1 of every rank's shard (one gather
// chunk; the whole shard when slot0 = 0, nslots = slots); global tile id g = f * T + t is held by rank
// g % N in slot g / N. One thread per row of a gathered tile: it copies the row's (clipped) tw x 3
// bytes to the frame, in 16-B pieces when both ends are 16-B aligned (tw = 16 at 1920 wide: always).
// Index math per tile row, not per byte (the per-pixel form's 64-bit divisions cost ~20 us per C4
// frame).
__global__ __launch_bounds__(kBlock) void k_assemble_tiles(const uint8_t *__restrict__ gathered, int32_t width,
                                                           int32_t height, int32_t tw, int32_t th, int32_t tiles_x,
                                                           int32_t tiles_total, int32_t nranks, int64_t slot0,
                                                           int64_t nslots, int32_t frames, uint8_t *__restrict__ out) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const int64_t tile = i / th;   // gathered tile (rank-major), row r of it
    const int r = static_cast<int>(i - tile * th);
    if (tile >= nranks * nslots) return;
    const int64_t rank = tile / nslots, slot = slot0 + (tile - rank * nslots);
    const int64_t g = slot * nranks + rank;   // < 2^30 (rt_render_tiles_device's bound)
    if (g >= static_cast<int64_t>(frames) * tiles_total) return;   // a padding slot
    const int f = static_cast<int>(g / tiles_total), t = static_cast<int>(g - static_cast<int64_t>(f) * tiles_total);
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const int y = ty * th + r, x0 = tx * tw;
    if (y >= height) return;
    const int n = min(tw, width - x0) * 3;
    const uint8_t *src = gathered + (tile * tw * th + static_cast<int64_t>(r) * tw) * 3;
    uint8_t *dst = out + ((static_cast<int64_t>(f) * height + y) * width + x0) * 3;
    int k = 0;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0)
        for (; k + 16 <= n; k += 16)
            *reinterpret_cast<uint4 *>(dst + k) = *reinterpret_cast<const uint4 *>(src + k);
    for (; k < n; ++k) dst[k] = src[k];
}

// The same un-permute with one thread per 16-B piece of a gathered tile row and the index math in 32
// bits through the host's multiply-high divisors (launch_assemble_tiles takes it when every piece
// index fits 32 bits): three times the threads of the per-row form and no 64-bit divisions. C4 at
// 8 ranks: 8 frames in 0.0555 ms with the per-row form (1.8 TB/s of reads + writes).
struct AssembleDivs { UDiv ppr, th, nslots, tiles_total, tiles_x; };
__global__ __launch_bounds__(kBlock) void k_assemble_pieces(const uint8_t *__restrict__ gathered, int32_t width, int32_t height,
                                                            int32_t tw, int32_t th, int32_t tiles_x, int32_t tiles_total,
                                                            int32_t nranks, uint32_t slot0, uint32_t nslots, int32_t frames,
                                                            uint32_t npieces, AssembleDivs dv, uint8_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * static_cast<uint32_t>(kBlock) + threadIdx.x;
    if (i >= npieces) return;
    const uint32_t row = udiv(i, dv.ppr), piece = i - row * dv.ppr.d;
    const uint32_t tile = udiv(row, dv.th), r = row - tile * static_cast<uint32_t>(th);   // gathered tile (rank-major), its row
    const uint32_t rank = udiv(tile, dv.nslots), slot = slot0 + (tile - rank * nslots);
    const uint32_t g = slot * static_cast<uint32_t>(nranks) + rank;   // < 2^30 (rt_render_tiles_device's bound)
    if (g >= static_cast<uint32_t>(frames) * static_cast<uint32_t>(tiles_total)) return;   // a padding slot
    const uint32_t f = udiv(g, dv.tiles_total), t = g - f * static_cast<uint32_t>(tiles_total);
    const uint32_t ty = udiv(t, dv.tiles_x), tx = t - ty * static_cast<uint32_t>(tiles_x);
    const int y = static_cast<int>(ty) * th + static_cast<int>(r), x0 = static_cast<int>(tx) * tw;
    if (y >= height) return;
    const int n = min(tw, width - x0) * 3, k = static_cast<int>(piece) * 16;
    if (k >= n) return;
    const uint8_t *src = gathered + (static_cast<int64_t>(tile) * tw * th + static_cast<int64_t>(r) * tw) * 3 + k;
    uint8_t *dst = out + ((static_cast<int64_t>(f) * height + y) * width + x0) * 3 + k;
    if (k + 16 <= n && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
        *reinterpret_cast<uint4 *>(dst) = *reinterpret_cast<const uint4 *>(src);
    } else {
        for (int b = 0; b < 16 && k + b < n; ++b) dst[b] = src[b];
    }
}

// The un-permute of a whole gather of 16x16 tiles into frames whose width is a multiple of 16, staged
// through LDS so that both sides move whole lines: a block takes kAsmTiles consecutive tiles of one
// frame's tile row, reads each from its rank's shard (768 contiguous bytes) into LDS and writes the 16
// frame rows they cover as runs of kAsmTiles x 48 contiguous bytes. (k_assemble_pieces reads tile rows
// in order but writes them as 48-byte pieces 5,760 bytes apart; here no store is narrower than a run.)
#ifndef RT_ASM_ROWS
#define RT_ASM_ROWS 1   // 0: every un-permute through k_assemble_pieces (A/B)
#endif
constexpr int kAsmTiles = 16;
constexpr int kAsmTileBytes = 16 * 16 * 3;          // 768
constexpr int kAsmLdsStride = kAsmTileBytes + 48;   // (a pad that spreads a row's three tile reads over banks)
struct AssembleRowDivs { UDiv nranks, chunks, tiles_y; };
__global__ __launch_bounds__(kBlock) void k_assemble_rows(const uint8_t *__restrict__ gathered, int32_t width, int32_t height,
                                                          int32_t tiles_x, int32_t tiles_total, int32_t nranks, uint32_t nslots,
                                                          AssembleRowDivs dv, uint8_t *__restrict__ out) {
    __shared__ uint4 stage[kAsmTiles * kAsmLdsStride / 16];
    // block -> (frame f, tile row ty, tile chunk c)
    const uint32_t b = blockIdx.x;
    const uint32_t fr = udiv(b, dv.chunks), c = b - fr * dv.chunks.d;
    const uint32_t f = udiv(fr, dv.tiles_y), ty = fr - f * dv.tiles_y.d;
    const int tx0 = static_cast<int>(c) * kAsmTiles;
    const int ntiles = min(kAsmTiles, tiles_x - tx0);
    // read: kAsmTiles x 48 pieces of 16 B, each tile's 48 from its rank's slot
    for (int q = threadIdx.x; q < kAsmTiles * 48; q += kBlock) {
        const int k = q / 48, w = q - k * 48;
        if (k >= ntiles) continue;
        const uint32_t g = f * static_cast<uint32_t>(tiles_total) + ty * static_cast<uint32_t>(tiles_x) + static_cast<uint32_t>(tx0 + k);
        const uint32_t slot = udiv(g, dv.nranks), rank = g - slot * dv.nranks.d;
        const int64_t tile = static_cast<int64_t>(rank) * nslots + slot;
        stage[(k * kAsmLdsStride) / 16 + w] = reinterpret_cast<const uint4 *>(gathered + tile * kAsmTileBytes)[w];
    }
    __syncthreads();
    // write: 16 frame rows of ntiles x 48 bytes
    const int run = ntiles * 3;   // pieces of 16 B per row
    for (int q = threadIdx.x; q < 16 * kAsmTiles * 3; q += kBlock) {
        const int r = q / (kAsmTiles * 3), w = q - r * (kAsmTiles * 3);
        const int y = static_cast<int>(ty) * 16 + r;
        if (w >= run || y >= height) continue;
        const int k = w / 3, part = w - 3 * k;
        const uint4 v = stage[(k * kAsmLdsStride + r * 48) / 16 + part];
        uint8_t *dst = out + ((static_cast<int64_t>(f) * height + y) * width + static_cast<int64_t>(tx0) * 16) * 3;
        reinterpret_cast<uint4 *>(dst)[w] = v;
    }
}

inline unsigned grid_for(int64_t n) { return static_cast<unsigned>((n + kBlock - 1) / kBlock); }

}  // namespace

bool tri_rcp_records() { return RT_TRI_RCP != 0; }   // the records' D slot holds rD (test_triangle)

// The geometry's divisors as multiply-high magic numbers (fastdiv.h), for the kernels' index decoding.
static FrameGeom with_divisors(FrameGeom g) {
    g.div_spp = make_udiv(static_cast<uint32_t>(g.pfx * g.pfy));
    g.div_tpx = make_udiv(static_cast<uint32_t>(g.tw * g.th));
    g.div_tiles = make_udiv(static_cast<uint32_t>(std::max(g.tiles_total, 1)));
    g.div_tx = make_udiv(static_cast<uint32_t>(std::max(g.tiles_x, 1)));
    g.div_tw = make_udiv(static_cast<uint32_t>(g.tw));
    g.div_pfy = make_udiv(static_cast<uint32_t>(g.pfy));
    return g;
}

void launch_gen_primary(const FrameGeom &g, const DevWork &w, hipStream_t stream, bool resets_only, float *samples) {
    const int64_t n = static_cast<int64_t>(g.ntiles) * g.tw * g.th * g.pfx * g.pfy;
    if (n <= 0) return;
    const int64_t clear = std::max<int64_t>(2 * kMaxStepsCounters, 2 * static_cast<int64_t>(w.steps) * kWqSlot);
    hipLaunchKernelGGL(k_gen_primary, dim3(grid_for(resets_only ? clear : std::max(n, clear))), dim3(kBlock), 0, stream,
                       with_divisors(g), w, resets_only ? 1 : 0,
                       (!resets_only && g.out_mode == 2 && g.sample_stride == 9) ? samples : nullptr);
}

void launch_gen_rays(const float4 *org, const float4 *dst, int32_t n, const DevWork &w, hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_gen_rays, dim3(grid_for(n)), dim3(kBlock), 0, stream, org, dst, n, w);
}

// LDS part of the traversal stack: lds_stack entries per lane (the rest overflows to global)
inline size_t bvh_lds(const DevScene &s, int lanes = kBvhBlock) {
    return sizeof(int32_t) * lanes * static_cast<size_t>(std::max(s.lds_stack, 1));
}
inline DevScene for_width(DevScene s, int) { return s; }

// Grid cap of the per-step BVH kernels (resident size at 7 waves per SIMD: a grid-stride walk).
constexpr int kMaxBvhGrid = 4096;
inline unsigned grid_bvh(int64_t n, int cap = kMaxBvhGrid) {
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + kBvhBlock - 1) / kBvhBlock, cap)));
}
inline unsigned grid_chunked(int64_t n) {
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n + kBlock * kPer - 1) / (kBlock * kPer), kMaxGrid)));
}

template <int W>
void launch_ch(const DevScene &s0, const DevWork &w, int step, int64_t capacity, hipStream_t stream) {
    const DevScene s = for_width(s0, W);
    auto k = s.work ? k_bvh_closest_hit<W, true> : k_bvh_closest_hit<W, false>;
    hipLaunchKernelGGL(k, dim3(grid_bvh(capacity, s.bvh_grid)), dim3(kBvhBlock), bvh_lds(s), stream, s,
                       w.q_org[step & 1], w.q_dst[step & 1], &w.counters[step], w.hit_idx, w.hit_I,
                       w.wq + (2 * step) * kWqSlot);
}

void launch_closest_hit(const DevScene &s, const DevWork &w, int step, int64_t capacity, hipStream_t stream) {
    if (capacity <= 0) return;
    if (s.use_bvh) {
        if (s.bvh_width == 4) launch_ch<4>(s, w, step, capacity, stream);
        else launch_ch<2>(s, w, step, capacity, stream);
        return;
    }
    if (s.work) {   // the counting pass: stages reached per test (the brute-force roofline's work)
        hipLaunchKernelGGL(k_closest_hit_stages, dim3(grid_for(capacity)), dim3(kBlock), 0, stream, s.tris, s.nt,
                           w.q_org[step & 1], w.q_dst[step & 1], &w.counters[step], w.hit_idx, w.hit_I, s.work + 2 * kWorkFields);
        return;
    }
    hipLaunchKernelGGL(k_closest_hit, dim3(grid_for(capacity)), dim3(kBlock), 0, stream, s.tris, s.nt,
                       w.q_org[step & 1], w.q_dst[step & 1], &w.counters[step], w.hit_idx, w.hit_I);
}

void launch_shadow_gen(const DevScene &, const DevWork &w, const ShadeParams &p, int64_t capacity, hipStream_t stream) {
    const int64_t n = capacity * p.n_lights;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_shadow_gen, dim3(grid_chunked(n)), dim3(kBlock), 0, stream, p, w);
}

template <int W>
void launch_sh(const DevScene &s0, const DevWork &w, const ShadowSource &src, int step, int64_t capacity,
               hipStream_t stream) {
    const DevScene s = for_width(s0, W);
    auto k = s.any_transparent ? k_bvh_shadow_hit<false, W, false> : k_bvh_shadow_hit<true, W, false>;
    if (s.work) k = s.any_transparent ? k_bvh_shadow_hit<false, W, true> : k_bvh_shadow_hit<true, W, true>;
    hipLaunchKernelGGL(k, dim3(grid_bvh(capacity, s.bvh_grid)), dim3(kBvhBlock), bvh_lds(s), stream, s, src, w.shadow,
                       w.wq + (2 * step + 1) * kWqSlot);
}

void launch_shadow_hit(const DevScene &s, const DevWork &w, const ShadeParams &p, bool virt, int64_t capacity,
                       hipStream_t stream) {
    if (capacity <= 0) return;
    const int step = p.step;
    ShadowSource src{};
    src.sq_org = w.sq_org;
    src.sq_dst = w.sq_dst;
    src.count = virt ? &w.counters[step] : &w.counters[kMaxStepsCounters + step];
    src.hit_idx = w.hit_idx;
    src.hit_I = w.hit_I;
    src.pair_count = &w.counters[kMaxStepsCounters + step];
    src.n_lights = p.n_lights;
    src.virt = virt ? 1 : 0;
    for (int l = 0; l < RT_MAX_LIGHTS; ++l)
        for (int k = 0; k < 3; ++k) src.lights[l][k] = p.lights[l][k];
    src.light_ext = p.light_ext;
    if (s.use_bvh) {
        if (s.bvh_width == 4) launch_sh<4>(s, w, src, step, capacity, stream);
        else launch_sh<2>(s, w, src, step, capacity, stream);
        return;
    }
    if (s.any_transparent)
        hipLaunchKernelGGL(k_shadow_hit<false>, dim3(grid_for(capacity)), dim3(kBlock), 0, stream, s.tris, s.nt, s.tri_mat,
                           s.mats, src, w.shadow);
    else
        hipLaunchKernelGGL(k_shadow_hit<true>, dim3(grid_for(capacity)), dim3(kBlock), 0, stream, s.tris, s.nt, s.tri_mat,
                           s.mats, src, w.shadow);
}

void launch_shade(const DevScene &s, const DevWork &w, const ShadeParams &p, int64_t capacity, hipStream_t stream) {
    if (capacity <= 0) return;
    const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((capacity + kShadeBlock - 1) / kShadeBlock, 1024)));
    hipLaunchKernelGGL(k_shade, dim3(grid), dim3(kShadeBlock), 0, stream, s, p, w);
}

int chain_spb(int fuse_spp) { return fuse_spp > 0 && fuse_spp <= kWave ? (kWave / fuse_spp) * fuse_spp : kWave; }

int64_t chain_batches(int64_t capacity, int fuse_spp) {
    const int spb = chain_spb(fuse_spp);
    return (capacity + spb - 1) / spb;
}

// k_chain's instantiations by width, any-hit shadows, work counting, fused frame and stealing
typedef void (*ChainKernel)(const DevScene, const ShadeParams, DevWork, int, int, uint8_t *, float *, int, int, int,
                            const FrameGeom, int, int, const FrameSet);
// The layout probe: a kernel with exactly k_chain's parameter list (both are ChainKernel, checked
// below), so its kernel-argument segment is laid out as every k_chain instantiation's. It runs
// chain_kernarg_mismatch once. (Inside k_chain, even behind an early return, the check moved the
// register allocation: spill 24 -> 36 B per lane.)
__global__ __launch_bounds__(64) void k_chain_kernarg_probe(const DevScene sc, const ShadeParams p, DevWork w, int first, int ordered,
                                                           uint8_t *__restrict__ out_u8, float *__restrict__ out_f32, int fuse_spp,
                                                           int spb, int nbatch, const FrameGeom g, int split, int split8,
                                                           const FrameSet fs) {
    if (blockIdx.x == 0 && threadIdx.x == 0)
        *reinterpret_cast<uint32_t *>(out_u8) = chain_kernarg_mismatch(first, ordered, out_u8, out_f32, fuse_spp, spb, nbatch, split,
                                                                       split8);
}
static_assert(std::is_same<decltype(&k_chain_kernarg_probe), ChainKernel>::value, "the probe must have k_chain's parameters");
static_assert(std::is_same<decltype(&k_chain<4, true, false, true, false>), ChainKernel>::value, "k_chain's parameters changed");

template <int W, bool kInLane, bool kSteal, bool kQuad = false, bool kMulti = false>
ChainKernel chain_kernel(bool anyhit, bool count) {
    return anyhit ? (count ? k_chain<W, true, true, kInLane, kSteal, kQuad, kMulti> : k_chain<W, true, false, kInLane, kSteal, kQuad, kMulti>)
                  : (count ? k_chain<W, false, true, kInLane, kSteal, kQuad, kMulti> : k_chain<W, false, false, kInLane, kSteal, kQuad, kMulti>);
}

// k_chain_kernarg_probe once (one wave, tagged structures, sentinel scalars): *bad = its word unless
// 0x80000000 (0: the layout matches ChainKernargs).
hipError_t probe_chain_kernargs(hipStream_t stream, uint32_t *bad, int *which) {
    *bad = 0;
    *which = -1;
    uint32_t *d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(uint32_t));
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(d, 0, sizeof(uint32_t), stream);
    // word i of each by-value argument = its tag + i (padding included): what the struct view must read
    auto tagged = [](auto &obj, uint32_t tag) {
        uint32_t wds[sizeof(obj) / 4];
        for (uint32_t i = 0; i < sizeof(obj) / 4; ++i) wds[i] = tag + i;
        std::memcpy(&obj, wds, sizeof(obj));
    };
    DevScene sc;
    ShadeParams sp;
    DevWork w;
    FrameGeom g;
    FrameSet fs;
    tagged(sc, kKargTagScene);
    tagged(sp, kKargTagShade);
    tagged(w, kKargTagWork);
    tagged(g, kKargTagGeom);
    tagged(fs, kKargTagFrames);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_chain_kernarg_probe, dim3(1), dim3(64), 0, stream, sc, sp, w, 0x11, -1, reinterpret_cast<uint8_t *>(d),
                           reinterpret_cast<float *>(static_cast<uintptr_t>(0x1234560)), 0x21, 0x31, 0x41, g, 0x51, 0x61, fs);
        e = hipGetLastError();
    }
    uint32_t h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    const hipError_t ef = hipFree(d);
    if (e != hipSuccess) return e;
    if (h != 0x80000000u) { *bad = h ? h : 1u; *which = 0; }
    return ef;
}

void launch_chain(const DevScene &s0, const DevWork &w, const ShadeParams &p, int first, int64_t capacity,
                  hipStream_t stream, bool ordered, uint8_t *out_u8, float *out_f32, int fuse_spp, const FrameGeom *g,
                  const FrameSet *fs) {
    if (capacity <= 0) return;
    const bool wide = s0.bvh_width == 4;
    const DevScene s = for_width(s0, wide ? 4 : 2);
    const bool anyhit = !s.any_transparent, count = s.work != nullptr;
    // fused pixel writes from step 0: each lane makes its primary ray and folds its own chain
    const bool fused = fuse_spp > 0 && fuse_spp <= kWave && first == 0 && g != nullptr;
    // in-wave work stealing (RT_TUNE_WAVE_STEAL; 2 = when the launch is at most two rounds of
    // resident waves, where a few long walks set the frame time): four-wide, fused launches
    const int64_t resident_lanes = static_cast<int64_t>(std::max(s.resident_grid, 1)) * kBvhBlock;
    const bool steal = wide && fused && (s.wave_steal == 1 || (s.wave_steal == 2 && capacity <= 2 * resident_lanes));
    const int spb = fused ? chain_spb(fuse_spp) : kWave;
    const int64_t nbatch = fused ? chain_batches(capacity, fuse_spp) : (capacity + kWave - 1) / kWave;
    // ordered launches over grid-stride batches: the longest batches run as eighth, quarter and half
    // waves (at most 1/RT_STEAL_SPLIT_DIV of the batches together; each part holds whole pixels, as
    // a pixel's sub-samples are summed within one wave's lanes), so the longest chains of the frame
    // run on more SIMDs at once; in the stealing kernel a part's idle lanes steal from its walks
    int s2 = 0, s4 = 0, s8 = 0;
    if (ordered && (s.chain_split & 3) == 0) {
        const int ppb = spb / (fused ? fuse_spp : 1);
        int64_t cap = nbatch / RT_STEAL_SPLIT_DIV;
        if (ppb >= 8) { s8 = static_cast<int>(std::min<int64_t>(cap, s.split_eighth)); cap -= s8; }
        if (ppb >= 4) { s4 = static_cast<int>(std::min<int64_t>(cap, s.steal_quarter)); cap -= s4; }
        if (ppb >= 2) s2 = static_cast<int>(std::min<int64_t>(cap, s.steal_half));
    }
    // the quarter tier as quad walks (RT_TUNE_QUAD_WALK) when a quarter holds at most 16 samples
    const int ppb_f = fused ? spb / fuse_spp : 0;
    const bool quad = wide && fused && !steal && s.quad_walk && s4 > 0 && ((ppb_f + 3) / 4) * fuse_spp <= kQuadSamples;
    const bool multi = fused && wide && !quad && fs && fs->count > 1;   // (host: 4-wide fused launches only)
    ChainKernel k = (steal && multi) ? chain_kernel<4, true, true, false, true>(anyhit, count)
                  : steal  ? chain_kernel<4, true, true>(anyhit, count)
                  : multi  ? chain_kernel<4, true, false, false, true>(anyhit, count)
                  : quad   ? chain_kernel<4, true, false, true>(anyhit, count)
                  : fused  ? (wide ? chain_kernel<4, true, false>(anyhit, count) : chain_kernel<2, true, false>(anyhit, count))
                           : (wide ? chain_kernel<4, false, false>(anyhit, count) : chain_kernel<2, false, false>(anyhit, count));
    const int split = s2 | (s4 << 16);
    const FrameGeom geom = g ? with_divisors(*g) : FrameGeom{};
    // distribution 4 (dynamic wave tasks): a resident grid, each wave takes tasks until none remain
    const int resident = multi ? s.resident_grid * RT_MULTI_WPE / RT_CHAIN_WPE : s.resident_grid;   // (its own waves per EU)
    const int grid_cap = (fused && s.chain_split == 4) ? std::max(1, std::min(s.bvh_grid, resident)) : s.bvh_grid;
    FrameSet frames{};
    frames.count = 1;
    if (multi) frames = *fs;
    hipLaunchKernelGGL(k, dim3(grid_bvh((nbatch + 7 * s8 + 3 * s4 + s2) * kWave * frames.count, grid_cap)), dim3(kBvhBlock), bvh_lds(s),
                       stream, s, p, w, first, ordered ? 1 : 0, out_u8, out_f32, fused ? fuse_spp : 0, spb, static_cast<int>(nbatch),
                       geom, split, s8, frames);
}

void launch_estimate(const DevScene &s0, const ShadeParams &p, const FrameGeom &g, int fuse_spp, int64_t capacity,
                     uint32_t *score, hipStream_t stream) {
    const int64_t nbatch = chain_batches(capacity, fuse_spp);
    if (nbatch <= 0) return;
    if (s0.cold_estimate == 2) {
        hipLaunchKernelGGL(k_estimate_center, dim3(grid_for(nbatch)), dim3(kBlock), 0, stream, with_divisors(g),
                           chain_spb(fuse_spp), static_cast<int>(nbatch), score);
        return;
    }
    const bool wide = s0.bvh_width == 4;
    const DevScene s = for_width(s0, wide ? 4 : 2);
    const unsigned grid = static_cast<unsigned>((nbatch + kBvhBlock - 1) / kBvhBlock);
    hipLaunchKernelGGL(wide ? k_estimate<4> : k_estimate<2>, dim3(grid), dim3(kBvhBlock), bvh_lds(s), stream, s, p,
                       with_divisors(g), chain_spb(fuse_spp), static_cast<int>(nbatch), score);
}

int chain_blocks_per_cu() { return 4 * RT_CHAIN_WPE * kWave / kBvhBlock; }
int chain_lds_record_steps() { return RT_LDS_RECORDS; }
int bvh_block_threads() { return kBvhBlock; }

void launch_frame(const FrameGeom &g, const DevWork &w, uint8_t *out_u8, float *out_f32, hipStream_t stream) {
    const int64_t n = static_cast<int64_t>(g.ntiles) * g.tw * g.th;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_frame, dim3(grid_for(n)), dim3(kBlock), 0, stream, with_divisors(g), w, out_u8, out_f32);
}

// A moving view's batch order (RT_TUNE_MOTION_ORDER): the durations of the previous view, dilated over
// the screen, so a long batch that moved by a few pixels since is still near the head. Per batch its
// duration (a split one's doubled, as order_bucket counts it) goes into the 8 x 8-pixel cell of its
// middle sample (atomicMax), then each batch takes the maximum over the (2r + 1)^2 cells around its own.
__device__ __forceinline__ uint32_t order_cost(uint32_t c) { return (c & kCostSplit) ? min((c & ~kCostSplit) * 2u, ~kCostSplit) : c; }
__device__ __forceinline__ int order_cell(const FrameGeom &g, int spb, int nq, int b, int cells_x) {
    const int first = b * spb, n = min(spb, nq - first);
    const uint32_t pix = udiv(static_cast<uint32_t>(first + n / 2), g.div_spp);
    int x, y;
    uint32_t slot;
    decode_pixel(g, pix, x, y, slot);
    // a batch whose middle sample lies in a tile's padding (past the frame's edge) takes the nearest
    // cell inside the frame, so the index stays below cells_x x cells_y
    x = min(max(x, 0), g.width - 1);
    y = min(max(y, 0), g.height - 1);
    return (y >> 3) * cells_x + (x >> 3);
}
__global__ __launch_bounds__(kBlock) void k_order_cells(const uint32_t *__restrict__ cost, int n, const FrameGeom g, int spb, int nq,
                                                        int cells_x, uint32_t *__restrict__ cells) {
    const int b = static_cast<int>(blockIdx.x) * kBlock + static_cast<int>(threadIdx.x);
    if (b >= n) return;
    atomicMax(&cells[order_cell(g, spb, nq, b, cells_x)], order_cost(cost[b]));
}
__global__ __launch_bounds__(kBlock) void k_order_dilate(int n, const FrameGeom g, int spb, int nq, int cells_x, int cells_y,
                                                         int radius, const uint32_t *__restrict__ cells, uint32_t *__restrict__ out) {
    const int b = static_cast<int>(blockIdx.x) * kBlock + static_cast<int>(threadIdx.x);
    if (b >= n) return;
    const int c = order_cell(g, spb, nq, b, cells_x), cx = c % cells_x, cy = c / cells_x;
    uint32_t m = 0;
    for (int dy = -radius; dy <= radius; ++dy)
        for (int dx = -radius; dx <= radius; ++dx) {
            const int x = cx + dx, y = cy + dy;
            if (x >= 0 && x < cells_x && y >= 0 && y < cells_y) m = max(m, cells[y * cells_x + x]);
        }
    out[b] = m;
}

hipError_t launch_order_batches_moving(const DevWork &w, int64_t nbatches, const FrameGeom &g, int fuse_spp, int radius,
                                       uint32_t *dil_cost, uint32_t *cells, int64_t cells_cap, hipStream_t stream) {
    if (nbatches <= 0) return hipSuccess;
    const FrameGeom gd = with_divisors(g);
    const int cells_x = (g.width + 7) / 8, cells_y = (g.height + 7) / 8;
    if (static_cast<int64_t>(cells_x) * cells_y > cells_cap) return launch_order_batches(w, nbatches, stream);
    const int n = static_cast<int>(nbatches), spb = chain_spb(fuse_spp);
    const int nq = static_cast<int>(static_cast<int64_t>(g.ntiles) * g.tw * g.th * g.pfx * g.pfy);
    hipError_t e = hipMemsetAsync(cells, 0, sizeof(uint32_t) * static_cast<size_t>(cells_x) * cells_y, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_order_cells, dim3(grid_for(n)), dim3(kBlock), 0, stream, w.batch_cost, n, gd, spb, nq, cells_x, cells);
    hipLaunchKernelGGL(k_order_dilate, dim3(grid_for(n)), dim3(kBlock), 0, stream, n, gd, spb, nq, cells_x, cells_y, radius, cells,
                       dil_cost);
    DevWork wd = w;
    wd.batch_cost = dil_cost;
    return launch_order_batches(wd, nbatches, stream);
}

hipError_t launch_order_batches(const DevWork &w, int64_t nbatches, hipStream_t stream) {
    if (nbatches <= 0) return hipSuccess;
    const int n = static_cast<int>(nbatches);
    const hipError_t e = hipMemsetAsync(w.order_scratch, 0, sizeof(int32_t) * kOrderBuckets, stream);
    if (e != hipSuccess) return e;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>((nbatches + kOrderBlock - 1) / kOrderBlock, 1024));
    hipLaunchKernelGGL(k_order_hist, dim3(grid), dim3(kOrderBlock), 0, stream, w.batch_cost, n, w.order_scratch);
    hipLaunchKernelGGL(k_order_scan, dim3(1), dim3(kOrderBuckets), 0, stream, w.order_scratch);
    hipLaunchKernelGGL(k_order_scatter, dim3(grid), dim3(kOrderBlock), 0, stream, w.batch_cost, n, w.order_scratch,
                       w.batch_order);
    return hipGetLastError();
}

void launch_fold_rays(const DevWork &w, int32_t n, float *rgb, hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_fold_rays, dim3(grid_for(n)), dim3(kBlock), 0, stream, w, n, rgb);
}

void launch_intersect_only(const DevScene &s0, const float4 *org, const float4 *dst, int32_t n, int32_t *idx,
                           float4 *I, hipStream_t stream) {
    if (n <= 0) return;
    if (s0.use_bvh) {
        const int W = s0.bvh_width == 4 ? 4 : 2;
        const DevScene s = for_width(s0, W);
        auto k = W == 4 ? (s.work ? k_bvh_intersect_only<4, true> : k_bvh_intersect_only<4, false>)
                        : (s.work ? k_bvh_intersect_only<2, true> : k_bvh_intersect_only<2, false>);
        hipLaunchKernelGGL(k, dim3(grid_bvh(n, s.bvh_grid)), dim3(kBvhBlock), bvh_lds(s), stream, s, org, dst, n, idx, I);
        return;
    }
    hipLaunchKernelGGL(k_intersect_only, dim3(grid_for(n)), dim3(kBlock), 0, stream, s0.tris, s0.nt, org, dst, n, idx, I);
}

void launch_normal_table(float4 *normals, float4 *ntab, int32_t nt, hipStream_t stream) {
    if (nt <= 0) return;
    hipLaunchKernelGGL(k_normal_table, dim3(grid_for(nt)), dim3(kBlock), 0, stream, normals, ntab, nt);
}

void launch_face_normals(const float *xyz, const uint32_t *tri_v, int32_t nt, float4 *normals, hipStream_t stream) {
    if (nt <= 0) return;
    hipLaunchKernelGGL(k_face_normals, dim3(grid_for(nt)), dim3(kBlock), 0, stream, xyz, tri_v, nt, normals);
}

void launch_ray_triangle_pairs(const float *R, const float *T, int32_t n, uint8_t *hit, float *I, hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_ray_triangle_pairs, dim3(grid_for(n)), dim3(kBlock), 0, stream, R, T, n, hit, I);
}

void launch_assemble_tiles(const uint8_t *gathered, int32_t width, int32_t height, int32_t tw, int32_t th, int32_t frames,
                           int32_t nranks, uint8_t *out, hipStream_t stream, int64_t slot0, int64_t nslots) {
    const int32_t tiles_x = (width + tw - 1) / tw, tiles_total = tiles_x * ((height + th - 1) / th);
    const int64_t slots = (static_cast<int64_t>(frames) * tiles_total + nranks - 1) / nranks;
    if (nslots < 0) nslots = slots - slot0;   // (default: the whole shard)
    const int64_t rows = static_cast<int64_t>(nranks) * nslots * th;   // one thread per gathered tile row
    if (rows <= 0 || static_cast<int64_t>(frames) * width * height <= 0) return;
    const int64_t ppr = (static_cast<int64_t>(tw) * 3 + 15) / 16, npieces = rows * ppr;
    const int32_t tiles_y = tiles_total / tiles_x;
    const int64_t chunks = (tiles_x + kAsmTiles - 1) / kAsmTiles, blocks = static_cast<int64_t>(frames) * tiles_y * chunks;
    if (RT_ASM_ROWS && tw == 16 && th == 16 && width % 16 == 0 && slot0 == 0 && nslots == slots &&
        ((reinterpret_cast<uintptr_t>(gathered) | reinterpret_cast<uintptr_t>(out)) & 15) == 0 &&
        static_cast<int64_t>(frames) * tiles_total < (int64_t(1) << 32) && blocks < (int64_t(1) << 31)) {
        const AssembleRowDivs dv{make_udiv(static_cast<uint32_t>(nranks)), make_udiv(static_cast<uint32_t>(chunks)),
                                 make_udiv(static_cast<uint32_t>(tiles_y))};
        hipLaunchKernelGGL(k_assemble_rows, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, stream, gathered, width, height,
                           tiles_x, tiles_total, nranks, static_cast<uint32_t>(nslots), dv, out);
        return;
    }
    if (npieces < (int64_t(1) << 32) - kBlock && slot0 + nslots < (int64_t(1) << 32)) {
        const AssembleDivs dv{make_udiv(static_cast<uint32_t>(ppr)), make_udiv(static_cast<uint32_t>(th)),
                              make_udiv(static_cast<uint32_t>(nslots)), make_udiv(static_cast<uint32_t>(tiles_total)),
                              make_udiv(static_cast<uint32_t>(tiles_x))};
        hipLaunchKernelGGL(k_assemble_pieces, dim3(static_cast<unsigned>((npieces + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                           gathered, width, height, tw, th, tiles_x, tiles_total, nranks, static_cast<uint32_t>(slot0),
                           static_cast<uint32_t>(nslots), frames, static_cast<uint32_t>(npieces), dv, out);
        return;
    }
    hipLaunchKernelGGL(k_assemble_tiles, dim3(static_cast<unsigned>((rows + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       gathered, width, height, tw, th, tiles_x, tiles_total, nranks, slot0, nslots, frames, out);
}

}  // namespace rt
