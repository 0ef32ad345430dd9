// rt_kernels.h — launch interface of the gfx950 kernels (rt_kernels.hip) used by the render
// driver (rt_capi.cpp). Host-only declarations; no kernel code here.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fastdiv.h"
#include "rt_internal.h"

namespace rt {

// Chain step states (how shade() combines a level with its child, raytracing.cpp:357-363)
enum : uint32_t { kChildNone = 0, kChildTrace = 1, kChildZero = 2 };

// Where samples come from and where finished pixels go.
struct FrameGeom {
    int32_t width, height, pfx, pfy;    // frame and sub-sample grid (main.cpp:347,360-362)
    float divX, divY;                   // float(W*pf - 1), float(H*pf - 1)
    int32_t tw, th, tiles_x;            // tile size and tiles per row of the tiled region
    int32_t first, stride;              // tile id of batch tile i = first + (tile0 + i) * stride
    int32_t tile0, ntiles;              // this batch
    int32_t ox, oy, cw, ch;             // tiled region origin / clip size (absolute pixels)
    int32_t out_mode;                   // 0: tile-major shard layout, 1: row-major in the clip rect, 2: every
                                        // sub-sample's unclamped colour, row-major pixels x (subx, suby) (f32)
    int32_t tiles_total;                // tiles per frame: ids wrap modulo this (multi-frame batches)
    int32_t stochastic;                 // RT_STOCHASTIC: jittered sub-samples
    uint32_t seed;                      // its hash seed
    int32_t sample_stride;              // out_mode 2: floats per sample record (3: rgb; 9: origin, dest, rgb)
    int32_t pix_order;                  // pixels of a tile in sample order: 0 row-major, 1 Morton (square
                                        // power-of-two tiles: a 64-sample batch covers 8x8 pixels)
    float corners[8][3];                // origin00,dest00,origin01,dest01,origin10,dest10,origin11,dest11
    // divisions by the geometry, as multiply-high + shifts (fastdiv.h); the launchers fill them
    UDiv div_spp, div_tpx, div_tiles, div_tx, div_tw, div_pfy;
};

// A multi-frame chain launch (rt_render_frames_device): frames 0..count-1 of one frame geometry that
// differ only in their corner rays (views) and outputs. The launch's wave tasks cycle over the frames
// (task t: frame t % count, the frame's own task t / count), so the frames' longest batches start side
// by side and their short ones fill the slots the others' tails free, in one launch on one queue.
constexpr int kMaxFramesPerLaunch = 8;
struct FrameSet {
    int32_t count;                                  // 1: a single frame (the FrameGeom's corners and outputs)
    float corners[kMaxFramesPerLaunch][8][3];
    uint8_t *out_u8[kMaxFramesPerLaunch];
    float *out_f32[kMaxFramesPerLaunch];
};

struct ShadeParams {
    int32_t max_lvl;
    uint32_t flags;
    int32_t n_lights;
    int32_t step;
    float lights[RT_MAX_LIGHTS][3];     // the first RT_MAX_LIGHTS lights
    float cam[3];
    float pad;
    float lnorm[RT_MAX_LIGHTS][3];      // diffuseOnly's lightpos.normalize() of the first lights (Vec3D.h:142-151),
                                        // made on the host with the same float operations (shade_params)
    const float *light_ext;             // n_lights > RT_MAX_LIGHTS: all n_lights x 3 (device), else null
};

// Where a shadow kernel's queries come from (isShadow, raytracing.cpp:241-261). Compacted: the
// shadow queue k_shadow_gen wrote (sq_org/sq_dst, count). Virtual: query j is pair (j / L, j % L)
// of the step's main queue, read straight from its hits (origin hit_I + 0.1, destination the
// light); pairs whose query missed are inactive and the kernel counts the active ones into
// pair_count (the shadow-ray statistic k_shadow_gen's compaction would have produced).
struct ShadowSource {
    const float4 *sq_org, *sq_dst;
    const int32_t *count;           // compacted: queue size; virtual: the main queue's size
    const int32_t *hit_idx;
    const float4 *hit_I;
    int32_t *pair_count;
    int32_t n_lights, virt;
    float lights[RT_MAX_LIGHTS][3];
    const float *light_ext;         // as ShadeParams::light_ext
};

// Device views of one scene and one render workspace.
struct DevScene {
    const TriRec *tris;
    const uint32_t *tri_mat;
    const float4 *normals;          // xyz = face normal; w = 1: ntab holds its normalize() states
    const float4 *ntab;             // per face [N(n), N(N(n))] where N(N(N(n))) == N(n) bitwise (shade's
                                    // repeated normal.normalize(), Vec3D.h:142-151), k_normal_table
    const DevMaterial *mats;
    const uint32_t *ties;           // powf(x,2) tie table
    int32_t nt, nm, n_ties, any_transparent;
    // BVH (use_bvh != 0): nodes, leaf-ordered records and their original indices, always list
    const BvhNode *nodes;
    const TriRec *leaf_recs;
    const uint32_t *leaf_idx;
    const uint32_t *always;
    const TriRec *always_recs;      // the always list's records, contiguous
    int32_t use_bvh, n_always;
    float scene_m1;
    int32_t bvh_depth;              // traversal stack entries needed (tree depth)
    const Bvh4F *nodes4f;           // the four-wide tree (bvh_width == 4), float child boxes
    int32_t bvh_width;              // 2 or 4 (RT_TUNE_BVH_WIDTH)
    int32_t lds_stack;              // stack entries per lane held in LDS (<= entries needed)
    int32_t *stack_ovf;             // deeper entries: [entry - lds_stack][grid lane], grid <= bvh_grid
    int32_t xcd_split;              // RT_TUNE_XCD_SPLIT
    int32_t bvh_grid;               // RT_TUNE_BVH_GRID
    unsigned long long *work;       // BVH kernels' work counters: [0, kWorkFields) closest-hit, then shadow
    int32_t chain_split;            // RT_TUNE_CHAIN_SPLIT: query distribution of k_chain (as xcd_split)
    int32_t wave_steal;             // RT_TUNE_WAVE_STEAL: 0 off, 1 on, 2 when the chain launch is <= 2 wave rounds
    int32_t resident_grid;          // chain-kernel blocks resident on the device at once (CUs x blocks per CU)
    int32_t steal_half;             // RT_TUNE_STEAL_HALF: half-wave batches of the ordered stealing launch
    int32_t steal_quarter;          // RT_TUNE_STEAL_QUARTER: quarter-wave batches before them
    int32_t split_eighth;           // RT_TUNE_SPLIT_EIGHTH: eighth-wave batches before those
    int32_t cold_estimate;          // RT_TUNE_COLD_ESTIMATE: 1 primary-walk score, 2 centre-out
    int32_t dyn_group_log2;         // RT_TUNE_DYN_GROUP: log2 of the consecutive wave tasks dealt to one XCD
    int32_t prio_batches;           // RT_TUNE_PRIORITY_BATCHES: longest batches run at raised wave priority
    int32_t shadow_helpers;         // RT_TUNE_SHADOW_HELPERS: split waves' idle lanes walk their owners' lights
    int32_t quad_walk;              // RT_TUNE_QUAD_WALK: the quarter tier's waves walk with four lanes per ray
};

struct DevWork {
    float4 *q_org[2], *q_dst[2];    // ping-pong main query queues; org.w = sample id, dst.w = lvl (int bits)
    int32_t *hit_idx;
    float4 *hit_I;
    float4 *sq_org, *sq_dst;        // shadow queue; org.w = output slot (query * n_lights + light)
    uint8_t *shadow;                // per (query, light): 1 = in shadow
    float4 *chain_local;            // [step][sample]: xyz = local colour, w = child state (bits)
    float4 *chain_coef;             // [step][sample]: xyz = coefficient on the child's colour
    uint8_t *depth;                 // per sample: number of chain steps
    int32_t *counters;              // [step] main queue sizes (step 0 dense, incl. inactive), [kMaxStepsCounters + step] shadow
    int32_t *counters_next;         // in-lane fused chain launch: the next launch's counters, zeroed by this one (or null)
    int32_t *wq;                    // [2 * step + shadow] work-queue slots of kWqSlot ints (RT_TUNE_XCD_SPLIT 2)
    uint32_t *batch_cost;           // chain launch: per wave batch (chain_spb samples), its wave's duration (100 MHz ticks)
    int32_t *batch_order;           // chain launch: dispatch order of the batches (cost descending), or unused
    int32_t *order_scratch;         // counting-sort scratch (kOrderBuckets histogram, then offsets)
    int64_t cap;                    // samples per batch
    int32_t steps;                  // chain steps allocated (max_lvl + 1)
    int64_t rec_cap;                // chain_local's samples per step: cap x the frames of a multi-frame launch whose
                                    // records reach past the LDS ones (frame f's at sample + f x cap), else cap
};

constexpr int kMaxStepsCounters = 4096;   // counters[step] for main queues; [kMaxStepsCounters + step] shadow
constexpr int kErrorSlot = 2 * kMaxStepsCounters - 1;   // set by kernels on an internal inconsistency
constexpr int kWorkFields = 6;               // = RT_WORK_FIELDS
constexpr int kDiagWords = 1 << 17;          // diagnostic words after the work counters (rt_diag_read)
constexpr int kWqStride = 16;                // one 64-B line per segment counter
constexpr int kWqSlot = 8 * kWqStride;       // eight segments (one per XCD) per launch
// RT_TUNE_CHAIN_SPLIT 4 (fused chain launches): the eight per-XCD wave-task counters live in the
// counter buffer, below the step counters' upper half, so the launch before (or k_gen_primary) has
// zeroed them with the rest; max_lvl <= 254 keeps the step counters below this slot.
constexpr int kWaveQueueSlot = kMaxStepsCounters - kWqSlot;

// Launchers (all asynchronous on `stream`).
// k_gen_primary zeroes w.counters (then counter 0 = the batch's samples) and w.wq, and writes the
// step-0 queue of primary rays; resets_only (a fused chain launch follows, which makes its primary
// rays itself): only the resets.
// samples (out_mode 2, sample_stride 9): each valid sample's ray goes to its record too.
void launch_gen_primary(const FrameGeom &g, const DevWork &w, hipStream_t stream, bool resets_only = false,
                        float *samples = nullptr);
void launch_gen_rays(const float4 *org, const float4 *dst, int32_t n, const DevWork &w, hipStream_t stream);
void launch_closest_hit(const DevScene &s, const DevWork &w, int step, int64_t capacity, hipStream_t stream);
void launch_shadow_gen(const DevScene &s, const DevWork &w, const ShadeParams &p, int64_t capacity, hipStream_t stream);
void launch_shadow_hit(const DevScene &s, const DevWork &w, const ShadeParams &p, bool virt, int64_t capacity,
                       hipStream_t stream);
void launch_shade(const DevScene &s, const DevWork &w, const ShadeParams &p, int64_t capacity, hipStream_t stream);
void launch_frame(const FrameGeom &g, const DevWork &w, uint8_t *out_u8, float *out_f32, hipStream_t stream);
// Steps first..max_lvl of every query in Q_first in one launch (closest-hit, shadows, shade per lane).
// fuse_spp > 0 (first == 0, g = the batch's frame geometry, fuse_spp = samples per pixel <= 64): the
// fused frame launch. Each lane makes its sample's primary ray, folds its chain in the lane, and each
// wave writes its pixels into out_u8/out_f32 with k_frame's arithmetic (no k_gen_primary queue, no
// k_frame); a wave batch then holds chain_spb(fuse_spp) samples (whole pixels). Otherwise the queue
// Q_first is traced and the chain records go to HBM for k_frame / k_fold_rays.
// ordered: dispatch the wave batches by w.batch_order (the previous launch's measured durations).
int chain_blocks_per_cu();   // blocks of the chain kernels resident per CU (4 SIMDs x waves per EU x 64 / block)
int bvh_block_threads();     // threads per block of the BVH and chain kernels (RT_BVH_BLOCK)
int chain_lds_record_steps();   // fused chain launches keep the records of steps below this in LDS (RT_LDS_RECORDS)
int chain_spb(int fuse_spp);                            // samples per wave batch of a fused launch
int64_t chain_batches(int64_t capacity, int fuse_spp);  // wave batches of a launch over `capacity` samples
// fs (fused launches only, may be null): a multi-frame launch over fs->count views of g (FrameSet).
void launch_chain(const DevScene &s, const DevWork &w, const ShadeParams &p, int first, int64_t capacity,
                  hipStream_t stream, bool ordered = false, uint8_t *out_u8 = nullptr, float *out_f32 = nullptr,
                  int fuse_spp = 0, const FrameGeom *g = nullptr, const FrameSet *fs = nullptr);
void launch_fold_rays(const DevWork &w, int32_t n, float *rgb, hipStream_t stream);
// The chain kernels read their arguments through a struct view of the kernel-argument segment
// (RT_OPAQUE_ARGS): a probe kernel with k_chain's parameter list checks that view against the bytes
// the runtime packed for each argument. *bad = 0 when it matches, else the probe's word (bit k:
// argument k of k_chain; *which = 0). Synchronises `stream`.
hipError_t probe_chain_kernargs(hipStream_t stream, uint32_t *bad, int *which);
// Batch order: the chain launch's wave batches sorted by the durations it measured, longest first
// (w.batch_cost -> w.batch_order); the next launch over the same batches dispatches in that order
// (launch_chain(..., ordered = true)). A counting sort: one fill and three small launches.
constexpr int kOrderBuckets = 128;
constexpr uint32_t kCostSplit = 0x80000000u;   // batch_cost flag: the batch ran split (lifetime in bits 0-30)
constexpr int kWaveBatch = 64;   // lanes per wave batch of the chain launch (one sample per lane)
constexpr int kChainMaxLights = RT_MAX_LIGHTS;   // the chain launch reads its lights from its arguments; more: per-step kernels
hipError_t launch_order_batches(const DevWork &w, int64_t nbatches, hipStream_t stream);
// The same for a moving view (a fused frame launch g of fuse_spp samples per pixel): the durations
// dilated over (2 radius + 1)^2 cells of 8 x 8 pixels first (dil_cost: nbatches entries, cells: cells_cap
// entries >= ceil(width / 8) x ceil(height / 8), else the plain sort).
hipError_t launch_order_batches_moving(const DevWork &w, int64_t nbatches, const FrameGeom &g, int fuse_spp, int radius,
                                       uint32_t *dil_cost, uint32_t *cells, int64_t cells_cap, hipStream_t stream);
// A cold launch's batch scores (no measured order yet): one primary walk per wave batch of a fused
// launch (g, fuse_spp, capacity as launch_chain's), scored into score[batch] for launch_order_batches.
void launch_estimate(const DevScene &s, const ShadeParams &p, const FrameGeom &g, int fuse_spp, int64_t capacity,
                     uint32_t *score, hipStream_t stream);
void launch_intersect_only(const DevScene &s, const float4 *org, const float4 *dst, int32_t n,
                           int32_t *idx, float4 *I, hipStream_t stream);
// calculateNormals on the device (face normal per triangle into normals[i].xyz)
void launch_face_normals(const float *xyz, const uint32_t *tri_v, int32_t nt, float4 *normals, hipStream_t stream);
// True when this build's test_triangle reads RN(1/D) from the records' D slot (RT_TRI_RCP): the
// uploads then pass every record through tri_rcp_slot (rt_internal.h).
bool tri_rcp_records();
void launch_normal_table(float4 *normals, float4 *ntab, int32_t nt, hipStream_t stream);
// Un-permute gathered tile shards ([nranks][slots][th][tw][3], tile g of the frames x T tiles in
// rank g % nranks, slot g / nranks) into frames x height x width x 3 bytes; with slot0 / nslots, a
// gather chunk holding slots [slot0, slot0 + nslots) of every rank ([nranks][nslots][th][tw][3]).
void launch_assemble_tiles(const uint8_t *gathered, int32_t width, int32_t height, int32_t tw, int32_t th, int32_t frames,
                           int32_t nranks, uint8_t *out, hipStream_t stream, int64_t slot0 = 0, int64_t nslots = -1);
// rayIntersectTriangle for n (ray, triangle) pairs: R = n x (origin, dest), T = n x 3 vertices
void launch_ray_triangle_pairs(const float *R, const float *T, int32_t n, uint8_t *hit, float *I, hipStream_t stream);

}  // namespace rt
