/*
 * raytracert_tune.h — launch-shape tuning and tuning diagnostics of librtamd.so.
 *
 * NOT part of the drop-in contract (include/raytracert.h is): these entries exist for the library's
 * own A/B measurements, tests and benchmarks, and may change between releases. No knob changes a
 * result: every output byte is the same under every value (tests/test_gpu_parity.py and
 * tests/test_gpu_configs.py check each knob against the default). Nothing in the reference
 * corresponds to them (its render loop has no launch shape).
 */
#ifndef RAYTRACERT_TUNE_H
#define RAYTRACERT_TUNE_H

#include "raytracert.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- tuning (launch-shape knobs; results never depend on them) ------------------------- */
#define RT_TUNE_XCD_SPLIT 0   /* BVH queue distribution: 0 grid-stride, 1 one static segment per XCD,
                                 2 per-XCD segments with work-stealing wave counters */
#define RT_TUNE_BVH_GRID  1   /* grid cap (blocks of 256 threads) of the BVH kernels; default 16384: the
                                 chain launch then gives each wave one 64-sample batch of a C4 frame
                                 and the dispatcher balances the blocks */
#define RT_TUNE_BVH_WIDTH 2   /* 4 (default): quantised four-wide nodes; 2: float binary nodes */
#define RT_TUNE_LDS_STACK 3   /* traversal stack entries per lane kept in LDS; deeper ones in HBM */
#define RT_TUNE_PIPES     4   /* 1-4 render pipelines (workspace + stream) a call's batches overlap on
                                 (default 1) */
#define RT_TUNE_WAVE_TRAVERSAL 8   /* retired in r03 (only 0 accepted): the wave-coherent walk of the
                                      four-wide tree measured no faster on C4, primaries included */
#define RT_TUNE_CHAIN_FROM 9     /* chain steps from this one on run in one launch, each lane carrying
                                    its ray through closest-hit, shadows and shade (default 0;
                                    >= max_lvl + 1: every step its own launches) */
#define RT_TUNE_BATCH_ORDER 15  /* 1 (default): the chain launch dispatches its wave batches longest
                                    first, by the durations the pipeline's previous launch over the
                                    same batches measured (the first launch runs in screen order);
                                    0: screen order */
#define RT_TUNE_ORDER_EVERY 17  /* batch order re-sorted every this many launches over the same batches
                                    (default 8; 1: every launch); the durations are measured every time */
#define RT_TUNE_FUSE_PIXELS 18  /* 1 (default): the chain launch writes each pixel when its samples'
                                    chains end (no separate frame pass) when pfx*pfy <= 64 (a wave
                                    batch holds floor(64 / spp) whole pixels); 0: always the frame pass */
#define RT_TUNE_CHAIN_REFILL 19  /* retired in r03 (only 0 accepted): per-lane pixel refill measured 1.5x
                                    slower on C4 (a wave's rays lose their shared chain step) */
#define RT_TUNE_REFILL_GRID 20   /* retired in r03 with it (only 0 accepted) */
#define RT_TUNE_WAVE_STEAL 21    /* in-wave work stealing in the chain launch: a lane whose query is done
                                    walks a subtree from another lane's stack with that lane's ray
                                    (four-wide tree). 0 off, 1 on, 2 (default, auto): the second and
                                    third launches over a frame geometry are timed without and with it
                                    and later ones use the faster (before that: on when the launch is at
                                    most two rounds of resident waves). C2 0.24 -> 0.18 ms, C3 -4%;
                                    C4 is faster without */
#define RT_TUNE_STEAL_HALF 22    /* ordered chain launches: at most this many of the longest batches (and at
                                    most 1/32 of all, with the quarter and eighth tiers) run as two waves
                                    of half the batch's pixels each, so the longest chains of a frame use
                                    more SIMDs at once; in the stealing kernel the idle lanes of each start
                                    as helpers (default 512; 0 off; needs >= 2 pixels per batch) */
#define RT_TUNE_COLD_ESTIMATE 24 /* how a fused launch over batches with no measured order (a new view's
                                    first frame) is ordered: 2 (default) centre-out, by the distance of
                                    each batch from the frame's centre (no walk); 1 a pre-pass that walks
                                    one primary ray per wave batch and scores the batch; 0 screen order.
                                    C4 cold frame 0.62 / 0.70 / 0.63 ms, C2 0.20 / 0.23 / 0.23 */
#define RT_TUNE_FORGET_ORDER 25  /* any value: drop every measured batch order and wave-steal trial, so the
                                    next launch runs as a new view's first frame (benchmarks, tests) */
#define RT_TUNE_STEAL_QUARTER 23 /* ... and before them this many of the longest run as four waves of a
                                    quarter of the pixels each (needs >= 4 pixels per batch); -1 (default):
                                    per view, the launch trials time the block-dispatch candidates with 0
                                    and with 64 (r03: ref_default 0.562 -> 0.509 ms, C3 0.215 -> 0.198,
                                    C2 0.158 -> 0.166, C4 equal) */
#define RT_TUNE_SPLIT_EIGHTH 26  /* ... and before those this many as eight waves of an eighth of the pixels
                                    (default 0; needs >= 8 pixels per batch) */
#define RT_TUNE_PRIORITY_BATCHES 27 /* ordered chain launches: the waves of this many of the longest batches
                                    (with their split parts) run at raised wave priority, so their
                                    SIMDs issue them first (the longest batch is the frame's critical
                                    path); default 0 */
#define RT_TUNE_PIXEL_ORDER 28   /* which pixels of a tile share a wave batch (samples are tile-major):
                                    0 row-major (a 64-sample batch of a 16x16 tile is 16x4 pixels),
                                    1 Morton order in square power-of-two tiles (8x8 pixels at pf 1,
                                    4x4 at pf 2: the rays of a batch stay closer together), 2 (default)
                                    Morton when pfx*pfy is a power of two and the launch is not one the
                                    stealing kernel may take (at most two rounds of resident waves),
                                    else row-major. C4 0.465 -> 0.430 ms, C5 8.47 -> 7.09 ms */
#define RT_TUNE_DYN_GROUP 29     /* RT_TUNE_CHAIN_SPLIT 4: 2^value consecutive wave tasks (of the batch order)
                                    go to one XCD before the next XCD's turn (default 2: four, as four
                                    consecutive 64-thread waves of a 256-thread block) */
#define RT_TUNE_SHADOW_HELPERS 30 /* in the split waves of a fused chain launch (RT_TUNE_STEAL_HALF and the
                                    quarter / eighth tiers, plain kernel) the lanes past the part's
                                    samples walk shadow rays for their owners: lane o + r x part takes
                                    lights r, r + roles, ... of sample o, so a sample's lights are walked
                                    side by side instead of one after another. 1 (default) on, 0 off,
                                    2 per view: the launch trials time the plain kernel both ways. C3
                                    0.263 -> 0.212 ms, C4 0.412 -> 0.397 ms, C5 equal. Placement only */
#define RT_TUNE_FRAMES_IN_FLIGHT 31 /* 1-4 (default 1): calls that render on one pipeline (the default)
                                    rotate over this many pipelines (workspace, batch order, trials), so
                                    a caller that queues consecutive frames on as many alternating
                                    streams keeps that many frames in flight: a frame's launch starts as
                                    the previous frame's short batches retire, beside its longest
                                    ones. Calls on one stream stay serialised. Setting it makes the
                                    other pipelines' streams, events and workspaces (pipeline 0's size)
                                    at once, not at their first frame. Placement only */
#define RT_TUNE_ADOPT_ORDER 32   /* 1 (default): a pipeline meeting a batch geometry that another pipeline has
                                    already ordered starts from that pipeline's measured order (frames in
                                    flight); 0: it learns its own from a cold launch. Placement only */
#define RT_TUNE_INFLIGHT_DYNAMIC 33 /* 1 (default): with RT_TUNE_FRAMES_IN_FLIGHT > 1 and RT_TUNE_CHAIN_SPLIT 5,
                                    ordered launches take dynamic wave tasks on a resident grid when the
                                    trials timed the chosen shape with them within 3% of the choice (the next
                                    frame's blocks then fill the slots the previous frame's tail frees; block
                                    dispatch runs two frames side by side from their first blocks: C4 0.387
                                    -> 0.377 ms per frame). The same for multi-frame launches (rt_render_frames_device),
                                    whose tasks of K frames fill the slots a frame's tail frees (C4, 4 frames per
                                    call: 0.3445 -> 0.3412 ms per frame, profiles/r05i_ab_multi_c4.txt);
                                    0: always the trials' distribution. Placement only */
#define RT_TUNE_INFLIGHT_STREAMS 34 /* 1: with RT_TUNE_FRAMES_IN_FLIGHT > 1, a single-pipeline call runs on its
                                    pipeline's own stream (forked from the caller's stream and joined back),
                                    so two frames in flight overlap whichever hardware queues the caller's
                                    streams share; 0 (default): on the caller's stream. Placement only */
#define RT_TUNE_QUAD_WALK 35      /* 1: the waves of the quarter tier (RT_TUNE_STEAL_QUARTER) walk with four lanes
                                    per ray: lane q of a quad tests child q of each four-wide node and a
                                    leaf's triangles side by side, so a ray's node visit costs ~60 instead of
                                    ~130 wave-instructions and the longest chains of the frame (its critical
                                    path) finish sooner; a part then holds at most 16 samples of whole pixels
                                    (pf 1, 2, 4; otherwise the plain quarter tier). 0 (default): off.
                                    Placement only */
#define RT_TUNE_MOTION_ORDER 36   /* r >= 1 (default 1): a fused frame whose corner rays differ from the previous
                                    launch of its pipeline over the same batches (a moving view: the trackball
                                    turned between 'r' presses) re-sorts the batch order after every launch,
                                    from the durations dilated over the screen (each batch takes the longest
                                    duration within the (2r + 1) x (2r + 1) cells of 8 x 8 pixels around it), so
                                    a long batch that moved by a few pixels is still near the head; 0: the
                                    static schedule (every RT_TUNE_ORDER_EVERY launches, undilated), 0-8.
                                    C4 orbit at 0.25 deg per frame, one in flight: r 1 0.456-0.461 ms, 2 0.50-0.52,
                                    3 0.54, 0 0.486 (profiles/r05h_orbit_ab.txt). Placement only */
#define RT_TUNE_ORDER_EARLY 37    /* 1: a re-sorted batch order is taken by the very next launch when its sort
                                    has already completed (hipEventQuery, no wait: frames one at a time, a moving
                                    view's order then comes from the previous view, not the one before); 0
                                    (default): always the launch after next (r02's double buffering). Measured
                                    neutral: C4 orbit one at a time 0.430-0.432 ms either way, cold and static
                                    frames equal (profiles/r06o_ab_order_early.txt). Placement only */
#define RT_TUNE_TOP_NODES 13     /* retired in r03 (0-85 accepted, no effect): an LDS copy of the four-wide
                                    tree's top levels; with float node rows loaded from global memory it
                                    measured slower (flat loads, 64-bit addresses) */
#define RT_TUNE_CHAIN_SPLIT 12   /* query distribution of the chain launch: as RT_TUNE_XCD_SPLIT, or 3: 64-query
                                    chunks dealt round-robin to the XCDs and taken dynamically within
                                    each, or 4 (fused frame launches; others use 0): a resident grid
                                    whose waves each take a first wave batch by position and later ones
                                    from per-XCD counters (RT_TUNE_DYN_GROUP consecutive batches per
                                    XCD), in batch order once one is measured, so no wave slot waits for
                                    the rest of its block to retire; 5 (default, auto): 4 for a cold
                                    launch, then the per-view trials (RT_TUNE_WAVE_STEAL) also time 0
                                    against 4 and keep the faster (rt_scene_trials) */
#define RT_TUNE_PIPE_BATCHES 6     /* split a call into at least pipes x this many batches */
#define RT_TUNE_PIPE_PRIORITY 7    /* 1 (default): pipelines after the first run at lower stream priority */
#define RT_TUNE_SHADOW_VIRTUAL 5   /* bit k: step k's shadow rays are read from its hits directly
                                      (no compacted shadow queue); default 1: step 0, whose
                                      queue is dense and mostly hits */
int rt_scene_tune(rt_scene *scene, int32_t knob, int32_t value);

/* ---- tuning diagnostics ---------------------------------------------------------------- */
/* The same counters in full: [0] tests, [1] node visits, [2] sum over wave tasks (64 queries side
 * by side) of the largest per-query visit count, [3] largest visit count of any query, [4] wave
 * tasks, [5] sum over wave tasks of the largest per-query test count. */
#define RT_WORK_FIELDS 6
int rt_work_detail(rt_scene *scene, int32_t kind, uint64_t out[RT_WORK_FIELDS]);
/* Diagnostic words reserved for diagnostic kernel builds (none in r03: the wave-time, region-count
 * and stamp builds were retired with the variants they measured); 0 in production builds.
 * Reads count words from offset (offset + count <= 131072); synchronises the device. */
int rt_diag_read(rt_scene *scene, int64_t offset, int64_t count, uint64_t *out);
/* The per-view launch trials of render pipeline 0 (RT_TUNE_WAVE_STEAL 2 x RT_TUNE_CHAIN_SPLIT 5 x
 * RT_TUNE_SHADOW_HELPERS 2 x RT_TUNE_STEAL_QUARTER -1): info = {candidates timed (0 while pending),
 * chosen candidate (-1 pending), its wave_steal, its chain distribution, its shadow helpers, its
 * quarter tier, its distribution with frames in flight (RT_TUNE_INFLIGHT_DYNAMIC)}; trial_ms (may be NULL) = each candidate's chain-launch time. Candidates, per
 * distribution (0, then 4): the plain kernel (without, then with shadow helpers), then the stealing
 * kernel, each at distribution 0 also with the quarter tier. After a warm-up launch each is timed
 * twice (two rounds) and its faster launch counts; the fastest candidate is kept unless within 2% of
 * candidate 0. Frames in flight: the other pipelines adopt pipeline 0's decision. Placement only. */
#define RT_TRIAL_INFO_FIELDS 7
#define RT_MAX_TRIALS 10
int rt_scene_trials(rt_scene *scene, int32_t info[RT_TRIAL_INFO_FIELDS], float trial_ms[RT_MAX_TRIALS]);

/* Per wave batch of the scene's latest chain launch (pipeline 0): the wave's duration in 100 MHz
 * ticks (s_memrealtime), in batch order (screen order of the batches, not dispatch order). *n_out =
 * the number of batches; up to capacity are copied. Synchronises the device. The longest batch is the
 * launch's critical path (what an N-GPU split of the frame cannot go below). */
int rt_batch_durations(rt_scene *scene, uint32_t *ticks, int64_t capacity, int64_t *n_out);
/* The render workspace of one pipeline for `cap` samples, `steps` = max_lvl + 1 chain steps and
 * `lights` lights, as the library carves it (no allocation, no device): total bytes and, per array
 * in carving order, (offset, bytes): q_org[0], q_dst[0], q_org[1], q_dst[1], hit_idx, hit_I, sq_org,
 * sq_dst, shadow, chain_local, chain_coef, depth, counters[0], counters[1], wq, cost[0], order[0],
 * cost[1], order[1], order_scratch. For tests of the sizing. */
#define RT_WS_ARRAYS 22
/* The render workspaces a scene holds now (every pipeline's), in bytes, and how many
 * rt_render_frames_device calls fell back to rendering their frames one by one because the one-launch
 * workspace could not be allocated (its frames' chain records past the LDS ones). */
int rt_workspace_bytes(rt_scene *s, uint64_t *bytes, uint64_t *multi_frame_fallbacks);
int rt_workspace_layout(int64_t cap, int32_t steps, int32_t lights, uint64_t *total_bytes,
                        uint64_t extents[2 * RT_WS_ARRAYS]);


#ifdef __cplusplus
}
#endif
#endif
