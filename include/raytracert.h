/*
 * raytracert.h — C-ABI of librtamd.so, the MI355X (gfx950) drop-in for the render path of
 * wmorssink/raytracert (CG_Project). Plain pointers and sizes only; no HIP or torch types.
 *
 * Reference interface each entry replaces (paths relative to the reference's CG_Project/):
 *   rt_scene_load_obj     init(char*)                       raytracing.h:19, raytracing.cpp:42-73
 *                         Mesh::loadMesh / Mesh::loadMtl    mesh.h:176-177, mesh.cpp:95-460
 *                         calculateNormals()                raytracing.h:41, raytracing.cpp:78-86
 *   rt_scene_reserve      the rest of init()'s set-up: buffers for the first frame (raytracing.cpp:42-73)
 *   rt_scene_create       Mesh(vertices, triangles) ctor    mesh.h:175 (+ materials, mesh.h:197-200)
 *   rt_scene_destroy      (globals live for the process: main.cpp:17-18,130)
 *   rt_scene_export       read access to MyMesh / normals   raytracing.h:8, raytracing.cpp:33
 *   rt_get_material       Material getMaterial(int)         raytracing.h:27, raytracing.cpp:373-376
 *   rt_ray_intersect_triangle  rayIntersectTriangle (batched pairs)  raytracing.cpp:99-154
 *   rt_intersect_mesh     intersectMesh (batched)           raytracing.cpp:161-192
 *   rt_trace_rays         Vec3Df performRayTracing(o, d)    raytracing.h:33, raytracing.cpp:410-416
 *   rt_debug_trace        debug key 'd' (shoot + trace)     raytracing.cpp:493-510
 *                         (batched; also trace(o,d,lvl) at lvl 0, raytracing.h:30)
 *   rt_render_tile        the 'r'-key frame loop            main.cpp:340-411 (loop :355-395,
 *                         + RGBValue clamp :24-42 + Image::writeImage quantisation :102-128)
 *   rt_render_tiles_device  same loop, interleaved tile shard into a device buffer (multi-GPU)
 *   rt_render_frame_device  same loop, the whole frame into a device buffer (single GPU)
 *   rt_render_frames_device  the loop for several views in one launch (consecutive 'r' presses)
 *   rt_render_frames_sharded  the same loop over N GPUs     (nothing in the reference: SURVEY.md §8e)
 *   rt_comm_*             RCCL communicator for it          (one process or host thread per GPU)
 *   rt_default_corners    produceRay for the 4 corners      main.cpp:300-325,355-358 (+ reshape :288-296)
 *   rt_write_ppm          Image::writeImage                 main.cpp:102-128
 *   rt_ppm_writer_*       the same file, kept mapped for a frame per 'r' press    main.cpp:405
 *
 * Errors: the reference has none (loadMesh returns true always, mesh.cpp:330; a missing OBJ
 * crashes at fclose(NULL), mesh.cpp:329). Here every entry returns RT_OK (0) or a negative
 * RT_E_* code, and rt_last_error_string() describes the last failure on the calling thread.
 */
#ifndef RAYTRACERT_H
#define RAYTRACERT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK        0
#define RT_E_IO     -1   /* OBJ cannot be opened / PPM cannot be written */
#define RT_E_PARSE  -2   /* malformed input the reference would read out of bounds */
#define RT_E_HIP    -3   /* a HIP runtime call or kernel launch failed */
#define RT_E_ARG    -4   /* invalid argument (NULL, negative size, bad tile, too many lights) */
#define RT_E_NOMEM  -5
#define RT_E_NODEV  -6   /* no usable gfx950 device */
#define RT_E_RCCL   -7   /* an RCCL call failed, or the communicator reported an asynchronous error */

/* Lights held inline in rt_params (the reference's MyLightPositions is an unbounded std::vector,
 * raytracing.h:9, grown by the 'L' key, main.cpp:334-336): up to RT_MAX_LIGHTS in lights[][], any
 * number (up to RT_LIGHTS_LIMIT) through rt_params.light_list. */
#define RT_MAX_LIGHTS 16
#define RT_LIGHTS_LIMIT 65536

/* Feature switches (raytracing.cpp:15-20; keyboard keys 1-6, raytracing.cpp:456-473). */
#define RT_AMBIENT    (1u << 0)
#define RT_DIFFUSE    (1u << 1)
#define RT_SPECULAR   (1u << 2)
#define RT_REFLECTION (1u << 3)
#define RT_SHADOWS    (1u << 4)
#define RT_REFRACTION (1u << 5)
#define RT_ALL_FEATURES 0x3Fu
/* Extension (the reference has only the regular pf x pf grid): each sub-sample
 * is jittered inside its grid cell by a counter-based hash of (pixel, sub-sample, seed), so a
 * stochastic frame is still a pure function of its parameters and the CPU restatement checks it
 * bit for bit. Sub-sample (subx, suby) of pixel (x, y): key = (y*width + x)*pfx*pfy + subx*pfy +
 * suby; h1 = fmix32(key ^ fmix32(seed)), h2 = fmix32(h1 + 0x9E3779B9) (MurmurHash3 finaliser);
 * jx = (h1 >> 8) * 2^-24, jy = (h2 >> 8) * 2^-24; xscale = 1 - (x*pfx + (subx + jx)) / divX and
 * likewise y, every operation in binary32. */
#define RT_STOCHASTIC (1u << 8)
#define RT_DEFAULT_SEED 0x5EED

/* Material "is set" flags (mesh.h:116-122). */
#define RT_HAS_KD    (1u << 0)
#define RT_HAS_KA    (1u << 1)
#define RT_HAS_KS    (1u << 2)
#define RT_HAS_NS    (1u << 3)
#define RT_HAS_NI    (1u << 4)
#define RT_HAS_TR    (1u << 5)
#define RT_HAS_ILLUM (1u << 6)

/* Layout-compatible with Vec3Df (Vec3D.h:272,291: float p[3], 12 bytes). */
typedef struct { float x, y, z; } rt_vec3;

/* Material (mesh.h:10-125) as plain data. Values of never-set fields are defined as 0. */
typedef struct {
    float Kd[3], Ka[3], Ks[3];
    float Ns, Ni, Tr;
    int32_t illum;
    uint32_t flags;      /* RT_HAS_* */
} rt_material;

/* Everything the reference reads from globals during a render. */
typedef struct {
    int32_t width, height;        /* WindowSize_X / WindowSize_Y (main.cpp:137-138) */
    int32_t pfx, pfy;             /* pixelfactorX / pixelfactorY (raytracing.cpp:23-25), >= 1 */
    int32_t max_lvl;              /* max recursion level (raytracing.cpp:29), >= 0 */
    uint32_t flags;               /* RT_AMBIENT ... RT_REFRACTION */
    int32_t n_lights;             /* MyLightPositions.size(): 0..RT_MAX_LIGHTS, or 0..RT_LIGHTS_LIMIT with light_list */
    int32_t seed;                 /* RT_STOCHASTIC only (else ignored): jitter hash seed */
    float lights[RT_MAX_LIGHTS][3];
    float camera_pos[3];          /* MyCameraPosition (raytracing.h:10) */
    float corners[8][3];          /* origin00,dest00, origin01,dest01, origin10,dest10, origin11,dest11 */
    /* NULL: the lights are lights[0..n_lights). Else n_lights x 3 floats (host memory, read during the
     * call; a std::vector<Vec3Df>'s data() is such an array) and lights[][] is ignored: any number of
     * lights, shaded in order as shade() loops over MyLightPositions (raytracing.cpp:342). */
    const float *light_list;
} rt_params;

typedef struct rt_scene rt_scene;

/* Pass as `device` to load/create a scene on the host only (loader and inspection; no HIP calls).
 * Render/intersect entries on such a scene return RT_E_NODEV. */
#define RT_HOST_ONLY (-1)

const char *rt_last_error_string(void);
/* Number of visible HIP devices. */
int rt_device_count(int32_t *count);

/* ---- scene ---------------------------------------------------------------------------- */
int  rt_scene_load_obj(const char *path, int32_t device, rt_scene **out);
/* load_flags: RT_LOAD_PARALLEL (what rt_scene_load_obj does: the file is parsed by up to 16
 * threads) or RT_LOAD_SEQUENTIAL (one fgets/sscanf pass, the reference loader restated line by
 * line). Both produce the same vertices, triangles, materials and normals bit for bit. */
#define RT_LOAD_PARALLEL   0
#define RT_LOAD_SEQUENTIAL 1
#define RT_LOAD_THREADS(n) ((n) << 8)   /* with RT_LOAD_PARALLEL: exactly n parser threads (tests) */
/* | RT_LOAD_TEXCOORDS: also keep Mesh::texcoords and Triangle::t (mesh.cpp:199-209, 263-268,
 * 290-316; the sequential parse), read back with rt_scene_texcoords. The tracer never uses them. */
#define RT_LOAD_TEXCOORDS  0x10
int  rt_scene_load_obj_ex(const char *path, int32_t device, int32_t load_flags, rt_scene **out);
/* Texture coordinates of a scene loaded with RT_LOAD_TEXCOORDS: *n_texcoords `vt` entries as 3
 * floats each (x, y, 0: the reference reads 2D coordinates into a Vec3Df), and per triangle its
 * three texture-coordinate indices (Triangle::t: the face's 1-based indices minus 1, as unsigned;
 * 0 for corners without one, mesh.cpp:290-291). Any pointer may be NULL; sizes 3*n, 3*nt. */
int  rt_scene_texcoords(const rt_scene *scene, int32_t *n_texcoords, float *texcoords, uint32_t *tri_t);
/* Mesh::loadMtl's parse (mesh.cpp:334-460) of one MTL file: every block the reference would
 * commit, in file order (unset values inherited from the previous block, `d` and `Tr` both set
 * Tr). Mesh::loadMtl then appends each block whose name is not yet in its materialIndex (the
 * first of a name wins). *n_blocks = the count; materials (capacity entries, may be NULL) and
 * names (NUL-separated, may be NULL; names_capacity must hold them all) receive them.
 * RT_E_IO if the file cannot be opened (the reference prints a warning and returns false). */
int  rt_load_mtl(const char *path, int32_t *n_blocks, rt_material *materials, int32_t capacity, char *names,
                 size_t names_capacity);
int  rt_scene_create(const float *xyz, int32_t n_vertices, const uint32_t *tri_v, const uint32_t *tri_mat,
                     int32_t n_triangles, const rt_material *materials, int32_t n_materials,
                     int32_t device, rt_scene **out);
void rt_scene_destroy(rt_scene *scene);
int  rt_scene_info(const rt_scene *scene, int32_t *n_vertices, int32_t *n_triangles, int32_t *n_materials);
/* Host copies of the loaded scene; any pointer may be NULL. Sizes: 3*nv, 3*nt, nt, nm, 3*nt.
 * face_normals of a device scene are the ones its renderer uses, computed on the device at upload
 * (calculateNormals, raytracing.cpp:78-86); of a host-only scene, the loader's (bit-identical). */
int  rt_scene_export(const rt_scene *scene, float *vertices, uint32_t *tri_v, uint32_t *tri_mat,
                     rt_material *materials, float *face_normals);
int  rt_get_material(const rt_scene *scene, int32_t triangle_index, rt_material *out);

/* ---- hot path ------------------------------------------------------------------------- */
/* rayIntersectTriangle (raytracing.cpp:99-154) for n independent (ray, triangle) pairs on device
 * `device`: rays = n x {origin, dest} (6 floats), tris = n x {T0, T1, T2} (9 floats), host arrays.
 * hit[i] = 1 and points[3*i..] = the intersection point (the reference's intersectOut), or 0 and
 * (0,0,0). No distance compare: a hit whose point is not finite is reported as the reference does. */
int rt_ray_intersect_triangle(int32_t device, const float *rays, const float *tris, int32_t n, uint8_t *hit,
                              float *points);
/* Batched intersectMesh: n rays (origin[i], dest[i], host arrays of 3*n floats).
 * index_out[i] = closest triangle or -1; point_out[3*i..] = hit point or (0,0,0). */
int rt_intersect_mesh(rt_scene *scene, const float *origins, const float *dests, int32_t n,
                      int32_t *index_out, float *point_out);
/* Batched performRayTracing: rgb_out[3*i..] = unclamped colour of ray i.
 * counts (may be NULL) receives {primary, secondary, shadow} intersectMesh-equivalent queries. */
int rt_trace_rays(rt_scene *scene, const rt_params *params, const float *origins, const float *dests,
                  int32_t n, float *rgb_out, uint64_t counts[3]);

/* Single-ray debug trace (the reference's key 'd', raytracing.cpp:493-510, which shoots one ray,
 * keeps (origin, intersection) for drawing and prints the traced colour): one record per trace()
 * call of the ray's chain, in order, with the outcome of each shadow ray its shade() cast. For
 * parity triage: compare against the oracle's ora_debug_trace to find the first bounce that
 * differs. Writes min(n, max_bounces) records; *n_bounces = n; rgb = performRayTracing(o, d). */
typedef struct {
    float origin[3], dest[3];     /* the ray trace() was called with */
    float hit[3];                 /* intersectMesh's point, (0,0,0) on a miss */
    int32_t triangle;             /* intersectMesh's index, -1 on a miss */
    int32_t level;                /* trace()'s lvl argument */
    uint32_t shadowed;            /* bit l: light l's shadow ray was blocked (isShadow true) */
    uint32_t lit;                 /* bit l: light l's shadow ray was traced and not blocked */
} rt_debug_bounce;
int rt_debug_trace(rt_scene *scene, const rt_params *params, const float origin[3], const float dest[3],
                   rt_debug_bounce *bounces, int32_t max_bounces, int32_t *n_bounces, float rgb[3]);
/* The frame loop for pixels [x0,x0+w) x [y0,y0+h) of the params->width x params->height frame.
 * rgb_u8 (w*h*3 bytes, row-major, top row first, as written to result.ppm) and rgb_f32
 * (w*h*3 clamped floats) are host buffers; either may be NULL. */
int rt_render_tile(rt_scene *scene, const rt_params *params, int32_t x0, int32_t y0, int32_t w, int32_t h,
                   uint8_t *rgb_u8, float *rgb_f32, uint64_t counts[3]);
/* Interleaved tile shard for multi-GPU rendering, fully device-resident. The frame is cut into
 * tile_w x tile_h tiles numbered row-major (tiles_x = ceil(width/tile_w), T tiles per frame); a batch
 * of `frames` frames of this view has tile ids g = f*T + t. This call renders ids first,
 * first+stride, first+2*stride, ... below frames*T and writes each as tile_w*tile_h*3 bytes (pixels
 * outside the frame are 0) into the DEVICE buffer d_out_u8 in that order. stream is the caller's
 * hipStream_t (NULL = the null stream): the work starts after what is already queued on it and
 * later work queued on it sees the finished tiles (the renderer forks its pipelines from it and
 * joins them back). The call returns after enqueueing (no host synchronisation) unless
 * counts != NULL. Returns the number of tiles written via n_tiles_out. */
/* Every sub-sample of the 'r' loop (main.cpp:369-388) for the frame params describes, in the loop's call
 * order: record k = ((y * width + x) * pfx + subx) * pfy + suby holds performRayTracing(origin, dest) of the
 * loop's ray for (x, y, subx, suby), unclamped (raytracing.cpp:410-416). layout RT_SAMPLES_RGB: 3 floats
 * per record, the colour; RT_SAMPLES_RAY_RGB: 9 floats, the ray's origin and dest as the device made them
 * (the loop's binary32 expressions, main.cpp:380-386), then the colour. A host that runs the loop unchanged
 * can answer each call from here once it finds the call's ray equal to the record's, bit for bit
 * (include/raytracert_dropin.hpp does). out is host memory of `capacity` floats (>= layout x width x height
 * x pfx x pfy, below 2^31 records); pinned memory from rt_host_alloc copies fastest. counts as
 * rt_render_tile. */
#define RT_SAMPLES_RGB     3
#define RT_SAMPLES_RAY_RGB 9
int rt_trace_frame_samples(rt_scene *scene, const rt_params *params, int32_t layout, float *out, size_t capacity,
                           uint64_t counts[3]);
/* Set-up without rendering: the render workspace of every pipeline a frame of params would use (tile_w x
 * tile_h tiles over the whole frame; with RT_TUNE_FRAMES_IN_FLIGHT F, all F), and with samples_layout
 * RT_SAMPLES_RGB / RT_SAMPLES_RAY_RGB the device staging of rt_trace_frame_samples. The first render of
 * such a frame then allocates nothing (a host can do this in init(), raytracing.cpp:42-73, so the first
 * 'r' press pays only the render). samples_layout 0: the workspace only. Synchronises the device's work
 * on the scene's stream. */
int rt_scene_reserve(rt_scene *scene, const rt_params *params, int32_t tile_w, int32_t tile_h, int32_t samples_layout);
/* Page-locked host memory (hipHostMalloc on the scene's device's runtime), for rt_trace_frame_samples'
 * output and other large device-to-host results. */
int  rt_host_alloc(size_t bytes, void **out);
void rt_host_free(void *ptr);
/* The whole frame, row-major (height x width x 3 bytes, the PPM's pixel order), into the DEVICE
 * buffer d_out_u8, rendered in tile_w x tile_h tiles; stream semantics as rt_render_tiles_device.
 * The single-GPU form of the shard + gather path (no un-permute needed). */
int rt_render_frame_device(rt_scene *scene, const rt_params *params, int32_t tile_w, int32_t tile_h, void *d_out_u8,
                           size_t out_capacity, void *stream, uint64_t counts[3]);
/* Several frames of one frame geometry, each its own view: params[f] (f < n_frames) may differ from
 * params[0] in their corner rays only (the trackball turned between 'r' presses, main.cpp:355-358), and
 * frame f goes row-major into the DEVICE buffer d_out_u8[f] (each out_capacity bytes). One chain launch
 * renders all of them when the frame is one batch of the four-wide tree (C4, C5, the reference's defaults): its wave tasks cycle
 * over the frames, so the frames' longest batches start side by side and the short ones of each fill
 * the slots the others' tails free, on one stream and one hardware queue (the overlap frames in flight
 * on two streams get, without depending on the runtime placing those streams on different hardware
 * queues). Otherwise the frames render one after another. Bytes equal the frames rendered one at a
 * time. counts: the sum over the frames. Stream semantics as rt_render_tiles_device. */
#define RT_MAX_FRAMES_PER_CALL 8
int rt_render_frames_device(rt_scene *scene, const rt_params *params, int32_t n_frames, int32_t tile_w, int32_t tile_h,
                            void *const *d_out_u8, size_t out_capacity, void *stream, uint64_t counts[3]);
int rt_render_tiles_device(rt_scene *scene, const rt_params *params, int32_t tile_w, int32_t tile_h,
                           int32_t frames, int32_t first, int32_t stride, void *d_out_u8, size_t out_capacity,
                           void *stream, int32_t *n_tiles_out, uint64_t counts[3]);

/* ---- multi-GPU ---------------------------------------------------------- */
/* One rank per GPU (a process or a host thread each). Rank 0 makes an id with rt_comm_unique_id
 * and the host hands its RT_COMM_ID_BYTES bytes to every rank (file, MPI, a TCP store...); every
 * rank then calls rt_comm_init (collective: it returns when all nranks have joined). RCCL
 * (librccl.so.1) is loaded on first use. */
#define RT_COMM_ID_BYTES 128
typedef struct rt_comm rt_comm;
int  rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
int  rt_comm_init(int32_t device, int32_t rank, int32_t nranks, const uint8_t id[RT_COMM_ID_BYTES], rt_comm **out);
void rt_comm_destroy(rt_comm *comm);
int  rt_comm_info(const rt_comm *comm, int32_t *rank, int32_t *nranks, int32_t *device);
/* Polls the communicator (ncclCommGetAsyncError): RT_OK or RT_E_RCCL with the error's text. */
int  rt_comm_check(rt_comm *comm);
/* The 'r' loop over the communicator's GPUs. Collective: every rank calls it with the same params,
 * tiling and frame count, its scene on its own device. `frames` frames of the view are cut into
 * tile_w x tile_h tiles, ids g = f*T + t; rank r renders ids r, r+N, ... (rt_render_tiles_device),
 * ONE gather (RCCL, equal-sized shards) brings the quantised tiles to rank 0, which un-permutes them
 * on the device into d_frames_out: frames x height x width x 3 bytes, row-major, the PPM's order
 * (other ranks: d_frames_out may be NULL). Bytes equal the one-GPU render's. Asynchronous on the
 * caller's `stream` unless counts != NULL (this rank's queries per kind; then it synchronises and
 * polls the communicator). */
int rt_render_frames_sharded(rt_scene *scene, const rt_params *params, rt_comm *comm, int32_t tile_w, int32_t tile_h,
                             int32_t frames, void *d_frames_out, size_t out_capacity, void *stream, uint64_t counts[3]);
/* Pipelining of rt_render_frames_sharded (collective: every rank sets the same depth; synchronises
 * the device). depth 1 (default): render, gather and un-permute in order on the caller's stream.
 * depth 2: call i renders on the communicator's render stream i % 2 into one of two alternating
 * shard buffers and gathers + un-permutes on its exchange stream; the caller's stream waits for
 * that call's un-permute (d_frames_out is ready in stream order, as at depth 1), but the next call's
 * render does not wait for the caller's stream, so it overlaps this call's gather and un-permute,
 * and this call's render too when the scene keeps frames in flight (RT_TUNE_FRAMES_IN_FLIGHT 2).
 * The gather and un-permute still follow the caller's work queued before the call.
 * The host must then keep d_frames_out of consecutive calls distinct until its stream has passed
 * them. Calls with counts != NULL drain the pipeline and run as at depth 1. */
int rt_comm_set_pipeline(rt_comm *comm, int32_t depth);
/* The un-permute step alone: d_gathered = nranks shards of slots = ceil(frames*T / nranks) tiles
 * each (tile g in shard g % nranks, slot g / nranks; tile_w*tile_h*3 bytes per tile, row-major
 * inside the tile) -> d_frames_out as above. For hosts that gather with their own transport. */
int rt_assemble_tiles_device(int32_t device, int32_t width, int32_t height, int32_t tile_w, int32_t tile_h, int32_t frames,
                             int32_t nranks, const void *d_gathered, size_t gathered_bytes, void *d_frames_out,
                             size_t out_capacity, void *stream);

/* ---- helpers -------------------------------------------------------------------------- */
/* Corner rays of the reference's default view (camera at (0,0,4), fovy 50, near 1, far 10). */
int rt_default_corners(int32_t width, int32_t height, float corners[8][3]);
/* Image::writeImage: "P6\n%i %i\n255\n" + w*h*3 bytes. */
int rt_write_ppm(const char *path, int32_t width, int32_t height, const uint8_t *rgb_u8);
/* A host that writes result.ppm after every frame (main.cpp:405): the file opened once, sized and kept
 * mapped; rt_ppm_writer_write copies a frame's w*h*3 bytes into it with `threads` threads (1-256), slice
 * by slice, and returns when they are in the file's page-cache pages. The file then holds the bytes
 * rt_write_ppm writes. (write() of one file does not scale with threads: the kernel serialises buffered
 * writes to one inode.) */
typedef struct rt_ppm_writer rt_ppm_writer;
int rt_ppm_writer_open(const char *path, int32_t width, int32_t height, int32_t threads, rt_ppm_writer **out);
int rt_ppm_writer_write(rt_ppm_writer *w, const uint8_t *rgb_u8);
void rt_ppm_writer_close(rt_ppm_writer *w);

/* ---- acceleration ------------------------------------------------------ */
/* The reference loops over every triangle for every ray (raytracing.cpp:174-189) and leaves its
 * KD-tree commented out (:167-172). RT_ACCEL_BVH visits only triangles whose padded acceptance
 * box the ray can reach; results (index, hit point, every output byte) are identical to
 * RT_ACCEL_BRUTE_FORCE by construction. Default: RT_ACCEL_BVH. */
#define RT_ACCEL_BRUTE_FORCE 0
#define RT_ACCEL_BVH         1
int rt_scene_set_accel(rt_scene *scene, int32_t mode);
int rt_scene_get_accel(const rt_scene *scene, int32_t *mode);
/* info[0] inner nodes of the binary tree, [1] its depth, [2] always-tested (ill-conditioned)
 * triangles, [3] never-accepted (degenerate) triangles, [4] triangles in leaves, [5] nodes of the
 * four-wide tree the kernels traverse by default, [6] its depth. Builds the BVH on demand. */
#define RT_BVH_INFO_FIELDS 7
int rt_scene_bvh_info(rt_scene *scene, int32_t info[RT_BVH_INFO_FIELDS]);
/* 64-bit FNV-1a digest of the BVH arrays the device receives (both trees, leaf order, always
 * list): equal digests = identical trees (the parallel and sequential builds are compared so). */
int rt_scene_bvh_digest(rt_scene *scene, uint64_t *digest);
/* Host-side structural check of the built BVH (containment, coverage, depth bound). */
int rt_scene_bvh_validate(rt_scene *scene);
/* The padded acceptance box of one triangle T = {T0, T1, T2} (9 floats), as the BVH uses it.
 * Returns 0 (box written), 1 (ill-conditioned: tested by every query) or 2 (never accepted). */
int rt_bvh_acceptance_box(const float T[9], float lo[3], float hi[3]);

/* ---- measurement ---------------------------------------------------------------------- */
/* Kernel kinds for rt_kernel_stats. */
#define RT_KERNEL_CLOSEST_HIT 0   /* closest-hit over all triangles (primary + secondary queries) */
#define RT_KERNEL_SHADOW      1   /* shadow queries (closest-hit or any-hit) */
#define RT_KERNEL_SHADE       2   /* shading / secondary-ray generation */
#define RT_KERNEL_FRAME       3   /* sample generation + fold + AA + quantise */
#define RT_KERNEL_CHAIN       4   /* closest-hit + shadows + shade of every step from chain_from on, per
                                     lane in one launch (RT_TUNE_CHAIN_FROM); tests = brute-force
                                     equivalent of all its closest-hit and shadow queries */
#define RT_KERNEL_KINDS       5
/* RT_PROFILE_TIMING: every launch of the scene is bracketed with hipEvents on its own stream and
 * the durations accumulated (one host sync per render call). RT_PROFILE_WORK additionally has the
 * BVH kernels count their work (rt_work_stats / rt_work_detail); the counting itself costs time,
 * so time and count in separate passes. */
#define RT_PROFILE_OFF    0
#define RT_PROFILE_TIMING 1
#define RT_PROFILE_WORK   2
int rt_set_profiling(rt_scene *scene, int32_t mode);
/* launches, summed milliseconds, and summed ray-triangle tests (closest-hit/shadow kinds). */
int rt_kernel_stats(rt_scene *scene, int32_t kind, uint64_t *launches, double *total_ms, double *tests);
int rt_reset_stats(rt_scene *scene);
/* Ray-triangle tests and BVH node visits executed by the BVH kernels of `kind`
 * (RT_KERNEL_CLOSEST_HIT or RT_KERNEL_SHADOW) while profiling was RT_PROFILE_WORK, since the last
 * reset (synchronises the device). */
int rt_work_stats(rt_scene *scene, int32_t kind, double *tests, double *node_visits);
/* Launch-shape tuning and the diagnostics of the tuning work (rt_scene_tune, rt_scene_trials,
 * rt_batch_durations, rt_work_detail, rt_diag_read, rt_workspace_layout) are declared in
 * raytracert_tune.h: they are not part of the drop-in contract, and no result depends on them. */

#ifdef __cplusplus
}
#endif
#endif
