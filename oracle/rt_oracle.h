/*
 * oracle/rt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * C interface of the CPU restatement of wmorssink/raytracert's render path
 * (CG_Project/raytracing.cpp, mesh.cpp, main.cpp). Only tests/, the
 * __graft_entry__.smoke() checker and bench.py's cpu_baseline leg may load
 * this library. The product (raytracert_amd/, librtamd.so) never links it.
 *
 * Parity status: PARTIALLY PINNED — see the header of rt_oracle.c.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_MAX_LIGHTS 16

/* Feature switches, raytracing.cpp:15-20 (all default true). */
#define ORA_AMBIENT    (1u << 0)
#define ORA_DIFFUSE    (1u << 1)
#define ORA_SPECULAR   (1u << 2)
#define ORA_REFLECTION (1u << 3)
#define ORA_SHADOWS    (1u << 4)
#define ORA_REFRACTION (1u << 5)
#define ORA_ALL_FEATURES 0x3Fu
#define ORA_STOCHASTIC (1u << 8)   /* = RT_STOCHASTIC: jittered sub-samples (extension) */

/* Material "is set" bits, mesh.h:116-122. */
#define ORA_HAS_KD (1u << 0)
#define ORA_HAS_KA (1u << 1)
#define ORA_HAS_KS (1u << 2)
#define ORA_HAS_NS (1u << 3)
#define ORA_HAS_NI (1u << 4)
#define ORA_HAS_TR (1u << 5)
#define ORA_HAS_ILLUM (1u << 6)

/* Same layout as rt_params in include/raytracert.h. */
typedef struct {
    int32_t width, height;        /* WindowSize_X / WindowSize_Y (main.cpp:137-138) */
    int32_t pfx, pfy;             /* pixelfactorX / pixelfactorY (raytracing.cpp:23-25) */
    int32_t max_lvl;              /* raytracing.cpp:29 */
    uint32_t flags;               /* ORA_AMBIENT ... ORA_REFRACTION */
    int32_t n_lights;             /* MyLightPositions.size() */
    int32_t seed;                 /* with flag bit 8 (RT_STOCHASTIC): jitter seed */
    float lights[ORA_MAX_LIGHTS][3];
    float camera_pos[3];          /* MyCameraPosition */
    float corners[8][3];          /* origin00,dest00, origin01,dest01, origin10,dest10, origin11,dest11 (main.cpp:348-358) */
    const float *light_list;      /* non-NULL: n_lights x 3 floats, any count (lights[][] ignored) */
} ora_params;

/* Material as loaded (mesh.h:10-125): 3+3+3 floats, Ns, Ni, Tr, illum, flags. */
typedef struct {
    float Kd[3], Ka[3], Ks[3];
    float Ns, Ni, Tr;
    int32_t illum;
    uint32_t flags;
} ora_material;

typedef struct ora_scene ora_scene;

/* Mesh::loadMesh + loadMtl + calculateNormals (mesh.cpp:95-460, raytracing.cpp:78-86).
 * Returns 0 on success, -1 if the OBJ cannot be opened. */
int  ora_load_obj(const char *path, ora_scene **out);
void ora_free(ora_scene *s);
void ora_counts(const ora_scene *s, int32_t *n_vertices, int32_t *n_triangles, int32_t *n_materials);
/* Copies out: vertices (3*nv floats), tri_v (3*nt), tri_mat (nt), materials (nm), normals (3*nt). Any may be NULL. */
void ora_export(const ora_scene *s, float *vertices, uint32_t *tri_v, uint32_t *tri_mat,
                ora_material *materials, float *normals);

/* rayIntersectTriangle (raytracing.cpp:99-154): R = {origin, dest}, T = 3 vertices. */
int ora_ray_intersect_triangle(const float R[6], const float T[9], float I[3]);
/* rayIntersectTriangle for n rays R[6n] against one triangle: hit[n] (0/1), I[3n]. */
void ora_ray_intersect_triangle_batch(const float *R, int32_t n, const float T[9], uint8_t *hit, float *I);
/* intersectMesh (raytracing.cpp:161-192). Returns triangle index or -1. */
int ora_intersect_mesh(const ora_scene *s, const float origin[3], const float dest[3], float I[3]);
/* performRayTracing (raytracing.cpp:410-416). counts (may be NULL): primary, secondary, shadow queries. */
/* = rt_debug_bounce (include/raytracert.h) */
typedef struct {
    float origin[3], dest[3], hit[3];
    int32_t triangle, level;
    uint32_t shadowed, lit;
} ora_debug_bounce;
int ora_debug_trace(const ora_scene *s, const ora_params *p, const float o[3], const float d[3],
                    ora_debug_bounce *out, int32_t max_bounces, float rgb[3]);
void ora_perform_ray_tracing(const ora_scene *s, const ora_params *p, const float origin[3],
                             const float dest[3], float rgb[3], uint64_t counts[3]);
/* The 'r' key render loop (main.cpp:355-395) + RGBValue clamp (main.cpp:24-42) + writeImage
 * quantisation (main.cpp:116-117), restricted to the pixel rectangle [x0,x0+w) x [y0,y0+h) of the
 * p->width x p->height frame. rgb_f32 (w*h*3, clamped floats) and rgb_u8 (w*h*3) may be NULL.
 * nthreads > 1 splits rows across pthreads. counts as above (may be NULL). */
void ora_render(const ora_scene *s, const ora_params *p, int32_t x0, int32_t y0, int32_t w, int32_t h,
                float *rgb_f32, uint8_t *rgb_u8, int32_t nthreads, uint64_t counts[3]);

/* Default camera of main.cpp:217-222,288-325: modelview = translate(0,0,-4), projection =
 * gluPerspective(50, w/h, 1, 10), viewport (0,0,w,h); corner rays by gluUnProject at win-z 0/1,
 * with double-precision matrices. Writes the 8 corner vectors (order as ora_params.corners). */
void ora_default_corners(int32_t width, int32_t height, float corners[8][3]);

#ifdef __cplusplus
}
#endif
#endif
