/*
 * oracle/rt_oracle.c — TEST INFRASTRUCTURE ONLY: the parity checker, never the product.
 *
 * A plain-C restatement of the render path of wmorssink/raytracert (TU Delft TI1805
 * "CG_Project"): OBJ/MTL loading, face normals, the brute-force closest-hit loop, the recursive
 * shade/shadow/reflection/refraction trace, and the 'r'-key frame loop with its PPM quantisation.
 * Every function cites the reference file:line it restates. Arithmetic follows the reference op
 * for op: IEEE binary32, round-to-nearest, no FMA contraction (built with -ffp-contract=off, as
 * the x86-64 reference build has no FMA), left-to-right Vec3D dot products, normalize() as a
 * multiply by a correctly rounded reciprocal, glibc powf/acosf/sqrtf.
 *
 * Who may use it: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only. The
 * product library (raytracert_amd/librtamd.so) does not link, load or call anything here.
 *
 * Parity status: PARTIALLY PINNED.
 *   The reference has no tests and no golden vectors, and it cannot be compiled in
 *   this image without writing stand-ins for <windows.h> and <GL/glut.h> (raytracing.cpp:10-11,
 *   mesh.cpp:8-9), which the build rules forbid, so oracle/_ref is not built. The restatement is
 *   pinned instead by (1) reference outputs recorded by the survey's own reference run in this
 *   container (SURVEY.md §6 / BASELINE.md: per-config ray counts, the all-black cube, the default
 *   camera corner vectors), committed as tests/golden/survey_pins.json, and (2) hand-derived
 *   known-answer tests for rayIntersectTriangle whose every operation is exact in binary32.
 *
 * Undefined behaviour in the reference is given a defined meaning here, identically in the
 * product (DESIGN.md §"Reference UB"): never-set Ns/Ni/Tr/illum read 0; an unknown or missing
 * `usemtl` maps to the default material 0; each loadMtl call starts from a zeroed Material.
 */
#include "rt_oracle.h"

#include <ctype.h>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------
 * Vec3D<float> (Vec3D.h:56-293): float p[3], every operator component-wise in binary32.
 * ---------------------------------------------------------------------------------------- */
typedef struct { float p[3]; } vec3;

static inline vec3 V(float x, float y, float z) { vec3 r = {{x, y, z}}; return r; }
/* operator+  Vec3D.h:24-26 */
static inline vec3 vadd(vec3 a, vec3 b) { return V(a.p[0] + b.p[0], a.p[1] + b.p[1], a.p[2] + b.p[2]); }
/* operator-  Vec3D.h:28-30 */
static inline vec3 vsub(vec3 a, vec3 b) { return V(a.p[0] - b.p[0], a.p[1] - b.p[1], a.p[2] - b.p[2]); }
/* unary -    Vec3D.h:32-34 */
static inline vec3 vneg(vec3 a) { return V(-a.p[0], -a.p[1], -a.p[2]); }
/* operator*(Vec,float) and operator*(float,Vec), Vec3D.h:12-18: p[i] * factor */
static inline vec3 vscale(vec3 a, float f) { return V(a.p[0] * f, a.p[1] * f, a.p[2] * f); }
/* operator*(Vec,Vec)  Vec3D.h:20-22 */
static inline vec3 vmul(vec3 a, vec3 b) { return V(a.p[0] * b.p[0], a.p[1] * b.p[1], a.p[2] * b.p[2]); }
/* operator/(Vec,float) Vec3D.h:36-38 */
static inline vec3 vdiv(vec3 a, float d) { return V(a.p[0] / d, a.p[1] / d, a.p[2] / d); }
/* dotProduct Vec3D.h:192-194: (a0*b0 + a1*b1) + a2*b2 */
static inline float vdot(vec3 a, vec3 b) { return a.p[0] * b.p[0] + a.p[1] * b.p[1] + a.p[2] * b.p[2]; }
/* crossProduct Vec3D.h:185-191 */
static inline vec3 vcross(vec3 a, vec3 b) {
    return V(a.p[1] * b.p[2] - a.p[2] * b.p[1],
             a.p[2] * b.p[0] - a.p[0] * b.p[2],
             a.p[0] * b.p[1] - a.p[1] * b.p[0]);
}
/* getLength Vec3D.h:138-140 (sqrt of a float; identical to sqrtf) */
static inline float vlen(vec3 a) { return sqrtf(vdot(a, a)); }
/* normalize Vec3D.h:142-151 */
static inline void vnormalize(vec3 *a) {
    float length = vlen(*a);
    if (length == 0.0f) return;
    float rez = 1.0f / length;
    a->p[0] *= rez; a->p[1] *= rez; a->p[2] *= rez;
}
/* distance Vec3D.h:199-202 */
static inline float vdistance(vec3 a, vec3 b) { return vlen(vsub(a, b)); }
/* std::max(a, b) = (a < b) ? b : a (libstdc++), as called at raytracing.cpp:202,225 */
static inline float fmax_std(float a, float b) { return (a < b) ? b : a; }

/* ------------------------------------------------------------------------------------------
 * Scene (mesh.h:10-201)
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    vec3 Kd, Ka, Ks;
    float Ns, Ni, Tr;
    int illum;
    unsigned flags;
    char name[128];
} material;

struct ora_scene {
    vec3 *verts; int nv, cap_v;
    uint32_t *tri;  int nt, cap_t;     /* 3 per triangle */
    uint32_t *tmat;                    /* per triangle */
    material *mats; int nm, cap_m;
    vec3 *normals;                     /* raytracing.cpp:33, filled by calculateNormals */
};

static void push_vert(ora_scene *s, vec3 v) {
    if (s->nv == s->cap_v) { s->cap_v = s->cap_v ? 2 * s->cap_v : 1024; s->verts = realloc(s->verts, sizeof(vec3) * s->cap_v); }
    s->verts[s->nv++] = v;
}
static void push_tri(ora_scene *s, uint32_t a, uint32_t b, uint32_t c, uint32_t m) {
    if (s->nt == s->cap_t) {
        s->cap_t = s->cap_t ? 2 * s->cap_t : 1024;
        s->tri = realloc(s->tri, sizeof(uint32_t) * 3 * s->cap_t);
        s->tmat = realloc(s->tmat, sizeof(uint32_t) * s->cap_t);
    }
    s->tri[3 * s->nt] = a; s->tri[3 * s->nt + 1] = b; s->tri[3 * s->nt + 2] = c;
    s->tmat[s->nt++] = m;
}
static int push_mat(ora_scene *s, const material *m) {
    if (s->nm == s->cap_m) { s->cap_m = s->cap_m ? 2 * s->cap_m : 16; s->mats = realloc(s->mats, sizeof(material) * s->cap_m); }
    s->mats[s->nm] = *m;
    return s->nm++;
}
static int find_mat(const ora_scene *s, const char *name) {
    /* std::map<string,uint> materialIndex (mesh.cpp:119): only MTL materials are keyed; index 0
     * (the default material) is never found by name. */
    for (int i = 1; i < s->nm; i++) if (strcmp(s->mats[i].name, name) == 0) return i;
    return -1;
}

#define LINE_LEN 256  /* mesh.cpp:22 */

/* Mesh::loadMtl, mesh.cpp:334-460 */
static int load_mtl(ora_scene *s, const char *filename) {
    FILE *in = fopen(filename, "r");
    if (!in) {
        fprintf(stderr, "  Warning! Material file '%s' not found!\n", filename);
        return 0;
    }
    char line[LINE_LEN];
    char key[LINE_LEN]; key[0] = 0;
    material mat; memset(&mat, 0, sizeof mat);  /* Material() -> cleanup(); unset floats read 0 (UB pinned) */
    float f1 = 0, f2 = 0, f3 = 0;
    int indef = 0;
    memset(line, 0, LINE_LEN);
    while (in && !feof(in)) {
        if (!fgets(line, LINE_LEN, in)) { /* line keeps its zeroed contents */ }
        if (line[0] == '#') { memset(line, 0, LINE_LEN); continue; }
        else if (isspace((unsigned char)line[0]) || line[0] == '\0') {
            if (indef && key[0] && (mat.flags & (ORA_HAS_KD | ORA_HAS_KA | ORA_HAS_KS | ORA_HAS_TR))) {
                if (find_mat(s, key) < 0) { snprintf(mat.name, sizeof mat.name, "%s", key); push_mat(s, &mat); }
                mat.flags = 0;  /* cleanup(): only the is_set flags (mesh.h:43-53) */
                snprintf(mat.name, sizeof mat.name, "empty");
            }
            if (line[0] == '\0') break;
        } else if (strncmp(line, "newmtl ", 7) == 0) {
            char *p0 = line + 6, *p1;
            while (isspace((unsigned char)*++p0)) {}
            p1 = p0;
            while (*p1 && !isspace((unsigned char)*p1)) ++p1;
            *p1 = '\0';
            snprintf(key, sizeof key, "%s", p0);
            indef = 1;
        } else if (strncmp(line, "Kd ", 3) == 0) {
            sscanf(line, "Kd %f %f %f", &f1, &f2, &f3); mat.Kd = V(f1, f2, f3); mat.flags |= ORA_HAS_KD;
        } else if (strncmp(line, "Ka ", 3) == 0) {
            sscanf(line, "Ka %f %f %f", &f1, &f2, &f3); mat.Ka = V(f1, f2, f3); mat.flags |= ORA_HAS_KA;
        } else if (strncmp(line, "Ks ", 3) == 0) {
            sscanf(line, "Ks %f %f %f", &f1, &f2, &f3); mat.Ks = V(f1, f2, f3); mat.flags |= ORA_HAS_KS;
        } else if (strncmp(line, "Ns ", 3) == 0) {
            sscanf(line, "Ns %f", &f1); mat.Ns = f1; mat.flags |= ORA_HAS_NS;
        } else if (strncmp(line, "Ni ", 3) == 0) {
            sscanf(line, "Ni %f", &f1); mat.Ni = f1; mat.flags |= ORA_HAS_NI;
        } else if (strncmp(line, "illum ", 6) == 0) {
            int illum = -1; sscanf(line, "illum %i", &illum); mat.illum = illum; mat.flags |= ORA_HAS_ILLUM;
        } else if (strncmp(line, "map_Kd ", 7) == 0) {
            /* texture name only (mesh.cpp:417-433); not used by the tracer */
        } else if (strncmp(line, "Tr ", 3) == 0) {
            sscanf(line, "Tr %f", &f1); mat.Tr = f1; mat.flags |= ORA_HAS_TR;
        } else if (strncmp(line, "d ", 2) == 0) {
            sscanf(line, "d %f", &f1); mat.Tr = f1; mat.flags |= ORA_HAS_TR;   /* no inversion, mesh.cpp:439-443 */
        }
        if (feof(in) && indef && (mat.flags & (ORA_HAS_KD | ORA_HAS_KA | ORA_HAS_KS | ORA_HAS_TR)) && key[0]) {
            if (find_mat(s, key) < 0) { snprintf(mat.name, sizeof mat.name, "%s", key); push_mat(s, &mat); }
        }
        memset(line, 0, LINE_LEN);
    }
    fclose(in);
    return 1;
}

/* Mesh::loadMesh, mesh.cpp:95-331 */
int ora_load_obj(const char *filename, ora_scene **out) {
    *out = NULL;
    FILE *in = fopen(filename, "r");
    if (!in) return -1;
    ora_scene *s = calloc(1, sizeof *s);

    /* defaultMat, mesh.cpp:108-117: Kd .5, Ka 0, Ks .5, Ns 96.7, illum 2; Ni/Tr never set (read 0) */
    material def; memset(&def, 0, sizeof def);
    def.Kd = V(0.5f, 0.5f, 0.5f); def.Ka = V(0.f, 0.f, 0.f); def.Ks = V(0.5f, 0.5f, 0.5f);
    def.Ns = 96.7f; def.illum = 2;
    def.flags = ORA_HAS_KD | ORA_HAS_KA | ORA_HAS_KS | ORA_HAS_NS | ORA_HAS_ILLUM;
    snprintf(def.name, sizeof def.name, "StandardMaterialInitFromTriMesh");
    push_mat(s, &def);

    /* path_ = directory of the OBJ with '\\' -> '/' (mesh.cpp:123-145) */
    char path_[4096];
    {
        char real[4096]; snprintf(real, sizeof real, "%s", filename);
        for (char *c = real; *c; c++) if (*c == '\\') *c = '/';
        char *slash = strrchr(real, '/');
        if (slash) { slash[1] = '\0'; snprintf(path_, sizeof path_, "%s", real); } else path_[0] = '\0';
    }

    char s_[LINE_LEN];
    char matname[LINE_LEN]; matname[0] = '\0';
    float x = 0, y = 0, z = 0;   /* persist across lines, mesh.cpp:121 */
    int vh[LINE_LEN]; int nvh;
    int th[LINE_LEN]; int nth;
    memset(s_, 0, LINE_LEN);
    while (!feof(in) && fgets(s_, LINE_LEN, in)) {
        if (s_[0] == '#' || isspace((unsigned char)s_[0]) || s_[0] == '\0') { memset(s_, 0, LINE_LEN); continue; }
        else if (strncmp(s_, "mtllib ", 7) == 0) {
            char *p0 = s_ + 6;
            while (isspace((unsigned char)*++p0)) {}
            int i = 0;
            while (p0[i] && !((signed char)p0[i] < 32)) i++;   /* t[i] < 32 || t[i] == 255, mesh.cpp:164-170 */
            size_t L = strlen(path_);
            snprintf(path_ + L, sizeof path_ - L, "%.*s", i, p0);   /* path_.append(...) mutates path_ */
            load_mtl(s, path_);
        } else if (strncmp(s_, "usemtl ", 7) == 0) {
            char *p0 = s_ + 6, *p1;
            while (isspace((unsigned char)*++p0)) {}
            p1 = p0;
            while (*p1 && !isspace((unsigned char)*p1)) ++p1;
            *p1 = '\0';
            snprintf(matname, sizeof matname, "%s", p0);
            if (find_mat(s, matname) < 0) {
                fprintf(stderr, "Warning! Material '%s' not defined in material file. Taking default!\n", matname);
                matname[0] = '\0';
            }
        } else if (strncmp(s_, "v ", 2) == 0) {
            sscanf(s_, "v %f %f %f", &x, &y, &z);
            push_vert(s, V(x, y, z));
        } else if (strncmp(s_, "vt ", 3) == 0) {
            /* texture coordinates: kept by the reference, unused by the tracer */
        } else if (strncmp(s_, "vn ", 3) == 0) {
            /* recalculated */
        } else if (strncmp(s_, "f ", 2) == 0) {
            /* tokenizer of mesh.cpp:218-288 */
            int component = 0, endOfVertex = 0;
            char *p0, *p1 = s_ + 2;
            nvh = 0; nth = 0;
            while (*p1 == ' ') ++p1;
            while (p1) {
                p0 = p1;
                while (*p1 != '/' && *p1 != '\r' && *p1 != '\n' && *p1 != ' ' && *p1 != '\0') ++p1;
                if (*p1 != '/') endOfVertex = 1;
                if (*p1 != '\0') { *p1 = '\0'; p1++; }
                if (*p1 == '\0' || *p1 == '\n') p1 = 0;
                if (*p0 != '\0') {
                    if (component == 0) vh[nvh++] = atoi(p0) - 1;
                    else if (component == 1) th[nth++] = atoi(p0) - 1;
                }
                ++component;
                if (endOfVertex) { component = 0; endOfVertex = 0; }
            }
            (void)th; (void)nth;
            /* material lookup (mesh.cpp:308,320); unknown / no usemtl -> default 0 (UB pinned) */
            int m = matname[0] ? find_mat(s, matname) : -1;
            if (m < 0) m = 0;
            int bad = 0;
            for (int i = 0; i < nvh; i++) if (vh[i] < 0) bad = 1;
            if (bad) { memset(s_, 0, LINE_LEN); continue; }
            if (nvh > 3) {
                for (int i = 0; i < nvh - 2; i++)   /* fan (0, i+1, i+2), mesh.cpp:293-315 (k = 0) */
                    push_tri(s, (uint32_t)vh[0], (uint32_t)vh[i + 1], (uint32_t)vh[i + 2], (uint32_t)m);
            } else if (nvh == 3) {
                push_tri(s, (uint32_t)vh[0], (uint32_t)vh[1], (uint32_t)vh[2], (uint32_t)m);
            }
        }
        memset(s_, 0, LINE_LEN);
    }
    fclose(in);

    /* Drop triangles whose vertex indices are out of range (reference: out-of-bounds read). */
    int k = 0;
    for (int i = 0; i < s->nt; i++) {
        if (s->tri[3 * i] < (uint32_t)s->nv && s->tri[3 * i + 1] < (uint32_t)s->nv && s->tri[3 * i + 2] < (uint32_t)s->nv) {
            s->tri[3 * k] = s->tri[3 * i]; s->tri[3 * k + 1] = s->tri[3 * i + 1]; s->tri[3 * k + 2] = s->tri[3 * i + 2];
            s->tmat[k] = s->tmat[i]; k++;
        }
    }
    s->nt = k;

    /* calculateNormals, raytracing.cpp:78-86 */
    s->normals = malloc(sizeof(vec3) * (s->nt ? s->nt : 1));
    for (int i = 0; i < s->nt; i++) {
        vec3 e01 = vsub(s->verts[s->tri[3 * i + 1]], s->verts[s->tri[3 * i]]);
        vec3 e02 = vsub(s->verts[s->tri[3 * i + 2]], s->verts[s->tri[3 * i]]);
        vec3 n = vcross(e01, e02);
        vnormalize(&n);
        s->normals[i] = n;
    }
    *out = s;
    return 0;
}

void ora_free(ora_scene *s) {
    if (!s) return;
    free(s->verts); free(s->tri); free(s->tmat); free(s->mats); free(s->normals); free(s);
}

void ora_counts(const ora_scene *s, int32_t *nv, int32_t *nt, int32_t *nm) {
    if (nv) *nv = s->nv;
    if (nt) *nt = s->nt;
    if (nm) *nm = s->nm;
}

void ora_export(const ora_scene *s, float *vertices, uint32_t *tri_v, uint32_t *tri_mat,
                ora_material *materials, float *normals) {
    if (vertices) memcpy(vertices, s->verts, sizeof(float) * 3 * s->nv);
    if (tri_v) memcpy(tri_v, s->tri, sizeof(uint32_t) * 3 * s->nt);
    if (tri_mat) memcpy(tri_mat, s->tmat, sizeof(uint32_t) * s->nt);
    if (normals) memcpy(normals, s->normals, sizeof(float) * 3 * s->nt);
    if (materials) {
        for (int i = 0; i < s->nm; i++) {
            const material *m = &s->mats[i];
            ora_material *o = &materials[i];
            memcpy(o->Kd, m->Kd.p, 12); memcpy(o->Ka, m->Ka.p, 12); memcpy(o->Ks, m->Ks.p, 12);
            o->Ns = m->Ns; o->Ni = m->Ni; o->Tr = m->Tr; o->illum = m->illum; o->flags = m->flags;
        }
    }
}

/* ------------------------------------------------------------------------------------------
 * Closest hit (raytracing.cpp:88-192)
 * ---------------------------------------------------------------------------------------- */

/* isNullVector, raytracing.cpp:92-94 */
static inline int is_null(vec3 v) { return v.p[0] == 0 && v.p[1] == 0 && v.p[2] == 0; }

/* rayIntersectTriangle, raytracing.cpp:99-154 */
static int ray_intersect_triangle(const vec3 R[2], const vec3 T[3], vec3 *intersectOut) {
    const float SMALL_NUM = 0.00001f;
    vec3 u = vsub(T[1], T[0]);
    vec3 v = vsub(T[2], T[0]);
    vec3 n = vcross(u, v);
    if (is_null(n)) return 0;                       /* degenerate */
    vec3 dir = vsub(R[1], R[0]);
    vec3 w0 = vsub(R[0], T[0]);
    float b = vdot(n, dir);
    float a = -vdot(n, w0);
    if (fabsf(b) < SMALL_NUM) return 0;             /* parallel; abs -> float overload */
    float r = a / b;
    if (r < 0) return 0;                            /* half-line: no r > 1 test */
    vec3 I = vadd(R[0], vscale(dir, r));
    float uu = vdot(u, u);
    float uv = vdot(u, v);
    float vv = vdot(v, v);
    vec3 w = vsub(I, T[0]);
    float wu = vdot(w, u);
    float wv = vdot(w, v);
    float D = uv * uv - uu * vv;
    float s = (uv * wv - vv * wu) / D;
    if (s < 0 || s > 1) return 0;
    float t = (uv * wu - uu * wv) / D;
    if (t < 0 || (s + t) > 1) return 0;
    *intersectOut = I;
    return 1;
}

/* intersectMesh, raytracing.cpp:161-192 */
static int intersect_mesh(const ora_scene *sc, vec3 origin, vec3 dest, vec3 *intersectOut) {
    vec3 intersect = V(0, 0, 0);
    int index = -1;
    float dist = FLT_MAX;
    vec3 R[2] = {origin, dest};
    for (int i = 0; i < sc->nt; i++) {
        vec3 tmp;
        vec3 T[3] = {sc->verts[sc->tri[3 * i]], sc->verts[sc->tri[3 * i + 1]], sc->verts[sc->tri[3 * i + 2]]};
        if (ray_intersect_triangle(R, T, &tmp)) {
            float td = vdistance(origin, tmp);
            if (td < dist) { dist = td; index = i; intersect = tmp; }
        }
    }
    *intersectOut = intersect;
    return index;
}

/* ------------------------------------------------------------------------------------------
 * Trace / shade (raytracing.cpp:194-416)
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    const ora_scene *sc;
    const ora_params *pr;
    uint64_t n_primary, n_secondary, n_shadow;
    ora_debug_bounce *dbg;   /* ora_debug_trace: one record per trace() call, in call order */
    int dbg_max, dbg_n, cur_light;
} ctx;

static vec3 trace(ctx *c, vec3 origin, vec3 dest, int lvl);

static inline int feat(const ctx *c, unsigned f) { return (c->pr->flags & f) != 0; }

/* diffuseOnly, raytracing.cpp:197-205 (normalizes the caller's normal in place) */
static vec3 diffuse_only(const material *m, vec3 *normal, vec3 lightpos) {
    vec3 Diffuse = V(0, 0, 0);
    vnormalize(normal);
    vnormalize(&lightpos);
    Diffuse = vadd(Diffuse, vscale(m->Kd, fmax_std(vdot(*normal, lightpos), 0.0f)));
    return Diffuse;
}

/* blinnPhongSpecularOnly, raytracing.cpp:210-232 */
static vec3 blinn_phong_specular_only(const ctx *c, vec3 vertexPos, vec3 *normal, const material *m, vec3 lightpos) {
    vec3 Specularity = V(0, 0, 0);
    vec3 cam = V(c->pr->camera_pos[0], c->pr->camera_pos[1], c->pr->camera_pos[2]);
    vec3 Vv = vsub(cam, vertexPos);
    vnormalize(normal);
    vnormalize(&Vv);
    vec3 L = vsub(lightpos, vertexPos);
    vnormalize(&L);
    vec3 H = vadd(Vv, L);
    vnormalize(&H);
    float spec = fmax_std(vdot(H, *normal), 0.0f);
    spec = powf(spec, m->Ns);
    Specularity = vadd(Specularity, vscale(m->Ks, spec));
    return Specularity;
}

/* isShadow, raytracing.cpp:241-261 */
static int is_shadow(ctx *c, vec3 intersection, vec3 light_pos) {
    if (feat(c, ORA_SHADOWS)) {
        vec3 out2;
        intersection = vadd(intersection, V(0.1f, 0.1f, 0.1f));
        c->n_shadow++;
        int index = intersect_mesh(c->sc, intersection, light_pos, &out2);
        int blocked = 1;
        if (index == -1) blocked = 0;
        else {
            const material *m = &c->sc->mats[c->sc->tmat[index]];   /* getMaterial, :373-376 */
            if ((m->flags & ORA_HAS_TR) && m->Tr < 1.0f) blocked = 0;
        }
        if (c->dbg && c->dbg_n >= 1 && c->dbg_n <= c->dbg_max) {
            ora_debug_bounce *b = &c->dbg[c->dbg_n - 1];   /* the trace whose shade() asks */
            if (c->cur_light < 32) {   /* (the record's masks hold lights 0-31) */
                if (blocked) b->shadowed |= 1u << c->cur_light; else b->lit |= 1u << c->cur_light;
            }
        }
        return blocked;
    }
    return 0;
}

/* addOffset, raytracing.cpp:266-271 */
static void add_offset(vec3 *point, const vec3 *towards) {
    vec3 v = vsub(*towards, *point);
    vnormalize(&v);
    v = vscale(v, 0.01f);            /* vector *= 0.01 -> float multiply */
    *point = vadd(*point, v);
}

/* reflection, raytracing.cpp:277-285 */
static vec3 reflection(ctx *c, vec3 ray, vec3 vertexPos, const vec3 *normal, int lvl) {
    vnormalize(&ray);
    vec3 R = vsub(ray, vscale(*normal, 2.0f * vdot(*normal, ray)));
    vec3 point = vertexPos;
    vec3 dest = vadd(vertexPos, R);
    add_offset(&point, &dest);
    return trace(c, point, dest, lvl);
}

/* refraction, raytracing.cpp:290-330 */
static vec3 refraction(ctx *c, vec3 ray, vec3 vertexPos, const vec3 *normal, const material *m, int lvl) {
    float ni = m->Ni;
    vnormalize(&ray);
    float check = vdot(ray, *normal);
    if (check < 0) {
        float angle = acosf(check);
        if (angle <= 2 && angle > 0)
            return vmul(m->Ks, reflection(c, ray, vertexPos, normal, lvl + 1));
        float nr = 1 / ni;
        float root = 1 - powf(nr, 2) * (1 - powf(vdot(*normal, ray), 2));
        if (root >= 0.0) {
            root = sqrtf(root);
            vec3 T = vsub(vscale(vsub(ray, vscale(*normal, vdot(*normal, ray))), nr), vscale(*normal, root));
            vec3 point = vertexPos;
            vec3 dest = vadd(vertexPos, T);
            add_offset(&point, &dest);
            return vscale(trace(c, point, dest, lvl + 1), 1 - m->Tr);
        }
    } else {
        float nr = ni;
        vec3 nn = vneg(*normal);
        float root = 1 - powf(nr, 2) * (1 - powf(vdot(nn, ray), 2));
        if (root >= 0.0) {
            root = sqrtf(root);
            vec3 T = vsub(vscale(vsub(ray, vscale(nn, vdot(nn, ray))), nr), vscale(nn, root));
            vec3 point = vertexPos;
            vec3 dest = vadd(point, T);
            add_offset(&point, &dest);
            return vscale(trace(c, point, dest, lvl + 1), 1 - m->Tr);
        }
    }
    return V(0, 0, 0);
}

/* shade, raytracing.cpp:335-368 */
static vec3 shade(ctx *c, vec3 ray, vec3 vertexPos, vec3 *normal, const material *m, int lvl) {
    vec3 pixelcolor = V(0, 0, 0);
    if (feat(c, ORA_AMBIENT) && (m->flags & ORA_HAS_KA)) pixelcolor = vadd(pixelcolor, m->Ka);
    for (int i = 0; i < c->pr->n_lights; i++) {
        /* MyLightPositions[i] (raytracing.h:9, an unbounded vector): the inline array or light_list */
        const float *li = c->pr->light_list ? c->pr->light_list + 3 * (size_t)i : c->pr->lights[i];
        vec3 L = V(li[0], li[1], li[2]);
        c->cur_light = i;
        if (!is_shadow(c, vertexPos, L)) {
            if (feat(c, ORA_DIFFUSE) && (m->flags & ORA_HAS_KD))
                pixelcolor = vadd(pixelcolor, vscale(diffuse_only(m, normal, L), m->Tr));
            if (feat(c, ORA_SPECULAR) && (m->flags & ORA_HAS_KS) && (m->flags & ORA_HAS_NS))
                pixelcolor = vadd(pixelcolor, vscale(blinn_phong_specular_only(c, vertexPos, normal, m, L), m->Tr));
        }
    }
    if (feat(c, ORA_REFRACTION) && (m->Tr < 1) && lvl < c->pr->max_lvl)
        pixelcolor = vadd(pixelcolor, refraction(c, ray, vertexPos, normal, m, lvl + 1));
    else if (feat(c, ORA_REFLECTION) && lvl < c->pr->max_lvl)
        pixelcolor = vadd(pixelcolor, vmul(m->Ks, reflection(c, ray, vertexPos, normal, lvl + 1)));
    return pixelcolor;
}

/* trace, raytracing.cpp:381-406 */
static vec3 trace(ctx *c, vec3 origin, vec3 dest, int lvl) {
    vec3 pixelcolor = V(0, 0, 0);
    vec3 intersectOut;
    if (lvl == 0) c->n_primary++; else c->n_secondary++;
    int index = intersect_mesh(c->sc, origin, dest, &intersectOut);
    if (c->dbg) {
        if (c->dbg_n < c->dbg_max) {
            ora_debug_bounce *b = &c->dbg[c->dbg_n];
            memset(b, 0, sizeof *b);
            memcpy(b->origin, origin.p, 12); memcpy(b->dest, dest.p, 12);
            if (index != -1) memcpy(b->hit, intersectOut.p, 12);
            b->triangle = index;
            b->level = lvl;
        }
        c->dbg_n++;
    }
    if (index == -1) return pixelcolor;
    vec3 ray = vsub(dest, origin);
    vec3 normal = c->sc->normals[index];
    const material *m = &c->sc->mats[c->sc->tmat[index]];
    return shade(c, ray, intersectOut, &normal, m, lvl);
}

/* ------------------------------------------------------------------------------------------
 * Public entry points
 * ---------------------------------------------------------------------------------------- */
int ora_ray_intersect_triangle(const float R[6], const float T[9], float I[3]) {
    vec3 r[2] = {V(R[0], R[1], R[2]), V(R[3], R[4], R[5])};
    vec3 t[3] = {V(T[0], T[1], T[2]), V(T[3], T[4], T[5]), V(T[6], T[7], T[8])};
    vec3 out = V(0, 0, 0);
    int hit = ray_intersect_triangle(r, t, &out);
    if (hit) memcpy(I, out.p, 12);
    return hit;
}

void ora_ray_intersect_triangle_batch(const float *R, int32_t n, const float T[9], uint8_t *hit, float *I) {
    for (int32_t i = 0; i < n; i++) hit[i] = (uint8_t)ora_ray_intersect_triangle(R + 6 * i, T, I + 3 * i);
}

int ora_intersect_mesh(const ora_scene *s, const float origin[3], const float dest[3], float I[3]) {
    vec3 out;
    int idx = intersect_mesh(s, V(origin[0], origin[1], origin[2]), V(dest[0], dest[1], dest[2]), &out);
    memcpy(I, out.p, 12);
    return idx;
}

/* Single-ray debug trace (reference key 'd', raytracing.cpp:493-510): every trace() call of the
 * chain in order, with its shadow-ray outcomes. Returns the number of trace() calls. */
int ora_debug_trace(const ora_scene *s, const ora_params *p, const float o[3], const float d[3],
                    ora_debug_bounce *out, int32_t max_bounces, float rgb[3]) {
    ctx c = {s, p, 0, 0, 0, out, max_bounces, 0, 0};
    vec3 col = trace(&c, V(o[0], o[1], o[2]), V(d[0], d[1], d[2]), 0);
    memcpy(rgb, col.p, 12);
    return c.dbg_n;
}

void ora_perform_ray_tracing(const ora_scene *s, const ora_params *p, const float o[3], const float d[3],
                             float rgb[3], uint64_t counts[3]) {
    ctx c = {s, p, 0, 0, 0, NULL, 0, 0, 0};
    vec3 col = trace(&c, V(o[0], o[1], o[2]), V(d[0], d[1], d[2]), 0);   /* performRayTracing :410-416 */
    memcpy(rgb, col.p, 12);
    if (counts) { counts[0] += c.n_primary; counts[1] += c.n_secondary; counts[2] += c.n_shadow; }
}

typedef struct {
    const ora_scene *s; const ora_params *p;
    int x0, y0, w, h, tid, nth;
    float *rgb_f32; uint8_t *rgb_u8;
    uint64_t counts[3];
} render_job;

/* MurmurHash3 32-bit finaliser (public domain algorithm), the jitter hash of RT_STOCHASTIC */
static uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

/* Frame loop of main.cpp:355-395, RGBValue clamp main.cpp:24-42, quantisation main.cpp:116-117 */
static void *render_rows(void *arg) {
    render_job *j = arg;
    const ora_params *p = j->p;
    ctx c = {j->s, p, 0, 0, 0, NULL, 0, 0, 0};
    vec3 o00 = V(p->corners[0][0], p->corners[0][1], p->corners[0][2]);
    vec3 d00 = V(p->corners[1][0], p->corners[1][1], p->corners[1][2]);
    vec3 o01 = V(p->corners[2][0], p->corners[2][1], p->corners[2][2]);
    vec3 d01 = V(p->corners[3][0], p->corners[3][1], p->corners[3][2]);
    vec3 o10 = V(p->corners[4][0], p->corners[4][1], p->corners[4][2]);
    vec3 d10 = V(p->corners[5][0], p->corners[5][1], p->corners[5][2]);
    vec3 o11 = V(p->corners[6][0], p->corners[6][1], p->corners[6][2]);
    vec3 d11 = V(p->corners[7][0], p->corners[7][1], p->corners[7][2]);
    unsigned pfx = (unsigned)p->pfx, pfy = (unsigned)p->pfy;
    float divX = (float)((unsigned)p->width * pfx - 1);    /* main.cpp:360 */
    float divY = (float)((unsigned)p->height * pfy - 1);   /* main.cpp:361 */
    int raysPerPixel = (int)(pfx * pfy);                   /* main.cpp:362 */
    for (int yy = j->tid; yy < j->h; yy += j->nth) {
        unsigned y = (unsigned)(j->y0 + yy);
        for (int xx = 0; xx < j->w; xx++) {
            unsigned x = (unsigned)(j->x0 + xx);
            vec3 rgb = V(0, 0, 0);
            for (int subx = 0; subx < (int)pfx; subx++) {
                for (int suby = 0; suby < (int)pfy; suby++) {
                    float xscale, yscale;
                    if (p->flags & ORA_STOCHASTIC) {
                        /* RT_STOCHASTIC (include/raytracert.h): jitter inside the grid cell */
                        uint32_t key = ((uint32_t)y * (uint32_t)p->width + x) * (pfx * pfy) + (uint32_t)subx * pfy + (uint32_t)suby;
                        uint32_t h1 = fmix32(key ^ fmix32((uint32_t)p->seed));
                        uint32_t h2 = fmix32(h1 + 0x9E3779B9u);
                        float jx = (float)(h1 >> 8) * 0x1p-24f, jy = (float)(h2 >> 8) * 0x1p-24f;
                        xscale = 1.0f - ((float)x * (float)pfx + ((float)subx + jx)) / divX;
                        yscale = 1.0f - ((float)y * (float)pfy + ((float)suby + jy)) / divY;
                    } else {
                        xscale = 1.0f - ((float)x * (float)pfx + (float)subx) / divX;
                        yscale = 1.0f - ((float)y * (float)pfy + (float)suby) / divY;
                    }
                    vec3 origin = vadd(vscale(vadd(vscale(o00, xscale), vscale(o10, 1 - xscale)), yscale),
                                       vscale(vadd(vscale(o01, xscale), vscale(o11, 1 - xscale)), 1 - yscale));
                    vec3 dest = vadd(vscale(vadd(vscale(d00, xscale), vscale(d10, 1 - xscale)), yscale),
                                     vscale(vadd(vscale(d01, xscale), vscale(d11, 1 - xscale)), 1 - yscale));
                    rgb = vadd(rgb, trace(&c, origin, dest, 0));
                }
            }
            rgb = vdiv(rgb, (float)raysPerPixel);
            size_t o = 3 * ((size_t)yy * j->w + xx);
            for (int k = 0; k < 3; k++) {
                float v = rgb.p[k];
                if (v > 1) v = 1.0f;
                if (v < 0) v = 0.0f;
                if (j->rgb_f32) j->rgb_f32[o + k] = v;
                if (j->rgb_u8) {
                    float q = v * 255.0f;
                    /* (unsigned char)(v*255.0f): truncation; NaN -> 0 as x86 cvttss2si gives */
                    j->rgb_u8[o + k] = (q == q) ? (uint8_t)(int)q : 0;
                }
            }
        }
    }
    j->counts[0] = c.n_primary; j->counts[1] = c.n_secondary; j->counts[2] = c.n_shadow;
    return NULL;
}

void ora_render(const ora_scene *s, const ora_params *p, int32_t x0, int32_t y0, int32_t w, int32_t h,
                float *rgb_f32, uint8_t *rgb_u8, int32_t nthreads, uint64_t counts[3]) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    render_job *jobs = calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *th = calloc((size_t)nthreads, sizeof *th);
    for (int t = 0; t < nthreads; t++) {
        render_job jj = {s, p, x0, y0, w, h, t, nthreads, rgb_f32, rgb_u8, {0, 0, 0}};
        jobs[t] = jj;
        if (nthreads > 1) pthread_create(&th[t], NULL, render_rows, &jobs[t]);
        else render_rows(&jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (counts) { counts[0] += jobs[t].counts[0]; counts[1] += jobs[t].counts[1]; counts[2] += jobs[t].counts[2]; }
    }
    free(jobs); free(th);
}

/* ------------------------------------------------------------------------------------------
 * Default camera: GLU restated (gluPerspective, gluUnProject with Mesa's cofactor inverse) for
 * the state main.cpp sets up: glTranslatef(0,0,-4) (:219), gluPerspective(50, w/h, 1, 10) (:294),
 * viewport (0,0,w,h) (:290); produceRay (:300-320) at win-z 0 and 1 with y_new = h - y.
 * ---------------------------------------------------------------------------------------- */
static void mat_mul_glu(const double a[16], const double b[16], double r[16]) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r[i * 4 + j] = a[i * 4 + 0] * b[0 * 4 + j] + a[i * 4 + 1] * b[1 * 4 + j] +
                           a[i * 4 + 2] * b[2 * 4 + j] + a[i * 4 + 3] * b[3 * 4 + j];
}

static int mat_inv_glu(const double m[16], double o[16]) {
    double inv[16], det;
    inv[0] = m[5]*m[10]*m[15] - m[5]*m[11]*m[14] - m[9]*m[6]*m[15] + m[9]*m[7]*m[14] + m[13]*m[6]*m[11] - m[13]*m[7]*m[10];
    inv[4] = -m[4]*m[10]*m[15] + m[4]*m[11]*m[14] + m[8]*m[6]*m[15] - m[8]*m[7]*m[14] - m[12]*m[6]*m[11] + m[12]*m[7]*m[10];
    inv[8] = m[4]*m[9]*m[15] - m[4]*m[11]*m[13] - m[8]*m[5]*m[15] + m[8]*m[7]*m[13] + m[12]*m[5]*m[11] - m[12]*m[7]*m[9];
    inv[12] = -m[4]*m[9]*m[14] + m[4]*m[10]*m[13] + m[8]*m[5]*m[14] - m[8]*m[6]*m[13] - m[12]*m[5]*m[10] + m[12]*m[6]*m[9];
    inv[1] = -m[1]*m[10]*m[15] + m[1]*m[11]*m[14] + m[9]*m[2]*m[15] - m[9]*m[3]*m[14] - m[13]*m[2]*m[11] + m[13]*m[3]*m[10];
    inv[5] = m[0]*m[10]*m[15] - m[0]*m[11]*m[14] - m[8]*m[2]*m[15] + m[8]*m[3]*m[14] + m[12]*m[2]*m[11] - m[12]*m[3]*m[10];
    inv[9] = -m[0]*m[9]*m[15] + m[0]*m[11]*m[13] + m[8]*m[1]*m[15] - m[8]*m[3]*m[13] - m[12]*m[1]*m[11] + m[12]*m[3]*m[9];
    inv[13] = m[0]*m[9]*m[14] - m[0]*m[10]*m[13] - m[8]*m[1]*m[14] + m[8]*m[2]*m[13] + m[12]*m[1]*m[10] - m[12]*m[2]*m[9];
    inv[2] = m[1]*m[6]*m[15] - m[1]*m[7]*m[14] - m[5]*m[2]*m[15] + m[5]*m[3]*m[14] + m[13]*m[2]*m[7] - m[13]*m[3]*m[6];
    inv[6] = -m[0]*m[6]*m[15] + m[0]*m[7]*m[14] + m[4]*m[2]*m[15] - m[4]*m[3]*m[14] - m[12]*m[2]*m[7] + m[12]*m[3]*m[6];
    inv[10] = m[0]*m[5]*m[15] - m[0]*m[7]*m[13] - m[4]*m[1]*m[15] + m[4]*m[3]*m[13] + m[12]*m[1]*m[7] - m[12]*m[3]*m[5];
    inv[14] = -m[0]*m[5]*m[14] + m[0]*m[6]*m[13] + m[4]*m[1]*m[14] - m[4]*m[2]*m[13] - m[12]*m[1]*m[6] + m[12]*m[2]*m[5];
    inv[3] = -m[1]*m[6]*m[11] + m[1]*m[7]*m[10] + m[5]*m[2]*m[11] - m[5]*m[3]*m[10] - m[9]*m[2]*m[7] + m[9]*m[3]*m[6];
    inv[7] = m[0]*m[6]*m[11] - m[0]*m[7]*m[10] - m[4]*m[2]*m[11] + m[4]*m[3]*m[10] + m[8]*m[2]*m[7] - m[8]*m[3]*m[6];
    inv[11] = -m[0]*m[5]*m[11] + m[0]*m[7]*m[9] + m[4]*m[1]*m[11] - m[4]*m[3]*m[9] - m[8]*m[1]*m[7] + m[8]*m[3]*m[5];
    inv[15] = m[0]*m[5]*m[10] - m[0]*m[6]*m[9] - m[4]*m[1]*m[10] + m[4]*m[2]*m[9] + m[8]*m[1]*m[6] - m[8]*m[2]*m[5];
    det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    if (det == 0) return 0;
    det = 1.0 / det;
    for (int i = 0; i < 16; i++) o[i] = inv[i] * det;
    return 1;
}

static void unproject(double winx, double winy, double winz, const double inv[16], const int vp[4], float out[3]) {
    double in[4] = {winx, winy, winz, 1.0}, o[4];
    in[0] = (in[0] - vp[0]) / vp[2];
    in[1] = (in[1] - vp[1]) / vp[3];
    in[0] = in[0] * 2 - 1; in[1] = in[1] * 2 - 1; in[2] = in[2] * 2 - 1;
    for (int i = 0; i < 4; i++)
        o[i] = in[0] * inv[0 * 4 + i] + in[1] * inv[1 * 4 + i] + in[2] * inv[2 * 4 + i] + in[3] * inv[3 * 4 + i];
    out[0] = (float)(o[0] / o[3]); out[1] = (float)(o[1] / o[3]); out[2] = (float)(o[2] / o[3]);
}

void ora_default_corners(int32_t w, int32_t h, float corners[8][3]) {
    double model[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, -4, 1};
    double proj[16] = {0};
    double aspect = (double)((float)w / (float)h);   /* (float)w/h at main.cpp:294 */
    double radians = 50.0 / 2 * 3.14159265358979323846 / 180;
    double sine = sin(radians), cotangent = cos(radians) / sine, zn = 1, zf = 10, dz = zf - zn;
    proj[0] = cotangent / aspect; proj[5] = cotangent; proj[10] = -(zf + zn) / dz;
    proj[11] = -1; proj[14] = -2 * zn * zf / dz; proj[15] = 0;
    double fin[16], inv[16];
    mat_mul_glu(model, proj, fin);
    mat_inv_glu(fin, inv);
    int vp[4] = {0, 0, w, h};
    int px[4][2] = {{0, 0}, {0, h - 1}, {w - 1, 0}, {w - 1, h - 1}};   /* produceRay calls, main.cpp:355-358 */
    for (int k = 0; k < 4; k++) {
        double yn = (double)(vp[3] - px[k][1]);
        unproject((double)px[k][0], yn, 0.0, inv, vp, corners[2 * k]);
        unproject((double)px[k][0], yn, 1.0, inv, vp, corners[2 * k + 1]);
    }
}
