/*
 * oracle.c — plain-C restatement of the reference path tracer's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker for the HIP product
 * and the CPU baseline timed by bench.py.  Never linked into libbwrt.so.
 *
 * Written to follow the reference's evaluation order operation by operation
 * (recursion included), so that it is the literal semantics the HIP kernel
 * must reproduce.  Citations are /root/reference/bwidman-raytracer/src/...
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp; never
 * -ffast-math: the reference's isnan() test must survive, Main.cu:139).
 *
 * Pin-sensitivity mutants (test infrastructure for
 * tests/golden/make_pin_sensitivity.py): -DORC_MUTANT=k replaces ONE
 * reference quirk by the "natural" formula, to measure
 * whether the only real-CUDA evidence (Renders/07 and 01 PNGs) can tell them
 * apart.  The default build has ORC_MUTANT 0: the reference semantics.
 *   1 A.5  jitter scale 0.001 * (W / 1000.0) instead of integer W / 1000
 *   2 A.6  half-pixel offset in pixelPosition
 *   3 A.9  unit triangle / quad shading normals
 *   4 A.10 tangent-frame helper test not inverted (no zero tangents on n ~ y)
 *   5 A.11 G1 with tan^2 instead of tan^4
 *   6 A.11 no isnan(G) guard
 *   7 A.12 forward-throughput evaluation of the rendering equation
 *   8 A.14/15 std::min / std::max semantics (NaN propagates) at the clamps
 *   9      libm sinf / cosf / atanf instead of the Cephes sequence
 *  (10     FMA contraction: the same source built with -ffp-contract=fast)
 */
#ifndef ORC_MUTANT
#define ORC_MUTANT 0
#endif
#include "oracle.h"

#include <math.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

_Static_assert(sizeof(orc_vec3) == 12, "vec3d layout");
_Static_assert(sizeof(orc_material) == 24, "material layout");
_Static_assert(sizeof(orc_sphere) == 40, "sphere layout");
_Static_assert(sizeof(orc_plane) == 60, "plane layout");
_Static_assert(sizeof(orc_triangle) == 60, "triangle layout");
_Static_assert(sizeof(orc_quad) == 72, "quad layout");
_Static_assert(sizeof(orc_camera) == 24, "camera layout");
_Static_assert(sizeof(orc_scene) == 88, "scene layout");

typedef orc_vec3 vec3;

/* Main.cu:28-29, Intersection.cuh:4, Math.cuh:5 */
#define SPECULAR_CHANCE 0.5f
#define NEAR_ZERO 0.0001f
#define ORC_PI 3.1415926535f

/* ---------------------------------------------------------------------- */
/* cuRAND XORWOW (CUDA 12.0 curand_kernel.h: _curand_init_scratch and
 * curand(curandStateXORWOW_t*)); called at Main.cu:377 and Math.cuh:278.
 * subsequence = offset = 0 at the only call site, so no skip-ahead. */
void orc_curand_init(unsigned long long seed, uint32_t st[6]) {
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    st[0] = 6615241u + t1 + t0;   /* d    */
    st[1] = 123456789u + t0;      /* v[0] */
    st[2] = 362436069u ^ t0;      /* v[1] */
    st[3] = 521288629u + t1;      /* v[2] */
    st[4] = 88675123u ^ t1;       /* v[3] */
    st[5] = 5783321u + t0;        /* v[4] */
}

uint32_t orc_curand(uint32_t st[6]) {
    uint32_t t = st[1] ^ (st[1] >> 2);
    st[1] = st[2];
    st[2] = st[3];
    st[3] = st[4];
    st[4] = st[5];
    st[5] = (st[5] ^ (st[5] << 4)) ^ (t ^ (t << 1));
    st[0] += 362437u;
    return st[5] + st[0];
}

/* Math.cuh:277-279: float(curand())/INT_MAX*0.5f*max; INT_MAX converts to
 * 2147483648.0f, so every step after the u32->float rounding is exact. */
static float rand_range(uint32_t st[6], float max) {
    float u = (float)orc_curand(st);
    return ((u / 2147483648.0f) * 0.5f) * max;
}

/* ---------------------------------------------------------------------- */
/* Transcendentals (Main.cu:175,179-182 call atan/sin/cos on floats).
 * The reference build used nvcc --use_fast_math (vcxproj:106,164), whose
 * __sinf/__cosf cannot be reproduced; both the oracle and the HIP kernel use
 * this single-precision Cody-Waite reduction + minimax polynomial sequence
 * (the classic Cephes sinf/cosf/atanf coefficients), evaluated without FMA
 * in exactly this order.  Accuracy vs libm is checked in
 * tests/test_oracle_math.py. */
#define FOPI 1.27323954473516f
#define DP1 0.78515625f
#define DP2 2.4187564849853515625e-4f
#define DP3 3.77489497744594108e-8f

static float poly_sin(float r, float z) {
    float p = -1.9515295891e-4f * z;
    p = p + 8.3321608736e-3f;
    p = p * z;
    p = p - 1.6666654611e-1f;
    p = p * z;
    p = p * r;
    return p + r;
}

static float poly_cos(float z) {
    float p = 2.443315711809948e-5f * z;
    p = p - 1.388731625493765e-3f;
    p = p * z;
    p = p + 4.166664568298827e-2f;
    p = p * z;
    p = p * z;
    p = p - 0.5f * z;
    return p + 1.0f;
}

static float reduce_quadrant(float x, int* jout) {
    int j = (int)(x * FOPI);
    float y = (float)j;
    if (j & 1) {
        j += 1;
        y += 1.0f;
    }
    *jout = j & 7;
    float r = x - y * DP1;
    r = r - y * DP2;
    r = r - y * DP3;
    return r;
}

float orc_sinf(float x) {
    int neg = 0;
    if (x < 0.0f) {
        x = -x;
        neg = 1;
    }
    int j;
    float r = reduce_quadrant(x, &j);
    if (j > 3) {
        neg = !neg;
        j -= 4;
    }
    float z = r * r;
    float p = (j == 1 || j == 2) ? poly_cos(z) : poly_sin(r, z);
    return neg ? -p : p;
}

float orc_cosf(float x) {
    if (x < 0.0f) x = -x;
    int j;
    float r = reduce_quadrant(x, &j);
    int neg = 0;
    if (j > 3) {
        neg = 1;
        j -= 4;
    }
    if (j > 1) neg = !neg;
    float z = r * r;
    float p = (j == 1 || j == 2) ? poly_sin(r, z) : poly_cos(z);
    return neg ? -p : p;
}

float orc_atanf(float x) {
    int neg = 0;
    if (x < 0.0f) {
        x = -x;
        neg = 1;
    }
    float y;
    if (x > 2.414213562373095f) {
        y = 1.5707963267948966f;
        x = -(1.0f / x);
    } else if (x > 0.4142135623730950f) {
        y = 0.7853981633974483f;
        x = (x - 1.0f) / (x + 1.0f);
    } else {
        y = 0.0f;
    }
    float z = x * x;
    float p = 8.05374449538e-2f * z;
    p = p - 1.38776856032e-1f;
    p = p * z;
    p = p + 1.99777106478e-1f;
    p = p * z;
    p = p - 3.33329491539e-1f;
    p = p * z;
    p = p * x;
    p = p + x;
    y = y + p;
    return neg ? -y : y;
}

/* ---------------------------------------------------------------------- */
/* Math.cuh:43-121 vector helpers, in the reference's operation order. */
static vec3 v3(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static vec3 add(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static vec3 sub(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static vec3 mulv(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static vec3 scale(float k, vec3 v) { return v3(k * v.x, k * v.y, k * v.z); }
static vec3 neg3(vec3 v) { return scale(-1.0f, v); }               /* Math.cuh:75-77 */
static vec3 addk(vec3 v, float k) { return v3(v.x + k, v.y + k, v.z + k); }
static vec3 divv(vec3 a, vec3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
static float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static vec3 cross(vec3 a, vec3 b) {                                   /* Math.cuh:103-108 */
    float i = a.y * b.z - a.z * b.y;
    float j = -(a.x * b.z - a.z * b.x);
    float k = a.x * b.y - a.y * b.x;
    return v3(i, j, k);
}
static float length3(vec3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
static vec3 normalize3(vec3 v) { return scale(1.0f / length3(v), v); } /* Math.cuh:119-121 */
static float square(float x) { return x * x; }
static float chi(float x) { return (x > 0.0f) ? 1.0f : 0.0f; }        /* Math.cuh:273-275 */

typedef struct { float m[3][3]; } mat3;
static vec3 row(const mat3* a, int r) { return v3(a->m[r][0], a->m[r][1], a->m[r][2]); }
static vec3 col(const mat3* a, int c) { return v3(a->m[0][c], a->m[1][c], a->m[2][c]); }
static vec3 matvec(const mat3* a, vec3 x) {                           /* Math.cuh:183-189 */
    return v3(dot(row(a, 0), x), dot(row(a, 1), x), dot(row(a, 2), x));
}
static mat3 matmul(const mat3* a, const mat3* b) {                    /* Math.cuh:191-199 */
    mat3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.m[i][j] = dot(row(a, i), col(b, j));
    return r;
}
static mat3 rot_x(float angle) {                                      /* Math.cuh:202-212 */
    float c = cosf(angle), s = sinf(angle);
    mat3 r = {{{1, 0, 0}, {0, c, -s}, {0, s, c}}};
    return r;
}
static mat3 rot_y(float angle) {                                      /* Math.cuh:215-225 */
    float c = cosf(angle), s = sinf(angle);
    mat3 r = {{{c, 0, s}, {0, 1, 0}, {-s, 0, c}}};
    return r;
}

/* ---------------------------------------------------------------------- */
/* Intersection.cuh */
typedef struct {
    vec3 intersection;
    float distance;
    vec3 normal;
    orc_material mat;
} hit_info;                                                            /* Intersection.cuh:6-11 */

static hit_info hit_init(void) {
    hit_info h;
    memset(&h, 0, sizeof h);
    h.distance = INFINITY;
    return h;
}

typedef struct { vec3 origin, direction; } ray3;

static int sphere_hit(const ray3* r, const orc_sphere* s, hit_info* closest) { /* :15-62 */
    vec3 p = s->position, x = r->origin, v = r->direction;
    float a = dot(v, v);
    float b = 2.0f * dot(sub(x, p), v);
    float c = dot(sub(x, p), sub(x, p)) - s->radius * s->radius;
    float disc = b * b - 4.0f * a * c;
    if (disc < 0.0f) return 0;
    float t = (-b - sqrtf(disc)) / (2.0f * a);
    if (t <= NEAR_ZERO || t > closest->distance) return 0;
    closest->distance = t;
    closest->intersection = add(r->origin, scale(t, r->direction));
    closest->normal = normalize3(sub(closest->intersection, s->position));
    closest->mat = s->mat;
    return 1;
}

static int plane_hit(const ray3* r, const orc_plane* pl, hit_info* closest) { /* :64-106 */
    vec3 normal = cross(pl->directions[0], pl->directions[1]);
    float nd = dot(normal, r->direction);
    if (fabsf(nd) < NEAR_ZERO) return 0;
    float d = -dot(normal, pl->origin);
    float t = -(dot(normal, r->origin) + d) / nd;
    if (t <= NEAR_ZERO || t > closest->distance) return 0;
    closest->intersection = add(r->origin, scale(t, r->direction));
    closest->distance = t;
    closest->normal = normal;
    closest->mat = pl->mat;
    return 1;
}

static int polygon_hit(const ray3* r, const vec3* v, int nv, const orc_material* mat,
                       hit_info* closest) {                           /* :108-173 */
    vec3 edges[4];
    for (int k = 0; k < nv; k++) edges[k] = sub(v[(k + 1) % nv], v[k]);
    orc_plane pl;
    pl.origin = v[0];
    pl.directions[0] = edges[0];
    pl.directions[1] = edges[1];
    pl.mat = *mat;
    hit_info info = hit_init();
    int hit = plane_hit(r, &pl, &info);
    if (!hit || info.distance <= NEAR_ZERO || info.distance > closest->distance) return 0;
    for (int k = 0; k < nv; k++) {
        vec3 inner = cross(info.normal, edges[k]);
        if (dot(inner, sub(info.intersection, v[k])) < 0.0f) return 0;
    }
    *closest = info;
#if ORC_MUTANT == 3
    closest->normal = normalize3(closest->normal);
#endif
    return 1;
}

/* ---------------------------------------------------------------------- */
/* Main.cu:111-206 BRDF helpers */
static float shadowing_masking(vec3 dir, vec3 n, vec3 m, float rough) { /* :112-120 */
    float vdn = dot(dir, n);
#if ORC_MUTANT == 8
    float tt = 1.0f / (vdn * vdn) - 1.0f;
    float tan_theta = (tt < 0.0f) ? 0.0f : tt;  /* std::max(tt, 0): NaN stays NaN */
#else
    float tan_theta = fmaxf(1.0f / (vdn * vdn) - 1.0f, 0.0f);
#endif
#if ORC_MUTANT == 5
    return chi(dot(dir, m) / vdn) * 2.0f / (1.0f + sqrtf(1.0f + rough * rough * tan_theta));
#else
    return chi(dot(dir, m) / vdn) * 2.0f /
           (1.0f + sqrtf(1.0f + rough * rough * tan_theta * tan_theta));
#endif
}

static float fresnel(vec3 incident, vec3 normal, float n1, float n2) { /* :122-133 */
    float c = fabsf(dot(incident, normal));
    float g_root = square(n2) / square(n1) - 1.0f + c * c;
    if (g_root < 0.0f) return 1.0f;
    float g = sqrtf(g_root);
    return 0.5f * square(g - c) / square(g + c) *
           (1.0f + square(c * (g + c) - 1.0f) / square(c * (g - c) + 1.0f));
}

static float specular_weight(vec3 i, vec3 o, vec3 n, vec3 m, float rough) { /* :135-147 */
    float g = shadowing_masking(i, n, m, rough) * shadowing_masking(o, n, m, rough);
#if ORC_MUTANT != 6
    if (isnan(g)) return 1.0f;
#endif
    float den = fabsf(dot(i, n) * dot(m, n));
    if (den == 0.0f) den = NEAR_ZERO;
    return fabsf(dot(i, m)) * g / den;
}

static vec3 base_around_normal(vec3 m, vec3 n) {                      /* :149-168 */
    vec3 some = v3(1, 0, 0);
#if ORC_MUTANT == 4
    if (!(fabsf(dot(n, some)) < 1.0f - NEAR_ZERO)) some = v3(0, 1, 0);
#else
    if (fabsf(dot(n, some)) < 1.0f - NEAR_ZERO) some = v3(0, 1, 0);
#endif
    vec3 t1 = cross(n, some);
    vec3 t2 = cross(n, t1);
    mat3 b = {{{t1.x, t2.x, n.x}, {t1.y, t2.y, n.y}, {t1.z, t2.z, n.z}}};
    return matvec(&b, m);
}

static vec3 microfacet_normal(float rough, uint32_t st[6]) {          /* :170-185 */
    float e1 = rand_range(st, 1.0f);
    float e2 = rand_range(st, 1.0f);
#if ORC_MUTANT == 9
#define orc_atanf atanf
#define orc_sinf sinf
#define orc_cosf cosf
#endif
    float theta = orc_atanf(rough * sqrtf(e1) / sqrtf(1.0f - e1));
    float phi = 2.0f * ORC_PI * e2;
    float st_ = orc_sinf(theta);
    float x = st_ * orc_cosf(phi);
    float y = st_ * orc_sinf(phi);
    float z = orc_cosf(theta);
#if ORC_MUTANT == 9
#undef orc_atanf
#undef orc_sinf
#undef orc_cosf
#endif
    return v3(x, y, z);
}

static vec3 reflect3(vec3 d, vec3 n) {                                /* :187-191 */
    return sub(d, scale(2.0f * dot(d, n), n));
}

static vec3 random_direction(uint32_t st[6], vec3 normal) {           /* :193-206 */
    vec3 r;
    do {
        float x = rand_range(st, 2.0f) - 1.0f;
        float y = rand_range(st, 2.0f) - 1.0f;
        float z = rand_range(st, 2.0f) - 1.0f;
        r = v3(x, y, z);
    } while (length3(r) > 1.0f);
    r = normalize3(r);
    if (dot(normal, r) < 0.0f) r = sub(r, scale(2.0f * dot(r, normal), normal));
    return r;
}

/* ---------------------------------------------------------------------- */
static unsigned long long g_queries, g_paths;
static vec3 g_background = {0.0f, 0.0f, 0.0f};                        /* Main.cu:27 */

void orc_set_background(float r, float g, float b) { g_background = v3(r, g, b); }

/* samplesPerPixel (Main.cu:27, 1 in the reference build) */
static int g_spp = 1;
void orc_set_samples_per_pixel(int n) { g_spp = n > 0 ? n : 1; }

static vec3 trace_path(ray3 in, const orc_scene* sc, uint32_t st[6], int bounces,
                       int max_bounces, unsigned long long* queries) { /* Main.cu:208-272 */
    vec3 out = g_background;                                          /* backgroundColor */
    if (bounces > max_bounces) return out;
    (*queries)++;
    hit_info closest = hit_init();
    int n = sc->sphere_count;                                         /* :217 */
    if (sc->plane_count > n) n = sc->plane_count;
    if (sc->triangle_count > n) n = sc->triangle_count;
    if (sc->quad_count > n) n = sc->quad_count;
    int hit = 0;
    for (int i = 0; i < n; i++) {                                     /* :221-234 */
        if (i < sc->sphere_count) hit |= sphere_hit(&in, &sc->spheres[i], &closest);
        if (i < sc->plane_count) hit |= plane_hit(&in, &sc->planes[i], &closest);
        if (i < sc->triangle_count)
            hit |= polygon_hit(&in, sc->triangles[i].vertices, 3, &sc->triangles[i].mat, &closest);
        if (i < sc->quad_count)
            hit |= polygon_hit(&in, sc->quads[i].vertices, 4, &sc->quads[i].mat, &closest);
    }
    if (hit) {                                                        /* :237-269 */
        vec3 emitted = scale(closest.mat.emittance, closest.mat.albedo);
        vec3 scatter, brdf;
        float choice = rand_range(st, 1.0f);
        if (choice < SPECULAR_CHANCE) {
            vec3 m = microfacet_normal(closest.mat.roughness, st);
            m = base_around_normal(m, closest.normal);
            scatter = reflect3(in.direction, m);
            float f = fresnel(neg3(in.direction), m, 1.0f, closest.mat.refractive_index);
            float s = specular_weight(neg3(in.direction), scatter, closest.normal, m,
                                      closest.mat.roughness);
            brdf = scale(s * f / SPECULAR_CHANCE, v3(1, 1, 1));
        } else {
            scatter = random_direction(st, closest.normal);
            brdf = scale((float)(2.0 / (1 - SPECULAR_CHANCE)), closest.mat.albedo);
        }
        ray3 next = {closest.intersection, scatter};
        vec3 incoming = trace_path(next, sc, st, bounces + 1, max_bounces, queries);
        float cos_angle = dot(scatter, closest.normal);
        out = add(emitted, scale(cos_angle, mulv(brdf, incoming)));
    }
    return out;
}

#if ORC_MUTANT == 7
/* mutant A.12: the same path, rendering equation evaluated forward
 * (acc += T * emitted, T *= brdf * cos) instead of innermost-first */
static vec3 trace_path_forward(ray3 in, const orc_scene* sc, uint32_t st[6], int max_bounces,
                               unsigned long long* queries) {
    vec3 acc = v3(0, 0, 0), T = v3(1, 1, 1);
    for (int bounces = 0;; bounces++) {
        if (bounces > max_bounces) return add(acc, mulv(T, g_background));
        (*queries)++;
        hit_info closest = hit_init();
        int n = sc->sphere_count;
        if (sc->plane_count > n) n = sc->plane_count;
        if (sc->triangle_count > n) n = sc->triangle_count;
        if (sc->quad_count > n) n = sc->quad_count;
        int hit = 0;
        for (int i = 0; i < n; i++) {
            if (i < sc->sphere_count) hit |= sphere_hit(&in, &sc->spheres[i], &closest);
            if (i < sc->plane_count) hit |= plane_hit(&in, &sc->planes[i], &closest);
            if (i < sc->triangle_count)
                hit |= polygon_hit(&in, sc->triangles[i].vertices, 3, &sc->triangles[i].mat, &closest);
            if (i < sc->quad_count)
                hit |= polygon_hit(&in, sc->quads[i].vertices, 4, &sc->quads[i].mat, &closest);
        }
        if (!hit) return add(acc, mulv(T, g_background));
        acc = add(acc, mulv(T, scale(closest.mat.emittance, closest.mat.albedo)));
        vec3 scatter, brdf;
        if (rand_range(st, 1.0f) < SPECULAR_CHANCE) {
            vec3 m = microfacet_normal(closest.mat.roughness, st);
            m = base_around_normal(m, closest.normal);
            scatter = reflect3(in.direction, m);
            float f = fresnel(neg3(in.direction), m, 1.0f, closest.mat.refractive_index);
            float s = specular_weight(neg3(in.direction), scatter, closest.normal, m, closest.mat.roughness);
            brdf = scale(s * f / SPECULAR_CHANCE, v3(1, 1, 1));
        } else {
            scatter = random_direction(st, closest.normal);
            brdf = scale((float)(2.0 / (1 - SPECULAR_CHANCE)), closest.mat.albedo);
        }
        T = mulv(T, scale(dot(scatter, closest.normal), brdf));
        in.origin = closest.intersection;
        in.direction = scatter;
    }
}
#define trace_path(in, sc, st, b, mb, q) trace_path_forward(in, sc, st, mb, q)
#endif

/* Math.cuh:245-262 */
static vec3 aces(vec3 c) {
    c = scale(0.6f, c);
    const float a = 2.51f, b = 0.03f, cc = 2.43f, d = 0.59f, e = 0.14f;
    vec3 r = divv(mulv(c, addk(scale(a, c), b)), addk(mulv(c, addk(scale(cc, c), d)), e));
#if ORC_MUTANT == 8
#define STD_MIN1(x) ((1.0f < (x)) ? 1.0f : (x)) /* std::min(x, 1): NaN stays NaN */
    return v3(STD_MIN1(r.x), STD_MIN1(r.y), STD_MIN1(r.z));
#else
    return v3(fminf(r.x, 1.0f), fminf(r.y, 1.0f), fminf(r.z, 1.0f));
#endif
}

static uint8_t to_u8(float v) {                                       /* Main.cu:312 */
    float r = roundf(v);
    if (r != r) return 0;          /* NaN -> 0 (cvt.rzi.u8 semantics) */
    if (r <= 0.0f) return 0;
    if (r >= 255.0f) return 255;
    return (uint8_t)r;
}

int orc_render_rows(const orc_scene* sc, int width, int height, int row_offset,
                    int row_stride, int rows, unsigned first_frame, int passes,
                    int max_bounces, uint32_t* rng, float* accum, uint8_t* rgba,
                    int init_rng, int threads) {
    if (!sc || width <= 0 || height <= 0 || rows < 0 || row_stride <= 0 || row_offset < 0 ||
        passes < 0 || max_bounces < 0 || !rng || !accum || first_frame == 0)
        return -1;
    /* host prelude, Main.cu:336-338 */
    const float screen_z = -(float)(width / 2) / tanf(sc->camera.fov / 2.0f);
    mat3 rl = rot_y(sc->camera.angle[0]);
    mat3 ru = rot_x(sc->camera.angle[1]);
    mat3 rot = matmul(&rl, &ru);
    /* Main.cu:291: 0.001 * (windowWidth / 1000), double then float */
#if ORC_MUTANT == 1
    const float jitter = (float)(0.001 * (width / 1000.0));
#else
    const float jitter = (float)(0.001 * (width / 1000));
#endif
    const size_t plane = (size_t)rows * (size_t)width;
    unsigned long long q_total = 0, p_total = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : q_total, p_total)
#endif
    for (int j = 0; j < rows; j++) {
        const int y = row_offset + j * row_stride;
        unsigned long long q = 0;
        for (int x = 0; x < width; x++) {
            const size_t p = (size_t)j * width + x;
            uint32_t st[6];
            if (init_rng) {
                orc_curand_init((unsigned long long)(y * width + x), st);
            } else {
                for (int k = 0; k < 6; k++) st[k] = rng[k * plane + p];
            }
            vec3 sum = v3(accum[3 * p], accum[3 * p + 1], accum[3 * p + 2]);
            unsigned frame = first_frame;
            for (int f = 0; f < passes; f++, frame++) {
#if ORC_MUTANT == 2
                vec3 pix = v3((float)(x - width / 2) + 0.5f, (float)(y - height / 2) + 0.5f, screen_z);
#else
                vec3 pix = v3((float)(x - width / 2), (float)(y - height / 2), screen_z);
#endif
                pix = matvec(&rot, pix);                              /* :288 */
                ray3 cam = {sc->camera.position, normalize3(pix)};
                cam.direction = add(cam.direction,
                                    scale(jitter, random_direction(st, cam.direction)));
                cam.direction = normalize3(cam.direction);            /* :292 */
                vec3 val = v3(0, 0, 0);
                for (int i = 0; i < g_spp; i++)                       /* :296-298: assigns */
                    val = trace_path(cam, sc, st, 0, max_bounces, &q);
                val = scale(1.0f / (float)g_spp, val);                /* :299, operator/= */
                if (frame == 1) sum = v3(0, 0, 0);                    /* :301-302 */
                sum = add(sum, val);                                  /* :304 */
                p_total++;
                if (f == passes - 1 && rgba) {
                    vec3 o = scale(1.0f / (float)frame, sum);          /* :305 */
                    o = aces(o);
                    o = v3(sqrtf(o.x), sqrtf(o.y), sqrtf(o.z));       /* Math.cuh:249-251 */
                    o = scale(255.0f, o);                             /* :311 */
                    rgba[4 * p + 0] = to_u8(o.x);
                    rgba[4 * p + 1] = to_u8(o.y);
                    rgba[4 * p + 2] = to_u8(o.z);
                    rgba[4 * p + 3] = 255;
                }
            }
            if (passes == 0 && rgba) {
                memset(&rgba[4 * p], 0, 3);
                rgba[4 * p + 3] = 255;
            }
            accum[3 * p] = sum.x;
            accum[3 * p + 1] = sum.y;
            accum[3 * p + 2] = sum.z;
            for (int k = 0; k < 6; k++) rng[k * plane + p] = st[k];
        }
        q_total += q;
    }
    g_queries = q_total;
    g_paths = p_total;
    return 0;
}

void orc_last_counters(unsigned long long* queries, unsigned long long* paths) {
    if (queries) *queries = g_queries;
    if (paths) *paths = g_paths;
}
