// rt_path.h — the per-ray arithmetic of the path tracer, shared by the HIP
// kernels (rt_kernels.hip, device pass) and the scalar C++ CPU fallback
// (rt_cpu.cpp, host pass).
//
// Reference (/root/reference/bwidman-raytracer/src):
//   vector helpers        Math.cuh:43-121          -> f3, add, sub, scale, dot, cross, normalize3
//   randRange + curand    Math.cuh:277-279         -> Xorwow, next_u32, rand_range, rand_pm1
//   curand_init           Main.cu:369-380          -> xorwow_seed
//   BRDF helpers          Main.cu:111-206          -> shadowing_masking, fresnel, specular_weight,
//                                                     random_direction, specular_scatter
//   intersections         Intersection.cuh:15-173  -> closest_hit_brute, leaf_test, slab_enter
//   camera ray            Main.cu:287-290          -> primary_dir
//   shading combine       Main.cu:262-268          -> fold_level
//   tone map / quantise   Math.cuh:245-262, Main.cu:305-312 -> tone_map
//
// Every function is __host__ __device__ and written once: the GPU kernels and
// the CPU fallback run the same float operations in the same order (both
// built with -ffp-contract=off, no fast-math), so the CPU fallback is
// bit-exact with the kernels and the oracle.  Only four primitives differ
// between the two compilation passes, all exactly specified operations:
//   rt_sqrt / rt_rcp / rt_inv_len  correctly rounded sqrt, 1/x, 1/sqrt (as
//       RN(1/RN(sqrt))): gfx950 sequences of rt_sqrt.h on the device (equal
//       to the compiler's sqrtf and 1.0f/x for all 2^32 inputs), IEEE sqrtss
//       / divss on the host;
//   rt_xor3  a ^ b ^ c: one gfx950 v_bitop3_b32 on the device;
// plus the address space of wave-uniform scene reads (scalar loads through
// the constant address space on the device, plain pointers on the host).
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>

#include "rt_layout.h"
#include "rt_sqrt.h"

#define RT_HD __host__ __device__ __forceinline__

namespace {

// ---- target primitives ----------------------------------------------------
RT_HD float rt_sqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return sqrt_cr(x);
#else
    return sqrtf(x);
#endif
}

RT_HD float rt_rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return rcp_cr(x);
#else
    return 1.0f / x;
#endif
}

// 1 / length as the reference's normalize computes it: RN(1 / RN(sqrt(s)))
RT_HD float rt_inv_len(float s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return inv_length_cr(s);
#else
    return 1.0f / sqrtf(s);
#endif
}

RT_HD unsigned rt_xor3(unsigned a, unsigned b, unsigned c) {
#if defined(__HIP_DEVICE_COMPILE__)
    // gfx950 three-input bitwise op, truth table 0x96 = a ^ b ^ c (the
    // compiler does not form it from the xors): one VALU op fewer per draw
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

// Scene records are read-only for the whole launch and indexed wave-
// uniformly: on the device they are read through the constant address space
// so they come in through scalar loads (s_load_dword*) into SGPRs even though
// the kernel stores to global memory inside the loop (which would otherwise
// make the compiler fall back to per-lane vector loads with a full vmcnt wait).
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) float* cfloat_ptr;
#else
typedef const float* cfloat_ptr;
#endif
RT_HD cfloat_ptr as_const(const float* p) { return (cfloat_ptr)p; }

RT_HD int rt_f2i(float x) { return __builtin_bit_cast(int, x); }
RT_HD float rt_i2f(int x) { return __builtin_bit_cast(float, x); }

// diagnostic builds only (-DRT_STAMPS -DRT_BRANCH_STATS, device): per-branch
// wave entries and active lanes -> K.stamps[17 + 2k], [18 + 2k]
#if defined(RT_STAMPS) && defined(RT_BRANCH_STATS) && defined(__HIP_DEVICE_COMPILE__)
#define RT_BRANCH_COUNT(K, k)                                                                          \
    do {                                                                                               \
        const unsigned long long _m = __ballot(1);                                                     \
        if (__builtin_amdgcn_mbcnt_hi((unsigned)(_m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)_m, 0u)) == 0 && \
            (K).stamps) {                                                                              \
            atomicAdd(&(K).stamps[17 + 2 * (k)], 1ull);                                                \
            atomicAdd(&(K).stamps[18 + 2 * (k)], (unsigned long long)__popcll(_m));                    \
        }                                                                                              \
    } while (0)
#else
#define RT_BRANCH_COUNT(K, k) \
    do {                      \
    } while (0)
#endif

// ---- vectors (Math.cuh:43-121, same operation order) ----------------------
struct f3 {
    float x, y, z;
};

RT_HD f3 mk(float x, float y, float z) {
    f3 r;
    r.x = x;
    r.y = y;
    r.z = z;
    return r;
}
RT_HD f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD f3 scale(float k, f3 v) { return mk(k * v.x, k * v.y, k * v.z); }
RT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_HD f3 cross(f3 a, f3 b) {  // Math.cuh:103-108 (negated j term)
    float i = a.y * b.z - a.z * b.y;
    float j = -(a.x * b.z - a.z * b.x);
    float k = a.x * b.y - a.y * b.x;
    return mk(i, j, k);
}
RT_HD float length3(f3 v) { return rt_sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
// scale(1 / length(v), v) (Math.cuh normalize)
RT_HD f3 normalize3(f3 v) { return scale(rt_inv_len(v.x * v.x + v.y * v.y + v.z * v.z), v); }
RT_HD float square(float x) { return x * x; }
RT_HD float chi(float x) { return (x > 0.0f) ? 1.0f : 0.0f; }

// ---- cuRAND XORWOW (curand_kernel.h, CUDA 12.0; Main.cu:377, Math.cuh:278)
struct Xorwow {
    unsigned d, v0, v1, v2, v3, v4;
};

// curand_init(seed, 0, 0) (Main.cu:377): seeding constants of the public
// header (recalled, not checkable offline: SURVEY §8c)
RT_HD Xorwow xorwow_seed(unsigned long long seed) {
    const unsigned s0 = (unsigned)seed ^ 0xaad26b49u;
    const unsigned s1 = (unsigned)(seed >> 32) ^ 0xf7dcefddu;
    const unsigned t0 = 1099087573u * s0;
    const unsigned t1 = 2591861531u * s1;
    Xorwow s;
    s.d = 6615241u + t1 + t0;
    s.v0 = 123456789u + t0;
    s.v1 = 362436069u ^ t0;
    s.v2 = 521288629u + t1;
    s.v3 = 88675123u ^ t1;
    s.v4 = 5783321u + t0;
    return s;
}

// the seed of pixel (x, y): the global index y*W + x (an int, Main.cu:377)
RT_HD unsigned long long pixel_seed(int x, int y, int width) { return (unsigned long long)(long long)(y * width + x); }

RT_HD unsigned next_u32(Xorwow& s) {
    unsigned t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1;
    s.v1 = s.v2;
    s.v2 = s.v3;
    s.v3 = s.v4;
    // v4 ^ (v4 << 4) ^ t ^ (t << 1): the first three in one rt_xor3
    s.v4 = rt_xor3(s.v4, s.v4 << 4, t) ^ (t << 1);
    s.d += 362437u;
    return s.v4 + s.d;
}

// Math.cuh:277-279: float(u)/INT_MAX*0.5f*max, INT_MAX -> 2^31 exactly
// Every step after the u32 -> float rounding is an exact power-of-two
// scaling, so the value equals u * (2^-32 * max) with max in {1, 2}.
RT_HD float rand_range(Xorwow& s, float max) {
    float u = (float)next_u32(s);
    return u * (2.3283064365386963e-10f * max);
}

// randRange(2) - 1 in one rounding: float(u) * 2^-31 is exact (power-of-two
// scaling of a float, no under/overflow), so fma(float(u), 2^-31, -1) =
// RN(RN(float(u) * 2^-31) - 1), bit-identical to the two-step reference.
RT_HD float rand_pm1(Xorwow& s) { return __builtin_fmaf((float)next_u32(s), 4.656612873077393e-10f, -1.0f); }

// ---- transcendentals: the exact operation sequence of oracle.c
// (Cody-Waite reduction + Cephes minimax polynomials, no FMA).
#define FOPI 1.27323954473516f
#define DP1 0.78515625f
#define DP2 2.4187564849853515625e-4f
#define DP3 3.77489497744594108e-8f

RT_HD float poly_sin(float r, float z) {
    float p = -1.9515295891e-4f * z;
    p = p + 8.3321608736e-3f;
    p = p * z;
    p = p - 1.6666654611e-1f;
    p = p * z;
    p = p * r;
    return p + r;
}

RT_HD float poly_cos(float z) {
    float p = 2.443315711809948e-5f * z;
    p = p - 1.388731625493765e-3f;
    p = p * z;
    p = p + 4.166664568298827e-2f;
    p = p * z;
    p = p * z;
    p = p - 0.5f * z;
    return p + 1.0f;
}

RT_HD float reduce_quadrant(float x, int& jout) {
    int j = (int)(x * FOPI);
    float y = (float)j;
    if (j & 1) {
        j += 1;
        y += 1.0f;
    }
    jout = j & 7;
    float r = x - y * DP1;
    r = r - y * DP2;
    r = r - y * DP3;
    return r;
}

// sin and cos of the same argument (shared reduction); sign handling as
// orc_sinf / orc_cosf: sin(-x) = -sin(x), cos(-x) = cos(x)
RT_HD void sincos_nn(float x, float& s, float& c) {
    const bool xneg = x < 0.0f;
    if (xneg) x = -x;
    int j;
    float r = reduce_quadrant(x, j);
    int sneg = 0, cneg = 0;
    if (j > 3) {
        sneg = 1;
        cneg = 1;
        j -= 4;
    }
    if (j > 1) cneg = !cneg;
    float z = r * r;
    float ps = poly_sin(r, z);
    float pc = poly_cos(z);
    bool swap = (j == 1 || j == 2);
    float sv = swap ? pc : ps;
    float cv = swap ? ps : pc;
    if (xneg) sneg = !sneg;
    s = sneg ? -sv : sv;
    c = cneg ? -cv : cv;
}

RT_HD float atan_nn(float x) {  // orc_atanf
    const bool xneg = x < 0.0f;
    if (xneg) x = -x;
    float y;
    if (x > 2.414213562373095f) {
        y = 1.5707963267948966f;
        x = -rt_rcp(x);
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
    return xneg ? -y : y;
}

// ---- BRDF helpers (Main.cu:111-206) ---------------------------------------
// rough2 = roughness * roughness (precomputed: the reference evaluates
// roughness * roughness * tanTheta * tanTheta left to right, Main.cu:119)
RT_HD float shadowing_masking(f3 dir, f3 n, f3 m, float rough2) {
    float vdn = dot(dir, n);
    float tan_theta = fmaxf(rt_rcp(vdn * vdn) - 1.0f, 0.0f);
    return chi(dot(dir, m) / vdn) * 2.0f / (1.0f + rt_sqrt(1.0f + rough2 * tan_theta * tan_theta));
}

// fresnel(i, m, 1, ior) with ior2m1 = ior*ior/(1*1) - 1 precomputed
RT_HD float fresnel(f3 incident, f3 normal, float ior2m1) {
    float c = fabsf(dot(incident, normal));
    float g_root = ior2m1 + c * c;
    if (g_root < 0.0f) return 1.0f;
    float g = rt_sqrt(g_root);
    return 0.5f * square(g - c) / square(g + c) * (1.0f + square(c * (g + c) - 1.0f) / square(c * (g - c) + 1.0f));
}

RT_HD float specular_weight(f3 i, f3 o, f3 n, f3 m, float rough2) {
    float g = shadowing_masking(i, n, m, rough2) * shadowing_masking(o, n, m, rough2);
    if (isnan(g)) return 1.0f;
    float den = fabsf(dot(i, n) * dot(m, n));
    if (den == 0.0f) den = RT_NEAR_ZERO;
    return fabsf(dot(i, m)) * g / den;
}

// genRandomDirection (Main.cu:193-206): rejection-sampled ball point,
// normalised, flipped into the hemisphere of `normal` (may be non-unit).
RT_HD f3 random_direction(Xorwow& s, f3 normal, int* iters = nullptr) {
    f3 r;
    do {
        if (iters) ++*iters;
        float x = rand_pm1(s);
        float y = rand_pm1(s);
        float z = rand_pm1(s);
        r = mk(x, y, z);
        // length(r) > 1 (Main.cu:197) <=> RN(x*x+y*y+z*z) > 1 + 2^-23: sqrt is
        // correctly rounded, so RN(sqrt(s)) > 1 iff s >= 1 + 2^-22 (checked
        // exhaustively in tests/test_numerics.py)
    } while (r.x * r.x + r.y * r.y + r.z * r.z > 1.00000012f);
    r = normalize3(r);
    if (dot(normal, r) < 0.0f) r = sub(r, scale(2.0f * dot(r, normal), normal));
    return r;
}

// Specular branch of tracePath after the brdfChoice draw (Main.cu:245-255):
// microfacet normal (genMicrofacetNormal :170-185) in the tangent frame
// (baseAroundNormalToRegular :149-168), mirror reflection (:187-191),
// Fresnel (:122-133) and the G-term weight (:112-147).  Returns the scatter
// direction; kspec = specularTerm * fresnelTerm / specularChance.
RT_HD f3 specular_scatter(Xorwow& rs, f3 d, f3 n, float rough, float rough2, float ior2m1, float& kspec) {
    const float e1 = rand_range(rs, 1.0f);
    const float e2 = rand_range(rs, 1.0f);
    const float theta = atan_nn(rough * rt_sqrt(e1) / rt_sqrt(1.0f - e1));
    const float phi = 2.0f * RT_PI * e2;
    float st, ct, sp, cp;
    sincos_nn(theta, st, ct);
    sincos_nn(phi, sp, cp);
    const f3 mloc = mk(st * cp, st * sp, ct);
    f3 some = mk(1.0f, 0.0f, 0.0f);
    if (fabsf(dot(n, some)) < 1.0f - RT_NEAR_ZERO) some = mk(0.0f, 1.0f, 0.0f);
    const f3 t1 = cross(n, some);
    const f3 t2 = cross(n, t1);
    const f3 m = mk(dot(mk(t1.x, t2.x, n.x), mloc), dot(mk(t1.y, t2.y, n.y), mloc), dot(mk(t1.z, t2.z, n.z), mloc));
    const f3 scatter = sub(d, scale(2.0f * dot(d, m), m));
    const f3 inc = scale(-1.0f, d);
    const float fr = fresnel(inc, m, ior2m1);
    const float sw = specular_weight(inc, scatter, n, m, rough2);
    kspec = sw * fr / RT_SPECULAR_CHANCE;
    return scatter;
}

// ---- closest hit over the whole scene (Main.cu:217-234 + Intersection.cuh)
// Only (t, primitive id) of the running closest hit are tracked; the hit
// point and attributes are recomputed for the winner, which is bit-identical
// to the reference's eager copies (same t, same expressions).
RT_HD bool polygon_edges(cfloat_ptr q, int nv, f3 P) {
    // q points at {v0[3], in0[3], v1[3], in1[3], ...}; reject if any
    // dot(inner_k, P - v_k) < 0 (Intersection.cuh:130-134 / :165-170)
    bool inside = true;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < nv) {
            f3 v = mk(q[6 * k + 0], q[6 * k + 1], q[6 * k + 2]);
            f3 in = mk(q[6 * k + 3], q[6 * k + 4], q[6 * k + 5]);
            if (dot(in, sub(P, v)) < 0.0f) inside = false;
        }
    }
    return inside;
}

// Conservative cull (approximate arithmetic, FMA allowed): skip the exact
// test when the ray's line passes the polygon's cull sphere {c, Rc^2} with
//   |w|^2 a (1 - 2^-14) - (w.d)^2 > Rc^2 a,   w = c - o,  a = |d|^2
// i.e. distance^2 > Rc^2 + 2^-14 |w|^2 (the 2^-14 term dominates the
// evaluation error, ~2^-22 |w|^2), and only for origins within the scene
// scale (rt_context.cpp cull_sphere: the reference rejects every such
// polygon).  NaN/inf rays compare false and are never culled.
struct CullRay {
    float a, a_k;  // |d|^2, |d|^2 (1 - 2^-14)
    bool ok;       // max|o_i| <= K.cull_omax and max|d_i| <= K.cull_dmax
};

RT_HD CullRay cull_ray(const rt_kparams& K, f3 o, f3 d, float a) {
    CullRay c;
    c.a = a;
    c.a_k = a * (1.0f - 6.103515625e-05f);
    c.ok = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) <= K.cull_omax &&
           fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z)) <= K.cull_dmax;
    return c;
}

RT_HD bool culled(cfloat_ptr cs, const CullRay& cr, f3 o, f3 d) {
    const float wx = cs[0] - o.x, wy = cs[1] - o.y, wz = cs[2] - o.z;
    const float ww = __builtin_fmaf(wx, wx, __builtin_fmaf(wy, wy, wz * wz));
    const float pj = __builtin_fmaf(wx, d.x, __builtin_fmaf(wy, d.y, wz * d.z));
    const float lhs = __builtin_fmaf(-pj, pj, ww * cr.a_k);
    return cr.ok && lhs > cs[3] * cr.a;
}

RT_HD void polygon_test(const rt_kparams& K, cfloat_ptr q, int nv, f3 o, f3 d, int id, const CullRay& cr,
                        float& best_t, int& best_id) {
    if (culled(q + (nv == 3 ? RT_TRI_CULL : RT_QUAD_CULL), cr, o, d)) return;
    RT_BRANCH_COUNT(K, 2);
    float nx = q[0], ny = q[1], nz = q[2], dd = q[3];
    float nd = nx * d.x + ny * d.y + nz * d.z;
    if (!(fabsf(nd) < RT_NEAR_ZERO)) {
        float t = -((nx * o.x + ny * o.y + nz * o.z) + dd) / nd;
        // plane part (fresh planeInfo, distance = INFINITY), then the
        // polygon's own distance test (Intersection.cuh:118-122)
        bool plane_hit = !(t <= RT_NEAR_ZERO || t > INFINITY);
        if (plane_hit && !(t <= RT_NEAR_ZERO || t > best_t)) {
            RT_BRANCH_COUNT(K, 3);
            f3 P = add(o, scale(t, d));
            if (polygon_edges(q + RT_POLY_EDGES, nv, P)) {
                best_t = t;
                best_id = id;
            }
        }
    }
}

// The reference's loop (Main.cu:217-234): index i over sphere i, plane i,
// triangle i, quad i interleaved; acceptance `nearZero < t <= closest`.
// QUADS = false: the scene has no quads (launch policy); the quad tests are
// compiled out, which shortens the loop body (config 3: 0.871 -> 0.865 ms)
// STEP = 2: only the indices i0, i0 + 2, ... (one half of a closest hit split
// over two lanes, combined by key, rt_kernels.hip "split"; rays that pass
// bvh_safe only)
#ifndef RT_HIT_UNROLL  // A/B knob: unroll factor of the brute-force loop (the build's -fno-unroll-loops otherwise)
#define RT_HIT_UNROLL 1
#endif
#define RT_PRAGMA(x) _Pragma(#x)
#define RT_PRAGMA_UNROLL(n) RT_PRAGMA(unroll n)
template <bool QUADS = true, int STEP = 1>
RT_HD void closest_hit_brute(const rt_kparams& K, f3 o, f3 d, float& best_t, int& best_id, int i0 = 0) {
    const float a = dot(d, d);
    const float a4 = 4.0f * a;
    const float a2 = 2.0f * a;
    best_t = INFINITY;
    best_id = -1;
    const int pln_base = K.n_sph;
    const int tri_base = K.n_sph + K.n_pln;
    const int quad_base = tri_base + K.n_tri;
    const CullRay cr = cull_ray(K, o, d, a);
    RT_BRANCH_COUNT(K, 4);
#if RT_HIT_UNROLL > 1
    RT_PRAGMA_UNROLL(RT_HIT_UNROLL)
#endif
    for (int i = i0; i < K.n_max; i += STEP) {
        if (i < K.n_sph) {  // Intersection.cuh:15-62
            const cfloat_ptr s = as_const(K.sph) + RT_SPH_FLOATS * i;
            f3 xp = mk(o.x - s[0], o.y - s[1], o.z - s[2]);
            float b = 2.0f * dot(xp, d);
            float c = dot(xp, xp) - s[3];
            float disc = b * b - a4 * c;
            // exact early-out: b >= 0 (finite disc, a2 > 0) gives -b - sqrt(disc) <= 0,
            // i.e. t <= 0 <= nearZero, rejected by the reference as well
            if (!(disc < 0.0f) && !(b >= 0.0f && disc == disc && a2 > 0.0f)) {
                RT_BRANCH_COUNT(K, 0);
                float t = (-b - rt_sqrt(disc)) / a2;
                if (!(t <= RT_NEAR_ZERO || t > best_t)) {
                    best_t = t;
                    best_id = i;
                }
            }
        }
        if (i < K.n_pln) {  // Intersection.cuh:64-106
            const cfloat_ptr q = as_const(K.pln) + RT_PLN_FLOATS * i;
            float nx = q[0], ny = q[1], nz = q[2], dd = q[3];
            float nd = nx * d.x + ny * d.y + nz * d.z;
            if (!(fabsf(nd) < RT_NEAR_ZERO)) {
                float t = -((nx * o.x + ny * o.y + nz * o.z) + dd) / nd;
                if (!(t <= RT_NEAR_ZERO || t > best_t)) {
                    best_t = t;
                    best_id = pln_base + i;
                }
            }
        }
        if (i < K.n_tri) polygon_test(K, as_const(K.tri) + RT_TRI_FLOATS * i, 3, o, d, tri_base + i, cr, best_t, best_id);
        if (QUADS && i < K.n_quad)
            polygon_test(K, as_const(K.quad) + RT_QUAD_FLOATS * i, 4, o, d, quad_base + i, cr, best_t, best_id);
    }
}

// ---- BVH pieces (large scenes, e.g. the 10k-triangle stress scene) ---------
// Exactness: every primitive is tested with the reference's own arithmetic
// (the same code as closest_hit_brute) and accepted when
//   t > nearZero  and  (t < best  or  (t == best and key > best_key)),
// so the winner is the minimum distance with ties resolved to the primitive
// the reference tests last (RT_KEY order) — exactly what the reference's
// running `t > closest` test in interleaved order returns, whatever order
// the BVH visits primitives in.  This needs distances that are never NaN:
// the reference ACCEPTS a NaN distance (its `t <= nearZero || t > closest`
// rejection is false for NaN) and then every later candidate, which only its
// own loop order reproduces.  Rays with a NaN/inf component, and finite rays
// whose primitive tests could overflow to NaN (bvh_safe), take the
// brute-force loop.  Node boxes are inflated far beyond float rounding and
// the slab test only ever prunes with margins, so no primitive the
// reference could hit is skipped.
RT_HD bool key_accept(float t, int key, float best_t, int best_key) {
    return !(t <= RT_NEAR_ZERO) && (t < best_t || (t == best_t && key > best_key));
}

// No bounded-primitive test of this ray can produce a NaN distance: with
// dm = max|d_i|, om = max|o_i|, S = K.ovf_sc (largest vertex / sphere
// centre coordinate + sphere radius), N = K.ovf_nm (largest component of
// a compiled triangle/quad normal cross(e0, e1), |n| = 2 area) and
// K.ovf_im (largest component of an inner edge normal cross(n, e_k)), the sphere
// test's b^2 and 4ac stay below 36 (dm (om + S))^2 < FLT_MAX and the polygon
// plane's n.d and n.o + d below 3 N dm and 3 N (om + 3 S): no inf - inf, no
// inf / inf.  Secondary rays are not unit vectors (the reference reflects
// about un-normalised triangle normals, Main.cu:187-191, Intersection.cuh:
// 108-138), so at scene scales >= 100 their direction reaches 1e16 and
// overflow does happen (tests/test_gpu_parity.py test_stress_bvh_scaled).
// Infinite distances need no special care: the reference and key_accept
// both keep the last of equal distances, and a box is only pruned against
// a finite closest hit.
RT_HD bool bvh_safe(const rt_kparams& K, f3 o, f3 d) {
    const float om = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float dm = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    // (NaN components fail every comparison, inf ones the first; dm > 1e-15
    // keeps a = |d|^2 normal, so a2 > 0 and (-b - sqrt(disc)) / a2 is never 0/0)
    // The polygon inside test dot(in_k, P - v_k) must not overflow either (a
    // NaN there passes it, so the reference accepts a hit anywhere on the
    // polygon's plane): P = o + t d with t <= |n.o + d| / 1e-4 (|n.d| >= 1e-4
    // or the plane is rejected), so |P - v_k| <= om + S + 1.8 dm 3e4 N (om + 3S)
    // and |in_k| <= K.ovf_im per component
    if (!(om + K.ovf_sc < 1e18f && dm < 1e18f && dm > 1e-15f && dm * (om + K.ovf_sc) < 1e18f &&
          K.ovf_nm * dm < 1e36f && K.ovf_nm * (om + 3.0f * K.ovf_sc) < 1e33f))
        return false;
    const float pm = om + K.ovf_sc + 6e4f * dm * (K.ovf_nm * (om + 3.0f * K.ovf_sc));
    return pm < 1e37f && K.ovf_im * pm < 3e36f;
}

// Planes are unbounded: a BVH walk tests every plane first
RT_HD void planes_first(const rt_kparams& K, f3 o, f3 d, float& best_t, int& best_id, int& best_key) {
    for (int i = 0; i < K.n_pln; i++) {
        const cfloat_ptr q = as_const(K.pln) + RT_PLN_FLOATS * i;
        const float nd = q[0] * d.x + q[1] * d.y + q[2] * d.z;
        if (!(fabsf(nd) < RT_NEAR_ZERO)) {
            const float t = -((q[0] * o.x + q[1] * o.y + q[2] * o.z) + q[3]) / nd;
            const int key = RT_KEY(1, i);
            if (key_accept(t, key, best_t, best_key)) {
                best_t = t;
                best_id = K.n_sph + i;
                best_key = key;
            }
        }
    }
}

// Slab-test set-up of a walk: a direction clamped away from 0 (sign kept, a
// conservative stand-in for the axis-parallel case), its reciprocal, the
// origin scaled by it, and the absolute margin m covering the rounding of
// o * inv (at most 2^-24 |o * inv| per axis) in the fma slab distances.
struct SlabRay {
    f3 inv, oinv;
    float m;
};

RT_HD SlabRay slab_ray(f3 o, f3 d) {
    const float tiny = 1e-20f;
    const f3 dc = mk(fabsf(d.x) < tiny ? copysignf(tiny, d.x) : d.x, fabsf(d.y) < tiny ? copysignf(tiny, d.y) : d.y,
                     fabsf(d.z) < tiny ? copysignf(tiny, d.z) : d.z);
    SlabRay s;
    s.inv = mk(rt_rcp(dc.x), rt_rcp(dc.y), rt_rcp(dc.z));
    s.oinv = mk(o.x * s.inv.x, o.y * s.inv.y, o.z * s.inv.z);
    s.m = 1e-6f + 9.5367431640625e-07f * fmaxf(fmaxf(fabsf(s.oinv.x), fabsf(s.oinv.y)), fabsf(s.oinv.z));
    return s;
}

// octant of the ray direction: the node array with near children first
RT_HD int ray_octant(const rt_kparams& K, f3 d) {
    return ((d.x < 0.0f) | ((d.y < 0.0f) << 1) | ((d.z < 0.0f) << 2)) & K.bvh_order_mask;
}

// The ray may enter box [lo, hi] before the closest hit so far: margins of
// 1e-5 relative + m absolute on the interval, and prune against the current
// closest distance only beyond the same margins
// (slab_test also returns the box's entry / exit distances)
RT_HD bool slab_test(float lx, float ly, float lz, float hx, float hy, float hz, const SlabRay& s, float best_t,
                     float& tmin, float& tmax) {
    const float tx0 = __builtin_fmaf(lx, s.inv.x, -s.oinv.x), tx1 = __builtin_fmaf(hx, s.inv.x, -s.oinv.x);
    const float ty0 = __builtin_fmaf(ly, s.inv.y, -s.oinv.y), ty1 = __builtin_fmaf(hy, s.inv.y, -s.oinv.y);
    const float tz0 = __builtin_fmaf(lz, s.inv.z, -s.oinv.z), tz1 = __builtin_fmaf(hz, s.inv.z, -s.oinv.z);
    tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    return tmin <= tmax * (1.0f + 1e-5f) + s.m && tmin <= best_t * (1.0f + 1e-5f) + (1e-5f + s.m);
}

RT_HD bool slab_enter(float lx, float ly, float lz, float hx, float hy, float hz, const SlabRay& s, float best_t) {
    float tmin, tmax;
    return slab_test(lx, ly, lz, hx, hy, hz, s, best_t, tmin, tmax);
}

// Leaf record (rt_layout.h RT_LEAF_FLOATS) {key, record...}: kind = key & 3,
// the primitive id follows from the index key >> 2 (no id / kind words: a
// triangle's plane and first edge are its first 48 bytes, one load round
// trip; config 5 89.8 -> 88.8 ms); each later edge loads only the 16-byte
// pieces it still needs, so a lane whose point fails an edge requests no
// further record bytes (the walk is bound by its L1 / L2 request traffic).
// VTX: the record in vertex form (rt_layout.h bvh_leafvtx)
template <bool VTX = false>
RT_HD void leaf_test(const rt_kparams& K, const float* r, f3 o, f3 d, float a2, float a4, float& best_t, int& best_id,
                     int& best_key) {
    const float4 c0 = *reinterpret_cast<const float4*>(r);      // key, n.xyz | key, c.xyz
    const float4 c1 = *reinterpret_cast<const float4*>(r + 4);  // d, v0.xyz   | r^2
    const float4 c2 = *reinterpret_cast<const float4*>(r + 8);  // in0.xyz, v1.x (RT_LEAF_VERTS: v2.yz, v3.xy)
#if defined(__HIP_DEVICE_COMPILE__)
    // issued with c0 and c1 (the compiler would sink it below the plane
    // test, one dependent round trip more): config 5 80.9 -> 78.3 ms, its
    // 1/8 shard 18.4 -> 18.1 (profiles/r05h/ab_hoist.txt); the whole record
    // up front needs 101 VGPRs (or spills at 96) and gains less.  (The
    // ray-refill kernel has since read the vertex form, VTX: 76.2 ms.)
    asm volatile("" ::"v"(c2.x), "v"(c2.y), "v"(c2.z), "v"(c2.w));
#endif
    const int key = rt_f2i(c0.x), kind = key & 3, idx = key >> 2;
    if (kind == 0) {  // sphere {c, r^2}, Intersection.cuh:15-62
        const f3 xp = mk(o.x - c0.y, o.y - c0.z, o.z - c0.w);
        const float b = 2.0f * dot(xp, d);
        const float c = dot(xp, xp) - c1.x;
        const float disc = b * b - a4 * c;
        if (!(disc < 0.0f) && !(b >= 0.0f)) {
            const float t = (-b - rt_sqrt(disc)) / a2;
            if (key_accept(t, key, best_t, best_key)) {
                best_t = t;
                best_id = idx;
                best_key = key;
            }
        }
        return;
    }
    if (VTX) {
        // {key, v0 | v1, v2.x | v2.yz, v3.xy | v3.z}: edges, normal, offset and
        // inner normals exactly as compile_polygon (rt_context.cpp) forms them
        const f3 v0 = mk(c0.y, c0.z, c0.w), v1 = mk(c1.x, c1.y, c1.z), v2 = mk(c1.w, c2.x, c2.y);
        const f3 n = cross(sub(v1, v0), sub(v2, v1));
        const float dd = -dot(n, v0);
        const float nd = n.x * d.x + n.y * d.y + n.z * d.z;
        if (fabsf(nd) < RT_NEAR_ZERO) return;
        const float t = -((n.x * o.x + n.y * o.y + n.z * o.z) + dd) / nd;
        if (!key_accept(t, key, best_t, best_key)) return;
        const f3 P = add(o, scale(t, d));
        // (the edges formed again where they are needed: fewer live registers)
        if (dot(cross(n, sub(v1, v0)), sub(P, v0)) < 0.0f) return;
        if (dot(cross(n, sub(v2, v1)), sub(P, v1)) < 0.0f) return;
        if (kind == 2) {
            if (dot(cross(n, sub(v0, v2)), sub(P, v2)) < 0.0f) return;
        } else {
            const float4 c3 = *reinterpret_cast<const float4*>(r + 12);  // v3.z
            const f3 v3 = mk(c2.z, c2.w, c3.x);
            if (dot(cross(n, sub(v3, v2)), sub(P, v2)) < 0.0f) return;
            if (dot(cross(n, sub(v0, v3)), sub(P, v3)) < 0.0f) return;
        }
        best_t = t;
        best_id = (kind == 2 ? K.n_sph + K.n_pln : K.n_sph + K.n_pln + K.n_tri) + idx;
        best_key = key;
        return;
    }
    const float nd = c0.y * d.x + c0.z * d.y + c0.w * d.z;
    if (fabsf(nd) < RT_NEAR_ZERO) return;
    const float t = -((c0.y * o.x + c0.z * o.y + c0.w * o.z) + c1.x) / nd;
    if (!key_accept(t, key, best_t, best_key)) return;
    const f3 P = add(o, scale(t, d));
    if (dot(mk(c2.x, c2.y, c2.z), sub(P, mk(c1.y, c1.z, c1.w))) < 0.0f) return;
    const float4 c3 = *reinterpret_cast<const float4*>(r + 12);  // v1.yz, in1.xy
    const float4 c4 = *reinterpret_cast<const float4*>(r + 16);  // in1.z, v2.xyz
#if defined(__HIP_DEVICE_COMPILE__)
    // c4 in one 16-byte load here (edge 2's v2 rides along): otherwise the
    // compiler loads in1.z alone and v2 again with in2, one more wave-load
    // of the same line
    asm volatile("" ::"v"(c4.y), "v"(c4.z), "v"(c4.w));
#endif
    if (dot(mk(c3.z, c3.w, c4.x), sub(P, mk(c2.w, c3.x, c3.y))) < 0.0f) return;
    const float4 c5 = *reinterpret_cast<const float4*>(r + 20);  // in2.xyz, v3.x
    if (dot(mk(c5.x, c5.y, c5.z), sub(P, mk(c4.y, c4.z, c4.w))) < 0.0f) return;
    if (kind == 3) {
        const float4 c6 = *reinterpret_cast<const float4*>(r + 24);  // v3.yz, in3.xy
        const float4 c7 = *reinterpret_cast<const float4*>(r + 28);  // in3.z
        if (dot(mk(c6.z, c6.w, c7.x), sub(P, mk(c5.w, c6.x, c6.y))) < 0.0f) return;
    }
    best_t = t;
    best_id = (kind == 2 ? K.n_sph + K.n_pln : K.n_sph + K.n_pln + K.n_tri) + idx;
    best_key = key;
}

// ---- camera, shading fold, output -------------------------------------------
// Main.cu:287-290: pixelPosition (integer W/2, H/2, no half-pixel offset),
// (rotLeft * rotUp) * pixelPosition, normalize
RT_HD f3 primary_dir(const rt_kparams& K, int x, int y) {
    const f3 pix = mk((float)(x - K.width / 2), (float)(y - K.height / 2), K.screen_z);
    const f3 pr = mk(K.rot[0] * pix.x + K.rot[1] * pix.y + K.rot[2] * pix.z,
                     K.rot[3] * pix.x + K.rot[4] * pix.y + K.rot[5] * pix.z,
                     K.rot[6] * pix.x + K.rot[7] * pix.y + K.rot[8] * pix.z);
    return normalize3(pr);
}

// Fold of the recursion innermost-first (Main.cu:262-268):
//   L = emitted + (brdf * L) * cosAngle,  emitted = emittance * albedo,
//   brdf = kspec * {1,1,1} (specular) or 4 * albedo (diffuse, :259).
RT_HD void fold_level(int c0, float k, float c, const float* hit_tab, float& lx, float& ly, float& lz) {
    // hit table (rt_context.cpp put_material): [4..6] emitted = emittance *
    // albedo, [12..14] diffuse brdf = (2/(1-specularChance)) * albedo, both
    // formed on the host with the same single float multiplications
    const bool spec = c0 < 0;
    const float* h = hit_tab + RT_HIT_FLOATS * (spec ? ~c0 : c0);
    const float4 e = *reinterpret_cast<const float4*>(h + 4);
    const float4 da = *reinterpret_cast<const float4*>(h + 12);
    const float bx = spec ? k : da.x, by = spec ? k : da.y, bz = spec ? k : da.z;
    lx = e.x + (bx * lx) * c;
    ly = e.y + (by * ly) * c;
    lz = e.z + (bz * lz) * c;
}

RT_HD unsigned to_u8(float v) {
    float r = roundf(v);
    if (r != r) return 0u;  // NaN -> 0
    if (r <= 0.0f) return 0u;
    if (r >= 255.0f) return 255u;
    return (unsigned)r;
}

// Main.cu:305-312: frameSum / n -> ACES (Math.cuh:253-262) -> gamma
// (Math.cuh:249-251) -> *255 -> round -> uchar4(r, g, b, 255)
RT_HD unsigned tone_map(float ax, float ay, float az, unsigned n) {
    const float inv = 1.0f / (float)n;
    float v[3] = {inv * ax, inv * ay, inv * az};
    unsigned px = 0xff000000u;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        float cc = 0.6f * v[ch];  // color *= 0.6
        float num = cc * (2.51f * cc + 0.03f);
        float den = cc * (2.43f * cc + 0.59f) + 0.14f;
        float tm = fminf(num / den, 1.0f);  // clamp(color, 1.0f): upper only
        float g = rt_sqrt(tm) * 255.0f;
        px |= to_u8(g) << (8 * ch);
    }
    return px;
}

}  // namespace
