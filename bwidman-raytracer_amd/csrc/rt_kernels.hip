// rt_kernels.hip — CDNA4 (gfx950) path-tracing kernels.
//
// Hot path of the reference (/root/reference/bwidman-raytracer/src):
//   launchRaytracer  Main.cu:274-315   -> rt_render_kernel
//   tracePath        Main.cu:208-272   -> iterative bounce loop + LDS record fold
//   BRDF helpers     Main.cu:111-206   -> shade()
//   intersections    Intersection.cuh  -> closest_hit()
//   initializeRand   Main.cu:368-380   -> rt_init_rand_kernel
//
// Design:
//  * one ray per lane (wave64), one pixel per lane, 256-lane workgroups;
//  * ALL `samples` progressive frames of a pixel run in ONE launch: the RNG
//    state (6 x u32) and the frameSum accumulator stay in VGPRs across
//    frames, so HBM sees 24+12 B read and 24+12+4 B written per pixel per
//    launch instead of per frame;
//  * in-lane path regeneration: a lane whose path terminated (miss or depth
//    limit) starts its next frame's camera ray in the very next iteration
//    instead of idling until the wave's longest path ends; a wave-wide
//    ballot decides when the wave is done.  Each pixel still consumes its
//    RNG stream and accumulates its frames strictly in order, so results are
//    identical to the frame-by-frame reference;
//  * the recursion's per-depth (emitted, brdf, cos) records live in an LDS
//    stack [(level*7+field)][lane] (conflict-free: bank = lane) and are
//    folded innermost-first when the path ends:
//        L = e_k + (b_k * L) * c_k   (Main.cu:268 evaluated by recursion)
//    which reproduces the recursive evaluation order bit for bit;
//  * the primitive loop index is wave-uniform, so primitive data come
//    through scalar loads (SGPR operands of the VALU tests), not VGPRs;
//  * every float op is one IEEE rounding in reference order (built with
//    -ffp-contract=off; correctly rounded div/sqrt); no MFMA (branchy
//    per-ray math, not a contraction).
#include <hip/hip_runtime.h>

#include "rt_layout.h"

namespace {

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) {
    f3 r;
    r.x = x;
    r.y = y;
    r.z = z;
    return r;
}
// Math.cuh:43-121, same operation order
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 scale(float k, f3 v) { return mk(k * v.x, k * v.y, k * v.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    float i = a.y * b.z - a.z * b.y;
    float j = -(a.x * b.z - a.z * b.x);
    float k = a.x * b.y - a.y * b.x;
    return mk(i, j, k);
}
__device__ __forceinline__ float length3(f3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
__device__ __forceinline__ f3 normalize3(f3 v) { return scale(1.0f / length3(v), v); }
__device__ __forceinline__ float square(float x) { return x * x; }
__device__ __forceinline__ float chi(float x) { return (x > 0.0f) ? 1.0f : 0.0f; }

// ---- cuRAND XORWOW (curand_kernel.h, CUDA 12.0; Main.cu:377, Math.cuh:278)
struct Xorwow {
    unsigned d, v0, v1, v2, v3, v4;
};

__device__ __forceinline__ unsigned next_u32(Xorwow& s) {
    unsigned t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1;
    s.v1 = s.v2;
    s.v2 = s.v3;
    s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v4 + s.d;
}

// Math.cuh:277-279: float(u)/INT_MAX*0.5f*max, INT_MAX -> 2^31 exactly
// Every step after the u32 -> float rounding is an exact power-of-two
// scaling, so the value equals u * (2^-32 * max) with max in {1, 2}.
__device__ __forceinline__ float rand_range(Xorwow& s, float max) {
    float u = (float)next_u32(s);
    return u * (2.3283064365386963e-10f * max);
}

// ---- transcendentals: the exact operation sequence of oracle.c
// (Cody-Waite reduction + Cephes minimax polynomials, no FMA).
#define FOPI 1.27323954473516f
#define DP1 0.78515625f
#define DP2 2.4187564849853515625e-4f
#define DP3 3.77489497744594108e-8f

__device__ __forceinline__ float poly_sin(float r, float z) {
    float p = -1.9515295891e-4f * z;
    p = p + 8.3321608736e-3f;
    p = p * z;
    p = p - 1.6666654611e-1f;
    p = p * z;
    p = p * r;
    return p + r;
}

__device__ __forceinline__ float poly_cos(float z) {
    float p = 2.443315711809948e-5f * z;
    p = p - 1.388731625493765e-3f;
    p = p * z;
    p = p + 4.166664568298827e-2f;
    p = p * z;
    p = p * z;
    p = p - 0.5f * z;
    return p + 1.0f;
}

__device__ __forceinline__ float reduce_quadrant(float x, int& jout) {
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
__device__ __forceinline__ void sincos_nn(float x, float& s, float& c) {
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

__device__ __forceinline__ float atan_nn(float x) {  // orc_atanf
    const bool xneg = x < 0.0f;
    if (xneg) x = -x;
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
    return xneg ? -y : y;
}

// ---- BRDF helpers (Main.cu:111-206)
// rough2 = roughness * roughness (precomputed: the reference evaluates
// roughness * roughness * tanTheta * tanTheta left to right, Main.cu:119)
__device__ __forceinline__ float shadowing_masking(f3 dir, f3 n, f3 m, float rough2) {
    float vdn = dot(dir, n);
    float tan_theta = fmaxf(1.0f / (vdn * vdn) - 1.0f, 0.0f);
    return chi(dot(dir, m) / vdn) * 2.0f / (1.0f + sqrtf(1.0f + rough2 * tan_theta * tan_theta));
}

// fresnel(i, m, 1, ior) with ior2m1 = ior*ior/(1*1) - 1 precomputed
__device__ __forceinline__ float fresnel(f3 incident, f3 normal, float ior2m1) {
    float c = fabsf(dot(incident, normal));
    float g_root = ior2m1 + c * c;
    if (g_root < 0.0f) return 1.0f;
    float g = sqrtf(g_root);
    return 0.5f * square(g - c) / square(g + c) *
           (1.0f + square(c * (g + c) - 1.0f) / square(c * (g - c) + 1.0f));
}

__device__ __forceinline__ float specular_weight(f3 i, f3 o, f3 n, f3 m, float rough2) {
    float g = shadowing_masking(i, n, m, rough2) * shadowing_masking(o, n, m, rough2);
    if (isnan(g)) return 1.0f;
    float den = fabsf(dot(i, n) * dot(m, n));
    if (den == 0.0f) den = RT_NEAR_ZERO;
    return fabsf(dot(i, m)) * g / den;
}

// genRandomDirection (Main.cu:193-206): rejection-sampled ball point,
// normalised, flipped into the hemisphere of `normal` (may be non-unit).
__device__ __forceinline__ f3 random_direction(Xorwow& s, f3 normal) {
    f3 r;
    do {
        float x = rand_range(s, 2.0f) - 1.0f;
        float y = rand_range(s, 2.0f) - 1.0f;
        float z = rand_range(s, 2.0f) - 1.0f;
        r = mk(x, y, z);
        // length(r) > 1 (Main.cu:197) <=> RN(x*x+y*y+z*z) > 1 + 2^-23: sqrt is
        // correctly rounded, so RN(sqrt(s)) > 1 iff s >= 1 + 2^-22 (checked
        // exhaustively in tests/test_numerics.py)
    } while (r.x * r.x + r.y * r.y + r.z * r.z > 1.00000012f);
    r = normalize3(r);
    if (dot(normal, r) < 0.0f) r = sub(r, scale(2.0f * dot(r, normal), normal));
    return r;
}

// ---- closest hit over the whole scene (Main.cu:217-234 + Intersection.cuh)
// The loop index is wave-uniform: primitive fields are scalar loads.  Only
// (t, primitive id) of the running closest hit are tracked; the hit point
// and attributes are recomputed for the winner, which is bit-identical to
// the reference's eager copies (same t, same expressions).
__device__ __forceinline__ bool polygon_edges(const float* __restrict__ q, int nv, f3 P) {
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

__device__ __forceinline__ void polygon_test(const float* __restrict__ q, int nv, f3 o, f3 d, int id,
                                             float& best_t, int& best_id) {
    float nx = q[0], ny = q[1], nz = q[2], dd = q[3];
    float nd = nx * d.x + ny * d.y + nz * d.z;
    if (!(fabsf(nd) < RT_NEAR_ZERO)) {
        float t = -((nx * o.x + ny * o.y + nz * o.z) + dd) / nd;
        // plane part (fresh planeInfo, distance = INFINITY), then the
        // polygon's own distance test (Intersection.cuh:118-122)
        bool plane_hit = !(t <= RT_NEAR_ZERO || t > INFINITY);
        if (plane_hit && !(t <= RT_NEAR_ZERO || t > best_t)) {
            f3 P = add(o, scale(t, d));
            if (polygon_edges(q + 4, nv, P)) {
                best_t = t;
                best_id = id;
            }
        }
    }
}

__device__ __forceinline__ void closest_hit(const rt_kparams& K, f3 o, f3 d, float& best_t, int& best_id) {
    const float a = dot(d, d);
    const float a4 = 4.0f * a;
    const float a2 = 2.0f * a;
    best_t = INFINITY;
    best_id = -1;
    const int pln_base = K.n_sph;
    const int tri_base = K.n_sph + K.n_pln;
    const int quad_base = tri_base + K.n_tri;
    for (int i = 0; i < K.n_max; i++) {
        if (i < K.n_sph) {  // Intersection.cuh:15-62
            const float* s = K.sph + RT_SPH_FLOATS * i;
            f3 xp = mk(o.x - s[0], o.y - s[1], o.z - s[2]);
            float b = 2.0f * dot(xp, d);
            float c = dot(xp, xp) - s[3];
            float disc = b * b - a4 * c;
            // exact early-out: b >= 0 (finite disc, a2 > 0) gives -b - sqrt(disc) <= 0,
            // i.e. t <= 0 <= nearZero, rejected by the reference as well
            if (!(disc < 0.0f) && !(b >= 0.0f && disc == disc && a2 > 0.0f)) {
                float t = (-b - sqrtf(disc)) / a2;
                if (!(t <= RT_NEAR_ZERO || t > best_t)) {
                    best_t = t;
                    best_id = i;
                }
            }
        }
        if (i < K.n_pln) {  // Intersection.cuh:64-106
            const float* q = K.pln + RT_PLN_FLOATS * i;
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
        if (i < K.n_tri) polygon_test(K.tri + RT_TRI_FLOATS * i, 3, o, d, tri_base + i, best_t, best_id);
        if (i < K.n_quad) polygon_test(K.quad + RT_QUAD_FLOATS * i, 4, o, d, quad_base + i, best_t, best_id);
    }
}

__device__ __forceinline__ unsigned to_u8(float v) {
    float r = roundf(v);
    if (r != r) return 0u;  // NaN -> 0
    if (r <= 0.0f) return 0u;
    if (r >= 255.0f) return 255u;
    return (unsigned)r;
}

// Main.cu:305-312: frameSum / n -> ACES (Math.cuh:253-262) -> gamma
// (Math.cuh:249-251) -> *255 -> round -> uchar4(r, g, b, 255)
__device__ __forceinline__ unsigned tone_map(float ax, float ay, float az, unsigned n) {
    const float inv = 1.0f / (float)n;
    float v[3] = {inv * ax, inv * ay, inv * az};
    unsigned px = 0xff000000u;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        float cc = 0.6f * v[ch];  // color *= 0.6
        float num = cc * (2.51f * cc + 0.03f);
        float den = cc * (2.43f * cc + 0.59f) + 0.14f;
        float tm = fminf(num / den, 1.0f);  // clamp(color, 1.0f): upper only
        float g = sqrtf(tm) * 255.0f;
        px |= to_u8(g) << (8 * ch);
    }
    return px;
}

// Per-lane pixel state ------------------------------------------------------
struct PixelState {
    long p;         // shard pixel index
    bool valid;
    Xorwow rs;
    float ax, ay, az;  // frameSum
    f3 d0;          // normalize(rot * pixelPosition): the same every frame
    int passes_left;
    unsigned frame;
};

__device__ __forceinline__ void load_pixel(const rt_kparams& K, long npix, long p, PixelState& s) {
    s.p = p;
    s.valid = p < npix;
    s.passes_left = 0;
    s.frame = K.first_frame;
    if (!s.valid) return;
    const int j = (int)(p / K.width);
    const int x = (int)(p - (long)j * K.width);
    const int y = K.row_offset + j * K.row_stride;
    s.rs.d = K.rng[0 * npix + p];
    s.rs.v0 = K.rng[1 * npix + p];
    s.rs.v1 = K.rng[2 * npix + p];
    s.rs.v2 = K.rng[3 * npix + p];
    s.rs.v3 = K.rng[4 * npix + p];
    s.rs.v4 = K.rng[5 * npix + p];
    s.ax = s.ay = s.az = 0.0f;
    if (K.first_frame != 1u) {
        s.ax = K.accum[0 * npix + p];
        s.ay = K.accum[1 * npix + p];
        s.az = K.accum[2 * npix + p];
    }
    // Main.cu:287-290: pixelPosition, rotLeft*rotUp*pixelPosition, normalize
    const f3 pix = mk((float)(x - K.width / 2), (float)(y - K.height / 2), K.screen_z);
    const f3 pr = mk(K.rot[0] * pix.x + K.rot[1] * pix.y + K.rot[2] * pix.z,
                     K.rot[3] * pix.x + K.rot[4] * pix.y + K.rot[5] * pix.z,
                     K.rot[6] * pix.x + K.rot[7] * pix.y + K.rot[8] * pix.z);
    s.d0 = normalize3(pr);
    s.passes_left = K.samples;
}

__device__ __forceinline__ void store_pixel(const rt_kparams& K, long npix, const PixelState& s) {
    const long p = s.p;
    K.rng[0 * npix + p] = s.rs.d;
    K.rng[1 * npix + p] = s.rs.v0;
    K.rng[2 * npix + p] = s.rs.v1;
    K.rng[3 * npix + p] = s.rs.v2;
    K.rng[4 * npix + p] = s.rs.v3;
    K.rng[5 * npix + p] = s.rs.v4;
    K.accum[0 * npix + p] = s.ax;
    K.accum[1 * npix + p] = s.ay;
    K.accum[2 * npix + p] = s.az;
    if (K.rgba) K.rgba[p] = tone_map(s.ax, s.ay, s.az, s.frame - 1u);
}

}  // namespace

// LDS layout: [hit table, n_prim*12 floats, if HIT_LDS] then the record stack
// of the recursion, 3 dwords per level per lane, lane-minor:
//   code[l][lane] (int: primitive id, ~id for a specular bounce),
//   kspec[l][lane] (specular brdf scalar), cosang[l][lane]
// (bank = lane: conflict-free for any per-lane depth).
//
// Persistent lanes: the grid covers the GPU once (occupancy-sized); lane g
// renders pixels g, g+T, g+2T, ... (T = lanes in the grid), each for all
// K.samples frames, regenerating its next path in the iteration after the
// previous one ends.  A wave ends when all its lanes ran out of pixels.
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 1
#endif

template <int BLOCK, bool HIT_LDS>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU)))
rt_render_kernel(rt_kparams K) {
    extern __shared__ float smem[];
    const int tid = threadIdx.x;
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    const float* hit_tab = K.hit;
    float* rec_base = smem;
    if (HIT_LDS) {
        for (int i = tid; i < n_prim * RT_HIT_FLOATS; i += BLOCK) smem[i] = K.hit[i];
        __syncthreads();
        hit_tab = smem;
        rec_base = smem + ((n_prim * RT_HIT_FLOATS + 3) & ~3);
    }
    int* rec_code = reinterpret_cast<int*>(rec_base) + tid;
    float* rec_k = rec_base + (K.max_bounces + 1) * BLOCK + tid;
    float* rec_c = rec_base + 2 * (K.max_bounces + 1) * BLOCK + tid;

    const long npix = (long)K.rows * K.width;
    const long T = (long)gridDim.x * BLOCK;
    PixelState px;
    load_pixel(K, npix, (long)blockIdx.x * BLOCK + tid, px);

    f3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
    int depth = -1;  // -1: needs a camera ray for its next frame
    const f3 cam = mk(K.cam_pos[0], K.cam_pos[1], K.cam_pos[2]);

    while (true) {
        // (1) regenerate: jittered camera ray (Main.cu:290-292)
        if (depth < 0 && px.passes_left > 0) {
            f3 jit = random_direction(px.rs, px.d0);
            d = normalize3(add(px.d0, scale(K.jitter, jit)));
            o = cam;
            depth = 0;
        }
        const bool active = depth >= 0;
        if (__ballot(active) == 0ull) break;
        if (active) {
            // (2) closest hit (Main.cu:214-234)
            float t;
            int id;
            closest_hit(K, o, d, t, id);

            bool finished = true;
            if (id >= 0) {
                // (3) shade (Main.cu:237-264)
                const float* h = hit_tab + RT_HIT_FLOATS * id;
                const float4 h0 = *reinterpret_cast<const float4*>(h);
                const float4 h1 = *reinterpret_cast<const float4*>(h + 4);
                const float4 h2 = *reinterpret_cast<const float4*>(h + 8);
                const f3 P = add(o, scale(t, d));
                f3 n = mk(h0.x, h0.y, h0.z);
                if (h0.w != 0.0f) n = normalize3(sub(P, n));  // sphere: centre -> normal
                const f3 albedo = mk(h1.x, h1.y, h1.z);
                const float rough = h2.x, ior2m1 = h2.y, rough2 = h2.z;

                f3 scatter;
                int code = id;
                float kspec = 0.0f;
                const float choice = rand_range(px.rs, 1.0f);
                if (choice < RT_SPECULAR_CHANCE) {
                    // genMicrofacetNormal (Main.cu:170-185)
                    const float e1 = rand_range(px.rs, 1.0f);
                    const float e2 = rand_range(px.rs, 1.0f);
                    const float theta = atan_nn(rough * sqrtf(e1) / sqrtf(1.0f - e1));
                    const float phi = 2.0f * RT_PI * e2;
                    float st, ct, sp, cp;
                    sincos_nn(theta, st, ct);
                    sincos_nn(phi, sp, cp);
                    const f3 mloc = mk(st * cp, st * sp, ct);
                    // baseAroundNormalToRegular (Main.cu:149-168)
                    f3 some = mk(1.0f, 0.0f, 0.0f);
                    if (fabsf(dot(n, some)) < 1.0f - RT_NEAR_ZERO) some = mk(0.0f, 1.0f, 0.0f);
                    const f3 t1 = cross(n, some);
                    const f3 t2 = cross(n, t1);
                    const f3 m = mk(dot(mk(t1.x, t2.x, n.x), mloc), dot(mk(t1.y, t2.y, n.y), mloc),
                                    dot(mk(t1.z, t2.z, n.z), mloc));
                    scatter = sub(d, scale(2.0f * dot(d, m), m));  // reflect, Main.cu:187-191
                    const f3 inc = scale(-1.0f, d);
                    const float fr = fresnel(inc, m, ior2m1);
                    const float sw = specular_weight(inc, scatter, n, m, rough2);
                    kspec = sw * fr / RT_SPECULAR_CHANCE;  // brdf = (s*F/0.5) * {1,1,1}
                    code = ~id;
                } else {
                    scatter = random_direction(px.rs, n);  // brdf = 4 * albedo
                }
                (void)albedo;
                rec_code[depth * BLOCK] = code;
                rec_k[depth * BLOCK] = kspec;
                rec_c[depth * BLOCK] = dot(scatter, n);  // cosAngle, Main.cu:264
                depth++;
                o = P;
                d = scatter;
                finished = depth > K.max_bounces;  // Main.cu:210
            }
            if (finished) {
                // (4) fold the recursion innermost-first (Main.cu:262-268):
                //     L = emitted + (brdf * L) * cosAngle
                float lx = 0.0f, ly = 0.0f, lz = 0.0f;  // backgroundColor
                for (int l = depth - 1; l >= 0; --l) {
                    const int c0 = rec_code[l * BLOCK];
                    const float k = rec_k[l * BLOCK];
                    const float c = rec_c[l * BLOCK];
                    const bool spec = c0 < 0;
                    const float4 mat = *reinterpret_cast<const float4*>(hit_tab + RT_HIT_FLOATS * (spec ? ~c0 : c0) + 4);
                    const float ex = mat.w * mat.x, ey = mat.w * mat.y, ez = mat.w * mat.z;  // emittance * albedo
                    const float dk = (float)(2.0 / (1 - RT_SPECULAR_CHANCE));                 // 4.0f
                    const float bx = spec ? k : dk * mat.x, by = spec ? k : dk * mat.y, bz = spec ? k : dk * mat.z;
                    lx = ex + (bx * lx) * c;
                    ly = ey + (by * ly) * c;
                    lz = ez + (bz * lz) * c;
                }
                // (5) progressive accumulation (Main.cu:299-304), spp = 1
                if (px.frame == 1u) {
                    px.ax = 0.0f;
                    px.ay = 0.0f;
                    px.az = 0.0f;
                }
                px.ax = px.ax + lx;
                px.ay = px.ay + ly;
                px.az = px.az + lz;
                px.frame++;
                px.passes_left--;
                depth = -1;
                if (px.passes_left == 0) {  // pixel done: write back, take the next one
                    store_pixel(K, npix, px);
                    load_pixel(K, npix, px.p + T, px);
                }
            }
        }
    }
}

// initializeRand (Main.cu:369-380): curand_init(y*W + x, 0, 0)
__global__ void __launch_bounds__(256) rt_init_rand_kernel(unsigned* rng, int width, int rows,
                                                           int row_offset, int row_stride) {
    const long npix = (long)rows * width;
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    const int j = (int)(p / width);
    const int x = (int)(p - (long)j * width);
    const int y = row_offset + j * row_stride;
    const unsigned long long seed = (unsigned long long)(long long)(y * width + x);
    const unsigned s0 = (unsigned)seed ^ 0xaad26b49u;
    const unsigned s1 = (unsigned)(seed >> 32) ^ 0xf7dcefddu;
    const unsigned t0 = 1099087573u * s0;
    const unsigned t1 = 2591861531u * s1;
    rng[0 * npix + p] = 6615241u + t1 + t0;
    rng[1 * npix + p] = 123456789u + t0;
    rng[2 * npix + p] = 362436069u ^ t0;
    rng[3 * npix + p] = 521288629u + t1;
    rng[4 * npix + p] = 88675123u ^ t1;
    rng[5 * npix + p] = 5783321u + t0;
}

// Multi-GPU gather epilogue: block r of `gathered` holds rows r, r+G, ...
__global__ void __launch_bounds__(256) rt_deinterleave_kernel(const unsigned* __restrict__ gathered,
                                                              unsigned* __restrict__ image, int width,
                                                              int height, int shards, int rows_per_shard) {
    const long n = (long)height * width;
    const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const int y = (int)(q / width);
    const int x = (int)(q - (long)y * width);
    const int r = y % shards;
    const int j = y / shards;
    image[q] = gathered[((long)r * rows_per_shard + j) * width + x];
}

// ---- launchers (host side) ------------------------------------------------
namespace {
template <int BLOCK, bool HIT_LDS>
hipError_t launch_render(const rt_kparams& K, size_t lds, int grid_cap, hipStream_t stream) {
    const long npix = (long)K.rows * K.width;
    long grid = (npix + BLOCK - 1) / BLOCK;
    if (grid_cap > 0 && grid > grid_cap) grid = grid_cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((rt_render_kernel<BLOCK, HIT_LDS>), dim3((unsigned)grid), dim3(BLOCK), lds, stream, K);
    return hipGetLastError();
}

template <int BLOCK, bool HIT_LDS>
int resident_blocks_per_cu(size_t lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rt_render_kernel<BLOCK, HIT_LDS>, BLOCK, lds) != hipSuccess)
        return 0;
    return n;
}
}  // namespace

// LDS bytes of one workgroup: hit table (if staged) + 3 record dwords per
// level per lane.
size_t rt_render_lds_bytes(const rt_kparams& K, int block, bool hit_lds) {
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    const size_t hit = hit_lds ? (size_t)((n_prim * RT_HIT_FLOATS + 3) & ~3) * sizeof(float) : 0;
    return hit + (size_t)3 * (K.max_bounces + 1) * block * sizeof(float);
}

// Host-side launch policy: 256-lane workgroups (64 for very deep paths),
// hit table in LDS when it fits in 16 KB, persistent grid of
// waves_per_cu-many resident workgroups per CU (0 = one per 256 pixels).
hipError_t rt_launch_render(const rt_kparams& K, int num_cus, int grid_mult, hipStream_t stream) {
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    const bool hit_lds = (size_t)n_prim * RT_HIT_FLOATS * sizeof(float) <= 16384;
    const bool small_block = (size_t)3 * (K.max_bounces + 1) * 256 * sizeof(float) > 32768;
    const int block = small_block ? 64 : 256;
    const size_t lds = rt_render_lds_bytes(K, block, hit_lds);
    int per_cu = 0;
    if (grid_mult > 0) {
        if (small_block)
            per_cu = hit_lds ? resident_blocks_per_cu<64, true>(lds) : resident_blocks_per_cu<64, false>(lds);
        else
            per_cu = hit_lds ? resident_blocks_per_cu<256, true>(lds) : resident_blocks_per_cu<256, false>(lds);
    }
    const int cap = (grid_mult > 0 && per_cu > 0) ? per_cu * num_cus * grid_mult : 0;
    if (small_block)
        return hit_lds ? launch_render<64, true>(K, lds, cap, stream) : launch_render<64, false>(K, lds, cap, stream);
    return hit_lds ? launch_render<256, true>(K, lds, cap, stream) : launch_render<256, false>(K, lds, cap, stream);
}

hipError_t rt_launch_init_rand(unsigned* rng, int width, int rows, int row_offset, int row_stride,
                               hipStream_t stream) {
    const long npix = (long)rows * width;
    const unsigned grid = (unsigned)((npix + 255) / 256);
    hipLaunchKernelGGL(rt_init_rand_kernel, dim3(grid), dim3(256), 0, stream, rng, width, rows,
                       row_offset, row_stride);
    return hipGetLastError();
}

hipError_t rt_launch_deinterleave(const unsigned* gathered, unsigned* image, int width, int height,
                                  int shards, int rows_per_shard, hipStream_t stream) {
    const long n = (long)height * width;
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(rt_deinterleave_kernel, dim3(grid), dim3(256), 0, stream, gathered, image,
                       width, height, shards, rows_per_shard);
    return hipGetLastError();
}
