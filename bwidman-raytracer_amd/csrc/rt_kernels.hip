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

#include <cstdio>
#include <type_traits>

#include "rt_diag.h"
#include "rt_layout.h"
#include "rt_path.h"

namespace {
// ---- BVH closest hit (wave-synchronous walk; rt_path.h has the pieces) ----
__device__ __forceinline__ void closest_hit_bvh(const rt_kparams& K, f3 o, f3 d, float& best_t, int& best_id) {
    if (!bvh_safe(K, o, d)) {  // NaN/inf rays, overflowing tests: the reference's interleaved loop
        closest_hit_brute(K, o, d, best_t, best_id);
        return;
    }
    const float a = dot(d, d);
    const float a4 = 4.0f * a;
    const float a2 = 2.0f * a;
    best_t = INFINITY;
    best_id = -1;
    int best_key = -1;
    planes_first(K, o, d, best_t, best_id, best_key);
    const SlabRay sr = slab_ray(o, d);
    // node array of the ray's direction octant (near children first)
    const float* nodes = K.bvh_nodes + (size_t)ray_octant(K, d) * K.bvh_order_stride;
    // speculative while-while traversal (Aila & Laine): a lane that reaches a
    // leaf its ray enters parks it and walks on; the parked leaves are tested
    // together once every lane has one parked (or ran out of nodes, or
    // reached a second leaf, where it waits), so the primitive tests run on
    // full waves and no lane idles in the node loop while others search.
    int node = 0;
    while (true) {
        int leaf = -1;
        while (true) {
            bool stalled = false;
            if (node >= 0) {
                RT_BRANCH_COUNT(K, 5);
                const float4 lo = *reinterpret_cast<const float4*>(nodes + 8 * node);
                const float4 hi = *reinterpret_cast<const float4*>(nodes + 8 * node + 4);
                const bool hit = slab_enter(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, sr, best_t);
                const int miss = __float_as_int(lo.w);
                const int lf = __float_as_int(hi.w);
                if (!hit) {
                    node = miss;
                } else if (lf < 0) {
                    node = node + 1;
                } else if (leaf < 0) {
                    leaf = lf;  // park it, walk on
                    node = miss;
                } else {
                    stalled = true;  // second leaf: revisit after the parked one
                }
            }
            if (__all(leaf >= 0 || node < 0 || stalled)) break;
        }
        if (!__any(leaf >= 0)) break;
        if (leaf >= 0) {
            const int first = leaf & 0xffffff, count = leaf >> 24;
            for (int k = 0; k < count; k++) {
                RT_BRANCH_COUNT(K, 6);
                leaf_test(K, K.bvh_leafrec + (size_t)RT_LEAF_FLOATS * (first + k), o, d, a2, a4, best_t, best_id,
                          best_key);
            }
        }
    }
}

template <bool BVH, bool QUADS = true>
__device__ __forceinline__ void closest_hit(const rt_kparams& K, f3 o, f3 d, float& best_t, int& best_id) {
    if (BVH)
        closest_hit_bvh(K, o, d, best_t, best_id);
    else
        closest_hit_brute<QUADS>(K, o, d, best_t, best_id);
}

// Per-lane pixel state ------------------------------------------------------
// RT_NT_PIXEL (default 3): the pixel-state streams (RNG, frameSum, RGBA8;
// each touched once per launch) as non-temporal loads (bit 0) and stores
// (bit 1).  Steady-state A/B (profiles/r06q, r06s): c3 -0.28 %, c4 -0.27 %,
// c5 -0.23 % kernel time, shards flat; HBM bytes +10 % (not the bound)
#ifndef RT_NT_PIXEL
#define RT_NT_PIXEL 3
#endif
// RT_NT_GREC (A/B knob, default 0): a global record's one read, at the path's
// fold, non-temporal
#ifndef RT_NT_GREC
#define RT_NT_GREC 0
#endif
template <typename T>
__device__ __forceinline__ T px_ld(const T* a) {
    if (RT_NT_PIXEL & 1) return __builtin_nontemporal_load(a);
    return *a;
}
template <typename T>
__device__ __forceinline__ void px_st(T* a, T v) {
    if (RT_NT_PIXEL & 2) __builtin_nontemporal_store(v, a);
    else *a = v;
}
struct PixelState {
    long w;         // work item (lane slot in the tiled launch order)
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
    s.rs.d = px_ld(&K.rng[0 * npix + p]);
    s.rs.v0 = px_ld(&K.rng[1 * npix + p]);
    s.rs.v1 = px_ld(&K.rng[2 * npix + p]);
    s.rs.v2 = px_ld(&K.rng[3 * npix + p]);
    s.rs.v3 = px_ld(&K.rng[4 * npix + p]);
    s.rs.v4 = px_ld(&K.rng[5 * npix + p]);
    s.ax = s.ay = s.az = 0.0f;
    if (K.first_frame != 1u) {
        s.ax = px_ld(&K.accum[0 * npix + p]);
        s.ay = px_ld(&K.accum[1 * npix + p]);
        s.az = px_ld(&K.accum[2 * npix + p]);
    }
    s.d0 = primary_dir(K, x, y);  // Main.cu:287-290
    s.passes_left = K.samples;
}

// Launch order: work item w -> pixel.  Items come in groups of 64 (one
// wave) covering a tile_w x (64/tile_w) pixel tile, tiles row-major over the
// shard; tile_w = 0 keeps the linear order (item = pixel).  Square-ish tiles
// keep a wave's rays spatially coherent (a pixel-scrambled order costs +45 %).
// tile_sq: every 4 consecutive waves form a 2 x 2 block of tiles (a 4-wave
// group then covers a square-ish patch), the tile grid padded to even sizes
__host__ __device__ inline long launch_items(const rt_kparams& K) {
    if (K.tile_w <= 0) return (long)K.rows * K.width;
    const int tw = K.tile_w, th = 64 / K.tile_w;
    long tiles_x = (K.width + tw - 1) / tw, tiles_y = (K.rows + th - 1) / th;
    if (K.tile_sq) {
        tiles_x += tiles_x & 1;
        tiles_y += tiles_y & 1;
    }
    return tiles_x * tiles_y * 64;
}

__device__ __forceinline__ long items_of(const rt_kparams& K, long npix) {
    return K.tile_w <= 0 ? npix : launch_items(K);
}

__device__ __forceinline__ long item_to_pixel(const rt_kparams& K, long npix, long w) {
    if (K.tile_w <= 0) return w < npix ? w : npix;
    const int tw = K.tile_w, th = 64 / K.tile_w;
    const long tiles_x = (K.width + tw - 1) / tw;
    const long wave = w >> 6;
    const int l = (int)(w & 63);
    long tx, ty;
    if (K.tile_sq) {
        const long sx = (tiles_x + 1) >> 1, sw = wave >> 2;
        tx = (sw % sx) * 2 + (wave & 1);
        ty = (sw / sx) * 2 + ((wave >> 1) & 1);
    } else {
        tx = wave % tiles_x;
        ty = wave / tiles_x;
    }
    const long x = tx * tw + (l % tw);
    const long j = ty * th + (l / tw);
    if (x >= K.width || j >= K.rows) return npix;
    return j * K.width + x;
}

__device__ __forceinline__ void load_item(const rt_kparams& K, long npix, long nitems, long w, PixelState& s) {
    load_pixel(K, npix, w < nitems ? item_to_pixel(K, npix, w) : npix, s);
    s.w = w;
}

__device__ __forceinline__ void store_pixel(const rt_kparams& K, long npix, const PixelState& s) {
    const long p = s.p;
    px_st(&K.rng[0 * npix + p], s.rs.d);
    px_st(&K.rng[1 * npix + p], s.rs.v0);
    px_st(&K.rng[2 * npix + p], s.rs.v1);
    px_st(&K.rng[3 * npix + p], s.rs.v2);
    px_st(&K.rng[4 * npix + p], s.rs.v3);
    px_st(&K.rng[5 * npix + p], s.rs.v4);
    px_st(&K.accum[0 * npix + p], s.ax);
    px_st(&K.accum[1 * npix + p], s.ay);
    px_st(&K.accum[2 * npix + p], s.az);
#if RT_NT_PIXEL & 2
    if (K.rgba) px_st(&K.rgba[p], tone_map(s.ax, s.ay, s.az, s.frame - 1u));
#else
    if (K.rgba) K.rgba[p] = tone_map(s.ax, s.ay, s.az, s.frame - 1u);
#endif
}

typedef __attribute__((address_space(3))) float lds_float;

__device__ __forceinline__ int lanes_below(unsigned long long mask) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                          __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

// RT_KEY of a primitive id (spheres, planes, triangles, quads in turn); -1 for -1
__device__ __forceinline__ int prim_key(const rt_kparams& K, int id) {
    const int e_pln = K.n_sph, e_tri = e_pln + K.n_pln, e_quad = e_tri + K.n_tri;
    return id < 0 ? -1
                  : id < e_pln ? RT_KEY(0, id)
                               : id < e_tri ? RT_KEY(1, id - e_pln)
                                            : id < e_quad ? RT_KEY(2, id - e_tri) : RT_KEY(3, id - e_quad);
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
// s_setprio of the wave that runs SPEC tasks during the execute step (the
// longest wave there; measured 0.882 -> 0.876 ms); 0 disables
// occupancy target of the sorted kernel with global-memory records (LDS no
// longer bounds it): 7 waves/SIMD (config 4: 6.36 -> 6.08 ms vs the default
// target; 8 spills and gains nothing)
#ifndef RT_GREC_WAVES
#define RT_GREC_WAVES 7
#endif
// global-record launches keep this many shallow record levels in LDS
// (3 dwords per level per lane; 2 still fits 7 waves/SIMD of the sorted kernel)
#ifndef RT_GREC_LDS_LEVELS
#define RT_GREC_LDS_LEVELS 2
#endif
#ifndef RT_SPEC_PRIO
#define RT_SPEC_PRIO 3
#endif
// occupancy target of the pair kernel
#ifndef RT_PAIR_WAVES
#define RT_PAIR_WAVES 7
#endif

template <int BLOCK, bool HIT_LDS, bool BVH>
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
    const long nitems = items_of(K, npix);
    PixelState px;
    load_item(K, npix, nitems, (long)blockIdx.x * BLOCK + tid, px);

    f3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
    int depth = -1;  // -1: needs a camera ray for its next frame
    const f3 cam = mk(K.cam_pos[0], K.cam_pos[1], K.cam_pos[2]);
    // samplesPerPixel (Main.cu:296-299): the frame's camera ray and the
    // paths still to trace from it
    f3 dcam = d;
    int inner = 1;

    while (true) {
        // (1) regenerate: jittered camera ray (Main.cu:290-292)
        if (depth < 0 && px.passes_left > 0) {
            f3 jit = random_direction(px.rs, px.d0);
            d = normalize3(add(px.d0, scale(K.jitter, jit)));
            o = cam;
            depth = 0;
            dcam = d;
            inner = K.spp_inner;
        }
        const bool active = depth >= 0;
        if (__ballot(active) == 0ull) break;
        if (active) {
            // (2) closest hit (Main.cu:214-234)
            float t;
            int id;
            closest_hit<BVH>(K, o, d, t, id);

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
                    const float theta = atan_nn(rough * sqrt_cr(e1) / sqrt_cr(1.0f - e1));
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
                float lx = K.bg[0], ly = K.bg[1], lz = K.bg[2];  // backgroundColor
                for (int l = depth - 1; l >= 0; --l)
                    fold_level(rec_code[l * BLOCK], rec_k[l * BLOCK], rec_c[l * BLOCK], hit_tab, lx, ly, lz);
                if (inner > 1) {  // `pixel = tracePath(...)` again from the same camera ray
                    inner--;
                    o = cam;
                    d = dcam;
                    depth = 0;
                    continue;
                }
                if (K.spp_inner != 1) {  // pixel /= samplesPerPixel: (1.0f / k) * pixel
                    const float k = 1.0f / (float)K.spp_inner;
                    lx = k * lx;
                    ly = k * ly;
                    lz = k * lz;
                }
                // (5) progressive accumulation (Main.cu:299-304)
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
                    load_item(K, npix, nitems, px.w + T, px);
                }
            }
        }
    }
}

#ifndef RT_TU_BVH  // defined once, in the main translation unit
// initializeRand (Main.cu:369-380): curand_init(y*W + x, 0, 0)
// Launch-order feedback: one workgroup turns the last launch's tile-group
// durations into the next launch's order, most expensive first (longest
// processing time first: the frame's last workgroups are then the cheap
// ones, so the chip drains quickly).  Counting sort over 512 logarithmic cost
// buckets (exponent and top 4 mantissa bits of float(cost): 1/16-octave
// steps, no max pass); the order within a bucket is whatever the LDS
// atomics give, which is harmless: every pixel's result is independent of
// when its group runs.
__device__ __forceinline__ int order_bucket(unsigned cost) {
    const int k = (int)(__float_as_uint((float)cost + 1.0f) >> 19) - (127 << 4);  // 0 .. 512
    return 511 - min(k, 511);
}

__global__ void __launch_bounds__(1024) rt_order_groups_kernel(const unsigned* __restrict__ cost,
                                                               int* __restrict__ order, int n) {
    __shared__ unsigned hist[512];
    __shared__ unsigned wsum[8];
    const int tid = threadIdx.x;
    if (tid < 512) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) atomicAdd(&hist[order_bucket(cost[i])], 1u);
    __syncthreads();
    // exclusive scan of the 512 buckets: waves 0..7, one bucket per lane
    unsigned v = 0, incl = 0;
    if (tid < 512) {
        v = hist[tid];
        incl = v;
        for (int m = 1; m < 64; m <<= 1) {
            const unsigned u = __shfl_up(incl, m);
            if ((tid & 63) >= m) incl += u;
        }
        if ((tid & 63) == 63) wsum[tid >> 6] = incl;
    }
    __syncthreads();
    if (tid < 512) {
        unsigned base = 0;
        for (int w = 0; w < (tid >> 6); w++) base += wsum[w];
        hist[tid] = base + incl - v;
    }
    __syncthreads();
    for (int i = tid; i < n; i += 1024) order[atomicAdd(&hist[order_bucket(cost[i])], 1u)] = i;
}

__global__ void __launch_bounds__(256) rt_init_rand_kernel(unsigned* rng, int width, int rows,
                                                           int row_offset, int row_stride) {
    const long npix = (long)rows * width;
    const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    const int j = (int)(p / width);
    const int x = (int)(p - (long)j * width);
    const int y = row_offset + j * row_stride;
    const Xorwow s = xorwow_seed(pixel_seed(x, y, width));
    rng[0 * npix + p] = s.d;
    rng[1 * npix + p] = s.v0;
    rng[2 * npix + p] = s.v1;
    rng[3 * npix + p] = s.v2;
    rng[4 * npix + p] = s.v3;
    rng[5 * npix + p] = s.v4;
}

// Multi-GPU gather epilogue: block r of `gathered` holds rows r, r+G, ...
// VEC = 4: 16 bytes (4 pixels) per lane (width % 4 == 0, 16-byte aligned
// buffers); a grid-stride loop, so the launch may cap its grid and leave the
// CUs to a render running beside it
template <int VEC>
__global__ void __launch_bounds__(256) rt_deinterleave_kernel(const unsigned* __restrict__ gathered,
                                                              unsigned* __restrict__ image, int width,
                                                              int height, int shards, int rows_per_shard) {
    typedef typename std::conditional<VEC == 4, uint4, unsigned>::type word;
    const int wv = width / VEC;
    const long n = (long)height * wv;
    for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x) {
        const int y = (int)(q / wv);
        const int x = (int)(q - (long)y * wv);
        const int r = y % shards;
        const int j = y / shards;
        reinterpret_cast<word*>(image)[q] = reinterpret_cast<const word*>(gathered)[((long)r * rows_per_shard + j) * wv + x];
    }
}
#endif  // RT_TU_BVH



enum { T_NONE = 0, T_REGEN = 1, T_DIFF = 2, T_SPEC = 3 };  // a lane's next task

// ===========================================================================
// Sorted task-queue megakernel (the product path).
//
// Divergence, not memory, bounds the simple one-path-per-lane kernel: in a
// wave, lanes that need a camera ray, a specular bounce or a diffuse bounce
// execute all three code paths one after the other (rocprof: 20 of 64 lanes
// active per VALU instruction).  Here each workgroup iterates in lock-step:
//
//   T-phase: every lane with pending work posts ONE task into an LDS queue:
//            RANDDIR tasks (camera-jitter direction for a new frame, or a
//            diffuse bounce: both are genRandomDirection, Main.cu:193-206)
//            fill slots from the front, SPEC tasks (Main.cu:245-255) from
//            the back; wave w then executes slots 64w..64w+63, so each wave
//            runs one task kind (at most one wave holds both).  The task
//            carries the lane's RNG state (6 x u32) and returns it updated,
//            so every pixel still consumes its own stream in reference order.
//   I-phase: every lane with a ray runs closest_hit (uniform code), draws its
//            brdfChoice, and posts the shading task for the next T-phase; a
//            miss (or the depth limit) folds the path's records, accumulates
//            the frame and schedules the pixel's next camera ray.
//
// LDS: [hit table][record stack 3 x levels x BLOCK]
//      [task slots 13 x BLOCK, field-major][2 x 2 queue counters]
// GREC: the record levels >= RT_GREC_LDS_LEVELS in global memory (deep paths
// and full frames, launch policy).  BVH scenes take the ray-refill kernel.
template <int BLOCK, bool HIT_LDS, bool GREC, bool ORDER = false, bool QUADS = true>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(GREC ? RT_GREC_WAVES : RT_WAVES_PER_EU)))
rt_render_sorted_kernel(rt_kparams K) {
    extern __shared__ float smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    const float* hit_tab = K.hit;
    float* rec_base = smem;
    if (HIT_LDS) {
        for (int i = tid; i < n_prim * RT_HIT_FLOATS; i += BLOCK) smem[i] = K.hit[i];
        hit_tab = smem;
        rec_base = smem + ((n_prim * RT_HIT_FLOATS + 3) & ~3);
    }
    // levels 0 .. max_bounces-1 in LDS; the deepest level (max_bounces) ends
    // the path in the round it is made, so it is folded straight from the
    // lane's own task slot (fields 4..6, free once the result is taken)
    const int levels = K.max_bounces;
    // record stack: LDS [level][field][lane] (a level's three fields BLOCK
    // dwords apart: one per-lane address, the fields as immediate offsets);
    // GREC: only the shallow levels 0 .. LL-1 in LDS, the deep ones (rarely
    // reached) in global memory, [group][level - LL][field][lane] (each
    // group's records contiguous and coalesced), so LDS leaves room for
    // RT_GREC_WAVES waves and few records ever leave the CU
    const int LL = GREC ? (levels < RT_GREC_LDS_LEVELS ? levels : RT_GREC_LDS_LEVELS) : levels;
    // (an LDS-address-space pointer: 32-bit address arithmetic, no 64-bit
    // base held across the loop)
    lds_float* rec = (lds_float*)(rec_base + tid);
    const int GL = levels - LL;
    float* grec = GREC ? K.rec + (long)blockIdx.x * 3 * GL * BLOCK + tid : rec_base;
    float* slots = rec_base + 3 * LL * BLOCK;
    int* counters = reinterpret_cast<int*>(slots + 13 * BLOCK);
    // counters[0..3]: queue fronts/backs (2 parities)
    const long npix = (long)K.rows * K.width;
    const long nitems = items_of(K, npix);
    if (tid < 4) counters[tid] = 0;
    diag_group_start(K);
    __syncthreads();
#define SLOT(f, i) slots[(f) * BLOCK + (i)]
// task results {r.xyz, kspec, rng[6]}, written back over the slot's own
// fields {0..3, 7..12}
#define RES(f, i) slots[((f) < 4 ? (f) : (f) + 3) * BLOCK + (i)]

    // tile-group of this workgroup (launch-order feedback, rt_layout.h)
    // (the start time is parked in group_cost[] itself: nothing stays live
    // across the loop)
    // ORDER: launch-order feedback instantiation (the pointers it needs after
    // the loop cost SGPRs, so launches without feedback use the plain one)
    const long group = ORDER && K.group_order ? (long)K.group_order[blockIdx.x] : (long)blockIdx.x;
    if (ORDER && tid == 0) K.group_cost[group] = (unsigned)__builtin_amdgcn_s_memrealtime();
    PixelState px;
    // (tid < BLOCK always holds; the guard keeps the register allocation and
    // schedule of the measured kernel: without it the instruction stream
    // differs in 55 places, `make asm`)
    load_item(K, npix, nitems, tid < BLOCK ? group * BLOCK + tid : nitems, px);
    int mode = px.passes_left > 0 ? T_REGEN : T_NONE;

    f3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
    f3 hn = o;  // pending hit's normal (its point is o)
    int hid = 0, depth = 0;
    bool has_ray = false;
    int parity = 0;
    const f3 cam = mk(K.cam_pos[0], K.cam_pos[1], K.cam_pos[2]);

    // path end: fold, accumulate (Main.cu:299-304), next frame / next pixel
    auto finish_path = [&](int slot) {
        // L = emitted + (brdf * L) * cosAngle, innermost level first; `x`
        // reads each record value (identity; opaque in RT_PHASE_TWICE == 4)
        auto fold_path = [&](auto x, float& lx, float& ly, float& lz) {
            if (depth > K.max_bounces)  // deepest level, parked in the slot
                fold_level(__float_as_int(x(SLOT(6, slot))), x(SLOT(4, slot)), x(SLOT(5, slot)), hit_tab, lx, ly, lz);
            const int nrec = depth > K.max_bounces ? K.max_bounces : depth;
            if (GREC)
                for (int l = nrec - 1; l >= LL; --l) {
                    const float* r = grec + 3 * (l - LL) * BLOCK;
#if RT_NT_GREC
                    // (the record's last read: non-temporal)
                    fold_level(__float_as_int(x(__builtin_nontemporal_load(&r[0]))), x(__builtin_nontemporal_load(&r[BLOCK])),
                               x(__builtin_nontemporal_load(&r[2 * BLOCK])), hit_tab, lx, ly, lz);
#else
                    fold_level(__float_as_int(x(r[0])), x(r[BLOCK]), x(r[2 * BLOCK]), hit_tab, lx, ly, lz);
#endif
                }
            for (int l = (nrec < LL ? nrec : LL) - 1; l >= 0; --l) {
                const lds_float* r = rec + 3 * l * BLOCK;
                fold_level(__float_as_int(x(r[0])), x(r[BLOCK]), x(r[2 * BLOCK]), hit_tab, lx, ly, lz);
            }
        };
        float lx = K.bg[0], ly = K.bg[1], lz = K.bg[2];  // backgroundColor (Main.cu:209-211)
        fold_path(DiagIdent(), lx, ly, lz);
        RT_TWICE_FOLD(K, fold_path);
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
        // one pixel per lane (the grid covers every work item): a finished
        // pixel is stored after the loop, by the whole wave at once, and the
        // camera set-up constants are not live inside the loop
        mode = px.passes_left > 0 ? T_REGEN : T_NONE;
    };
    bool ended = false;  // path ended this round: finish_path() once, after the I-phase

    SortedStamps dg;  // diagnostic builds only (rt_diag.h)
    while (true) {
        const int task = mode;
        dg.stamp(7);
        // every owner has read its previous task result out of the slots
        // before any wave overwrites them with this round's tasks
        __syncthreads();
        dg.stamp(0);

        // ---- T-phase: enqueue (front: RANDDIR, back: SPEC)
        int* cnt = counters + 2 * parity;
        const bool front = task == T_REGEN || task == T_DIFF;
        const unsigned long long mf = __ballot(front);
        const unsigned long long mbk = __ballot(task == T_SPEC);
        int base_f = 0, base_b = 0;
        if (lane == 0) {
            if (mf) base_f = atomicAdd(&cnt[0], __popcll(mf));
            if (mbk) base_b = atomicAdd(&cnt[1], __popcll(mbk));
        }
        base_f = __builtin_amdgcn_readfirstlane(base_f);
        base_b = __builtin_amdgcn_readfirstlane(base_b);
        int slot = -1;
        if (front) slot = base_f + lanes_below(mf);
        if (task == T_SPEC) slot = BLOCK - 1 - (base_b + lanes_below(mbk));
        if (slot >= 0) {
            const f3 nrm = task == T_REGEN ? px.d0 : hn;
            SLOT(0, slot) = nrm.x;
            SLOT(1, slot) = nrm.y;
            SLOT(2, slot) = nrm.z;
            SLOT(3, slot) = d.x;
            SLOT(4, slot) = d.y;
            SLOT(5, slot) = d.z;
            // code: primitive id (bounce) or -1 (camera ray)
            SLOT(6, slot) = __int_as_float(task == T_REGEN ? -1 : hid);
            SLOT(7, slot) = __uint_as_float(px.rs.d);
            SLOT(8, slot) = __uint_as_float(px.rs.v0);
            SLOT(9, slot) = __uint_as_float(px.rs.v1);
            SLOT(10, slot) = __uint_as_float(px.rs.v2);
            SLOT(11, slot) = __uint_as_float(px.rs.v3);
            SLOT(12, slot) = __uint_as_float(px.rs.v4);
        }
        dg.stamp(1);
        __syncthreads();
        dg.stamp(2);
        // no task anywhere in the workgroup: every lane is idle (rays are
        // always consumed in the round that made them), so the group is done
        const int nf = cnt[0], nb = cnt[1];
        if (nf + nb == 0) break;

        // ---- T-phase: execute slot `tid`
        {
            const bool do_front = tid < nf;
            const bool do_spec = tid >= BLOCK - nb;
#if RT_SPEC_PRIO
            // the SPEC wave is the longest of the execute step: let it issue first
            const int wave_first = (int)__builtin_amdgcn_readfirstlane((unsigned)(tid & ~63));
            const bool spec_wave = wave_first + 63 >= BLOCK - nb;
            if (spec_wave) __builtin_amdgcn_s_setprio(RT_SPEC_PRIO);
#endif
            if (do_front || do_spec) {
                Xorwow rs;
                rs.d = __float_as_uint(SLOT(7, tid));
                rs.v0 = __float_as_uint(SLOT(8, tid));
                rs.v1 = __float_as_uint(SLOT(9, tid));
                rs.v2 = __float_as_uint(SLOT(10, tid));
                rs.v3 = __float_as_uint(SLOT(11, tid));
                rs.v4 = __float_as_uint(SLOT(12, tid));
                const f3 nrm = mk(SLOT(0, tid), SLOT(1, tid), SLOT(2, tid));
                const int code = __float_as_int(SLOT(6, tid));
                f3 r;
                if (do_front) {
                    RT_TWICE_RANDDIR(rs, nrm);
                    r = random_direction(rs, nrm, dg.rej_ptr());
                    if (code < 0) r = normalize3(add(nrm, scale(K.jitter, r)));  // camera jitter, Main.cu:291-292
                } else {
                    const f3 dd = mk(SLOT(3, tid), SLOT(4, tid), SLOT(5, tid));
                    const float4 h2 = *reinterpret_cast<const float4*>(hit_tab + RT_HIT_FLOATS * code + 8);
                    float kspec;
                    RT_TWICE_SPEC(rs, dd, nrm, h2);
                    r = specular_scatter(rs, dd, nrm, h2.x, h2.z, h2.y, kspec);
                    RES(3, tid) = kspec;
                }
                RES(0, tid) = r.x;
                RES(1, tid) = r.y;
                RES(2, tid) = r.z;
                RES(4, tid) = __uint_as_float(rs.d);
                RES(5, tid) = __uint_as_float(rs.v0);
                RES(6, tid) = __uint_as_float(rs.v1);
                RES(7, tid) = __uint_as_float(rs.v2);
                RES(8, tid) = __uint_as_float(rs.v3);
                RES(9, tid) = __uint_as_float(rs.v4);
            }
            dg.exec(do_front, do_spec);
        }
        dg.stamp(3);
#if RT_SPEC_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        __syncthreads();
        dg.stamp(4);
        if (tid == 0) {
            counters[2 * (parity ^ 1)] = 0;
            counters[2 * (parity ^ 1) + 1] = 0;
        }
        parity ^= 1;

        // ---- owner: take the task result back.  The result direction goes
        // straight into d and the pending hit point already is o (I-phase),
        // so no ray registers are copied here
        if (slot >= 0) {
            d = mk(RES(0, slot), RES(1, slot), RES(2, slot));
            px.rs.d = __float_as_uint(RES(4, slot));
            px.rs.v0 = __float_as_uint(RES(5, slot));
            px.rs.v1 = __float_as_uint(RES(6, slot));
            px.rs.v2 = __float_as_uint(RES(7, slot));
            px.rs.v3 = __float_as_uint(RES(8, slot));
            px.rs.v4 = __float_as_uint(RES(9, slot));
            mode = T_NONE;
            if (task == T_REGEN) {
                o = cam;
                depth = 0;
                has_ray = true;
            } else {
                const int code = task == T_SPEC ? ~hid : hid;
                const float kspec = task == T_SPEC ? RES(3, slot) : 0.0f;
                const float cosang = dot(d, hn);  // cosAngle, Main.cu:264
                if (depth < K.max_bounces) {
                    if (!GREC || depth < LL) {  // (separate stores: LDS and global address spaces)
                        lds_float* r = rec + 3 * depth * BLOCK;
                        r[0] = __int_as_float(code);
                        r[BLOCK] = kspec;
                        r[2 * BLOCK] = cosang;
                    } else {
                        float* r = grec + 3 * (depth - LL) * BLOCK;
                        r[0] = __int_as_float(code);
                        r[BLOCK] = kspec;
                        r[2 * BLOCK] = cosang;
                    }
                    has_ray = true;  // from the hit point o along d
                } else {  // next query would exceed maxBounces (Main.cu:210): the path ends
                    SLOT(4, slot) = kspec;
                    SLOT(5, slot) = cosang;
                    SLOT(6, slot) = __int_as_float(code);
                    ended = true;
                }
                depth++;
            }
        }

        dg.stamp(5);
        dg.rays(has_ray);
        // ---- I-phase: closest hit + brdfChoice (Main.cu:214-245)
        float t = INFINITY;
        int id = -1;
        if (has_ray) {
            RT_TWICE_HIT(QUADS, K, o, d);
            closest_hit_brute<QUADS>(K, o, d, t, id);
        }
        if (has_ray) {
            has_ray = false;
            if (id >= 0) {
                const float4 h0 = *reinterpret_cast<const float4*>(hit_tab + RT_HIT_FLOATS * id);
                o = add(o, scale(t, d));  // the hit point: the next ray's origin
                hn = mk(h0.x, h0.y, h0.z);
                if (h0.w != 0.0f) hn = normalize3(sub(o, hn));  // sphere normal
                hid = id;
                // brdfChoice (Main.cu:243): specular or diffuse bounce next round
                mode = rand_range(px.rs, 1.0f) < RT_SPECULAR_CHANCE ? T_SPEC : T_DIFF;
            } else {
                ended = true;
            }
        }
        if (ended) {
            ended = false;
            finish_path(slot);
        }
        dg.stamp(6);
    }
    if (px.valid && px.passes_left == 0 && px.frame != K.first_frame) store_pixel(K, npix, px);
    // the loop exit is group-uniform (the round that posts no task), so one
    // lane's clock after the loop closes the group's span
    if (ORDER && tid == 0) {
        // the pointers re-read from the kernel arguments (volatile), so they
        // are not held in SGPRs across the loop
        const volatile __attribute__((address_space(4))) rt_kparams* kp =
            (const volatile __attribute__((address_space(4))) rt_kparams*)__builtin_amdgcn_kernarg_segment_ptr();
        int* const ord = kp->group_order;
        unsigned* const cost = kp->group_cost;
        const long g = ord ? (long)__builtin_nontemporal_load(&ord[blockIdx.x]) : (long)blockIdx.x;
        cost[g] = (unsigned)__builtin_amdgcn_s_memrealtime() - cost[g];
    }
    diag_group_end<true>(K);
    dg.flush(K);
#undef SLOT
#undef RES
}

// ---- pair kernel (small frames and shards) --------------------------------
// A 128-lane group of two waves for 64 pixels: wave 0 owns them (lane j
// pixel j of the group's tile), wave 1 is their helper (lane 64 + j works
// for owner j only), so no queue, no counters and no compaction — a wave
// holds at most 64 tasks anyway.  A round (3 barriers):
//   X  execute: the owner runs its pixel's diffuse bounce or camera ray in
//      place (genRandomDirection, Main.cu:193-206, 290-292) and posts the
//      next ray; the helper runs the owner's SPEC task (Main.cu:245-255) from
//      its slot and posts that ray;
//   H  closest hit (Main.cu:214-235): the owner takes its SPEC result back
//      and records the bounce; owner and helper each test every other index
//      i of the reference's interleaved loop on the posted ray, the helper
//      the even ones (index 0 carries the planes), the owner the odd ones
//      (rays that fail bvh_safe: the whole loop on the owner);
//   S  owner and helper merge the halves the same way (the smaller
//      distance, ties to the larger RT_KEY); the helper computes the hit
//      point and normal (Main.cu:237-241) for both, the owner draws
//      brdfChoice (:243), parks a finished path for its fold in the next X
//      phase (Main.cu:262-268, 299-304) and posts a SPEC task.
// Every pixel consumes its RNG stream in the reference's order, so results
// equal the sorted kernel's and the oracle's bit for bit.
// LDS: [hit table][records 3 x max_bounces x 64][exchange PF x 64][live flag]
#define RT_PAIR_FIELDS 25
template <bool HIT_LDS, bool ORDER, bool QUADS>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(RT_PAIR_WAVES)))
rt_render_pair_kernel(rt_kparams K) {
    extern __shared__ float smem[];
    const int tid = threadIdx.x;
    const int j = tid & 63;           // the pixel this lane works for
    const bool owner = tid < 64;      // (wave-uniform)
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    const float* hit_tab = K.hit;
    float* rec_base = smem;
    if (HIT_LDS) {
        for (int i = tid; i < n_prim * RT_HIT_FLOATS; i += 128) smem[i] = K.hit[i];
        hit_tab = smem;
        rec_base = smem + ((n_prim * RT_HIT_FLOATS + 3) & ~3);
    }
    const int levels = K.max_bounces;
    // record stack [level][field][pixel] (the owner's only)
    lds_float* rec = (lds_float*)(rec_base + j);
    // exchange [field][pixel]: 0-2 ray origin (in S the helper overwrites it
    // with the hit point), 3-5 ray direction, 6 ray flag (0 none, 1 split
    // closest hit, 2 whole loop on the owner), 7-8 the helper's half (t, id),
    // 9-11 the hit's normal (written by the helper in S), 12-14 SPEC
    // scattered direction out, 15 SPEC kspec out, 16-21 RNG state (SPEC in /
    // out), 22 SPEC flag (1 posted, 3 posted and its ray traced), 23-24 the
    // owner's (t, id)
    lds_float* xb = (lds_float*)(rec_base + 3 * levels * 64) + j;
#define XF(f) xb[(f) * 64]
    int* live_flag = reinterpret_cast<int*>(rec_base + 3 * levels * 64 + RT_PAIR_FIELDS * 64);
    const long npix = (long)K.rows * K.width;
    const long nitems = items_of(K, npix);
    diag_group_start(K);
    const long group = ORDER && K.group_order ? (long)K.group_order[blockIdx.x] : (long)blockIdx.x;
    if (ORDER && tid == 0) K.group_cost[group] = (unsigned)__builtin_amdgcn_s_memrealtime();
    PixelState px;
    load_item(K, npix, nitems, owner ? group * 64 + j : nitems, px);  // (helpers: no pixel)
    int mode = px.passes_left > 0 ? T_REGEN : T_NONE;  // the owner's task this round
    f3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f), hn = o;
    int hid = 0, depth = 0;
    bool hit = false;   // (owner) last S found a hit: its point and normal come from the helper
    int hflag = 0;      // (helper) the ray flag of this round
    const f3 cam = mk(K.cam_pos[0], K.cam_pos[1], K.cam_pos[2]);
    if (owner) XF(22) = __int_as_float(0);
    __syncthreads();

    bool fold = false;  // a finished path waits for its fold (run in the owner's X phase)
    while (true) {
        // ---- X: execute
        bool has_ray = false, ended = false;
        int dcode = 0;              // deepest level (a bounce at depth max_bounces)
        float dk = 0.0f, dc = 0.0f;
        if (owner) {
            if (fold) {  // fold innermost-first (Main.cu:262-268), accumulate (:299-304)
                fold = false;
                float lx = K.bg[0], ly = K.bg[1], lz = K.bg[2];  // backgroundColor (Main.cu:209-211)
                if (depth > K.max_bounces)  // (the deepest level, parked in XF(6..8))
                    fold_level(__float_as_int(XF(6)), XF(7), XF(8), hit_tab, lx, ly, lz);
                const int nrec = depth > K.max_bounces ? K.max_bounces : depth;
                for (int l = nrec - 1; l >= 0; --l) {
                    const lds_float* q = rec + 3 * l * 64;
                    fold_level(__float_as_int(q[0]), q[64], q[128], hit_tab, lx, ly, lz);
                }
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
            }
            if (hit) {  // the hit point and normal the helper computed in S
                hit = false;
                o = mk(XF(0), XF(1), XF(2));
                hn = mk(XF(9), XF(10), XF(11));
            }
            if (mode == T_REGEN || mode == T_DIFF) {
                f3 r = random_direction(px.rs, mode == T_REGEN ? px.d0 : hn);
                if (mode == T_REGEN) {  // jittered camera ray, Main.cu:290-292
                    d = normalize3(add(px.d0, scale(K.jitter, r)));
                    o = cam;
                    depth = 0;
                    has_ray = true;
                } else {  // diffuse bounce, Main.cu:257-264: brdf = 4 * albedo (fold)
                    const float cosang = dot(r, hn);
                    if (depth < K.max_bounces) {
                        lds_float* q = rec + 3 * depth * 64;
                        q[0] = __int_as_float(hid);
                        q[64] = 0.0f;
                        q[128] = cosang;
                        d = r;
                        has_ray = true;
                    } else {
                        dcode = hid;
                        dc = cosang;
                        ended = true;
                    }
                    depth++;
                }
            }
            if (mode != T_SPEC) {  // (a SPEC lane's ray flag is the helper's)
                const int flag = has_ray ? (bvh_safe(K, o, d) ? 1 : 2) : 0;
                XF(0) = o.x;
                XF(1) = o.y;
                XF(2) = o.z;
                XF(3) = d.x;
                XF(4) = d.y;
                XF(5) = d.z;
                XF(6) = __int_as_float(flag);
            }
        } else {
            const int sf = __float_as_int(XF(22));
            if (sf & 1) {  // the owner's SPEC task, Main.cu:245-255
                Xorwow rs;
                rs.d = __float_as_uint(XF(16));
                rs.v0 = __float_as_uint(XF(17));
                rs.v1 = __float_as_uint(XF(18));
                rs.v2 = __float_as_uint(XF(19));
                rs.v3 = __float_as_uint(XF(20));
                rs.v4 = __float_as_uint(XF(21));
                const f3 nrm = mk(XF(9), XF(10), XF(11));
                const f3 dd = mk(XF(3), XF(4), XF(5));  // the incoming ray
                const float4 h2 = *reinterpret_cast<const float4*>(hit_tab + RT_HIT_FLOATS * hid + 8);
                float kspec;
                const f3 r = specular_scatter(rs, dd, nrm, h2.x, h2.z, h2.y, kspec);
                XF(12) = r.x;
                XF(13) = r.y;
                XF(14) = r.z;
                XF(15) = kspec;
                XF(16) = __uint_as_float(rs.d);
                XF(17) = __uint_as_float(rs.v0);
                XF(18) = __uint_as_float(rs.v1);
                XF(19) = __uint_as_float(rs.v2);
                XF(20) = __uint_as_float(rs.v3);
                XF(21) = __uint_as_float(rs.v4);
                int flag = 0;
                if (sf & 2) {  // traced: the ray from the hit point (posted in XF(0..2))
                    XF(3) = r.x;
                    XF(4) = r.y;
                    XF(5) = r.z;
                    flag = bvh_safe(K, mk(XF(0), XF(1), XF(2)), r) ? 1 : 2;
                }
                XF(6) = __int_as_float(flag);
            }
        }
        __syncthreads();

        // ---- H: SPEC take-back, closest hit halves
        float t = INFINITY;
        int id = -1;
        int rflag = 0;
        if (owner) {
            if (mode == T_SPEC) {
                const f3 r = mk(XF(12), XF(13), XF(14));
                const float kspec = XF(15);
                px.rs.d = __float_as_uint(XF(16));
                px.rs.v0 = __float_as_uint(XF(17));
                px.rs.v1 = __float_as_uint(XF(18));
                px.rs.v2 = __float_as_uint(XF(19));
                px.rs.v3 = __float_as_uint(XF(20));
                px.rs.v4 = __float_as_uint(XF(21));
                const float cosang = dot(r, hn);  // cosAngle, Main.cu:264
                if (depth < K.max_bounces) {
                    lds_float* q = rec + 3 * depth * 64;
                    q[0] = __int_as_float(~hid);
                    q[64] = kspec;
                    q[128] = cosang;
                    d = r;
                    has_ray = true;
                } else {
                    dcode = ~hid;
                    dk = kspec;
                    dc = cosang;
                    ended = true;
                }
                depth++;
            }
            if (has_ray) {
                rflag = __float_as_int(XF(6));
                if (rflag == 1)  // (the odd indices: the owner also took its SPEC result back)
                    closest_hit_brute<QUADS, 2>(K, o, d, t, id, 1);
                else
                    closest_hit_brute<QUADS>(K, o, d, t, id);
                XF(23) = t;
                XF(24) = __int_as_float(id);
            }
        } else {
            hflag = __float_as_int(XF(6));
            if (hflag == 1) {
                closest_hit_brute<QUADS, 2>(K, mk(XF(0), XF(1), XF(2)), mk(XF(3), XF(4), XF(5)), t, id, 0);
                XF(7) = t;
                XF(8) = __int_as_float(id);
            }
        }
        __syncthreads();

        // ---- S: merge, shade, fold, post
        int live = 0;
        if (owner) {
            if (rflag == 1) {  // the helper's half: smaller distance, ties to the larger key
                const float t2 = XF(7);
                const int id2 = __float_as_int(XF(8));
                if (id2 >= 0 && (t2 < t || (t2 == t && prim_key(K, id2) > prim_key(K, id)))) {
                    t = t2;
                    id = id2;
                }
            }
            mode = T_NONE;
            if (has_ray) {
                if (id >= 0) {  // Main.cu:237-245 (the helper computes the point and normal)
                    hid = id;
                    hit = true;
                    mode = rand_range(px.rs, 1.0f) < RT_SPECULAR_CHANCE ? T_SPEC : T_DIFF;  // brdfChoice
                } else {
                    ended = true;
                }
            }
            if (ended) {
                // the fold runs in the next X phase, beside the helper's SPEC
                // tasks (the longer half of X); the deepest level waits in
                // XF(6..8), free until the owner posts its next ray there
                fold = true;
                XF(6) = __int_as_float(dcode);
                XF(7) = dk;
                XF(8) = dc;
                mode = px.passes_left > 1 ? T_REGEN : T_NONE;
            }
            int sf = 0;
            if (mode == T_SPEC) {  // the helper's task next round (its hit, normal and ray it has)
                XF(16) = __uint_as_float(px.rs.d);
                XF(17) = __uint_as_float(px.rs.v0);
                XF(18) = __uint_as_float(px.rs.v1);
                XF(19) = __uint_as_float(px.rs.v2);
                XF(20) = __uint_as_float(px.rs.v3);
                XF(21) = __uint_as_float(px.rs.v4);
                sf = depth < K.max_bounces ? 3 : 1;  // 3: its scattered ray is traced from the hit point
            }
            XF(22) = __int_as_float(sf);
            live = __ballot(mode != T_NONE || fold) != 0ull;
            if (j == 0) *live_flag = live;
        } else if (hflag != 0) {
            // the same merge as the owner's, then the hit point and normal
            // (Main.cu:237-241; the same float operations), for the owner's
            // next X phase and the SPEC task
            float tt = XF(23);
            int ii = __float_as_int(XF(24));
            if (hflag == 1 && id >= 0 && (t < tt || (t == tt && prim_key(K, id) > prim_key(K, ii)))) {
                tt = t;
                ii = id;
            }
            if (ii >= 0) {
                const float4 h0 = *reinterpret_cast<const float4*>(hit_tab + RT_HIT_FLOATS * ii);
                const f3 hp = add(mk(XF(0), XF(1), XF(2)), scale(tt, mk(XF(3), XF(4), XF(5))));
                f3 nn = mk(h0.x, h0.y, h0.z);
                if (h0.w != 0.0f) nn = normalize3(sub(hp, nn));  // sphere normal
                XF(0) = hp.x;
                XF(1) = hp.y;
                XF(2) = hp.z;
                XF(9) = nn.x;
                XF(10) = nn.y;
                XF(11) = nn.z;
                hid = ii;
            }
        }
        __syncthreads();
        if (!owner) live = *live_flag;
        if (!live) break;  // (group-uniform)
    }
#undef XF
    if (px.valid && px.passes_left == 0 && px.frame != K.first_frame) store_pixel(K, npix, px);
    if (ORDER && tid == 0) {
        const volatile __attribute__((address_space(4))) rt_kparams* kp =
            (const volatile __attribute__((address_space(4))) rt_kparams*)__builtin_amdgcn_kernarg_segment_ptr();
        int* const ord = kp->group_order;
        unsigned* const cost = kp->group_cost;
        const long g = ord ? (long)__builtin_nontemporal_load(&ord[blockIdx.x]) : (long)blockIdx.x;
        cost[g] = (unsigned)__builtin_amdgcn_s_memrealtime() - cost[g];
    }
    diag_group_end<true>(K);
}

#ifdef RT_TU_BVH
// ---- BVH kernel with ray refill (large scenes) --------------------------------
// One path per lane like rt_render_kernel, but the BVH walk is not a
// wave-synchronous call: each lane keeps its walk state (node, parked leaf,
// closest hit) across iterations, and once K.refill lanes of a wave have
// finished their walks, those lanes shade their hit and set up their next
// ray while the others stay parked mid-walk (persistent traversal with ray
// refill, Aila & Laine 2009), so the node loop runs on fuller waves instead
// of waiting for each round's slowest ray.  A ray's tests and their
// (t, RT_KEY) acceptance are exactly those of closest_hit_bvh (planes
// first, then every primitive of every leaf whose inflated box the ray may
// enter), so the result does not depend on when the lane walks.
// refill threshold K.refill (of 64, relative to the lanes that still hold a
// pixel; rt_layout.h RT_REFILL): with the spatial-split tree and leaf batches
// at 58 ready lanes, config 5 at 32 / 36 / 40 / 48: 96.4 / 95.0 / 94.9 / 97.8
// ms, its 1/8 shard 21.6 / 21.6 / 22.1 / 22.3 ms
// leaf-test batch threshold K.leaf_batch (lanes of 64 ready; rt_layout.h
// RT_LEAF_BATCH): with one parked leaf, config 5 at 52 / 54 / 56 / 58 / 60 /
// 62 / 64 (all lanes, Aila & Laine's rule): 102.2 / 99.1 / 98.1 / 97.3 / 98.2
// / 101.1 / 118.0 ms, its 1/8 shard 24.8 / 23.4 / 23.0 / 22.3 / 22.2 / 22.3 /
// 25.5 ms; with two, 60 / 62: 91.8 / 92.6 ms, 1/8 shard 21.3 / 20.2 ms
// fp16 bits -> float (exact)
__device__ __forceinline__ float h2f(unsigned bits) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(bits & 0xffffu));
}

// N16: 16-byte nodes (rt_layout.h bvh_nodes16) — one gather per node visit
// instead of two; the walk, its tests and its order are the same.
// ORDER: launch-order feedback as in the sorted kernel (workgroup g renders
// tile-group group_order[g] and records its duration in group_cost[])
// Leaf records in vertex form (rt_layout.h bvh_leafvtx: 64 bytes, the plane
// and inner normals formed in the kernel): config 5 78.6 -> 75.6 ms, 1/2
// shard 43.0 -> 41.4, 1/8 17.63 -> 17.56 (profiles/r05h/ab_vtx_policy.txt);
// the kernel held to 5 waves per SIMD (96 VGPRs; 12 bytes of spills on the
// pixel-load and shading paths)
#ifndef RT_REFILL_WAVES
#define RT_REFILL_WAVES 5
#endif
#ifndef RT_NODE_PAIR
#define RT_NODE_PAIR 1
#endif
template <int BLOCK, bool N16, bool ORDER = false>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(RT_REFILL_WAVES)))
rt_render_bvh_refill_kernel(rt_kparams K) {
    extern __shared__ float smem[];
    const int tid = threadIdx.x;
    const float* hit_tab = K.hit;
    int* rec_code = reinterpret_cast<int*>(smem) + tid;
    float* rec_k = smem + (K.max_bounces + 1) * BLOCK + tid;
    float* rec_c = smem + 2 * (K.max_bounces + 1) * BLOCK + tid;
    const long npix = (long)K.rows * K.width;
    const long T = (long)gridDim.x * BLOCK;
    const long nitems = items_of(K, npix);
    const long group = ORDER && K.group_order ? (long)K.group_order[blockIdx.x] : (long)blockIdx.x;
    if (ORDER && tid == 0) K.group_cost[group] = (unsigned)__builtin_amdgcn_s_memrealtime();
    PixelState px;
    load_item(K, npix, nitems, group * BLOCK + tid, px);
    const f3 cam = mk(K.cam_pos[0], K.cam_pos[1], K.cam_pos[2]);
    diag_group_start(K);
    LaneDone lane_done;  // diagnostic builds only (rt_diag.h)

    f3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
    int depth = -1;          // -1: the next ray is a camera ray
    bool walking = false;    // a BVH walk is in flight
    bool pending = false;    // a finished query waits to be shaded
    bool idle = false;       // no pixel left
    int node = -1, leaf = -1, leaf2 = -1;  // two parked leaves per lane
    float best_t = INFINITY;
    int best_id = -1, best_key = -1;
    SlabRay sr;
    sr.inv = o;
    sr.oinv = o;
    sr.m = 0.0f;
    float a2 = 0.0f, a4 = 0.0f;
    const float* nodes = K.bvh_nodes;
    const unsigned* nodes16 = K.bvh_nodes16;
    const int nn = K.bvh_n_nodes;
    // a walk is live while its node indexes the array: -1 (done) and nn (past
    // a leaf that ends the array: a leaf's miss link is simply node + 1) fail
    // the same unsigned compare, and the leaf test reuses the decoded flag —
    // 39 -> 34 VALU per node step: config 5 86.5 -> 85.7 ms, its 1/8 shard
    // 20.1 -> 19.65 (profiles/r05h/ab_node_step.txt); the 16-byte step below
    // (one address instruction, ~w parked directly, one compare per parked
    // leaf) 34 -> 30 VALU, with leaf records loaded in six 16-byte loads
    // instead of seven (rt_path.h leaf_test): 84.8 -> 84.0 ms, 1/8 shard
    // 19.64 -> 19.36 (profiles/r05h/ab_node_step3.txt).  Keeping the parked
    // leaves as loop-carried lane masks (28 VALU) costs more in mask
    // bookkeeping than it saves: +3 %
#define NODE_LIVE(n) ((unsigned)(n) < (unsigned)nn)
    RefillStamps dg;  // diagnostic builds only (rt_diag.h)
    while (true) {
        dg.count(3);
        // (A) lanes without a walk: shade the finished query, start the next ray
        while (!walking && !idle) {
            if (pending) {
                pending = false;
                diag_bvh_check(K, o, d, best_t, best_id, depth);
                bool finished = true;
                if (best_id >= 0) {  // shade (Main.cu:237-264), as rt_render_kernel
                    const float* h = hit_tab + RT_HIT_FLOATS * best_id;
                    const float4 h0 = *reinterpret_cast<const float4*>(h);
                    const float4 h2 = *reinterpret_cast<const float4*>(h + 8);
                    const f3 P = add(o, scale(best_t, d));
                    f3 n = mk(h0.x, h0.y, h0.z);
                    if (h0.w != 0.0f) n = normalize3(sub(P, n));  // sphere: centre -> normal
                    f3 scatter;
                    int code = best_id;
                    float kspec = 0.0f;
                    const float choice = rand_range(px.rs, 1.0f);
                    if (choice < RT_SPECULAR_CHANCE) {
                        scatter = specular_scatter(px.rs, d, n, h2.x, h2.z, h2.y, kspec);
                        code = ~best_id;
                    } else {
                        scatter = random_direction(px.rs, n);  // brdf = 4 * albedo
                    }
                    rec_code[depth * BLOCK] = code;
                    rec_k[depth * BLOCK] = kspec;
                    rec_c[depth * BLOCK] = dot(scatter, n);  // cosAngle, Main.cu:264
                    depth++;
                    o = P;
                    d = scatter;
                    finished = depth > K.max_bounces;  // Main.cu:210
                }
                if (finished) {  // fold (Main.cu:262-268), accumulate (Main.cu:299-304)
                    float lx = K.bg[0], ly = K.bg[1], lz = K.bg[2];
                    for (int l = depth - 1; l >= 0; --l)
                        fold_level(rec_code[l * BLOCK], rec_k[l * BLOCK], rec_c[l * BLOCK], hit_tab, lx, ly, lz);
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
                    if (px.passes_left == 0) {
                        store_pixel(K, npix, px);
                        load_item(K, npix, nitems, px.w + T, px);
                    }
                }
            }
            if (depth < 0) {
                if (px.passes_left <= 0) {
                    idle = true;
                    lane_done.mark(K);
                    break;
                }
                // jittered camera ray (Main.cu:290-292)
                const f3 jit = random_direction(px.rs, px.d0);
                d = normalize3(add(px.d0, scale(K.jitter, jit)));
                o = cam;
                depth = 0;
            }
            // set up the walk of (o, d): closest_hit_bvh's prologue
            best_t = INFINITY;
            best_id = -1;
            best_key = -1;
            if (!bvh_safe(K, o, d)) {  // NaN/inf rays, overflowing tests: the reference's interleaved loop
                closest_hit_brute(K, o, d, best_t, best_id);
                pending = true;
                continue;
            }
            const float a = dot(d, d);
            a4 = 4.0f * a;
            a2 = 2.0f * a;
            planes_first(K, o, d, best_t, best_id, best_key);  // planes are unbounded: always tested
            sr = slab_ray(o, d);
            const int order = ray_octant(K, d);
            if (N16)
                nodes16 = K.bvh_nodes16 + (size_t)order * nn * 4;
            else
                nodes = K.bvh_nodes + (size_t)order * K.bvh_order_stride;
            node = 0;
            leaf = -1;
            leaf2 = -1;
            walking = true;
        }
        dg.stamp(0);
        if (__ballot(walking) == 0ull) break;  // every lane idle

        // (B) walk until K.refill lanes are waiting for a new ray
        while (true) {
            while (true) {  // node steps; a lane parks the first two leaves its ray enters
                bool stalled = false;
                if (NODE_LIVE(node)) {  // (a live node implies a walk)
                    RT_BRANCH_COUNT(K, 5);
                    // branch-free step: miss -> skip the subtree; internal -> first
                    // child; leaf -> park it (or stall on a third one)
                    if (N16) {
#define RT_N16_STEP(q)                                                                                        \
    do {                                                                                                      \
        const int w = (int)(q).w; /* miss link (internal) or ~leaf (a leaf's miss link is node + 1) */        \
        const bool lnode = w < -1;                                                                            \
        const bool hit = slab_enter(h2f((q).x), h2f((q).x >> 16), h2f((q).y), h2f((q).y >> 16), h2f((q).z), \
                                    h2f((q).z >> 16), sr, best_t);                                            \
        const bool is_leaf = hit && lnode;                                                                    \
        const bool park = is_leaf && leaf2 < 0;                                                               \
        stalled = is_leaf != park;                                                                            \
        const bool first = park && leaf < 0;                                                                  \
        leaf2 = park != first ? ~w : leaf2;                                                                   \
        leaf = first ? ~w : leaf;                                                                             \
        node = !hit && !lnode ? w : (stalled ? node : node + 1);                                              \
    } while (0)
                        const uint4* nq = reinterpret_cast<const uint4*>(nodes16);
                        const uint4 q = nq[(unsigned)node];
#if RT_NODE_PAIR
                        // the next node in array order is loaded with this one:
                        // a step that moves to node + 1 (an internal hit, a
                        // parked or missed leaf) takes it without a second
                        // round trip — config 5 75.9 -> 74.6 ms, its 1/8
                        // shard flat (profiles/r05h/ab_node_pair.txt); the
                        // node after it too (node + 2): 80.0 ms
                        const int node0 = node;
                        const uint4 q1 = nq[min((unsigned)node + 1u, (unsigned)nn - 1u)];
                        RT_N16_STEP(q);
                        asm volatile("" ::"v"(q1.x), "v"(q1.y), "v"(q1.z), "v"(q1.w));
                        if (node == node0 + 1 && NODE_LIVE(node)) RT_N16_STEP(q1);
#else
                        RT_N16_STEP(q);
#endif
#undef RT_N16_STEP
                    } else {
                        const float4 lo = *reinterpret_cast<const float4*>(nodes + 8 * node);
                        const float4 hi = *reinterpret_cast<const float4*>(nodes + 8 * node + 4);
                        const bool hit = slab_enter(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, sr, best_t);
                        const int miss = __float_as_int(lo.w);
                        const int lf = __float_as_int(hi.w);
                        const bool is_leaf = hit && lf >= 0;
                        const bool park = is_leaf && leaf2 < 0;
                        stalled = is_leaf != park;
                        const bool first = park && leaf < 0;
                        leaf2 = park != first ? lf : leaf2;
                        leaf = first ? lf : leaf;
                        node = !hit || park ? miss : (is_leaf ? node : node + 1);
                    }
                }
                // test the parked leaves once K.leaf_batch of the 64 lanes are
                // ready (a leaf parked, the walk done or stalled, no walk);
                // the rest walk on and join a later batch
                dg.count(4);
                // (a lane without a walk has a dead node, and a stalled lane
                // has a parked leaf; two compare masks OR'd on the scalar
                // side: a ballot of anything but one compare costs a
                // v_cndmask + v_cmp per step — config 5 83.9 -> 81.3 ms, its
                // 1/8 shard 19.2 -> 18.3, profiles/r05h/ab_ballot.txt)
                if (__popcll(__ballot(leaf >= 0) | __ballot(!NODE_LIVE(node))) >= K.leaf_batch) break;
            }
            dg.stamp(1);
            dg.count(5);
            if (leaf >= 0) {
                const int first = leaf & 0xffffff, count = leaf >> 24;
                for (int k = 0; k < count; k++) {
                    RT_BRANCH_COUNT(K, 6);
                    leaf_test<true>(K, K.bvh_leafvtx + (size_t)RT_LEAF_VFLOATS * (first + k), o, d, a2, a4, best_t,
                                    best_id, best_key);
                }
                leaf = -1;
            }
            if (leaf2 >= 0) {
                const int first = leaf2 & 0xffffff, count = leaf2 >> 24;
                for (int k = 0; k < count; k++)
                    leaf_test<true>(K, K.bvh_leafvtx + (size_t)RT_LEAF_VFLOATS * (first + k), o, d, a2, a4, best_t,
                                    best_id, best_key);
                leaf2 = -1;
            }
            dg.stamp(2);
            if (walking && !NODE_LIVE(node)) {  // walk complete: the query result is best_t / best_id
                walking = false;
                pending = true;
            }
            const unsigned long long w = __ballot(walking);
            // K.refill of 64 relative to the lanes that still have a pixel, so a
            // wave's tail (pixels done, lanes idle) keeps refilling: config 5
            // 120.4 -> 117.4 ms, its 1/8 shard 26.6 -> 25.6 ms (absolute count)
            // (all 64 lanes are active here: the finished ones are ~w & ~idle)
            const unsigned long long live = ~__ballot(idle);
            if (w == 0ull || 64 * __popcll(~w & live) >= K.refill * __popcll(live)) break;
        }
    }
    if (ORDER && tid == 0) {  // the loop exit is wave-uniform (one wave per group)
        const long g = K.group_order ? (long)K.group_order[blockIdx.x] : (long)blockIdx.x;
        K.group_cost[g] = (unsigned)__builtin_amdgcn_s_memrealtime() - K.group_cost[g];
    }
    diag_group_end<false>(K);
    dg.flush(K);
#undef NODE_LIVE
}
#endif  // RT_TU_BVH

// ---- launchers (host side) ------------------------------------------------
// launch-order feedback applies to grids of more than RT_ORDER_MIN_GEN
// generations of resident groups: 1.5 -> 1.1 turns it on for the c3 1/4
// shard (1.32 generations: 0.297 -> 0.285 ms, two rounds, tools/shard_sweep.py;
// c2 / c3 / c4 at the other shard sizes unchanged within noise)
#ifndef RT_ORDER_MIN_GEN
#define RT_ORDER_MIN_GEN 1.1
#endif
// launch-order feedback: the grid of the last launch that sorted its
// tile-group costs into group_order (0 = none; the context resets it before
// each launch and keeps the value as the order's grid)
extern thread_local long rt_order_groups_last;
// the render kernel the last launch on this thread took (rt_last_kernel_name)
extern thread_local char rt_launched_kernel[96];
hipError_t rt_launch_order_groups(const unsigned* cost, int* order, long n, hipStream_t stream);

namespace {
// render kernels: one path per lane (A/B reference, samplesPerPixel > 1),
// the sorted task-queue kernel (full frames), the pair kernel (small frames
// and shards: 128 lanes for 64 pixels)
enum { K_SIMPLE = 0, K_SORTED = 1, K_PAIR = 2 };

template <int KIND, int BLOCK, bool HIT_LDS, bool BVH = false, bool GREC = false, bool ORDER = false, bool QUADS = true>
void* kernel_ptr() {
    if constexpr (KIND == K_PAIR) return reinterpret_cast<void*>(&rt_render_pair_kernel<HIT_LDS, ORDER, QUADS>);
    if constexpr (KIND == K_SORTED)
        return reinterpret_cast<void*>(&rt_render_sorted_kernel<BLOCK, HIT_LDS, GREC, ORDER, QUADS>);
    return reinterpret_cast<void*>(&rt_render_kernel<BLOCK, HIT_LDS, BVH>);
}

template <int KIND, int BLOCK, bool HIT_LDS, bool GREC, bool ORDER, bool QUADS>
void launch_kind(const rt_kparams& K, long grid, size_t lds, hipStream_t stream) {
    if constexpr (KIND == K_PAIR)
        hipLaunchKernelGGL((rt_render_pair_kernel<HIT_LDS, ORDER, QUADS>), dim3((unsigned)grid), dim3(128), lds, stream, K);
    else
        hipLaunchKernelGGL((rt_render_sorted_kernel<BLOCK, HIT_LDS, GREC, ORDER, QUADS>), dim3((unsigned)grid),
                           dim3(BLOCK), lds, stream, K);
}

template <int KIND, int BLOCK, bool HIT_LDS, bool BVH = false, bool GREC = false>
hipError_t launch_render(const rt_kparams& K0, size_t lds, int grid_mult, int num_cus, hipStream_t stream) {
    static_assert(KIND != K_PAIR || (BLOCK == 128 && HIT_LDS && !BVH && !GREC), "pair launches: 128 lanes, 64 pixels");
    static_assert(KIND == K_SIMPLE || !BVH, "BVH scenes: the ray-refill kernel");
    constexpr int OWN = KIND == K_PAIR ? 64 : BLOCK;  // pixels per workgroup
    rt_kparams K = K0;
    const long nitems = launch_items(K);
    long grid = (nitems + OWN - 1) / OWN;  // streaming needs a resident grid only
    if (grid_mult > 0 && KIND == K_SIMPLE) {  // persistent (simple kernel): grid_mult x resident groups per CU x CUs
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel_ptr<KIND, BLOCK, HIT_LDS, BVH>(), BLOCK, lds) ==
                hipSuccess &&
            per_cu > 0) {
            const long cap = (long)per_cu * num_cus * grid_mult;
            if (grid > cap) grid = cap;
        }
    }
    if (grid < 1) grid = 1;
    K.rec_stride = (int)(grid * OWN);
    // launch-order feedback: only where the grid covers every item once
    // (group g <-> tile-group g) and the buffers hold the grid, and only
    // where the grid runs in more than RT_ORDER_MIN_GEN generations of
    // resident groups: LPT order shortens the drain at the end of a
    // multi-generation grid, while a grid that is resident all at once only
    // gets its expensive groups packed onto the same CUs (c3 at 1/8: 0.264
    // vs 0.243 ms with the order; 1/2: 0.493 vs 0.522)
    bool feedback = KIND != K_SIMPLE && K.group_cost && K.group_order && grid <= K.order_cap;
    if (feedback) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel_ptr<KIND, BLOCK, HIT_LDS, BVH, GREC>(), BLOCK,
                                                         lds) != hipSuccess ||
            per_cu <= 0)
            per_cu = 1;
        // (pair launches always: their grid is about one generation, and the
        // order still helped there: c3 1/8 0.212 -> 0.206 ms, 1/16 0.187 ->
        // 0.183, profiles/r04/spread/ab_pair.txt vs ab_prio.txt)
        feedback = KIND == K_PAIR || (double)grid > RT_ORDER_MIN_GEN * (double)per_cu * num_cus;
    }
    if (!feedback) {
        K.group_cost = nullptr;
        K.group_order = nullptr;
    } else if (K.order_n != grid) {
        K.group_order = nullptr;  // no order for this grid yet: blockIdx order
    }
    // brute-force scenes without quads: the quad tests compiled out
    const bool quads = BVH || K.n_quad > 0;
    if constexpr (KIND == K_SIMPLE) {
        hipLaunchKernelGGL((rt_render_kernel<BLOCK, HIT_LDS, BVH>), dim3((unsigned)grid), dim3(BLOCK), lds, stream, K);
    } else {
        if (feedback && quads)
            launch_kind<KIND, BLOCK, HIT_LDS, GREC, true, true>(K, grid, lds, stream);
        else if (feedback)
            launch_kind<KIND, BLOCK, HIT_LDS, GREC, true, false>(K, grid, lds, stream);
        else if (quads)
            launch_kind<KIND, BLOCK, HIT_LDS, GREC, false, true>(K, grid, lds, stream);
        else
            launch_kind<KIND, BLOCK, HIT_LDS, GREC, false, false>(K, grid, lds, stream);
    }
    std::snprintf(rt_launched_kernel, sizeof rt_launched_kernel, "%s<%d%s%s%s>%s",
                  KIND == K_PAIR ? "rt_render_pair_kernel" : KIND == K_SORTED ? "rt_render_sorted_kernel" : "rt_render_kernel",
                  KIND == K_PAIR ? 128 : BLOCK, HIT_LDS ? "" : ",hit_global", GREC ? ",grec" : "", BVH ? ",bvh" : "",
                  feedback ? "+order" : "");
    hipError_t e = hipGetLastError();
    // the sort runs when asked, and always for a grid without an order yet
    if (e == hipSuccess && feedback && (K0.order_sort || K0.order_n != grid)) {
        e = rt_launch_order_groups(K0.group_cost, K0.group_order, grid, stream);
        if (e == hipSuccess) rt_order_groups_last = grid;
    }
    return e;
}

}  // namespace

#ifdef RT_TU_BVH
// The BVH instantiations live in their own translation unit
// (rt_kernels_bvh.hip), built at -O3: the traversal loops want the full
// optimizer while the brute-force kernels are faster at -O1.
// BVH scenes: the ray-refill kernel, 64-lane groups (no barriers)
hipError_t rt_launch_render_bvh_refill(const rt_kparams& K0, int num_cus, hipStream_t s) {
    constexpr int BLOCK = 64;
    rt_kparams K = K0;
    const long nitems = launch_items(K);
    const long grid = (nitems + BLOCK - 1) / BLOCK < 1 ? 1 : (nitems + BLOCK - 1) / BLOCK;
    const size_t lds = (size_t)3 * (K.max_bounces + 1) * BLOCK * sizeof(float);
    // launch-order feedback (as launch_render): only for grids of more than
    // RT_ORDER_MIN_GEN generations of resident groups
    bool feedback = K.group_cost && K.group_order && grid <= K.order_cap;
    if (feedback) {
        int per_cu = 0;
        const void* kp = K.bvh_nodes16 ? reinterpret_cast<const void*>(&rt_render_bvh_refill_kernel<BLOCK, true, true>)
                                       : reinterpret_cast<const void*>(&rt_render_bvh_refill_kernel<BLOCK, false, true>);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, BLOCK, lds) != hipSuccess || per_cu <= 0)
            per_cu = 1;
        feedback = (double)grid > RT_ORDER_MIN_GEN * (double)per_cu * num_cus;
    }
    if (!feedback) {
        K.group_cost = nullptr;
        K.group_order = nullptr;
    } else if (K.order_n != grid) {
        K.group_order = nullptr;  // no order for this grid yet: blockIdx order
    }
    const bool n16 = K.bvh_nodes16 != nullptr;
    if (feedback && n16)
        hipLaunchKernelGGL((rt_render_bvh_refill_kernel<BLOCK, true, true>), dim3((unsigned)grid), dim3(BLOCK), lds, s, K);
    else if (feedback)
        hipLaunchKernelGGL((rt_render_bvh_refill_kernel<BLOCK, false, true>), dim3((unsigned)grid), dim3(BLOCK), lds, s, K);
    else if (n16)
        hipLaunchKernelGGL((rt_render_bvh_refill_kernel<BLOCK, true>), dim3((unsigned)grid), dim3(BLOCK), lds, s, K);
    else
        hipLaunchKernelGGL((rt_render_bvh_refill_kernel<BLOCK, false>), dim3((unsigned)grid), dim3(BLOCK), lds, s, K);
    std::snprintf(rt_launched_kernel, sizeof rt_launched_kernel, "rt_render_bvh_refill_kernel<64%s>%s",
                  n16 ? ",n16" : "", feedback ? "+order" : "");
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && feedback && (K0.order_sort || K0.order_n != grid)) {
        e = rt_launch_order_groups(K0.group_cost, K0.group_order, grid, s);
        if (e == hipSuccess) rt_order_groups_last = grid;
    }
    return e;
}

// BVH scenes with samplesPerPixel > 1 (or BWRT_KERNEL=simple): the
// one-path-per-lane kernel with the wave-synchronous BVH walk
hipError_t rt_launch_render_bvh_simple(const rt_kparams& K, int block, size_t lds, int grid_mult, int num_cus,
                                       hipStream_t s) {
    return block == 64 ? launch_render<K_SIMPLE, 64, false, true>(K, lds, grid_mult, num_cus, s)
                       : launch_render<K_SIMPLE, 256, false, true>(K, lds, grid_mult, num_cus, s);
}
#else
hipError_t rt_launch_render_bvh_simple(const rt_kparams& K, int block, size_t lds, int grid_mult, int num_cus,
                                       hipStream_t s);
hipError_t rt_launch_render_bvh_refill(const rt_kparams& K, int num_cus, hipStream_t s);

size_t rt_render_lds_bytes(const rt_kparams& K, int block, bool hit_lds, bool sorted);
// LDS bytes of one pair-kernel group (hit table in LDS)
size_t rt_pair_lds_bytes(const rt_kparams& K) {
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    return (size_t)((n_prim * RT_HIT_FLOATS + 3) & ~3) * sizeof(float) +
           (size_t)(3 * (K.max_bounces > 0 ? K.max_bounces : 0) + RT_PAIR_FIELDS) * 64 * sizeof(float) + 4 * sizeof(int);
}

namespace {
template <int BLOCK, int KIND>
hipError_t launch_block(const rt_kparams& K, bool hit_lds, size_t lds, int grid_mult, int num_cus, hipStream_t s) {
    if constexpr (KIND == K_SIMPLE) {
        if (K.bvh_nodes)  // large scenes: hit table in global memory, BVH traversal
            return rt_launch_render_bvh_simple(K, BLOCK, lds, grid_mult, num_cus, s);
    }
    if (KIND == K_SORTED && K.rec)  // record stack in global memory
        return hit_lds ? launch_render<KIND, BLOCK, true, false, true>(K, lds, grid_mult, num_cus, s)
                       : launch_render<KIND, BLOCK, false, false, true>(K, lds, grid_mult, num_cus, s);
    return hit_lds ? launch_render<KIND, BLOCK, true>(K, lds, grid_mult, num_cus, s)
                   : launch_render<KIND, BLOCK, false>(K, lds, grid_mult, num_cus, s);
}
}  // namespace

// Launch policy for the sorted kernel's record stack: global memory when the
// LDS stack (3 dwords per level per lane) would hold the brute-force kernel
// below RT_WAVES_PER_EU waves per SIMD, i.e. deep paths.  Measured: config
// 4 (maxBounces 6) 4 -> 7 waves/SIMD, 7.61 -> 6.34 ms.
// Also when global records let more 256-lane groups reside per CU (runtime
// occupancy of both instantiations) and the frame runs at least
// RT_GREC_MIN_GEN generations of them: config 3 (maxBounces 4) 6 -> 7
// waves/SIMD, 0.816 -> 0.801 ms (three alternating runs); re-measured in
// round 5 on its row shards (`profiles/r05b/ab_grec_shards.txt`): 1/2 (2.26
// generations) 0.460 -> 0.453 ms, 1/3 (1.51) 0.335 -> 0.322, but 1/4 (1.13)
// 0.270 -> 0.277; config 2 gains no group.  A third shape, one LDS level at
// 8 waves per SIMD (64 VGPRs, 8-byte spill), makes the 1/4 shard one resident
// generation (0.99) instead of 1.32, and loses there: 0.298 vs 0.270 ms with
// LDS records, 1/2 0.455 vs 0.42, full frame flat (round 6, two alternating
// runs, profiles/r06a/ab_grec.txt; the code: profiles/r06a/grec8_shape.diff)
#ifndef RT_GREC_MIN_GEN
#define RT_GREC_MIN_GEN 1.4
#endif
bool rt_render_wants_global_records(const rt_kparams& K, int num_cus) {
    if (K.bvh_nodes || K.max_bounces <= 0) return false;
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    const bool hit_lds = (size_t)n_prim * RT_HIT_FLOATS * sizeof(float) <= 16384;
    rt_kparams L = K;
    L.rec = nullptr;
    const size_t lds = rt_render_lds_bytes(L, 256, hit_lds, true);
    const long groups = (long)(160 * 1024) / (long)(lds ? lds : 1);  // 256-lane groups per CU: 1 wave per SIMD each
    if (groups < RT_WAVES_PER_EU) return true;
    // resident 256-lane groups per CU with LDS / global records
    L.rec = reinterpret_cast<float*>(&L);  // any non-null: the global-record LDS size
    const size_t lds_g = rt_render_lds_bytes(L, 256, hit_lds, true);
    int occ_l = 0, occ_g = 0;
    const void* kl = hit_lds ? kernel_ptr<K_SORTED, 256, true>() : kernel_ptr<K_SORTED, 256, false>();
    const void* kg = hit_lds ? kernel_ptr<K_SORTED, 256, true, false, true>() : kernel_ptr<K_SORTED, 256, false, false, true>();
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_l, kl, 256, lds) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_g, kg, 256, lds_g) != hipSuccess || occ_g <= occ_l)
        return false;
    const double gens = (double)((long)K.rows * K.width) / (256.0 * occ_g * (num_cus > 0 ? num_cus : 1));
    return gens >= RT_GREC_MIN_GEN;
}

// Floats of a global-memory record stack for one launch: 3 dwords per level
// kept in global memory (levels RT_GREC_LDS_LEVELS .. max_bounces-1; the
// shallow ones stay in LDS) per lane of the grid (the grid covers every work
// item, rounded up to the largest workgroup), [group][level][field][lane].  At least one float, so a
// forced global-record launch with no global level still gets a buffer.
size_t rt_render_rec_floats(const rt_kparams& K) {
    const long nitems = launch_items(K);
    const int lds_levels = K.max_bounces < RT_GREC_LDS_LEVELS ? K.max_bounces : RT_GREC_LDS_LEVELS;
    const size_t planes = (size_t)3 * (K.max_bounces - lds_levels);
    return planes ? planes * (size_t)((nitems + 255) / 256 * 256) : 1;
}

// LDS bytes of one workgroup: hit table (if staged) + 3 record dwords per
// level per lane + 13 task-slot dwords per lane and 4 queue counters (sorted).
size_t rt_render_lds_bytes(const rt_kparams& K, int block, bool hit_lds, bool sorted) {
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
    const size_t hit = hit_lds ? (size_t)((n_prim * RT_HIT_FLOATS + 3) & ~3) * sizeof(float) : 0;
    // record stack: max_bounces + 1 levels (simple kernel), max_bounces (sorted)
    const int lds_levels = sorted && K.rec ? (K.max_bounces < RT_GREC_LDS_LEVELS ? K.max_bounces : RT_GREC_LDS_LEVELS)
                                           : K.max_bounces + (sorted ? 0 : 1);
    size_t b = hit + (size_t)3 * (lds_levels > 0 ? lds_levels : 0) * block * sizeof(float);
    if (sorted) b += (size_t)13 * block * sizeof(float) + 8 * sizeof(int);  // + queue counters
    return b;
}

// Host-side launch policy: BVH scenes take the ray-refill kernel; otherwise
// 256-lane workgroups (64 when the record stack of very deep paths would not
// fit), hit table in LDS when it fits in 16 KB, sorted task-queue kernel
// unless `simple` (one pixel per lane: its grid always covers every item);
// for the simple kernel grid_mult > 0 caps the grid at grid_mult x resident
// workgroups per CU (persistent lanes).
// pair_req: 1 / 0 forces the pair kernel on / off (BWRT_SPREAD), -1 the
// policy: frames and shards of at most RT_SPREAD_PIX pixels per CU (about
// 1.5 generations of 7 waves per SIMD, 32 pixels per wave) take 128-lane
// pair groups owning 64 pixels each.  Measured on c3 row shards: 1/8 0.252
// -> 0.194 ms, 1/16 0.254 -> 0.167 (profiles/r04g/shards_c3.txt); 1/4
// (2,025 pixels per CU) keeps the sorted kernel
#ifndef RT_SPREAD_PIX
#define RT_SPREAD_PIX 1400
#endif
#ifndef RT_PAIR_MIN_CHAIN
#define RT_PAIR_MIN_CHAIN 8
#endif
hipError_t rt_launch_render(const rt_kparams& K, int num_cus, int grid_mult, bool simple, int block_req,
                            hipStream_t stream, int pair_req) {
    // samplesPerPixel > 1 (the reference's in-frame loop, off by default):
    // only the one-path-per-lane kernel implements it
    simple = simple || K.spp_inner > 1;
    if (K.bvh_nodes && !simple) return rt_launch_render_bvh_refill(K, num_cus, stream);
    const int n_prim = K.n_sph + K.n_pln + K.n_tri + K.n_quad;
#ifdef RT_NO_HIT_LDS  // A/B builds: hit table read from global memory
    const bool hit_lds = false;
#else
    const bool hit_lds = !K.bvh_nodes && (size_t)n_prim * RT_HIT_FLOATS * sizeof(float) <= 16384;
#endif
    const bool small_block = (size_t)3 * (K.max_bounces + 1) * 256 * sizeof(float) > 49152;
    const int block = small_block ? 64 : 256;
    const size_t lds = rt_render_lds_bytes(K, block, hit_lds, !simple);
    if (simple)
        return small_block ? launch_block<64, K_SIMPLE>(K, hit_lds, lds, grid_mult, num_cus, stream)
                           : launch_block<256, K_SIMPLE>(K, hit_lds, lds, grid_mult, num_cus, stream);
#ifndef RT_SORTED_BLOCK
#define RT_SORTED_BLOCK 256
#endif
    if (small_block) return launch_block<64, K_SORTED>(K, hit_lds, lds, grid_mult, num_cus, stream);
    const long items = (long)K.rows * K.width;
    // (the pair kernel shortens long per-pixel chains: frames of at most
    // RT_PAIR_MIN_CHAIN queries per pixel keep the sorted kernel — config 1,
    // 1 frame x 2 queries: 10.3 vs 10.9 us, profiles/r05c/session.txt)
    const bool pair = hit_lds && !K.rec && (block_req == 0 || block_req == 128) &&
                      (pair_req > 0 || (pair_req < 0 && block_req == 0 && items <= (long)num_cus * RT_SPREAD_PIX &&
                                        (long)K.samples * (K.max_bounces + 1) >= RT_PAIR_MIN_CHAIN));
    if (pair)
        return launch_render<K_PAIR, 128, true>(K, rt_pair_lds_bytes(K), grid_mult, num_cus, stream);
    if (block_req == 64 || block_req == 128 || block_req == 256) {  // explicit (BWRT_BLOCK)
        const size_t lds_r = rt_render_lds_bytes(K, block_req, hit_lds, true);
        if (lds_r <= 65536) {
            if (block_req == 64) return launch_block<64, K_SORTED>(K, hit_lds, lds_r, grid_mult, num_cus, stream);
            if (block_req == 128) return launch_block<128, K_SORTED>(K, hit_lds, lds_r, grid_mult, num_cus, stream);
            return launch_block<256, K_SORTED>(K, hit_lds, lds_r, grid_mult, num_cus, stream);
        }
    }
    const size_t lds_s = rt_render_lds_bytes(K, RT_SORTED_BLOCK, hit_lds, true);
    // deep paths (large max_bounces) make the LDS record stack big: take
    // 128-lane groups when they keep more waves resident per CU (LDS 160 KB,
    // VGPR-bound at 4 x RT_WAVES_PER_EU waves)
    auto waves_per_cu = [](size_t lds_bytes, int block) {
        const long by_lds = (long)(160 * 1024 / (lds_bytes ? lds_bytes : 1)) * (block / 64);
        return by_lds < 4L * RT_WAVES_PER_EU ? by_lds : 4L * RT_WAVES_PER_EU;
    };
    // small frames / shards (one rank of an 8-GPU frame): fewer than 4
    // full-size groups per CU leave CUs with unequal shares of the critical
    // path (every group is resident at once); 128-lane groups spread it
    // (measured on c3 row shards of 1/8: 0.249 vs 0.264 ms; 1/4: 0.312 vs
    // 0.291), and the pair kernel (above) spreads it further
    const bool few_groups = items < (long)num_cus * 4 * RT_SORTED_BLOCK;
    if (RT_SORTED_BLOCK > 128 &&
        (few_groups ||
         waves_per_cu(rt_render_lds_bytes(K, 128, hit_lds, true), 128) > waves_per_cu(lds_s, RT_SORTED_BLOCK))) {
        const size_t lds_128 = rt_render_lds_bytes(K, 128, hit_lds, true);
        return launch_block<128, K_SORTED>(K, hit_lds, lds_128, grid_mult, num_cus, stream);
    }
    return launch_block<RT_SORTED_BLOCK, K_SORTED>(K, hit_lds, lds_s, grid_mult, num_cus, stream);
}

thread_local long rt_order_groups_last = 0;
thread_local char rt_launched_kernel[96] = "";

hipError_t rt_launch_order_groups(const unsigned* cost, int* order, long n, hipStream_t stream) {
    hipLaunchKernelGGL(rt_order_groups_kernel, dim3(1), dim3(1024), 0, stream, cost, order, (int)n);
    return hipGetLastError();
}

hipError_t rt_launch_init_rand(unsigned* rng, int width, int rows, int row_offset, int row_stride,
                               hipStream_t stream) {
    const long npix = (long)rows * width;
    const unsigned grid = (unsigned)((npix + 255) / 256);
    hipLaunchKernelGGL(rt_init_rand_kernel, dim3(grid), dim3(256), 0, stream, rng, width, rows,
                       row_offset, row_stride);
    return hipGetLastError();
}

// max_blocks > 0 caps the grid (the loop strides over the rest)
hipError_t rt_launch_deinterleave(const unsigned* gathered, unsigned* image, int width, int height,
                                  int shards, int rows_per_shard, int max_blocks, hipStream_t stream) {
    const bool vec = width % 4 == 0 && ((reinterpret_cast<uintptr_t>(gathered) | reinterpret_cast<uintptr_t>(image)) & 15) == 0;
    const long n = (long)height * (vec ? width / 4 : width);
    long grid = (n + 255) / 256;
    if (max_blocks > 0 && grid > max_blocks) grid = max_blocks;
    if (vec)
        hipLaunchKernelGGL(rt_deinterleave_kernel<4>, dim3((unsigned)grid), dim3(256), 0, stream, gathered, image,
                           width, height, shards, rows_per_shard);
    else
        hipLaunchKernelGGL(rt_deinterleave_kernel<1>, dim3((unsigned)grid), dim3(256), 0, stream, gathered, image,
                           width, height, shards, rows_per_shard);
    return hipGetLastError();
}
#endif  // RT_TU_BVH
