// rt_cpu.cpp — scalar C++ CPU fallback of the render kernel (host only).
//
// The same path as the HIP kernels (reference /root/reference/bwidman-raytracer/src:
// launchRaytracer Main.cu:274-315, tracePath Main.cu:208-272, Intersection.cuh:
// 15-173), one pixel per loop iteration, all `samples` progressive frames of a
// pixel in a row with its RNG state and frameSum in registers, built from the
// per-ray functions of rt_path.h that the kernels use (compiled here for the
// host: -ffp-contract=off, IEEE sqrtss/divss, hardware fma for the exactly
// specified fma steps), so every pixel is bit-identical to the GPU result and
// to the oracle (tests/test_cpu_fallback.py).
//
// Threads take 256-pixel chunks of the shard from an atomic counter
// (std::thread; the calling thread works too).  Scenes with a BVH walk the
// same threaded fp32 node arrays as the kernels, scalar: a leaf is tested as
// soon as the walk reaches it, with the same (t, RT_KEY) acceptance, so the
// result does not depend on the visiting order (rt_path.h key_accept).
//
// This is an explicit backend: only contexts made by rt_create_cpu() render
// here (include/rt_abi.h).  A GPU context never falls back to it.
#include <atomic>
#include <thread>

#include <xmmintrin.h>  // MXCSR
#include <vector>

#include "rt_path.h"

namespace {

// scalar threaded-BVH walk: the kernels' closest_hit_bvh without the wave
// scheduling (no leaf parking)
void closest_hit_bvh_cpu(const rt_kparams& K, f3 o, f3 d, float& best_t, int& best_id) {
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
    const float* nodes = K.bvh_nodes + (size_t)ray_octant(K, d) * K.bvh_order_stride;
    int node = 0;
    while (node >= 0) {
        const float* nd = nodes + 8 * (size_t)node;  // {bmin, miss, bmax, leaf}
        const int miss = rt_f2i(nd[3]);
        if (!slab_enter(nd[0], nd[1], nd[2], nd[4], nd[5], nd[6], sr, best_t)) {
            node = miss;
            continue;
        }
        const int lf = rt_f2i(nd[7]);
        if (lf < 0) {  // internal: first child next
            node = node + 1;
            continue;
        }
        const int first = lf & 0xffffff, count = lf >> 24;
        for (int k = 0; k < count; k++)
            leaf_test(K, K.bvh_leafrec + (size_t)RT_LEAF_FLOATS * (first + k), o, d, a2, a4, best_t, best_id, best_key);
        node = miss;
    }
}

// One path from (o, d) (tracePath, Main.cu:208-272, iteratively): the
// per-level records, folded innermost-first into the returned radiance
f3 trace_path(const rt_kparams& K, Xorwow& rs, f3 o, f3 d) {
    // recursion records (code, kspec, cosAngle): at most max_bounces + 1 hits
    int rec_code[RT_MAX_LEVELS];
    float rec_k[RT_MAX_LEVELS], rec_c[RT_MAX_LEVELS];
    int depth = 0;
    while (true) {
        float t;
        int id;
        if (K.bvh_nodes)
            closest_hit_bvh_cpu(K, o, d, t, id);
        else
            closest_hit_brute(K, o, d, t, id);
        if (id < 0) break;  // miss: backgroundColor (Main.cu:269-271)
        // shade (Main.cu:237-264)
        const float* h = K.hit + RT_HIT_FLOATS * id;
        const f3 P = add(o, scale(t, d));
        f3 n = mk(h[0], h[1], h[2]);
        if (h[3] != 0.0f) n = normalize3(sub(P, n));  // sphere: centre -> normal
        f3 scatter;
        int code = id;
        float kspec = 0.0f;
        if (rand_range(rs, 1.0f) < RT_SPECULAR_CHANCE) {  // brdfChoice (Main.cu:243)
            scatter = specular_scatter(rs, d, n, h[8], h[10], h[9], kspec);
            code = ~id;
        } else {
            scatter = random_direction(rs, n);  // brdf = 4 * albedo
        }
        rec_code[depth] = code;
        rec_k[depth] = kspec;
        rec_c[depth] = dot(scatter, n);  // cosAngle, Main.cu:264
        depth++;
        o = P;
        d = scatter;
        if (depth > K.max_bounces) break;  // the next call returns background (Main.cu:210)
    }
    // fold the recursion innermost-first (Main.cu:262-268)
    float lx = K.bg[0], ly = K.bg[1], lz = K.bg[2];
    for (int l = depth - 1; l >= 0; --l) fold_level(rec_code[l], rec_k[l], rec_c[l], K.hit, lx, ly, lz);
    return mk(lx, ly, lz);
}

// Every frame of shard pixel p (Main.cu:285-312 per frame, frames in order)
void render_pixel(const rt_kparams& K, long npix, long p) {
    const int j = (int)(p / K.width);
    const int x = (int)(p - (long)j * K.width);
    const int y = K.row_offset + j * K.row_stride;
    Xorwow rs;
    rs.d = K.rng[0 * npix + p];
    rs.v0 = K.rng[1 * npix + p];
    rs.v1 = K.rng[2 * npix + p];
    rs.v2 = K.rng[3 * npix + p];
    rs.v3 = K.rng[4 * npix + p];
    rs.v4 = K.rng[5 * npix + p];
    float ax = 0.0f, ay = 0.0f, az = 0.0f;
    if (K.first_frame != 1u) {
        ax = K.accum[0 * npix + p];
        ay = K.accum[1 * npix + p];
        az = K.accum[2 * npix + p];
    }
    const f3 d0 = primary_dir(K, x, y);
    const f3 cam = mk(K.cam_pos[0], K.cam_pos[1], K.cam_pos[2]);
    unsigned frame = K.first_frame;
    for (int s = 0; s < K.samples; s++) {
        // jittered camera ray (Main.cu:290-292)
        const f3 jit = random_direction(rs, d0);
        const f3 dcam = normalize3(add(d0, scale(K.jitter, jit)));
        // samplesPerPixel paths from it; the last one is kept (Main.cu:296-298)
        f3 L = trace_path(K, rs, cam, dcam);
        for (int i = 1; i < K.spp_inner; i++) L = trace_path(K, rs, cam, dcam);
        float lx = L.x, ly = L.y, lz = L.z;
        if (K.spp_inner != 1) {  // pixel /= samplesPerPixel: (1.0f / k) * pixel (Math.cuh:91-97)
            const float k = 1.0f / (float)K.spp_inner;
            lx = k * lx;
            ly = k * ly;
            lz = k * lz;
        }
        // progressive accumulation (Main.cu:299-304)
        if (frame == 1u) {
            ax = 0.0f;
            ay = 0.0f;
            az = 0.0f;
        }
        ax = ax + lx;
        ay = ay + ly;
        az = az + lz;
        frame++;
    }
    K.rng[0 * npix + p] = rs.d;
    K.rng[1 * npix + p] = rs.v0;
    K.rng[2 * npix + p] = rs.v1;
    K.rng[3 * npix + p] = rs.v2;
    K.rng[4 * npix + p] = rs.v3;
    K.rng[5 * npix + p] = rs.v4;
    K.accum[0 * npix + p] = ax;
    K.accum[1 * npix + p] = ay;
    K.accum[2 * npix + p] = az;
    if (K.rgba) K.rgba[p] = tone_map(ax, ay, az, frame - 1u);
}

}  // namespace

// The host can run this translation unit (built for x86-64-v3); checked with
// baseline instructions only
__attribute__((target("arch=x86-64"))) bool rt_cpu_supported() {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
}

// curand_init(y*W + x, 0, 0) for every shard pixel (Main.cu:369-380), planes
void rt_cpu_init_rand(unsigned* rng, int width, int rows, int row_offset, int row_stride) {
    const long npix = (long)rows * width;
    for (long p = 0; p < npix; p++) {
        const int j = (int)(p / width);
        const int x = (int)(p - (long)j * width);
        const Xorwow s = xorwow_seed(pixel_seed(x, row_offset + j * row_stride, width));
        rng[0 * npix + p] = s.d;
        rng[1 * npix + p] = s.v0;
        rng[2 * npix + p] = s.v1;
        rng[3 * npix + p] = s.v2;
        rng[4 * npix + p] = s.v3;
        rng[5 * npix + p] = s.v4;
    }
}

// Render K.samples frames of the shard in K (host pointers) on `threads`
// threads (>= 1).  Returns the threads actually used.
int rt_cpu_render(const rt_kparams& K, int threads) {
    const long npix = (long)K.rows * K.width;
    constexpr long kChunk = 256;
    const long chunks = (npix + kChunk - 1) / kChunk;
    if (threads < 1) threads = 1;
    if ((long)threads > chunks) threads = (int)(chunks > 0 ? chunks : 1);
    std::atomic<long> next(0);
    auto work = [&]() {
        // IEEE float state for the whole render, whatever the calling thread
        // holds (a -ffast-math library or torch.set_flush_denormal may have
        // set FTZ / DAZ, and new threads inherit it): round to nearest, no
        // denormal flushing — the GPU keeps f32 denormals — restored after
        const unsigned saved = _mm_getcsr();
        _mm_setcsr((saved & ~(_MM_ROUND_MASK | _MM_FLUSH_ZERO_MASK | 0x0040u)) | _MM_ROUND_NEAREST);  // 0x40 = DAZ
        for (long c = next.fetch_add(1); c < chunks; c = next.fetch_add(1)) {
            const long end = (c + 1) * kChunk < npix ? (c + 1) * kChunk : npix;
            for (long p = c * kChunk; p < end; p++) render_pixel(K, npix, p);
        }
        _mm_setcsr(saved);
    };
    std::vector<std::thread> pool;
    pool.reserve((size_t)threads - 1);
    for (int t = 1; t < threads; t++) {
        try {
            pool.emplace_back(work);
        } catch (...) {  // no more threads: the ones running (and this one) finish the work
            break;
        }
    }
    work();
    for (std::thread& t : pool) t.join();
    return (int)pool.size() + 1;
}
