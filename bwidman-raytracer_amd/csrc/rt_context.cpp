// rt_context.cpp — implementation of the C ABI (include/rt_abi.h).
//
// Host-side replacement of the reference's render driver
// (/root/reference/bwidman-raytracer/src/Main.cu:38-109 allocateScene,
// :317-366 render, :401-496 main's state handling): the context owns the
// device copy of the (compiled) scene, the per-pixel RNG state and frameSum
// accumulator of one pixel-row shard, a HIP stream and timing events.
//
// Compiled with -ffp-contract=off: the host-side scene compilation and the
// camera prelude (Main.cu:336-338) use the reference's float operations in
// the reference's order, so the kernel sees bit-identical inputs.
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <xmmintrin.h>
#include <vector>

#include "../../include/rt_abi.h"
#include "rt_layout.h"

size_t rt_render_rec_floats(const rt_kparams& K);
bool rt_render_wants_global_records(const rt_kparams& K, int num_cus);
hipError_t rt_launch_render(const rt_kparams& K, int num_cus, int grid_mult, bool simple, int block_req,
                            hipStream_t stream, int pair_req);
hipError_t rt_launch_init_rand(unsigned* rng, int width, int rows, int row_offset, int row_stride,
                               hipStream_t stream);
extern thread_local long rt_order_groups_last;
extern thread_local char rt_launched_kernel[96];
hipError_t rt_launch_deinterleave(const unsigned* gathered, unsigned* image, int width, int height,
                                  int shards, int rows_per_shard, int max_blocks, hipStream_t stream);
// scalar C++ CPU fallback (rt_cpu.cpp)
int rt_cpu_render(const rt_kparams& K, int threads);
void rt_cpu_init_rand(unsigned* rng, int width, int rows, int row_offset, int row_stride);
bool rt_cpu_supported();

static_assert(sizeof(rt_vec3) == 12, "vec3d layout (Math.cuh:35-39)");
static_assert(sizeof(rt_material) == 24, "material layout (WorldTypes.cuh:15-20)");
static_assert(sizeof(rt_sphere) == 40 && offsetof(rt_sphere, mat) == 16, "sphere layout");
static_assert(sizeof(rt_plane) == 60 && offsetof(rt_plane, mat) == 36, "plane layout");
static_assert(sizeof(rt_triangle) == 60 && offsetof(rt_triangle, mat) == 36, "triangle layout");
static_assert(sizeof(rt_quad) == 72 && offsetof(rt_quad, mat) == 48, "quad layout");
static_assert(sizeof(rt_camera) == 24, "camera layout (WorldTypes.cuh:9-13)");
static_assert(sizeof(rt_scene) == 88 && offsetof(rt_scene, spheres) == 24 &&
                  offsetof(rt_scene, sphere_count) == 32 && offsetof(rt_scene, planes) == 40 &&
                  offsetof(rt_scene, triangles) == 56 && offsetof(rt_scene, quads) == 72 &&
                  offsetof(rt_scene, quad_count) == 80,
              "scene layout (WorldTypes.cuh:44-53)");

namespace {

struct V3 {
    float x, y, z;
};
V3 v3(const rt_vec3& a) { return {a.x, a.y, a.z}; }
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 cross(V3 a, V3 b) {  // Math.cuh:103-108
    float i = a.y * b.z - a.z * b.y;
    float j = -(a.x * b.z - a.z * b.x);
    float k = a.x * b.y - a.y * b.x;
    return {i, j, k};
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct rt_context {
    int device = 0;
    int num_cus = 256;
    bool simple = false;  // BWRT_KERNEL=simple: one-path-per-lane kernel (A/B reference)
    int grid_mult = 0;  // persistent grid = grid_mult x resident workgroups per CU x CUs
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr;  // start of the last render (timing)
    // end of the last render launch (on `render_stream`, possibly a caller's
    // stream): a launch on another stream waits for it, and host-side state
    // writes wait for it (the kernels read and write the same shard state).
    // Events, not stream handles, so a caller may destroy its streams.
    hipEvent_t ev_render = nullptr;
    hipStream_t render_stream = nullptr;
    bool render_recorded = false;
    // the last render ran on the context's own stream and its end event is
    // not recorded yet (rt_get_stream): flush_render() records it on demand
    bool render_pending = false;
    // end of the last de-interleave on a caller's stream (rt_synchronize)
    hipEvent_t ev_aux = nullptr;
    bool aux_recorded = false;
    // CPU backend (rt_create_cpu): host copies instead of device buffers, the
    // scalar fallback of rt_cpu.cpp instead of the kernels
    bool cpu = false;
    int threads = 1;
    float cpu_ms = -1.0f;
    std::vector<float> scene_h;
    std::vector<unsigned> rng_h, rgba_h;
    std::vector<float> accum_h;
    bool timed = false;
    bool ktiming = true;  // start marker ev0 before each launch (rt_set_kernel_timing)
    std::string err;

    // compiled scene
    bool has_scene = false;
    rt_camera camera{};
    int n_sph = 0, n_pln = 0, n_tri = 0, n_quad = 0;
    float cull_omax = 0.0f;  // polygon culling bound (rt_layout.h)
    float background[3] = {0.0f, 0.0f, 0.0f};  // backgroundColor, Main.cu:27
    int bvh_nodes_per_order = 0;
    int bvh_order_mask = 7;
    DevBuf scene_buf;  // spheres | planes | triangles | quads | hit table | bvh nodes | bvh prims
    size_t off_bvh = 0, off_bvh_prims = 0, off_bvh_vtx = 0;  // in floats; 0 = no BVH
    size_t off_bvh16 = 0;                   // 16-byte nodes (0 = none: boxes beyond fp16)
    float ovf_sc = 0.0f, ovf_nm = 0.0f, ovf_im = 0.0f;  // overflow bounds (rt_layout.h)
    float cull_dmax = -1.0f;                            // culled rays: max|d_i| bound
    size_t off_pln = 0, off_tri = 0, off_quad = 0, off_hit = 0;  // in floats

    // shard state
    int width = 0, height = 0, row_offset = 0, row_stride = 1, rows = 0;
    DevBuf rng, accum, rgba;
    DevBuf rec;  // sorted kernel's record stack in global memory (deep paths)
    // launch-order feedback (rt_layout.h): tile-group costs of the last
    // launch and the order sorted from them, valid for a grid of order_n groups
    DevBuf gcost, gorder;
    long order_n = 0;
    // re-sort the launch order every order_period-th launch (BWRT_ORDER_PERIOD;
    // a grid without an order is always sorted): the per-group costs follow
    // the image, so a kept order is as good as a fresh one, and the sort
    // kernel plus its launch gap cost ~8 us per launch.  Config 3 bench kernel
    // average, three alternating runs: every launch 0.7567 / 0.7543 / 0.7535,
    // every 4th 0.7479 / 0.7461 / 0.7476, every 16th 0.7462 / 0.7430 / 0.7469,
    // never again 0.7451 / 0.7458 / 0.7484 ms (profiles/r03f/order_period_ab.txt);
    // config 2 0.1503 / 0.1515 vs 0.1555 / 0.1565, config 4 5.50 vs 5.52 ms
    int order_period = 16;
    // the kept order was measured on another image (new scene, camera or
    // shard): the next launch re-sorts its costs whatever the period
    bool order_stale = true;
    unsigned long long launches = 0;
    bool order_feedback = true;  // BWRT_ORDER=0: blockIdx order
    int grec = -1;  // BWRT_GREC: 1 / 0 force global / LDS records; -1 = launch policy
    void* host_rgba = nullptr;  // pinned staging for rt_render_multi
    size_t host_rgba_bytes = 0;
    int block = 0;               // BWRT_BLOCK: sorted-kernel workgroup lanes (0 = launch policy)
    int tile_w = -1;             // BWRT_TILE: wave tile width (0 = linear order; -1 = launch policy)
    int tile_sq = 0;             // BWRT_TILE_SQ: a 4-wave group's tiles as 2 x 2 (experiment)
    int leaf_batch = -1;         // BWRT_LEAF_BATCH: BVH refill kernel leaf-batch threshold (-1 = launch policy)
    int refill = -1;             // BWRT_REFILL: BVH refill kernel refill threshold (-1 = launch policy)
    int spread = -1;             // BWRT_SPREAD: 1 / 0 force the pair kernel on / off (-1 = launch policy)
    int deint_blocks = 0;        // BWRT_DEINT_BLOCKS: cap on the de-interleave grid (0 = one thread per 16 bytes)
    std::string kernel_name;     // the render kernel of the last launch (rt_last_kernel_name)
    unsigned frame = 1;
    int max_bounces = RT_DEFAULT_MAX_BOUNCES;
    int spp_inner = 1;  // samplesPerPixel, Main.cu:27
};

namespace {

// Tuning and diagnostic knobs (BWRT_BLOCK, BWRT_TILE, BWRT_GREC, BWRT_SPREAD,
// BWRT_ORDER*, BWRT_BVH_*, BWRT_STAMPS, ...; listed in rt_abi.h) are read
// only when the process sets BWRT_TUNING=1: a default context always takes
// the measured launch policy, whatever else the environment holds.
// IEEE float state for the library's host-side float work (scene compile,
// camera set-up, controls): round to nearest, no FTZ / DAZ, whatever the
// calling thread holds (a -ffast-math library or torch.set_flush_denormal
// may have set them), restored on return — the GPU keeps f32 denormals and
// the compiled scene must not depend on the caller
struct HostFpEnv {
    unsigned saved;
    HostFpEnv() : saved(_mm_getcsr()) {
        _mm_setcsr((saved & ~(_MM_ROUND_MASK | _MM_FLUSH_ZERO_MASK | 0x0040u)) | _MM_ROUND_NEAREST);  // 0x40 = DAZ
    }
    ~HostFpEnv() { _mm_setcsr(saved); }
};

const char* tuning_env(const char* name) {
    const char* t = std::getenv("BWRT_TUNING");
    return t && std::strcmp(t, "1") == 0 ? std::getenv(name) : nullptr;
}

// Record the end event of a render launched on the context's own stream
// whose recording was deferred (see launch)
hipError_t flush_render(rt_context* c) {
    if (!c->render_pending) return hipSuccess;
    c->render_pending = false;
    const hipError_t e = hipEventRecord(c->ev_render, c->stream);
    if (e == hipSuccess) c->render_recorded = true;
    return e;
}

int fail(rt_context* c, int code, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

int hip_fail(rt_context* c, hipError_t e, const char* what) {
    return fail(c, e == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_HIP, "%s: %s", what,
                hipGetErrorString(e));
}

#define HIP_TRY(ctx, expr)                                  \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #expr); \
    } while (0)

void free_buf(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

// Host-side writes of context state (scene, RNG seeds, frameSum, checkpoint
// restore) and buffer reallocation must not overlap a render still running
// on a caller's stream (rt_render_device): wait for the last render launch
// (its event, recorded on whatever stream it ran on).  Work on c->stream is
// already ordered by the stream itself.
int quiesce(rt_context* c) {
    if (c->cpu) return RT_OK;
    HIP_TRY(c, flush_render(c));
    if (!c->render_recorded) return RT_OK;
    HIP_TRY(c, hipEventSynchronize(c->ev_render));
    return RT_OK;
}

int ensure_buf(rt_context* c, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return RT_OK;
    if (b.p) {  // the old buffer may still be in use by queued work
        int rc = quiesce(c);
        if (rc) return rc;
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    free_buf(b);
    if (bytes == 0) return RT_OK;
    HIP_TRY(c, hipMalloc(&b.p, bytes));
    b.bytes = bytes;
    return RT_OK;
}

int shard_rows(int height, int row_offset, int row_stride) {
    if (height <= 0 || row_offset < 0 || row_stride <= 0 || row_offset >= height) return 0;
    return (height - row_offset + row_stride - 1) / row_stride;
}

void put_material(float* h, const rt_material& m) {
    // emittedLight = emittance * albedo (Main.cu:238)
    h[4] = m.emittance * m.albedo.x;
    h[5] = m.emittance * m.albedo.y;
    h[6] = m.emittance * m.albedo.z;
    h[7] = 0.0f;
    h[8] = m.roughness;
    // fresnel(): square(ior)/square(1.0f) - 1.0f (Main.cu:125)
    h[9] = (m.refractive_index * m.refractive_index) / (1.0f * 1.0f) - 1.0f;
    h[10] = m.roughness * m.roughness;  // Main.cu:119 evaluates roughness*roughness first
    h[11] = 0.0f;
    // diffuse brdf = 2 / (1 - specularChance) * albedo (Main.cu:259): the
    // double constant narrows to 4.0f; scaling by 4 is exact
    const float dk = (float)(2.0 / (1 - 0.5f));
    h[12] = dk * m.albedo.x;
    h[13] = dk * m.albedo.y;
    h[14] = dk * m.albedo.z;
    h[15] = 0.0f;
}

// Triangle / quad record: {n, d, v0, in0, v1, in1, ...}; Intersection.cuh:109-127
// Cull sphere of a triangle, used by polygon_test to skip the exact test for
// rays whose LINE passes farther than Rc from the centre.  Such a ray's
// plane hit P (as the reference computes it, with float rounding) is at
// least Rc - R from the triangle; outside a triangle with smallest angle
// alpha some edge function dot(in_k, P - v_k) is then below
// -|in_k| * (Rc - R) * sin(alpha / 2), and the inflation
//   Rc = R (1 + 2^-20) + 2^-14 * scale / (0.25 sin alpha)
// (scale >= every coordinate of the scene and of any culled ray origin)
// keeps that margin > 2^-14 * scale, several hundred times the rounding of
// the reference's P = o + t d and of its edge dots (~2^-21 * scale).  So the
// reference rejects every culled triangle.  Degenerate/skinny triangles
// (sin alpha < 2^-10) and quads (possibly non-convex / non-planar) are never
// culled (Rc^2 = inf).
void cull_sphere(float* cs, const rt_vec3* verts, int nv, double scale) {
    cs[0] = cs[1] = cs[2] = 0.0f;
    cs[3] = INFINITY;
    if (nv != 3) return;
    double v[3][3];
    for (int k = 0; k < 3; k++) {
        v[k][0] = verts[k].x;
        v[k][1] = verts[k].y;
        v[k][2] = verts[k].z;
    }
    double c[3], r = 0.0, min_sin = 1.0;
    for (int a = 0; a < 3; a++) c[a] = (v[0][a] + v[1][a] + v[2][a]) / 3.0;
    for (int k = 0; k < 3; k++) {
        double d2 = 0.0, e1[3], e2[3], l1 = 0.0, l2 = 0.0, dp = 0.0;
        for (int a = 0; a < 3; a++) {
            d2 += (v[k][a] - c[a]) * (v[k][a] - c[a]);
            e1[a] = v[(k + 1) % 3][a] - v[k][a];
            e2[a] = v[(k + 2) % 3][a] - v[k][a];
            l1 += e1[a] * e1[a];
            l2 += e2[a] * e2[a];
            dp += e1[a] * e2[a];
        }
        r = std::max(r, std::sqrt(d2));
        const double cosang = (l1 > 0.0 && l2 > 0.0) ? dp / std::sqrt(l1 * l2) : 1.0;
        min_sin = std::min(min_sin, std::sqrt(std::max(0.0, 1.0 - cosang * cosang)));
    }
    if (!(min_sin >= 1.0 / 1024.0) || !std::isfinite(r) || !std::isfinite(scale)) return;
    const double rc = r * (1.0 + std::ldexp(1.0, -20)) + std::ldexp(1.0, -14) * scale / (0.25 * min_sin);
    const double rc2 = rc * rc * (1.0 + std::ldexp(1.0, -20));
    if (!(rc2 < 1e30)) return;
    cs[0] = (float)c[0];
    cs[1] = (float)c[1];
    cs[2] = (float)c[2];
    cs[3] = (float)rc2;
}

void compile_polygon(float* q, float* h, const rt_vec3* verts, int nv, const rt_material& m, double scale) {
    V3 v[4], e[4];
    for (int k = 0; k < nv; k++) v[k] = v3(verts[k]);
    for (int k = 0; k < nv; k++) e[k] = sub(v[(k + 1) % nv], v[k]);
    V3 n = cross(e[0], e[1]);   // plane {v0, {e0, e1}}: normal = cross(d0, d1)
    float d = -dot(n, v[0]);    // Intersection.cuh:83
    q[0] = n.x;
    q[1] = n.y;
    q[2] = n.z;
    q[3] = d;
    for (int k = 0; k < nv; k++) {
        V3 in = cross(n, e[k]);  // Intersection.cuh:125-127
        float* r = q + RT_POLY_EDGES + 6 * k;
        r[0] = v[k].x;
        r[1] = v[k].y;
        r[2] = v[k].z;
        r[3] = in.x;
        r[4] = in.y;
        r[5] = in.z;
    }
    h[0] = n.x;
    h[1] = n.y;
    h[2] = n.z;
    h[3] = 0.0f;
    put_material(h, m);
    // cull sphere (centre, Rc^2), appended after the edge data
    float* cs = q + (nv == 3 ? RT_TRI_CULL : RT_QUAD_CULL);
    cull_sphere(cs, verts, nv, scale);
}

// ---- BVH over spheres / triangles / quads (large scenes) -------------------
// Binned-SAH binary tree, emitted as EIGHT threaded (stackless) node arrays,
// one per ray-direction octant: in array k the children of every node are
// laid out near side of the node's split axis first for that octant, each
// node holding its "miss" link (next node once the subtree is skipped).  A
// lane walks the array of its ray's octant, so boxes come front to back
// along every split and the running closest hit prunes the rest
// (multiple-threaded BVH).  Boxes are inflated by 1e-3 + 1e-4 * |coordinate|
// — orders of magnitude beyond the rounding of the reference's hit tests —
// so every hit the reference can accept lies inside its leaf's box.
struct BvhItem {
    float lo[3], hi[3], c[3];
    int id;
};

struct BvhNode {
    float lo[3], hi[3];
    int left = -1, right = -1;  // children (internal)
    int axis = 0;               // split axis (internal): left child holds the smaller centroids
    int first = 0, count = 0;   // prims range (leaf)
};

struct BvhBuilder {
    static constexpr int kBins = 16;
    int max_leaf = 8;         // BWRT_BVH_LEAF
    float trav_cost = 0.0f;   // BWRT_BVH_CT: SAH cost of one node step relative to one primitive test
    int order_mask = 7;       // octant bits that get their own node array (set from the scene extents; BWRT_BVH_ORDER_MASK)
    std::vector<BvhItem> items;
    std::vector<BvhNode> tree;
    std::vector<int> prims;
    std::vector<float> nodes;  // 8 orders x n_nodes x 8 floats
    // the same threaded arrays as 16-byte nodes (rt_layout.h bvh_nodes16):
    // boxes in fp16 rounded outward; n16 = every box fits the fp16 range
    std::vector<uint32_t> nodes16;  // 8 orders x n_nodes x 4 words
    bool n16 = false;
    int n_nodes = 0;

    // fp16 bits of the largest half <= v (down) or the smallest half >= v
    // (up); false if |v| exceeds the finite fp16 range
    static bool half_bound(float v, bool up, uint16_t& out) {
        if (!(std::fabs(v) <= 65504.0f)) return false;
        if (std::fabs(v) < 6.103515625e-05f) {  // below the smallest normal: +-2^-14
            out = up ? 0x0400 : 0x8400;
            return true;
        }
        uint32_t f;
        std::memcpy(&f, &v, 4);
        const uint32_t sign = (f >> 16) & 0x8000u;
        const int e = (int)((f >> 23) & 0xff) - 127 + 15;  // 1..30 here
        uint32_t m = (f >> 13) & 0x3ffu;                   // truncated toward zero
        uint16_t h = (uint16_t)(sign | ((uint32_t)e << 10) | m);
        const bool inexact = (f & 0x1fffu) != 0;
        // truncation moved |v| down: step one ulp outward when that is the wrong way
        if (inexact && (up != (sign != 0))) h = (uint16_t)(h + 1);  // away from zero
        if (((h >> 10) & 0x1f) == 0x1f) return false;             // stepped to infinity
        out = h;
        return true;
    }

    static float inflate(float v) { return 1e-3f + 1e-4f * std::fabs(v); }
    static float area(const float* lo, const float* hi) {
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return (dx < 0 || dy < 0 || dz < 0) ? 0.0f : 2.0f * (dx * dy + dy * dz + dz * dx);
    }

    int make_leaf(int node, int b, int e) {
        tree[node].first = (int)prims.size();
        tree[node].count = e - b;
        for (int i = b; i < e; i++) prims.push_back(items[i].id);
        return node;
    }

    int build(int b, int e) {
        const int node = (int)tree.size();
        tree.emplace_back();
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < e; i++)
            for (int a = 0; a < 3; a++) {
                lo[a] = std::min(lo[a], items[i].lo[a]);
                hi[a] = std::max(hi[a], items[i].hi[a]);
                clo[a] = std::min(clo[a], items[i].c[a]);
                chi[a] = std::max(chi[a], items[i].c[a]);
            }
        for (int a = 0; a < 3; a++) {
            tree[node].lo[a] = lo[a];
            tree[node].hi[a] = hi[a];
        }
        const int n = e - b;
        if (n <= 2) return make_leaf(node, b, e);
        // binned SAH over the three axes
        float best_cost = INFINITY;
        int best_axis = -1, best_bin = -1;
        for (int a = 0; a < 3; a++) {
            const float ext = chi[a] - clo[a];
            if (!(ext > 0.0f)) continue;
            int cnt[kBins] = {0};
            float blo[kBins][3], bhi[kBins][3];
            for (int k = 0; k < kBins; k++)
                for (int q = 0; q < 3; q++) {
                    blo[k][q] = INFINITY;
                    bhi[k][q] = -INFINITY;
                }
            for (int i = b; i < e; i++) {
                int k = (int)((items[i].c[a] - clo[a]) / ext * kBins);
                k = std::min(std::max(k, 0), kBins - 1);
                cnt[k]++;
                for (int q = 0; q < 3; q++) {
                    blo[k][q] = std::min(blo[k][q], items[i].lo[q]);
                    bhi[k][q] = std::max(bhi[k][q], items[i].hi[q]);
                }
            }
            float rarea[kBins];
            int rcnt[kBins];
            float rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
            int rc = 0;
            for (int k = kBins - 1; k > 0; k--) {
                rc += cnt[k];
                for (int q = 0; q < 3; q++) {
                    rl[q] = std::min(rl[q], blo[k][q]);
                    rh[q] = std::max(rh[q], bhi[k][q]);
                }
                rarea[k] = area(rl, rh);
                rcnt[k] = rc;
            }
            float ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
            int lc = 0;
            for (int k = 0; k < kBins - 1; k++) {
                lc += cnt[k];
                for (int q = 0; q < 3; q++) {
                    ll[q] = std::min(ll[q], blo[k][q]);
                    lh[q] = std::max(lh[q], bhi[k][q]);
                }
                if (lc == 0 || rcnt[k + 1] == 0) continue;
                const float cost = area(ll, lh) * lc + rarea[k + 1] * rcnt[k + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_bin = k;
                }
            }
        }
        const float leaf_cost = area(lo, hi) * n;
        best_cost += trav_cost * area(lo, hi);
        int mid;
        if (best_axis >= 0 && (best_cost < leaf_cost || n > max_leaf)) {
            const int a = best_axis;
            const float ext = chi[a] - clo[a];
            auto it = std::partition(items.begin() + b, items.begin() + e, [&](const BvhItem& x) {
                int k = (int)((x.c[a] - clo[a]) / ext * kBins);
                k = std::min(std::max(k, 0), kBins - 1);
                return k <= best_bin;
            });
            mid = (int)(it - items.begin());
        } else if (n <= max_leaf) {
            return make_leaf(node, b, e);
        } else {  // all centroids equal: split in the middle
            mid = (b + e) / 2;
        }
        if (mid <= b || mid >= e) mid = (b + e) / 2;
        const int l = build(b, mid);
        const int r = build(mid, e);
        tree[node].axis = best_axis >= 0 ? best_axis : 0;
        tree[node].left = l;
        tree[node].right = r;
        return node;
    }

    // threaded array for the ray-direction octant `order` (bit a set: d[a] < 0):
    // at every node the child on the near side of its split axis comes first
    void emit(int order, int node, std::vector<int>& pos, std::vector<int>& seq) {
        pos[node] = (int)seq.size();
        seq.push_back(node);
        const BvhNode& t = tree[node];
        if (t.left < 0) return;
        const bool left_first = !((order >> t.axis) & 1);
        emit(order, left_first ? t.left : t.right, pos, seq);
        emit(order, left_first ? t.right : t.left, pos, seq);
    }

    void finish() {
        n_nodes = (int)tree.size();
        nodes.assign((size_t)8 * n_nodes * 8, 0.0f);
        nodes16.assign((size_t)8 * n_nodes * 4, 0u);
        n16 = true;
        std::vector<int> pos(n_nodes), seq, end(n_nodes);
        for (int order = 0; order < 8; order++) {
            if (order & ~order_mask) continue;  // never selected by the kernel
            seq.clear();
            emit(order, 0, pos, seq);
            // subtree end in this order: position after the last descendant
            for (int i = n_nodes - 1; i >= 0; i--) {
                const BvhNode& t = tree[seq[i]];
                end[i] = t.left < 0 ? i + 1 : std::max(end[pos[t.left]], end[pos[t.right]]);
            }
            float* base = nodes.data() + (size_t)order * n_nodes * 8;
            for (int i = 0; i < n_nodes; i++) {
                const BvhNode& t = tree[seq[i]];
                float* nd = base + (size_t)i * 8;
                for (int a = 0; a < 3; a++) {
                    nd[a] = t.lo[a];
                    nd[4 + a] = t.hi[a];
                }
                const int miss = end[i] < n_nodes ? end[i] : -1;
                const int leaf = t.left < 0 ? ((t.count << 24) | t.first) : -1;
                std::memcpy(&nd[3], &miss, 4);
                std::memcpy(&nd[7], &leaf, 4);
                // 16-byte node: {lo.x | lo.y, lo.z | hi.x, hi.y | hi.z} in fp16
                // (lo rounded down, hi up) + w: the miss link of an internal node
                // (-1 = done) or ~leaf of a leaf (count >= 1, so w < -2^24; a
                // leaf's miss link is always the next node, i + 1)
                uint16_t hb[6];
                for (int a = 0; a < 3; a++)
                    n16 = n16 && half_bound(t.lo[a], false, hb[a]) && half_bound(t.hi[a], true, hb[3 + a]);
                uint32_t* q = nodes16.data() + ((size_t)order * n_nodes + i) * 4;
                q[0] = hb[0] | (uint32_t)hb[1] << 16;
                q[1] = hb[2] | (uint32_t)hb[3] << 16;
                q[2] = hb[4] | (uint32_t)hb[5] << 16;
                const int w = t.left < 0 ? ~leaf : miss;
                std::memcpy(&q[3], &w, 4);
            }
        }
    }

    // ---- spatial splits (SBVH, Stich, Friedrich & Dietrich 2009) ----------
    // A reference is a primitive cut down to a region of space: its box
    // bounds the part of the primitive inside every split plane it was cut
    // by (polygons clipped in double precision, spheres by their box).  A
    // primitive may sit in several leaves; testing it more than once changes
    // nothing ((t, key) acceptance), and the union of its references' boxes
    // covers the whole primitive.  Boxes are inflated as above when stored.
    struct Ref {
        double lo[3], hi[3];
        int id;
    };
    std::vector<double> geo;  // per primitive id: up to 4 vertices, 12 doubles
    std::vector<int> geo_nv;  // 3 / 4: polygon vertices; 0: clipped by its box
    double root_area = 0.0;
    size_t ref_budget = 0, n_refs = 0;
    double split_alpha = 1e-5;  // try spatial splits when the object split's children overlap > alpha * root area
    static constexpr int kSpatialBins = 32;

    static double dinflate(double v) { return 1e-3 + 1e-4 * std::fabs(v); }
    static float fdown(double v) {
        float f = (float)v;
        if ((double)f > v) f = std::nextafter(f, -INFINITY);
        return f;
    }
    static float fup(double v) {
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, INFINITY);
        return f;
    }
    static double darea(const double* lo, const double* hi) {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return (dx < 0 || dy < 0 || dz < 0) ? 0.0 : 2.0 * (dx * dy + dy * dz + dz * dx);
    }

    // the part of r with s0 <= x_a <= s1; false if there is none
    bool clip(const Ref& r, int a, double s0, double s1, Ref& out) const {
        out = r;
        out.lo[a] = std::max(r.lo[a], s0);
        out.hi[a] = std::min(r.hi[a], s1);
        if (out.lo[a] > out.hi[a]) return false;
        const int nv = geo_nv[r.id];
        if (nv < 3) return true;
        double poly[8][3], tmp[8][3];
        int n = nv;
        for (int k = 0; k < nv; k++)
            for (int q = 0; q < 3; q++) poly[k][q] = geo[(size_t)12 * r.id + 3 * k + q];
        for (int side = 0; side < 2 && n > 0; side++) {
            int m = 0;
            for (int k = 0; k < n; k++) {
                const double* p = poly[k];
                const double* q = poly[(k + 1) % n];
                const double dp = side == 0 ? p[a] - s0 : s1 - p[a];
                const double dq = side == 0 ? q[a] - s0 : s1 - q[a];
                if (dp >= 0.0)
                    for (int c = 0; c < 3; c++) tmp[m][c] = p[c];
                if (dp >= 0.0) m++;
                if ((dp >= 0.0) != (dq >= 0.0)) {
                    const double t = dp / (dp - dq);
                    for (int c = 0; c < 3; c++) tmp[m][c] = p[c] + t * (q[c] - p[c]);
                    m++;
                }
            }
            n = m;
            for (int k = 0; k < n; k++)
                for (int c = 0; c < 3; c++) poly[k][c] = tmp[k][c];
        }
        // no part of the polygon in the slab (a sliver on its boundary is
        // covered by the neighbouring reference's inflated box)
        if (n == 0) return false;
        double plo[3] = {INFINITY, INFINITY, INFINITY}, phi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int k = 0; k < n; k++)
            for (int c = 0; c < 3; c++) {
                plo[c] = std::min(plo[c], poly[k][c]);
                phi[c] = std::max(phi[c], poly[k][c]);
            }
        for (int c = 0; c < 3; c++) {
            out.lo[c] = std::max(out.lo[c], plo[c]);
            out.hi[c] = std::min(out.hi[c], phi[c]);
            if (out.lo[c] > out.hi[c]) {  // rounding: keep a degenerate box at the slab
                out.lo[c] = out.hi[c] = std::min(std::max(0.5 * (plo[c] + phi[c]), out.lo[c]), out.hi[c]);
            }
        }
        return true;
    }

    int build_s(std::vector<Ref>& refs) {
        const int node = (int)tree.size();
        tree.emplace_back();
        const int n = (int)refs.size();
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (const Ref& r : refs)
            for (int a = 0; a < 3; a++) {
                lo[a] = std::min(lo[a], r.lo[a]);
                hi[a] = std::max(hi[a], r.hi[a]);
                const double c = 0.5 * (r.lo[a] + r.hi[a]);
                clo[a] = std::min(clo[a], c);
                chi[a] = std::max(chi[a], c);
            }
        for (int a = 0; a < 3; a++) {
            tree[node].lo[a] = fdown(lo[a] - dinflate(lo[a]));
            tree[node].hi[a] = fup(hi[a] + dinflate(hi[a]));
        }
        auto leaf = [&]() {
            tree[node].first = (int)prims.size();
            tree[node].count = n;
            for (const Ref& r : refs) prims.push_back(r.id);
            return node;
        };
        if (n <= 2) return leaf();
        // object split: binned SAH over the reference centroids
        double best_cost = INFINITY, ov_area = 0.0;
        int best_axis = -1, best_bin = -1;
        for (int a = 0; a < 3; a++) {
            const double ext = chi[a] - clo[a];
            if (!(ext > 0.0)) continue;
            int cnt[kBins] = {0};
            double blo[kBins][3], bhi[kBins][3];
            for (int k = 0; k < kBins; k++)
                for (int q = 0; q < 3; q++) blo[k][q] = INFINITY, bhi[k][q] = -INFINITY;
            for (const Ref& r : refs) {
                int k = (int)((0.5 * (r.lo[a] + r.hi[a]) - clo[a]) / ext * kBins);
                k = std::min(std::max(k, 0), kBins - 1);
                cnt[k]++;
                for (int q = 0; q < 3; q++) blo[k][q] = std::min(blo[k][q], r.lo[q]), bhi[k][q] = std::max(bhi[k][q], r.hi[q]);
            }
            double rl[kBins][3], rh[kBins][3];
            int rc[kBins];
            double al[3] = {INFINITY, INFINITY, INFINITY}, ah[3] = {-INFINITY, -INFINITY, -INFINITY};
            int c = 0;
            for (int k = kBins - 1; k > 0; k--) {
                c += cnt[k];
                for (int q = 0; q < 3; q++) al[q] = std::min(al[q], blo[k][q]), ah[q] = std::max(ah[q], bhi[k][q]);
                for (int q = 0; q < 3; q++) rl[k][q] = al[q], rh[k][q] = ah[q];
                rc[k] = c;
            }
            double ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
            int lc = 0;
            for (int k = 0; k < kBins - 1; k++) {
                lc += cnt[k];
                for (int q = 0; q < 3; q++) ll[q] = std::min(ll[q], blo[k][q]), lh[q] = std::max(lh[q], bhi[k][q]);
                if (lc == 0 || rc[k + 1] == 0) continue;
                const double cost = darea(ll, lh) * lc + darea(rl[k + 1], rh[k + 1]) * rc[k + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_bin = k;
                    double ol[3], oh[3];
                    for (int q = 0; q < 3; q++) ol[q] = std::max(ll[q], rl[k + 1][q]), oh[q] = std::min(lh[q], rh[k + 1][q]);
                    ov_area = darea(ol, oh);
                }
            }
        }
        // spatial split: chop the references into spatial bins
        bool spatial = false;
        double split_pos = 0.0;
        if (n_refs < ref_budget && ov_area > split_alpha * root_area) {
            for (int a = 0; a < 3; a++) {
                const double ext = hi[a] - lo[a];
                if (!(ext > 0.0)) continue;
                const double w = ext / kSpatialBins;
                int ent[kSpatialBins] = {0}, ext_[kSpatialBins] = {0};
                double blo[kSpatialBins][3], bhi[kSpatialBins][3];
                for (int k = 0; k < kSpatialBins; k++)
                    for (int q = 0; q < 3; q++) blo[k][q] = INFINITY, bhi[k][q] = -INFINITY;
                for (const Ref& r : refs) {
                    int k0 = (int)((r.lo[a] - lo[a]) / w), k1 = (int)((r.hi[a] - lo[a]) / w);
                    k0 = std::min(std::max(k0, 0), kSpatialBins - 1);
                    k1 = std::min(std::max(k1, k0), kSpatialBins - 1);
                    bool any = false;
                    int first = -1, last = -1;
                    for (int k = k0; k <= k1; k++) {
                        const double s0 = k == 0 ? -INFINITY : lo[a] + k * w;
                        const double s1 = k == kSpatialBins - 1 ? INFINITY : lo[a] + (k + 1) * w;
                        Ref part;
                        if (!clip(r, a, s0, s1, part)) continue;
                        any = true;
                        if (first < 0) first = k;
                        last = k;
                        for (int q = 0; q < 3; q++) blo[k][q] = std::min(blo[k][q], part.lo[q]), bhi[k][q] = std::max(bhi[k][q], part.hi[q]);
                    }
                    if (!any) {  // (rounding) count it in its box's first bin
                        first = last = k0;
                        for (int q = 0; q < 3; q++) blo[k0][q] = std::min(blo[k0][q], r.lo[q]), bhi[k0][q] = std::max(bhi[k0][q], r.hi[q]);
                    }
                    ent[first]++;
                    ext_[last]++;
                }
                double rl[kSpatialBins][3], rh[kSpatialBins][3];
                int rc[kSpatialBins];
                double al[3] = {INFINITY, INFINITY, INFINITY}, ah[3] = {-INFINITY, -INFINITY, -INFINITY};
                int c = 0;
                for (int k = kSpatialBins - 1; k > 0; k--) {
                    c += ext_[k];
                    for (int q = 0; q < 3; q++) al[q] = std::min(al[q], blo[k][q]), ah[q] = std::max(ah[q], bhi[k][q]);
                    for (int q = 0; q < 3; q++) rl[k][q] = al[q], rh[k][q] = ah[q];
                    rc[k] = c;
                }
                double ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
                int lc = 0;
                for (int k = 0; k < kSpatialBins - 1; k++) {
                    lc += ent[k];
                    for (int q = 0; q < 3; q++) ll[q] = std::min(ll[q], blo[k][q]), lh[q] = std::max(lh[q], bhi[k][q]);
                    if (lc == 0 || rc[k + 1] == 0) continue;
                    const double cost = darea(ll, lh) * lc + darea(rl[k + 1], rh[k + 1]) * rc[k + 1];
                    if (cost < best_cost) {
                        best_cost = cost;
                        best_axis = a;
                        spatial = true;
                        split_pos = lo[a] + (k + 1) * w;
                    }
                }
            }
        }
        const double leaf_cost = darea(lo, hi) * n;
        best_cost += trav_cost * darea(lo, hi);
        if (best_axis < 0 || (best_cost >= leaf_cost && n <= max_leaf)) {
            if (n <= max_leaf) return leaf();
        }
        std::vector<Ref> L, R;
        if (best_axis >= 0 && spatial) {
            const int a = best_axis;
            for (const Ref& r : refs) {
                if (r.hi[a] <= split_pos) {
                    L.push_back(r);
                } else if (r.lo[a] >= split_pos) {
                    R.push_back(r);
                } else {
                    Ref pl, pr;
                    const bool hl = clip(r, a, -INFINITY, split_pos, pl), hr = clip(r, a, split_pos, INFINITY, pr);
                    if (hl) L.push_back(pl);
                    if (hr) R.push_back(pr);
                    if (!hl && !hr) L.push_back(r);
                }
            }
        } else if (best_axis >= 0) {
            const int a = best_axis;
            const double ext = chi[a] - clo[a];
            for (const Ref& r : refs) {
                int k = (int)((0.5 * (r.lo[a] + r.hi[a]) - clo[a]) / ext * kBins);
                k = std::min(std::max(k, 0), kBins - 1);
                (k <= best_bin ? L : R).push_back(r);
            }
        }
        if (L.empty() || R.empty()) {  // no usable split: halve the list along the widest centroid axis
            L.clear();
            R.clear();
            int a = 0;
            for (int q = 1; q < 3; q++)
                if (chi[q] - clo[q] > chi[a] - clo[a]) a = q;
            std::sort(refs.begin(), refs.end(),
                      [a](const Ref& x, const Ref& y) { return x.lo[a] + x.hi[a] < y.lo[a] + y.hi[a]; });
            L.assign(refs.begin(), refs.begin() + n / 2);
            R.assign(refs.begin() + n / 2, refs.end());
            best_axis = a;
        }
        n_refs += L.size() + R.size() - (size_t)n;
        std::vector<Ref>().swap(refs);
        const int l = build_s(L);
        const int r = build_s(R);
        tree[node].axis = best_axis;
        tree[node].left = l;
        tree[node].right = r;
        return node;
    }

    void add(int id, const float* lo, const float* hi) {
        BvhItem it;
        for (int a = 0; a < 3; a++) {
            it.lo[a] = lo[a] - inflate(lo[a]);
            it.hi[a] = hi[a] + inflate(hi[a]);
            it.c[a] = 0.5f * (lo[a] + hi[a]);
        }
        it.id = id;
        items.push_back(it);
    }
};

}  // namespace

extern "C" {

const char* rt_version(void) { return "0.1.0"; }

rt_material rt_material_default(void) {
    rt_material m;
    m.albedo = {0.0f, 0.0f, 0.0f};
    m.emittance = 0.0f;
    m.roughness = 1.0f;
    m.refractive_index = 1.05f;  // WorldTypes.cuh:19 (double 1.05 -> float)
    return m;
}

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rt_create(int device, rt_context** out) {
    if (!out) return RT_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return RT_ERR_INVALID_ARGUMENT;
    rt_context* c = new rt_context();
    c->device = device;
    // the context's stream at the device's highest priority: its render
    // workgroups dispatch ahead of other streams' work, e.g. the multi-GPU
    // gather and de-interleave of the previous frame that overlap the next
    // render (world size 1, ms per step: 0.761-0.765 vs 0.780-0.785 at
    // normal priority, single-GPU renders unchanged; profiles/r06e/);
    // BWRT_STREAM_PRIO=0: normal priority
    int prio_lo = 0, prio_hi = 0;
    const char* sp = tuning_env("BWRT_STREAM_PRIO");
    const bool high = !(sp && std::atoi(sp) == 0) && hipSetDevice(device) == hipSuccess &&
                      hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) == hipSuccess;
    if (hipSetDevice(device) != hipSuccess ||
        (high ? hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi)
              : hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev_render) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_aux, hipEventDisableTiming) != hipSuccess) {
        rt_destroy(c);
        return RT_ERR_HIP;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->num_cus = prop.multiProcessorCount;
    if (const char* gm = tuning_env("BWRT_GRID_MULT")) c->grid_mult = std::atoi(gm);
    if (const char* db = tuning_env("BWRT_DEINT_BLOCKS")) c->deint_blocks = std::max(std::atoi(db), 0);
    if (const char* kk = tuning_env("BWRT_KERNEL")) c->simple = std::strcmp(kk, "simple") == 0;
    if (const char* bk = tuning_env("BWRT_BLOCK")) c->block = std::atoi(bk);
    if (const char* tw = tuning_env("BWRT_TILE")) {
        const int t = std::atoi(tw);
        if (t >= 0 && t <= 64 && (t & (t - 1)) == 0) c->tile_w = t;
    }
    if (const char* g = tuning_env("BWRT_TILE_SQ")) c->tile_sq = std::atoi(g) != 0;
    if (const char* g = tuning_env("BWRT_GREC")) c->grec = std::atoi(g) ? 1 : 0;
    if (const char* g = tuning_env("BWRT_LEAF_BATCH")) c->leaf_batch = std::min(std::max(std::atoi(g), 1), 64);
    if (const char* g = tuning_env("BWRT_REFILL")) c->refill = std::min(std::max(std::atoi(g), 1), 64);
    if (const char* g = tuning_env("BWRT_SPREAD")) c->spread = std::atoi(g) ? 1 : 0;
    if (const char* g = tuning_env("BWRT_ORDER")) c->order_feedback = std::atoi(g) != 0;
    if (const char* g = tuning_env("BWRT_ORDER_PERIOD")) c->order_period = std::max(std::atoi(g), 1);
    *out = c;
    return RT_OK;
}

int rt_create_cpu(int threads, rt_context** out) {
    if (!out) return RT_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (threads < 0) return RT_ERR_INVALID_ARGUMENT;
    // rt_cpu.cpp is built for x86-64-v3 (hardware fma for the exactly
    // specified fma steps of rt_path.h)
    if (!rt_cpu_supported()) return RT_ERR_UNSUPPORTED;
    rt_context* c = new rt_context();
    c->cpu = true;
    c->device = -1;
    c->threads = threads > 0 ? threads : rt_cpu_threads();
    *out = c;
    return RT_OK;
}

int rt_cpu_threads(void) {
    // the CPUs this process may run on (sched affinity), not the machine's,
    // capped by a cgroup v2 CPU quota (cpu.max "quota period", rounded up):
    // a container may see every CPU of the host but be granted a share
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    if (n <= 0) n = 1;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char quota[32] = {0};
        long period = 0;
        if (std::fscanf(f, "%31s %ld", quota, &period) == 2 && std::strcmp(quota, "max") != 0 && period > 0) {
            const long q = std::atol(quota);
            const int share = (int)((q + period - 1) / period);
            if (share > 0 && share < n) n = share;
        }
        std::fclose(f);
    }
    return n;
}

void rt_destroy(rt_context* c) {
    if (!c) return;
    if (c->cpu) {
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->render_pending = false;  // its launch is done: the stream is synchronised
    if (c->render_recorded) (void)hipEventSynchronize(c->ev_render);
    if (c->aux_recorded) (void)hipEventSynchronize(c->ev_aux);
    free_buf(c->scene_buf);
    free_buf(c->rng);
    free_buf(c->accum);
    free_buf(c->rgba);
    free_buf(c->rec);
    free_buf(c->gcost);
    free_buf(c->gorder);
    if (c->host_rgba) (void)hipHostFree(c->host_rgba);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev_render) (void)hipEventDestroy(c->ev_render);
    if (c->ev_aux) (void)hipEventDestroy(c->ev_aux);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int rt_set_scene(rt_context* c, const rt_scene* s) {
    const HostFpEnv fp;
    if (!c || !s) return fail(c, RT_ERR_INVALID_ARGUMENT, "null argument");
    if (s->sphere_count < 0 || s->plane_count < 0 || s->triangle_count < 0 || s->quad_count < 0)
        return fail(c, RT_ERR_INVALID_ARGUMENT, "negative primitive count");
    if ((s->sphere_count && !s->spheres) || (s->plane_count && !s->planes) ||
        (s->triangle_count && !s->triangles) || (s->quad_count && !s->quads))
        return fail(c, RT_ERR_INVALID_ARGUMENT, "null primitive array with non-zero count");
    if (!c->cpu) HIP_TRY(c, hipSetDevice(c->device));
    const int ns = s->sphere_count, np = s->plane_count, nt = s->triangle_count, nq = s->quad_count;
    const size_t off_pln = (size_t)ns * RT_SPH_FLOATS;
    const size_t off_tri = off_pln + (size_t)np * RT_PLN_FLOATS;
    const size_t off_quad = off_tri + (size_t)nt * RT_TRI_FLOATS;
    const size_t off_hit = off_quad + (size_t)nq * RT_QUAD_FLOATS;
    const size_t total = off_hit + (size_t)(ns + np + nt + nq) * RT_HIT_FLOATS + 4;
    std::vector<float> h(total, 0.0f);
    float* hit = h.data() + off_hit;
    int id = 0;
    for (int i = 0; i < ns; i++, id++) {  // Intersection.cuh:32-38
        const rt_sphere& sp = s->spheres[i];
        float* q = h.data() + (size_t)i * RT_SPH_FLOATS;
        q[0] = sp.position.x;
        q[1] = sp.position.y;
        q[2] = sp.position.z;
        q[3] = sp.radius * sp.radius;
        float* hh = hit + (size_t)id * RT_HIT_FLOATS;
        hh[0] = sp.position.x;
        hh[1] = sp.position.y;
        hh[2] = sp.position.z;
        hh[3] = 1.0f;  // sphere: normal = normalize(P - centre)
        put_material(hh, sp.mat);
    }
    for (int i = 0; i < np; i++, id++) {  // Intersection.cuh:69,83
        const rt_plane& pl = s->planes[i];
        V3 n = cross(v3(pl.directions[0]), v3(pl.directions[1]));
        float d = -dot(n, v3(pl.origin));
        float* q = h.data() + off_pln + (size_t)i * RT_PLN_FLOATS;
        q[0] = n.x;
        q[1] = n.y;
        q[2] = n.z;
        q[3] = d;
        float* hh = hit + (size_t)id * RT_HIT_FLOATS;
        hh[0] = n.x;
        hh[1] = n.y;
        hh[2] = n.z;
        hh[3] = 0.0f;
        put_material(hh, pl.mat);
    }
    // scene scale for polygon culling: >= every primitive coordinate and the
    // camera position; rays whose origin lies beyond it are never culled
    double scale = 1.0;
    auto grow = [&](const rt_vec3& v, double extra) {
        scale = std::max(scale, std::max(std::fabs((double)v.x), std::max(std::fabs((double)v.y), std::fabs((double)v.z))) + extra);
    };
    grow(s->camera.position, 0.0);
    for (int i = 0; i < ns; i++) grow(s->spheres[i].position, std::fabs((double)s->spheres[i].radius));
    for (int i = 0; i < nt; i++)
        for (int k = 0; k < 3; k++) grow(s->triangles[i].vertices[k], 0.0);
    for (int i = 0; i < nq; i++)
        for (int k = 0; k < 4; k++) grow(s->quads[i].vertices[k], 0.0);
    scale *= 2.0;
    if (!std::isfinite(scale) || scale > 1e30 || tuning_env("BWRT_NO_CULL")) scale = INFINITY;
    c->cull_omax = std::isfinite(scale) ? (float)scale : -1.0f;  // -1: no ray is culled
    for (int i = 0; i < nt; i++, id++)
        compile_polygon(h.data() + off_tri + (size_t)i * RT_TRI_FLOATS, hit + (size_t)id * RT_HIT_FLOATS,
                        s->triangles[i].vertices, 3, s->triangles[i].mat, scale);
    for (int i = 0; i < nq; i++, id++)
        compile_polygon(h.data() + off_quad + (size_t)i * RT_QUAD_FLOATS, hit + (size_t)id * RT_HIT_FLOATS,
                        s->quads[i].vertices, 4, s->quads[i].mat, scale);
    // overflow bounds of the bounded primitives' tests (rt_layout.h ovf_*;
    // a NaN or inf input makes its bound infinite, so no ray is culled and
    // every BVH ray takes the brute-force loop)
    {
        double sc = 0.0, rmax = 0.0, nm = 0.0, im = 0.0;
        auto upd = [](double& b, float x) {
            const double a = std::fabs((double)x);
            if (!(a <= b)) b = std::isnan(a) ? INFINITY : a;
        };
        for (int i = 0; i < ns; i++) {
            const rt_sphere& sp = s->spheres[i];
            upd(sc, sp.position.x);
            upd(sc, sp.position.y);
            upd(sc, sp.position.z);
            upd(rmax, sp.radius);
        }
        auto polyb = [&](const rt_vec3* v, int nv, const float* rec) {
            for (int k = 0; k < nv; k++) {
                upd(sc, v[k].x);
                upd(sc, v[k].y);
                upd(sc, v[k].z);
            }
            for (int a = 0; a < 3; a++) upd(nm, rec[a]);
            for (int k = 0; k < nv; k++)  // {v_k[3], in_k[3]} from float 4 on
                for (int a = 0; a < 3; a++) upd(im, rec[RT_POLY_EDGES + 6 * k + 3 + a]);
        };
        for (int i = 0; i < nt; i++) polyb(s->triangles[i].vertices, 3, h.data() + off_tri + (size_t)i * RT_TRI_FLOATS);
        for (int i = 0; i < nq; i++) polyb(s->quads[i].vertices, 4, h.data() + off_quad + (size_t)i * RT_QUAD_FLOATS);
        const double S = (sc + rmax) * (1.0 + 1e-6), N = nm * (1.0 + 1e-6), I = im * (1.0 + 1e-6);
        c->ovf_sc = (float)std::min(S, 3e38);
        c->ovf_nm = (float)std::min(N, 3e38);
        c->ovf_im = (float)std::min(I, 3e38);
        // culling (polygon_test) skips only polygons whose exact test rejects
        // the ray; a NaN in the inside test would instead accept it, so rays
        // are culled only when, for every origin within cull_omax, no polygon
        // test can overflow: max|d_i| <= cull_dmax (the bounds of the
        // kernel's bvh_safe with om = cull_omax, halved)
        double dmax = INFINITY;
        if (c->cull_omax > 0.0f) {
            const double om = c->cull_omax;
            dmax = std::min(dmax, 1e18 / (om + S));
            if (N > 0.0) {
                dmax = std::min(dmax, 1e36 / N);
                dmax = std::min(dmax, (1e37 - om - S) / (6e4 * N * (om + 3.0 * S)));  // P finite
                if (I > 0.0) dmax = std::min(dmax, (3e36 / I - om - S) / (6e4 * N * (om + 3.0 * S)));
                if (!(N * (om + 3.0 * S) < 1e33)) dmax = -1.0;  // t = num / nd may overflow
            }
            dmax *= 0.5;
        }
        c->cull_dmax = std::isfinite(dmax) ? (float)std::min(dmax, 3e38) : (dmax > 0.0 ? INFINITY : -1.0f);
        if (!(c->cull_dmax > 0.0f)) c->cull_dmax = -1.0f;
    }
    // BVH for large scenes (BWRT_BVH_MIN primitives, default 64)
    size_t off_bvh = 0, off_bvh_prims = 0, off_bvh_vtx = 0, off_bvh16 = 0;
    {
        int bvh_min = 64;
        if (const char* e = tuning_env("BWRT_BVH_MIN")) bvh_min = std::atoi(e);
        const int nb = ns + nt + nq;
        if (nb > 0 && nb >= bvh_min) {
            // leaf encoding: 24-bit index of a leaf's first primitive record
            if (nb >= (1 << 24))
                return fail(c, RT_ERR_UNSUPPORTED, "%d bounded primitives: the BVH holds at most 2^24 - 1", nb);
            BvhBuilder B;
            B.items.reserve(nb);
            for (int i = 0; i < ns; i++) {
                const rt_sphere& sp = s->spheres[i];
                const float r = std::fabs(sp.radius);
                const float lo[3] = {sp.position.x - r, sp.position.y - r, sp.position.z - r};
                const float hi[3] = {sp.position.x + r, sp.position.y + r, sp.position.z + r};
                B.add(i, lo, hi);
            }
            auto poly = [&](int id, const rt_vec3* v, int nv) {
                float lo[3] = {v[0].x, v[0].y, v[0].z}, hi[3] = {v[0].x, v[0].y, v[0].z};
                for (int k = 1; k < nv; k++) {
                    const float p[3] = {v[k].x, v[k].y, v[k].z};
                    for (int a = 0; a < 3; a++) {
                        lo[a] = std::min(lo[a], p[a]);
                        hi[a] = std::max(hi[a], p[a]);
                    }
                }
                B.add(id, lo, hi);
            };
            for (int i = 0; i < nt; i++) poly(ns + np + i, s->triangles[i].vertices, 3);
            for (int i = 0; i < nq; i++) poly(ns + np + nt + i, s->quads[i].vertices, 4);
            B.tree.reserve(2 * (size_t)nb);
            // leaf = (count << 24) | first in an int: count <= 127 keeps the sign
            // bit clear (a negative value means "internal node" to the kernels)
            if (const char* e = tuning_env("BWRT_BVH_LEAF")) B.max_leaf = std::min(std::max(std::atoi(e), 1), 127);
            if (const char* e = tuning_env("BWRT_BVH_CT")) B.trav_cost = (float)std::atof(e);
            // spatial splits (BWRT_BVH_SBVH=0: object splits only), references
            // up to BWRT_BVH_REFS x the primitives (default 2)
            bool sbvh = true;
            if (const char* e = tuning_env("BWRT_BVH_SBVH")) sbvh = std::atoi(e) != 0;
            if (sbvh) {
                B.geo.assign((size_t)12 * (ns + np + nt + nq), 0.0);
                B.geo_nv.assign((size_t)(ns + np + nt + nq), 0);
                auto geo = [&](int id, const rt_vec3* v, int nv) {
                    B.geo_nv[id] = nv;
                    for (int k = 0; k < nv; k++) {
                        B.geo[(size_t)12 * id + 3 * k + 0] = v[k].x;
                        B.geo[(size_t)12 * id + 3 * k + 1] = v[k].y;
                        B.geo[(size_t)12 * id + 3 * k + 2] = v[k].z;
                    }
                };
                for (int i = 0; i < nt; i++) geo(ns + np + i, s->triangles[i].vertices, 3);
                for (int i = 0; i < nq; i++) geo(ns + np + nt + i, s->quads[i].vertices, 4);
                std::vector<BvhBuilder::Ref> refs;
                refs.reserve(nb);
                double rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
                auto addref = [&](int id, const double* lo, const double* hi) {
                    BvhBuilder::Ref r;
                    for (int a = 0; a < 3; a++) {
                        r.lo[a] = lo[a];
                        r.hi[a] = hi[a];
                        rlo[a] = std::min(rlo[a], lo[a]);
                        rhi[a] = std::max(rhi[a], hi[a]);
                    }
                    r.id = id;
                    refs.push_back(r);
                };
                for (int i = 0; i < ns; i++) {
                    const rt_sphere& sp = s->spheres[i];
                    const double r = std::fabs((double)sp.radius);
                    const double lo[3] = {sp.position.x - r, sp.position.y - r, sp.position.z - r};
                    const double hi[3] = {sp.position.x + r, sp.position.y + r, sp.position.z + r};
                    addref(i, lo, hi);
                }
                auto polyref = [&](int id, const rt_vec3* v, int nv) {
                    double lo[3] = {v[0].x, v[0].y, v[0].z}, hi[3] = {v[0].x, v[0].y, v[0].z};
                    for (int k = 1; k < nv; k++) {
                        const double p[3] = {v[k].x, v[k].y, v[k].z};
                        for (int a = 0; a < 3; a++) lo[a] = std::min(lo[a], p[a]), hi[a] = std::max(hi[a], p[a]);
                    }
                    addref(id, lo, hi);
                };
                for (int i = 0; i < nt; i++) polyref(ns + np + i, s->triangles[i].vertices, 3);
                for (int i = 0; i < nq; i++) polyref(ns + np + nt + i, s->quads[i].vertices, 4);
                double refs_x = 2.0;
                if (const char* e = tuning_env("BWRT_BVH_REFS")) refs_x = std::atof(e);
                if (const char* e = tuning_env("BWRT_BVH_ALPHA")) B.split_alpha = std::atof(e);
                B.root_area = BvhBuilder::darea(rlo, rhi);
                B.ref_budget = (size_t)(refs_x * nb);
                B.n_refs = (size_t)nb;
                B.build_s(refs);
                if (B.prims.size() >= (1u << 24))
                    return fail(c, RT_ERR_UNSUPPORTED, "%zu BVH references: at most 2^24 - 1", B.prims.size());
            } else {
                B.build(0, nb);
            }
            // octant arrays only along the scene's long axes (extent >= half
            // the longest): each bit doubles the node data the walks spread
            // over the caches, and a short axis buys little front-to-back
            // order.  Config 5 (extents ~25 / 9 / 31): x and z, 157 -> 147 ms
            // with 16-byte nodes (all three axes; z alone 187, x alone 272)
            {
                const BvhNode& root = B.tree[0];
                float ext[3], mx = 0.0f;
                for (int a = 0; a < 3; a++) mx = std::max(mx, ext[a] = root.hi[a] - root.lo[a]);
                B.order_mask = 0;
                for (int a = 0; a < 3; a++)
                    if (!(ext[a] < 0.5f * mx)) B.order_mask |= 1 << a;
            }
            if (const char* e = tuning_env("BWRT_BVH_ORDER_MASK")) B.order_mask = std::atoi(e) & 7;
            B.finish();
            if (tuning_env("BWRT_BVH_STATS")) {  // diagnostics (tests, tuning)
                long ax[3] = {0, 0, 0}, inner = 0;
                for (const BvhNode& t : B.tree)
                    if (t.left >= 0) ax[t.axis]++, inner++;
                std::fprintf(stderr, "bvh: %d nodes, %ld internal, %zu references of %d primitives, split axes x %ld y %ld z %ld, octant mask %d, n16 %d\n",
                             (int)B.tree.size(), inner, B.prims.size(), nb, ax[0], ax[1], ax[2], B.order_mask, B.n16 ? 1 : 0);
            }
            c->bvh_nodes_per_order = B.n_nodes;
            c->bvh_order_mask = B.order_mask;
            off_bvh = (total + 3) & ~(size_t)3;
            // leaf records, RT_LEAF_FLOATS (128 B) each, start on a 128-byte
            // boundary: a record spans one cache line
            off_bvh_prims = (off_bvh + B.nodes.size() + 31) & ~(size_t)31;
            // vertex-form leaf records after them (64 B each, 64-byte aligned;
            // the GPU's ray-refill kernel reads these, the CPU walk the full
            // form), then the 16-byte nodes, again from a 128-byte boundary
            // (eight nodes per line, the same lines for every scene)
            off_bvh_vtx = off_bvh_prims + B.prims.size() * RT_LEAF_FLOATS;
            off_bvh16 = B.n16 ? (off_bvh_vtx + B.prims.size() * RT_LEAF_VFLOATS + 31) & ~(size_t)31 : 0;
            h.resize((B.n16 ? off_bvh16 + B.nodes16.size() : off_bvh_vtx + B.prims.size() * RT_LEAF_VFLOATS) + 4, 0.0f);
            std::memcpy(h.data() + off_bvh, B.nodes.data(), B.nodes.size() * sizeof(float));
            if (B.n16) std::memcpy(h.data() + off_bvh16, B.nodes16.data(), B.nodes16.size() * sizeof(uint32_t));
            for (size_t j = 0; j < B.prims.size(); j++) {
                const int id = B.prims[j];
                float* r = h.data() + off_bvh_prims + j * RT_LEAF_FLOATS;
                int kind, idx, nf;
                const float* src;
                if (id < ns) {
                    kind = 0, idx = id, nf = RT_SPH_FLOATS, src = h.data() + (size_t)idx * RT_SPH_FLOATS;
                } else if (id < ns + np + nt) {  // (the BVH does not cull: no cull sphere)
                    kind = 2, idx = id - ns - np, nf = RT_TRI_CULL, src = h.data() + off_tri + (size_t)idx * RT_TRI_FLOATS;
                } else {
                    kind = 3, idx = id - ns - np - nt, nf = RT_QUAD_CULL,
                    src = h.data() + off_quad + (size_t)idx * RT_QUAD_FLOATS;
                }
                // {key, record...} (rt_layout.h): kind = key & 3, the id
                // follows from the index; polygons as {n, d, edges} without
                // the cull sphere wherever the compiled record keeps it
                const int key = RT_KEY(kind, idx);
                std::memcpy(&r[0], &key, 4);
                float* rv = h.data() + off_bvh_vtx + j * RT_LEAF_VFLOATS;  // vertex form
                std::memcpy(&rv[0], &key, 4);
                if (kind == 0) {
                    std::memcpy(&r[1], src, (size_t)nf * sizeof(float));
                    std::memcpy(&rv[1], src, (size_t)nf * sizeof(float));
                } else {
                    std::memcpy(&r[1], src, 4 * sizeof(float));
                    std::memcpy(&r[5], src + RT_POLY_EDGES, (size_t)(kind == 2 ? 18 : 24) * sizeof(float));
                    for (int k = 0; k < (kind == 2 ? 3 : 4); k++)
                        std::memcpy(&rv[1 + 3 * k], src + RT_POLY_EDGES + 6 * k, 3 * sizeof(float));
                }
            }
        }
    }
    if (c->cpu) {
        c->scene_h.swap(h);
    } else {
        const size_t bytes = h.size() * sizeof(float);
        int rc = quiesce(c);  // a render on a caller's stream may still read the scene
        if (!rc) rc = ensure_buf(c, c->scene_buf, bytes);
        if (rc) return rc;
        HIP_TRY(c, hipMemcpyAsync(c->scene_buf.p, h.data(), bytes, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    c->n_sph = ns;
    c->n_pln = np;
    c->n_tri = nt;
    c->n_quad = nq;
    c->off_pln = off_pln;
    c->off_tri = off_tri;
    c->off_quad = off_quad;
    c->off_hit = off_hit;
    c->off_bvh = off_bvh;
    c->off_bvh_prims = off_bvh_prims;
    c->off_bvh_vtx = off_bvh_vtx;
    c->off_bvh16 = tuning_env("BWRT_BVH_N16") && !std::atoi(tuning_env("BWRT_BVH_N16")) ? 0 : off_bvh16;
    c->camera = s->camera;
    c->has_scene = true;
    c->frame = 1;
    c->order_stale = true;
    return RT_OK;
}

int rt_set_camera(rt_context* c, const rt_camera* cam) {
    if (!c || !cam) return fail(c, RT_ERR_INVALID_ARGUMENT, "null argument");
    c->camera = *cam;
    c->frame = 1;  // Controls.cuh: any movement sets accumulatedFrames = 1
    c->order_stale = true;
    return RT_OK;
}

int rt_set_background(rt_context* c, float r, float g, float b) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    c->background[0] = r;
    c->background[1] = g;
    c->background[2] = b;
    return RT_OK;
}

int rt_get_camera(const rt_context* c, rt_camera* cam) {
    if (!c || !cam) return RT_ERR_INVALID_ARGUMENT;
    *cam = c->camera;
    return RT_OK;
}

// Controls.cuh:5-75 in the reference's float operation order: the direction
// vectors are rotY * rotX (matrix product, Math.cuh:191-199) times a basis
// vector (mat * vec = row dots, Math.cuh:144-150); position +/-= k * dir.
int rt_apply_controls(rt_camera* cam, unsigned keys, float dt) {
    if (!cam) return RT_ERR_INVALID_ARGUMENT;
    const HostFpEnv fp;
    const float move = 5 * dt;
    const float rot = 2 * dt;
    const float cy = cosf(cam->angle[0]), sy = sinf(cam->angle[0]);  // rotationMatrix3DY
    const float cx = cosf(cam->angle[1]), sx = sinf(cam->angle[1]);  // rotationMatrix3DX
    const float L[3][3] = {{cy, 0, sy}, {0, 1, 0}, {-sy, 0, cy}};
    const float U[3][3] = {{1, 0, 0}, {0, cx, -sx}, {0, sx, cx}};
    float M[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) M[i][j] = L[i][0] * U[0][j] + L[i][1] * U[1][j] + L[i][2] * U[2][j];
    auto mul = [&](float x, float y, float z) {
        return V3{M[0][0] * x + M[0][1] * y + M[0][2] * z, M[1][0] * x + M[1][1] * y + M[1][2] * z,
                  M[2][0] * x + M[2][1] * y + M[2][2] * z};
    };
    const V3 front = mul(0, 0, -1), right = mul(1, 0, 0);
    rt_vec3& p = cam->position;
    int flags = 0;
    auto add = [&](float k, V3 v, float sign) {  // position (+|-)= k * v
        const V3 kv{k * v.x, k * v.y, k * v.z};
        if (sign > 0) {
            p.x = p.x + kv.x;
            p.y = p.y + kv.y;
            p.z = p.z + kv.z;
        } else {
            p.x = p.x - kv.x;
            p.y = p.y - kv.y;
            p.z = p.z - kv.z;
        }
        flags |= RT_CONTROLS_MOVED;
    };
    if (keys & RT_KEY_W) add(move, front, +1);
    if (keys & RT_KEY_A) add(move, right, -1);
    if (keys & RT_KEY_S) add(move, front, -1);
    if (keys & RT_KEY_D) add(move, right, +1);
    if (keys & RT_KEY_SPACE) {
        p.y += move;
        flags |= RT_CONTROLS_MOVED;
    }
    if (keys & RT_KEY_LEFT_SHIFT) {
        p.y -= move;
        flags |= RT_CONTROLS_MOVED;
    }
    if (keys & RT_KEY_LEFT) {
        cam->angle[0] += rot;
        flags |= RT_CONTROLS_MOVED;
    }
    if (keys & RT_KEY_RIGHT) {
        cam->angle[0] -= rot;
        flags |= RT_CONTROLS_MOVED;
    }
    if (keys & RT_KEY_UP) {
        cam->angle[1] += rot;
        flags |= RT_CONTROLS_MOVED;
    }
    if (keys & RT_KEY_DOWN) {
        cam->angle[1] -= rot;
        flags |= RT_CONTROLS_MOVED;
    }
    if (keys & RT_KEY_ESCAPE) flags |= RT_CONTROLS_QUIT;
    return flags;
}

int rt_controls(rt_context* c, unsigned keys, float dt) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    const int flags = rt_apply_controls(&c->camera, keys, dt);
    if (flags > 0 && (flags & RT_CONTROLS_MOVED)) {
        c->frame = 1;  // accumulatedFrames = 1
        c->order_stale = true;
    }
    return flags;
}

int rt_reset_accumulation(rt_context* c) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    c->frame = 1;
    return RT_OK;
}

unsigned rt_frame_counter(const rt_context* c) { return c ? c->frame : 0u; }

int rt_set_max_bounces(rt_context* c, int mb) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    if (mb < 0) return fail(c, RT_ERR_INVALID_ARGUMENT, "max_bounces < 0");
    if (mb > RT_MAX_BOUNCES) return fail(c, RT_ERR_UNSUPPORTED, "max_bounces > %d", RT_MAX_BOUNCES);
    c->max_bounces = mb;
    return RT_OK;
}

int rt_set_samples_per_pixel(rt_context* c, int n) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    if (n < 1) return fail(c, RT_ERR_INVALID_ARGUMENT, "samples per pixel < 1");
    if (n > RT_MAX_SAMPLES_PER_PIXEL)
        return fail(c, RT_ERR_UNSUPPORTED, "samples per pixel > %d", RT_MAX_SAMPLES_PER_PIXEL);
    c->spp_inner = n;
    return RT_OK;
}

int rt_set_kernel_timing(rt_context* c, int enable) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    c->ktiming = enable != 0;
    if (!c->ktiming) c->timed = false;  // no stale duration from an earlier launch
    return RT_OK;
}

int rt_shard_rows(int height, int row_offset, int row_stride) {
    return shard_rows(height, row_offset, row_stride == 0 ? 1 : row_stride);
}

int rt_init_rand(rt_context* c, int width, int height, int row_offset, int row_stride) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    if (row_stride == 0) row_stride = 1;
    if (width <= 0 || height <= 0 || row_offset < 0 || row_stride < 0 || row_offset >= height)
        return fail(c, RT_ERR_INVALID_ARGUMENT, "bad shard %dx%d offset %d stride %d", width, height,
                    row_offset, row_stride);
    if ((long long)width * height > (1ll << 31))
        return fail(c, RT_ERR_UNSUPPORTED, "image larger than 2^31 pixels");
    const int rows = shard_rows(height, row_offset, row_stride);
    const size_t npix = (size_t)rows * width;
    if (c->cpu) {
        try {
            c->rng_h.assign(npix * 6, 0u);
            c->accum_h.assign(npix * 3, 0.0f);
            c->rgba_h.assign(npix, 0u);
        } catch (...) {
            return fail(c, RT_ERR_OUT_OF_MEMORY, "host state for %zu pixels", npix);
        }
        rt_cpu_init_rand(c->rng_h.data(), width, rows, row_offset, row_stride);
    }
    if (c->cpu) {
        c->width = width;
        c->height = height;
        c->row_offset = row_offset;
        c->row_stride = row_stride;
        c->rows = rows;
        c->frame = 1;
        return RT_OK;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = quiesce(c);  // a render on a caller's stream may still use the state
    if (!rc) rc = ensure_buf(c, c->rng, npix * 6 * sizeof(unsigned));
    if (!rc) rc = ensure_buf(c, c->accum, npix * 3 * sizeof(float));
    if (rc) return rc;
    HIP_TRY(c, hipMemsetAsync(c->accum.p, 0, npix * 3 * sizeof(float), c->stream));
    HIP_TRY(c, rt_launch_init_rand((unsigned*)c->rng.p, width, rows, row_offset, row_stride, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->width = width;
    c->height = height;
    c->row_offset = row_offset;
    c->row_stride = row_stride;
    c->rows = rows;
    c->frame = 1;
    c->order_stale = true;
    return RT_OK;
}

static int prepare(rt_context* c, const rt_render_params* p, rt_kparams& K, unsigned& first) {
    const HostFpEnv fp;
    if (!c || !p) return fail(c, RT_ERR_INVALID_ARGUMENT, "null argument");
    if (!c->has_scene) return fail(c, RT_ERR_NO_SCENE, "rt_set_scene() not called");
    const int stride = p->row_stride == 0 ? 1 : p->row_stride;
    if (p->width <= 0 || p->height <= 0 || p->samples <= 0 || p->row_offset < 0 || stride < 0 ||
        p->row_offset >= p->height)
        return fail(c, RT_ERR_INVALID_ARGUMENT, "bad render params %dx%d samples %d shard %d/%d", p->width,
                    p->height, p->samples, p->row_offset, stride);
    if (p->max_bounces < 0) return fail(c, RT_ERR_INVALID_ARGUMENT, "max_bounces < 0");
    if (p->max_bounces > RT_MAX_BOUNCES)
        return fail(c, RT_ERR_UNSUPPORTED, "max_bounces %d > %d", p->max_bounces, RT_MAX_BOUNCES);
    if (c->width != p->width || c->height != p->height || c->row_offset != p->row_offset ||
        c->row_stride != stride || (c->cpu ? c->rng_h.empty() : !c->rng.p)) {
        int rc = rt_init_rand(c, p->width, p->height, p->row_offset, stride);
        if (rc) return rc;
    }
    first = p->first_frame ? p->first_frame : c->frame;
    if ((unsigned long long)first + (unsigned)p->samples > 0xffffffffull)
        return fail(c, RT_ERR_INVALID_ARGUMENT, "frame counter overflow");
    if (!c->cpu) HIP_TRY(c, hipSetDevice(c->device));

    std::memset(&K, 0, sizeof K);
    K.width = p->width;
    K.height = p->height;
    K.row_offset = p->row_offset;
    K.row_stride = stride;
    K.rows = c->rows;
    K.samples = p->samples;
    K.max_bounces = p->max_bounces;
    K.first_frame = first;
    // host prelude, Main.cu:336-338
    const rt_camera& cam = c->camera;
    K.cam_pos[0] = cam.position.x;
    K.cam_pos[1] = cam.position.y;
    K.cam_pos[2] = cam.position.z;
    K.screen_z = -(float)(p->width / 2) / tanf(cam.fov / 2.0f);
    {
        const float cy = cosf(cam.angle[0]), sy = sinf(cam.angle[0]);  // rotationMatrix3DY
        const float cx = cosf(cam.angle[1]), sx = sinf(cam.angle[1]);  // rotationMatrix3DX
        const float L[3][3] = {{cy, 0, sy}, {0, 1, 0}, {-sy, 0, cy}};
        const float U[3][3] = {{1, 0, 0}, {0, cx, -sx}, {0, sx, cx}};
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)  // dot(a.row(i), b.col(j)), Math.cuh:191-199
                K.rot[3 * i + j] = L[i][0] * U[0][j] + L[i][1] * U[1][j] + L[i][2] * U[2][j];
    }
    K.jitter = (float)(0.001 * (p->width / 1000));  // Main.cu:291
    K.bg[0] = c->background[0];
    K.bg[1] = c->background[1];
    K.bg[2] = c->background[2];
    K.n_sph = c->n_sph;
    K.n_pln = c->n_pln;
    K.n_tri = c->n_tri;
    K.n_quad = c->n_quad;
    K.cull_omax = c->cull_omax;
    K.bvh_order_stride = c->bvh_nodes_per_order * 8;
    K.bvh_order_mask = c->bvh_order_mask;
    int nmax = c->n_sph;  // Main.cu:217
    if (c->n_pln > nmax) nmax = c->n_pln;
    if (c->n_tri > nmax) nmax = c->n_tri;
    if (c->n_quad > nmax) nmax = c->n_quad;
    K.n_max = nmax;
    const float* base = c->cpu ? c->scene_h.data() : (const float*)c->scene_buf.p;
    K.sph = base;
    K.pln = base + c->off_pln;
    K.tri = base + c->off_tri;
    K.quad = base + c->off_quad;
    K.hit = base + c->off_hit;
    K.bvh_nodes = c->off_bvh ? base + c->off_bvh : nullptr;
    K.bvh_leafrec = c->off_bvh ? base + c->off_bvh_prims : nullptr;
    K.bvh_leafvtx = c->off_bvh ? base + c->off_bvh_vtx : nullptr;
    K.bvh_nodes16 = c->off_bvh && c->off_bvh16 ? reinterpret_cast<const unsigned*>(base + c->off_bvh16) : nullptr;
    K.bvh_n_nodes = c->bvh_nodes_per_order;
    K.ovf_sc = c->ovf_sc;
    K.ovf_nm = c->ovf_nm;
    K.ovf_im = c->ovf_im;
    K.cull_dmax = c->cull_dmax;
    K.spp_inner = c->spp_inner;
    K.rng = c->cpu ? c->rng_h.data() : (unsigned*)c->rng.p;
    K.accum = c->cpu ? c->accum_h.data() : (float*)c->accum.p;
    return RT_OK;
}

// The CPU backend's render: rt_cpu.cpp over the host state, synchronous
static int cpu_render(rt_context* c, const rt_render_params* p, int threads, uint8_t* rgba_out, float* accum_out) {
    rt_kparams K;
    unsigned first = 0;
    int rc = prepare(c, p, K, first);
    if (rc) return rc;
    const size_t npix = (size_t)c->rows * c->width;
    K.rgba = c->rgba_h.data();
    const auto t0 = std::chrono::steady_clock::now();
    rt_cpu_render(K, threads > 0 ? threads : c->threads);
    c->cpu_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->frame = first + (unsigned)p->samples;  // Main.cu:480 accumulatedFrames++
    if (rgba_out) std::memcpy(rgba_out, c->rgba_h.data(), npix * 4);
    if (accum_out)
        for (size_t i = 0; i < npix; i++)
            for (int ch = 0; ch < 3; ch++) accum_out[3 * i + ch] = c->accum_h[ch * npix + i];
    return RT_OK;
}

static int launch(rt_context* c, rt_kparams& K, hipStream_t s, unsigned first, int samples) {
    // wave tiles: 8 x 8 pixels; on small shards (one rank of a multi-GPU
    // frame, below 1024 pixels per CU) 32 x 2 (config 3 at 1/8: 0.249 ->
    // 0.244 ms); BVH scenes 4 x 16 on small shards: squarer tiles keep a
    // wave's rays closer together (config 5: 170.4 -> 167.7 ms; at 1/8 38.5 ->
    // 35.2).  Full brute-force frames took 16 x 4 until late in round 3; with
    // the kernel of then, 8 x 8 is ahead (bench kernel average, config 3,
    // three alternating runs: 0.7495 / 0.7535 / 0.7497 vs 0.7579 / 0.7616 /
    // 0.7559 ms; c2 -3 %, c4 5.51 vs 5.53 ms; 1/2 shard -2 %, 1/4 flat;
    // profiles/r03e/c3_knobs.txt, profiles/r03e/tiles/)
    const bool small = (long)K.rows * K.width <= (long)c->num_cus * 1024;
    K.tile_w = c->tile_w >= 0 ? c->tile_w : K.bvh_nodes ? (small ? 4 : 8) : (small ? 32 : 8);
    K.tile_sq = c->tile_sq;
    // BVH refill kernel: test the parked leaves once this many of a wave's 64
    // lanes are ready; small shards (every wave resident at once, the frame
    // ends with the slowest waves) batch later
    K.leaf_batch = c->leaf_batch > 0 ? c->leaf_batch : small ? RT_LEAF_BATCH_SMALL : RT_LEAF_BATCH;
    K.refill = c->refill > 0 ? c->refill : small ? RT_REFILL_SMALL : RT_REFILL;
    // deep paths: the sorted kernel's record stack in global memory (launch policy)
    K.rec = nullptr;
    if (!c->simple && (c->grec == 1 || (c->grec < 0 && rt_render_wants_global_records(K, c->num_cus)))) {
        const int rc = ensure_buf(c, c->rec, rt_render_rec_floats(K) * sizeof(float));
        if (rc) return rc;
        K.rec = (float*)c->rec.p;
    }
    unsigned long long* stamps = nullptr;
    const int NST = 40;  // 8 per-phase wave-cycle sums + utilisation / branch counters
    if (tuning_env("BWRT_STAMPS")) {  // diagnostic builds (-DRT_STAMPS)
        if (hipMalloc(&stamps, NST * sizeof(unsigned long long)) == hipSuccess)
            (void)hipMemsetAsync(stamps, 0, NST * sizeof(unsigned long long), s);
        K.stamps = stamps;
    }
    const char* gtimes = tuning_env("BWRT_GTIMES");  // diagnostic builds (-DRT_GTIMES): group times file
    const size_t NGT = (size_t)RT_GTIMES_WORDS;
    if (gtimes && !stamps) {
        if (hipMalloc(&stamps, NGT * sizeof(unsigned long long)) == hipSuccess)
            (void)hipMemsetAsync(stamps, 0, NGT * sizeof(unsigned long long), s);
        K.stamps = stamps;
    }
    // launch-order feedback: room for a grid of 64-lane groups over the
    // padded wave tiles (any block size needs fewer groups)
    if (c->order_feedback && !c->simple) {
        const size_t cap = ((size_t)K.width + 128) * ((size_t)K.rows + 128) / 64 + 1;  // tiles padded to 2 x 2
        const void* before = c->gorder.p;
        int rc = ensure_buf(c, c->gcost, cap * sizeof(unsigned));
        if (!rc) rc = ensure_buf(c, c->gorder, cap * sizeof(int));
        if (rc) return rc;
        if (c->gorder.p != before) c->order_n = 0;  // fresh buffer: no order yet
        K.group_cost = (unsigned*)c->gcost.p;
        K.group_order = (int*)c->gorder.p;
        K.order_n = c->order_n;
        K.order_cap = (long)(c->gorder.bytes / sizeof(int));
        // BVH scenes re-sort every launch: their order keeps improving when
        // sorted from costs measured under the previous order (config 5: 85.8
        // / 86.3 / 86.1 ms every launch vs 86.7 / 87.0 / 87.0 every 16th), and
        // the sort is 6.5 us of an 86 ms frame (profiles/r03g/order_period_configs_ab.txt)
        K.order_sort = K.bvh_nodes || c->order_stale || c->launches % (unsigned long long)c->order_period == 0;
        c->order_stale = false;
    }
    // renders continue each other's RNG / frameSum state: a launch on a
    // different stream than the previous one waits for it (no host sync)
    if (c->render_stream && c->render_stream != s) {
        HIP_TRY(c, flush_render(c));
        HIP_TRY(c, hipStreamWaitEvent(s, c->ev_render, 0));
    }
    rt_order_groups_last = 0;
    rt_launched_kernel[0] = 0;
    // every event recorded here is a marker packet the GPU drains between two
    // renders (~5 us each on MI355X, tools/ev_ab.sh): the start marker only
    // with kernel timing on, and one end event that serves both the ordering
    // of later calls (ev_render) and the timing
    if (c->ktiming) HIP_TRY(c, hipEventRecord(c->ev0, s));
    hipError_t e = rt_launch_render(K, c->num_cus, c->grid_mult, c->simple, c->block, s, c->spread);
    if (e == hipSuccess && rt_order_groups_last > 0) c->order_n = rt_order_groups_last;
    c->kernel_name = rt_launched_kernel;
    c->launches++;
    if (gtimes && stamps) {
        std::vector<unsigned long long> h(NGT);
        (void)hipMemcpyAsync(h.data(), stamps, NGT * sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        if (FILE* f = std::fopen(gtimes, "wb")) {
            std::fwrite(h.data(), sizeof(unsigned long long), NGT, f);
            std::fclose(f);
        }
        (void)hipFree(stamps);
        stamps = nullptr;
    }
    if (stamps) {
        unsigned long long h[NST] = {0};
        (void)hipMemcpyAsync(h, stamps, sizeof h, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        std::fprintf(stderr, "stamps");
        for (int k = 0; k < NST; k++) std::fprintf(stderr, " %llu", h[k]);
        std::fprintf(stderr, "\n");
        (void)hipFree(stamps);
    }
    if (e != hipSuccess) return hip_fail(c, e, "rt_render_kernel launch");
    c->render_stream = s;
    if (s == c->stream && !c->ktiming) {
        // the context's own stream, which lives as long as the context: the
        // end event is recorded only when a later call needs it (flush_render),
        // so back-to-back renders carry no marker packet between them
        c->render_pending = true;
    } else {
        c->render_pending = false;
        HIP_TRY(c, hipEventRecord(c->ev_render, s));
        c->render_recorded = true;
    }
    c->timed = c->ktiming;
    c->frame = first + (unsigned)samples;  // Main.cu:480 accumulatedFrames++
    return RT_OK;
}

int rt_render_ex(rt_context* c, const rt_render_params* p, uint8_t* rgba_out, float* accum_out) {
    if (c && c->cpu) return cpu_render(c, p, 0, rgba_out, accum_out);
    rt_kparams K;
    unsigned first = 0;
    int rc = prepare(c, p, K, first);
    if (rc) return rc;
    const size_t npix = (size_t)c->rows * c->width;
    rc = ensure_buf(c, c->rgba, npix * 4);
    if (rc) return rc;
    K.rgba = (unsigned*)c->rgba.p;
    rc = launch(c, K, c->stream, first, p->samples);
    if (rc) return rc;
    if (rgba_out) HIP_TRY(c, hipMemcpyAsync(rgba_out, c->rgba.p, npix * 4, hipMemcpyDeviceToHost, c->stream));
    if (accum_out) {
        std::vector<float> planes(npix * 3);
        HIP_TRY(c, hipMemcpyAsync(planes.data(), c->accum.p, npix * 3 * sizeof(float), hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (size_t i = 0; i < npix; i++)
            for (int ch = 0; ch < 3; ch++) accum_out[3 * i + ch] = planes[ch * npix + i];
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_render(rt_context* c, int width, int height, int samples, uint8_t* rgba_out) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    rt_render_params p;
    p.width = width;
    p.height = height;
    p.samples = samples;
    p.max_bounces = c->max_bounces;
    p.first_frame = 0;
    p.row_offset = 0;
    p.row_stride = 1;
    return rt_render_ex(c, &p, rgba_out, nullptr);
}

// Single-process multi-GPU (the C++ host's counterpart of bench.py's one
// process per GPU): context i renders rows y = i (mod n) on its own stream,
// all launches in flight at once; the shards come back through pinned host
// buffers and are interleaved on the host.
int rt_render_multi(rt_context* const* ctxs, int n, int width, int height, int samples, uint8_t* rgba_out) {
    if (!ctxs || n <= 0 || width <= 0 || height <= 0 || samples <= 0) return RT_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < n; i++) {
        if (!ctxs[i]) return RT_ERR_INVALID_ARGUMENT;
        if (ctxs[i]->cpu) return fail(ctxs[i], RT_ERR_UNSUPPORTED, "rt_render_multi: CPU context");
        for (int j = 0; j < i; j++)
            if (ctxs[j] == ctxs[i]) return fail(ctxs[i], RT_ERR_INVALID_ARGUMENT, "context listed twice");
    }
    const int active = n < height ? n : height;  // contexts beyond the image height get no rows
    // a failure at context i leaves contexts 0..i-1 with renders and copies
    // into their pinned buffers in flight: drain them before returning, so a
    // later call cannot reuse host_rgba under a running copy
    auto drain = [&](int launched, int rc) {
        for (int j = 0; j < launched; j++) {
            (void)hipSetDevice(ctxs[j]->device);
            (void)hipStreamSynchronize(ctxs[j]->stream);
        }
        return rc;
    };
    for (int i = 0; i < active; i++) {
        rt_context* c = ctxs[i];
        rt_render_params p;
        p.width = width;
        p.height = height;
        p.samples = samples;
        p.max_bounces = c->max_bounces;
        p.first_frame = 0;
        p.row_offset = i;
        p.row_stride = n;
        rt_kparams K;
        unsigned first = 0;
        int rc = prepare(c, &p, K, first);
        if (rc) return drain(i, rc);
        const size_t bytes = (size_t)c->rows * width * 4;
        rc = ensure_buf(c, c->rgba, bytes);
        if (rc) return drain(i, rc);
        if (c->host_rgba_bytes < bytes) {
            rc = quiesce(c);
            if (rc) return drain(i, rc);
            if (hipStreamSynchronize(c->stream) != hipSuccess) return drain(i, fail(c, RT_ERR_HIP, "stream sync"));
            if (c->host_rgba) (void)hipHostFree(c->host_rgba);
            c->host_rgba = nullptr;
            c->host_rgba_bytes = 0;
            const hipError_t e = hipHostMalloc(&c->host_rgba, bytes, hipHostMallocDefault);
            if (e != hipSuccess) return drain(i, hip_fail(c, e, "hipHostMalloc"));
            c->host_rgba_bytes = bytes;
        }
        K.rgba = (unsigned*)c->rgba.p;
        rc = launch(c, K, c->stream, first, samples);
        if (rc) return drain(i + 1, rc);
        const hipError_t e = hipMemcpyAsync(c->host_rgba, c->rgba.p, bytes, hipMemcpyDeviceToHost, c->stream);
        if (e != hipSuccess) return drain(i + 1, hip_fail(c, e, "hipMemcpyAsync"));
    }
    for (int i = 0; i < active; i++) {
        rt_context* c = ctxs[i];
        HIP_TRY(c, hipSetDevice(c->device));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if (!rgba_out) continue;
        const uint8_t* src = (const uint8_t*)c->host_rgba;
        for (int j = 0; j < c->rows; j++)
            std::memcpy(rgba_out + ((size_t)(i + j * n) * width) * 4, src + (size_t)j * width * 4, (size_t)width * 4);
    }
    return RT_OK;
}

int rt_render_device(rt_context* c, const rt_render_params* p, void* rgba_device, void* stream) {
    if (c && c->cpu) return fail(c, RT_ERR_UNSUPPORTED, "rt_render_device: CPU context");
    rt_kparams K;
    unsigned first = 0;
    int rc = prepare(c, p, K, first);
    if (rc) return rc;
    if (rgba_device && ((uintptr_t)rgba_device & 3u))
        return fail(c, RT_ERR_INVALID_ARGUMENT, "rgba_device not 4-byte aligned");
    K.rgba = (unsigned*)rgba_device;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return launch(c, K, s, first, p->samples);
}

int rt_synchronize(rt_context* c) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    if (c->cpu) return RT_OK;  // CPU renders are synchronous
    HIP_TRY(c, hipSetDevice(c->device));
    // record a deferred end event first, so ev_render always marks the last
    // render (later renders on a caller's stream wait on it)
    HIP_TRY(c, flush_render(c));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->render_recorded) HIP_TRY(c, hipEventSynchronize(c->ev_render));
    if (c->aux_recorded) HIP_TRY(c, hipEventSynchronize(c->ev_aux));
    return RT_OK;
}

void* rt_get_stream(rt_context* c) { return c && !c->cpu ? (void*)c->stream : nullptr; }

float rt_last_kernel_ms(rt_context* c) {
    if (c && c->cpu) return c->cpu_ms;
    if (!c || !c->timed) return -1.0f;
    if (hipEventSynchronize(c->ev_render) != hipSuccess) return -1.0f;
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev_render) != hipSuccess) return -1.0f;
    return ms;
}

int rt_deinterleave_rows_device(rt_context* c, const void* gathered, void* image, int width, int height,
                                int shards, int rows_per_shard, void* stream) {
    if (!c || !gathered || !image) return fail(c, RT_ERR_INVALID_ARGUMENT, "null argument");
    if (width <= 0 || height <= 0 || shards <= 0 || rows_per_shard * shards < height)
        return fail(c, RT_ERR_INVALID_ARGUMENT, "bad deinterleave geometry");
    if (c->cpu) return fail(c, RT_ERR_UNSUPPORTED, "rt_deinterleave_rows_device: CPU context");
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    HIP_TRY(c, rt_launch_deinterleave((const unsigned*)gathered, (unsigned*)image, width, height, shards,
                                      rows_per_shard, c->deint_blocks, s));
    HIP_TRY(c, hipEventRecord(c->ev_aux, s));
    c->aux_recorded = true;
    return RT_OK;
}

int rt_get_state(rt_context* c, uint32_t* rng, float* accum) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    const size_t npix = (size_t)c->rows * c->width;
    if (c->cpu) {
        if (c->rng_h.empty()) return fail(c, RT_ERR_INVALID_ARGUMENT, "no shard state (render or rt_init_rand first)");
        if (rng) std::memcpy(rng, c->rng_h.data(), npix * 6 * sizeof(unsigned));
        if (accum)
            for (size_t i = 0; i < npix; i++)
                for (int ch = 0; ch < 3; ch++) accum[3 * i + ch] = c->accum_h[ch * npix + i];
        return RT_OK;
    }
    if (!c->rng.p) return fail(c, RT_ERR_INVALID_ARGUMENT, "no shard state (render or rt_init_rand first)");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const int qrc = quiesce(c);  // the last render, on whatever stream it ran
    if (qrc) return qrc;
    if (rng) HIP_TRY(c, hipMemcpy(rng, c->rng.p, npix * 6 * sizeof(unsigned), hipMemcpyDeviceToHost));
    if (accum) {
        std::vector<float> planes(npix * 3);
        HIP_TRY(c, hipMemcpy(planes.data(), c->accum.p, npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < npix; i++)
            for (int ch = 0; ch < 3; ch++) accum[3 * i + ch] = planes[ch * npix + i];
    }
    return RT_OK;
}

int rt_set_state(rt_context* c, const uint32_t* rng, const float* accum, unsigned frame_counter) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    if (c->cpu ? c->rng_h.empty() : !c->rng.p) return fail(c, RT_ERR_INVALID_ARGUMENT, "no shard state (rt_init_rand first)");
    if (frame_counter == 0) return fail(c, RT_ERR_INVALID_ARGUMENT, "frame_counter must be >= 1");
    const size_t npix = (size_t)c->rows * c->width;
    if (c->cpu) {
        if (rng) std::memcpy(c->rng_h.data(), rng, npix * 6 * sizeof(unsigned));
        if (accum)
            for (size_t i = 0; i < npix; i++)
                for (int ch = 0; ch < 3; ch++) c->accum_h[ch * npix + i] = accum[3 * i + ch];
        c->frame = frame_counter;
        return RT_OK;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    const int rc = quiesce(c);  // a render on a caller's stream may still use the state
    if (rc) return rc;
    std::vector<float> planes;
    if (rng)
        HIP_TRY(c, hipMemcpyAsync(c->rng.p, rng, npix * 6 * sizeof(unsigned), hipMemcpyHostToDevice, c->stream));
    if (accum) {
        planes.resize(npix * 3);
        for (size_t i = 0; i < npix; i++)
            for (int ch = 0; ch < 3; ch++) planes[ch * npix + i] = accum[3 * i + ch];
        HIP_TRY(c, hipMemcpyAsync(c->accum.p, planes.data(), npix * 3 * sizeof(float), hipMemcpyHostToDevice,
                                  c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->frame = frame_counter;
    return RT_OK;
}

const char* rt_error_string(int status) {
    switch (status) {
        case RT_OK: return "ok";
        case RT_ERR_INVALID_ARGUMENT: return "invalid argument";
        case RT_ERR_NO_DEVICE: return "no HIP device";
        case RT_ERR_HIP: return "HIP runtime error";
        case RT_ERR_OUT_OF_MEMORY: return "out of device memory";
        case RT_ERR_NO_SCENE: return "no scene";
        case RT_ERR_UNSUPPORTED: return "unsupported";
        default: return "unknown status";
    }
}

const char* rt_last_error(const rt_context* c) { return c ? c->err.c_str() : ""; }

const char* rt_last_kernel_name(const rt_context* c) { return c ? c->kernel_name.c_str() : ""; }

int rt_render_cpu(rt_context* c, const rt_render_params* p, int threads, uint8_t* rgba_out, float* accum_out) {
    if (!c) return RT_ERR_INVALID_ARGUMENT;
    if (!c->cpu) return fail(c, RT_ERR_INVALID_ARGUMENT, "rt_render_cpu: not a CPU context (rt_create_cpu)");
    if (threads < 0) return fail(c, RT_ERR_INVALID_ARGUMENT, "threads < 0");
    return cpu_render(c, p, threads, rgba_out, accum_out);
}

int rt_context_threads(const rt_context* c) { return c && c->cpu ? c->threads : 0; }

}  // extern "C"
