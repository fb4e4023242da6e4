// rt_layout.h — device-side data layout shared by the host scene compiler
// (rt_context.cpp) and the HIP kernels (rt_kernels.hip).
//
// The scene is "compiled" once on upload: every quantity the reference
// recomputes per ray but that depends only on the primitive (plane normal
// cross(d0,d1) Intersection.cuh:69, d = -dot(n,origin) :83, triangle/quad
// edges + normal + inner edge normals :109-127 / :142-162, r*r :38,
// ior^2/1^2 - 1 Main.cu:125) is precomputed with the SAME float operations
// in the same order, so the per-ray arithmetic stays bit-identical to the
// reference semantics while doing less work.
//
// HBM layout (all float32, records padded to 16 B):
//   spheres   : n_sph  x  4 floats  {cx, cy, cz, r*r}
//   planes    : n_pln  x  4 floats  {nx, ny, nz, d}
//   triangles : n_tri  x 28 floats  {nx,ny,nz,d, v0[3],in0[3], v1[3],in1[3], v2[3],in2[3], pad2,
//                                    cull sphere {cx,cy,cz,Rc^2}}
//   quads     : n_quad x 32 floats  {nx,ny,nz,d, v0[3],in0[3], .. v3[3],in3[3], cull {.., Rc^2 = inf}}
//   hit table : n_prim x 16 floats  {n_or_centre[3], is_sphere,
//                                    emittance*albedo[3], 0,
//                                    roughness, ior^2-1, roughness^2, 0,
//                                    4*albedo[3], 0}
//   primitive id = index within its kind + kind offset, kinds ordered
//   spheres, planes, triangles, quads.
//
// Per-pixel progressive state (SoA planes over the shard's pixels
// p = j*width + x, so a wave's 64 lanes touch 256 contiguous bytes):
//   rng   : 6 planes of u32 {d, v0, v1, v2, v3, v4}   (24 B/pixel)
//   accum : 3 planes of f32 {r, g, b}                 (12 B/pixel)
//   rgba  : 1 plane of u32 (bytes r,g,b,255)          ( 4 B/pixel)
#pragma once

#define RT_SPH_FLOATS 4
#define RT_PLN_FLOATS 4
#define RT_TRI_FLOATS 28
#define RT_QUAD_FLOATS 32
#define RT_TRI_CULL 24   // offset of the cull sphere in a triangle record
#define RT_QUAD_CULL 28
#define RT_POLY_EDGES 4  // offset of {v0, in0, v1, in1, ...} in a polygon record
#define RT_LEAF_FLOATS 32  // BVH leaf record: RT_KEY + the record without its cull sphere (<= 28 floats)
#define RT_LEAF_VFLOATS 16 // BVH leaf record, vertex form: RT_KEY + a sphere's {c, r^2} or a polygon's vertices
#ifndef RT_HIT_FLOATS
#define RT_HIT_FLOATS 16
#endif

#define RT_NEAR_ZERO 0.0001f       // Intersection.cuh:4
#define RT_SPECULAR_CHANCE 0.5f    // Main.cu:29
#define RT_PI 3.1415926535f        // Math.cuh:5
#define RT_MAX_LEVELS 33           // recursion records per path: RT_MAX_BOUNCES (rt_abi.h) + 1

// diagnostic builds (-DRT_GTIMES, BWRT_GTIMES): words of the group / lane
// time buffer (rt_diag.h; rt_context.cpp allocates it)
#define RT_GTIMES_WORDS (1ull << 22)

struct rt_kparams {
    int width, height;          // full image
    int row_offset, row_stride; // shard rows y = row_offset + j*row_stride
    int rows;                   // shard rows
    int samples;                // progressive frames in this launch
    int max_bounces;
    unsigned first_frame;
    float cam_pos[3];
    float rot[9];               // rotationMatrix3DY(a0) * rotationMatrix3DX(a1), row-major
    float screen_z;             // Main.cu:336
    float jitter;               // (float)(0.001 * (width / 1000)), Main.cu:291
    float bg[3];                // backgroundColor, Main.cu:27
    int n_sph, n_pln, n_tri, n_quad, n_max;
    const float* sph;
    const float* pln;
    const float* tri;
    const float* quad;
    const float* hit;
    unsigned* rng;              // 6 planes of rows*width
    float* accum;               // 3 planes of rows*width
    unsigned* rgba;             // rows*width (may be null)
    unsigned long long* stamps; // diagnostic builds (-DRT_STAMPS) only: per-phase cycle sums
    int tile_w;                 // wave tile width in pixels (1..64, power of 2); 0 = linear order
    int tile_sq;                // waves of a 4-wave group as 2 x 2 tiles (else 4 tiles in a row)
    // bounding-volume hierarchy over spheres/triangles/quads (large scenes;
    // null = brute-force loop): 8 threaded node arrays (one per ray-direction
    // octant, bit a = d[a] < 0; bvh_order_stride floats apart).  Node: 8
    // floats {bmin.xyz, miss, bmax.xyz, leaf}, depth-first (first child =
    // node + 1, near side of the split first for that octant), miss = next node when
    // the subtree is skipped (-1 = done), leaf = -1 (internal) or
    // (count << 24) | first index into bvh_leafrec: {RT_KEY (kind = key & 3:
    // 0 sphere, 2 triangle, 3 quad; index = key >> 2), then the compiled
    // record without its cull sphere}.
    const float* bvh_nodes;
    const float* bvh_leafrec;   // leaf records in leaf order, RT_LEAF_FLOATS each
    // the same leaves in vertex form (RT_LEAF_VFLOATS each: polygons as
    // {key, v0, v1, v2[, v3]}, the kernel forms their planes and inner
    // normals with compile_polygon's own float operations: three loads in
    // one round trip instead of six in three) — the ray-refill kernel's form
    const float* bvh_leafvtx;
    int bvh_order_stride;
    int bvh_order_mask;         // octant bits with their own arrays (7 = all three axes)
    // the same arrays as 16-byte nodes (null when a box exceeds the fp16
    // range), bvh_n_nodes x 4 words per octant: {lo.x | lo.y << 16,
    // lo.z | hi.x << 16, hi.y | hi.z << 16} as fp16 rounded outward (lo down,
    // hi up: the boxes only grow) and w = the miss link of an internal node
    // (-1 = done) or ~leaf for a leaf, whose miss link is the next node
    const unsigned* bvh_nodes16;
    int bvh_n_nodes;
    // overflow bounds of the bounded primitives' tests (kernel bvh_safe):
    // largest |coordinate| of a vertex / sphere centre plus the largest
    // radius, largest |component| of a triangle / quad normal cross(e0, e1)
    // and of an inner edge normal cross(n, e_k)
    float ovf_sc, ovf_nm, ovf_im;
    // conservative polygon culling (see polygon_test): only rays whose origin
    // satisfies max|o_i| <= cull_omax and whose direction max|d_i| <=
    // cull_dmax (no polygon test can overflow) may skip a polygon's exact test
    float cull_omax;
    float cull_dmax;
    // recursion record stack in global memory (sorted kernel, deep paths and
    // full frames): levels 0 .. RT_GREC_LDS_LEVELS-1 stay in LDS, the deeper
    // ones take 3 * (max_bounces - RT_GREC_LDS_LEVELS) floats per lane of the
    // grid, [group][level - RT_GREC_LDS_LEVELS][field][lane]; null = all
    // records in LDS
    float* rec;
    int rec_stride;             // lanes in the grid (set by the launcher)
    // launch-order feedback (sorted kernel): workgroup g renders tile-group
    // group_order[g] (null = g itself; a permutation of the grid's groups,
    // valid only when order_n equals this launch's grid) and writes that
    // tile-group's duration to group_cost[]; the launcher then sorts the
    // costs so the next launch starts the most expensive tile-groups first
    // and the frame ends on cheap ones.  Null group_cost = feature off.
    int* group_order;
    unsigned* group_cost;
    long order_n;               // grid the current group_order was built for (0 = none)
    long order_cap;             // capacity of group_order / group_cost
    int order_sort;             // sort this launch's costs into group_order (else the order is kept)
    int leaf_batch;             // BVH refill kernel: leaf tests once this many lanes are ready
    int refill;                 // BVH refill kernel: new rays once this many of 64 (relative) wait
    // samplesPerPixel (Main.cu:27, 296-299): paths traced per frame from the
    // frame's one jittered camera ray; the LAST one, scaled by 1/n, is the
    // frame's sample.  1 (the reference build) everywhere but the simple
    // kernel and the CPU fallback, which the launch policy picks for n > 1
    int spp_inner;
};

// leaf-batch thresholds of the launch policy (full frames / small shards)
#ifndef RT_LEAF_BATCH
#define RT_LEAF_BATCH 60
#endif
#ifndef RT_LEAF_BATCH_SMALL
#define RT_LEAF_BATCH_SMALL 62
#endif
// (refill 40 on full frames since the round-5 node-step trimming: config 5
// 80.8 -> 80.1 ms over five alternating pairs; small shards flat between 28
// and 36, profiles/r05h/ab_refill5.txt)
#ifndef RT_REFILL
#define RT_REFILL 40
#endif
// (small shards: 32 since the round-5 leaf-load change, config 5's 1/8
// shard 17.86 -> 17.64 ms over two alternating pairs and ahead in the
// earlier sweep too, profiles/r05h/ab_refill5.txt, ab_knobs6.txt)
#ifndef RT_REFILL_SMALL
#define RT_REFILL_SMALL 32
#endif

// Interleaved test order of Main.cu:221-234 (sphere i, plane i, triangle i,
// quad i, then i+1): a primitive's key; among equal distances the reference
// keeps the LAST tested primitive, i.e. the largest key.
#define RT_KEY(kind, i) ((i) * 4 + (kind))
