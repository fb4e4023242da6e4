/*
 * rt_abi.h — C ABI of the MI355X-native path tracer (libbwrt.so).
 *
 * This is the drop-in boundary for the reference renderer's hot path
 * (IndaPlus22/bwidman-raytracer, paths relative to /root/reference):
 *
 *   reference                                   | replaced by
 *   --------------------------------------------+-----------------------------------------
 *   structs vec3d/material/sphere/plane/        | rt_vec3 / rt_material / rt_sphere /
 *   triangle/quad/camera/scene                  | rt_plane / rt_triangle / rt_quad /
 *   (Math.cuh:35-39, WorldTypes.cuh:9-53)       | rt_camera / rt_scene (byte-compatible)
 *   scene allocateScene()  (Main.cu:38-109)     | rt_set_scene()  (library uploads a copy)
 *   initializeRand<<<>>>   (Main.cu:369-380)    | done lazily by the first render of a frame
 *   cudaMalloc randStates/frameSum              |   size (rt_init_rand() forces it)
 *   (Main.cu:460-465)                           |
 *   render(scene,grid,block,cell,randStates,    | rt_render() / rt_render_ex() /
 *          accumulatedFrames,frameSum)          | rt_render_device()
 *   (Main.cu:317-366, kernel Main.cu:274-315)   |
 *   accumulatedFrames++ / controls() reset      | frame counter kept in the context;
 *   (Main.cu:467,480; Controls.cuh:15..69)      | rt_reset_accumulation(), rt_set_camera()
 *
 * Conventions
 *  - Every function returns RT_OK (0) or a negative rt_status; no exceptions
 *    cross the ABI.  rt_last_error() gives a human-readable message.
 *  - One context = one GPU (HIP device) and one pixel-row shard.  A context
 *    must be used by one host thread at a time.  All calls except
 *    rt_render_device()/rt_deinterleave_rows_device() are synchronous.
 *  - Output RGBA8 buffers are row-major, row 0 = BOTTOM of the screen
 *    (the reference draws texcoord (0,0) at the bottom-left, Main.cu:358).
 *  - Semantics of one "sample" (progressive frame) follow the reference
 *    exactly: jittered camera ray, one path of up to max_bounces+1
 *    closest-hit queries, frameSum reset when the frame number is 1,
 *    frameSum/n -> ACES -> gamma -> *255 -> round -> u8.
 *  - The per-pixel RNG is cuRAND-XORWOW seeded with the global pixel index
 *    y*width+x (Main.cu:377); results are independent of sharding.
 *  - Launch-policy overrides for tuning and diagnostics are environment
 *    variables read ONLY when the process sets BWRT_TUNING=1 (otherwise a
 *    context always takes the measured launch policy); none changes a
 *    result, only kernel choice and speed:
 *      at rt_create:    BWRT_KERNEL=simple, BWRT_BLOCK, BWRT_TILE, BWRT_TILE_SQ,
 *                       BWRT_GREC, BWRT_GRID_MULT, BWRT_LEAF_BATCH, BWRT_REFILL,
 *                       BWRT_SPREAD, BWRT_ORDER, BWRT_ORDER_PERIOD,
 *                       BWRT_STREAM_PRIO=0 (the context's stream at normal
 *                       instead of the highest priority), BWRT_DEINT_BLOCKS
 *      at rt_set_scene: BWRT_BVH_MIN, BWRT_BVH_LEAF, BWRT_BVH_CT, BWRT_BVH_SBVH,
 *                       BWRT_BVH_REFS, BWRT_BVH_ALPHA, BWRT_BVH_ORDER_MASK,
 *                       BWRT_BVH_N16, BWRT_NO_CULL, BWRT_BVH_STATS (report)
 *      per launch:      BWRT_STAMPS, BWRT_GTIMES (diagnostic builds only)
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define RT_API __attribute__((visibility("default")))
#else
#define RT_API
#endif

/* ---- world types (byte-compatible with the reference) ------------------ */

/* Math.cuh:35-39 (vec3d, also used as `color`): 12 bytes */
typedef struct rt_vec3 {
    float x, y, z;
} rt_vec3;

/* WorldTypes.cuh:15-20: 24 bytes.
 * Reference defaults: albedo {0,0,0}, emittance 0, roughness 1,
 * refractiveIndex 1.05 (see rt_material_default()). */
typedef struct rt_material {
    rt_vec3 albedo;
    float emittance;
    float roughness;
    float refractive_index;
} rt_material;

/* WorldTypes.cuh:22-26: 40 bytes (mat at offset 16) */
typedef struct rt_sphere {
    rt_vec3 position;
    float radius;
    rt_material mat;
} rt_sphere;

/* WorldTypes.cuh:28-32: 60 bytes (mat at offset 36).
 * The plane normal is cross(directions[0], directions[1]), NOT normalised
 * (Intersection.cuh:69). */
typedef struct rt_plane {
    rt_vec3 origin;
    rt_vec3 directions[2];
    rt_material mat;
} rt_plane;

/* WorldTypes.cuh:34-37: 60 bytes */
typedef struct rt_triangle {
    rt_vec3 vertices[3];
    rt_material mat;
} rt_triangle;

/* WorldTypes.cuh:39-42: 72 bytes */
typedef struct rt_quad {
    rt_vec3 vertices[4];
    rt_material mat;
} rt_quad;

/* WorldTypes.cuh:9-13: 24 bytes.  angle[0] = yaw (RotY), angle[1] = pitch
 * (RotX), fov in radians (horizontal). */
typedef struct rt_camera {
    rt_vec3 position;
    float angle[2];
    float fov;
} rt_camera;

/* WorldTypes.cuh:44-53: 88 bytes on LP64 (same offsets).  Unlike the
 * reference (device pointers produced by allocateScene), the pointers here
 * are HOST pointers: rt_set_scene() copies the arrays to the GPU; the caller
 * keeps ownership of its arrays. */
typedef struct rt_scene {
    rt_camera camera;
    const rt_sphere* spheres;
    int sphere_count;
    const rt_plane* planes;
    int plane_count;
    const rt_triangle* triangles;
    int triangle_count;
    const rt_quad* quads;
    int quad_count;
} rt_scene;

/* ---- status codes ------------------------------------------------------- */

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARGUMENT = -1,
    RT_ERR_NO_DEVICE = -2,
    RT_ERR_HIP = -3,         /* a HIP runtime call or kernel launch failed */
    RT_ERR_OUT_OF_MEMORY = -4,
    RT_ERR_NO_SCENE = -5,    /* render before rt_set_scene()              */
    RT_ERR_UNSUPPORTED = -6  /* e.g. max_bounces above RT_MAX_BOUNCES      */
} rt_status;

#define RT_MAX_BOUNCES 32
#define RT_DEFAULT_MAX_BOUNCES 5 /* Main.cu:26 */

/* Render request for the extended entry points. */
typedef struct rt_render_params {
    int width;          /* full image width  (Main.cu:23, windowWidth)  */
    int height;         /* full image height (Main.cu:24, windowHeight) */
    int samples;        /* progressive frames rendered by this call (>=1)  */
    int max_bounces;    /* Main.cu:26; B allows B+1 closest-hit queries    */
    unsigned first_frame; /* accumulatedFrames of the first frame of this
                             call; 1 restarts accumulation (Main.cu:301);
                             0 = continue from the context's frame counter */
    int row_offset;     /* shard: render global rows y = row_offset +      */
    int row_stride;     /*        j*row_stride, j = 0..rows-1 (0,1 = all)  */
} rt_render_params;

/* ---- context ------------------------------------------------------------ */

typedef struct rt_context rt_context;

/* Library / ABI version, "major.minor.patch". */
RT_API const char* rt_version(void);

/* Reference material defaults (WorldTypes.cuh:16-19). */
RT_API rt_material rt_material_default(void);

/* Number of visible HIP devices (0 when none; never fails). */
RT_API int rt_device_count(void);

/* Create a context on HIP device `device`.  Without a HIP device this
 * returns RT_ERR_NO_DEVICE: a GPU context never falls back to the CPU. */
RT_API int rt_create(int device, rt_context** out);
RT_API void rt_destroy(rt_context* ctx);

/* ---- scalar C++ CPU fallback ------------------------------------------------
 * The same per-ray arithmetic as the HIP kernels (csrc/rt_path.h, compiled
 * for the host), bit-identical results, one pixel per loop iteration on a
 * pool of `threads` host threads (256-pixel chunks).  It is an explicit
 * backend, never chosen implicitly: only a context made by rt_create_cpu()
 * renders on the CPU, and every entry point above behaves on it as on a GPU
 * context (rt_set_scene, rt_init_rand, rt_render, rt_render_ex, rt_controls,
 * rt_get_state / rt_set_state, ...; rt_last_kernel_ms gives the last render's
 * wall time) except rt_render_device, rt_render_multi and
 * rt_deinterleave_rows_device (RT_ERR_UNSUPPORTED: no device memory).
 * Replaces the reference's config-1 CPU path and is the CPU baseline of
 * bench.py (SURVEY §8(b) rt_render_cpu, §8(d)). */

/* Host threads the process may run on: its sched affinity, capped by a
 * cgroup v2 CPU quota (/sys/fs/cgroup/cpu.max) when one is set. */
RT_API int rt_cpu_threads(void);

/* Create a CPU context rendering on `threads` host threads (0 = all of
 * rt_cpu_threads()).  Needs an x86-64-v3 host (AVX2 + FMA), else
 * RT_ERR_UNSUPPORTED. */
RT_API int rt_create_cpu(int threads, rt_context** out);

/* Host threads of a CPU context (0 for a GPU context). */
RT_API int rt_context_threads(const rt_context* ctx);

/* rt_render_ex() on a CPU context with an explicit thread count for this call
 * (0 = the context's).  RT_ERR_INVALID_ARGUMENT on a GPU context. */
RT_API int rt_render_cpu(rt_context* ctx, const rt_render_params* p, int threads,
                         uint8_t* rgba_out, float* accum_out);

/* Upload a copy of the scene (≈ allocateScene, Main.cu:38-109).  Resets the
 * frame counter to 1, like any camera change in controls().  Waits for a
 * render still running on a caller's stream (rt_render_device) first; so do
 * rt_init_rand and rt_set_state.  Scenes with 2^24 or more spheres +
 * triangles + quads in the BVH return RT_ERR_UNSUPPORTED. */
RT_API int rt_set_scene(rt_context* ctx, const rt_scene* scene);

/* Move the camera (controls(), Controls.cuh:5-75): resets accumulation. */
RT_API int rt_set_camera(rt_context* ctx, const rt_camera* camera);

/* accumulatedFrames = 1 (Controls.cuh:15..69).  RNG streams continue. */
RT_API int rt_reset_accumulation(rt_context* ctx);

/* The frame number the next continuing render will use (accumulatedFrames). */
RT_API unsigned rt_frame_counter(const rt_context* ctx);

/* Default max_bounces for rt_render() (initially RT_DEFAULT_MAX_BOUNCES). */
RT_API int rt_set_max_bounces(rt_context* ctx, int max_bounces);

/* backgroundColor (Main.cu:27, a compile-time constant {0,0,0} there): the
 * radiance of a miss and of the depth cut-off (Main.cu:209-211).  Takes
 * effect at the next render; does not reset accumulation. */
RT_API int rt_set_background(rt_context* ctx, float r, float g, float b);

/* samplesPerPixel (Main.cu:27, a compile-time constant 1 there): each
 * progressive frame traces n paths from the frame's one jittered camera ray
 * and, like the reference's loop (Main.cu:296-299, `pixel = tracePath(...)`
 * assigns), keeps the LAST one, scaled by 1/n; the RNG draws of all n are
 * consumed.  Default 1, the reference build (and the only value whose frames
 * are unbiased).  n > 1 renders with the one-path-per-lane kernel.  Takes
 * effect at the next render; does not reset accumulation. */
#define RT_MAX_SAMPLES_PER_PIXEL 1024
RT_API int rt_set_samples_per_pixel(rt_context* ctx, int n);

/* Copy of the context's current camera (after rt_controls()). */
RT_API int rt_get_camera(const rt_context* ctx, rt_camera* camera);

/* ---- camera controls (Controls.cuh:5-75) ----------------------------------
 * `keys` = OR of the RT_KEY_* held during the frame, `delta_time` = that
 * frame's duration in seconds (Main.cu:482).  Movement speed 5/s, rotation
 * speed 2 rad/s, directions from rotY(angle[0]) * rotX(angle[1]) applied to
 * (0,0,-1) / (1,0,0), evaluated in float in the reference's operation order.
 * Returns an OR of RT_CONTROLS_MOVED (any movement key: accumulation restarts,
 * accumulatedFrames = 1) and RT_CONTROLS_QUIT (escape), or a negative
 * rt_status. */
#define RT_KEY_W          (1u << 0)  /* forward */
#define RT_KEY_A          (1u << 1)  /* left */
#define RT_KEY_S          (1u << 2)  /* back */
#define RT_KEY_D          (1u << 3)  /* right */
#define RT_KEY_SPACE      (1u << 4)  /* up (world y) */
#define RT_KEY_LEFT_SHIFT (1u << 5)  /* down (world y) */
#define RT_KEY_LEFT       (1u << 6)  /* yaw +   (angle[0]) */
#define RT_KEY_RIGHT      (1u << 7)  /* yaw -   */
#define RT_KEY_UP         (1u << 8)  /* pitch + (angle[1]) */
#define RT_KEY_DOWN       (1u << 9)  /* pitch - */
#define RT_KEY_ESCAPE     (1u << 10) /* glfwSetWindowShouldClose */
#define RT_CONTROLS_MOVED 1
#define RT_CONTROLS_QUIT 2

/* Apply one frame of controls to a camera (no context, no GPU). */
RT_API int rt_apply_controls(rt_camera* camera, unsigned keys, float delta_time);

/* Apply one frame of controls to the context's camera; on movement the
 * frame counter restarts at 1 (the next render resets frameSum). */
RT_API int rt_controls(rt_context* ctx, unsigned keys, float delta_time);

/* Allocate and seed the per-pixel state for a (width,height) image shard:
 * curand_init(y*width+x, 0, 0) per pixel (Main.cu:369-380) and a frameSum
 * buffer (Main.cu:464-465).  Called implicitly by the render entry points
 * when the shard changes; calling it again reseeds the RNG. */
RT_API int rt_init_rand(rt_context* ctx, int width, int height,
                        int row_offset, int row_stride);

/* Drop-in render(width, height, samples): renders `samples` progressive
 * frames continuing the context's frame counter, with the context's
 * max_bounces, over the full image, and writes the final RGBA8 image
 * (width*height*4 bytes, row 0 = bottom) to host memory.  rgba_out may be
 * NULL. */
RT_API int rt_render(rt_context* ctx, int width, int height, int samples,
                     uint8_t* rgba_out);

/* Extended synchronous render.  Output rows are the shard's rows in order
 * (rows = number of y with y = row_offset + j*row_stride < height).
 * rgba_out: rows*width*4 bytes or NULL; accum_out: rows*width*3 floats
 * (frameSum, interleaved r,g,b) or NULL. */
RT_API int rt_render_ex(rt_context* ctx, const rt_render_params* p,
                        uint8_t* rgba_out, float* accum_out);

/* Asynchronous render into DEVICE memory (rows*width*4 bytes, 4-byte
 * aligned) on HIP stream `stream` (hipStream_t; NULL = the context's own
 * stream).  Returns after the launch; the frame counter advances.  A render
 * on a different stream than the context's previous render is ordered after
 * it on the device (stream wait on an event; no host synchronisation). */
RT_API int rt_render_device(rt_context* ctx, const rt_render_params* p,
                            void* rgba_device, void* stream);

/* The context's own HIP stream (hipStream_t), valid until rt_destroy (NULL
 * for a CPU context), created at the device's highest stream priority, so a
 * render on it dispatches ahead of work on the caller's other streams (a
 * gather of the previous frame).  Renders on it (rt_render_device with this stream or
 * NULL) record their completion event lazily — when a later call needs it:
 * a render on another stream, a state read or write, rt_synchronize — so
 * back-to-back renders carry no marker packet between them (1.5-3 us per
 * launch on MI355X).  Such a deferred event is recorded at the end of the
 * stream when the later call comes, so it also covers any work the caller
 * queued on this stream after the render (a gather, a copy): calls that wait
 * for the render wait for that work too.  A render on a caller's stream
 * records it at once (the caller may destroy that stream). */
RT_API void* rt_get_stream(rt_context* ctx);

/* Wait for all work of the context: its stream, the last render launch
 * (also on a caller's stream, rt_render_device) and the last
 * rt_deinterleave_rows_device. */
RT_API int rt_synchronize(rt_context* ctx);

/* One image across n contexts in ONE process (one context per GPU, the same
 * scene / camera / max_bounces set on each; the C++ host's multi-GPU path,
 * SURVEY §8e): context i renders rows y = i (mod n) of the frames that
 * continue its own frame counter, all contexts concurrently on their own
 * streams; the RGBA8 rows are gathered into rgba_out (host, width*height*4,
 * row 0 = bottom; may be NULL).  Keep the contexts' frame counters in step by
 * always rendering them together.  Equal to one context rendering the whole
 * image (tests/test_gpu_parity.py).  On failure every context's queued work
 * has finished when the call returns, but the contexts that did launch have
 * advanced their RNG state and frame counter while the others have not:
 * re-seed all of them (rt_init_rand) before rendering together again. */
RT_API int rt_render_multi(rt_context* const* ctxs, int n, int width, int height, int samples,
                           uint8_t* rgba_out);

/* Duration (ms, HIP events on the launch stream) of the last render kernel
 * launch; -1 when unavailable (no render yet, or kernel timing off).
 * Synchronises on that launch's end event. */
RT_API float rt_last_kernel_ms(rt_context* ctx);

/* Name of the render kernel the context's last GPU render launched, with
 * its workgroup lanes and variant, e.g. "rt_render_sorted_kernel<256,grec>+order"
 * (full frames), "rt_render_pair_kernel<128>+order" (small frames and
 * shards), "rt_render_bvh_refill_kernel<64,n16>" (BVH scenes); "" before
 * the first render and on a CPU context.  A diagnostic of the launch
 * policy (tests assert which kernel a workload runs); valid until the next
 * render on the context.  The reference launches one kernel, Main.cu:342. */
RT_API const char* rt_last_kernel_name(const rt_context* ctx);

/* Per-launch kernel timing (default on): every render records a start event
 * before its kernels; its end event (recorded either way: later calls are
 * ordered after it) closes the interval rt_last_kernel_ms reports.  Each event
 * is a marker packet the GPU drains between two launches (MI355X, config 3:
 * the start marker costs 5-7 us per launch, ~1 %; tools/ev_ab.sh,
 * profiles/r03d/launch_events/).  Off, rt_last_kernel_ms returns -1.  The
 * reference times nothing on the device (it prints host-side FPS,
 * Main.cu:486-495). */
RT_API int rt_set_kernel_timing(rt_context* ctx, int enable);

/* Number of pixel rows in the shard (row_offset, row_stride) of `height`. */
RT_API int rt_shard_rows(int height, int row_offset, int row_stride);

/* Multi-GPU gather epilogue: `gathered` holds `shards` consecutive blocks
 * of rows_per_shard*width RGBA8 pixels, block r = rows r, r+shards, ...
 * (row_stride = shards) padded to rows_per_shard.  Writes the full
 * height*width image to `image` (both device pointers) on `stream`. */
RT_API int rt_deinterleave_rows_device(rt_context* ctx, const void* gathered,
                                       void* image, int width, int height,
                                       int shards, int rows_per_shard,
                                       void* stream);

/* Checkpoint / resume of the progressive state of the current shard.
 * rng: 6*rows*width uint32 as planes (d, v0..v4), accum: 3*rows*width floats
 * interleaved r,g,b.  Either pointer may be NULL. */
RT_API int rt_get_state(rt_context* ctx, uint32_t* rng, float* accum);
RT_API int rt_set_state(rt_context* ctx, const uint32_t* rng,
                        const float* accum, unsigned frame_counter);

RT_API const char* rt_error_string(int status);
RT_API const char* rt_last_error(const rt_context* ctx);

#ifdef __cplusplus
}
#endif

#endif /* RT_ABI_H */
