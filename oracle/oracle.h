/*
 * oracle.h — CPU restatement of the reference path tracer (TEST
 * INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline — never as the
 * thing measured or shipped.  The product (libbwrt.so) does not link it and
 * has no CPU fallback.
 *
 * Parity pinning: the reference cannot be built here
 * (its kernel needs CUDA headers — cuda_runtime.h, curand_kernel.h,
 * host_defines.h — that the image lacks), so this restatement is pinned by
 * the reference's own rendered outputs: Renders/01_red_circle.png (disc
 * geometry) and Renders/07_specular_BRDF.png (converged image, block means),
 * through fixtures under tests/golden/.  The exact cuRAND stream and the
 * nvcc --use_fast_math transcendentals are NOT pinnable (parity unpinned for
 * those two aspects; statistical parity only).
 */
#ifndef BWRT_ORACLE_H
#define BWRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* WorldTypes.cuh / Math.cuh layouts (same bytes as include/rt_abi.h). */
typedef struct { float x, y, z; } orc_vec3;
typedef struct { orc_vec3 albedo; float emittance, roughness, refractive_index; } orc_material;
typedef struct { orc_vec3 position; float radius; orc_material mat; } orc_sphere;
typedef struct { orc_vec3 origin; orc_vec3 directions[2]; orc_material mat; } orc_plane;
typedef struct { orc_vec3 vertices[3]; orc_material mat; } orc_triangle;
typedef struct { orc_vec3 vertices[4]; orc_material mat; } orc_quad;
typedef struct { orc_vec3 position; float angle[2]; float fov; } orc_camera;
typedef struct {
    orc_camera camera;
    const orc_sphere* spheres;   int sphere_count;
    const orc_plane* planes;     int plane_count;
    const orc_triangle* triangles; int triangle_count;
    const orc_quad* quads;       int quad_count;
} orc_scene;

/* cuRAND XORWOW restated (CUDA 12.0 curand_kernel.h, external dependency,
 * not in /root/reference).  state = {d, v0, v1, v2, v3, v4}. */
void orc_curand_init(unsigned long long seed, uint32_t state[6]);
uint32_t orc_curand(uint32_t state[6]);

/* Transcendentals used on the path (Main.cu:175-182): single-precision
 * Cody-Waite + minimax approximations, specified in DESIGN.md; the product
 * kernel implements the same operation sequence. */
float orc_atanf(float x);
float orc_sinf(float x);
float orc_cosf(float x);

/* Render `passes` progressive frames (frame numbers first_frame ..
 * first_frame+passes-1) for the shard rows y = row_offset + j*row_stride,
 * j < rows.  State arrays are per shard pixel p = j*width + x:
 *   rng:   6 planes of rows*width uint32 (d, v0..v4)
 *   accum: rows*width*3 floats (frameSum, interleaved)
 *   rgba:  rows*width*4 bytes (may be NULL)
 * If init_rng != 0 the RNG is seeded first with curand_init(y*W+x,0,0).
 * threads <= 0 uses the OpenMP default.  Returns 0 or -1 on bad arguments. */
int orc_render_rows(const orc_scene* scene, int width, int height,
                    int row_offset, int row_stride, int rows,
                    unsigned first_frame, int passes, int max_bounces,
                    uint32_t* rng, float* accum, uint8_t* rgba,
                    int init_rng, int threads);

/* backgroundColor (Main.cu:27; {0,0,0} in the reference build) used by the
 * next orc_render_rows calls. */
void orc_set_background(float r, float g, float b);

/* samplesPerPixel (Main.cu:27; 1 in the reference build): the in-frame loop
 * of Main.cu:296-299 traces that many paths from the frame's one jittered
 * camera ray, keeps the LAST (assignment, not a sum) and scales it by
 * 1/samplesPerPixel.  Used by the next orc_render_rows calls. */
void orc_set_samples_per_pixel(int n);

/* Work counters of the last orc_render_rows call (closest-hit queries and
 * paths), for the measured work profile in DESIGN.md. */
void orc_last_counters(unsigned long long* queries, unsigned long long* paths);

#ifdef __cplusplus
}
#endif

#endif
