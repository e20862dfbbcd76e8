/*
 * sr_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's per-pixel hot path
 * (assets/shaders/black_hole.frag:208-936) and of the press-R CPU geodesic
 * (src/main.cpp:73-124). It is the checker for the HIP kernel and the
 * `cpu_baseline` leg of bench.py; the product (libsr.so) never links, loads or
 * calls it. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * may use it.
 *
 * Pinning: the restatement is checked against golden RGBA8 frames rendered by
 * the reference shader itself on SwiftShader in the build container
 * (tests/golden/make_golden.py), within the tolerance budget stated in
 * tests/test_oracle_golden.py. See DESIGN.md §3.
 *
 * Arithmetic contract (shared with the kernel):
 *   - IEEE binary32 everywhere, no FMA contraction, GLSL left-to-right order;
 *   - division and sqrt correctly rounded;
 *   - sin/cos/tan/atan2/asin/pow: the binary64 function rounded to binary32;
 *   - normalize(v) = v * (1 / sqrt(dot(v, v))).
 */
#ifndef SR_ORACLE_H
#define SR_ORACLE_H

#include <stdint.h>
#include "../include/sr/sr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* params->filter_mode of the oracle only (test infrastructure): SwiftShader
 * 4.1's fixed-point RGBA8 sampler (sr_oracle.c sample_swiftshader), the
 * filter the golden renders ran with. The library accepts SR_FILTER_LERP and
 * SR_FILTER_WEIGHTED only. */
#define SRO_FILTER_SWIFTSHADER 2

typedef struct {
    const uint8_t* bg; /* skybox, rows bottom-up, NULL = incomplete texture */
    int bg_w, bg_h, bg_channels;
    const uint8_t* arr; /* texture array, layer-major, rows bottom-up */
    int arr_w, arr_h, arr_layers, arr_channels;
} sro_textures;

/* Render rows [row_begin, row_end) of a width x height frame. Any of the
 * output pointers may be NULL. Dense rows. nthreads <= 0: all cores. */
int sro_render(const sr_scene* scene, const sr_test_ray* test_ray, const sro_textures* tex,
               const sr_camera* cam, const sr_params* params, int width, int height,
               int row_begin, int row_end, uint8_t* rgba8, float* rgba32, int32_t* steps,
               int nthreads);

/* One texture() lookup of the oracle's sampler (GL_LINEAR + GL_REPEAT) on
 * one RGBA8 / RGB8 image (rows bottom-up), mode SR_FILTER_* or
 * SRO_FILTER_SWIFTSHADER. 0, or -1 on bad arguments. */
int sro_sample_texture(const uint8_t* base, int width, int height, int channels, float u, float v, int mode,
                       float out_rgba[4]);

/* One pixel (px, py), GL order. Returns the number of executed steps. */
int sro_shade_pixel(const sr_scene* scene, const sr_test_ray* test_ray, const sro_textures* tex,
                    const sr_camera* cam, const sr_params* params, int width, int height,
                    int px, int py, float out_rgba[4]);

/* press-R test ray: src/main.cpp:94-124 with MAX_STEPS/MAX_REVOLUTIONS as
 * arguments. Returns the point count (<= max_points written). */
int sro_test_ray_points(const float pos[3], const float forward[3], int max_steps,
                        int max_revolutions, float* out_xyz, int max_points);

/* CPU baseline: the press-R loop swept over the pixels of
 * rows [row_begin, row_end) of a width x height frame, dir = the shader's
 * camera ray of that pixel (frag:859-863), one growable point vector per ray.
 * Returns the total number of points (a checksum of the work). */
int64_t sro_pressr_sweep(const sr_camera* cam, int width, int height, int row_begin,
                         int row_end, int max_steps, int max_revolutions, int nthreads);

#ifdef __cplusplus
}
#endif

#endif
