/*
 * sr.h — C-ABI of the MI355X-native Schwarzschild geodesic renderer.
 *
 * This is the drop-in boundary that replaces the reference's GL shader-program
 * interface (Yachim/schwarzschild-raytracer):
 *
 *   reference                                              replaced by
 *   -----------------------------------------------------  -------------------------
 *   glDrawElements(full-screen quad)  src/main.cpp:318-319  sr_render / sr_render_blocks
 *   Camera::loadShader                camera.cpp:41-50      sr_camera argument
 *   ObjectLoader::load                objectLoader.cpp:27   sr_set_scene (snapshot)
 *   loadTexture(bg) + unit 0          image_utils.cpp:7-40  sr_set_background
 *   loadTextureArray + unit 1         image_utils.cpp:42    sr_set_texture_array
 *   glUniform percent_black/max_steps src/main.cpp:295-297  sr_params
 *   glUniform raytrace_type/...       src/main.cpp:394-427  sr_params
 *   test-ray uniforms (press R)       src/main.cpp:375-391  sr_set_test_ray
 *   calculateTestRayPoints            src/main.cpp:94-124   sr_test_ray_points
 *
 * The structs below are POD mirrors of the GLSL uniform block of
 * assets/shaders/black_hole.frag:15-192: same field names, same capacities.
 * Matrices are column-major 3x3 exactly as uploaded by
 * glUniformMatrix3fv(..., GL_FALSE, &m_axes[0].x) (transform.cpp:67-68):
 * axes[0..2] = column 0 (right), axes[3..5] = column 1 (up),
 * axes[6..8] = column 2 (forward).
 *
 * Conventions: extern "C", no exceptions cross the ABI, every call returns an
 * sr_status (0 = ok, < 0 = error). A context is bound to one HIP device and is
 * not thread-safe (one host thread per context), like the reference's single
 * GL context (SURVEY §8b "Threading").
 */
#ifndef SR_SR_H
#define SR_SR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Capacities — black_hole.frag:63,67,88,96,113,121,130,140,149,159,178,182 */
#define SR_MAX_LIGHTS       4
#define SR_MAX_TEXTURES     10
#define SR_MAX_MATERIALS    10
#define SR_MAX_SPHERES      3
#define SR_MAX_PLANES       3
#define SR_MAX_DISKS        3
#define SR_MAX_HOLLOW_DISKS 3
#define SR_MAX_CYLINDERS    3
#define SR_MAX_RECTANGLES   3
#define SR_MAX_BOXES        3
#define SR_MAX_OBJECTS      21
#define SR_MAX_POINTS       1000
/* max_steps limit: the integrate -> shade hand-off packs a ray's step count into 24 bits */
#define SR_MAX_STEPS        ((1 << 24) - 1)

/* Object type codes — black_hole.frag:162-171 == ObjectType (object.h:7-19) */
#define SR_OBJECT_SPHERE      0
#define SR_OBJECT_PLANE       1
#define SR_OBJECT_DISK        2
#define SR_OBJECT_HOLLOW_DISK 3
#define SR_OBJECT_CYLINDER    4 /* ObjectType::LATERAL_CYLINDER */
#define SR_OBJECT_RECTANGLE   5
#define SR_OBJECT_BOX         6

/* Raytrace modes — black_hole.frag:32-35 == RaytraceType (camera.h:14-19) */
#define SR_RAYTRACE_CURVED      0
#define SR_RAYTRACE_FLAT        1
#define SR_RAYTRACE_HALF_WIDTH  2
#define SR_RAYTRACE_HALF_HEIGHT 3

/* Bilinear filter arithmetic. The GL spec leaves the weight
 * arithmetic to the implementation; it decides whether an opaque textured hit
 * reaches alpha == 1.0 exactly (black_hole.frag:932).
 *   SR_FILTER_LERP     : lerp form, exactly 1.0 on all-opaque texels (hardware TMU-like).
 *   SR_FILTER_WEIGHTED : four-weight sum (SwiftShader-like; may give 0.99999994). */
#define SR_FILTER_LERP     0
#define SR_FILTER_WEIGHTED 1

typedef enum {
    SR_OK = 0,
    SR_E_INVALID = -1,   /* bad argument (null pointer, bad size, bad mode) */
    SR_E_CAPACITY = -2,  /* more objects/lights/... than the GLSL arrays hold */
    SR_E_HIP = -3,       /* a HIP runtime call failed */
    SR_E_NOMEM = -4,     /* host or device allocation failed */
    SR_E_NOT_READY = -5, /* sr_render before sr_set_scene */
    SR_E_NO_DEVICE = -6, /* no HIP device / bad device ordinal */
    SR_E_IO = -7         /* a file could not be written (sr_write_png) */
} sr_status;

/* struct Transform — black_hole.frag:41-44 */
typedef struct {
    float pos[3];
    float axes[9]; /* column-major: right, up, forward */
} sr_transform;

/* struct Camera — black_hole.frag:46-49 (fov: horizontal, degrees) */
typedef struct {
    sr_transform transform;
    float fov;
} sr_camera;

/* struct Light — black_hole.frag:54-61 */
typedef struct {
    sr_transform transform;
    float color[3];
    float intensity;
    float attenuation_constant;
    float attenuation_linear;
    float attenuation_quadratic;
} sr_light;

/* struct Material — black_hole.frag:72-86 (bools as int32) */
typedef struct {
    float color[4];
    float ambient;
    float diffuse;
    float specular;
    float shininess;
    int32_t texture_index;    /* < 0 disables */
    int32_t normal_map_index; /* < 0 disables */
    int32_t invert_uv_x;
    int32_t invert_uv_y;
    int32_t swap_uvs;
    int32_t double_sided_normals;
    int32_t flip_normals;
} sr_material;

/* struct Sphere — black_hole.frag:91-94 */
typedef struct {
    sr_transform transform;
    float radius;
} sr_sphere;

/* struct Plane — black_hole.frag:106-111 */
typedef struct {
    sr_transform transform;
    float texture_offset[2];
    int32_t repeat_texture;
    float texture_size[2];
} sr_plane;

/* struct Disk — black_hole.frag:116-119 */
typedef struct {
    sr_plane plane;
    float radius;
} sr_disk;

/* struct HollowDisk — black_hole.frag:124-128 */
typedef struct {
    sr_plane plane;
    float inner_radius;
    float outer_radius;
} sr_hollow_disk;

/* struct Cylinder (lateral surface only) — black_hole.frag:134-138 */
typedef struct {
    sr_transform transform;
    float height;
    float radius;
} sr_cylinder;

/* struct Rectangle — black_hole.frag:143-147 */
typedef struct {
    sr_plane plane;
    float width;
    float height;
} sr_rectangle;

/* struct Box — black_hole.frag:152-157 */
typedef struct {
    sr_transform transform;
    float width;
    float depth;
    float height;
} sr_box;

/* struct Object — black_hole.frag:172-176 */
typedef struct {
    int32_t type;
    int32_t index;          /* into the per-type array */
    int32_t material_index; /* into materials[]; ObjectLoader starts at 1 */
} sr_object;

/* The scene half of the uniform block (what ObjectLoader::load and
 * loadTextureArray upload once): black_hole.frag:64-65, 68-69, 89, 97-160,
 * 179-180. */
typedef struct {
    int32_t num_objects;
    sr_object objects[SR_MAX_OBJECTS];
    sr_sphere spheres[SR_MAX_SPHERES];
    sr_plane planes[SR_MAX_PLANES];
    sr_disk disks[SR_MAX_DISKS];
    sr_hollow_disk hollow_disks[SR_MAX_HOLLOW_DISKS];
    sr_cylinder cylinders[SR_MAX_CYLINDERS];
    sr_rectangle rectangles[SR_MAX_RECTANGLES];
    sr_box boxes[SR_MAX_BOXES];
    sr_material materials[SR_MAX_MATERIALS];
    int32_t num_lights;
    sr_light lights[SR_MAX_LIGHTS];
    float texture_sizes[SR_MAX_TEXTURES][2];
    float max_texture_size[2];
} sr_scene;

/* Per-frame parameters: black_hole.frag:15-39 uniforms. Defaults (sr_params_default)
 * are the shader's initializers, with max_revolutions = 2 (the app's glUniform1f
 * upload into an int uniform is rejected, src/main.cpp:297). */
typedef struct {
    int32_t max_steps;          /* frag:19 */
    int32_t max_revolutions;    /* frag:20 */
    float u_f;                  /* frag:22 */
    int32_t crosshair;          /* frag:24 */
    int32_t raytrace_type;      /* frag:36 */
    float curved_percentage;    /* frag:37 */
    float percent_black;        /* frag:39; < 0 disables the noise mask */
    float time;                 /* frag:16 (declared, unused by the shader) */
    int32_t filter_mode;        /* SR_FILTER_* (texture() arithmetic) */
} sr_params;

/* Test-ray overlay uniforms: black_hole.frag:182-192 (set on key R, src/main.cpp:375-391). */
typedef struct {
    int32_t visible;                  /* test_ray_visible */
    float radius;                     /* test_ray_radius (0.025) */
    float extended_length;            /* test_ray_extended_length (1000) */
    float curved_color[4];            /* (1,0,0,1) */
    float flat_color[4];              /* (0,1,0,1) */
    float flat_origin[3];
    float flat_dir[3];
    int32_t num_curved_points;
    float curved_points[SR_MAX_POINTS][3];
} sr_test_ray;

typedef struct sr_ctx sr_ctx;
typedef struct ihipStream_t* sr_stream; /* == hipStream_t; NULL = default stream */

/* Library / defaults -------------------------------------------------------- */
const char* sr_version(void);
const char* sr_status_string(int status);
void sr_params_default(sr_params* out);
void sr_test_ray_default(sr_test_ray* out);
void sr_scene_clear(sr_scene* out);
/* The app's hard-coded scene and camera (src/main.cpp:222-268), textures
 * described by texture_sizes (uv_checker 600x600, cubemap 1601x1201). */
void sr_default_scene(sr_scene* out);
void sr_default_camera(sr_camera* out);
/* The app's H-key flyby (src/main.cpp:404-410 -> Camera::hyperbolicTrajectory,
 * camera.cpp:20-33, then lookAt(origin), camera.cpp:35-39): moves *cam along
 * the hyperbola of the given initial / closest distance at eased time t in
 * [0, 1] (the app: 30, 10, elapsed / HYPERBOLIC_TRAJECTORY_DURATION). The fov
 * is kept. Host-only, per frame. */
int sr_camera_hyperbolic_trajectory(sr_camera* cam, float initial_distance, float closest_distance,
                                    float time);

/* Context ------------------------------------------------------------------- */
int sr_create(sr_ctx** out, int hip_device);
void sr_destroy(sr_ctx* ctx);

/* Skybox: already flipped as stbi_set_flip_vertically_on_load(true) leaves it
 * (row 0 = v 0). channels 3 (GL_RGB: alpha reads 1) or 4. Synchronous copy. */
int sr_set_background(sr_ctx* ctx, const uint8_t* pixels, int width, int height, int channels);
/* Texture array image exactly as glTexImage3D receives it (already padded to the
 * max size; layer-major, rows bottom-up). channels 3 or 4. */
int sr_set_texture_array(sr_ctx* ctx, const uint8_t* pixels, int width, int height,
                         int layers, int channels);
/* Snapshot copy of the scene (ObjectLoader::load semantics). Validates types,
 * per-type indices and material indices: SR_E_CAPACITY instead of the
 * reference's silent glUniform drop. */
int sr_set_scene(sr_ctx* ctx, const sr_scene* scene);
int sr_set_test_ray(sr_ctx* ctx, const sr_test_ray* test_ray);

/* Render rows [row_begin, row_end) of a width x height frame (GL order: row 0
 * is the bottom row) into dev_rgba8 (device memory, row r at
 * dev_rgba8 + (r - row_begin) * pitch_bytes). Asynchronous on `stream`.
 * A context reuses its per-frame scratch (pixel state, launch order), so its
 * renders are ordered: a launch on another stream than the context's last
 * one first waits (hipStreamWaitEvent on an event recorded at the end of that
 * launch) for the work of that stream. Between launches the context frees
 * replaced buffers in stream order on its last launch's stream, and the calls
 * that wait for the context's frames (sr_set_*, sr_wave_costs, sr_destroy)
 * synchronise it: keep that stream alive until the context's next launch (on
 * any stream) or sr_destroy. */
int sr_render(sr_ctx* ctx, const sr_camera* cam, const sr_params* params, int width,
              int height, int row_begin, int row_end, uint8_t* dev_rgba8,
              size_t pitch_bytes, sr_stream stream);

/* Block-cyclic row bands for multi-GPU tiling: frame rows are cut in blocks of
 * `block_rows`; this call renders blocks b = block_first + k*block_step
 * (k = 0, 1, ...) and packs them densely: block k's row j lands at
 * dev_rgba8 + (k*block_rows + j) * pitch_bytes. */
int sr_render_blocks(sr_ctx* ctx, const sr_camera* cam, const sr_params* params, int width,
                     int height, int block_rows, int block_first, int block_step,
                     uint8_t* dev_rgba8, size_t pitch_bytes, sr_stream stream);

/* Frames in one launch (not in the reference; the pixels are unchanged): the
 * rows sr_render_blocks would render, for n_frames (1 .. 32) frames that
 * differ only in the camera (cams[f]), frame f packed at dev_rgba8 + f *
 * frame_stride_bytes. One launch carries n_frames times the work, so a GPU
 * holding a small share of each frame (multi-GPU row tiling) runs it as
 * efficiently as a whole frame; the launch order and split tiles follow the
 * costliest tiles over the batch. SR_E_CAPACITY above 32 frames. */
int sr_render_blocks_batch(sr_ctx* ctx, const sr_camera* cams, int n_frames, const sr_params* params,
                           int width, int height, int block_rows, int block_first, int block_step,
                           uint8_t* dev_rgba8, size_t pitch_bytes, size_t frame_stride_bytes, sr_stream stream);

/* A rank's cost-balanced rows (not in the reference; the pixels are
 * unchanged): like sr_render_blocks_batch, but output row k of each frame's
 * tile renders frame row blocks[k / block_rows] * block_rows + k % block_rows
 * for an explicit list of n_blocks block indices (-1: padding, rows left
 * unwritten). The list is copied to the device once per distinct list and
 * kept with the context. schwarzschild-raytracer_amd/dist.py balanced_blocks
 * builds equal-length lists of about equal cost for the ranks of a node. */
int sr_render_block_list(sr_ctx* ctx, const sr_camera* cams, int n_frames, const sr_params* params, int width,
                         int height, int block_rows, const int* blocks, int n_blocks, uint8_t* dev_rgba8,
                         size_t pitch_bytes, size_t frame_stride_bytes, sr_stream stream);

/* Per-wave cost map of one whole frame (not in the reference), for
 * cost-balanced multi-GPU shares: renders the frame (no image output, split
 * tiles off for this launch) and writes, for each 8x8 wave tile (row block
 * b = y / 8, column c = x / 8), dev_out[(b * ceil(width / 8) + c) * 2] = the
 * wave's longest ray's executed steps and [... + 1] = its budget events
 * (DESIGN.md §5): int32 [ceil(height / 8)][ceil(width / 8)][2]. Deterministic,
 * so every rank of a node derives the same block lists from it. */
int sr_wave_costs(sr_ctx* ctx, const sr_camera* cam, const sr_params* params, int width, int height,
                  int32_t* dev_out, sr_stream stream);

/* ---- Multi-GPU frame partition (not in the reference, whose frame is one
 * draw on one GPU, src/main.cpp:318-319). A frame's rows are cut
 * into blocks of block_rows (8: one 8x8 wave tile tall); every rank of a node
 * renders an equal-length list of blocks of about equal cost with
 * sr_render_block_list, the tiles are gathered to the root (the caller's
 * RCCL collective: ncclGather of equal-size tiles, examples/sr_multi_gpu.cpp)
 * and sr_assemble_blocks puts the frame back together. */

/* Per-block cost from an sr_wave_costs map copied to the host
 * ([n_blocks][waves_per_block][2] = {steps, events} per 8x8 wave): out_cost[b]
 * = sum over the block's waves of steps + event_steps x events (a wave runs
 * until its longest ray ends; a budget event costs about 8 wave-steps,
 * DESIGN.md §8). Same values as dist.block_costs. */
int sr_block_costs(const int32_t* wave_cost, int n_blocks, int waves_per_block, double event_steps,
                   double* out_cost);

/* Equal-length block lists of about equal cost for `world` ranks:
 * out_lists[r * per + s] (-1: padding), *out_per = ceil(n_blocks / world);
 * SR_E_CAPACITY when world * per > max_entries. Blocks by descending cost to
 * the least-loaded rank with room, then pairwise swaps out of the most
 * loaded rank while one lowers the pair's maximum; the block-cyclic lists
 * when they are at least as even. Deterministic, binary64, the same lists as
 * dist.balanced_blocks: every rank derives identical lists from identical
 * costs (or the root computes and broadcasts them). */
int sr_balanced_blocks(const double* cost, int n_blocks, int world, int* out_lists, int max_entries, int* out_per);

/* Reassembles n_frames frames from gathered tiles: rank r's tile of frame f
 * starts at stacked + r * rank_stride + f * in_frame_stride, its slot s holds
 * the block_rows rows of frame block lists[r * per + s] (dense rows of
 * row_bytes); frame f's row y lands at out + f * out_frame_stride + y *
 * row_bytes (rows >= height dropped, -1 slots skipped). on_device != 0: every
 * pointer, `lists` included, is device memory and the copy is a kernel on
 * `stream` (asynchronous); 0: host memory, synchronous. */
int sr_assemble_blocks(const uint8_t* stacked, size_t rank_stride, size_t in_frame_stride, const int* lists,
                       int world, int per, int height, int block_rows, size_t row_bytes, uint8_t* out,
                       size_t out_frame_stride, int n_frames, int on_device, sr_stream stream);

/* Debug/parity variant: unclamped FragColor as float RGBA (dev_rgba32, may be
 * NULL), the RGBA8 pixel (dev_rgba8, may be NULL) and the number of executed
 * geodesic steps per pixel (dev_steps, may be NULL). Dense rows. */
int sr_render_debug(sr_ctx* ctx, const sr_camera* cam, const sr_params* params, int width,
                    int height, int row_begin, int row_end, float* dev_rgba32,
                    uint8_t* dev_rgba8, int32_t* dev_steps, sr_stream stream);

/* Split tiles (not in the reference; a latency knob, the pixels are unchanged):
 * the next frames run the max_tiles costliest 16x16 workgroup tiles of the
 * previous frame on this context whose longest ray took at least min_steps
 * steps as waves of lanes_per_wave (16, 4 or 1) rays instead of 64. A wave's
 * budget events are the union of its rays' events, so the frame's longest
 * rays finish sooner in sparse waves, at the cost of more waves for those
 * tiles. max_tiles 0 (the default) turns it off. For one
 * headline frame at a time (1920x1080, 2000 steps) sr_set_split(ctx, 32, 16,
 * 1200) measured 1.148 ms against 1.163 ms without (profiles/r04/s16), and
 * 1.067-1.075 ms against 1.106-1.116 ms timed round robin (profiles/r04/s24). */
int sr_set_split(sr_ctx* ctx, int max_tiles, int lanes_per_wave, int min_steps);

/* Latency mode (not in the reference; the pixels are unchanged): on != 0 runs
 * the next frames' step loop with two fast-loop steps per iteration instead of
 * three: one frame alone finishes sooner (its longest rays' dependency
 * chain: 1.277 -> 1.128 ms in profiles/r04/s8_split_sweep.jsonl), frames in
 * flight run ~2 % slower. For an interactive caller that draws one frame at
 * a time (src/main.cpp:318-319) without split tiles: with them it measured
 * slower than split tiles alone. Off by default. */
int sr_set_latency_mode(sr_ctx* ctx, int on);

/* Rows a sr_render_blocks call with these arguments writes. */
int sr_blocks_row_count(int height, int block_rows, int block_first, int block_step);

/* Runtime invariant counters of a context (not in the reference), after its
 * launched frames are done: out[0] = pixels the shade kernel found stopped at
 * a hit classified opaque in the step loop whose shaded alpha was not 1 (the
 * classification is exact where it claims, DESIGN.md §5, so this stays 0; a
 * non-zero count means such rays were written without the rest of their
 * path), out[1] = stream-ordered frees (hipFreeAsync) that failed (a leak).
 * Writes min(n, 2) counters. */
int sr_diag_counters(sr_ctx* ctx, int64_t* out, int n);

/* sizeof of the ABI structs, for binding checks: sr_camera, sr_params,
 * sr_scene, sr_test_ray, sr_material, sr_light (in that order). */
int sr_abi_struct_sizes(size_t* out, int n);

/* Presentation (not in the hot path): writes a frame in host memory as an
 * RGBA8 PNG. Replaces the reference's window present (src/main.cpp:318-319
 * draw, :432 glfwSwapBuffers) for offline use. Rows are read bottom-up as GL
 * and sr_render leave them when flip_rows != 0 (row 0 = the image's bottom).
 * SR_E_IO when the file cannot be written. */
int sr_write_png(const char* path, const uint8_t* rgba8, int width, int height, size_t pitch_bytes,
                 int flip_rows);

/* Host-side press-R geodesic (src/main.cpp:94-124): writes up to max_points
 * xyz triples into out_xyz and the count into *out_count. */
int sr_test_ray_points(const float cam_pos[3], const float cam_forward[3], int max_steps,
                       int max_revolutions, float* out_xyz, int max_points, int* out_count);

#ifdef __cplusplus
}
#endif

#endif /* SR_SR_H */
