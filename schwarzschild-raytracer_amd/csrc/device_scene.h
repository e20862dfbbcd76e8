// device_scene.h — the launch-invariant scene image the kernel reads with
// wave-uniform (scalar) loads. Built once per sr_set_scene / sr_set_test_ray
// by the host packer (sr_api.cpp) from the GLSL-shaped sr_scene; every derived
// value (box faces, test-ray frames, bounding spheres) is computed on the host
// with the same float operations the shader performs per call, so the kernel's
// results are bit-identical to evaluating them per step.
#ifndef SR_DEVICE_SCENE_H
#define SR_DEVICE_SCENE_H

#include <stdint.h>

#include "sr/sr.h"

#define SR_OBJ_FLOATS 120

// Record float layout (f[]):
//   [0..2] pos   [3..11] axes (column-major)
//   sphere   : [12] radius
//   plane*   : [12,13] texture_offset [14] repeat_texture [15,16] texture_size
//   disk     : plane* + [17] radius
//   hollow   : plane* + [17] inner_radius [18] outer_radius
//   rectangle: plane* + [17] width [18] height
//   cylinder : [12] height [13] radius
//   box      : [12] width [13] depth [14] height, then 6 faces (bot, top,
//              front, back, left, right; frag:649) at 16 + 14*face:
//              pos[3] c0[3] c1[3] c2[3] width height
#define SR_F_POS 0
#define SR_F_AXES 3
#define SR_F_P0 12
#define SR_F_BOX_FACE0 16
#define SR_F_FACE_STRIDE 14

// How the step loop may skip an object's exact test (never changes a result):
//   SR_KIND_EXACT  : always tested (non-finite bounds, non-orthonormal frames)
//   SR_KIND_BUDGET : held in a per-lane budget slot, skipped while the path
//                    since the slot's anchor is below its clearance (kernel:
//                    clearance / budget_step); planes by plane distance alone
//   SR_KIND_CHORD  : per-chord segment/bounding-sphere test (budget slots full)
#define SR_KIND_EXACT 0
#define SR_KIND_BUDGET 1
#define SR_KIND_CHORD 2
// Rounding margins, relative to S = |o|_1 + len + 1 of the chord:
// a planar primitive's accepted hit point lies on the chord and passes a direct
// distance test (error ~ eps * S); a quadratic's near-tangent root can wander
// ~ sqrt(eps) * |o - c| (spheres, the black hole).
#define SR_MU_PLANAR 1.0e-4f
#define SR_MU_QUADRATIC 2.0e-3f
// Cylinders: the lateral-surface quadratic's computed discriminant is the
// exact one of a radius r' with |r'^2 - r^2| <= ~12 eps (|X|^2 + r^2) for
// every chord direction (|X| <= |o - pos|: each rounding is a multiple of
// |d_perp|^2), so an accepted point lies within min(SR_CYL_QMARGIN Sc^2 / r,
// 2 SR_MU_QUADRATIC (Sc + r)) of the lateral surface, Sc = S + |pos|_1
// (tests/test_cyl_lateral_margin.py finds at most 1/25
// of it). Its root error along the chord grows as 1 / |d_perp|^2 (the
// round-2 margin divided by |d_perp|^2 for that), but moves the point along
// the surface, not off it.
#define SR_CYL_QMARGIN 4.0e-6f
// Budgeted cylinders: chords with |d_perp|^2 < SR_BUDGET_DPMIN are tested per
// chord; the budget window is capped at SR_BUDGET_TMAX of path so the
// quadratic margin can be bounded at the anchor.
#ifndef SR_BUDGET_DPMIN
#define SR_BUDGET_DPMIN 0.02f
#endif
#ifndef SR_BUDGET_TMAX
#define SR_BUDGET_TMAX 32.0f
#endif
// Objects held in per-lane budget slots (slot 0 is the black hole): every
// object of a full scene (SR_MAX_OBJECTS). The integrate kernel is
// instantiated for 6 (the default scene), 8 and all 21 slots
// (geodesic.hip sr_launch_geodesic).
#ifndef SR_MAX_BUDGET
#define SR_MAX_BUDGET SR_MAX_OBJECTS
#endif

typedef struct {
    int32_t type;
    int32_t index;
    int32_t material_index;
    int32_t kind;    // SR_KIND_*
    float bc[3];     // bounding-sphere centre
    float br;        // bounding-sphere radius + static margin (per-chord test)
    float rb;        // budget radius: br + SR_MU_QUADRATIC * (1 + |bc|_1 + br)
    float mu;        // per-chord margin factor (SR_MU_*)
    float mp;        // distance-to-primitive margin SR_MU_QUADRATIC * (1 + |pos|_1 + R), +inf: bounding sphere only
    float pl1;       // |pos|_1 (cylinder margins scale with |o - pos|)
    float f[SR_OBJ_FLOATS - 4];
} sr_dev_obj;  // 512 B

// A budget slot's object in the compact form the budget events read (slot j
// >= 1 is slots[j - 1]): one scalar-load batch instead of chains through
// budget_idx and the 512 B record. Extents x0..x2 by type:
//   rectangle: width, height, -      box: width, depth, height
//   disk: radius, -, -               hollow disk: inner, outer radius, -
//   cylinder: height, radius, -      sphere: -
typedef struct {
    int32_t type;
    int32_t cyl;     // k among the budgeted cylinders (budget_cyl_mask bit order), -1 otherwise
    float rb, mp, br, mu, pl1;  // as in sr_dev_obj
    float qk;        // cylinders: SR_CYL_QMARGIN / (radius SR_BUDGET_DPMIN), rounded away from zero
    float bc[3], x0;
    float pos[3], x1;
    float a0[3], x2;  // axes[0..2] (columns)
    float a1[3], rf;  // rf: the farthest the object's accepted points reach from the origin (outward_slot)
    float a2[3], cn;  // cn: |bc| x 1.001, rounded up (outward_clear)
} sr_dev_slot;  // 128 B

// Per-pixel state passed between the integrate / shade / resume kernels
// (geodesic.hip PS_*), floats per pixel: a 16-byte record {packed word
// (status, hit count, steps), rd[3]}, SR_PS_HITS 32-byte hit
// records {p[3], key | steps << 8, chord dir[3], -}, then planes of the
// resumable / flat-ray state (step, frag[4], ro, nv, tv, u, du). Written only
// where the next kernel reads them.
#define SR_PS_HITS 4
#define SR_PS_FIELDS (4 + 8 * SR_PS_HITS + 16)
// Texture-array opacity bitmap radius (texels), see sr_api.cpp make_opacity_map
#define SR_OPQ_RADIUS 2

// One test-ray cylinder: pos[3] axes[9] height radius, then 1 when its frame
// is orthonormal (the budget's segment refinement), padded to 16 floats.
#define SR_SEG_FLOATS 16
// Culling bounds of the curved test ray (geodesic.hip test_ray_hits_culled),
// after the segments in the same buffer: blocks of SR_TR_BLOCK consecutive
// segments, then groups of SR_TR_GROUP blocks. A bound is {centre[3], R,
// cone axis[3], cos alpha, sin alpha, max |pos|_1, always (1: no culling),
// lateral-margin scale}: every segment's accepted points lie within R of the
// centre and within the scale x lat_margin of its (frame's) lateral surface
// (sr_api.cpp frame_norms: 1 + 1e-6 for an orthonormal frame); every segment
// axis within alpha of the cone axis (unused since round 6).
#define SR_TR_BLOCK 8
#define SR_TR_GROUP 8
#define SR_TR_BLOCKS ((SR_MAX_POINTS - 1 + SR_TR_BLOCK - 1) / SR_TR_BLOCK)
#define SR_TR_GROUPS ((SR_TR_BLOCKS + SR_TR_GROUP - 1) / SR_TR_GROUP)
#define SR_TR_BOUND_FLOATS 12
#define SR_SEGS_BUF_FLOATS ((SR_MAX_POINTS - 1) * SR_SEG_FLOATS + (SR_TR_BLOCKS + SR_TR_GROUPS) * SR_TR_BOUND_FLOATS)

typedef struct {
    int32_t num_objects;
    int32_t num_lights;
    int32_t tr_visible;
    int32_t tr_num_segments;  // num_test_ray_curved_points - 1 (>= 0)
    int32_t tr_num_blocks;    // culling blocks / groups of the segments (SR_TR_BLOCK, SR_TR_GROUP)
    int32_t tr_num_groups;
    float tr_radius;
    float tr_extended_length;
    // the test ray's budget (geodesic.hip clearance_tr, round 6): the farthest
    // accepted point's distance from the origin bound (every segment's sphere
    // and the flat cylinder's ends, +inf when unbounded) and the largest
    // |pos|_1 of its cylinders
    float tr_far;
    float tr_pl1;
    // the flat cylinder's budget: {M^-1 (0, 1, 0) (its accepted points' axis
    // direction), |M^-1| (0: not budgeted), |M^-1| |M|^2 (the lateral
    // margin's scale), the axis' rounding over its length, the largest
    // lateral-margin scale of the flat cylinder and every bound, -}
    float tr_fg[8];
    int32_t num_budget;       // objects of SR_KIND_BUDGET (<= SR_MAX_BUDGET)
    int32_t budget_idx[SR_MAX_OBJECTS];  // their indices in objs[]
    int32_t budget_cyl_mask;  // bit j-1 set: budget slot j is a cylinder
    sr_dev_slot slots[SR_MAX_BUDGET];  // budget slots 1..num_budget
    int32_t num_step;         // objects of SR_KIND_EXACT / SR_KIND_CHORD (tested every step)
    int32_t step_idx[SR_MAX_OBJECTS];
    // an unbounded ray (the flat intersect, frag:895-897) from beyond this
    // radius squared that does not approach the origin misses every object
    // and the black hole (+inf: planes or unbounded objects)
    float flat_miss_r2;
    float tr_curved_color[4];
    float tr_flat_color[4];
    float tr_flat[SR_SEG_FLOATS];  // flat test-ray cylinder
    sr_dev_obj objs[SR_MAX_OBJECTS];
    sr_material materials[SR_MAX_MATERIALS];
    sr_light lights[SR_MAX_LIGHTS];
    sr_plane planes[SR_MAX_PLANES];
    float texture_sizes[SR_MAX_TEXTURES][2];
    float max_texture_size[2];
} sr_dev_scene;

// One frame's camera (Camera::loadShader, camera.cpp:41-50).
typedef struct {
    float pos[3];
    float axes[9];
    float ray_forward;  // 1 / tan(fov/360*PI), computed once on the host (frag:859)
} sr_dev_cam;

// Frames one launch renders (sr_render_blocks_batch): the same rows of
// `batch` frames that differ only in the camera.
#define SR_MAX_BATCH 32

// Per-launch constants (kernel argument, scalar-loaded).
typedef struct {
    sr_dev_cam cam[SR_MAX_BATCH];  // cam[f]: frame f of the batch
    int32_t batch;      // frames in the launch (1 .. SR_MAX_BATCH)
    int32_t tiles;      // 16x16 workgroup tiles per frame
    int64_t out_frame_stride;  // bytes between the frames' output tiles
    float max_angle;    // 2 * max_revolutions * PI (frag:860)
    float res_x, res_y; // resolution uniform == frame size
    float u_f;
    float uf_radius;    // 1 / u_f (frag:893)
    float uf_radius2;   // uf_radius * uf_radius in binary32 (sphere_intersect's r * r, frag:461)
    float percent_black;
    float curved_percentage;
    int32_t max_steps;
    int32_t raytrace_type;
    int32_t crosshair;
    int32_t filter_mode;
    int32_t cull;       // segment culling on/off (off = the reference's exhaustive loop)
    int32_t width, height;
    // output row mapping: output row k renders frame row
    //   y = row_base + (k / block_rows) * block_stride + (k % block_rows)
    int32_t nrows;
    int32_t row_base;
    int32_t block_rows;
    int32_t block_stride;
    // or, when block_list is set (sr_render_block_list): output row k renders
    //   y = block_list[k / block_rows] * block_rows + (k % block_rows), none for -1
    const int32_t* block_list;
    // optional (sr_wave_costs): per 8x8 wave of the frame, {max steps, budget
    // events} at [(f * ceil(nrows / 8) + k / 8) * ceil(width / 8) + x / 8]
    int32_t* wave_cost;
    // 1 - (max_angle / max_steps)^2 / 8, rounded down: a chord between two
    // orbit points at radii >= a stays at least a x out_dip from the origin
    float out_dip;
    // textures (RGBA8 texels)
    int32_t bg_w, bg_h;
    int32_t arr_w, arr_h, arr_layers;
    // split tiles (sr_set_split): the split_tiles costliest workgroup tiles of
    // the previous frame (max steps >= split_min_steps) run as 64 >> split_log2
    // workgroups of 2^split_log2-lane waves; 0 = off
    int32_t split_tiles;
    int32_t split_log2;
    int32_t split_min_steps;
    // 1: every chord origin lies within r = 100 (u_f >= 0.01 and the cameras
    // inside), where the black hole's u window holds (geodesic.hip SR_BH_WINDOW)
    int32_t win_ok;
    // the scene's budget slots (sr_dev_scene.num_budget): picks the integrate
    // kernel's slot capacity (geodesic.hip SR_NB_SMALL)
    int32_t num_budget;
    // the scene's budgeted cylinders (popcount of sr_dev_scene.budget_cyl_mask;
    // the small instantiation handles SR_NC_SMALL)
    int32_t num_budget_cyl;
    // 1: the test ray is visible (sr_dev_scene.tr_visible): the integrate and
    // resume kernels' test-ray instantiations, which budget it (geodesic.hip
    // clearance_tr) instead of testing every chord
    int32_t tr_visible;
    // sqrt(8 (1 - out_dip)), rounded up: at least the step angle (the budget
    // events' directional plane window, geodesic.hip plane_window)
    float max_dphi;
    // fast-loop steps per iteration of the integrate kernel:
    // SR_FAST_UNROLL_DEFAULT, or 2 in the latency mode (sr_set_latency_mode;
    // DESIGN.md §7)
    int32_t fast_unroll;
    // S_max = (sqrt 3 + 3) R + 1 (x 1.001, rounded up) for R = 1 / u_f: bounds
    // |o|_1 + len + 1 of every chord from inside the u_f sphere to within 2 R
    // (geodesic.hip budget_frame's orbital-plane exclusion); +inf when u_f <= 0
    float xplane_s;
    // the inner black-hole window's upper bounds on u (geodesic.hip
    // SR_BH_WINDOW2): out_dip / (1 + SR_BH_G2) for every lane (chords stay
    // SR_BH_G2 off the shell, above the discriminant's error at tangency),
    // and out_dip / (1 + SR_BH_G3) for steep falling lanes (E >= SR_BH_E_MIN)
    // when max_dphi <= SR_BH_S_DPHI (else bh_u2); both rounded down
    float bh_u2, bh_u3;
    // per budget slot j - 1: the orbital-plane distance of its bounding centre
    // beyond which no chord of a low-energy orbit (u < 0.6, u'^2 + u^2 (1 -
    // u) <= SR_XCYL_EMAX) can reach it (geodesic.hip SR_XCYL, sr_api.cpp
    // xlow_need); +inf: never excluded
    float xlow_need[SR_MAX_BUDGET];
    // per budget slot j - 1: the orbit energy at or below which a low-energy
    // orbit's periapsis lies beyond every chord that could reach the object
    // (geodesic.hip SR_XPERI, sr_api.cpp xperi_e); -1: never excluded
    float xperi_e[SR_MAX_BUDGET];
} sr_dev_frame;

// the orbit energy below which a cylinder's orbital-plane exclusion applies
// (under the photon orbit's 4/27: such an orbit outside the photon sphere
// stays at u <= 0.58, so |u'| <= sqrt(E) and |u''| <= 1/6 along it)
#define SR_XCYL_EMAX 0.14f

// the integrate kernel's default fast-loop steps per iteration (geodesic.hip
// SR_FAST_UNROLL)
#define SR_FAST_UNROLL_DEFAULT 4
// the largest step angle (max_angle / max_steps, here max_dphi) at which the
// low-energy exclusions apply (sr_api.cpp clear_radius): their premises (E
// conserved within 2 %, one step moving u by at most kappa, u never past the
// periapsis root) are checked on the kernel's own binary32 RK4 up to it by
// tests/test_low_energy_bounds.py (the app's MAX_STEPS 100 at up to three
// revolutions: 0.1885); coarser schedules exclude nothing
#define SR_XLOW_DPHI_MAX 0.2f

// the inner black-hole window's margins (sr_api.cpp build_frame, geodesic.hip)
#define SR_BH_G2 1.5e-3
#define SR_BH_G3 6.0e-5
#define SR_BH_S_DPHI 0.0132f
#define SR_BH_E_MIN 0.1452f
// u at r = 1 - 1e-3 and r = 1 - SR_BH_G3, rounded up: an end point past these
// (with the chord's start in the window) has certainly entered the shell
#define SR_BH_UIN2 1.00100112f
#define SR_BH_UIN3 1.00006008f

#endif
