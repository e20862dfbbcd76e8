// sr_api.cpp — the C-ABI of include/sr/sr.h: device context, texture and
// scene uploads, launch-invariant precomputation, and kernel dispatch.
// Replaces the reference's GL program interface: the draw call of
// src/main.cpp:318-319 becomes sr_render, the loadShader uniform uploads
// become sr_set_scene / sr_set_test_ray snapshots.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <tuple>
#include <utility>
#include <vector>

#include "device_scene.h"
#include "sr/sr.h"

// Round 6: budgeted cylinders take the lateral margin SR_CYL_QMARGIN Sc^2 / r
// for every chord direction (0: the round-2 margin over SR_BUDGET_DPMIN, and
// the kernel's direction tests and slab budgets for nearly parallel chords)
#ifndef SR_CYL_DIRFREE
#define SR_CYL_DIRFREE 1
#endif

extern "C" hipError_t sr_launch_geodesic(const sr_dev_scene* sc, const float4* tbl, const float* segs,
                                         const uint32_t* bg, const uint32_t* arr, const uint8_t* opq,
                                         const sr_dev_frame* fr,
                                         uint8_t* out, size_t pitch, float* dbg_rgba, int32_t* dbg_steps,
                                         float* ps, size_t ps_n, int* list, int* count, int* order, int* cost,
                                         int* diag, hipEvent_t* ev4, hipStream_t stream);

namespace {

constexpr float kPi = 3.1415926535f;  // frag:10

struct Table {
    float4* dev = nullptr;
    int steps = 0;
    std::vector<float4> host;  // source of the stream-ordered upload, kept until the entry goes
    uint64_t used = 0;
};

// Device caches of a context (step tables, launch orders, block lists) hold at
// most this many entries each; the least recently used goes, its buffers
// freed in stream order after the context's in-flight frames.
constexpr size_t kCacheEntries = 8;

}  // namespace

struct sr_ctx {
    int device = 0;
    sr_dev_scene* d_scene = nullptr;
    float* d_segs = nullptr;
    uint32_t* d_bg = nullptr;
    int bg_w = 0, bg_h = 0;
    uint32_t* d_arr = nullptr;
    int arr_w = 0, arr_h = 0, arr_layers = 0;
    uint8_t* d_opq = nullptr;  // texture-array opacity bitmap (make_opacity_map)
    bool scene_set = false;
    bool cull = true;
    sr_dev_scene h_scene;
    // xlow_need's and xperi_e's last inputs and results (build_frame; cleared by sr_set_scene)
    float xc_uf = NAN, xc_dphi = NAN;
    float xc_need[SR_MAX_BUDGET];
    float xc_peri[SR_MAX_BUDGET];
    // pixel pipeline scratch (geodesic.hip): SR_PS_FIELDS planes of ps_n floats,
    // the resume worklist and its counter; grown on demand, reused per frame.
    // Renders on one context are ordered on its stream(s) by the caller.
    float* d_ps = nullptr;
    int* d_list = nullptr;
    int* d_count = nullptr;
    size_t ps_n = 0;
    // workgroup-tile launch order (costliest first) and per-tile cost of the
    // last frame, one pair per grid shape (geodesic.hip order_tiles): kept
    // for the context's lifetime, so a shape change never frees a buffer an
    // in-flight frame still reads
    struct Order {
        int* order = nullptr;
        int* cost = nullptr;
        std::vector<int> host;  // source of the stream-ordered upload
        uint64_t used = 0;
    };
    // (gx, gy, split_tiles, split_log2, block list): a block list's tiles have
    // their own costs; the list is its device copy, one per distinct content
    std::map<std::tuple<int, int, int, int, const int*>, Order> orders;
    // device copies of the block lists of sr_render_block_list, by content
    // (the key is the upload's source)
    struct BlockList {
        int* dev = nullptr;
        uint64_t used = 0;
    };
    std::map<std::vector<int>, BlockList> block_lists;
    uint64_t tick = 0;  // LRU clock of the caches
    // synchronous uploads (sr_set_*) run on this non-blocking stream, never
    // on the null stream (which would wait for other contexts' work)
    hipStream_t upload = nullptr;
    // split tiles (sr_set_split): 0 = off
    int split_tiles = 0, split_log2 = 4, split_min_steps = 1;
    int fast_unroll = SR_FAST_UNROLL_DEFAULT;  // sr_set_latency_mode: 2
    const int* last_order = nullptr;  // the launch codes of the context's last frame (its next frame's order)
    size_t last_slots = 0;
    // the stream of the context's last launch: a context is used from one
    // stream, so waiting for it waits for every frame that
    // may still read the context's buffers, and for nothing else on the device
    hipStream_t last_stream = nullptr;
    bool launched = false;
    // a launch on another stream than the last one first waits for it (this
    // event, recorded on the old stream): the context's scratch and the
    // stream-ordered frees on last_stream stay ordered after every launch
    hipEvent_t order_ev = nullptr;
    // stream-ordered frees whose hipFreeAsync failed (sr_diag_counters)
    int64_t free_errors = 0;
    // device counter of the shade kernel's invariant check (sr_diag_counters)
    int* d_diag = nullptr;
    // optional per-kernel timing: 4 events per frame (before integrate, after
    // integrate, after shade, after resume), a ring of `timing_cap` frames
    std::vector<hipEvent_t> tev;
    int timing_cap = 0;
    int timing_n = 0;
    std::map<std::pair<int, int>, Table> tables;  // (max_steps, max_revolutions) -> table
};

namespace {

// ---- small float helpers with the kernel's evaluation order ----------------
struct V3 {
    float x, y, z;
};
inline V3 v3(float x, float y, float z) { return {x, y, z}; }
inline V3 ld(const float* p) { return {p[0], p[1], p[2]}; }
inline void st(float* p, V3 v) {
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 scl(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float len(V3 a) { return std::sqrt(dot(a, a)); }
inline V3 nrm(V3 a) { return scl(a, 1.0f / std::sqrt(dot(a, a))); }
// columns c0, c1, c2: (c0*v.x + c1*v.y) + c2*v.z
inline V3 mv(V3 c0, V3 c1, V3 c2, V3 v) { return add(add(scl(c0, v.x), scl(c1, v.y)), scl(c2, v.z)); }
inline float l1norm(V3 a) { return std::fabs(a.x) + std::fabs(a.y) + std::fabs(a.z); }

bool orthonormal(V3 a, V3 b, V3 c) {
    const float tol = 1e-5f;
    return std::fabs(dot(a, a) - 1.f) < tol && std::fabs(dot(b, b) - 1.f) < tol &&
           std::fabs(dot(c, c) - 1.f) < tol && std::fabs(dot(a, b)) < tol &&
           std::fabs(dot(a, c)) < tol && std::fabs(dot(b, c)) < tol;
}

// Bounding sphere (c, R) of everything the object's exact test can accept.
void set_bound(sr_dev_obj& o, V3 c, float R, int kind, float mu) {
    if (!std::isfinite(R) || !std::isfinite(c.x) || !std::isfinite(c.y) || !std::isfinite(c.z)) {
        o.kind = SR_KIND_EXACT;
        return;
    }
    st(o.bc, c);
    o.br = R + mu * (1.f + l1norm(c) + R);
    o.rb = R + SR_MU_QUADRATIC * (1.f + l1norm(c) + R);
    o.mu = mu;
    o.kind = kind;
    // distance-to-primitive clearance (kernel clearance()): disks need a unit
    // normal axes[1]; rectangles, boxes and cylinders are only budgeted with an
    // orthonormal frame. Margin for the primitives' in-plane / height / radius
    // tests, relative to their magnitudes.
    V3 n = ld(o.f + SR_F_AXES + 3);
    bool typed = o.type == SR_OBJECT_DISK || o.type == SR_OBJECT_HOLLOW_DISK || o.type == SR_OBJECT_RECTANGLE ||
                 o.type == SR_OBJECT_BOX || o.type == SR_OBJECT_CYLINDER;
    // Planar primitives (disks, annuli, rectangles, box faces) accept a point
    // of the chord within a few eps S of the plane and of their in-plane
    // bounds, so their per-chord factor (SR_MU_PLANAR, ~100x that) serves
    // here too; the cylinder's height and radius keep the quadratic one.
    const float md = o.type == SR_OBJECT_CYLINDER ? SR_MU_QUADRATIC : mu;
    o.mp = typed && std::fabs(dot(n, n) - 1.f) < 1e-5f ? md * (1.f + l1norm(ld(o.f + SR_F_POS)) + R) : INFINITY;
    o.pl1 = l1norm(ld(o.f + SR_F_POS));
}

// The accepted region of rect_test (frag:573-584) for a frame that need not
// be orthonormal: the points pos + q with c1 . q = 0 (the plane through pos
// with normal c1), 0 <= c0 . q <= w and 0 <= c2 . q <= h, a parallelogram
// with the corners q = M^-1 (alpha, 0, beta) for M's rows c0, c1, c2.
// Appends its corners (binary64); kappa = |M|_F |M^-1|_F >= the condition
// number, which scales the rounding of an accepted point's position. False
// for a singular or non-finite frame.
bool parallelogram_corners(V3 pos, V3 c0, V3 c1, V3 c2, float w, float h, std::vector<std::array<double, 3>>& out,
                           double& kappa) {
    const double m[3][3] = {{c0.x, c0.y, c0.z}, {c1.x, c1.y, c1.z}, {c2.x, c2.y, c2.z}};
    const double det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
                       m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                       m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    if (!std::isfinite(det) || std::fabs(det) < 1e-6 || !(w >= 0.f) || !(h >= 0.f)) return false;
    double inv[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const int i1 = (j + 1) % 3, i2 = (j + 2) % 3, j1 = (i + 1) % 3, j2 = (i + 2) % 3;
            inv[i][j] = (m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1]) / det;  // adjugate / det
        }
    double fm = 0, fi = 0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            fm += m[i][j] * m[i][j];
            fi += inv[i][j] * inv[i][j];
        }
    kappa = std::sqrt(fm * fi);
    for (int k = 0; k < 4; k++) {
        const double al = (k & 1) ? w : 0.0, be = (k & 2) ? h : 0.0;  // M q = (al, 0, be)
        std::array<double, 3> q;
        for (int i = 0; i < 3; i++) q[i] = (double)(&pos.x)[i] + inv[i][0] * al + inv[i][2] * be;
        out.push_back(q);
    }
    return std::isfinite(kappa);
}

// Bounding sphere of a non-orthonormal rectangle's or box's accepted region
// (the parallelograms of its faces): budgeted like an orthonormal one but by
// that sphere alone (mp = +inf: no distance-to-primitive refinement, no
// directional plane window), its planar margin factor scaled by the frame's
// condition number. A scene with such an object no longer tests every chord
// exactly (round 6: the max-capacity scene's skewed rectangle had turned
// lazy chords off for the whole frame).
bool set_bound_corners(sr_dev_obj& o, const std::vector<std::array<double, 3>>& pts, double kappa) {
    if (pts.empty() || !(kappa < 1e3)) return false;
    double c[3] = {0, 0, 0};
    for (const auto& q : pts)
        for (int i = 0; i < 3; i++) c[i] += q[i] / (double)pts.size();
    double R = 0;
    for (const auto& q : pts)
        R = std::max(R, std::sqrt((q[0] - c[0]) * (q[0] - c[0]) + (q[1] - c[1]) * (q[1] - c[1]) +
                                  (q[2] - c[2]) * (q[2] - c[2])));
    const V3 cf = v3((float)c[0], (float)c[1], (float)c[2]);
    const double slack = 1e-5 * (std::fabs(c[0]) + std::fabs(c[1]) + std::fabs(c[2]) + R);  // the centre's rounding
    set_bound(o, cf, (float)((R + slack) * (1.0 + 1e-6)), SR_KIND_BUDGET, (float)(SR_MU_PLANAR * std::max(1.0, kappa)));
    o.mp = INFINITY;  // the frame's distances are not Euclidean: the bounding sphere alone
    return o.kind == SR_KIND_BUDGET;
}

void put_transform(float* f, const sr_transform& t) {
    std::memcpy(f + SR_F_POS, t.pos, 3 * sizeof(float));
    std::memcpy(f + SR_F_AXES, t.axes, 9 * sizeof(float));
}
void put_plane(float* f, const sr_plane& p) {
    put_transform(f, p.transform);
    f[12] = p.texture_offset[0];
    f[13] = p.texture_offset[1];
    f[14] = (float)p.repeat_texture;
    f[15] = p.texture_size[0];
    f[16] = p.texture_size[1];
}

// One rectangle face of a box (frag:587-647): pos, columns, width, height.
void put_face(float* g, V3 pos, V3 c0, V3 c1, V3 c2, float w, float h) {
    st(g, pos);
    st(g + 3, c0);
    st(g + 6, c1);
    st(g + 9, c2);
    g[12] = w;
    g[13] = h;
}

int pack_object(const sr_scene& s, int i, sr_dev_obj& o) {
    const sr_object& so = s.objects[i];
    std::memset(&o, 0, sizeof o);
    o.type = so.type;
    o.index = so.index;
    o.material_index = so.material_index;
    if (so.material_index < 0 || so.material_index >= SR_MAX_MATERIALS) return SR_E_CAPACITY;
    const int k = so.index;
    float* f = o.f;
    switch (so.type) {
    case SR_OBJECT_SPHERE: {
        if (k < 0 || k >= SR_MAX_SPHERES) return SR_E_CAPACITY;
        put_transform(f, s.spheres[k].transform);
        f[SR_F_P0] = s.spheres[k].radius;
        set_bound(o, ld(f), std::fabs(f[SR_F_P0]), SR_KIND_BUDGET, SR_MU_QUADRATIC);
        return SR_OK;
    }
    case SR_OBJECT_PLANE:
        if (k < 0 || k >= SR_MAX_PLANES) return SR_E_CAPACITY;
        put_plane(f, s.planes[k]);
        o.kind = SR_KIND_EXACT;
        {  // unbounded: budgeted by its plane distance alone (rb = +inf)
            V3 pos = ld(f + SR_F_POS), n = ld(f + SR_F_AXES + 3);
            if (std::isfinite(l1norm(pos)) && std::fabs(dot(n, n) - 1.f) < 1e-5f) {
                st(o.bc, pos);
                o.br = INFINITY;
                o.rb = INFINITY;
                o.mu = SR_MU_PLANAR;
                o.mp = SR_MU_QUADRATIC * (1.f + l1norm(pos));  // plane distance only
                o.pl1 = l1norm(pos);
                o.kind = SR_KIND_BUDGET;
            }
        }
        return SR_OK;
    case SR_OBJECT_DISK: {
        if (k < 0 || k >= SR_MAX_DISKS) return SR_E_CAPACITY;
        put_plane(f, s.disks[k].plane);
        f[17] = s.disks[k].radius;
        set_bound(o, ld(f), std::fabs(f[17]), SR_KIND_BUDGET, SR_MU_PLANAR);
        return SR_OK;
    }
    case SR_OBJECT_HOLLOW_DISK: {
        if (k < 0 || k >= SR_MAX_HOLLOW_DISKS) return SR_E_CAPACITY;
        put_plane(f, s.hollow_disks[k].plane);
        f[17] = s.hollow_disks[k].inner_radius;
        f[18] = s.hollow_disks[k].outer_radius;
        set_bound(o, ld(f), std::fabs(f[18]), SR_KIND_BUDGET, SR_MU_PLANAR);
        return SR_OK;
    }
    case SR_OBJECT_CYLINDER: {
        if (k < 0 || k >= SR_MAX_CYLINDERS) return SR_E_CAPACITY;
        put_transform(f, s.cylinders[k].transform);
        float h = s.cylinders[k].height, r = s.cylinders[k].radius;
        f[SR_F_P0] = h;
        f[SR_F_P0 + 1] = r;
        V3 a0 = ld(f + 3), a1 = ld(f + 6), a2 = ld(f + 9);
        if (orthonormal(a0, a1, a2) && h >= 0.f && r > 0.f) {
            double hh = 0.5 * h;
            set_bound(o, add(ld(f), scl(a1, (float)hh)), (float)std::sqrt((double)r * r + hh * hh),
                      SR_KIND_BUDGET, SR_MU_PLANAR);
        }
        return SR_OK;
    }
    case SR_OBJECT_RECTANGLE: {
        if (k < 0 || k >= SR_MAX_RECTANGLES) return SR_E_CAPACITY;
        put_plane(f, s.rectangles[k].plane);
        float w = s.rectangles[k].width, h = s.rectangles[k].height;
        f[17] = w;
        f[18] = h;
        V3 a0 = ld(f + 3), a1 = ld(f + 6), a2 = ld(f + 9);
        if (orthonormal(a0, a1, a2) && w >= 0.f && h >= 0.f) {
            V3 c = add(ld(f), add(scl(a0, 0.5f * w), scl(a2, 0.5f * h)));
            set_bound(o, c, (float)std::sqrt(0.25 * w * w + 0.25 * h * h), SR_KIND_BUDGET, SR_MU_PLANAR);
        } else {
            std::vector<std::array<double, 3>> pts;
            double kappa = 0;
            o.kind = SR_KIND_EXACT;
            if (parallelogram_corners(ld(f), a0, a1, a2, w, h, pts, kappa)) set_bound_corners(o, pts, kappa);
        }
        return SR_OK;
    }
    case SR_OBJECT_BOX: {
        if (k < 0 || k >= SR_MAX_BOXES) return SR_E_CAPACITY;
        const sr_box& b = s.boxes[k];
        put_transform(f, b.transform);
        f[12] = b.width;
        f[13] = b.depth;
        f[14] = b.height;
        V3 p = ld(b.transform.pos);
        V3 a0 = ld(b.transform.axes), a1 = ld(b.transform.axes + 3), a2 = ld(b.transform.axes + 6);
        float* F = f + SR_F_BOX_FACE0;
        const int S = SR_F_FACE_STRIDE;
        // frag:587-647, order bot, top, front, back, left, right (frag:649)
        put_face(F + 0 * S, add(p, scl(a2, b.depth)), a0, neg(a1), neg(a2), b.width, b.depth);
        put_face(F + 1 * S, add(p, scl(a1, b.height)), a0, a1, a2, b.width, b.depth);
        put_face(F + 2 * S, add(p, mv(a0, a1, a2, v3(0.f, b.height, b.depth))), a0, a2, neg(a1), b.width,
                 b.height);
        put_face(F + 3 * S, add(p, mv(a0, a1, a2, v3(b.width, b.height, 0.f))), neg(a0), neg(a2), neg(a1),
                 b.width, b.height);
        put_face(F + 4 * S, add(p, scl(a1, b.height)), a2, neg(a0), neg(a1), b.depth, b.height);
        put_face(F + 5 * S, add(p, mv(a0, a1, a2, v3(b.width, b.height, b.depth))), neg(a2), a0, neg(a1),
                 b.depth, b.height);
        if (orthonormal(a0, a1, a2) && b.width >= 0.f && b.depth >= 0.f && b.height >= 0.f) {
            V3 c = add(p, mv(a0, a1, a2, v3(0.5f * b.width, 0.5f * b.height, 0.5f * b.depth)));
            double R = 0.5 * std::sqrt((double)b.width * b.width + (double)b.height * b.height +
                                       (double)b.depth * b.depth);
            set_bound(o, c, (float)R, SR_KIND_BUDGET, SR_MU_PLANAR);
        } else {
            // the six faces' parallelograms (box_intersect tests each face's rect_test)
            std::vector<std::array<double, 3>> pts;
            double kappa = 1, kf = 0;
            bool ok = true;
            o.kind = SR_KIND_EXACT;
            for (int fc = 0; fc < 6 && ok; fc++) {
                const float* g = F + fc * S;
                ok = parallelogram_corners(ld(g), ld(g + 3), ld(g + 6), ld(g + 9), g[12], g[13], pts, kf);
                kappa = std::max(kappa, kf);
            }
            if (ok) set_bound_corners(o, pts, kappa);
        }
        return SR_OK;
    }
    default:
        return SR_E_INVALID;
    }
}

// The spectral norms of M (rows a0, a1, a2) and of M^-1, and M^-1 itself
// (binary64): the extreme eigenvalues of M M^T in closed form (symmetric
// 3x3). False for a singular, ill-conditioned (|M| |M^-1| >= 1e3) or
// non-finite frame. A cylinder test in this frame accepts points q - pos =
// M^-1 (x, y, z) with x^2 + z^2 within the lateral margin of r^2 and y in
// its height slab (geodesic.hip lat_margin: the analysis holds in the
// frame's coordinates), so |M^-1| scales its radius and |M^-1| |M|^2 its
// lateral margin in world distances.
bool frame_norms(V3 a0, V3 a1, V3 a2, double& nm, double& ninv, double inv[3][3]) {
    const double m[3][3] = {{a0.x, a0.y, a0.z}, {a1.x, a1.y, a1.z}, {a2.x, a2.y, a2.z}};
    double g[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) g[i][j] = m[i][0] * m[j][0] + m[i][1] * m[j][1] + m[i][2] * m[j][2];
    const double p1 = g[0][1] * g[0][1] + g[0][2] * g[0][2] + g[1][2] * g[1][2];
    const double q = (g[0][0] + g[1][1] + g[2][2]) / 3.0;
    double emax = q, emin = q;
    const double p2 = (g[0][0] - q) * (g[0][0] - q) + (g[1][1] - q) * (g[1][1] - q) + (g[2][2] - q) * (g[2][2] - q) + 2.0 * p1;
    if (p2 > 0.0) {
        const double p = std::sqrt(p2 / 6.0);
        double b[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) b[i][j] = (g[i][j] - (i == j ? q : 0.0)) / p;
        double r = 0.5 * (b[0][0] * (b[1][1] * b[2][2] - b[1][2] * b[2][1]) - b[0][1] * (b[1][0] * b[2][2] - b[1][2] * b[2][0]) +
                          b[0][2] * (b[1][0] * b[2][1] - b[1][1] * b[2][0]));
        r = std::min(1.0, std::max(-1.0, r));
        const double phi = std::acos(r) / 3.0;
        emax = q + 2.0 * p * std::cos(phi);
        emin = q + 2.0 * p * std::cos(phi + 2.0 * 3.14159265358979323846 / 3.0);
    }
    const double det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                       m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    if (!std::isfinite(det) || det == 0.0 || !(emin > 0.0) || !std::isfinite(emax)) return false;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const int i1 = (j + 1) % 3, i2 = (j + 2) % 3, j1 = (i + 1) % 3, j2 = (i + 2) % 3;
            inv[i][j] = (m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1]) / det;  // adjugate / det
        }
    // a relative allowance for the closed form's rounding
    nm = std::sqrt(emax) * (1.0 + 1e-9);
    ninv = 1.0 / std::sqrt(emin) * (1.0 + 1e-9);
    return nm * ninv < 1e3;
}

// Culling bounds of the curved test ray's segments (device_scene.h
// SR_TR_BLOCK / SR_TR_GROUP; geodesic.hip test_ray_hits_culled). Per segment
// k the sphere may_hit would use for a budgeted cylinder of that pose (set_bound:
// bc = pos + a1 h / 2, br = R + 1e-4 (1 + |bc|_1 + R), R = sqrt(r^2 + (h / 2)^2))
// and its axis a1; a bound covers its segments' spheres (R_bound >= |bc_k - c|
// + br_k) and axes (within alpha of the cone axis), with |pos|_1 at most pl1.
// Segments whose frame is not orthonormal (or not finite), a zero radius,
// make their block and group `always` (no culling).
void test_ray_bounds(float* buf, int nseg, float r, int& nblocks, int& ngroups) {
    struct Seg {
        double bc[3], br, ax[3], pl1, ls;
        bool ok;
    };
    std::vector<Seg> sg((size_t)nseg);
    for (int k = 0; k < nseg; k++) {
        const float* g = buf + (size_t)k * SR_SEG_FLOATS;
        Seg& q = sg[(size_t)k];
        const V3 a0 = ld(g + 3), a1 = ld(g + 6), a2 = ld(g + 9);
        const float h = g[12];
        // round 6: any well-conditioned frame (the reference's gram_schmidt of
        // d.xzy, d, d.zxy leaves some segments' frames ~1e-2 off orthonormal,
        // which made their blocks test every chord): the sphere of M^-1's
        // image of the frame's cylinder, its lateral margin scaled (ls)
        double nm = 1, ninv = 1, inv[3][3];
        q.ok = frame_norms(a0, a1, a2, nm, ninv, inv) && h >= 0.f && r > 0.f && std::isfinite(h) && std::isfinite(r);
        const double hh = 0.5 * (double)h;
        for (int i = 0; i < 3; i++) q.bc[i] = (double)g[i] + inv[i][1] * hh;  // pos + M^-1 (0, h / 2, 0)
        const double R = ninv * std::sqrt((double)r * r + hh * hh);
        q.br = (R + 1e-4 * (1.0 + std::fabs(q.bc[0]) + std::fabs(q.bc[1]) + std::fabs(q.bc[2]) + R)) * (1.0 + 1e-6);
        q.ax[0] = a1.x, q.ax[1] = a1.y, q.ax[2] = a1.z;
        q.pl1 = std::fabs((double)g[0]) + std::fabs((double)g[1]) + std::fabs((double)g[2]);
        q.ls = ninv * nm * nm * (1.0 + 1e-6);
        q.ok = q.ok && std::isfinite(q.br) && std::isfinite(q.pl1) && std::isfinite(q.ls);
    }
    // bound of segments [k0, k1) into out[SR_TR_BOUND_FLOATS]
    auto bound = [&](int k0, int k1, float* out) {
        double c[3] = {0, 0, 0}, ca[3] = {0, 0, 0};
        bool ok = k1 > k0;
        for (int k = k0; k < k1; k++) {
            ok = ok && sg[(size_t)k].ok;
            for (int i = 0; i < 3; i++) {
                c[i] += sg[(size_t)k].bc[i] / (k1 - k0);
                ca[i] += sg[(size_t)k].ax[i];
            }
        }
        const double cn = std::sqrt(ca[0] * ca[0] + ca[1] * ca[1] + ca[2] * ca[2]);
        double Rb = 0.0, cosa = 1.0, pl1 = 0.0, ls = 1.0;
        for (int k = k0; k < k1 && ok && cn > 0.0; k++) {
            const Seg& q = sg[(size_t)k];
            const double dx = q.bc[0] - c[0], dy = q.bc[1] - c[1], dz = q.bc[2] - c[2];
            Rb = std::max(Rb, std::sqrt(dx * dx + dy * dy + dz * dz) + q.br);
            cosa = std::min(cosa, (q.ax[0] * ca[0] + q.ax[1] * ca[1] + q.ax[2] * ca[2]) / cn);
            pl1 = std::max(pl1, q.pl1);
            ls = std::max(ls, q.ls);
        }
        cosa -= 1e-6;  // the float axes and the kernel's dot products
        ok = ok && cn > 0.0 && cosa > 0.0 && std::isfinite(Rb);
        for (int i = 0; i < 3; i++) {
            out[i] = (float)c[i];
            out[4 + i] = ok ? (float)(ca[i] / cn) : 0.f;
        }
        // centre rounded to float: grow R by that, and 1e-5 relative
        const double cr = 1e-6 * (std::fabs(c[0]) + std::fabs(c[1]) + std::fabs(c[2]));
        out[3] = ok ? (float)((Rb + cr) * (1.0 + 1e-5) + 1e-5) : INFINITY;
        out[7] = ok ? (float)cosa : 0.f;
        out[8] = ok ? (float)std::min(1.0, std::sqrt(std::max(0.0, 1.0 - cosa * cosa)) + 1e-6) : 1.f;
        out[9] = (float)(pl1 * (1.0 + 1e-6));
        out[10] = ok ? 0.f : 1.f;
        out[11] = ok ? std::nextafter((float)ls, INFINITY) : 1.f;  // the lateral margin's scale (>= 1)
    };
    float* blocks = buf + (size_t)(SR_MAX_POINTS - 1) * SR_SEG_FLOATS;
    float* groups = blocks + (size_t)SR_TR_BLOCKS * SR_TR_BOUND_FLOATS;
    nblocks = (nseg + SR_TR_BLOCK - 1) / SR_TR_BLOCK;
    ngroups = (nblocks + SR_TR_GROUP - 1) / SR_TR_GROUP;
    for (int b = 0; b < nblocks; b++)
        bound(b * SR_TR_BLOCK, std::min(nseg, (b + 1) * SR_TR_BLOCK), blocks + (size_t)b * SR_TR_BOUND_FLOATS);
    for (int g = 0; g < ngroups; g++)
        bound(g * SR_TR_GROUP * SR_TR_BLOCK, std::min(nseg, (g + 1) * SR_TR_GROUP * SR_TR_BLOCK),
              groups + (size_t)g * SR_TR_BOUND_FLOATS);
}

// gram_schmidt(mat3(d.xzy, d, d.zxy)), frag:739-753, 764, 789
void test_ray_frame(V3 d, float* axes9) {
    V3 m0 = v3(d.x, d.z, d.y), m1 = d, m2 = v3(d.z, d.x, d.y);
    auto project = [](V3 v, V3 t) { return scl(t, dot(v, t) / dot(t, t)); };
    m0 = sub(m0, project(m0, m1));
    m2 = sub(sub(m2, project(m2, m1)), project(m2, m0));
    st(axes9, nrm(m0));
    st(axes9 + 3, nrm(m1));
    st(axes9 + 6, nrm(m2));
}

inline bool hip_ok(hipError_t e) { return e == hipSuccess; }

// Frees a device buffer in stream order: after the context's in-flight
// frames (its last launch stream; `s` before its first launch). hipFree would
// synchronise the whole device.
void release(sr_ctx* ctx, void* p, hipStream_t s) {
    if (p && !hip_ok(hipFreeAsync(p, ctx->launched ? ctx->last_stream : s))) ctx->free_errors++;
}

// LRU eviction down to kCacheEntries - 1 entries (one is about to be added).
template <class Map, class Free>
void evict_lru(sr_ctx* ctx, Map& m, Free&& free_entry) {
    while (m.size() >= kCacheEntries) {
        auto victim = m.begin();
        for (auto it = m.begin(); it != m.end(); ++it)
            if (it->second.used < victim->second.used) victim = it;
        free_entry(victim->second);
        m.erase(victim);
    }
}

void evict_tables(sr_ctx* ctx) {
    evict_lru(ctx, ctx->tables, [&](Table& t) { release(ctx, t.dev, ctx->last_stream); });
}

int ensure_table(sr_ctx* ctx, int max_steps, int max_revs, hipStream_t s, const float4** out) {
    auto key = std::make_pair(max_steps, max_revs);
    auto it = ctx->tables.find(key);
    if (it != ctx->tables.end()) {
        it->second.used = ++ctx->tick;
        *out = it->second.dev;
        return SR_OK;
    }
    // frag:860, 914-915, 925: the angle sequence depends only on the step index
    const float max_angle = 2.0f * (float)max_revs * kPi;
    // entry i = one float4 {step_size, step_size / 6, cos phi, sin phi} (RK4
    // forms 0.5 step_size products exactly, geodesic.hip half_step). Four
    // padding entries: the step loop loads up to four steps ahead.
    std::vector<float4> h((size_t)max_steps + 4, make_float4(0.f, 0.f, 0.f, 0.f));
    float phi = 0.0f;
    for (int i = 0; i < max_steps; i++) {
        float step = (max_angle - phi) / (float)(max_steps - i);
        phi += step;
        const float c = (float)std::cos((double)phi), sn = (float)std::sin((double)phi);
        h[(size_t)i] = make_float4(step, step / 6.0f, c, sn);
    }
    evict_tables(ctx);
    Table& t = ctx->tables[key];
    t.steps = max_steps;
    t.host = std::move(h);
    t.used = ++ctx->tick;
    // stream-ordered: allocated and filled on the caller's stream, ahead of
    // the launch that reads it (no device-wide synchronisation)
    if (!hip_ok(hipMallocAsync(reinterpret_cast<void**>(&t.dev), t.host.size() * sizeof(float4), s))) {
        ctx->tables.erase(key);
        return SR_E_NOMEM;
    }
    if (!hip_ok(hipMemcpyAsync(t.dev, t.host.data(), t.host.size() * sizeof(float4), hipMemcpyHostToDevice, s))) {
        release(ctx, t.dev, s);
        ctx->tables.erase(key);
        return SR_E_HIP;
    }
    *out = t.dev;
    return SR_OK;
}

// Synchronous upload of host bytes into a fresh device buffer on the
// context's private upload stream (the previous buffer is freed in stream
// order after the context's in-flight frames).
int upload_bytes(sr_ctx* ctx, const void* src, size_t bytes, void** dev) {
    release(ctx, *dev, ctx->upload);
    *dev = nullptr;
    if (!hip_ok(hipMallocAsync(dev, bytes, ctx->upload))) return SR_E_NOMEM;
    if (!hip_ok(hipMemcpyAsync(*dev, src, bytes, hipMemcpyHostToDevice, ctx->upload)) ||
        !hip_ok(hipStreamSynchronize(ctx->upload)))
        return SR_E_HIP;
    return SR_OK;
}

int upload_rgba(sr_ctx* ctx, const uint8_t* px, int w, int h, int layers, int ch, uint32_t** dev) {
    size_t n = (size_t)w * h * layers;
    std::vector<uint32_t> rgba(n);
    for (size_t i = 0; i < n; i++) {
        const uint8_t* p = px + i * ch;
        uint32_t a = ch == 4 ? p[3] : 255u;  // GL_RGB reads alpha 1
        rgba[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | (a << 24);
    }
    return upload_bytes(ctx, rgba.data(), n * sizeof(uint32_t), reinterpret_cast<void**>(dev));
}

// Waits for this context's in-flight frames (its last launch stream), not
// for the device: other contexts' frames and collectives run on.
bool wait_ctx(sr_ctx* ctx) {
    if (!ctx->launched) return true;
    return hip_ok(hipStreamSynchronize(ctx->last_stream));
}

void free_pixel_state(sr_ctx* ctx, hipStream_t s) {
    release(ctx, ctx->d_ps, s);
    release(ctx, ctx->d_list, s);
    release(ctx, ctx->d_count, s);
    ctx->d_ps = nullptr;
    ctx->d_list = nullptr;
    ctx->d_count = nullptr;
    ctx->ps_n = 0;
}

// Grows the pixel-state planes in stream order: the old buffers are freed
// after the context's in-flight frames, the new ones allocated and cleared
// on the caller's stream ahead of the launch (no host wait, no device-wide
// synchronisation).
int ensure_pixel_state(sr_ctx* ctx, size_t n, hipStream_t s) {
    if (n <= ctx->ps_n) return SR_OK;
    free_pixel_state(ctx, s);
    if (!hip_ok(hipMallocAsync(reinterpret_cast<void**>(&ctx->d_ps), n * SR_PS_FIELDS * sizeof(float), s)) ||
        !hip_ok(hipMallocAsync(reinterpret_cast<void**>(&ctx->d_list), n * sizeof(int), s)) ||
        !hip_ok(hipMallocAsync(reinterpret_cast<void**>(&ctx->d_count), 2 * sizeof(int), s))) {
        free_pixel_state(ctx, s);
        return SR_E_NOMEM;
    }
    // [0]: the shade kernel's resume queue
    if (!hip_ok(hipMemsetAsync(ctx->d_count, 0, 2 * sizeof(int), s))) {
        free_pixel_state(ctx, s);
        return SR_E_HIP;
    }
    ctx->ps_n = n;
    return SR_OK;
}

// Opacity bitmap of the texture array for the step loop's hit classification
// (geodesic.hip hit_opacity): bit (layer, y, x) is set when every texel within
// +-SR_OPQ_RADIUS of (x, y), wrapping like the sampler, has alpha 255. A
// bilinear footprint {x0, x0 + 1} x {y0, y0 + 1} whose floor lies within one
// texel of (x, y) then reads alpha 1 exactly (LERP filtering).
int make_opacity_map(sr_ctx* ctx, const uint8_t* px, int w, int h, int layers, int ch, uint8_t** dev) {
    const size_t stride = ((size_t)w + 7) / 8;
    std::vector<uint8_t> bits(stride * (size_t)h * (size_t)layers, 0);
    std::vector<uint8_t> row((size_t)w * h);
    std::vector<uint8_t> tmp((size_t)w * h);
    const int R = SR_OPQ_RADIUS;
    for (int l = 0; l < layers; l++) {
        for (size_t i = 0; i < (size_t)w * h; i++) {
            const uint8_t* p = px + ((size_t)l * w * h + i) * ch;
            row[i] = ch == 4 ? (p[3] == 255) : 1;
        }
        for (int y = 0; y < h; y++)  // horizontal min, wrapping
            for (int x = 0; x < w; x++) {
                uint8_t m = 1;
                for (int d = -R; d <= R && m; d++) m = row[(size_t)y * w + (((x + d) % w) + w) % w];
                tmp[(size_t)y * w + x] = m;
            }
        for (int y = 0; y < h; y++)  // vertical min, wrapping
            for (int x = 0; x < w; x++) {
                uint8_t m = 1;
                for (int d = -R; d <= R && m; d++) m = tmp[(size_t)((((y + d) % h) + h) % h) * w + x];
                if (m) bits[((size_t)l * h + y) * stride + (x >> 3)] |= (uint8_t)(1u << (x & 7));
            }
    }
    return upload_bytes(ctx, bits.data(), bits.size(), reinterpret_cast<void**>(dev));
}

void evict_orders(sr_ctx* ctx) {
    evict_lru(ctx, ctx->orders, [&](sr_ctx::Order& o) {
        if (ctx->last_order == o.order) {
            ctx->last_order = nullptr;
            ctx->last_slots = 0;
        }
        release(ctx, o.order, ctx->last_stream);
        release(ctx, o.cost, ctx->last_stream);
    });
}

// Launch order for a grid shape: tiles nearest the frame centre first (where
// the black hole usually is) until a frame has measured the costs. One
// buffer pair per shape and split setting, allocated on first use. Entries
// are launch codes (geodesic.hip order_tiles): tile << 8 for a whole
// tile, -1 for the split grid's slots no tile uses yet.
int ensure_order(sr_ctx* ctx, int gx, int gy, const int* list, hipStream_t s, int** order, int** cost) {
    const int split = ctx->split_tiles;
    const auto key = std::make_tuple(gx, gy, split, split ? ctx->split_log2 : 0, list);
    auto it = ctx->orders.find(key);
    if (it != ctx->orders.end()) {
        it->second.used = ++ctx->tick;
        *order = it->second.order;
        *cost = it->second.cost;
        return SR_OK;
    }
    const size_t n = (size_t)gx * gy;
    const size_t slots = n + (size_t)((64 >> (split ? ctx->split_log2 : 6)) - 1) * (size_t)split;
    std::vector<int> ord(n);
    std::vector<double> d(n);
    for (size_t i = 0; i < n; i++) {
        ord[i] = (int)i;
        const double x = (double)(i % gx) + 0.5 - 0.5 * gx, y = (double)(i / gx) + 0.5 - 0.5 * gy;
        d[i] = x * x + y * y;
    }
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return d[a] < d[b]; });
    for (int& v : ord) v <<= 8;
    ord.resize(slots, -1);
    evict_orders(ctx);
    sr_ctx::Order& o = ctx->orders[key];
    o.host = std::move(ord);
    o.used = ++ctx->tick;
    // stream-ordered, on the caller's stream ahead of the launch
    if (!hip_ok(hipMallocAsync(reinterpret_cast<void**>(&o.order), slots * sizeof(int), s)) ||
        !hip_ok(hipMallocAsync(reinterpret_cast<void**>(&o.cost), n * sizeof(int), s))) {
        release(ctx, o.order, s);
        ctx->orders.erase(key);
        return SR_E_NOMEM;
    }
    if (!hip_ok(hipMemcpyAsync(o.order, o.host.data(), slots * sizeof(int), hipMemcpyHostToDevice, s)) ||
        !hip_ok(hipMemsetAsync(o.cost, 0, n * sizeof(int), s))) {
        release(ctx, o.order, s);
        release(ctx, o.cost, s);
        ctx->orders.erase(key);
        return SR_E_HIP;
    }
    *order = o.order;
    *cost = o.cost;
    return SR_OK;
}

// The device copy of a block list (sr_render_block_list), uploaded once per
// distinct list on the caller's stream and kept for the context's lifetime (a
// rank's balanced list does not change between frames).
int ensure_block_list(sr_ctx* ctx, const int* blocks, int n, hipStream_t s, const int** dev) {
    std::vector<int> key(blocks, blocks + n);
    auto it = ctx->block_lists.find(key);
    if (it != ctx->block_lists.end()) {
        it->second.used = ++ctx->tick;
        *dev = it->second.dev;
        return SR_OK;
    }
    if (ctx->block_lists.size() >= kCacheEntries) {
        // an evicted list's launch orders go with it (they are keyed by its device copy)
        evict_lru(ctx, ctx->block_lists, [&](sr_ctx::BlockList& b) {
            for (auto o = ctx->orders.begin(); o != ctx->orders.end();) {
                if (std::get<4>(o->first) == b.dev) {
                    if (ctx->last_order == o->second.order) {
                        ctx->last_order = nullptr;
                        ctx->last_slots = 0;
                    }
                    release(ctx, o->second.order, ctx->last_stream);
                    release(ctx, o->second.cost, ctx->last_stream);
                    o = ctx->orders.erase(o);
                } else {
                    ++o;
                }
            }
            release(ctx, b.dev, ctx->last_stream);
        });
    }
    // the map's key is the source of the stream-ordered upload: it lives as long as the entry
    auto ins = ctx->block_lists.emplace(std::move(key), sr_ctx::BlockList{});
    sr_ctx::BlockList& b = ins.first->second;
    b.used = ++ctx->tick;
    if (!hip_ok(hipMallocAsync(reinterpret_cast<void**>(&b.dev), (size_t)n * sizeof(int), s))) {
        ctx->block_lists.erase(ins.first);
        return SR_E_NOMEM;
    }
    if (!hip_ok(hipMemcpyAsync(b.dev, ins.first->first.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice, s))) {
        release(ctx, b.dev, s);
        ctx->block_lists.erase(ins.first);
        return SR_E_HIP;
    }
    *dev = b.dev;
    return SR_OK;
}

// Camera::loadShader (camera.cpp:41-50) and frag:859's launch invariant
void build_cam(const sr_camera* cam, sr_dev_cam& dc) {
    std::memcpy(dc.pos, cam->transform.pos, sizeof dc.pos);
    std::memcpy(dc.axes, cam->transform.axes, sizeof dc.axes);
    dc.ray_forward = 1.0f / (float)std::tan((double)(cam->fov / 360.0f * kPi));
}

// The orbital-plane exclusion of a budgeted cylinder (geodesic.hip SR_XCYL)
// for a low-energy orbit: u < 0.6 and E = u'^2 + u^2 (1 - u) <= SR_XCYL_EMAX
// at its start. E is conserved along the orbit (u'' = -u + 1.5 u^2; RK4's
// drift over a frame is orders below the 2 % allowed here), so u stays below
// 0.58, |u'| <= sqrt(E) and |u''| <= 1/6, and one step changes u by at most
// kappa = sqrt(E) dphi + dphi^2 / 12. A chord whose nearer end lies at r_lo
// has its farther end within r_hi = 1 / (1 / r_lo - kappa) (and within 2 /
// u_f unless it is forced, budget_event), so S = |o|_1 + len + 1 <= (sqrt 3
// + 1) r_hi + r_lo + 1, and the chord stays r_lo cos(dphi) from the origin.
// may_hit accepts it only within br + mu S + qk (S + |pos|_1)^2 of the
// bounding centre (chords off the axis by SR_BUDGET_DPMIN; the nearly
// parallel ones are the slab budget's). Chords with r_lo >= r_c, where
// r_lo cos(dphi) - |bc| exceeds that reach, cannot hit; the others have S <=
// S(r_c), so a bounding centre farther than reach(S(r_c)) from the orbital
// plane cannot be reached by any chord of the orbit. r_c is found on a
// geometric grid, each interval [r_i, r_i+1] checked with its worst ends.
// Both return r_c with reach(S(r_c)) (clear_radius; r_c = +inf: none).
struct ClearRadius {
    double rc, need, rhi;
};
static ClearRadius clear_radius(const sr_dev_slot& sl, float u_f, float max_dphi) {
    ClearRadius out{INFINITY, INFINITY, INFINITY};
    if (!(u_f > 0.0f) || !(max_dphi > 0.0f) || !std::isfinite(sl.br) || !std::isfinite(sl.cn)) return out;
    if (!(max_dphi <= SR_XLOW_DPHI_MAX)) return out;  // the premises are proven up to this step angle
    const double d = (double)max_dphi * 1.001;
    const double kap = std::sqrt((double)SR_XCYL_EMAX) * 1.02 * d + d * d / 12.0 * 1.02 + 1e-6;
    const double R2 = 2.0 / (double)u_f * (1.0 + 1e-5);
    const auto rhi = [&](double r) {
        const double v = 1.0 / r - kap;
        return v > 1.0 / R2 ? 1.0 / v : R2;
    };
    const auto S = [&](double r) { return (std::sqrt(3.0) + 1.0) * rhi(r) * (1.0 + 1e-5) + r + 1.0; };
    const auto reach = [&](double s) {
        const double sc = s + (double)sl.pl1;
        return ((double)sl.br + (double)sl.mu * s + (double)sl.qk * sc * sc) * 1.001 + 1e-4;
    };
    const double c = (1.0 - d * d / 2.0) * (1.0 - 1e-4);
    // from the top (R2) down while every interval clears by distance
    double hi = R2, rc = R2;
    for (;;) {
        const double lo = std::max(1.0, hi / 1.002);
        if (!(lo * c - (double)sl.cn - reach(S(hi)) > 0.0)) break;
        rc = lo;
        if (lo <= 1.0) break;
        hi = lo;
    }
    if (rc >= R2) return out;
    out.rc = rc;
    out.need = reach(S(rc)) + 1e-6 * rhi(rc);
    out.rhi = rhi(rc);
    return out;
}
// (every bounded slot: for spheres mu S(r_c) replaces the orbital-plane
// exclusion's mu S_max, 0.96 for the quadratic factor; for a cylinder it is
// the only plane exclusion; + 1e-5 |bc| for the plane distance's rounding)
static float xlow_need(const sr_dev_slot& sl, float u_f, float max_dphi) {
    if (sl.type == SR_OBJECT_PLANE || (sl.type == SR_OBJECT_CYLINDER && !(sl.x1 > 0.0f))) return INFINITY;
    const ClearRadius c = clear_radius(sl, u_f, max_dphi);
    return std::isfinite(c.need) ? std::nextafter((float)(c.need + 1e-5 * (double)sl.cn), INFINITY) : INFINITY;
}
// The periapsis exclusion (geodesic.hip SR_XPERI): a low-energy orbit stays
// at u <= u_t, the root of u^2 (1 - u) = E below 2/3 (f(u) = u^2 (1 - u)
// increases there), so its chords' nearer ends lie at r >= 1 / u_t (end
// points within 2e-5 of their radius). When that is beyond r_c (x 1.001), no
// chord of the orbit can reach the object by distance from the origin alone:
// E <= f(1 / (1.001 r_c)), less 0.1 % and 1e-6 for the energy's drift and
// rounding, and at most SR_XCYL_EMAX (the step bound's premise). Planes and
// the black hole are never excluded.
static float xperi_e(const sr_dev_slot& sl, float u_f, float max_dphi) {
    if (sl.type == SR_OBJECT_PLANE) return -1.0f;
    const ClearRadius c = clear_radius(sl, u_f, max_dphi);
    if (!std::isfinite(c.rc)) return -1.0f;
    const double w = 1.0 / (c.rc * 1.001);
    double e = w < 2.0 / 3.0 ? w * w * (1.0 - w) * (1.0 - 1e-3) - 1e-6 : (double)SR_XCYL_EMAX;
    e = std::min(e, (double)SR_XCYL_EMAX);
    return e > 0.0 ? std::nextafter((float)e, 0.0f) : -1.0f;
}

int build_frame(sr_ctx* ctx, const sr_camera* cam, const sr_params* p, int width, int height, sr_dev_frame& fr) {
    if (!cam || !p || width <= 0 || height <= 0) return SR_E_INVALID;
    if (p->raytrace_type < 0 || p->raytrace_type > 3) return SR_E_INVALID;
    if (p->filter_mode != SR_FILTER_LERP && p->filter_mode != SR_FILTER_WEIGHTED) return SR_E_INVALID;
    // the hand-off packs a ray's step count into 24 bits (geodesic.hip ps_word)
    if (p->max_steps < 0 || p->max_steps > SR_MAX_STEPS) return SR_E_INVALID;
    std::memset(&fr, 0, sizeof fr);
    for (int j = 0; j < SR_MAX_BUDGET; j++) fr.xlow_need[j] = INFINITY;  // launch() sets them
    for (int j = 0; j < SR_MAX_BUDGET; j++) fr.xperi_e[j] = -1.0f;
    build_cam(cam, fr.cam[0]);
    fr.batch = 1;
    // frag:860 (launch invariant, same float ops)
    fr.max_angle = 2.0f * (float)p->max_revolutions * kPi;
    fr.res_x = (float)width;
    fr.res_y = (float)height;
    fr.u_f = p->u_f;
    fr.uf_radius = 1.0f / p->u_f;
    fr.uf_radius2 = fr.uf_radius * fr.uf_radius;  // binary32, as the kernel would compute it
    {
        // chords start within R = 1 / u_f and end within 2 R, or are forced
        // (geodesic.hip budget_frame): S <= (sqrt 3 + 3) R + 1
        const double R = p->u_f > 0.0f ? 1.0 / (double)p->u_f : INFINITY;
        // (x 1.005: the chord ends' 4e-7 r off the orbital plane, as mu >= SR_MU_PLANAR)
        const double S = ((std::sqrt(3.0) + 3.0) * R * (1.0 + 1e-5) + 1.0) * 1.001 * 1.005;
        fr.xplane_s = S < 1.0e30 ? std::nextafter((float)S, INFINITY) : INFINITY;
#ifdef SR_XS_FIXED  // timing experiments only: a fixed S_max (not exact for every u_f)
        fr.xplane_s = SR_XS_FIXED;
#endif
    }
    fr.percent_black = p->percent_black;
    fr.curved_percentage = p->curved_percentage;
    fr.max_steps = p->max_steps;
    fr.raytrace_type = p->raytrace_type;
    fr.crosshair = p->crosshair;
    fr.filter_mode = p->filter_mode;
    fr.cull = ctx->cull ? 1 : 0;
    fr.width = width;
    fr.height = height;
    fr.bg_w = ctx->bg_w;
    fr.bg_h = ctx->bg_h;
    fr.arr_w = ctx->arr_w;
    fr.arr_h = ctx->arr_h;
    fr.arr_layers = ctx->arr_layers;
    {
        const double dphi = (double)fr.max_angle / (p->max_steps > 0 ? p->max_steps : 1);
        fr.out_dip = (float)(1.0 - dphi * dphi / 8.0 - 1e-6);
        fr.max_dphi = std::nextafter((float)std::sqrt(8.0 * (1.0 - (double)fr.out_dip)), INFINITY);
        // the inner black-hole window's bounds (geodesic.hip SR_BH_WINDOW2)
        fr.bh_u2 = std::nextafter((float)((double)fr.out_dip / (1.0 + SR_BH_G2)), 0.0f);
        fr.bh_u3 = fr.max_dphi <= SR_BH_S_DPHI
                       ? std::nextafter((float)((double)fr.out_dip / (1.0 + SR_BH_G3)), 0.0f)
                       : fr.bh_u2;
    }
    fr.split_tiles = ctx->split_tiles;
    fr.split_log2 = ctx->split_log2;
    fr.split_min_steps = ctx->split_min_steps;
    fr.fast_unroll = ctx->fast_unroll;
    return SR_OK;
}

// Renders the same rows of n_frames frames (cams[f]; output f at out + f *
// frame_stride) in one launch of each kernel.
int launch(sr_ctx* ctx, const sr_camera* cams, int n_frames, const sr_params* params, int width, int height,
           int nrows, int row_base, int block_rows, int block_stride, uint8_t* out, size_t pitch,
           size_t frame_stride, float* dbg_rgba, int32_t* dbg_steps, sr_stream stream,
           const int* d_block_list = nullptr, int32_t* d_wave_cost = nullptr) {
    if (!ctx) return SR_E_INVALID;
    if (!ctx->scene_set) return SR_E_NOT_READY;
    if (!cams || n_frames < 1) return SR_E_INVALID;
    if (n_frames > SR_MAX_BATCH) return SR_E_CAPACITY;
    sr_dev_frame fr;
    int rc = build_frame(ctx, cams, params, width, height, fr);
    if (rc != SR_OK) return rc;
    for (int f = 1; f < n_frames; f++) build_cam(&cams[f], fr.cam[f]);
    fr.batch = n_frames;
    // the black hole's u window (geodesic.hip SR_BH_WINDOW): chord origins within r = 100
    fr.num_budget = ctx->h_scene.num_budget;
    fr.num_budget_cyl = __builtin_popcount((unsigned)ctx->h_scene.budget_cyl_mask);
    fr.tr_visible = ctx->h_scene.tr_visible ? 1 : 0;
    fr.win_ok = fr.uf_radius <= 100.0f;
    {  // the low-energy exclusions (xlow_need, xperi_e), per (u_f, step angle)
        if (!(ctx->xc_uf == fr.u_f && ctx->xc_dphi == fr.max_dphi)) {
            for (int j = 0; j < SR_MAX_BUDGET; j++) ctx->xc_need[j] = INFINITY;
            for (int j = 0; j < SR_MAX_BUDGET; j++) ctx->xc_peri[j] = -1.0f;
            for (int j = 0; j < ctx->h_scene.num_budget; j++) {
                const sr_dev_slot& sl = ctx->h_scene.slots[j];
                ctx->xc_need[j] = xlow_need(sl, fr.u_f, fr.max_dphi);
                ctx->xc_peri[j] = xperi_e(sl, fr.u_f, fr.max_dphi);
            }
            ctx->xc_uf = fr.u_f;
            ctx->xc_dphi = fr.max_dphi;
        }
        for (int j = 0; j < SR_MAX_BUDGET; j++) fr.xlow_need[j] = ctx->xc_need[j];
        for (int j = 0; j < SR_MAX_BUDGET; j++) fr.xperi_e[j] = ctx->xc_peri[j];
    }
    for (int f = 0; f < n_frames; f++) {
        const float* q = fr.cam[f].pos;
        if (!((double)q[0] * q[0] + (double)q[1] * q[1] + (double)q[2] * q[2] <= 1.0e4)) fr.win_ok = 0;
    }
    if (nrows < 0 || block_rows <= 0) return SR_E_INVALID;
    if (out && pitch < (size_t)width * 4) return SR_E_INVALID;
    if (n_frames > 1 && (!out || frame_stride < pitch * (size_t)nrows || dbg_rgba || dbg_steps)) return SR_E_INVALID;
    fr.out_frame_stride = (int64_t)frame_stride;
    fr.tiles = ((width + 15) / 16) * ((nrows + 15) / 16);
    fr.nrows = nrows;
    fr.row_base = row_base;
    fr.block_rows = block_rows;
    fr.block_stride = block_stride;
    fr.block_list = d_block_list;
    fr.wave_cost = d_wave_cost;
    if (!hip_ok(hipSetDevice(ctx->device))) return SR_E_HIP;
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (ctx->launched && s != ctx->last_stream) {
        // ordered after the launches on the previous stream: order_ev was
        // recorded at the end of the last launch, so the old stream's handle
        // is not touched here (the caller may have destroyed it since)
        if (!hip_ok(hipStreamWaitEvent(s, ctx->order_ev, 0))) return SR_E_HIP;
    }
    // every stream-ordered free from here on (ensure_*'s evictions) goes to s
    ctx->last_stream = s;
    const float4* tbl = nullptr;
    rc = ensure_table(ctx, params->max_steps, params->max_revolutions, s, &tbl);
    if (rc != SR_OK) return rc;
    rc = ensure_pixel_state(ctx, (size_t)fr.tiles * (size_t)n_frames * 256, s);
    if (rc != SR_OK) return rc;
    int* order = nullptr;
    int* cost = nullptr;
    if (nrows > 0) {
        rc = ensure_order(ctx, (width + 15) / 16, (nrows + 15) / 16, d_block_list, s, &order, &cost);
        if (rc != SR_OK) return rc;
        ctx->last_order = order;
        ctx->last_slots = (size_t)((width + 15) / 16) * (size_t)((nrows + 15) / 16) +
                          (size_t)((64 >> (ctx->split_tiles ? ctx->split_log2 : 6)) - 1) * (size_t)ctx->split_tiles;
    }
    hipError_t e = sr_launch_geodesic(ctx->d_scene, tbl, ctx->d_segs, ctx->d_bg, ctx->d_arr, ctx->d_opq, &fr, out, pitch,
                                      dbg_rgba, dbg_steps, ctx->d_ps, ctx->ps_n, ctx->d_list, ctx->d_count, order, cost,
                                      ctx->d_diag,
                                      ctx->timing_n < ctx->timing_cap ? &ctx->tev[4 * (size_t)ctx->timing_n++] : nullptr,
                                      s);
    if (hip_ok(e)) e = hipEventRecord(ctx->order_ev, s);
    ctx->launched = true;
    return hip_ok(e) ? SR_OK : SR_E_HIP;
}

}  // namespace

extern "C" hipError_t sr_assemble_blocks_device(const uint8_t* stacked, size_t rank_stride, size_t in_frame_stride,
                                                const int* dev_lists, int world, int per, int height, int block_rows,
                                                size_t row_bytes, uint8_t* out, size_t out_frame_stride, int n_frames,
                                                hipStream_t stream);
extern "C" int sr_assemble_blocks_host(const uint8_t* stacked, size_t rank_stride, size_t in_frame_stride,
                                       const int* lists, int world, int per, int height, int block_rows,
                                       size_t row_bytes, uint8_t* out, size_t out_frame_stride, int n_frames);

extern "C" {

int sr_assemble_blocks(const uint8_t* stacked, size_t rank_stride, size_t in_frame_stride, const int* lists,
                       int world, int per, int height, int block_rows, size_t row_bytes, uint8_t* out,
                       size_t out_frame_stride, int n_frames, int on_device, sr_stream stream) {
    if (!stacked || !lists || !out || world <= 0 || per < 0 || height <= 0 || block_rows <= 0 || row_bytes == 0 ||
        n_frames < 1)
        return SR_E_INVALID;
    if (!on_device)
        return sr_assemble_blocks_host(stacked, rank_stride, in_frame_stride, lists, world, per, height, block_rows,
                                       row_bytes, out, out_frame_stride, n_frames);
    const hipError_t e = sr_assemble_blocks_device(stacked, rank_stride, in_frame_stride, lists, world, per, height,
                                                   block_rows, row_bytes, out, out_frame_stride, n_frames,
                                                   reinterpret_cast<hipStream_t>(stream));
    return hip_ok(e) ? SR_OK : SR_E_HIP;
}

const char* sr_version(void) { return "schwarzschild-mi355x 0.1 (gfx950)"; }

const char* sr_status_string(int s) {
    switch (s) {
    case SR_OK: return "ok";
    case SR_E_INVALID: return "invalid argument";
    case SR_E_CAPACITY: return "capacity exceeded";
    case SR_E_HIP: return "HIP runtime error";
    case SR_E_NOMEM: return "out of memory";
    case SR_E_NOT_READY: return "scene not set";
    case SR_E_NO_DEVICE: return "no HIP device";
    case SR_E_IO: return "file write failed";
    default: return "unknown status";
    }
}

int sr_create(sr_ctx** out, int hip_device) {
    if (!out) return SR_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (!hip_ok(hipGetDeviceCount(&n)) || n <= 0) return SR_E_NO_DEVICE;
    if (hip_device < 0 || hip_device >= n) return SR_E_NO_DEVICE;
    if (!hip_ok(hipSetDevice(hip_device))) return SR_E_HIP;
    sr_ctx* c = new (std::nothrow) sr_ctx();
    if (!c) return SR_E_NOMEM;
    c->device = hip_device;
    std::memset(&c->h_scene, 0, sizeof c->h_scene);
    c->h_scene.flat_miss_r2 = INFINITY;  // set by sr_set_scene
    if (!hip_ok(hipStreamCreateWithFlags(&c->upload, hipStreamNonBlocking))) {
        c->upload = nullptr;
        sr_destroy(c);
        return SR_E_HIP;
    }
    if (!hip_ok(hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming))) {
        c->order_ev = nullptr;
        sr_destroy(c);
        return SR_E_HIP;
    }
    if (!hip_ok(hipMalloc(&c->d_scene, sizeof(sr_dev_scene))) ||
        !hip_ok(hipMalloc(&c->d_segs, (size_t)SR_SEGS_BUF_FLOATS * sizeof(float))) ||
        !hip_ok(hipMalloc(reinterpret_cast<void**>(&c->d_diag), sizeof(int)))) {
        sr_destroy(c);
        return SR_E_NOMEM;
    }
    if (!hip_ok(hipMemsetAsync(c->d_scene, 0, sizeof(sr_dev_scene), c->upload)) ||
        !hip_ok(hipMemsetAsync(c->d_diag, 0, sizeof(int), c->upload)) ||
        !hip_ok(hipMemsetAsync(c->d_segs, 0, (size_t)SR_SEGS_BUF_FLOATS * sizeof(float),
                               c->upload)) ||
        !hip_ok(hipStreamSynchronize(c->upload))) {
        sr_destroy(c);
        return SR_E_HIP;
    }
    sr_test_ray tr;
    sr_test_ray_default(&tr);
    int rc = sr_set_test_ray(c, &tr);
    if (rc != SR_OK) {
        sr_destroy(c);
        return rc;
    }
    *out = c;
    return SR_OK;
}

void sr_destroy(sr_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)wait_ctx(c);
    if (c->d_scene) (void)hipFree(c->d_scene);
    if (c->d_segs) (void)hipFree(c->d_segs);
    if (c->d_diag) (void)hipFree(c->d_diag);
    // the rest came from the stream-ordered allocator: freed the same way,
    // then waited for (the context's frames are done: wait_ctx)
    const hipStream_t s = c->upload;
    if (s) {
        c->launched = false;  // release() frees on `s`
        release(c, c->d_bg, s);
        release(c, c->d_arr, s);
        release(c, c->d_opq, s);
        for (auto& kv : c->tables) release(c, kv.second.dev, s);
        free_pixel_state(c, s);
        for (auto& kv : c->orders) {
            release(c, kv.second.order, s);
            release(c, kv.second.cost, s);
        }
        for (auto& kv : c->block_lists) release(c, kv.second.dev, s);
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
    for (hipEvent_t e : c->tev) (void)hipEventDestroy(e);
    if (c->order_ev) (void)hipEventDestroy(c->order_ev);
    delete c;
}

int sr_diag_counters(sr_ctx* c, int64_t* out, int n) {
    if (!c || !out || n < 0) return SR_E_INVALID;
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    int dropped = 0;
    if (!hip_ok(hipMemcpyAsync(&dropped, c->d_diag, sizeof(int), hipMemcpyDeviceToHost, c->upload)) ||
        !hip_ok(hipStreamSynchronize(c->upload)))
        return SR_E_HIP;
    const int64_t v[2] = {dropped, c->free_errors};
    for (int i = 0; i < n && i < 2; i++) out[i] = v[i];
    return SR_OK;
}

int sr_set_background(sr_ctx* c, const uint8_t* px, int w, int h, int ch) {
    if (!c || !px || w <= 0 || h <= 0 || (ch != 3 && ch != 4)) return SR_E_INVALID;
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    int rc = upload_rgba(c, px, w, h, 1, ch, &c->d_bg);
    if (rc != SR_OK) {
        c->bg_w = c->bg_h = 0;
        return rc;
    }
    c->bg_w = w;
    c->bg_h = h;
    return SR_OK;
}

int sr_set_texture_array(sr_ctx* c, const uint8_t* px, int w, int h, int layers, int ch) {
    if (!c || !px || w <= 0 || h <= 0 || layers <= 0 || (ch != 3 && ch != 4)) return SR_E_INVALID;
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    int rc = upload_rgba(c, px, w, h, layers, ch, &c->d_arr);
    if (rc == SR_OK) rc = make_opacity_map(c, px, w, h, layers, ch, &c->d_opq);
    if (rc != SR_OK) {
        c->arr_w = c->arr_h = c->arr_layers = 0;
        return rc;
    }
    c->arr_w = w;
    c->arr_h = h;
    c->arr_layers = layers;
    return SR_OK;
}

// The compact copy of a budgeted object (device_scene.h sr_dev_slot).
// The farthest any point the object's exact test accepts can lie from the
// origin (geodesic.hip outward_slot): the primitive's farthest point F plus
// the larger of its static margins (the bounding sphere's and the
// distance-to-primitive one, mp), x 1.001, rounded up; the per-chord terms
// (mu S, a cylinder's quadratic margin) are outward_clear's. A disk's or a
// rim's farthest point is sqrt((c . n)^2 + (|c_perp| + R)^2), a rectangle's
// a corner, a sphere's |c| + R. At most cn + br (the bounding sphere's),
// which boxes, planes and frames without a unit normal keep.
static float far_reach(const sr_dev_obj& o, float cn) {
    const double sphere = (double)cn + (double)o.br;
    if (!(o.mp < INFINITY) || !std::isfinite(sphere)) return (float)sphere;
    const float* f = o.f;
    const double p[3] = {f[SR_F_POS], f[SR_F_POS + 1], f[SR_F_POS + 2]};
    double a0[3], a1[3], a2[3];
    for (int i = 0; i < 3; i++) {
        a0[i] = f[SR_F_AXES + i];
        a1[i] = f[SR_F_AXES + 3 + i];
        a2[i] = f[SR_F_AXES + 6 + i];
    }
    const auto norm = [](const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); };
    const auto rim = [&](const double* c, double R) {  // circle centre c, normal a1, radius R
        const double cn1 = c[0] * a1[0] + c[1] * a1[1] + c[2] * a1[2];
        const double cp = std::sqrt(std::max(0.0, c[0] * c[0] + c[1] * c[1] + c[2] * c[2] - cn1 * cn1));
        return std::sqrt(cn1 * cn1 + (cp + R) * (cp + R));
    };
    double F;
    switch (o.type) {
    case SR_OBJECT_DISK: F = rim(p, std::fabs((double)f[17])); break;
    case SR_OBJECT_HOLLOW_DISK: F = rim(p, std::fabs((double)f[18])); break;
    case SR_OBJECT_CYLINDER: {
        const double h = f[SR_F_P0], R = std::fabs((double)f[SR_F_P0 + 1]);
        const double top[3] = {p[0] + a1[0] * h, p[1] + a1[1] * h, p[2] + a1[2] * h};
        F = std::max(rim(p, R), rim(top, R));
        break;
    }
    case SR_OBJECT_RECTANGLE: {
        const double w = f[17], h = f[18];
        F = 0.0;
        for (int i = 0; i < 4; i++) {
            const double al = (i & 1) ? w : 0.0, be = (i & 2) ? h : 0.0;
            const double c[3] = {p[0] + a0[0] * al + a2[0] * be, p[1] + a0[1] * al + a2[1] * be,
                                 p[2] + a0[2] * al + a2[2] * be};
            F = std::max(F, norm(c));
        }
        break;
    }
    default:
        return (float)sphere;
    }
    // the bounding sphere's static margin mu (1 + |c|_1 + R) with R <= br, or mp
    const double l1c = std::fabs((double)o.bc[0]) + std::fabs((double)o.bc[1]) + std::fabs((double)o.bc[2]);
    const double margin = std::max((double)o.mu * (1.0 + l1c + (double)o.br), (double)o.mp);
    const double rf = (F + margin) * 1.001;
    if (!std::isfinite(rf) || !(rf < sphere)) return (float)sphere;
    return std::nextafter((float)rf, INFINITY);
}

static void pack_slot(const sr_dev_obj& o, int cyl, sr_dev_slot& sl) {
    std::memset(&sl, 0, sizeof sl);
    const float* f = o.f;
    sl.type = o.type;
    sl.cyl = cyl;
    sl.rb = o.rb;
    sl.mp = o.mp;
    sl.br = o.br;
    sl.mu = o.mu;
    sl.pl1 = o.pl1;
    std::memcpy(sl.bc, o.bc, sizeof sl.bc);
    sl.cn = std::nextafter((float)(std::sqrt((double)o.bc[0] * o.bc[0] + (double)o.bc[1] * o.bc[1] +
                                             (double)o.bc[2] * o.bc[2]) * 1.001),
                           INFINITY);
    std::memcpy(sl.pos, f + SR_F_POS, 3 * sizeof(float));
    std::memcpy(sl.a0, f + SR_F_AXES, 3 * sizeof(float));
    std::memcpy(sl.a1, f + SR_F_AXES + 3, 3 * sizeof(float));
    std::memcpy(sl.a2, f + SR_F_AXES + 6, 3 * sizeof(float));
    sl.rf = far_reach(o, sl.cn);
    switch (o.type) {
    case SR_OBJECT_RECTANGLE:
    case SR_OBJECT_HOLLOW_DISK:
        sl.x0 = f[17];
        sl.x1 = f[18];
        break;
    case SR_OBJECT_DISK:
        sl.x0 = f[17];
        break;
    case SR_OBJECT_BOX:
        sl.x0 = f[12];
        sl.x1 = f[13];
        sl.x2 = f[14];
        break;
    case SR_OBJECT_CYLINDER: {
        sl.x0 = f[SR_F_P0];
        sl.x1 = f[SR_F_P0 + 1];
        // a margin factor: rounded away from zero so the product bounds the
        // quotient the margin was specified with. SR_CYL_DIRFREE: the lateral
        // margin SR_CYL_QMARGIN Sc^2 / r holds for every chord direction
        // (tests/test_cyl_lateral_margin.py), so the
        // direction floor SR_BUDGET_DPMIN no longer divides it
        const double q = (double)SR_CYL_QMARGIN / ((double)sl.x1 * (SR_CYL_DIRFREE ? 1.0 : (double)SR_BUDGET_DPMIN));
        sl.qk = (float)(q * (1.0 + 1e-5));
        break;
    }
    default:
        break;
    }
}

int sr_set_scene(sr_ctx* c, const sr_scene* s) {
    if (!c || !s) return SR_E_INVALID;
    if (s->num_objects < 0 || s->num_lights < 0) return SR_E_INVALID;
    if (s->num_objects > SR_MAX_OBJECTS || s->num_lights > SR_MAX_LIGHTS) return SR_E_CAPACITY;
    sr_dev_scene d = c->h_scene;  // keeps the test-ray part
    d.num_objects = s->num_objects;
    d.num_lights = s->num_lights;
    std::memset(d.objs, 0, sizeof d.objs);
    d.num_budget = 0;
    d.num_step = 0;
    d.budget_cyl_mask = 0;
    for (int i = 0; i < s->num_objects; i++) {
        int rc = pack_object(*s, i, d.objs[i]);
        if (rc != SR_OK) return rc;
        sr_dev_obj& o = d.objs[i];
        // the per-lane budget registers hold SR_MAX_BUDGET objects; further
        // bounded objects fall back to per-chord bounding-sphere tests
        if (o.kind == SR_KIND_BUDGET && d.num_budget >= SR_MAX_BUDGET) o.kind = SR_KIND_CHORD;
        if (o.kind == SR_KIND_BUDGET) {
            // SR_CYL_DIRFREE: no budgeted cylinder needs the direction tests
            // (chord_parallel) or the slab budget of chords nearly parallel
            // to its axis: its distance budget covers every direction
            const bool dirs = !SR_CYL_DIRFREE && o.type == SR_OBJECT_CYLINDER;
            pack_slot(o, dirs ? __builtin_popcount((unsigned)d.budget_cyl_mask) : -1, d.slots[d.num_budget]);
            if (dirs) d.budget_cyl_mask |= 1 << d.num_budget;
            d.budget_idx[d.num_budget++] = i;
        } else {
            d.step_idx[d.num_step++] = i;
        }
    }
    {  // the flat intersect's far-field miss radius (geodesic.hip flat_misses)
        double R = 1.0 + SR_MU_QUADRATIC * 3.0;  // the black hole
        for (int i = 0; i < s->num_objects && std::isfinite(R); i++) {
            const sr_dev_obj& o = d.objs[i];
            const double bc = std::sqrt((double)o.bc[0] * o.bc[0] + (double)o.bc[1] * o.bc[1] + (double)o.bc[2] * o.bc[2]);
            if (o.kind == SR_KIND_EXACT || o.type == SR_OBJECT_PLANE || !std::isfinite(o.br) || !std::isfinite(bc))
                R = INFINITY;
            else
                R = std::max(R, bc + (double)o.br);
        }
        // beyond twice that plus one, with a margin far above any rounding of
        // the tests' quadratics and slab distances at that range
        const double r = 2.0 * R + 1.0;
        d.flat_miss_r2 = std::isfinite(r) ? std::nextafter((float)(r * r), INFINITY) : INFINITY;
    }
    std::memcpy(d.materials, s->materials, sizeof d.materials);
    std::memcpy(d.lights, s->lights, sizeof d.lights);
    std::memcpy(d.planes, s->planes, sizeof d.planes);
    std::memcpy(d.texture_sizes, s->texture_sizes, sizeof d.texture_sizes);
    std::memcpy(d.max_texture_size, s->max_texture_size, sizeof d.max_texture_size);
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    if (!hip_ok(hipMemcpyAsync(c->d_scene, &d, sizeof d, hipMemcpyHostToDevice, c->upload)) ||
        !hip_ok(hipStreamSynchronize(c->upload)))
        return SR_E_HIP;
    c->h_scene = d;
    c->xc_uf = c->xc_dphi = NAN;  // xlow_need, xperi_e again at the next launch
    c->scene_set = true;
    return SR_OK;
}

int sr_set_test_ray(sr_ctx* c, const sr_test_ray* t) {
    if (!c || !t) return SR_E_INVALID;
    if (t->num_curved_points < 0 || t->num_curved_points > SR_MAX_POINTS) return SR_E_CAPACITY;
    sr_dev_scene d = c->h_scene;
    d.tr_visible = t->visible ? 1 : 0;
    d.tr_radius = t->radius;
    d.tr_extended_length = t->extended_length;
    std::memcpy(d.tr_curved_color, t->curved_color, sizeof d.tr_curved_color);
    std::memcpy(d.tr_flat_color, t->flat_color, sizeof d.tr_flat_color);
    std::memset(d.tr_flat, 0, sizeof d.tr_flat);
    st(d.tr_flat, ld(t->flat_origin));
    test_ray_frame(ld(t->flat_dir), d.tr_flat + 3);
    d.tr_flat[12] = t->extended_length;
    d.tr_flat[13] = t->radius;
    const int n = t->num_curved_points;
    const int nseg = n >= 2 ? n - 1 : 0;
    std::vector<float> segs((size_t)SR_SEGS_BUF_FLOATS, 0.f);
    for (int i = 0; i < nseg; i++) {  // frag:777-793
        float* g = segs.data() + (size_t)i * SR_SEG_FLOATS;
        V3 pi = ld(t->curved_points[i]);
        V3 diff = sub(ld(t->curved_points[i + 1]), pi);
        float h = len(diff);
        if (i == n - 2 && len(ld(t->curved_points[n - 1])) < 1.0f) h = t->extended_length;
        st(g, pi);
        test_ray_frame(diff, g + 3);
        g[12] = h;
        g[13] = t->radius;
        // 1: an orthonormal frame (tolerance 1e-5) whose own capsule bounds its
        // accepted points (geodesic.hip clearance_tr's segment refinement)
        g[14] = orthonormal(ld(g + 3), ld(g + 6), ld(g + 9)) && std::isfinite(h) && h >= 0.f ? 1.f : 0.f;
    }
    d.tr_num_segments = nseg;
    test_ray_bounds(segs.data(), nseg, t->radius, d.tr_num_blocks, d.tr_num_groups);
    // the test ray's budget (geodesic.hip clearance_tr): the flat cylinder's
    // accepted points lie within |M^-1| (r + its lateral margin) of the
    // segment [pos, pos + L M^-1 (0, 1, 0)] (frame_norms); the farthest
    // accepted point and the largest |pos|_1 for outward lanes
    {
        const V3 fp = ld(d.tr_flat), a0 = ld(d.tr_flat + 3), a1 = ld(d.tr_flat + 6), a2 = ld(d.tr_flat + 9);
        const float L = d.tr_flat[12], r = d.tr_flat[13];
        double nm = 1, ninv = 1, inv[3][3];
        bool ok = frame_norms(a0, a1, a2, nm, ninv, inv) && std::isfinite(fp.x) && std::isfinite(fp.y) &&
                  std::isfinite(fp.z) && L >= 0.f && std::isfinite(L) && r > 0.f && std::isfinite(r);
        const double g[3] = {inv[0][1], inv[1][1], inv[2][1]};
        std::memset(d.tr_fg, 0, sizeof d.tr_fg);
        if (ok) {
            for (int i = 0; i < 3; i++) d.tr_fg[i] = (float)g[i];
            // the float axis g's rounding over the length L: radius and margin grown by it
            const double gerr = 1e-7 * (std::fabs(g[0]) + std::fabs(g[1]) + std::fabs(g[2])) * (double)L;
            d.tr_fg[3] = std::nextafter((float)(ninv * (1.0 + 1e-6)), INFINITY);
            d.tr_fg[4] = std::nextafter((float)(ninv * nm * nm * (1.0 + 1e-6)), INFINITY);
            d.tr_fg[5] = std::nextafter((float)(gerr + 1e-6 * (std::fabs((double)fp.x) + std::fabs((double)fp.y) +
                                                             std::fabs((double)fp.z))), INFINITY);
        }
        const auto n3 = [](double x, double y, double z) { return std::sqrt(x * x + y * y + z * z); };
        double far = ok ? std::max(n3(fp.x, fp.y, fp.z), n3(fp.x + g[0] * L, fp.y + g[1] * L, fp.z + g[2] * L)) +
                              ninv * r + (double)d.tr_fg[5]
                        : INFINITY;
        double pl1 = std::fabs((double)fp.x) + std::fabs((double)fp.y) + std::fabs((double)fp.z);
        const float* groups = segs.data() + (size_t)(SR_MAX_POINTS - 1) * SR_SEG_FLOATS +
                              (size_t)SR_TR_BLOCKS * SR_TR_BOUND_FLOATS;
        float ls = d.tr_fg[4];  // the largest lateral-margin scale (outward lanes)
        for (int g = 0; g < d.tr_num_groups; g++) {
            const float* B = groups + (size_t)g * SR_TR_BOUND_FLOATS;
            far = B[10] != 0.f ? INFINITY : std::max(far, n3(B[0], B[1], B[2]) + (double)B[3]);
            pl1 = std::max(pl1, (double)B[9]);
            ls = std::max(ls, B[11]);
        }
        d.tr_fg[6] = ls;
        // the float centre's distance and a 1e-5 relative allowance
        d.tr_far = std::isfinite(far) ? std::nextafter((float)(far * (1.0 + 1e-5) + 1e-5), INFINITY) : INFINITY;
        d.tr_pl1 = std::nextafter((float)(pl1 * (1.0 + 1e-6)), INFINITY);
    }
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    if (!hip_ok(hipMemcpyAsync(c->d_segs, segs.data(), segs.size() * sizeof(float), hipMemcpyHostToDevice,
                               c->upload)) ||
        !hip_ok(hipMemcpyAsync(c->d_scene, &d, sizeof d, hipMemcpyHostToDevice, c->upload)) ||
        !hip_ok(hipStreamSynchronize(c->upload)))
        return SR_E_HIP;
    c->h_scene = d;
    return SR_OK;
}

int sr_render(sr_ctx* c, const sr_camera* cam, const sr_params* p, int width, int height, int row_begin,
              int row_end, uint8_t* out, size_t pitch, sr_stream stream) {
    if (!out || row_begin < 0 || row_end > height || row_begin > row_end) return SR_E_INVALID;
    int n = row_end - row_begin;
    return launch(c, cam, 1, p, width, height, n, row_begin, n > 0 ? n : 1, 0, out, pitch, 0, nullptr, nullptr,
                  stream);
}

int sr_blocks_row_count(int height, int block_rows, int block_first, int block_step) {
    if (height <= 0 || block_rows <= 0 || block_first < 0 || block_step <= 0) return 0;
    int rows = 0;
    for (int b = block_first; b * block_rows < height; b += block_step) {
        int r = height - b * block_rows;
        rows += r < block_rows ? r : block_rows;
    }
    return rows;
}

int sr_render_blocks(sr_ctx* c, const sr_camera* cam, const sr_params* p, int width, int height, int block_rows,
                     int block_first, int block_step, uint8_t* out, size_t pitch, sr_stream stream) {
    if (!out || block_rows <= 0 || block_first < 0 || block_step <= 0) return SR_E_INVALID;
    int nblocks = 0;
    for (int b = block_first; b * block_rows < height; b += block_step) nblocks++;
    return launch(c, cam, 1, p, width, height, nblocks * block_rows, block_first * block_rows, block_rows,
                  block_step * block_rows, out, pitch, 0, nullptr, nullptr, stream);
}

int sr_wave_costs(sr_ctx* c, const sr_camera* cam, const sr_params* p, int width, int height, int32_t* dev_out,
                  sr_stream stream) {
    if (!c || !cam || !dev_out || width <= 0 || height <= 0) return SR_E_INVALID;
    // split tiles off for this launch: every wave is a whole 8x8 wave tile
    const int split = c->split_tiles;
    c->split_tiles = 0;
    const int rc = launch(c, cam, 1, p, width, height, height, 0, height, height, nullptr, (size_t)width * 4, 0,
                          nullptr, nullptr, stream, nullptr, dev_out);
    c->split_tiles = split;
    return rc;
}

int sr_render_block_list(sr_ctx* c, const sr_camera* cams, int n_frames, const sr_params* p, int width, int height,
                         int block_rows, const int* blocks, int n_blocks, uint8_t* out, size_t pitch,
                         size_t frame_stride, sr_stream stream) {
    if (!c || !out || !blocks || block_rows <= 0 || n_blocks <= 0 || height <= 0) return SR_E_INVALID;
    if ((long long)n_blocks * block_rows > (1 << 24)) return SR_E_INVALID;
    const int nb = (height + block_rows - 1) / block_rows;
    for (int i = 0; i < n_blocks; i++)
        if (blocks[i] < -1 || blocks[i] >= nb) return SR_E_INVALID;
    if (!hip_ok(hipSetDevice(c->device))) return SR_E_HIP;
    const int* d = nullptr;
    const int rc = ensure_block_list(c, blocks, n_blocks, reinterpret_cast<hipStream_t>(stream), &d);
    if (rc != SR_OK) return rc;
    return launch(c, cams, n_frames, p, width, height, n_blocks * block_rows, 0, block_rows, block_rows, out, pitch,
                  frame_stride, nullptr, nullptr, stream, d);
}

int sr_render_blocks_batch(sr_ctx* c, const sr_camera* cams, int n_frames, const sr_params* p, int width,
                           int height, int block_rows, int block_first, int block_step, uint8_t* out, size_t pitch,
                           size_t frame_stride, sr_stream stream) {
    if (!out || block_rows <= 0 || block_first < 0 || block_step <= 0) return SR_E_INVALID;
    int nblocks = 0;
    for (int b = block_first; b * block_rows < height; b += block_step) nblocks++;
    return launch(c, cams, n_frames, p, width, height, nblocks * block_rows, block_first * block_rows, block_rows,
                  block_step * block_rows, out, pitch, frame_stride, nullptr, nullptr, stream);
}

int sr_render_debug(sr_ctx* c, const sr_camera* cam, const sr_params* p, int width, int height, int row_begin,
                    int row_end, float* dbg_rgba, uint8_t* out, int32_t* dbg_steps, sr_stream stream) {
    if (row_begin < 0 || row_end > height || row_begin > row_end) return SR_E_INVALID;
    if (!dbg_rgba && !out && !dbg_steps) return SR_E_INVALID;
    int n = row_end - row_begin;
    return launch(c, cam, 1, p, width, height, n, row_begin, n > 0 ? n : 1, 0, out, (size_t)width * 4, 0, dbg_rgba,
                  dbg_steps, stream);
}

int sr_abi_struct_sizes(size_t* out, int n) {
    const size_t sz[6] = {sizeof(sr_camera), sizeof(sr_params), sizeof(sr_scene),
                          sizeof(sr_test_ray), sizeof(sr_material), sizeof(sr_light)};
    if (!out || n < 0) return SR_E_INVALID;
    for (int i = 0; i < n && i < 6; i++) out[i] = sz[i];
    return SR_OK;
}

int sr_set_split(sr_ctx* c, int max_tiles, int lanes_per_wave, int min_steps) {
    if (!c || max_tiles < 0 || max_tiles > (1 << 16) || min_steps < 0) return SR_E_INVALID;
    int lg;
    switch (lanes_per_wave) {
    case 16: lg = 4; break;
    case 4: lg = 2; break;
    case 1: lg = 0; break;
    default: return SR_E_INVALID;
    }
    c->split_tiles = max_tiles;
    c->split_log2 = lg;
    c->split_min_steps = min_steps;
    return SR_OK;
}

int sr_set_latency_mode(sr_ctx* c, int on) {
    if (!c) return SR_E_INVALID;
    c->fast_unroll = on ? 2 : SR_FAST_UNROLL_DEFAULT;
    return SR_OK;
}

// Not in sr.h's public set: the launch codes order_tiles wrote at the end
// of the context's last frame (the next frame of that shape runs them; tile
// << 8, | 0x80 | sub for split workgroups, -1 unused). Waits for the frame.
int sr_debug_last_order(sr_ctx* c, int* out, int max_n, int* n) {
    if (!c || !n || max_n < 0 || (max_n && !out)) return SR_E_INVALID;
    *n = (int)c->last_slots;
    if (!c->last_order) return SR_OK;
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    const size_t k = c->last_slots < (size_t)max_n ? c->last_slots : (size_t)max_n;
    if (k && (!hip_ok(hipMemcpyAsync(out, c->last_order, k * sizeof(int), hipMemcpyDeviceToHost, c->upload)) ||
              !hip_ok(hipStreamSynchronize(c->upload))))
        return SR_E_HIP;
    return SR_OK;
}

// Not in sr.h's public set: a host copy of the integrate -> shade hand-off
// (geodesic.hip PS_*: SR_PS_FIELDS floats per pixel id in its planes) after
// the context's last frame, for post-mortems of single pixels without
// instrumenting the kernel. *n_px = pixel ids the buffer holds; copies
// min(max_floats, n_px * SR_PS_FIELDS) floats.
int sr_debug_pixel_state(sr_ctx* c, float* out, size_t max_floats, size_t* n_px) {
    if (!c || !n_px || (max_floats && !out)) return SR_E_INVALID;
    *n_px = c->ps_n;
    if (!max_floats || !c->d_ps) return SR_OK;
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    size_t k = c->ps_n * SR_PS_FIELDS;
    if (k > max_floats) k = max_floats;
    if (!hip_ok(hipMemcpyAsync(out, c->d_ps, k * sizeof(float), hipMemcpyDeviceToHost, c->upload)) ||
        !hip_ok(hipStreamSynchronize(c->upload)))
        return SR_E_HIP;
    return SR_OK;
}

// Not in sr.h's public set: toggles segment culling (parity tests compare
// culled and exhaustive renders bit for bit).
int sr_debug_set_culling(sr_ctx* c, int enabled) {
    if (!c) return SR_E_INVALID;
    c->cull = enabled != 0;
    return SR_OK;
}

// Not in sr.h's public set: per-kernel HIP-event timing of the next
// `capacity` frames (0: off). bench.py reads the integrate kernel's duration
// for its roofline line from here.
int sr_debug_set_timing(sr_ctx* c, int capacity) {
    if (!c || capacity < 0 || capacity > (1 << 16)) return SR_E_INVALID;
    if (!hip_ok(hipSetDevice(c->device)) || !wait_ctx(c)) return SR_E_HIP;
    for (hipEvent_t e : c->tev) (void)hipEventDestroy(e);
    c->tev.assign(4 * (size_t)capacity, nullptr);
    c->timing_cap = 0;
    c->timing_n = 0;
    for (auto& e : c->tev)
        if (!hip_ok(hipEventCreate(&e))) return SR_E_HIP;
    c->timing_cap = capacity;
    return SR_OK;
}

// Waits for the recorded frames and writes ms[3 * f + j] (j = integrate,
// shade, resume) for up to max_frames of them; *n_frames = frames recorded.
// Restarts the recording.
int sr_debug_kernel_times(sr_ctx* c, float* ms, int max_frames, int* n_frames) {
    if (!c || !n_frames || max_frames < 0 || (max_frames && !ms)) return SR_E_INVALID;
    *n_frames = c->timing_n;
    const int n = c->timing_n < max_frames ? c->timing_n : max_frames;
    for (int f = 0; f < n; f++) {
        hipEvent_t* e = &c->tev[4 * (size_t)f];
        if (!hip_ok(hipEventSynchronize(e[3]))) return SR_E_HIP;
        for (int j = 0; j < 3; j++)
            if (!hip_ok(hipEventElapsedTime(&ms[3 * f + j], e[j], e[j + 1]))) return SR_E_HIP;
    }
    c->timing_n = 0;
    return SR_OK;
}

}  // extern "C"
