// geodesic.hip — the per-pixel Schwarzschild null-geodesic kernel for gfx950.
//
// Hot path of the reference: assets/shaders/black_hole.frag:843-936 (one GLSL
// fragment per pixel). Here: one wave64 lane per ray, each wave renders an
// 8x8 pixel tile (four waves = a 16x16 workgroup tile). All scene/camera data
// are launch-invariant and read with wave-uniform scalar loads; the per-step
// angle table {dphi_i, phi_i, cos phi_i, sin phi_i} depends only on the step
// index i (frag:914-915, 925), which is wave-uniform inside the step loop, so
// the two transcendentals and the division of every step become one s_load.
//
// Arithmetic contract (shared with oracle/sr_oracle.c): binary32,
// no contraction (-ffp-contract=off), correctly rounded div/sqrt, binary64
// transcendentals rounded to binary32, GLSL evaluation order.
#include <hip/hip_runtime.h>

#include "../device_scene.h"

namespace {

#define SR_PI 3.1415926535f
#define SR_EPS 0.0000001f

struct f2 { float x, y; };
struct f3 { float x, y, z; };
struct f4 { float x, y, z, w; };
struct m3 { f3 c0, c1, c2; };

__device__ __forceinline__ f2 F2(float x, float y) { f2 r; r.x = x; r.y = y; return r; }
__device__ __forceinline__ f3 F3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f4 F4(float x, float y, float z, float w) { f4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return F3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return F3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator-(f3 a) { return F3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return F3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return F3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return F3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ f4 operator+(f4 a, f4 b) { return F4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len(f3 a) { return sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 nrm(f3 a) { float k = 1.0f / sqrtf(dot(a, a)); return a * k; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return F3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
__device__ __forceinline__ f3 mv(const m3& m, f3 v) { return (m.c0 * v.x + m.c1 * v.y) + m.c2 * v.z; }
__device__ __forceinline__ f3 mtv(const m3& m, f3 v) { return F3(dot(m.c0, v), dot(m.c1, v), dot(m.c2, v)); }
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }

// binary64 function, rounded once to binary32
__device__ __forceinline__ float t_sin(float x) { __builtin_amdgcn_sched_barrier(0); float r_ = (float)sin((double)x); __builtin_amdgcn_sched_barrier(0); return r_; }
__device__ __forceinline__ float t_cos(float x) { __builtin_amdgcn_sched_barrier(0); float r_ = (float)cos((double)x); __builtin_amdgcn_sched_barrier(0); return r_; }
__device__ __forceinline__ float t_asin(float x) { __builtin_amdgcn_sched_barrier(0); float r_ = (float)asin((double)x); __builtin_amdgcn_sched_barrier(0); return r_; }
__device__ __forceinline__ float t_atan2(float y, float x) { __builtin_amdgcn_sched_barrier(0); float r_ = (float)atan2((double)y, (double)x); __builtin_amdgcn_sched_barrier(0); return r_; }
__device__ __forceinline__ float t_pow(float x, float y) { __builtin_amdgcn_sched_barrier(0); float r_ = (float)pow((double)x, (double)y); __builtin_amdgcn_sched_barrier(0); return r_; }

__device__ __forceinline__ f3 ld3(const float* p) { return F3(p[0], p[1], p[2]); }
__device__ __forceinline__ m3 ldm(const float* a) {
    m3 m;
    m.c0 = F3(a[0], a[1], a[2]);
    m.c1 = F3(a[3], a[4], a[5]);
    m.c2 = F3(a[6], a[7], a[8]);
    return m;
}

// Closest-hit record. slot >= 0: scene object; SLOT_BH: the black hole
// (OBJECT_TYPE_SPECIAL); SLOT_TR_FLAT / SLOT_TR_CURVED: test-ray cylinders.
enum { SLOT_NONE = -100, SLOT_BH = -1, SLOT_TR_FLAT = -2, SLOT_TR_CURVED = -3 };
struct Hit {
    float dist;
    f3 p;
    int slot;
    int face;  // box face, or test-ray segment
    int key;   // visiting order in the reference's intersect()
};

struct Tex {
    const uint32_t* __restrict__ bg;
    const uint32_t* __restrict__ arr;
};

// ---- primitive tests: return the reference's is_hit and fill p ------------
// sphere_intersect, frag:457-478
__device__ __forceinline__ bool sphere_test(f3 o, f3 d, f3 c, float r, float max_lambda, f3& p) {
    f3 oc = o - c;
    float b = dot(d, oc);
    float D = b * b - dot(oc, oc) + r * r;
    if (D < 0.0f) return false;
    float sq = sqrtf(D);
    float first = -dot(d, oc);
    float l1 = first - sq, l2 = first + sq;
    float lam = -1.0f;  // min_positive, frag:441-454
    if (l1 > 0.0f && l2 > 0.0f) lam = gmin(l1, l2);
    else if (l1 > 0.0f) lam = l1;
    else if (l2 > 0.0f) lam = l2;
    bool hit = lam >= 0.0f && (max_lambda < 0.0f || lam <= max_lambda);
    if (hit) p = o + d * lam;
    return hit;
}

// plane_intersect, frag:483-500 (normal = axes[1])
__device__ __forceinline__ bool plane_test(f3 o, f3 d, f3 pos, f3 n, float max_lambda, f3& p) {
    float denom = dot(n, d);
    if (fabsf(denom) < SR_EPS) return false;
    float lam = dot(n, pos - o) / denom;
    bool hit = lam >= 0.0f && (max_lambda < 0.0f || lam <= max_lambda);
    if (hit) p = o + d * lam;
    return hit;
}

// rectangle_intersect, frag:573-584
__device__ __forceinline__ bool rect_test(f3 o, f3 d, f3 pos, f3 c0, f3 c1, f3 c2, float w, float h,
                                          float max_lambda, f3& p) {
    if (!plane_test(o, d, pos, c1, max_lambda, p)) return false;
    f3 q = p - pos;
    float alpha = dot(q, c0);
    float beta = dot(q, c2);
    return (alpha >= 0.0f && alpha <= w) && (beta >= 0.0f && beta <= h);
}

// cylinder_intersect, frag:523-571 (lateral surface, local frame transpose(axes))
__device__ __forceinline__ bool cyl_test(f3 o, f3 d, f3 pos, const m3& A, float height, float radius,
                                         float max_lambda, f3& p) {
    f3 lo = mtv(A, o - pos);
    f3 ld = mtv(A, d);
    float opsq = (lo.x * lo.x + lo.z * lo.z) + 0.0f * 0.0f;
    float dpsq = (ld.x * ld.x + ld.z * ld.z) + 0.0f * 0.0f;
    float a = lo.x * ld.x + lo.z * ld.z;
    float D = a * a + dpsq * (radius * radius - opsq);
    if (D < 0.0f) return false;
    float l1 = -(a + sqrtf(D)) / dpsq;
    float l2 = -(a - sqrtf(D)) / dpsq;
    f3 p1 = o + d * l1, p2 = o + d * l2;
    float h1 = dot(p1 - pos, A.c1), h2 = dot(p2 - pos, A.c1);
    bool in1 = h1 >= 0.0f && h1 <= height;
    bool in2 = h2 >= 0.0f && h2 <= height;
    if (!in1 && !in2) return false;
    float lam = -1.0f;
    if (in1 && in2) {
        if (l1 > 0.0f && l2 > 0.0f) lam = gmin(l1, l2);
        else if (l1 > 0.0f) lam = l1;
        else if (l2 > 0.0f) lam = l2;
    } else if (in1) {
        lam = l1;
    } else {
        lam = l2;
    }
    p = o + d * lam;
    return lam >= 0.0f && (max_lambda < 0.0f || lam <= max_lambda);
}

// intersect() visits the black hole, the flat test ray, the curved test-ray
// segments and then objects[] in order, and a later hit replaces the current
// one only at a strictly smaller distance (frag:757-814): the result is the
// minimum of (dist, visiting order). These keys let candidates be evaluated in
// any order (or skipped) with the same winner.
enum { KEY_BH = 0, KEY_TR_FLAT = 1, KEY_TR_CURVED0 = 2, KEY_OBJ0 = 2 + SR_MAX_POINTS };

__device__ __forceinline__ void consider(Hit& best, bool hit, f3 p, f3 o, int slot, int face, int key) {
    if (!hit) return;
    float dist = len(p - o);
    if (best.slot == SLOT_NONE || dist < best.dist || (dist == best.dist && key < best.key)) {
        best.dist = dist;
        best.p = p;
        best.slot = slot;
        best.face = face;
        best.key = key;
    }
}

// Conservative segment culling (not part of the reference; exact by margin):
// every primitive's accepted hit point lies on the chord [o, o + len*d] up to
// rounding and inside the object's bounding sphere, so a chord whose distance
// from the sphere exceeds it by the rounding margin cannot report a hit.
__device__ __forceinline__ bool may_hit(const sr_dev_obj& ob, f3 o, f3 d, float seg_len, float S) {
    f3 w = ld3(ob.bc) - o;
    float t = dot(w, d);
    t = t < 0.0f ? 0.0f : t;
    t = t > seg_len ? seg_len : t;
    f3 q = w - d * t;
    float d2 = dot(q, q);
    float R = ob.br + ob.mu * S;
    if (ob.type == SR_OBJECT_CYLINDER) {
        // the quadratic's root error grows as S^2 / (r * |d_perp|^2)
        float ca = dot(d, ld3(ob.f + SR_F_AXES + 3));
        float dp = 1.0f - ca * ca;
        float r = ob.f[SR_F_P0 + 1];
        if (!(dp > 1.0e-6f) || !(r > 0.0f)) return true;
        R = R + 4.0e-6f * S * S * __builtin_amdgcn_rcpf(r * dp);
    }
    return !(d2 > R * R);
}

__device__ __forceinline__ Hit no_hit() {
    Hit h;
    h.slot = SLOT_NONE;
    h.dist = 0.0f;
    h.p = F3(0.0f, 0.0f, 0.0f);
    h.face = 0;
    h.key = 0;
    return h;
}

// intersect_object, frag:697-736, folded into the running closest hit
__device__ __forceinline__ void test_object(Hit& best, const sr_dev_obj& ob, int k, f3 o, f3 d, float max_lambda) {
    const float* f = ob.f;
    const f3 pos = ld3(f + SR_F_POS);
    const int key = KEY_OBJ0 + k;
    f3 p;
    switch (ob.type) {
    case SR_OBJECT_SPHERE:
        consider(best, sphere_test(o, d, pos, f[SR_F_P0], max_lambda, p), p, o, k, 0, key);
        break;
    case SR_OBJECT_PLANE:
        consider(best, plane_test(o, d, pos, ld3(f + SR_F_AXES + 3), max_lambda, p), p, o, k, 0, key);
        break;
    case SR_OBJECT_DISK: {  // frag:502-508
        bool h = plane_test(o, d, pos, ld3(f + SR_F_AXES + 3), max_lambda, p);
        if (h) {
            f3 q = p - pos;
            h = dot(q, q) <= f[17] * f[17];
        }
        consider(best, h, p, o, k, 0, key);
        break;
    }
    case SR_OBJECT_HOLLOW_DISK: {  // frag:510-517
        bool h = plane_test(o, d, pos, ld3(f + SR_F_AXES + 3), max_lambda, p);
        if (h) {
            f3 q = p - pos;
            float sq = dot(q, q);
            h = sq >= f[17] * f[17] && sq <= f[18] * f[18];
        }
        consider(best, h, p, o, k, 0, key);
        break;
    }
    case SR_OBJECT_CYLINDER: {
        m3 A = ldm(f + SR_F_AXES);
        consider(best, cyl_test(o, d, pos, A, f[SR_F_P0], f[SR_F_P0 + 1], max_lambda, p), p, o, k, 0, key);
        break;
    }
    case SR_OBJECT_RECTANGLE: {
        m3 A = ldm(f + SR_F_AXES);
        consider(best, rect_test(o, d, pos, A.c0, A.c1, A.c2, f[17], f[18], max_lambda, p), p, o, k, 0, key);
        break;
    }
    case SR_OBJECT_BOX: {
        // box_intersect frag:586-695: the closest face, earlier faces win ties
        Hit bh = no_hit();
#pragma unroll
        for (int face = 0; face < 6; face++) {
            const float* g = f + SR_F_BOX_FACE0 + SR_F_FACE_STRIDE * face;
            bool h = rect_test(o, d, ld3(g), ld3(g + 3), ld3(g + 6), ld3(g + 9), g[12], g[13], max_lambda, p);
            consider(bh, h, p, o, k, face, face);
        }
        if (bh.slot != SLOT_NONE) consider(best, true, bh.p, o, k, bh.face, key);
        break;
    }
    default:
        break;
    }
}

// Clearance budget (not part of the reference; exact by margin). Every point
// of the chords that follow an anchor point A on the ray's polyline lies
// within T = (summed chord lengths since A) of A, so while
//     T * (1 + 3 mu) < min_k(|A - c_k| - rb_k) - 1.8 mu |A|
// no chord can come within rb_k (bounding radius + the per-chord rounding
// margin mu * (|o|_1 + len + 1 + |c|_1 + R), |o|_1 <= 1.8 (|A| + T)) of any
// budgeted object k or of the black hole: their exact tests cannot hit and
// are skipped. Computed with hardware sqrt: its error is far below the margin.
// Planar primitives (disk, hollow disk, rectangle) also accept only points
// within ~eps*S of their plane (p = o + d*num/den leaves |n.(p - pos)| ~ eps*|num|),
// so their clearance is the larger of the bounding-sphere and plane distances:
// a thin accretion disk around the hole no longer exhausts the budget.
#define SR_BUDGET_SLACK 1.006f
__device__ __forceinline__ float anchor_budget(const sr_dev_scene* __restrict__ sc, f3 A) {
    const float a = __builtin_amdgcn_sqrtf(dot(A, A));
    float B = a - (1.0f + SR_MU_QUADRATIC * 3.0f);  // black hole: c = 0, R = 1
    const int nb = sc->num_budget;
    for (int j = 0; j < nb; j++) {
        const sr_dev_obj& ob = sc->objs[sc->budget_idx[j]];
        f3 w = A - ld3(ob.bc);
        float clear = __builtin_amdgcn_sqrtf(dot(w, w)) - ob.rb;
        if (ob.type == SR_OBJECT_DISK || ob.type == SR_OBJECT_HOLLOW_DISK || ob.type == SR_OBJECT_RECTANGLE) {
            f3 q = A - ld3(ob.f + SR_F_POS);
            clear = fmaxf(clear, fabsf(dot(q, ld3(ob.f + SR_F_AXES + 3))) - ob.mp);
        }
        B = fminf(B, clear);
    }
    return B - 1.8f * SR_MU_QUADRATIC * a;
}

// intersect(), frag:755-814: the closest hit along [o, o + max_lambda*d]
// (max_lambda < 0: unbounded). `cull` enables skipping exact tests that
// provably miss: budgeted objects and the black hole unless `near`, chord-
// culled objects when the chord misses their bounding sphere.
__device__ __forceinline__ Hit closest_hit(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs, f3 o, f3 d,
                           float max_lambda, bool cull, bool near) {
    Hit best = no_hit();
    f3 p;
    cull = cull && max_lambda >= 0.0f;
    if (!cull || near)  // BLACK_HOLE: sphere of radius 1 at the origin (frag:104, 757)
        consider(best, sphere_test(o, d, F3(0.0f, 0.0f, 0.0f), 1.0f, max_lambda, p), p, o, SLOT_BH, 0, KEY_BH);

    if (sc->tr_visible) {  // frag:760-803
        const float* t = sc->tr_flat;
        m3 A = ldm(t + 3);
        consider(best, cyl_test(o, d, ld3(t), A, t[12], t[13], max_lambda, p), p, o, SLOT_TR_FLAT, 0, KEY_TR_FLAT);
        int ns = sc->tr_num_segments;
        for (int s = 0; s < ns; s++) {
            const float* g = segs + s * SR_SEG_FLOATS;
            m3 B = ldm(g + 3);
            consider(best, cyl_test(o, d, ld3(g), B, g[12], g[13], max_lambda, p), p, o, SLOT_TR_CURVED, 0,
                     KEY_TR_CURVED0 + s);
        }
    }

    if (!cull) {
        const int n = sc->num_objects;
        for (int k = 0; k < n; k++) test_object(best, sc->objs[k], k, o, d, max_lambda);
        return best;
    }
    // objects tested every step (planes: always; cylinders: unless the chord
    // misses their bounding sphere), then the budgeted ones when near
    const float S = (fabsf(o.x) + fabsf(o.y) + fabsf(o.z)) + max_lambda + 1.0f;
    const int ns = sc->num_step;
    for (int j = 0; j < ns; j++) {
        const int k = sc->step_idx[j];
        const sr_dev_obj& ob = sc->objs[k];
        if (ob.kind == SR_KIND_CHORD && !may_hit(ob, o, d, max_lambda, S)) continue;
        test_object(best, ob, k, o, d, max_lambda);
    }
    if (near) {
        const int nb = sc->num_budget;
        for (int j = 0; j < nb; j++) {
            const int k = sc->budget_idx[j];
            const sr_dev_obj& ob = sc->objs[k];
            if (!may_hit(ob, o, d, max_lambda, S)) continue;
            test_object(best, ob, k, o, d, max_lambda);
        }
    }
    return best;
}

// ---- textures ------------------------------------------------
// UNORM8 -> float: b / 255 correctly rounded, tabulated at compile time (the
// constant-folded quotients are the IEEE results of the runtime division).
struct Unorm8Table {
    float v[256];
    constexpr Unorm8Table() : v() {
        for (int i = 0; i < 256; i++) v[i] = (float)i / 255.0f;
    }
};
__constant__ constexpr Unorm8Table k_unorm8{};

__device__ __forceinline__ f4 texel(const uint32_t* base, int w, int x, int y) {
    uint32_t v = base[(size_t)y * (size_t)w + (size_t)x];
    return F4(k_unorm8.v[v & 0xffu], k_unorm8.v[(v >> 8) & 0xffu], k_unorm8.v[(v >> 16) & 0xffu],
              k_unorm8.v[v >> 24]);
}
__device__ __forceinline__ int wrap_rep(float f, int n) {
    int i = (int)f;
    int m = i % n;
    return m < 0 ? m + n : m;
}
__device__ __forceinline__ f4 lerp4(f4 a, f4 b, float t) {
    return F4(a.x + (b.x - a.x) * t, a.y + (b.y - a.y) * t, a.z + (b.z - a.z) * t, a.w + (b.w - a.w) * t);
}
__device__ f4 bilinear(const uint32_t* base, int w, int h, float u, float v, int mode) {
    float s = u * (float)w - 0.5f;
    float t = v * (float)h - 0.5f;
    if (!(fabsf(s) < 16777216.0f)) s = 0.0f;
    if (!(fabsf(t) < 16777216.0f)) t = 0.0f;
    float fs = floorf(s), ft = floorf(t);
    float a = s - fs, b = t - ft;
    int x0 = wrap_rep(fs, w), x1 = wrap_rep(fs + 1.0f, w);
    int y0 = wrap_rep(ft, h), y1 = wrap_rep(ft + 1.0f, h);
    f4 t00 = texel(base, w, x0, y0), t10 = texel(base, w, x1, y0);
    f4 t01 = texel(base, w, x0, y1), t11 = texel(base, w, x1, y1);
    if (mode == SR_FILTER_WEIGHTED) {
        float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b);
        float w01 = (1.0f - a) * b, w11 = a * b;
        return F4(((t00.x * w00 + t10.x * w10) + t01.x * w01) + t11.x * w11,
                  ((t00.y * w00 + t10.y * w10) + t01.y * w01) + t11.y * w11,
                  ((t00.z * w00 + t10.z * w10) + t01.z * w01) + t11.z * w11,
                  ((t00.w * w00 + t10.w * w10) + t01.w * w01) + t11.w * w11);
    }
    return lerp4(lerp4(t00, t10, a), lerp4(t01, t11, a), b);
}
// get_bg, frag:829-837
__device__ __forceinline__ f4 get_bg(const sr_dev_frame& fr, const Tex& tx, f3 dir) {
    float u = t_atan2(dir.z, dir.x) / SR_PI;
    if (u < 0.0f) u += 2.0f;
    u *= 0.5f;
    float v = t_asin(dir.y) / SR_PI + 0.5f;
    if (!tx.bg || fr.bg_w <= 0 || fr.bg_h <= 0) return F4(0.0f, 0.0f, 0.0f, 1.0f);
    return bilinear(tx.bg, fr.bg_w, fr.bg_h, u, v, fr.filter_mode);
}
__device__ f4 tex_array(const sr_dev_frame& fr, const Tex& tx, f2 uv, int layer) {
    if (!tx.arr || fr.arr_w <= 0 || fr.arr_h <= 0 || fr.arr_layers <= 0) return F4(0.0f, 0.0f, 0.0f, 1.0f);
    if (layer < 0) layer = 0;
    if (layer > fr.arr_layers - 1) layer = fr.arr_layers - 1;
    const uint32_t* base = tx.arr + (size_t)layer * (size_t)fr.arr_w * (size_t)fr.arr_h;
    return bilinear(base, fr.arr_w, fr.arr_h, uv.x, uv.y, fr.filter_mode);
}

// ---- tangent spaces (frag:208-333) + calculate_lighting (frag:365-438) ---------
// The reference builds the full [tangent, bitangent, normal] frame for every
// hit; only the normal and uv reach the lighting unless a normal map is used,
// so the frame's tangent columns (cos/sin of phi and theta) are built on
// demand by surface_frame() with the same expressions.
struct Surface {
    f3 n;         // tangent_space[2]
    f2 uv;        // tangent_coordinates
    float phi;    // sphere / disks / cylinder
    float theta;  // sphere
};

__device__ __forceinline__ float phi_of(f3 local) {
    float phi = t_atan2(local.x, local.z);
    if (phi < 0.0f) phi += 2.0f * SR_PI;
    return phi;
}

__device__ __forceinline__ f2 planar_uv(f3 p, f3 pos, const m3& A, float w, float h, bool scaled) {
    f3 local = mtv(A, p - pos);
    f2 uv = scaled ? F2(local.x / w, local.z / h) : F2(local.x, local.z);
    uv.y = 1.0f - uv.y;
    return uv;
}

__device__ __forceinline__ m3 box_face(const float* f, int face) {
    const float* g = f + SR_F_BOX_FACE0 + SR_F_FACE_STRIDE * face;
    m3 F;
    F.c0 = ld3(g + 3);
    F.c1 = ld3(g + 6);
    F.c2 = ld3(g + 9);
    return F;
}

__device__ Surface surface_of(const sr_dev_obj& ob, const Hit& h) {
    const float* f = ob.f;
    f3 pos = ld3(f + SR_F_POS);
    m3 A = ldm(f + SR_F_AXES);
    f3 disp = h.p - pos;
    Surface s;
    s.phi = 0.0f;
    s.theta = 0.0f;
    switch (ob.type) {
    case SR_OBJECT_SPHERE: {  // frag:209-232
        s.n = nrm(disp);
        f3 local = mtv(A, disp);
        s.phi = phi_of(local);
        s.theta = t_asin(local.y / f[SR_F_P0]);
        s.uv = F2(s.phi / (2.0f * SR_PI), s.theta / SR_PI + 0.5f);
        return s;
    }
    case SR_OBJECT_DISK:
    case SR_OBJECT_HOLLOW_DISK: {  // frag:249-295
        f3 local = mtv(A, disp);
        s.phi = phi_of(local);
        if (ob.type == SR_OBJECT_DISK) s.uv = F2(len(local) / f[17], s.phi / (2.0f * SR_PI));
        else s.uv = F2((len(local) - f[17]) / (f[18] - f[17]), s.phi / (2.0f * SR_PI));
        s.n = A.c1;
        return s;
    }
    case SR_OBJECT_CYLINDER: {  // frag:297-318
        s.n = nrm(disp);
        f3 local = mtv(A, disp);
        s.phi = phi_of(local);
        s.uv = F2(s.phi / (2.0f * SR_PI), local.y / f[SR_F_P0]);
        return s;
    }
    case SR_OBJECT_RECTANGLE:  // frag:320-333
        s.uv = planar_uv(h.p, pos, A, f[17], f[18], true);
        s.n = A.c1;
        return s;
    case SR_OBJECT_BOX: {  // frag:665-692
        const float* g = f + SR_F_BOX_FACE0 + SR_F_FACE_STRIDE * h.face;
        m3 F = box_face(f, h.face);
        s.uv = planar_uv(h.p, ld3(g), F, g[12], g[13], true);
        switch (h.face) {
        case 0: s.uv.x += 1.0f; break;
        case 1: s.uv.x += 1.0f; s.uv.y += 2.0f; break;
        case 2: s.uv.x += 1.0f; s.uv.y += 1.0f; break;
        case 3: s.uv.x += 3.0f; s.uv.y += 1.0f; break;
        case 4: s.uv.y += 1.0f; break;
        default: s.uv.x += 2.0f; s.uv.y += 1.0f; break;
        }
        s.uv.x /= 4.0f;
        s.uv.y /= 3.0f;
        s.n = F.c1;
        return s;
    }
    default:  // plane, frag:234-247
        s.uv = planar_uv(h.p, pos, A, 1.0f, 1.0f, false);
        s.n = A.c1;
        return s;
    }
}

// The full tangent_space matrix (normal-map path only); n is the (possibly
// flipped) normal column.
__device__ __forceinline__ m3 surface_frame(const sr_dev_obj& ob, const Hit& h, const Surface& s, f3 n) {
    const float* f = ob.f;
    m3 A = ldm(f + SR_F_AXES);
    m3 ts;
    ts.c2 = n;
    switch (ob.type) {
    case SR_OBJECT_SPHERE:
        ts.c0 = mv(A, F3(t_cos(s.phi), 0.0f, -t_sin(s.phi)));
        ts.c1 = mv(A, F3(t_sin(s.phi) * t_cos(s.theta), t_sin(s.theta), t_cos(s.phi) * t_cos(s.theta)));
        return ts;
    case SR_OBJECT_DISK:
    case SR_OBJECT_HOLLOW_DISK:
        ts.c0 = nrm(h.p - ld3(f + SR_F_POS));
        ts.c1 = mv(A, F3(t_cos(s.phi), 0.0f, -t_sin(s.phi)));
        return ts;
    case SR_OBJECT_CYLINDER:
        ts.c0 = mv(A, F3(t_cos(s.phi), 0.0f, -t_sin(s.phi)));
        ts.c1 = A.c1;
        return ts;
    case SR_OBJECT_BOX: {
        m3 F = box_face(f, h.face);
        ts.c0 = F.c0;
        ts.c1 = -F.c2;
        return ts;
    }
    default:  // plane, rectangle
        ts.c0 = A.c0;
        ts.c1 = -A.c2;
        return ts;
    }
}

// Called by shade() for lanes that share one (slot, face): both are re-read as
// wave-uniform values so the object record is fetched with scalar loads.
__device__ __forceinline__ f4 shade_hit(const sr_dev_scene* __restrict__ sc, const sr_dev_frame& fr, const Tex& tx,
                        Hit h, f3 view_dir) {
    h.slot = __builtin_amdgcn_readfirstlane(h.slot);
    h.face = __builtin_amdgcn_readfirstlane(h.face);
    if (h.slot == SLOT_BH) return F4(0.0f, 0.0f, 0.0f, 1.0f);
    if (h.slot == SLOT_TR_CURVED)
        return F4(sc->tr_curved_color[0], sc->tr_curved_color[1], sc->tr_curved_color[2], sc->tr_curved_color[3]);
    if (h.slot == SLOT_TR_FLAT)
        return F4(sc->tr_flat_color[0], sc->tr_flat_color[1], sc->tr_flat_color[2], sc->tr_flat_color[3]);
#ifdef SR_TIMING_CONST_SHADE  // timing experiments only: wrong colours
    return F4(0.5f, 0.5f, 0.5f, 1.0f);
#endif
    const sr_dev_obj& ob = sc->objs[h.slot];
    int mi = ob.material_index;
    if (mi < 0 || mi >= SR_MAX_MATERIALS) mi = 0;
    const sr_material& m = sc->materials[mi];
    Surface s = surface_of(ob, h);
    if (m.flip_normals) s.n = s.n * -1.0f;
    if (!m.double_sided_normals && dot(s.n, view_dir) < 0.0f) return F4(0.0f, 0.0f, 0.0f, 0.0f);
    f2 uv = s.uv;
    const bool is_plane = ob.type == SR_OBJECT_PLANE;
    int pi = ob.index;
    if (pi < 0 || pi >= SR_MAX_PLANES) pi = 0;
    const sr_plane& pl = sc->planes[pi];
    if (m.swap_uvs) uv = F2(uv.y, uv.x);
    if (m.invert_uv_x) uv.x = (is_plane ? pl.texture_size[0] : 1.0f) - uv.x;
    if (m.invert_uv_y) uv.y = (is_plane ? pl.texture_size[1] : 1.0f) - uv.y;

    f4 base = F4(m.color[0], m.color[1], m.color[2], m.color[3]);
    if (m.texture_index >= 0) {
        int ti = m.texture_index < SR_MAX_TEXTURES ? m.texture_index : 0;
        f2 r = F2((uv.x * sc->texture_sizes[ti][0]) / sc->max_texture_size[0],
                  (uv.y * sc->texture_sizes[ti][1]) / sc->max_texture_size[1]);
        bool render = true;
        if (is_plane) {
            r = F2(r.x - pl.texture_offset[0], r.y - pl.texture_offset[1]);
            f2 puv = F2(r.x / pl.texture_size[0], r.y / pl.texture_size[1]);
            r.x = r.x - pl.texture_size[0] * floorf(r.x / pl.texture_size[0]);
            r.y = r.y - pl.texture_size[1] * floorf(r.y / pl.texture_size[1]);
            r = F2(r.x / pl.texture_size[0], r.y / pl.texture_size[1]);
            render = pl.repeat_texture || ((puv.x >= 0.0f && puv.x <= 1.0f) && (puv.y >= 0.0f && puv.y <= 1.0f));
        }
        if (render) base = tex_array(fr, tx, r, m.texture_index);
    }
    f3 brgb = F3(base.x, base.y, base.z);
    f3 col = brgb * m.ambient;
    f3 normal = s.n;
    if (m.normal_map_index >= 0) {
        int ni = m.normal_map_index < SR_MAX_TEXTURES ? m.normal_map_index : 0;
        f2 r = F2((uv.x * sc->texture_sizes[ni][0]) / sc->max_texture_size[0],
                  (uv.y * sc->texture_sizes[ni][1]) / sc->max_texture_size[1]);
        f4 nm = tex_array(fr, tx, r, m.normal_map_index);
        normal = nrm(mv(surface_frame(ob, h, s, s.n), F3(nm.x, nm.y, nm.z)));
    }
    int nl = sc->num_lights;
    if (nl > SR_MAX_LIGHTS) nl = SR_MAX_LIGHTS;
    for (int i = 0; i < nl; i++) {
        const sr_light& L = sc->lights[i];
        f3 lpos = ld3(L.transform.pos);
        f3 lcol = ld3(L.color);
        f3 ldir = nrm(lpos - h.p);
        float dist = len(lpos - h.p);
        float att = 1.0f / (L.attenuation_constant + L.attenuation_linear * dist +
                            L.attenuation_quadratic * dist * dist);
        float diff = gmax(dot(normal, ldir), 0.0f);
        f3 diffuse = (lcol * (m.diffuse * diff)) * brgb;
        f3 I = -ldir;
        f3 refl = I - normal * (2.0f * dot(normal, I));
        float spec = t_pow(gmax(dot(view_dir, refl), 0.0f), m.shininess);
        f3 specular = lcol * (m.specular * spec);
        col = col + ((diffuse + specular) * att) * L.intensity;
    }
    return F4(col.x, col.y, col.z, base.w);
}

// calculate_lighting for the active lanes' hits: a waterfall over the distinct
// (object, face) keys present in the wave, so shade_hit sees wave-uniform
// object data (scalar loads) instead of per-lane gathers of scene records.
__device__ __forceinline__ f4 shade(const sr_dev_scene* __restrict__ sc, const sr_dev_frame& fr, const Tex& tx,
                                    const Hit& h, f3 view_dir) {
    const int key = h.slot * 8 + h.face;
    f4 c;
    for (;;) {
        const int first = __builtin_amdgcn_readfirstlane(key);
        if (key == first) {
            c = shade_hit(sc, fr, tx, h, view_dir);
            break;
        }
    }
    return c;
}

__device__ __forceinline__ f4 intersect_color(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                              const sr_dev_frame& fr, const Tex& tx, f3 o, f3 d,
                                              float max_lambda, bool cull, bool near) {
    Hit h = closest_hit(sc, segs, o, d, max_lambda, cull, near);
    if (h.slot == SLOT_NONE) return F4(0.0f, 0.0f, 0.0f, 0.0f);
    return shade(sc, fr, tx, h, -d);
}

__device__ __forceinline__ uint32_t unorm8(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x >= 1.0f) return 255u;
    return (uint32_t)floorf(x * 255.0f + 0.5f);
}

}  // namespace

// Exit modes of the step loop
#define MODE_DONE 1   // FragColor final
#define MODE_FLAT 2   // unbounded intersect(ray), then get_bg if alpha != 1 (frag:874-876, 895-897, 903-905)
#define MODE_BG 3     // get_bg(ray.dir) (frag:921-922 break, 935)

#ifndef SR_MIN_WAVES_PER_EU
#define SR_MIN_WAVES_PER_EU 1
#endif

template <bool DEBUG>
__global__ __launch_bounds__(256, SR_MIN_WAVES_PER_EU) void sr_geodesic_kernel(const sr_dev_scene* __restrict__ sc,
                                                          const float4* __restrict__ tbl,
                                                          const float* __restrict__ segs,
                                                          const uint32_t* __restrict__ bg,
                                                          const uint32_t* __restrict__ arr,
                                                          sr_dev_frame fr, uint8_t* __restrict__ out,
                                                          size_t pitch, float* __restrict__ dbg_rgba,
                                                          int32_t* __restrict__ dbg_steps) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int px = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int k = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (px >= fr.width || k >= fr.nrows) return;
    const int py = fr.row_base + (k / fr.block_rows) * fr.block_stride + (k % fr.block_rows);
    if (py >= fr.height) return;

    Tex tx;
    tx.bg = bg;
    tx.arr = arr;
    const bool cull = fr.cull != 0;

    // full_screen_quad.vert:7-10: uv = NDC of the pixel centre
    f2 uv = F2((float)(2 * px + 1) / (float)fr.width - 1.0f, (float)(2 * py + 1) / (float)fr.height - 1.0f);
    f4 frag = F4(0.0f, 0.0f, 0.0f, 0.0f);
    if (fr.crosshair) {  // frag:845-857
        float hx = fabsf(uv.x * fr.res_x / 2.0f), hy = fabsf(uv.y * fr.res_y / 2.0f);
        if ((hx < 1.0f && hy > 5.0f && hy < 15.0f) || (hy < 1.0f && hx > 5.0f && hx < 15.0f))
            frag = F4(0.5f, 0.5f, 0.5f, 0.5f);
    }
    // frag:859-863
    f2 uvv = F2(uv.x, uv.y * fr.res_y / fr.res_x);
    m3 cam = ldm(fr.cam_axes);
    f3 ro = ld3(fr.cam_pos);
    f3 rd = nrm(mv(cam, F3(uvv.x, uvv.y, fr.ray_forward)));
    f3 nv = nrm(ro);
    int steps = 0;
    int mode;
    const bool flat = fr.raytrace_type == SR_RAYTRACE_FLAT ||
                      (fr.raytrace_type == SR_RAYTRACE_HALF_WIDTH && uv.x > 2.0f * fr.curved_percentage + -1.0f) ||
                      (fr.raytrace_type == SR_RAYTRACE_HALF_HEIGHT && uv.y > 2.0f * fr.curved_percentage + -1.0f);
    if (flat || fabsf(dot(rd, nv)) >= 1.0f - SR_EPS) {
        mode = MODE_FLAT;
    } else if (fr.percent_black >= 0.0f &&
               [&] {  // rand(uv_vec) <= percent_black, frag:839-841, 879; rand is in [0, 1)
                   float x = t_sin(uvv.x * 12.9898f + uvv.y * 78.233f) * 43758.5453f;
                   return x - floorf(x) <= fr.percent_black;
               }()) {
        mode = MODE_DONE;
    } else {
        // frag:883-889
        f3 tv = nrm(cross(cross(nv, rd), nv));
        float u = 1.0f / len(ro);
        float du = -u * dot(rd, nv) / dot(rd, tv);
        mode = MODE_BG;
        const int N = fr.max_steps;
        // clearance budget of the polyline since the last anchor (anchor_budget)
        float T = 0.0f;
        float B = cull ? anchor_budget(sc, ro) : 0.0f;
        int i = 0;
        // Rounds: integrate until this lane's chord hits something (or the ray
        // ends), shade the wave's pending hits together, and resume the lanes
        // whose hit was not opaque (frag:930-932) at the next step. Shading
        // stays out of the step loop's registers and runs once per round.
        for (;;) {
            Hit hit = no_hit();
            for (; i < N; i++) {
                // {step_size, step_size / 6, cos phi, sin phi} of step i (wave-uniform)
                const float4 e = tbl[i];
                steps++;
                if (u < fr.u_f) {  // frag:891-912
                    f3 q;
                    if (!sphere_test(ro, rd, F3(0.0f, 0.0f, 0.0f), fr.uf_radius, -1.0f, q)) {
                        mode = MODE_FLAT;
                        break;
                    }
                    nv = nrm(q);
                    if (fabsf(dot(rd, nv)) >= 1.0f - SR_EPS) {
                        mode = MODE_FLAT;
                        break;
                    }
                    tv = nrm(cross(cross(nv, rd), nv));
                    u = 1.0f / len(q);
                    du = -u * dot(rd, nv) / dot(rd, tv);
                }
                // frag:914-919
                const float h = e.x;
                {  // rk4_step, frag:341-355 (`delta_phi / 6.` is e.y, computed on the host)
                    float k1 = du;
                    float l1 = -u * (1.0f - 1.5f * u);
                    float k2 = du + 0.5f * l1 * h;
                    float ua = u + 0.5f * k1 * h;
                    float l2 = -ua * (1.0f - 1.5f * ua);
                    float k3 = du + 0.5f * l2 * h;
                    float ub = u + 0.5f * k2 * h;
                    float l3 = -ub * (1.0f - 1.5f * ub);
                    float k4 = du + l3 * h;
                    float uc = u + k3 * h;
                    float l4 = -uc * (1.0f - 1.5f * uc);
                    u += e.y * (k1 + 2.0f * k2 + 2.0f * k3 + k4);
                    du += e.y * (l1 + 2.0f * l2 + 2.0f * l3 + l4);
                }
                if (u < 0.0f) break;  // frag:921-922 -> get_bg
                // frag:924-930
                f3 prev = ro;
                ro = (nv * e.z + tv * e.w) / u;
                f3 delta = ro - prev;
                float seg = len(delta);
                rd = delta / seg;
                T += seg;
                // wave-uniform: a wave runs the near path if any lane needs it, so
                // every active lane tests and re-anchors together (keeps the
                // lanes' anchors in step and the skipped steps coherent)
                const bool near = __ballot(!(T * SR_BUDGET_SLACK < B)) != 0;
                hit = closest_hit(sc, segs, prev, rd, seg, cull, near);
                if (cull && near) {  // re-anchor at the chord's end
                    B = anchor_budget(sc, ro);
                    T = 0.0f;
                }
                if (hit.slot != SLOT_NONE) break;
            }
            if (hit.slot == SLOT_NONE) break;
            f4 c = shade(sc, fr, tx, hit, -rd);
            frag = frag + c;
            if (c.w == 1.0f) {  // frag:932
                mode = MODE_DONE;
                break;
            }
            i++;
        }
    }
    if (mode == MODE_FLAT) {
        f4 c = intersect_color(sc, segs, fr, tx, ro, rd, -1.0f, false, true);
        frag = frag + c;
        mode = c.w != 1.0f ? MODE_BG : MODE_DONE;
    }
    if (mode == MODE_BG) frag = frag + get_bg(fr, tx, rd);

    uint32_t pix = unorm8(frag.x) | (unorm8(frag.y) << 8) | (unorm8(frag.z) << 16) | (unorm8(frag.w) << 24);
    if (out) *reinterpret_cast<uint32_t*>(out + (size_t)k * pitch + (size_t)px * 4) = pix;
    if (DEBUG) {
        size_t i = (size_t)k * (size_t)fr.width + (size_t)px;
        if (dbg_rgba) {
            dbg_rgba[4 * i + 0] = frag.x;
            dbg_rgba[4 * i + 1] = frag.y;
            dbg_rgba[4 * i + 2] = frag.z;
            dbg_rgba[4 * i + 3] = frag.w;
        }
        if (dbg_steps) dbg_steps[i] = steps;
    }
}

extern "C" hipError_t sr_launch_geodesic(const sr_dev_scene* sc, const float4* tbl, const float* segs,
                                         const uint32_t* bg, const uint32_t* arr, const sr_dev_frame* fr,
                                         uint8_t* out, size_t pitch, float* dbg_rgba, int32_t* dbg_steps,
                                         hipStream_t stream) {
    dim3 block(256);
    dim3 grid((fr->width + 15) / 16, (fr->nrows + 15) / 16);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    if (dbg_rgba || dbg_steps)
        hipLaunchKernelGGL(sr_geodesic_kernel<true>, grid, block, 0, stream, sc, tbl, segs, bg, arr, *fr, out,
                           pitch, dbg_rgba, dbg_steps);
    else
        hipLaunchKernelGGL(sr_geodesic_kernel<false>, grid, block, 0, stream, sc, tbl, segs, bg, arr, *fr, out,
                           pitch, dbg_rgba, dbg_steps);
    return hipGetLastError();
}
