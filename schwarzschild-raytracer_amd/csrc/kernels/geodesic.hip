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

#include <cstdint>
#include <type_traits>

// constant address space: wave-uniform loads through it are scalar loads
typedef float sr_v4f __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) sr_v4f sr_cfloat4;
__device__ __forceinline__ float4 ldc(const sr_cfloat4* p) {
    const sr_v4f v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}

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
__device__ __forceinline__ float t_sin(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float t_cos(float x) { return (float)cos((double)x); }
// asin / atan2 / pow are called only by the shading kernels: out of line, the
// binary64 code's registers do not add to the lighting's (sr_shade_kernel 215
// -> 117 VGPRs, 2 -> 4 waves per SIMD: 0.104 -> 0.060 ms per headline frame,
// profiles/r02/s7_shade_noinline.jsonl)
__device__ __attribute__((noinline)) float t_asin(float x) { return (float)asin((double)x); }
__device__ __attribute__((noinline)) float t_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
__device__ __attribute__((noinline)) float t_pow(float x, float y) { return (float)pow((double)x, (double)y); }

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
    const uint8_t* __restrict__ opq;  // texture-array opacity bitmap (sr_api.cpp make_opacity_map)
};

#include "probes.h"

// ---- primitive tests: return the reference's is_hit and fill p ------------
// sphere_intersect, frag:457-478 (r2: the float square r * r of the radius):
// whether it hits, and its lambda (the point is o + d * lam, sphere_test_r2)
__device__ __forceinline__ bool sphere_lambda_r2(f3 o, f3 d, f3 c, float r2, float max_lambda, float& lam_out) {
    f3 oc = o - c;
    float b = dot(d, oc);
    float D = b * b - dot(oc, oc) + r2;
    if (D < 0.0f) return false;
    float sq = sqrtf(D);
    float first = -dot(d, oc);
    float l1 = first - sq, l2 = first + sq;
    float lam = -1.0f;  // min_positive, frag:441-454
    if (l1 > 0.0f && l2 > 0.0f) lam = gmin(l1, l2);
    else if (l1 > 0.0f) lam = l1;
    else if (l2 > 0.0f) lam = l2;
    lam_out = lam;
    return lam >= 0.0f && (max_lambda < 0.0f || lam <= max_lambda);
}
__device__ __forceinline__ bool sphere_test_r2(f3 o, f3 d, f3 c, float r2, float max_lambda, f3& p) {
    float lam;
    const bool hit = sphere_lambda_r2(o, d, c, r2, max_lambda, lam);
    if (hit) p = o + d * lam;
    return hit;
}
__device__ __forceinline__ bool sphere_test(f3 o, f3 d, f3 c, float r, float max_lambda, f3& p) {
    return sphere_test_r2(o, d, c, r * r, max_lambda, p);
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

// p by reference: callers pass the point their own test argument writes
// (consider(best, test(..., p), p, ...)), and the order in which a call's
// arguments are evaluated is unspecified, so a by-value copy could be taken
// before the test ran.
__device__ __forceinline__ void consider(Hit& best, bool hit, const f3& p, f3 o, int slot, int face, int key) {
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

// The lateral margin of a cylinder test (device_scene.h SR_CYL_QMARGIN, round
// 6): an accepted point lies within this of the lateral surface for every
// chord direction, Sc >= S + |pos|_1 of the chord.
#ifndef SR_REACH_LAT  // slot_reachable's cylinder margin: lat_margin (1) or round 2's over |d_perp|^2 (0;
                      // conservative too: 1 measured no faster, profiles/r06/s43)
#define SR_REACH_LAT 0
#endif
__device__ __forceinline__ float lat_margin(float Sc, float r) {
    return fminf(SR_CYL_QMARGIN * Sc * Sc * __builtin_amdgcn_rcpf(r), 2.0f * SR_MU_QUADRATIC * (Sc + r)) * 1.001f;
}
// The same for a chord of length at most len (round 6, the test rays): an
// accepted point has frame-lateral distance ~r at a parameter in [0, len], so
// the chord origin's lateral offset |X| is at most (r + len) (1 + 1e-3), and
// the discriminant's radius r' obeys |r'^2 - r^2| <= 12 u q, q = (r + len)^2 +
// r^2; the origin's and the point's own roundings add ~3 u Sc. In the
// frame's coordinates (world distances: the bound's scale |M^-1| |M|^2).
// Constants ~8x the derivation's (tests/test_cyl_lateral_margin.py: at most
// 1/40 of this).
__device__ __forceinline__ float lat_margin_len(float len, float Sc, float r) {
    const float rl = r + len;
    const float q = __builtin_fmaf(rl, rl, r * r);
    return (fminf(6.0e-6f * q * __builtin_amdgcn_rcpf(r), 7.0e-3f * __builtin_amdgcn_sqrtf(q)) + 2.0e-6f * Sc) * 1.001f;
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
        // an accepted point lies within lat_margin of the lateral surface,
        // whatever the chord's direction (round 6; the root's error along
        // the chord, S^2 / (r |d_perp|^2), moves it along the surface)
        const float r = ob.f[SR_F_P0 + 1];
        if (!(r > 0.0f)) return true;
        R = R + lat_margin(S + ob.pl1, r);  // |o - pos| <= S + |pos|_1
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

// Clearance budgets (not part of the reference; exact by margin). Budget slot
// 0 is the black hole, slot j >= 1 the object sc->objs[sc->budget_idx[j - 1]].
// From an anchor point A on the ray's polyline, every point of the chords that
// follow lies within T = (summed chord lengths since A) of A, so while
//     T * SR_PATH_SLACK < clearance_j(A)
// no chord can come within the per-chord acceptance region of slot j and its
// exact test cannot hit: it is skipped. clearance_j(A) is
//     max(|A - c| - rb, |n.(A - pos)| - mp)  (planar objects: the plane bound)
//     - 1.8 mu |A|                           (chord origins |o|_1 <= 1.8 (|A| + T); mu = slot_mu)
// with rb = bounding radius + mu_q (1 + |c|_1 + R) and the path slack covering
// the T-proportional part of the rounding margins. Cylinders also subtract
// their quadratic margin SR_CYL_QMARGIN S^2 / (r SR_BUDGET_DPMIN) for the
// largest S a chord of the window can have (a window is at most the
// clearance before this margin, capped at SR_BUDGET_TMAX); chords closer than
// SR_BUDGET_DPMIN to the cylinder axis direction are covered by the slab
// budget instead (clearance_slab, chord_parallel). Computed with
// hardware sqrt: its error is far below the margins.
#define SR_PATH_SLACK 1.01f
// Ball form of the budgets (SR_BALL): a budget bounds the
// displacement from the last budget event's end point instead of the path
// since it, so the step loop tests the step's end point against a ball
// (sign of a quadratic in u, no reciprocal or square root) instead of
// summing chord-length bounds. Every margin below that assumed chords within
// a window of path W holds for chords within a ball of radius W, except the
// chord length (up to 2 W) and the directional plane window (a path bound,
// converted in plane_window).
#ifndef SR_NEAR
#define SR_NEAR 1.0f
#endif
#ifndef SR_CYL_INSIDE
#define SR_CYL_INSIDE 1
#endif
#ifndef SR_XPLANE  // orbital-plane exclusion of bounded slots (budget_frame)
#define SR_XPLANE 1
#endif
// The margin factor of a slot's distance tests: a planar primitive's
// per-chord factor (SR_MU_PLANAR: it accepts a chord point within a few eps
// S of its plane and bounds), the quadratic one for spheres and cylinders
// (sr_api.cpp set_bound; the slab and in-plane margins sl.mp use the same).
__device__ __forceinline__ float slot_mu(const sr_dev_slot& sl) {
    return sl.type == SR_OBJECT_CYLINDER ? SR_MU_QUADRATIC : sl.mu;
}
__device__ __forceinline__ float clearance_obj(const sr_dev_slot& sl, f3 A, float a) {
    float c;
    {
        f3 w = A - ld3(sl.bc);
        c = __builtin_amdgcn_sqrtf(dot(w, w)) - sl.rb;
        // distance to the primitive itself (orthonormal frame). When every lane
        // of the wave is far from the object (beyond SR_NEAR (rb + 1) of its
        // bounding sphere) that sphere's distance is close to it: skip it.
        if (sl.mp < INFINITY && __ballot(c < SR_NEAR * (sl.rb + 1.0f))) {
            const f3 q = A - ld3(sl.pos);
            const float y = dot(q, ld3(sl.a1));  // along axes[1] (plane normal / height)
            float d2;
            if (sl.type == SR_OBJECT_PLANE) {
                d2 = y * y;
            } else if (sl.type == SR_OBJECT_RECTANGLE || sl.type == SR_OBJECT_BOX) {
                const float x = dot(q, ld3(sl.a0)), z = dot(q, ld3(sl.a2));
                const bool box = sl.type == SR_OBJECT_BOX;
                const float ex = fmaxf(0.0f, fmaxf(-x, x - sl.x0)), ez = fmaxf(0.0f, fmaxf(-z, z - sl.x1));
                const float ey = box ? fmaxf(0.0f, fmaxf(-y, y - sl.x2)) : y;
                d2 = ex * ex + ey * ey + ez * ez;
            } else {  // disk, hollow disk, cylinder: radial distance from axes[1]
                const float rho = __builtin_amdgcn_sqrtf(fmaxf(0.0f, dot(q, q) - y * y));
                float er, ey = y;
                if (sl.type == SR_OBJECT_DISK) {
                    er = fmaxf(0.0f, rho - sl.x0);
                } else if (sl.type == SR_OBJECT_HOLLOW_DISK) {
                    er = fmaxf(0.0f, fmaxf(sl.x0 - rho, rho - sl.x1));
                } else {
                    // the lateral surface alone (no caps): inside the tube
                    // too, its distance is |rho - radius| (SR_CYL_INSIDE; a
                    // solid cylinder's 0 made every step of a ray travelling
                    // up the tube an event)
                    er = SR_CYL_INSIDE ? fabsf(rho - sl.x1) : fmaxf(0.0f, rho - sl.x1);
                    ey = fmaxf(0.0f, fmaxf(-y, y - sl.x0));
                }
                d2 = er * er + ey * ey;
            }
            c = fmaxf(c, __builtin_amdgcn_sqrtf(d2) - sl.mp);
        }
        if (sl.type == SR_OBJECT_CYLINDER) {
            // quadratic margin SR_CYL_QMARGIN Sb^2 / (r SR_BUDGET_DPMIN), the
            // quotient folded into sl.qk on the host
            // the window's path is at most this clearance (capped): chord
            // origins stay within sqrt(3) W of A, chords within W long
            const float W = fminf(c, SR_BUDGET_TMAX);
            // (chords of a ball of radius W are up to 2 W long: SR_BALL)
            float Sb = (fabsf(A.x) + fabsf(A.y) + fabsf(A.z)) + sl.pl1 + (4.0f * W + 1.0f);
            float qm = (Sb * Sb) * sl.qk;
            c = fminf(c - qm, SR_BUDGET_TMAX);
        }
    }
    return c - 1.8f * slot_mu(sl) * a;
}
// black hole: sphere_test accepts only its entry or exit point, on the r = 1
// shell (a ray can cross the shell between steps and go on inside)
__device__ __forceinline__ float clearance_bh(float a) {
    return (fabsf(a - 1.0f) - SR_MU_QUADRATIC * 3.0f) - 1.8f * SR_MU_QUADRATIC * a;
}
// Outward lanes: past the photon orbit (u < 0.6) with u' < 0, u'' = -u (1 -
// 1.5 u) < 0 keeps u falling, so every later orbit point lies farther from
// the origin than the anchor (distance a), and every later chord stays
// beyond a x out_dip. Slot j cannot be hit again once that exceeds the
// farthest reach of its per-chord acceptance region, |c| + br + mu S (plus a
// cylinder's quadratic margin qk (S + |pos|_1)^2 while no chord of the orbit
// can be nearly parallel to its axis, bs.cm), for the chords there (S <= 2 a
// + 1 + 0.01 a^2 covers |o|_1 + len + 1 of an orbit chord at radius up to
// 110; the bound grows slower than a, so it holds for every later chord
// too). The black hole's region is the r = 1 shell; planes are unbounded. A
// new orbital frame (reseed) re-anchors every slot. Escaping rays stop
// re-anchoring the hole and the objects they have passed: events 686 k ->
// 552 k per headline frame, -6 % frame time (profiles/r02/s18_*).
__device__ __forceinline__ bool outward_clear(float cn, float br, float mu, float qk, float pl1, float a, float dip) {
    const float S = __builtin_fmaf(0.01f * a, a, __builtin_fmaf(2.0f, a, 1.0f));
    const float Sc = S + pl1;
    return a * dip > (cn + br + __builtin_fmaf(mu, S, qk * Sc * Sc)) * 1.001f;
}
// Directional budget of a planar primitive (plane, disk, annulus, rectangle):
// the path a lane needs before it can reach the primitive's acceptance slab
// |y| <= m (y: signed distance to the plane, m as in slot_reachable). The
// orbit's curvature is 1.5 u^5 / (u^2 + u'^2)^(3/2) <= 1.5 / r^2; within a
// window of path L <= a / 2 from the anchor (distance a from the origin) r >=
// a / 2, so the direction turns by at most theta0 + kappa s, kappa = 6 / a^2,
// theta0 bounding the angle between the last chord and the tangent at the
// anchor. The approach to the plane is then at most (c + theta0) L + kappa
// L^2 / 2 (c: the chord direction's component toward the plane), and chords
// between the path's points stay between their plane distances. L is that
// bound's root for |y| - m, capped at a / 2, shortened by 0.2 % for the
// polyline's length against the arc's. Returns 0 when nothing is known. Rays
// heading for a rectangle or a disk get there in one or two events instead
// of a geometric series of distance budgets: events 552 k -> 446 k per
// headline frame, -2.5 % frame time (profiles/r02/s22_*).
// SR_BALL: the budget bounds the displacement from B, not the path. Along
// the path the direction stays within theta(s) = theta0 + kappa s of the last
// chord's, so the displacement's projection on that direction after a path
// s is at least the integral of cos theta >= 1 - theta^2 / 2, i.e. s - (th1^3
// - theta0^3) / (6 kappa) = s (1 - (th1^2 + th1 theta0 + theta0^2) / 6) with
// th1 = theta(s), and it grows while theta < pi / 2. The first end point past
// a path Lc is at most one chord further (<= 1.5 a dphi: r <= 1.5 a): with
// Lc capped so that r >= a / 2 (kappa's bound) and theta <= 1.5 still hold
// there, an end point within that projection bound of B has a path below Lc.
__device__ __forceinline__ float plane_window(const sr_dev_slot& sl, f3 A, f3 B, float a, float perr, float dphi) {
    const f3 dv = B - A;
    const f3 nrm_ = ld3(sl.a1);
    const float y = dot(B - ld3(sl.pos), nrm_);
    const float len = __builtin_amdgcn_sqrtf(dot(dv, dv));
    // the chord lies within len of B: r >= a - len >= a / 2 on it, so kappa <= 6 / a^2 there too
    if (!(len > 1e-6f) || !(len < 0.5f * a) || !(a > 1.0f)) return 0.0f;
    const float il = __builtin_amdgcn_rcpf(len);
    const float a2 = a * a;
    const float kap = 6.06f * __builtin_amdgcn_rcpf(a2);  // 6 / a^2 plus 1 %
    const float c = (y > 0.0f ? -1.0f : 1.0f) * dot(dv, nrm_) * il;
    const float th0 = __builtin_fmaf(kap, len, __builtin_fmaf(2.0f * perr, il, 1e-4f));
    const float m = (sl.mp + sl.mu * __builtin_fmaf(3.1f, a, 1.0f)) * 1.001f + perr;  // S <= 3.1 a + 1 (planar)
    const float R = fabsf(y) - m;
    if (!(R > 0.0f)) return 0.0f;
    const float b = c + th0;
    const float L = (__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, 2.0f * kap * R)) - b) * (a2 * (1.0f / 6.06f));
    const float ch = 1.5f * a * dphi;  // the next chord
    const float Lc = fminf(L, fminf(__builtin_fmaf(0.5f, a, -ch), (1.5f - th0) * (a2 * (1.0f / 6.06f)) - ch));
    const float th1 = __builtin_fmaf(kap, Lc, th0);
    const float f = 1.0f - (th1 * th1 + th1 * th0 + th0 * th0) * (1.0f / 6.0f);
    return (Lc > 0.0f && f > 0.0f) ? Lc * f * 0.998f : 0.0f;
}
// The same window from a ray's start (budget_init): the anchor A is the
// camera (or a reseed point), where the orbit's tangent is the ray direction
// d itself (the frame nv, tv and u' = -u (d . nv) / (d . tv) are built from
// it: the tangent (nv cos phi + tv sin phi) / u differentiated at phi = 0 is
// parallel to d, to rounding), so theta0 is that rounding's 1e-4 and no chord
// enters it. Before it, every ray of a frame started with the distance budget
// of the same camera point, and the rectangle in front of the default camera
// (3.6 away) ran out on every wave at the same step: one event per wave.
#ifndef SR_INIT_WINDOW
#define SR_INIT_WINDOW 1
#endif
__device__ __forceinline__ float plane_window_start(const sr_dev_slot& sl, f3 A, f3 d, float a, float perr, float dphi) {
    const f3 nrm_ = ld3(sl.a1);
    const float y = dot(A - ld3(sl.pos), nrm_);
    if (!(a > 1.0f)) return 0.0f;
    const float a2 = a * a;
    const float kap = 6.06f * __builtin_amdgcn_rcpf(a2);  // 6 / a^2 plus 1 %
    const float c = (y > 0.0f ? -1.0f : 1.0f) * dot(d, nrm_);
    const float th0 = 1e-4f;
    const float m = (sl.mp + sl.mu * __builtin_fmaf(3.1f, a, 1.0f)) * 1.001f + perr;  // S <= 3.1 a + 1 (planar)
    const float R = fabsf(y) - m;
    if (!(R > 0.0f)) return 0.0f;
    const float b = c + th0;
    const float L = (__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, 2.0f * kap * R)) - b) * (a2 * (1.0f / 6.06f));
    const float ch = 1.5f * a * dphi;  // the next chord
    const float Lc = fminf(L, fminf(__builtin_fmaf(0.5f, a, -ch), (1.5f - th0) * (a2 * (1.0f / 6.06f)) - ch));
    const float th1 = __builtin_fmaf(kap, Lc, th0);
    const float f = 1.0f - (th1 * th1 + th1 * th0 + th0 * th0) * (1.0f / 6.0f);
    return (Lc > 0.0f && f > 0.0f) ? Lc * f * 0.998f : 0.0f;
}
// slot j >= 1 for an outward lane at distance a (cyl_par: bs.cm's bit for a budgeted cylinder)
// Round 5: a cylinder is excluded for outward lanes whose orbital plane can
// hold a chord nearly parallel to its axis (bs.cm) too. Its distance budget
// covers only chords with |d_perp|^2 >= SR_BUDGET_DPMIN (sl.qk's margin);
// nearly parallel ones are the slab budget's (the cylinder-plane fast loop's
// ball min(m, mh) and budget_event's forced bit), which the exclusion leaves
// alone. Escaping lanes of the frame's centre column (orbital planes through
// the cylinder's axis) re-anchored its 32-unit window every step or two on
// their way out to u_f: the slowest waves' most frequent event.
#ifndef SR_OUT_CYL_CM
#define SR_OUT_CYL_CM 1
#endif
// Round 5: an outward lane clears an object once it is beyond the object's
// farthest accepted point (sr_dev_slot.rf) rather than its bounding sphere's
// far side: a disk seen edge-on from the origin, a rectangle or a cylinder's
// rim lie well inside |bc| + br.
#ifndef SR_OUT_FAR
#define SR_OUT_FAR 1
#endif
__device__ __forceinline__ bool outward_slot(const sr_dev_slot& sl, bool cyl_par, float a, float dip) {
    if (SR_OUT_CYL_CM) cyl_par = false;
    if (sl.type == SR_OBJECT_PLANE || (sl.type == SR_OBJECT_CYLINDER && (cyl_par || !(sl.x1 > 0.0f)))) return false;
    if (SR_OUT_FAR)  // the object's own farthest point (sr_api.cpp far_reach), not its bounding sphere's
        return outward_clear(sl.rf, 0.0f, slot_mu(sl), sl.type == SR_OBJECT_CYLINDER ? sl.qk : 0.0f, sl.pl1, a, dip);
    return outward_clear(sl.cn, sl.br, sl.mu, sl.type == SR_OBJECT_CYLINDER ? sl.qk : 0.0f, sl.pl1, a, dip);
}

// A budget slot's record read in one batch of scalar loads: every field is
// pinned to an SGPR where it is loaded, so the type-specific code that
// follows does not wait on a chain of lazily issued loads.
#define SR_PIN(x) asm volatile("" : "+s"(x))
__device__ __forceinline__ sr_dev_slot pin_slot(const sr_dev_slot& g) {
    sr_dev_slot sl = g;
    SR_PIN(sl.type);
    SR_PIN(sl.rb);
    SR_PIN(sl.mp);
    SR_PIN(sl.br);
    SR_PIN(sl.mu);
    SR_PIN(sl.pl1);
    SR_PIN(sl.qk);
    SR_PIN(sl.bc[0]);
    SR_PIN(sl.bc[1]);
    SR_PIN(sl.bc[2]);
    SR_PIN(sl.x0);
    SR_PIN(sl.pos[0]);
    SR_PIN(sl.pos[1]);
    SR_PIN(sl.pos[2]);
    SR_PIN(sl.x1);
    SR_PIN(sl.a0[0]);
    SR_PIN(sl.a0[1]);
    SR_PIN(sl.a0[2]);
    SR_PIN(sl.x2);
    SR_PIN(sl.a1[0]);
    SR_PIN(sl.a1[1]);
    SR_PIN(sl.a1[2]);
    SR_PIN(sl.a2[0]);
    SR_PIN(sl.a2[1]);
    SR_PIN(sl.a2[2]);
    return sl;
}

// Direction-independent part of a budgeted cylinder's clearance: the distance
// from A to its height slab (0 <= (p - pos) . axes[1] <= height). cyl_test
// accepts only a point p = o + lambda d with 0 <= lambda <= len, i.e. on the
// chord up to rounding, whose computed height passes that window, so this
// bound holds however ill-conditioned the lateral quadratic is (chords nearly
// parallel to the axis). Same margins as clearance_obj(); -inf without a unit axis.
__device__ __forceinline__ float clearance_slab(const sr_dev_slot& sl, f3 A, float a) {
    if (!(sl.mp < INFINITY)) return -INFINITY;
    const float y = dot(A - ld3(sl.pos), ld3(sl.a1));
    const float ey = fmaxf(0.0f, fmaxf(-y, y - sl.x0));
    return ey - sl.mp - 1.8f * SR_MU_QUADRATIC * a;
}

// NaN-propagating minimum: a NaN clearance must force the exact tests. IEEE
// minimum (v_minimum3_f32 on gfx950): NaN if either operand is NaN, one
// instruction (the select form it replaces, `!(e >= m) ? e : m`, took two and
// dropped an earlier NaN when a later operand was a number).
__device__ __forceinline__ float nmin(float m, float e) { return __builtin_elementwise_minimum(m, e); }

// Per-lane budget state: E[j] = clearance_j(anchor_j) - slacked path from
// anchor_j to the last budget event, T = slacked path since that event,
// m = min_j E[j]. Slots re-anchor independently: only those whose budget is
// spent are re-anchored (and tested if the chord may reach them). Unused
// slots hold +inf. (pa, pb)[k] = (nv, tv) . axis of the k-th budgeted
// cylinder (budget_cyl_mask bit order) for the chord-direction test.
// E lives in LDS, one column per thread (E[j * SR_WG], conflict-free): the
// event loop indexes it with the wave-uniform slot j in a compact runtime
// loop, and the step loop's registers hold only T and m.
// SR_WG: threads per workgroup of the integrate and resume kernels (64, 128
// or 256: one, two or four of a 16x16 tile's 8x8 waves). A workgroup's LDS
// (72 B per thread) is held until its last wave ends: with 256-thread
// workgroups a CU fills up with tiles whose one long wave runs on beside
// three finished ones (busy wave slots 0.84 of the chip's over a headline
// launch); one wave per workgroup frees each slot as its wave ends (0.94):
// 1.27 -> 1.22 ms per headline frame, 1/8 share 0.185 -> 0.171
// (profiles/r02/s10_wg_*).
#ifndef SR_WG
#define SR_WG 64
#endif
#define SR_WG_PER_TILE (256 / SR_WG)
#define SR_E_STRIDE SR_WG
// Budgeted cylinders whose nearly parallel chords the kernel handles apart
// (chord_parallel, slab budgets, the cylinder-plane fast loops) in the
// general and large instantiations and the resume kernel: none since round 6
// (sr_api.cpp SR_CYL_DIRFREE: the lateral margin holds for every direction);
// SR_MAX_CYLINDERS for a host built with SR_CYL_DIRFREE=0
#ifndef SR_NC_KERNEL
#define SR_NC_KERNEL 0
#endif
#ifndef SR_AHEAD
#define SR_AHEAD 2.0f
#endif
#ifndef SR_FAST_UNROLL  // fast-loop steps per iteration (1 .. 4; the step table has 4 padding entries);
                        // the latency mode's instantiation runs 2 (sr_set_latency_mode). 4 since round 6:
                        // at 7 waves per SIMD 0.5 % more frames per second than 3 in two A/Bs
                        // (profiles/r06/s18, s19), one frame alone level
#define SR_FAST_UNROLL SR_FAST_UNROLL_DEFAULT
#endif
#ifndef SR_AHEAD_T
#define SR_AHEAD_T 1.0f
#endif
#ifndef SR_CM_ITER  // the cylinder-plane fast loop tests the chord direction once per iteration (integrate)
#define SR_CM_ITER 1
#endif
#ifndef SR_COAST  // the RK4-only fast loop of waves whose every budget is +inf (integrate)
#define SR_COAST 1
#endif
// The budget state's LDS rows (one column per thread) for an
// instantiation with NB budget slots and NC budgeted cylinders: E[0..NB],
// then pa[k], pb[k] (rows PA0 + 2k, + 1) and the slab budgets H[k] (SLAB0 +
// k) of the cylinders, then the budget's per-lane scalars (Budget::T() ...
// uhi()), which the fast loop does not need, so they wait in LDS instead of
// registers (held in VGPRs across it they were spilled to scratch and
// reloaded at every event). The default scene's kernel (6 slots, 1 cylinder)
// takes 17 rows, 4.25 KiB per 64-lane wave.
template <int NB, int NC, bool TR = false>
struct BudgetLayout {
    static constexpr int PA0 = NB + 1;
    static constexpr int SLAB0 = PA0 + 2 * NC;
    static constexpr int BT = SLAB0 + NC;
    static constexpr int BM = BT + 1, BCX = BT + 2, BCY = BT + 3, BMH = BT + 4, BCM = BT + 5, BUHI = BT + 6;
    static constexpr int BTR = BT + 7;  // the test ray's budget (TR instantiations, clearance_tr)
    static constexpr int ROWS = BT + 7 + (TR ? 1 : 0);
};
// reach bit of the test ray (budget_event, closest_hit_chord)
#define SR_REACH_TR (1u << 30)
// The black hole's u window (SR_BH_WINDOW). Every chord of the step loop
// joins two orbit points at radii 1/u (within 3e-6 relative) and subtends
// the step's angle dphi at the origin, so it stays in the half-plane beyond
// the chord between the same directions at the smaller radius: at least
// min(rA, rB) cos(dphi / 2) >= min(rA, rB) out_dip from the origin. While u
// <= SR_BH_U (r >= 1.0142) at both ends and out_dip > SR_BH_DIP, every point
// of a chord is at least r_e = 1.0076 from the origin, and sphere_test
// cannot accept it: a root on the r = 1 sphere needs a computed discriminant
// b^2 - c >= 0 (true value 1 - rho^2 for the line at distance rho) and a root
// inside [0, len], i.e. within the segment, whose end is sqrt(r_e^2 - rho^2)
// - sqrt(1 - rho^2) >= (r_e^2 - 1) / (2 r_e) = 0.0076 along the line from
// the true root (the line's foot point beyond it when rho >= r_e). With the
// chord origin o within r = 100 (sr_dev_frame.win_ok: u_f >= 0.01, cameras
// inside) the discriminant is computed within 4 eps |o|^2 = 4.8e-3 and the
// root within that over 2 sqrt(disc) (or its square root, 0.07, near
// tangency, where the distance is 0.12 or more): at most 0.0024 at rho = 0
// and 3x below the distance everywhere. So a lane beyond that radius needs
// no distance budget for the hole: its slot-0 budget is +inf and the step
// loop exits on u > uhi = SR_BH_U instead (one compare per step), where slot
// 0 re-anchors and the chord is reach-tested. Lanes inside the band (or the
// shell) keep the distance budget, uhi = SR_U_NOWIN. Ring rays orbit the photon
// sphere at r ~ 1.5 for hundreds of steps: their distance budgets (0.5 at r =
// 1.5) ran out every ~50 steps per lane and made the hole the most frequent
// event (profiles/r03/s19_*: its re-anchors 186 k -> 93 k per headline frame,
// a frame alone -8 %).
#ifndef SR_BH_WINDOW
#define SR_BH_WINDOW 1
#endif
#define SR_BH_U 0.986f      // u at r = 1.01420
// A lane without a window keeps uhi = the largest float below 1e30, not
// +inf: a ray through the singularity (u past 1e30, then +inf, where RK4
// keeps u = u' = +inf) leaves the fast loop there for the slow path's
// degenerate chord (integrate: degen; the reference's chord of zero length
// and NaN direction ends the ray). Its ball test alone does not catch it: a
// ball around the origin holds every such end point (vb -> -inf). Round 6:
// a stress-scene ray that passed the shell behind an alpha-0 texel ran on to
// max_steps (found once that scene's lazy chords were switched on).
#define SR_U_NOWIN 0x1.93e592p+99f
#define SR_BH_RWIN 1.0143f  // an anchor beyond this radius (by perr) starts a window
// The inner window (SR_BH_WINDOW2): chords whose two ends both lie at r in
// [1.00402, 1.1] (u in [SR_BH_ULO2, 0.996]) with a step angle below 0.063
// (out_dip > SR_BH_DIP2) stay at least 1.00402 x 0.9995 = 1.00352 from the
// origin. sphere_test computes their discriminant within 12 eps (|o|^2 + 1)
// <= 1.6e-6 (|o| <= 1.1), so a root it accepts lies within sqrt(1.6e-6) =
// 1.26e-3 of a true root (near tangency; less elsewhere), while the segment
// ends at least 3.5e-3 from the sphere along the line: none is accepted. A
// lane there needs no distance budget for the hole either; the step loop
// exits on u > 0.996 or u < SR_BH_ULO2 (climbing past r = 1.1; the u_f
// compare, per lane). Rays falling in crossed the band r < 1.0142 with an
// event on every step (their distance budget was below one step).
#ifndef SR_BH_WINDOW2
#define SR_BH_WINDOW2 1
#endif
// Round 5: the window's upper bound follows the frame's step angle instead
// of r = 1.004 (sr_dev_frame.bh_u2 = out_dip / (1 + SR_BH_G2)): a chord with
// both ends at u <= bh_u2 stays min(rA, rB) out_dip >= 1 + SR_BH_G2 = 1.0015
// from the origin (less the end points' 2.2e-6), above the 1.26e-3 a root
// can move at tangency. Falling lanes steep enough (the orbit's invariant E =
// u'^2 + u^2 - u^3 >= SR_BH_E_MIN at the window's anchor, and max_dphi <=
// SR_BH_S_DPHI) get bh_u3 = out_dip / (1 + SR_BH_G3), 6e-5 off the shell:
// u'' > 0 for u > 2/3, so u' only grows on the way in (each RK4 stage adds a
// positive term), u' >= sqrt(E - u^2 (1 - u)) >= 0.367 once u >= 0.99 (E
// drifts by < 3e-5 over the window), and a chord from u_A to u_B >= 0.998
// rises u_B - u_A >= 0.367 dphi (u_A >= 0.99) or >= 0.008 >= 0.6 dphi (u_A <
// 0.99): its line passes within rho^2 <= rA rB / (1 + (u_B - u_A)^2 / (u_A
// u_B dphi^2)) <= 0.9 of the origin (2 (1 - cos) >= sin^2 in the chord's
// length), so sphere_test's discriminant is >= 0.1 and its roots move by at
// most 1.6e-6 / 0.316 + 3e-7 < 6e-6, ten times below the clearance. The
// same bounds make a crossing certain (the integrate slow path): a chord from
// inside the window (u_A <= uhi) to u_B >= SR_BH_UIN3 (steep lanes; inside
// r = 1 - 6e-5) or >= SR_BH_UIN2 (any lane: inside 1 - 1e-3, so the line
// passes within 0.999 of the origin, the discriminant is >= 2e-3 and a root
// moves by < 4e-5) has its entry root at least 5.8e-5 from both ends: the
// computed lambda1 is positive, below the length, and the smaller positive
// root. With the lane's other slots covered by its ball (vb < 0, no forced
// chord, no per-chord objects) the hole is the closest hit: ST_BH (the shade
// kernel reads its status and step count only) without the event.
#define SR_BH_ULO2 0.90910f   // u at r = 1.09999
// an anchor within this radius (by perr) and at u <= the window's bound
// (budget_event: (a - perr) uw > 1) starts an inner window
#define SR_BH_RMAX2 1.0999f
#define SR_BH_DIP2 0.9995f
#define SR_BH_DIP 0.9935f   // 1.0142 x 0.9935 = 1.0076

// SR_BALL: the step loop's test for the end point X = (cos phi, sin phi) / u
// of each step (orbital-plane coordinates) against the ball of radius R / 1.01
// around the centre C: inside when 1 + u (bn cos phi + bt sin phi + Q u) < 0,
// bn = -2 C.x, bt = -2 C.y, Q = |C|^2 - Rq^2 (that is (|X - C|^2 - Rq^2) u^2).
// Rq leaves room for the reference's rounding of the chord end point (1.1e-6
// r, r <= |C| + R), the centre's embedding (nv C.x + tv C.y within 1e-6 |C|
// of the event's end point and of budget_init's anchor), the frame's
// non-orthonormality (1e-6 relative) and the test's own float evaluation
// (below 7 eps (|C| + Rq)^2 in |X - C|^2). +inf: always inside (every budget
// infinite); -inf, NaN or a ball too small for its margins: never inside.
__device__ __forceinline__ float ball_q(float R, float cx, float cy) {
    if (!(R < INFINITY)) return R == INFINITY ? -INFINITY : INFINITY;
    const float c = fabsf(cx) + fabsf(cy);  // >= |C|
    const float Rt = R * (1.0f / 1.0101f) - 3.0e-6f * (c + R);
    if (!(Rt > 0.0f)) return INFINITY;
    const float s = c + Rt;
    return __builtin_fmaf(2.0e-6f * s, s, (cx * cx + cy * cy) - Rt * Rt);
}

template <int NB_, int NC_, bool TR_ = false>
struct Budget {
    using L = BudgetLayout<NB_, NC_, TR_>;
    static constexpr int NB = NB_, NC = NC_;
    static constexpr bool TR = TR_;
    float* E;  // &lds[threadIdx.x]: E[j * SR_E_STRIDE], then pa[k], pb[k] (below)
    // Scalars in LDS rows (L::BT ..), read with volatile loads so that no
    // register holds them across the fast loop:
    //   T   the charge since the last event (slacked path; SR_BALL: displacement)
    //   m   min_j E[j]
    //   cx, cy  SR_BALL: the ball's centre, the last event's end point in the orbital plane (nv, tv)
    //   mh  min_k of the cylinders' slab budgets H[k] (E[SLAB0 + k]): the bound
    //       that covers chords nearly parallel to an axis
    //   cm  budgeted cylinders (bit k) whose axis this orbital plane may nearly contain
    //   uhi the step loop's exit bound on u for the black hole (SR_BH_WINDOW; SR_U_NOWIN: none; bh_u2 /
    //       bh_u3: the inner window, whose lower bound is SR_BH_ULO2 instead of u_f: ulo_of())
    __device__ __forceinline__ float ld(int row) const { return E[row * SR_E_STRIDE]; }
    __device__ __forceinline__ void st(int row, float v) const { E[row * SR_E_STRIDE] = v; }
    __device__ __forceinline__ float T() const { return ld(L::BT); }
    __device__ __forceinline__ void setT(float v) const { st(L::BT, v); }
    __device__ __forceinline__ float m() const { return ld(L::BM); }
    __device__ __forceinline__ void setM(float v) const { st(L::BM, v); }
    __device__ __forceinline__ float cx() const { return ld(L::BCX); }
    __device__ __forceinline__ float cy() const { return ld(L::BCY); }
    __device__ __forceinline__ void setC(float x, float y) const {
        st(L::BCX, x);
        st(L::BCY, y);
    }
    __device__ __forceinline__ float mh() const { return ld(L::BMH); }
    __device__ __forceinline__ void setMh(float v) const { st(L::BMH, v); }
    // the L::BCM row holds cm in bits 0..7 and the orbit's excluded slots
    // (bit 8 + j: slot j, budget_frame) above
    __device__ __forceinline__ uint32_t cm() const { return __float_as_uint(ld(L::BCM)) & 0xffu; }
    __device__ __forceinline__ uint32_t excl() const { return __float_as_uint(ld(L::BCM)) >> 8; }
    __device__ __forceinline__ void setCm(uint32_t cm, uint32_t excl) const {
        st(L::BCM, __uint_as_float(cm | (excl << 8)));
    }
    __device__ __forceinline__ float etr() const { return ld(L::BTR); }
    __device__ __forceinline__ void setEtr(float v) const { st(L::BTR, v); }
    __device__ __forceinline__ float uhi() const { return ld(L::BUHI); }
    __device__ __forceinline__ void setUhi(float v) const { st(L::BUHI, v); }
    // the inner window (uhi in (SR_BH_U, 1): sr_dev_frame.bh_u2 / bh_u3)
    static __device__ __forceinline__ bool inner(float uhi) { return uhi > SR_BH_U && uhi < 1.0f; }
    static __device__ __forceinline__ float ulo_of(float uhi, float u_f) { return inner(uhi) ? SR_BH_ULO2 : u_f; }
    SR_PROBE_BUDGET_FIELDS  // measurement builds only (probes.h)
};

// The orbital frame's projections (pa, pb) on the budgeted cylinders' axes.
// Every chord lies in span(nv, tv), so its direction d has (d . axis)^2 <=
// pa^2 + pb^2 (Cauchy-Schwarz): when that is below 1 - 2 SR_BUDGET_DPMIN (with
// a rounding allowance far above the frame's non-orthonormality) no chord of
// this orbit can be near-parallel to the axis and bit k of bs.cm stays clear:
// chord_parallel skips the cylinder for this lane.
// slot j's orbital-plane exclusion bit (below), n = nv x tv, nn = |n|^2
// (xs = sr_dev_frame.xplane_s: S_max of the orbit's chords, +inf: no
// exclusion; it carries 0.5 % on top, which covers the end points' 4e-7 r
// off the plane as mu >= SR_MU_PLANAR)
__device__ __forceinline__ uint32_t xplane_bit(const sr_dev_slot& sl, int j, f3 n, float nn, float xs) {
    if (sl.type == SR_OBJECT_PLANE || sl.type == SR_OBJECT_CYLINDER) return 0u;
    const float h = dot(ld3(sl.bc), n);  // |h| / |n|: bc's distance from the plane
    const float need = (sl.br + sl.mu * xs) * 1.001f + 1.0e-4f + 1.0e-5f * sl.cn;
    // |h| / sqrt(nn) > need without a square root; NaN frames exclude nothing
    return (uint32_t)(h * h > (need * need) * (nn * 1.0002f)) << j;
}
// A bounded slot off a low-energy orbit's plane (SR_XCYL): need =
// sr_dev_frame.xlow_need[j - 1] (sr_api.cpp xlow_need has the bound: the
// chords that could come near the object by distance from the origin stay
// short, so its margin mu S, and a cylinder's quadratic one, are small; the
// orbital-plane exclusion's S_max gave a cylinder 31 units). A cylinder's
// slab budget (nearly parallel chords) is left alone, as for outward lanes
// (outward_slot).
#ifndef SR_XCYL
#define SR_XCYL 1
#endif
__device__ __forceinline__ uint32_t xcyl_bit(const sr_dev_slot& sl, int j, f3 n, float nn, float need) {
    const float h = dot(ld3(sl.bc), n);
    return (uint32_t)(h * h > (need * need) * (nn * 1.0002f)) << j;
}
// The orbit's energy E = u'^2 + u^2 (1 - u) for the exclusions of low-energy
// orbits (SR_XCYL, SR_XPERI: u < 0.6 and E <= SR_XCYL_EMAX), +inf otherwise
// (NaN compares false too)
__device__ __forceinline__ float orbit_e(float u, float du) {
    return u < 0.6f ? __builtin_fmaf(du, du, u * u * (1.0f - u)) : INFINITY;
}
// Periapsis exclusion (SR_XPERI): a low-energy orbit never comes closer to
// the origin than its periapsis, and an object whose every reachable chord
// (sr_api.cpp clear_radius) lies inside that sphere is excluded for the
// orbit, like an orbital-plane exclusion (bits 8 + j, budget_frame). The
// accretion disk, within r = 5 of the hole, is the default scene's case.
#ifndef SR_XPERI
#define SR_XPERI 1
#endif
// the cylinders' (pa, pb) rows and the cm bits (budget_frame, budget_init)
template <class BS>
__device__ __forceinline__ uint32_t budget_cyl_frame(const sr_dev_scene* __restrict__ sc, BS& bs, f3 nv, f3 tv) {
    uint32_t c = (uint32_t)sc->budget_cyl_mask;
    uint32_t cm = 0;
#pragma unroll
    for (int k = 0; k < BS::NC; k++) {
        if (c) {
            const f3 ax = ld3(sc->slots[__builtin_ctz(c)].a1);
            const float pa = dot(nv, ax), pb = dot(tv, ax);
            bs.E[(BS::L::PA0 + 2 * k) * SR_E_STRIDE] = pa;
            bs.E[(BS::L::PA0 + 1 + 2 * k) * SR_E_STRIDE] = pb;
            // NaN frames keep the test (the comparison is false)
            cm |= (uint32_t)(!(pa * pa + pb * pb < 1.0f - 2.0f * SR_BUDGET_DPMIN - 1.0e-3f)) << k;
            c &= c - 1;
        }
    }
    return cm;
}
template <class BS>
__device__ __forceinline__ void budget_frame(const sr_dev_scene* __restrict__ sc, BS& bs, f3 nv, f3 tv, float xs,
                                             const float* xneed, const float* xperi, float eo) {
    const uint32_t cm = budget_cyl_frame(sc, bs, nv, tv);
    uint32_t x = 0;
#if SR_XPLANE
    // Orbital-plane exclusion (per orbit): every chord of this orbit joins two
    // end points (nv cos phi + tv sin phi) / u computed in binary32, within
    // 4e-7 r of the plane span(nv, tv) through the origin, and an object's
    // exact test accepts only points within br + mu S of its bounding
    // sphere's centre bc (may_hit). Every applied step of an orbit but its
    // last has u >= u_f, so a chord starts within R = 1 / u_f, and it ends
    // within 2 R unless it is that last one (the step to u < u_f: a reseed or
    // the ray's end follows) with u < u_f / 2. So S = |o|_1 + len + 1 <=
    // (sqrt 3 + 3) R + 1 = S_max (sr_dev_frame.xplane_s, the host's bound,
    // +inf when u_f <= 0), and when bc lies farther from that plane than br +
    // mu S_max plus the rounding, no such chord can reach the object: its
    // budget is +inf until the next reseed (a new plane). A chord ending
    // beyond 2 R is an event with the excluded slots forced (integrate,
    // budget_event: rare, a near-radial escape). Planes (unbounded) and cylinders (their quadratic margin
    // grows near the axis direction) are never excluded. Of the default scene
    // the sphere and the box lie off most rays' planes (the pencil of planes
    // through the camera and the hole).
    {
        const f3 n = cross(nv, tv);  // |n| within 1e-5 of 1
        const float nn = dot(n, n);
        const int nb = sc->num_budget;
        for (int j = 1; j <= nb; j++) {
            x |= xplane_bit(sc->slots[j - 1], j, n, nn, xs);
            if (SR_XCYL && eo <= SR_XCYL_EMAX) x |= xcyl_bit(sc->slots[j - 1], j, n, nn, xneed[j - 1]);
            if (SR_XPERI && eo <= xperi[j - 1]) x |= 1u << j;
        }
    }
#endif
    bs.setCm(cm, x);
}

// bs.cm's bit for slot j (budgeted cylinders; false for other slots)
template <class BS>
__device__ __forceinline__ bool cyl_par_bit(const sr_dev_scene* __restrict__ sc, const BS& bs, int j) {
    const uint32_t cyl = (uint32_t)sc->budget_cyl_mask;
    if (!((cyl >> (j - 1)) & 1u)) return false;
    return (bs.cm() >> __builtin_popcount(cyl & ((1u << (j - 1)) - 1u))) & 1u;
}

__device__ float clearance_tr(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs, f3 A, bool outward,
                              float a, float dip, float rlen, uint32_t& gm);

// START_WINDOW: d is the orbit's tangent at A (a ray's start, sr_integrate_kernel),
// so the planar slots may take plane_window_start's directional budget
template <bool START_WINDOW, class BS>
__device__ __forceinline__ void budget_init(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                            BS& bs, f3 A, f3 nv, f3 tv,
                                            bool outward, float dip, bool bh_ok, bool falling, float xs, float u2w,
                                            const float* xneed, const float* xperi, float eo, f3 d, float dphi) {
    const float a = __builtin_amdgcn_sqrtf(dot(A, A));
    const int nb = sc->num_budget;
    bs.setT(0.0f);
    // the ball's centre: A in the orbital plane (A lies in it: the camera, or a
    // chord end point), within 1e-6 a of A; the budgets give that up
    bs.setC(dot(A, nv), dot(A, tv));
    const float m0 = 2.0e-6f * (a + 1.0f);
    float m = INFINITY;
    // the cm bits first (outward_slot); the exclusion bits in the slot loop
    const uint32_t cm = budget_cyl_frame(sc, bs, nv, tv);
    bs.setCm(cm, 0u);
    const f3 xn = cross(nv, tv);
    const float xnn = dot(xn, xn);
    uint32_t xcl = 0;
    {
        float e = clearance_bh(a);
        float uhi = SR_U_NOWIN;
        if (SR_BH_WINDOW && bh_ok && a > SR_BH_RWIN) {
            e = INFINITY;
            uhi = SR_BH_U;
        }
        if (SR_BH_WINDOW2 && dip > SR_BH_DIP2 && a * u2w > 1.000001f && a < SR_BH_RMAX2 && (falling || !(a > SR_BH_RWIN))) {
            e = INFINITY;
            uhi = u2w;
        }
        bs.setUhi(uhi);
        if (outward && outward_clear(1.0f, 0.0f, SR_MU_QUADRATIC, 0.0f, 0.0f, a, dip)) e = INFINITY;
        e -= m0;
        bs.E[0] = e;
        m = nmin(m, e);
    }
    if constexpr (BS::TR) {  // the test ray (clearance_tr)
        uint32_t gm;
        const float e = clearance_tr(sc, segs, A, outward, a, dip, -1.0f, gm) - m0;
        bs.setEtr(e);
        m = nmin(m, e);
    }
    // One pass over the slots; slot j + 1's record is loaded while slot j
    // is worked on (one batch of scalar loads per slot, waited a slot later:
    // waited at once they serialised the loop's latency, SR_PROF section 22)
    sr_dev_slot nxt;
    if (nb > 0) nxt = sc->slots[0];
#pragma unroll 1
    for (int j = 1; j <= nb; j++) {
        const sr_dev_slot sl = pin_slot(nxt);
        if (j < nb) nxt = sc->slots[j];
        if (SR_XPLANE) xcl |= xplane_bit(sl, j, xn, xnn, xs);
        if (SR_XCYL && eo <= SR_XCYL_EMAX) xcl |= xcyl_bit(sl, j, xn, xnn, xneed[j - 1]);
        if (SR_XPERI && eo <= xperi[j - 1]) xcl |= 1u << j;
        float e = clearance_obj(sl, A, a) - m0;
        if (START_WINDOW && SR_INIT_WINDOW && (sl.type == SR_OBJECT_RECTANGLE || sl.type == SR_OBJECT_DISK ||
                               sl.type == SR_OBJECT_HOLLOW_DISK || sl.type == SR_OBJECT_PLANE) &&
            sl.mp < INFINITY && e < 0.5f * a) {
            const float w = plane_window_start(sl, A, d, a, m0, dphi);
            e = w > e ? w : e;  // NaN e stays NaN
        }
        if (outward && outward_slot(sl, cyl_par_bit(sc, bs, j), a, dip)) e = INFINITY;
        if ((xcl >> j) & 1u) e = INFINITY;  // off this orbit's plane (budget_frame)
        bs.E[j * SR_E_STRIDE] = e;
        m = nmin(m, e);
    }
    bs.setCm(cm, xcl);
    bs.setM(m);
    float mh = INFINITY;
    uint32_t c = (uint32_t)sc->budget_cyl_mask;
#pragma unroll
    for (int k = 0; k < BS::NC; k++) {
        if (c) {
            const float e = clearance_slab(sc->slots[__builtin_ctz(c)], A, a) - m0;
            bs.E[(BS::L::SLAB0 + k) * SR_E_STRIDE] = e;
            mh = nmin(mh, e);
            c &= c - 1;
        }
    }
    bs.setMh(mh);
}

// The orbit's (pa, pb) on each budgeted cylinder's axis (budget_frame),
// read from LDS once per fast loop: they change only at reseeds.
template <int NC>
struct CylDirs {
    float pa[NC > 0 ? NC : 1], pb[NC > 0 ? NC : 1];
};
template <class BS>
__device__ __forceinline__ CylDirs<BS::NC> cyl_dirs(const sr_dev_scene* __restrict__ sc, const BS& bs) {
    CylDirs<BS::NC> d;
    uint32_t c = (uint32_t)sc->budget_cyl_mask;
#pragma unroll
    for (int k = 0; k < BS::NC; k++) {
        d.pa[k] = d.pb[k] = 0.0f;
        if (c) {
            d.pa[k] = bs.E[(BS::L::PA0 + 2 * k) * SR_E_STRIDE];
            d.pb[k] = bs.E[(BS::L::PA0 + 1 + 2 * k) * SR_E_STRIDE];
            c &= c - 1;
        }
    }
    return d;
}

// Whether the chord with in-plane components (a, b) (chord = nv a + tv b, up
// to perr absolute) may be closer than SR_BUDGET_DPMIN to a budgeted
// cylinder's axis direction; bit k of the result: cylinder k (bit order of
// budget_cyl_mask). Decided with twice the threshold and forced when the
// direction is not known to 0.4%. Branch-free over the cylinder capacity
// (unused slots have pa = pb = 0 and no bit in cm).
template <int NC>
__device__ __forceinline__ uint32_t chord_parallel(uint32_t cm, const CylDirs<NC>& cd, float a, float b, float perr) {
    const float dd = a * a + b * b;
    const bool vague = !(perr * perr <= 1.6e-5f * dd);
    uint32_t par = 0;
#pragma unroll
    for (int k = 0; k < NC; k++) {
        const float ca = a * cd.pa[k] + b * cd.pb[k];
        const bool near = vague | !(dd - ca * ca >= 2.0f * SR_BUDGET_DPMIN * dd);
        par |= (uint32_t)near << k;
    }
    return par & cm;
}

// Conservative: may the exact chord, within perr of the segment [A, B], come
// within reach of slot j's exact test (per-chord margins of may_hit)?
__device__ __forceinline__ bool slot_reachable(const sr_dev_slot* slp, int j, f3 A, f3 B, float perr) {
    const f3 dv = B - A;
    const float dd = dot(dv, dv);
    const float len = __builtin_amdgcn_sqrtf(dd);
    const float S = ((fabsf(A.x) + fabsf(A.y) + fabsf(A.z)) + len + 1.0f) * 1.001f + perr;
    if (!(S < 1.0e30f)) return true;  // non-finite chord: the exact tests decide
    f3 c;
    float R;
    if (j == 0) {
        c = F3(0.0f, 0.0f, 0.0f);
        R = 1.0f + SR_MU_QUADRATIC * S;  // the black hole: sphere r = 1 at the origin
        // a chord inside the shell (both ends, by the margin) cannot reach it
        const float ri = (1.0f - SR_MU_QUADRATIC * S) * 0.999f - perr;
        if (dot(A, A) < ri * ri && dot(B, B) < ri * ri && ri > 0.0f) return false;
    } else {
        const sr_dev_slot& sl = *slp;
        c = ld3(sl.bc);
        R = sl.br + sl.mu * S;
        if (sl.mp < INFINITY) {  // orthonormal frame: tighter regions than the bounding sphere
            const float m = (sl.mp + slot_mu(sl) * S) * 1.001f + perr;
            const f3 pos = ld3(sl.pos);
            const f3 a1 = ld3(sl.a1);
            const float yA = dot(A - pos, a1), yB = dot(B - pos, a1);
            if (sl.type == SR_OBJECT_PLANE || sl.type == SR_OBJECT_DISK || sl.type == SR_OBJECT_HOLLOW_DISK ||
                sl.type == SR_OBJECT_RECTANGLE) {
                // planar: the chord must reach the plane's acceptance slab
                if ((yA > m && yB > m) || (yA < -m && yB < -m)) return false;
            } else if (sl.type == SR_OBJECT_BOX) {
                // the chord must reach the box grown by the margin (slab test in the box frame)
                const f3 a0 = ld3(sl.a0), a2 = ld3(sl.a2);
                const float xA = dot(A - pos, a0), xB = dot(B - pos, a0);
                const float zA = dot(A - pos, a2), zB = dot(B - pos, a2);
                float t0 = 0.0f, t1 = 1.0f;
                auto slab = [&](float pA, float pB, float hi) {
                    const float lo_ = -m, hi_ = hi + m, dpv = pB - pA;
                    if (fabsf(dpv) < 1e-30f) {
                        if (pA < lo_ || pA > hi_) t1 = -1.0f;
                        return;
                    }
                    const float inv = __builtin_amdgcn_rcpf(dpv);  // the margin covers its rounding
                    float ta = (lo_ - pA) * inv, tb = (hi_ - pA) * inv;
                    if (ta > tb) {
                        const float tt = ta;
                        ta = tb;
                        tb = tt;
                    }
                    t0 = fmaxf(t0, ta);
                    t1 = fminf(t1, tb);
                };
                slab(xA, xB, sl.x0);
                slab(yA, yB, sl.x2);
                slab(zA, zB, sl.x1);
                if (t0 > t1 + 1e-6f) return false;
            } else if (sl.type == SR_OBJECT_CYLINDER) {
                // the chord must reach the height slab (clearance_slab), in any direction
                const float hc = sl.x0;
                if ((yA < -m && yB < -m) || (yA > hc + m && yB > hc + m)) return false;
            }
        }
        if (sl.type == SR_OBJECT_CYLINDER) {
            const float r = sl.x1;
#if SR_REACH_LAT  // the lateral margin for every chord direction (lat_margin, round 6)
            if (!(r > 0.0f)) return true;
            R = R + lat_margin(S + sl.pl1, r);
#else
            const float ca = dot(dv, ld3(sl.a1));
            const float dp = (dd - ca * ca) * __builtin_amdgcn_rcpf(dd) * 0.5f;
            if (!(dp > 1.0e-6f) || !(r > 0.0f)) return true;
            const float Sc = S + sl.pl1;
            R = R + SR_CYL_QMARGIN * Sc * Sc * __builtin_amdgcn_rcpf(r * dp);
#endif
        }
    }
    R = R * 1.001f + perr;
    const f3 w = c - A;
    float t = dot(w, dv) * __builtin_amdgcn_rcpf(dd);
    t = t > 0.0f ? t : 0.0f;  // NaN -> 0
    t = t < 1.0f ? t : 1.0f;
    const f3 q = w - dv * t;
    return !(dot(q, q) > R * R);
}

// Budget event for the chord of this step, known approximately as [A, B]
// (exact end points within perr; bs.T already charged with it). Slots whose
// budget is spent re-anchor at B (clearance - perr); returns the
// wave-uniform mask of those the chord may reach: their exact tests need the
// exact chord. A budgeted cylinder's E covers chords at least SR_BUDGET_DPMIN
// off its axis direction; chords that may be closer (par, bit k = cylinder k)
// are covered by its slab budget H[k] instead, and the slot re-anchors when
// that is spent too. reanchor_cyl: a new orbital frame (reseed) re-anchors
// every cylinder slot.
// Two phases: every budget is read at once and compared (unrolled over the
// slot capacity, no per-slot branches or LDS round trips), then only the
// slots some lane has spent - usually one - run their clearance and reach
// tests; all lanes re-anchor those.
template <class BS>
__device__ __forceinline__ uint32_t budget_event(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                                 uint32_t& trmask, BS& bs, f3 A, f3 B,
                                                 float perr, uint32_t par, bool reanchor_cyl, float ahead,
                                                 bool outward, float dip, float dphi, bool bhx, bool bh_ok,
                                                 bool falling, bool par_recompute, float u_f, float u2, float u3,
                                                 bool steep) {
    constexpr int NB = BS::NB, NC = BS::NC;
    constexpr int NS = NB + 1;  // the slots this kernel instantiation handles (sc->num_budget <= NB)
    const int nb = sc->num_budget;
    const uint32_t cyl = (uint32_t)sc->budget_cyl_mask;  // budget index (slot - 1) of each budgeted cylinder
    const float T = bs.T();
    float e[NS], h[NC > 0 ? NC : 1];
#pragma unroll
    for (int j = 0; j < NS; j++) e[j] = bs.E[j * SR_E_STRIDE];
    {
        uint32_t c = cyl;  // only the scene's cylinders' rows exist in the packed layout
#pragma unroll
        for (int k = 0; k < NC; k++) {
            h[k] = INFINITY;
            if (c) {
                h[k] = bs.E[(BS::L::SLAB0 + k) * SR_E_STRIDE];
                c &= c - 1;
            }
        }
    }
    if (par_recompute) {
        // the event chord's direction against the budgeted cylinders' axes
        // (chord_parallel in 3-D on the approximate chord; the fast loop's
        // CMV 2 tested only its iteration's first chord)
        par = 0;
        const f3 dv = B - A;
        const float dd = dot(dv, dv);
        const bool vague = !(perr * perr <= 1.6e-5f * dd);
        uint32_t c = cyl;
#pragma unroll
        for (int k = 0; k < NC; k++) {
            if (c) {
                const float ca = dot(dv, ld3(sc->slots[__builtin_ctz(c)].a1));
                par |= (uint32_t)(vague | !(dd - ca * ca >= 2.0f * SR_BUDGET_DPMIN * dd)) << k;
                c &= c - 1;
            }
        }
        par &= bs.cm();
    }
    // this lane's slots whose E does not cover the chord (bit 0: the chord
    // left the black hole's u window, bhx)
    uint32_t forced = (uint32_t)bhx;
    {
        uint32_t c = cyl;
#pragma unroll
        for (int k = 0; k < NC; k++) {
            if (c) {
                const bool f = reanchor_cyl || (((par >> k) & 1u) && !(T < h[k]));
                forced |= (uint32_t)f << (__builtin_ctz(c) + 1);
                c &= c - 1;
            }
        }
    }
    if (reanchor_cyl) forced |= (2u << nb) - 1u;  // a new orbital frame: outward budgets start over
    // the orbital-plane exclusions hold for chords ending within 2 / u_f
    // (budget_frame): beyond (|B| >= 2 / u_f (1 - 1e-5) > 1.9 / u_f for a
    // chord to u < u_f / 2, integrate's event) this lane's excluded slots are forced
    if (SR_XPLANE && dot(B, B) * (u_f * u_f) > 3.61f) forced |= bs.excl();
    uint32_t spent = 0;  // wave-uniform: slots some lane has spent or is about to
    // one ballot per slot of a single compare (written straight to an SGPR
    // pair); forced slots, rare (reseeds, near-axis chords), balloted apart
#pragma unroll
    for (int j = 0; j < NS; j++) {
        if (__ballot(!(T + ahead < e[j]))) spent |= 1u << j;
    }
    if (__ballot(forced != 0u)) {
#pragma unroll
        for (int j = 0; j < NS; j++)
            if (__ballot((forced >> j) & 1u)) spent |= 1u << j;
    }
    spent &= (2u << nb) - 1u;
    // uniform by construction (ballots); said so, so that the slot records
    // below stay scalar loads in every build (pin_slot's SGPR constraints)
    spent = __builtin_amdgcn_readfirstlane(spent);
    SR_PTB(20);
    SR_PROBE(probe_event_phase1(bs, T, e[0], forced, spent));
    // the others run on: charge them the path since the last event
    float m = INFINITY, mh = INFINITY;
#pragma unroll
    for (int j = 0; j < NS; j++) {
        if (j <= nb && !((spent >> j) & 1u)) {
            const float v = e[j] - T;
            bs.E[j * SR_E_STRIDE] = v;
            m = nmin(m, v);
        }
    }
    {
        uint32_t c = cyl;
#pragma unroll
        for (int k = 0; k < NC; k++) {
            if (c) {
                if (!((spent >> (__builtin_ctz(c) + 1)) & 1u)) {
                    const float v = h[k] - T;
                    bs.E[(BS::L::SLAB0 + k) * SR_E_STRIDE] = v;
                    mh = nmin(mh, v);
                }
                c &= c - 1;
            }
        }
    }
    SR_PTB(3);
    // the spent ones re-anchor at B
    const float a = __builtin_amdgcn_sqrtf(dot(B, B));
    uint32_t reach = 0;
    if constexpr (BS::TR) {  // the test ray's budget: spent (or a new frame) re-anchors it for every lane
        const float et = bs.etr();
        if (__ballot(!(T + ahead < et)) || __ballot(reanchor_cyl)) {
            const bool h = reanchor_cyl || !(T < et);  // this lane's budget did not cover the chord
            // the chord lies within its length (+ the end points' error) of B:
            // the groups (and the flat cylinder) whose clearance from B
            // exceeds that cannot be reached by it (trmask, clearance_tr)
            const f3 dv = B - A;
            const float rlen = __builtin_fmaf(__builtin_amdgcn_sqrtf(dot(dv, dv)), 1.001f, 2.0f * perr + 1.0e-6f);
            const float v = clearance_tr(sc, segs, B, outward, a, dip, rlen, trmask) - perr;
            bs.setEtr(v);
            m = nmin(m, v);
            SR_STAT(22, 1);  // (the small instantiation's counter of slot 8, which it lacks)
            if (__ballot(h && trmask != 0u)) {
                reach |= SR_REACH_TR;
                SR_STAT(10, 1);
            }
        } else {
            const float v = et - T;
            bs.setEtr(v);
            m = nmin(m, v);
        }
    }
    const uint32_t xcl = SR_XPLANE ? bs.excl() : 0u;  // slots off this orbit's plane (budget_frame)
    for (uint32_t w = spent; w; w &= w - 1) {
        const int j = __builtin_ctz(w);
        if (j <= 8) SR_STAT(14 + j, 1);
        SR_PROBE(if (j < 8) SR_PROF_BUMP(bs.prof, 8 + j, 1));
        // only lanes whose budget did not cover the chord can reach the slot
        // (the others re-anchor early: look-ahead, or another lane spent it)
        // (its E is still the uncharged one in LDS: spent slots are only written below)
        const bool h = ((forced >> j) & 1u) || !(T < bs.E[j * SR_E_STRIDE]);
        if (j == 0) {
            // beyond the band: the u window instead of a distance budget
            const bool win1 = SR_BH_WINDOW && bh_ok && a - perr > SR_BH_RWIN;
            // the inner window from an anchor already inside its bound (u <= uw:
            // a re-anchor near the shell, e.g. by another lane's event, keeps it)
            const float uw = steep ? u3 : u2;
            const bool win2 = SR_BH_WINDOW2 && dip > SR_BH_DIP2 && (a - perr) * uw > 1.000001f &&
                              a + perr < SR_BH_RMAX2 && (falling || !win1);
            const bool win = win1 || win2;
            bs.setUhi(win2 ? uw : win1 ? SR_BH_U : SR_U_NOWIN);
            const float v = (win || (outward && outward_clear(1.0f, 0.0f, SR_MU_QUADRATIC, 0.0f, 0.0f, a, dip)))
                                ? INFINITY
                                : clearance_bh(a) - perr;
            bs.E[0] = v;
            m = nmin(m, v);
            if (__ballot(h) && __ballot(h && slot_reachable(nullptr, 0, A, B, perr))) reach |= 1u;
            continue;
        }
        const sr_dev_slot sl = pin_slot(sc->slots[j - 1]);
        // One straight-line copy per object type (the type a compile-time
        // constant in it): the clearance and the reach test interleave.
        auto reanchor = [&](auto ty_tag) {
            constexpr int TY = decltype(ty_tag)::value;
            sr_dev_slot st = sl;
            st.type = TY;
            float v = clearance_obj(st, B, a) - perr;
            if ((TY == SR_OBJECT_RECTANGLE || TY == SR_OBJECT_DISK || TY == SR_OBJECT_HOLLOW_DISK ||
                 TY == SR_OBJECT_PLANE) && st.mp < INFINITY && v < 0.5f * a) {
                // the window's slot-independent terms (chord length, curvature
                // bound) recomputed here: hoisted out of the slot loop they
                // were spilled and reloaded one scratch round trip at a time
                float ao = a;
                asm volatile("" : "+v"(A.x), "+v"(A.y), "+v"(A.z), "+v"(B.x), "+v"(B.y), "+v"(B.z));
                asm volatile("" : "+v"(ao), "+v"(perr));
                const float w = plane_window(st, A, B, ao, perr, dphi);
                v = w > v ? w : v;  // NaN v stays NaN
            }
            if (TY != SR_OBJECT_PLANE && outward &&
                outward_slot(st, TY == SR_OBJECT_CYLINDER &&
                                     ((bs.cm() >> __builtin_popcount(cyl & ((1u << (j - 1)) - 1u))) & 1u),
                             a, dip))
                v = INFINITY;
            if (TY != SR_OBJECT_PLANE && ((xcl >> j) & 1u)) v = INFINITY;  // budget_frame (cylinders: SR_XCYL)
            bs.E[j * SR_E_STRIDE] = v;
            m = nmin(m, v);
            if (TY == SR_OBJECT_CYLINDER) {
                const int k = __builtin_popcount(cyl & ((1u << (j - 1)) - 1u));
                const float vh = clearance_slab(st, B, a) - perr;
                bs.E[(BS::L::SLAB0 + k) * SR_E_STRIDE] = vh;
                mh = nmin(mh, vh);
            }
            if (__ballot(h) && __ballot(h && slot_reachable(&st, j, A, B, perr))) reach |= 1u << j;
        };
        switch (sl.type) {
        case SR_OBJECT_DISK: reanchor(std::integral_constant<int, SR_OBJECT_DISK>{}); break;
        case SR_OBJECT_HOLLOW_DISK: reanchor(std::integral_constant<int, SR_OBJECT_HOLLOW_DISK>{}); break;
        case SR_OBJECT_RECTANGLE: reanchor(std::integral_constant<int, SR_OBJECT_RECTANGLE>{}); break;
        case SR_OBJECT_BOX: reanchor(std::integral_constant<int, SR_OBJECT_BOX>{}); break;
        case SR_OBJECT_CYLINDER: reanchor(std::integral_constant<int, SR_OBJECT_CYLINDER>{}); break;
        case SR_OBJECT_PLANE: reanchor(std::integral_constant<int, SR_OBJECT_PLANE>{}); break;
        default: reanchor(std::integral_constant<int, SR_OBJECT_SPHERE>{}); break;
        }
    }
    bs.setT(0.0f);
    bs.setM(m);
    bs.setMh(mh);
    return reach;
}

// The test rays (frag:760-803), visited right after the black hole.
__device__ __forceinline__ void test_ray_hits(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                              Hit& best, f3 o, f3 d, float max_lambda) {
    if (!sc->tr_visible) return;
    f3 p;
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

// Culled test-ray hits for one exact chord [o, o + seg d] of the step loop
// (frag:760-803: the flat cylinder, then every curved segment). A segment is
// skipped only when the chord stays beyond the reach of its accepted points:
// its bounding sphere (as may_hit's for a cylinder of that pose) grown by mu
// S and the lateral margin lat_margin (round 6: for every chord direction;
// round 5 divided the quadratic's margin by |d_perp|^2 and tested every
// segment of a block whose cone of axes held a chord's direction); decided
// for a whole block or group of segments at once (sr_api.cpp
// test_ray_bounds: every segment's sphere lies within R of the bound's
// centre). The survivors are the exhaustive loop's tests with the same keys,
// so the winner is the same.
__device__ __forceinline__ bool tr_bound_may_hit(const float* __restrict__ B, f3 o, f3 d, float seg, float S, float r) {
    if (B[10] != 0.0f || !(r > 0.0f)) return true;  // a segment without a proven bound
    const f3 w = ld3(B) - o;
    float t = dot(w, d);
    t = t < 0.0f ? 0.0f : t;
    t = t > seg ? seg : t;
    const f3 q = w - d * t;
    const float d2 = dot(q, q);
    const float R = (B[3] + SR_MU_PLANAR * S) * 1.001f + lat_margin_len(seg, S + B[9], r) * B[11];
    return !(d2 > R * R);
}
// MASK (the test-ray instantiations): gm from the event's clearance_tr, bit g
// (group g) / bit 31 (the flat cylinder) clear where this chord cannot reach
// that part; it replaces the groups' per-chord bound tests
template <bool MASK = false>
__device__ __forceinline__ void test_ray_hits_culled(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                                     Hit& best, f3 o, f3 d, float seg, uint32_t gm = 0xffffffffu) {
    if (!sc->tr_visible) return;
    f3 p;
    const float* t = sc->tr_flat;
    const m3 A = ldm(t + 3);
    if (!MASK || __ballot((gm >> 31) & 1u))
        consider(best, cyl_test(o, d, ld3(t), A, t[12], t[13], seg, p), p, o, SLOT_TR_FLAT, 0, KEY_TR_FLAT);
    const float S = (fabsf(o.x) + fabsf(o.y) + fabsf(o.z)) + seg + 1.0f;  // as closest_hit_chord's may_hit
    const float r = sc->tr_radius;
    const float* blocks = segs + (SR_MAX_POINTS - 1) * SR_SEG_FLOATS;
    const float* groups = blocks + SR_TR_BLOCKS * SR_TR_BOUND_FLOATS;
    const int ns = sc->tr_num_segments, nb = sc->tr_num_blocks, ng = sc->tr_num_groups;
    for (int g = 0; g < ng; g++) {
        const bool hg = MASK ? (bool)((gm >> g) & 1u) : tr_bound_may_hit(groups + g * SR_TR_BOUND_FLOATS, o, d, seg, S, r);
        if (!__ballot(hg)) continue;
        const int b1 = min(nb, (g + 1) * SR_TR_GROUP);
        for (int b = g * SR_TR_GROUP; b < b1; b++) {
            const bool hb = hg && tr_bound_may_hit(blocks + b * SR_TR_BOUND_FLOATS, o, d, seg, S, r);
            if (!__ballot(hb)) continue;
            const int s1 = min(ns, (b + 1) * SR_TR_BLOCK);
            for (int s = b * SR_TR_BLOCK; s < s1; s++) {
                if (!hb) continue;
                const float* q = segs + s * SR_SEG_FLOATS;
                const m3 B = ldm(q + 3);
                consider(best, cyl_test(o, d, ld3(q), B, q[12], q[13], seg, p), p, o, SLOT_TR_CURVED, 0,
                         KEY_TR_CURVED0 + s);
            }
        }
    }
}

// The test ray's budget (round 6; the test-ray instantiations, TR): a
// lane's clearance from every test-ray cylinder, for the chords of a ball
// around the anchor A as the budget slots' (clearance_obj), so that a chord
// inside the lane's ball needs no test-ray test at all; before it, every
// chord of every ray was exact and tested while the overlay was visible
// (frag:760-803 in every step of frag:890-933). An accepted point of a
// cylinder test lies on the chord, within lat_margin of the lateral surface
// for every chord direction and within its height slab up to mu S: within
// a block's or group's bound radius of its centre (test_ray_bounds), or of
// the flat cylinder's axis segment by its radius, grown by those margins.
// For chords in a ball of radius W <= the clearance around A, S <= |A|_1 +
// 4 W + 1 (clearance_obj), W capped at SR_BUDGET_TMAX. Groups closer than
// SR_TR_REFINE take the better of their own bound and their blocks'.
#ifndef SR_TR_REFINE
#define SR_TR_REFINE 2.0f
#endif
#ifndef SR_TR_SKIP  // round 6: +5 % on the overlay at the headline size (profiles/r06/s51)
#define SR_TR_SKIP 1
#endif
// Blocks closer than SR_TR_SEG take the better of their bound and their
// segments' own capsules (orthonormal frames only: the segment's float frame
// measures lateral distance within 1e-5 of the true one there)
#ifndef SR_TR_SEG
#define SR_TR_SEG 0.5f
#endif
__device__ __forceinline__ float tr_clear_bound(const float* __restrict__ B, f3 A, float l1A, float r) {
    const f3 w = A - ld3(B);
    const float dist = __builtin_amdgcn_sqrtf(dot(w, w));
    const float d0 = dist - B[3];
    const float W = fminf(fmaxf(d0, 0.0f), SR_BUDGET_TMAX);
    const float Sb = l1A + __builtin_fmaf(4.0f, W, 1.0f);
    const float m = SR_MU_PLANAR * 1.001f * Sb + lat_margin_len(2.0f * W, Sb + B[9], r) * B[11] + 3.0e-5f * dist;
    return B[10] != 0.0f ? -INFINITY : d0 - m;
}
// One segment's capsule (its axis segment [pos, pos + h c1], radius r):
// -inf unless its frame is orthonormal (q[14], sr_api.cpp); the frame's
// 1e-5 tolerance moves lateral distances and the axis by at most 1e-5 of
// them, inside the 3e-5 allowance
__device__ __forceinline__ float tr_clear_segment(const float* __restrict__ q, f3 A, float l1A, float r) {
    const f3 w = A - ld3(q);
    const f3 ax = ld3(q + 6);
    float t = dot(w, ax);
    t = t > 0.0f ? t : 0.0f;
    t = t < q[12] ? t : q[12];
    const f3 d = w - ax * t;
    const float d0 = __builtin_amdgcn_sqrtf(dot(d, d)) - r;
    const float W = fminf(fmaxf(d0, 0.0f), SR_BUDGET_TMAX);
    const float Sb = l1A + __builtin_fmaf(4.0f, W, 1.0f);
    const float pl1 = fabsf(q[0]) + fabsf(q[1]) + fabsf(q[2]);
    const float m = SR_MU_PLANAR * 1.001f * Sb + lat_margin_len(2.0f * W, Sb + pl1, r) * 1.0001f +
                    3.0e-5f * (fabsf(w.x) + fabsf(w.y) + fabsf(w.z) + q[12] + r);
    return q[14] != 0.0f ? d0 - m : -INFINITY;
}
// gm (rlen >= 0): bit g for group g, bit 31 for the flat cylinder, set
// unless that part's clearance from A exceeds rlen (a chord within rlen of A
// cannot reach it: the S bound of a ball of radius W >= its clearance holds
// for it while rlen < SR_BUDGET_TMAX); NaN keeps the bit.
__device__ float clearance_tr(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs, f3 A, bool outward,
                              float a, float dip, float rlen, uint32_t& gm) {
    gm = 0xffffffffu;
    if (!(rlen < SR_BUDGET_TMAX)) rlen = INFINITY;
    const float r = sc->tr_radius;
    if (!(r > 0.0f)) return -INFINITY;
    // outward lanes (outward_clear's premises and S bound) beyond every accepted point
    if (outward) {
        const float S = __builtin_fmaf(0.01f * a, a, __builtin_fmaf(2.0f, a, 1.0f));
        if (a * dip > (sc->tr_far + SR_MU_PLANAR * S) * 1.001f + lat_margin_len(S, S + sc->tr_pl1, r) * sc->tr_fg[6]) {
            gm = 0u;
            return INFINITY;
        }
    }
    uint32_t mk = 0u;
    const float l1A = fabsf(A.x) + fabsf(A.y) + fabsf(A.z);
    float e;
    {  // the flat cylinder: within |M^-1| r (+ margins) of [pos, pos + length g] (sr_dev_scene.tr_fg)
        const float* t = sc->tr_flat;
        const float* fg = sc->tr_fg;
        const f3 w = A - ld3(t);
        const f3 g = ld3(fg);
        // the closest point of the axis segment, as a parameter in [0, length] (g . g within 1e-5 of 1)
        float h = dot(w, g) * __builtin_amdgcn_rcpf(dot(g, g));
        h = h > 0.0f ? h : 0.0f;
        h = h < t[12] ? h : t[12];
        const f3 q = w - g * h;
        const float d0 = __builtin_amdgcn_sqrtf(dot(q, q)) - r * fg[3];
        const float W = fminf(fmaxf(d0, 0.0f), SR_BUDGET_TMAX);
        const float Sb = l1A + __builtin_fmaf(4.0f, W, 1.0f);
        const float pl1 = fabsf(t[0]) + fabsf(t[1]) + fabsf(t[2]);
        const float m = SR_MU_PLANAR * 1.001f * Sb + lat_margin_len(2.0f * W, Sb + pl1, r) * fg[4] + fg[5] +
                        3.0e-5f * (fabsf(w.x) + fabsf(w.y) + fabsf(w.z) + t[12]);
        e = fg[3] > 0.0f ? d0 - m : -INFINITY;
        mk |= (uint32_t)!(e > rlen) << 31;
    }
    const float* blocks = segs + (SR_MAX_POINTS - 1) * SR_SEG_FLOATS;
    const float* groups = blocks + SR_TR_BLOCKS * SR_TR_BOUND_FLOATS;
    const int nb = sc->tr_num_blocks, ng = sc->tr_num_groups;
#if SR_TR_SKIP
    // SR_TR_SKIP: a group whose distance beyond its radius exceeds both this
    // lane's clearance so far and rlen by the largest margin any part can
    // take here (W at its cap) can neither lower the clearance nor be reached:
    // when that holds for every lane the group costs a distance test only
    const float Smax = l1A + __builtin_fmaf(4.0f, SR_BUDGET_TMAX, 1.0f);
    const float mmax = SR_MU_PLANAR * 1.001f * Smax + lat_margin_len(2.0f * SR_BUDGET_TMAX, Smax + sc->tr_pl1, r) * sc->tr_fg[6];
#endif
    for (int g = 0; g < ng; g++) {
#if SR_TR_SKIP
        {
            const float* B = groups + g * SR_TR_BOUND_FLOATS;
            const f3 w = A - ld3(B);
            const float lim = (fmaxf(e, rlen) + B[3] + mmax) * 1.0001f;
            if (!__ballot(!(dot(w, w) > lim * lim && lim > 0.0f && B[10] == 0.0f))) continue;
        }
#endif
        float eg = tr_clear_bound(groups + g * SR_TR_BOUND_FLOATS, A, l1A, r);
        if (__ballot(eg < SR_TR_REFINE)) {
            float eb = INFINITY;
            const int b1 = min(nb, (g + 1) * SR_TR_GROUP);
            for (int b = g * SR_TR_GROUP; b < b1; b++) {
                float ebb = tr_clear_bound(blocks + b * SR_TR_BOUND_FLOATS, A, l1A, r);
                if (SR_TR_SEG > 0.0f && __ballot(ebb < SR_TR_SEG)) {
                    float es = INFINITY;
                    const int s1 = min(sc->tr_num_segments, (b + 1) * SR_TR_BLOCK);
                    for (int k = b * SR_TR_BLOCK; k < s1; k++) es = nmin(es, tr_clear_segment(segs + k * SR_SEG_FLOATS, A, l1A, r));
                    ebb = es > ebb ? es : ebb;  // both bound the block's segments; NaN ebb stays NaN
                }
                eb = nmin(eb, ebb);
            }
            eg = eb > eg ? eb : eg;  // both bound the group's segments; NaN eg stays NaN
        }
        mk |= (uint32_t)!(eg > rlen) << g;
        e = nmin(e, eg);
    }
    gm = mk;
    return nmin(e, SR_BUDGET_TMAX);
}

// intersect(), frag:755-814, exhaustively: the closest hit along
// [o, o + max_lambda*d] (max_lambda < 0: unbounded).
__device__ __forceinline__ Hit closest_hit_all(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                               f3 o, f3 d, float max_lambda) {
    Hit best = no_hit();
    f3 p;
    consider(best, sphere_test(o, d, F3(0.0f, 0.0f, 0.0f), 1.0f, max_lambda, p), p, o, SLOT_BH, 0, KEY_BH);
    test_ray_hits(sc, segs, best, o, d, max_lambda);
    const int n = sc->num_objects;
    for (int k = 0; k < n; k++) test_object(best, sc->objs[k], k, o, d, max_lambda);
    return best;
}

// intersect() for one exact chord of the step loop with culling: the test
// rays, the objects tested every step (chord-culled ones only when the chord
// reaches their bounding sphere) and the budget slots in `reach`. Same
// winner as closest_hit_all (lexicographic keys, skipped tests provably
// miss). One copy of each exact test: candidates go into a wave-uniform
// object mask first.
// TR: the test rays are tested only when the test ray's budget may be reached
// (SR_REACH_TR; elsewhere every chord tests them)
template <bool TR = false>
__device__ __forceinline__ Hit closest_hit_chord(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                                 uint32_t reach, f3 o, f3 d, float seg, uint32_t trmask = 0xffffffffu) {
    Hit best = no_hit();
    if (!TR) test_ray_hits_culled(sc, segs, best, o, d, seg);
    else if (reach & SR_REACH_TR) test_ray_hits_culled<true>(sc, segs, best, o, d, seg, trmask);
    uint32_t om = 0;  // objects to test (wave-uniform)
    const int ns = sc->num_step;
    for (int j = 0; j < ns; j++) om |= 1u << sc->step_idx[j];
    if (reach & 1u) {  // BLACK_HOLE: sphere of radius 1 at the origin (frag:104, 757)
        f3 p;
        consider(best, sphere_test(o, d, F3(0.0f, 0.0f, 0.0f), 1.0f, seg, p), p, o, SLOT_BH, 0, KEY_BH);
    }
    for (uint32_t c = reach >> 1; c; c &= c - 1) om |= 1u << sc->budget_idx[__builtin_ctz(c)];
    if (om) {
        const float S = (fabsf(o.x) + fabsf(o.y) + fabsf(o.z)) + seg + 1.0f;
        for (; om; om &= om - 1) {
            const int k = __builtin_ctz(om);
            const sr_dev_obj& ob = sc->objs[k];
            if (ob.kind != SR_KIND_EXACT && !may_hit(ob, o, d, seg, S)) continue;
            SR_STAT(12, 1);
            test_object(best, ob, k, o, d, seg);
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

// APPROX: the binary32 library atan2 (a few ulp from the binary64-rounded
// value) for the step loop's opacity classification; `ok` turns false near the
// 0 / 2pi seam, where the two can land on opposite sides.
template <bool APPROX>
__device__ __forceinline__ float phi_of(f3 local, bool& ok) {
    float phi;
    if (APPROX) {
        phi = atan2f(local.x, local.z);
        ok = ok && fabsf(phi) > 1.0e-3f;
    } else {
        phi = t_atan2(local.x, local.z);
    }
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

// tangent_space + tangent_coordinates of a hit (frag:208-333). APPROX (the step
// loop's opacity test): binary32 atan2 / asin, `ok` false where that may
// move the uv across a seam; every other operation is the exact one.
template <bool APPROX>
__device__ __forceinline__ Surface surface_of_t(const sr_dev_obj& ob, const Hit& h, bool& ok) {
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
        s.phi = phi_of<APPROX>(local, ok);
        s.theta = APPROX ? asinf(local.y / f[SR_F_P0]) : t_asin(local.y / f[SR_F_P0]);
        s.uv = F2(s.phi / (2.0f * SR_PI), s.theta / SR_PI + 0.5f);
        return s;
    }
    case SR_OBJECT_DISK:
    case SR_OBJECT_HOLLOW_DISK: {  // frag:249-295
        f3 local = mtv(A, disp);
        s.phi = phi_of<APPROX>(local, ok);
        if (ob.type == SR_OBJECT_DISK) s.uv = F2(len(local) / f[17], s.phi / (2.0f * SR_PI));
        else s.uv = F2((len(local) - f[17]) / (f[18] - f[17]), s.phi / (2.0f * SR_PI));
        s.n = A.c1;
        return s;
    }
    case SR_OBJECT_CYLINDER: {  // frag:297-318
        s.n = nrm(disp);
        f3 local = mtv(A, disp);
        s.phi = phi_of<APPROX>(local, ok);
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

__device__ Surface surface_of(const sr_dev_obj& ob, const Hit& h) {
    bool ok = true;
    return surface_of_t<false>(ob, h, ok);
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

// Opacity of calculate_lighting's result for a chord hit, decided in the step
// loop without lighting (exact where it claims):
//   OP_OPAQUE: alpha == 1 exactly, the ray ends here (frag:932)
//   OP_ZERO  : vec4(0) (a single-sided surface seen from behind, frag:370-374):
//              adding it leaves frag unchanged (frag starts at +0 or 0.5 and
//              is never -0), the ray goes on
//   OP_MAYBE : anything else; the hit is queued for shading and the ray goes on
// Textured alpha: the bilinear footprint is located with binary32 uv (within
// far less than a texel of the shaded one) and is opaque when the opacity
// bitmap says every texel within SR_OPQ_RADIUS of it has alpha 255 (LERP
// filtering of four 1.0 alphas is exactly 1.0).
#define OP_OPAQUE 0
#define OP_ZERO 1
#define OP_MAYBE 2
__device__ __forceinline__ int hit_opacity_uniform(const sr_dev_scene* __restrict__ sc, const sr_dev_frame& fr,
                                                   const Tex& tx, int slot, int face, const Hit& hit, f3 view_dir,
                                                   bool zero_only) {
    if (slot == SLOT_BH) return OP_OPAQUE;
    if (slot == SLOT_TR_CURVED) return sc->tr_curved_color[3] == 1.0f ? OP_OPAQUE : OP_MAYBE;
    if (slot == SLOT_TR_FLAT) return sc->tr_flat_color[3] == 1.0f ? OP_OPAQUE : OP_MAYBE;
    const sr_dev_obj& ob = sc->objs[slot];
    int mi = ob.material_index;
    if (mi < 0 || mi >= SR_MAX_MATERIALS) mi = 0;
    const sr_material& m = sc->materials[mi];
    if (!m.double_sided_normals) {  // surface_of's normal, then flip_normals (shade_hit)
        const float* f = ob.f;
        f3 n;
        if (ob.type == SR_OBJECT_SPHERE || ob.type == SR_OBJECT_CYLINDER)
            n = nrm(hit.p - ld3(f + SR_F_POS));
        else if (ob.type == SR_OBJECT_BOX)
            n = ld3(f + SR_F_BOX_FACE0 + SR_F_FACE_STRIDE * face + 6);
        else
            n = ld3(f + SR_F_AXES + 3);
        if (m.flip_normals) n = n * -1.0f;
        if (dot(n, view_dir) < 0.0f) return OP_ZERO;
    }
    if (zero_only) return OP_MAYBE;
    if (m.texture_index < 0) return m.color[3] == 1.0f ? OP_OPAQUE : OP_MAYBE;
    if (ob.type == SR_OBJECT_PLANE || fr.filter_mode != SR_FILTER_LERP || !tx.opq || !tx.arr || fr.arr_w <= 0 ||
        fr.arr_h <= 0 || fr.arr_layers <= 0)
        return OP_MAYBE;
    Hit hh = hit;
    hh.face = face;
    bool ok = true;
    f2 uv = surface_of_t<true>(ob, hh, ok).uv;
    if (!ok) return OP_MAYBE;
    if (m.swap_uvs) uv = F2(uv.y, uv.x);
    if (m.invert_uv_x) uv.x = 1.0f - uv.x;
    if (m.invert_uv_y) uv.y = 1.0f - uv.y;
    const int ti = m.texture_index < SR_MAX_TEXTURES ? m.texture_index : 0;
    // the sizes pinned here: hoisted out of the step loop (their float
    // conversions, the divisors' scalings and the wrap's magic reciprocals)
    // they stayed live across it and were spilled
    float tsx = sc->texture_sizes[ti][0], tsy = sc->texture_sizes[ti][1];
    float msx = sc->max_texture_size[0], msy = sc->max_texture_size[1];
    int aw = fr.arr_w, ah = fr.arr_h;
    asm volatile("" : "+s"(tsx), "+s"(tsy), "+s"(msx), "+s"(msy), "+s"(aw), "+s"(ah));
    f2 r = F2((uv.x * tsx) / msx, (uv.y * tsy) / msy);
    int layer = m.texture_index;
    if (layer > fr.arr_layers - 1) layer = fr.arr_layers - 1;
    const float s = r.x * (float)aw - 0.5f;  // bilinear()
    const float t = r.y * (float)ah - 0.5f;
    if (!(fabsf(s) < 4194304.0f) || !(fabsf(t) < 4194304.0f)) return OP_MAYBE;
    const int x = wrap_rep(floorf(s), aw), y = wrap_rep(floorf(t), ah);
    const size_t stride = ((size_t)aw + 7) >> 3;
    const uint8_t bits = tx.opq[((size_t)layer * (size_t)ah + (size_t)y) * stride + (size_t)(x >> 3)];
    return (bits >> (x & 7)) & 1 ? OP_OPAQUE : OP_MAYBE;
}

__device__ __forceinline__ int hit_opacity(const sr_dev_scene* __restrict__ sc, const sr_dev_frame& fr,
                                           const Tex& tx, const Hit& hit, f3 view_dir, bool zero_only) {
    const int key = hit.slot * 8 + hit.face;
    int op;
    for (;;) {  // waterfall: object data as wave-uniform loads
        const int first = __builtin_amdgcn_readfirstlane(key);
        if (key == first) {
            op = hit_opacity_uniform(sc, fr, tx, __builtin_amdgcn_readfirstlane(hit.slot),
                                     __builtin_amdgcn_readfirstlane(hit.face), hit, view_dir, zero_only);
            break;
        }
    }
    return op;
}

__device__ __forceinline__ f4 intersect_color(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                              const sr_dev_frame& fr, const Tex& tx, f3 o, f3 d,
                                              float max_lambda) {
    Hit h = closest_hit_all(sc, segs, o, d, max_lambda);
    if (h.slot == SLOT_NONE) return F4(0.0f, 0.0f, 0.0f, 0.0f);
    return shade(sc, fr, tx, h, -d);
}

__device__ __forceinline__ uint32_t unorm8(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x >= 1.0f) return 255u;
    return (uint32_t)floorf(x * 255.0f + 0.5f);
}

// ---- pixel pipeline ---------------------------------------------------------
// A frame is three launches on one stream:
//   sr_integrate_kernel : camera ray + RK4 step loop (integration registers
//                         only). Chord hits are classified by hit_opacity:
//                         back faces are skipped, hits that may be translucent
//                         are recorded and the ray goes on, the first opaque
//                         hit (or the end of the ray) stops it
//   sr_shade_kernel     : calculate_lighting of the recorded hits in order,
//                         skybox / unbounded flat intersect, final pixels; a
//                         pixel whose recorded hits were all translucent and
//                         whose ray stopped early is queued for resumption
//   sr_resume_kernel    : the queued pixels (dense worklist), integrated and
//                         shaded in rounds to completion
// Pixel state between launches lives in SoA planes ps[field * n + id], id = the
// pixel's thread index in the launch grid (coalesced for every kernel).
#define ST_DONE 0  // no ray (percent_black): frag = the crosshair colour
#define ST_HIT 1   // stopped at an opaque-classified hit (the last recorded one)
#define ST_MORE 2  // stopped with SR_PS_HITS translucent hits recorded
#define ST_FLAT 3  // unbounded intersect(ray), then get_bg if alpha != 1 (frag:874-876, 895-897, 903-905)
#define ST_BG 4    // get_bg(rd) (frag:921-922 break, 935)
#define ST_BH 5    // stopped in the black hole (opaque black) after the logged hits

// The hand-off is written only where the next kernel reads it, in records
// that one lane writes whole (partial writes of shared sectors by scattered
// lanes cost whole sectors: as SoA planes the sparse hit records made the
// hand-off 2.4x its size):
//   every pixel      one 16-byte store {packed word, rd} (rd: the final
//                    direction, read by escaped and flat rays)
//   logged hits      one 32-byte record each {p, key | steps << 8, dir},
//                    hit-major (hit j of neighbouring pixels adjacent: a
//                    wave's records share lines, 150 -> 126 MB per headline
//                    frame); a ray that ends in the black hole gets status
//                    ST_BH instead (its colour is a constant, shade_hit)
//   ST_FLAT          ro (plane)
//   ST_MORE          the resumable state (planes): the log filled with
//                    translucent hits; sr_resume_kernel continues the ray
// An ST_HIT pixel's last logged hit is opaque exactly (hit_opacity), so the
// shade kernel always finishes it: it keeps no resumable state.
enum {
    PS_REC = 0,                       // [4 floats / px] word, rd[3]
    PS_HITS = 4,                      // [8 floats / hit, (j * n + id) * 8] p[3], (key + 24) | steps << 8, dir[3], -
    PS_PLANES = 4 + 8 * SR_PS_HITS,   // planes (field * n + id) from here:
    PS_I = 0, PS_FRAG = 1, PS_RO = 5, PS_NV = 8, PS_TV = 11, PS_U = 14, PS_DU = 15
};
static_assert(PS_PLANES + 16 == SR_PS_FIELDS, "pixel-state layout");
// key = slot * 8 + face in [-24, 167]: slots -3 .. SR_MAX_OBJECTS - 1
#define PS_KEY_BIAS 24
static_assert((SR_MAX_OBJECTS - 1) * 8 + 7 + PS_KEY_BIAS < 256, "hit key fits 8 bits");
// steps <= SR_MAX_STEPS (sr_api.cpp build_frame): 24 bits
static_assert(SR_MAX_STEPS < (1 << 24), "step count fits the packed word");
__device__ __forceinline__ int ps_word(int st, int nh, int steps) {
    return (int)((uint32_t)st | ((uint32_t)nh << 3) | ((uint32_t)steps << 8));
}

struct Ray {
    f3 ro, rd, nv, tv;
    float u, du;
    int i, steps;
    SR_PROBE_RAY_FIELDS  // measurement builds only (probes.h)
};

struct Pix {
    int px, k, py;
};

// 16x16 workgroup tile of four 8x8 wave tiles; false for threads off the frame
__device__ __forceinline__ bool pixel_of(const sr_dev_frame& fr, int block, int t, Pix& q) {
    const int gx = (fr.width + 15) >> 4;
    const int bx = block % gx, by = block / gx;
    const int lane = t & 63, wave = t >> 6;
    q.px = bx * 16 + (wave & 1) * 8 + (lane & 7);
    q.k = by * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (q.px >= fr.width || q.k >= fr.nrows) return false;
    if (fr.block_list) {  // sr_render_block_list: a rank's cost-balanced blocks
        const int b = fr.block_list[q.k / fr.block_rows];
        if (b < 0) return false;
        q.py = b * fr.block_rows + (q.k % fr.block_rows);
    } else {
        q.py = fr.row_base + (q.k / fr.block_rows) * fr.block_stride + (q.k % fr.block_rows);
    }
    return q.py < fr.height;
}

struct PS {
    float* __restrict__ p;
    size_t n;
    // the 16-byte record and the hit records (one lane, whole records)
    __device__ __forceinline__ void put_rec(size_t id, int w, f3 rd) const {
        *reinterpret_cast<float4*>(p + 4 * id) = make_float4(__int_as_float(w), rd.x, rd.y, rd.z);
    }
    __device__ __forceinline__ float4 get_rec(size_t id) const { return *reinterpret_cast<const float4*>(p + 4 * id); }
    __device__ __forceinline__ float* hit(size_t id, int j) const {
        float* const row = p + 4 * n + (size_t)j * n * 8;  // hit j's plane
        return row + id * 8;
    }
    // the same for a 32-bit id (the integrate kernel's LDS pixel ids): one
    // 32 x 32 + 64-bit multiply-add, no zero-extended id (the compiler kept
    // that zero in a register spilled across the step loop)
    __device__ __forceinline__ float* hit32(uint32_t id, int j) const {
        const uint64_t row = reinterpret_cast<uint64_t>(p + 4 * n + (size_t)j * n * 8);
        uint64_t a, carry;
        asm("v_mad_u64_u32 %0, %1, %2, 32, %3" : "=v"(a), "=s"(carry) : "v"(id), "v"(row));
        return reinterpret_cast<float*>(a);
    }
    // planes of the resumable / flat-ray state
    __device__ __forceinline__ float& at(int f, size_t id) const { return p[(size_t)(PS_PLANES + f) * n + id]; }
    __device__ __forceinline__ void put3(int f, size_t id, f3 v) const {
        at(f, id) = v.x;
        at(f + 1, id) = v.y;
        at(f + 2, id) = v.z;
    }
    __device__ __forceinline__ f3 get3(int f, size_t id) const { return F3(at(f, id), at(f + 1, id), at(f + 2, id)); }
    __device__ __forceinline__ void puti(int f, size_t id, int v) const { at(f, id) = __int_as_float(v); }
    __device__ __forceinline__ int geti(int f, size_t id) const { return __float_as_int(at(f, id)); }
    __device__ __forceinline__ void put4(int f, size_t id, f4 v) const {
        at(f, id) = v.x;
        at(f + 1, id) = v.y;
        at(f + 2, id) = v.z;
        at(f + 3, id) = v.w;
    }
    __device__ __forceinline__ f4 get4(int f, size_t id) const {
        return F4(at(f, id), at(f + 1, id), at(f + 2, id), at(f + 3, id));
    }
};

// frag:845-857: the crosshair's initial FragColor
__device__ __forceinline__ f4 crosshair_frag(const sr_dev_frame& fr, const Pix& q) {
    f4 frag = F4(0.0f, 0.0f, 0.0f, 0.0f);
    if (fr.crosshair) {
        f2 uv = F2((float)(2 * q.px + 1) / (float)fr.width - 1.0f, (float)(2 * q.py + 1) / (float)fr.height - 1.0f);
        float hx = fabsf(uv.x * fr.res_x / 2.0f), hy = fabsf(uv.y * fr.res_y / 2.0f);
        if ((hx < 1.0f && hy > 5.0f && hy < 15.0f) || (hy < 1.0f && hx > 5.0f && hx < 15.0f))
            frag = F4(0.5f, 0.5f, 0.5f, 0.5f);
    }
    return frag;
}

// frag:859-889: camera ray, flat / percent_black early outs and the initial
// (u, du) of the geodesic. Returns ST_FLAT, ST_DONE or -1 (integrate).
__device__ __forceinline__ int init_pixel(const sr_dev_frame& fr, const sr_dev_cam& cam, const Pix& q, Ray& r) {
    // full_screen_quad.vert:7-10: uv = NDC of the pixel centre
    f2 uv = F2((float)(2 * q.px + 1) / (float)fr.width - 1.0f, (float)(2 * q.py + 1) / (float)fr.height - 1.0f);
    f2 uvv = F2(uv.x, uv.y * fr.res_y / fr.res_x);
    m3 axes = ldm(cam.axes);
    r.ro = ld3(cam.pos);
    r.rd = nrm(mv(axes, F3(uvv.x, uvv.y, cam.ray_forward)));
    r.nv = nrm(r.ro);
    r.steps = 0;
    r.i = 0;
    SR_PROBE(probe_ray_init(r));
    const bool flat = fr.raytrace_type == SR_RAYTRACE_FLAT ||
                      (fr.raytrace_type == SR_RAYTRACE_HALF_WIDTH && uv.x > 2.0f * fr.curved_percentage + -1.0f) ||
                      (fr.raytrace_type == SR_RAYTRACE_HALF_HEIGHT && uv.y > 2.0f * fr.curved_percentage + -1.0f);
    if (flat || fabsf(dot(r.rd, r.nv)) >= 1.0f - SR_EPS) return ST_FLAT;
    if (fr.percent_black >= 0.0f) {  // rand(uv_vec) <= percent_black, frag:839-841, 879; rand is in [0, 1)
        float x = t_sin(uvv.x * 12.9898f + uvv.y * 78.233f) * 43758.5453f;
        if (x - floorf(x) <= fr.percent_black) return ST_DONE;
    }
    // frag:883-889
    r.tv = nrm(cross(cross(r.nv, r.rd), r.nv));
    r.u = 1.0f / len(r.ro);
    r.du = -r.u * dot(r.rd, r.nv) / dot(r.rd, r.tv);
    return -1;
}

// Where integrate() records translucent hits (sr_integrate_kernel only)
// The integrate kernel's pixel ids, one LDS word per thread: read where a hit
// is logged and at the hand-off, not held in registers across the step loop
// (a 64-bit id there was spilled to scratch for the whole loop).
__shared__ uint32_t sr_lds_pid[SR_WG];
struct HitLog {
    PS ps;
    int n;
    // a volatile read where it is used: the hit-record address is not hoisted
    // out of the step loop (a 64-bit VGPR pair there was spilled), through an
    // LDS-typed pointer: a ds_read with a 32-bit address (a generic pointer is
    // a flat load with a 64-bit one, also spilled); the index passes through
    // an empty asm so that the LDS address is formed here too (hoisted, it was
    // one more register live across the step loop, spilled)
    __device__ __forceinline__ uint32_t id() const {
        typedef volatile const __attribute__((address_space(3))) uint32_t lds_u32;
        uint32_t t = threadIdx.x;
        asm volatile("" : "+v"(t));
        return *(lds_u32*)&sr_lds_pid[t];
    }
};

// Chord end point of step j, frag:924: (nv cos phi_j + tv sin phi_j) / u_j
__device__ __forceinline__ f3 point_at(const Ray& r, float u, float c, float s) { return (r.nv * c + r.tv * s) / u; }

// The same point from an approximate radius rad ~ 1/u (no division): within
// 1.1e-6 rad of the exact float evaluation
__device__ __forceinline__ f3 point_near(const Ray& r, float rad, float c, float s) {
    return r.nv * (rad * c) + r.tv * (rad * s);
}

// absolute error bound of point_near / chord components for radii rA, rB
__device__ __forceinline__ float point_err(float rA, float rB) { return 4.0e-6f * (rA + rB); }

// ddu, frag:336-338
__device__ __forceinline__ float ddu(float u) { return -u * (1.0f - 1.5f * u); }

// rk4_step, frag:341-355, plus the `u += .x; du += .y` of frag:918-919 (h6 =
// `delta_phi / 6.` and hh = 0.5 h, computed on the host):
//   (ua, k2) = (u, u') + (k1, l1) hh           l2 = ddu(ua)
//   (ub, k3) = (u, u') + (k2, l2) hh           l3 = ddu(ub)
//   (uc, k4) = (u, u') + (k3, l3) h            l4 = ddu(uc)
//   (u, u') += h6 ((fma(2, (k3, l3), fma(2, (k2, l2), (k1, l1)))) + (k4, l4))
// in scalar binary32 instructions. The u and u' halves of a stage are the
// same operations on different operands; as packed pairs (v_pk_mul_f32 /
// v_pk_add_f32 / v_pk_fma_f32; round 3, removed since) they are half the instructions
// but each takes the SIMD's issue for twice as long as a scalar one, and
// need hazard s_nops: with six waves per SIMD the scalar form renders 2.9 %
// more frames per second (one frame alone, latency bound, is 3.5 % slower;
// profiles/r03/s13_*). Bit-identical to the reference's expressions: (0.5 q) h and q (0.5 h) are
// both the rounding of the same product, as scaling by 0.5 is exact for
// non-subnormal q (the stage values here are never subnormal: DESIGN.md §4);
// and 2 q is exact, so fma(2, q, a) is the rounding of a + 2 q, as the
// reference's a + (2. * q).
// The step table's entry is one float4 {h, h / 6, cos phi, sin phi} (16
// bytes), and the reference's a + 0.5 q h (frag:345-349: (0.5 q) h) is
// computed as fma(0.5, q h, a): (0.5 q) h and 0.5 (q h) are the rounding of
// the same product (scaling by 0.5 is exact), and the fused add of the exact
// 0.5 (q h) rounds once, as the reference's separate add does. Against a
// 32-byte entry that carried 0.5 h: half the scalar loads and SGPRs of the
// fast loop's prefetch, 0.854 -> 0.843 ms per frame in the pipeline A/B,
// one frame alone 1.193 -> 1.122 ms (profiles/r05/s4_ab_*.log).
__device__ __forceinline__ float half_step(float a, float q, float h) { return __builtin_fmaf(0.5f, q * h, a); }
__device__ __forceinline__ void rk4_step(float u, float du, float h, float h6, float& un, float& dun) {
    const float k1 = du;
    const float l1 = ddu(u);
    const float k2 = half_step(du, l1, h);
    const float l2 = ddu(half_step(u, k1, h));
    const float k3 = half_step(du, l2, h);
    const float l3 = ddu(half_step(u, k2, h));
    const float k4 = du + l3 * h;
    const float l4 = ddu(u + k3 * h);
    un = u + h6 * (__builtin_fmaf(2.0f, k3, __builtin_fmaf(2.0f, k2, k1)) + k4);
    dun = du + h6 * (__builtin_fmaf(2.0f, l3, __builtin_fmaf(2.0f, l2, l1)) + l4);
}

// The flat intersect of a ray that left the u_f sphere (frag:895-897,
// 903-905) when it provably hits nothing: from ro beyond sc->flat_miss_r2
// (twice the reach of every object's acceptance region and the black hole,
// plus one) and not approaching the origin (ro . rd >= 0, within rounding
// far below that factor), every point of the ray is at least |ro| from the
// origin. Its colour is then get_bg(rd) alone (intersect adds vec4(0), frag
// is never -0), exactly ST_BG's: the shade kernel skips the exhaustive
// intersect, and the hand-off the ray origin (1.65 M of the headline frame's
// 2.07 M pixels end this way).
__device__ __forceinline__ bool flat_misses(const sr_dev_scene* __restrict__ sc, f3 ro, f3 rd) {
    return !sc->tr_visible && dot(ro, rd) >= 0.0f && dot(ro, ro) > sc->flat_miss_r2;
}

// The step loop, frag:890-933, from step r.i (entry: r.u = u after step
// r.i - 1, r.ro / r.rd = that step's chord end and direction).
//
// Lazy chords (CULL): the reference computes every chord exactly (two
// divisions by u, a sqrt and three divisions by its length); here a step
// only advances (u, du) and tests its end point against the lane's ball
// (ball_q: every budget covers the chords whose ends lie in it).
// When a budget is spent (or the chord may be near-parallel to a budgeted
// cylinder) the wave runs a budget event on the approximate chord
// (point_near); only when a slot may be reached is the exact chord
// materialised - the reference's float expressions on the same operands, so
// bit-identical - and tested. Exits and reseeds materialise it too.
//
// Hits that contribute vec4(0) are skipped. RECORD (sr_integrate_kernel):
// possibly translucent hits are logged and the ray goes on; it stops at an
// opaque-classified hit (ST_HIT, logged last) or when the log is full
// (ST_MORE). Otherwise (resume): stops at the first hit not skipped (ST_HIT,
// in `hit`). r.i = the stopping step. Ends of the ray: ST_FLAT / ST_BG.
// sr_wave_costs: budget events of each wave of the integrate kernel's workgroup
__shared__ int sr_lds_ev[SR_WG / 64];

template <bool CULL, bool RECORD, bool WCOST = false, int NB = SR_MAX_BUDGET, int FU = SR_FAST_UNROLL,
          int NC = SR_NC_KERNEL, bool TR = false>
__device__ __forceinline__ int integrate(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                         const float4* __restrict__ tbl, const sr_dev_frame& fr, const Tex& tx,
                                         Ray& r, Hit& hit, HitLog& log) {
    using BS = Budget<NB, NC, TR && CULL>;
    __shared__ float lds_E[BS::L::ROWS * SR_E_STRIDE];  // blockDim.x == SR_E_STRIDE
    BS bs;
    bs.E = lds_E + threadIdx.x;
    SR_PROBE(SR_PROF_CLOCK(prof_bi_));  // budget_init's cycles (section 22)
    if (!CULL) bs.setUhi(INFINITY);
    if (CULL)
        // the ray's start (sr_integrate_kernel): r.rd is the orbit's tangent at
        // r.ro; a resumed ray's is a chord direction, so no start window. (Round
        // 6: the resume passed a NaN direction "to get 0", but fminf drops a NaN
        // operand, and plane_window_start returned its caps: a window toward a
        // plane the resumed ray was heading into, missing its hit whenever no
        // wave-mate's event re-anchored the slot first - three pixels of a
        // four-frame batch of the stress scene, varying run to run with the
        // worklist's order, tests/test_gpu_parity.py test_resumed_rays_*.)
        budget_init<RECORD>(sc, segs, bs, r.ro, r.nv, r.tv, r.du < 0.0f && r.u < 0.6f, fr.out_dip,
                            fr.win_ok && fr.out_dip > SR_BH_DIP, r.du > 0.0f, fr.xplane_s, fr.bh_u2, fr.xlow_need,
                            fr.xperi_e, orbit_e(r.u, r.du), r.rd, fr.max_dphi);
    SR_PROBE(FireProbe<Ray, BS> fire_probe_(r, bs));
    const int N = fr.max_steps;
    // every chord is tested exactly when objects outside the budget slots or
    // the test rays are present (wave-uniform); the test-ray instantiations
    // budget the test rays (clearance_tr)
    const bool every = !CULL || sc->num_step > 0 || (sc->tr_visible && !BS::TR);
    // Chord bookkeeping: im = the step whose chord r.ro / r.rd hold; up = u
    // after step i - 2 (outside the fast loop: it leaves `up` behind and
    // recover_up() recomputes it); rA ~ 1 / u after step i - 1. r.steps =
    // sbase + (steps begun). In sr_integrate_kernel the step index i is
    // wave-uniform.
    int im = r.i - 1;
    float up = 0.0f;
    float rA = __builtin_amdgcn_rcpf(r.u);
    const int sbase = r.steps - r.i;
    // {cos phi, sin phi} after step j (step -1: the camera, phi = 0)
    auto phi_cs = [&](int j) -> f2 {
        if (j < 0) return F2(1.0f, 0.0f);
        const float4 t = tbl[j];
        return F2(t.z, t.w);
    };
    // materialise the chord of step i - 1 (its end point from r.u, its start
    // from r.ro when that is step i - 2, else from up)
    auto settle_prev = [&](int i) {
        if (im == i - 1) return;
        const f2 p1 = phi_cs(i - 1);
        f3 A;
        if (im == i - 2) {
            A = r.ro;
        } else {
            const f2 p2 = phi_cs(i - 2);
            A = point_at(r, up, p2.x, p2.y);
        }
        f3 B = point_at(r, r.u, p1.x, p1.y);
        f3 delta = B - A;
        float seg = len(delta);
        r.rd = delta / seg;
        r.ro = B;
        im = i - 1;
    };
    bool force = false;  // this lane's next chord is charged exactly (new orbital frame)
    int i = r.i;
    SR_PROBE(LoopProbe lp(i); SR_PROF_LOOP_START(r, bs, prof_bi_));
    for (;;) {
        if (RECORD) i = __builtin_amdgcn_readfirstlane(i);  // every lane started at step 0: keep i scalar
        // (sr_resume_kernel's lanes are unrelated rays at their own steps)
        if (i >= N) break;
        // frag:891-912, the top of step i (the fast loop below leaves a step
        // early whenever some lane's u drops below u_f, so this is where
        // every reseed happens)
        SR_PT(21);
        if (__ballot(r.u < fr.u_f)) {
            if (r.u < fr.u_f) {
                r.i = i;
                r.steps = sbase + i + 1;
                settle_prev(i);
                // the new orbital plane has its own coordinates: charge the
                // displacement from the old centre to the chord start r.ro
                // here, the new chord at the forced event (reseeded)
                if (CULL)
                {
                    const float ocx = bs.cx(), ocy = bs.cy();
                    bs.setT(__builtin_fmaf(len(r.ro - (r.nv * ocx + r.tv * ocy)), 1.0101f,
                                           3.0e-6f * (fabsf(ocx) + fabsf(ocy) + 1.0f)));
                }
                float lam;
                if (!sphere_lambda_r2(r.ro, r.rd, F3(0.0f, 0.0f, 0.0f), fr.uf_radius2, -1.0f, lam))
                    return flat_misses(sc, r.ro, r.rd) ? ST_BG : ST_FLAT;
                const f3 q = r.ro + r.rd * lam;  // sphere_intersect's point (computed past the exit)
                r.nv = nrm(q);
                if (fabsf(dot(r.rd, r.nv)) >= 1.0f - SR_EPS) return flat_misses(sc, r.ro, r.rd) ? ST_BG : ST_FLAT;
                r.tv = nrm(cross(cross(r.nv, r.rd), r.nv));
                r.u = 1.0f / len(q);
                r.du = -r.u * dot(r.rd, r.nv) / dot(r.rd, r.tv);
                if (CULL) budget_frame(sc, bs, r.nv, r.tv, fr.xplane_s, fr.xlow_need, fr.xperi_e,
                                          orbit_e(r.u, r.du));
                force = true;  // the chord starts at the exact r.ro
            }
            SR_PT(1);
        }
        // ---- fast loop: RK4, the ball test of the step's end point and
        // the u compares per step, the same instructions on every lane and
        // wave-uniform exits only. The wave leaves with step i computed but
        // not applied when some lane needs attention: a budget event (the
        // end point left its ball, ball_q; an empty ball while every chord is
        // tested or this lane's chord is forced), an exit (u < 0) or a reseed
        // at the next step (u < u_f).
        // Only numbers leave the loop (lane-mask booleans carried out of it
        // cost exec-mask bookkeeping on every step).
        const float bm = bs.m();
        const float lim0 = (every || force) ? -INFINITY : bm;
        const float uhi = bs.uhi();  // u > uhi: the chord left the black hole's u window
        // u < ulo: a reseed or exit at the next step, or the inner window's end
        const float ulo = BS::ulo_of(uhi, fr.u_f);
        const float bcx = CULL ? bs.cx() : 0.0f, bcy = CULL ? bs.cy() : 0.0f;
        const float bn = -2.0f * bcx, bt = -2.0f * bcy;
        const float q0 = (!CULL || every || force) ? INFINITY : ball_q(bm, bcx, bcy);
        float vb;  // the step's ball test (< 0: inside)
        // some lane's orbital plane nearly contains a budgeted cylinder's axis
        // (bs.cm changes only at reseeds, outside the fast loop)
        const uint32_t bcm = CULL ? bs.cm() : 0u;
        // (an instantiation without budgeted cylinders, NC = 0, has no such lane)
        const bool any_cm = CULL && NC > 0 && __ballot(bcm != 0u);
        // {step_size, step_size / 6, cos phi, sin phi}, {g, 0.5 step_size, K_i, -},
        // read through the constant address space: scalar loads
        const sr_cfloat4* tp = (const sr_cfloat4*)(tbl + i);
        float4 e;
        float un, dun, rB;
        uint32_t par;
        // Three versions of the loop: without a lane whose orbital plane nearly
        // contains a budgeted cylinder's axis (the usual case, CMV 0) the
        // limit is fixed and there is no direction test; with one, the chord's
        // direction is tested on every step (CMV 1) or, when every lane is in
        // a black-hole u window, on the first step of each FU-step
        // iteration only (CMV 2, SR_CM_ITER): with u <= uhi < 1 at every
        // applied step's ends the orbit's tangent turns by at most 1.5 u per
        // radian of phi (dpsi/dphi = 1.5 u^3 / (u^2 + u'^2)), and a chord's
        // direction is the tangent's at a point of its own step, so the next
        // FU - 1 chords lie within 1.515 FU max_dphi of the tested one's
        // direction (4.55 max_dphi at three steps; round 6: the bound was
        // still the three-step one when the loop went to four), below
        // the 0.0555 rad between chord_parallel's threshold (|d_perp|^2 <
        // 2 SR_BUDGET_DPMIN, direction known to 0.004) and the margin's
        // (|d_perp|^2 >= SR_BUDGET_DPMIN). The exit step's chord is tested
        // again in the slow path (its end may lie beyond the window).
        auto fast = [&](auto cm_tag) {
            constexpr int CMV = decltype(cm_tag)::value;
            constexpr bool CM = CMV != 0;
            par = 0;
            e = ldc(tp);
            f2 pc = CM ? phi_cs(i - 1) : F2(0.0f, 0.0f);  // {cos, sin} phi after the previous step
            const CylDirs<NC> cd = CM ? cyl_dirs(sc, bs) : CylDirs<NC>{};
            const float qh = CM ? ((every || force) ? INFINITY : ball_q(nmin(bm, bs.mh()), bcx, bcy)) : q0;
            // the LDS reads land before the loop: a wait for them inside it
            // would also wait for the step table's prefetch (one counter)
            if (CM) __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            float qit = q0;  // CMV 2: the iteration's ball
            // Step i from entry e: RK4, the ball test of its end point and the
            // exit test; true when some lane needs attention (the step is then
            // computed but not applied). k: the step's place in the iteration.
            auto compute = [&](int k) -> bool {
                rk4_step(r.u, r.du, e.x, e.y, un, dun);  // frag:914-919
                // the end point against the ball (ball_q): a multiply and three FMAs
                float q = q0;
                if (CULL && CMV == 1) {
                    rB = __builtin_amdgcn_rcpf(un);
                    par = chord_parallel(bcm, cd, rB * e.z - rA * pc.x, rB * e.w - rA * pc.y, point_err(rA, rB));
                    q = par ? qh : q0;
                }
                if (CULL && CMV == 2) {
                    if (k == 0) {
                        const float ra = __builtin_amdgcn_rcpf(r.u);
                        rB = __builtin_amdgcn_rcpf(un);
                        par = chord_parallel(bcm, cd, rB * e.z - ra * pc.x, rB * e.w - ra * pc.y, point_err(ra, rB));
                        qit = par ? qh : q0;
                    }
                    q = qit;
                }
                vb = __builtin_fmaf(__builtin_fmaf(q, un, __builtin_fmaf(bt, e.w, bn * e.z)), un, 1.0f);
                SR_STAT(0, 1);
                SR_STAT(13, __popcll(__ballot(1)));
                SR_PROBE(if (CM) SR_STAT_MAIN(31, 1));  // wave-steps of the cylinder-plane fast loop
                SR_PROBE(if (!(un < 1.0e20f)) SR_TRACE_AT("fast i=%d u=%g un=%g dun=%g vb=%g q=%g\n", i, r.u, un,
                                                            dun, vb, q));
                return __ballot(!(vb < 0.0f) || un < ulo || un > uhi);
            };
            // apply step i and move to entry en of step i + 1
            auto apply = [&](float4 en) -> bool {
                r.u = un;
                r.du = dun;
                if (CMV == 1) rA = rB;
                tp += 1;
                if (CM) pc = F2(e.z, e.w);
                e = en;
                return ++i >= N;
            };
            // FU (SR_FAST_UNROLL) steps per iteration: the entries of steps i + 1
            // .. i + FU are loaded together at its top (the table
            // holds max_steps + 4 entries), so step i + 1 waits only for loads
            // issued a step earlier, and the copies rename the registers one
            // step would rotate. A use on each exit path keeps the loads where
            // they are issued (sunk to their first use, they would be waited
            // at once).
            for (;;) {
                float4 nx[FU];
#pragma unroll
                for (int k = 0; k < FU; k++) nx[k] = ldc(tp + 1 + k);
                __builtin_amdgcn_sched_barrier(0);
                bool leave = false;
#pragma unroll
                for (int k = 0; k < FU && !leave; k++) {
                    if (compute(k)) {
#pragma unroll
                        for (int j = k; j < FU; j++) asm volatile("; keep %0" ::"s"(nx[j].x));
                        leave = true;
                    } else {
                        leave = apply(nx[k]);
                    }
                }
                if (leave) break;
            }
        };
        // Coasting: when every lane's limit is +inf (escaping rays that have
        // passed every object: outward_clear gave all their budgets +inf),
        // nothing but u < u_f (or the end of the loop) can stop a lane until
        // its next event or reseed, which re-anchors every slot: a step is
        // RK4 and that compare. The chord bound and its path T are skipped
        // (T is reset at that re-anchor; rB is restored on the way out), so
        // the iterates are the same. Only outward lanes (u < 0.6 falling)
        // coast: u stays finite.
        auto coast = [&]() {
            e = ldc(tp);
            for (;;) {
                float4 nx[FU];
#pragma unroll
                for (int k = 0; k < FU; k++) nx[k] = ldc(tp + 1 + k);
                __builtin_amdgcn_sched_barrier(0);
                bool leave = false;
#pragma unroll
                for (int k = 0; k < FU && !leave; k++) {
                    rk4_step(r.u, r.du, e.x, e.y, un, dun);  // frag:914-919
                    SR_STAT(0, 1);
                    SR_STAT(11, 1);  // coasting wave-steps
                    SR_STAT(13, __popcll(__ballot(1)));
                    if (__ballot(!(un >= ulo && un <= uhi))) {  // NaN leaves too
#pragma unroll
                        for (int j = k; j < FU; j++) asm volatile("; keep %0" ::"s"(nx[j].x));
                        leave = true;
                    } else {
                        r.u = un;
                        r.du = dun;
                        tp += 1;
                        e = nx[k];
                        leave = ++i >= N;
                    }
                }
                if (leave) break;
            }
            // the state the full loop leaves: step i's radius, no charge (every budget is +inf)
            rA = __builtin_amdgcn_rcpf(r.u);
            rB = __builtin_amdgcn_rcpf(un);
            par = 0;
            vb = -1.0f;  // inside every (infinite) budget
        };
        // The fast loop does not carry `up` (u after step i - 2): the copy
        // cost a register move per step in its rotation (42.3 -> 41.7 VALU
        // per step). The two exits that need it - u < 0 (the previous chord,
        // frag:921-922) and the end of the loop - recompute it from the
        // loop's entry state with the same RK4 steps (bit-identical).
        const int ick = i;
        const float uck = r.u, duck = r.du, upck = up;
        auto recover_up = [&](int ie) -> float {  // u after step ie - 2
            if (ie == ick) return upck;
            float u = uck, du = duck;
            for (int j = ick; j < ie - 1; j++) {  // steps ick .. ie - 2
                const float4 t0 = tbl[j];
                float un2, dun2;
                rk4_step(u, du, t0.x, t0.y, un2, dun2);  // the fast loop's operands
                u = un2;
                du = dun2;
            }
            return u;
        };
        // CMV 2 needs every lane in a u window (u <= uhi < 1 at applied steps)
        // and the iteration's chords' turning 1.5 x 1.01 x FU max_dphi within 0.05
        const bool cm_iter = SR_CM_ITER && any_cm && !__ballot(!(uhi < 1.0f)) &&
                             (1.515f * (float)FU) * fr.max_dphi < 0.05f;
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        if constexpr (NC > 0) {
            if (cm_iter) fast(I2{});
            else if (any_cm) fast(I1{});
            else if (CULL && SR_COAST && !__ballot(!(lim0 == INFINITY))) coast();
            else fast(I0{});
        } else {
            if (CULL && SR_COAST && !__ballot(!(lim0 == INFINITY))) coast();
            else fast(I0{});
        }
        SR_PT(0);
        if (i >= N) {
            SR_PROBE(SR_STAT_STEPHIST(56, N - 1 - ick); SR_STAT_STEPHIST(57, 1));  // recover_up's replayed steps
            up = recover_up(N);
            break;
        }
        SR_PROBE(SR_PROF_BUMP(r.prof, 19, 1));
        // Past the singularity: u before and after the step both +inf or NaN.
        // RK4 keeps u there (inf + x is inf or NaN, NaN stays NaN) and no
        // compare of the loop fires (u < 0, u < u_f, the hole's window), so
        // the reference runs on to max_steps, and every chord from here has
        // both ends at +-0 or NaN (point_at divides by u): length 0 or NaN,
        // direction 0 / 0 or NaN / x, NaN in all three components. Each
        // primitive test then misses whatever its origin: sphere_test's and
        // cyl_test's discriminant is NaN (not < 0) and so are their roots
        // (lam stays -1 / in1, in2 false); plane_test's denominator is NaN
        // (not < eps) and so is lam (not >= 0), which fails the disks,
        // rectangles and boxes too. So the ray ends at max_steps with no
        // further hit and a final direction of three NaNs, whose get_bg
        // (bilinear's s = t = 0 for any NaN, whatever its sign or payload)
        // is the loop's: leave the loop for its end (r.i = N; up = r.u makes
        // settle_prev(N)'s chord one of those). The stress scene's rays
        // through an object's translucent skin at the shell ran ~1800 such
        // steps, each an event with every slot tested (round 6: its frame
        // alone 31.0 -> 4.6 ms). Here, before the slow path proper, the check
        // left the hot instantiation's allocation as it was; placed after the
        // degenerate-chord flag or in the event it cost ~0.8 % per frame
        // (profiles/r06/s20_s31).
        if (CULL && !(r.u < INFINITY) && !(un < INFINITY)) {
            up = r.u;
            break;
        }
        // ---- slow path of step i
        r.i = i;
        r.steps = sbase + i + 1;
        if (un < 0.0f) {
            SR_PROBE(if (i > ick) SR_STAT_STEPHIST(58, i - 1 - ick); SR_STAT_STEPHIST(59, 1));  // (u < 0 exit)
            up = recover_up(i);
            settle_prev(i);
            return ST_BG;
        }
        // the chord left the black hole's u window (or the inner one outward)
        const bool bhx = un > uhi || (un < SR_BH_ULO2 && BS::inner(uhi));
        // a chord ending beyond 2 / u_f, which the orbital-plane exclusions do
        // not cover (budget_frame): an event that forces them (budget_event)
        // a ray through the singularity (u past 1e30: its chord points round
        // to the origin, then inf / NaN): the exact chord is degenerate (zero
        // length, NaN direction) and the exact tests decide what its NaN
        // arithmetic hits, so every slot is tested (reach below)
        const bool degen = CULL && !(un < 1.0e30f && r.u < 1.0e30f);
        const bool event = !(vb < 0.0f) || bhx || (SR_XPLANE && un < 0.5f * fr.u_f) || degen;
        SR_PROBE(SR_TRACE_AT("slow i=%d u=%.9g un=%.9g uhi=%.9g vb=%g force=%d event=%d bhx=%d m=%g\n", i, r.u, un,
                             uhi, vb, (int)force, (int)event, (int)bhx, bm));
#ifndef SR_BH_CROSS
#define SR_BH_CROSS 1
#endif
        // a certain crossing of the shell from inside the inner window (its
        // proof at SR_BH_WINDOW2): the hole is this chord's closest hit
        if (RECORD && CULL && SR_BH_CROSS && !every && __ballot(BS::inner(uhi) && un >= SR_BH_UIN3)) {
            const float uin = (uhi == fr.bh_u3 && fr.bh_u3 != fr.bh_u2) ? SR_BH_UIN3 : SR_BH_UIN2;
            if (BS::inner(uhi) && un >= uin && un < 1.0e30f && vb < 0.0f && !force) return ST_BH;
        }
        if (CULL) {  // the radii of the step's ends (the fast loop carries none)
            rA = __builtin_amdgcn_rcpf(r.u);
            rB = __builtin_amdgcn_rcpf(un);
        }
        up = r.u;
        r.u = un;
        r.du = dun;
        const float rAold = rA;
        rA = rB;
        const bool reseeded = force;
        force = false;
        do {  // `break`: on to step i + 1
            if (!__ballot(event)) break;
            uint32_t reach = 0xffffffffu;
            uint32_t trmask = 0xffffffffu;  // test-ray parts this lane's chord may reach (budget_event)
            const f2 p1 = phi_cs(i - 1);
            if (CULL) {
                // the approximate chord (exact start when materialised)
                const bool exact_start = im == i - 1;
                const f3 Ap = exact_start ? r.ro : point_near(r, rAold, p1.x, p1.y);
                const f3 Bp = point_near(r, rB, e.z, e.w);
                const float pe = point_err(exact_start ? 0.0f : rAold, rB);
                // the displacement from the ball's centre to the step's end
                // point Bp, which becomes the centre: bs.T bounds 1.01 x the
                // distance between the centres' embeddings and between the
                // reference's end point and the old centre (the chord is
                // covered by slot j when bs.T < E[j]: both its ends are in
                // the ball). After a reseed: the charge from the reseed plus
                // the chord from the exact r.ro.
                float ahead;
                {
                    const float cx = rB * e.z, cy = rB * e.w;  // Bp = nv cx + tv cy (point_near)
                    const f3 dv = Bp - Ap;
                    const float cl = __builtin_amdgcn_sqrtf(dot(dv, dv));
                    float T;
                    if (reseeded) {
                        T = bs.T() + (cl * 1.0001f + pe) * SR_PATH_SLACK;
                    } else {
                        const float ocx = bs.cx(), ocy = bs.cy();
                        const float dx = cx - ocx, dy = cy - ocy;
                        T = __builtin_fmaf(__builtin_amdgcn_sqrtf(dx * dx + dy * dy), 1.0101f,
                                           3.0e-6f * (rB + fabsf(ocx) + fabsf(ocy)));
                    }
                    bs.setT(T);
                    ahead = SR_AHEAD * SR_PATH_SLACK * cl + SR_AHEAD_T * T;
                    bs.setC(cx, cy);
                }
                SR_STAT(1, 1);
                SR_PROBE(probe_event(sc, bs, r, lp, i, event, vb, q0, bhx, reseeded, ahead, any_cm));
                // sr_wave_costs: the wave's event count (one lane, its own LDS word)
                if (WCOST && (int)__lane_id() == __builtin_ctzll(__ballot(1)))
                    sr_lds_ev[threadIdx.x >> 6] += 1;
                // a new frame (reseed): the cylinders' direction tests start over
                SR_PT(2);
                // the inner window's bound for this lane: steep falling lanes get bh_u3
                const bool steep = r.du > 0.0f && __builtin_fmaf(r.du, r.du, r.u * r.u * (1.0f - r.u)) >= SR_BH_E_MIN;
                reach = budget_event(sc, segs, trmask, bs, Ap, Bp, pe, par, reseeded, ahead, r.du < 0.0f && r.u < 0.6f, fr.out_dip,
                                     fr.max_dphi, bhx, fr.win_ok && fr.out_dip > SR_BH_DIP, r.du > 0.0f, cm_iter,
                                     fr.u_f, fr.bh_u2, fr.bh_u3, steep);
                if (__ballot(degen)) {
                    reach |= ((2u << sc->num_budget) - 1u) | SR_REACH_TR;
                    trmask = 0xffffffffu;
                }
                SR_PT(6);
                SR_PROBE(probe_reach(r, reach));
                SR_PROBE(SR_TRACE_AT("  event reach=%x uhi'=%.9g m'=%g E0=%g\n", reach, bs.uhi(), bs.m(), bs.ld(0)));
                if (!__ballot(reach != 0u || every)) break;
                SR_PROBE(probe_fire(bs));
            }
            // frag:924-930: the exact chord of step i
            SR_PROBE(probe_exact_chord(r));
            f3 prev = im == i - 1 ? r.ro : point_at(r, up, p1.x, p1.y);
            r.ro = point_at(r, r.u, e.z, e.w);
            im = i;
            f3 delta = r.ro - prev;
            float seg = len(delta);
            r.rd = delta / seg;
            hit = CULL ? closest_hit_chord<BS::TR>(sc, segs, reach, prev, r.rd, seg, trmask)
                       : closest_hit_all(sc, segs, prev, r.rd, seg);
            SR_PT(4);
            SR_PROBE(SR_TRACE_AT("  chord i=%d seg=%g slot=%d\n", i, seg, hit.slot));
            if (hit.slot != SLOT_NONE) {
                const int op = hit_opacity(sc, fr, tx, hit, -r.rd, !RECORD);
                SR_PT(5);
                if (op == OP_ZERO) break;  // frag + vec4(0), alpha != 1: the ray goes on (frag:930-932)
                if (!RECORD) return ST_HIT;
                if (hit.slot == SLOT_BH) return ST_BH;  // opaque black (shade_hit): no record
                // r.steps: the ray's step count if this hit ends it
                // the whole 32-byte sector in two 16-byte stores (a partial
                // sector costs a read-modify-write)
                // log.n < SR_PS_HITS by construction (ST_MORE below); the clamp
                // keeps the store inside the hit planes whatever a miscompiled
                // register holds (a 7-wave build of round
                // 5's source counted 7 .. 31 hits and wrote past the planes)
                float4* h = reinterpret_cast<float4*>(
                    log.ps.hit32(log.id(), min((uint32_t)log.n, (uint32_t)(SR_PS_HITS - 1))));
                h[0] = make_float4(hit.p.x, hit.p.y, hit.p.z,
                                   __int_as_float((int)((uint32_t)(hit.slot * 8 + hit.face + PS_KEY_BIAS) |
                                                                  ((uint32_t)r.steps << 8))));
                h[1] = make_float4(r.rd.x, r.rd.y, r.rd.z, hit.p.x);  // .w unread (a zero here was a spilled register)
                log.n++;
                if (op == OP_OPAQUE) return ST_HIT;
                if (log.n == SR_PS_HITS) return ST_MORE;
            }
        } while (false);
        i++;
    }
    r.i = N;
    r.steps = sbase + N;
    settle_prev(N);
    return ST_BG;
}

// The ray's ending (frag:874-876, 895-897, 903-905, 935) after its hits.
__device__ __forceinline__ void finish_ray(const sr_dev_scene* __restrict__ sc, const float* __restrict__ segs,
                                           const sr_dev_frame& fr, const Tex& tx, int st, f3 ro, f3 rd, f4& frag) {
    if (st == ST_FLAT) {
        f4 c = intersect_color(sc, segs, fr, tx, ro, rd, -1.0f);
        frag = frag + c;
        if (c.w == 1.0f) return;
        st = ST_BG;
    }
    if (st == ST_BG) frag = frag + get_bg(fr, tx, rd);
}

__device__ __forceinline__ void write_pixel(const sr_dev_frame& fr, uint8_t* __restrict__ out, size_t pitch,
                                            float* __restrict__ dbg_rgba, int32_t* __restrict__ dbg_steps,
                                            const Pix& q, f4 frag, int steps) {
    uint32_t pix = unorm8(frag.x) | (unorm8(frag.y) << 8) | (unorm8(frag.z) << 16) | (unorm8(frag.w) << 24);
    if (out) *reinterpret_cast<uint32_t*>(out + (size_t)q.k * pitch + (size_t)q.px * 4) = pix;
    const size_t i = (size_t)q.k * (size_t)fr.width + (size_t)q.px;
    if (dbg_rgba) {
        dbg_rgba[4 * i + 0] = frag.x;
        dbg_rgba[4 * i + 1] = frag.y;
        dbg_rgba[4 * i + 2] = frag.z;
        dbg_rgba[4 * i + 3] = frag.w;
    }
    if (dbg_steps) dbg_steps[i] = steps;
}

}  // namespace

#ifndef SR_MIN_WAVES_PER_EU  // the Makefile's WAVES (7 since round 6)
#define SR_MIN_WAVES_PER_EU 7
#endif
#ifndef SR_NB_SMALL
#define SR_NB_SMALL 6
#endif
// budgeted cylinders of the small instantiation: its cylinder loops (phase 1,
// chord_parallel in the cylinder-plane fast loop) run over one, and its LDS
// layout holds 17 rows instead of 25 (no VGPR spills left in it)
#ifndef SR_NC_SMALL  // round 6: 0 (no budgeted cylinder needs the direction tests, sr_api.cpp SR_CYL_DIRFREE)
#define SR_NC_SMALL 0
#endif
#ifndef SR_GENERAL_WAVES_PER_EU
#define SR_GENERAL_WAVES_PER_EU 5
#endif
// the general instantiation: 8 slots, 3 cylinders (25 LDS rows); scenes with
// more budget slots run the large one (every object budgeted: SR_MAX_BUDGET
// slots; 29 rows, 7.5 KiB of LDS per wave since round 6: 21 waves per CU)
#define SR_NB_GENERAL 8
#define SR_NC_GENERAL SR_NC_KERNEL
// the large instantiation at 5 waves per SIMD since round 6 (96 VGPRs, no
// spills, 7.5 KiB of LDS per wave once the cylinder rows went: the stress
// scene 1.832 -> 1.647 ms per frame, profiles/r06/s45/stress)
#ifndef SR_LARGE_WAVES_PER_EU
#define SR_LARGE_WAVES_PER_EU 5
#endif

// Waves per SIMD the integrate kernel is built for: SR_MIN_WAVES_PER_EU (7:
// 72 VGPRs, since round 6: 1.5 % more frames per second and one frame alone
// 1.9 % sooner than 6 waves at 80, profiles/r06/s5) for the frame kernels of
// scenes that fit the small instantiation; 5 (96 VGPRs) for the general one (8 slots, 3 cylinders),
// whose event path then keeps every value in registers (at 6 it spilled 9 in
// the reseed path), its 6.5 KiB of LDS per wave allowing 24 waves per CU
constexpr int sr_integrate_waves(int nb, int nc) {
    return nb > SR_NB_GENERAL ? SR_LARGE_WAVES_PER_EU
                              : (nb > SR_NB_SMALL || nc > SR_NC_SMALL) ? SR_GENERAL_WAVES_PER_EU : SR_MIN_WAVES_PER_EU;
}

// Launch codes (order_tiles): tile << 8 for a whole 16x16 workgroup tile;
// tile << 8 | SR_SPLIT | sub for workgroup `sub` of a split tile; -1 for an
// unused slot of the grid.
#define SR_SPLIT 0x80

// The thread index (in the tile's own 256-thread numbering, pixel_of) that
// thread `tid` of split workgroup `sub` stands for, or -1 (idle lane). A split
// tile's 256 pixels are cut into cells of L = 2^lg pixels (4x4, 2x2 or 1x1
// squares inside the tile's 8x8 wave tiles); split workgroup `sub` runs cells
// 4 sub .. 4 sub + 3, one per wave, in lanes 0 .. L - 1. A ray's result does
// not depend on its wave-mates (every culling decision is exact), so the
// cells' pixels are bit-identical to the whole tile's.
__device__ __forceinline__ int split_thread(int sub, int tid, int lg) {
    const int lane = tid & 63;
    if (lane >= (1 << lg)) return -1;
    const int cell = sub * 4 + (tid >> 6);
    const int side = lg >> 1;                 // cell side 2^side
    const int cpq = 64 >> lg;                 // cells per 8x8 wave tile
    const int quad = cell / cpq, qc = cell % cpq;
    const int per_row = 8 >> side;
    const int x8 = ((qc % per_row) << side) + (lane & ((1 << side) - 1));
    const int y8 = ((qc / per_row) << side) + (lane >> side);
    return quad * 64 + y8 * 8 + x8;
}

// 1-D grid: workgroup s = (slot * B + f) * SR_WG_PER_TILE + part renders
// part `part` (SR_WG threads) of launch code order[slot] of frame f of the
// batch (costliest tiles of every frame first, order_tiles), and records
// the tile's cost (max steps of its rays over the batch).
// WCOST: the sr_wave_costs instantiation (per-wave steps and events to
// fr.wave_cost); the frame kernels carry none of its code.
// NB: budget slots the event path handles (>= the scene's sc->num_budget;
// sr_launch_geodesic picks SR_NB_SMALL when it suffices: the default scene
// has six, and phase 1 of an event runs over every slot of the capacity).
// NC: budgeted cylinders it handles (SR_NC_SMALL with SR_NB_SMALL).
// TR: the test-ray instantiation (the test ray budgeted, clearance_tr)
template <bool CULL, bool WCOST = false, int NB = SR_MAX_BUDGET, int FU = SR_FAST_UNROLL, int NC = SR_NC_KERNEL,
          bool TR = false>
__global__ __launch_bounds__(SR_WG, sr_integrate_waves(NB, NC)) void sr_integrate_kernel(
    const sr_dev_scene* __restrict__ sc, const float4* __restrict__ tbl, const float* __restrict__ segs,
    const uint32_t* __restrict__ arr, const uint8_t* __restrict__ opq, sr_dev_frame fr, float* __restrict__ ps_base,
    size_t ps_n, int* __restrict__ count, const int* __restrict__ order, int* __restrict__ cost) {
    const unsigned B = (unsigned)fr.batch;
    const unsigned bid = blockIdx.x;
    const unsigned wg = bid / SR_WG_PER_TILE;  // the tile's workgroup index (slot * B + f)
    const int frame = B > 1 ? (int)(wg % B) : 0;
    const unsigned slot = B > 1 ? wg / B : wg;
    const int code = order ? order[slot] : ((int)slot << 8);
    if (blockIdx.x == 0 && threadIdx.x == 0) *count = 0;  // the shade kernel's queue (stream-ordered)
    if (code < 0) return;  // unused slot of a split grid
    const int block = code >> 8;
    const int ttid = (int)(bid % SR_WG_PER_TILE) * SR_WG + (int)threadIdx.x;  // thread of the tile's 256
    const int tid = (code & SR_SPLIT) ? split_thread(code & 0x3f, ttid, fr.split_log2) : ttid;
#ifndef SR_PRIO_BLOCKS
#define SR_PRIO_BLOCKS 256
#endif
    // The costliest tiles (launched first) are the frame's critical path: a
    // 2000-step ray sharing its SIMD with four other waves would run 3x longer
    // than the rest of the grid. Raised issue priority keeps them near their
    // own latency bound while the other waves fill the idle issue slots.
#ifdef SR_PRIO_SPLIT
    if (order && ((code & SR_SPLIT) || wg < SR_PRIO_BLOCKS)) __builtin_amdgcn_s_setprio(3);
#else
    if (order && wg < SR_PRIO_BLOCKS) __builtin_amdgcn_s_setprio(3);
#endif
    SR_PROBE(WaveProbe wp);  // measurement builds only (probes.h)
    Pix q;
    int steps = 0;
    if (WCOST && (threadIdx.x & 63) == 0) sr_lds_ev[threadIdx.x >> 6] = 0;
    if (tid >= 0 && pixel_of(fr, block, tid, q)) {
        sr_lds_pid[threadIdx.x] = (uint32_t)(((size_t)frame * (size_t)fr.tiles + (size_t)block) * 256 + tid);
        Tex tx;
        tx.bg = nullptr;
        tx.arr = arr;
        tx.opq = opq;
        HitLog log{PS{ps_base, ps_n}, 0};
        const PS& ps = log.ps;
        Ray r;
        Hit hit;
        int st = init_pixel(fr, fr.cam[frame], q, r);
        SR_PROBE(st = wp.lane_mask(q.px, q.py, fr.width, st, ST_DONE); wp.ray_start(r));
        if (st < 0) st = integrate<CULL, true, WCOST, NB, FU, NC, TR>(sc, segs, tbl, fr, tx, r, hit, log);
        const size_t id = log.id();
        ps.put_rec(id, ps_word(st, log.n, r.steps), r.rd);
        SR_PROBE(wp.pixel(st, log.n));
        if (st == ST_FLAT || st == ST_MORE) ps.put3(PS_RO, id, r.ro);
        if (st == ST_MORE) {  // resumable (sr_resume_kernel)
            ps.puti(PS_I, id, r.i);
            ps.put3(PS_NV, id, r.nv);
            ps.put3(PS_TV, id, r.tv);
            ps.at(PS_U, id) = r.u;
            ps.at(PS_DU, id) = r.du;
        }
        steps = r.steps;
        SR_PROBE(wp.ray_end(r));
    }
    SR_PROBE(wp.finish(frame, fr.tiles, block, ttid, steps));
    if (cost) {  // all 64 lanes are active here
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) steps = max(steps, __shfl_xor(steps, off));
        if ((threadIdx.x & 63) == 0) atomicMax(&cost[block], steps);
    }
    if (WCOST && !(code & SR_SPLIT)) {  // sr_wave_costs (split tiles off)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) steps = max(steps, __shfl_xor(steps, off));
        if ((threadIdx.x & 63) == 0) {
            const int wave = ttid >> 6, gxt = (fr.width + 15) >> 4;
            const int b8 = (block / gxt) * 2 + (wave >> 1), c8 = (block % gxt) * 2 + (wave & 1);
            const int nb8 = (fr.nrows + 7) >> 3, nc8 = (fr.width + 7) >> 3;
            if (b8 < nb8 && c8 < nc8) {
                int* o = fr.wave_cost + (((size_t)frame * nb8 + b8) * nc8 + c8) * 2;
                o[0] = steps;
                o[1] = sr_lds_ev[threadIdx.x >> 6];
            }
        }
    }
}

// Launch order for the next frame: workgroup tiles by descending cost of this
// frame (counting sort on 256 cost buckets), so the long rays - those
// orbiting near the photon sphere run to max_steps - start first instead of
// forming a latency-bound tail. With split tiles, the first min(split_tiles,
// tiles of cost >= split_min_steps) tiles are emitted as 64 >> split_log2
// split workgroups each (their waves carry a few rays: a wave's budget events
// are the union of its lanes', so the longest rays run with fewer events);
// the grid's remaining slots get -1. Resets the costs. One workgroup.
// One 256-thread workgroup (a wave per SIMD): with 1024 threads it needed
// sixteen wave slots on one CU, which the integrate launches of the other
// streams rarely left free, and its stream waited up to 6.5 ms behind it
// (mean 0.35 ms per launch, profiles/r04/s6_kernel_stats.csv).
#define SR_ORDER_WG 256
// Round 6: one workgroup of the shade kernel (the grid's first, so it is
// dispatched before the shading ones) instead of a kernel of its own after
// it: the launch order of the next frame is off this frame's critical path
// (a frame alone spent 0.038 ms in the resume and order kernels after its
// shade kernel, tools/frame_parts.py), and the buckets' offsets are a
// parallel scan instead of one thread's loop over the 256 buckets.
__device__ __forceinline__ void order_tiles(int* __restrict__ cost, int n, int max_cost, int* __restrict__ order,
                                            int split_tiles, int split_log2, int split_min) {
    __shared__ int hist[256];
    __shared__ int offs[256];
    __shared__ int wsum[SR_ORDER_WG / 64];
    __shared__ int nsplit;
    const int t = threadIdx.x;
    // 256 cost buckets, descending cost = descending bucket. With split
    // tiles the split threshold is a bucket boundary (costs >= split_min in
    // 128..255, below it in 0..127), so exactly the tiles of cost >=
    // split_min may be split; without, the buckets span [0, max_cost].
    const int smin = split_min < 1 ? 1 : split_min;
    auto bucket = [&](int c) {
        c = c < 0 ? 0 : c;
        long long b;
        if (split_tiles == 0) b = (long long)c * 256 / ((long long)max_cost + 1);
        else if (c >= smin) b = 128 + (long long)(c - smin) * 128 / ((long long)(max_cost > smin ? max_cost : smin) - smin + 1);
        else b = (long long)c * 128 / smin;
        return (int)(b < 0 ? 0 : b > 255 ? 255 : b);
    };
    hist[t] = 0;
    __syncthreads();
    for (int i = t; i < n; i += SR_ORDER_WG) atomicAdd(&hist[bucket(cost[i])], 1);
    __syncthreads();
    // thread t holds bucket 255 - t (descending cost): an inclusive scan over
    // the threads gives each bucket's end, its exclusive prefix its offset
    const int lane = t & 63, wv = t >> 6;
    const int h = hist[255 - t];
    int x = h;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int base = 0;
    for (int k = 0; k < wv; k++) base += wsum[k];
    offs[255 - t] = base + x - h;
    // tiles in the top half of the buckets (cost >= split_min with split tiles)
    if (t == 127) nsplit = split_tiles < base + x ? split_tiles : base + x;
    __syncthreads();
    const int S = 64 >> split_log2;  // split workgroups per tile
    const int ns = nsplit;
    for (int i = t; i < n; i += SR_ORDER_WG) {
        const int p = atomicAdd(&offs[bucket(cost[i])], 1);
        if (p < ns) {
            for (int sub = 0; sub < S; sub++) order[p * S + sub] = (i << 8) | SR_SPLIT | sub;
        } else {
            order[ns * S + (p - ns)] = i << 8;
        }
        cost[i] = 0;
    }
    for (int j = n + (S - 1) * ns + t; j < n + (S - 1) * split_tiles; j += SR_ORDER_WG) order[j] = -1;
}
// the next frame's launch order (order_tiles) in the shade kernel's first workgroup
struct OrderArgs {
    int* cost;
    int* order;
    int n, max_cost, split_tiles, split_log2, split_min;
};

#ifndef SR_SHADE_WAVES_PER_EU
#define SR_SHADE_WAVES_PER_EU 1
#endif
__global__ __launch_bounds__(256, SR_SHADE_WAVES_PER_EU) void sr_shade_kernel(const sr_dev_scene* __restrict__ sc,
                                                      const float* __restrict__ segs,
                                                      const uint32_t* __restrict__ bg,
                                                      const uint32_t* __restrict__ arr, sr_dev_frame fr,
                                                      float* __restrict__ ps_base, size_t ps_n,
                                                      uint8_t* __restrict__ out, size_t pitch,
                                                      float* __restrict__ dbg_rgba, int32_t* __restrict__ dbg_steps,
                                                      int* __restrict__ list, int* __restrict__ count,
                                                      int* __restrict__ diag, OrderArgs oa) {
    // with a launch order to compute, grid row 0 is its workgroup's (block
    // (0, 0)) and the frames' tiles follow in rows 1 ..
    const int row0 = oa.order ? 1 : 0;
    if ((int)blockIdx.y < row0) {
        if (blockIdx.x == 0)
            order_tiles(oa.cost, oa.n, oa.max_cost, oa.order, oa.split_tiles, oa.split_log2, oa.split_min);
        return;
    }
    const int vblock = ((int)blockIdx.y - row0) * gridDim.x + blockIdx.x;  // frame f's tiles are rows f*gy ..
    const int f = vblock / fr.tiles, block = vblock - f * fr.tiles;
    Pix q;
    if (!pixel_of(fr, block, threadIdx.x, q)) return;
    const size_t id = (size_t)vblock * 256 + threadIdx.x;
    if (out) out += (size_t)f * (size_t)fr.out_frame_stride;
    if (dbg_rgba) dbg_rgba += (size_t)f * (size_t)fr.width * (size_t)fr.nrows * 4;
    if (dbg_steps) dbg_steps += (size_t)f * (size_t)fr.width * (size_t)fr.nrows;
    const PS ps{ps_base, ps_n};
    Tex tx;
    tx.bg = bg;
    tx.arr = arr;
    tx.opq = nullptr;
    const float4 rec = ps.get_rec(id);
    const int w0 = __float_as_int(rec.x);
    const int st = w0 & 7, nh = min((w0 >> 3) & 7, SR_PS_HITS);  // <= SR_PS_HITS written (memory safety)
    f4 frag = crosshair_frag(fr, q);
    bool done = false;
    int steps_at = -1;
    for (int j = 0; j < nh && !done; j++) {  // frag:930-932 for each recorded hit, in order
        const float4* h4 = reinterpret_cast<const float4*>(ps.hit(id, j));
        const float4 a = h4[0], b = h4[1];
        Hit h = no_hit();
        const int hw = __float_as_int(a.w);
        const int key = (hw & 0xff) - PS_KEY_BIAS;
        h.slot = key >> 3;
        h.face = key & 7;
        h.p = F3(a.x, a.y, a.z);
        f4 c = shade(sc, fr, tx, h, -F3(b.x, b.y, b.z));
        frag = frag + c;
        done = c.w == 1.0f;
        if (done) steps_at = (int)((unsigned)hw >> 8);
    }
    if (!done && st == ST_BH) {  // the ray's end in the black hole: vec4(0, 0, 0, 1) (shade_hit)
        frag = frag + F4(0.0f, 0.0f, 0.0f, 1.0f);
        done = true;
        steps_at = (int)((unsigned)w0 >> 8);
    }
    if (!done) {
        if (st == ST_MORE) {
            // every hit so far translucent, the ray stopped with its log
            // full: accumulate and queue for sr_resume_kernel (an ST_HIT
            // pixel ends at its last hit, opaque exactly: done above)
            ps.put4(PS_FRAG, id, frag);
            list[atomicAdd(count, 1)] = (int)id;
            return;
        }
        // an ST_HIT pixel ends at an opaque-classified hit (hit_opacity, exact
        // where it claims): its shaded alpha is 1. Counted if ever not
        // (sr_diag_counters; the tests assert 0): such a ray has no
        // resumable state and is written without the rest of its path.
        if (st == ST_HIT) atomicAdd(diag, 1);
        if (st == ST_FLAT || st == ST_BG)  // ro only for the flat intersect
            finish_ray(sc, segs, fr, tx, st, st == ST_FLAT ? ps.get3(PS_RO, id) : F3(0.0f, 0.0f, 0.0f),
                       F3(rec.y, rec.z, rec.w), frag);
    }
    if (dbg_steps && steps_at < 0) steps_at = (int)((unsigned)w0 >> 8);
    write_pixel(fr, out, pitch, dbg_rgba, dbg_steps, q, frag, steps_at);
}

template <bool CULL, bool TR = false>
__global__ __launch_bounds__(SR_WG) void sr_resume_kernel(const sr_dev_scene* __restrict__ sc,
                                                       const float4* __restrict__ tbl,
                                                       const float* __restrict__ segs,
                                                       const uint32_t* __restrict__ bg,
                                                       const uint32_t* __restrict__ arr, sr_dev_frame fr,
                                                       float* __restrict__ ps_base, size_t ps_n,
                                                       uint8_t* __restrict__ out, size_t pitch,
                                                       float* __restrict__ dbg_rgba, int32_t* __restrict__ dbg_steps,
                                                       const int* __restrict__ list, const int* __restrict__ count) {
    const int total = *count;
    const PS ps{ps_base, ps_n};
    Tex tx;
    tx.bg = bg;
    tx.arr = arr;
    tx.opq = nullptr;
    for (int w = blockIdx.x * SR_WG + threadIdx.x; w < total; w += gridDim.x * SR_WG) {
        const int id = list[w];
        const int f = (id >> 8) / fr.tiles;
        Pix q;
        pixel_of(fr, (id >> 8) - f * fr.tiles, id & 255, q);
        Ray r;
        f4 frag = ps.get4(PS_FRAG, id);
        const float4 rec = ps.get_rec(id);
        r.ro = ps.get3(PS_RO, id);
        r.rd = F3(rec.y, rec.z, rec.w);
        r.nv = ps.get3(PS_NV, id);
        r.tv = ps.get3(PS_TV, id);
        r.u = ps.at(PS_U, id);
        r.du = ps.at(PS_DU, id);
        r.i = ps.geti(PS_I, id) + 1;
        r.steps = (int)((unsigned)__float_as_int(rec.x) >> 8);
        HitLog log{ps, 0};  // RECORD = false: nothing is logged
        for (;;) {  // rounds: integrate to the next hit, shade, resume if not opaque
            Hit hit = no_hit();
            const int st = integrate<CULL, false, false, SR_MAX_BUDGET, SR_FAST_UNROLL, SR_NC_KERNEL, TR>(
                sc, segs, tbl, fr, tx, r, hit, log);
            if (st == ST_HIT) {
                f4 c = shade(sc, fr, tx, hit, -r.rd);
                frag = frag + c;
                if (c.w == 1.0f) break;  // frag:932
                r.i++;
                continue;
            }
            finish_ray(sc, segs, fr, tx, st, r.ro, r.rd, frag);
            break;
        }
        const size_t fo = (size_t)f * (size_t)fr.width * (size_t)fr.nrows;
        write_pixel(fr, out ? out + (size_t)f * (size_t)fr.out_frame_stride : nullptr, pitch,
                    dbg_rgba ? dbg_rgba + 4 * fo : nullptr, dbg_steps ? dbg_steps + fo : nullptr, q, frag, r.steps);
    }
}

// order/cost (optional, one int per workgroup tile): the launch order and
// the cost feedback of order_tiles
extern "C" hipError_t sr_launch_geodesic(const sr_dev_scene* sc, const float4* tbl, const float* segs,
                                         const uint32_t* bg, const uint32_t* arr, const uint8_t* opq,
                                         const sr_dev_frame* fr, uint8_t* out, size_t pitch, float* dbg_rgba,
                                         int32_t* dbg_steps, float* ps, size_t ps_n, int* list, int* count,
                                         int* order, int* cost, int* diag, hipEvent_t* ev4, hipStream_t stream) {
    dim3 block(256);
    dim3 grid((fr->width + 15) / 16, (fr->nrows + 15) / 16);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    const unsigned nblocks = grid.x * grid.y;
    const unsigned B = (unsigned)fr->batch;
    if (B < 1 || B > SR_MAX_BATCH || fr->tiles != (int)nblocks) return hipErrorInvalidValue;
    if ((size_t)nblocks * B * 256 > ps_n || (size_t)nblocks * B * 256 > (size_t)INT32_MAX) return hipErrorInvalidValue;
    if ((order == nullptr) != (cost == nullptr)) return hipErrorInvalidValue;
    // split tiles need the launch order (their codes come from order_tiles)
    const int split = order ? fr->split_tiles : 0;
    if (split < 0 || (split && (fr->split_log2 < 0 || fr->split_log2 > 4 || (fr->split_log2 & 1))))
        return hipErrorInvalidValue;
    if (nblocks > (1u << 22)) return hipErrorInvalidValue;  // tile << 8 stays a positive int
    const unsigned slots = nblocks + ((64u >> (split ? fr->split_log2 : 6)) - 1u) * (unsigned)split;
    const bool cull = fr->cull != 0;
    // the small instantiation (6 slots, 1 cylinder: 17 LDS rows) when the
    // scene fits it, the general one (8 slots) or the large one (every object)
    const bool small = cull && fr->num_budget <= SR_NB_SMALL && fr->num_budget_cyl <= SR_NC_SMALL;
    const bool general = fr->num_budget <= SR_NB_GENERAL;
    const bool tr = cull && fr->tr_visible != 0;
    // cylinders with direction tests beyond what the instantiations handle (a
    // host built with SR_CYL_DIRFREE=0 against a kernel without them)
    if (cull && fr->num_budget_cyl > SR_NC_KERNEL && !small) return hipErrorInvalidValue;
    if (ev4) (void)hipEventRecord(ev4[0], stream);
    if (fr->wave_cost && general)
        hipLaunchKernelGGL((sr_integrate_kernel<true, true, SR_NB_GENERAL, SR_FAST_UNROLL, SR_NC_GENERAL>),
                           dim3(slots * B * SR_WG_PER_TILE), dim3(SR_WG), 0, stream,
                           sc, tbl, segs, arr, opq, *fr, ps, ps_n, count, order, cost);
    else if (fr->wave_cost)
        hipLaunchKernelGGL((sr_integrate_kernel<true, true>), dim3(slots * B * SR_WG_PER_TILE), dim3(SR_WG), 0, stream,
                           sc, tbl, segs, arr, opq, *fr, ps, ps_n, count, order, cost);
    else if (small && tr)  // the test-ray instantiations (the overlay visible)
        hipLaunchKernelGGL((sr_integrate_kernel<true, false, SR_NB_SMALL, SR_FAST_UNROLL, SR_NC_SMALL, true>),
                           dim3(slots * B * SR_WG_PER_TILE), dim3(SR_WG), 0, stream, sc, tbl, segs, arr, opq, *fr, ps,
                           ps_n, count, order, cost);
    else if (cull && general && tr)
        hipLaunchKernelGGL((sr_integrate_kernel<true, false, SR_NB_GENERAL, SR_FAST_UNROLL, SR_NC_GENERAL, true>),
                           dim3(slots * B * SR_WG_PER_TILE), dim3(SR_WG), 0, stream, sc, tbl, segs, arr, opq, *fr, ps,
                           ps_n, count, order, cost);
    else if (cull && tr)
        hipLaunchKernelGGL((sr_integrate_kernel<true, false, SR_MAX_BUDGET, SR_FAST_UNROLL, SR_NC_KERNEL, true>),
                           dim3(slots * B * SR_WG_PER_TILE), dim3(SR_WG), 0, stream, sc, tbl, segs, arr, opq, *fr, ps,
                           ps_n, count, order, cost);
    else if (small && fr->fast_unroll == 2)  // latency mode (sr_set_latency_mode)
        hipLaunchKernelGGL((sr_integrate_kernel<true, false, SR_NB_SMALL, 2, SR_NC_SMALL>), dim3(slots * B * SR_WG_PER_TILE),
                           dim3(SR_WG), 0, stream, sc, tbl, segs, arr, opq, *fr, ps, ps_n, count, order, cost);
    else if (small)
        hipLaunchKernelGGL((sr_integrate_kernel<true, false, SR_NB_SMALL, SR_FAST_UNROLL, SR_NC_SMALL>),
                           dim3(slots * B * SR_WG_PER_TILE),
                           dim3(SR_WG), 0, stream, sc, tbl, segs, arr, opq, *fr, ps, ps_n, count, order, cost);
    else if (cull && general)
        hipLaunchKernelGGL((sr_integrate_kernel<true, false, SR_NB_GENERAL, SR_FAST_UNROLL, SR_NC_GENERAL>),
                           dim3(slots * B * SR_WG_PER_TILE), dim3(SR_WG), 0, stream, sc,
                           tbl, segs, arr, opq, *fr, ps, ps_n, count, order, cost);
    else if (cull)
        hipLaunchKernelGGL(sr_integrate_kernel<true>, dim3(slots * B * SR_WG_PER_TILE), dim3(SR_WG), 0, stream, sc,
                           tbl, segs, arr, opq, *fr, ps, ps_n, count, order, cost);
    else  // the reference's loop (no budgets: the smallest LDS layout)
        hipLaunchKernelGGL((sr_integrate_kernel<false, false, 1, SR_FAST_UNROLL, 1>), dim3(slots * B * SR_WG_PER_TILE),
                           dim3(SR_WG), 0, stream, sc, tbl, segs, arr, opq, *fr, ps, ps_n, count, order, cost);
    if (ev4) (void)hipEventRecord(ev4[1], stream);
    OrderArgs oa{cost, order, (int)nblocks, fr->max_steps, split, split ? fr->split_log2 : 6, fr->split_min_steps};
    hipLaunchKernelGGL(sr_shade_kernel, dim3(grid.x, grid.y * B + (order ? 1u : 0u)), block, 0, stream, sc, segs, bg,
                       arr, *fr, ps, ps_n, out, pitch, dbg_rgba, dbg_steps, list, count, diag, oa);
    if (ev4) (void)hipEventRecord(ev4[2], stream);
#ifndef SR_RESUME_TILES  // the resume kernel's grid-stride grid, in 256-thread tiles
#define SR_RESUME_TILES 1024u
#endif
    unsigned nb = (nblocks * B < SR_RESUME_TILES ? nblocks * B : SR_RESUME_TILES) * SR_WG_PER_TILE;
    if (tr)
        hipLaunchKernelGGL((sr_resume_kernel<true, true>), dim3(nb), dim3(SR_WG), 0, stream, sc, tbl, segs, bg, arr, *fr,
                           ps, ps_n, out, pitch, dbg_rgba, dbg_steps, list, count);
    else if (cull)
        hipLaunchKernelGGL(sr_resume_kernel<true>, dim3(nb), dim3(SR_WG), 0, stream, sc, tbl, segs, bg, arr, *fr, ps, ps_n,
                           out, pitch, dbg_rgba, dbg_steps, list, count);
    else
        hipLaunchKernelGGL(sr_resume_kernel<false>, dim3(nb), dim3(SR_WG), 0, stream, sc, tbl, segs, bg, arr, *fr, ps, ps_n,
                           out, pitch, dbg_rgba, dbg_steps, list, count);
    if (ev4) (void)hipEventRecord(ev4[3], stream);
    return hipGetLastError();
}
