/*
 * sr_oracle.c — CPU ORACLE (test infrastructure; never shipped, never measured
 * as the product). Restates assets/shaders/black_hole.frag (reference
 * Yachim/schwarzschild-raytracer @ 2025-03-02) function by function; every
 * function cites the GLSL lines it follows. See sr_oracle.h for the
 * arithmetic contract and how the restatement is pinned.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no -ffast-math).
 */
#include "sr_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* frag:10 — `#define PI 3.1415926535`, a float literal in GLSL */
#define PI_F 3.1415926535f
/* frag:30 */
#define EPSILON_F 0.0000001f

/* ---- arithmetic contract helpers -------------------------------------- */
static inline float f_sin(float x) { return (float)sin((double)x); }
static inline float f_cos(float x) { return (float)cos((double)x); }
static inline float f_tan(float x) { return (float)tan((double)x); }
static inline float f_asin(float x) { return (float)asin((double)x); }
static inline float f_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
static inline float f_pow(float x, float y) { return (float)pow((double)x, (double)y); }
/* GLSL min/max: min(x,y) = y < x ? y : x */
static inline float f_min(float x, float y) { return y < x ? y : x; }
static inline float f_max(float x, float y) { return x < y ? y : x; }

typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;
typedef struct { v3 c[3]; } m3; /* columns */

static inline v2 V2(float x, float y) { v2 r = {x, y}; return r; }
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scl3(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 div3s(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float dot2(v2 a, v2 b) { return a.x * b.x + a.y * b.y; }
static inline float len3(v3 a) { return sqrtf(dot3(a, a)); }
static inline v3 norm3(v3 a) { float k = 1.0f / sqrtf(dot3(a, a)); return scl3(a, k); }
static inline v3 cross3(v3 a, v3 b) {
    return V3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
/* m * v, column-major: (m0*v.x + m1*v.y) + m2*v.z */
static inline v3 mv3(m3 m, v3 v) {
    return add3(add3(scl3(m.c[0], v.x), scl3(m.c[1], v.y)), scl3(m.c[2], v.z));
}
/* transpose(m) * v */
static inline v3 mtv3(m3 m, v3 v) { return V3(dot3(m.c[0], v), dot3(m.c[1], v), dot3(m.c[2], v)); }
static inline m3 M3(v3 a, v3 b, v3 c) { m3 r; r.c[0] = a; r.c[1] = b; r.c[2] = c; return r; }
static inline v4 add4(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
/* frag:357-363 — square_vector(vec2) goes through vec3(v, 0.) */
static inline float sqv2(v2 v) { return (v.x * v.x + v.y * v.y) + 0.0f * 0.0f; }
static inline float f_fract(float x) { return x - floorf(x); }
static inline float f_mod(float x, float y) { return x - y * floorf(x / y); }

static inline v3 load_v3(const float* p) { return V3(p[0], p[1], p[2]); }
static inline m3 load_m3(const float* a) {
    return M3(V3(a[0], a[1], a[2]), V3(a[3], a[4], a[5]), V3(a[6], a[7], a[8]));
}

/* ---- GLSL structs (frag:41-206) ---------------------------------------- */
typedef struct { v3 pos; m3 axes; } Transform;
typedef struct { Transform transform; float radius; } Sphere;
typedef struct { Transform transform; v2 texture_offset; int repeat_texture; v2 texture_size; } Plane;
typedef struct { Plane plane; float radius; } Disk;
typedef struct { Plane plane; float inner_radius, outer_radius; } HollowDisk;
typedef struct { Transform transform; float height, radius; } Cylinder;
typedef struct { Plane plane; float width, height; } Rectangle;
typedef struct { Transform transform; float width, depth, height; } Box;
typedef struct { int type, index, material_index; } Object;
typedef struct { v3 origin, dir; } Ray;
typedef struct {
    int is_hit;
    float dist;
    v3 intersection_point;
    m3 tangent_space;
    v2 tangent_coordinates;
    Object object;
} HitInfo;

enum {
    OBJECT_TYPE_TEST_RAY_CURVED = -99,
    OBJECT_TYPE_TEST_RAY_FLAT = -98,
    OBJECT_TYPE_SPECIAL = -42
};

typedef struct {
    const sr_scene* scene;
    const sr_test_ray* tr;
    const sro_textures* tex;
    const sr_camera* cam;
    const sr_params* prm;
    float res_x, res_y;
} Ctx;

static Transform to_transform(const sr_transform* t) {
    Transform r;
    r.pos = load_v3(t->pos);
    r.axes = load_m3(t->axes);
    return r;
}
static Plane to_plane(const sr_plane* p) {
    Plane r;
    r.transform = to_transform(&p->transform);
    r.texture_offset = V2(p->texture_offset[0], p->texture_offset[1]);
    r.repeat_texture = p->repeat_texture != 0;
    r.texture_size = V2(p->texture_size[0], p->texture_size[1]);
    return r;
}

static HitInfo miss(void) {
    HitInfo h;
    memset(&h, 0, sizeof h);
    h.is_hit = 0;
    return h;
}

/* ---- textures (image_utils.cpp:12-18, 111-114) ---------- */
static v4 fetch_texel(const uint8_t* base, int w, int ch, int x, int y) {
    const uint8_t* p = base + ((size_t)y * (size_t)w + (size_t)x) * (size_t)ch;
    float a = ch == 4 ? (float)p[3] / 255.0f : 1.0f;
    return V4((float)p[0] / 255.0f, (float)p[1] / 255.0f, (float)p[2] / 255.0f, a);
}
static int wrap_repeat(float f, int n) {
    long i = (long)f;
    long m = i % n;
    if (m < 0) m += n;
    return (int)m;
}
static v4 lerp4(v4 a, v4 b, float t) {
    return V4(a.x + (b.x - a.x) * t, a.y + (b.y - a.y) * t, a.z + (b.z - a.z) * t,
              a.w + (b.w - a.w) * t);
}
static v4 wsum4(v4 t00, v4 t10, v4 t01, v4 t11, float a, float b) {
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b);
    float w01 = (1.0f - a) * b, w11 = a * b;
    return V4(((t00.x * w00 + t10.x * w10) + t01.x * w01) + t11.x * w11,
              ((t00.y * w00 + t10.y * w10) + t01.y * w01) + t11.y * w11,
              ((t00.z * w00 + t10.z * w10) + t01.z * w01) + t11.z * w11,
              ((t00.w * w00 + t10.w * w10) + t01.w * w01) + t11.w * w11);
}
/* SwiftShader 4.1's GL_LINEAR + GL_REPEAT sampler of an RGBA8 / RGB8 texture
 * (test only: the filter the golden renders ran with; the library has no
 * such mode). Measured on the SwiftShader of this image with a probe shader
 * of our own over random textures (POT and NPOT, array and 2D, RGB and RGBA)
 * and coordinates, bit-exact on every sample
 * (tests/golden/probe_swiftshader_filter.py):
 *   - the coordinate is a 0.16 fixed-point fraction of the texture: U =
 *     trunc(float32(x * 65536)) (x86 truncation: out of range -> low bits 0),
 *     minus half a texel 0x8000 / n, mod 2^16; texel i0 = (U0 n) >> 16 with
 *     fraction f = (U0 n) mod 2^16, texel i1 from U0 + 2 (0x8000 / n) the
 *     same way (so i1 == i0 when f is small on an NPOT size);
 *   - texels widen to 16 bits (c * 257); weights MulHigh(~f_u or f_u, ~f_v or
 *     f_v) with ~f = 0xFFFF - f, MulHigh(a, b) = (a b) >> 16; the result
 *     (MulHigh(c00, w00) + MulHigh(c10, w10)) + (MulHigh(c01, w01) +
 *     MulHigh(c11, w11)) is a UNORM16, returned as float32(K) * (1 / 65535);
 *   - a 3-channel texture reads alpha 1.0.
 * An opaque texel therefore reads alpha 65527..65533 / 65535 < 1: the
 * reference's `alpha == 1.` (frag:932) never stops a ray at a textured
 * object there. */
static int ss_coord(float x, int n, int* i0, int* i1) {
    const float xf = x * 65536.0f;
    const uint32_t U = fabsf(xf) < 2147483648.0f ? (uint32_t)(int32_t)xf : 0x80000000u;  /* truncation */
    const uint32_t U0 = (U - (uint32_t)(0x8000 / n)) & 0xFFFFu;
    const uint32_t U1 = (U0 + 2u * (uint32_t)(0x8000 / n)) & 0xFFFFu;  /* one texel: twice the half */
    const uint32_t p = U0 * (uint32_t)n;
    *i0 = (int)(p >> 16);
    *i1 = (int)((U1 * (uint32_t)n) >> 16);
    return (int)(p & 0xFFFFu);
}
static uint32_t ss_mh(uint32_t a, uint32_t b) { return (a * b) >> 16; }
static v4 sample_swiftshader(const uint8_t* base, int w, int h, int ch, float u, float v) {
    int x0, x1, y0, y1;
    const uint32_t fu = (uint32_t)ss_coord(u, w, &x0, &x1), fv = (uint32_t)ss_coord(v, h, &y0, &y1);
    const uint32_t nfu = 0xFFFFu - fu, nfv = 0xFFFFu - fv;
    const uint32_t w00 = ss_mh(nfu, nfv), w10 = ss_mh(fu, nfv), w01 = ss_mh(nfu, fv), w11 = ss_mh(fu, fv);
    const uint8_t* t00 = base + ((size_t)y0 * (size_t)w + (size_t)x0) * (size_t)ch;
    const uint8_t* t10 = base + ((size_t)y0 * (size_t)w + (size_t)x1) * (size_t)ch;
    const uint8_t* t01 = base + ((size_t)y1 * (size_t)w + (size_t)x0) * (size_t)ch;
    const uint8_t* t11 = base + ((size_t)y1 * (size_t)w + (size_t)x1) * (size_t)ch;
    float r[4];
    for (int k = 0; k < 4; k++) {
        if (k == 3 && ch < 4) {
            r[k] = 1.0f;
            continue;
        }
        const uint32_t K = (ss_mh(t00[k] * 257u, w00) + ss_mh(t10[k] * 257u, w10)) +
                           (ss_mh(t01[k] * 257u, w01) + ss_mh(t11[k] * 257u, w11));
        r[k] = (float)K * (1.0f / 65535.0f);
    }
    return V4(r[0], r[1], r[2], r[3]);
}

/* GL_LINEAR + GL_REPEAT, texel centres at (i + 1/2) / size, no mipmaps. A
 * non-finite or out-of-range coordinate reads texel 0 (GLSL leaves it undefined). */
static v4 sample_bilinear(const uint8_t* base, int w, int h, int ch, float u, float v, int mode) {
    if (mode == SRO_FILTER_SWIFTSHADER) return sample_swiftshader(base, w, h, ch, u, v);
    float s = u * (float)w - 0.5f;
    float t = v * (float)h - 0.5f;
    if (!(fabsf(s) < 16777216.0f)) s = 0.0f;
    if (!(fabsf(t) < 16777216.0f)) t = 0.0f;
    float fs = floorf(s), ft = floorf(t);
    float a = s - fs, b = t - ft;
    int x0 = wrap_repeat(fs, w), x1 = wrap_repeat(fs + 1.0f, w);
    int y0 = wrap_repeat(ft, h), y1 = wrap_repeat(ft + 1.0f, h);
    v4 t00 = fetch_texel(base, w, ch, x0, y0), t10 = fetch_texel(base, w, ch, x1, y0);
    v4 t01 = fetch_texel(base, w, ch, x0, y1), t11 = fetch_texel(base, w, ch, x1, y1);
    if (mode == SR_FILTER_WEIGHTED) return wsum4(t00, t10, t01, t11, a, b);
    return lerp4(lerp4(t00, t10, a), lerp4(t01, t11, a), b);
}
int sro_sample_texture(const uint8_t* base, int width, int height, int channels, float u, float v, int mode,
                       float out_rgba[4]) {
    if (!base || width <= 0 || height <= 0 || (channels != 3 && channels != 4) || !out_rgba) return -1;
    const v4 r = sample_bilinear(base, width, height, channels, u, v, mode);
    out_rgba[0] = r.x;
    out_rgba[1] = r.y;
    out_rgba[2] = r.z;
    out_rgba[3] = r.w;
    return 0;
}
static v4 texture_bg(const Ctx* c, v2 uv) {
    const sro_textures* t = c->tex;
    if (!t || !t->bg || t->bg_w <= 0 || t->bg_h <= 0) return V4(0, 0, 0, 1);
    return sample_bilinear(t->bg, t->bg_w, t->bg_h, t->bg_channels, uv.x, uv.y,
                           c->prm->filter_mode);
}
static v4 texture_array(const Ctx* c, v2 uv, int layer_index) {
    const sro_textures* t = c->tex;
    if (!t || !t->arr || t->arr_w <= 0 || t->arr_h <= 0 || t->arr_layers <= 0)
        return V4(0, 0, 0, 1);
    int layer = layer_index;
    if (layer < 0) layer = 0;
    if (layer > t->arr_layers - 1) layer = t->arr_layers - 1;
    const uint8_t* base =
        t->arr + (size_t)layer * (size_t)t->arr_w * (size_t)t->arr_h * (size_t)t->arr_channels;
    return sample_bilinear(base, t->arr_w, t->arr_h, t->arr_channels, uv.x, uv.y,
                           c->prm->filter_mode);
}

/* ---- tangent spaces (frag:208-333) ------------------------------------- */
/* frag:209-232 */
static void sphere_tangent_space(HitInfo* h, const Sphere* s) {
    Transform tr = s->transform;
    v3 displacement = sub3(h->intersection_point, tr.pos);
    v3 normal = norm3(displacement);
    v3 local = mtv3(tr.axes, displacement);
    float phi = f_atan2(local.x, local.z);
    if (phi < 0.0f) phi += 2.0f * PI_F;
    float theta = f_asin(local.y / s->radius);
    h->tangent_coordinates = V2(phi / (2.0f * PI_F), theta / PI_F + 0.5f);
    v3 tangent = V3(f_cos(phi), 0.0f, -f_sin(phi));
    v3 bitangent = V3(f_sin(phi) * f_cos(theta), f_sin(theta), f_cos(phi) * f_cos(theta));
    tangent = mv3(tr.axes, tangent);
    bitangent = mv3(tr.axes, bitangent);
    h->tangent_space = M3(tangent, bitangent, normal);
}
/* frag:234-247 */
static void plane_tangent_space(HitInfo* h, const Plane* p) {
    Transform tr = p->transform;
    v3 displacement = sub3(h->intersection_point, tr.pos);
    v3 local = mtv3(tr.axes, displacement);
    h->tangent_coordinates = V2(local.x, local.z);
    h->tangent_coordinates.y = 1.0f - h->tangent_coordinates.y;
    h->tangent_space = M3(tr.axes.c[0], neg3(tr.axes.c[2]), tr.axes.c[1]);
}
/* frag:249-271 */
static void disk_tangent_space(HitInfo* h, const Disk* d) {
    Transform tr = d->plane.transform;
    v3 displacement = sub3(h->intersection_point, tr.pos);
    v3 local = mtv3(tr.axes, displacement);
    float phi = f_atan2(local.x, local.z);
    if (phi < 0.0f) phi += 2.0f * PI_F;
    h->tangent_coordinates = V2(len3(local) / d->radius, phi / (2.0f * PI_F));
    v3 tangent = norm3(displacement);
    v3 bitangent = V3(f_cos(phi), 0.0f, -f_sin(phi));
    bitangent = mv3(tr.axes, bitangent);
    h->tangent_space = M3(tangent, bitangent, tr.axes.c[1]);
}
/* frag:273-295 */
static void hollow_disk_tangent_space(HitInfo* h, const HollowDisk* d) {
    Transform tr = d->plane.transform;
    v3 displacement = sub3(h->intersection_point, tr.pos);
    v3 local = mtv3(tr.axes, displacement);
    float phi = f_atan2(local.x, local.z);
    if (phi < 0.0f) phi += 2.0f * PI_F;
    h->tangent_coordinates = V2((len3(local) - d->inner_radius) / (d->outer_radius - d->inner_radius),
                                phi / (2.0f * PI_F));
    v3 tangent = norm3(displacement);
    v3 bitangent = V3(f_cos(phi), 0.0f, -f_sin(phi));
    bitangent = mv3(tr.axes, bitangent);
    h->tangent_space = M3(tangent, bitangent, tr.axes.c[1]);
}
/* frag:297-318 */
static void cylinder_tangent_space(HitInfo* h, const Cylinder* cy) {
    Transform tr = cy->transform;
    v3 displacement = sub3(h->intersection_point, tr.pos);
    v3 normal = norm3(displacement);
    v3 bitangent = tr.axes.c[1];
    v3 local = mtv3(tr.axes, displacement);
    float phi = f_atan2(local.x, local.z);
    if (phi < 0.0f) phi += 2.0f * PI_F;
    h->tangent_coordinates = V2(phi / (2.0f * PI_F), local.y / cy->height);
    v3 tangent = mv3(tr.axes, V3(f_cos(phi), 0.0f, -f_sin(phi)));
    h->tangent_space = M3(tangent, bitangent, normal);
}
/* frag:320-333 */
static void rectangle_tangent_space(HitInfo* h, const Rectangle* r) {
    Transform tr = r->plane.transform;
    v3 displacement = sub3(h->intersection_point, tr.pos);
    v3 local = mtv3(tr.axes, displacement);
    h->tangent_coordinates = V2(local.x / r->width, local.z / r->height);
    h->tangent_coordinates.y = 1.0f - h->tangent_coordinates.y;
    h->tangent_space = M3(tr.axes.c[0], neg3(tr.axes.c[2]), tr.axes.c[1]);
}

/* ---- Binet equation + RK4 (frag:336-355) ------------------------------- */
static inline float ddu(float u) { return -u * (1.0f - 1.5f * u); }
static inline v2 rk4_step(float u_i, float du_i, float delta_phi) {
    float k1 = du_i;
    float l1 = ddu(u_i);
    float k2 = du_i + 0.5f * l1 * delta_phi;
    float l2 = ddu(u_i + 0.5f * k1 * delta_phi);
    float k3 = du_i + 0.5f * l2 * delta_phi;
    float l3 = ddu(u_i + 0.5f * k2 * delta_phi);
    float k4 = du_i + l3 * delta_phi;
    float l4 = ddu(u_i + k3 * delta_phi);
    return V2(delta_phi / 6.0f * (k1 + 2.0f * k2 + 2.0f * k3 + k4),
              delta_phi / 6.0f * (l1 + 2.0f * l2 + 2.0f * l3 + l4));
}

/* ---- lighting (frag:365-438) ------------------------------------------- */
static v4 calculate_lighting(const Ctx* c, HitInfo h, v3 view_dir) {
    const sr_scene* sc = c->scene;
    if (h.object.type == OBJECT_TYPE_SPECIAL) return V4(0, 0, 0, 1);
    if (h.object.type == OBJECT_TYPE_TEST_RAY_CURVED) {
        const float* k = c->tr->curved_color;
        return V4(k[0], k[1], k[2], k[3]);
    }
    if (h.object.type == OBJECT_TYPE_TEST_RAY_FLAT) {
        const float* k = c->tr->flat_color;
        return V4(k[0], k[1], k[2], k[3]);
    }
    int mi = h.object.material_index;
    if (mi < 0 || mi >= SR_MAX_MATERIALS) mi = 0; /* GLSL: out-of-range array read is undefined */
    const sr_material* m = &sc->materials[mi];
    if (m->flip_normals) h.tangent_space.c[2] = scl3(h.tangent_space.c[2], -1.0f);
    if (!m->double_sided_normals && dot3(h.tangent_space.c[2], view_dir) < 0.0f)
        return V4(0, 0, 0, 0);
    v2 object_uv = h.tangent_coordinates;

    int is_plane = h.object.type == SR_OBJECT_PLANE;
    int pi = h.object.index;
    if (pi < 0 || pi >= SR_MAX_PLANES) pi = 0;
    Plane plane_obj = to_plane(&sc->planes[pi]);

    if (m->swap_uvs) object_uv = V2(object_uv.y, object_uv.x);
    if (m->invert_uv_x) object_uv.x = (is_plane ? plane_obj.texture_size.x : 1.0f) - object_uv.x;
    if (m->invert_uv_y) object_uv.y = (is_plane ? plane_obj.texture_size.y : 1.0f) - object_uv.y;

    v4 base_color = V4(m->color[0], m->color[1], m->color[2], m->color[3]);
    if (m->texture_index >= 0) {
        int ti = m->texture_index < SR_MAX_TEXTURES ? m->texture_index : 0;
        v2 ts = V2(sc->texture_sizes[ti][0], sc->texture_sizes[ti][1]);
        v2 mts = V2(sc->max_texture_size[0], sc->max_texture_size[1]);
        v2 rescaled_uv = V2((object_uv.x * ts.x) / mts.x, (object_uv.y * ts.y) / mts.y);
        int render_color = 1;
        if (is_plane) {
            Plane plane = plane_obj;
            rescaled_uv = V2(rescaled_uv.x - plane.texture_offset.x, rescaled_uv.y - plane.texture_offset.y);
            v2 plane_uv = V2(rescaled_uv.x / plane.texture_size.x, rescaled_uv.y / plane.texture_size.y);
            rescaled_uv.x = f_mod(rescaled_uv.x, plane.texture_size.x);
            rescaled_uv.y = f_mod(rescaled_uv.y, plane.texture_size.y);
            rescaled_uv = V2(rescaled_uv.x / plane.texture_size.x, rescaled_uv.y / plane.texture_size.y);
            render_color = plane.repeat_texture ||
                           ((plane_uv.x >= 0.0f && plane_uv.x <= 1.0f) &&
                            (plane_uv.y >= 0.0f && plane_uv.y <= 1.0f));
        }
        if (render_color) base_color = texture_array(c, rescaled_uv, m->texture_index);
    }
    v3 base_rgb = V3(base_color.x, base_color.y, base_color.z);
    v3 final_color = scl3(base_rgb, m->ambient);

    v3 normal = h.tangent_space.c[2];
    if (m->normal_map_index >= 0) {
        int ni = m->normal_map_index < SR_MAX_TEXTURES ? m->normal_map_index : 0;
        v2 ts = V2(sc->texture_sizes[ni][0], sc->texture_sizes[ni][1]);
        v2 mts = V2(sc->max_texture_size[0], sc->max_texture_size[1]);
        v2 rescaled_uv = V2((object_uv.x * ts.x) / mts.x, (object_uv.y * ts.y) / mts.y);
        v4 nm = texture_array(c, rescaled_uv, m->normal_map_index);
        normal = norm3(mv3(h.tangent_space, V3(nm.x, nm.y, nm.z)));
    }

    int nl = sc->num_lights;
    if (nl > SR_MAX_LIGHTS) nl = SR_MAX_LIGHTS;
    for (int i = 0; i < nl; i++) {
        const sr_light* L = &sc->lights[i];
        v3 lpos = load_v3(L->transform.pos);
        v3 lcol = load_v3(L->color);
        v3 light_dir = norm3(sub3(lpos, h.intersection_point));
        float distance = len3(sub3(lpos, h.intersection_point));
        float attenuation = 1.0f / (L->attenuation_constant + L->attenuation_linear * distance +
                                    L->attenuation_quadratic * distance * distance);
        float diff = f_max(dot3(normal, light_dir), 0.0f);
        v3 diffuse = mul3(scl3(lcol, m->diffuse * diff), base_rgb);
        /* reflect(I, N) = I - 2 * dot(N, I) * N */
        v3 I = neg3(light_dir);
        v3 reflect_dir = sub3(I, scl3(normal, 2.0f * dot3(normal, I)));
        float spec = f_pow(f_max(dot3(view_dir, reflect_dir), 0.0f), m->shininess);
        v3 specular = scl3(lcol, m->specular * spec);
        final_color = add3(final_color, scl3(scl3(add3(diffuse, specular), attenuation), L->intensity));
    }
    return V4(final_color.x, final_color.y, final_color.z, base_color.w);
}

/* ---- intersections (frag:440-736) -------------------------------------- */
/* frag:441-454 */
static float min_positive(float n1, float n2) {
    float n = -1.0f;
    if (n1 > 0.0f && n2 > 0.0f) n = f_min(n1, n2);
    else if (n1 > 0.0f) n = n1;
    else if (n2 > 0.0f) n = n2;
    return n;
}
/* frag:457-478 */
static HitInfo sphere_intersect(Ray ray, const Sphere* s, float max_lambda) {
    HitInfo res = miss();
    v3 oc = sub3(ray.origin, s->transform.pos);
    float b = dot3(ray.dir, oc);
    float D = b * b - dot3(oc, oc) + s->radius * s->radius;
    if (D < 0.0f) return res;
    float sqrt_D = sqrtf(D);
    float first_term = -dot3(ray.dir, oc);
    float lambda1 = first_term - sqrt_D;
    float lambda2 = first_term + sqrt_D;
    float lambda = min_positive(lambda1, lambda2);
    res.is_hit = lambda >= 0.0f && (max_lambda < 0.0f || lambda <= max_lambda);
    if (!res.is_hit) return res;
    res.intersection_point = add3(ray.origin, scl3(ray.dir, lambda));
    res.dist = len3(sub3(res.intersection_point, ray.origin));
    sphere_tangent_space(&res, s);
    return res;
}
/* frag:483-500 */
static HitInfo plane_intersect(Ray ray, const Plane* p, float max_lambda) {
    HitInfo res = miss();
    v3 normal = p->transform.axes.c[1];
    float denom = dot3(normal, ray.dir);
    if (fabsf(denom) < EPSILON_F) return res;
    float lambda = dot3(normal, sub3(p->transform.pos, ray.origin)) / denom;
    res.is_hit = lambda >= 0.0f && (max_lambda < 0.0f || lambda <= max_lambda);
    if (!res.is_hit) return res;
    res.intersection_point = add3(ray.origin, scl3(ray.dir, lambda));
    res.dist = len3(sub3(res.intersection_point, ray.origin));
    plane_tangent_space(&res, p);
    return res;
}
/* frag:502-508 */
static HitInfo disk_intersect(Ray ray, const Disk* d, float max_lambda) {
    HitInfo res = plane_intersect(ray, &d->plane, max_lambda);
    v3 q = sub3(res.intersection_point, d->plane.transform.pos);
    res.is_hit = res.is_hit && dot3(q, q) <= d->radius * d->radius;
    if (!res.is_hit) return res;
    disk_tangent_space(&res, d);
    return res;
}
/* frag:510-517 */
static HitInfo hollow_disk_intersect(Ray ray, const HollowDisk* d, float max_lambda) {
    HitInfo res = plane_intersect(ray, &d->plane, max_lambda);
    v3 q = sub3(res.intersection_point, d->plane.transform.pos);
    float squared_dist = dot3(q, q);
    res.is_hit = res.is_hit && squared_dist >= d->inner_radius * d->inner_radius &&
                 squared_dist <= d->outer_radius * d->outer_radius;
    if (!res.is_hit) return res;
    hollow_disk_tangent_space(&res, d);
    return res;
}
/* frag:519-521 */
static int is_in_range(float n, float lo, float hi) { return n >= lo && n <= hi; }
/* frag:523-571 */
static HitInfo cylinder_intersect(Ray ray, const Cylinder* cy, float max_lambda) {
    v3 pos = cy->transform.pos;
    m3 axes = cy->transform.axes;
    v3 axis = axes.c[1];
    float height = cy->height;
    float radius = cy->radius;
    v3 local_origin = mtv3(axes, sub3(ray.origin, pos));
    v3 local_dir = mtv3(axes, ray.dir);
    float origin_parallel_sq = sqv2(V2(local_origin.x, local_origin.z));
    float dir_parallel_sq = sqv2(V2(local_dir.x, local_dir.z));
    float a = local_origin.x * local_dir.x + local_origin.z * local_dir.z;
    float D = a * a + dir_parallel_sq * (radius * radius - origin_parallel_sq);
    HitInfo res = miss();
    if (D < 0.0f) return res;
    float lambda1 = -(a + sqrtf(D)) / dir_parallel_sq;
    float lambda2 = -(a - sqrtf(D)) / dir_parallel_sq;
    v3 p1 = add3(ray.origin, scl3(ray.dir, lambda1));
    v3 p2 = add3(ray.origin, scl3(ray.dir, lambda2));
    int in1 = is_in_range(dot3(sub3(p1, pos), axis), 0.0f, height);
    int in2 = is_in_range(dot3(sub3(p2, pos), axis), 0.0f, height);
    if (!in1 && !in2) return res;
    float lambda = -1.0f;
    if (in1 && in2) lambda = min_positive(lambda1, lambda2);
    else if (in1) lambda = lambda1;
    else if (in2) lambda = lambda2;
    res.intersection_point = add3(ray.origin, scl3(ray.dir, lambda));
    res.is_hit = lambda >= 0.0f && (max_lambda < 0.0f || lambda <= max_lambda);
    if (!res.is_hit) return res;
    res.dist = len3(sub3(res.intersection_point, ray.origin));
    cylinder_tangent_space(&res, cy);
    return res;
}
/* frag:573-584 */
static HitInfo rectangle_intersect(Ray ray, const Rectangle* r, float max_lambda) {
    HitInfo res = plane_intersect(ray, &r->plane, max_lambda);
    if (!res.is_hit) return res;
    Transform tr = r->plane.transform;
    float alpha = dot3(sub3(res.intersection_point, tr.pos), tr.axes.c[0]);
    float beta = dot3(sub3(res.intersection_point, tr.pos), tr.axes.c[2]);
    res.is_hit = is_in_range(alpha, 0.0f, r->width) && is_in_range(beta, 0.0f, r->height);
    if (!res.is_hit) return res;
    rectangle_tangent_space(&res, r);
    return res;
}
static Rectangle make_rect(v3 pos, m3 axes, float w, float h) {
    Rectangle r;
    memset(&r, 0, sizeof r);
    r.plane.transform.pos = pos;
    r.plane.transform.axes = axes;
    r.width = w;
    r.height = h;
    return r;
}
/* frag:586-695 */
static HitInfo box_intersect(Ray ray, const Box* b, float max_lambda) {
    v3 p = b->transform.pos;
    m3 A = b->transform.axes;
    v3 a0 = A.c[0], a1 = A.c[1], a2 = A.c[2];
    Rectangle rects[6];
    rects[0] = make_rect(add3(p, scl3(a2, b->depth)), M3(a0, neg3(a1), neg3(a2)), b->width, b->depth);
    rects[1] = rects[0];
    rects[1].plane.transform.pos = add3(p, scl3(a1, b->height));
    rects[1].plane.transform.axes = A;
    rects[3] = make_rect(add3(p, mv3(A, V3(b->width, b->height, 0.0f))), M3(neg3(a0), neg3(a2), neg3(a1)),
                         b->width, b->height);
    rects[2] = rects[3];
    rects[2].plane.transform.pos = add3(p, mv3(A, V3(0.0f, b->height, b->depth)));
    rects[2].plane.transform.axes = M3(a0, a2, neg3(a1));
    rects[4] = make_rect(add3(p, scl3(a1, b->height)), M3(a2, neg3(a0), neg3(a1)), b->depth, b->height);
    rects[5] = rects[4];
    rects[5].plane.transform.pos = add3(p, mv3(A, V3(b->width, b->height, b->depth)));
    rects[5].plane.transform.axes = M3(neg3(a2), a0, neg3(a1));
    /* order: bot, top, front, back, left, right (frag:649) */
    HitInfo res = miss();
    int closest_index = -1;
    for (int i = 0; i < 6; i++) {
        HitInfo hi = rectangle_intersect(ray, &rects[i], max_lambda);
        if (!hi.is_hit) continue;
        if (closest_index < 0 || hi.dist < res.dist) {
            res = hi;
            closest_index = i;
        }
    }
    if (!res.is_hit) return res;
    rectangle_tangent_space(&res, &rects[closest_index]);
    static const float off[6][2] = {{1, 0}, {1, 2}, {1, 1}, {3, 1}, {0, 1}, {2, 1}};
    if (off[closest_index][0] != 0.0f) res.tangent_coordinates.x += off[closest_index][0];
    if (off[closest_index][1] != 0.0f) res.tangent_coordinates.y += off[closest_index][1];
    res.tangent_coordinates.x /= 4.0f;
    res.tangent_coordinates.y /= 3.0f;
    return res;
}
/* frag:697-736 */
static HitInfo intersect_object(const Ctx* c, Ray ray, Object o, float max_lambda) {
    const sr_scene* sc = c->scene;
    HitInfo res = miss();
    int k = o.index;
    switch (o.type) {
    case SR_OBJECT_SPHERE:
        if (k >= 0 && k < SR_MAX_SPHERES) {
            Sphere s;
            s.transform = to_transform(&sc->spheres[k].transform);
            s.radius = sc->spheres[k].radius;
            res = sphere_intersect(ray, &s, max_lambda);
        }
        break;
    case SR_OBJECT_PLANE:
        if (k >= 0 && k < SR_MAX_PLANES) {
            Plane p = to_plane(&sc->planes[k]);
            res = plane_intersect(ray, &p, max_lambda);
        }
        break;
    case SR_OBJECT_DISK:
        if (k >= 0 && k < SR_MAX_DISKS) {
            Disk d;
            d.plane = to_plane(&sc->disks[k].plane);
            d.radius = sc->disks[k].radius;
            res = disk_intersect(ray, &d, max_lambda);
        }
        break;
    case SR_OBJECT_HOLLOW_DISK:
        if (k >= 0 && k < SR_MAX_HOLLOW_DISKS) {
            HollowDisk d;
            d.plane = to_plane(&sc->hollow_disks[k].plane);
            d.inner_radius = sc->hollow_disks[k].inner_radius;
            d.outer_radius = sc->hollow_disks[k].outer_radius;
            res = hollow_disk_intersect(ray, &d, max_lambda);
        }
        break;
    case SR_OBJECT_CYLINDER:
        if (k >= 0 && k < SR_MAX_CYLINDERS) {
            Cylinder cy;
            cy.transform = to_transform(&sc->cylinders[k].transform);
            cy.height = sc->cylinders[k].height;
            cy.radius = sc->cylinders[k].radius;
            res = cylinder_intersect(ray, &cy, max_lambda);
        }
        break;
    case SR_OBJECT_RECTANGLE:
        if (k >= 0 && k < SR_MAX_RECTANGLES) {
            Rectangle r;
            r.plane = to_plane(&sc->rectangles[k].plane);
            r.width = sc->rectangles[k].width;
            r.height = sc->rectangles[k].height;
            res = rectangle_intersect(ray, &r, max_lambda);
        }
        break;
    case SR_OBJECT_BOX:
        if (k >= 0 && k < SR_MAX_BOXES) {
            Box b;
            b.transform = to_transform(&sc->boxes[k].transform);
            b.width = sc->boxes[k].width;
            b.depth = sc->boxes[k].depth;
            b.height = sc->boxes[k].height;
            res = box_intersect(ray, &b, max_lambda);
        }
        break;
    default:
        break;
    }
    res.object = o;
    return res;
}
/* frag:739-741 */
static v3 project(v3 v, v3 target) { return scl3(target, dot3(v, target) / dot3(target, target)); }
/* frag:744-753 */
static m3 gram_schmidt(m3 m) {
    m.c[0] = sub3(m.c[0], project(m.c[0], m.c[1]));
    m.c[2] = sub3(sub3(m.c[2], project(m.c[2], m.c[1])), project(m.c[2], m.c[0]));
    m.c[0] = norm3(m.c[0]);
    m.c[1] = norm3(m.c[1]);
    m.c[2] = norm3(m.c[2]);
    return m;
}
static m3 test_ray_frame(v3 d) { return gram_schmidt(M3(V3(d.x, d.z, d.y), d, V3(d.z, d.x, d.y))); }

/* frag:755-822 */
static v4 intersect(const Ctx* c, Ray ray, float max_lambda) {
    static const Sphere BLACK_HOLE = {{{0, 0, 0}, {{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}}}, 1.0f};
    HitInfo closest = sphere_intersect(ray, &BLACK_HOLE, max_lambda);
    closest.object.type = OBJECT_TYPE_SPECIAL;

    const sr_test_ray* tr = c->tr;
    if (tr && tr->visible) {
        Cylinder cy;
        cy.transform.pos = load_v3(tr->flat_origin);
        cy.transform.axes = test_ray_frame(load_v3(tr->flat_dir));
        cy.height = tr->extended_length;
        cy.radius = tr->radius;
        HitInfo hit = cylinder_intersect(ray, &cy, max_lambda);
        hit.object.type = OBJECT_TYPE_TEST_RAY_FLAT;
        if (hit.is_hit && (!closest.is_hit || hit.dist < closest.dist)) closest = hit;

        int n = tr->num_curved_points;
        if (n > SR_MAX_POINTS) n = SR_MAX_POINTS;
        for (int i = 0; i < n - 1; i++) {
            if (n < 2) break;
            v3 pi = load_v3(tr->curved_points[i]);
            v3 diff = sub3(load_v3(tr->curved_points[i + 1]), pi);
            float test_ray_length = len3(diff);
            if (i == n - 2 && len3(load_v3(tr->curved_points[n - 1])) < 1.0f)
                test_ray_length = tr->extended_length;
            Cylinder seg;
            seg.transform.pos = pi;
            seg.transform.axes = test_ray_frame(diff);
            seg.height = test_ray_length;
            seg.radius = tr->radius;
            HitInfo h2 = cylinder_intersect(ray, &seg, max_lambda);
            h2.object.type = OBJECT_TYPE_TEST_RAY_CURVED;
            if (!h2.is_hit) continue;
            if (!closest.is_hit || h2.dist < closest.dist) closest = h2;
        }
    }

    int no = c->scene->num_objects;
    if (no > SR_MAX_OBJECTS) no = SR_MAX_OBJECTS;
    for (int i = 0; i < no; i++) {
        const sr_object* so = &c->scene->objects[i];
        Object o = {so->type, so->index, so->material_index};
        HitInfo hit = intersect_object(c, ray, o, max_lambda);
        if (!hit.is_hit) continue;
        if (!closest.is_hit || hit.dist < closest.dist) closest = hit;
    }

    v4 color = V4(0, 0, 0, 0);
    if (closest.is_hit) color = calculate_lighting(c, closest, neg3(ray.dir));
    return color;
}

/* frag:829-837 */
static v4 get_bg(const Ctx* c, v3 dir) {
    float u = f_atan2(dir.z, dir.x) / PI_F;
    if (u < 0.0f) u += 2.0f;
    u *= 0.5f;
    float v = f_asin(dir.y) / PI_F + 0.5f;
    return texture_bg(c, V2(u, v));
}
/* frag:839-841 */
static float rand_glsl(v2 co) {
    return f_fract(f_sin(dot2(co, V2(12.9898f, 78.233f))) * 43758.5453f);
}

/* frag:843-936, one fragment. uv = pixel-centre NDC (full_screen_quad.vert:7-10). */
static int shade(const Ctx* c, v2 uv, v4* frag_out) {
    const sr_params* P = c->prm;
    v4 frag = V4(0, 0, 0, 0);
    int steps = 0;
    /* frag:845-857 */
    if (P->crosshair) {
        float hx = fabsf(uv.x * c->res_x / 2.0f), hy = fabsf(uv.y * c->res_y / 2.0f);
        const float cw = 2.0f, cs = 5.0f, cl = 10.0f;
        if ((hx < cw / 2.0f && hy > cs && hy < cl + cs) || (hy < cw / 2.0f && hx > cs && hx < cl + cs))
            frag = V4(0.5f, 0.5f, 0.5f, 0.5f);
    }
    /* frag:859-863 */
    float ray_forward = 1.0f / f_tan(c->cam->fov / 360.0f * PI_F);
    float max_angle = 2.0f * (float)P->max_revolutions * PI_F;
    v2 uv_vec = V2(uv.x, uv.y * c->res_y / c->res_x);
    m3 cam_axes = load_m3(c->cam->transform.axes);
    Ray ray;
    ray.origin = load_v3(c->cam->transform.pos);
    ray.dir = norm3(mv3(cam_axes, V3(uv_vec.x, uv_vec.y, ray_forward)));

    /* frag:865-881 */
    v3 normal_vec = norm3(ray.origin);
    int flat = P->raytrace_type == SR_RAYTRACE_FLAT ||
               (P->raytrace_type == SR_RAYTRACE_HALF_WIDTH && uv.x > 2.0f * P->curved_percentage + -1.0f) ||
               (P->raytrace_type == SR_RAYTRACE_HALF_HEIGHT && uv.y > 2.0f * P->curved_percentage + -1.0f);
    if (flat || fabsf(dot3(ray.dir, normal_vec)) >= 1.0f - EPSILON_F) {
        v4 ic = intersect(c, ray, -1.0f);
        frag = add4(frag, ic);
        if (ic.w != 1.0f) frag = add4(frag, get_bg(c, ray.dir));
        *frag_out = frag;
        return steps;
    } else if (rand_glsl(uv_vec) <= P->percent_black) {
        *frag_out = frag;
        return steps;
    }

    /* frag:883-889 */
    v3 tangent_vec = norm3(cross3(cross3(normal_vec, ray.dir), normal_vec));
    v3 prev_ray_pos;
    float u = 1.0f / len3(ray.origin);
    float du = -u * dot3(ray.dir, normal_vec) / dot3(ray.dir, tangent_vec);
    float phi = 0.0f;
    const float uf_radius = 1.0f / P->u_f;
    for (int i = 0; i < P->max_steps; i++) {
        steps++;
        /* frag:891-912 */
        if (u < P->u_f) {
            Sphere uf;
            uf.transform.pos = V3(0, 0, 0);
            uf.transform.axes = M3(V3(1, 0, 0), V3(0, 1, 0), V3(0, 0, 1));
            uf.radius = uf_radius;
            HitInfo uh = sphere_intersect(ray, &uf, -1.0f);
            if (!uh.is_hit) {
                v4 ic = intersect(c, ray, -1.0f);
                frag = add4(frag, ic);
                if (ic.w != 1.0f) frag = add4(frag, get_bg(c, ray.dir));
                *frag_out = frag;
                return steps;
            }
            normal_vec = norm3(uh.intersection_point);
            if (fabsf(dot3(ray.dir, normal_vec)) >= 1.0f - EPSILON_F) {
                v4 ic = intersect(c, ray, -1.0f);
                frag = add4(frag, ic);
                if (ic.w != 1.0f) frag = add4(frag, get_bg(c, ray.dir));
                *frag_out = frag;
                return steps;
            }
            tangent_vec = norm3(cross3(cross3(normal_vec, ray.dir), normal_vec));
            u = 1.0f / len3(uh.intersection_point);
            du = -u * dot3(ray.dir, normal_vec) / dot3(ray.dir, tangent_vec);
        }
        /* frag:914-922 */
        float step_size = (max_angle - phi) / (float)(P->max_steps - i);
        phi += step_size;
        v2 r = rk4_step(u, du, step_size);
        u += r.x;
        du += r.y;
        if (u < 0.0f) break;
        /* frag:924-932 */
        prev_ray_pos = ray.origin;
        ray.origin = div3s(add3(scl3(normal_vec, f_cos(phi)), scl3(tangent_vec, f_sin(phi))), u);
        v3 delta_ray = sub3(ray.origin, prev_ray_pos);
        float ray_length = len3(delta_ray);
        ray.dir = div3s(delta_ray, ray_length);
        Ray chord = {prev_ray_pos, ray.dir};
        v4 ic = intersect(c, chord, ray_length);
        frag = add4(frag, ic);
        if (ic.w == 1.0f) {
            *frag_out = frag;
            return steps;
        }
    }
    /* frag:935 */
    frag = add4(frag, get_bg(c, ray.dir));
    *frag_out = frag;
    return steps;
}

static inline v2 pixel_uv(int px, int py, int W, int H) {
    return V2((float)(2 * px + 1) / (float)W - 1.0f, (float)(2 * py + 1) / (float)H - 1.0f);
}
/* GL RGBA8 UNORM store: clamp to [0,1], round to nearest; NaN stores 0. */
static inline uint8_t to_unorm8(float x) {
    if (!(x > 0.0f)) return 0;
    if (x >= 1.0f) return 255;
    return (uint8_t)floorf(x * 255.0f + 0.5f);
}

int sro_shade_pixel(const sr_scene* scene, const sr_test_ray* test_ray, const sro_textures* tex,
                    const sr_camera* cam, const sr_params* params, int width, int height, int px,
                    int py, float out_rgba[4]) {
    Ctx c = {scene, test_ray, tex, cam, params, (float)width, (float)height};
    v4 f;
    int s = shade(&c, pixel_uv(px, py, width, height), &f);
    out_rgba[0] = f.x;
    out_rgba[1] = f.y;
    out_rgba[2] = f.z;
    out_rgba[3] = f.w;
    return s;
}

typedef struct {
    Ctx c;
    int W, H, row_begin, row_end, tid, nthreads;
    uint8_t* rgba8;
    float* rgba32;
    int32_t* steps;
} RenderJob;

static void* render_worker(void* arg) {
    RenderJob* j = (RenderJob*)arg;
    for (int y = j->row_begin + j->tid; y < j->row_end; y += j->nthreads) {
        size_t row = (size_t)(y - j->row_begin) * (size_t)j->W;
        for (int x = 0; x < j->W; x++) {
            v4 f;
            int s = shade(&j->c, pixel_uv(x, y, j->W, j->H), &f);
            size_t i = row + (size_t)x;
            if (j->rgba8) {
                j->rgba8[4 * i + 0] = to_unorm8(f.x);
                j->rgba8[4 * i + 1] = to_unorm8(f.y);
                j->rgba8[4 * i + 2] = to_unorm8(f.z);
                j->rgba8[4 * i + 3] = to_unorm8(f.w);
            }
            if (j->rgba32) {
                j->rgba32[4 * i + 0] = f.x;
                j->rgba32[4 * i + 1] = f.y;
                j->rgba32[4 * i + 2] = f.z;
                j->rgba32[4 * i + 3] = f.w;
            }
            if (j->steps) j->steps[i] = s;
        }
    }
    return NULL;
}

static int resolve_threads(int nthreads) {
    if (nthreads > 0) return nthreads;
    long n = sysconf(_SC_NPROCESSORS_ONLN);
    return n > 0 ? (int)n : 1;
}

int sro_render(const sr_scene* scene, const sr_test_ray* test_ray, const sro_textures* tex,
               const sr_camera* cam, const sr_params* params, int width, int height, int row_begin,
               int row_end, uint8_t* rgba8, float* rgba32, int32_t* steps, int nthreads) {
    if (!scene || !cam || !params || width <= 0 || height <= 0 || row_begin < 0 ||
        row_end > height || row_begin > row_end)
        return SR_E_INVALID;
    int nt = resolve_threads(nthreads);
    if (nt > 256) nt = 256;
    pthread_t th[256];
    RenderJob jobs[256];
    for (int t = 0; t < nt; t++) {
        RenderJob* j = &jobs[t];
        Ctx c = {scene, test_ray, tex, cam, params, (float)width, (float)height};
        j->c = c;
        j->W = width;
        j->H = height;
        j->row_begin = row_begin;
        j->row_end = row_end;
        j->tid = t;
        j->nthreads = nt;
        j->rgba8 = rgba8;
        j->rgba32 = rgba32;
        j->steps = steps;
        if (nt == 1) render_worker(j);
        else pthread_create(&th[t], NULL, render_worker, j);
    }
    if (nt > 1)
        for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
    return SR_OK;
}

/* ====================================================================== *
 * press-R CPU path, src/main.cpp:73-124. The reference compiles it as C++  *
 * against glm with double literals mixed into float code; the casts below  *
 * spell out where C++ evaluates in double and narrows.         *
 * ====================================================================== */
/* src/main.cpp:73-75 — `-u * (1. - 1.5 * u)` in double, narrowed on return */
static float c1_ddu(float u) { return (float)((double)(-u) * (1.0 - 1.5 * (double)u)); }
/* src/main.cpp:78-92 */
static void c1_rk4_step(float u_i, float du_i, float delta_phi, float* out_du, float* out_ddu) {
    float k1 = du_i;
    float l1 = c1_ddu(u_i);
    float k2 = (float)((double)du_i + 0.5 * (double)l1 * (double)delta_phi);
    float l2 = c1_ddu((float)((double)u_i + 0.5 * (double)k1 * (double)delta_phi));
    float k3 = (float)((double)du_i + 0.5 * (double)l2 * (double)delta_phi);
    float l3 = c1_ddu((float)((double)u_i + 0.5 * (double)k2 * (double)delta_phi));
    float k4 = du_i + l3 * delta_phi;
    float l4 = c1_ddu(u_i + k3 * delta_phi);
    /* glm::vec2(double, double): narrowed per component */
    *out_du = (float)((double)delta_phi / 6.0 *
                      ((double)k1 + 2.0 * (double)k2 + 2.0 * (double)k3 + (double)k4));
    *out_ddu = (float)((double)delta_phi / 6.0 *
                       ((double)l1 + 2.0 * (double)l2 + 2.0 * (double)l3 + (double)l4));
}

/* glm semantics: dot = (x*x' + y*y') + z*z', normalize = v * (1 / sqrt(dot)) */
static int c1_trace(v3 origin, v3 dir, int max_steps, int max_revolutions, float* out_xyz,
                    int max_points, v3** vec_out, int* vec_cap) {
    /* src/main.cpp:98-102 */
    v3 normal_vec = norm3(origin);
    v3 tangent_vec = norm3(cross3(cross3(normal_vec, dir), normal_vec));
    float u = (float)(1.0 / (double)len3(origin));
    float du = -u * dot3(dir, normal_vec) / dot3(dir, tangent_vec);
    int count = 0;
#define C1_PUSH(P)                                                                        \
    do {                                                                                  \
        if (out_xyz && count < max_points) {                                              \
            out_xyz[3 * count + 0] = (P).x;                                               \
            out_xyz[3 * count + 1] = (P).y;                                               \
            out_xyz[3 * count + 2] = (P).z;                                               \
        }                                                                                 \
        if (vec_out) {                                                                    \
            if (count >= *vec_cap) {                                                      \
                int nc = *vec_cap ? 2 * *vec_cap : 1;                                     \
                v3* nv = (v3*)realloc(*vec_out, (size_t)nc * sizeof(v3));                 \
                if (nv) { *vec_out = nv; *vec_cap = nc; }                                 \
            }                                                                             \
            if (count < *vec_cap) (*vec_out)[count] = (P);                                \
        }                                                                                 \
        count++;                                                                          \
    } while (0)
    /* src/main.cpp:104 — unqualified abs(float) resolves to ::abs(int) in that
     * translation unit: the float is truncated to int first. */
    if (abs((int)dot3(dir, normal_vec)) >= 1.0 - 0.000001) {
        v3 p1 = origin, p2 = add3(origin, dir);
        C1_PUSH(p1);
        C1_PUSH(p2);
        return count;
    }
    C1_PUSH(origin);
    /* MAX_TEST_RAY_ANGLE expands to `2. * float(MAX_REVOLUTIONS) * M_PI` (double) */
    const double max_angle = 2.0 * (double)(float)max_revolutions * M_PI;
    float phi = 0.0f;
    for (int i = 0; i < max_steps; i++) {
        float step_size = (float)((max_angle - (double)phi) / (double)(float)(max_steps - i));
        phi += step_size;
        float r_du, r_ddu;
        c1_rk4_step(u, du, step_size, &r_du, &r_ddu);
        u += r_du;
        if ((double)u < 0.0 || (double)u > 1.0) break;
        du += r_ddu;
        /* (float(cos(phi)) * n + float(sin(phi)) * t) / u — ::cos(double) */
        float cphi = (float)cos((double)phi), sphi = (float)sin((double)phi);
        v3 p = div3s(add3(scl3(normal_vec, cphi), scl3(tangent_vec, sphi)), u);
        C1_PUSH(p);
    }
#undef C1_PUSH
    return count;
}

int sro_test_ray_points(const float pos[3], const float forward[3], int max_steps,
                        int max_revolutions, float* out_xyz, int max_points) {
    /* src/main.cpp:95-96: origin = pos + dir * float(TEST_RAY_OFFSET) */
    v3 dir = load_v3(forward);
    v3 origin = add3(load_v3(pos), scl3(dir, 1.0f));
    return c1_trace(origin, dir, max_steps, max_revolutions, out_xyz, max_points, NULL, NULL);
}

/* BASELINE config 1: one press-R ray (src/main.cpp:94-124, a std::vector of
 * points per call) traced `reps` times on this thread, for a per-ray time.
 * Returns the points of one trace. */
int sro_pressr_ray_repeat(const float pos[3], const float forward[3], int max_steps, int max_revolutions,
                          int reps) {
    v3 dir = load_v3(forward);
    v3 origin = add3(load_v3(pos), scl3(dir, 1.0f));
    int n = 0;
    for (int k = 0; k < reps; k++) {
        v3* vec = NULL;
        int cap = 0;
        n = c1_trace(origin, dir, max_steps, max_revolutions, NULL, 0, &vec, &cap);
        free(vec);
    }
    return n;
}

typedef struct {
    const sr_camera* cam;
    int W, H, row_begin, row_end, tid, nthreads, max_steps, max_revolutions;
    int64_t total;
} SweepJob;

static void* sweep_worker(void* arg) {
    SweepJob* j = (SweepJob*)arg;
    float ray_forward = 1.0f / f_tan(j->cam->fov / 360.0f * PI_F);
    m3 axes = load_m3(j->cam->transform.axes);
    v3 pos = load_v3(j->cam->transform.pos);
    float aspect_scale = (float)j->H / (float)j->W;
    int64_t total = 0;
    for (int y = j->row_begin + j->tid; y < j->row_end; y += j->nthreads) {
        for (int x = 0; x < j->W; x++) {
            v2 uv = pixel_uv(x, y, j->W, j->H);
            v3 dir = norm3(mv3(axes, V3(uv.x, uv.y * (float)j->H / (float)j->W, ray_forward)));
            (void)aspect_scale;
            v3 origin = add3(pos, scl3(dir, 1.0f));
            v3* vec = NULL; /* one std::vector per ray */
            int cap = 0;
            total += c1_trace(origin, dir, j->max_steps, j->max_revolutions, NULL, 0, &vec, &cap);
            free(vec);
        }
    }
    j->total = total;
    return NULL;
}

int64_t sro_pressr_sweep(const sr_camera* cam, int width, int height, int row_begin, int row_end,
                         int max_steps, int max_revolutions, int nthreads) {
    if (!cam || width <= 0 || height <= 0 || row_begin < 0 || row_end > height || row_begin > row_end)
        return -1;
    int nt = resolve_threads(nthreads);
    if (nt > 256) nt = 256;
    pthread_t th[256];
    SweepJob jobs[256];
    for (int t = 0; t < nt; t++) {
        SweepJob* j = &jobs[t];
        j->cam = cam;
        j->W = width;
        j->H = height;
        j->row_begin = row_begin;
        j->row_end = row_end;
        j->tid = t;
        j->nthreads = nt;
        j->max_steps = max_steps;
        j->max_revolutions = max_revolutions;
        j->total = 0;
        if (nt == 1) sweep_worker(j);
        else pthread_create(&th[t], NULL, sweep_worker, j);
    }
    int64_t total = 0;
    for (int t = 0; t < nt; t++) {
        if (nt > 1) pthread_join(th[t], NULL);
        total += jobs[t].total;
    }
    return total;
}
