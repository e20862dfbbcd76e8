// vecmath.hpp — the small float vector library the host-side scene classes
// use in place of glm (glm is not vendored by the reference and is absent
// here). The operations the reference's scene code calls are given glm's
// evaluation order, so host-built scenes carry the same float bits:
//   dot(a, b)     = (a.x*b.x + a.y*b.y) + a.z*b.z
//   normalize(v)  = v * (1 / sqrt(dot(v, v)))     (glm inversesqrt)
//   cross(a, b)   = (a.y*b.z - b.y*a.z, a.z*b.x - b.z*a.x, a.x*b.y - b.x*a.y)
//   angleAxis / toMat3 as glm's quaternion routines.
// Compile users with -ffp-contract=off.
#ifndef SR_VECMATH_HPP
#define SR_VECMATH_HPP

#include <cmath>

namespace sr {

struct vec2 {
    float x = 0.f, y = 0.f;
    vec2() = default;
    vec2(float a, float b) : x(a), y(b) {}
};

struct vec3 {
    float x = 0.f, y = 0.f, z = 0.f;
    vec3() = default;
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};

struct vec4 {
    float x = 0.f, y = 0.f, z = 0.f, w = 0.f;
    vec4() = default;
    vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
};

inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator/(vec3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline vec3& operator+=(vec3& a, vec3 b) { a = a + b; return a; }
inline vec3& operator/=(vec3& a, float s) { a = a / s; return a; }

inline float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float length(vec3 a) { return std::sqrt(dot(a, a)); }
inline vec3 normalize(vec3 a) { return a * (1.0f / std::sqrt(dot(a, a))); }
inline vec3 cross(vec3 a, vec3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}

// Column-major 3x3 (m[c] is column c), as glm::mat3.
struct mat3 {
    vec3 c[3] = {vec3(1, 0, 0), vec3(0, 1, 0), vec3(0, 0, 1)};
    mat3() = default;
    mat3(vec3 c0, vec3 c1, vec3 c2) : c{c0, c1, c2} {}
    vec3& operator[](int i) { return c[i]; }
    const vec3& operator[](int i) const { return c[i]; }
};
inline vec3 operator*(const mat3& m, vec3 v) { return (m.c[0] * v.x + m.c[1] * v.y) + m.c[2] * v.z; }

struct quat {
    float w = 1.f, x = 0.f, y = 0.f, z = 0.f;
};

// glm::angleAxis: (cos(a/2), axis * sin(a/2)), std:: float trig.
inline quat angleAxis(float angle, vec3 axis) {
    float s = std::sin(angle * 0.5f);
    quat q;
    q.w = std::cos(angle * 0.5f);
    vec3 v = axis * s;
    q.x = v.x;
    q.y = v.y;
    q.z = v.z;
    return q;
}

// glm::mat3_cast / toMat3
inline mat3 toMat3(const quat& q) {
    float qxx = q.x * q.x, qyy = q.y * q.y, qzz = q.z * q.z;
    float qxz = q.x * q.z, qxy = q.x * q.y, qyz = q.y * q.z;
    float qwx = q.w * q.x, qwy = q.w * q.y, qwz = q.w * q.z;
    mat3 r;
    r.c[0].x = 1.f - 2.f * (qyy + qzz);
    r.c[0].y = 2.f * (qxy + qwz);
    r.c[0].z = 2.f * (qxz - qwy);
    r.c[1].x = 2.f * (qxy - qwz);
    r.c[1].y = 1.f - 2.f * (qxx + qzz);
    r.c[1].z = 2.f * (qyz + qwx);
    r.c[2].x = 2.f * (qxz + qwy);
    r.c[2].y = 2.f * (qyz - qwx);
    r.c[2].z = 1.f - 2.f * (qxx + qyy);
    return r;
}

}  // namespace sr

#endif
