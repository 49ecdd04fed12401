// gvrt_math.h — the float32 vector/matrix subset the reference's host camera code uses, with glm's
// memory layout (column-major, m[col][row]) and glm's operation order, so that the matrices this host
// layer hands to the renderer are bit-identical to the reference's (checked against the reference's own
// camera.hpp / LoadCamera.hpp / vendored glm built from its sources: tests/test_host_cpp.py).
//
// Operation order follows glm 0.9.8 as vendored by the reference (external/glm):
//   dot3 = (x*x' + y*y') + z*z'; normalize(v) = v * (1 / sqrt(dot(v, v))); cross as compute_cross;
//   lookAtRH (gtc/matrix_transform.inl); perspective_Vulkan_no_depth_reverse (:276-290);
//   translate: Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3];
//   inverse: compute_inverse<mat4> cofactor form (detail/func_matrix.inl:299-354);
//   quat_cast (gtc/quaternion.inl); radians(deg) = deg * float(0.0174532925...).
// Build with -ffp-contract=off on x86-64 (SSE float arithmetic, as the reference's own build): every
// expression below is one IEEE binary32 operation per operator.
#pragma once
#include <cmath>

namespace gm {

struct vec3 {
    float x = 0, y = 0, z = 0;
    vec3() = default;
    constexpr vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};
struct vec4 {
    float x = 0, y = 0, z = 0, w = 0;
    vec4() = default;
    constexpr vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    vec4(const vec3& v, float d) : x(v.x), y(v.y), z(v.z), w(d) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};
struct quat {  // glm::quat member order (x, y, z, w)
    float x = 0, y = 0, z = 0, w = 1;
};

inline vec3 operator+(const vec3& a, const vec3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(const vec3& a, const vec3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator-(const vec3& a) { return {-a.x, -a.y, -a.z}; }
inline vec3 operator*(const vec3& a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator/(const vec3& a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline vec3& operator+=(vec3& a, const vec3& b) { return a = a + b; }
inline vec3& operator-=(vec3& a, const vec3& b) { return a = a - b; }
inline vec4 operator+(const vec4& a, const vec4& b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline vec4 operator*(const vec4& a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline vec4 operator*(const vec4& a, const vec4& b) { return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
inline vec4 operator-(const vec4& a, const vec4& b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline bool operator==(const vec3& a, const vec3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

inline float dot(const vec3& a, const vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline vec3 cross(const vec3& x, const vec3& y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline float inversesqrt(float x) { return 1.0f / std::sqrt(x); }
inline vec3 normalize(const vec3& v) { return v * inversesqrt(dot(v, v)); }
inline float length(const vec3& v) { return std::sqrt(dot(v, v)); }
inline float radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }

// 3x3 and 4x4, column-major: m[c] is column c (glm::mat3 / glm::mat4)
struct mat3 {
    vec3 c[3];
    mat3() : c{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}} {}
    vec3& operator[](int i) { return c[i]; }
    const vec3& operator[](int i) const { return c[i]; }
};
struct mat4 {
    vec4 c[4];
    mat4() : mat4(1.0f) {}
    explicit mat4(float d) : c{{d, 0, 0, 0}, {0, d, 0, 0}, {0, 0, d, 0}, {0, 0, 0, d}} {}
    mat4(const vec4& a, const vec4& b, const vec4& d, const vec4& e) : c{a, b, d, e} {}
    explicit mat4(const mat3& m) : c{vec4(m[0], 0), vec4(m[1], 0), vec4(m[2], 0), {0, 0, 0, 1}} {}
    vec4& operator[](int i) { return c[i]; }
    const vec4& operator[](int i) const { return c[i]; }
    const float* data() const { return &c[0].x; }  // glm::value_ptr: the 16 floats of the UBO
};
inline bool operator==(const mat4& a, const mat4& b) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            if (a[i][j] != b[i][j]) return false;
    return true;
}
inline bool operator!=(const mat4& a, const mat4& b) { return !(a == b); }

inline mat3 mat3_of(const mat4& m) {
    mat3 r;
    for (int i = 0; i < 3; ++i) r[i] = {m[i].x, m[i].y, m[i].z};
    return r;
}
inline mat3 transpose(const mat3& m) {
    mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[i][j] = m[j][i];
    return r;
}
inline mat4 transpose(const mat4& m) {
    mat4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r[i][j] = m[j][i];
    return r;
}
inline mat3 operator-(const mat3& m) {
    mat3 r;
    for (int i = 0; i < 3; ++i) r[i] = -m[i];
    return r;
}
inline vec3 operator*(const mat3& m, const vec3& v) {
    return {m[0][0] * v.x + m[1][0] * v.y + m[2][0] * v.z, m[0][1] * v.x + m[1][1] * v.y + m[2][1] * v.z,
            m[0][2] * v.x + m[1][2] * v.y + m[2][2] * v.z};
}

inline mat4 translate(const mat4& m, const vec3& v) {
    mat4 r(m);
    r[3] = m[0] * v[0] + m[1] * v[1] + m[2] * v[2] + m[3];
    return r;
}

inline mat4 lookAt(const vec3& eye, const vec3& center, const vec3& up) {  // lookAtRH
    const vec3 f(normalize(center - eye));
    const vec3 s(normalize(cross(f, up)));
    const vec3 u(cross(s, f));
    mat4 r(1.0f);
    r[0][0] = s.x;
    r[1][0] = s.y;
    r[2][0] = s.z;
    r[0][1] = u.x;
    r[1][1] = u.y;
    r[2][1] = u.z;
    r[0][2] = -f.x;
    r[1][2] = -f.y;
    r[2][2] = -f.z;
    r[3][0] = -dot(s, eye);
    r[3][1] = -dot(u, eye);
    r[3][2] = dot(f, eye);
    return r;
}

// The reference's modified glm (matrix_transform.inl:276-290): [1][1] = -1/tan, so image row 0 is the top.
inline mat4 perspective_Vulkan_no_depth_reverse(float fovy, float aspect, float zNear, float zFar) {
    const float tanHalfFovy = std::tan(fovy / 2.0f);
    mat4 r(0.0f);
    r[0][0] = 1.0f / (aspect * tanHalfFovy);
    r[1][1] = -1.0f / (tanHalfFovy);
    r[2][3] = -1.0f;
    r[2][2] = -zFar / (zFar - zNear);
    r[3][2] = -(zFar * zNear) / (zFar - zNear);
    return r;
}

inline mat4 inverse(const mat4& m) {
    const float c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3],
                c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    const float c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3], c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3],
                c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    const float c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2], c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2],
                c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    const float c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3], c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3],
                c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    const float c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2], c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2],
                c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    const float c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1], c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1],
                c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    const vec4 f0(c00, c00, c02, c03), f1(c04, c04, c06, c07), f2(c08, c08, c10, c11);
    const vec4 f3(c12, c12, c14, c15), f4(c16, c16, c18, c19), f5(c20, c20, c22, c23);
    const vec4 v0(m[1][0], m[0][0], m[0][0], m[0][0]), v1(m[1][1], m[0][1], m[0][1], m[0][1]);
    const vec4 v2(m[1][2], m[0][2], m[0][2], m[0][2]), v3(m[1][3], m[0][3], m[0][3], m[0][3]);
    const vec4 i0(v1 * f0 - v2 * f1 + v3 * f2), i1(v0 * f0 - v2 * f3 + v3 * f4);
    const vec4 i2(v0 * f1 - v1 * f3 + v3 * f5), i3(v0 * f2 - v1 * f4 + v2 * f5);
    const vec4 sa(+1, -1, +1, -1), sb(-1, +1, -1, +1);
    const mat4 inv(i0 * sa, i1 * sb, i2 * sa, i3 * sb);
    const vec4 row0(inv[0][0], inv[1][0], inv[2][0], inv[3][0]);
    const vec4 d0(m[0] * row0);
    const float d1 = (d0.x + d0.y) + (d0.z + d0.w);
    const float one_over_det = 1.0f / d1;
    return mat4(inv[0] * one_over_det, inv[1] * one_over_det, inv[2] * one_over_det, inv[3] * one_over_det);
}

// glm::quat_cast(mat3) (gtc/quaternion.inl): the largest of w, x, y, z picks the branch.
inline quat quat_cast(const mat3& m) {
    const float fourXSquaredMinus1 = m[0][0] - m[1][1] - m[2][2];
    const float fourYSquaredMinus1 = m[1][1] - m[0][0] - m[2][2];
    const float fourZSquaredMinus1 = m[2][2] - m[0][0] - m[1][1];
    const float fourWSquaredMinus1 = m[0][0] + m[1][1] + m[2][2];
    int biggestIndex = 0;
    float fourBiggestSquaredMinus1 = fourWSquaredMinus1;
    if (fourXSquaredMinus1 > fourBiggestSquaredMinus1) {
        fourBiggestSquaredMinus1 = fourXSquaredMinus1;
        biggestIndex = 1;
    }
    if (fourYSquaredMinus1 > fourBiggestSquaredMinus1) {
        fourBiggestSquaredMinus1 = fourYSquaredMinus1;
        biggestIndex = 2;
    }
    if (fourZSquaredMinus1 > fourBiggestSquaredMinus1) {
        fourBiggestSquaredMinus1 = fourZSquaredMinus1;
        biggestIndex = 3;
    }
    const float biggestVal = std::sqrt(fourBiggestSquaredMinus1 + 1.0f) * 0.5f;
    const float mult = 0.25f / biggestVal;
    quat q;
    switch (biggestIndex) {
        case 0:
            q.w = biggestVal;
            q.x = (m[1][2] - m[2][1]) * mult;
            q.y = (m[2][0] - m[0][2]) * mult;
            q.z = (m[0][1] - m[1][0]) * mult;
            break;
        case 1:
            q.w = (m[1][2] - m[2][1]) * mult;
            q.x = biggestVal;
            q.y = (m[0][1] + m[1][0]) * mult;
            q.z = (m[2][0] + m[0][2]) * mult;
            break;
        case 2:
            q.w = (m[2][0] - m[0][2]) * mult;
            q.x = (m[0][1] + m[1][0]) * mult;
            q.y = biggestVal;
            q.z = (m[1][2] + m[2][1]) * mult;
            break;
        default:
            q.w = (m[0][1] - m[1][0]) * mult;
            q.x = (m[2][0] + m[0][2]) * mult;
            q.y = (m[1][2] + m[2][1]) * mult;
            q.z = biggestVal;
            break;
    }
    return q;
}

}  // namespace gm
