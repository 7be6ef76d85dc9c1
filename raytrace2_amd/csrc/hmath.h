// hmath.h — host-side float math with the reference's glm semantics.
// Used by the scene loader/compiler and the Camera. Compiled with -ffp-contract=off so every
// operation rounds exactly as the reference's non-FMA x86-64 build.
#pragma once
#include <cfloat>
#include <cmath>

namespace rt2 {

constexpr float kInfinity = FLT_MAX;  // Defs.hpp:17

struct vec3 {
  float x = 0, y = 0, z = 0;
  vec3() = default;
  constexpr vec3(float a, float b, float c) : x(a), y(b), z(c) {}
  explicit constexpr vec3(float s) : x(s), y(s), z(s) {}
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator/(vec3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }
inline float dot(vec3 a, vec3 b) {
  float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
  return (px + py) + pz;
}
inline vec3 cross(vec3 a, vec3 b) {
  return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
inline vec3 normalize(vec3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

struct vec4 {
  float v[4] = {0, 0, 0, 0};
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
};
inline vec4 operator+(const vec4& a, const vec4& b) {
  return {{a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]}};
}
inline vec4 operator-(const vec4& a, const vec4& b) {
  return {{a[0] - b[0], a[1] - b[1], a[2] - b[2], a[3] - b[3]}};
}
inline vec4 operator*(const vec4& a, const vec4& b) {
  return {{a[0] * b[0], a[1] * b[1], a[2] * b[2], a[3] * b[3]}};
}
inline vec4 operator*(const vec4& a, float s) { return {{a[0] * s, a[1] * s, a[2] * s, a[3] * s}}; }

// Column-major 4x4 like glm::mat4: col[c][r].
struct mat4 {
  vec4 col[4];
  static mat4 identity() {
    mat4 m;
    for (int i = 0; i < 4; i++) m.col[i][i] = 1.0f;
    return m;
  }
  vec4& operator[](int c) { return col[c]; }
  const vec4& operator[](int c) const { return col[c]; }
};

// glm mat4 * vec4 = (c0*x + c1*y) + (c2*z + c3*w)
inline vec4 transform4(const mat4& m, const vec4& v) {
  return (m[0] * v[0] + m[1] * v[1]) + (m[2] * v[2] + m[3] * v[3]);
}
inline vec3 transform_point(const mat4& m, vec3 p) {
  vec4 r = transform4(m, vec4{{p.x, p.y, p.z, 1.0f}});
  return {r[0], r[1], r[2]};
}
// glm mat4 * mat4: Result[i] = ((A0*B[i][0] + A1*B[i][1]) + A2*B[i][2]) + A3*B[i][3]
inline mat4 matmul(const mat4& a, const mat4& b) {
  mat4 r;
  for (int i = 0; i < 4; i++) r[i] = ((a[0] * b[i][0] + a[1] * b[i][1]) + a[2] * b[i][2]) + a[3] * b[i][3];
  return r;
}

// glm::inverse for mat4 (cofactor expansion, glm/detail/func_matrix.inl compute_inverse<4,4>)
mat4 inverse(const mat4& m);

}  // namespace rt2
