// glm_restated.h — TEST INFRASTRUCTURE (the CPU oracle's own vector math).
//
// The reference does every vector operation on the hot path through glm
// 0.9.8.4 (g-truc/glm, pinned at ray/cmake/glm.cmake:11,15; not vendored in
// /root/reference, not available offline).  This header restates, for the
// oracle only, the published glm 0.9.8.4 implementation of the operations the
// reference calls (call sites RayTracer.cpp:77,
// scene.h:57-62,127-128, light.cpp:21-73, material.cpp:34-69, camera.cpp:21-31),
// written in glm's own structure — tvec3 component-wise operators, the
// detail::compute_dot / compute_normalize / inversesqrt helpers, the
// column-vector form of tmat4x4 * tvec4 and tmat3x3 * tvec3 — rather than as
// the product's hand-flattened formulas (csrc/common/rt_math.h).  The oracle
// never includes rt_math.h (oracle/Makefile; tests/test_oracle_math.py checks
// the two bit for bit on random and edge inputs), so a slip in the product's
// operation order is visible to the parity tests instead of being shared by
// checker and product.
//
// Only the POD vector types (rt_types.h: x, y, z storage) are shared; every
// operation below is the oracle's.  Compiled with -ffp-contract=off like the
// reference's own flags would need to be for these orders to hold.
#pragma once

#include <cmath>
#include <cstdint>

#include "../cs378hgraphics-raytracer_amd/csrc/common/rt_types.h"

namespace glmr {

using rtm::dvec2;
using rtm::dvec3;

// ---- tvec3<double> component-wise operators (glm/detail/type_vec3.inl:
// operator+(tvec3, tvec3) = tvec3(v1.x + v2.x, v1.y + v2.y, v1.z + v2.z),
// operator*(T, tvec3) = tvec3(s * v.x, ...), operator/(tvec3, T) divides)
inline dvec3 vec3(double x, double y, double z) { return dvec3{x, y, z}; }
inline dvec3 vec3(double s) { return dvec3{s, s, s}; }  // tvec3(T scalar)
inline dvec3 operator+(const dvec3& v1, const dvec3& v2) { return vec3(v1.x + v2.x, v1.y + v2.y, v1.z + v2.z); }
inline dvec3 operator-(const dvec3& v1, const dvec3& v2) { return vec3(v1.x - v2.x, v1.y - v2.y, v1.z - v2.z); }
inline dvec3 operator*(const dvec3& v1, const dvec3& v2) { return vec3(v1.x * v2.x, v1.y * v2.y, v1.z * v2.z); }
inline dvec3 operator*(const dvec3& v, double s) { return vec3(v.x * s, v.y * s, v.z * s); }
inline dvec3 operator*(double s, const dvec3& v) { return vec3(s * v.x, s * v.y, s * v.z); }
inline dvec3 operator/(const dvec3& v, double s) { return vec3(v.x / s, v.y / s, v.z / s); }
inline dvec3 operator-(const dvec3& v) { return vec3(-v.x, -v.y, -v.z); }
inline dvec3& operator+=(dvec3& a, const dvec3& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  return a;
}
inline dvec3& operator*=(dvec3& a, const dvec3& b) {
  a.x *= b.x;
  a.y *= b.y;
  a.z *= b.z;
  return a;
}
inline dvec3& operator*=(dvec3& a, double s) {
  a.x *= s;
  a.y *= s;
  a.z *= s;
  return a;
}

namespace detail {
// glm/detail/func_geometric.inl: compute_dot<tvec3>::call —
//   tvec3<T, P> tmp(a * b); return tmp.x + tmp.y + tmp.z;
inline double compute_dot(const dvec3& a, const dvec3& b) {
  const dvec3 tmp(a * b);
  return tmp.x + tmp.y + tmp.z;
}
// glm/detail/func_exponential.inl: inversesqrt(x) = static_cast<genType>(1) / sqrt(x)
inline double inversesqrt(double x) { return static_cast<double>(1) / std::sqrt(x); }
// compute_normalize::call(v) = v * inversesqrt(dot(v, v))
inline dvec3 compute_normalize(const dvec3& v) { return v * inversesqrt(compute_dot(v, v)); }
}  // namespace detail

inline double dot(const dvec3& x, const dvec3& y) { return detail::compute_dot(x, y); }
// length(v) = sqrt(dot(v, v)) (compute_length)
inline double length(const dvec3& v) { return std::sqrt(dot(v, v)); }
inline dvec3 normalize(const dvec3& x) { return detail::compute_normalize(x); }
// distance(p0, p1) = length(p1 - p0) (compute_distance)
inline double distance(const dvec3& p0, const dvec3& p1) { return length(p1 - p0); }
// cross (func_geometric.inl): tvec3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y)
inline dvec3 cross(const dvec3& x, const dvec3& y) {
  return vec3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}

// func_common.inl: min(x, y) = (y < x) ? y : x, max(x, y) = (x < y) ? y : x,
// clamp(x, lo, hi) = min(max(x, lo), hi) (NaN in x passes through)
inline double min(double x, double y) { return (y < x) ? y : x; }
inline double max(double x, double y) { return (x < y) ? y : x; }
inline double clamp(double x, double lo, double hi) { return min(max(x, lo), hi); }
inline dvec3 min(const dvec3& a, const dvec3& b) { return vec3(min(a.x, b.x), min(a.y, b.y), min(a.z, b.z)); }
inline dvec3 max(const dvec3& a, const dvec3& b) { return vec3(max(a.x, b.x), max(a.y, b.y), max(a.z, b.z)); }
// min / max (tvec3, T): against tvec3(y) (compute_min_vector / compute_max_vector)
inline dvec3 min(const dvec3& x, double y) { return min(x, vec3(y)); }
inline dvec3 max(const dvec3& x, double y) { return max(x, vec3(y)); }
// clamp(tvec3, T, T) = min(max(x, tvec3(lo)), tvec3(hi)) (compute_clamp_vector)
inline dvec3 clamp(const dvec3& x, double lo, double hi) { return min(max(x, vec3(lo)), vec3(hi)); }
// pow(tvec3, tvec3) = component-wise std::pow (func_exponential.inl)
inline dvec3 pow(const dvec3& b, const dvec3& e) { return vec3(std::pow(b.x, e.x), std::pow(b.y, e.y), std::pow(b.z, e.z)); }

// tmat4x4<double> * tvec4<double> (glm/detail/type_mat4x4.inl), the
// column-vector form:  Mov_k = tvec4(v[k]);  Add0 = m[0] * Mov0 + m[1] * Mov1;
// Add1 = m[2] * Mov2 + m[3] * Mov3;  result = Add0 + Add1.  `m` column-major
// m[c * 4 + r] (rtxh::Mat4).
struct dvec4 {
  double x, y, z, w;
};
inline dvec4 operator*(const dvec4& a, const dvec4& b) { return dvec4{a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
inline dvec4 operator+(const dvec4& a, const dvec4& b) { return dvec4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline dvec4 mat4_mul(const double* m, const dvec4& v) {
  const dvec4 col0{m[0], m[1], m[2], m[3]}, col1{m[4], m[5], m[6], m[7]};
  const dvec4 col2{m[8], m[9], m[10], m[11]}, col3{m[12], m[13], m[14], m[15]};
  const dvec4 Mov0{v.x, v.x, v.x, v.x}, Mov1{v.y, v.y, v.y, v.y};
  const dvec4 Mov2{v.z, v.z, v.z, v.z}, Mov3{v.w, v.w, v.w, v.w};
  const dvec4 Mul0 = col0 * Mov0;
  const dvec4 Mul1 = col1 * Mov1;
  const dvec4 Add0 = Mul0 + Mul1;
  const dvec4 Mul2 = col2 * Mov2;
  const dvec4 Mul3 = col3 * Mov3;
  const dvec4 Add1 = Mul2 + Mul3;
  return Add0 + Add1;
}
// operator*(dmat4x4, dvec3) of scene.h:57-62: glm::dvec4(v, 1.0), the
// product, its xyz
inline dvec3 mat4_mul_point(const double* m, const dvec3& v) {
  const dvec4 r = mat4_mul(m, dvec4{v.x, v.y, v.z, 1.0});
  return vec3(r.x, r.y, r.z);
}
// tmat3x3<double> * tvec3<double> (type_mat3x3.inl):
//   tvec3(m[0][0] * v.x + m[1][0] * v.y + m[2][0] * v.z, ...)  — column-major m[c * 3 + r]
inline dvec3 mat3_mul(const double* m, const dvec3& v) {
  return vec3(m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z,
              m[2] * v.x + m[5] * v.y + m[8] * v.z);
}

// (not glm) RayTracer::setPixel (RayTracer.cpp:388-394): pixel[k] =
// (int)(255.0 * c) stored in an unsigned char (the low byte).  c is clamped
// to [0, 1] or NaN (glm::clamp passes NaN through, RayTracer.cpp:77); on
// x86-64 the conversion of NaN (cvttsd2si) gives INT_MIN, whose low byte is 0.
inline uint8_t set_pixel_byte(double c) {
  if (std::isnan(c)) return 0;
  const int v = static_cast<int>(255.0 * c);
  return static_cast<uint8_t>(v & 0xff);
}

}  // namespace glmr
