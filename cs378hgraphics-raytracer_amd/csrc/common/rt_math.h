// rt_math.h — FP64 vector math shared by the host loader and the gfx950 kernels.
//
// Every operation reproduces the evaluation order of glm 0.9.8.4 (the version
// pinned at ray/cmake/glm.cmake:11,15 of the reference), because hit indices
// must be bit-exact against the CPU restatement:
//   dot(a,b)      = (a.x*b.x + a.y*b.y) + a.z*b.z        (glm compute_dot)
//   length(v)     = sqrt(dot(v,v))
//   normalize(v)  = v * (1.0 / sqrt(dot(v,v)))            (glm inversesqrt)
//   distance(a,b) = length(b - a)
//   min/max       = (y < x) ? y : x  /  (x < y) ? y : x   (glm func_common)
//   clamp(x,l,h)  = min(max(x,l),h)
//   mat4*vec4     = (c0*x + c1*y) + (c2*z + c3*w)         (glm type_mat4x4.inl)
//   mat3*vec3     = row r: (m[0][r]*x + m[1][r]*y) + m[2][r]*z
// Everything must be compiled with -ffp-contract=off (host and device).
#pragma once

#include <math.h>
#include <stdint.h>

#include "rt_types.h"

namespace rtm {

RT_HD dvec3 splat3(double s) { return mk3(s, s, s); }

RT_HD double get(const dvec3& v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
RT_HD void set(dvec3& v, int i, double s) {
  if (i == 0) v.x = s; else if (i == 1) v.y = s; else v.z = s;
}

RT_HD dvec3 operator+(const dvec3& a, const dvec3& b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD dvec3 operator-(const dvec3& a, const dvec3& b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD dvec3 operator*(const dvec3& a, const dvec3& b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD dvec3 operator*(const dvec3& a, double s) { return mk3(a.x * s, a.y * s, a.z * s); }
RT_HD dvec3 operator*(double s, const dvec3& a) { return mk3(s * a.x, s * a.y, s * a.z); }
RT_HD dvec3 operator/(const dvec3& a, double s) { return mk3(a.x / s, a.y / s, a.z / s); }
RT_HD dvec3 operator-(const dvec3& a) { return mk3(-a.x, -a.y, -a.z); }
RT_HD dvec3& operator+=(dvec3& a, const dvec3& b) { a.x += b.x; a.y += b.y; a.z += b.z; return a; }
RT_HD dvec3& operator*=(dvec3& a, const dvec3& b) { a.x *= b.x; a.y *= b.y; a.z *= b.z; return a; }
RT_HD dvec3& operator*=(dvec3& a, double s) { a.x *= s; a.y *= s; a.z *= s; return a; }

RT_HD double dot(const dvec3& a, const dvec3& b) {
  double tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
  return (tx + ty) + tz;
}
RT_HD dvec3 cross(const dvec3& x, const dvec3& y) {
  return mk3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
RT_HD double length(const dvec3& v) { return sqrt(dot(v, v)); }
RT_HD dvec3 normalize(const dvec3& v) {
  double inv = 1.0 / sqrt(dot(v, v));
  return v * inv;
}
RT_HD double distance(const dvec3& p0, const dvec3& p1) { return length(p1 - p0); }

RT_HD double gmin(double x, double y) { return (y < x) ? y : x; }
RT_HD double gmax(double x, double y) { return (x < y) ? y : x; }
RT_HD double gclamp(double x, double lo, double hi) { return gmin(gmax(x, lo), hi); }
// setPixel's (int)(255 * c) (RayTracer.cpp:388-394) for c in [0, 1] or NaN
// (glm::clamp passes NaN through): x86 cvttsd2si turns NaN into INT_MIN,
// whose low byte is 0; both paths write that 0 explicitly.
RT_HD uint8_t to_byte(double c) { return (c != c) ? uint8_t(0) : uint8_t(int(255.0 * c)); }
RT_HD dvec3 gclamp3(const dvec3& v, double lo, double hi) {
  return mk3(gclamp(v.x, lo, hi), gclamp(v.y, lo, hi), gclamp(v.z, lo, hi));
}
RT_HD dvec3 gmin3(const dvec3& a, const dvec3& b) { return mk3(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
RT_HD dvec3 gmax3(const dvec3& a, const dvec3& b) { return mk3(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }

// Scalar pow.  On the device it is an out-of-line call: the FP64 pow of the
// device math library is long, and three inlined copies interleaved by the
// scheduler dominated the register peak of the shading kernel.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __attribute__((noinline)) inline double rpow(double b, double e) { return ::pow(b, e); }
#elif defined(__HIPCC__)
__host__ inline double rpow(double b, double e) { return ::pow(b, e); }
#else
inline double rpow(double b, double e) { return pow(b, e); }
#endif

// glm::pow(dvec3, dvec3(s)) — componentwise std::pow.
RT_HD dvec3 pow3(const dvec3& b, double e) { return mk3(rpow(b.x, e), rpow(b.y, e), rpow(b.z, e)); }

// ray::at (scene/ray.h:40): p + (t * d)
RT_HD dvec3 ray_at(const dvec3& p, const dvec3& d, double t) { return p + (t * d); }

// Affine transform with glm mat4*vec4 pairing, w = 1 (scene.h:57-62).
// m is column-major: m[c*3 + r] for columns c = 0..3 and rows r = 0..2.
RT_HD dvec3 xform_point(const double* m, const dvec3& v) {
  dvec3 r;
  // component r: (m0r*x + m1r*y) + (m2r*z + m3r*1)
  r.x = (m[0] * v.x + m[3] * v.y) + (m[6] * v.z + m[9] * 1.0);
  r.y = (m[1] * v.x + m[4] * v.y) + (m[7] * v.z + m[10] * 1.0);
  r.z = (m[2] * v.x + m[5] * v.y) + (m[8] * v.z + m[11] * 1.0);
  return r;
}

// glm mat3*vec3, column-major m[c*3 + r].
RT_HD dvec3 mat3_mul(const double* m, const dvec3& v) {
  dvec3 r;
  r.x = (m[0] * v.x + m[3] * v.y) + m[6] * v.z;
  r.y = (m[1] * v.x + m[4] * v.y) + m[7] * v.z;
  r.z = (m[2] * v.x + m[5] * v.y) + m[8] * v.z;
  return r;
}

}  // namespace rtm
