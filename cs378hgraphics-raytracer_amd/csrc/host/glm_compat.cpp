// glm_compat.cpp — the glm 0.9.8.4 matrix operations the reference uses on
// the host (translate/rotate/scale/transpose/inverse/mat4*mat4), restated
// with glm's evaluation order.  glm is not vendored in the reference
// (ray/cmake/glm.cmake:11,15 clones it), so these follow glm 0.9.8's
// published sources: matrix_transform.inl (translate, rotate, scale),
// func_matrix.inl (compute_inverse for mat3/mat4), type_mat4x4.inl
// (operator* for mat4*mat4 and mat4*vec4).  Used by the .ray loader only;
// CPU oracle and GPU kernels consume the resulting matrices, so CPU/GPU
// parity does not depend on this file.
#include <cmath>

#include "scene_model.h"
#include "../common/rt_math.h"

namespace rtxh {

Mat4 mat4_identity() {
  Mat4 r;
  for (int i = 0; i < 16; ++i) r.m[i] = (i % 5 == 0) ? 1.0 : 0.0;
  return r;
}

Mat3 mat3_identity() {
  Mat3 r;
  for (int i = 0; i < 9; ++i) r.m[i] = (i % 4 == 0) ? 1.0 : 0.0;
  return r;
}

// glm: Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3]
Mat4 mat4_mul(const Mat4& a, const Mat4& b) {
  Mat4 r;
  for (int c = 0; c < 4; ++c) {
    for (int row = 0; row < 4; ++row) {
      double s = a.m[0 * 4 + row] * b.m[c * 4 + 0];
      s = s + a.m[1 * 4 + row] * b.m[c * 4 + 1];
      s = s + a.m[2 * 4 + row] * b.m[c * 4 + 2];
      s = s + a.m[3 * 4 + row] * b.m[c * 4 + 3];
      r.m[c * 4 + row] = s;
    }
  }
  return r;
}

// glm::translate(mat4(1), v): Result[3] = m0*v0 + m1*v1 + m2*v2 + m3
Mat4 mat4_translate(const dvec3& v) {
  Mat4 id = mat4_identity();
  Mat4 r = id;
  for (int row = 0; row < 4; ++row) {
    double s = id.m[0 * 4 + row] * v.x;
    s = s + id.m[1 * 4 + row] * v.y;
    s = s + id.m[2 * 4 + row] * v.z;
    s = s + id.m[3 * 4 + row];
    r.m[3 * 4 + row] = s;
  }
  return r;
}

// glm::scale(mat4(1), v)
Mat4 mat4_scale(const dvec3& v) {
  Mat4 id = mat4_identity();
  Mat4 r;
  for (int row = 0; row < 4; ++row) {
    r.m[0 * 4 + row] = id.m[0 * 4 + row] * v.x;
    r.m[1 * 4 + row] = id.m[1 * 4 + row] * v.y;
    r.m[2 * 4 + row] = id.m[2 * 4 + row] * v.z;
    r.m[3 * 4 + row] = id.m[3 * 4 + row];
  }
  return r;
}

// glm::rotate(angle, axis) = rotate(mat4(1), angle, axis)  (Parser.cpp:287)
Mat4 mat4_rotate(double angle, const dvec3& v) {
  const double a = angle;
  const double c = std::cos(a);
  const double s = std::sin(a);
  dvec3 axis = rtm::normalize(v);
  dvec3 temp = (1.0 - c) * axis;
  double R[3][3];
  R[0][0] = c + temp.x * axis.x;
  R[0][1] = temp.x * axis.y + s * axis.z;
  R[0][2] = temp.x * axis.z - s * axis.y;
  R[1][0] = temp.y * axis.x - s * axis.z;
  R[1][1] = c + temp.y * axis.y;
  R[1][2] = temp.y * axis.z + s * axis.x;
  R[2][0] = temp.z * axis.x + s * axis.y;
  R[2][1] = temp.z * axis.y - s * axis.x;
  R[2][2] = c + temp.z * axis.z;
  Mat4 m = mat4_identity();
  Mat4 r;
  for (int col = 0; col < 3; ++col) {
    for (int row = 0; row < 4; ++row) {
      double acc = m.m[0 * 4 + row] * R[col][0];
      acc = acc + m.m[1 * 4 + row] * R[col][1];
      acc = acc + m.m[2 * 4 + row] * R[col][2];
      r.m[col * 4 + row] = acc;
    }
  }
  for (int row = 0; row < 4; ++row) r.m[3 * 4 + row] = m.m[3 * 4 + row];
  return r;
}

Mat4 mat4_transpose(const Mat4& a) {
  Mat4 r;
  for (int c = 0; c < 4; ++c)
    for (int row = 0; row < 4; ++row) r.m[c * 4 + row] = a.m[row * 4 + c];
  return r;
}

// glm 0.9.8 compute_inverse<tmat4x4> (func_matrix.inl)
Mat4 mat4_inverse(const Mat4& A) {
  auto m = [&](int c, int r) { return A.m[c * 4 + r]; };
  double Coef00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3);
  double Coef02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
  double Coef03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3);
  double Coef04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
  double Coef06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3);
  double Coef07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
  double Coef08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2);
  double Coef10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
  double Coef11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2);
  double Coef12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
  double Coef14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3);
  double Coef15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
  double Coef16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2);
  double Coef18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
  double Coef19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2);
  double Coef20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
  double Coef22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1);
  double Coef23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);

  double Fac0[4] = {Coef00, Coef00, Coef02, Coef03};
  double Fac1[4] = {Coef04, Coef04, Coef06, Coef07};
  double Fac2[4] = {Coef08, Coef08, Coef10, Coef11};
  double Fac3[4] = {Coef12, Coef12, Coef14, Coef15};
  double Fac4[4] = {Coef16, Coef16, Coef18, Coef19};
  double Fac5[4] = {Coef20, Coef20, Coef22, Coef23};

  double Vec0[4] = {m(1, 0), m(0, 0), m(0, 0), m(0, 0)};
  double Vec1[4] = {m(1, 1), m(0, 1), m(0, 1), m(0, 1)};
  double Vec2[4] = {m(1, 2), m(0, 2), m(0, 2), m(0, 2)};
  double Vec3[4] = {m(1, 3), m(0, 3), m(0, 3), m(0, 3)};

  double Inv[4][4];
  for (int k = 0; k < 4; ++k) {
    Inv[0][k] = (Vec1[k] * Fac0[k] - Vec2[k] * Fac1[k]) + Vec3[k] * Fac2[k];
    Inv[1][k] = (Vec0[k] * Fac0[k] - Vec2[k] * Fac3[k]) + Vec3[k] * Fac4[k];
    Inv[2][k] = (Vec0[k] * Fac1[k] - Vec1[k] * Fac3[k]) + Vec3[k] * Fac5[k];
    Inv[3][k] = (Vec0[k] * Fac2[k] - Vec1[k] * Fac4[k]) + Vec2[k] * Fac5[k];
  }
  const double SignA[4] = {+1, -1, +1, -1};
  const double SignB[4] = {-1, +1, -1, +1};
  double Inverse[4][4];
  for (int k = 0; k < 4; ++k) {
    Inverse[0][k] = Inv[0][k] * SignA[k];
    Inverse[1][k] = Inv[1][k] * SignB[k];
    Inverse[2][k] = Inv[2][k] * SignA[k];
    Inverse[3][k] = Inv[3][k] * SignB[k];
  }
  double Row0[4] = {Inverse[0][0], Inverse[1][0], Inverse[2][0], Inverse[3][0]};
  double Dot0[4];
  for (int k = 0; k < 4; ++k) Dot0[k] = m(0, k) * Row0[k];
  double Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
  double OneOverDeterminant = 1.0 / Dot1;
  Mat4 r;
  for (int c = 0; c < 4; ++c)
    for (int row = 0; row < 4; ++row) r.m[c * 4 + row] = Inverse[c][row] * OneOverDeterminant;
  return r;
}

Mat3 mat3_from4(const Mat4& a) {
  Mat3 r;
  for (int c = 0; c < 3; ++c)
    for (int row = 0; row < 3; ++row) r.m[c * 3 + row] = a.m[c * 4 + row];
  return r;
}

// glm 0.9.8 compute_inverse<tmat3x3>
Mat3 mat3_inverse(const Mat3& A) {
  auto m = [&](int c, int r) { return A.m[c * 3 + r]; };
  double OneOverDeterminant =
      1.0 / ((+m(0, 0) * (m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) -
              m(1, 0) * (m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2))) +
             m(2, 0) * (m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2)));
  Mat3 r;
  auto set = [&](int c, int row, double v) { r.m[c * 3 + row] = v; };
  set(0, 0, +(m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) * OneOverDeterminant);
  set(1, 0, -(m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2)) * OneOverDeterminant);
  set(2, 0, +(m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1)) * OneOverDeterminant);
  set(0, 1, -(m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2)) * OneOverDeterminant);
  set(1, 1, +(m(0, 0) * m(2, 2) - m(2, 0) * m(0, 2)) * OneOverDeterminant);
  set(2, 1, -(m(0, 0) * m(2, 1) - m(2, 0) * m(0, 1)) * OneOverDeterminant);
  set(0, 2, +(m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2)) * OneOverDeterminant);
  set(1, 2, -(m(0, 0) * m(1, 2) - m(1, 0) * m(0, 2)) * OneOverDeterminant);
  set(2, 2, +(m(0, 0) * m(1, 1) - m(1, 0) * m(0, 1)) * OneOverDeterminant);
  return r;
}

Mat3 mat3_transpose(const Mat3& a) {
  Mat3 r;
  for (int c = 0; c < 3; ++c)
    for (int row = 0; row < 3; ++row) r.m[c * 3 + row] = a.m[row * 3 + c];
  return r;
}

// glm mat4 * vec4: (c0*x + c1*y) + (c2*z + c3*w)
void mat4_mul_vec4(const Mat4& M, const double v[4], double out[4]) {
  for (int row = 0; row < 4; ++row) {
    double mul0 = M.m[0 * 4 + row] * v[0];
    double mul1 = M.m[1 * 4 + row] * v[1];
    double mul2 = M.m[2 * 4 + row] * v[2];
    double mul3 = M.m[3 * 4 + row] * v[3];
    out[row] = (mul0 + mul1) + (mul2 + mul3);
  }
}

dvec3 mat4_mul_point(const Mat4& M, const dvec3& v) {
  double in[4] = {v.x, v.y, v.z, 1.0};
  double out[4];
  mat4_mul_vec4(M, in, out);
  return dvec3{out[0], out[1], out[2]};
}

// TransformNode ctor (scene/scene.h:119-129)
Transform make_transform(const Transform* parent, const Mat4& local) {
  Transform t;
  t.xform = parent ? mat4_mul(parent->xform, local) : local;
  t.inverse = mat4_inverse(t.xform);
  t.normi = mat3_transpose(mat3_inverse(mat3_from4(t.xform)));
  return t;
}

}  // namespace rtxh
