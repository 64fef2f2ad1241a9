// oracle_math.hpp — TEST INFRASTRUCTURE ONLY (parity checker / CPU baseline), never the product.
//
// Small fixed-size FP64 matrices and Eigen-compatible quaternion helpers used by the CPU oracle.
// Written independently of the GPU kernels (which use their own fused arithmetic in
// okvis2-x_amd/csrc/okvisgpu_math.hpp) so that parity compares two separate restatements.
//
// Quaternion conventions follow Eigen as used by the reference: coefficient storage (x, y, z, w),
// Hamilton product, toRotationMatrix() formula of Eigen::QuaternionBase.
#pragma once

#include <cmath>
#include <cstring>
#include <algorithm>

namespace oracle {

template <int R, int C>
struct Mat {
  double a[R * C];
  double& operator()(int r, int c) { return a[r * C + c]; }
  double operator()(int r, int c) const { return a[r * C + c]; }
  static Mat Zero() { Mat m; std::memset(m.a, 0, sizeof(m.a)); return m; }
  static Mat Identity() {
    Mat m = Zero();
    for (int i = 0; i < (R < C ? R : C); ++i) m(i, i) = 1.0;
    return m;
  }
  Mat<C, R> T() const {
    Mat<C, R> t;
    for (int r = 0; r < R; ++r)
      for (int c = 0; c < C; ++c) t(c, r) = (*this)(r, c);
    return t;
  }
  template <int BR, int BC>
  Mat<BR, BC> block(int r0, int c0) const {
    Mat<BR, BC> b;
    for (int r = 0; r < BR; ++r)
      for (int c = 0; c < BC; ++c) b(r, c) = (*this)(r0 + r, c0 + c);
    return b;
  }
  template <int BR, int BC>
  void setBlock(int r0, int c0, const Mat<BR, BC>& b) {
    for (int r = 0; r < BR; ++r)
      for (int c = 0; c < BC; ++c) (*this)(r0 + r, c0 + c) = b(r, c);
  }
  double squaredNorm() const {
    double s = 0;
    for (int i = 0; i < R * C; ++i) s += a[i] * a[i];
    return s;
  }
  double norm() const { return std::sqrt(squaredNorm()); }
};

template <int R, int K, int C>
inline Mat<R, C> operator*(const Mat<R, K>& x, const Mat<K, C>& y) {
  Mat<R, C> z = Mat<R, C>::Zero();
  for (int r = 0; r < R; ++r)
    for (int k = 0; k < K; ++k) {
      const double v = x(r, k);
      for (int c = 0; c < C; ++c) z(r, c) += v * y(k, c);
    }
  return z;
}
template <int R, int C>
inline Mat<R, C> operator+(const Mat<R, C>& x, const Mat<R, C>& y) {
  Mat<R, C> z;
  for (int i = 0; i < R * C; ++i) z.a[i] = x.a[i] + y.a[i];
  return z;
}
template <int R, int C>
inline Mat<R, C> operator-(const Mat<R, C>& x, const Mat<R, C>& y) {
  Mat<R, C> z;
  for (int i = 0; i < R * C; ++i) z.a[i] = x.a[i] - y.a[i];
  return z;
}
template <int R, int C>
inline Mat<R, C> operator-(const Mat<R, C>& x) {
  Mat<R, C> z;
  for (int i = 0; i < R * C; ++i) z.a[i] = -x.a[i];
  return z;
}
template <int R, int C>
inline Mat<R, C> operator*(double s, const Mat<R, C>& x) {
  Mat<R, C> z;
  for (int i = 0; i < R * C; ++i) z.a[i] = s * x.a[i];
  return z;
}
template <int R, int C>
inline Mat<R, C>& operator+=(Mat<R, C>& x, const Mat<R, C>& y) {
  for (int i = 0; i < R * C; ++i) x.a[i] += y.a[i];
  return x;
}

using M3 = Mat<3, 3>;
using V3 = Mat<3, 1>;
using M4 = Mat<4, 4>;
using V4 = Mat<4, 1>;

inline V3 v3(double x, double y, double z) { V3 v; v.a[0] = x; v.a[1] = y; v.a[2] = z; return v; }

inline V3 cross(const V3& a, const V3& b) {
  return v3(a.a[1] * b.a[2] - a.a[2] * b.a[1], a.a[2] * b.a[0] - a.a[0] * b.a[2],
            a.a[0] * b.a[1] - a.a[1] * b.a[0]);
}

// okvis_kinematics/include/okvis/kinematics/operators.hpp:40-60
inline M3 crossMx(double x, double y, double z) {
  M3 C;
  C(0, 0) = 0.0; C(0, 1) = -z;  C(0, 2) = y;
  C(1, 0) = z;   C(1, 1) = 0.0; C(1, 2) = -x;
  C(2, 0) = -y;  C(2, 1) = x;   C(2, 2) = 0.0;
  return C;
}
inline M3 crossMx(const V3& v) { return crossMx(v.a[0], v.a[1], v.a[2]); }

struct Quat {
  double x, y, z, w;
};
inline Quat qmake(double w, double x, double y, double z) { return Quat{x, y, z, w}; }
inline Quat qmul(const Quat& a, const Quat& b) {  // Eigen Hamilton product a*b
  return Quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
              a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
              a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x,
              a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
inline double qnorm(const Quat& q) { return std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w); }
inline Quat qnormalized(const Quat& q) {
  const double n = qnorm(q);
  return Quat{q.x / n, q.y / n, q.z / n, q.w / n};
}
inline Quat qconj(const Quat& q) { return Quat{-q.x, -q.y, -q.z, q.w}; }
inline Quat qinverse(const Quat& q) {  // Eigen: conjugate / squaredNorm
  const double n2 = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
  return Quat{-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
}
inline V3 qvec(const Quat& q) { return v3(q.x, q.y, q.z); }
inline M3 qrot(const Quat& q) {  // Eigen QuaternionBase::toRotationMatrix
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  M3 R;
  R(0, 0) = 1 - (tyy + tzz); R(0, 1) = txy - twz;       R(0, 2) = txz + twy;
  R(1, 0) = txy + twz;       R(1, 1) = 1 - (txx + tzz); R(1, 2) = tyz - twx;
  R(2, 0) = txz - twy;       R(2, 1) = tyz + twx;       R(2, 2) = 1 - (txx + tyy);
  return R;
}

// operators.hpp:64-76: plus(q_AB) with q_AB*q_BC = plus(q_AB)*q_BC.coeffs()
inline M4 qplusMat(const Quat& qq) {
  const double q[4] = {qq.x, qq.y, qq.z, qq.w};
  M4 Q;
  Q(0,0) =  q[3]; Q(0,1) = -q[2]; Q(0,2) =  q[1]; Q(0,3) =  q[0];
  Q(1,0) =  q[2]; Q(1,1) =  q[3]; Q(1,2) = -q[0]; Q(1,3) =  q[1];
  Q(2,0) = -q[1]; Q(2,1) =  q[0]; Q(2,2) =  q[3]; Q(2,3) =  q[2];
  Q(3,0) = -q[0]; Q(3,1) = -q[1]; Q(3,2) = -q[2]; Q(3,3) =  q[3];
  return Q;
}
// operators.hpp:78-90: oplus(q_BC) with q_AB*q_BC = oplus(q_BC)*q_AB.coeffs()
inline M4 qoplusMat(const Quat& qq) {
  const double q[4] = {qq.x, qq.y, qq.z, qq.w};
  M4 Q;
  Q(0,0) =  q[3]; Q(0,1) =  q[2]; Q(0,2) = -q[1]; Q(0,3) =  q[0];
  Q(1,0) = -q[2]; Q(1,1) =  q[3]; Q(1,2) =  q[0]; Q(1,3) =  q[1];
  Q(2,0) =  q[1]; Q(2,1) = -q[0]; Q(2,2) =  q[3]; Q(2,3) =  q[2];
  Q(3,0) = -q[0]; Q(3,1) = -q[1]; Q(3,2) = -q[2]; Q(3,3) =  q[3];
  return Q;
}

// okvis_kinematics/include/okvis/kinematics/implementation/Transformation.hpp:30-43
inline double sinc(double x) {
  if (std::fabs(x) > 1.0e-6) return std::sin(x) / x;
  const double c_2 = 1.0 / 6.0, c_4 = 1.0 / 120.0, c_6 = 1.0 / 5040.0;
  const double x_2 = x * x, x_4 = x_2 * x_2, x_6 = x_2 * x_2 * x_2;
  return 1.0 - c_2 * x_2 + c_4 * x_4 - c_6 * x_6;
}
// Transformation.hpp:45-52
inline Quat deltaQ(const V3& dAlpha) {
  const double halfnorm = 0.5 * dAlpha.norm();
  const double s = sinc(halfnorm);
  return Quat{s * 0.5 * dAlpha.a[0], s * 0.5 * dAlpha.a[1], s * 0.5 * dAlpha.a[2], std::cos(halfnorm)};
}
// Transformation.hpp:55-67 (Forster et al. RSS 2015 eq. 8)
inline M3 rightJacobian(const V3& PhiVec) {
  const double Phi = PhiVec.norm();
  M3 ret = M3::Identity();
  const M3 Phi_x = crossMx(PhiVec);
  const M3 Phi_x2 = Phi_x * Phi_x;
  if (Phi < 1.0e-4) {
    ret += (-0.5) * Phi_x + (1.0 / 6.0) * Phi_x2;
  } else {
    const double Phi2 = Phi * Phi, Phi3 = Phi2 * Phi;
    ret += (-(1.0 - std::cos(Phi)) / Phi2) * Phi_x + ((Phi - std::sin(Phi)) / Phi3) * Phi_x2;
  }
  return ret;
}

// okvis::Duration::toSec of a signed nanosecond difference: sec/nsec normalised so 0 <= nsec < 1e9
// (okvis_time/include/okvis/Duration.hpp:107-109, normalizeSecNSecSigned).
inline double durToSec(long long dns) {
  long long sec = dns / 1000000000LL;
  long long nsec = dns % 1000000000LL;
  if (nsec < 0) { nsec += 1000000000LL; sec -= 1; }
  return (double)sec + 1e-9 * (double)nsec;
}

}  // namespace oracle
