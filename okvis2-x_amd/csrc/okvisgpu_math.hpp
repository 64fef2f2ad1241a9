// okvisgpu_math.hpp — FP64 small-matrix / quaternion / camera helpers for the HIP kernels
// (and the host-side synthetic generator). Register-resident, fully unrolled.
//
// Conventions follow the reference's Eigen usage: quaternion coefficients (x, y, z, w), Hamilton
// product, Eigen::QuaternionBase::toRotationMatrix(). Formulas cite the okvis source they restate.
#pragma once
#include <cfloat>

#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

#define OKG_HD __host__ __device__ __forceinline__

namespace okg {

// Pointers loaded from the device descriptor are generic (flat) to the compiler; re-qualifying
// them as global lets it emit global_load (vmcnt only) and batch independent loads.
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
using gptr = const __attribute__((address_space(1))) T*;
#else
template <typename T>
using gptr = const T*;
#endif
template <typename T>
__device__ __forceinline__ gptr<T> gmem(const T* p) {
  return (gptr<T>)p;
}
// Writable global pointer (global_store: counts in vmcnt only; a flat store also counts in
// lgkmcnt, so every LDS wait would wait for it too).
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
using gwptr = __attribute__((address_space(1))) T*;
#else
template <typename T>
using gwptr = T*;
#endif
template <typename T>
__device__ __forceinline__ gwptr<T> gmemw(T* p) {
  return (gwptr<T>)p;
}

// One of two buffer pointers (parameter set / linearisation buffer xcur, lcur) picked by a loaded
// flag. The pointers are made opaque first: otherwise the select of P.x[0] / P.x[1] is folded into
// an indexed load P.x[flag], one more dependent load before the data.
template <typename T>
__device__ __forceinline__ T* pick2(int flag, T* p0, T* p1) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+s"(p0));
  asm("" : "+s"(p1));
#endif
  return flag ? p1 : p0;
}

// Workgroup barrier that orders LDS only: __syncthreads() also waits for every outstanding global
// load (vmcnt(0)), which defeats loads prefetched across the barrier.
__device__ __forceinline__ void ldsBarrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct Q {
  double x, y, z, w;
};

OKG_HD Q qmul(const Q& a, const Q& b) {
  return Q{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
           a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
OKG_HD Q qnormalize(const Q& q) {
  const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return Q{q.x / n, q.y / n, q.z / n, q.w / n};
}
OKG_HD Q qinv(const Q& q) {  // Eigen Quaternion::inverse (conjugate / squared norm)
  const double n2 = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
  return Q{-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
}
// Eigen toRotationMatrix; R row-major [9]
OKG_HD void qrot(const Q& q, double R[9]) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
// okvis::kinematics::plus(q) (operators.hpp:64-76), 4x4 row-major
OKG_HD void qplusM(const Q& q, double M[16]) {
  M[0] = q.w;  M[1] = -q.z; M[2] = q.y;   M[3] = q.x;
  M[4] = q.z;  M[5] = q.w;  M[6] = -q.x;  M[7] = q.y;
  M[8] = -q.y; M[9] = q.x;  M[10] = q.w;  M[11] = q.z;
  M[12] = -q.x; M[13] = -q.y; M[14] = -q.z; M[15] = q.w;
}
// okvis::kinematics::oplus(q) (operators.hpp:78-90)
OKG_HD void qoplusM(const Q& q, double M[16]) {
  M[0] = q.w;  M[1] = q.z;  M[2] = -q.y;  M[3] = q.x;
  M[4] = -q.z; M[5] = q.w;  M[6] = q.x;   M[7] = q.y;
  M[8] = q.y;  M[9] = -q.x; M[10] = q.w;  M[11] = q.z;
  M[12] = -q.x; M[13] = -q.y; M[14] = -q.z; M[15] = q.w;
}

// kinematics::sinc / ode::sinc (Transformation.hpp:30-43, ode.hpp:34-46)
OKG_HD double sinc(double x) {
  if (fabs(x) > 1.0e-6) return sin(x) / x;
  const double x_2 = x * x, x_4 = x_2 * x_2, x_6 = x_2 * x_2 * x_2;
  return 1.0 - (1.0 / 6.0) * x_2 + (1.0 / 120.0) * x_4 - (1.0 / 5040.0) * x_6;
}
// kinematics::deltaQ (Transformation.hpp:45-52)
OKG_HD Q deltaQ(double a0, double a1, double a2) {
  const double halfnorm = 0.5 * sqrt(a0 * a0 + a1 * a1 + a2 * a2);
  const double s = sinc(halfnorm) * 0.5;
  return Q{s * a0, s * a1, s * a2, cos(halfnorm)};
}

// 3x3 row-major helpers
OKG_HD void mm3(const double A[9], const double B[9], double C[9]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) C[r * 3 + c] = A[r * 3 + 0] * B[0 * 3 + c] + A[r * 3 + 1] * B[1 * 3 + c] + A[r * 3 + 2] * B[2 * 3 + c];
}
OKG_HD void mv3(const double A[9], const double v[3], double o[3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r) o[r] = A[r * 3 + 0] * v[0] + A[r * 3 + 1] * v[1] + A[r * 3 + 2] * v[2];
}
OKG_HD void mtv3(const double A[9], const double v[3], double o[3]) {  // A^T v
#pragma unroll
  for (int r = 0; r < 3; ++r) o[r] = A[0 * 3 + r] * v[0] + A[1 * 3 + r] * v[1] + A[2 * 3 + r] * v[2];
}
OKG_HD void crossMx(const double v[3], double C[9]) {
  C[0] = 0.0;   C[1] = -v[2]; C[2] = v[1];
  C[3] = v[2];  C[4] = 0.0;   C[5] = -v[0];
  C[6] = -v[1]; C[7] = v[0];  C[8] = 0.0;
}
// kinematics::rightJacobian (Transformation.hpp:55-67)
OKG_HD void rightJacobian(const double p[3], double J[9]) {
  const double Phi = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
  double X[9], X2[9];
  crossMx(p, X);
  mm3(X, X, X2);
  double a, b;
  if (Phi < 1.0e-4) {
    a = -0.5;
    b = 1.0 / 6.0;
  } else {
    const double Phi2 = Phi * Phi, Phi3 = Phi2 * Phi;
    a = -(1.0 - cos(Phi)) / Phi2;
    b = (Phi - sin(Phi)) / Phi3;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) J[i] = a * X[i] + b * X2[i];
  J[0] += 1.0; J[4] += 1.0; J[8] += 1.0;
}

// rightJacobian with sin / cos of Phi from sin / cos of Phi / 2 (one sincos per IMU step, shared
// with dq = exp(w dt / 2)): 1 - cos Phi = 2 sin^2(Phi/2) and sin Phi = 2 sin(Phi/2) cos(Phi/2), equal
// to the reference's a, b up to rounding (the form above loses ~1e-10 of a to cancellation at the
// small angles of one IMU step; either way a few 1e-16 of J).
OKG_HD void rightJacobianHalf(const double p[3], double sh, double ch, double J[9]) {
  const double Phi = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
  double X[9], X2[9];
  crossMx(p, X);
  mm3(X, X, X2);
  double a, b;
  if (Phi < 1.0e-4) {
    a = -0.5;
    b = 1.0 / 6.0;
  } else {
    const double Phi2 = Phi * Phi, Phi3 = Phi2 * Phi;
    a = -(2.0 * sh * sh) / Phi2;
    b = (Phi - 2.0 * sh * ch) / Phi3;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) J[i] = a * X[i] + b * X2[i];
  J[0] += 1.0; J[4] += 1.0; J[8] += 1.0;
}

// okvis::Duration::toSec of a signed nanosecond difference (Duration.hpp:107-109)
OKG_HD double durToSec(int64_t dns) {
  // sec = 0 for [0, 1 s): the same double as (double)0 + 1e-9 * nsec, without the 64-bit division
  if (dns >= 0 && dns < 1000000000LL) return 1e-9 * (double)dns;
  int64_t sec = dns / 1000000000LL;
  int64_t nsec = dns % 1000000000LL;
  if (nsec < 0) { nsec += 1000000000LL; sec -= 1; }
  return (double)sec + 1e-9 * (double)nsec;
}

// ------------------------------------------------------------------ camera (okvis_cv)
struct Cam {
  int dist;
  double fu, fv, cu, cv;
  double d0, d1, d2, d3, d4, d5, d6, d7;
};
// [dist, fu, fv, cu, cv, d0..d7] (DevProblem::cam)
OKG_HD Cam loadCam(const double* c) {
  return Cam{(int)c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[11], c[12]};
}

// distortion_.distort (RadialTangentialDistortion.hpp:89-137, EquidistantDistortion.hpp:87-188)
OKG_HD void distort(const Cam& c, double u0, double u1, double& o0, double& o1, double Jd[4], bool wantJ) {
  if (c.dist == 1) {
    const double k1 = c.d0, k2 = c.d1, p1 = c.d2, p2 = c.d3;
    const double mx_u = u0 * u0, my_u = u1 * u1, mxy_u = u0 * u1;
    const double rho_u = mx_u + my_u;
    const double rad = k1 * rho_u + k2 * rho_u * rho_u;
    o0 = u0 + u0 * rad + 2.0 * p1 * mxy_u + p2 * (rho_u + 2.0 * mx_u);
    o1 = u1 + u1 * rad + 2.0 * p2 * mxy_u + p1 * (rho_u + 2.0 * my_u);
    if (wantJ) {
      Jd[0] = 1 + rad + k1 * 2.0 * mx_u + k2 * rho_u * 4 * mx_u + 2.0 * p1 * u1 + 6 * p2 * u0;
      Jd[2] = k1 * 2.0 * u0 * u1 + k2 * 4 * rho_u * u0 * u1 + p1 * 2.0 * u0 + 2.0 * p2 * u1;
      Jd[1] = Jd[2];
      Jd[3] = 1 + rad + k1 * 2.0 * my_u + k2 * rho_u * 4 * my_u + 6 * p1 * u1 + 2.0 * p2 * u0;
    }
  } else if (c.dist == 3) {
    // RadialTangentialDistortion8 (k1 k2 p1 p2 k3 k4 k5 k6): rational radial model. The reference
    // returns false for rho > 9 and then reads uninitialised outputs; the model is evaluated there.
    const double k1 = c.d0, k2 = c.d1, p1 = c.d2, p2 = c.d3, k3 = c.d4, k4 = c.d5, k5 = c.d6, k6 = c.d7;
    const double mx_u = u0 * u0, my_u = u1 * u1, mxy_u = u0 * u1;
    const double rho_u = mx_u + my_u;
    const double num = 1.0 + ((k3 * rho_u + k2) * rho_u + k1) * rho_u;
    const double den = 1.0 + ((k6 * rho_u + k5) * rho_u + k4) * rho_u;
    const double rad = num / den;
    o0 = u0 * rad + 2.0 * p1 * mxy_u + p2 * (rho_u + 2.0 * mx_u);
    o1 = u1 * rad + 2.0 * p2 * mxy_u + p1 * (rho_u + 2.0 * my_u);
    if (wantJ) {
      // d rad / d rho = (num' den - num den') / den^2, d rho / du = 2u
      const double dnum = k1 + rho_u * (2.0 * k2 + 3.0 * k3 * rho_u);
      const double dden = k4 + rho_u * (2.0 * k5 + 3.0 * k6 * rho_u);
      const double drad = (dnum * den - num * dden) / (den * den);
      Jd[0] = rad + 2.0 * mx_u * drad + 2.0 * p1 * u1 + 6.0 * p2 * u0;
      Jd[1] = 2.0 * mxy_u * drad + 2.0 * p1 * u0 + 2.0 * p2 * u1;
      Jd[2] = Jd[1];
      Jd[3] = rad + 2.0 * my_u * drad + 6.0 * p1 * u1 + 2.0 * p2 * u0;
    }
  } else if (c.dist == 2) {
    const double k1 = c.d0, k2 = c.d1, k3 = c.d2, k4 = c.d3;
    const double r2 = u0 * u0 + u1 * u1;
    const double r = sqrt(r2);
    const double th = atan(r);
    const double th2 = th * th, th4 = th2 * th2, th6 = th4 * th2, th8 = th4 * th4;
    const double poly = 1.0 + k1 * th2 + k2 * th4 + k3 * th6 + k4 * th8;
    const double thd = th * poly;
    const double s = (r > 1e-8) ? thd / r : 1.0;
    o0 = s * u0;
    o1 = s * u1;
    if (wantJ) {
      if (r > 1e-8) {
        // d(s*u)/du = s I + u (ds/dr) u^T / r ; ds/dr = (dthd/dth * dth/dr * r - thd) / r^2
        const double dpoly = 2.0 * k1 * th + 4.0 * k2 * th2 * th + 6.0 * k3 * th4 * th + 8.0 * k4 * th6 * th;
        const double dthd = poly + th * dpoly;
        const double dth_dr = 1.0 / (1.0 + r2);
        const double ds = (dthd * dth_dr * r - thd) / r2;
        const double f = ds / r;
        Jd[0] = s + f * u0 * u0;
        Jd[1] = f * u0 * u1;
        Jd[2] = Jd[1];
        Jd[3] = s + f * u1 * u1;
      } else {
        Jd[0] = 1; Jd[1] = 0; Jd[2] = 0; Jd[3] = 1;
      }
    }
  } else {
    o0 = u0;
    o1 = u1;
    if (wantJ) { Jd[0] = 1; Jd[1] = 0; Jd[2] = 0; Jd[3] = 1; }
  }
}

// PinholeCamera::projectHomogeneous (PinholeCamera.hpp:497-518) -> project (:288-366).
// J: 2x3 point Jacobian (the 4th homogeneous column is zero). kp/J = 0 when |z| < 1e-12.
OKG_HD void projectHomogeneous(const Cam& c, double x, double y, double z, double w, double kp[2],
                               double J[6], bool wantJ) {
  if (w < 0) { x = -x; y = -y; z = -z; }
  if (fabs(z) < 1.0e-12) {
    kp[0] = kp[1] = 0.0;
    if (wantJ) for (int i = 0; i < 6; ++i) J[i] = 0.0;
    return;
  }
  const double rz = 1.0 / z;
  const double rz2 = rz * rz;
  double d0, d1, Jd[4];
  distort(c, x * rz, y * rz, d0, d1, Jd, wantJ);
  if (wantJ) {
    J[0] = c.fu * Jd[0] * rz;
    J[1] = c.fu * Jd[1] * rz;
    J[2] = -c.fu * (x * Jd[0] + y * Jd[1]) * rz2;
    J[3] = c.fv * Jd[2] * rz;
    J[4] = c.fv * Jd[3] * rz;
    J[5] = -c.fv * (x * Jd[2] + y * Jd[3]) * rz2;
  }
  kp[0] = c.fu * d0 + c.cu;
  kp[1] = c.fv * d1 + c.cv;
}

// Minimal reprojection Jacobians from the stored linearisation (ReprojectionError.hpp:71-220 in the
// fused form): with A = L Jh C_CW (2x3, Cauchy-scaled) and p = hp_W.xyz - t_WS w at the
// linearisation point, J_pose = [w A, -A [p]x] (2x6) and J_landmark = -A (2x3).
OKG_HD void obsJacobians(const double A[6], const double p[3], double w, double Jp[12], double Jl[6]) {
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const double a0 = A[r * 3 + 0], a1 = A[r * 3 + 1], a2 = A[r * 3 + 2];
    Jp[r * 6 + 0] = w * a0;
    Jp[r * 6 + 1] = w * a1;
    Jp[r * 6 + 2] = w * a2;
    Jp[r * 6 + 3] = -(a1 * p[2] - a2 * p[1]);
    Jp[r * 6 + 4] = -(a2 * p[0] - a0 * p[2]);
    Jp[r * 6 + 5] = -(a0 * p[1] - a1 * p[0]);
    Jl[r * 3 + 0] = -a0;
    Jl[r * 3 + 1] = -a1;
    Jl[r * 3 + 2] = -a2;
  }
}

// Minimal Jacobian of the weighted reprojection residual w.r.t. the extrinsics T_SC
// (implementation/ReprojectionError.hpp:186-214): J2 = Jh_w [C_CS w, -C_CS [p_S]x] with
// Jh_w C_CS = A C_WS, p_S = C_SW p - t_SC w (p = hp.xyz - t_WS w); A as stored (Cauchy-scaled).
OKG_HD void extrJacobian(const double A[6], const double C_WS[9], const double p[3], double w, const double* ex,
                         double Je[12]) {
  double pS[3];
  mtv3(C_WS, p, pS);
  pS[0] -= ex[0] * w;
  pS[1] -= ex[1] * w;
  pS[2] -= ex[2] * w;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    // b = (A C_WS) row r
    const double b0 = A[r * 3 + 0] * C_WS[0] + A[r * 3 + 1] * C_WS[3] + A[r * 3 + 2] * C_WS[6];
    const double b1 = A[r * 3 + 0] * C_WS[1] + A[r * 3 + 1] * C_WS[4] + A[r * 3 + 2] * C_WS[7];
    const double b2 = A[r * 3 + 0] * C_WS[2] + A[r * 3 + 1] * C_WS[5] + A[r * 3 + 2] * C_WS[8];
    Je[r * 6 + 0] = w * b0;
    Je[r * 6 + 1] = w * b1;
    Je[r * 6 + 2] = w * b2;
    Je[r * 6 + 3] = -(b1 * pS[2] - b2 * pS[1]);
    Je[r * 6 + 4] = -(b2 * pS[0] - b0 * pS[2]);
    Je[r * 6 + 5] = -(b0 * pS[1] - b1 * pS[0]);
  }
}

// ReprojectionError<G>::EvaluateWithMinimalJacobians in the factored form
// (implementation/ReprojectionError.hpp:71-220): weighted residual r = L (meas - kp) (no loss) and
// A = L Jh C_CS C_SW (2x3), so that J_pose = [w A, -A [p]x] and J_landmark = -A (obsJacobians)
// with p = hp.xyz - t_WS w returned in p.
OKG_HD void reprojectA(const Cam& cam, const double* pose, const double* hp, const double* ex, const double* L,
                       const double* meas, double r[2], double A[6], double p[3]) {
  double C_WS[9], C_SC[9];
  qrot(qnormalize(Q{pose[3], pose[4], pose[5], pose[6]}), C_WS);
  qrot(qnormalize(Q{ex[3], ex[4], ex[5], ex[6]}), C_SC);
  const double w4 = hp[3];
  p[0] = hp[0] - pose[0] * w4;
  p[1] = hp[1] - pose[1] * w4;
  p[2] = hp[2] - pose[2] * w4;
  double hS[3];
  mtv3(C_WS, p, hS);
  const double q3[3] = {hS[0] - ex[0] * w4, hS[1] - ex[1] * w4, hS[2] - ex[2] * w4};
  double hC[3];
  mtv3(C_SC, q3, hC);
  double kp[2], Jh[6];
  projectHomogeneous(cam, hC[0], hC[1], hC[2], w4, kp, Jh, true);
  const double e0 = meas[0] - kp[0], e1 = meas[1] - kp[1];
  r[0] = L[0] * e0 + L[1] * e1;
  r[1] = L[2] * e0 + L[3] * e1;
  double Jw[6], B[6];
  for (int c = 0; c < 3; ++c) {
    Jw[c] = L[0] * Jh[c] + L[1] * Jh[3 + c];
    Jw[3 + c] = L[2] * Jh[c] + L[3] * Jh[3 + c];
  }
  for (int rr = 0; rr < 2; ++rr)
    for (int k = 0; k < 3; ++k)
      B[rr * 3 + k] = Jw[rr * 3 + 0] * C_SC[k * 3 + 0] + Jw[rr * 3 + 1] * C_SC[k * 3 + 1] + Jw[rr * 3 + 2] * C_SC[k * 3 + 2];
  for (int rr = 0; rr < 2; ++rr)
    for (int c = 0; c < 3; ++c)
      A[rr * 3 + c] = B[rr * 3 + 0] * C_WS[c * 3 + 0] + B[rr * 3 + 1] * C_WS[c * 3 + 1] + B[rr * 3 + 2] * C_WS[c * 3 + 2];
}

// ReprojectionError<G>::EvaluateWithMinimalJacobians + the Cauchy(1) corrector in the fused form of
// the device (implementation/ReprojectionError.hpp:71-220, ViGraph.cpp:235,338): residual r = L (m -
// kp) and, with wantA, A = L Jh C_CS C_SW (2x3), both scaled by the corrector's sqrt(rho'), and the
// robustified cost. C_WS = R(q_WS) of the pose (formed once per pose by the callers), ex = T_SC.
// (k_eval_obs; without wantA only r and the cost.)
OKG_HD void obsCore(const Cam& cam, const double L[4], const double m[2], const double* pose, const double C_WS[9],
                    const double hp[4], const double ex[7], bool loss, bool wantA, double r[2], double A[6],
                    double& cost) {
  double C_SC[9];
  qrot(qnormalize(Q{ex[3], ex[4], ex[5], ex[6]}), C_SC);
  const double w4 = hp[3];
  // p = hp_W.xyz - t_WS w ; hp_S = C_SW p ; hp_C = C_CS (hp_S - t_SC w)
  const double p[3] = {hp[0] - pose[0] * w4, hp[1] - pose[1] * w4, hp[2] - pose[2] * w4};
  double hS[3];
  mtv3(C_WS, p, hS);
  const double q3[3] = {hS[0] - ex[0] * w4, hS[1] - ex[1] * w4, hS[2] - ex[2] * w4};
  double hC[3];
  mtv3(C_SC, q3, hC);
  double kp[2], Jh[6];
  projectHomogeneous(cam, hC[0], hC[1], hC[2], w4, kp, Jh, wantA);
  const double e0 = m[0] - kp[0], e1 = m[1] - kp[1];
  const double r0 = L[0] * e0 + L[1] * e1;
  const double r1 = L[2] * e0 + L[3] * e1;
  // Cauchy(1) corrector (rho'' < 0 branch: scale residual and Jacobian by sqrt(rho'))
  const double sq = r0 * r0 + r1 * r1;
  double sc = 1.0;
  if (loss) {
    const double sum = 1.0 + sq;
    cost = 0.5 * log(sum);
    sc = sqrt(fmax(DBL_MIN, 1.0 / sum));
  } else {
    cost = 0.5 * sq;
  }
  r[0] = r0 * sc;
  r[1] = r1 * sc;
  if (!wantA) return;
  // Jh_w = L Jh (2x3); C_CW = C_SC^T C_WS^T ; A = Jh_w C_CW
  double Jw[6];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    Jw[c] = L[0] * Jh[c] + L[1] * Jh[3 + c];
    Jw[3 + c] = L[2] * Jh[c] + L[3] * Jh[3 + c];
  }
  double B[6];  // Jh_w C_CS = Jh_w C_SC^T : B[r][k] = sum_j Jw[r][j] C_SC[k][j]
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      B[rr * 3 + k] = Jw[rr * 3 + 0] * C_SC[k * 3 + 0] + Jw[rr * 3 + 1] * C_SC[k * 3 + 1] + Jw[rr * 3 + 2] * C_SC[k * 3 + 2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr)  // B C_SW = B C_WS^T : A[r][c] = sum_k B[r][k] C_WS[c][k]
#pragma unroll
    for (int c = 0; c < 3; ++c)
      A[rr * 3 + c] = (B[rr * 3 + 0] * C_WS[c * 3 + 0] + B[rr * 3 + 1] * C_WS[c * 3 + 1] + B[rr * 3 + 2] * C_WS[c * 3 + 2]) * sc;
}

// Symmetric eigen-decomposition A = V diag(lam) V^T by cyclic Jacobi (Eigen's
// SelfAdjointEigenSolver restated; eigenvalues ascending, eigenvector signs arbitrary). A is
// destroyed. N <= 6, one thread.
template <int N>
OKG_HD void jacobiEigenSym(double* A, double lam[N], double V[N * N]) {
  for (int i = 0; i < N * N; ++i) V[i] = (i % (N + 1)) == 0 ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 32; ++sweep) {
    double off = 0.0, dg = 0.0;
    for (int i = 0; i < N; ++i) {
      dg += A[i * N + i] * A[i * N + i];
      for (int j = i + 1; j < N; ++j) off += A[i * N + j] * A[i * N + j];
    }
    if (off <= 1e-36 * dg || off == 0.0) break;
    for (int p = 0; p < N - 1; ++p)
      for (int q = p + 1; q < N; ++q) {
        const double apq = A[p * N + q];
        if (apq == 0.0) continue;
        const double theta = (A[q * N + q] - A[p * N + p]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < N; ++k) {
          const double akp = A[k * N + p], akq = A[k * N + q];
          A[k * N + p] = c * akp - s * akq;
          A[k * N + q] = s * akp + c * akq;
        }
        for (int k = 0; k < N; ++k) {
          const double apk = A[p * N + k], aqk = A[q * N + k];
          A[p * N + k] = c * apk - s * aqk;
          A[q * N + k] = s * apk + c * aqk;
        }
        A[p * N + q] = A[q * N + p] = 0.0;
        for (int k = 0; k < N; ++k) {
          const double vkp = V[k * N + p], vkq = V[k * N + q];
          V[k * N + p] = c * vkp - s * vkq;
          V[k * N + q] = s * vkp + c * vkq;
        }
      }
  }
  for (int i = 0; i < N; ++i) lam[i] = A[i * N + i];
  for (int i = 1; i < N; ++i)  // insertion sort, ascending, columns of V follow
    for (int j = i; j > 0 && lam[j] < lam[j - 1]; --j) {
      const double t = lam[j]; lam[j] = lam[j - 1]; lam[j - 1] = t;
      for (int k = 0; k < N; ++k) {
        const double v = V[k * N + j]; V[k * N + j] = V[k * N + j - 1]; V[k * N + j - 1] = v;
      }
    }
}

}  // namespace okg
