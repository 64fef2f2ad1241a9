// functors.cpp — TEST INFRASTRUCTURE ONLY (oracle). CPU restatement of the okvis cost functors,
// manifolds and camera projection. Each function cites the reference file:line it follows.
#include "oracle.hpp"

#include <cfloat>
#include <cstdio>

namespace oracle {

// ============================================================ cameras
// RadialTangentialDistortion::distort (RadialTangentialDistortion.hpp:89-137) and
// EquidistantDistortion::distort (EquidistantDistortion.hpp:87-188). NoDistortion: identity.
static void distort(const Camera& cam, double u0, double u1, double out[2], double Jd[4]) {
  if (cam.dist == OKVISGPU_DIST_RADTAN) {
    const double k1 = cam.d[0], k2 = cam.d[1], p1 = cam.d[2], p2 = cam.d[3];
    const double mx_u = u0 * u0, my_u = u1 * u1, mxy_u = u0 * u1;
    const double rho_u = mx_u + my_u;
    const double rad_dist_u = k1 * rho_u + k2 * rho_u * rho_u;
    out[0] = u0 + u0 * rad_dist_u + 2.0 * p1 * mxy_u + p2 * (rho_u + 2.0 * mx_u);
    out[1] = u1 + u1 * rad_dist_u + 2.0 * p2 * mxy_u + p1 * (rho_u + 2.0 * my_u);
    if (Jd) {
      Jd[0] = 1 + rad_dist_u + k1 * 2.0 * mx_u + k2 * rho_u * 4 * mx_u + 2.0 * p1 * u1 + 6 * p2 * u0;
      Jd[2] = k1 * 2.0 * u0 * u1 + k2 * 4 * rho_u * u0 * u1 + p1 * 2.0 * u0 + 2.0 * p2 * u1;
      Jd[1] = Jd[2];
      Jd[3] = 1 + rad_dist_u + k1 * 2.0 * my_u + k2 * rho_u * 4 * my_u + 6 * p1 * u1 + 2.0 * p2 * u0;
    }
  } else if (cam.dist == OKVISGPU_DIST_EQUIDISTANT) {
    const double k1 = cam.d[0], k2 = cam.d[1], k3 = cam.d[2], k4 = cam.d[3];
    const double r = std::sqrt(u0 * u0 + u1 * u1);
    const double theta = std::atan(r);
    const double theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2,
                 theta8 = theta4 * theta4;
    const double thetad = theta * (1.0 + k1 * theta2 + k2 * theta4 + k3 * theta6 + k4 * theta8);
    const double scaling = (r > 1e-8) ? thetad / r : 1.0;
    out[0] = scaling * u0;
    out[1] = scaling * u1;
    if (Jd) {
      if (r > 1e-8) {
        double t2 = u0 * u0, t3 = u1 * u1, t4 = t2 + t3;
        double t6 = std::atan(std::sqrt(t4));
        double t7 = t6 * t6;
        double t8 = 1.0 / std::sqrt(t4);
        double t9 = t7 * t7;
        double t11 = 1.0 / ((t2 + t3) + 1.0);
        double t17 = (((k1 * t7 + k2 * t9) + k3 * t7 * t9) + k4 * (t9 * t9)) + 1.0;
        double t18 = 1.0 / t4;
        double t19 = 1.0 / std::sqrt(t4 * t4 * t4);
        double t20 = t6 * t8 * t17;
        double t25 = ((k2 * t6 * t7 * t8 * t11 * u1 * 4.0 + k3 * t6 * t8 * t9 * t11 * u1 * 6.0) +
                      k4 * t6 * t7 * t8 * t9 * t11 * u1 * 8.0) +
                     k1 * t6 * t8 * t11 * u1 * 2.0;
        t4 = ((k2 * t6 * t7 * t8 * t11 * u0 * 4.0 + k3 * t6 * t8 * t9 * t11 * u0 * 6.0) +
              k4 * t6 * t7 * t8 * t9 * t11 * u0 * 8.0) +
             k1 * t6 * t8 * t11 * u0 * 2.0;
        t7 = t11 * t17 * t18 * u0 * u1;
        Jd[1] = (t7 + t6 * t8 * t25 * u0) - t6 * t17 * t19 * u0 * u1;
        Jd[3] = ((t20 - t3 * t6 * t17 * t19) + t3 * t11 * t17 * t18) + t6 * t8 * t25 * u1;
        Jd[0] = ((t20 - t2 * t6 * t17 * t19) + t2 * t11 * t17 * t18) + t6 * t8 * t4 * u0;
        Jd[2] = (t7 + t6 * t8 * t4 * u1) - t6 * t17 * t19 * u0 * u1;
      } else {
        Jd[0] = 1; Jd[1] = 0; Jd[2] = 0; Jd[3] = 1;
      }
    }
  } else if (cam.dist == OKVISGPU_DIST_RADTAN8) {
    // RadialTangentialDistortion8::distort (RadialTangentialDistortion8.hpp:88-170). The reference
    // returns false for rho > 9 and PinholeCamera::project (PinholeCamera.hpp:311-354) still writes
    // the keypoint from the (then uninitialised) outputs while ReprojectionError ignores the status;
    // here the model is evaluated there too.
    const double k1 = cam.d[0], k2 = cam.d[1], p1 = cam.d[2], p2 = cam.d[3];
    const double k3 = cam.d[4], k4 = cam.d[5], k5 = cam.d[6], k6 = cam.d[7];
    const double mx_u = u0 * u0, my_u = u1 * u1, mxy_u = u0 * u1;
    const double rho_u = mx_u + my_u;
    const double num = rho_u * (k1 + rho_u * (k2 + k3 * rho_u)) + 1.0;
    const double den = rho_u * (k4 + rho_u * (k5 + k6 * rho_u)) + 1.0;
    const double rad = num / den;
    out[0] = u0 * rad + 2.0 * p1 * mxy_u + p2 * (rho_u + 2.0 * mx_u);
    out[1] = u1 * rad + 2.0 * p2 * mxy_u + p1 * (rho_u + 2.0 * my_u);
    if (Jd) {
      // d num / d u_j and d den / d u_j, expanded as in the reference's J(i, j) expressions
      const double dn[2] = {rho_u * (u0 * (k2 + k3 * rho_u) * 2.0 + k3 * u0 * rho_u * 2.0) +
                                u0 * (k1 + rho_u * (k2 + k3 * rho_u)) * 2.0,
                            rho_u * (u1 * (k2 + k3 * rho_u) * 2.0 + k3 * u1 * rho_u * 2.0) +
                                u1 * (k1 + rho_u * (k2 + k3 * rho_u)) * 2.0};
      const double dd[2] = {rho_u * (u0 * (k5 + k6 * rho_u) * 2.0 + k6 * u0 * rho_u * 2.0) +
                                u0 * (k4 + rho_u * (k5 + k6 * rho_u)) * 2.0,
                            rho_u * (u1 * (k5 + k6 * rho_u) * 2.0 + k6 * u1 * rho_u * 2.0) +
                                u1 * (k4 + rho_u * (k5 + k6 * rho_u)) * 2.0};
      const double c2 = den * den;
      Jd[0] = p1 * u1 * 2.0 + p2 * u0 * 6.0 + rad + u0 * dn[0] / den - u0 * dd[0] * num / c2;
      Jd[1] = p1 * u0 * 2.0 + p2 * u1 * 2.0 + u0 * dn[1] / den - u0 * dd[1] * num / c2;
      Jd[2] = p1 * u0 * 2.0 + p2 * u1 * 2.0 + u1 * dn[0] / den - u1 * dd[0] * num / c2;
      Jd[3] = p1 * u1 * 6.0 + p2 * u0 * 2.0 + rad + u1 * dn[1] / den - u1 * dd[1] * num / c2;
    }
  } else {
    out[0] = u0;
    out[1] = u1;
    if (Jd) { Jd[0] = 1; Jd[1] = 0; Jd[2] = 0; Jd[3] = 1; }
  }
}

// PinholeCamera<D>::project (PinholeCamera.hpp:248-285 without, :288-366 with Jacobian)
bool cameraProject(const Camera& cam, const V3& p, double kp[2], double J[6]) {
  if (std::fabs(p.a[2]) < 1.0e-12) return false;
  const double rz = 1.0 / p.a[2];
  const double rz2 = rz * rz;
  const double u0 = p.a[0] * rz, u1 = p.a[1] * rz;
  double d[2], Jd[4];
  distort(cam, u0, u1, d, J ? Jd : nullptr);
  if (J) {
    J[0] = cam.fu * Jd[0] * rz;
    J[1] = cam.fu * Jd[1] * rz;
    J[2] = -cam.fu * (p.a[0] * Jd[0] + p.a[1] * Jd[1]) * rz2;
    J[3] = cam.fv * Jd[2] * rz;
    J[4] = cam.fv * Jd[3] * rz;
    J[5] = -cam.fv * (p.a[0] * Jd[2] + p.a[1] * Jd[3]) * rz2;
  }
  kp[0] = cam.fu * d[0] + cam.cu;
  kp[1] = cam.fv * d[1] + cam.cv;
  return true;
}

bool cameraProjectHomogeneous(const Camera& cam, const V4& hp, double kp[2], double J[8]) {
  V3 head = v3(hp.a[0], hp.a[1], hp.a[2]);
  if (hp.a[3] < 0) head = -head;
  double J3[6];
  // The reference leaves kp / J uninitialised when project() bails out at |z|<1e-12; the oracle
  // (and the GPU path) define them as zero in that case.
  kp[0] = kp[1] = 0.0;
  for (int i = 0; i < 6; ++i) J3[i] = 0.0;
  const bool ok = cameraProject(cam, head, kp, J ? J3 : nullptr);
  if (J) {
    J[0] = J3[0]; J[1] = J3[1]; J[2] = J3[2]; J[3] = 0.0;
    J[4] = J3[3]; J[5] = J3[4]; J[6] = J3[5]; J[7] = 0.0;
  }
  return ok;
}

// ============================================================ manifolds
void posePlus(const double* x, const double* delta, double* out) {  // PoseLocalParameterization.cpp:29-50
  const Quat dq = deltaQ(v3(delta[3], delta[4], delta[5]));
  const Quat q = qnormalized(qmul(dq, qnormalized(qmake(x[6], x[3], x[4], x[5]))));
  out[0] = x[0] + delta[0];
  out[1] = x[1] + delta[1];
  out[2] = x[2] + delta[2];
  out[3] = q.x; out[4] = q.y; out[5] = q.z; out[6] = q.w;
}
void posePlusJacobian(const double* x, double* J) {  // PoseLocalParameterization.cpp:56-68
  for (int i = 0; i < 42; ++i) J[i] = 0.0;
  J[0 * 6 + 0] = J[1 * 6 + 1] = J[2 * 6 + 2] = 1.0;
  const M4 Q = qoplusMat(qmake(x[6], x[3], x[4], x[5]));
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 3; ++c) J[(3 + r) * 6 + 3 + c] = Q(r, c) * 0.5;
}
void poseMinusJacobian(const double* x, double* J) {  // PoseLocalParameterization.cpp:89-103
  for (int i = 0; i < 42; ++i) J[i] = 0.0;
  J[0 * 7 + 0] = J[1 * 7 + 1] = J[2 * 7 + 2] = 1.0;
  const Quat qinv = qmake(x[6], -x[3], -x[4], -x[5]);
  const M4 Qplus = qoplusMat(qinv);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) J[(3 + r) * 7 + 3 + c] = 2.0 * Qplus(r, c);
}
void pointPlus(const double* x, const double* delta, double* out) {
  out[0] = x[0] + delta[0];
  out[1] = x[1] + delta[1];
  out[2] = x[2] + delta[2];
  out[3] = x[3];
}

// ============================================================ ReprojectionError
void reprojectionEvaluate(const Camera& cam, const double* meas, const double* L, const double* pose,
                          const double* hpW, const double* extr, double* r, double* J0,
                          double* J1, double* J2, double* J0min, double* J1min, double* J2min) {
  // implementation/ReprojectionError.hpp:80-106
  const V3 t_WS = v3(pose[0], pose[1], pose[2]);
  const Quat q_WS = qnormalized(qmake(pose[6], pose[3], pose[4], pose[5]));
  V4 hp_W; for (int i = 0; i < 4; ++i) hp_W.a[i] = hpW[i];
  const V3 t_SC = v3(extr[0], extr[1], extr[2]);
  const Quat q_SC = qnormalized(qmake(extr[6], extr[3], extr[4], extr[5]));
  const M3 C_SC = qrot(q_SC);
  const M3 C_CS = C_SC.T();
  M4 T_CS = M4::Identity();
  T_CS.setBlock(0, 0, C_CS);
  T_CS.setBlock(0, 3, -(C_CS * t_SC));
  const M3 C_WS = qrot(q_WS);
  const M3 C_SW = C_WS.T();
  M4 T_SW = M4::Identity();
  T_SW.setBlock(0, 0, C_SW);
  T_SW.setBlock(0, 3, -(C_SW * t_WS));
  const V4 hp_S = T_SW * hp_W;
  const V4 hp_C = T_CS * hp_S;

  const bool wantJ = (J0 || J1 || J2 || J0min || J1min || J2min);
  double kp[2], Jh[8];
  cameraProjectHomogeneous(cam, hp_C, kp, wantJ ? Jh : nullptr);
  const double e0 = meas[0] - kp[0], e1 = meas[1] - kp[1];
  r[0] = L[0] * e0 + L[1] * e1;
  r[1] = L[2] * e0 + L[3] * e1;
  if (!wantJ) return;

  Mat<2, 4> Jh_w;
  for (int rr = 0; rr < 2; ++rr)
    for (int c = 0; c < 4; ++c) Jh_w(rr, c) = L[rr * 2 + 0] * Jh[0 * 4 + c] + L[rr * 2 + 1] * Jh[1 * 4 + c];

  if (J0 || J0min) {  // :134-165
    const V3 p = v3(hp_W.a[0], hp_W.a[1], hp_W.a[2]) - hp_W.a[3] * t_WS;
    Mat<4, 6> J = Mat<4, 6>::Zero();
    J.setBlock(0, 0, hp_W.a[3] * C_SW);
    J.setBlock(0, 3, -(C_SW * crossMx(p)));
    const Mat<2, 6> Jmin = (Jh_w * T_CS) * J;
    if (J0min) for (int i = 0; i < 12; ++i) J0min[i] = Jmin.a[i];
    if (J0) {
      Mat<6, 7> Jl; poseMinusJacobian(pose, Jl.a);
      const Mat<2, 7> Ja = Jmin * Jl;
      for (int i = 0; i < 14; ++i) J0[i] = Ja.a[i];
    }
  }
  if (J1 || J1min) {  // :166-185
    const M4 T_CW = T_CS * T_SW;
    const Mat<2, 4> J = -(Jh_w * T_CW);
    if (J1) for (int i = 0; i < 8; ++i) J1[i] = J.a[i];
    if (J1min)
      for (int rr = 0; rr < 2; ++rr)
        for (int c = 0; c < 3; ++c) J1min[rr * 3 + c] = J(rr, c);
  }
  if (J2 || J2min) {  // :186-216
    const V3 p = v3(hp_S.a[0], hp_S.a[1], hp_S.a[2]) - hp_S.a[3] * t_SC;
    Mat<4, 6> J = Mat<4, 6>::Zero();
    J.setBlock(0, 0, hp_S.a[3] * C_CS);
    J.setBlock(0, 3, -(C_CS * crossMx(p)));
    const Mat<2, 6> Jmin = Jh_w * J;
    if (J2min) for (int i = 0; i < 12; ++i) J2min[i] = Jmin.a[i];
    if (J2) {
      Mat<6, 7> Jl; poseMinusJacobian(extr, Jl.a);
      const Mat<2, 7> Ja = Jmin * Jl;
      for (int i = 0; i < 14; ++i) J2[i] = Ja.a[i];
    }
  }
}

// ============================================================ PseudoInverse::symmSqrtU
// Eigen-decomposition a = V diag(lambda) V^T (cyclic Jacobi, converged to machine precision), then
// result = diag(sqrt(1/lambda or 1/tol)) V^T with tol = max(eps, eps*n*max(lambda))
// (PseudoInverse.hpp:132-158). The eigenvector basis/sign convention differs from Eigen's
// SelfAdjointEigenSolver; only result^T*result (the information matrix) is basis-invariant, which
// is what the solver consumes.
void symmSqrtU(const Mat<15, 15>& a_in, Mat<15, 15>& result) {
  const int n = 15;
  Mat<15, 15> A = a_in;
  Mat<15, 15> V = Mat<15, 15>::Identity();
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0, diag = 0.0;
    for (int i = 0; i < n; ++i) {
      diag += A(i, i) * A(i, i);
      for (int j = i + 1; j < n; ++j) off += A(i, j) * A(i, j);
    }
    if (off <= 1e-36 * diag || off == 0.0) break;
    for (int p = 0; p < n - 1; ++p) {
      for (int q = p + 1; q < n; ++q) {
        const double apq = A(p, q);
        if (apq == 0.0) continue;
        const double app = A(p, p), aqq = A(q, q);
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0);
        const double s = t * c;
        for (int k = 0; k < n; ++k) {  // A <- A J  (columns p,q)
          const double akp = A(k, p), akq = A(k, q);
          A(k, p) = c * akp - s * akq;
          A(k, q) = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {  // A <- J^T A (rows p,q)
          const double apk = A(p, k), aqk = A(q, k);
          A(p, k) = c * apk - s * aqk;
          A(q, k) = s * apk + c * aqk;
        }
        A(p, q) = A(q, p) = 0.0;
        for (int k = 0; k < n; ++k) {  // V <- V J
          const double vkp = V(k, p), vkq = V(k, q);
          V(k, p) = c * vkp - s * vkq;
          V(k, q) = s * vkp + c * vkq;
        }
      }
    }
  }
  double lmax = -1e300;
  for (int i = 0; i < n; ++i) lmax = std::max(lmax, A(i, i));
  const double eps = DBL_EPSILON;
  const double tol = std::max(eps, eps * n * lmax);
  for (int i = 0; i < n; ++i) {
    const double li = A(i, i);
    const double s = std::sqrt(li > tol ? 1.0 / li : 1.0 / tol);
    for (int j = 0; j < n; ++j) result(i, j) = s * V(j, i);
  }
}

// ============================================================ ImuError
ImuError::ImuError() {
  for (int j = 0; j < 4; ++j) dPdsigma[j] = Mat<15, 15>::Zero();
}

void ImuError::loadState(const double* s) {
  redoCounter = (int)s[0];
  redo = s[1] != 0.0;
  Delta_q = Quat{s[2], s[3], s[4], s[5]};
  for (int i = 0; i < 9; ++i) {
    C_integral.a[i] = s[6 + i];
    C_doubleintegral.a[i] = s[15 + i];
    dalpha_db_g.a[i] = s[30 + i];
    dv_db_g.a[i] = s[39 + i];
    dp_db_g.a[i] = s[48 + i];
    sb_ref[i] = s[57 + i];
  }
  for (int i = 0; i < 3; ++i) {
    acc_integral.a[i] = s[24 + i];
    acc_doubleintegral.a[i] = s[27 + i];
  }
  for (int i = 0; i < 225; ++i) sqrtInfo.a[i] = s[66 + i];
  lastSteps = (int)s[291];
  // the append state (ABI 4): cross_ and P_delta_. The four dPdsigma_ of the last integration
  // are not stored; P = sum_j sigma_j^2 dPdsigma_j, and every later use (append) is linear in
  // them, so P is carried as dPdsigma_0 = P / sigma_g^2 (or through the first non-zero sigma).
  for (int i = 0; i < 9; ++i) cross.a[i] = s[292 + i];
  for (int i = 0; i < 225; ++i) P_delta.a[i] = s[301 + i];
  const double sig[4] = {params.sigma_g_c, params.sigma_a_c, params.sigma_gw_c, params.sigma_aw_c};
  for (int j = 0; j < 4; ++j) dPdsigma[j] = Mat<15, 15>::Zero();
  for (int j = 0; j < 4; ++j)
    if (sig[j] != 0.0) {
      dPdsigma[j] = (1.0 / (sig[j] * sig[j])) * P_delta;
      break;
    }
}
void ImuError::storeState(double* s) const {
  s[0] = redoCounter;
  s[1] = redo ? 1.0 : 0.0;
  s[2] = Delta_q.x; s[3] = Delta_q.y; s[4] = Delta_q.z; s[5] = Delta_q.w;
  for (int i = 0; i < 9; ++i) {
    s[6 + i] = C_integral.a[i];
    s[15 + i] = C_doubleintegral.a[i];
    s[30 + i] = dalpha_db_g.a[i];
    s[39 + i] = dv_db_g.a[i];
    s[48 + i] = dp_db_g.a[i];
    s[57 + i] = sb_ref[i];
  }
  for (int i = 0; i < 3; ++i) {
    s[24 + i] = acc_integral.a[i];
    s[27 + i] = acc_doubleintegral.a[i];
  }
  for (int i = 0; i < 225; ++i) s[66 + i] = sqrtInfo.a[i];
  s[291] = lastSteps;
  for (int i = 0; i < 9; ++i) s[292 + i] = cross.a[i];
  for (int i = 0; i < 225; ++i) s[301 + i] = P_delta.a[i];
}

// ImuError::append (ImuError.cpp:63-255). The reference loops over the appended deque `m` and
// compares with the end of the merged member deque; the loop always leaves at nexttime == t_1
// first because m covers t_1 (checked), which is what this restatement does.
int ImuError::append(const double* sb, const std::vector<ImuSample>& m, long long t_1) {
  // merge the deques (:74-81)
  size_t first = 0;
  while (first < m.size() && !(m[first].t > meas.back().t)) ++first;
  meas.insert(meas.end(), m.begin() + first, m.end());
  long long time = t1;
  const long long end = t_1;
  t1 = t_1;  // setT1
  if (m.empty() || !(m.back().t >= end)) return -1;
  const V3 bg = v3(sb[3], sb[4], sb[5]);
  const V3 ba = v3(sb[6], sb[7], sb[8]);
  bool hasStarted = false;
  int i = 0;
  const int N = (int)m.size();
  for (int it = 0; it + 1 < N; ++it) {
    V3 omega_S_0 = v3(m[it].g[0], m[it].g[1], m[it].g[2]);
    V3 acc_S_0 = v3(m[it].a[0], m[it].a[1], m[it].a[2]);
    V3 omega_S_1 = v3(m[it + 1].g[0], m[it + 1].g[1], m[it + 1].g[2]);
    V3 acc_S_1 = v3(m[it + 1].a[0], m[it + 1].a[1], m[it + 1].a[2]);
    long long nexttime = m[it + 1].t;
    double dt = durToSec(nexttime - time);
    if (end < nexttime) {
      const double interval = durToSec(nexttime - m[it].t);
      nexttime = t1;
      dt = durToSec(nexttime - time);
      const double r = dt / interval;
      omega_S_1 = (1.0 - r) * omega_S_0 + r * omega_S_1;
      acc_S_1 = (1.0 - r) * acc_S_0 + r * acc_S_1;
    }
    if (dt <= 0.0) continue;
    if (!hasStarted) {
      hasStarted = true;
      const double r = dt / durToSec(nexttime - m[it].t);
      omega_S_0 = r * omega_S_0 + (1.0 - r) * omega_S_1;
      acc_S_0 = r * acc_S_0 + (1.0 - r) * acc_S_1;
    }
    double gyr_sat_mult = 1.0, acc_sat_mult = 1.0;
    for (int k = 0; k < 3; ++k)
      if (std::fabs(omega_S_0.a[k]) > params.g_max || std::fabs(omega_S_1.a[k]) > params.g_max) {
        gyr_sat_mult *= 100; break;
      }
    for (int k = 0; k < 3; ++k)
      if (std::fabs(acc_S_0.a[k]) > params.a_max || std::fabs(acc_S_1.a[k]) > params.a_max) {
        acc_sat_mult *= 100; break;
      }
    // (:160-190) orientation, rotation (double) integrals
    const V3 omega_S_true = 0.5 * (omega_S_0 + omega_S_1) - bg;
    const double theta_half = omega_S_true.norm() * 0.5 * dt;
    const double sinc_theta_half = sinc(theta_half);
    const double cos_theta_half = std::cos(theta_half);
    const V3 dqv = (sinc_theta_half * 0.5 * dt) * omega_S_true;
    const Quat dq{dqv.a[0], dqv.a[1], dqv.a[2], cos_theta_half};
    const Quat Delta_q_1 = qmul(Delta_q, dq);
    const M3 C = qrot(Delta_q);
    const M3 C_1 = qrot(Delta_q_1);
    const V3 acc_S_true = 0.5 * (acc_S_0 + acc_S_1) - ba;
    const M3 CC1 = C + C_1;
    const M3 C_integral_1 = C_integral + (0.5 * dt) * CC1;
    const V3 acc_integral_1 = acc_integral + (0.5 * dt) * (CC1 * acc_S_true);
    C_doubleintegral += dt * C_integral + (0.25 * dt * dt) * CC1;
    acc_doubleintegral += dt * acc_integral + (0.25 * dt * dt) * (CC1 * acc_S_true);
    // (:192-200) Jacobian parts
    const M3 Jr = rightJacobian(dt * omega_S_true);
    dalpha_db_g += dt * (C_1 * Jr);
    const M3 cross_1 = qrot(qinverse(dq)) * cross + dt * Jr;
    const M3 acc_S_x = crossMx(acc_S_true);
    const M3 X = C * acc_S_x * cross + C_1 * acc_S_x * cross_1;
    const M3 dv_db_g_1 = dv_db_g + (0.5 * dt) * X;
    dp_db_g += dt * dv_db_g + (0.25 * dt * dt) * X;
    // (:202-233) covariance derivatives
    Mat<15, 15> F = Mat<15, 15>::Identity();
    F.setBlock(0, 3, -crossMx(dt * acc_integral + (0.25 * dt * dt) * (CC1 * acc_S_true)));
    F.setBlock(0, 6, dt * M3::Identity());
    F.setBlock(0, 9, dt * dv_db_g + (0.25 * dt * dt) * X);
    F.setBlock(0, 12, -(dt * C_integral) + (0.25 * dt * dt) * CC1);
    F.setBlock(3, 9, -(dt * C_1));
    F.setBlock(6, 3, -crossMx((0.5 * dt) * (CC1 * acc_S_true)));
    F.setBlock(6, 9, (0.5 * dt) * X);
    F.setBlock(6, 12, -((0.5 * dt) * CC1));
    Mat<15, 15> K[4];
    for (int j = 0; j < 4; ++j) K[j] = Mat<15, 15>::Zero();
    for (int k = 0; k < 3; ++k) {
      K[0](3 + k, 3 + k) = gyr_sat_mult * dt;
      K[1](k, k) = 0.5 * dt * dt * dt * acc_sat_mult * acc_sat_mult * acc_sat_mult;
      K[1](6 + k, 6 + k) = acc_sat_mult * dt;
      K[2](9 + k, 9 + k) = dt;
      K[3](12 + k, 12 + k) = dt;
    }
    const Mat<15, 15> Ft = F.T();
    for (int j = 0; j < 4; ++j) dPdsigma[j] = F * dPdsigma[j] * Ft + K[j];
    Delta_q = Delta_q_1;
    C_integral = C_integral_1;
    acc_integral = acc_integral_1;
    cross = cross_1;
    dv_db_g = dv_db_g_1;
    time = nexttime;
    ++i;
    if (nexttime == t1) break;
  }
  // (:236-252) weighting; speedAndBiases_ref_, redo_ and the redo counter are left as they are
  for (int j = 0; j < 4; ++j) dPdsigma[j] = 0.5 * dPdsigma[j] + 0.5 * dPdsigma[j].T();
  P_delta = (params.sigma_g_c * params.sigma_g_c) * dPdsigma[0];
  P_delta += (params.sigma_a_c * params.sigma_a_c) * dPdsigma[1];
  P_delta += (params.sigma_gw_c * params.sigma_gw_c) * dPdsigma[2];
  P_delta += (params.sigma_aw_c * params.sigma_aw_c) * dPdsigma[3];
  symmSqrtU(P_delta, sqrtInfo);
  lastSteps = i;
  return i;
}

// ImuError::redoPreintegration (ImuError.cpp:258-466), literal 4-derivative covariance recursion.
int ImuError::redoPreintegration(const double* sb) {
  long long time = t0;
  const long long end = t1;
  if (!(meas.back().t >= end)) return -1;
  Delta_q = Quat{0, 0, 0, 1};
  C_integral = M3::Zero(); C_doubleintegral = M3::Zero();
  acc_integral = V3::Zero(); acc_doubleintegral = V3::Zero();
  cross = M3::Zero();
  dalpha_db_g = M3::Zero(); dv_db_g = M3::Zero(); dp_db_g = M3::Zero();
  P_delta = Mat<15, 15>::Zero();
  for (int j = 0; j < 4; ++j) dPdsigma[j] = Mat<15, 15>::Zero();
  const V3 bg = v3(sb[3], sb[4], sb[5]);
  const V3 ba = v3(sb[6], sb[7], sb[8]);

  bool hasStarted = false;
  int i = 0;
  const int N = (int)meas.size();
  for (int it = 0; it < N; ++it) {
    // (it+1) is always valid here: the loop breaks at nexttime == t1 <= back().timeStamp.
    const int nx = (it + 1 < N) ? it + 1 : it;
    V3 omega_S_0 = v3(meas[it].g[0], meas[it].g[1], meas[it].g[2]);
    V3 acc_S_0 = v3(meas[it].a[0], meas[it].a[1], meas[it].a[2]);
    V3 omega_S_1 = v3(meas[nx].g[0], meas[nx].g[1], meas[nx].g[2]);
    V3 acc_S_1 = v3(meas[nx].a[0], meas[nx].a[1], meas[nx].a[2]);
    long long nexttime = (it + 1 == N) ? t1 : meas[it + 1].t;
    double dt = durToSec(nexttime - time);
    if (end < nexttime) {
      const double interval = durToSec(nexttime - meas[it].t);
      nexttime = t1;
      dt = durToSec(nexttime - time);
      const double r = dt / interval;
      omega_S_1 = (1.0 - r) * omega_S_0 + r * omega_S_1;
      acc_S_1 = (1.0 - r) * acc_S_0 + r * acc_S_1;
    }
    if (dt <= 0.0) continue;
    if (!hasStarted) {
      hasStarted = true;
      const double r = dt / durToSec(nexttime - meas[it].t);
      omega_S_0 = r * omega_S_0 + (1.0 - r) * omega_S_1;
      acc_S_0 = r * acc_S_0 + (1.0 - r) * acc_S_1;
    }
    double gyr_sat_mult = 1.0, acc_sat_mult = 1.0;
    for (int k = 0; k < 3; ++k)
      if (std::fabs(omega_S_0.a[k]) > params.g_max || std::fabs(omega_S_1.a[k]) > params.g_max) {
        gyr_sat_mult *= 100; break;
      }
    for (int k = 0; k < 3; ++k)
      if (std::fabs(acc_S_0.a[k]) > params.a_max || std::fabs(acc_S_1.a[k]) > params.a_max) {
        acc_sat_mult *= 100; break;
      }
    // orientation (:362-370)
    const V3 omega_S_true = 0.5 * (omega_S_0 + omega_S_1) - bg;
    const double theta_half = omega_S_true.norm() * 0.5 * dt;
    const double sinc_theta_half = sinc(theta_half);
    const double cos_theta_half = std::cos(theta_half);
    const V3 dqv = (sinc_theta_half * 0.5 * dt) * omega_S_true;
    const Quat dq{dqv.a[0], dqv.a[1], dqv.a[2], cos_theta_half};
    const Quat Delta_q_1 = qmul(Delta_q, dq);
    const M3 C = qrot(Delta_q);
    const M3 C_1 = qrot(Delta_q_1);
    const V3 acc_S_true = 0.5 * (acc_S_0 + acc_S_1) - ba;
    const M3 CC1 = C + C_1;
    const M3 C_integral_1 = C_integral + (0.5 * dt) * CC1;
    const V3 acc_integral_1 = acc_integral + (0.5 * dt) * (CC1 * acc_S_true);
    C_doubleintegral += dt * C_integral + (0.25 * dt * dt) * CC1;
    acc_doubleintegral += dt * acc_integral + (0.25 * dt * dt) * (CC1 * acc_S_true);
    // Jacobian parts (:385-392)
    const M3 Jr = rightJacobian(dt * omega_S_true);
    dalpha_db_g += dt * (C_1 * Jr);
    const M3 cross_1 = qrot(qinverse(dq)) * cross + dt * Jr;
    const M3 acc_S_x = crossMx(acc_S_true);
    const M3 X = C * acc_S_x * cross + C_1 * acc_S_x * cross_1;
    const M3 dv_db_g_1 = dv_db_g + (0.5 * dt) * X;
    dp_db_g += dt * dv_db_g + (0.25 * dt * dt) * X;
    // covariance propagation (:395-426)
    Mat<15, 15> F = Mat<15, 15>::Identity();
    F.setBlock(0, 3, -crossMx(dt * acc_integral + (0.25 * dt * dt) * (CC1 * acc_S_true)));
    F.setBlock(0, 6, dt * M3::Identity());
    F.setBlock(0, 9, dt * dv_db_g + (0.25 * dt * dt) * X);
    F.setBlock(0, 12, -(dt * C_integral) + (0.25 * dt * dt) * CC1);
    F.setBlock(3, 9, -(dt * C_1));
    F.setBlock(6, 3, -crossMx((0.5 * dt) * (CC1 * acc_S_true)));
    F.setBlock(6, 9, (0.5 * dt) * X);
    F.setBlock(6, 12, -((0.5 * dt) * CC1));
    Mat<15, 15> K[4];
    for (int j = 0; j < 4; ++j) K[j] = Mat<15, 15>::Zero();
    for (int k = 0; k < 3; ++k) {
      K[0](3 + k, 3 + k) = gyr_sat_mult * dt;
      K[1](k, k) = 0.5 * dt * dt * dt * acc_sat_mult * acc_sat_mult * acc_sat_mult;
      K[1](6 + k, 6 + k) = acc_sat_mult * dt;
      K[2](9 + k, 9 + k) = dt;
      K[3](12 + k, 12 + k) = dt;
    }
    const Mat<15, 15> Ft = F.T();
    for (int j = 0; j < 4; ++j) dPdsigma[j] = F * dPdsigma[j] * Ft + K[j];
    // memory shift
    Delta_q = Delta_q_1;
    C_integral = C_integral_1;
    acc_integral = acc_integral_1;
    cross = cross_1;
    dv_db_g = dv_db_g_1;
    time = nexttime;
    ++i;
    if (nexttime == t1) break;
  }
  for (int k = 0; k < 9; ++k) sb_ref[k] = sb[k];
  for (int j = 0; j < 4; ++j) dPdsigma[j] = 0.5 * dPdsigma[j] + 0.5 * dPdsigma[j].T();
  P_delta = (params.sigma_g_c * params.sigma_g_c) * dPdsigma[0];
  P_delta += (params.sigma_a_c * params.sigma_a_c) * dPdsigma[1];
  P_delta += (params.sigma_gw_c * params.sigma_gw_c) * dPdsigma[2];
  P_delta += (params.sigma_aw_c * params.sigma_aw_c) * dPdsigma[3];
  symmSqrtU(P_delta, sqrtInfo);
  return i;
}

// ImuError::EvaluateWithMinimalJacobians (ImuError.cpp:797-1003)
bool ImuError::evaluate(const double* const* prm, double* residuals, double** jac, double** jacMin,
                        bool redoAlways) {
  bool success = true;
  const V3 r0 = v3(prm[0][0], prm[0][1], prm[0][2]);
  const Quat q0 = qnormalized(qmake(prm[0][6], prm[0][3], prm[0][4], prm[0][5]));
  const V3 r1 = v3(prm[2][0], prm[2][1], prm[2][2]);
  const Quat q1 = qnormalized(qmake(prm[2][6], prm[2][3], prm[2][4], prm[2][5]));
  const double* sb0 = prm[1];
  const double* sb1 = prm[3];
  const M3 C_WS_0 = qrot(q0);
  const M3 C_S0_W = C_WS_0.T();
  const double Delta_t = durToSec(t1 - t0);
  Mat<6, 1> Delta_b;
  for (int k = 0; k < 6; ++k) Delta_b.a[k] = sb0[3 + k] - sb_ref[3 + k];
  const double dbg = std::sqrt(Delta_b.a[0] * Delta_b.a[0] + Delta_b.a[1] * Delta_b.a[1] +
                               Delta_b.a[2] * Delta_b.a[2]);
  redo = redo || (dbg > 0.0003);
  if ((redo && (((int)meas.size() < 50) || redoAlways)) || redoCounter == 0) {
    const int steps = redoPreintegration(sb0);
    lastSteps = steps;
    if (steps == 0) success = false;  // "hack it away" (ImuError.cpp:849-853)
    redoCounter++;
    Delta_b = Mat<6, 1>::Zero();
    redo = false;
  }

  const V3 g_W = v3(0, 0, params.g);  // g * (0,0,6371009).normalized()
  Mat<15, 15> F0 = Mat<15, 15>::Identity();
  const V3 sv0 = v3(sb0[0], sb0[1], sb0[2]);
  const V3 sv1 = v3(sb1[0], sb1[1], sb1[2]);
  const V3 delta_p_est_W = r0 - r1 + Delta_t * sv0 - (0.5 * Delta_t * Delta_t) * g_W;
  const V3 delta_v_est_W = sv0 - sv1 - Delta_t * g_W;
  const Mat<3, 1> dbg3 = Delta_b.block<3, 1>(0, 0);
  const Quat Dq = qmul(deltaQ(-(dalpha_db_g * dbg3)), Delta_q);
  F0.setBlock(0, 0, C_S0_W);
  F0.setBlock(0, 3, C_S0_W * crossMx(delta_p_est_W));
  F0.setBlock(0, 6, Delta_t * C_S0_W);
  F0.setBlock(0, 9, dp_db_g);
  F0.setBlock(0, 12, -C_doubleintegral);
  {
    const M4 m = qplusMat(qmul(Dq, qinverse(q1))) * qoplusMat(q0);
    F0.setBlock(3, 3, m.block<3, 3>(0, 0));
  }
  {
    const M4 m = qoplusMat(qmul(qinverse(q1), q0)) * qoplusMat(Dq);
    F0.setBlock(3, 9, m.block<3, 3>(0, 0) * (-dalpha_db_g));
  }
  F0.setBlock(6, 3, C_S0_W * crossMx(delta_v_est_W));
  F0.setBlock(6, 6, C_S0_W);
  F0.setBlock(6, 9, dv_db_g);
  F0.setBlock(6, 12, -C_integral);
  Mat<15, 15> F1 = -Mat<15, 15>::Identity();
  F1.setBlock(0, 0, -C_S0_W);
  {
    const M4 m = qplusMat(Dq) * qoplusMat(q0) * qplusMat(qinverse(q1));
    F1.setBlock(3, 3, -m.block<3, 3>(0, 0));
  }
  F1.setBlock(6, 6, -C_S0_W);

  Mat<15, 1> error;
  {
    const V3 e0 = C_S0_W * delta_p_est_W + acc_doubleintegral + F0.block<3, 6>(0, 9) * Delta_b;
    const Quat qe = qmul(Dq, qmul(qinverse(q1), q0));
    const V3 e6 = C_S0_W * delta_v_est_W + acc_integral + F0.block<3, 6>(6, 9) * Delta_b;
    for (int k = 0; k < 3; ++k) {
      error.a[k] = e0.a[k];
      error.a[6 + k] = e6.a[k];
    }
    error.a[3] = 2 * qe.x; error.a[4] = 2 * qe.y; error.a[5] = 2 * qe.z;
    for (int k = 0; k < 6; ++k) error.a[9 + k] = sb0[3 + k] - sb1[3 + k];
  }
  if (!success) error = Mat<15, 1>::Zero();
  const Mat<15, 1> we = sqrtInfo * error;
  for (int k = 0; k < 15; ++k) residuals[k] = we.a[k];

  const bool any = jac || jacMin;
  if (!any) return true;
  auto want = [&](int i) { return (jac && jac[i]) || (jacMin && jacMin[i]); };
  if (want(0)) {
    Mat<15, 6> J0m = sqrtInfo * F0.block<15, 6>(0, 0);
    if (!success) J0m = Mat<15, 6>::Zero();
    if (jac && jac[0]) {
      Mat<6, 7> Jl; poseMinusJacobian(prm[0], Jl.a);
      const Mat<15, 7> J = J0m * Jl;
      for (int i = 0; i < 105; ++i) jac[0][i] = J.a[i];
    }
    if (jacMin && jacMin[0]) for (int i = 0; i < 90; ++i) jacMin[0][i] = J0m.a[i];
  }
  if (want(1)) {
    Mat<15, 9> J1 = sqrtInfo * F0.block<15, 9>(0, 6);
    if (!success) J1 = Mat<15, 9>::Zero();
    if (jac && jac[1]) for (int i = 0; i < 135; ++i) jac[1][i] = J1.a[i];
    if (jacMin && jacMin[1]) for (int i = 0; i < 135; ++i) jacMin[1][i] = J1.a[i];
  }
  if (want(2)) {
    Mat<15, 6> J2m = sqrtInfo * F1.block<15, 6>(0, 0);
    if (!success) J2m = Mat<15, 6>::Zero();
    if (jac && jac[2]) {
      Mat<6, 7> Jl; poseMinusJacobian(prm[2], Jl.a);
      const Mat<15, 7> J = J2m * Jl;
      for (int i = 0; i < 105; ++i) jac[2][i] = J.a[i];
    }
    if (jacMin && jacMin[2]) for (int i = 0; i < 90; ++i) jacMin[2][i] = J2m.a[i];
  }
  if (want(3)) {
    Mat<15, 9> J3 = sqrtInfo * F1.block<15, 9>(0, 6);
    if (!success) J3 = Mat<15, 9>::Zero();
    if (jac && jac[3]) for (int i = 0; i < 135; ++i) jac[3][i] = J3.a[i];
    if (jacMin && jacMin[3]) for (int i = 0; i < 135; ++i) jacMin[3][i] = J3.a[i];
  }
  return true;
}

// ============================================================ PoseError / SpeedAndBiasError
void poseErrorEvaluate(const double* meas, const double* L, const double* pose, double* r, double* J,
                       double* Jmin) {
  // T_WS with normalised q; dp = measurement * T_WS^-1 (PoseError.cpp:81-90)
  const Quat q = qnormalized(qmake(pose[6], pose[3], pose[4], pose[5]));
  const Quat qm = qmake(meas[6], meas[3], meas[4], meas[5]);
  const Quat dq = qmul(qm, qinverse(q));
  double e[6];
  e[0] = meas[0] - pose[0];
  e[1] = meas[1] - pose[1];
  e[2] = meas[2] - pose[2];
  e[3] = 2 * dq.x; e[4] = 2 * dq.y; e[5] = 2 * dq.z;
  for (int i = 0; i < 6; ++i) {
    double s = 0;
    for (int k = 0; k < 6; ++k) s += L[i * 6 + k] * e[k];
    r[i] = s;
  }
  if (!J && !Jmin) return;
  Mat<6, 6> J0m = -Mat<6, 6>::Identity();  // :104-110
  const M4 P = qplusMat(dq);
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) J0m(3 + a, 3 + b) = -P(a, b);
  Mat<6, 6> Lm; for (int i = 0; i < 36; ++i) Lm.a[i] = L[i];
  const Mat<6, 6> Jw = Lm * J0m;
  if (Jmin) for (int i = 0; i < 36; ++i) Jmin[i] = Jw.a[i];
  if (J) {
    Mat<6, 7> Jl; poseMinusJacobian(pose, Jl.a);
    const Mat<6, 7> Ja = Jw * Jl;
    for (int i = 0; i < 42; ++i) J[i] = Ja.a[i];
  }
}

void sbErrorEvaluate(const double* meas, const double* L, const double* sb, double* r, double* J) {
  double e[9];
  for (int i = 0; i < 9; ++i) e[i] = meas[i] - sb[i];
  for (int i = 0; i < 9; ++i) {
    double s = 0;
    for (int k = 0; k < 9; ++k) s += L[i * 9 + k] * e[k];
    r[i] = s;
  }
  if (J) for (int i = 0; i < 81; ++i) J[i] = -L[i];
}

}  // namespace oracle
