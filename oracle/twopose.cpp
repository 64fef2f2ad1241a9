// twopose.cpp — TEST INFRASTRUCTURE ONLY (parity oracle). CPU restatement of the relative-pose
// (pose-graph) edge that okvis leaves in the window after marginalising keyframe observations:
//   TwoPoseStandardGraphError::compute            okvis_ceres/src/TwoPoseGraphError.cpp:162-397
//   TwoPoseStandardGraphError(Const)::Evaluate... okvis_ceres/src/TwoPoseGraphError.cpp:467-606,
//                                                 :631-767 (both classes evaluate identically)
//   PseudoInverse::symmSqrt                       okvis_ceres/include/okvis/PseudoInverse.hpp:101-129
//   RelativePoseError::EvaluateWithMinimalJacobians okvis_ceres/src/RelativePoseError.cpp:59-140
// Eigen's SelfAdjointEigenSolver is restated as a cyclic Jacobi eigen-solve with eigenvalues sorted
// ascending; eigenvector signs are arbitrary in both, and everything the solver consumes (J_^T J_,
// DeltaX_, the marginalised H00_ / b0_) is sign-invariant.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "oracle.hpp"

namespace oracle {

// Cyclic Jacobi: A = V diag(lam) V^T, lam ascending (columns of V are the eigenvectors).
template <int N>
void jacobiEigen(const Mat<N, N>& a_in, double lam[N], Mat<N, N>& Vout) {
  Mat<N, N> A = a_in;
  Mat<N, N> V = Mat<N, N>::Identity();
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0, diag = 0.0;
    for (int i = 0; i < N; ++i) {
      diag += A(i, i) * A(i, i);
      for (int j = i + 1; j < N; ++j) off += A(i, j) * A(i, j);
    }
    if (off <= 1e-36 * diag || off == 0.0) break;
    for (int p = 0; p < N - 1; ++p)
      for (int q = p + 1; q < N; ++q) {
        const double apq = A(p, q);
        if (apq == 0.0) continue;
        const double theta = (A(q, q) - A(p, p)) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < N; ++k) {
          const double akp = A(k, p), akq = A(k, q);
          A(k, p) = c * akp - s * akq;
          A(k, q) = s * akp + c * akq;
        }
        for (int k = 0; k < N; ++k) {
          const double apk = A(p, k), aqk = A(q, k);
          A(p, k) = c * apk - s * aqk;
          A(q, k) = s * apk + c * aqk;
        }
        A(p, q) = A(q, p) = 0.0;
        for (int k = 0; k < N; ++k) {
          const double vkp = V(k, p), vkq = V(k, q);
          V(k, p) = c * vkp - s * vkq;
          V(k, q) = s * vkp + c * vkq;
        }
      }
  }
  int idx[N];
  for (int i = 0; i < N; ++i) idx[i] = i;
  std::sort(idx, idx + N, [&](int x, int y) { return A(x, x) < A(y, y); });
  for (int i = 0; i < N; ++i) {
    lam[i] = A(idx[i], idx[i]);
    for (int k = 0; k < N; ++k) Vout(k, i) = V(k, idx[i]);
  }
}

namespace {

struct Pose {
  V3 r;
  Quat q;  // normalised (okvis::kinematics::Transformation normalises on construction)
};
Pose poseOf(const double* p) { return Pose{v3(p[0], p[1], p[2]), qnormalized(qmake(p[6], p[3], p[4], p[5]))}; }
Pose inverse(const Pose& T) {  // Transformation.hpp:187-190
  const Quat qi = qinverse(T.q);
  return Pose{-(qrot(T.q).T() * T.r), qnormalized(qi)};
}
Pose compose(const Pose& A, const Pose& B) {  // Transformation operator*: r_A + C_A r_B, q_A q_B
  return Pose{A.r + qrot(A.q) * B.r, qnormalized(qmul(A.q, B.q))};
}

}  // namespace

// TwoPoseGraphError.cpp:467-606 / :631-767. Jmin0 (reference pose), Jmin1 (other pose): 6x6
// row-major minimal Jacobians; J0/J1: ambient 6x7 (= Jmin * PoseManifold::minusJacobian).
void relPoseEvaluate(const double* dx, const double* Jsq, const double* lin, const double* pose0,
                     const double* pose1, double* r, double* Jmin0, double* Jmin1, double* J0, double* J1) {
  const Pose T_WS0 = poseOf(pose0);
  const Pose T_S0W = inverse(T_WS0);
  const Pose T_WSi = poseOf(pose1);
  const Pose T_S0Si = compose(T_S0W, T_WSi);
  const V3 r_lin = v3(lin[0], lin[1], lin[2]);
  const Quat q_lin = qnormalized(qmake(lin[6], lin[3], lin[4], lin[5]));
  Mat<6, 1> err;
  const V3 dr = T_S0Si.r - r_lin;
  const Quat dq = qmul(T_S0Si.q, qinverse(q_lin));
  const double dX[6] = {dr.a[0], dr.a[1], dr.a[2], 2.0 * dq.x, 2.0 * dq.y, 2.0 * dq.z};
  for (int i = 0; i < 6; ++i) err.a[i] = dx[i] + dX[i];
  Mat<6, 6> J_;
  for (int i = 0; i < 36; ++i) J_.a[i] = Jsq[i];
  const Mat<6, 1> e = J_ * err;
  for (int i = 0; i < 6; ++i) r[i] = e.a[i];
  if (!Jmin0 && !Jmin1 && !J0 && !J1) return;
  const M3 C_S0W = qrot(T_S0W.q);
  Mat<6, 6> Jerr = Mat<6, 6>::Zero();
  Jerr.setBlock(0, 0, C_S0W);
  const M4 Pm = qplusMat(qinverse(T_WS0.q)) * qoplusMat(qmul(T_WSi.q, qinverse(q_lin)));
  const M3 B = Pm.block<3, 3>(0, 0);
  Jerr.setBlock(3, 3, B);
  Mat<6, 6> JerrRef = Mat<6, 6>::Zero();
  JerrRef.setBlock(0, 0, -C_S0W);
  JerrRef.setBlock(0, 3, C_S0W * crossMx(T_WSi.r - T_WS0.r));
  JerrRef.setBlock(3, 3, -B);
  const Mat<6, 6> Jm1 = J_ * Jerr, Jm0 = J_ * JerrRef;
  if (Jmin0) for (int i = 0; i < 36; ++i) Jmin0[i] = Jm0.a[i];
  if (Jmin1) for (int i = 0; i < 36; ++i) Jmin1[i] = Jm1.a[i];
  if (J0) {
    Mat<6, 7> Jl; poseMinusJacobian(pose0, Jl.a);
    const Mat<6, 7> Ja = Jm0 * Jl;
    for (int i = 0; i < 42; ++i) J0[i] = Ja.a[i];
  }
  if (J1) {
    Mat<6, 7> Jl; poseMinusJacobian(pose1, Jl.a);
    const Mat<6, 7> Ja = Jm1 * Jl;
    for (int i = 0; i < 42; ++i) J1[i] = Ja.a[i];
  }
}

// RelativePoseError::EvaluateWithMinimalJacobians (RelativePoseError.cpp:59-140): T_AB measured,
// L = LLT(information).L^T; parameters T_WA (pose0), T_WB (pose1).
void relativePoseErrorEvaluate(const double* Tab, const double* Lsq, const double* pose0, const double* pose1,
                               double* r, double* Jmin0, double* Jmin1, double* J0, double* J1) {
  const Pose T_WA = poseOf(pose0), T_WB = poseOf(pose1), T_ABm = poseOf(Tab);
  const Pose T_AW = inverse(T_WA), T_BW = inverse(T_WB);
  const Pose T_AB = compose(T_AW, T_WB);
  const V3 dr = T_ABm.r - T_AB.r;
  const Quat dq = qmul(T_ABm.q, qinverse(T_AB.q));
  const double e[6] = {dr.a[0], dr.a[1], dr.a[2], 2.0 * dq.x, 2.0 * dq.y, 2.0 * dq.z};
  Mat<6, 6> L;
  for (int i = 0; i < 36; ++i) L.a[i] = Lsq[i];
  for (int i = 0; i < 6; ++i) {
    double s = 0;
    for (int k = 0; k < 6; ++k) s += L(i, k) * e[k];
    r[i] = s;
  }
  if (!Jmin0 && !Jmin1 && !J0 && !J1) return;
  const M3 C_AW = qrot(T_AW.q);
  const M4 Pm = qplusMat(qmul(T_ABm.q, T_BW.q)) * qoplusMat(T_WA.q);
  const M3 B = Pm.block<3, 3>(0, 0);
  Mat<6, 6> A0 = Mat<6, 6>::Identity(), A1 = Mat<6, 6>::Identity();
  A0.setBlock(0, 0, C_AW);
  A0.setBlock(0, 3, -(C_AW * crossMx(T_WB.r - T_WA.r)));
  A0.setBlock(3, 3, B);
  A1.setBlock(0, 0, -C_AW);
  A1.setBlock(3, 3, -B);
  const Mat<6, 6> Jm0 = L * A0, Jm1 = L * A1;
  if (Jmin0) for (int i = 0; i < 36; ++i) Jmin0[i] = Jm0.a[i];
  if (Jmin1) for (int i = 0; i < 36; ++i) Jmin1[i] = Jm1.a[i];
  if (J0) {
    Mat<6, 7> Jl; poseMinusJacobian(pose0, Jl.a);
    const Mat<6, 7> Ja = Jm0 * Jl;
    for (int i = 0; i < 42; ++i) J0[i] = Ja.a[i];
  }
  if (J1) {
    Mat<6, 7> Jl; poseMinusJacobian(pose1, Jl.a);
    const Mat<6, 7> Ja = Jm1 * Jl;
    for (int i = 0; i < 42; ++i) J1[i] = Ja.a[i];
  }
}

// TwoPoseStandardGraphError::compute (TwoPoseGraphError.cpp:162-397) for edge e of the batch.
void twoPoseCompute(const okvisgpu_twopose_edges* E, int e, double* deltaX, double* Jsq, double* linPoint,
                    double* H00out, double* b0out) {
  const Pose T_WS0 = poseOf(&E->ref_pose[7 * e]);
  const Pose T_S0W = inverse(T_WS0);
  const Pose T_S0S1 = compose(T_S0W, poseOf(&E->other_pose[7 * e]));
  std::vector<Camera> cams;
  for (int c = 0; c < E->n_cameras; ++c) {
    const okvisgpu_camera& k = E->cameras[c];
    cams.push_back(cameraOf(k));
  }
  bool relPoseSet = false;
  Mat<6, 6> H00_ = Mat<6, 6>::Zero(), mH = Mat<6, 6>::Zero();
  Mat<6, 1> b0_ = Mat<6, 1>::Zero(), mb = Mat<6, 1>::Zero();
  const double identity[7] = {0, 0, 0, 0, 0, 0, 1};
  double relPose[7];
  for (int i = 0; i < 3; ++i) relPose[i] = T_S0S1.r.a[i];
  relPose[3] = T_S0S1.q.x; relPose[4] = T_S0S1.q.y; relPose[5] = T_S0S1.q.z; relPose[6] = T_S0S1.q.w;
  for (int l = E->landmark_begin[e]; l < E->landmark_begin[e + 1]; ++l) {
    Mat<6, 6> H00 = Mat<6, 6>::Zero();
    Mat<6, 1> b0 = Mat<6, 1>::Zero();
    Mat<6, 3> H01 = Mat<6, 3>::Zero();
    M3 H11 = M3::Zero();
    V3 b1 = V3::Zero();
    // landmark in S0 coordinates (:198-205), minimal distance (:208)
    const double* hw = &E->landmarks[4 * l];
    const M3 C = qrot(T_S0W.q);
    const V3 xyz = C * v3(hw[0], hw[1], hw[2]) + hw[3] * T_S0W.r;
    const double hpS0[4] = {xyz.a[0], xyz.a[1], xyz.a[2], hw[3]};
    const double minDist = hpS0[2] / hpS0[3];
    for (int o = E->obs_begin[l]; o < E->obs_begin[l + 1]; ++o) {
      const bool isReference = E->obs_other[o] == 0;
      if (!isReference && !relPoseSet) relPoseSet = true;  // :267-270
      const int ci = E->obs_camera[o];
      double r[2], J0[12], J1[6];
      reprojectionEvaluate(cams[ci], &E->obs_keypoint[2 * o], &E->obs_sqrt_info[4 * o],
                           isReference ? identity : relPose, hpS0, &E->extrinsics[7 * ci], r, nullptr,
                           nullptr, nullptr, J0, J1, nullptr);
      if (std::sqrt(r[0] * r[0] + r[1] * r[1]) > 3.0) continue;  // :285-288 obvious outliers
      const bool cauchy = E->obs_cauchy ? E->obs_cauchy[o] != 0 : true;
      if (cauchy) {  // Corrector (:290-337); CauchyLoss rho'' < 0: scale by sqrt(rho')
        const double sq = r[0] * r[0] + r[1] * r[1];
        const double s = std::sqrt(std::max(DBL_MIN, 1.0 / (1.0 + sq)));
        for (double& v : J0) v *= s;
        for (double& v : J1) v *= s;
        r[0] *= s;
        r[1] *= s;
      }
      if (!isReference)  // :340-344
        for (int a = 0; a < 6; ++a) {
          for (int b = 0; b < 6; ++b) H00(a, b) += J0[a] * J0[b] + J0[6 + a] * J0[6 + b];
          b0.a[a] -= J0[a] * r[0] + J0[6 + a] * r[1];
          for (int b = 0; b < 3; ++b) H01(a, b) += J0[a] * J1[b] + J0[6 + a] * J1[3 + b];
        }
      for (int a = 0; a < 3; ++a) {  // :346-347
        for (int b = 0; b < 3; ++b) H11(a, b) += J1[a] * J1[b] + J1[3 + a] * J1[3 + b];
        b1.a[a] -= J1[a] * r[0] + J1[3 + a] * r[1];
      }
    }
    // marginalise the landmark (:354-368): symmSqrt(V, 1e-7) => M M^T = W V^+ W^T
    double lam[3];
    M3 Ev;
    jacobiEigen<3>(H11, lam, Ev);
    const double tol = std::max(1.0e-7, 1.0e-7 * 3 * lam[2]);
    int rank = 0;
    for (int i = 0; i < 3; ++i) rank += lam[i] > tol;
    if (rank < 3 && minDist < 2.99) continue;
    M3 Vsqrt;  // E diag(sqrt(1/lambda or 1/tol))
    for (int i = 0; i < 3; ++i) {
      const double f = std::sqrt(lam[i] > tol ? 1.0 / lam[i] : 1.0 / tol);
      for (int k = 0; k < 3; ++k) Vsqrt(k, i) = Ev(k, i) * f;
    }
    H00_ += H00;
    b0_ += b0;
    const Mat<6, 3> M = H01 * Vsqrt;
    mH += M * M.T();
    mb += M * (Vsqrt.T() * b1);
  }
  H00_ = H00_ - mH;
  b0_ = b0_ - mb;
  // J_ and DeltaX_ from the eigen-decomposition of H00_ (:376-385)
  double lam[6];
  Mat<6, 6> Ev;
  jacobiEigen<6>(H00_, lam, Ev);
  const double tol = 1.0e-8 * 6.0 * lam[5];
  Mat<6, 1> Etb = Ev.T() * b0_;
  for (int i = 0; i < 6; ++i) {
    const bool keep = lam[i] > tol;
    const double ds = keep ? std::sqrt(lam[i]) : 0.0;
    for (int k = 0; k < 6; ++k) Jsq[i * 6 + k] = ds * Ev(k, i);
    Etb.a[i] = keep ? Etb.a[i] / lam[i] : 0.0;
  }
  const Mat<6, 1> dxv = Ev * Etb;
  for (int i = 0; i < 6; ++i) deltaX[i] = -dxv.a[i];
  if (relPoseSet) {
    for (int i = 0; i < 7; ++i) linPoint[i] = relPose[i];
  } else {
    for (int i = 0; i < 7; ++i) linPoint[i] = identity[i];
  }
  if (H00out) for (int i = 0; i < 36; ++i) H00out[i] = H00_.a[i];
  if (b0out) for (int i = 0; i < 6; ++i) b0out[i] = b0_.a[i];
}

void relPoseBlockEvaluate(const okvisgpu_problem* p, int i, const double* pose0, const double* pose1, double* r,
                          double* Jmin0, double* Jmin1, double* J0, double* J1) {
  if (p->relpose_kind && p->relpose_kind[i] == 1)
    relativePoseErrorEvaluate(&p->relpose_lin_point[7 * i], &p->relpose_sqrt_info[36 * i], pose0, pose1, r, Jmin0,
                              Jmin1, J0, J1);
  else
    relPoseEvaluate(&p->relpose_delta_x[6 * i], &p->relpose_sqrt_info[36 * i], &p->relpose_lin_point[7 * i], pose0,
                    pose1, r, Jmin0, Jmin1, J0, J1);
}

}  // namespace oracle

extern "C" {

int oracle_twopose_compute(const okvisgpu_twopose_edges* E, double* delta_x, double* sqrt_info, double* lin_point,
                           double* H00, double* b0) {
  if (!E || E->n_edges < 0) return OKVISGPU_ERR_INVALID_ARGUMENT;
  for (int e = 0; e < E->n_edges; ++e)
    oracle::twoPoseCompute(E, e, &delta_x[6 * e], &sqrt_info[36 * e], &lin_point[7 * e], H00 ? &H00[36 * e] : nullptr,
                           b0 ? &b0[6 * e] : nullptr);
  return OKVISGPU_OK;
}

}  // extern "C"
