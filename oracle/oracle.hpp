// oracle.hpp — TEST INFRASTRUCTURE ONLY. CPU restatement of the okvis_ceres hot path (the parity
// oracle and the CPU baseline "port"). Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load liboracle.so; the product library never links it.
//
// Parity status: the cost functors are pinned by the reference's own test properties
// (numeric-vs-analytic Jacobians with jacobiansCorrect semantics, ErrorInterface.cpp:44-163;
// camera round trips, TestPinholeCamera.cpp; convergence thresholds of TestReprojectionError.cpp
// and TestImuError.cpp). The reference ships no golden vectors and cannot be built here (no Eigen,
// no Ceres: SURVEY.md §8c), so the DOGLEG/DENSE_SCHUR solver semantics (ceres-solver, un-vendored
// submodule, version >= 2.1) are restated from Ceres' published algorithm and are
// "parity unpinned" at the per-iterate level.
#pragma once

#include <cstdint>
#include <vector>
#include "oracle_math.hpp"
#include "../include/okvisgpu.h"

namespace oracle {

// ------------------------------------------------------------------ cameras (okvis_cv)
struct Camera {
  int dist;
  double fu, fv, cu, cv;
  double d[8];
};
inline Camera cameraOf(const okvisgpu_camera& k) {
  return Camera{k.distortion, k.fu, k.fv, k.cu, k.cv,
                {k.dist[0], k.dist[1], k.dist[2], k.dist[3], k.dist[4], k.dist[5], k.dist[6], k.dist[7]}};
}
// PinholeCamera<D>::project with point Jacobian (PinholeCamera.hpp:288-366). Returns false when
// |z| < 1e-12 (ProjectionStatus::Invalid before any output is written).
bool cameraProject(const Camera& cam, const V3& p, double kp[2], double J[6] /*2x3 or null*/);
// projectHomogeneous (PinholeCamera.hpp:497-518): projects -head for w<0 without negating J.
bool cameraProjectHomogeneous(const Camera& cam, const V4& hp, double kp[2], double J[8] /*2x4*/);

// ------------------------------------------------------------------ manifolds
// PoseLocalParameterization.cpp:29-107
void posePlus(const double* x, const double* delta, double* x_plus_delta);
void posePlusJacobian(const double* x, double* J /*7x6 row-major*/);
void poseMinusJacobian(const double* x, double* J /*6x7 row-major*/);
// HomogeneousPointLocalParameterization.cpp:27-90
void pointPlus(const double* x, const double* delta, double* x_plus_delta);

// ------------------------------------------------------------------ cost functors
// ReprojectionError<G>::EvaluateWithMinimalJacobians (implementation/ReprojectionError.hpp:71-220).
// jac (ambient): J0 2x7, J1 2x4, J2 2x7; jacMin: 2x6, 2x3, 2x6. Any may be null.
void reprojectionEvaluate(const Camera& cam, const double* meas, const double* sqrtInfo /*2x2*/,
                          const double* pose, const double* hp, const double* extr, double* r,
                          double* J0, double* J1, double* J2, double* J0min, double* J1min,
                          double* J2min);

struct ImuSample {
  long long t;
  double g[3], a[3];
};

// okvis::ceres::ImuError (ImuError.hpp:41-306, ImuError.cpp) with its mutable preintegration state.
class ImuError {
 public:
  okvisgpu_imu_params params;
  std::vector<ImuSample> meas;
  long long t0 = 0, t1 = 0;
  // mutable preintegration state (ImuError.hpp:273-304)
  Quat Delta_q{0, 0, 0, 1};
  M3 C_integral = M3::Zero(), C_doubleintegral = M3::Zero();
  V3 acc_integral = V3::Zero(), acc_doubleintegral = V3::Zero();
  M3 cross = M3::Zero(), dalpha_db_g = M3::Zero(), dv_db_g = M3::Zero(), dp_db_g = M3::Zero();
  Mat<15, 15> P_delta = Mat<15, 15>::Zero();
  Mat<15, 15> dPdsigma[4];
  double sb_ref[9] = {0};
  bool redo = true;
  int redoCounter = 0;
  int lastSteps = 1;
  Mat<15, 15> sqrtInfo = Mat<15, 15>::Zero();

  ImuError();
  int redoPreintegration(const double* sb);                          // ImuError.cpp:258-466
  // ImuError::append (ImuError.cpp:63-255): continue the preintegration from t1 to t_1 over the
  // next link's measurements m with the eliminated state's speed/bias sb (IMU-merge elimination,
  // ViGraphEstimator.cpp:38-171). Returns the integrated steps, -1 if m does not cover t_1.
  int append(const double* sb, const std::vector<ImuSample>& m, long long t_1);
  // ImuError.cpp:797-1003. jac (ambient) J0 15x7, J1 15x9, J2 15x7, J3 15x9; jacMin 15x6,15x9,15x6,15x9.
  bool evaluate(const double* const* params, double* r, double** jac, double** jacMin,
                bool redoAlways);
  void loadState(const double* s);
  void storeState(double* s) const;
};

// PseudoInverse::symmSqrtU (okvis_ceres/include/okvis/PseudoInverse.hpp:132-158) via cyclic Jacobi.
void symmSqrtU(const Mat<15, 15>& a, Mat<15, 15>& result);

// PoseError::EvaluateWithMinimalJacobians (PoseError.cpp:73-125).
void poseErrorEvaluate(const double* meas, const double* sqrtInfo /*6x6*/, const double* pose,
                       double* r, double* J /*6x7 ambient*/, double* Jmin /*6x6*/);
// SpeedAndBiasError::EvaluateWithMinimalJacobians (SpeedAndBiasError.cpp:67-101).
void sbErrorEvaluate(const double* meas, const double* sqrtInfo /*9x9*/, const double* sb,
                     double* r, double* J /*9x9*/);

// TwoPoseStandardGraphError(Const)::EvaluateWithMinimalJacobians (TwoPoseGraphError.cpp:467-606,
// :631-767): dx = DeltaX_ [6], Jsq = J_ [36], lin = linearisationPoint_T_S0S1_ [7]. Jmin0/Jmin1 6x6
// (reference / other pose), J0/J1 ambient 6x7. Any output Jacobian may be null.
void relPoseEvaluate(const double* dx, const double* Jsq, const double* lin, const double* pose0,
                     const double* pose1, double* r, double* Jmin0, double* Jmin1, double* J0, double* J1);
// RelativePoseError::EvaluateWithMinimalJacobians (RelativePoseError.cpp:59-140), twopose.cpp.
void relativePoseErrorEvaluate(const double* Tab, const double* Lsq, const double* pose0, const double* pose1,
                               double* r, double* Jmin0, double* Jmin1, double* J0, double* J1);
// The relative-pose residual block i of a problem: kind 0 graph edge, 1 RelativePoseError.
void relPoseBlockEvaluate(const okvisgpu_problem* p, int i, const double* pose0, const double* pose1, double* r,
                          double* Jmin0, double* Jmin1, double* J0, double* J1);
// TwoPoseStandardGraphError::compute (TwoPoseGraphError.cpp:162-397) of edge e (twopose.cpp).
void twoPoseCompute(const okvisgpu_twopose_edges* E, int e, double* deltaX, double* Jsq, double* linPoint,
                    double* H00, double* b0);

}  // namespace oracle

// ------------------------------------------------------------------ C API (ctypes)
extern "C" {
int oracle_solve(const okvisgpu_problem* p, const okvisgpu_options* o, okvisgpu_summary* s);
int oracle_evaluate(const okvisgpu_problem* p, double* cost);
int oracle_linearize_reduce(const okvisgpu_problem* p, int32_t jacobi_scaling, double mu, double* S,
                            double* rhs, double* cost, int32_t* dim_out);
int oracle_eval_reprojection(const okvisgpu_problem* p, double* r, double* Jp, double* Jl);
int oracle_eval_imu(const okvisgpu_problem* p, int32_t redo_always, double* r, double* J);
/* numeric-vs-analytic Jacobian check with jacobiansCorrect semantics (ErrorInterface.cpp:44-163):
 * kind 0 = reprojection obs, 1 = imu factor, 2 = pose prior, 3 = sb prior, 4 = relative pose. Returns the max over
 * parameter blocks of ||Ja - Jn||_F / min(||Ja||_F, ||Jn||_F) in max_rel. */
int oracle_check_jacobians(const okvisgpu_problem* p, int32_t kind, int32_t index, double delta,
                           double* max_rel);
int oracle_eval_relpose(const okvisgpu_problem* p, double* r, double* J /*[n][6][12] minimal*/);
/* host-evaluated factors (ABI 5), no loss: r [n][15], J [n][15][30] minimal in the IMU column layout */
int oracle_eval_host(const okvisgpu_problem* p, double* r, double* J);
/* IMU-merge elimination of the state between factors f and f+1 (ViGraphEstimator.cpp:38-171):
 * factor f's ImuError (its state from p->imu_state, integrated first if never integrated) appended
 * with factor f+1's measurements up to its t1 at the speed/bias sb (ImuError::append,
 * ImuError.cpp:63-255). Writes the merged state [OKVISGPU_IMU_STATE_DOUBLES]; returns the steps. */
int oracle_imu_merge(const okvisgpu_problem* p, int32_t f, const double* sb, double* state_out);
int oracle_twopose_compute(const okvisgpu_twopose_edges* E, double* delta_x, double* sqrt_info, double* lin_point,
                           double* H00, double* b0);
/* okvisgpu_imu_append on the CPU: same batch, same in/out state layout, steps[n] (-1 untouched). */
int oracle_imu_append(const okvisgpu_imu_append_batch* b, int32_t* steps);
int oracle_project(const okvisgpu_camera* cam, const double* hp4, double* kp2, double* J24);
void oracle_pose_plus(const double* x, const double* delta, double* out);
void oracle_pose_plus_jacobian(const double* x, double* J76);
void oracle_pose_minus_jacobian(const double* x, double* J67);
int oracle_dense_cholesky(int32_t n, double* A, int32_t num_threads); /* lower, in place; 0 = ok */
/* ::ceres::LossFunction::Evaluate restated (rho, rho', rho''), okvisgpu_loss_kind */
int oracle_loss_evaluate(const okvisgpu_loss* loss, double s, double* rho);
/* Ceres' Corrector on one residual block: r [nres] and J [nres][ncols] (may be NULL) corrected in
 * place, cost = rho(|r|^2)/2 */
int oracle_loss_correct(const okvisgpu_loss* loss, int32_t nres, int32_t ncols, double* r, double* J, double* cost);
}
