// C++ consumer of the okvisgpu::Problem facade (include/okvisgpu_problem.hpp), compiled with g++
// only. It drives the facade the way okvis drives ::ceres::Problem (ViGraph.cpp:327-385,433-459,
// 597-637; ViGraphEstimator.cpp:216-331): parameter blocks with manifolds, typeInfo()-recognised
// residual blocks, freeze / unfreeze, removal, ::ceres::Solve.
//   facade_test cpu  bookkeeping, graph flattening and error paths (no GPU needed)
//   facade_test gpu  the TestReprojectionError.cpp:48-164 scene through the facade (its thresholds),
//                    and an S10 window through the facade vs the same window through the C ABI
//                    directly (also after a freeze between solves)
#include <algorithm>
#include <array>
#include <cmath>
#include <memory>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "okvisgpu.h"
#include "okvisgpu_problem.hpp"

static int g_fail = 0;
#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                            \
    }                                                                      \
  } while (0)

namespace {

struct Quat { double x, y, z, w; };
Quat qmul(Quat a, Quat b) {
  return {a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
          a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
void rot(Quat q, double R[9]) {
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  const double x = q.x / n, y = q.y / n, z = q.z / n, w = q.w / n;
  const double r[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                       2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                       2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
  for (int i = 0; i < 9; ++i) R[i] = r[i];
}
struct Pose { double t[3]; Quat q; };
// Transformation::setRandom (Transformation.hpp:199-208), Random() uniform in [-1, 1]
Pose setRandom(std::mt19937_64& g, double tmax, double rmax) {
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  double a[3] = {rmax * U(g), rmax * U(g), rmax * U(g)};
  Pose p;
  for (double& v : p.t) v = tmax * U(g);
  const double ang = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  const double s = std::sin(ang / 2) / ang;
  p.q = {a[0] * s, a[1] * s, a[2] * s, std::cos(ang / 2)};
  return p;
}
Pose compose(const Pose& A, const Pose& B) {
  double R[9];
  rot(A.q, R);
  Pose o;
  for (int i = 0; i < 3; ++i) o.t[i] = A.t[i] + R[3 * i] * B.t[0] + R[3 * i + 1] * B.t[1] + R[3 * i + 2] * B.t[2];
  o.q = qmul(A.q, B.q);
  return o;
}
void toArray(const Pose& p, double* a) {
  a[0] = p.t[0]; a[1] = p.t[1]; a[2] = p.t[2]; a[3] = p.q.x; a[4] = p.q.y; a[5] = p.q.z; a[6] = p.q.w;
}
double rotErr(Quat a, Quat b) {  // 2 |vec(a b^-1)|
  const Quat d = qmul(a, Quat{-b.x, -b.y, -b.z, b.w});
  return 2 * std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
}

// Stand-ins with the member names (and defaults) of ceres::Solver::Options / Summary that okvis
// uses (Ceres is not in this image): the ::ceres::Solve-shaped facade call is a template over them.
enum class CeresLikeTermination { CONVERGENCE, NO_CONVERGENCE, FAILURE, USER_SUCCESS, USER_FAILURE };
struct CeresLikeOptions {
  int max_num_iterations = 50, num_threads = 1, max_num_consecutive_invalid_steps = 5;
  bool jacobi_scaling = true, minimizer_progress_to_stdout = false;
  double function_tolerance = 1e-6, gradient_tolerance = 1e-10, parameter_tolerance = 1e-8;
  double initial_trust_region_radius = 1e4, max_trust_region_radius = 1e16, min_trust_region_radius = 1e-32;
  double min_relative_decrease = 1e-3, min_lm_diagonal = 1e-6, max_lm_diagonal = 1e32;
};
struct CeresLikeSummary {
  double initial_cost = -1, final_cost = -1, total_time_in_seconds = -1;
  double preprocessor_time_in_seconds = -2, minimizer_time_in_seconds = -2, postprocessor_time_in_seconds = -2;
  double linear_solver_time_in_seconds = -2, residual_evaluation_time_in_seconds = -2,
         jacobian_evaluation_time_in_seconds = -2;
  int num_successful_steps = -1, num_unsuccessful_steps = -1;
  CeresLikeTermination termination_type = CeresLikeTermination::FAILURE;
};

okvisgpu_options zeroTol(int iters) {
  okvisgpu_options o;
  okvisgpu_default_options(&o);
  o.max_num_iterations = iters;
  o.function_tolerance = o.gradient_tolerance = o.parameter_tolerance = 0.0;
  return o;
}

// a cost function the GPU path does not know and that is no HostCostFunction either
struct OtherError final : okvisgpu::CostFunction {
  std::string typeInfo() const override { return "GpsErrorSynchronous"; }
  int residualDim() const override { return 3; }
  std::vector<int> parameterBlockSizes() const override { return {7}; }
};

void skew(const double v[3], double S[9]) {
  S[0] = 0; S[1] = -v[2]; S[2] = v[1]; S[3] = v[2]; S[4] = 0; S[5] = -v[0]; S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
// PoseManifold lift Jacobian (6x7, PoseLocalParameterization.cpp:89-103): I3 | 2 oplus(q^-1)_{0:3,:}
void liftJacobian(const double* T, double L[42]) {
  for (int i = 0; i < 42; ++i) L[i] = 0.0;
  L[0] = L[8] = L[16] = 1.0;
  const double x = -T[3], y = -T[4], z = -T[5], w = T[6];
  const double Q[3][4] = {{w, z, -y, x}, {-z, w, x, y}, {y, -x, w, z}};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) L[(3 + r) * 7 + 3 + c] = 2.0 * Q[r][c];
}

// A ceres::SizedCostFunction<3, 7, 9, 7>-shaped functor with okvis' GpsErrorAsynchronous block
// layout (GpsErrorAsynchronous.hpp:42-55): pose T_WS, speed/bias, alignment T_GW;
// r = (p_meas - (R_GW (r_WS + v dt + R_WS r_SA) + r_GW)) / sigma, ambient Jacobians = minimal x lift
// (how okvis' functors produce them). Used through okvisgpu::HostFunctor<GpsFunctor>.
struct GpsFunctor {
  double meas[3] = {0, 0, 0}, dt = 0.02, r_SA[3] = {0.05, -0.02, 0.1}, sigma = 0.05;
  std::vector<int32_t> sizes{7, 9, 7};
  std::string typeInfo() const { return "GpsErrorAsynchronous"; }
  int num_residuals() const { return 3; }
  const std::vector<int32_t>& parameter_block_sizes() const { return sizes; }
  void predict(const double* T, const double* sb, const double* G, double pG[3], double a[3], double pW[3],
               double RG[9]) const {
    double RS[9];
    rot(Quat{T[3], T[4], T[5], T[6]}, RS);
    rot(Quat{G[3], G[4], G[5], G[6]}, RG);
    for (int i = 0; i < 3; ++i) a[i] = RS[3 * i] * r_SA[0] + RS[3 * i + 1] * r_SA[1] + RS[3 * i + 2] * r_SA[2];
    for (int i = 0; i < 3; ++i) pW[i] = T[i] + sb[i] * dt + a[i];
    for (int i = 0; i < 3; ++i) pG[i] = RG[3 * i] * pW[0] + RG[3 * i + 1] * pW[1] + RG[3 * i + 2] * pW[2] + G[i];
  }
  bool Evaluate(double const* const* p, double* r, double** J) const {
    double pG[3], a[3], pW[3], RG[9];
    predict(p[0], p[1], p[2], pG, a, pW, RG);
    const double s = 1.0 / sigma;
    for (int i = 0; i < 3; ++i) r[i] = s * (meas[i] - pG[i]);
    if (!J) return true;
    double Sa[9], RSa[9], g[3], Sg[9];
    skew(a, Sa);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) RSa[3 * i + j] = RG[3 * i] * Sa[j] + RG[3 * i + 1] * Sa[3 + j] + RG[3 * i + 2] * Sa[6 + j];
    for (int i = 0; i < 3; ++i) g[i] = RG[3 * i] * pW[0] + RG[3 * i + 1] * pW[1] + RG[3 * i + 2] * pW[2];
    skew(g, Sg);
    double Jt[18], Jg[18];  // minimal 3x6
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        Jt[6 * i + j] = -s * RG[3 * i + j];
        Jt[6 * i + 3 + j] = s * RSa[3 * i + j];
        Jg[6 * i + j] = i == j ? -s : 0.0;
        Jg[6 * i + 3 + j] = s * Sg[3 * i + j];
      }
    const double* mins[3] = {Jt, nullptr, Jg};
    for (int k = 0; k < 3; k += 2) {
      if (!J[k]) continue;
      double L[42];
      liftJacobian(p[k], L);
      for (int i = 0; i < 3; ++i)
        for (int c = 0; c < 7; ++c) {
          double v = 0;
          for (int m = 0; m < 6; ++m) v += mins[k][6 * i + m] * L[m * 7 + c];
          J[k][7 * i + c] = v;
        }
    }
    if (J[1])
      for (int i = 0; i < 3; ++i)
        for (int c = 0; c < 9; ++c) J[1][9 * i + c] = c < 3 ? -s * RG[3 * i + c] * dt : 0.0;
    return true;
  }
};

// okvis-shaped functor getters for the fromOkvis* adapters (Eigen-like call operators)
struct Vec { double v[3]; double operator()(int i) const { return v[i]; } };
struct Mat2 { double m[4]; double operator()(int r, int c) const { return m[2 * r + c]; } };
struct MockReprojection {
  Vec meas{{310.5, 120.25, 0}};
  Mat2 info{{4.0, 1.0, 1.0, 9.0}};
  const Vec& measurement() const { return meas; }
  const Mat2& information() const { return info; }
};
// Records an okvisgpu_problem (e.g. a synthetic window) into a facade, block by block and residual
// by residual, the way ViGraph adds them; parameter memory = the problem's own arrays.
struct Recorded {
  okvisgpu::PoseManifold poseManifold;
  okvisgpu::HomogeneousPointManifold pointManifold;
  okvisgpu::CauchyLoss cauchy{1.0};
  std::vector<std::unique_ptr<okvisgpu::CostFunction>> costs;
  std::vector<okvisgpu::ResidualBlockId> ids;  // in the order recorded: observations, IMU, priors
};

void record(okvisgpu::Problem& P, const okvisgpu_problem* p, Recorded& R) {
  for (int i = 0; i < p->n_poses; ++i) {
    P.AddParameterBlock(&p->poses[7 * i], 7, &R.poseManifold);
    if (p->pose_constant && p->pose_constant[i]) P.SetParameterBlockConstant(&p->poses[7 * i]);
  }
  for (int i = 0; i < p->n_speed_biases; ++i) {
    P.AddParameterBlock(&p->speed_biases[9 * i], 9);
    if (p->speed_bias_constant && p->speed_bias_constant[i]) P.SetParameterBlockConstant(&p->speed_biases[9 * i]);
  }
  for (int c = 0; c < p->n_cameras; ++c) {
    P.AddParameterBlock(&p->extrinsics[7 * c], 7, &R.poseManifold);
    P.SetParameterBlockConstant(&p->extrinsics[7 * c]);  // do_extrinsics: false (ViGraph.cpp:385)
  }
  for (int l = 0; l < p->n_landmarks; ++l) {
    P.AddParameterBlock(&p->landmarks[4 * l], 4, &R.pointManifold);
    if (p->landmark_constant && p->landmark_constant[l]) P.SetParameterBlockConstant(&p->landmarks[4 * l]);
  }
  for (int o = 0; o < p->n_observations; ++o) {
    const int c = p->obs_camera[o];
    R.costs.emplace_back(new okvisgpu::ReprojectionError(p->cameras[c], &p->obs_keypoint[2 * o], &p->obs_sqrt_info[4 * o]));
    R.ids.push_back(P.AddResidualBlock(R.costs.back().get(), (!p->obs_cauchy || p->obs_cauchy[o]) ? &R.cauchy : nullptr,
                                       &p->poses[7 * p->obs_pose[o]], &p->landmarks[4 * p->obs_landmark[o]],
                                       &p->extrinsics[7 * c]));
  }
  for (int f = 0; f < p->n_imu; ++f) {
    const int s0 = p->imu_sample_begin[f], s1 = p->imu_sample_begin[f + 1];
    std::vector<int64_t> ts(p->imu_sample_t_ns + s0, p->imu_sample_t_ns + s1);
    std::vector<double> ga(p->imu_sample_gyr_acc + 6 * s0, p->imu_sample_gyr_acc + 6 * s1);
    auto* e = new okvisgpu::ImuError(ts, ga, p->imu_params, p->imu_t0_ns[f], p->imu_t1_ns[f]);
    R.costs.emplace_back(e);
    const int* b = &p->imu_blocks[4 * f];
    R.ids.push_back(P.AddResidualBlock(e, nullptr, &p->poses[7 * b[0]], &p->speed_biases[9 * b[1]],
                                       &p->poses[7 * b[2]], &p->speed_biases[9 * b[3]]));
  }
  for (int i = 0; i < p->n_pose_priors; ++i) {
    R.costs.emplace_back(new okvisgpu::PoseError(&p->pose_prior_meas[7 * i], &p->pose_prior_sqrt_info[36 * i]));
    P.AddResidualBlock(R.costs.back().get(), nullptr, &p->poses[7 * p->pose_prior_block[i]]);
  }
  for (int i = 0; i < p->n_sb_priors; ++i) {
    R.costs.emplace_back(new okvisgpu::SpeedAndBiasError(&p->sb_prior_meas[9 * i], &p->sb_prior_sqrt_info[81 * i]));
    P.AddResidualBlock(R.costs.back().get(), nullptr, &p->speed_biases[9 * p->sb_prior_block[i]]);
  }
}

int cpuTests() {
  okvisgpu::Problem P;
  okvisgpu::PoseManifold pm;
  okvisgpu::HomogeneousPointManifold hm;
  okvisgpu::CauchyLoss cauchy(1.0);
  double T0[7] = {0, 0, 0, 0, 0, 0, 1}, T1[7] = {1, 0, 0, 0, 0, 0, 1}, Tsc[7] = {0, 0, 0, 0, 0, 0, 1};
  double sb0[9] = {0}, sb1[9] = {0};
  double L0[4] = {0, 0, 5, 1}, L1[4] = {1, 1, 6, 1};
  P.AddParameterBlock(T0, 7, &pm);
  P.AddParameterBlock(sb0, 9);
  P.AddParameterBlock(T1, 7, &pm);
  P.AddParameterBlock(sb1, 9);
  P.AddParameterBlock(Tsc, 7, &pm);
  P.SetParameterBlockConstant(Tsc);
  P.AddParameterBlock(L0, 4, &hm);
  P.AddParameterBlock(L1, 4, &hm);
  P.AddParameterBlock(L1, 4);  // re-adding is a no-op (Ceres)
  CHECK(P.NumParameterBlocks() == 7);
  CHECK(P.HasParameterBlock(T0) && !P.HasParameterBlock(T0 + 1));
  CHECK(P.IsParameterBlockConstant(Tsc) && !P.IsParameterBlockConstant(T1));
  CHECK(P.GetManifold(L0) == &hm && P.GetManifold(sb0) == nullptr);
  okvisgpu_camera cam{};
  cam.distortion = OKVISGPU_DIST_NONE;
  cam.width = 752; cam.height = 480; cam.fu = 350; cam.fv = 360; cam.cu = 378; cam.cv = 238;
  const double kp[2] = {378, 238}, Li[4] = {1, 0, 0, 1};
  okvisgpu::ReprojectionError e00(cam, kp, Li), e01(cam, kp, Li), e10(cam, kp, Li);
  auto r00 = P.AddResidualBlock(&e00, &cauchy, T0, L0, Tsc);
  auto r01 = P.AddResidualBlock(&e01, &cauchy, T0, L1, Tsc);
  auto r10 = P.AddResidualBlock(&e10, &cauchy, T1, L0, Tsc);
  std::vector<int64_t> ts = {0, 5000000, 10000000};
  std::vector<double> ga(18, 0.0);
  okvisgpu_imu_params ip{};
  okvisgpu::ImuError imu(ts, ga, ip, 1000000, 9000000);
  auto rimu = P.AddResidualBlock(&imu, nullptr, T0, sb0, T1, sb1);
  const double pm7[7] = {0, 0, 0, 0, 0, 0, 1}, pL[36] = {0};
  okvisgpu::PoseError prior(pm7, pL), extrPrior(pm7, pL);
  P.AddResidualBlock(&prior, nullptr, T0);
  P.AddResidualBlock(&extrPrior, nullptr, Tsc);
  CHECK(P.NumResidualBlocks() == 6);
  std::vector<double*> blocks;
  P.GetParameterBlocksForResidualBlock(rimu, &blocks);
  CHECK(blocks.size() == 4 && blocks[0] == T0 && blocks[3] == sb1);
  std::vector<okvisgpu::ResidualBlockId> rs;
  P.GetResidualBlocksForParameterBlock(L0, &rs);
  CHECK(rs.size() == 2 && rs[0] == r00 && rs[1] == r10);
  CHECK(P.GetCostFunctionForResidualBlock(r01) == &e01 && P.GetLossFunctionForResidualBlock(rimu) == nullptr);
  // the flattened C-ABI problem: Tsc is an extrinsics block (third block of a reprojection), not a pose
  const okvisgpu_problem& v = P.view();
  CHECK(v.n_poses == 2 && v.n_speed_biases == 2 && v.n_landmarks == 2 && v.n_cameras == 1);
  CHECK(v.n_observations == 3 && v.n_imu == 1 && v.n_pose_priors == 1 && v.n_extrinsics_priors == 1);
  CHECK(v.obs_pose[2] == 1 && v.obs_landmark[1] == 1 && v.obs_cauchy[0] == 1 && v.extrinsics_constant[0] == 1);
  CHECK(v.imu_blocks[0] == 0 && v.imu_blocks[1] == 0 && v.imu_blocks[2] == 1 && v.imu_blocks[3] == 1);
  CHECK(v.imu_sample_begin[1] == 3 && v.imu_t1_ns[0] == 9000000);
  // §8b host fallback: a ceres-shaped functor through HostFunctor<F> keeps its call site; the view
  // carries its blocks (functor order, extrinsics as pose-kind n_poses + camera) and a trampoline
  // that reaches the functor
  {
    GpsFunctor f;
    bool hthrew = false;
    okvisgpu::HostFunctor<GpsFunctor> hf(&f);
    CHECK(hf.typeInfo() == "GpsErrorAsynchronous" && hf.residualDim() == 3 && hf.parameterBlockSizes().size() == 3);
    auto rg = P.AddResidualBlock(&hf, nullptr, T0, sb0, Tsc);
    const okvisgpu_problem& w = P.view();
    CHECK(w.n_host == 1 && w.host_dim[0] == 3 && w.host_cauchy == nullptr && w.host_loss[0].kind == OKVISGPU_LOSS_NONE);
    CHECK(w.host_param_kind[0] == 0 && w.host_param_kind[1] == 1 && w.host_param_kind[2] == 0 && w.host_param_kind[3] == -1);
    CHECK(w.host_param_index[0] == 0 && w.host_param_index[1] == 0 && w.host_param_index[2] == w.n_poses);
    const double* prm[3] = {T0, sb0, Tsc};
    double r1[3], r2[3], Ja[21], Jb[27], Jc[21];
    double* jac[3] = {Ja, Jb, Jc};
    CHECK(w.host_evaluate(w.host_user, 0, prm, r1, jac) == 1);
    f.Evaluate(prm, r2, nullptr);
    CHECK(r1[0] == r2[0] && r1[1] == r2[1] && r1[2] == r2[2]);
    // EvaluateResidualBlock (ViGraph.hpp:553) of a host term: on the host, raw without a loss
    double ec = -1, er[3];
    CHECK(P.EvaluateResidualBlock(rg, true, &ec, er, nullptr));
    CHECK(er[0] == r2[0] && er[1] == r2[1] && er[2] == r2[2]);
    CHECK(std::fabs(ec - 0.5 * (r2[0] * r2[0] + r2[1] * r2[1] + r2[2] * r2[2])) <= 1e-15 * ec);
    P.RemoveResidualBlock(rg);
    CHECK(P.view().n_host == 0);
    // the fallback's limits: no landmark block, at most 2 pose-kind blocks
    struct LmHost final : okvisgpu::HostCostFunction {
      int residualDim() const override { return 1; }
      std::vector<int> parameterBlockSizes() const override { return {7, 4}; }
      bool Evaluate(double const* const*, double*, double**) const override { return true; }
    } lmh;
    struct ThreePoses final : okvisgpu::HostCostFunction {
      int residualDim() const override { return 6; }
      std::vector<int> parameterBlockSizes() const override { return {7, 7, 7}; }
      bool Evaluate(double const* const*, double*, double**) const override { return true; }
    } tp;
    hthrew = false;
    try { P.AddResidualBlock(&lmh, nullptr, T1, L1); } catch (const okvisgpu::Unsupported&) { hthrew = true; }
    CHECK(hthrew);
    hthrew = false;
    try { P.AddResidualBlock(&tp, nullptr, T0, T1, Tsc); } catch (const okvisgpu::Unsupported&) { hthrew = true; }
    CHECK(hthrew);
  }
  // okvis functors through their getters (ReprojectionErrorBase.hpp:75-91)
  {
    const MockReprojection mr;
    const okvisgpu::ReprojectionError re = okvisgpu::fromOkvisReprojectionError(mr, cam);
    CHECK(re.keypoint[0] == 310.5 && re.keypoint[1] == 120.25);
    const double* U = re.sqrt_info;  // U^T U = information, U upper triangular
    CHECK(U[2] == 0.0 && std::fabs(U[0] * U[0] - 4.0) < 1e-15 && std::fabs(U[0] * U[1] - 1.0) < 1e-15 &&
          std::fabs(U[1] * U[1] + U[3] * U[3] - 9.0) < 1e-14);
    // (fromOkvisImuError also reads the protected preintegration state: okvis_roundtrip.cpp, against
    // stand-ins with okvis' member layout)
  }
  // removal (RemoveParameterBlock drops its residual blocks too)
  P.RemoveResidualBlock(r01);
  CHECK(P.NumResidualBlocks() == 5);
  P.RemoveParameterBlock(L0);
  CHECK(P.NumResidualBlocks() == 3 && !P.HasParameterBlock(L0));
  CHECK(P.view().n_observations == 0 && P.view().n_landmarks == 1);
  // unknown functor -> Unsupported (OKVISGPU_ERR_UNSUPPORTED); wrong block -> Error
  OtherError gps;
  bool threw = false;
  try { P.AddResidualBlock(&gps, nullptr, T0); } catch (const okvisgpu::Unsupported& u) { threw = u.status() == OKVISGPU_ERR_UNSUPPORTED; }
  CHECK(threw);
  threw = false;
  try { P.AddResidualBlock(&prior, nullptr, sb0); } catch (const okvisgpu::Error&) { threw = true; }
  CHECK(threw);
  // the four losses ViGraph's constructor builds (ViGraph.cpp:235-238), ::ceres::LossFunction::Evaluate
  {
    okvisgpu::CauchyLoss cauchyLoss(1.0), cauchyGpsLoss(3.0);
    okvisgpu::TukeyLoss tukeyDepthLoss(0.1), tukeyLidarLoss(2.0);
    double rho[3];
    cauchyGpsLoss.Evaluate(9.0, rho);  // b log(1 + s/b), b = 9
    CHECK(std::fabs(rho[0] - 9.0 * std::log(2.0)) < 1e-14 && std::fabs(rho[1] - 0.5) < 1e-15 &&
          std::fabs(rho[2] + 1.0 / 36.0) < 1e-15);
    cauchyLoss.Evaluate(3.0, rho);
    CHECK(std::fabs(rho[0] - std::log(4.0)) < 1e-15 && rho[1] == 0.25);
    tukeyLidarLoss.Evaluate(1.0, rho);  // a^2/3 (1 - (1 - s/a^2)^3), rho' = (1 - s/a^2)^2
    CHECK(std::fabs(rho[0] - 4.0 / 3.0 * (1.0 - 27.0 / 64.0)) < 1e-15 && rho[1] == 0.5625 && rho[2] == -0.375);
    tukeyLidarLoss.Evaluate(5.0, rho);  // outlier: constant cost, no gradient
    CHECK(std::fabs(rho[0] - 4.0 / 3.0) < 1e-15 && rho[1] == 0.0 && rho[2] == 0.0);
    tukeyDepthLoss.Evaluate(0.02, rho);
    CHECK(rho[1] == 0.0 && std::fabs(rho[0] - 0.01 / 3.0) < 1e-17);
    CHECK(std::string(tukeyLidarLoss.name()) == "TukeyLoss" && cauchyGpsLoss.a() == 3.0);
    // reprojections take CauchyLoss(1.0) only (the device's); host factors take any of them
    okvisgpu::Problem Q;
    double Ta[7] = {0, 0, 0, 0, 0, 0, 1}, Tb[7] = {1, 0, 0, 0, 0, 0, 1}, Ex[7] = {0, 0, 0, 0, 0, 0, 1};
    double La[4] = {0, 0, 5, 1}, sa[9] = {};
    Q.AddParameterBlock(Ta, 7, &pm);
    Q.AddParameterBlock(Tb, 7, &pm);
    Q.AddParameterBlock(Ex, 7, &pm);
    Q.AddParameterBlock(La, 4, &hm);
    okvisgpu::ReprojectionError ea(cam, kp, Li);
    threw = false;
    try { Q.AddResidualBlock(&ea, &cauchyGpsLoss, Ta, La, Ex); } catch (const okvisgpu::Unsupported&) { threw = true; }
    CHECK(threw);
    Q.AddResidualBlock(&ea, &cauchyLoss, Ta, La, Ex);
    GpsFunctor g;
    okvisgpu::HostFunctor<GpsFunctor> hg(&g);
    struct SubmapLike final : okvisgpu::HostCostFunction {  // SubmapIcpError's blocks: (pose A, pose B)
      int residualDim() const override { return 1; }
      std::vector<int> parameterBlockSizes() const override { return {7, 7}; }
      bool Evaluate(double const* const*, double* r, double**) const override { r[0] = 0.0; return true; }
    } sm;
    Q.AddResidualBlock(&hg, &cauchyGpsLoss, Ta, sa, Ex);
    Q.AddResidualBlock(&sm, &tukeyLidarLoss, Ta, Tb);
    Q.AddResidualBlock(&sm, &tukeyDepthLoss, Ta, Tb);
    const okvisgpu_problem& v = Q.view();
    CHECK(v.n_host == 3 && v.host_loss[0].kind == OKVISGPU_LOSS_CAUCHY && v.host_loss[0].a == 3.0);
    CHECK(v.host_loss[1].kind == OKVISGPU_LOSS_TUKEY && v.host_loss[1].a == 2.0 && v.host_loss[2].a == 0.1);
    CHECK(v.obs_cauchy[0] == 1);
    threw = false;
    try { okvisgpu::TukeyLoss bad(-1.0); (void)bad; } catch (const okvisgpu::Error&) { threw = true; }
    CHECK(threw);
    // EvaluateResidualBlock with the loss applied (Ceres' Corrector on r): CauchyLoss(3) on the GPS
    // term, cost b log(1 + s/b), r scaled by sqrt(rho')
    {
      const double* prm[3] = {Ta, sa, Ex};
      double raw[3], ec = -1, er[3];
      g.Evaluate(prm, raw, nullptr);
      const double sq = raw[0] * raw[0] + raw[1] * raw[1] + raw[2] * raw[2];
      std::vector<okvisgpu::ResidualBlockId> ids;
      Q.GetResidualBlocksForParameterBlock(sa, &ids);
      CHECK(ids.size() == 1 && Q.EvaluateResidualBlock(ids[0], true, &ec, er, nullptr));
      CHECK(std::fabs(ec - 0.5 * 9.0 * std::log1p(sq / 9.0)) <= 1e-14 * ec);
      const double sc = 1.0 / std::sqrt(1.0 + sq / 9.0);
      CHECK(std::fabs(er[0] - raw[0] * sc) <= 1e-15 * std::fabs(raw[0]) + 1e-300);
      CHECK(Q.EvaluateResidualBlock(ids[0], false, &ec, er, nullptr) && er[1] == raw[1] && ec == 0.5 * sq);
      threw = false;
      double* jac[3] = {nullptr, nullptr, nullptr};
      try { Q.EvaluateResidualBlock(ids[0], false, &ec, er, jac); } catch (const okvisgpu::Unsupported&) { threw = true; }
      CHECK(threw);
    }
  }
  // one VARIABLE extrinsics block seen with two different intrinsics would become two independent
  // ABI blocks: rejected (a constant one is fine: two ABI cameras sharing the same constant T_SC)
  {
    okvisgpu::Problem Q;
    double Ta[7] = {0, 0, 0, 0, 0, 0, 1}, Ex[7] = {0, 0, 0, 0, 0, 0, 1}, La[4] = {0, 0, 5, 1};
    Q.AddParameterBlock(Ta, 7, &pm);
    Q.AddParameterBlock(Ex, 7, &pm);
    Q.AddParameterBlock(La, 4, &hm);
    okvisgpu_camera cam2 = cam;
    cam2.fu = 351;
    okvisgpu::ReprojectionError ea(cam, kp, Li), eb(cam2, kp, Li);
    Q.AddResidualBlock(&ea, &cauchy, Ta, La, Ex);
    Q.AddResidualBlock(&eb, &cauchy, Ta, La, Ex);
    Q.SetParameterBlockConstant(Ex);
    CHECK(Q.view().n_cameras == 2);
    Q.SetParameterBlockVariable(Ex);
    threw = false;
    try { (void)Q.view(); } catch (const okvisgpu::Unsupported&) { threw = true; }
    CHECK(threw);
  }
  // ::ceres::Solve-shaped call: the ceres::Solver::Options / Summary member names okvis uses
  {
    CeresLikeOptions co;
    co.max_num_iterations = 7;
    co.num_threads = 3;
    co.function_tolerance = 1e-3;
    co.minimizer_progress_to_stdout = true;
    const okvisgpu_options o = okvisgpu::toOptions(co, false, 0.05, 2);
    okvisgpu_options d;
    okvisgpu_default_options(&d);
    CHECK(o.max_num_iterations == 7 && o.num_threads == 3 && o.function_tolerance == 1e-3 && o.verbose == 1);
    CHECK(o.linear_solver == OKVISGPU_SPARSE_NORMAL_CHOLESKY && o.trust_region_strategy == OKVISGPU_DOGLEG);
    CHECK(o.time_limit_s == 0.05 && o.min_iterations == 2);
    // every other field keeps the Ceres default the mock carries (= the C ABI's defaults)
    CHECK(o.gradient_tolerance == d.gradient_tolerance && o.parameter_tolerance == d.parameter_tolerance);
    CHECK(o.initial_trust_region_radius == d.initial_trust_region_radius &&
          o.max_trust_region_radius == d.max_trust_region_radius &&
          o.min_trust_region_radius == d.min_trust_region_radius);
    CHECK(o.min_relative_decrease == d.min_relative_decrease && o.min_lm_diagonal == d.min_lm_diagonal &&
          o.max_lm_diagonal == d.max_lm_diagonal && o.jacobi_scaling == d.jacobi_scaling &&
          o.max_num_consecutive_invalid_steps == d.max_num_consecutive_invalid_steps);
    okvisgpu_summary s{};
    s.initial_cost = 3.0; s.final_cost = 1.0; s.num_successful_steps = 4; s.num_unsuccessful_steps = 2;
    s.termination_type = OKVISGPU_USER_SUCCESS; s.total_time_s = 0.5;
    s.preprocessor_time_s = 0.1; s.minimizer_time_s = 0.3; s.postprocessor_time_s = 0.1;
    s.linear_solver_time_s = 0.2; s.residual_evaluation_time_s = 0.04; s.jacobian_evaluation_time_s = 0.05;
    CeresLikeSummary cs;
    okvisgpu::toSummary(s, &cs);
    CHECK(cs.initial_cost == 3.0 && cs.final_cost == 1.0 && cs.num_successful_steps == 4 &&
          cs.num_unsuccessful_steps == 2 && cs.termination_type == CeresLikeTermination::USER_SUCCESS &&
          cs.total_time_in_seconds == 0.5);
    CHECK(cs.preprocessor_time_in_seconds == 0.1 && cs.minimizer_time_in_seconds == 0.3 &&
          cs.postprocessor_time_in_seconds == 0.1 && cs.linear_solver_time_in_seconds == 0.2 &&
          cs.residual_evaluation_time_in_seconds == 0.04 && cs.jacobian_evaluation_time_in_seconds == 0.05);
  }
  // no device in this container: Solve reports the C ABI's status instead of crashing
  int32_t ndev = 0;
  okvisgpu_device_count(&ndev);
  if (ndev == 0) {
    okvisgpu_summary s;
    CHECK(P.Solve(zeroTol(2), &s) == OKVISGPU_ERR_DEVICE);
    CeresLikeSummary cs;
    CHECK(okvisgpu::Solve(CeresLikeOptions{}, &P, &cs) == OKVISGPU_ERR_DEVICE);
  }
  std::printf("facade_test cpu %s\n", g_fail ? "FAILED" : "ok");
  return g_fail ? 1 : 0;
}

// TestReprojectionError.cpp:48-164 through the facade
int reprojectionScene(uint64_t seed) {
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  const Pose T_WS = setRandom(g, 10.0, M_PI);
  const Pose T_dist = setRandom(g, 1.0, 0.01);
  const Pose T_SC = setRandom(g, 0.2, M_PI);
  double pose[7], extr[7];
  toArray(compose(T_WS, T_dist), pose);
  toArray(T_SC, extr);
  okvisgpu::Problem P;
  okvisgpu::PoseManifold pm;
  okvisgpu::HomogeneousPointManifold hm;
  P.AddParameterBlock(pose, 7, &pm);
  P.AddParameterBlock(extr, 7, &pm);
  P.SetParameterBlockVariable(pose);
  P.SetParameterBlockConstant(extr);
  okvisgpu_camera cam{};
  cam.distortion = OKVISGPU_DIST_NONE;
  cam.width = 752; cam.height = 480; cam.fu = 350; cam.fv = 360; cam.cu = 378; cam.cv = 238;
  const Pose T_WC = compose(T_WS, T_SC);
  double R[9];
  rot(T_WC.q, R);
  std::vector<std::array<double, 4>> lms(99);
  std::vector<std::unique_ptr<okvisgpu::ReprojectionError>> errs;
  const double Li[4] = {1, 0, 0, 1};
  for (int i = 1; i < 100; ++i) {
    const double minD = (i % 10) * 3 + 2.0, maxD = 10.0;
    const double u = (U(g) + 1) * 0.5 * (752 - 0.022) + 0.011, v = (U(g) + 1) * 0.5 * (480 - 0.022) + 0.011;
    const double d = U(g);
    double ray[3] = {(u - 378) / 350, (v - 238) / 360, 1.0};
    const double n = std::sqrt(ray[0] * ray[0] + ray[1] * ray[1] + 1.0), depth = 0.5 * (maxD - minD) * (d + 1) + minD;
    for (double& x : ray) x *= depth / n;
    auto& L = lms[i - 1];
    for (int r = 0; r < 3; ++r) L[r] = T_WC.t[r] + R[3 * r] * ray[0] + R[3 * r + 1] * ray[1] + R[3 * r + 2] * ray[2];
    L[3] = 1.0;
    P.AddParameterBlock(L.data(), 4, &hm);
    P.SetParameterBlockConstant(L.data());
    const double kp[2] = {350 * ray[0] / ray[2] + 378 + U(g), 360 * ray[1] / ray[2] + 238 + U(g)};
    errs.emplace_back(new okvisgpu::ReprojectionError(cam, kp, Li));
    P.AddResidualBlock(errs.back().get(), nullptr, pose, L.data(), extr);
  }
  okvisgpu_options o;
  okvisgpu_default_options(&o);
  okvisgpu_summary s;
  const int rc = P.Solve(o, &s);
  CHECK(rc == OKVISGPU_OK);
  const double dt = std::sqrt(std::pow(pose[0] - T_WS.t[0], 2) + std::pow(pose[1] - T_WS.t[1], 2) +
                              std::pow(pose[2] - T_WS.t[2], 2));
  const double dr = rotErr(T_WS.q, Quat{pose[3], pose[4], pose[5], pose[6]});
  CHECK(dr < 1e-2);  // TestReprojectionError.cpp:158-160
  CHECK(dt < 1e-1);  // :161-163
  std::printf("reprojection scene %llu: rc %d, %d iterations, termination %d, rot %.3g, trans %.3g\n",
              (unsigned long long)seed, rc, s.num_iterations, s.termination_type, dr, dt);
  return 0;
}

int windowVsDirect() {
  okvisgpu_synth_config cfg;
  okvisgpu_synth_default_config(&cfg, 10, 500, 4000, 20251015u);
  okvisgpu_synth_window *wa = nullptr, *wb = nullptr;
  CHECK(okvisgpu_synth_create(&cfg, &wa) == OKVISGPU_OK && okvisgpu_synth_create(&cfg, &wb) == OKVISGPU_OK);
  const okvisgpu_problem* pa = okvisgpu_synth_problem(wa);
  const okvisgpu_problem* pb = okvisgpu_synth_problem(wb);
  okvisgpu::Problem P;
  Recorded R;
  record(P, pa, R);
  // EvaluateResidualBlock (ViGraph.hpp:553) of GPU terms against the C ABI's evaluation hooks on the
  // same values: reprojections bit for bit (raw, and with the CauchyLoss(1) Corrector), IMU |r|^2
  {
    okvisgpu_ctx* ec = nullptr;
    CHECK(okvisgpu_ctx_create(0, &ec) == OKVISGPU_OK && okvisgpu_set_problems(ec, pb, 1) == OKVISGPU_OK);
    const int no = pb->n_observations, ni = pb->n_imu;
    std::vector<double> ro(2 * (size_t)no), ri(15 * (size_t)ni);
    CHECK(okvisgpu_eval_reprojection(ec, 0, ro.data(), nullptr, nullptr) == OKVISGPU_OK);
    CHECK(okvisgpu_eval_imu(ec, 0, 0, ri.data(), nullptr) == OKVISGPU_OK);
    double worst = 0.0;
    for (int o : {0, 1234, no - 1}) {
      double c = -1, r[2];
      CHECK(P.EvaluateResidualBlock(R.ids[o], false, &c, r, nullptr));
      CHECK(r[0] == ro[2 * o] && r[1] == ro[2 * o + 1]);
      const double sq = r[0] * r[0] + r[1] * r[1];
      CHECK(P.EvaluateResidualBlock(R.ids[o], true, &c, r, nullptr));
      CHECK(std::fabs(c - 0.5 * std::log1p(sq)) <= 1e-15 * c + 1e-300);
      worst = std::max(worst, std::fabs(r[0] - ro[2 * o] / std::sqrt(1.0 + sq)));
    }
    CHECK(worst <= 1e-12);
    for (int f : {0, ni - 1}) {
      double c = -1, r[15], s2 = 0.0;
      CHECK(P.EvaluateResidualBlock(R.ids[no + f], true, &c, r, nullptr));
      for (int i = 0; i < 15; ++i) s2 += ri[15 * f + i] * ri[15 * f + i];
      CHECK(std::fabs(c - 0.5 * s2) <= 1e-12 * c);
    }
    std::printf("EvaluateResidualBlock: reprojections equal to the C ABI hooks, IMU cost to 1e-12\n");
    okvisgpu_ctx_destroy(ec);
  }
  okvisgpu_summary sa, sb;
  CHECK(P.Solve(zeroTol(5), &sa) == OKVISGPU_OK);
  okvisgpu_ctx* ctx = nullptr;
  CHECK(okvisgpu_ctx_create(0, &ctx) == OKVISGPU_OK);
  CHECK(okvisgpu_set_problems(ctx, pb, 1) == OKVISGPU_OK);
  const okvisgpu_options o5 = zeroTol(5), o3 = zeroTol(3);
  CHECK(okvisgpu_solve(ctx, &o5, &sb) == OKVISGPU_OK);
  double dev = 0;
  for (int i = 0; i < 7 * pa->n_poses; ++i) dev = std::max(dev, std::fabs(pa->poses[i] - pb->poses[i]));
  CHECK(sa.num_iterations == sb.num_iterations);
  CHECK(std::fabs(sa.final_cost - sb.final_cost) <= 1e-9 * sb.final_cost);
  CHECK(dev <= 1e-9);
  std::printf("S10 facade vs C ABI: cost %.12g / %.12g, max pose deviation %.3g\n", sa.final_cost, sb.final_cost, dev);
  // freeze pose 3 between solves (the cheap set_block_constant path) and continue both
  P.SetParameterBlockConstant(&pa->poses[21]);
  CHECK(okvisgpu_set_block_constant(ctx, 0, 0, 3, 1) == OKVISGPU_OK);
  const double p3[7] = {pa->poses[21], pa->poses[22], pa->poses[23], pa->poses[24], pa->poses[25], pa->poses[26], pa->poses[27]};
  CHECK(P.Solve(zeroTol(3), &sa) == OKVISGPU_OK);
  CHECK(okvisgpu_update_params(ctx) == OKVISGPU_OK);
  CHECK(okvisgpu_solve(ctx, &o3, &sb) == OKVISGPU_OK);
  dev = 0;
  for (int i = 0; i < 7 * pa->n_poses; ++i) dev = std::max(dev, std::fabs(pa->poses[i] - pb->poses[i]));
  bool frozen = true;
  for (int i = 0; i < 7; ++i) frozen = frozen && pa->poses[21 + i] == p3[i];
  CHECK(frozen);
  CHECK(std::fabs(sa.final_cost - sb.final_cost) <= 1e-9 * sb.final_cost && dev <= 1e-9);
  std::printf("after freezing pose 3: cost %.12g / %.12g, max pose deviation %.3g\n", sa.final_cost, sb.final_cost, dev);
  // online calibration switched on between solves (ViGraph::setExtrinsicsVariable, ViGraph.cpp:1733-1739):
  // the facade queues okvisgpu_set_block_constant kind 3 (no problem re-upload) like the direct caller
  P.SetParameterBlockVariable(&pa->extrinsics[0]);
  CHECK(okvisgpu_set_block_constant(ctx, 0, 3, 0, 0) == OKVISGPU_OK);
  CHECK(P.Solve(zeroTol(3), &sa) == OKVISGPU_OK);
  CHECK(okvisgpu_update_params(ctx) == OKVISGPU_OK);
  CHECK(okvisgpu_solve(ctx, &o3, &sb) == OKVISGPU_OK);
  dev = 0;
  for (int i = 0; i < 7 * pa->n_poses; ++i) dev = std::max(dev, std::fabs(pa->poses[i] - pb->poses[i]));
  double dext = 0, moved = 0;
  for (int i = 0; i < 7; ++i) {
    dext = std::max(dext, std::fabs(pa->extrinsics[i] - pb->extrinsics[i]));
    moved = std::max(moved, std::fabs(pa->extrinsics[i] - pa->extrinsics[7 + i]));
  }
  CHECK(std::fabs(sa.final_cost - sb.final_cost) <= 1e-9 * sb.final_cost && dev <= 1e-9 && dext <= 1e-9);
  std::printf("after T_SC0 variable: cost %.12g / %.12g, max pose deviation %.3g, extrinsics %.3g\n", sa.final_cost,
              sb.final_cost, dev, dext);
  okvisgpu_ctx_destroy(ctx);
  okvisgpu_synth_destroy(wa);
  okvisgpu_synth_destroy(wb);
  return 0;
}

// §8b fallback end to end: an S10 window plus one GpsFunctor per keyframe on (pose k, speed/bias k,
// camera 0's constant T_SC as the alignment block) under CauchyLoss(3.0), through the facade
// (HostFunctor<GpsFunctor>, okvisgpu::CauchyLoss) and through the C ABI directly (host_* arrays,
// host_loss, a C callback): same solve.
int gpsHostFallback() {
  okvisgpu_synth_config cfg;
  okvisgpu_synth_default_config(&cfg, 10, 500, 4000, 20251016u);
  okvisgpu_synth_window *wa = nullptr, *wb = nullptr;
  CHECK(okvisgpu_synth_create(&cfg, &wa) == OKVISGPU_OK && okvisgpu_synth_create(&cfg, &wb) == OKVISGPU_OK);
  const okvisgpu_problem* pa = okvisgpu_synth_problem(wa);
  const okvisgpu_problem* pb = okvisgpu_synth_problem(wb);
  const int n = pa->n_poses;
  std::vector<double> gt(7 * n), gsb(9 * n);
  CHECK(okvisgpu_synth_ground_truth(wa, gt.data(), nullptr, gsb.data()) == OKVISGPU_OK);
  std::vector<GpsFunctor> gps(n);
  for (int k = 0; k < n; ++k) {  // measurements from the ground truth, aligned by T_SC0
    gps[k].dt = 0.005 * k;
    double pG[3], a[3], pW[3], RG[9];
    gps[k].predict(&gt[7 * k], &gsb[9 * k], &pa->extrinsics[0], pG, a, pW, RG);
    for (int i = 0; i < 3; ++i) gps[k].meas[i] = pG[i] + 0.01 * ((k + i) % 3 - 1);
  }
  okvisgpu::Problem P;
  Recorded R;
  record(P, pa, R);
  // GPS factors as ViGraph adds them: with cauchyGpsLossFunctionPtr_ = CauchyLoss(3.0)
  // (ViGraph.cpp:236,999); keyframe 4's measurement carries a gross error
  gps[4].meas[0] += 1.5;
  okvisgpu::CauchyLoss cauchyGpsLoss(3.0);
  std::vector<std::unique_ptr<okvisgpu::HostFunctor<GpsFunctor>>> hf;
  for (int k = 0; k < n; ++k) {
    hf.emplace_back(new okvisgpu::HostFunctor<GpsFunctor>(&gps[k]));
    P.AddResidualBlock(hf.back().get(), &cauchyGpsLoss, &pa->poses[7 * k], &pa->speed_biases[9 * k], &pa->extrinsics[0]);
  }
  okvisgpu_options o = zeroTol(8);
  o.num_threads = 2;
  okvisgpu_summary sa, sb;
  CHECK(P.Solve(o, &sa) == OKVISGPU_OK);
  // the same through the C ABI
  okvisgpu_problem q = *pb;
  std::vector<int32_t> dim(n, 3), kind, idx;
  for (int k = 0; k < n; ++k) {
    kind.insert(kind.end(), {0, 1, 0, -1});
    idx.insert(idx.end(), {k, k, pb->n_poses + 0, -1});
  }
  q.n_host = n;
  q.host_dim = dim.data();
  q.host_param_kind = kind.data();
  q.host_param_index = idx.data();
  q.host_cauchy = nullptr;
  const std::vector<okvisgpu_loss> losses(n, okvisgpu_loss{OKVISGPU_LOSS_CAUCHY, 0, 3.0, 0.0});
  q.host_loss = losses.data();
  q.host_user = &gps;
  q.host_evaluate = [](void* user, int32_t f, const double* const* prm, double* r, double** J) -> int {
    return (*static_cast<std::vector<GpsFunctor>*>(user))[f].Evaluate(prm, r, J) ? 1 : 0;
  };
  okvisgpu_ctx* ctx = nullptr;
  CHECK(okvisgpu_ctx_create(0, &ctx) == OKVISGPU_OK);
  CHECK(okvisgpu_set_problems(ctx, &q, 1) == OKVISGPU_OK);
  CHECK(okvisgpu_solve(ctx, &o, &sb) == OKVISGPU_OK);
  double dev = 0;
  for (int i = 0; i < 7 * n; ++i) dev = std::max(dev, std::fabs(pa->poses[i] - pb->poses[i]));
  CHECK(sa.num_iterations == sb.num_iterations && sa.termination_type == sb.termination_type);
  CHECK(std::fabs(sa.final_cost - sb.final_cost) <= 1e-9 * sb.final_cost && dev <= 1e-9);
  CHECK(sa.final_cost < 1e-2 * sa.initial_cost);
  std::printf("S10 + GPS host factors, facade vs C ABI: cost %.12g / %.12g (initial %.6g), max pose deviation %.3g\n",
              sa.final_cost, sb.final_cost, sa.initial_cost, dev);
  okvisgpu_ctx_destroy(ctx);
  okvisgpu_synth_destroy(wa);
  okvisgpu_synth_destroy(wb);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  if (mode == "cpu") return cpuTests();
  for (uint64_t seed = 1; seed <= 5; ++seed) reprojectionScene(seed);
  windowVsDirect();
  gpsHostFallback();
  std::printf("facade_test gpu %s\n", g_fail ? "FAILED" : "ok");
  return g_fail ? 1 : 0;
}
