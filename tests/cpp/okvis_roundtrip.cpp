// okvis objects across the boundary and back (the facade's okvis_access adapters, against the
// stand-ins of tests/cpp/okvis_standins.hpp, which mirror the okvis headers' protected members).
//   okvis_roundtrip cpu         accessor read / write of every adapted functor (no GPU needed)
//   okvis_roundtrip gpu <dump>  a window whose ImuError terms are live views of okvis ImuError
//                               objects (OkvisImuError<E>) and whose priors / pose-graph edges come
//                               from okvis objects through fromOkvis*; three solves:
//                                 1. Problem P1, then its write-back into the objects
//                                 2. a NEW Problem P2 over the same objects (the realtime ->
//                                    full-graph copy, ViSlamBackend.cpp:925-997): the state must
//                                    come in from the objects, or >= 50-sample factors would be
//                                    re-integrated at the current bias (ImuError.cpp:834-858)
//                                 3. P2 again (no structural change: the state is re-read)
//                               after each, the parameters and the objects' states (read back
//                               through the accessor) are appended to <dump> as raw doubles;
//                               tests/test_okvis_roundtrip.py replays the same solves on the oracle.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "okvisgpu.h"
#include "okvisgpu_problem.hpp"
#include "okvis_standins.hpp"

static int g_fail = 0;
#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c);  \
      ++g_fail;                                                                  \
    }                                                                            \
  } while (0)

namespace {

using okvis::ceres::ImuError;
using Members = okvisgpu::okvis_access::ImuErrorMembers<ImuError>;

// A test subclass that can set the protected members directly (what redoPreintegration would).
struct ImuErrorFiller : ImuError {
  using ImuError::ImuError;
  void fill(double base) {
    Delta_q_ = mini::Quaterniond(0.9, 0.1 * base, -0.2, 0.3);
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) {
        C_integral_(r, c) = base + r + 0.1 * c;
        C_doubleintegral_(r, c) = 2 * base - r + 0.01 * c;
        dalpha_db_g_(r, c) = 3 * base + 0.5 * r - c;
        dv_db_g_(r, c) = -base + r * c;
        dp_db_g_(r, c) = 0.25 * base + r - 2 * c;
        cross_(r, c) = 0.125 * (r + 1) * (c + 2) + base;
      }
      acc_integral_(r) = 4 * base + r;
      acc_doubleintegral_(r) = 5 * base - r;
    }
    for (int i = 0; i < 9; ++i) speedAndBiases_ref_(i) = 0.01 * i + base;
    for (int r = 0; r < 15; ++r)
      for (int c = 0; c < 15; ++c) {
        squareRootInformation_(r, c) = c >= r ? 1.0 / (1 + r + c) + base : 0.0;
        P_delta_(r, c) = 1e-6 * (1 + std::min(r, c)) + (r == c ? 1e-3 : 0.0);
      }
    redo_ = false;
    redoCounter_ = 7;
  }
  const mini::Matrix<15, 15>& info() const { return information_; }
  const mini::AlignedVector<mini::Matrix<15, 15>>& dP() const { return dPdsigma_; }
  // four distinct per-sigma derivatives (what okvis' own integration leaves)
  void setDistinctDp() {
    dPdsigma_.resize(4);
    for (int k = 0; k < 4; ++k)
      for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 15; ++c) dPdsigma_[k](r, c) = 0.5 * k + 0.01 * r - 0.002 * c;
  }
};

int cpuTests() {
  okvis::ImuParameters ip;
  okvis::ImuMeasurementDeque m;
  for (int i = 0; i < 4; ++i) {
    okvis::ImuMeasurement s;
    s.timeStamp = okvis::Time::fromNSec(1000000000ll + 5000000ll * i);
    for (int k = 0; k < 3; ++k) {
      s.measurement.gyroscopes(k) = 0.1 * (i + k);
      s.measurement.accelerometers(k) = 9.0 + i - k;
    }
    m.push_back(s);
  }
  ImuErrorFiller e(m, ip, okvis::Time::fromNSec(1001000000ll), okvis::Time::fromNSec(1014000000ll));
  // a fresh okvis factor: counter 0, redo_ true, identity Delta_q (ImuError.hpp:276-297)
  std::vector<double> s(OKVISGPU_IMU_STATE_DOUBLES);
  Members::read(e, s.data());
  CHECK(s[0] == 0.0 && s[1] == 1.0 && s[2] == 0.0 && s[5] == 1.0 && s[66] == 0.0);
  // the members land in the blob layout of okvisgpu.h (OKVISGPU_IMU_STATE_DOUBLES)
  e.fill(0.5);
  Members::read(e, s.data());
  CHECK(s[0] == 7.0 && s[1] == 0.0);
  CHECK(s[2] == 0.05 && s[3] == -0.2 && s[4] == 0.3 && s[5] == 0.9);
  CHECK(s[6 + 3 * 1 + 2] == 0.5 + 1 + 0.2);        // C_integral_(1, 2), row-major
  CHECK(s[15 + 3 * 2 + 0] == 1.0 - 2);              // C_doubleintegral_(2, 0)
  CHECK(s[24 + 2] == 4.0 && s[27 + 1] == 2.5 - 1);  // acc_integral_(2), acc_doubleintegral_(1)
  CHECK(s[30 + 3 * 2 + 1] == 1.5 + 1.0 - 1);        // dalpha_db_g_(2, 1)
  CHECK(s[39 + 3 * 2 + 2] == -0.5 + 4);             // dv_db_g_(2, 2)
  CHECK(s[48 + 1] == 0.125 - 2);                    // dp_db_g_(0, 1)
  CHECK(s[57 + 8] == 0.08 + 0.5);                   // speedAndBiases_ref_(8)
  CHECK(s[66 + 15 * 0 + 14] == 1.0 / 15 + 0.5 && s[66 + 15 * 14] == 0.0);
  CHECK(s[292 + 3 * 1 + 0] == 0.125 * 2 * 2 + 0.5);  // cross_(1, 0)
  CHECK(s[301 + 15 * 3 + 7] == 1e-6 * 4);            // P_delta_(3, 7)
  // write: every blob field lands in its member; information_ = U^T U; dPdsigma_ continues P_delta_
  std::vector<double> t(s);
  for (int i = 2; i < 66; ++i) t[i] = 0.001 * i - 0.3;
  for (int i = 292; i < 301; ++i) t[i] = -0.002 * i;
  t[0] = 3;
  t[1] = 1;
  ImuErrorFiller f(m, ip, e.t0(), e.t1());
  Members::write(t.data(), f);
  std::vector<double> u(OKVISGPU_IMU_STATE_DOUBLES);
  Members::read(f, u.data());
  CHECK(std::memcmp(t.data(), u.data(), sizeof(double) * 291) == 0);
  CHECK(std::memcmp(t.data() + 292, u.data() + 292, sizeof(double) * (OKVISGPU_IMU_STATE_DOUBLES - 292)) == 0);
  double dinfo = 0.0, ddp = 0.0;
  for (int r = 0; r < 15; ++r)
    for (int c = 0; c < 15; ++c) {
      double v = 0;
      for (int k = 0; k < 15; ++k) v += t[66 + 15 * k + r] * t[66 + 15 * k + c];
      dinfo = std::max(dinfo, std::fabs(f.info()(r, c) - v));
      const double p = f.dP()[0](r, c) * ip.sigma_g_c * ip.sigma_g_c + f.dP()[1](r, c) * ip.sigma_a_c * ip.sigma_a_c +
                       f.dP()[2](r, c) * ip.sigma_gw_c * ip.sigma_gw_c + f.dP()[3](r, c) * ip.sigma_aw_c * ip.sigma_aw_c;
      ddp = std::max(ddp, std::fabs(p - t[301 + 15 * r + c]) / 1e-3);
    }
  CHECK(f.dP().size() == 4 && dinfo < 1e-14 && ddp < 1e-14);
  // fromOkvisImuError copies samples, times and state; OkvisImuError is a live view
  okvisgpu::ImuError term = okvisgpu::fromOkvisImuError(e);
  CHECK(term.t0_ns == 1001000000ll && term.t1_ns == 1014000000ll && term.sample_t_ns.size() == 4);
  CHECK(term.gyr_acc[6 * 3 + 2] == 0.1 * 5 && term.gyr_acc[6 * 2 + 3] == 11.0);
  CHECK(std::memcmp(term.state.data(), s.data(), sizeof(double) * OKVISGPU_IMU_STATE_DOUBLES) == 0);
  CHECK(term.params.sigma_gw_c == ip.sigma_gw_c && term.params.g == ip.g);
  okvisgpu::OkvisImuError<ImuError> view(&f);
  CHECK(std::memcmp(view.state.data(), u.data(), sizeof(double) * OKVISGPU_IMU_STATE_DOUBLES) == 0);
  view.state[0] = 11;  // what a solve's write-back leaves in the term
  view.state[57 + 3] = 0.123;
  f.setDistinctDp();  // P_delta_ unchanged by the "solve": the object's own dPdsigma_ stays
  view.pushState();
  Members::read(f, u.data());
  CHECK(u[0] == 11 && u[60] == 0.123);
  CHECK(f.dP().size() == 4 && f.dP()[2](3, 5) == 0.5 * 2 + 0.01 * 3 - 0.002 * 5 && f.dP()[0](1, 1) == 0.01 - 0.002);
  e.fill(0.75);  // the object changed between solves (ImuError::append): the view re-reads it
  okvisgpu::OkvisImuError<ImuError> view2(&e);
  e.fill(0.25);
  view2.pullState();
  Members::read(e, u.data());
  CHECK(std::memcmp(view2.state.data(), u.data(), sizeof(double) * OKVISGPU_IMU_STATE_DOUBLES) == 0);
  // the facade flattens a view's state into the C-ABI problem, and writes the okvis object back
  {
    okvisgpu::Problem P;
    okvisgpu::PoseManifold pm;
    double T0[7] = {0, 0, 0, 0, 0, 0, 1}, T1[7] = {1, 0, 0, 0, 0, 0, 1}, sb0[9] = {0}, sb1[9] = {0};
    P.AddParameterBlock(T0, 7, &pm);
    P.AddParameterBlock(T1, 7, &pm);
    P.AddResidualBlock(&view2, nullptr, T0, sb0, T1, sb1);
    const okvisgpu_problem& v = P.view();
    CHECK(v.n_imu == 1 && v.imu_state[0] == 7.0 && v.imu_state[57] == 0.25 && v.imu_t1_ns[0] == 1014000000ll);
    CHECK(v.imu_sample_begin[1] == 4 && v.imu_sample_gyr_acc[6 * 3 + 2] == 0.1 * 5);
  }
  // pose-graph edges, relative pose, priors
  double dx[6] = {0.1, -0.2, 0.3, 0.01, -0.02, 0.03}, J[36], lp[7] = {1, 2, 3, 0.1, 0.2, 0.3, 0.9};
  for (int i = 0; i < 36; ++i) J[i] = (i % 7 == 0 ? 10.0 : 0.0) + 0.1 * i;
  mini::Matrix<6, 1> DX;
  mini::Matrix<6, 6> JM;
  for (int i = 0; i < 6; ++i) DX(i) = dx[i];
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 6; ++c) JM(r, c) = J[6 * r + c];
  const okvis::kinematics::Transformation LP(lp);
  okvis::ceres::TwoPoseStandardGraphErrorConst tc(DX, JM, LP);
  okvis::ceres::TwoPoseStandardGraphError ts(dx, J, lp);
  const okvisgpu::TwoPoseGraphError a = okvisgpu::fromOkvisTwoPoseGraphError(tc);
  const okvisgpu::TwoPoseGraphError b = okvisgpu::fromOkvisTwoPoseGraphError(ts);
  CHECK(a.is_const && a.typeInfo() == "TwoPoseStandardGraphErrorConst");
  CHECK(!b.is_const && b.typeInfo() == "TwoPoseStandardGraphError");
  CHECK(std::memcmp(a.delta_x, dx, sizeof dx) == 0 && std::memcmp(b.delta_x, dx, sizeof dx) == 0);
  CHECK(std::memcmp(a.J, J, sizeof J) == 0 && std::memcmp(b.J, J, sizeof J) == 0);
  CHECK(std::memcmp(a.lin_point, lp, sizeof lp) == 0 && std::memcmp(b.lin_point, lp, sizeof lp) == 0);
  okvis::ceres::RelativePoseError rp(J, LP);
  const okvisgpu::RelativePoseError c = okvisgpu::fromOkvisRelativePoseError(rp);
  CHECK(std::memcmp(c.T_AB, lp, sizeof lp) == 0 && std::memcmp(c.sqrt_info, J, sizeof J) == 0);
  // the first-state prior's diagonal information (ViGraph.cpp:348-368) has zero yaw / pitch
  // entries: its stored square root is sqrt(diag), read as such (an LLT of information() fails)
  const double diag[6] = {1e8, 1e8, 1e8, 0, 0, 1e2};
  okvis::ceres::PoseError pe(LP, diag);
  const okvisgpu::PoseError d = okvisgpu::fromOkvisPoseError(pe);
  CHECK(std::memcmp(d.meas, lp, sizeof lp) == 0 && d.sqrt_info[0] == 1e4 && d.sqrt_info[21] == 0.0 &&
        d.sqrt_info[28] == 0.0 && d.sqrt_info[35] == 10.0 && d.sqrt_info[1] == 0.0);
  okvis::SpeedAndBias sbm;
  double L9[81];
  for (int i = 0; i < 9; ++i) sbm(i) = 0.5 * i;
  for (int i = 0; i < 81; ++i) L9[i] = i % 10 == 0 ? 3.0 + i : 0.0;
  okvis::ceres::SpeedAndBiasError se(sbm, L9);
  const okvisgpu::SpeedAndBiasError g = okvisgpu::fromOkvisSpeedAndBiasError(se);
  CHECK(g.meas[8] == 4.0 && std::memcmp(g.sqrt_info, L9, sizeof L9) == 0);
  std::printf("okvis_roundtrip cpu %s\n", g_fail ? "FAILED" : "ok");
  return g_fail ? 1 : 0;
}

// ------------------------------------------------------------------ GPU round trip
struct OkvisWindow {  // what ViGraph holds: okvis functor objects (here: the stand-ins)
  std::vector<std::unique_ptr<ImuError>> imu;
  std::vector<std::unique_ptr<okvis::ceres::PoseError>> posePriors;
  std::vector<std::unique_ptr<okvis::ceres::SpeedAndBiasError>> sbPriors;
  std::vector<std::unique_ptr<okvis::ceres::TwoPoseStandardGraphErrorConst>> edgesConst;
  std::vector<std::unique_ptr<okvis::ceres::TwoPoseStandardGraphError>> edges;
  std::vector<std::unique_ptr<okvis::ceres::RelativePoseError>> relpose;
  std::vector<int> relKind;  // per relpose record: 0 const edge, 1 edge, 2 relative pose error
  std::vector<int> relIndex;
};

OkvisWindow okvisObjects(const okvisgpu_problem* p) {
  OkvisWindow W;
  okvis::ImuParameters ip;
  ip.a_max = p->imu_params.a_max; ip.g_max = p->imu_params.g_max; ip.sigma_g_c = p->imu_params.sigma_g_c;
  ip.sigma_a_c = p->imu_params.sigma_a_c; ip.sigma_gw_c = p->imu_params.sigma_gw_c;
  ip.sigma_aw_c = p->imu_params.sigma_aw_c; ip.g = p->imu_params.g;
  for (int f = 0; f < p->n_imu; ++f) {
    okvis::ImuMeasurementDeque m;
    for (int s = p->imu_sample_begin[f]; s < p->imu_sample_begin[f + 1]; ++s) {
      okvis::ImuMeasurement x;
      x.timeStamp = okvis::Time::fromNSec(p->imu_sample_t_ns[s]);
      for (int k = 0; k < 3; ++k) {
        x.measurement.gyroscopes(k) = p->imu_sample_gyr_acc[6 * s + k];
        x.measurement.accelerometers(k) = p->imu_sample_gyr_acc[6 * s + 3 + k];
      }
      m.push_back(x);
    }
    W.imu.emplace_back(new ImuError(m, ip, okvis::Time::fromNSec(p->imu_t0_ns[f]), okvis::Time::fromNSec(p->imu_t1_ns[f])));
  }
  for (int i = 0; i < p->n_pose_priors; ++i)
    W.posePriors.emplace_back(new okvis::ceres::PoseError(okvis::kinematics::Transformation(&p->pose_prior_meas[7 * i]),
                                                          &p->pose_prior_sqrt_info[36 * i], 0));
  for (int i = 0; i < p->n_sb_priors; ++i) {
    okvis::SpeedAndBias m;
    for (int k = 0; k < 9; ++k) m(k) = p->sb_prior_meas[9 * i + k];
    W.sbPriors.emplace_back(new okvis::ceres::SpeedAndBiasError(m, &p->sb_prior_sqrt_info[81 * i]));
  }
  for (int i = 0; i < p->n_relpose; ++i) {
    const okvis::kinematics::Transformation lp(&p->relpose_lin_point[7 * i]);
    if (p->relpose_kind[i] == 1) {
      W.relKind.push_back(2);
      W.relIndex.push_back((int)W.relpose.size());
      W.relpose.emplace_back(new okvis::ceres::RelativePoseError(&p->relpose_sqrt_info[36 * i], lp));
    } else if (i % 2 == 0) {
      mini::Matrix<6, 1> dx;
      mini::Matrix<6, 6> J;
      for (int k = 0; k < 6; ++k) dx(k) = p->relpose_delta_x[6 * i + k];
      for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) J(r, c) = p->relpose_sqrt_info[36 * i + 6 * r + c];
      W.relKind.push_back(0);
      W.relIndex.push_back((int)W.edgesConst.size());
      W.edgesConst.emplace_back(new okvis::ceres::TwoPoseStandardGraphErrorConst(dx, J, lp));
    } else {
      W.relKind.push_back(1);
      W.relIndex.push_back((int)W.edges.size());
      W.edges.emplace_back(new okvis::ceres::TwoPoseStandardGraphError(&p->relpose_delta_x[6 * i],
                                                                       &p->relpose_sqrt_info[36 * i],
                                                                       &p->relpose_lin_point[7 * i]));
    }
  }
  return W;
}

struct Terms {  // the facade terms of one Problem (owned by the caller, as in Ceres)
  okvisgpu::PoseManifold poseManifold;
  okvisgpu::HomogeneousPointManifold pointManifold;
  okvisgpu::CauchyLoss cauchy{1.0};
  std::vector<std::unique_ptr<okvisgpu::CostFunction>> costs;
};

// ViGraph's graph over the okvis objects: parameter memory = the problem's arrays
void record(okvisgpu::Problem& P, const okvisgpu_problem* p, OkvisWindow& W, Terms& T) {
  for (int i = 0; i < p->n_poses; ++i) {
    P.AddParameterBlock(&p->poses[7 * i], 7, &T.poseManifold);
    if (p->pose_constant && p->pose_constant[i]) P.SetParameterBlockConstant(&p->poses[7 * i]);
  }
  for (int i = 0; i < p->n_speed_biases; ++i) P.AddParameterBlock(&p->speed_biases[9 * i], 9);
  for (int c = 0; c < p->n_cameras; ++c) {
    P.AddParameterBlock(&p->extrinsics[7 * c], 7, &T.poseManifold);
    P.SetParameterBlockConstant(&p->extrinsics[7 * c]);
  }
  for (int l = 0; l < p->n_landmarks; ++l) P.AddParameterBlock(&p->landmarks[4 * l], 4, &T.pointManifold);
  for (int o = 0; o < p->n_observations; ++o) {
    const int c = p->obs_camera[o];
    T.costs.emplace_back(new okvisgpu::ReprojectionError(p->cameras[c], &p->obs_keypoint[2 * o], &p->obs_sqrt_info[4 * o]));
    P.AddResidualBlock(T.costs.back().get(), (!p->obs_cauchy || p->obs_cauchy[o]) ? &T.cauchy : nullptr,
                       &p->poses[7 * p->obs_pose[o]], &p->landmarks[4 * p->obs_landmark[o]], &p->extrinsics[7 * c]);
  }
  for (int f = 0; f < p->n_imu; ++f) {
    T.costs.emplace_back(new okvisgpu::OkvisImuError<ImuError>(W.imu[f].get()));
    const int* b = &p->imu_blocks[4 * f];
    P.AddResidualBlock(T.costs.back().get(), nullptr, &p->poses[7 * b[0]], &p->speed_biases[9 * b[1]],
                       &p->poses[7 * b[2]], &p->speed_biases[9 * b[3]]);
  }
  for (int i = 0; i < p->n_pose_priors; ++i) {
    T.costs.emplace_back(new okvisgpu::PoseError(okvisgpu::fromOkvisPoseError(*W.posePriors[i])));
    P.AddResidualBlock(T.costs.back().get(), nullptr, &p->poses[7 * p->pose_prior_block[i]]);
  }
  for (int i = 0; i < p->n_sb_priors; ++i) {
    T.costs.emplace_back(new okvisgpu::SpeedAndBiasError(okvisgpu::fromOkvisSpeedAndBiasError(*W.sbPriors[i])));
    P.AddResidualBlock(T.costs.back().get(), nullptr, &p->speed_biases[9 * p->sb_prior_block[i]]);
  }
  for (int i = 0; i < p->n_relpose; ++i) {
    const int k = W.relIndex[i];
    if (W.relKind[i] == 0)
      T.costs.emplace_back(new okvisgpu::TwoPoseGraphError(okvisgpu::fromOkvisTwoPoseGraphError(*W.edgesConst[k])));
    else if (W.relKind[i] == 1)
      T.costs.emplace_back(new okvisgpu::TwoPoseGraphError(okvisgpu::fromOkvisTwoPoseGraphError(*W.edges[k])));
    else
      T.costs.emplace_back(new okvisgpu::RelativePoseError(okvisgpu::fromOkvisRelativePoseError(*W.relpose[k])));
    P.AddResidualBlock(T.costs.back().get(), nullptr, &p->poses[7 * p->relpose_blocks[2 * i]],
                       &p->poses[7 * p->relpose_blocks[2 * i + 1]]);
  }
}

okvisgpu_options zeroTol(int iters) {
  okvisgpu_options o;
  okvisgpu_default_options(&o);
  o.max_num_iterations = iters;
  o.function_tolerance = o.gradient_tolerance = o.parameter_tolerance = 0.0;
  return o;
}

void dump(FILE* f, const okvisgpu_problem* p, const OkvisWindow& W, const okvisgpu_summary& s) {
  const double head[4] = {s.initial_cost, s.final_cost, (double)s.num_iterations, (double)s.termination_type};
  std::fwrite(head, sizeof(double), 4, f);
  std::fwrite(p->poses, sizeof(double), 7 * (size_t)p->n_poses, f);
  std::fwrite(p->speed_biases, sizeof(double), 9 * (size_t)p->n_speed_biases, f);
  std::fwrite(p->landmarks, sizeof(double), 4 * (size_t)p->n_landmarks, f);
  std::vector<double> s1(OKVISGPU_IMU_STATE_DOUBLES);
  for (const auto& e : W.imu) {  // the okvis objects' members, read back through the accessor
    Members::read(*e, s1.data());
    std::fwrite(s1.data(), sizeof(double), s1.size(), f);
  }
}

int gpuRoundTrip(const char* path, int kf, int lm, int obs, double kf_dt, uint64_t seed, int n_relpose) {
  okvisgpu_synth_config cfg;
  okvisgpu_synth_default_config(&cfg, kf, lm, obs, seed);
  cfg.kf_dt_s = kf_dt;
  cfg.n_relpose = n_relpose;
  cfg.relpose_stride = 2;
  cfg.relpose_kind = 2;
  okvisgpu_synth_window* w = nullptr;
  CHECK(okvisgpu_synth_create(&cfg, &w) == OKVISGPU_OK);
  const okvisgpu_problem* p = okvisgpu_synth_problem(w);
  OkvisWindow W = okvisObjects(p);
  FILE* f = std::fopen(path, "wb");
  CHECK(f != nullptr);
  okvisgpu_summary s;
  {
    okvisgpu::Problem P1;
    Terms T1;
    record(P1, p, W, T1);
    CHECK(P1.Solve(zeroTol(4), &s) == OKVISGPU_OK);
    dump(f, p, W, s);
    std::printf("solve 1: %d iterations, cost %.12g -> %.12g\n", s.num_iterations, s.initial_cost, s.final_cost);
  }
  okvisgpu::Problem P2;
  Terms T2;
  record(P2, p, W, T2);
  CHECK(P2.Solve(zeroTol(3), &s) == OKVISGPU_OK);
  dump(f, p, W, s);
  std::printf("solve 2 (new Problem): %d iterations, cost %.12g -> %.12g\n", s.num_iterations, s.initial_cost, s.final_cost);
  CHECK(P2.Solve(zeroTol(3), &s) == OKVISGPU_OK);
  dump(f, p, W, s);
  std::printf("solve 3 (same Problem): %d iterations, cost %.12g -> %.12g\n", s.num_iterations, s.initial_cost, s.final_cost);
  std::fclose(f);
  okvisgpu_synth_destroy(w);
  std::printf("okvis_roundtrip gpu %s\n", g_fail ? "FAILED" : "ok");
  return g_fail ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  if (mode == "cpu") return cpuTests();
  if (argc < 9) {
    std::fprintf(stderr, "usage: okvis_roundtrip gpu <dump> <kf> <lm> <obs> <kf_dt> <seed> <n_relpose>\n");
    return 2;
  }
  return gpuRoundTrip(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), std::atof(argv[6]),
                      (uint64_t)std::atoll(argv[7]), std::atoi(argv[8]));
}
