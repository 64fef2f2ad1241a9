// okvisgpu_problem.hpp — C++ facade with the subset of the `::ceres::Problem` API that okvis drives,
// recording the graph and solving it through the okvisgpu C ABI (okvisgpu.h). Header-only, C++17,
// no Ceres / Eigen / HIP types: it compiles with any host compiler and links against
// libokvisgpu.so.
//
// What it replaces: `ViGraph::problem_` (a `::ceres::Problem`,
// okvis_ceres/include/okvis/ViGraph.hpp:27-39) and the `::ceres::Solve(options_, problem_.get(),
// &summary_)` call of `ViGraph::optimise` (ViGraph.cpp:1884). Method names, argument meaning and
// ownership follow the call sites:
//   AddParameterBlock(ptr, size[, manifold])          ViGraph.cpp:327-345, ViGraphEstimator.cpp:84-126
//   AddResidualBlock(cost, loss, ptrs...)             ViGraph.cpp:367-385,433-459; ViGraph.hpp:336-340
//   RemoveResidualBlock / RemoveParameterBlock        ViGraph.cpp:597,611,626-637,700-702
//   SetParameterBlockConstant / Variable              ViGraphEstimator.cpp:216-331, ViSlamBackend.cpp:854-863
//   HasParameterBlock, IsParameterBlockConstant, NumResidualBlocks, NumParameterBlocks,
//   GetParameterBlocksForResidualBlock, GetResidualBlocksForParameterBlock,
//   GetCostFunctionForResidualBlock, GetLossFunctionForResidualBlock, GetManifold, SetManifold
// Cost functions are recognised by their `typeInfo()` string, as okvis' ErrorInterface::typeInfo()
// (okvis_ceres/include/okvis/ceres/ErrorInterface.hpp:78) names them: "ReprojectionError",
// "ImuError", "PoseError", "SpeedAndBiasError", "TwoPoseStandardGraphError(Const)",
// "RelativePoseError". The term classes below carry the constants the adapter reads from the okvis
// functors' getters (fromOkvisReprojectionError / fromOkvisImuError read them).
// Any other cost function on pose-kind / speed-bias blocks (GPS, user factors) joins the solve as a
// HostCostFunction (or HostFunctor<F> around the caller's ceres::CostFunction-shaped functor): the
// §8b host-evaluated fallback. Cost functions the fallback cannot take either (landmark blocks:
// OneSidedDepthError) are rejected at AddResidualBlock with okvisgpu::Unsupported
// (OKVISGPU_ERR_UNSUPPORTED): the caller keeps its Ceres solve for such a graph.
//
// Ownership: like `Problem::Options{DO_NOT_TAKE_OWNERSHIP}` (ViGraph.cpp:239-247), the facade never
// deletes cost functions, losses or manifolds; parameter memory stays the caller's and is read
// before and written after every Solve (the reference's in-place ParameterBlock semantics).
// Errors: misuse (unknown block, wrong sizes) throws okvisgpu::Error (a std::runtime_error, as
// OKVIS_THROW does); Solve returns the okvisgpu_status of the C ABI.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "okvisgpu.h"

namespace okvisgpu {

struct Error : std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error("okvisgpu: " + m) {}
};
struct Unsupported : Error {
  explicit Unsupported(const std::string& m) : Error(m) {}
  int status() const { return OKVISGPU_ERR_UNSUPPORTED; }
};

// ---------------------------------------------------------------- manifolds (ceres::Manifold)
class Manifold {
 public:
  virtual ~Manifold() = default;
  virtual int AmbientSize() const = 0;
  virtual int TangentSize() const = 0;
  virtual const char* name() const = 0;
};
// PoseManifold (okvis_ceres/src/PoseLocalParameterization.cpp:29-107): [t, q xyzw], 7 -> 6
class PoseManifold final : public Manifold {
 public:
  int AmbientSize() const override { return 7; }
  int TangentSize() const override { return 6; }
  const char* name() const override { return "PoseManifold"; }
};
// HomogeneousPointManifold (HomogeneousPointLocalParameterization.cpp:27-90): 4 -> 3
class HomogeneousPointManifold final : public Manifold {
 public:
  int AmbientSize() const override { return 4; }
  int TangentSize() const override { return 3; }
  const char* name() const override { return "HomogeneousPointManifold"; }
};

// ---------------------------------------------------------------- losses (ceres::LossFunction)
// The Ceres loss family with ::ceres::LossFunction::Evaluate(s, rho) (evaluated by the library,
// okvisgpu_loss_evaluate: the same restatement the backend applies). okvis builds four of them in
// ViGraph's constructor (ViGraph.cpp:235-238): CauchyLoss(1.0) (every reprojection, :338; Cauchy
// submap alignment, :1505), CauchyLoss(3.0) (GPS, :88,:999,:1408), TukeyLoss(0.1) / TukeyLoss(2.0)
// (depth / LiDAR submap alignment, :1513 / :1510). The GPU evaluates reprojections with
// CauchyLoss(1) only; host-evaluated factors take any of these.
class LossFunction {
 public:
  virtual ~LossFunction() = default;
  virtual const char* name() const = 0;
  virtual okvisgpu_loss descriptor() const = 0;
  // rho[0..2] = rho(s), rho'(s), rho''(s) of the squared residual norm s
  void Evaluate(double s, double rho[3]) const {
    const okvisgpu_loss d = descriptor();
    if (okvisgpu_loss_evaluate(&d, s, rho) != OKVISGPU_OK) throw Error(std::string(name()) + ": invalid scale");
  }
};
namespace detail {
template <int Kind>
class ScaledLoss : public LossFunction {
 public:
  explicit ScaledLoss(double a, double b = 0.0) : a_(a), b_(b) {
    const okvisgpu_loss d = descriptor();
    double rho[3];
    if (okvisgpu_loss_evaluate(&d, 0.0, rho) != OKVISGPU_OK) throw Error("loss function with an invalid scale");
  }
  okvisgpu_loss descriptor() const override { return okvisgpu_loss{Kind, 0, a_, b_}; }
  double a() const { return a_; }

 protected:
  double a_, b_;
};
}  // namespace detail
class CauchyLoss final : public detail::ScaledLoss<OKVISGPU_LOSS_CAUCHY> {
 public:
  explicit CauchyLoss(double a = 1.0) : ScaledLoss(a) {}
  const char* name() const override { return "CauchyLoss"; }
};
class TukeyLoss final : public detail::ScaledLoss<OKVISGPU_LOSS_TUKEY> {
 public:
  explicit TukeyLoss(double a) : ScaledLoss(a) {}
  const char* name() const override { return "TukeyLoss"; }
};
class HuberLoss final : public detail::ScaledLoss<OKVISGPU_LOSS_HUBER> {
 public:
  explicit HuberLoss(double a) : ScaledLoss(a) {}
  const char* name() const override { return "HuberLoss"; }
};
class SoftLOneLoss final : public detail::ScaledLoss<OKVISGPU_LOSS_SOFTLONE> {
 public:
  explicit SoftLOneLoss(double a) : ScaledLoss(a) {}
  const char* name() const override { return "SoftLOneLoss"; }
};
class ArctanLoss final : public detail::ScaledLoss<OKVISGPU_LOSS_ARCTAN> {
 public:
  explicit ArctanLoss(double a) : ScaledLoss(a) {}
  const char* name() const override { return "ArctanLoss"; }
};
class TolerantLoss final : public detail::ScaledLoss<OKVISGPU_LOSS_TOLERANT> {
 public:
  TolerantLoss(double a, double b) : ScaledLoss(a, b) {}
  const char* name() const override { return "TolerantLoss"; }
};

// ---------------------------------------------------------------- cost functions
// The okvis functors' constants (what the GPU evaluates from); typeInfo() as ErrorInterface.
class CostFunction {
 public:
  virtual ~CostFunction() = default;
  virtual std::string typeInfo() const = 0;
  virtual int residualDim() const = 0;
  virtual std::vector<int> parameterBlockSizes() const = 0;  // ambient sizes, in call order
};

// ReprojectionError<PinholeCamera<D>> (implementation/ReprojectionError.hpp:49-220): parameters
// (T_WS pose, hp_W landmark, T_SC extrinsics); camera = the functor's cameraGeometry_.
class ReprojectionError final : public CostFunction {
 public:
  ReprojectionError(const okvisgpu_camera& camera, const double keypoint[2], const double sqrt_info[4])
      : camera(camera) {
    std::memcpy(this->keypoint, keypoint, sizeof(this->keypoint));
    std::memcpy(this->sqrt_info, sqrt_info, sizeof(this->sqrt_info));
  }
  std::string typeInfo() const override { return "ReprojectionError"; }
  int residualDim() const override { return 2; }
  std::vector<int> parameterBlockSizes() const override { return {7, 4, 7}; }
  okvisgpu_camera camera;
  double keypoint[2];   // measurement_
  double sqrt_info[4];  // squareRootInformation_ (row-major)
};

// ImuError (ImuError.cpp:63-1003): parameters (pose0, sb0, pose1, sb1). `state` is the functor's
// mutable preintegration state (OKVISGPU_IMU_STATE_DOUBLES layout), written back after a solve.
// A term that is a live view of an okvis ImuError object (OkvisImuError<E> below) overrides the
// hooks: pull() refreshes samples, times and state from the object when the graph is flattened,
// pullState() the state before every solve, pushState() writes the solved state back into it.
class ImuError : public CostFunction {
 public:
  ImuError(std::vector<int64_t> sample_t_ns, std::vector<double> gyr_acc, const okvisgpu_imu_params& params,
           int64_t t0_ns, int64_t t1_ns)
      : sample_t_ns(std::move(sample_t_ns)), gyr_acc(std::move(gyr_acc)), params(params), t0_ns(t0_ns),
        t1_ns(t1_ns), state(OKVISGPU_IMU_STATE_DOUBLES, 0.0) {
    if (this->gyr_acc.size() != 6 * this->sample_t_ns.size()) throw Error("ImuError: gyr_acc must hold 6 per sample");
  }
  std::string typeInfo() const override { return "ImuError"; }
  int residualDim() const override { return 15; }
  std::vector<int> parameterBlockSizes() const override { return {7, 9, 7, 9}; }
  virtual void pull() {}
  virtual void pullState() {}
  virtual void pushState() {}
  std::vector<int64_t> sample_t_ns;
  std::vector<double> gyr_acc;
  okvisgpu_imu_params params;
  int64_t t0_ns, t1_ns;
  std::vector<double> state;
};

// PoseError (PoseError.cpp:73-125): a prior on a pose or an extrinsics block.
class PoseError final : public CostFunction {
 public:
  PoseError(const double measurement[7], const double sqrt_info[36]) {
    std::memcpy(meas, measurement, sizeof(meas));
    std::memcpy(this->sqrt_info, sqrt_info, sizeof(this->sqrt_info));
  }
  std::string typeInfo() const override { return "PoseError"; }
  int residualDim() const override { return 6; }
  std::vector<int> parameterBlockSizes() const override { return {7}; }
  double meas[7];
  double sqrt_info[36];
};

// SpeedAndBiasError (SpeedAndBiasError.cpp:67-101).
class SpeedAndBiasError final : public CostFunction {
 public:
  SpeedAndBiasError(const double measurement[9], const double sqrt_info[81]) {
    std::memcpy(meas, measurement, sizeof(meas));
    std::memcpy(this->sqrt_info, sqrt_info, sizeof(this->sqrt_info));
  }
  std::string typeInfo() const override { return "SpeedAndBiasError"; }
  int residualDim() const override { return 9; }
  std::vector<int> parameterBlockSizes() const override { return {9}; }
  double meas[9];
  double sqrt_info[81];
};

// TwoPoseStandardGraphError / ...Const (TwoPoseGraphError.cpp:467-606,631-767): parameters
// (reference pose, other pose); DeltaX_, J_, linearisationPoint_T_S0S1_.
class TwoPoseGraphError final : public CostFunction {
 public:
  TwoPoseGraphError(const double delta_x[6], const double J[36], const double lin_point[7], bool is_const = true)
      : is_const(is_const) {
    std::memcpy(this->delta_x, delta_x, sizeof(this->delta_x));
    std::memcpy(this->J, J, sizeof(this->J));
    std::memcpy(this->lin_point, lin_point, sizeof(this->lin_point));
  }
  std::string typeInfo() const override {
    return is_const ? "TwoPoseStandardGraphErrorConst" : "TwoPoseStandardGraphError";
  }
  int residualDim() const override { return 6; }
  std::vector<int> parameterBlockSizes() const override { return {7, 7}; }
  double delta_x[6], J[36], lin_point[7];
  bool is_const;
};

// RelativePoseError (RelativePoseError.cpp:59-140, ViGraph::addRelativePoseConstraint): (A, B).
class RelativePoseError final : public CostFunction {
 public:
  RelativePoseError(const double T_AB[7], const double sqrt_info[36]) {
    std::memcpy(this->T_AB, T_AB, sizeof(this->T_AB));
    std::memcpy(this->sqrt_info, sqrt_info, sizeof(this->sqrt_info));
  }
  std::string typeInfo() const override { return "RelativePoseError"; }
  int residualDim() const override { return 6; }
  std::vector<int> parameterBlockSizes() const override { return {7, 7}; }
  double T_AB[7], sqrt_info[36];
};

// Host-evaluated residual (ABI 5, SURVEY.md §8b fallback): any cost function the GPU path has no
// functor for (GpsErrorSynchronous / GpsErrorAsynchronous, user factors) on pose-kind (7, state pose
// or extrinsics) and speed/bias (9) blocks, at most 2 of each, <= 15 residuals. Evaluate has the
// ::ceres::CostFunction::Evaluate contract: ambient Jacobians (the backend applies the blocks'
// PoseManifold), return false on failure. It is called from up to options.num_threads host threads
// at every point the solver evaluates; any loss of the family above may be attached at
// AddResidualBlock (CauchyLoss(3.0) for GPS, TukeyLoss for submap alignment: ViGraph.cpp:999,1510).
class HostCostFunction : public CostFunction {
 public:
  std::string typeInfo() const override { return "HostCostFunction"; }
  virtual bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const = 0;
};

// A ceres::CostFunction-shaped functor object (okvis' GpsErrorAsynchronous, a
// ceres::SizedCostFunction, ...) used as a host cost function through its own getters, so the call
// site keeps its type: F must provide Evaluate(double const* const*, double*, double**) const,
// num_residuals() and parameter_block_sizes() (ceres::CostFunction), and typeInfo()
// (ErrorInterface.hpp:78). The functor is not owned.
template <class F>
class HostFunctor final : public HostCostFunction {
 public:
  explicit HostFunctor(const F* functor) : f_(functor) {}
  std::string typeInfo() const override { return f_->typeInfo(); }
  int residualDim() const override { return (int)f_->num_residuals(); }
  std::vector<int> parameterBlockSizes() const override {
    const auto& s = f_->parameter_block_sizes();
    return std::vector<int>(s.begin(), s.end());
  }
  bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const override {
    return f_->Evaluate(parameters, residuals, jacobians);
  }

 private:
  const F* f_;
};

// ---- okvis functors -> GPU-evaluated terms, through the functors' getters (templates: no okvis /
// Eigen types are named here; anything with the getters' shape works)
// ReprojectionError<PinholeCamera<D>>: measurement() (2-vector), information() (2x2)
// (ReprojectionErrorBase.hpp:75-91, ReprojectionError.hpp:94-105); squareRootInformation_ =
// LLT(information).matrixL()^T (ReprojectionError.hpp:49-57). The camera is the caller's
// okvisgpu_camera of cameraGeometry_ (its intrinsics).
template <class E>
ReprojectionError fromOkvisReprojectionError(const E& e, const okvisgpu_camera& camera) {
  const auto& m = e.measurement();
  const auto& I = e.information();
  const double kp[2] = {(double)m(0), (double)m(1)};
  const double l00 = std::sqrt((double)I(0, 0)), l10 = (double)I(1, 0) / l00;
  const double l11 = std::sqrt((double)I(1, 1) - l10 * l10);
  const double L[4] = {l00, l10, 0.0, l11};  // L^T row-major
  return ReprojectionError(camera, kp, L);
}
// ---- okvis functor internals. The members okvis keeps the solver state in are protected and have
// no getters (ImuError.hpp:266-305, TwoPoseGraphError.hpp:178,283-284,364-372,
// RelativePoseError.hpp:148-150, PoseError.hpp:166-170, SpeedAndBiasError.hpp:163-168). Each
// accessor below is a class derived from the okvis functor type E that is never instantiated:
// naming a protected member through it (&Members::Delta_q_) forms a pointer to E's member that
// applies to any E object ([class.protected]), so the okvis headers stay unpatched. Eigen objects
// are used only through their call operators / coefficient accessors (m(r, c), v(i), q.x(), ...).
namespace okvis_access {
template <class M>
void matIn(const M& m, int R, int Cn, double* out) {
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < Cn; ++c) out[r * Cn + c] = (double)m(r, c);
}
template <class M>
void matOut(const double* in, int R, int Cn, M& m) {
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < Cn; ++c) m(r, c) = in[r * Cn + c];
}
template <class V>
void vecIn(const V& v, int n, double* out) {
  for (int i = 0; i < n; ++i) out[i] = (double)v(i);
}
template <class T>  // kinematics::Transformation: coeffs() = [r_AB, q_AB xyzw] (Transformation.hpp:122-123)
void transformationIn(const T& t, double* out) {
  const auto& c = t.coeffs();
  for (int i = 0; i < 7; ++i) out[i] = (double)c(i);
}

// okvis::ceres::ImuError's preintegration members <-> the OKVISGPU_IMU_STATE_DOUBLES blob.
template <class E>
struct ImuErrorMembers : E {
  static void read(const E& e, double* s) {
    for (int i = 0; i < OKVISGPU_IMU_STATE_DOUBLES; ++i) s[i] = 0.0;
    s[0] = (double)(e.*(&ImuErrorMembers::redoCounter_));
    s[1] = (e.*(&ImuErrorMembers::redo_)) ? 1.0 : 0.0;
    const auto& q = e.*(&ImuErrorMembers::Delta_q_);
    s[2] = q.x(); s[3] = q.y(); s[4] = q.z(); s[5] = q.w();
    matIn(e.*(&ImuErrorMembers::C_integral_), 3, 3, s + 6);
    matIn(e.*(&ImuErrorMembers::C_doubleintegral_), 3, 3, s + 15);
    vecIn(e.*(&ImuErrorMembers::acc_integral_), 3, s + 24);
    vecIn(e.*(&ImuErrorMembers::acc_doubleintegral_), 3, s + 27);
    matIn(e.*(&ImuErrorMembers::dalpha_db_g_), 3, 3, s + 30);
    matIn(e.*(&ImuErrorMembers::dv_db_g_), 3, 3, s + 39);
    matIn(e.*(&ImuErrorMembers::dp_db_g_), 3, 3, s + 48);
    vecIn(e.*(&ImuErrorMembers::speedAndBiases_ref_), 9, s + 57);
    matIn(e.*(&ImuErrorMembers::squareRootInformation_), 15, 15, s + 66);
    matIn(e.*(&ImuErrorMembers::cross_), 3, 3, s + 292);
    matIn(e.*(&ImuErrorMembers::P_delta_), 15, 15, s + 301);
  }
  // The members are `mutable` in okvis, but a pointer to member cannot modify a const object
  // ([expr.mptr.oper]), hence E&. information_ = U^T U as redoPreintegration / append set it
  // (ImuError.cpp:463,252). dPdsigma_ (the four covariance derivatives ImuError::append continues
  // from, ImuError.cpp:220-223,242-248) is touched only when the GPU changed P_delta_ (it redid or
  // appended the preintegration): it is then written as P_delta_ / sigma_k^2 in the slot of the
  // first non-zero noise density and zero in the others. append's recursion is linear in them, so it
  // continues P_delta_ exactly as from the four separate matrices. Limitation: the four per-sigma
  // matrices themselves are not reproduced after a GPU re-integration (the device carries their
  // sigma^2-weighted sum only), so ImuError::EvaluateWithSigmaGradientAndHessian (not called by
  // okvis' solve) would see the folded slot; a factor the GPU did not re-integrate keeps its own.
  static void write(const double* s, E& e) {
    e.*(&ImuErrorMembers::redoCounter_) = (int)s[0];
    e.*(&ImuErrorMembers::redo_) = s[1] != 0.0;
    auto& q = e.*(&ImuErrorMembers::Delta_q_);
    q.x() = s[2]; q.y() = s[3]; q.z() = s[4]; q.w() = s[5];
    matOut(s + 6, 3, 3, e.*(&ImuErrorMembers::C_integral_));
    matOut(s + 15, 3, 3, e.*(&ImuErrorMembers::C_doubleintegral_));
    auto& ai = e.*(&ImuErrorMembers::acc_integral_);
    auto& ad = e.*(&ImuErrorMembers::acc_doubleintegral_);
    for (int i = 0; i < 3; ++i) { ai(i) = s[24 + i]; ad(i) = s[27 + i]; }
    matOut(s + 30, 3, 3, e.*(&ImuErrorMembers::dalpha_db_g_));
    matOut(s + 39, 3, 3, e.*(&ImuErrorMembers::dv_db_g_));
    matOut(s + 48, 3, 3, e.*(&ImuErrorMembers::dp_db_g_));
    auto& sb = e.*(&ImuErrorMembers::speedAndBiases_ref_);
    for (int i = 0; i < 9; ++i) sb(i) = s[57 + i];
    matOut(s + 66, 15, 15, e.*(&ImuErrorMembers::squareRootInformation_));
    matOut(s + 292, 3, 3, e.*(&ImuErrorMembers::cross_));
    bool pChanged = false;
    {
      const auto& P0 = e.*(&ImuErrorMembers::P_delta_);
      for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 15; ++c) pChanged = pChanged || (double)P0(r, c) != s[301 + 15 * r + c];
    }
    matOut(s + 301, 15, 15, e.*(&ImuErrorMembers::P_delta_));
    const double* U = s + 66;
    auto& info = e.*(&ImuErrorMembers::information_);
    for (int r = 0; r < 15; ++r)
      for (int c = 0; c < 15; ++c) {
        double v = 0.0;
        for (int k = 0; k < 15; ++k) v += U[k * 15 + r] * U[k * 15 + c];
        info(r, c) = v;
      }
    if (!pChanged) return;  // the okvis object's own dPdsigma_ stays (it produced this P_delta_)
    const auto& p = e.imuParameters();
    const double sig[4] = {(double)p.sigma_g_c, (double)p.sigma_a_c, (double)p.sigma_gw_c, (double)p.sigma_aw_c};
    int k0 = -1;
    for (int k = 0; k < 4 && k0 < 0; ++k)
      if (sig[k] != 0.0) k0 = k;
    auto& dP = e.*(&ImuErrorMembers::dPdsigma_);
    dP.resize(4);
    for (int k = 0; k < 4; ++k)
      for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 15; ++c) dP[k](r, c) = k == k0 ? s[301 + 15 * r + c] / (sig[k] * sig[k]) : 0.0;
  }
};

// TwoPoseStandardGraphError(Const): DeltaX_, J_, linearisationPoint_T_S0S1_.
template <class E>
struct TwoPoseMembers : E {
  static void read(const E& e, double* delta_x, double* J, double* lin_point) {
    vecIn(e.*(&TwoPoseMembers::DeltaX_), 6, delta_x);
    matIn(e.*(&TwoPoseMembers::J_), 6, 6, J);
    transformationIn(e.*(&TwoPoseMembers::linearisationPoint_T_S0S1_), lin_point);
  }
};
// RelativePoseError: T_AB_, squareRootInformation_ (RelativePoseError.hpp:148-150).
template <class E>
struct RelativePoseMembers : E {
  static void read(const E& e, double* T_AB, double* sqrt_info) {
    transformationIn(e.*(&RelativePoseMembers::T_AB_), T_AB);
    matIn(e.*(&RelativePoseMembers::squareRootInformation_), 6, 6, sqrt_info);
  }
};
// PoseError: measurement_, squareRootInformation_ (PoseError.hpp:166-170). The stored square root
// is the one Evaluate uses; the diagonal constructor (PoseError.cpp:34-39) sets it to sqrt(diag),
// which for the first-state prior's zero yaw/pitch entries (ViGraph.cpp:348-368) is not an LLT of
// information() (singular), so the member is read rather than recomputed.
template <class E>
struct PoseErrorMembers : E {
  static void read(const E& e, double* meas, double* sqrt_info) {
    transformationIn(e.*(&PoseErrorMembers::measurement_), meas);
    matIn(e.*(&PoseErrorMembers::squareRootInformation_), 6, 6, sqrt_info);
  }
};
// SpeedAndBiasError: measurement_, squareRootInformation_ (SpeedAndBiasError.hpp:163-167).
template <class E>
struct SpeedAndBiasMembers : E {
  static void read(const E& e, double* meas, double* sqrt_info) {
    vecIn(e.*(&SpeedAndBiasMembers::measurement_), 9, meas);
    matIn(e.*(&SpeedAndBiasMembers::squareRootInformation_), 9, 9, sqrt_info);
  }
};

template <class E>
okvisgpu_imu_params imuParams(const E& e) {  // imuParameters() (ImuError.hpp:216-218)
  const auto& p = e.imuParameters();
  okvisgpu_imu_params ip;
  ip.a_max = p.a_max; ip.g_max = p.g_max; ip.sigma_g_c = p.sigma_g_c; ip.sigma_a_c = p.sigma_a_c;
  ip.sigma_gw_c = p.sigma_gw_c; ip.sigma_aw_c = p.sigma_aw_c; ip.g = p.g;
  return ip;
}
template <class E>  // imuMeasurements() (ImuError.hpp:221-223): okvis::Time stamps via toNSec()
void imuSamples(const E& e, std::vector<int64_t>& t, std::vector<double>& ga) {
  t.clear();
  ga.clear();
  for (const auto& m : e.imuMeasurements()) {
    t.push_back((int64_t)m.timeStamp.toNSec());
    for (int k = 0; k < 3; ++k) ga.push_back((double)m.measurement.gyroscopes(k));
    for (int k = 0; k < 3; ++k) ga.push_back((double)m.measurement.accelerometers(k));
  }
}
}  // namespace okvis_access

// A live view of an okvis ImuError object as a GPU-evaluated term: samples, t0 / t1 and the whole
// preintegration state are read from the object when the graph is flattened (so a factor that okvis
// already evaluated keeps its linearisation point, redo flag and counter: ImuError.cpp:834-858), the
// state again before every solve (ImuError::append between solves, ImuError.cpp:63-255), and the
// solved state is written back into the object after the solve, as Ceres' in-place evaluation
// leaves it there. The object is not owned.
template <class E>
class OkvisImuError final : public ImuError {
 public:
  explicit OkvisImuError(E* e)
      : ImuError({}, {}, okvis_access::imuParams(*e), (int64_t)e->t0().toNSec(), (int64_t)e->t1().toNSec()), e_(e) {
    pull();
  }
  void pull() override {
    params = okvis_access::imuParams(*e_);
    t0_ns = (int64_t)e_->t0().toNSec();
    t1_ns = (int64_t)e_->t1().toNSec();
    okvis_access::imuSamples(*e_, sample_t_ns, gyr_acc);
    pullState();
  }
  void pullState() override { okvis_access::ImuErrorMembers<E>::read(*e_, state.data()); }
  void pushState() override { okvis_access::ImuErrorMembers<E>::write(state.data(), *e_); }
  E* object() const { return e_; }

 private:
  E* e_;
};

// ImuError: imuParameters(), imuMeasurements() (deque of Measurement<ImuSensorReadings>), t0(), t1()
// (ImuError.hpp:89-92,216-224) and, through the accessor, the preintegration state. A copy: the
// solved state stays in the returned term (use OkvisImuError<E> to write it back into the object).
template <class E>
ImuError fromOkvisImuError(const E& e) {
  std::vector<int64_t> t;
  std::vector<double> ga;
  okvis_access::imuSamples(e, t, ga);
  ImuError r(std::move(t), std::move(ga), okvis_access::imuParams(e), (int64_t)e.t0().toNSec(),
             (int64_t)e.t1().toNSec());
  okvis_access::ImuErrorMembers<E>::read(e, r.state.data());
  return r;
}
// Writes a term's solved state into the okvis object (what OkvisImuError::pushState does).
template <class E>
void toOkvisImuError(const ImuError& term, E& e) {
  okvis_access::ImuErrorMembers<E>::write(term.state.data(), e);
}
// TwoPoseStandardGraphError / TwoPoseStandardGraphErrorConst (the kind from typeInfo(),
// TwoPoseGraphError.hpp:360-362): DeltaX_, J_, linearisationPoint_T_S0S1_. These are constant
// during a solve (compute() / the const clone set them), so nothing is written back.
template <class E>
TwoPoseGraphError fromOkvisTwoPoseGraphError(const E& e) {
  double dx[6], J[36], lp[7];
  okvis_access::TwoPoseMembers<E>::read(e, dx, J, lp);
  return TwoPoseGraphError(dx, J, lp, std::string(e.typeInfo()) == "TwoPoseStandardGraphErrorConst");
}
// RelativePoseError (ViGraph::addRelativePoseConstraint, ViGraph.cpp:786-808).
template <class E>
RelativePoseError fromOkvisRelativePoseError(const E& e) {
  double T[7], L[36];
  okvis_access::RelativePoseMembers<E>::read(e, T, L);
  return RelativePoseError(T, L);
}
// PoseError: the first-state and extrinsics priors (ViGraph.cpp:348-386).
template <class E>
PoseError fromOkvisPoseError(const E& e) {
  double m[7], L[36];
  okvis_access::PoseErrorMembers<E>::read(e, m, L);
  return PoseError(m, L);
}
// SpeedAndBiasError: the first-state speed / bias prior (ViGraph.cpp:363-370).
template <class E>
SpeedAndBiasError fromOkvisSpeedAndBiasError(const E& e) {
  double m[9], L[81];
  okvis_access::SpeedAndBiasMembers<E>::read(e, m, L);
  return SpeedAndBiasError(m, L);
}

// ---------------------------------------------------------------- Problem
struct ResidualBlock;
using ResidualBlockId = ResidualBlock*;

struct ResidualBlock {
  CostFunction* cost;
  LossFunction* loss;
  std::vector<double*> blocks;
};

class Problem {
 public:
  explicit Problem(int device = 0) : device_(device) {}
  ~Problem() {
    if (ctx_) okvisgpu_ctx_destroy(ctx_);
  }
  Problem(const Problem&) = delete;
  Problem& operator=(const Problem&) = delete;

  // ---- parameter blocks
  void AddParameterBlock(double* values, int size, Manifold* manifold = nullptr) {
    if (!values) throw Error("AddParameterBlock: null pointer");
    if (size != 4 && size != 7 && size != 9) throw Unsupported("parameter block of size " + std::to_string(size));
    auto it = params_.find(values);
    if (it != params_.end()) {  // Ceres: re-adding with the same size is a no-op
      if (it->second.size != size) throw Error("AddParameterBlock: block re-added with another size");
      if (manifold) it->second.manifold = manifold;
      return;
    }
    checkManifold(size, manifold);
    Param p;
    p.size = size;
    p.manifold = manifold;
    p.order = nextOrder_++;
    params_[values] = p;
    dirty_ = true;
  }
  void SetManifold(double* values, Manifold* manifold) {
    Param& p = param(values, "SetManifold");
    checkManifold(p.size, manifold);
    p.manifold = manifold;
    dirty_ = true;
  }
  const Manifold* GetManifold(const double* values) const { return param(values, "GetManifold").manifold; }
  bool HasParameterBlock(const double* values) const { return params_.count(const_cast<double*>(values)) != 0; }
  int NumParameterBlocks() const { return (int)params_.size(); }
  int ParameterBlockSize(const double* values) const { return param(values, "ParameterBlockSize").size; }

  void SetParameterBlockConstant(const double* values) { setConstant(values, true); }
  void SetParameterBlockVariable(double* values) { setConstant(values, false); }
  bool IsParameterBlockConstant(const double* values) const { return param(values, "IsParameterBlockConstant").constant; }

  // Removes the block and every residual block that depends on it (Ceres semantics).
  void RemoveParameterBlock(const double* values) {
    Param& p = param(values, "RemoveParameterBlock");
    std::vector<ResidualBlockId> deps(p.residuals.begin(), p.residuals.end());
    for (ResidualBlockId r : deps) RemoveResidualBlock(r);
    params_.erase(const_cast<double*>(values));
    dirty_ = true;
  }

  // ---- residual blocks
  ResidualBlockId AddResidualBlock(CostFunction* cost, LossFunction* loss, const std::vector<double*>& blocks) {
    if (!cost) throw Error("AddResidualBlock: null cost function");
    const std::string t = cost->typeInfo();
    static const std::set<std::string> known = {"ReprojectionError", "ImuError", "PoseError", "SpeedAndBiasError",
                                                "TwoPoseStandardGraphError", "TwoPoseStandardGraphErrorConst",
                                                "RelativePoseError"};
    const bool host = dynamic_cast<const HostCostFunction*>(cost) != nullptr;
    if (!host && !known.count(t))
      throw Unsupported("cost function \"" + t + "\" has no GPU evaluation (wrap it in a HostCostFunction)");
    if (loss && !host && t != "ReprojectionError") throw Unsupported(t + " with a loss function (okvis adds none)");
    if (loss && t == "ReprojectionError") {  // the device applies CauchyLoss(1) to reprojections
      const okvisgpu_loss d = loss->descriptor();
      if (d.kind != OKVISGPU_LOSS_CAUCHY || d.a != 1.0)
        throw Unsupported(t + " with loss \"" + loss->name() + "\" (reprojections take CauchyLoss(1.0), ViGraph.cpp:338)");
    }
    const std::vector<int> sizes = cost->parameterBlockSizes();
    if (host) {  // the §8b fallback's limits (okvisgpu.h host_*)
      int np = 0, ns = 0;
      for (int s : sizes) {
        if (s == 7) ++np;
        else if (s == 9) ++ns;
        else throw Unsupported(t + ": host-evaluated blocks must be pose-kind (7) or speed/bias (9)");
      }
      if (np > 2 || ns > 2 || sizes.empty())
        throw Unsupported(t + ": host-evaluated factors take 1-4 blocks, at most 2 of each kind");
      if (cost->residualDim() < 1 || cost->residualDim() > OKVISGPU_HOST_MAX_RESIDUALS)
        throw Unsupported(t + ": host-evaluated factors have 1-15 residuals");
    }
    if (sizes.size() != blocks.size()) throw Error("AddResidualBlock: " + t + " expects " + std::to_string(sizes.size()) + " blocks");
    for (size_t k = 0; k < blocks.size(); ++k) {
      auto it = params_.find(blocks[k]);
      if (it == params_.end()) {
        AddParameterBlock(blocks[k], sizes[k]);  // Ceres adds unknown blocks implicitly
        it = params_.find(blocks[k]);
      }
      if (it->second.size != sizes[k]) throw Error("AddResidualBlock: block " + std::to_string(k) + " of " + t + " has size " +
                                                   std::to_string(it->second.size));
    }
    auto rb = std::unique_ptr<ResidualBlock>(new ResidualBlock{cost, loss, blocks});
    ResidualBlockId id = rb.get();
    for (double* b : blocks) params_[b].residuals.insert(id);
    residuals_.push_back(std::move(rb));
    dirty_ = true;
    return id;
  }
  template <class... Ts>
  ResidualBlockId AddResidualBlock(CostFunction* cost, LossFunction* loss, double* x0, Ts*... xs) {
    return AddResidualBlock(cost, loss, std::vector<double*>{x0, xs...});
  }
  void RemoveResidualBlock(ResidualBlockId id) {
    auto it = std::find_if(residuals_.begin(), residuals_.end(), [&](const auto& r) { return r.get() == id; });
    if (it == residuals_.end()) throw Error("RemoveResidualBlock: unknown residual block");
    for (double* b : id->blocks) {
      auto p = params_.find(b);
      if (p != params_.end()) p->second.residuals.erase(id);
    }
    residuals_.erase(it);
    dirty_ = true;
  }
  int NumResidualBlocks() const { return (int)residuals_.size(); }
  void GetParameterBlocksForResidualBlock(const ResidualBlockId id, std::vector<double*>* out) const {
    *out = find(id)->blocks;
  }
  void GetResidualBlocksForParameterBlock(const double* values, std::vector<ResidualBlockId>* out) const {
    const Param& p = param(values, "GetResidualBlocksForParameterBlock");
    out->clear();
    for (const auto& r : residuals_)  // insertion order
      if (p.residuals.count(r.get())) out->push_back(r.get());
  }
  const CostFunction* GetCostFunctionForResidualBlock(const ResidualBlockId id) const { return find(id)->cost; }
  const LossFunction* GetLossFunctionForResidualBlock(const ResidualBlockId id) const { return find(id)->loss; }

  // ---- solve: ::ceres::Solve(options, &problem, &summary) (ViGraph.cpp:1884)
  int Solve(const okvisgpu_options& options, okvisgpu_summary* summary) {
    int rc = ensureContext();
    if (rc != OKVISGPU_OK) return rc;
    if (dirty_ || !uploaded_) {
      build();
      rc = okvisgpu_set_problems(ctx_, &view_, 1);
      if (rc != OKVISGPU_OK) return rc;
      uploaded_ = true;
      dirty_ = false;
      constDirty_.clear();
    } else {
      gatherValues();
      for (const auto& kv : constDirty_) {  // freeze / unfreeze without re-uploading the problem
        rc = okvisgpu_set_block_constant(ctx_, 0, kv.first.first, kv.first.second, kv.second);
        if (rc != OKVISGPU_OK) return rc;
      }
      constDirty_.clear();
      rc = okvisgpu_update_params(ctx_);
      if (rc != OKVISGPU_OK) return rc;
    }
    okvisgpu_summary s;
    rc = okvisgpu_solve(ctx_, &options, &s);
    if (rc != OKVISGPU_OK) return rc;
    scatterValues();
    if (summary) *summary = s;
    return OKVISGPU_OK;
  }

  // Problem::Evaluate(total cost) at the caller's current parameter values.
  int EvaluateCost(double* cost) {
    int rc = ensureContext();
    if (rc != OKVISGPU_OK) return rc;
    build();
    rc = okvisgpu_set_problems(ctx_, &view_, 1);
    if (rc != OKVISGPU_OK) return rc;
    uploaded_ = true;
    dirty_ = false;
    constDirty_.clear();
    return okvisgpu_evaluate(ctx_, 0, cost);
  }

  // ::ceres::Problem::EvaluateResidualBlock(id, apply_loss_function, &cost, residuals, jacobians) at the
  // caller's current parameter values (okvis: the GPS residual dump, ViGraph.hpp:553, which passes no
  // Jacobians). Host cost functions are evaluated on the host through their Evaluate; the GPU terms
  // (ReprojectionError, ImuError, TwoPose / RelativePose edges) through the C ABI's evaluation hooks
  // (the problem is uploaded or its values refreshed first). With apply_loss_function the cost is
  // rho(|r|^2)/2 and r is corrected as Ceres' Corrector does; else cost = |r|^2/2 and the raw r. An
  // ImuError residual is U e with the device's square-root information U (any U with U^T U = the
  // reference's information, DESIGN.md §5: |r| and the cost are the reference's, the components may
  // differ by an orthogonal factor), and the evaluation may re-integrate on the device as
  // ImuError::Evaluate would (not written back into the term). Returns false if a host term's
  // Evaluate fails; Jacobians and the prior terms (PoseError, SpeedAndBiasError) throw Unsupported.
  bool EvaluateResidualBlock(ResidualBlockId id, bool apply_loss_function, double* cost, double* residuals,
                             double** jacobians) {
    const ResidualBlock* rb = find(id);
    if (jacobians) throw Unsupported("EvaluateResidualBlock with Jacobians (okvis requests none, ViGraph.hpp:553)");
    const int dim = rb->cost->residualDim();
    double r[OKVISGPU_HOST_MAX_RESIDUALS];
    if (const auto* h = dynamic_cast<const HostCostFunction*>(rb->cost)) {
      std::vector<const double*> prm(rb->blocks.begin(), rb->blocks.end());
      if (!h->Evaluate(prm.data(), r, nullptr)) return false;
    } else {
      const std::string t = rb->cost->typeInfo();
      const bool rp = t == "TwoPoseStandardGraphError" || t == "TwoPoseStandardGraphErrorConst" || t == "RelativePoseError";
      if (t != "ReprojectionError" && t != "ImuError" && !rp)
        throw Unsupported("EvaluateResidualBlock of " + t + " (no device evaluation hook)");
      if (!refreshDevice()) throw Error(std::string("EvaluateResidualBlock: ") + last_error());
      int idx = 0;  // position among the residuals of the same ABI kind (the order build() emits them)
      for (const auto& o : residuals_) {
        if (o.get() == id) break;
        const std::string u = o->cost->typeInfo();
        const bool urp = u == "TwoPoseStandardGraphError" || u == "TwoPoseStandardGraphErrorConst" || u == "RelativePoseError";
        if (rp ? urp : u == t) ++idx;
      }
      int rc;
      if (t == "ReprojectionError") {
        std::vector<double> all(2 * (size_t)view_.n_observations);
        rc = okvisgpu_eval_reprojection(ctx_, 0, all.data(), nullptr, nullptr);
        if (rc == OKVISGPU_OK) std::copy(all.begin() + 2 * idx, all.begin() + 2 * idx + 2, r);
      } else if (t == "ImuError") {
        std::vector<double> all(15 * (size_t)view_.n_imu);
        rc = okvisgpu_eval_imu(ctx_, 0, 0, all.data(), nullptr);
        if (rc == OKVISGPU_OK) std::copy(all.begin() + 15 * idx, all.begin() + 15 * idx + 15, r);
      } else {
        std::vector<double> all(6 * (size_t)view_.n_relpose);
        rc = okvisgpu_eval_relpose(ctx_, 0, all.data(), nullptr);
        if (rc == OKVISGPU_OK) std::copy(all.begin() + 6 * idx, all.begin() + 6 * idx + 6, r);
      }
      if (rc != OKVISGPU_OK) throw Error(std::string("EvaluateResidualBlock: ") + last_error());
    }
    double sq = 0.0;
    for (int i = 0; i < dim; ++i) sq += r[i] * r[i];
    double c = 0.5 * sq, scale = 1.0;
    if (apply_loss_function && rb->loss) {  // Ceres' Corrector on the residual (corrector.cc)
      double rho[3];
      rb->loss->Evaluate(sq, rho);
      c = 0.5 * rho[0];
      scale = std::sqrt(rho[1]);
      if (sq != 0.0 && rho[2] > 0.0) scale /= std::sqrt(1.0 + 2.0 * sq * rho[2] / rho[1]);  // / (1 - alpha)
    }
    if (cost) *cost = c;
    if (residuals)
      for (int i = 0; i < dim; ++i) residuals[i] = r[i] * scale;
    return true;
  }

  const char* last_error() const { return ctx_ ? okvisgpu_last_error(ctx_) : okvisgpu_last_error(nullptr); }

  // The C-ABI problem the facade hands to okvisgpu_set_problems (rebuilt from the recorded graph;
  // pointers valid until the next structural change). Exposed for inspection and tests.
  const okvisgpu_problem& view() {
    if (dirty_ || !built_) build();
    return view_;
  }
  // Block indices in the view (-1 if not a block of that kind).
  int poseIndex(const double* v) const { return indexIn(poseIdx_, v); }
  int speedBiasIndex(const double* v) const { return indexIn(sbIdx_, v); }
  int landmarkIndex(const double* v) const { return indexIn(lmIdx_, v); }

 private:
  struct Param {
    int size = 0;
    Manifold* manifold = nullptr;
    bool constant = false;
    int64_t order = 0;
    std::set<ResidualBlockId> residuals;
  };
  struct Cam {  // one ABI camera = (extrinsics block, intrinsics)
    double* extr;
    okvisgpu_camera cam;
  };

  static bool sameCamera(const okvisgpu_camera& a, const okvisgpu_camera& b) {
    return a.distortion == b.distortion && a.width == b.width && a.height == b.height && a.fu == b.fu &&
           a.fv == b.fv && a.cu == b.cu && a.cv == b.cv && std::memcmp(a.dist, b.dist, sizeof(a.dist)) == 0;
  }
  static void checkManifold(int size, const Manifold* m) {
    if (m && m->AmbientSize() != size) throw Error(std::string(m->name()) + " on a block of size " + std::to_string(size));
    if (size == 7 && m && std::strcmp(m->name(), "PoseManifold") != 0) throw Unsupported("7-dim block without PoseManifold");
  }
  Param& param(const double* v, const char* what) {
    auto it = params_.find(const_cast<double*>(v));
    if (it == params_.end()) throw Error(std::string(what) + ": unknown parameter block");
    return it->second;
  }
  const Param& param(const double* v, const char* what) const {
    auto it = params_.find(const_cast<double*>(v));
    if (it == params_.end()) throw Error(std::string(what) + ": unknown parameter block");
    return it->second;
  }
  const ResidualBlock* find(ResidualBlockId id) const {
    for (const auto& r : residuals_)
      if (r.get() == id) return id;
    throw Error("unknown residual block");
  }
  static int indexIn(const std::map<double*, int>& m, const double* v) {
    auto it = m.find(const_cast<double*>(v));
    return it == m.end() ? -1 : it->second;
  }
  void setConstant(const double* values, bool c) {
    Param& p = param(values, c ? "SetParameterBlockConstant" : "SetParameterBlockVariable");
    if (p.constant == c) return;
    p.constant = c;
    double* v = const_cast<double*>(values);
    int kind = -1, index = -1;
    if ((index = indexIn(poseIdx_, v)) >= 0) kind = 0;
    else if ((index = indexIn(sbIdx_, v)) >= 0) kind = 1;
    else if ((index = indexIn(lmIdx_, v)) >= 0) kind = 2;
    else if ((index = extrinsicsCamera(v)) >= 0) kind = 3;  // ViSlamBackend.cpp:866-872 freeze
    if (kind < 0 || dirty_ || !uploaded_) dirty_ = true;  // structure rebuilt at the next Solve anyway
    else constDirty_[{kind, index}] = c ? 1 : 0;
  }
  // The ABI camera of an extrinsics block (-1: none, or shared by several cameras).
  int extrinsicsCamera(const double* v) const {
    int ci = -1;
    for (size_t i = 0; i < extrPtr_.size(); ++i)
      if (extrPtr_[i] == v) {
        if (ci >= 0) return -1;
        ci = (int)i;
      }
    return ci;
  }
  int ensureContext() {
    if (ctx_) return OKVISGPU_OK;
    return okvisgpu_ctx_create(device_, &ctx_);
  }
  // the device holds the recorded graph with the caller's current values (as Solve prepares it)
  bool refreshDevice() {
    if (ensureContext() != OKVISGPU_OK) return false;
    if (dirty_ || !uploaded_) {
      build();
      if (okvisgpu_set_problems(ctx_, &view_, 1) != OKVISGPU_OK) return false;
      uploaded_ = true;
      dirty_ = false;
      constDirty_.clear();
      return true;
    }
    gatherValues();
    for (const auto& kv : constDirty_)
      if (okvisgpu_set_block_constant(ctx_, 0, kv.first.first, kv.first.second, kv.second) != OKVISGPU_OK) return false;
    constDirty_.clear();
    return okvisgpu_update_params(ctx_) == OKVISGPU_OK;
  }

  // Flatten the recorded graph into the SoA arrays of okvisgpu_problem. Blocks are ordered by
  // insertion; a 7-dim block is an extrinsics block if it is the third block of a reprojection
  // error, a pose otherwise.
  void build() {
    std::vector<std::pair<int64_t, double*>> order;
    for (auto& kv : params_) order.push_back({kv.second.order, kv.first});
    std::sort(order.begin(), order.end());
    std::set<double*> extrBlocks;
    for (const auto& r : residuals_)
      if (r->cost->typeInfo() == "ReprojectionError") extrBlocks.insert(r->blocks[2]);
    poseIdx_.clear(); sbIdx_.clear(); lmIdx_.clear();
    posePtr_.clear(); sbPtr_.clear(); lmPtr_.clear();
    for (auto& o : order) {
      const Param& p = params_[o.second];
      if (p.size == 7 && !extrBlocks.count(o.second)) { poseIdx_[o.second] = (int)posePtr_.size(); posePtr_.push_back(o.second); }
      else if (p.size == 9) { sbIdx_[o.second] = (int)sbPtr_.size(); sbPtr_.push_back(o.second); }
      else if (p.size == 4) { lmIdx_[o.second] = (int)lmPtr_.size(); lmPtr_.push_back(o.second); }
    }
    A_ = Arrays();
    for (double* b : posePtr_) A_.pose_c.push_back(params_[b].constant);
    for (double* b : sbPtr_) A_.sb_c.push_back(params_[b].constant);
    for (double* b : lmPtr_) A_.lm_c.push_back(params_[b].constant);
    std::vector<Cam> cams;
    auto camIndex = [&](double* extr, const okvisgpu_camera& c) {
      for (size_t i = 0; i < cams.size(); ++i)
        if (cams[i].extr == extr && sameCamera(cams[i].cam, c)) return (int)i;
      cams.push_back(Cam{extr, c});
      return (int)cams.size() - 1;
    };
    auto pidx = [&](double* b, const char* what) {
      const int i = indexIn(poseIdx_, b);
      if (i < 0) throw Error(std::string(what) + ": block is not a pose");
      return i;
    };
    auto sidx = [&](double* b) {
      const int i = indexIn(sbIdx_, b);
      if (i < 0) throw Error("ImuError: block is not a speed/bias block");
      return i;
    };
    A_.imu_begin.push_back(0);
    imuTerms_.clear();
    for (const auto& r : residuals_) {
      const std::string t = r->cost->typeInfo();
      if (t == "ReprojectionError") {
        const auto* e = static_cast<const ReprojectionError*>(r->cost);
        A_.obs_pose.push_back(pidx(r->blocks[0], "ReprojectionError"));
        const int l = indexIn(lmIdx_, r->blocks[1]);
        if (l < 0) throw Error("ReprojectionError: block 1 is not a landmark");
        A_.obs_lm.push_back(l);
        A_.obs_cam.push_back(camIndex(r->blocks[2], e->camera));
        A_.obs_kp.insert(A_.obs_kp.end(), e->keypoint, e->keypoint + 2);
        A_.obs_L.insert(A_.obs_L.end(), e->sqrt_info, e->sqrt_info + 4);
        A_.obs_cauchy.push_back(r->loss != nullptr);
      } else if (t == "ImuError") {
        auto* e = static_cast<ImuError*>(r->cost);
        e->pull();  // a live view re-reads its okvis object (samples may have grown by append)
        const int32_t b[4] = {pidx(r->blocks[0], "ImuError"), sidx(r->blocks[1]), pidx(r->blocks[2], "ImuError"),
                              sidx(r->blocks[3])};
        A_.imu_blocks.insert(A_.imu_blocks.end(), b, b + 4);
        A_.imu_t0.push_back(e->t0_ns);
        A_.imu_t1.push_back(e->t1_ns);
        A_.imu_ts.insert(A_.imu_ts.end(), e->sample_t_ns.begin(), e->sample_t_ns.end());
        A_.imu_ga.insert(A_.imu_ga.end(), e->gyr_acc.begin(), e->gyr_acc.end());
        A_.imu_begin.push_back((int32_t)A_.imu_ts.size());
        A_.imu_state.insert(A_.imu_state.end(), e->state.begin(), e->state.end());
        if (imuTerms_.empty()) A_.imu_params = e->params;
        else if (std::memcmp(&A_.imu_params, &e->params, sizeof(e->params)) != 0)
          throw Unsupported("ImuError terms with different ImuParameters in one graph");
        imuTerms_.push_back(e);
      } else if (t == "PoseError") {
        const auto* e = static_cast<const PoseError*>(r->cost);
        if (extrBlocks.count(r->blocks[0])) {
          A_.ep_cam_ptr.push_back(r->blocks[0]);
          A_.ep_meas.insert(A_.ep_meas.end(), e->meas, e->meas + 7);
          A_.ep_L.insert(A_.ep_L.end(), e->sqrt_info, e->sqrt_info + 36);
        } else {
          A_.pp_block.push_back(pidx(r->blocks[0], "PoseError"));
          A_.pp_meas.insert(A_.pp_meas.end(), e->meas, e->meas + 7);
          A_.pp_L.insert(A_.pp_L.end(), e->sqrt_info, e->sqrt_info + 36);
        }
      } else if (t == "SpeedAndBiasError") {
        const auto* e = static_cast<const SpeedAndBiasError*>(r->cost);
        A_.sbp_block.push_back(sidx(r->blocks[0]));
        A_.sbp_meas.insert(A_.sbp_meas.end(), e->meas, e->meas + 9);
        A_.sbp_L.insert(A_.sbp_L.end(), e->sqrt_info, e->sqrt_info + 81);
      } else if (t == "TwoPoseStandardGraphError" || t == "TwoPoseStandardGraphErrorConst") {
        const auto* e = static_cast<const TwoPoseGraphError*>(r->cost);
        A_.rp_blocks.push_back(pidx(r->blocks[0], t.c_str()));
        A_.rp_blocks.push_back(pidx(r->blocks[1], t.c_str()));
        A_.rp_dx.insert(A_.rp_dx.end(), e->delta_x, e->delta_x + 6);
        A_.rp_J.insert(A_.rp_J.end(), e->J, e->J + 36);
        A_.rp_lp.insert(A_.rp_lp.end(), e->lin_point, e->lin_point + 7);
        A_.rp_kind.push_back(0);
      } else if (t == "RelativePoseError") {
        const auto* e = static_cast<const RelativePoseError*>(r->cost);
        A_.rp_blocks.push_back(pidx(r->blocks[0], t.c_str()));
        A_.rp_blocks.push_back(pidx(r->blocks[1], t.c_str()));
        A_.rp_dx.insert(A_.rp_dx.end(), 6, 0.0);
        A_.rp_J.insert(A_.rp_J.end(), e->sqrt_info, e->sqrt_info + 36);
        A_.rp_lp.insert(A_.rp_lp.end(), e->T_AB, e->T_AB + 7);
        A_.rp_kind.push_back(1);
      }
    }
    // cameras / extrinsics (one ABI camera per distinct (extrinsics block, intrinsics) pair). A
    // variable extrinsics block is ONE Ceres block: seen with two intrinsics it would become two
    // independently optimised ABI blocks, so that graph is rejected.
    for (size_t i = 0; i < cams.size(); ++i)
      for (size_t j = 0; j < i; ++j)
        if (cams[i].extr == cams[j].extr && !params_[cams[i].extr].constant)
          throw Unsupported("a variable extrinsics block observed with two different camera intrinsics");
    extrPtr_.clear();
    for (const Cam& c : cams) {
      A_.cams.push_back(c.cam);
      A_.extr.insert(A_.extr.end(), c.extr, c.extr + 7);
      A_.extr_c.push_back(params_[c.extr].constant);
      extrPtr_.push_back(c.extr);
    }
    for (double* e : A_.ep_cam_ptr) {
      int ci = -1;
      for (size_t i = 0; i < extrPtr_.size(); ++i)
        if (extrPtr_[i] == e) { ci = (int)i; break; }
      A_.ep_cam.push_back(ci);
    }
    // host-evaluated residuals: blocks as (kind, index) in the functor's order; an extrinsics block
    // is the pose-kind block n_poses + camera
    hostTerms_.clear();
    for (const auto& r : residuals_) {
      const auto* h = dynamic_cast<const HostCostFunction*>(r->cost);
      if (!h) continue;
      int32_t kind[4] = {-1, -1, -1, -1}, idx[4] = {-1, -1, -1, -1};
      for (size_t k = 0; k < r->blocks.size(); ++k) {
        double* b = r->blocks[k];
        if (params_[b].size == 9) {
          kind[k] = 1;
          idx[k] = indexIn(sbIdx_, b);
          continue;
        }
        kind[k] = 0;
        if ((idx[k] = indexIn(poseIdx_, b)) >= 0) continue;
        const int c = extrinsicsCamera(b);
        if (c < 0) throw Unsupported(h->typeInfo() + ": an extrinsics block shared by several cameras");
        idx[k] = (int32_t)posePtr_.size() + c;
      }
      A_.host_kind.insert(A_.host_kind.end(), kind, kind + 4);
      A_.host_index.insert(A_.host_index.end(), idx, idx + 4);
      A_.host_dim.push_back(h->residualDim());
      A_.host_loss.push_back(r->loss ? r->loss->descriptor() : okvisgpu_loss{OKVISGPU_LOSS_NONE, 0, 1.0, 0.0});
      hostTerms_.push_back(h);
    }
    gatherValues();
    okvisgpu_problem& P = view_;
    std::memset(&P, 0, sizeof(P));
    P.n_poses = (int32_t)posePtr_.size();
    P.poses = A_.pose.data();
    P.pose_constant = A_.pose_c.data();
    P.n_speed_biases = (int32_t)sbPtr_.size();
    P.speed_biases = A_.sb.data();
    P.speed_bias_constant = A_.sb_c.data();
    P.n_landmarks = (int32_t)lmPtr_.size();
    P.landmarks = A_.lm.data();
    P.landmark_constant = A_.lm_c.data();
    P.n_cameras = (int32_t)A_.cams.size();
    P.cameras = A_.cams.data();
    P.extrinsics = A_.extr.data();
    P.extrinsics_constant = A_.extr_c.data();
    P.n_observations = (int32_t)A_.obs_pose.size();
    P.obs_pose = A_.obs_pose.data();
    P.obs_landmark = A_.obs_lm.data();
    P.obs_camera = A_.obs_cam.data();
    P.obs_keypoint = A_.obs_kp.data();
    P.obs_sqrt_info = A_.obs_L.data();
    P.obs_cauchy = A_.obs_cauchy.data();
    P.n_imu = (int32_t)imuTerms_.size();
    P.imu_blocks = A_.imu_blocks.data();
    P.imu_t0_ns = A_.imu_t0.data();
    P.imu_t1_ns = A_.imu_t1.data();
    P.imu_sample_begin = A_.imu_begin.data();
    P.imu_sample_t_ns = A_.imu_ts.data();
    P.imu_sample_gyr_acc = A_.imu_ga.data();
    P.imu_params = A_.imu_params;
    P.imu_state = A_.imu_state.data();
    P.n_pose_priors = (int32_t)A_.pp_block.size();
    P.pose_prior_block = A_.pp_block.data();
    P.pose_prior_meas = A_.pp_meas.data();
    P.pose_prior_sqrt_info = A_.pp_L.data();
    P.n_sb_priors = (int32_t)A_.sbp_block.size();
    P.sb_prior_block = A_.sbp_block.data();
    P.sb_prior_meas = A_.sbp_meas.data();
    P.sb_prior_sqrt_info = A_.sbp_L.data();
    P.n_relpose = (int32_t)A_.rp_kind.size();
    P.relpose_blocks = A_.rp_blocks.data();
    P.relpose_delta_x = A_.rp_dx.data();
    P.relpose_sqrt_info = A_.rp_J.data();
    P.relpose_lin_point = A_.rp_lp.data();
    P.relpose_kind = A_.rp_kind.data();
    P.n_extrinsics_priors = (int32_t)A_.ep_cam.size();
    P.extrinsics_prior_camera = A_.ep_cam.data();
    P.extrinsics_prior_meas = A_.ep_meas.data();
    P.extrinsics_prior_sqrt_info = A_.ep_L.data();
    P.n_host = (int32_t)hostTerms_.size();
    P.host_dim = A_.host_dim.data();
    P.host_param_kind = A_.host_kind.data();
    P.host_param_index = A_.host_index.data();
    P.host_cauchy = nullptr;
    P.host_loss = A_.host_loss.data();
    P.host_evaluate = &Problem::hostTrampoline;
    P.host_user = this;
    built_ = true;
  }
  static int hostTrampoline(void* user, int32_t factor, const double* const* parameters, double* residuals,
                            double** jacobians) {
    try {
      return static_cast<const Problem*>(user)->hostTerms_[factor]->Evaluate(parameters, residuals, jacobians) ? 1 : 0;
    } catch (...) {  // no exception crosses the C ABI: an evaluation failure
      return 0;
    }
  }
  // caller's parameter memory -> SoA (before a solve)
  void gatherValues() {
    A_.pose.resize(7 * posePtr_.size());
    A_.sb.resize(9 * sbPtr_.size());
    A_.lm.resize(4 * lmPtr_.size());
    for (size_t i = 0; i < posePtr_.size(); ++i) std::memcpy(&A_.pose[7 * i], posePtr_[i], 7 * sizeof(double));
    for (size_t i = 0; i < sbPtr_.size(); ++i) std::memcpy(&A_.sb[9 * i], sbPtr_[i], 9 * sizeof(double));
    for (size_t i = 0; i < lmPtr_.size(); ++i) std::memcpy(&A_.lm[4 * i], lmPtr_[i], 4 * sizeof(double));
    for (size_t i = 0; i < extrPtr_.size() && 7 * i < A_.extr.size(); ++i)
      std::memcpy(&A_.extr[7 * i], extrPtr_[i], 7 * sizeof(double));
    for (size_t f = 0; f < imuTerms_.size(); ++f) {
      imuTerms_[f]->pullState();
      std::memcpy(&A_.imu_state[f * OKVISGPU_IMU_STATE_DOUBLES], imuTerms_[f]->state.data(),
                  OKVISGPU_IMU_STATE_DOUBLES * sizeof(double));
    }
  }
  // SoA -> caller's parameter memory (after a solve): the in-place write-back of Ceres
  void scatterValues() {
    for (size_t i = 0; i < posePtr_.size(); ++i) std::memcpy(posePtr_[i], &A_.pose[7 * i], 7 * sizeof(double));
    for (size_t i = 0; i < sbPtr_.size(); ++i) std::memcpy(sbPtr_[i], &A_.sb[9 * i], 9 * sizeof(double));
    for (size_t i = 0; i < lmPtr_.size(); ++i) std::memcpy(lmPtr_[i], &A_.lm[4 * i], 4 * sizeof(double));
    for (size_t i = 0; i < extrPtr_.size(); ++i) std::memcpy(extrPtr_[i], &A_.extr[7 * i], 7 * sizeof(double));
    for (size_t f = 0; f < imuTerms_.size(); ++f) {
      std::memcpy(imuTerms_[f]->state.data(), &A_.imu_state[f * OKVISGPU_IMU_STATE_DOUBLES],
                  OKVISGPU_IMU_STATE_DOUBLES * sizeof(double));
      imuTerms_[f]->pushState();  // into the okvis object of a live view
    }
  }

  struct Arrays {
    std::vector<double> pose, sb, lm, extr, obs_kp, obs_L, imu_ga, imu_state, pp_meas, pp_L, sbp_meas, sbp_L, rp_dx,
        rp_J, rp_lp, ep_meas, ep_L;
    std::vector<uint8_t> pose_c, sb_c, lm_c, extr_c, obs_cauchy, rp_kind;
    std::vector<okvisgpu_loss> host_loss;
    std::vector<int32_t> obs_pose, obs_lm, obs_cam, imu_blocks, imu_begin, pp_block, sbp_block, rp_blocks, ep_cam,
        host_kind, host_index, host_dim;
    std::vector<int64_t> imu_t0, imu_t1, imu_ts;
    std::vector<okvisgpu_camera> cams;
    std::vector<double*> ep_cam_ptr;
    okvisgpu_imu_params imu_params{};
  };

  int device_;
  okvisgpu_ctx* ctx_ = nullptr;
  std::map<double*, Param> params_;
  std::vector<std::unique_ptr<ResidualBlock>> residuals_;
  int64_t nextOrder_ = 0;
  bool dirty_ = true, uploaded_ = false, built_ = false;
  std::map<std::pair<int, int>, int> constDirty_;
  std::map<double*, int> poseIdx_, sbIdx_, lmIdx_;
  std::vector<double*> posePtr_, sbPtr_, lmPtr_, extrPtr_;
  std::vector<ImuError*> imuTerms_;
  std::vector<const HostCostFunction*> hostTerms_;
  Arrays A_;
  okvisgpu_problem view_{};
};

// ---- the ::ceres::Solve(options_, problem_.get(), &summary_) call shape (ViGraph.cpp:1884), so the
// call site keeps its ceres::Solver::Options / Summary objects. Templates over the caller's types
// (no Ceres type is named here): the options fields okvis sets or relies on (ViGraph.cpp:248-249,
// 1854-1861; Ceres defaults otherwise) are read by their ceres::Solver::Options names. The linear
// solver is passed as a flag (the caller compares `options_.linear_solver_type == ::ceres::
// DENSE_SCHUR`), the trust region is DOGLEG (ViGraph.cpp:249), and the CeresIterationCallback
// time limit / iteration minimum (CeresIterationCallback.cpp:30-38) come as arguments. The summary
// fields are written under their ceres::Solver::Summary names; termination_type is cast to the
// member's enum (okvisgpu_termination follows ceres::TerminationType: CONVERGENCE, NO_CONVERGENCE,
// FAILURE, USER_SUCCESS).
template <class SolverOptions>
okvisgpu_options toOptions(const SolverOptions& o, bool denseSchur = true, double timeLimitS = -1.0,
                           int minIterations = 0) {
  okvisgpu_options r;
  okvisgpu_default_options(&r);
  r.max_num_iterations = o.max_num_iterations;
  r.num_threads = o.num_threads;
  r.linear_solver = denseSchur ? OKVISGPU_DENSE_SCHUR : OKVISGPU_SPARSE_NORMAL_CHOLESKY;
  r.trust_region_strategy = OKVISGPU_DOGLEG;
  r.jacobi_scaling = o.jacobi_scaling ? 1 : 0;
  r.function_tolerance = o.function_tolerance;
  r.gradient_tolerance = o.gradient_tolerance;
  r.parameter_tolerance = o.parameter_tolerance;
  r.initial_trust_region_radius = o.initial_trust_region_radius;
  r.max_trust_region_radius = o.max_trust_region_radius;
  r.min_trust_region_radius = o.min_trust_region_radius;
  r.min_relative_decrease = o.min_relative_decrease;
  r.min_lm_diagonal = o.min_lm_diagonal;
  r.max_lm_diagonal = o.max_lm_diagonal;
  r.max_num_consecutive_invalid_steps = o.max_num_consecutive_invalid_steps;
  r.verbose = o.minimizer_progress_to_stdout ? 1 : 0;
  r.time_limit_s = timeLimitS;
  r.min_iterations = minIterations;
  return r;
}
template <class SolverSummary>
void toSummary(const okvisgpu_summary& s, SolverSummary* out) {
  out->initial_cost = s.initial_cost;
  out->final_cost = s.final_cost;
  out->num_successful_steps = s.num_successful_steps;
  out->num_unsuccessful_steps = s.num_unsuccessful_steps;
  out->termination_type = static_cast<decltype(out->termination_type)>(s.termination_type);
  out->total_time_in_seconds = s.total_time_s;
  // the Summary timing fields FullReport prints (ViGraph.cpp:1887-1889); the device phase times
  // are filled when the solve ran with options.verbose (minimizer_progress_to_stdout), else -1
  out->preprocessor_time_in_seconds = s.preprocessor_time_s;
  out->minimizer_time_in_seconds = s.minimizer_time_s;
  out->postprocessor_time_in_seconds = s.postprocessor_time_s;
  out->linear_solver_time_in_seconds = s.linear_solver_time_s;
  out->residual_evaluation_time_in_seconds = s.residual_evaluation_time_s;
  out->jacobian_evaluation_time_in_seconds = s.jacobian_evaluation_time_s;
}
template <class SolverOptions, class SolverSummary>
int Solve(const SolverOptions& options, Problem* problem, SolverSummary* summary, bool denseSchur = true,
          double timeLimitS = -1.0, int minIterations = 0) {
  okvisgpu_summary s;
  const int rc = problem->Solve(toOptions(options, denseSchur, timeLimitS, minIterations), &s);
  if (rc == OKVISGPU_OK && summary) toSummary(s, summary);
  return rc;
}

}  // namespace okvisgpu
