// solver.cpp — TEST INFRASTRUCTURE ONLY (oracle / CPU baseline "port").
//
// CPU restatement of what `::ceres::Solve` does for okvis' realtime window
// (ViGraph::optimise, okvis_ceres/src/ViGraph.cpp:1844-1890; DENSE_SCHUR at ViSlamBackend.cpp:877,
// DOGLEG at ViGraph.cpp:249). The solver algorithm lives in ceres-solver (un-vendored submodule,
// Ceres >= 2.1, pinned commit not recorded: SURVEY.md §8c) and is restated from its published
// design: TrustRegionMinimizer (Jacobi column scaling fixed at iteration 0, step quality,
// parameter/function/gradient tolerances), DoglegStrategy (traditional dogleg, LM-regularised
// Gauss-Newton step with mu in [1e-8, 1], radius update 0.25/0.75), Corrector for CauchyLoss,
// SchurComplementSolver with dense LLT of the reduced camera matrix. Per-iterate parity with real
// Ceres is UNPINNED (no Ceres in this container); see DESIGN.md.
#include <atomic>
#include <chrono>
#include <cfloat>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <thread>
#include <vector>

#include "oracle.hpp"

namespace oracle {
namespace {

enum Kind { kPose = 0, kSb = 1, kLm = 2, kExt = 3 };  // kExt: extrinsics T_SC (PoseParameterBlock + PoseManifold)
enum RKind { rReproj = 0, rImu = 1, rPosePrior = 2, rSbPrior = 3, rRelPose = 4, rExtPrior = 5, rHost = 6 };

struct PBlock {
  int kind, index;
  int amb, loc;
  bool constant;
  bool active = false;  // used by at least one residual block and not constant
  bool is_e = false;
  int xoff = -1;        // ambient offset in x (active only)
  int toff = -1;        // tangent offset (active only)
};

struct RBlock {
  int kind, index, nres;
  int pb[4];            // parameter block ids (-1 = none)
  int npb;
  bool fixed = false;   // all parameter blocks constant (Ceres removes these; fixed_cost)
  int roff = 0;         // residual offset
  int jacoff = 0;       // offset into the jacobian value store
  int jcols = 0;        // sum of tangent sizes of its ACTIVE blocks
};

struct Program {
  const okvisgpu_problem* p;
  std::vector<PBlock> pbs;
  std::vector<RBlock> rbs;
  std::vector<Camera> cams;
  std::vector<ImuError> imus;
  int poseBase, sbBase, lmBase, extBase;
  int nx = 0, nt = 0, nres = 0, njac = 0;
  int ne = 0;                    // number of active e-blocks (landmarks)
  int eTangent = 0;              // tangent size of all e-blocks (they come first)
  std::vector<int> fblocks;      // active non-e blocks in reduced ordering
  std::vector<int> fOffset;      // per pblock: offset in the reduced system (-1)
  int fdim = 0;
  std::vector<std::vector<int>> chunkRows;  // per e-block (in e order): residual blocks touching it
  std::vector<int> eOrder;       // pblock ids of e-blocks in order
  std::vector<int> noERows;      // non-fixed residual blocks touching no e-block
  std::vector<double> constVals; // ambient values of constant blocks (by pblock id offset)
  std::vector<int> constOff;
  std::atomic<int> hostFailures{0};  // host_evaluate calls that returned 0 (ABI 5 host factors)
};

const double* blockValues(const Program& P, const std::vector<double>& x, int id) {
  const PBlock& b = P.pbs[id];
  if (b.active) return &x[b.xoff];
  return &P.constVals[P.constOff[id]];
}

void buildProgram(const okvisgpu_problem* p, Program& P, bool loadImuState) {
  P.p = p;
  P.poseBase = 0;
  P.sbBase = p->n_poses;
  P.lmBase = p->n_poses + p->n_speed_biases;
  for (int i = 0; i < p->n_poses; ++i)
    P.pbs.push_back(PBlock{kPose, i, 7, 6, p->pose_constant ? p->pose_constant[i] != 0 : false});
  for (int i = 0; i < p->n_speed_biases; ++i)
    P.pbs.push_back(PBlock{kSb, i, 9, 9, p->speed_bias_constant ? p->speed_bias_constant[i] != 0 : false});
  for (int i = 0; i < p->n_landmarks; ++i)
    P.pbs.push_back(PBlock{kLm, i, 4, 3, p->landmark_constant ? p->landmark_constant[i] != 0 : false});
  // one extrinsics block per camera, shared by all states (ViGraph.cpp:330-336,469-473); constant
  // unless online calibration (ViGraph.cpp:372-386)
  P.extBase = (int)P.pbs.size();
  for (int c = 0; c < p->n_cameras; ++c)
    P.pbs.push_back(PBlock{kExt, c, 7, 6, p->extrinsics_constant ? p->extrinsics_constant[c] != 0 : true});
  for (int c = 0; c < p->n_cameras; ++c) {
    const okvisgpu_camera& k = p->cameras[c];
    P.cams.push_back(cameraOf(k));
  }
  auto addR = [&](int kind, int index, int nres, std::initializer_list<int> ids) {
    RBlock r;
    r.kind = kind; r.index = index; r.nres = nres; r.npb = 0;
    for (int id : ids) r.pb[r.npb++] = id;
    P.rbs.push_back(r);
  };
  for (int o = 0; o < p->n_observations; ++o)
    addR(rReproj, o, 2, {P.poseBase + p->obs_pose[o], P.lmBase + p->obs_landmark[o], P.extBase + p->obs_camera[o]});
  for (int f = 0; f < p->n_imu; ++f) {
    const int* b = &p->imu_blocks[4 * f];
    addR(rImu, f, 15, {P.poseBase + b[0], P.sbBase + b[1], P.poseBase + b[2], P.sbBase + b[3]});
    ImuError e;
    e.params = p->imu_params;
    e.t0 = p->imu_t0_ns[f];
    e.t1 = p->imu_t1_ns[f];
    for (int s = p->imu_sample_begin[f]; s < p->imu_sample_begin[f + 1]; ++s) {
      ImuSample m;
      m.t = p->imu_sample_t_ns[s];
      for (int k = 0; k < 3; ++k) {
        m.g[k] = p->imu_sample_gyr_acc[6 * s + k];
        m.a[k] = p->imu_sample_gyr_acc[6 * s + 3 + k];
      }
      e.meas.push_back(m);
    }
    if (loadImuState && p->imu_state) e.loadState(&p->imu_state[(size_t)f * OKVISGPU_IMU_STATE_DOUBLES]);
    P.imus.push_back(e);
  }
  for (int i = 0; i < p->n_pose_priors; ++i) addR(rPosePrior, i, 6, {P.poseBase + p->pose_prior_block[i]});
  for (int i = 0; i < p->n_sb_priors; ++i) addR(rSbPrior, i, 9, {P.sbBase + p->sb_prior_block[i]});
  for (int i = 0; i < p->n_relpose; ++i)
    addR(rRelPose, i, 6, {P.poseBase + p->relpose_blocks[2 * i], P.poseBase + p->relpose_blocks[2 * i + 1]});
  for (int i = 0; i < p->n_extrinsics_priors; ++i)  // PoseError on T_SC (ViGraph.cpp:372-382)
    addR(rExtPrior, i, 6, {P.extBase + p->extrinsics_prior_camera[i]});
  // host-evaluated residual blocks (ABI 5): a user CostFunction on pose-kind / speed-bias blocks,
  // in the functor's parameter order (Ceres ResidualBlock with the blocks' manifolds)
  for (int h = 0; h < p->n_host; ++h) {
    RBlock r;
    r.kind = rHost; r.index = h; r.nres = p->host_dim[h]; r.npb = 0;
    for (int k = 0; k < 4 && p->host_param_kind[4 * h + k] >= 0; ++k) {
      const int kind = p->host_param_kind[4 * h + k], idx = p->host_param_index[4 * h + k];
      r.pb[r.npb++] = kind == 1 ? P.sbBase + idx : idx < p->n_poses ? P.poseBase + idx : P.extBase + idx - p->n_poses;
    }
    P.rbs.push_back(r);
  }

  // Active blocks (Ceres Program::RemoveFixedBlocks: unused or constant blocks removed).
  for (RBlock& r : P.rbs) {
    bool allConst = true;
    for (int k = 0; k < r.npb; ++k)
      if (!P.pbs[r.pb[k]].constant) allConst = false;
    r.fixed = allConst;
    if (!allConst)
      for (int k = 0; k < r.npb; ++k)
        if (!P.pbs[r.pb[k]].constant) P.pbs[r.pb[k]].active = true;
  }
  // Ordering: e-blocks (active landmarks) first, then f-blocks in the reduced ordering convention.
  int xo = 0, to = 0;
  for (size_t id = 0; id < P.pbs.size(); ++id) {
    PBlock& b = P.pbs[id];
    if (b.kind == kLm && b.active) {
      b.is_e = true;
      b.xoff = xo; b.toff = to;
      xo += b.amb; to += b.loc;
      P.eOrder.push_back((int)id);
    }
  }
  P.ne = (int)P.eOrder.size();
  P.eTangent = to;
  P.fOffset.assign(P.pbs.size(), -1);
  const int nmax = std::max(p->n_poses, p->n_speed_biases);
  int fo = 0;
  for (int i = 0; i < nmax; ++i) {
    for (int kind = 0; kind < 2; ++kind) {
      if (kind == 0 && i >= p->n_poses) continue;
      if (kind == 1 && i >= p->n_speed_biases) continue;
      const int id = (kind == 0 ? P.poseBase : P.sbBase) + i;
      PBlock& b = P.pbs[id];
      if (!b.active) continue;
      b.xoff = xo; b.toff = to;
      xo += b.amb; to += b.loc;
      P.fblocks.push_back(id);
      P.fOffset[id] = fo;
      fo += b.loc;
    }
  }
  // variable extrinsics after all states (the reduced ordering of the GPU path: band + border)
  for (int c = 0; c < p->n_cameras; ++c) {
    const int id = P.extBase + c;
    PBlock& b = P.pbs[id];
    if (!b.active) continue;
    b.xoff = xo; b.toff = to;
    xo += b.amb; to += b.loc;
    P.fblocks.push_back(id);
    P.fOffset[id] = fo;
    fo += b.loc;
  }
  P.fdim = fo;
  P.nx = xo;
  P.nt = to;
  // constants store
  P.constOff.assign(P.pbs.size(), -1);
  for (size_t id = 0; id < P.pbs.size(); ++id) {
    const PBlock& b = P.pbs[id];
    if (b.active) continue;
    P.constOff[id] = (int)P.constVals.size();
    const double* src = b.kind == kPose ? &p->poses[7 * b.index]
                        : b.kind == kSb ? &p->speed_biases[9 * b.index]
                        : b.kind == kExt ? &p->extrinsics[7 * b.index]
                                        : &p->landmarks[4 * b.index];
    for (int k = 0; k < b.amb; ++k) P.constVals.push_back(src[k]);
  }
  // residual / jacobian layout and chunks
  std::vector<int> eIndexOf(P.pbs.size(), -1);
  for (int e = 0; e < P.ne; ++e) eIndexOf[P.eOrder[e]] = e;
  P.chunkRows.assign(P.ne, {});
  int ro = 0, jo = 0;
  for (size_t ri = 0; ri < P.rbs.size(); ++ri) {
    RBlock& r = P.rbs[ri];
    if (r.fixed) continue;
    r.roff = ro;
    ro += r.nres;
    r.jcols = 0;
    for (int k = 0; k < r.npb; ++k)
      if (P.pbs[r.pb[k]].active) r.jcols += P.pbs[r.pb[k]].loc;
    r.jacoff = jo;
    jo += r.nres * r.jcols;
    int eb = -1;
    for (int k = 0; k < r.npb; ++k)
      if (P.pbs[r.pb[k]].active && P.pbs[r.pb[k]].is_e) eb = eIndexOf[r.pb[k]];
    if (eb >= 0) P.chunkRows[eb].push_back((int)ri);
    else P.noERows.push_back((int)ri);
  }
  P.nres = ro;
  P.njac = jo;
}

void gatherX(const Program& P, std::vector<double>& x) {
  x.assign(P.nx, 0.0);
  const okvisgpu_problem* p = P.p;
  for (const PBlock& b : P.pbs) {
    if (!b.active) continue;
    const double* src = b.kind == kPose ? &p->poses[7 * b.index]
                        : b.kind == kSb ? &p->speed_biases[9 * b.index]
                        : b.kind == kExt ? &p->extrinsics[7 * b.index]
                                        : &p->landmarks[4 * b.index];
    for (int k = 0; k < b.amb; ++k) x[b.xoff + k] = src[k];
  }
}
void scatterX(const Program& P, const std::vector<double>& x) {
  const okvisgpu_problem* p = P.p;
  for (const PBlock& b : P.pbs) {
    if (!b.active) continue;
    double* dst = b.kind == kPose ? &p->poses[7 * b.index]
                  : b.kind == kSb ? &p->speed_biases[9 * b.index]
                  : b.kind == kExt ? &p->extrinsics[7 * b.index]
                                  : &p->landmarks[4 * b.index];
    for (int k = 0; k < b.amb; ++k) dst[k] = x[b.xoff + k];
  }
}

// Manifold Plus over the whole state (Evaluator::Plus).
void plusAll(const Program& P, const std::vector<double>& x, const double* delta, std::vector<double>& out) {
  out.resize(P.nx);
  for (const PBlock& b : P.pbs) {
    if (!b.active) continue;
    if (b.kind == kPose || b.kind == kExt) posePlus(&x[b.xoff], &delta[b.toff], &out[b.xoff]);
    else if (b.kind == kLm) pointPlus(&x[b.xoff], &delta[b.toff], &out[b.xoff]);
    else for (int k = 0; k < 9; ++k) out[b.xoff + k] = x[b.xoff + k] + delta[b.toff + k];
  }
}

// Persistent worker pool behind parallelFor (Ceres' ThreadPool + ParallelFor: workers are created
// once, not per call). Work is split into nthreads static contiguous chunks, so every result is
// independent of scheduling.
class Pool {
 public:
  static Pool& get() {
    static Pool pool;
    return pool;
  }
  // run job(t) for t in [0, n) on n workers (the caller runs t = 0)
  void run(int n, const std::function<void(int)>& job) {
    std::lock_guard<std::mutex> serial(callMutex_);
    ensure(n - 1);
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &job;
      want_ = n - 1;
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    job(0);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  void ensure(int workers) {
    while ((int)th_.size() < workers) {
      const int id = (int)th_.size() + 1;
      const uint64_t g = gen_;  // only run() (serialised by callMutex_) advances gen_
      th_.emplace_back([this, id, g] { loop(id, g); });
    }
  }
  void loop(int id, uint64_t seen) {  // joins from the job after generation `seen` on
    for (;;) {
      const std::function<void(int)>* job = nullptr;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        if (id > want_) continue;
        job = job_;
      }
      (*job)(id);
      std::lock_guard<std::mutex> lk(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::mutex callMutex_, m_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int want_ = 0, pending_ = 0;
  bool stop_ = false;
};

template <class F>
void parallelFor(int n, int nthreads, F f) {
  if (nthreads <= 1 || n < 64) { for (int i = 0; i < n; ++i) f(i); return; }
  const int chunk = (n + nthreads - 1) / nthreads;
  const int nt = (n + chunk - 1) / chunk;
  const std::function<void(int)> job = [&](int t) {
    const int b = t * chunk, e = std::min(n, b + chunk);
    for (int i = b; i < e; ++i) f(i);
  };
  Pool::get().run(nt, job);
}

// ::ceres::LossFunction::Evaluate of the loss family a problem can attach to host-evaluated
// factors (okvisgpu.h "robust losses"): rho = (rho(s), rho'(s), rho''(s)) as published in
// ceres-solver >= 2.1 internal/ceres/loss_function.cc (un-vendored submodule);
// okvis constructs CauchyLoss(1.0), CauchyLoss(3.0), TukeyLoss(0.1), TukeyLoss(2.0)
// (okvis_ceres/src/ViGraph.cpp:235-238).
void lossEvaluate(const okvisgpu_loss& L, double s, double rho[3]) {
  const double a = L.a, dmin = std::numeric_limits<double>::min();
  switch (L.kind) {
    case OKVISGPU_LOSS_CAUCHY: {  // b = a^2, c = 1/b: b log(1 + s c)
      const double b = a * a, c = 1.0 / b, sum = 1.0 + s * c, inv = 1.0 / sum;
      rho[0] = b * std::log(sum);
      rho[1] = std::max(dmin, inv);
      rho[2] = -c * (inv * inv);
      break;
    }
    case OKVISGPU_LOSS_TUKEY: {  // a^2/3 (1 - (1 - s/a^2)^3) inside, a^2/3 outside
      const double a2 = a * a;
      if (s <= a2) {
        const double v = 1.0 - s / a2, v2 = v * v;
        rho[0] = a2 / 3.0 * (1.0 - v2 * v);
        rho[1] = v2;
        rho[2] = -2.0 / a2 * v;
      } else {
        rho[0] = a2 / 3.0;
        rho[1] = 0.0;
        rho[2] = 0.0;
      }
      break;
    }
    case OKVISGPU_LOSS_HUBER: {
      const double b = a * a;
      if (s > b) {
        const double r = std::sqrt(s);
        rho[0] = 2.0 * a * r - b;
        rho[1] = std::max(dmin, a / r);
        rho[2] = -rho[1] / (2.0 * s);
      } else {
        rho[0] = s;
        rho[1] = 1.0;
        rho[2] = 0.0;
      }
      break;
    }
    case OKVISGPU_LOSS_SOFTLONE: {
      const double b = a * a, c = 1.0 / b, sum = 1.0 + s * c, t = std::sqrt(sum);
      rho[0] = 2.0 * b * (t - 1.0);
      rho[1] = std::max(dmin, 1.0 / t);
      rho[2] = -(c * rho[1]) / (2.0 * sum);
      break;
    }
    case OKVISGPU_LOSS_ARCTAN: {
      const double b = 1.0 / (a * a), sum = 1.0 + s * s * b, inv = 1.0 / sum;
      rho[0] = a * std::atan2(s, a);
      rho[1] = std::max(dmin, inv);
      rho[2] = -2.0 * s * b * (inv * inv);
      break;
    }
    case OKVISGPU_LOSS_TOLERANT: {  // b log(1 + e^((s-a)/b)) - b log(1 + e^(-a/b))
      const double b = L.b, c = b * std::log(1.0 + std::exp(-a / b)), x = (s - a) / b;
      if (x > 36.7) {  // ln(2^53): 1 + e^x == e^x
        rho[0] = s - a - c;
        rho[1] = 1.0;
        rho[2] = 0.0;
      } else {
        const double e = std::exp(x);
        rho[0] = b * std::log(1.0 + e) - c;
        rho[1] = std::max(dmin, e / (1.0 + e));
        rho[2] = 0.5 / (b * (1.0 + std::cosh(x)));
      }
      break;
    }
    default:
      rho[0] = s;
      rho[1] = 1.0;
      rho[2] = 0.0;
  }
}

// Ceres' Corrector (internal/ceres/corrector.cc; okvis restates it at TwoPoseGraphError.cpp:292-337)
// on the raw residual rr (squared norm sq) and the minimal (tangent-space) Jacobian, as Ceres'
// ResidualBlock applies it after the manifold: returns the cost rho(sq)/2; res (may be NULL) =
// corrected residual; jac (may be NULL; row-major nres x ncols) corrected in place. rho'' <= 0 or
// sq = 0: r and J scaled by sqrt(rho'); rho'' > 0: alpha = 1 - sqrt(1 + 2 sq rho''/rho'), r scaled by
// sqrt(rho')/(1 - alpha), J <- sqrt(rho') (J - alpha/sq r (r^T J)), column by column.
double applyCorrector(const okvisgpu_loss& loss, int nres, int ncols, const double* rr, double sq, double* res,
                      double* jac) {
  double rho[3];
  lossEvaluate(loss, sq, rho);
  const double sqrtRho1 = std::sqrt(rho[1]);
  double scale = sqrtRho1, alphaSq = 0.0;
  if (sq != 0.0 && rho[2] > 0.0) {
    const double D = 1.0 + 2.0 * sq * rho[2] / rho[1];
    const double alpha = 1.0 - std::sqrt(D);
    scale = sqrtRho1 / (1.0 - alpha);
    alphaSq = alpha / sq;
  }
  if (res)
    for (int i = 0; i < nres; ++i) res[i] = rr[i] * scale;
  if (jac)
    for (int c = 0; c < ncols; ++c) {
      if (alphaSq == 0.0) {
        for (int i = 0; i < nres; ++i) jac[i * ncols + c] *= sqrtRho1;
        continue;
      }
      double rtj = 0.0;
      for (int i = 0; i < nres; ++i) rtj += jac[i * ncols + c] * rr[i];
      for (int i = 0; i < nres; ++i) jac[i * ncols + c] = sqrtRho1 * (jac[i * ncols + c] - alphaSq * rr[i] * rtj);
    }
  return 0.5 * rho[0];
}

// Evaluate one residual block: residuals (corrected), local Jacobian (corrected, row-major
// nres x jcols over the ACTIVE blocks in parameter order), cost contribution.
double evalResidual(Program& P, const std::vector<double>& x, int ri, double* res, double* jac,
                    bool redoAlways) {
  RBlock& r = P.rbs[ri];
  const okvisgpu_problem* p = P.p;
  const double* prm[4];
  for (int k = 0; k < r.npb; ++k) prm[k] = blockValues(P, x, r.pb[k]);
  double ambJ[4][15 * 9];
  double* ja[4] = {nullptr, nullptr, nullptr, nullptr};
  if (jac)
    for (int k = 0; k < r.npb; ++k)
      if (P.pbs[r.pb[k]].active) ja[k] = ambJ[k];
  double rr[15];
  bool useLoss = false;
  okvisgpu_loss loss{OKVISGPU_LOSS_CAUCHY, 0, 1.0, 0.0};  // CauchyLoss(1) unless a host factor says otherwise
  switch (r.kind) {
    case rReproj: {
      const int o = r.index;
      const int cam = p->obs_camera[o];
      reprojectionEvaluate(P.cams[cam], &p->obs_keypoint[2 * o], &p->obs_sqrt_info[4 * o], prm[0], prm[1],
                           prm[2], rr, ja[0], ja[1], ja[2], nullptr, nullptr, nullptr);
      useLoss = p->obs_cauchy ? p->obs_cauchy[o] != 0 : true;
      break;
    }
    case rImu: {
      double* jj[4] = {ja[0], ja[1], ja[2], ja[3]};
      P.imus[r.index].evaluate(prm, rr, jac ? jj : nullptr, nullptr, redoAlways);
      break;
    }
    case rPosePrior:
      poseErrorEvaluate(&p->pose_prior_meas[7 * r.index], &p->pose_prior_sqrt_info[36 * r.index], prm[0], rr,
                        ja[0], nullptr);
      break;
    case rSbPrior:
      sbErrorEvaluate(&p->sb_prior_meas[9 * r.index], &p->sb_prior_sqrt_info[81 * r.index], prm[0], rr, ja[0]);
      break;
    case rExtPrior:
      poseErrorEvaluate(&p->extrinsics_prior_meas[7 * r.index], &p->extrinsics_prior_sqrt_info[36 * r.index], prm[0],
                        rr, ja[0], nullptr);
      break;
    case rRelPose:  // no loss function (ViGraphEstimator.cpp:770, ViGraph.cpp:801)
      relPoseBlockEvaluate(p, r.index, prm[0], prm[1], rr, nullptr, nullptr, ja[0], ja[1]);
      break;
    case rHost: {  // the caller's Evaluate; Jacobians always requested (okvisgpu.h host_evaluate)
      double* jall[4] = {ambJ[0], ambJ[1], ambJ[2], ambJ[3]};
      for (int k = 0; k < 4; ++k) std::memset(ambJ[k], 0, sizeof(ambJ[k]));
      for (int i = 0; i < 15; ++i) rr[i] = 0.0;
      if (!p->host_evaluate(p->host_user, r.index, prm, rr, jall)) {  // Ceres: cost = max, step rejected
        P.hostFailures.fetch_add(1);
        if (res) for (int i = 0; i < r.nres; ++i) res[i] = 0.0;
        if (jac) for (int i = 0; i < r.nres * r.jcols; ++i) jac[i] = 0.0;
        return HUGE_VAL;
      }
      if (p->host_loss) {  // ABI 6: the factor's own loss
        loss = p->host_loss[r.index];
        useLoss = loss.kind != OKVISGPU_LOSS_NONE;
      } else {
        useLoss = p->host_cauchy ? p->host_cauchy[r.index] != 0 : false;
      }
      break;
    }
  }
  double sq = 0;
  for (int i = 0; i < r.nres; ++i) sq += rr[i] * rr[i];
  double cost = 0.5 * sq;
  if (res)
    for (int i = 0; i < r.nres; ++i) res[i] = rr[i];
  if (jac) {
    // local Jacobian = ambient * PlusJacobian (Ceres ResidualBlock with manifold)
    int col = 0;
    for (int k = 0; k < r.npb; ++k) {
      const PBlock& b = P.pbs[r.pb[k]];
      if (!b.active) continue;
      if (b.kind == kPose || b.kind == kExt) {
        double Jp[42];
        posePlusJacobian(prm[k], Jp);
        for (int i = 0; i < r.nres; ++i)
          for (int c = 0; c < 6; ++c) {
            double s = 0;
            for (int a = 0; a < 7; ++a) s += ambJ[k][i * 7 + a] * Jp[a * 6 + c];
            jac[i * r.jcols + col + c] = s;
          }
      } else if (b.kind == kLm) {
        for (int i = 0; i < r.nres; ++i)
          for (int c = 0; c < 3; ++c) jac[i * r.jcols + col + c] = ambJ[k][i * 4 + c];
      } else {
        for (int i = 0; i < r.nres; ++i)
          for (int c = 0; c < 9; ++c) jac[i * r.jcols + col + c] = ambJ[k][i * 9 + c];
      }
      col += b.loc;
    }
  }
  if (useLoss) cost = applyCorrector(loss, r.nres, r.jcols, rr, sq, res, jac);
  return cost;
}

struct Linearization {
  std::vector<double> res, jac;
};

// ProgramEvaluator::Evaluate. Returns false never (functors always succeed).
double evaluateAll(Program& P, const std::vector<double>& x, Linearization* lin, int nthreads,
                   bool redoAlways) {
  const int nr = (int)P.rbs.size();
  std::vector<double> costs(nr, 0.0);
  if (lin) { lin->res.assign(P.nres, 0.0); lin->jac.assign(P.njac, 0.0); }
  parallelFor(nr, nthreads, [&](int ri) {
    const RBlock& r = P.rbs[ri];
    if (r.fixed) return;
    costs[ri] = evalResidual(P, x, ri, lin ? &lin->res[r.roff] : nullptr, lin ? &lin->jac[r.jacoff] : nullptr,
                             redoAlways);
  });
  double c = 0;
  for (int ri = 0; ri < nr; ++ri) c += costs[ri];
  return c;
}

double fixedCost(Program& P, int nthreads, bool redoAlways) {
  std::vector<double> x;  // no active blocks referenced by fixed residuals
  double c = 0;
  for (size_t ri = 0; ri < P.rbs.size(); ++ri) {
    if (!P.rbs[ri].fixed) continue;
    double rr[15];
    c += evalResidual(P, x, (int)ri, rr, nullptr, redoAlways);
  }
  (void)nthreads;
  return c;
}

// Per-column (tangent) helpers over the block-sparse Jacobian.
template <class F>
void forEachJacBlock(const Program& P, int ri, F f) {
  const RBlock& r = P.rbs[ri];
  int col = 0;
  for (int k = 0; k < r.npb; ++k) {
    const PBlock& b = P.pbs[r.pb[k]];
    if (!b.active) continue;
    f(b, col);
    col += b.loc;
  }
}

void squaredColumnNorm(const Program& P, const Linearization& L, std::vector<double>& out) {
  out.assign(P.nt, 0.0);
  for (size_t ri = 0; ri < P.rbs.size(); ++ri) {
    const RBlock& r = P.rbs[ri];
    if (r.fixed) continue;
    const double* J = &L.jac[r.jacoff];
    forEachJacBlock(P, (int)ri, [&](const PBlock& b, int col) {
      for (int i = 0; i < r.nres; ++i)
        for (int c = 0; c < b.loc; ++c) out[b.toff + c] += J[i * r.jcols + col + c] * J[i * r.jcols + col + c];
    });
  }
}
void scaleColumns(const Program& P, Linearization& L, const std::vector<double>& s) {
  for (size_t ri = 0; ri < P.rbs.size(); ++ri) {
    const RBlock& r = P.rbs[ri];
    if (r.fixed) continue;
    double* J = &L.jac[r.jacoff];
    forEachJacBlock(P, (int)ri, [&](const PBlock& b, int col) {
      for (int i = 0; i < r.nres; ++i)
        for (int c = 0; c < b.loc; ++c) J[i * r.jcols + col + c] *= s[b.toff + c];
    });
  }
}
// y += J^T v
void leftMultiply(const Program& P, const Linearization& L, const double* v, double* y) {
  for (size_t ri = 0; ri < P.rbs.size(); ++ri) {
    const RBlock& r = P.rbs[ri];
    if (r.fixed) continue;
    const double* J = &L.jac[r.jacoff];
    forEachJacBlock(P, (int)ri, [&](const PBlock& b, int col) {
      for (int i = 0; i < r.nres; ++i)
        for (int c = 0; c < b.loc; ++c) y[b.toff + c] += J[i * r.jcols + col + c] * v[r.roff + i];
    });
  }
}
// y += J v
void rightMultiply(const Program& P, const Linearization& L, const double* v, double* y) {
  for (size_t ri = 0; ri < P.rbs.size(); ++ri) {
    const RBlock& r = P.rbs[ri];
    if (r.fixed) continue;
    const double* J = &L.jac[r.jacoff];
    forEachJacBlock(P, (int)ri, [&](const PBlock& b, int col) {
      for (int i = 0; i < r.nres; ++i) {
        double s = 0;
        for (int c = 0; c < b.loc; ++c) s += J[i * r.jcols + col + c] * v[b.toff + c];
        y[r.roff + i] += s;
      }
    });
  }
}

}  // namespace

// ------------------------------------------------------------------ dense LLT (Eigen LLT semantics)
// Blocked right-looking Cholesky of the lower triangle of a row-major n x n matrix, in place.
// Fails (returns k+1) at the first non-positive pivot like Eigen::LLT (x <= 0).
// Envelope (profile) aware: with first[i] the column of row i's first non-zero, the factor keeps
// that envelope (no fill left of it), so only products inside it are formed. The reduced camera
// matrix of a sliding window is block-banded, so this does O(n b^2) instead of O(n^3 / 3) work;
// the values are those of the dense algorithm (the skipped terms are exact zeros).
int denseCholesky(int n, double* A, int nthreads) {
  const int nb = 64;
  std::vector<int> first(n);
  for (int i = 0; i < n; ++i) {
    const double* Ai = &A[(size_t)i * n];
    int j = 0;
    while (j < i && Ai[j] == 0.0) ++j;
    first[i] = j;
  }
  std::vector<int> rows;
  for (int k0 = 0; k0 < n; k0 += nb) {
    const int k1 = std::min(n, k0 + nb);
    // unblocked factorisation of the diagonal block
    for (int k = k0; k < k1; ++k) {
      const int jk = std::max(k0, first[k]);
      double d = A[(size_t)k * n + k];
      for (int j = jk; j < k; ++j) d -= A[(size_t)k * n + j] * A[(size_t)k * n + j];
      if (!(d > 0.0)) return k + 1;
      d = std::sqrt(d);
      A[(size_t)k * n + k] = d;
      for (int i = k + 1; i < k1; ++i) {
        if (first[i] > k) continue;
        double s = A[(size_t)i * n + k];
        for (int j = std::max(jk, first[i]); j < k; ++j) s -= A[(size_t)i * n + j] * A[(size_t)k * n + j];
        A[(size_t)i * n + k] = s / d;
      }
    }
    if (k1 >= n) break;
    // rows below the block whose envelope reaches into it
    rows.clear();
    for (int i = k1; i < n; ++i)
      if (first[i] < k1) rows.push_back(i);
    const int nr = (int)rows.size();
    // panel: L_ik = (A_ik - sum_j<k L_ij L_kj) / L_kk
    parallelFor(nr, nthreads, [&](int ii) {
      const int i = rows[ii];
      double* Ai = &A[(size_t)i * n];
      for (int k = std::max(k0, first[i]); k < k1; ++k) {
        double s = Ai[k];
        const double* Ak = &A[(size_t)k * n];
        for (int j = std::max(std::max(k0, first[i]), first[k]); j < k; ++j) s -= Ai[j] * Ak[j];
        Ai[k] = s / Ak[k];
      }
    });
    // trailing update: A_ij -= L_i(k0:k1) . L_j(k0:k1) for rows i, j of the list, j <= i
    parallelFor(nr, nthreads, [&](int ii) {
      const int i = rows[ii];
      double* Ai = &A[(size_t)i * n];
      for (int jj = 0; jj <= ii; ++jj) {
        const int j = rows[jj];
        const int lo = std::max(k0, std::max(first[i], first[j]));
        const double* Li = Ai;
        const double* Lj = &A[(size_t)j * n];
        double s = 0;
        for (int k = lo; k < k1; ++k) s += Li[k] * Lj[k];
        Ai[j] -= s;
      }
    });
  }
  return 0;
}

namespace {

void choleskySolve(int n, const double* L, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int j = 0; j < i; ++j) s -= L[(size_t)i * n + j] * b[j];
    b[i] = s / L[(size_t)i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < n; ++j) s -= L[(size_t)j * n + i] * b[j];
    b[i] = s / L[(size_t)i * n + i];
  }
}

// Invert a small SPD matrix via LLT (InvertPSDMatrix, assume full rank). Returns false if not PD.
bool invertSpd3(const double* A, double* inv) {
  double L[9] = {0};
  for (int k = 0; k < 3; ++k) {
    double d = A[k * 3 + k];
    for (int j = 0; j < k; ++j) d -= L[k * 3 + j] * L[k * 3 + j];
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    L[k * 3 + k] = d;
    for (int i = k + 1; i < 3; ++i) {
      double s = A[i * 3 + k];
      for (int j = 0; j < k; ++j) s -= L[i * 3 + j] * L[k * 3 + j];
      L[i * 3 + k] = s / d;
    }
  }
  for (int c = 0; c < 3; ++c) {
    double e[3] = {0, 0, 0};
    e[c] = 1.0;
    choleskySolve(3, L, e);
    for (int r = 0; r < 3; ++r) inv[r * 3 + c] = e[r];
  }
  return true;
}

// SchurComplementSolver (DENSE_SCHUR): build the reduced system for J (already column scaled),
// residuals b and diagonal D. Outputs lhs (fdim^2, full symmetric), rhs (fdim), and per-e-block
// inverse(E^T E + D_e^2) / g_e for the back substitution.
struct Reduced {
  std::vector<double> lhs, rhs;
  std::vector<double> einv;  // [ne][9]
  bool ok = true;
};

void buildReduced(const Program& P, const Linearization& L, const double* D, Reduced& R, int nthreads) {
  const int fd = P.fdim;
  R.lhs.assign((size_t)fd * fd, 0.0);
  R.rhs.assign(fd, 0.0);
  R.einv.assign((size_t)P.ne * 9, 0.0);
  R.ok = true;
  // Rows without e-blocks: lhs += F^T F, rhs += F^T b (SchurEliminator NoEBlockRowsUpdate).
  for (int ri : P.noERows) {
    const RBlock& r = P.rbs[ri];
    const double* J = &L.jac[r.jacoff];
    const double* b = &L.res[r.roff];
    std::vector<std::pair<int, int>> cols;  // (fOffset, local col)
    forEachJacBlock(P, ri, [&](const PBlock& pb, int col) {
      const int id = (int)(&pb - &P.pbs[0]);
      cols.push_back({P.fOffset[id], col});
      (void)pb;
    });
    int ci = 0;
    for (int k = 0; k < r.npb; ++k) {
      const PBlock& pa = P.pbs[r.pb[k]];
      if (!pa.active) continue;
      const int fa = cols[ci].first, ca = cols[ci].second;
      ++ci;
      for (int u = 0; u < pa.loc; ++u) {
        double g = 0;
        for (int i = 0; i < r.nres; ++i) g += J[i * r.jcols + ca + u] * b[i];
        R.rhs[fa + u] += g;
      }
      int cj = 0;
      for (int m = 0; m < r.npb; ++m) {
        const PBlock& pc = P.pbs[r.pb[m]];
        if (!pc.active) continue;
        const int fc = cols[cj].first, cc = cols[cj].second;
        ++cj;
        for (int u = 0; u < pa.loc; ++u)
          for (int v = 0; v < pc.loc; ++v) {
            double s = 0;
            for (int i = 0; i < r.nres; ++i) s += J[i * r.jcols + ca + u] * J[i * r.jcols + cc + v];
            R.lhs[(size_t)(fa + u) * fd + fc + v] += s;
          }
      }
    }
  }
  // Chunks: one per e-block (landmark). Phase 1 (parallel over landmarks): per landmark and
  // f-block the local F^T F, F^T b and W = F^T E, then (E^T E + D^2)^-1 and z. Phase 2 (parallel
  // over owners of f-block rows): every lhs / rhs row is accumulated by one thread, landmark by
  // landmark in e order, so the result does not depend on the thread count.
  struct FAcc { int fid; int foff; int loc; double W[27]; double H[81]; double g[9]; };
  // F^T F between two different f-blocks of one row (a reprojection error with variable
  // extrinsics touches the pose and the extrinsics: SchurEliminator's EBlockRowOuterProduct)
  struct Cross { int fa, fc; int la, lc; double H[81]; };
  struct Chunk { std::vector<FAcc> f; std::vector<Cross> x; double z[3]; };
  std::vector<Chunk> chunks(P.ne);
  std::vector<int> failed(P.ne, 0);
  parallelFor(P.ne, nthreads, [&](int e) {
    const int eid = P.eOrder[e];
    const PBlock& eb = P.pbs[eid];
    double ete[9] = {0}, ge[3] = {0};
    std::vector<FAcc>& facc = chunks[e].f;
    for (int ri : P.chunkRows[e]) {
      const RBlock& r = P.rbs[ri];
      const double* J = &L.jac[r.jacoff];
      const double* b = &L.res[r.roff];
      int ecol = -1;
      forEachJacBlock(P, ri, [&](const PBlock& pb, int col) { if (&pb == &eb) ecol = col; });
      for (int u = 0; u < 3; ++u) {
        for (int v = 0; v < 3; ++v) {
          double s = 0;
          for (int i = 0; i < r.nres; ++i) s += J[i * r.jcols + ecol + u] * J[i * r.jcols + ecol + v];
          ete[u * 3 + v] += s;
        }
        double g = 0;
        for (int i = 0; i < r.nres; ++i) g += J[i * r.jcols + ecol + u] * b[i];
        ge[u] += g;
      }
      forEachJacBlock(P, ri, [&](const PBlock& pb, int col) {
        if (&pb == &eb) return;
        const int id = (int)(&pb - &P.pbs[0]);
        FAcc* a = nullptr;
        for (auto& x : facc) if (x.fid == id) a = &x;
        if (!a) {
          facc.push_back(FAcc{id, P.fOffset[id], pb.loc, {0}, {0}, {0}});
          a = &facc.back();
        }
        for (int u = 0; u < pb.loc; ++u)
          for (int v = 0; v < 3; ++v) {
            double s = 0;
            for (int i = 0; i < r.nres; ++i) s += J[i * r.jcols + col + u] * J[i * r.jcols + ecol + v];
            a->W[u * 3 + v] += s;
          }
        // F^T F (diagonal f block) and F^T b
        for (int u = 0; u < pb.loc; ++u) {
          double g = 0;
          for (int i = 0; i < r.nres; ++i) g += J[i * r.jcols + col + u] * b[i];
          a->g[u] += g;
          for (int v = 0; v < pb.loc; ++v) {
            double s = 0;
            for (int i = 0; i < r.nres; ++i) s += J[i * r.jcols + col + u] * J[i * r.jcols + col + v];
            a->H[u * pb.loc + v] += s;
          }
        }
        // F^T F with the row's other f-blocks
        forEachJacBlock(P, ri, [&](const PBlock& pc, int col2) {
          if (&pc == &eb || &pc == &pb) return;
          const int id2 = (int)(&pc - &P.pbs[0]);
          Cross* x = nullptr;
          for (auto& y : chunks[e].x) if (y.fa == id && y.fc == id2) x = &y;
          if (!x) {
            chunks[e].x.push_back(Cross{id, id2, pb.loc, pc.loc, {0}});
            x = &chunks[e].x.back();
          }
          for (int u = 0; u < pb.loc; ++u)
            for (int v = 0; v < pc.loc; ++v) {
              double s = 0;
              for (int i = 0; i < r.nres; ++i) s += J[i * r.jcols + col + u] * J[i * r.jcols + col2 + v];
              x->H[u * pc.loc + v] += s;
            }
        });
      });
    }
    if (D)
      for (int u = 0; u < 3; ++u) ete[u * 3 + u] += D[eb.toff + u] * D[eb.toff + u];
    double inv[9];
    if (!invertSpd3(ete, inv)) { failed[e] = 1; return; }
    for (int k = 0; k < 9; ++k) R.einv[(size_t)e * 9 + k] = inv[k];
    for (int u = 0; u < 3; ++u)
      chunks[e].z[u] = inv[u * 3 + 0] * ge[0] + inv[u * 3 + 1] * ge[1] + inv[u * 3 + 2] * ge[2];
  });
  for (int e = 0; e < P.ne; ++e)
    if (failed[e]) { R.ok = false; return; }
  // phase 2: thread t owns the f-blocks t, t + T, ... (rows of lhs / rhs)
  const int nf = (int)P.fblocks.size();
  std::vector<int> ownerOf(P.pbs.size(), -1);
  const int T = std::max(1, std::min(nthreads, nf));
  for (int k = 0; k < nf; ++k) ownerOf[P.fblocks[k]] = k % T;
  auto rowPass = [&](int t) {
    for (int e = 0; e < P.ne; ++e) {
      const Chunk& c = chunks[e];
      const double* inv = &R.einv[(size_t)e * 9];
      for (const Cross& x : c.x) {
        if (ownerOf[x.fa] != t) continue;
        const int fa = P.fOffset[x.fa], fc = P.fOffset[x.fc];
        for (int u = 0; u < x.la; ++u)
          for (int v = 0; v < x.lc; ++v) R.lhs[(size_t)(fa + u) * fd + fc + v] += x.H[u * x.lc + v];
      }
      for (const FAcc& a : c.f) {
        if (ownerOf[a.fid] != t) continue;
        for (int u = 0; u < a.loc; ++u) {
          R.rhs[a.foff + u] += a.g[u];
          for (int v = 0; v < a.loc; ++v) R.lhs[(size_t)(a.foff + u) * fd + a.foff + v] += a.H[u * a.loc + v];
        }
        // rhs_f -= W_f z
        for (int u = 0; u < a.loc; ++u)
          R.rhs[a.foff + u] -= a.W[u * 3 + 0] * c.z[0] + a.W[u * 3 + 1] * c.z[1] + a.W[u * 3 + 2] * c.z[2];
        // Y = W_f inv  (loc x 3); lhs_ac -= Y W_c^T
        double Y[27];
        for (int u = 0; u < a.loc; ++u)
          for (int v = 0; v < 3; ++v)
            Y[u * 3 + v] = a.W[u * 3 + 0] * inv[0 * 3 + v] + a.W[u * 3 + 1] * inv[1 * 3 + v] + a.W[u * 3 + 2] * inv[2 * 3 + v];
        for (const FAcc& cc : c.f)
          for (int u = 0; u < a.loc; ++u)
            for (int v = 0; v < cc.loc; ++v)
              R.lhs[(size_t)(a.foff + u) * fd + cc.foff + v] -=
                  Y[u * 3 + 0] * cc.W[v * 3 + 0] + Y[u * 3 + 1] * cc.W[v * 3 + 1] + Y[u * 3 + 2] * cc.W[v * 3 + 2];
      }
    }
  };
  if (T <= 1) rowPass(0);
  else {
    const std::function<void(int)> job = rowPass;
    Pool::get().run(T, job);
  }
  if (D)
    for (int f : P.fblocks) {
      const PBlock& b = P.pbs[f];
      const int fo = P.fOffset[f];
      for (int u = 0; u < b.loc; ++u) R.lhs[(size_t)(fo + u) * fd + fo + u] += D[b.toff + u] * D[b.toff + u];
    }
}

// Back substitution y_e = (E^T E + D^2)^-1 (E^T b - E^T F y_f) for every chunk.
void backSubstitute(const Program& P, const Linearization& L, const Reduced& R, const double* yf, double* y) {
  for (int f : P.fblocks) {
    const PBlock& b = P.pbs[f];
    for (int u = 0; u < b.loc; ++u) y[b.toff + u] = yf[P.fOffset[f] + u];
  }
  for (int e = 0; e < P.ne; ++e) {
    const int eid = P.eOrder[e];
    const PBlock& eb = P.pbs[eid];
    double rhs[3] = {0, 0, 0};
    for (int ri : P.chunkRows[e]) {
      const RBlock& r = P.rbs[ri];
      const double* J = &L.jac[r.jacoff];
      const double* bb = &L.res[r.roff];
      int ecol = -1;
      forEachJacBlock(P, ri, [&](const PBlock& pb, int col) { if (&pb == &eb) ecol = col; });
      for (int i = 0; i < r.nres; ++i) {
        double sj = bb[i];
        forEachJacBlock(P, ri, [&](const PBlock& pb, int col) {
          if (&pb == &eb) return;
          const int id = (int)(&pb - &P.pbs[0]);
          for (int c = 0; c < pb.loc; ++c) sj -= J[i * r.jcols + col + c] * yf[P.fOffset[id] + c];
        });
        for (int u = 0; u < 3; ++u) rhs[u] += J[i * r.jcols + ecol + u] * sj;
      }
    }
    const double* inv = &R.einv[(size_t)e * 9];
    for (int u = 0; u < 3; ++u)
      y[eb.toff + u] = inv[u * 3 + 0] * rhs[0] + inv[u * 3 + 1] * rhs[1] + inv[u * 3 + 2] * rhs[2];
  }
}

double nowS() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double vnorm(const std::vector<double>& v) {
  double s = 0;
  for (double x : v) s += x * x;
  return std::sqrt(s);
}

// ------------------------------------------------------------------ TrustRegionMinimizer + Dogleg
struct Minimizer {
  Program& P;
  const okvisgpu_options& o;
  int nthreads;
  bool redoAlways;
  // state
  std::vector<double> x, cand, jscale, gradient;  // gradient: J^T r (Ceres Evaluator gradient, local)
  Linearization lin;
  double x_cost = 0, cand_cost = 0, fixed = 0, x_norm = 0, minimum_cost = 0;
  double grad_max_norm = 0, grad_norm = 0;
  // dogleg
  double radius, mu = 1e-8, dogleg_step_norm = 0, alpha = 0, model_cost_change = 0;
  bool reuse = false;
  std::vector<double> diag, dgrad, gn, step, delta;

  Minimizer(Program& P_, const okvisgpu_options& o_)
      : P(P_), o(o_), nthreads(std::max(1, o_.num_threads)), redoAlways(o_.redo_propagation_always != 0) {
    radius = o.initial_trust_region_radius;
  }

  void evaluateGradientAndJacobian(int iteration) {
    x_cost = evaluateAll(P, x, &lin, nthreads, redoAlways);
    gradient.assign(P.nt, 0.0);
    leftMultiply(P, lin, lin.res.data(), gradient.data());  // unscaled J^T r
    if (o.jacobi_scaling) {
      if (iteration == 0) {
        squaredColumnNorm(P, lin, jscale);
        for (double& s : jscale) s = 1.0 / (1.0 + std::sqrt(s));
      }
      scaleColumns(P, lin, jscale);
    }
    // |x - Plus(x, -g)| (TrustRegionMinimizer::EvaluateGradientAndJacobian)
    std::vector<double> ng(P.nt), proj;
    for (int i = 0; i < P.nt; ++i) ng[i] = -gradient[i];
    plusAll(P, x, ng.data(), proj);
    grad_max_norm = 0;
    double s = 0;
    for (int i = 0; i < P.nx; ++i) {
      const double d = x[i] - proj[i];
      grad_max_norm = std::max(grad_max_norm, std::fabs(d));
      s += d * d;
    }
    grad_norm = std::sqrt(s);
  }

  // DoglegStrategy::ComputeGaussNewtonStep (single attempt per mu; failure handled by caller loop)
  // Returns 0 ok, 1 failure (mu exhausted).
  int computeGaussNewtonStep() {
    const int n = P.nt;
    while (mu < 1.0) {
      std::vector<double> D(n);
      for (int i = 0; i < n; ++i) D[i] = diag[i] * std::sqrt(mu);
      Reduced R;
      buildReduced(P, lin, D.data(), R, nthreads);
      bool ok = R.ok;
      std::vector<double> y(n, 0.0);
      if (ok) {
        std::vector<double> lhs = R.lhs;
        if (denseCholesky(P.fdim, lhs.data(), nthreads) != 0) ok = false;
        if (ok) {
          std::vector<double> yf = R.rhs;
          choleskySolve(P.fdim, lhs.data(), yf.data());
          backSubstitute(P, lin, R, yf.data(), y.data());
          for (double v : y) if (!std::isfinite(v)) ok = false;
        }
      }
      if (!ok) { mu *= 10.0; continue; }
      gn.assign(n, 0.0);
      for (int i = 0; i < n; ++i) gn[i] = -diag[i] * y[i];
      return 0;
    }
    return 1;
  }

  void computeTraditionalDoglegStep() {
    const int n = P.nt;
    step.assign(n, 0.0);
    double gnorm = 0, gnn = 0, gdotgn = 0;
    for (int i = 0; i < n; ++i) { gnorm += dgrad[i] * dgrad[i]; gnn += gn[i] * gn[i]; gdotgn += dgrad[i] * gn[i]; }
    gnorm = std::sqrt(gnorm);
    gnn = std::sqrt(gnn);
    if (gnn <= radius) {
      for (int i = 0; i < n; ++i) step[i] = gn[i] / diag[i];
      dogleg_step_norm = gnn;
      return;
    }
    if (gnorm * alpha >= radius) {
      for (int i = 0; i < n; ++i) step[i] = (-(radius / gnorm) * dgrad[i]) / diag[i];
      dogleg_step_norm = radius;
      return;
    }
    const double b_dot_a = -alpha * gdotgn;
    const double a_squared_norm = std::pow(alpha * gnorm, 2.0);
    const double b_minus_a_squared_norm = a_squared_norm - 2 * b_dot_a + std::pow(gnn, 2);
    const double c = b_dot_a - a_squared_norm;
    const double d = std::sqrt(c * c + b_minus_a_squared_norm * (std::pow(radius, 2.0) - a_squared_norm));
    const double beta = (c <= 0) ? (d - c) / b_minus_a_squared_norm : (radius * radius - a_squared_norm) / (d + c);
    double sn = 0;
    for (int i = 0; i < n; ++i) {
      const double v = (-alpha * (1.0 - beta)) * dgrad[i] + beta * gn[i];
      sn += v * v;
      step[i] = v / diag[i];
    }
    dogleg_step_norm = std::sqrt(sn);
  }

  // DoglegStrategy::ComputeStep; returns 0 ok, 1 linear solver failure
  int computeStep() {
    const int n = P.nt;
    if (reuse) {
      computeTraditionalDoglegStep();
      return 0;
    }
    reuse = true;
    squaredColumnNorm(P, lin, diag);
    for (double& d : diag) d = std::sqrt(std::min(std::max(d, o.min_lm_diagonal), o.max_lm_diagonal));
    // ComputeGradient: gradient_ = J^T r / diagonal
    dgrad.assign(n, 0.0);
    leftMultiply(P, lin, lin.res.data(), dgrad.data());
    for (int i = 0; i < n; ++i) dgrad[i] /= diag[i];
    // ComputeCauchyPoint: alpha = |g|^2 / |J (g / diag)|^2
    std::vector<double> sg(n), Jg(P.nres, 0.0);
    for (int i = 0; i < n; ++i) sg[i] = dgrad[i] / diag[i];
    rightMultiply(P, lin, sg.data(), Jg.data());
    double g2 = 0, jg2 = 0;
    for (double v : dgrad) g2 += v * v;
    for (double v : Jg) jg2 += v * v;
    alpha = g2 / jg2;
    if (computeGaussNewtonStep() != 0) return 1;
    computeTraditionalDoglegStep();
    return 0;
  }

  void stepAccepted(double q) {
    if (q < 0.25) radius *= 0.5;
    if (q > 0.75) radius = std::max(radius, 3.0 * dogleg_step_norm);
    radius = std::min(radius, o.max_trust_region_radius);
    mu = std::max(1e-8, 2.0 * mu / 10.0);
    reuse = false;
  }

  void run(okvisgpu_summary* S) {
    const double t_start = nowS();
    gatherX(P, x);
    fixed = fixedCost(P, nthreads, redoAlways);
    x_norm = vnorm(x);
    evaluateGradientAndJacobian(0);
    S->initial_cost = x_cost + fixed;
    if (P.hostFailures.load() != 0) {  // initial evaluation failed: the solve ends there
      S->final_cost = x_cost + fixed;
      S->num_iterations = 0;
      S->num_successful_steps = 1;
      S->num_unsuccessful_steps = 0;
      S->termination_type = OKVISGPU_FAILURE;
      S->total_time_s = nowS() - t_start;
      S->final_radius = radius;
      S->final_mu = mu;
      return;
    }
    minimum_cost = std::numeric_limits<double>::max();
    int iteration = 0, num_succ = 0, num_unsucc = 0, consecutive_invalid = 0;
    bool step_successful = true;
    int termination = OKVISGPU_NO_CONVERGENCE;
    double iter_start = t_start;
    std::vector<double> best = x;
    while (true) {
      // FinalizeIterationAndCheckIfMinimizerCanContinue
      if (step_successful) {
        ++num_succ;
        if (x_cost < minimum_cost) { minimum_cost = x_cost; best = x; }
      } else {
        ++num_unsucc;
      }
      const double now = nowS();
      const double iter_time = now - iter_start, cum_time = now - t_start;
      if (o.time_limit_s >= 0 && iteration >= o.min_iterations && cum_time + iter_time > o.time_limit_s) {
        termination = OKVISGPU_USER_SUCCESS;
        break;
      }
      if (iteration >= o.max_num_iterations) { termination = OKVISGPU_NO_CONVERGENCE; break; }
      if (grad_max_norm <= o.gradient_tolerance) { termination = OKVISGPU_CONVERGENCE; break; }
      if (radius <= o.min_trust_region_radius) { termination = OKVISGPU_CONVERGENCE; break; }
      // next iteration
      iter_start = nowS();
      ++iteration;
      step_successful = false;
      const int status = computeStep();
      bool valid = false;
      if (status == 0) {
        // model_cost_change = -(J step).(r + J step / 2)
        std::vector<double> mr(P.nres, 0.0);
        rightMultiply(P, lin, step.data(), mr.data());
        double mcc = 0;
        for (int i = 0; i < P.nres; ++i) mcc -= mr[i] * (lin.res[i] + mr[i] / 2.0);
        model_cost_change = mcc;
        valid = model_cost_change > 0.0;
        if (valid) {
          delta.assign(P.nt, 0.0);
          for (int i = 0; i < P.nt; ++i) delta[i] = step[i] * (o.jacobi_scaling ? jscale[i] : 1.0);
          consecutive_invalid = 0;
        }
      }
      if (!valid) {  // HandleInvalidStep: the next FinalizeIteration counts it as unsuccessful
        if (++consecutive_invalid >= o.max_num_consecutive_invalid_steps) {
          // Ceres returns before FinalizeIteration records this iteration: not counted
          // (TrustRegionMinimizer::Minimize, `if (!HandleInvalidStep()) return;`)
          termination = OKVISGPU_FAILURE;
          --iteration;
          break;
        }
        mu *= 10.0;  // StepIsInvalid
        reuse = false;
        continue;
      }
      // ComputeCandidatePointAndEvaluateCost
      plusAll(P, x, delta.data(), cand);
      cand_cost = evaluateAll(P, cand, nullptr, nthreads, redoAlways);
      // ParameterToleranceReached
      double sn = 0;
      for (int i = 0; i < P.nx; ++i) sn += (x[i] - cand[i]) * (x[i] - cand[i]);
      sn = std::sqrt(sn);
      // (Ceres returns before the iteration's summary is recorded: it is not counted)
      if (sn <= o.parameter_tolerance * (x_norm + o.parameter_tolerance)) { termination = OKVISGPU_CONVERGENCE; --iteration; break; }
      // FunctionToleranceReached
      const double cost_change = x_cost - cand_cost;
      if (std::fabs(cost_change) <= o.function_tolerance * x_cost) { termination = OKVISGPU_CONVERGENCE; --iteration; break; }
      // IsStepSuccessful
      const double rel = (cand_cost >= std::numeric_limits<double>::max())
                             ? std::numeric_limits<double>::lowest()
                             : (x_cost - cand_cost) / model_cost_change;
      if (rel > o.min_relative_decrease) {  // HandleSuccessfulStep
        x = cand;
        x_norm = vnorm(x);
        evaluateGradientAndJacobian(iteration);
        step_successful = true;
        stepAccepted(rel);
      } else {  // HandleUnsuccessfulStep
        radius *= 0.5;
        reuse = true;
      }
    }
    // final: best parameters
    if (minimum_cost < std::numeric_limits<double>::max()) x = best;
    scatterX(P, x);
    S->final_cost = std::min(minimum_cost, x_cost) + fixed;
    S->num_iterations = iteration;
    S->num_successful_steps = num_succ;
    S->num_unsuccessful_steps = num_unsucc;
    S->termination_type = termination;
    S->total_time_s = nowS() - t_start;
    S->final_radius = radius;
    S->final_mu = mu;
  }
};

void storeImuStates(const Program& P) {
  if (!P.p->imu_state) return;
  for (size_t f = 0; f < P.imus.size(); ++f)
    P.imus[f].storeState(&P.p->imu_state[f * OKVISGPU_IMU_STATE_DOUBLES]);
}

}  // namespace
}  // namespace oracle

using namespace oracle;

extern "C" {

int oracle_solve(const okvisgpu_problem* p, const okvisgpu_options* o, okvisgpu_summary* s) {
  if (!p || !o) return OKVISGPU_ERR_INVALID_ARGUMENT;
  Program P;
  buildProgram(p, P, true);
  Minimizer M(P, *o);
  okvisgpu_summary tmp;
  std::memset(&tmp, 0, sizeof(tmp));
  M.run(&tmp);
  storeImuStates(P);
  if (s) *s = tmp;
  return OKVISGPU_OK;
}

int oracle_evaluate(const okvisgpu_problem* p, double* cost) {
  Program P;
  buildProgram(p, P, true);
  std::vector<double> x;
  gatherX(P, x);
  const double c = evaluateAll(P, x, nullptr, 1, false) + fixedCost(P, 1, false);
  if (cost) *cost = c;
  return OKVISGPU_OK;
}

int oracle_linearize_reduce(const okvisgpu_problem* p, int32_t jacobi_scaling, double mu, double* S,
                            double* rhs, double* cost, int32_t* dim_out) {
  Program P;
  buildProgram(p, P, true);
  std::vector<double> x;
  gatherX(P, x);
  Linearization L;
  const double c = evaluateAll(P, x, &L, 1, false);
  if (jacobi_scaling) {
    std::vector<double> js;
    squaredColumnNorm(P, L, js);
    for (double& v : js) v = 1.0 / (1.0 + std::sqrt(v));
    scaleColumns(P, L, js);
  }
  std::vector<double> diag;
  squaredColumnNorm(P, L, diag);
  for (double& d : diag) d = std::sqrt(std::min(std::max(d, 1e-6), 1e32)) * std::sqrt(mu);
  Reduced R;
  buildReduced(P, L, mu > 0 ? diag.data() : nullptr, R, 1);
  if (dim_out) *dim_out = P.fdim;
  if (S) std::memcpy(S, R.lhs.data(), sizeof(double) * R.lhs.size());
  if (rhs) std::memcpy(rhs, R.rhs.data(), sizeof(double) * R.rhs.size());
  if (cost) *cost = c + fixedCost(P, 1, false);
  storeImuStates(P);
  return R.ok ? OKVISGPU_OK : OKVISGPU_ERR_NUMERICAL;
}

int oracle_eval_reprojection(const okvisgpu_problem* p, double* r, double* Jp, double* Jl) {
  std::vector<Camera> cams;
  for (int c = 0; c < p->n_cameras; ++c) {
    const okvisgpu_camera& k = p->cameras[c];
    cams.push_back(cameraOf(k));
  }
  for (int o = 0; o < p->n_observations; ++o) {
    const int cam = p->obs_camera[o];
    double rr[2], j0[12], j1[6];
    reprojectionEvaluate(cams[cam], &p->obs_keypoint[2 * o], &p->obs_sqrt_info[4 * o], &p->poses[7 * p->obs_pose[o]],
                         &p->landmarks[4 * p->obs_landmark[o]], &p->extrinsics[7 * cam], rr, nullptr, nullptr,
                         nullptr, j0, j1, nullptr);
    if (r) { r[2 * o] = rr[0]; r[2 * o + 1] = rr[1]; }
    if (Jp) for (int i = 0; i < 12; ++i) Jp[12 * o + i] = j0[i];
    if (Jl) for (int i = 0; i < 6; ++i) Jl[6 * o + i] = j1[i];
  }
  return OKVISGPU_OK;
}

int oracle_imu_merge(const okvisgpu_problem* p, int32_t f, const double* sb, double* state_out) {
  if (!p || f < 0 || f + 1 >= p->n_imu) return -2;
  Program P;
  buildProgram(p, P, true);
  ImuError& e = P.imus[f];
  if (e.redoCounter == 0) {  // first use integrates (ImuError.cpp:837)
    const int* b = &p->imu_blocks[4 * f];
    const double* prm[4] = {&p->poses[7 * b[0]], &p->speed_biases[9 * b[1]], &p->poses[7 * b[2]],
                            &p->speed_biases[9 * b[3]]};
    double rr[15];
    e.evaluate(prm, rr, nullptr, nullptr, false);
  }
  const int steps = e.append(sb, P.imus[f + 1].meas, p->imu_t1_ns[f + 1]);
  e.storeState(state_out);
  return steps;
}

// okvisgpu_imu_append semantics on the CPU (ImuError::append, ImuError.cpp:63-255, for a batch):
// every factor continues from its stored state (t1 = t1_old) over the given samples to t1_new with
// the eliminated state's speed/bias; -1 leaves the state untouched.
int oracle_imu_append(const okvisgpu_imu_append_batch* b, int32_t* steps) {
  if (!b || b->n < 0 || (b->n > 0 && (!b->state || !b->sample_begin || !b->speed_biases))) return -2;
  for (int f = 0; f < b->n; ++f) {
    oracle::ImuError e;
    e.params = b->imu_params;
    double* st = b->state + (size_t)f * OKVISGPU_IMU_STATE_DOUBLES;
    e.loadState(st);
    std::vector<oracle::ImuSample> m;
    for (int s = b->sample_begin[f]; s < b->sample_begin[f + 1]; ++s) {
      oracle::ImuSample x;
      x.t = b->sample_t_ns[s];
      for (int k = 0; k < 3; ++k) {
        x.g[k] = b->sample_gyr_acc[6 * s + k];
        x.a[k] = b->sample_gyr_acc[6 * s + 3 + k];
      }
      m.push_back(x);
    }
    int n = -1;
    if (!m.empty()) {
      e.meas.push_back(m.front());  // the link's own samples only feed the merged deque
      e.t1 = b->t1_old_ns[f];
      n = e.append(&b->speed_biases[9 * f], m, b->t1_new_ns[f]);
      if (n >= 0) e.storeState(st);
    }
    if (steps) steps[f] = n;
  }
  return OKVISGPU_OK;
}

int oracle_eval_imu(const okvisgpu_problem* p, int32_t redo_always, double* r, double* J) {
  Program P;
  buildProgram(p, P, true);
  for (int f = 0; f < p->n_imu; ++f) {
    const int* b = &p->imu_blocks[4 * f];
    const double* prm[4] = {&p->poses[7 * b[0]], &p->speed_biases[9 * b[1]], &p->poses[7 * b[2]],
                            &p->speed_biases[9 * b[3]]};
    double rr[15], j0[90], j1[135], j2[90], j3[135];
    double* jm[4] = {j0, j1, j2, j3};
    P.imus[f].evaluate(prm, rr, nullptr, jm, redo_always != 0);
    if (r) for (int i = 0; i < 15; ++i) r[15 * f + i] = rr[i];
    if (J)
      for (int i = 0; i < 15; ++i) {
        double* row = &J[(size_t)f * 450 + i * 30];
        for (int c = 0; c < 6; ++c) row[c] = j0[i * 6 + c];
        for (int c = 0; c < 9; ++c) row[6 + c] = j1[i * 9 + c];
        for (int c = 0; c < 6; ++c) row[15 + c] = j2[i * 6 + c];
        for (int c = 0; c < 9; ++c) row[21 + c] = j3[i * 9 + c];
      }
  }
  storeImuStates(P);
  return OKVISGPU_OK;
}

// jacobiansCorrect (ErrorInterface.cpp:44-163): central differences in the tangent space.
int oracle_check_jacobians(const okvisgpu_problem* p, int32_t kind, int32_t index, double delta,
                           double* max_rel) {
  Program P;
  buildProgram(p, P, true);
  std::vector<std::vector<double>> blocks;
  std::vector<int> kinds;
  Camera cam{};
  int nres = 0;
  if (kind == 0) {
    blocks.push_back(std::vector<double>(&p->poses[7 * p->obs_pose[index]], &p->poses[7 * p->obs_pose[index]] + 7));
    blocks.push_back(std::vector<double>(&p->landmarks[4 * p->obs_landmark[index]], &p->landmarks[4 * p->obs_landmark[index]] + 4));
    blocks.push_back(std::vector<double>(&p->extrinsics[7 * p->obs_camera[index]], &p->extrinsics[7 * p->obs_camera[index]] + 7));
    kinds = {kPose, kLm, kPose};
    cam = P.cams[p->obs_camera[index]];
    nres = 2;
  } else if (kind == 1) {
    const int* b = &p->imu_blocks[4 * index];
    blocks.push_back(std::vector<double>(&p->poses[7 * b[0]], &p->poses[7 * b[0]] + 7));
    blocks.push_back(std::vector<double>(&p->speed_biases[9 * b[1]], &p->speed_biases[9 * b[1]] + 9));
    blocks.push_back(std::vector<double>(&p->poses[7 * b[2]], &p->poses[7 * b[2]] + 7));
    blocks.push_back(std::vector<double>(&p->speed_biases[9 * b[3]], &p->speed_biases[9 * b[3]] + 9));
    kinds = {kPose, kSb, kPose, kSb};
    nres = 15;
  } else if (kind == 2) {
    blocks.push_back(std::vector<double>(&p->poses[7 * p->pose_prior_block[index]], &p->poses[7 * p->pose_prior_block[index]] + 7));
    kinds = {kPose};
    nres = 6;
  } else if (kind == 3) {
    blocks.push_back(std::vector<double>(&p->speed_biases[9 * p->sb_prior_block[index]], &p->speed_biases[9 * p->sb_prior_block[index]] + 9));
    kinds = {kSb};
    nres = 9;
  } else {
    const int* b = &p->relpose_blocks[2 * index];
    blocks.push_back(std::vector<double>(&p->poses[7 * b[0]], &p->poses[7 * b[0]] + 7));
    blocks.push_back(std::vector<double>(&p->poses[7 * b[1]], &p->poses[7 * b[1]] + 7));
    kinds = {kPose, kPose};
    nres = 6;
  }
  const int nb = (int)blocks.size();
  auto eval = [&](const std::vector<std::vector<double>>& bl, double* r, double** jmin) {
    const double* prm[4];
    for (int i = 0; i < nb; ++i) prm[i] = bl[i].data();
    if (kind == 0) {
      reprojectionEvaluate(cam, &p->obs_keypoint[2 * index], &p->obs_sqrt_info[4 * index], prm[0], prm[1], prm[2], r,
                           nullptr, nullptr, nullptr, jmin ? jmin[0] : nullptr, jmin ? jmin[1] : nullptr,
                           jmin ? jmin[2] : nullptr);
    } else if (kind == 1) {
      P.imus[index].evaluate(prm, r, nullptr, jmin, false);
    } else if (kind == 2) {
      poseErrorEvaluate(&p->pose_prior_meas[7 * index], &p->pose_prior_sqrt_info[36 * index], prm[0], r, nullptr,
                        jmin ? jmin[0] : nullptr);
    } else if (kind == 3) {
      sbErrorEvaluate(&p->sb_prior_meas[9 * index], &p->sb_prior_sqrt_info[81 * index], prm[0], r,
                      jmin ? jmin[0] : nullptr);
    } else {
      relPoseBlockEvaluate(p, index, prm[0], prm[1], r, jmin ? jmin[0] : nullptr, jmin ? jmin[1] : nullptr, nullptr,
                           nullptr);
    }
  };
  std::vector<std::vector<double>> Ja(nb);
  std::vector<double*> jp(nb);
  for (int i = 0; i < nb; ++i) {
    const int loc = kinds[i] == kPose ? 6 : kinds[i] == kLm ? 3 : 9;
    Ja[i].assign(nres * loc, 0.0);
    jp[i] = Ja[i].data();
  }
  double r0[15];
  eval(blocks, r0, jp.data());
  double worst = 0;
  for (int i = 0; i < nb; ++i) {
    const int loc = kinds[i] == kPose ? 6 : kinds[i] == kLm ? 3 : 9;
    std::vector<double> Jn(nres * loc);
    for (int j = 0; j < loc; ++j) {
      double dp[9] = {0}, dm[9] = {0};
      dp[j] = delta;
      dm[j] = -delta;
      auto bp = blocks, bm = blocks;
      if (kinds[i] == kPose) {
        posePlus(blocks[i].data(), dp, bp[i].data());
        posePlus(blocks[i].data(), dm, bm[i].data());
      } else if (kinds[i] == kLm) {
        pointPlus(blocks[i].data(), dp, bp[i].data());
        pointPlus(blocks[i].data(), dm, bm[i].data());
      } else {
        for (int k = 0; k < 9; ++k) { bp[i][k] += dp[k]; bm[i][k] += dm[k]; }
      }
      double rp[15], rm[15];
      eval(bp, rp, nullptr);
      eval(bm, rm, nullptr);
      for (int rr = 0; rr < nres; ++rr) Jn[rr * loc + j] = (rp[rr] - rm[rr]) / (2.0 * delta);
    }
    double dn = 0, na = 0, nn = 0;
    for (int k = 0; k < nres * loc; ++k) {
      dn += (Ja[i][k] - Jn[k]) * (Ja[i][k] - Jn[k]);
      na += Ja[i][k] * Ja[i][k];
      nn += Jn[k] * Jn[k];
    }
    const double den = std::sqrt(std::min(na, nn));
    const double rel = den > 0 ? std::sqrt(dn) / den : std::sqrt(dn);
    worst = std::max(worst, rel);
  }
  if (max_rel) *max_rel = worst;
  return OKVISGPU_OK;
}

int oracle_eval_relpose(const okvisgpu_problem* p, double* r, double* J) {
  for (int i = 0; i < p->n_relpose; ++i) {
    const int* b = &p->relpose_blocks[2 * i];
    double J0[36], J1[36], rr6[6];
    relPoseBlockEvaluate(p, i, &p->poses[7 * b[0]], &p->poses[7 * b[1]], rr6, J0, J1, nullptr, nullptr);
    if (r) for (int k = 0; k < 6; ++k) r[6 * i + k] = rr6[k];
    if (J)
      for (int rr = 0; rr < 6; ++rr)
        for (int c = 0; c < 6; ++c) {
          J[72 * i + rr * 12 + c] = J0[rr * 6 + c];
          J[72 * i + rr * 12 + 6 + c] = J1[rr * 6 + c];
        }
  }
  return OKVISGPU_OK;
}

// Host-evaluated factors at the problem's values, no loss: r [n][15], minimal J [n][15][30] in the
// IMU column layout (k-th pose-kind block of the functor at 0 / 15, k-th speed/bias at 6 / 21),
// the manifold applied as Ceres' ResidualBlock does (ambient J times the plus Jacobian).
int oracle_eval_host(const okvisgpu_problem* p, double* r, double* J) {
  for (int h = 0; h < p->n_host; ++h) {
    const double* prm[4] = {nullptr, nullptr, nullptr, nullptr};
    double amb[4][15 * 9] = {};
    double* ja[4] = {amb[0], amb[1], amb[2], amb[3]};
    int col[4] = {0, 0, 0, 0}, kind[4] = {0, 0, 0, 0}, nb = 0, npk = 0, nsb = 0;
    for (; nb < 4 && p->host_param_kind[4 * h + nb] >= 0; ++nb) {
      kind[nb] = p->host_param_kind[4 * h + nb];
      const int idx = p->host_param_index[4 * h + nb];
      if (kind[nb] == 0) {
        prm[nb] = idx < p->n_poses ? &p->poses[7 * idx] : &p->extrinsics[7 * (idx - p->n_poses)];
        col[nb] = npk++ == 0 ? 0 : 15;
      } else {
        prm[nb] = &p->speed_biases[9 * idx];
        col[nb] = nsb++ == 0 ? 6 : 21;
      }
    }
    double rr[15] = {};
    const int dim = p->host_dim[h];
    if (!p->host_evaluate(p->host_user, h, prm, rr, ja)) return OKVISGPU_ERR_NUMERICAL;
    if (r) for (int i = 0; i < 15; ++i) r[15 * h + i] = i < dim ? rr[i] : 0.0;
    if (!J) continue;
    double* Jh = J + 450 * (size_t)h;
    for (int i = 0; i < 450; ++i) Jh[i] = 0.0;
    for (int k = 0; k < nb; ++k) {
      if (kind[k] == 1) {
        for (int i = 0; i < dim; ++i)
          for (int c = 0; c < 9; ++c) Jh[i * 30 + col[k] + c] = amb[k][i * 9 + c];
        continue;
      }
      double Jp[42];
      posePlusJacobian(prm[k], Jp);
      for (int i = 0; i < dim; ++i)
        for (int c = 0; c < 6; ++c) {
          double s = 0;
          for (int a = 0; a < 7; ++a) s += amb[k][i * 7 + a] * Jp[a * 6 + c];
          Jh[i * 30 + col[k] + c] = s;
        }
    }
  }
  return OKVISGPU_OK;
}

int oracle_project(const okvisgpu_camera* k, const double* hp4, double* kp2, double* J24) {
  Camera cam = cameraOf(*k);
  V4 hp;
  for (int i = 0; i < 4; ++i) hp.a[i] = hp4[i];
  return cameraProjectHomogeneous(cam, hp, kp2, J24) ? 0 : 1;
}
void oracle_pose_plus(const double* x, const double* delta, double* out) { posePlus(x, delta, out); }
void oracle_pose_plus_jacobian(const double* x, double* J) { posePlusJacobian(x, J); }
void oracle_pose_minus_jacobian(const double* x, double* J) { poseMinusJacobian(x, J); }
int oracle_dense_cholesky(int32_t n, double* A, int32_t num_threads) { return denseCholesky(n, A, num_threads); }

int oracle_loss_evaluate(const okvisgpu_loss* loss, double s, double* rho) {
  if (!loss || !rho) return OKVISGPU_ERR_INVALID_ARGUMENT;
  lossEvaluate(*loss, s, rho);
  return OKVISGPU_OK;
}

int oracle_loss_correct(const okvisgpu_loss* loss, int32_t nres, int32_t ncols, double* r, double* J, double* cost) {
  if (!loss || !r || nres < 1 || nres > 15) return OKVISGPU_ERR_INVALID_ARGUMENT;
  double rr[15], sq = 0.0;
  for (int i = 0; i < nres; ++i) {
    rr[i] = r[i];
    sq += r[i] * r[i];
  }
  const double c = applyCorrector(*loss, nres, ncols, rr, sq, r, J);
  if (cost) *cost = c;
  return OKVISGPU_OK;
}

}  // extern "C"
