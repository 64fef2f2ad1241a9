// runtime.cpp — host runtime of the okvisgpu C ABI (include/okvisgpu.h).
//
// The drop-in replacement for `::ceres::Solve(options_, problem_.get(), &summary_)` in
// okvis::ViGraph::optimise (okvis_ceres/src/ViGraph.cpp:1844-1890): structure analysis of each
// window (residual blocks, constant flags, Schur ordering with landmarks as e-blocks, the
// reduced-system contribution lists), one HBM arena per context, upload, and the trust-region
// iteration as a captured hipGraph that is replayed max_num_iterations times with every decision
// taken on the device (kernels_control.hip). The host synchronises once per solve (plus once per
// iteration only when a CeresIterationCallback-style time limit is requested).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/okvisgpu.h"
#include "device_problem.hpp"
#include "launch.hpp"
#include "okvisgpu_math.hpp"

using namespace okg;

namespace {

struct HipError {
  std::string msg;
  int code;
};

#define HIPCHK(x)                                                                             \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess)                                                                     \
      throw HipError{std::string(#x) + ": " + hipGetErrorString(e_),                          \
                     e_ == hipErrorOutOfMemory ? OKVISGPU_ERR_OUT_OF_MEMORY : OKVISGPU_ERR_DEVICE}; \
  } while (0)

struct ArgError {
  std::string msg;
};
struct UnsupportedError {
  std::string msg;
};

double nowS() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Per-window host copies (parameter staging / write-back) split over host threads: contiguous
// window ranges, one thread per range. Small batches run on the calling thread. The thread count
// follows OMP_NUM_THREADS (the job's CPU share) and is capped at 16.
template <class F>
void forWindows(int n, F&& fn) {
  static const int cap = [] {
    const char* e = std::getenv("OMP_NUM_THREADS");
    int t = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 16));
  }();
  const int nt = std::min(cap, n / 64);
  if (nt <= 1) {
    for (int w = 0; w < n; ++w) fn(w);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t]() {
      for (int w = (int)((int64_t)n * t / nt); w < (int)((int64_t)n * (t + 1) / nt); ++w) fn(w);
    });
  for (auto& x : th) x.join();
}

// Host mirror of everything uploaded (built by analyse()).
struct HostBatch {
  int n_win = 0;
  std::vector<const okvisgpu_problem*> probs;
  // bases per window
  std::vector<int> pose_base, sb_base, lm_base, cam_base, obs_base, imu_base, pp_base, sbp_base, rp_base, sample_base;
  // parameters (initial copies)
  std::vector<double> pose, sb, lm, extr, cam;
  std::vector<int32_t> lm_perm;  // internal landmark k of window w is the caller's landmark lm_perm[lm_base[w] + k]
  // extrinsics: camera c of window w is pose-kind block cam_pose[cam_base[w] + c] (after the states)
  std::vector<int32_t> cam_pose;
  std::vector<uint8_t> win_ext_free;  // window has a variable extrinsics block (write-back)
  // extrinsic visits (landmark, variable camera): observation lists (global obs index), the group's
  // range, segment slots; pose-extrinsics cross blocks (state pose, variable camera) with their obs
  std::vector<int32_t> xvisit_pose, xvisit_lm, xvisit_obs_begin, xvisit_obs, xvisit_slot, lmg_xbegin;
  std::vector<int32_t> pe_pose, pe_ext, pe_obs_begin, pe_obs;
  std::vector<int32_t> pose_win, sb_win, lm_win, pose_f, sb_f;
  std::vector<uint8_t> lm_free, pose_active, sb_active;
  // obs (sorted) + permutation to the caller's order (within the window)
  std::vector<int32_t> obs_pose, obs_lm, obs_cam, obs_win, obs_orig;
  std::vector<uint8_t> obs_flags;
  std::vector<double> obs_kp, obs_L;
  std::vector<double> obs_Ls;  // isotropic batches: L = diag(s, s) per observation, s only (obs_iso)
  bool obs_iso = false;
  // visits
  std::vector<int32_t> lm_visit_begin, visit_pose, visit_obs_begin, visit_lm, lmg_begin;
  std::vector<int32_t> lmg_info;  // [n_lmg+1][kLmgInfo]: first landmark, first visit, window, first segment,
                                  // first partial block, first landmark-pair product
  // visit segments: per landmark group, the visits of one free pose (k_lm_visit pre-sums them)
  std::vector<int32_t> seg_gbegin, seg_pose, seg_range, visit_slot;
  // partial Schur blocks: per landmark group and pose pair, sum of Z_a Z_b^T over the group's landmarks
  std::vector<int32_t> part_gbegin, part_cbegin, part_contrib;
  // imu
  std::vector<int32_t> imu_blocks, imu_win, imu_sbegin;
  std::vector<uint8_t> imu_flags;
  std::vector<int64_t> imu_t0, imu_t1, imu_ts;
  std::vector<double> imu_ga, imu_par, imu_state;
  // host-evaluated factors (ABI 5): global factor index n_imu_total + h, after every IMU factor;
  // slot[k] = IMU-layout slot (0 pose0, 1 sb0, 2 pose1, 3 sb1) of the functor's k-th block
  struct HostFactor { int win, local, np, dim; int8_t slot[4]; okvisgpu_loss loss; };
  int n_imu_total = 0;
  std::vector<HostFactor> hf;
  std::vector<int32_t> host_blocks, host_win, win_host_range;
  std::vector<uint8_t> host_flags;
  // priors
  std::vector<int32_t> pp_block, pp_win, sbp_block, sbp_win;
  std::vector<double> pp_meas, pp_L, sbp_meas, sbp_L;
  // relative-pose edges
  std::vector<int32_t> rp_blocks, rp_win;
  std::vector<uint8_t> rp_flags, rp_kind;
  std::vector<double> rp_dx, rp_J, rp_lp;
  // reduced structure
  std::vector<int32_t> win_foff, win_fdim, win_fpad;
  std::vector<int64_t> win_soff, win_linvoff, win_fwdoff;
  std::vector<int32_t> win_lmg_range;
  std::vector<int32_t> win_pose_range, win_sb_range, win_lm_range, win_obs_range, win_imu_range, win_pp_range,
      win_sbp_range, win_rp_range;
  std::vector<int32_t> fb_win, fb_kind, fb_index, fb_off, fb_cbegin;
  // S offset of every f-block: fb_off, plus the window's gap rows after the left part of a
  // nested-dissection order (win_sgap: f offset of the gap, gap length; 0 0 without one); natural
  // index of every f entry (-1: gap row) and natural dimension per window
  std::vector<int32_t> win_sgap, f_nat, win_fnat, win_bsplit;
  std::vector<int64_t> win_defoff;
  int64_t defer_total = 0;
  bool any_split = false;
  bool nd = false;  // order the windows' states for the tile-parallel schedule (nested dissection)
  int lmg_visits = kLmGroupVisits, lmg_lms = kLmGroupMax;  // landmark-group bounds (k_lm_visit workgroups)
  std::vector<int32_t> chol_root_items;  // (w, d, first-root-of-window flag): tiles no update writes
  int n_chol_launches = 1;
  std::vector<Contrib> fb_contrib;
  std::vector<int32_t> pair_win, pair_fi, pair_fj, pair_cbegin, pair_runs;
  std::vector<int32_t> asm_pp_items, asm_sb_items, asm_ppl_items;
  std::vector<int32_t> chol_upd_items, chol_upd_begin, tile_items;
  int64_t n_panels = 0;  // structurally non-zero tiles below the diagonal (panel products)
  int64_t n_band_updates = 0;
  int64_t n_band_updates_diag = 0;  // of which symmetric updates of a diagonal tile (SYRK)
  std::vector<Contrib> pair_contrib;
  int64_t s_total = 0, linv_total = 0, fwd_total = 0;
  std::vector<std::vector<uint8_t>> tileNz;
  std::vector<uint8_t> tile_nz;
  std::vector<std::vector<int16_t>> tileFu;
  std::vector<int16_t> tile_fu;
  std::vector<int64_t> win_tnzoff;
  std::vector<int> tileT;
  int f_total = 0;
  int max_fpad = 0;
  int max_panels = 0;  // most non-zero tiles below a diagonal tile (panels of one Cholesky step)
};

template <class T>
void appendN(std::vector<T>& v, const T* src, size_t n) {
  if (n) v.insert(v.end(), src, src + n);
}

// ---- robust losses (okvisgpu.h "robust losses"): ::ceres::LossFunction::Evaluate of the Ceres
// loss family (ceres-solver >= 2.1 loss_function.cc, restated: CauchyLoss, TukeyLoss, HuberLoss,
// SoftLOneLoss, ArctanLoss, TolerantLoss), rho[0..2] = rho(s), rho'(s), rho''(s)
bool lossValid(const okvisgpu_loss& L) {
  switch (L.kind) {
    case OKVISGPU_LOSS_NONE: return true;
    case OKVISGPU_LOSS_TOLERANT: return L.a >= 0.0 && L.b > 0.0 && std::isfinite(L.a) && std::isfinite(L.b);
    case OKVISGPU_LOSS_CAUCHY: case OKVISGPU_LOSS_TUKEY: case OKVISGPU_LOSS_HUBER: case OKVISGPU_LOSS_SOFTLONE:
    case OKVISGPU_LOSS_ARCTAN: return L.a > 0.0 && std::isfinite(L.a);
  }
  return false;
}

void lossRho(const okvisgpu_loss& L, double s, double* rho) {
  const double a = L.a;
  switch (L.kind) {
    case OKVISGPU_LOSS_CAUCHY: {
      const double b = a * a, c = 1.0 / b;
      const double sum = 1.0 + s * c, inv = 1.0 / sum;
      rho[0] = b * std::log(sum);
      rho[1] = std::max(DBL_MIN, inv);
      rho[2] = -c * (inv * inv);
      return;
    }
    case OKVISGPU_LOSS_TUKEY: {
      const double a2 = a * a;
      if (s <= a2) {  // inlier region
        const double v = 1.0 - s / a2, v2 = v * v;
        rho[0] = a2 / 3.0 * (1.0 - v2 * v);
        rho[1] = v2;
        rho[2] = -2.0 / a2 * v;
      } else {  // outlier region: constant cost, no gradient
        rho[0] = a2 / 3.0;
        rho[1] = 0.0;
        rho[2] = 0.0;
      }
      return;
    }
    case OKVISGPU_LOSS_HUBER: {
      const double b = a * a;
      if (s > b) {
        const double r = std::sqrt(s);
        rho[0] = 2.0 * a * r - b;
        rho[1] = std::max(DBL_MIN, a / r);
        rho[2] = -rho[1] / (2.0 * s);
      } else {
        rho[0] = s;
        rho[1] = 1.0;
        rho[2] = 0.0;
      }
      return;
    }
    case OKVISGPU_LOSS_SOFTLONE: {
      const double b = a * a, c = 1.0 / b;
      const double sum = 1.0 + s * c, t = std::sqrt(sum);
      rho[0] = 2.0 * b * (t - 1.0);
      rho[1] = std::max(DBL_MIN, 1.0 / t);
      rho[2] = -(c * rho[1]) / (2.0 * sum);
      return;
    }
    case OKVISGPU_LOSS_ARCTAN: {
      const double b = 1.0 / (a * a);
      const double sum = 1.0 + s * s * b, inv = 1.0 / sum;
      rho[0] = a * std::atan2(s, a);
      rho[1] = std::max(DBL_MIN, inv);
      rho[2] = -2.0 * s * b * (inv * inv);
      return;
    }
    case OKVISGPU_LOSS_TOLERANT: {
      const double b = L.b, c = b * std::log(1.0 + std::exp(-a / b));
      const double x = (s - a) / b;
      if (x > 36.7) {  // 1 + e^x == e^x in double beyond ln(2^53)
        rho[0] = s - a - c;
        rho[1] = 1.0;
        rho[2] = 0.0;
      } else {
        const double ex = std::exp(x);
        rho[0] = b * std::log(1.0 + ex) - c;
        rho[1] = std::max(DBL_MIN, ex / (1.0 + ex));
        rho[2] = 0.5 / (b * (1.0 + std::cosh(x)));
      }
      return;
    }
    default:
      rho[0] = s;
      rho[1] = 1.0;
      rho[2] = 0.0;
  }
}

// the loss of host factor h: host_loss (ABI 6), else CauchyLoss(1) where host_cauchy is set
okvisgpu_loss hostLoss(const okvisgpu_problem* p, int h) {
  if (p->host_loss) return p->host_loss[h];
  okvisgpu_loss L{OKVISGPU_LOSS_NONE, 0, 1.0, 0.0};
  if (p->host_cauchy && p->host_cauchy[h]) L.kind = OKVISGPU_LOSS_CAUCHY;
  return L;
}

void validate(const okvisgpu_problem* p, int w) {
  auto bad = [&](const std::string& m) { throw ArgError{"window " + std::to_string(w) + ": " + m}; };
  if (p->n_poses < 0 || p->n_speed_biases < 0 || p->n_landmarks < 0 || p->n_observations < 0 || p->n_imu < 0 ||
      p->n_pose_priors < 0 || p->n_sb_priors < 0 || p->n_cameras < 0 || p->n_relpose < 0)
    bad("negative count");
  if (p->n_poses && !p->poses) bad("poses == NULL");
  if (p->n_speed_biases && !p->speed_biases) bad("speed_biases == NULL");
  if (p->n_landmarks && !p->landmarks) bad("landmarks == NULL");
  if (p->n_observations) {
    if (!p->obs_pose || !p->obs_landmark || !p->obs_camera || !p->obs_keypoint || !p->obs_sqrt_info)
      bad("observation arrays missing");
    if (!p->cameras || !p->extrinsics) bad("cameras / extrinsics missing");
    for (int o = 0; o < p->n_observations; ++o) {
      if (p->obs_pose[o] < 0 || p->obs_pose[o] >= p->n_poses) bad("obs_pose out of range");
      if (p->obs_landmark[o] < 0 || p->obs_landmark[o] >= p->n_landmarks) bad("obs_landmark out of range");
      if (p->obs_camera[o] < 0 || p->obs_camera[o] >= p->n_cameras) bad("obs_camera out of range");
    }
  }
  for (int c = 0; c < p->n_cameras; ++c)
    if (p->cameras[c].distortion < 0 || p->cameras[c].distortion > 3) bad("unknown distortion model");
  if (p->n_extrinsics_priors < 0) bad("negative count");
  if (p->n_extrinsics_priors && (!p->extrinsics_prior_camera || !p->extrinsics_prior_meas || !p->extrinsics_prior_sqrt_info))
    bad("extrinsics prior arrays missing");
  for (int i = 0; i < p->n_extrinsics_priors; ++i)
    if (p->extrinsics_prior_camera[i] < 0 || p->extrinsics_prior_camera[i] >= p->n_cameras)
      bad("extrinsics prior camera out of range");
  if (p->n_cameras && !p->extrinsics) bad("extrinsics == NULL");
  if (p->n_imu) {
    if (!p->imu_blocks || !p->imu_t0_ns || !p->imu_t1_ns || !p->imu_sample_begin || !p->imu_sample_t_ns ||
        !p->imu_sample_gyr_acc)
      bad("imu arrays missing");
    for (int f = 0; f < p->n_imu; ++f) {
      const int* b = &p->imu_blocks[4 * f];
      if (b[0] < 0 || b[0] >= p->n_poses || b[2] < 0 || b[2] >= p->n_poses || b[1] < 0 ||
          b[1] >= p->n_speed_biases || b[3] < 0 || b[3] >= p->n_speed_biases)
        bad("imu block index out of range");
      if (p->imu_sample_begin[f + 1] < p->imu_sample_begin[f]) bad("imu_sample_begin not monotone");
    }
  }
  for (int i = 0; i < p->n_pose_priors; ++i)
    if (p->pose_prior_block[i] < 0 || p->pose_prior_block[i] >= p->n_poses) bad("pose prior block out of range");
  for (int i = 0; i < p->n_sb_priors; ++i)
    if (p->sb_prior_block[i] < 0 || p->sb_prior_block[i] >= p->n_speed_biases) bad("sb prior block out of range");
  if (p->n_relpose) {
    if (!p->relpose_blocks || !p->relpose_delta_x || !p->relpose_sqrt_info || !p->relpose_lin_point)
      bad("relative-pose arrays missing");
    for (int i = 0; i < p->n_relpose; ++i) {
      const int a = p->relpose_blocks[2 * i], b = p->relpose_blocks[2 * i + 1];
      if (a < 0 || a >= p->n_poses || b < 0 || b >= p->n_poses) bad("relative-pose block out of range");
      if (a == b) bad("relative-pose edge connects a pose to itself");
      if (p->relpose_kind && p->relpose_kind[i] > 1) bad("unknown relative-pose kind");
    }
  }
  if (p->n_host < 0) bad("negative count");
  if (p->n_host) {
    if (!p->host_dim || !p->host_param_kind || !p->host_param_index || !p->host_evaluate)
      bad("host factor arrays / host_evaluate missing");
    for (int h = 0; h < p->n_host; ++h) {
      const std::string f = "host factor " + std::to_string(h) + ": ";
      if (p->host_dim[h] < 1 || p->host_dim[h] > OKVISGPU_HOST_MAX_RESIDUALS) bad(f + "residual dimension out of range");
      int np = 0, ns = 0, nb = 0;
      for (int k = 0; k < 4; ++k) {
        const int kind = p->host_param_kind[4 * h + k], idx = p->host_param_index[4 * h + k];
        if (kind < 0) break;
        ++nb;
        if (kind == 0) {
          if (idx < 0 || idx >= p->n_poses + p->n_cameras) bad(f + "pose-kind block out of range");
          ++np;
        } else if (kind == 1) {
          if (idx < 0 || idx >= p->n_speed_biases) bad(f + "speed/bias block out of range");
          ++ns;
        } else {
          throw UnsupportedError{"window " + std::to_string(w) + ": " + f +
                                 "only pose-kind and speed/bias blocks can be host-evaluated"};
        }
        for (int j = 0; j < k; ++j)
          if (p->host_param_kind[4 * h + j] == kind && p->host_param_index[4 * h + j] == idx)
            bad(f + "parameter block repeated");
        if (p->host_loss && !lossValid(p->host_loss[h])) bad(f + "unknown loss kind or non-positive loss scale");
      }
      for (int k = nb; k < 4; ++k)
        if (p->host_param_kind[4 * h + k] >= 0) bad(f + "parameter blocks must be leading (kind -1 = none)");
      if (nb == 0) bad(f + "no parameter block");
      if (np > 2 || ns > 2)
        throw UnsupportedError{"window " + std::to_string(w) + ": " + f +
                               "more than 2 pose-kind or 2 speed/bias blocks"};
    }
  }
}

// Development: host-time split of analyse() (build with -DOKG_ANALYSE_TIMING; printed per build).
#ifdef OKG_ANALYSE_TIMING
double g_atime[16];
std::chrono::steady_clock::time_point g_alast;
#define ATIME(i)                                                                                    \
  {                                                                                                 \
    const auto now = std::chrono::steady_clock::now();                                             \
    g_atime[i] += std::chrono::duration<double, std::milli>(now - g_alast).count();                 \
    g_alast = now;                                                                                  \
  }
#else
#define ATIME(i)
#endif

// Build the batch. `constOverride` carries okvisgpu_set_block_constant() edits.
// ---- tile-level symbolic factorisation and the tile-parallel launch schedule -------------------
// Fill of LLT inside the envelope, on the tile pattern nz (T x T, lower triangle).
void symbolicFill(std::vector<uint8_t>& nz, int T) {
  for (int k = 0; k < T; ++k)
    for (int i = k + 1; i < T; ++i)
      if (nz[(size_t)i * T + k])
        for (int j = k + 1; j <= i; ++j)
          if (nz[(size_t)j * T + k]) nz[(size_t)i * T + j] = 1;
}
// Launch schedule of the tile-parallel factorisation for a window's (filled) tile pattern: step k's
// band updates (tiles (i, j), k < j <= i, L_ik and L_jk non-zero) run in launch L[k] >= 1; launch 0
// factors the root tiles (those no update writes); any other tile is factored by the workgroup of
// its last update, so step k starts one launch after that; no tile is written by two updates of
// one launch. last[] holds each tile's last update launch (-1: none). For a block-banded pattern
// this is launch k + 1 for step k (the pre-round-4 schedule); for a nested-dissection order the
// independent parts share launches. Returns the number of launches.
int cholSchedule(const std::vector<uint8_t>& nz, int T, std::vector<int>& L, std::vector<int>& last) {
  L.assign(T, 0);
  last.assign((size_t)T * T, -1);
  int n = 1;
  for (int k = 0; k < T; ++k) {
    int lk = std::max(1, last[(size_t)k * T + k] + 1);
    bool any = false;
    for (int i = k + 1; i < T; ++i)
      if (nz[(size_t)i * T + k])
        for (int j = k + 1; j <= i; ++j)
          if (nz[(size_t)j * T + k]) {
            lk = std::max(lk, last[(size_t)i * T + j] + 1);
            any = true;
          }
    L[k] = lk;
    if (!any) continue;
    for (int i = k + 1; i < T; ++i)
      if (nz[(size_t)i * T + k])
        for (int j = k + 1; j <= i; ++j)
          if (nz[(size_t)j * T + k]) last[(size_t)i * T + j] = lk;
    n = std::max(n, lk + 1);
  }
  return n;
}
inline int pad64(int x) { return (x + kTile - 1) / kTile * kTile; }
// One level of nested dissection of a window's state slots (few windows: the latency of a solve is
// the chain of the tile-parallel launches). Slots [0, a) (left) and [b, n) (right) share no factor
// once the separator [a, b) is eliminated last: order left | right reversed | separator, left padded
// to a tile boundary in S, so the two parts factor as independent chains that each reach the
// separator only at their ends (the right part in natural order would touch it from its first
// tile on, and every step would write the separator's tiles). dim[u] = f scalars of slot u,
// reach[u] = largest slot coupled to u (landmarks seen from both, IMU links, edges, host factors).
// The split is chosen on the launch count of the estimated tile pattern (interval couplings);
// returns {-1, -1} unless it saves two launches or more with at most one tile more.
std::pair<int, int> chooseNd(const std::vector<int>& dim, const std::vector<int>& reach) {
  const int n = (int)dim.size();
  auto estimate = [&](int a, int b, int& tiles) {
    std::vector<int> order;  // (a = 0: the natural order)
    for (int u = 0; u < (a > 0 ? a : n); ++u) order.push_back(u);
    if (a > 0) {
      for (int u = n - 1; u >= b; --u) order.push_back(u);
      for (int u = a; u < b; ++u) order.push_back(u);
    }
    std::vector<int> off(n, 0);
    int o = 0;
    for (int t = 0; t < n; ++t) {
      if (t == a && a > 0 && a < n) o = pad64(o);
      off[order[t]] = o;
      o += dim[order[t]];
    }
    const int T = std::max(1, pad64(o) / kTile);
    tiles = T;
    std::vector<uint8_t> nz((size_t)T * T, 0);
    for (int i = 0; i < T; ++i) nz[(size_t)i * T + i] = 1;
    for (int u = 0; u < n; ++u) {
      if (!dim[u]) continue;
      for (int v = u; v <= reach[u]; ++v) {
        if (!dim[v]) continue;
        for (int ti = off[u] / kTile; ti <= (off[u] + dim[u] - 1) / kTile; ++ti)
          for (int tj = off[v] / kTile; tj <= (off[v] + dim[v] - 1) / kTile; ++tj)
            nz[(size_t)std::max(ti, tj) * T + std::min(ti, tj)] = 1;
      }
    }
    symbolicFill(nz, T);
    std::vector<int> L, last;
    return cholSchedule(nz, T, L, last);
  };
  int t0 = 0;
  const int base = estimate(0, 0, t0);
  std::vector<int> pm(n + 1, -1);
  for (int u = 0; u < n; ++u) pm[u + 1] = std::max(pm[u], reach[u]);
  int best = base, ba = -1, bb = -1;
  const int stride = n > 64 ? n / 32 : 1;
  for (int a = std::max(1, n > 64 ? n / 4 : 1); a < (n > 64 ? 3 * n / 4 : n - 1); a += stride) {
    const int b = std::max(a, pm[a] + 1);
    if (b >= n) continue;
    int t = 0;
    const int lv = estimate(a, b, t);
    if (t <= t0 + 1 && lv < best) {
      best = lv;
      ba = a;
      bb = b;
    }
  }
  return best <= base - 2 ? std::make_pair(ba, bb) : std::make_pair(-1, -1);
}

void analyse(const std::vector<const okvisgpu_problem*>& probs,
             const std::map<std::tuple<int, int, int>, int>& constOverride, HostBatch& B) {
  B.seg_gbegin.push_back(0);
  B.part_gbegin.push_back(0);
  B.n_win = (int)probs.size();
  B.probs = probs;
  {  // capacity for the per-observation / per-landmark arrays of the whole batch (no regrowth)
    size_t no = 0, nl = 0;
    for (const okvisgpu_problem* p : probs) {
      no += (size_t)std::max(0, p->n_observations);
      nl += (size_t)std::max(0, p->n_landmarks);
    }
    for (auto* v : {&B.obs_pose, &B.obs_lm, &B.obs_cam, &B.obs_win, &B.obs_orig, &B.visit_pose, &B.visit_lm,
                    &B.visit_obs_begin})
      v->reserve(no + 1);
    B.obs_flags.reserve(no);
    B.obs_kp.reserve(2 * no);
    B.obs_L.reserve(4 * no);
    B.lm.reserve(4 * nl);
    B.lm_perm.reserve(nl);
    B.lm_visit_begin.reserve(nl + 1);
    B.lm_win.reserve(nl);
    B.lm_free.reserve(nl);
  }
  B.n_imu_total = 0;  // host factors are numbered after every IMU factor of the batch
  for (const okvisgpu_problem* p : probs) B.n_imu_total += std::max(0, p->n_imu);
  for (int w = 0; w < B.n_win; ++w) {
    ATIME(0)
    const okvisgpu_problem* p = probs[w];
    validate(p, w);
    const int pb = (int)B.pose_win.size(), sbb = (int)B.sb_win.size(), lb = (int)B.lm_win.size();
    const int cb = (int)(B.cam.size() / kCamDoubles), ob = (int)B.obs_win.size(), ib = (int)B.imu_win.size();
    const int ppb = (int)B.pp_win.size(), sbpb = (int)B.sbp_win.size(), rpb = (int)B.rp_win.size();
    B.pose_base.push_back(pb); B.sb_base.push_back(sbb); B.lm_base.push_back(lb); B.cam_base.push_back(cb);
    B.obs_base.push_back(ob); B.imu_base.push_back(ib); B.pp_base.push_back(ppb); B.sbp_base.push_back(sbpb);
    B.rp_base.push_back(rpb);
    auto isConst = [&](int kind, int idx, const uint8_t* flags) {
      auto it = constOverride.find(std::make_tuple(w, kind, idx));
      if (it != constOverride.end()) return it->second != 0;
      return flags ? flags[idx] != 0 : false;
    };
    // pose-kind blocks of the window: the states' poses [0, np), then one extrinsics block per
    // camera [np, np + ncam) (okvis: PoseParameterBlocks with the PoseManifold, ViGraph.cpp:330-336)
    const int np = p->n_poses, ncam = p->n_cameras, npx = np + ncam;
    std::vector<uint8_t> pc(npx), sc(p->n_speed_biases), lc(p->n_landmarks);
    for (int i = 0; i < np; ++i) pc[i] = isConst(0, i, p->pose_constant);
    for (int c = 0; c < ncam; ++c) {  // constant unless flagged variable (do_extrinsics: false)
      auto it = constOverride.find(std::make_tuple(w, 3, c));
      pc[np + c] = it != constOverride.end() ? it->second != 0
                                             : (p->extrinsics_constant ? p->extrinsics_constant[c] != 0 : 1);
    }
    for (int i = 0; i < p->n_speed_biases; ++i) sc[i] = isConst(1, i, p->speed_bias_constant);
    for (int i = 0; i < p->n_landmarks; ++i) lc[i] = isConst(2, i, p->landmark_constant);
    // parameters
    appendN(B.pose, p->poses, (size_t)7 * p->n_poses);
    appendN(B.pose, p->extrinsics, (size_t)7 * ncam);
    appendN(B.sb, p->speed_biases, (size_t)9 * p->n_speed_biases);
    // internal landmark order: by first observing pose (then caller order), so that the visits of
    // neighbouring keyframes are close in memory whatever order the caller numbers landmarks in
    // (okvis numbers them by creation, which is nearly this order already)
    std::vector<int> perm(p->n_landmarks), inv(p->n_landmarks);
    {
      std::vector<int> firstPose(p->n_landmarks, p->n_poses);
      for (int o = 0; o < p->n_observations; ++o)
        firstPose[p->obs_landmark[o]] = std::min(firstPose[p->obs_landmark[o]], p->obs_pose[o]);
      std::iota(perm.begin(), perm.end(), 0);
      std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return firstPose[a] < firstPose[b]; });
      for (int k = 0; k < p->n_landmarks; ++k) inv[perm[k]] = k;
    }
    for (int k = 0; k < p->n_landmarks; ++k) {
      appendN(B.lm, &p->landmarks[4 * (size_t)perm[k]], 4);
      B.lm_perm.push_back(perm[k]);
    }
    for (int c = 0; c < p->n_cameras; ++c) {
      const okvisgpu_camera& k = p->cameras[c];
      const double cv[kCamDoubles] = {(double)k.distortion, k.fu, k.fv, k.cu, k.cv, k.dist[0], k.dist[1],
                                      k.dist[2], k.dist[3], k.dist[4], k.dist[5], k.dist[6], k.dist[7]};
      appendN(B.cam, cv, kCamDoubles);
      appendN(B.extr, &p->extrinsics[7 * c], 7);
      B.cam_pose.push_back(pb + np + c);
    }
    for (int i = 0; i < npx; ++i) B.pose_win.push_back(w);
    for (int i = 0; i < p->n_speed_biases; ++i) B.sb_win.push_back(w);
    for (int i = 0; i < p->n_landmarks; ++i) B.lm_win.push_back(w);
    ATIME(1)
    // active blocks: free and used by a residual block that is not entirely constant
    std::vector<uint8_t> pa(npx, 0), sa(p->n_speed_biases, 0), la(p->n_landmarks, 0);
    std::vector<uint8_t> ofix(p->n_observations), ifix(p->n_imu);
    for (int o = 0; o < p->n_observations; ++o) {
      const int ps = p->obs_pose[o], l = p->obs_landmark[o], xe = np + p->obs_camera[o];
      ofix[o] = pc[ps] && lc[l] && pc[xe];
      if (!pc[ps]) pa[ps] = 1;
      if (!lc[l]) la[l] = 1;
      if (!pc[xe]) pa[xe] = 1;
    }
    for (int f = 0; f < p->n_imu; ++f) {
      const int* b = &p->imu_blocks[4 * f];
      ifix[f] = pc[b[0]] && sc[b[1]] && pc[b[2]] && sc[b[3]];
      if (!pc[b[0]]) pa[b[0]] = 1;
      if (!sc[b[1]]) sa[b[1]] = 1;
      if (!pc[b[2]]) pa[b[2]] = 1;
      if (!sc[b[3]]) sa[b[3]] = 1;
    }
    // PoseError priors on pose-kind blocks: the states' (pose_prior_*) then the extrinsics'
    // (extrinsics_prior_*, ViGraph.cpp:372-382), one prior list on the device
    struct PPrior { int blk; const double* meas; const double* L; };
    std::vector<PPrior> pps;
    for (int i = 0; i < p->n_pose_priors; ++i)
      pps.push_back(PPrior{p->pose_prior_block[i], &p->pose_prior_meas[7 * i], &p->pose_prior_sqrt_info[36 * i]});
    for (int i = 0; i < p->n_extrinsics_priors; ++i)
      pps.push_back(PPrior{np + p->extrinsics_prior_camera[i], &p->extrinsics_prior_meas[7 * i],
                           &p->extrinsics_prior_sqrt_info[36 * i]});
    for (const PPrior& q : pps)
      if (!pc[q.blk]) pa[q.blk] = 1;
    for (int i = 0; i < p->n_sb_priors; ++i)
      if (!sc[p->sb_prior_block[i]]) sa[p->sb_prior_block[i]] = 1;
    std::vector<uint8_t> rfix(p->n_relpose);
    for (int i = 0; i < p->n_relpose; ++i) {
      const int a = p->relpose_blocks[2 * i], b = p->relpose_blocks[2 * i + 1];
      rfix[i] = pc[a] && pc[b];
      if (!pc[a]) pa[a] = 1;
      if (!pc[b]) pa[b] = 1;
    }
    // host-evaluated factors: IMU-layout slots (pose-kind blocks fill slots 0 then 2, speed/bias
    // blocks 1 then 3, in the functor's order) and window-local block per slot (-1 unused)
    const int hfBase = (int)B.hf.size();
    std::vector<std::array<int, 4>> hslot(p->n_host);
    std::vector<uint8_t> hfix(p->n_host);
    for (int h = 0; h < p->n_host; ++h) {
      HostBatch::HostFactor F{w, h, 0, p->host_dim[h], {-1, -1, -1, -1}, hostLoss(p, h)};
      std::array<int, 4>& s = hslot[h];
      s = {-1, -1, -1, -1};
      int npk = 0, nsb = 0;
      bool allConst = true;
      for (int k = 0; k < 4 && p->host_param_kind[4 * h + k] >= 0; ++k) {
        const int kind = p->host_param_kind[4 * h + k], idx = p->host_param_index[4 * h + k];
        const int q = kind == 0 ? 2 * npk++ : 1 + 2 * nsb++;
        F.slot[k] = (int8_t)q;
        F.np = k + 1;
        s[q] = idx;
        const bool c = kind == 0 ? pc[idx] != 0 : sc[idx] != 0;
        allConst = allConst && c;
        if (!c) (kind == 0 ? pa[idx] : sa[idx]) = 1;
      }
      hfix[h] = allConst;
      B.hf.push_back(F);
    }
    // f-blocks in the reduced ordering: pose i, then speed/bias i, state slot by slot; for the
    // tile-parallel schedule (few windows) possibly in a nested-dissection order of the slots
    std::vector<int> posef(npx, -1), sbf(p->n_speed_biases, -1), poseFb(npx, -1), sbFb(p->n_speed_biases, -1);
    int fo = 0;
    const int nmax = std::max(p->n_poses, p->n_speed_biases);
    const int fbBase = (int)B.fb_win.size();
    std::vector<int> slotOrder(nmax);
    std::iota(slotOrder.begin(), slotOrder.end(), 0);
    int ndLeft = 0, ndSep = 0;  // slots of the left part (0: natural order); order index of the separator
    const bool extFree = std::any_of(pa.begin() + np, pa.end(), [](uint8_t a) { return a != 0; });
    if (B.nd && !extFree && nmax >= 8) {  // (variable extrinsics couple every state: no split)
      std::vector<int> dim(nmax, 0), reach(nmax);
      for (int i = 0; i < nmax; ++i) {
        dim[i] = (i < p->n_poses && pa[i] ? 6 : 0) + (i < p->n_speed_biases && sa[i] ? 9 : 0);
        reach[i] = i;
      }
      auto couple = [&](int lo, int hi) {
        if (lo >= 0 && hi > lo) reach[lo] = std::max(reach[lo], hi);
      };
      {  // landmarks: the free poses observing a free landmark are coupled by its elimination
        std::vector<int> lo(p->n_landmarks, INT_MAX), hi(p->n_landmarks, -1);
        for (int o = 0; o < p->n_observations; ++o) {
          const int l = p->obs_landmark[o], ps = p->obs_pose[o];
          if (!la[l] || !pa[ps]) continue;
          lo[l] = std::min(lo[l], ps);
          hi[l] = std::max(hi[l], ps);
        }
        for (int l = 0; l < p->n_landmarks; ++l)
          if (hi[l] >= 0) couple(lo[l], hi[l]);
      }
      auto coupleSet = [&](std::initializer_list<int> slots) {
        int lo = INT_MAX, hi = -1;
        for (int u : slots)
          if (u >= 0) { lo = std::min(lo, u); hi = std::max(hi, u); }
        if (hi >= 0) couple(lo, hi);
      };
      for (int f = 0; f < p->n_imu; ++f) {
        const int* b = &p->imu_blocks[4 * f];
        coupleSet({pa[b[0]] ? b[0] : -1, sa[b[1]] ? b[1] : -1, pa[b[2]] ? b[2] : -1, sa[b[3]] ? b[3] : -1});
      }
      for (int i = 0; i < p->n_relpose; ++i) {
        const int a = p->relpose_blocks[2 * i], b = p->relpose_blocks[2 * i + 1];
        coupleSet({a < np && pa[a] ? a : -1, b < np && pa[b] ? b : -1});
      }
      for (int h = 0; h < p->n_host; ++h) {
        int lo = INT_MAX, hi = -1;
        for (int k = 0; k < 4 && p->host_param_kind[4 * h + k] >= 0; ++k) {
          const int kind = p->host_param_kind[4 * h + k], idx = p->host_param_index[4 * h + k];
          const bool act = kind == 0 ? (idx < np && pa[idx]) : sa[idx] != 0;
          if (act) { lo = std::min(lo, idx); hi = std::max(hi, idx); }
        }
        if (hi >= 0) couple(lo, hi);
      }
      const auto ab = chooseNd(dim, reach);
      if (ab.first > 0) {
        slotOrder.clear();
        for (int u = 0; u < ab.first; ++u) slotOrder.push_back(u);
        for (int u = nmax - 1; u >= ab.second; --u) slotOrder.push_back(u);
        for (int u = ab.first; u < ab.second; ++u) slotOrder.push_back(u);
        ndLeft = ab.first;
        ndSep = ab.first + (nmax - ab.second);
      }
    }
    // (nested dissection: the left part ends on a tile boundary; the gap rows between are identity
    // rows of S with zero rhs, so the f-vector and S share one index)
    int gapAt = 0, gap = 0, rightAt = 0, sepAt = 0;
    for (int t = 0; t < nmax; ++t) {
      const int i = slotOrder[t];
      if (ndLeft && t == ndLeft) {
        gapAt = fo;
        fo = pad64(fo);
        gap = fo - gapAt;
        rightAt = fo;
      }
      if (ndLeft && t == ndSep) sepAt = fo;
      if (i < p->n_poses && pa[i]) {
        posef[i] = fo;
        poseFb[i] = (int)B.fb_win.size();
        B.fb_win.push_back(w); B.fb_kind.push_back(0); B.fb_index.push_back(pb + i); B.fb_off.push_back(fo);
        fo += 6;
      }
      if (i < p->n_speed_biases && sa[i]) {
        sbf[i] = fo;
        sbFb[i] = (int)B.fb_win.size();
        B.fb_win.push_back(w); B.fb_kind.push_back(1); B.fb_index.push_back(sbb + i); B.fb_off.push_back(fo);
        fo += 9;
      }
    }
    // variable extrinsics after all states: S keeps the states' band plus a dense border
    for (int c = 0; c < ncam; ++c) {
      const int i = np + c;
      if (!pa[i]) continue;
      posef[i] = fo;
      poseFb[i] = (int)B.fb_win.size();
      B.fb_win.push_back(w); B.fb_kind.push_back(0); B.fb_index.push_back(pb + i); B.fb_off.push_back(fo);
      fo += 6;
    }
    B.win_ext_free.push_back(fo > 0 && extFree);
    B.win_sgap.push_back(gap ? gapAt : 0);
    B.win_sgap.push_back(gap);
    // natural order of the f entries (pose i, speed/bias i slot by slot, then extrinsics: the order
    // of okvisgpu_linearize_reduce's export and of the oracle)
    {
      std::vector<int32_t> nat(fo, -1);
      int no = 0;
      auto put = [&](int f, int n) {
        for (int c = 0; c < n; ++c) nat[f + c] = no++;
      };
      for (int i = 0; i < nmax; ++i) {
        if (i < p->n_poses && posef[i] >= 0) put(posef[i], 6);
        if (i < p->n_speed_biases && sbf[i] >= 0) put(sbf[i], 9);
      }
      for (int c = 0; c < ncam; ++c)
        if (posef[np + c] >= 0) put(posef[np + c], 6);
      B.f_nat.insert(B.f_nat.end(), nat.begin(), nat.end());
      B.win_fnat.push_back(no);
    }
    for (int i = 0; i < npx; ++i) { B.pose_f.push_back(posef[i]); B.pose_active.push_back(pa[i]); }
    for (int i = 0; i < p->n_speed_biases; ++i) { B.sb_f.push_back(sbf[i]); B.sb_active.push_back(sa[i]); }
    std::vector<uint8_t> laNew(p->n_landmarks);
    for (int k = 0; k < p->n_landmarks; ++k) laNew[k] = la[perm[k]];
    for (int k = 0; k < p->n_landmarks; ++k) B.lm_free.push_back(laNew[k]);
    const int fpad = pad64(fo);  // S dimension (leading dimension of the window's S)
    B.win_foff.push_back(B.f_total);
    B.win_fdim.push_back(fo);
    B.win_fpad.push_back(fpad);
    B.win_soff.push_back(B.s_total);
    B.win_linvoff.push_back(B.linv_total);
    B.win_fwdoff.push_back(B.fwd_total);
    B.fwd_total += fpad;
    B.f_total += fo;
    B.s_total += (int64_t)fpad * fpad;
    B.linv_total += (int64_t)(fpad / kTile) * kTile * kTile;
    B.max_fpad = std::max(B.max_fpad, fpad);

    ATIME(2)
    // observations sorted by (internal landmark, pose, camera, original index)
    // (counting sort by landmark, then insertion sort of each landmark's few observations: the
    // order of a stable sort on that key, in linear time)
    std::vector<int> order(p->n_observations);
    {
      std::vector<int> start(p->n_landmarks + 1, 0);
      for (int o = 0; o < p->n_observations; ++o) ++start[inv[p->obs_landmark[o]] + 1];
      for (int l = 0; l < p->n_landmarks; ++l) start[l + 1] += start[l];
      std::vector<int> fill(start.begin(), start.end() - 1);
      for (int o = 0; o < p->n_observations; ++o) order[fill[inv[p->obs_landmark[o]]]++] = o;
      auto before = [&](int a, int b) {
        if (p->obs_pose[a] != p->obs_pose[b]) return p->obs_pose[a] < p->obs_pose[b];
        if (p->obs_camera[a] != p->obs_camera[b]) return p->obs_camera[a] < p->obs_camera[b];
        return a < b;
      };
      for (int l = 0; l < p->n_landmarks; ++l)
        for (int i = start[l] + 1; i < start[l + 1]; ++i) {
          const int x = order[i];
          int j = i - 1;
          for (; j >= start[l] && before(x, order[j]); --j) order[j + 1] = order[j];
          order[j + 1] = x;
        }
    }
    ATIME(3)
    // visits and landmark -> visit ranges
    const int vBase = (int)B.visit_pose.size();
    std::vector<int> lmVisitBegin(p->n_landmarks + 1, 0);
    std::vector<std::vector<int>> visitsAtPose(p->n_poses);
    {
      int prevL = -1, prevP = -1;
      std::vector<int> vcount(p->n_landmarks, 0);
      // per-observation arrays written in place (sized once; push_back per element dominated)
      const size_t nob = (size_t)p->n_observations;
      for (auto* v : {&B.obs_pose, &B.obs_lm, &B.obs_cam, &B.obs_win, &B.obs_orig}) v->resize(ob + nob);
      B.obs_flags.resize(ob + nob);
      B.obs_kp.resize(2 * (ob + nob));
      B.obs_L.resize(4 * (ob + nob));
      int32_t *oPose = B.obs_pose.data() + ob, *oLm = B.obs_lm.data() + ob, *oCam = B.obs_cam.data() + ob,
              *oWin = B.obs_win.data() + ob, *oOrig = B.obs_orig.data() + ob;
      uint8_t* oFl = B.obs_flags.data() + ob;
      double *oKp = B.obs_kp.data() + 2 * (size_t)ob, *oL = B.obs_L.data() + 4 * (size_t)ob;
      for (int k = 0; k < p->n_observations; ++k) {
        const int o = order[k];
        const int l = inv[p->obs_landmark[o]], ps = p->obs_pose[o], cam = p->obs_camera[o];
        oPose[k] = pb + ps;
        oLm[k] = lb + l;
        oCam[k] = cb + cam;
        oWin[k] = w;
        oOrig[k] = o;
        uint8_t fl = 0;
        if (p->obs_cauchy ? p->obs_cauchy[o] != 0 : true) fl |= 1;
        if (ofix[o]) fl |= 2;
        if (posef[np + cam] >= 0) fl |= 4;  // variable extrinsics
        oFl[k] = fl;
        oKp[2 * k] = p->obs_keypoint[2 * o];
        oKp[2 * k + 1] = p->obs_keypoint[2 * o + 1];
        for (int i = 0; i < 4; ++i) oL[4 * k + i] = p->obs_sqrt_info[4 * o + i];
        if (l != prevL || ps != prevP) {
          B.visit_pose.push_back(pb + ps);
          B.visit_lm.push_back(lb + l);
          B.visit_obs_begin.push_back(ob + k);
          visitsAtPose[ps].push_back((int)B.visit_pose.size() - 1);
          vcount[l]++;
          prevL = l;
          prevP = ps;
        }
      }
      int acc = vBase;
      for (int l = 0; l < p->n_landmarks; ++l) {
        lmVisitBegin[l] = acc;
        acc += vcount[l];
      }
      lmVisitBegin[p->n_landmarks] = acc;
      for (int l = 0; l < p->n_landmarks; ++l) B.lm_visit_begin.push_back(lmVisitBegin[l]);
    }
    ATIME(4)
    // extrinsic visits: per landmark and variable camera, the landmark's (non-fixed) observations
    // through that camera (the extrinsics block is the third parameter block of their
    // ReprojectionErrors); global indices, in landmark order like the visits
    std::vector<int> lmXBegin(p->n_landmarks + 1, (int)B.xvisit_pose.size());
    {
      std::vector<int> freeCams;
      for (int c = 0; c < ncam; ++c)
        if (posef[np + c] >= 0) freeCams.push_back(c);
      int k = 0;
      for (int l = 0; l < p->n_landmarks; ++l) {
        lmXBegin[l] = (int)B.xvisit_pose.size();
        const int k0 = k;
        while (k < p->n_observations && inv[p->obs_landmark[order[k]]] == l) ++k;
        for (int c : freeCams) {
          std::vector<int32_t> obs;
          for (int j = k0; j < k; ++j)
            if (p->obs_camera[order[j]] == c && !ofix[order[j]]) obs.push_back(ob + j);
          if (obs.empty()) continue;
          B.xvisit_pose.push_back(pb + np + c);
          B.xvisit_lm.push_back(lb + l);
          B.xvisit_obs_begin.push_back((int32_t)B.xvisit_obs.size());
          B.xvisit_obs.insert(B.xvisit_obs.end(), obs.begin(), obs.end());
          B.xvisit_slot.push_back(-1);
        }
      }
      lmXBegin[p->n_landmarks] = (int)B.xvisit_pose.size();
    }
    ATIME(5)
    // landmark groups of k_lm_visit (consecutive whole landmarks of this window, <= kLmGroupVisits
    // visits and <= kLmGroupMax landmarks; one workgroup, one thread per visit) and their visit
    // segments: the visits of a group that belong to one free pose, pre-summed by k_lm_visit into
    // one H | g and one U z record (ascending pose; members in visit order)
    std::vector<std::vector<int>> segsAtPose(npx);
    std::vector<std::pair<int, int>> partKeys;  // f-block pair of each partial block of this window
    const int partBase = (int)B.part_cbegin.size();
    {
      // each visit of a free pose gets the slot of its position in the group's (pose, visit)
      // order, so a segment is a contiguous slot range [seg_range.x, seg_range.y)
      // A group's threads: its pose visits first (thread t = v - gv0), then its extrinsic visits
      // (thread t = nvg + xv - gx0).
      std::vector<std::pair<int, int>> mem, gitems, gprod;  // scratch reused by every group
      std::vector<int> glocal, gcount, gfill, fbLocal(std::max(1, (int)B.fb_off.size()), -1);
      std::vector<int32_t> gsorted;
      auto closeGroup = [&](int gl0, int gl1) {
        const int gv0 = lmVisitBegin[gl0], gv1 = lmVisitBegin[gl1], nvg = gv1 - gv0;
        const int gx0 = lmXBegin[gl0], gx1 = lmXBegin[gl1];
        // members (v >= 0 visit, -1 - xv extrinsic visit) grouped by pose-kind block, ascending,
        // each block's members in visit order
        mem.clear();
        for (int v = gv0; v < gv1; ++v) {
          const int ps = B.visit_pose[v] - pb;
          if (posef[ps] >= 0) mem.push_back({ps, v});
          else B.visit_slot[v] = -1;
        }
        for (int xv = gx0; xv < gx1; ++xv) mem.push_back({B.xvisit_pose[xv] - pb, -1 - xv});
        std::stable_sort(mem.begin(), mem.end(),
                         [](const std::pair<int, int>& a, const std::pair<int, int>& b) { return a.first < b.first; });
        int slot = 0;
        for (size_t m = 0; m < mem.size();) {
          const int ps = mem[m].first;
          segsAtPose[ps].push_back((int)B.seg_pose.size());
          B.seg_pose.push_back(pb + ps);
          B.seg_range.push_back(slot);
          for (; m < mem.size() && mem[m].first == ps; ++m) {
            const int v = mem[m].second;
            if (v >= 0) B.visit_slot[v] = slot++;
            else B.xvisit_slot[-1 - v] = slot++;
          }
          B.seg_range.push_back(slot);
        }
        // partial Schur blocks (k_lm_visit): per f-block pair (row >= col by f offset) the products
        // Z_a Z_b^T of the group's free landmarks; contributions packed as (a | b << 16), thread
        // offsets within the group
        // products keyed by f-block pair, in (row f-block, col f-block) order, each key's products
        // in generation order: the group's f-blocks get dense local indices in ascending order and
        // the products are counting-sorted by (local row, local col)
        std::vector<std::pair<int, int>>& items = gitems;  // (thread, f-block) of one landmark's free visits
        glocal.clear();
        for (int v = gv0; v < gv1; ++v)
          if (laNew[B.visit_lm[v] - lb] && poseFb[B.visit_pose[v] - pb] >= 0) glocal.push_back(poseFb[B.visit_pose[v] - pb]);
        for (int xv = gx0; xv < gx1; ++xv)
          if (laNew[B.xvisit_lm[xv] - lb]) glocal.push_back(poseFb[B.xvisit_pose[xv] - pb]);
        std::sort(glocal.begin(), glocal.end());
        glocal.erase(std::unique(glocal.begin(), glocal.end()), glocal.end());
        const int nloc = (int)glocal.size();
        for (int i = 0; i < nloc; ++i) fbLocal[glocal[i]] = i;
        gprod.clear();
        for (int l = gl0; l < gl1; ++l) {
          if (!laNew[l]) continue;
          items.clear();
          for (int va = lmVisitBegin[l]; va < lmVisitBegin[l + 1]; ++va) {
            const int fa = poseFb[B.visit_pose[va] - pb];
            if (fa >= 0) items.push_back({va - gv0, fa});
          }
          for (int xv = lmXBegin[l]; xv < lmXBegin[l + 1]; ++xv)
            items.push_back({nvg + xv - gx0, poseFb[B.xvisit_pose[xv] - pb]});
          for (const auto& a : items)
            for (const auto& b : items) {
              if (B.fb_off[a.second] < B.fb_off[b.second]) continue;
              gprod.push_back({fbLocal[a.second] * nloc + fbLocal[b.second], a.first | (b.first << 16)});
            }
        }
        gcount.assign((size_t)nloc * nloc + 1, 0);
        for (const auto& x : gprod) ++gcount[x.first + 1];
        for (int k = 0; k < nloc * nloc; ++k) gcount[k + 1] += gcount[k];
        gsorted.resize(gprod.size());
        gfill.assign(gcount.begin(), gcount.end() - 1);
        for (const auto& x : gprod) gsorted[gfill[x.first]++] = x.second;
        // long blocks are split into chunks of <= kPartChunk products (separate records, summed
        // in order by k_assemble_pp) so that no k_lm_visit thread serialises a whole block
        constexpr int kPartChunk = 24;  // measured: 6 / 12 / 24 / unsplit on 2048 S50 windows
        for (int key = 0; key < nloc * nloc; ++key) {
          const int k0 = gcount[key], k1 = gcount[key + 1];
          for (int c0 = k0; c0 < k1; c0 += kPartChunk) {
            const int c1 = std::min(k1, c0 + kPartChunk);
            partKeys.push_back({glocal[key / nloc], glocal[key % nloc]});
            B.part_cbegin.push_back((int)B.part_contrib.size());
            B.part_contrib.insert(B.part_contrib.end(), gsorted.begin() + c0, gsorted.begin() + c1);
          }
        }
        B.lmg_begin.push_back(lb + gl0);
        B.lmg_xbegin.push_back(gx0);
        B.seg_gbegin.push_back((int)B.seg_pose.size());
        B.part_gbegin.push_back((int)B.part_cbegin.size());
      };
      // landmark-pair products a group stages in LDS (kLmPartStage) bound the group as well; only
      // visits of free poses form products. A landmark with more products than the stage holds
      // (>= 64 free observing poses, e.g. a long track in a full graph) gets a group of its own
      // whose products k_lm_visit streams from HBM instead.
      auto pairCount = [&](int l) {
        if (!laNew[l]) return 0;
        int nf = lmXBegin[l + 1] - lmXBegin[l];
        for (int v = lmVisitBegin[l]; v < lmVisitBegin[l + 1]; ++v) nf += posef[B.visit_pose[v] - pb] >= 0;
        return nf * (nf + 1) / 2;
      };
      int gpc = 0;
      B.visit_slot.resize(B.visit_pose.size(), -1);
      int g0 = 0, gl = 0;
      for (int l = 0; l < p->n_landmarks; ++l) {
        const int nv = lmVisitBegin[l + 1] - lmVisitBegin[l] + lmXBegin[l + 1] - lmXBegin[l];
        if (nv > kLmGroupVisits)
          throw ArgError{"landmark with more than " + std::to_string(kLmGroupVisits) + " observing poses"};
        const int gv = lmVisitBegin[l] - lmVisitBegin[g0] + lmXBegin[l] - lmXBegin[g0];
        const int pcl = pairCount(l);
        if (l > g0 && (gv + nv > B.lmg_visits || gl == B.lmg_lms || gpc + pcl > kLmPartStage)) {
          closeGroup(g0, l);
          g0 = l;
          gl = 0;
          gpc = 0;
        }
        ++gl;
        gpc += pcl;
      }
      if (p->n_landmarks > 0) closeGroup(g0, p->n_landmarks);
    }
    ATIME(6)
    // imu
    const int sBase = (int)B.imu_ts.size();
    for (int f = 0; f < p->n_imu; ++f) {
      const int* b = &p->imu_blocks[4 * f];
      const int32_t gb[4] = {pb + b[0], sbb + b[1], pb + b[2], sbb + b[3]};
      appendN(B.imu_blocks, gb, 4);
      B.imu_win.push_back(w);
      B.imu_flags.push_back(ifix[f] ? 2 : 0);
      B.imu_t0.push_back(p->imu_t0_ns[f]);
      B.imu_t1.push_back(p->imu_t1_ns[f]);
      B.imu_sbegin.push_back(sBase + p->imu_sample_begin[f] - p->imu_sample_begin[0]);
    }
    if (p->n_imu) {
      const int s0 = p->imu_sample_begin[0], s1 = p->imu_sample_begin[p->n_imu];
      appendN(B.imu_ts, &p->imu_sample_t_ns[s0], (size_t)(s1 - s0));
      appendN(B.imu_ga, &p->imu_sample_gyr_acc[6 * (size_t)s0], (size_t)6 * (s1 - s0));
    }
    {
      const okvisgpu_imu_params& ip = p->imu_params;
      const double par[7] = {ip.a_max, ip.g_max, ip.sigma_g_c, ip.sigma_a_c, ip.sigma_gw_c, ip.sigma_aw_c, ip.g};
      appendN(B.imu_par, par, 7);
    }
    for (int f = 0; f < p->n_imu; ++f) {
      if (p->imu_state) appendN(B.imu_state, &p->imu_state[(size_t)f * OKVISGPU_IMU_STATE_DOUBLES], OKVISGPU_IMU_STATE_DOUBLES);
      else B.imu_state.insert(B.imu_state.end(), OKVISGPU_IMU_STATE_DOUBLES, 0.0);
    }
    // host-evaluated factors (global pose-kind / speed-bias indices per slot)
    const int hgBase = B.n_imu_total + hfBase;  // global factor index of this window's first
    for (int h = 0; h < p->n_host; ++h) {
      const std::array<int, 4>& s = hslot[h];
      const int32_t gb[4] = {s[0] < 0 ? -1 : pb + s[0], s[1] < 0 ? -1 : sbb + s[1], s[2] < 0 ? -1 : pb + s[2],
                             s[3] < 0 ? -1 : sbb + s[3]};
      appendN(B.host_blocks, gb, 4);
      B.host_win.push_back(w);
      B.host_flags.push_back(hfix[h] ? 2 : 0);
    }
    {
      const int r_host[2] = {hgBase, hgBase + p->n_host};
      appendN(B.win_host_range, r_host, 2);
    }
    // priors
    for (const PPrior& q : pps) {
      B.pp_block.push_back(pb + q.blk);
      B.pp_win.push_back(w);
      appendN(B.pp_meas, q.meas, 7);
      appendN(B.pp_L, q.L, 36);
    }
    for (int i = 0; i < p->n_sb_priors; ++i) {
      B.sbp_block.push_back(sbb + p->sb_prior_block[i]);
      B.sbp_win.push_back(w);
      appendN(B.sbp_meas, &p->sb_prior_meas[9 * i], 9);
      appendN(B.sbp_L, &p->sb_prior_sqrt_info[81 * i], 81);
    }
    for (int i = 0; i < p->n_relpose; ++i) {
      B.rp_blocks.push_back(pb + p->relpose_blocks[2 * i]);
      B.rp_blocks.push_back(pb + p->relpose_blocks[2 * i + 1]);
      B.rp_win.push_back(w);
      B.rp_flags.push_back(rfix[i] ? 2 : 0);
      B.rp_kind.push_back(p->relpose_kind ? p->relpose_kind[i] : 0);
      appendN(B.rp_dx, &p->relpose_delta_x[6 * i], 6);
      appendN(B.rp_J, &p->relpose_sqrt_info[36 * i], 36);
      appendN(B.rp_lp, &p->relpose_lin_point[7 * i], 7);
    }
    // ranges
    const int r_pose[2] = {pb, pb + npx}, r_sb[2] = {sbb, sbb + p->n_speed_biases},
              r_lm[2] = {lb, lb + p->n_landmarks}, r_obs[2] = {ob, ob + p->n_observations},
              r_imu[2] = {ib, ib + p->n_imu}, r_pp[2] = {ppb, ppb + (int)pps.size()},
              r_sbp[2] = {sbpb, sbpb + p->n_sb_priors}, r_rp[2] = {rpb, rpb + p->n_relpose};
    appendN(B.win_pose_range, r_pose, 2); appendN(B.win_sb_range, r_sb, 2); appendN(B.win_lm_range, r_lm, 2);
    appendN(B.win_obs_range, r_obs, 2); appendN(B.win_imu_range, r_imu, 2); appendN(B.win_pp_range, r_pp, 2);
    appendN(B.win_sbp_range, r_sbp, 2);
    appendN(B.win_rp_range, r_rp, 2);

    ATIME(7)
    // ---- f-block gradient / diagonal contribution lists
    const int nFb = (int)B.fb_win.size() - fbBase;
    std::vector<std::vector<Contrib>> fbc(nFb);
    for (int i = 0; i < npx; ++i) {
      if (poseFb[i] < 0) continue;
      for (int sg : segsAtPose[i]) fbc[poseFb[i] - fbBase].push_back(Contrib{C_VISIT, sg, 0, 0});
    }
    const int imuCol[4] = {0, 6, 15, 21};
    for (int f = 0; f < p->n_imu; ++f) {
      if (ifix[f]) continue;
      const int* b = &p->imu_blocks[4 * f];
      const int fbs[4] = {poseFb[b[0]], sbFb[b[1]], poseFb[b[2]], sbFb[b[3]]};
      for (int q = 0; q < 4; ++q)
        if (fbs[q] >= 0) fbc[fbs[q] - fbBase].push_back(Contrib{C_IMU, ib + f, imuCol[q], imuCol[q]});
    }
    // host factors' slot f-blocks (-1: unused slot or constant block)
    auto hostFbs = [&](int h, int* fbs) {
      const std::array<int, 4>& s = hslot[h];
      for (int q = 0; q < 4; ++q) fbs[q] = s[q] < 0 ? -1 : (q & 1) ? sbFb[s[q]] : poseFb[s[q]];
    };
    for (int h = 0; h < p->n_host; ++h) {
      if (hfix[h]) continue;
      int fbs[4];
      hostFbs(h, fbs);
      for (int q = 0; q < 4; ++q)
        if (fbs[q] >= 0) fbc[fbs[q] - fbBase].push_back(Contrib{C_IMU, hgBase + h, imuCol[q], imuCol[q]});
    }
    for (size_t i = 0; i < pps.size(); ++i) {
      const int fb = poseFb[pps[i].blk];
      if (fb >= 0) fbc[fb - fbBase].push_back(Contrib{C_PPRIOR, ppb + (int)i, 0, 0});
    }
    for (int i = 0; i < p->n_sb_priors; ++i) {
      const int fb = sbFb[p->sb_prior_block[i]];
      if (fb >= 0) fbc[fb - fbBase].push_back(Contrib{C_SBPRIOR, sbpb + i, 0, 0});
    }
    for (int i = 0; i < p->n_relpose; ++i) {
      if (rfix[i]) continue;
      for (int q = 0; q < 2; ++q) {
        const int fb = poseFb[p->relpose_blocks[2 * i + q]];
        if (fb >= 0) fbc[fb - fbBase].push_back(Contrib{C_RELPOSE, rpb + i, 6 * q, 6 * q});
      }
    }
    for (int k = 0; k < nFb; ++k) {
      B.fb_cbegin.push_back((int)B.fb_contrib.size());
      B.fb_contrib.insert(B.fb_contrib.end(), fbc[k].begin(), fbc[k].end());
    }
    ATIME(8)
    // ---- block pairs (fi >= fj by reduced offset) and their contribution lists
    std::map<std::pair<int, int>, std::vector<Contrib>> pairs;
    auto key = [&](int fa, int fb2) {  // row = larger offset
      return B.fb_off[fa] >= B.fb_off[fb2] ? std::make_pair(fa, fb2) : std::make_pair(fb2, fa);
    };
    for (int i = 0; i < npx; ++i) {
      if (poseFb[i] < 0) continue;
      auto& lst = pairs[std::make_pair(poseFb[i], poseFb[i])];
      for (int sg : segsAtPose[i]) lst.push_back(Contrib{C_VISIT, sg, 0, 0});
    }
    for (size_t k = 0; k < partKeys.size(); ++k)  // partial Schur blocks, group order
      pairs[partKeys[k]].push_back(Contrib{C_PAIR, partBase + (int)k, 0, 0});
    for (int f = 0; f < p->n_imu; ++f) {
      if (ifix[f]) continue;
      const int* b = &p->imu_blocks[4 * f];
      const int fbs[4] = {poseFb[b[0]], sbFb[b[1]], poseFb[b[2]], sbFb[b[3]]};
      for (int u = 0; u < 4; ++u)
        for (int v = 0; v < 4; ++v) {
          if (fbs[u] < 0 || fbs[v] < 0) continue;
          if (B.fb_off[fbs[u]] < B.fb_off[fbs[v]]) continue;
          pairs[key(fbs[u], fbs[v])].push_back(Contrib{C_IMU, ib + f, imuCol[u], imuCol[v]});
        }
    }
    for (int h = 0; h < p->n_host; ++h) {
      if (hfix[h]) continue;
      int fbs[4];
      hostFbs(h, fbs);
      for (int u = 0; u < 4; ++u)
        for (int v = 0; v < 4; ++v) {
          if (fbs[u] < 0 || fbs[v] < 0) continue;
          if (B.fb_off[fbs[u]] < B.fb_off[fbs[v]]) continue;
          pairs[key(fbs[u], fbs[v])].push_back(Contrib{C_IMU, hgBase + h, imuCol[u], imuCol[v]});
        }
    }
    for (size_t i = 0; i < pps.size(); ++i) {
      const int fb = poseFb[pps[i].blk];
      if (fb >= 0) pairs[std::make_pair(fb, fb)].push_back(Contrib{C_PPRIOR, ppb + (int)i, 0, 0});
    }
    // pose-extrinsics cross blocks: sum over the observations of a free state pose through a
    // variable camera of J_e^T J_p (k_pose_extr); row = the extrinsics block (after all states)
    for (int ps = 0; ps < np; ++ps) {
      if (poseFb[ps] < 0) continue;
      for (int c = 0; c < ncam; ++c) {
        if (poseFb[np + c] < 0) continue;
        std::vector<int32_t> obs;
        for (int k = 0; k < p->n_observations; ++k) {
          const int o = order[k];
          if (p->obs_pose[o] == ps && p->obs_camera[o] == c && !ofix[o]) obs.push_back(ob + k);
        }
        if (obs.empty()) continue;
        pairs[key(poseFb[np + c], poseFb[ps])].push_back(Contrib{C_PEXT, (int)B.pe_pose.size(), 0, 0});
        B.pe_pose.push_back(pb + ps);
        B.pe_ext.push_back(pb + np + c);
        B.pe_obs_begin.push_back((int32_t)B.pe_obs.size());
        B.pe_obs.insert(B.pe_obs.end(), obs.begin(), obs.end());
      }
    }
    for (int i = 0; i < p->n_sb_priors; ++i) {
      const int fb = sbFb[p->sb_prior_block[i]];
      if (fb >= 0) pairs[std::make_pair(fb, fb)].push_back(Contrib{C_SBPRIOR, sbpb + i, 0, 0});
    }
    for (int i = 0; i < p->n_relpose; ++i) {
      if (rfix[i]) continue;
      const int fbs[2] = {poseFb[p->relpose_blocks[2 * i]], poseFb[p->relpose_blocks[2 * i + 1]]};
      for (int u = 0; u < 2; ++u)
        for (int v = 0; v < 2; ++v) {
          if (fbs[u] < 0 || fbs[v] < 0) continue;
          if (B.fb_off[fbs[u]] < B.fb_off[fbs[v]]) continue;
          pairs[key(fbs[u], fbs[v])].push_back(Contrib{C_RELPOSE, rpb + i, 6 * u, 6 * v});
        }
    }
    ATIME(9)
    // diagonal pairs must exist for every f-block (they carry the damping, diag and rhs)
    for (int k = fbBase; k < (int)B.fb_win.size(); ++k) pairs[std::make_pair(k, k)];
    // tile-level structure of S and its symbolic LLT (fill within the envelope)
    {
      const int T = fpad / kTile;
      std::vector<uint8_t> nz((size_t)T * T, 0);
      for (int i = 0; i < T; ++i) nz[(size_t)i * T + i] = 1;
      for (auto& kv : pairs) {
        const int fa = kv.first.first, fb2 = kv.first.second;
        const int na = B.fb_kind[fa] == 0 ? 6 : 9, nb = B.fb_kind[fb2] == 0 ? 6 : 9;
        for (int ti = B.fb_off[fa] / kTile; ti <= (B.fb_off[fa] + na - 1) / kTile; ++ti)
          for (int tj = B.fb_off[fb2] / kTile; tj <= (B.fb_off[fb2] + nb - 1) / kTile; ++tj)
            nz[(size_t)std::max(ti, tj) * T + std::min(ti, tj)] = 1;
      }
      symbolicFill(nz, T);
      // first band update of every tile (a step k < j with L_ik and L_jk non-zero): until then the
      // factorisation reads the tile from the assembled S, afterwards from its working copy W
      std::vector<int16_t> fu((size_t)T * T, kNoUpdate);
      for (int i = 0; i < T; ++i)
        for (int j = 0; j <= i; ++j)
          for (int k = 0; k < j; ++k)
            if (nz[(size_t)i * T + k] && nz[(size_t)j * T + k]) {
              fu[(size_t)i * T + j] = (int16_t)k;
              break;
            }
      // backward substitution split (nested dissection): the tiles of the left part [0, tL) and of
      // the right part [tL, tS) share no non-zero tile, so once the separator's tiles [tS, T) are
      // solved the two parts are independent (k_chol_bsub: one workgroup each)
      int tL = rightAt / kTile, tS = sepAt / kTile;
      bool split = ndLeft > 0 && tL > 0 && tS > tL;
      for (int i = tL; split && i < tS; ++i)
        for (int j = 0; j < tL; ++j)
          if (nz[(size_t)i * T + j]) split = false;
      B.win_bsplit.push_back(split ? tL : 0);
      B.win_bsplit.push_back(split ? tS : 0);
      B.win_defoff.push_back(B.defer_total);
      if (split) B.defer_total += (int64_t)(T - tS) * (tS - tL) * kTile;
      B.any_split = B.any_split || split;
      B.tileFu.push_back(fu);
      B.tileNz.push_back(nz);
      B.tileT.push_back(T);
    }
    for (auto& kv : pairs) {
      B.pair_win.push_back(w);
      B.pair_fi.push_back(kv.first.first);
      B.pair_fj.push_back(kv.first.second);
      B.pair_cbegin.push_back((int)B.pair_contrib.size());
      // contributions are grouped by kind (visits, landmark pairs, then factor blocks); the
      // kernels stream each run separately
      {
        const int base = (int)B.pair_contrib.size();
        int np = 0, nv = 0;
        for (const Contrib& c : kv.second) { nv += c.type == C_VISIT; np += c.type == C_PAIR; }
        for (size_t i = 0; i < kv.second.size(); ++i) {
          const int t = kv.second[i].type;
          const bool ok = (int)i < nv ? t == C_VISIT : ((int)i < nv + np ? t == C_PAIR : (t != C_VISIT && t != C_PAIR));
          if (!ok) throw std::logic_error("pair contribution runs out of order");
        }
        B.pair_runs.push_back(base + nv);
        B.pair_runs.push_back(base + nv + np);
      }
      B.pair_contrib.insert(B.pair_contrib.end(), kv.second.begin(), kv.second.end());
    }
  }
  // tile-parallel schedule (cholSchedule): launch 0 factors every window's root tiles; launch
  // l >= 1 runs the band updates of the steps scheduled there, each item (w, i, j, mode | k << 8):
  // mode bit 0 = update of tile (i, j) by step k (panels formed from X_k), bit 1 = factor tile
  // i (= j) afterwards (the item is its last update)
  {
    std::vector<std::vector<int32_t>> byLaunch(1);
    for (int w = 0; w < B.n_win; ++w) {
      const int T = B.tileT[w];
      const auto& nz = B.tileNz[w];
      std::vector<int> L, last;
      const int nl = cholSchedule(nz, T, L, last);
      B.n_chol_launches = std::max(B.n_chol_launches, nl);
      if ((int)byLaunch.size() < nl) byLaunch.resize(nl);
      bool first = true;
      for (int d = 0; d < T; ++d)
        if (last[(size_t)d * T + d] < 0) {
          B.chol_root_items.push_back(w);
          B.chol_root_items.push_back(d);
          B.chol_root_items.push_back(first ? 1 : 0);
          first = false;
        }
      for (int k = 0; k < T; ++k)
        for (int i = k + 1; i < T; ++i)
          if (nz[(size_t)i * T + k]) ++B.n_panels;
      for (int k = 0; k < T; ++k)
        for (int i = k + 1; i < T; ++i)
          if (nz[(size_t)i * T + k])
            for (int j = k + 1; j <= i; ++j)
              if (nz[(size_t)j * T + k]) {
                const bool fac = i == j && last[(size_t)i * T + i] == L[k];
                auto& v = byLaunch[L[k]];
                v.push_back(w); v.push_back(i); v.push_back(j); v.push_back((fac ? 3 : 1) | (k << 8));
                ++B.n_band_updates;
                if (i == j) ++B.n_band_updates_diag;
              }
    }
    for (size_t l = 0; l < byLaunch.size(); ++l) {
      B.chol_upd_begin.push_back((int)B.chol_upd_items.size() / 4);
      B.chol_upd_items.insert(B.chol_upd_items.end(), byLaunch[l].begin(), byLaunch[l].end());
    }
    B.chol_upd_begin.push_back((int)B.chol_upd_items.size() / 4);
  }
  // assembly work lists: pose-pose pairs (one wavefront each, 4 per workgroup) are grouped so
  // that workgroups b, b+8, ... (one XCD under round-robin placement; speed only) walk the pairs of
  // the same windows and share their visit blocks in that XCD's L2
  // Off-diagonal pairs with few contributions (no visits; partial blocks and factor blocks only)
  // take a 16-lane quarter of a wavefront each (k_assemble_pp_light, 16 per workgroup).
  {
    constexpr int kXcd = 8;
    const int nq = B.n_win >= kXcd ? kXcd : 1;
    std::vector<std::vector<int32_t>> q(nq), ql(nq);
    for (int k = 0; k < (int)B.pair_win.size(); ++k) {
      const bool pp = B.fb_kind[B.pair_fi[k]] == 0 && B.fb_kind[B.pair_fj[k]] == 0;
      const int kend = k + 1 < (int)B.pair_cbegin.size() ? B.pair_cbegin[k + 1] : (int)B.pair_contrib.size();
      const bool light = B.n_win >= kManyWindows && B.pair_fi[k] != B.pair_fj[k] &&
                         B.pair_runs[2 * k] == B.pair_cbegin[k] && kend - B.pair_cbegin[k] <= kAsmLightMax;
      if (!pp) B.asm_sb_items.push_back(k);
      else if (light) ql[B.pair_win[k] % nq].push_back(k);
      else q[B.pair_win[k] % nq].push_back(k);
    }
    auto interleave = [&](std::vector<std::vector<int32_t>>& qq, int perWG, std::vector<int32_t>& out) {
      std::vector<size_t> pos(nq, 0);
      bool more = true;
      while (more) {
        more = false;
        for (int x = 0; x < nq; ++x)
          for (int i = 0; i < perWG; ++i) {
            const bool has = pos[x] < qq[x].size();
            out.push_back(has ? qq[x][pos[x]++] : -1);
          }
        for (int x = 0; x < nq; ++x) more = more || pos[x] < qq[x].size();
      }
      while (!out.empty() && out.back() < 0) out.pop_back();
    };
    interleave(q, 4, B.asm_pp_items);
    interleave(ql, 16, B.asm_ppl_items);
  }
  for (int w = 0; w < B.n_win; ++w) {
    B.win_tnzoff.push_back((int64_t)B.tile_nz.size());
    B.tile_nz.insert(B.tile_nz.end(), B.tileNz[w].begin(), B.tileNz[w].end());
    B.tile_fu.insert(B.tile_fu.end(), B.tileFu[w].begin(), B.tileFu[w].end());
    const int T = B.tileT[w];
    for (int k = 0; k < T; ++k) {
      int np = 0;
      for (int i = k + 1; i < T; ++i) np += B.tileNz[w][(size_t)i * T + k] ? 1 : 0;
      B.max_panels = std::max(B.max_panels, np);
    }
  }
  for (int w = 0; w < B.n_win; ++w) {
    const int T = B.tileT[w];
    for (int i = 0; i < T; ++i)
      for (int j = 0; j <= i; ++j)
        if (B.tileNz[w][(size_t)i * T + j]) { B.tile_items.push_back(w); B.tile_items.push_back(i); B.tile_items.push_back(j); }
  }
  B.lm_visit_begin.push_back((int)B.visit_pose.size());
  B.lmg_begin.push_back((int)B.lm_win.size());  // groups: begin of each, then the end
  {  // each window's groups are contiguous (built window by window)
    B.win_lmg_range.assign(2 * (size_t)B.n_win, 0);
    const int ng = (int)B.lmg_begin.size() - 1;
    std::vector<int> first(B.n_win, -1), last(B.n_win, -1);
    for (int g = 0; g < ng; ++g) {
      const int w = B.lm_win[B.lmg_begin[g]];
      if (first[w] < 0) first[w] = g;
      last[w] = g;
    }
    for (int w = 0; w < B.n_win; ++w)
      if (first[w] >= 0) {
        B.win_lmg_range[2 * w] = first[w];
        B.win_lmg_range[2 * w + 1] = last[w] + 1;
      }
  }
  B.lmg_xbegin.push_back((int)B.xvisit_pose.size());
  B.xvisit_obs_begin.push_back((int)B.xvisit_obs.size());
  B.pe_obs_begin.push_back((int)B.pe_obs.size());
  B.part_cbegin.push_back((int)B.part_contrib.size());
  B.visit_obs_begin.push_back((int)B.obs_win.size());
  B.imu_sbegin.push_back((int)B.imu_ts.size());
  // host-evaluated factors share the IMU factors' per-factor arrays, after all of them
  B.imu_blocks.insert(B.imu_blocks.end(), B.host_blocks.begin(), B.host_blocks.end());
  B.imu_win.insert(B.imu_win.end(), B.host_win.begin(), B.host_win.end());
  B.imu_flags.insert(B.imu_flags.end(), B.host_flags.begin(), B.host_flags.end());
  B.fb_cbegin.push_back((int)B.fb_contrib.size());
  B.pair_cbegin.push_back((int)B.pair_contrib.size());
  {  // per-group record (two 16-byte loads; the terminal entry closes the last group)
    const int ng = (int)B.lmg_begin.size() - 1;
    B.lmg_info.assign(kLmgInfo * (size_t)(ng + 1), 0);
    for (int g = 0; g <= ng; ++g) {
      const int l0 = B.lmg_begin[g];
      int32_t* r = &B.lmg_info[kLmgInfo * (size_t)g];
      r[0] = l0;
      r[1] = B.lm_visit_begin[l0];
      r[2] = g < ng ? B.lm_win[l0] : -1;
      r[3] = B.seg_gbegin[g];
      r[4] = B.part_gbegin[g];
      r[5] = B.part_cbegin[B.part_gbegin[g]];
    }
  }
  ATIME(10)
}

// A single hipMalloc arena carved into the device arrays.
struct Arena {
  char* base = nullptr;
  size_t size = 0, used = 0;
  std::vector<std::pair<size_t, size_t>> plan;
  size_t reserve(size_t bytes) {
    const size_t off = (size + 255) & ~size_t(255);
    size = off + std::max<size_t>(bytes, 8);
    return off;
  }
  template <class T>
  T* at(size_t off) const { return reinterpret_cast<T*>(base + off); }
};

}  // namespace

// Persistent host worker threads of one context: the host-evaluated factors (ABI 5) are evaluated
// at every point the solver evaluates, from the HIP callback thread of the iteration graph's host
// node, so the workers are created once (grown on demand) instead of per evaluation. run(n, f)
// calls f(0..n-1) on n workers and returns when all are done.
class HostWorkers {
 public:
  ~HostWorkers() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    wake_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(int n, const std::function<void(int)>& f) {
    while ((int)th_.size() < n) {
      const int id = (int)th_.size();
      th_.emplace_back([this, id]() { loop(id); });
    }
    std::unique_lock<std::mutex> l(m_);
    job_ = &f;
    njob_ = n;
    pending_ = n;
    ++gen_;
    wake_.notify_all();
    done_.wait(l, [&]() { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int id) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> l(m_);
    for (;;) {
      wake_.wait(l, [&]() { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      if (id >= njob_) continue;
      const std::function<void(int)>* f = job_;
      l.unlock();
      (*f)(id);
      l.lock();
      if (--pending_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable wake_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int njob_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct okvisgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side[3] = {nullptr, nullptr, nullptr};  // fork streams of the captured iteration graph
  std::vector<hipEvent_t> forkEv;
  size_t forkEvUsed = 0;  // events of forkEv taken by the capture in progress
  std::string last_error;
  HostBatch B;
  std::vector<const okvisgpu_problem*> probs;
  std::map<std::tuple<int, int, int>, int> constOverride;
  void* hostStage = nullptr;  // pinned staging of the uploaded arrays (kept between set_problems)
  size_t hostStageBytes = 0;
  size_t arenaCap = 0;        // bytes allocated at `arena` (reused while a new batch fits)
  bool structureDirty = false;
  DevProblem P{};
  void* arena = nullptr;
  size_t arenaBytes = 0;
  hipGraphExec_t iterGraph = nullptr;
  // kGraphIters iterations captured as one graph as well (iterGraphK): consecutive launches of one
  // graph are ~8 us apart on the device (4.5 % of the S10 single-window iteration; batches +0.2-0.3 %,
  // r05bk), so solve_iterate runs n iterations as n / K launches of it and n mod K of the single one.
  static constexpr int kGraphIters = 4;
  hipGraphExec_t iterGraphK = nullptr;
  int graphIters = 1;
  int cuCount = 256;
  size_t ldsPerBlock = 65536;
  bool persistentFits() const { return cholesky_persistent_fits(P.max_fpad, ldsPerBlock); }
  bool pipeFits() const { return cholesky_pipe_fits(P.max_fpad, ldsPerBlock); }
  // S is cleared by the build's arena memset; its padded diagonal (rows >= fdim) is set once per
  // build before the first factorisation (k_zero_S setup mode). The factorisation works in W and
  // the assembly overwrites its blocks, so S needs no clearing per iteration.
  bool sNeedsInit = true;
  void ensureS(hipStream_t s) {
    if (!sNeedsInit) return;
    launch_zero_S(P, s, 2);
    sNeedsInit = false;
  }
  bool haveProblem = false;
  // split-solve state
  bool inSolve = false;
  okvisgpu_options opts{};
  int replays = 0;
  double solveT0 = 0.0;
  // summary timings (okvisgpu_summary, ABI 6): wall clock of begin / iterations / write-back, and
  // the iterations' device time per phase when the solve ran them eagerly (options.verbose)
  double tPre = 0.0, tIterStart = 0.0, tMin = 0.0, tPost = 0.0;
  bool phasesTimed = false;
  double phaseMs[OKVISGPU_N_PHASES] = {};
  // host-evaluated factors (ABI 5): pinned copies of host_in / host_out and per-factor failure
  // flags of the last evaluation, written by hostEvaluate() on the HIP callback thread
  double* hostIn = nullptr;
  double* hostOut = nullptr;
  int hostBufFactors = 0;
  std::vector<uint8_t> hostFail;
  HostWorkers hostWorkers;

  void fillSummaries(const std::vector<WinState>& st, okvisgpu_summary* sums) {
    if (!sums) return;
    const double t1 = nowS();
    for (int w = 0; w < P.n_win; ++w) {
      const WinState& s = st[w];
      okvisgpu_summary& S = sums[w];
      std::memset(&S, 0, sizeof(S));
      S.initial_cost = s.initial_cost;
      S.final_cost = std::min(s.min_cost, s.x_cost) + s.fixed_cost;
      S.num_iterations = s.iteration;
      S.num_successful_steps = s.num_succ + 1;  // Ceres counts iteration 0
      S.num_unsuccessful_steps = s.num_unsucc;
      S.termination_type = s.done ? s.termination : OKVISGPU_NO_CONVERGENCE;
      S.total_time_s = t1 - solveT0;
      S.final_radius = s.radius;
      S.final_mu = s.mu;
      S.preprocessor_time_s = tPre;
      S.minimizer_time_s = tMin;
      S.postprocessor_time_s = tPost;
      S.linear_solver_time_s = S.residual_evaluation_time_s = S.jacobian_evaluation_time_s = S.step_time_s = -1.0;
      if (phasesTimed) {  // phase ids: kPhaseNames
        auto sum = [&](std::initializer_list<int> ids) {
          double t = 0.0;
          for (int i : ids) t += phaseMs[i];
          return t * 1e-3;
        };
        S.linear_solver_time_s = sum({0, 1, 2, 3, 4, 5, 6, 7});
        S.step_time_s = sum({8});
        S.residual_evaluation_time_s = sum({9, 10, 11, 12});
        S.jacobian_evaluation_time_s = sum({13, 14});
      }
    }
  }

  // end of a solve: iterations done (states were just read back), write-back, summaries
  void finish(const std::vector<WinState>& st, okvisgpu_summary* sums) {
    const double t = nowS();
    tMin = t - tIterStart;
    for (int w = 0; w < P.n_win; ++w)
      if (st[w].dev_error) {
        inSolve = false;
        throw HipError{"window " + std::to_string(w) + ": the pipelined Cholesky's team wait reached its limit",
                       OKVISGPU_ERR_DEVICE};
      }
    downloadParams();
    inSolve = false;
    tPost = nowS() - t;
    fillSummaries(st, sums);
  }

  // One trust-region iteration as eager launches on the context's stream with HIP events between
  // the phases (the captured graph's kernels in the same order: the same bits); ms[phase] += the
  // phase's device time. okvisgpu_profile_iteration and the verbose solve.
  void profiledIteration(double* ms) {
    hipStream_t s = stream;
    std::vector<hipEvent_t> ev;
    std::vector<int> phaseOf;
    auto mark = [&](int phase) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      HIPCHK(hipEventRecord(e, s));
      ev.push_back(e);
      phaseOf.push_back(phase);
    };
    mark(-1);
    launch_lm_prep(P, s); mark(0);
    mark(1);  // (S is no longer cleared per iteration: phase kept for the ABI's phase list)
    launch_assemble(P, s); mark(2);
    launch_cholesky(P, s); mark(3);
    mark(5);  // (gn_finalize: fused into the Cholesky's back substitution; phase kept for the ABI list)
    launch_lm_backsub(P, s); mark(4);
    mark(6);  // (jv: the trailing workgroups of lm_backsub; phase kept for the ABI list)
    mark(7);  // (the J*v reduction runs inside k_dogleg)
    launch_dogleg(P, s); mark(8);
    launch_eval_obs(P, 1, s); mark(9);
    launch_eval_imu(P, 1, s); mark(10);
    launch_eval_priors(P, 1, s);
    evalHost(1, s); mark(11);  // host-evaluated factors at the candidate (counted with the priors)
    launch_reduce(P, R_COST_CAND, s); mark(12);
    launch_linearization_blocks(P, 1, s); mark(13);
    launch_gradnorm(P, 1, s); mark(14);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    for (size_t i = 1; i < ev.size(); ++i) {
      float t = 0.f;
      HIPCHK(hipEventElapsedTime(&t, ev[i - 1], ev[i]));
      ms[phaseOf[i]] += t;
    }
    for (auto e : ev) (void)hipEventDestroy(e);
  }

  ~okvisgpu_ctx() {
    dropGraph();
    if (arena) (void)hipFree(arena);
    if (hostStage) (void)hipHostFree(hostStage);
    if (hostIn) (void)hipHostFree(hostIn);
    if (hostOut) (void)hipHostFree(hostOut);
    for (hipEvent_t e : forkEv) (void)hipEventDestroy(e);
    for (hipStream_t q : side)
      if (q) (void)hipStreamDestroy(q);
    if (stream) (void)hipStreamDestroy(stream);
  }

  void dropGraph() {
    if (iterGraph) {
      (void)hipGraphExecDestroy(iterGraph);
      iterGraph = nullptr;
    }
    if (iterGraphK) {
      (void)hipGraphExecDestroy(iterGraphK);
      iterGraphK = nullptr;
    }
    graphIters = 1;
  }
  // n iterations of the captured graph(s), in stream order
  void launchIterations(int n) {
    int k = 0;
    if (iterGraphK)
      for (; k + graphIters <= n; k += graphIters) HIPCHK(hipGraphLaunch(iterGraphK, stream));
    for (; k < n; ++k) HIPCHK(hipGraphLaunch(iterGraph, stream));
  }

  // ---- host-evaluated factors (SURVEY.md §8b fallback) ------------------------------------------
  // Every evaluation point (initial, each candidate) runs, in stream order: k_host_gather (the
  // blocks' values of the factors the eval mode selects) -> copy to pinned memory -> host node
  // (hostEvaluate: the caller's Evaluate on options.num_threads threads, manifold + loss applied
  // here) -> copy back -> k_host_scatter into the IMU-layout linearisation records. All of it is
  // graph-capturable (the host step is a host node of the captured iteration).
  void ensureHostBuffers() {
    hostFail.assign((size_t)P.n_host, 0);
    if (P.n_host <= hostBufFactors) return;
    if (hostIn) HIPCHK(hipHostFree(hostIn));
    if (hostOut) HIPCHK(hipHostFree(hostOut));
    hostIn = hostOut = nullptr;
    hostBufFactors = 0;
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&hostIn), sizeof(double) * kHostIn * P.n_host, hipHostMallocDefault));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&hostOut), sizeof(double) * kHostOut * P.n_host, hipHostMallocDefault));
    hostBufFactors = P.n_host;
  }

  // PoseManifold plus Jacobian at x, 7x6 row-major (PoseLocalParameterization.cpp:56-68): the
  // minimal Jacobian of a pose-kind block is J_ambient * this, as Ceres applies a block's manifold.
  static void posePlusJacobian(const double* x, double* J) {
    for (int i = 0; i < 42; ++i) J[i] = 0.0;
    J[0 * 6 + 0] = J[1 * 6 + 1] = J[2 * 6 + 2] = 1.0;
    const double qx = x[3], qy = x[4], qz = x[5], qw = x[6];
    const double Q[4][3] = {{qw, qz, -qy}, {-qz, qw, qx}, {qy, -qx, qw}, {-qx, -qy, -qz}};  // oplus(q), cols 0..2
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 3; ++c) J[(3 + r) * 6 + 3 + c] = Q[r][c] * 0.5;
  }

  // One host factor: Evaluate at the gathered point; r and the minimal Jacobian (IMU column
  // layout), corrected for the factor's loss (Ceres' Corrector, both branches) unless mode 3 (raw
  // evaluation), into its host_out record. Failure: cost +inf, r = J = 0.
  void hostEvaluateOne(int h) {
    const double* in = hostIn + (size_t)h * kHostIn;
    double* out = hostOut + (size_t)h * kHostOut;
    if (in[0] == 0.0) return;
    const int mode = (int)in[1];
    const HostBatch::HostFactor& F = B.hf[h];
    const okvisgpu_problem* p = probs[F.win];
    static const int at[4] = {8, 15, 24, 31}, col[4] = {0, 6, 15, 21};
    const double* prm[4] = {nullptr, nullptr, nullptr, nullptr};
    double amb[4][OKVISGPU_HOST_MAX_RESIDUALS * 9];
    double* jac[4] = {nullptr, nullptr, nullptr, nullptr};
    double r[OKVISGPU_HOST_MAX_RESIDUALS];
    for (int k = 0; k < F.np; ++k) {
      prm[k] = in + at[F.slot[k]];
      jac[k] = amb[k];
      std::memset(amb[k], 0, sizeof(amb[k]));
    }
    std::memset(r, 0, sizeof(r));
    std::memset(out, 0, sizeof(double) * kHostOut);
    int ok = 0;
    try {
      ok = p->host_evaluate(p->host_user, F.local, prm, r, jac);
    } catch (...) {
      ok = 0;
    }
    hostFail[h] = ok ? 0 : 1;
    if (!ok) {
      out[0] = HUGE_VAL;
      return;
    }
    double sq = 0.0;
    for (int i = 0; i < F.dim; ++i) sq += r[i] * r[i];
    // minimal Jacobian (IMU column layout): ambient * PoseManifold plus Jacobian for pose-kind
    // blocks, identity for speed/bias
    double* J = out + 1 + 15;
    for (int k = 0; k < F.np; ++k) {
      const int q = F.slot[k];
      if (q & 1) {  // speed/bias: identity manifold
        for (int i = 0; i < F.dim; ++i)
          for (int c = 0; c < 9; ++c) J[i * 30 + col[q] + c] = amb[k][i * 9 + c];
      } else {
        double Jp[42];
        posePlusJacobian(prm[k], Jp);
        for (int i = 0; i < F.dim; ++i)
          for (int c = 0; c < 6; ++c) {
            double s = 0.0;
            for (int a = 0; a < 7; ++a) s += amb[k][i * 7 + a] * Jp[a * 6 + c];
            J[i * 30 + col[q] + c] = s;
          }
      }
    }
    for (int i = 0; i < F.dim; ++i) out[1 + i] = r[i];
    if (F.loss.kind == OKVISGPU_LOSS_NONE || mode == 3) {
      out[0] = 0.5 * sq;
      return;
    }
    // Ceres' Corrector (internal/ceres/corrector.cc; okvis restates it at TwoPoseGraphError.cpp:
    // 292-337), applied to the minimal Jacobian as Ceres' ResidualBlock does after the manifold
    double rho[3];
    lossRho(F.loss, sq, rho);
    out[0] = 0.5 * rho[0];
    const double sqrtRho1 = std::sqrt(rho[1]);
    double rScale = sqrtRho1, alphaSq = 0.0;
    if (sq != 0.0 && rho[2] > 0.0) {  // second-order (Triggs) correction
      const double D = 1.0 + 2.0 * sq * rho[2] / rho[1];
      const double alpha = 1.0 - std::sqrt(D);
      rScale = sqrtRho1 / (1.0 - alpha);
      alphaSq = alpha / sq;
    }
    for (int k = 0; k < F.np; ++k) {
      const int q = F.slot[k], nc = (q & 1) ? 9 : 6;
      for (int c = 0; c < nc; ++c) {
        double* Jc = J + col[q] + c;
        if (alphaSq == 0.0) {
          for (int i = 0; i < F.dim; ++i) Jc[i * 30] *= sqrtRho1;
          continue;
        }
        double rtj = 0.0;
        for (int i = 0; i < F.dim; ++i) rtj += Jc[i * 30] * r[i];
        for (int i = 0; i < F.dim; ++i) Jc[i * 30] = sqrtRho1 * (Jc[i * 30] - alphaSq * r[i] * rtj);
      }
    }
    for (int i = 0; i < F.dim; ++i) out[1 + i] = r[i] * rScale;
  }

  void hostEvaluate() {
    const int n = P.n_host;
    const int nt = std::min(std::max(1, std::min(16, opts.num_threads)), n / 8);
    if (nt <= 1) {
      for (int h = 0; h < n; ++h) hostEvaluateOne(h);
      return;
    }
    hostWorkers.run(nt, [this, n, nt](int t) {
      for (int h = (int)((int64_t)n * t / nt); h < (int)((int64_t)n * (t + 1) / nt); ++h) hostEvaluateOne(h);
    });
  }
  static void hostEvaluateCallback(void* self) { static_cast<okvisgpu_ctx*>(self)->hostEvaluate(); }

  void evalHost(int mode, hipStream_t s) {
    if (P.n_host == 0) return;
    launch_host_gather(P, mode, s);
    HIPCHK(hipMemcpyAsync(hostIn, P.host_in, sizeof(double) * kHostIn * P.n_host, hipMemcpyDeviceToHost, s));
    HIPCHK(hipLaunchHostFunc(s, hostEvaluateCallback, this));
    HIPCHK(hipMemcpyAsync(P.host_out, hostOut, sizeof(double) * kHostOut * P.n_host, hipMemcpyHostToDevice, s));
    launch_host_scatter(P, s);
  }
  // every residual of the batch at one evaluation point (mode: launch.hpp)
  void evalAll(int mode, hipStream_t s) {
    launch_eval(P, mode, s);
    evalHost(mode, s);
  }
  // after the initial evaluation: a window whose host factor failed there ends with FAILURE
  // (Ceres: "Residual and Jacobian evaluation failed" at iteration 0)
  void failInitialHostEvaluations() {
    if (P.n_host == 0) return;
    HIPCHK(hipStreamSynchronize(stream));
    std::vector<uint8_t> bad(P.n_win, 0);
    bool any = false;
    for (int h = 0; h < P.n_host; ++h)
      if (hostFail[h]) any = bad[B.hf[h].win] = 1;
    if (!any) return;
    std::vector<WinState> st = readStates();
    for (int w = 0; w < P.n_win; ++w)
      if (bad[w]) {
        st[w].done = 1;
        st[w].termination = OKVISGPU_FAILURE;
      }
    HIPCHK(hipMemcpyAsync(P.st, st.data(), sizeof(WinState) * st.size(), hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }

  // (Re)build the device problem. Nothing of the previous batch survives a failure: the context
  // holds no problem until a build completes (entry points then return OKVISGPU_ERR_NO_PROBLEM).
  void build() {
    haveProblem = false;
    inSolve = false;
    dropGraph();
    const bool timing = std::getenv("OKVISGPU_BUILD_TIMING") != nullptr;  // development: host cost split
    const auto tb0 = std::chrono::steady_clock::now();
    {
      HostBatch nb;
      // nested-dissection order where the tile-parallel or the split persistent schedule will run
      // (at most one window per CU, setOptions): the chain of a window's factorisation is the
      // latency there. The order is a function of the window and this flag only, so a window's
      // bits depend on the batch just through it.
      nb.nd = (int)probs.size() < cuCount;
#ifdef OKG_ND_OVERRIDE
      if (const char* e = std::getenv("OKVISGPU_ND")) nb.nd = e[0] == '1';  // (development A/B builds only)
#endif
      // smaller landmark groups where a window's linearisation is a latency chain (fewWindows: one
      // workgroup per group, ~16 us of phases for a 256-visit group): 64 visits / 16 landmarks
      // (one S50 window: 36 -> 144 groups; steady iteration 0.3144 -> 0.3121 ms, S10 0.1580 ->
      // 0.1541 ms, profiles/r06_lmg_ab.txt). Like the state order, a function of the batch size only.
      if (fewWindows((int)probs.size(), cuCount)) {
        nb.lmg_visits = 64;
        nb.lmg_lms = 16;
      }
#ifdef OKG_LMG_OVERRIDE  // (development A/B builds only: OKVISGPU_LMG=visits,landmarks)
      if (const char* e = std::getenv("OKVISGPU_LMG")) {
        int v = 0, m = 0;
        if (std::sscanf(e, "%d,%d", &v, &m) == 2 && v >= 1 && v <= kLmGroupVisits && m >= 1 && m <= kLmGroupMax) {
          nb.lmg_visits = v;
          nb.lmg_lms = m;
        }
      }
#endif
      analyse(probs, constOverride, nb);  // may throw: B is untouched until it succeeds
      B = std::move(nb);
    }
    const auto tb1 = std::chrono::steady_clock::now();
    // the uploaded arrays are laid out first (one contiguous host -> device copy from a pinned
    // staging buffer), the scratch arrays after them (one memset); a scratch offset carries
    // kScratchTag until the two regions are placed
    constexpr size_t kScratchTag = size_t(1) << 62;
    Arena A, AS;
    DevProblem& D = P;
    D = DevProblem{};
    D.n_win = B.n_win;
    D.n_pose = (int)B.pose_win.size();
    D.n_sb = (int)B.sb_win.size();
    D.n_lm = (int)B.lm_win.size();
    D.n_obs = (int)B.obs_win.size();
    D.n_visit = (int)B.visit_pose.size();
    D.cu_count = cuCount;
    D.lin_prep = -1;
    D.n_imu = B.n_imu_total;
    D.n_host = (int)B.hf.size();
    D.n_fac = D.n_imu + D.n_host;
    D.n_pprior = (int)B.pp_win.size();
    D.n_sbprior = (int)B.sbp_win.size();
    D.n_relpose = (int)B.rp_win.size();
    D.n_cam = (int)(B.cam.size() / kCamDoubles);
    D.n_fblock = (int)B.fb_win.size();
    D.n_pair = (int)B.pair_win.size();
    D.max_fpad = B.max_fpad;
    D.max_tiles = B.max_fpad / kTile;
    D.obs_stride = ((int64_t)D.n_obs + 63) / 64 * 64;
    // ---- plan
    struct Up { size_t off; const void* src; size_t bytes; };
    std::vector<Up> ups;
    auto upl = [&](const auto& vec) -> size_t {
      using T = typename std::decay_t<decltype(vec)>::value_type;
      const size_t bytes = vec.size() * sizeof(T);
      const size_t off = A.reserve(bytes);
      ups.push_back(Up{off, vec.data(), bytes});
      return off;
    };
    auto scratch = [&](size_t bytes) { return kScratchTag | AS.reserve(bytes); };
    const size_t o_pose0 = upl(B.pose), o_pose1 = upl(B.pose), o_sb0 = upl(B.sb), o_sb1 = upl(B.sb);
    const size_t o_lm0 = upl(B.lm), o_lm1 = upl(B.lm), o_extr = upl(B.extr), o_cam = upl(B.cam);
    const size_t o_pose_win = upl(B.pose_win), o_sb_win = upl(B.sb_win), o_lm_win = upl(B.lm_win);
    const size_t o_pose_f = upl(B.pose_f), o_sb_f = upl(B.sb_f), o_lm_free = upl(B.lm_free);
    const size_t o_pose_act = upl(B.pose_active), o_sb_act = upl(B.sb_active);
    const size_t o_obs_pose = upl(B.obs_pose), o_obs_lm = upl(B.obs_lm), o_obs_cam = upl(B.obs_cam),
                 o_obs_win = upl(B.obs_win), o_obs_flags = upl(B.obs_flags), o_obs_kp = upl(B.obs_kp),
                 o_obs_L = upl(B.obs_L);
    // every reprojection's square-root information diag(s, s) (okvis' keypoint-size information;
    // +0.0 off the diagonal): k_eval_obs then reads s alone (8 instead of 32 bytes per observation)
    // and forms the same products with the constant zeros, so the same bits
    B.obs_iso = D.n_obs > 0;
    B.obs_Ls.assign(std::max(1, D.n_obs), 0.0);
    for (int o = 0; o < D.n_obs && B.obs_iso; ++o) {
      const double* L = B.obs_L.data() + 4 * (size_t)o;
      B.obs_iso = L[1] == 0.0 && !std::signbit(L[1]) && L[2] == 0.0 && !std::signbit(L[2]) && L[0] == L[3] &&
                  std::signbit(L[0]) == std::signbit(L[3]);
      B.obs_Ls[o] = L[0];
    }
    const size_t o_obs_Ls = upl(B.obs_Ls);
    const size_t o_obs_lin0 = scratch(sizeof(double) * kObsLin * D.obs_stride);
    const size_t o_obs_lin1 = scratch(sizeof(double) * kObsLin * D.obs_stride);
    const size_t o_obs_cost0 = scratch(sizeof(double) * D.n_obs), o_obs_cost1 = scratch(sizeof(double) * D.n_obs);
    const size_t o_grp_red = scratch(sizeof(double) * kGrpRed * std::max<size_t>(1, B.lmg_begin.size()));
    const size_t o_lmvb = upl(B.lm_visit_begin), o_vpose = upl(B.visit_pose), o_vob = upl(B.visit_obs_begin),
                 o_vlm = upl(B.visit_lm), o_lmg_b = upl(B.lmg_begin), o_lmg_info = upl(B.lmg_info);
    const size_t o_lmV = scratch(sizeof(double) * 6 * D.n_lm), o_lmg = scratch(sizeof(double) * 3 * D.n_lm),
                 o_lmVi = scratch(sizeof(double) * 9 * D.n_lm), o_lmz = scratch(sizeof(double) * 3 * D.n_lm);
    D.n_seg = (int)B.seg_pose.size();
    const size_t o_seg_gb = upl(B.seg_gbegin), o_seg_pose = upl(B.seg_pose), o_seg_rg = upl(B.seg_range),
                 o_vslot = upl(B.visit_slot);
    D.n_part = (int)B.part_cbegin.size() - 1;
    const size_t o_pgb = upl(B.part_gbegin), o_pcb2 = upl(B.part_cbegin), o_pcon = upl(B.part_contrib),
                 o_partS = scratch(sizeof(double) * 36 * std::max(1, D.n_part));
    const size_t o_shg = scratch(sizeof(double) * kSegHG * D.n_seg), o_suz = scratch(sizeof(double) * kSegUz * D.n_seg);
    D.n_xvisit = (int)B.xvisit_pose.size();
    D.n_pe = (int)B.pe_pose.size();
    const size_t o_cpose = upl(B.cam_pose), o_xvp = upl(B.xvisit_pose), o_xvl = upl(B.xvisit_lm),
                 o_xvob = upl(B.xvisit_obs_begin), o_xvo = upl(B.xvisit_obs), o_xvs = upl(B.xvisit_slot),
                 o_lmgx = upl(B.lmg_xbegin), o_pep = upl(B.pe_pose), o_pee = upl(B.pe_ext), o_peob = upl(B.pe_obs_begin),
                 o_peo = upl(B.pe_obs), o_peH = scratch(sizeof(double) * 36 * std::max(1, D.n_pe));
    const size_t o_imu_blocks = upl(B.imu_blocks), o_imu_win = upl(B.imu_win), o_imu_flags = upl(B.imu_flags),
                 o_imu_t0 = upl(B.imu_t0), o_imu_t1 = upl(B.imu_t1), o_imu_sb = upl(B.imu_sbegin),
                 o_imu_ts = upl(B.imu_ts), o_imu_ga = upl(B.imu_ga), o_imu_par = upl(B.imu_par),
                 o_imu_state = upl(B.imu_state);
    const size_t o_imu_lin0 = scratch(sizeof(double) * kImuLin * D.n_fac),
                 o_imu_lin1 = scratch(sizeof(double) * kImuLin * D.n_fac);
    const size_t o_imu_cost0 = scratch(sizeof(double) * D.n_fac), o_imu_cost1 = scratch(sizeof(double) * D.n_fac),
                 o_imu_jv = scratch(sizeof(double) * 3 * D.n_fac),
                 o_imu_H = scratch(sizeof(double) * kImuHess * D.n_fac);
    const size_t o_whr = upl(B.win_host_range), o_host_in = scratch(sizeof(double) * kHostIn * D.n_host),
                 o_host_out = scratch(sizeof(double) * kHostOut * D.n_host);
    const size_t o_pp_block = upl(B.pp_block), o_pp_win = upl(B.pp_win), o_pp_meas = upl(B.pp_meas),
                 o_pp_L = upl(B.pp_L);
    const size_t o_pp_lin0 = scratch(sizeof(double) * 42 * D.n_pprior), o_pp_lin1 = scratch(sizeof(double) * 42 * D.n_pprior),
                 o_pp_cost0 = scratch(sizeof(double) * D.n_pprior), o_pp_cost1 = scratch(sizeof(double) * D.n_pprior),
                 o_pp_jv = scratch(sizeof(double) * 3 * D.n_pprior);
    const size_t o_sbp_block = upl(B.sbp_block), o_sbp_win = upl(B.sbp_win), o_sbp_meas = upl(B.sbp_meas),
                 o_sbp_L = upl(B.sbp_L);
    const size_t o_sbp_lin0 = scratch(sizeof(double) * 90 * D.n_sbprior),
                 o_sbp_lin1 = scratch(sizeof(double) * 90 * D.n_sbprior),
                 o_sbp_cost0 = scratch(sizeof(double) * D.n_sbprior), o_sbp_cost1 = scratch(sizeof(double) * D.n_sbprior),
                 o_sbp_jv = scratch(sizeof(double) * 3 * D.n_sbprior);
    const size_t o_rp_blocks = upl(B.rp_blocks), o_rp_win = upl(B.rp_win), o_rp_flags = upl(B.rp_flags),
                 o_rp_kind = upl(B.rp_kind),
                 o_rp_dx = upl(B.rp_dx), o_rp_J = upl(B.rp_J), o_rp_lp = upl(B.rp_lp);
    const size_t o_rp_lin0 = scratch(sizeof(double) * kRelPoseLin * D.n_relpose),
                 o_rp_lin1 = scratch(sizeof(double) * kRelPoseLin * D.n_relpose),
                 o_rp_cost0 = scratch(sizeof(double) * D.n_relpose), o_rp_cost1 = scratch(sizeof(double) * D.n_relpose),
                 o_rp_jv = scratch(sizeof(double) * 3 * D.n_relpose), o_wrpr = upl(B.win_rp_range);
    const size_t o_wfoff = upl(B.win_foff), o_wfdim = upl(B.win_fdim), o_wfpad = upl(B.win_fpad),
                 o_wsoff = upl(B.win_soff), o_wlinv = upl(B.win_linvoff), o_wfwd = upl(B.win_fwdoff), o_wpr = upl(B.win_pose_range), o_wsr = upl(B.win_sb_range),
                 o_wlr = upl(B.win_lm_range), o_wlgr = upl(B.win_lmg_range), o_wor = upl(B.win_obs_range), o_wir = upl(B.win_imu_range),
                 o_wppr = upl(B.win_pp_range), o_wsbpr = upl(B.win_sbp_range);
    const size_t o_fbw = upl(B.fb_win), o_fbk = upl(B.fb_kind), o_fbi = upl(B.fb_index), o_fbo = upl(B.fb_off),
                 o_fbcb = upl(B.fb_cbegin), o_fbc = upl(B.fb_contrib);
    const size_t o_pw = upl(B.pair_win), o_pfi = upl(B.pair_fi), o_pfj = upl(B.pair_fj), o_pcb = upl(B.pair_cbegin),
                 o_pc = upl(B.pair_contrib);
    const size_t o_pruns = upl(B.pair_runs);
    const size_t o_tnz = upl(B.tile_nz), o_tnzoff = upl(B.win_tnzoff), o_tfu = upl(B.tile_fu);
    const size_t o_app = upl(B.asm_pp_items), o_asb = upl(B.asm_sb_items), o_appl = upl(B.asm_ppl_items);
    const size_t o_ti = upl(B.tile_items);
    const size_t o_cri = upl(B.chol_root_items), o_cui = upl(B.chol_upd_items), o_cub = upl(B.chol_upd_begin);
    const size_t o_wsgap = upl(B.win_sgap), o_wbsp = upl(B.win_bsplit), o_wdef = upl(B.win_defoff);
    const size_t nf = std::max(1, B.f_total), nl3 = std::max<size_t>(1, (size_t)3 * D.n_lm);
    const size_t o_S = scratch(sizeof(double) * std::max<int64_t>(1, B.s_total));
    const size_t o_W = scratch(sizeof(double) * std::max<int64_t>(1, B.s_total));
    const size_t o_Linv = scratch(sizeof(double) * std::max<int64_t>(1, B.linv_total));
    const size_t o_fwd = scratch(sizeof(double) * std::max<int64_t>(1, B.fwd_total));
    const size_t o_defer = scratch(sizeof(double) * std::max<int64_t>(1, B.defer_total));
    size_t of[10], ol[7];
    for (int i = 0; i < 10; ++i) of[i] = scratch(sizeof(double) * nf);
    for (int i = 0; i < 7; ++i) ol[i] = scratch(sizeof(double) * nl3);
    const size_t o_st = scratch(sizeof(WinState) * D.n_win);
    const size_t o_self = scratch(sizeof(DevProblem));
    // ---- allocate (reusing the arena while the batch fits) + upload
    const size_t upSize = (A.size + 255) & ~size_t(255);
    const size_t total = upSize + AS.size;
    if (!arena || total > arenaCap) {
      if (arena) {
        HIPCHK(hipFree(arena));
        arena = nullptr;
        arenaCap = 0;
      }
      HIPCHK(hipMalloc(&arena, total));
      arenaCap = total;
    }
    arenaBytes = total;
    char* base = static_cast<char*>(arena);
    if (A.size > hostStageBytes) {
      if (hostStage) HIPCHK(hipHostFree(hostStage));
      hostStage = nullptr;
      hostStageBytes = 0;
      HIPCHK(hipHostMalloc(&hostStage, A.size, hipHostMallocDefault));
      hostStageBytes = A.size;
    }
    HIPCHK(hipStreamSynchronize(stream));  // the staging buffer is free (previous upload done)
    const auto tb2 = std::chrono::steady_clock::now();
    for (const Up& u : ups)
      if (u.bytes) std::memcpy(static_cast<char*>(hostStage) + u.off, u.src, u.bytes);
    const auto tb3 = std::chrono::steady_clock::now();
    if (timing) {
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      std::fprintf(stderr, "okvisgpu build: analyse %.3f ms, layout+alloc %.3f ms, stage %.3f ms (%zu B)\n", ms(tb0, tb1),
                   ms(tb1, tb2), ms(tb2, tb3), A.size);
    }
    if (A.size) HIPCHK(hipMemcpyAsync(base, hostStage, A.size, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemsetAsync(base + upSize, 0, AS.size, stream));
    sNeedsInit = true;
    auto place = [&](size_t off) { return (off & kScratchTag) ? upSize + (off & ~kScratchTag) : off; };
    auto dp = [&](size_t off) { return reinterpret_cast<double*>(base + place(off)); };
    auto ip = [&](size_t off) { return reinterpret_cast<int32_t*>(base + place(off)); };
    auto lp = [&](size_t off) { return reinterpret_cast<int64_t*>(base + place(off)); };
    auto up = [&](size_t off) { return reinterpret_cast<uint8_t*>(base + place(off)); };
    D.pose[0] = dp(o_pose0); D.pose[1] = dp(o_pose1); D.sb[0] = dp(o_sb0); D.sb[1] = dp(o_sb1);
    D.lm[0] = dp(o_lm0); D.lm[1] = dp(o_lm1); D.extr = dp(o_extr); D.cam = dp(o_cam);
    D.pose_win = ip(o_pose_win); D.sb_win = ip(o_sb_win); D.lm_win = ip(o_lm_win);
    D.pose_f = ip(o_pose_f); D.sb_f = ip(o_sb_f); D.lm_free = up(o_lm_free);
    D.pose_active = up(o_pose_act); D.sb_active = up(o_sb_act);
    D.obs_pose = ip(o_obs_pose); D.obs_lm = ip(o_obs_lm); D.obs_cam = ip(o_obs_cam); D.obs_win = ip(o_obs_win);
    D.obs_flags = up(o_obs_flags); D.obs_kp = dp(o_obs_kp); D.obs_L = dp(o_obs_L);
    D.obs_Ls = dp(o_obs_Ls); D.obs_iso = B.obs_iso;
    D.obs_lin[0] = dp(o_obs_lin0); D.obs_lin[1] = dp(o_obs_lin1);
    D.obs_cost[0] = dp(o_obs_cost0); D.obs_cost[1] = dp(o_obs_cost1); D.grp_red = dp(o_grp_red);
    D.lm_visit_begin = ip(o_lmvb); D.visit_pose = ip(o_vpose); D.visit_obs_begin = ip(o_vob); D.visit_lm = ip(o_vlm);
    D.lm_V = dp(o_lmV); D.lm_g = dp(o_lmg); D.lm_Linv = dp(o_lmVi); D.lm_zz = dp(o_lmz);
    D.part_gbegin = ip(o_pgb); D.part_cbegin = ip(o_pcb2); D.part_contrib = ip(o_pcon); D.part_S = dp(o_partS);
    D.seg_hg = dp(o_shg); D.seg_uz = dp(o_suz);
    D.seg_gbegin = ip(o_seg_gb); D.seg_pose = ip(o_seg_pose); D.seg_range = ip(o_seg_rg); D.visit_slot = ip(o_vslot);
    D.cam_pose = ip(o_cpose);
    D.xvisit_pose = ip(o_xvp); D.xvisit_lm = ip(o_xvl); D.xvisit_obs_begin = ip(o_xvob); D.xvisit_obs = ip(o_xvo);
    D.xvisit_slot = ip(o_xvs); D.lmg_xbegin = ip(o_lmgx);
    D.pe_pose = ip(o_pep); D.pe_ext = ip(o_pee); D.pe_obs_begin = ip(o_peob); D.pe_obs = ip(o_peo); D.pe_H = dp(o_peH);
    D.lmg_info = ip(o_lmg_info);
    D.lmg_begin = ip(o_lmg_b); D.n_lmg = B.lmg_begin.empty() ? 0 : (int)B.lmg_begin.size() - 1;
    D.imu_blocks = ip(o_imu_blocks); D.imu_win = ip(o_imu_win); D.imu_flags = up(o_imu_flags);
    D.imu_t0 = lp(o_imu_t0); D.imu_t1 = lp(o_imu_t1); D.imu_sbegin = ip(o_imu_sb); D.imu_ts = lp(o_imu_ts);
    D.imu_ga = dp(o_imu_ga); D.imu_par = dp(o_imu_par); D.imu_state = dp(o_imu_state);
    D.imu_lin[0] = dp(o_imu_lin0); D.imu_lin[1] = dp(o_imu_lin1);
    D.imu_cost[0] = dp(o_imu_cost0); D.imu_cost[1] = dp(o_imu_cost1); D.imu_jv = dp(o_imu_jv);
    D.imu_H = dp(o_imu_H);
    D.win_host_range = ip(o_whr); D.host_in = dp(o_host_in); D.host_out = dp(o_host_out);
    D.pp_block = ip(o_pp_block); D.pp_win = ip(o_pp_win); D.pp_meas = dp(o_pp_meas); D.pp_L = dp(o_pp_L);
    D.pp_lin[0] = dp(o_pp_lin0); D.pp_lin[1] = dp(o_pp_lin1); D.pp_cost[0] = dp(o_pp_cost0);
    D.pp_cost[1] = dp(o_pp_cost1); D.pp_jv = dp(o_pp_jv);
    D.sbp_block = ip(o_sbp_block); D.sbp_win = ip(o_sbp_win); D.sbp_meas = dp(o_sbp_meas); D.sbp_L = dp(o_sbp_L);
    D.sbp_lin[0] = dp(o_sbp_lin0); D.sbp_lin[1] = dp(o_sbp_lin1); D.sbp_cost[0] = dp(o_sbp_cost0);
    D.sbp_cost[1] = dp(o_sbp_cost1); D.sbp_jv = dp(o_sbp_jv);
    D.win_foff = ip(o_wfoff); D.win_fdim = ip(o_wfdim); D.win_fpad = ip(o_wfpad); D.win_soff = lp(o_wsoff);
    D.win_pose_range = ip(o_wpr); D.win_sb_range = ip(o_wsr); D.win_lm_range = ip(o_wlr); D.win_lmg_range = ip(o_wlgr);
    D.win_obs_range = ip(o_wor); D.win_imu_range = ip(o_wir); D.win_pp_range = ip(o_wppr);
    D.win_sbp_range = ip(o_wsbpr);
    D.win_rp_range = ip(o_wrpr);
    D.rp_blocks = ip(o_rp_blocks); D.rp_win = ip(o_rp_win); D.rp_flags = up(o_rp_flags); D.rp_kind = up(o_rp_kind);
    D.rp_dx = dp(o_rp_dx); D.rp_J = dp(o_rp_J); D.rp_lp = dp(o_rp_lp);
    D.rp_lin[0] = dp(o_rp_lin0); D.rp_lin[1] = dp(o_rp_lin1);
    D.rp_cost[0] = dp(o_rp_cost0); D.rp_cost[1] = dp(o_rp_cost1); D.rp_jv = dp(o_rp_jv);
    D.fb_win = ip(o_fbw); D.fb_kind = ip(o_fbk); D.fb_index = ip(o_fbi); D.fb_off = ip(o_fbo);
    D.fb_cbegin = ip(o_fbcb); D.fb_contrib = reinterpret_cast<const Contrib*>(base + place(o_fbc));
    D.pair_win = ip(o_pw); D.pair_fi = ip(o_pfi); D.pair_fj = ip(o_pfj); D.pair_cbegin = ip(o_pcb);
    D.pair_contrib = reinterpret_cast<const Contrib*>(base + place(o_pc));
    D.pair_runs = ip(o_pruns);
    D.tile_nz = reinterpret_cast<const uint8_t*>(base + place(o_tnz));
    D.tile_fu = reinterpret_cast<const int16_t*>(base + place(o_tfu));
    D.win_tnzoff = reinterpret_cast<const int64_t*>(base + place(o_tnzoff));
    D.chol_root_items = ip(o_cri);
    D.n_chol_roots = (int)B.chol_root_items.size() / 3;
    D.n_chol_launches = B.n_chol_launches;
    D.chol_upd_items = ip(o_cui); D.chol_upd_begin = ip(o_cub);
    D.h_upd_begin = B.chol_upd_begin.data();
    D.win_sgap = ip(o_wsgap);
    D.win_bsplit = ip(o_wbsp);
    D.chol_schedule = 1;
    D.asm_pp_items = ip(o_app); D.asm_sb_items = ip(o_asb);
    D.n_asm_pp = (int)B.asm_pp_items.size(); D.n_asm_sb = (int)B.asm_sb_items.size();
    D.asm_ppl_items = ip(o_appl); D.n_asm_ppl = (int)B.asm_ppl_items.size();
    D.tile_items = ip(o_ti);
    D.n_tiles = (int)(B.tile_items.size() / 3);
    D.S = dp(o_S);
    D.W = dp(o_W);
    D.Linv = dp(o_Linv);
    D.win_linvoff = lp(o_wlinv);
    D.fwdF = dp(o_fwd);
    D.chol_defer = dp(o_defer);
    D.win_defoff = lp(o_wdef);
    D.win_fwdoff = lp(o_wfwd);
    double** fv[10] = {&D.sF, &D.diagF, &D.hdF, &D.gF, &D.rhsF, &D.yF, &D.gnF, &D.dgF, &D.vF, &D.stepF};
    for (int i = 0; i < 10; ++i) *fv[i] = dp(of[i]);
    double** lv[7] = {&D.sL, &D.diagL, &D.stepL, &D.yL, &D.gnL, &D.dgL, &D.vL};
    for (int i = 0; i < 7; ++i) *lv[i] = dp(ol[i]);
    D.gL = D.lm_g;  // the landmark gradient is the accumulated J_l^T r
    D.st = reinterpret_cast<WinState*>(base + place(o_st));
    D.self = reinterpret_cast<const DevProblem*>(base + place(o_self));
    HIPCHK(hipStreamSynchronize(stream));
    uploadDescriptor();
    ensureHostBuffers();
    haveProblem = true;
    structureDirty = false;
  }

  // Kernels read the descriptor through one pointer to device memory (a 1.3 KB by-value kernarg is
  // re-fetched field by field on every dependent access).
  void uploadDescriptor() {
    HIPCHK(hipMemcpyAsync(const_cast<DevProblem*>(P.self), &P, sizeof(DevProblem), hipMemcpyHostToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }

  void setOptions(const okvisgpu_options& o) {
    DevOptions& d = P.opt;
    d.max_num_iterations = o.max_num_iterations;
    d.jacobi_scaling = o.jacobi_scaling;
    d.max_num_consecutive_invalid_steps = o.max_num_consecutive_invalid_steps;
    d.redo_propagation_always = o.redo_propagation_always;
    d.function_tolerance = o.function_tolerance;
    d.gradient_tolerance = o.gradient_tolerance;
    d.parameter_tolerance = o.parameter_tolerance;
    d.initial_radius = o.initial_trust_region_radius;
    d.max_radius = o.max_trust_region_radius;
    d.min_radius = o.min_trust_region_radius;
    d.min_relative_decrease = o.min_relative_decrease;
    d.min_lm_diagonal = o.min_lm_diagonal;
    d.max_lm_diagonal = o.max_lm_diagonal;
    // Cholesky schedule (measured on MI355X, S50 windows, bench window-it/s, round 4 with the
    // nested-dissection order (nd) below one window per CU: 64 windows: schedule 1 65.2k, 2 (nd)
    // 72.2k; 128: 1 103.6k, 3 (nd) 107.9k, 2 (nd) 98.2k; 256: 1 159.7k, 3 (nd) 152.8k; 512: 1
    // 186.5k, 3 (nd) 166.0k; gpurun_out r04g / r04h nd_probe; round 5, the pipelined two-team
    // kernel (4), gpurun_out r05g: 64: 2 74.1k, 4 67.0k; 128: 3 110.1k, 4 105.7k; 256: 1 161.0k,
    // 4 170.1k; 512: 1 186.7k, 4 178.7k; the split schedule with pipelined parts (5), r05s: 64: 2
    // 73.9k, 3 70.4k, 5 73.7k; 128: 3 109.8k, 5 114.5k; 192: 4 133.6k, 3 127.3k, 5 120.7k; one S50
    // window: 2 2,765, 5 2,336, 3 2,233, 4 1,858 it/s): below half a window per CU the
    // tile-parallel launches spread each window over many CUs; at half a window per CU the split
    // schedule with each part pipelined; up to one window per CU the pipelined kernel (its step is
    // the factor plus one panel and one update); from there one persistent workgroup per window,
    // two per CU. (A wave-specialised kernel and a persistent variant with the panel tiles in LDS were
    // measured slower at every batch size and removed in round 4; a two-window pipelined
    // workgroup, round 5, ran 166.8k against 199.4k at 2,048 windows and was removed.)
    int sched = o.cholesky_schedule >= 1 && o.cholesky_schedule <= 5 ? o.cholesky_schedule : 0;
    if (sched == 0)
      sched = 2 * P.n_win < cuCount ? 2 : (2 * P.n_win <= cuCount && B.any_split ? 5 : (P.n_win <= cuCount ? 4 : 1));
    if (sched == 3 && !B.any_split) sched = 1;  // (no window with a nested-dissection split)
    if (sched == 5 && !B.any_split) sched = 4;
    // the persistent kernel keeps the window's rhs / y in dynamic LDS next to its static tiles:
    // a reduced dimension beyond what fits falls back to the tile-parallel launches
    if (sched == 5 && !(pipeFits() && persistentFits())) sched = 3;
    if (sched == 4 && !pipeFits()) sched = 1;
    if ((sched == 1 || sched == 3) && !persistentFits()) sched = 2;
    if (sched != P.chol_schedule) dropGraph();
    P.chol_schedule = sched;
    uploadDescriptor();
  }

  void resetStates(double mu) {
    std::vector<WinState> s(P.n_win);
    for (auto& x : s) {
      std::memset(&x, 0, sizeof(x));
      x.radius = P.opt.initial_radius;
      x.mu = mu;
      x.need_gn = 1;
      x.z_mu = -1.0;
      x.termination = OKVISGPU_NO_CONVERGENCE;
    }
    HIPCHK(hipMemcpyAsync(P.st, s.data(), sizeof(WinState) * s.size(), hipMemcpyHostToDevice, stream));
  }

  // Pinned staging for the parameter copies: the set_problems staging buffer (it holds both
  // parameter sets and the IMU states, so it is large enough), grown if ever needed.
  char* paramStage(size_t bytes) {
    HIPCHK(hipStreamSynchronize(stream));  // no copy out of / into it is still in flight
    if (bytes > hostStageBytes) {
      if (hostStage) HIPCHK(hipHostFree(hostStage));
      hostStage = nullptr;
      hostStageBytes = 0;
      HIPCHK(hipHostMalloc(&hostStage, bytes, hipHostMallocDefault));
      hostStageBytes = bytes;
    }
    return static_cast<char*>(hostStage);
  }

  // Upload current host parameter values into both parameter sets (+ IMU state): the windows are
  // packed into pinned memory in device order (host threads over windows), set 0 and the IMU
  // states go up in one copy each, and set 1 is a device-side copy of set 0.
  void uploadParams() {
    const size_t np = 7 * (size_t)P.n_pose, ns = 9 * (size_t)P.n_sb, nl = 4 * (size_t)P.n_lm,
                 ni = (size_t)P.n_imu * kImuState;
    double* pose = reinterpret_cast<double*>(paramStage((np + ns + nl + ni) * 8));
    double *sb = pose + np, *lm = sb + ns, *imu = lm + nl;
    forWindows(B.n_win, [&](int w) {
      const okvisgpu_problem* p = probs[w];
      double* q = pose + 7 * (size_t)B.pose_base[w];
      std::memcpy(q, p->poses, sizeof(double) * 7 * p->n_poses);
      std::memcpy(q + 7 * (size_t)p->n_poses, p->extrinsics, sizeof(double) * 7 * p->n_cameras);
      std::memcpy(sb + 9 * (size_t)B.sb_base[w], p->speed_biases, sizeof(double) * 9 * p->n_speed_biases);
      double* l = lm + 4 * (size_t)B.lm_base[w];
      const int* perm = &B.lm_perm[B.lm_base[w]];
      for (int k = 0; k < p->n_landmarks; ++k) std::memcpy(l + 4 * (size_t)k, &p->landmarks[4 * (size_t)perm[k]], 32);
      double* f = imu + (size_t)B.imu_base[w] * kImuState;
      if (p->imu_state) std::memcpy(f, p->imu_state, sizeof(double) * kImuState * p->n_imu);
      else std::memset(f, 0, sizeof(double) * kImuState * p->n_imu);
    });
    if (np) HIPCHK(hipMemcpyAsync(P.pose[0], pose, np * 8, hipMemcpyHostToDevice, stream));
    if (ns) HIPCHK(hipMemcpyAsync(P.sb[0], sb, ns * 8, hipMemcpyHostToDevice, stream));
    if (nl) HIPCHK(hipMemcpyAsync(P.lm[0], lm, nl * 8, hipMemcpyHostToDevice, stream));
    if (ni) HIPCHK(hipMemcpyAsync(P.imu_state, imu, ni * 8, hipMemcpyHostToDevice, stream));
    if (np) HIPCHK(hipMemcpyAsync(P.pose[1], P.pose[0], np * 8, hipMemcpyDeviceToDevice, stream));
    if (ns) HIPCHK(hipMemcpyAsync(P.sb[1], P.sb[0], ns * 8, hipMemcpyDeviceToDevice, stream));
    if (nl) HIPCHK(hipMemcpyAsync(P.lm[1], P.lm[0], nl * 8, hipMemcpyDeviceToDevice, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }

  // Write device results back into the caller's arrays: k_select_current gathers every window's
  // current parameter set into set 0 (WinState::xcur on the device), then one copy per array into
  // pinned memory and a threaded scatter into the windows' arrays.
  void downloadParams() {
    const size_t np = 7 * (size_t)P.n_pose, ns = 9 * (size_t)P.n_sb, nl = 4 * (size_t)P.n_lm,
                 ni = (size_t)P.n_imu * kImuState;
    double* pose = reinterpret_cast<double*>(paramStage((np + ns + nl + ni) * 8));
    double *sb = pose + np, *lm = sb + ns, *imu = lm + nl;
    launch_select_current(P, stream);
    HIPCHK(hipGetLastError());
    if (np) HIPCHK(hipMemcpyAsync(pose, P.pose[0], np * 8, hipMemcpyDeviceToHost, stream));
    if (ns) HIPCHK(hipMemcpyAsync(sb, P.sb[0], ns * 8, hipMemcpyDeviceToHost, stream));
    if (nl) HIPCHK(hipMemcpyAsync(lm, P.lm[0], nl * 8, hipMemcpyDeviceToHost, stream));
    if (ni) HIPCHK(hipMemcpyAsync(imu, P.imu_state, ni * 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    forWindows(B.n_win, [&](int w) {
      const okvisgpu_problem* p = probs[w];
      const double* q = pose + 7 * (size_t)B.pose_base[w];
      std::memcpy(p->poses, q, sizeof(double) * 7 * p->n_poses);
      if (B.win_ext_free[w])  // variable extrinsics are written back like every other block
        std::memcpy(p->extrinsics, q + 7 * (size_t)p->n_poses, sizeof(double) * 7 * p->n_cameras);
      std::memcpy(p->speed_biases, sb + 9 * (size_t)B.sb_base[w], sizeof(double) * 9 * p->n_speed_biases);
      const double* l = lm + 4 * (size_t)B.lm_base[w];
      const int* perm = &B.lm_perm[B.lm_base[w]];
      for (int k = 0; k < p->n_landmarks; ++k) std::memcpy(&p->landmarks[4 * (size_t)perm[k]], l + 4 * (size_t)k, 32);
      if (p->imu_state && p->n_imu)
        std::memcpy(p->imu_state, imu + (size_t)B.imu_base[w] * kImuState, sizeof(double) * kImuState * p->n_imu);
    });
  }

  std::vector<WinState> readStates() {
    std::vector<WinState> s(P.n_win);
    HIPCHK(hipMemcpyAsync(s.data(), P.st, sizeof(WinState) * s.size(), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return s;
  }

  void launchInit(int evalMode) {
    evalAll(evalMode, stream);
    launch_reduce(P, R_COST_INIT, stream);
    launch_linearization_blocks(P, 0, stream);
    launch_gradnorm(P, 0, stream);
    if (lin_runs_prep(P)) launch_lm_prep(P, stream);  // (the first iteration's; later ones: k_lin_few)
    HIPCHK(hipGetLastError());
  }

  // One iteration. Few windows (a latency chain of small launches): the gradient test of an
  // iteration runs inside the next iteration's assembly launch (k_assemble_few; it reads nothing the
  // assembly writes, and a window it ends is skipped from the Cholesky on), and the captured
  // graph ends with one standalone test (graphTail), so that every graph launch leaves complete
  // window states. The test is idempotent (the same state gives the same norms and decision), so
  // the repeat at the start of the next graph launch is harmless.
  bool fusedGradnorm() const { return fewWindows(P.n_win, P.cu_count); }
  void launchIteration() {
    if (!lin_runs_prep(P)) launch_lm_prep(P, stream);
    if (fusedGradnorm()) launch_assemble_gradnorm_few(P, stream);
    else launch_assemble(P, stream);
    launch_cholesky(P, stream);
    launch_gn_backsub(P, stream);  // (with the factors' J*v)
    launch_dogleg(P, stream);
    evalAll(1, stream);
    launch_reduce(P, R_COST_CAND, stream);
    launch_linearization_blocks(P, 1, stream);
    if (!fusedGradnorm()) launch_gradnorm(P, 1, stream);
  }
  void graphTail(bool serial) {
    if (serial && fusedGradnorm()) launch_gradnorm(P, 1, stream);
  }

  // The captured iteration with the independent kernels of a phase on fork streams, so the graph
  // runs them concurrently (the latency of a single window is a chain of small kernels); the data
  // they touch is disjoint (eval: obs / IMU / prior records; linearisation: landmark groups / IMU
  // Hessians; J*v: reprojection rows / factor rows; S tiles zeroed vs. landmark-group records;
  // pose-pose vs. speed/bias blocks of S).
  void launchIterationForked() {
    size_t& ne = forkEvUsed;  // (distinct events for every fork / join of one capture)
    auto ev = [&]() {
      if (ne == forkEv.size()) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        forkEv.push_back(e);
      }
      return forkEv[ne++];
    };
    auto fork = [&](hipStream_t to) {
      hipEvent_t e = ev();
      HIPCHK(hipEventRecord(e, stream));
      HIPCHK(hipStreamWaitEvent(to, e, 0));
    };
    auto join = [&](hipStream_t from) {
      hipEvent_t e = ev();
      HIPCHK(hipEventRecord(e, from));
      HIPCHK(hipStreamWaitEvent(stream, e, 0));
    };
    // Gauss-Newton system: the stale Z rebuilt (few windows after the first iteration), then the
    // assembly kernels and the clearing of the tile entries they do not write, on four streams
    // (disjoint entries of S)
    launch_lm_prep(P, stream);
    fork(side[0]);
    launch_assemble_sb(P, side[0]);
    launch_assemble_pp(P, stream);
    join(side[0]);
    launch_cholesky(P, stream);  // (with the f-blocks' GN vectors, formerly k_gn_finalize)
    launch_lm_backsub(P, stream);  // (with the factors' J*v)
    launch_dogleg(P, stream);
    // candidate evaluation
    fork(side[0]);
    fork(side[1]);
    launch_eval_imu(P, 1, side[0]);
    launch_eval_priors(P, 1, side[1]);
    evalHost(1, side[1]);
    launch_eval_obs(P, 1, stream);
    join(side[0]);
    join(side[1]);
    launch_reduce(P, R_COST_CAND, stream);
    // linearisation at the accepted point
    fork(side[0]);
    launch_imu_hess(P, 1, side[0]);
    launch_lm_blocks(P, 1, stream);
    join(side[0]);
    launch_fgrad(P, 1, stream);
    launch_gradnorm(P, 1, stream);
  }

  void ensureGraph() {
    if (iterGraph) return;
    hipGraph_t g;
    HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    // Few windows: one stream (a cross-stream edge of the graph costs ~10 us, more than the
    // overlap of a single window's small kernels gains: S50 1488 -> 1614 it/s); a full batch
    // keeps the fork streams (2,048 S50 windows: 135.7k -> 138.5k window-it/s). Env override
    // OKVISGPU_SERIAL_GRAPH=0|1 (measurements).
    const char* ser = std::getenv("OKVISGPU_SERIAL_GRAPH");
    const bool serial = ser && (ser[0] == '0' || ser[0] == '1') ? ser[0] == '1' : P.n_win < cuCount;
    forkEvUsed = 0;
    if (serial) launchIteration();
    else launchIterationForked();
    graphTail(serial);
    HIPCHK(hipStreamEndCapture(stream, &g));
    HIPCHK(hipGraphInstantiate(&iterGraph, g, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(g));
    // Env override OKVISGPU_GRAPH_ITERS=<K> (measurements; 1 = single-iteration graph only).
    const char* gi = std::getenv("OKVISGPU_GRAPH_ITERS");
    const int K = gi && *gi ? std::max(1, std::min(std::atoi(gi), 64)) : kGraphIters;
    if (K > 1) {
      HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
      forkEvUsed = 0;
      for (int k = 0; k < K; ++k) {
        if (serial) launchIteration();
        else launchIterationForked();
      }
      graphTail(serial);
      HIPCHK(hipStreamEndCapture(stream, &g));
      HIPCHK(hipGraphInstantiate(&iterGraphK, g, nullptr, nullptr, 0));
      HIPCHK(hipGraphDestroy(g));
      graphIters = K;
    }
  }
};

namespace {

thread_local std::string g_err;

int fail(okvisgpu_ctx* c, int code, const std::string& m) {
  if (c) c->last_error = m;
  g_err = m;
  return code;
}

template <class F>
int guarded(okvisgpu_ctx* c, F f) {
  try {
    return f();
  } catch (const HipError& e) {
    return fail(c, e.code, e.msg);
  } catch (const ArgError& e) {
    return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, e.msg);
  } catch (const UnsupportedError& e) {
    return fail(c, OKVISGPU_ERR_UNSUPPORTED, e.msg);
  } catch (const std::bad_alloc&) {
    return fail(c, OKVISGPU_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(c, OKVISGPU_ERR_DEVICE, e.what());
  }
}

}  // namespace

extern "C" {

int okvisgpu_abi_version(void) { return OKVISGPU_ABI_VERSION; }

int okvisgpu_loss_evaluate(const okvisgpu_loss* loss, double s, double* rho) {
  if (!loss || !rho || !lossValid(*loss)) return fail(nullptr, OKVISGPU_ERR_INVALID_ARGUMENT, "loss_evaluate: bad loss");
  lossRho(*loss, s, rho);
  return OKVISGPU_OK;
}

void okvisgpu_default_options(okvisgpu_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->max_num_iterations = 50;  // ::ceres::Solver::Options default
  o->linear_solver = OKVISGPU_DENSE_SCHUR;
  o->trust_region_strategy = OKVISGPU_DOGLEG;
  o->jacobi_scaling = 1;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_relative_decrease = 1e-3;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->max_num_consecutive_invalid_steps = 5;
  o->time_limit_s = -1.0;
  o->min_iterations = 0;
  o->redo_propagation_always = 0;
  o->num_threads = 1;
  o->verbose = 0;
  o->cholesky_schedule = 0;
}

int okvisgpu_device_count(int32_t* count) {
  if (!count) return OKVISGPU_ERR_INVALID_ARGUMENT;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return OKVISGPU_OK;
}

int okvisgpu_ctx_create(int32_t device, okvisgpu_ctx** out) {
  if (!out) return OKVISGPU_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(nullptr, OKVISGPU_ERR_DEVICE, "no HIP device");
  if (device < 0 || device >= n) return fail(nullptr, OKVISGPU_ERR_INVALID_ARGUMENT, "bad device index");
  auto* c = new okvisgpu_ctx();
  c->device = device;
  const int rc = guarded(c, [&]() {
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
      throw HipError{std::string("okvisgpu is built for gfx950 only; device is ") + prop.gcnArchName,
                     OKVISGPU_ERR_DEVICE};
    c->cuCount = prop.multiProcessorCount;
    c->ldsPerBlock = prop.sharedMemPerBlock;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (hipStream_t& q : c->side) HIPCHK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
    return (int)OKVISGPU_OK;
  });
  if (rc != OKVISGPU_OK) {
    delete c;
    return rc;
  }
  *out = c;
  return OKVISGPU_OK;
}

int okvisgpu_ctx_destroy(okvisgpu_ctx* c) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  (void)hipSetDevice(c->device);
  delete c;
  return OKVISGPU_OK;
}

const char* okvisgpu_last_error(const okvisgpu_ctx* c) { return c ? c->last_error.c_str() : g_err.c_str(); }

int okvisgpu_set_problems(okvisgpu_ctx* c, const okvisgpu_problem* problems, int32_t n) {
  if (!c || !problems || n <= 0) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "set_problems: bad arguments");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    c->probs.clear();
    for (int i = 0; i < n; ++i) c->probs.push_back(&problems[i]);
    c->constOverride.clear();
    c->build();
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_update_params(okvisgpu_ctx* c) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    c->uploadParams();
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_set_block_constant(okvisgpu_ctx* c, int32_t window, int32_t kind, int32_t index, int32_t is_const) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (window < 0 || window >= (int)c->probs.size() || kind < 0 || kind > 3)
    return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "set_block_constant: bad window/kind");
  const okvisgpu_problem* p = c->probs[window];
  const int n = kind == 0 ? p->n_poses : kind == 1 ? p->n_speed_biases : kind == 2 ? p->n_landmarks : p->n_cameras;
  if (index < 0 || index >= n) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "set_block_constant: bad index");
  c->constOverride[std::make_tuple(window, kind, index)] = is_const ? 1 : 0;
  c->structureDirty = true;
  return OKVISGPU_OK;
}

int okvisgpu_get_params(okvisgpu_ctx* c) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    c->downloadParams();
    return (int)OKVISGPU_OK;
  });
}

static int checkSolveOptions(okvisgpu_ctx* c, const okvisgpu_options* o) {
  if (!c || !o) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  // SPARSE_NORMAL_CHOLESKY (the full graph's option, ViGraph.cpp:248) solves the same normal
  // equations; the step is formed through the exact tile-sparse Schur complement either way
  if ((o->linear_solver != OKVISGPU_DENSE_SCHUR && o->linear_solver != OKVISGPU_SPARSE_NORMAL_CHOLESKY) ||
      o->trust_region_strategy != OKVISGPU_DOGLEG)
    return fail(c, OKVISGPU_ERR_UNSUPPORTED,
                "linear solver must be DENSE_SCHUR or SPARSE_NORMAL_CHOLESKY and the strategy DOGLEG");
  if (o->max_num_iterations < 0) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "max_num_iterations < 0");
  return OKVISGPU_OK;
}

int okvisgpu_solve_begin(okvisgpu_ctx* c, const okvisgpu_options* o) {
  const int rc = checkSolveOptions(c, o);
  if (rc != OKVISGPU_OK) return rc;
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    c->solveT0 = nowS();
    c->opts = *o;
    c->replays = 0;
    if (c->structureDirty) c->build();  // freeze / unfreeze changed the free set
    c->setOptions(*o);
    c->dropGraph();  // options are baked into the captured kernel arguments
    c->P.lin_prep = -1;  // the GN prep's placement: decided once, used by launchInit and the capture
    c->P.lin_prep = lin_runs_prep(c->P) ? 1 : 0;
    c->uploadParams();
    c->resetStates(1e-8);
    c->ensureS(c->stream);
    c->launchInit(2);
    c->failInitialHostEvaluations();
    c->ensureGraph();
    c->inSolve = true;
    c->phasesTimed = false;
    for (double& t : c->phaseMs) t = 0.0;
    c->tIterStart = nowS();
    c->tPre = c->tIterStart - c->solveT0;
    c->tMin = c->tPost = 0.0;
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_solve_iterate(okvisgpu_ctx* c, int32_t n) {
  if (!c || n < 0) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->inSolve) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "solve_iterate without solve_begin");
  return guarded(c, [&]() {
    c->launchIterations(n);
    c->replays += n;
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_synchronize(okvisgpu_ctx* c) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  return guarded(c, [&]() {
    HIPCHK(hipStreamSynchronize(c->stream));
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_solve_end(okvisgpu_ctx* c, okvisgpu_summary* sums) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->inSolve) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "solve_end without solve_begin");
  return guarded(c, [&]() {
    const okvisgpu_options& o = c->opts;
    const int maxReplays = std::max(1, o.max_num_iterations) * 8 + 8;
    std::vector<WinState> st = c->readStates();
    // windows that consumed passes on mu-retries (ComputeGaussNewtonStep loop) finish here
    while (c->replays < maxReplays) {
      bool allDone = true;
      for (auto& s : st) allDone = allDone && s.done;
      if (allDone) break;
      HIPCHK(hipGraphLaunch(c->iterGraph, c->stream));
      ++c->replays;
      st = c->readStates();
    }
    c->finish(st, sums);
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_solve(okvisgpu_ctx* c, const okvisgpu_options* o, okvisgpu_summary* sums) {
  int rc = okvisgpu_solve_begin(c, o);
  if (rc != OKVISGPU_OK) return rc;
  if (o->time_limit_s < 0.0 && !o->verbose) {
    rc = okvisgpu_solve_iterate(c, o->max_num_iterations);
    if (rc != OKVISGPU_OK) return rc;
    return okvisgpu_solve_end(c, sums);
  }
  // One iteration at a time (states read back after each): CeresIterationCallback
  // (CeresIterationCallback.cpp:30-38): after the minimum number of iterations, stop once the next
  // iteration would exceed the time budget; verbose: eager iterations timed per phase (the Ceres
  // Summary timing fields, FullReport at ViGraph.cpp:1887-1889).
  return guarded(c, [&]() {
    c->phasesTimed = o->verbose != 0;
    std::vector<WinState> st = c->readStates();
    double iterStart = nowS();
    const int maxReplays = std::max(1, o->max_num_iterations) * 8 + 8;
    while (c->replays < maxReplays) {
      bool allDone = true;
      for (auto& s : st) allDone = allDone && s.done;
      if (allDone) break;
      const double now = nowS();
      const double iterTime = now - iterStart, cum = now - c->solveT0;
      bool changed = false;
      for (auto& s : st)
        if (o->time_limit_s >= 0.0 && !s.done && s.iteration >= o->min_iterations && cum + iterTime > o->time_limit_s) {
          s.done = 1;
          s.termination = OKVISGPU_USER_SUCCESS;
          changed = true;
        }
      if (changed) {
        HIPCHK(hipMemcpyAsync(c->P.st, st.data(), sizeof(WinState) * st.size(), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        continue;
      }
      iterStart = nowS();
      if (o->verbose) c->profiledIteration(c->phaseMs);
      else HIPCHK(hipGraphLaunch(c->iterGraph, c->stream));
      ++c->replays;
      st = c->readStates();
    }
    c->finish(st, sums);
    return (int)OKVISGPU_OK;
  });
}

static const char* kPhaseNames[OKVISGPU_N_PHASES] = {
    "lm_prep",     "zero_S",   "assemble",   "cholesky",  "lm_backsub", "gn_finalize",
    "jv",          "reduce_jv", "dogleg",   "eval_obs",
    "eval_imu",    "eval_priors", "reduce_cand", "lin_blocks", "gradnorm"};

const char* okvisgpu_phase_name(int32_t i) { return (i >= 0 && i < OKVISGPU_N_PHASES) ? kPhaseNames[i] : ""; }

int okvisgpu_profile_iteration(okvisgpu_ctx* c, double* ms) {
  if (!c || !ms) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->inSolve) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "profile_iteration needs solve_begin");
  return guarded(c, [&]() {
    for (int i = 0; i < OKVISGPU_N_PHASES; ++i) ms[i] = 0.0;
    c->profiledIteration(ms);
    c->replays += 1;
    return (int)OKVISGPU_OK;
  });
}

// ---- per-kernel timing with algorithmic work models (bench.py's roofline) ------------------
namespace {
enum KernelId {
  K_ASSEMBLE_PP, K_ASSEMBLE_SB, K_CHOLESKY, K_LM_VISIT, K_LM_VISIT_PREP, K_EVAL_IMU, K_EVAL_OBS, K_JV,
  K_FGRAD, K_LM_BACKSUB, K_COUNT
};
const char* kKernelNames[K_COUNT] = {"k_assemble_pp", "k_assemble_sb", "k_cholesky", "k_lm_visit", "k_lm_visit_prep",
                                     "k_eval_imu",    "k_eval_obs",    "k_jv",       "k_fgrad",
                                     "k_lm_backsub_jv"};
// bound: 0 = HBM bytes, 1 = FP64 matrix-core FLOPs
const int kKernelBound[K_COUNT] = {0, 0, 1, 0, 0, 0, 0, 0, 0, 0};

// Algorithmic work of one iteration's launches of kernel k over the whole batch: compulsory HBM
// bytes (every operand read once, every result written once) or FP64 FLOPs.
double kernelWork(const HostBatch& B, const DevProblem& P, int k) {
  const double d8 = 8.0;
  const double nObs = P.n_obs, nVis = P.n_visit, nLm = P.n_lm, nImu = P.n_imu;
  switch (k) {
    case K_ASSEMBLE_PP: {
      double desc = 0, pairs = 0;
      for (const auto* list : {&B.asm_pp_items, &B.asm_ppl_items})
        for (int it : *list)
          if (it >= 0) { desc += B.pair_cbegin[it + 1] - B.pair_cbegin[it]; pairs += 1; }
      return desc * 16 + (double)P.n_part * 36 * d8 + (double)P.n_seg * (21 + 6) * d8 + pairs * (36 + 12) * d8;
    }
    case K_ASSEMBLE_SB: {
      double desc = 0, entries = 0;
      for (int it : B.asm_sb_items) {
        desc += B.pair_cbegin[it + 1] - B.pair_cbegin[it];
        const int ni = B.fb_kind[B.pair_fi[it]] == 0 ? 6 : 9, nj = B.fb_kind[B.pair_fj[it]] == 0 ? 6 : 9;
        entries += ni * nj;
      }
      return desc * 16 + nImu * kImuLin * d8 + entries * d8;
    }
    case K_CHOLESKY: {
      // algorithmic FLOPs of the tile-sparse LLT and its two triangular solves, per structurally
      // non-zero 64x64 tile (n = 64; VERDICT r05 "Next" 1, SURVEY §8d "LLT d^3/3"):
      //   diagonal potrf n^3/3, panel TRSM n^3, diagonal band update (SYRK) n^2(n+1), off-diagonal
      //   band update (GEMM) 2n^3, forward + backward substitution 2n^2 per diagonal tile and 4n^2
      //   per panel tile. The kernel's own extras (X = L_kk^-1, full 64-column MFMA blocks) are not
      //   counted; the issued-MFMA figure sits beside this in bench.py (frac_issued).
      const double n = 64.0;
      double diag = 0;
      for (int w = 0; w < P.n_win; ++w) diag += B.tileT[w];
      const double panels = (double)B.n_panels, syrk = (double)B.n_band_updates_diag,
                   gemm = (double)(B.n_band_updates - B.n_band_updates_diag);
      return diag * (n * n * n / 3.0 + 2.0 * n * n) + panels * (n * n * n + 4.0 * n * n) +
             syrk * n * n * (n + 1.0) + gemm * 2.0 * n * n * n;
    }
    case K_LM_VISIT:  // obs linearisation + params in; segments, partial blocks, landmark blocks out
      return nObs * (kObsLin * d8 + 1) + nVis * (7 * d8 + 16) + (double)P.n_seg * (27 + 6) * d8 +
             (double)B.part_contrib.size() * 4 + (double)P.n_part * 36 * d8 + nLm * 40 * d8;
    case K_LM_VISIT_PREP:  // W recomputed from the obs linearisation; U z, partial blocks, L^-1 out
      return nObs * (kObsLin * d8 + 1) + nVis * (7 * d8 + 16) + (double)P.n_seg * 6 * d8 +
             (double)B.part_contrib.size() * 4 + (double)P.n_part * 36 * d8 + nLm * 34 * d8;
    case K_EVAL_IMU: return nImu * (2.0 * kImuState + kImuLin + 2 * 16) * d8 + (double)B.imu_ts.size() * 7 * d8;
    case K_EVAL_OBS: return nObs * (16 + (P.obs_iso ? 8 : 32) + 13 + kObsLin * d8 + 8) + nLm * 4 * d8 + (double)B.pose_f.size() * 7 * d8;
    case K_JV:  // factors: IMU linearisation, prior / edge Jacobians in, their J*v forms out
      return nImu * (kImuLin + 3) * d8 + (double)P.n_pprior * (42 + 3) * d8 + (double)P.n_sbprior * (90 + 3) * d8 +
             (double)P.n_relpose * (kRelPoseLin + 3) * d8;
    case K_LM_BACKSUB:  // obs linearisation (A, flags) once; pose / landmark parameters and vectors once per
                        // block; landmark step + dogleg vectors and the visits' J*v forms out
      return nObs * (6 * d8 + 1) + nVis * (3 * d8 + 16) + (double)P.n_pose * (7 + 18) * d8 +
             nLm * (4 + 9 + 3 + 3 + 3 + 3 + 12) * d8;
    case K_FGRAD: return (double)P.n_seg * 27 * d8 + nImu * kImuLin * d8 + (double)B.fb_contrib.size() * 16;
  }
  return 0.0;
}
}  // namespace

int okvisgpu_kernel_count(void) { return K_COUNT; }
const char* okvisgpu_kernel_name(int32_t k) { return (k >= 0 && k < K_COUNT) ? kKernelNames[k] : ""; }

int okvisgpu_time_kernel(okvisgpu_ctx* c, int32_t kernel, int32_t reps, double* avg_ms, double* work,
                         int32_t* bound) {
  if (!c || kernel < 0 || kernel >= K_COUNT || reps < 1) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (c->inSolve) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "time_kernel: call after solve_end");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    const DevProblem& P = c->P;
    hipStream_t s = c->stream;
    // re-arm every window (the linearisation of the finished solve stays resident); the solve
    // state is scratch afterwards and is rebuilt by the next solve_begin
    std::vector<WinState> st = c->readStates();
    for (WinState& w : st) {
      w.done = 0; w.need_gn = 1; w.gn_failed = 0; w.eval_cand = 1; w.accepted = 1; w.step_valid = 2;
      w.z_mu = -1.0;  // stale: the prep mode recomputes Z
    }
    HIPCHK(hipMemcpyAsync(P.st, st.data(), sizeof(WinState) * st.size(), hipMemcpyHostToDevice, s));
    std::vector<hipEvent_t> ev;
    size_t used = 0;
    auto event = [&]() {
      if (used == ev.size()) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        ev.push_back(e);
      }
      HIPCHK(hipEventRecord(ev[used], s));
      return used++;
    };
    std::vector<std::pair<size_t, size_t>> spans;
    auto timed = [&](auto&& launch) {
      const size_t a = event();
      launch();
      const size_t b = event();
      spans.emplace_back(a, b);
    };
    for (int r = 0; r < reps; ++r) {
      switch (kernel) {
        case K_ASSEMBLE_PP: timed([&] { launch_assemble_pp(P, s); }); break;
        case K_ASSEMBLE_SB: timed([&] { launch_assemble_sb(P, s); }); break;
        case K_LM_VISIT: timed([&] { launch_lm_visit(P, 1, s); }); break;
        case K_LM_VISIT_PREP: timed([&] { launch_lm_visit(P, 2, s); }); break;
        case K_EVAL_IMU:
          // redo counter := 0 forces the re-preintegration the candidate evaluations of a solve
          // mostly perform (the device-side IMU state is scratch afterwards)
          if (P.n_imu > 0)
            HIPCHK(hipMemset2DAsync(P.imu_state, sizeof(double) * kImuState, 0, sizeof(double), P.n_imu, s));
          timed([&] { launch_eval_imu_as_solved(P, 1, s); });
          break;
        case K_EVAL_OBS: timed([&] { launch_eval_obs(P, 1, s); }); break;
        case K_JV: timed([&] { launch_jv(P, s); }); break;
        case K_LM_BACKSUB: timed([&] { launch_lm_backsub(P, s); }); break;
        case K_FGRAD: timed([&] { launch_fgrad(P, 1, s); }); break;
        case K_CHOLESKY:  // (the factorisation reads the assembled S and works in W: repeatable)
          c->ensureS(s);
          launch_assemble(P, s);
          timed([&] { launch_cholesky(P, s); });
          break;
      }
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    double tot = 0.0;
    for (auto& sp : spans) {
      float t = 0.f;
      HIPCHK(hipEventElapsedTime(&t, ev[sp.first], ev[sp.second]));
      tot += t;
    }
    for (auto e : ev) (void)hipEventDestroy(e);
    if (avg_ms) *avg_ms = tot / reps;
    if (work) *work = kernelWork(c->B, P, kernel);
    if (bound) *bound = kKernelBound[kernel];
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_get_stats(okvisgpu_ctx* c, okvisgpu_problem_stats* st) {
  if (!c || !st) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  const HostBatch& B = c->B;
  const DevProblem& P = c->P;
  std::memset(st, 0, sizeof(*st));
  st->n_windows = B.n_win;
  st->n_poses = P.n_pose;
  st->n_speed_biases = P.n_sb;
  st->n_landmarks = P.n_lm;
  for (int w = 0; w < B.n_win; ++w) {
    const okvisgpu_problem* p = B.probs[w];
    for (int c = 0; c < p->n_cameras; ++c) st->n_extrinsics_free += B.pose_f[B.pose_base[w] + p->n_poses + c] >= 0;
  }
  for (uint8_t f : B.lm_free) st->n_landmarks_free += f != 0;
  st->n_observations = P.n_obs;
  st->n_visits = P.n_visit;
  st->n_imu = P.n_imu;
  st->n_imu_samples = (int64_t)B.imu_ts.size();
  st->n_pose_priors = P.n_pprior;
  st->n_sb_priors = P.n_sbprior;
  st->n_relpose = P.n_relpose;
  st->cholesky_launches = B.n_chol_launches;
  st->reduced_dim = 0;
  for (int d : B.win_fnat) st->reduced_dim += d;
  st->s_tiles_nonzero = (int64_t)B.tile_items.size() / 3;
  for (int T : B.tileT) st->s_tiles_dense += (int64_t)T * (T + 1) / 2;
  st->n_block_pairs = P.n_pair;
  st->n_visit_segments = P.n_seg;
  st->n_partial_blocks = P.n_part;
  st->arena_bytes = (int64_t)c->arenaBytes;
  st->cholesky_split_windows = 0;
  for (size_t w = 0; w + 1 < c->B.win_bsplit.size(); w += 2) st->cholesky_split_windows += c->B.win_bsplit[w + 1] > 0;
  return OKVISGPU_OK;
}

int okvisgpu_plan_window(const okvisgpu_problem* p, int32_t nested_dissection, int64_t* info, uint8_t* tile_nz,
                         int32_t* step_launch, int32_t* natural) {
  if (!p) return OKVISGPU_ERR_INVALID_ARGUMENT;
  try {
    HostBatch B;
    B.nd = nested_dissection != 0;
#ifdef OKG_ANALYSE_TIMING
    for (double& x : g_atime) x = 0.0;
    g_alast = std::chrono::steady_clock::now();
#endif
    analyse({p}, {}, B);
#ifdef OKG_ANALYSE_TIMING
    std::fprintf(stderr, "analyse ms:");
    for (int i = 0; i < 11; ++i) std::fprintf(stderr, " [%d] %.3f", i, g_atime[i]);
    std::fprintf(stderr, "\n");
#endif
    const int T = B.tileT[0], fpad = B.win_fpad[0];
    const auto& nz = B.tileNz[0];
    std::vector<int> L, last;
    const int nl = cholSchedule(nz, T, L, last);
    if (info) {
      int64_t nnz = 0;
      for (uint8_t v : nz) nnz += v;
      const int64_t v[8] = {B.win_fnat[0], fpad, T, nnz, nl, B.win_bsplit[0], B.win_bsplit[1], B.win_sgap[1]};
      std::copy(v, v + 8, info);
    }
    if (tile_nz) std::copy(nz.begin(), nz.end(), tile_nz);
    if (step_launch)
      for (int k = 0; k < T; ++k) {
        bool any = false;
        for (int i = k + 1; i < T && !any; ++i) any = nz[(size_t)i * T + k] != 0;
        step_launch[k] = any ? L[k] : 0;
      }
    if (natural)
      for (int r = 0; r < fpad; ++r) natural[r] = r < B.win_fdim[0] ? B.f_nat[r] : -1;
    return OKVISGPU_OK;
  } catch (const std::exception&) {
    return OKVISGPU_ERR_INVALID_ARGUMENT;
  }
}

int okvisgpu_evaluate(okvisgpu_ctx* c, int32_t window, double* cost) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (window < 0 || window >= c->P.n_win) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "bad window");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    okvisgpu_options o;
    okvisgpu_default_options(&o);
    c->setOptions(o);
    c->resetStates(1e-8);
    c->evalAll(2, c->stream);
    launch_reduce(c->P, R_COST_INIT, c->stream);
    HIPCHK(hipGetLastError());
    auto st = c->readStates();
    if (cost) *cost = st[window].x_cost + st[window].fixed_cost;
    // a failed host_evaluate leaves +inf in the cost; report it like okvisgpu_eval_host does
    // (ceres::Problem::Evaluate returns false)
    const int h0 = c->B.win_host_range[2 * window], h1 = c->B.win_host_range[2 * window + 1];
    for (int h = h0; h < h1; ++h)
      if (c->hostFail[h - c->P.n_imu]) return fail(c, OKVISGPU_ERR_NUMERICAL, "host_evaluate failed");
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_linearize_reduce(okvisgpu_ctx* c, int32_t window, int32_t jacobi_scaling, double mu, double* S,
                              double* rhs, double* cost, int32_t* dim_out) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (window < 0 || window >= c->P.n_win) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "bad window");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    okvisgpu_options o;
    okvisgpu_default_options(&o);
    o.jacobi_scaling = jacobi_scaling;
    c->setOptions(o);
    c->resetStates(mu);
    c->launchInit(2);
    launch_gn_reduce(c->P, c->stream);
    HIPCHK(hipGetLastError());
    auto st = c->readStates();
    // exported in the natural order (pose i, speed/bias i, ..., extrinsics), whatever order the
    // window's S is held in (nested dissection: permuted slots and gap rows)
    const int fdim = c->B.win_fdim[window], fpad = c->B.win_fpad[window], dn = c->B.win_fnat[window];
    const int32_t* nat = c->B.f_nat.data() + c->B.win_foff[window];
    if (dim_out) *dim_out = dn;
    if (cost) *cost = st[window].x_cost + st[window].fixed_cost;
    if (S && dn) {
      std::vector<double> full((size_t)fpad * fpad);
      HIPCHK(hipMemcpy(full.data(), c->P.S + c->B.win_soff[window], full.size() * 8, hipMemcpyDeviceToHost));
      for (int r = 0; r < fdim; ++r)
        for (int q = 0; q <= r; ++q) {
          const int a = nat[r], b = nat[q];
          if (a < 0 || b < 0) continue;
          S[(size_t)a * dn + b] = full[(size_t)r * fpad + q];
          S[(size_t)b * dn + a] = full[(size_t)r * fpad + q];
        }
    }
    if (rhs && dn) {
      std::vector<double> v(fdim);
      HIPCHK(hipMemcpy(v.data(), c->P.rhsF + c->B.win_foff[window], sizeof(double) * fdim, hipMemcpyDeviceToHost));
      for (int r = 0; r < fdim; ++r)
        if (nat[r] >= 0) rhs[nat[r]] = v[r];
    }
    if (st[window].gn_failed) return fail(c, OKVISGPU_ERR_NUMERICAL, "landmark block not positive definite");
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_eval_reprojection(okvisgpu_ctx* c, int32_t window, double* r, double* Jp, double* Jl) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (window < 0 || window >= c->P.n_win) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "bad window");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    c->resetStates(1e-8);
    launch_eval(c->P, 3, c->stream);
    HIPCHK(hipGetLastError());
    const int64_t S = c->P.obs_stride;
    std::vector<double> lin((size_t)kObsLin * S);
    HIPCHK(hipMemcpyAsync(lin.data(), c->P.obs_lin[0], lin.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const okvisgpu_problem* pr = c->probs[window];
    const int ob = c->B.obs_base[window], n = pr->n_observations;
    for (int k = 0; k < n; ++k) {
      const int g = ob + k, o = c->B.obs_orig[g];
      if (r) for (int i = 0; i < 2; ++i) r[2 * o + i] = lin[(size_t)i * S + g];
      double A[6], Jpo[12], Jlo[6];
      for (int i = 0; i < 6; ++i) A[i] = lin[(size_t)(2 + i) * S + g];
      const double* hp = &pr->landmarks[4 * pr->obs_landmark[o]];
      const double* tw = &pr->poses[7 * pr->obs_pose[o]];
      const double p3[3] = {hp[0] - tw[0] * hp[3], hp[1] - tw[1] * hp[3], hp[2] - tw[2] * hp[3]};
      obsJacobians(A, p3, hp[3], Jpo, Jlo);
      if (Jp) for (int i = 0; i < 12; ++i) Jp[12 * o + i] = Jpo[i];
      if (Jl) for (int i = 0; i < 6; ++i) Jl[6 * o + i] = Jlo[i];
    }
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_eval_imu(okvisgpu_ctx* c, int32_t window, int32_t redo_always, double* r, double* J) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (window < 0 || window >= c->P.n_win) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "bad window");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    okvisgpu_options o;
    okvisgpu_default_options(&o);
    o.redo_propagation_always = redo_always;
    c->setOptions(o);
    c->resetStates(1e-8);
    launch_eval(c->P, 3, c->stream);
    HIPCHK(hipGetLastError());
    const int n = c->probs[window]->n_imu, ib = c->B.imu_base[window];
    std::vector<double> lin((size_t)kImuLin * std::max(1, n));
    if (n) HIPCHK(hipMemcpyAsync(lin.data(), c->P.imu_lin[0] + (size_t)ib * kImuLin, (size_t)kImuLin * n * 8,
                                 hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int f = 0; f < n; ++f) {
      if (r) for (int i = 0; i < 15; ++i) r[15 * f + i] = lin[(size_t)f * kImuLin + i];
      if (J) for (int i = 0; i < 450; ++i) J[450 * (size_t)f + i] = lin[(size_t)f * kImuLin + 15 + i];
    }
    // keep the caller's ImuError state in sync (the evaluation may have re-integrated)
    c->downloadParams();
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_eval_relpose(okvisgpu_ctx* c, int32_t window, double* r, double* J) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (window < 0 || window >= c->P.n_win) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "bad window");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    c->resetStates(1e-8);
    launch_eval(c->P, 3, c->stream);
    HIPCHK(hipGetLastError());
    const int n = c->probs[window]->n_relpose, rb = c->B.rp_base[window];
    std::vector<double> lin((size_t)kRelPoseLin * std::max(1, n));
    if (n) HIPCHK(hipMemcpyAsync(lin.data(), c->P.rp_lin[0] + (size_t)rb * kRelPoseLin, (size_t)kRelPoseLin * n * 8,
                                 hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; ++i) {
      if (r) for (int k = 0; k < 6; ++k) r[6 * i + k] = lin[(size_t)i * kRelPoseLin + k];
      if (J) for (int k = 0; k < 72; ++k) J[72 * (size_t)i + k] = lin[(size_t)i * kRelPoseLin + 6 + k];
    }
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_eval_host(okvisgpu_ctx* c, int32_t window, double* r, double* J) {
  if (!c) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (!c->haveProblem) return fail(c, OKVISGPU_ERR_NO_PROBLEM, "no problem set");
  if (window < 0 || window >= c->P.n_win) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "bad window");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    c->resetStates(1e-8);
    c->evalHost(3, c->stream);
    HIPCHK(hipGetLastError());
    const int h0 = c->B.win_host_range[2 * window], n = c->B.win_host_range[2 * window + 1] - h0;
    std::vector<double> lin((size_t)kImuLin * std::max(1, n));
    if (n) HIPCHK(hipMemcpyAsync(lin.data(), c->P.imu_lin[0] + (size_t)h0 * kImuLin, (size_t)kImuLin * n * 8,
                                 hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int f = 0; f < n; ++f) {
      if (r) for (int i = 0; i < 15; ++i) r[15 * f + i] = lin[(size_t)f * kImuLin + i];
      if (J) for (int i = 0; i < 450; ++i) J[450 * (size_t)f + i] = lin[(size_t)f * kImuLin + 15 + i];
    }
    for (int f = 0; f < n; ++f)
      if (c->hostFail[h0 - c->P.n_imu + f]) return fail(c, OKVISGPU_ERR_NUMERICAL, "host_evaluate failed");
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_imu_append(okvisgpu_ctx* c, const okvisgpu_imu_append_batch* A, int32_t* steps) {
  if (!c || !A || A->n < 0) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "imu_append: bad arguments");
  if (A->n == 0) return OKVISGPU_OK;
  if (!A->state || !A->t1_old_ns || !A->t1_new_ns || !A->speed_biases || !A->sample_begin)
    return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "imu_append: missing arrays");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    const int n = A->n;
    if (A->sample_begin[0] != 0) throw ArgError{"imu_append: sample_begin must start at 0"};
    for (int i = 0; i < n; ++i)
      if (A->sample_begin[i + 1] < A->sample_begin[i]) throw ArgError{"imu_append: sample_begin not monotone"};
    const int ns = A->sample_begin[n];
    if (ns && (!A->sample_t_ns || !A->sample_gyr_acc)) throw ArgError{"imu_append: sample arrays missing"};
    std::vector<int32_t> blk(4 * (size_t)n);
    for (int i = 0; i < n; ++i) { blk[4 * i] = 0; blk[4 * i + 1] = i; blk[4 * i + 2] = 0; blk[4 * i + 3] = i; }
    const okvisgpu_imu_params& ip = A->imu_params;
    const double par[7] = {ip.a_max, ip.g_max, ip.sigma_g_c, ip.sigma_a_c, ip.sigma_gw_c, ip.sigma_aw_c, ip.g};
    Arena M;
    const size_t o_blk = M.reserve(blk.size() * 4), o_t0 = M.reserve(8 * (size_t)n), o_t1 = M.reserve(8 * (size_t)n),
                 o_sb = M.reserve(4 * (size_t)(n + 1)), o_ts = M.reserve(8 * (size_t)std::max(1, ns)),
                 o_ga = M.reserve(48 * (size_t)std::max(1, ns)), o_par = M.reserve(sizeof(par)),
                 o_st = M.reserve(sizeof(double) * kImuState * n), o_bias = M.reserve(72 * (size_t)n),
                 o_self = M.reserve(sizeof(DevProblem));
    char* base = nullptr;
    HIPCHK(hipMalloc(&base, M.size));
    std::unique_ptr<char, void (*)(char*)> guard(base, [](char* p) { (void)hipFree(p); });
    auto up = [&](size_t off, const void* src, size_t bytes) {
      if (bytes) HIPCHK(hipMemcpyAsync(base + off, src, bytes, hipMemcpyHostToDevice, c->stream));
    };
    up(o_blk, blk.data(), blk.size() * 4);
    up(o_t0, A->t1_old_ns, 8 * (size_t)n);
    up(o_t1, A->t1_new_ns, 8 * (size_t)n);
    up(o_sb, A->sample_begin, 4 * (size_t)(n + 1));
    up(o_ts, A->sample_t_ns, 8 * (size_t)ns);
    up(o_ga, A->sample_gyr_acc, 48 * (size_t)ns);
    up(o_par, par, sizeof(par));
    up(o_st, A->state, sizeof(double) * kImuState * n);
    up(o_bias, A->speed_biases, 72 * (size_t)n);
    // a descriptor holding only what the append mode of k_eval_imu reads
    DevProblem D{};
    D.n_imu = n;
    D.n_fac = n;
    D.imu_blocks = reinterpret_cast<const int32_t*>(base + o_blk);
    D.imu_t0 = reinterpret_cast<const int64_t*>(base + o_t0);
    D.imu_t1 = reinterpret_cast<const int64_t*>(base + o_t1);
    D.imu_sbegin = reinterpret_cast<const int32_t*>(base + o_sb);
    D.imu_ts = reinterpret_cast<const int64_t*>(base + o_ts);
    D.imu_ga = reinterpret_cast<const double*>(base + o_ga);
    D.imu_par = reinterpret_cast<const double*>(base + o_par);
    D.imu_state = reinterpret_cast<double*>(base + o_st);
    D.sb[0] = D.sb[1] = reinterpret_cast<double*>(base + o_bias);
    D.self = reinterpret_cast<const DevProblem*>(base + o_self);
    up(o_self, &D, sizeof(D));
    launch_imu_append(D, c->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(A->state, D.imu_state, sizeof(double) * kImuState * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (steps)
      for (int i = 0; i < n; ++i) {
        const int s0 = A->sample_begin[i], s1 = A->sample_begin[i + 1];
        const bool covered = s1 > s0 && A->sample_t_ns[s1 - 1] >= A->t1_new_ns[i];
        steps[i] = covered ? (int32_t)A->state[(size_t)i * kImuState + 291] : -1;
      }
    return (int)OKVISGPU_OK;
  });
}

int okvisgpu_twopose_compute(okvisgpu_ctx* c, const okvisgpu_twopose_edges* E, double* delta_x, double* sqrt_info,
                             double* lin_point, double* H00, double* b0) {
  if (!c || !E || E->n_edges < 0) return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "twopose_compute: bad arguments");
  if (E->n_edges == 0) return OKVISGPU_OK;
  if (!E->ref_pose || !E->other_pose || !E->landmark_begin || !E->obs_begin || !delta_x || !sqrt_info || !lin_point)
    return fail(c, OKVISGPU_ERR_INVALID_ARGUMENT, "twopose_compute: missing arrays");
  return guarded(c, [&]() {
    HIPCHK(hipSetDevice(c->device));
    const int ne = E->n_edges;
    const int nl = E->landmark_begin[ne] - E->landmark_begin[0];
    if (E->landmark_begin[0] != 0 || nl < 0) throw ArgError{"twopose_compute: landmark_begin must start at 0"};
    for (int e = 0; e < ne; ++e)
      if (E->landmark_begin[e + 1] < E->landmark_begin[e]) throw ArgError{"twopose_compute: landmark_begin not monotone"};
    const int no = nl ? E->obs_begin[nl] - E->obs_begin[0] : 0;
    if (nl && (E->obs_begin[0] != 0 || no < 0)) throw ArgError{"twopose_compute: obs_begin must start at 0"};
    for (int l = 0; l < nl; ++l)
      if (E->obs_begin[l + 1] < E->obs_begin[l]) throw ArgError{"twopose_compute: obs_begin not monotone"};
    if (no && (!E->landmarks || !E->obs_other || !E->obs_camera || !E->obs_keypoint || !E->obs_sqrt_info ||
               !E->cameras || !E->extrinsics))
      throw ArgError{"twopose_compute: observation arrays missing"};
    for (int o = 0; o < no; ++o)
      if (E->obs_camera[o] < 0 || E->obs_camera[o] >= E->n_cameras) throw ArgError{"twopose_compute: obs_camera out of range"};
    std::vector<double> cam((size_t)kCamDoubles * std::max(1, E->n_cameras));
    for (int k = 0; k < E->n_cameras; ++k) {
      const okvisgpu_camera& q = E->cameras[k];
      if (q.distortion < 0 || q.distortion > 3) throw ArgError{"twopose_compute: unknown distortion model"};
      const double cv[kCamDoubles] = {(double)q.distortion, q.fu, q.fv, q.cu, q.cv, q.dist[0], q.dist[1],
                                      q.dist[2], q.dist[3], q.dist[4], q.dist[5], q.dist[6], q.dist[7]};
      std::memcpy(&cam[kCamDoubles * (size_t)k], cv, sizeof(cv));
    }
    std::vector<uint8_t> cauchy(std::max(1, no), 1);
    if (E->obs_cauchy) for (int o = 0; o < no; ++o) cauchy[o] = E->obs_cauchy[o] ? 1 : 0;
    // one scratch allocation for inputs and outputs
    Arena A;
    auto put = [&](size_t bytes) { return A.reserve(bytes); };
    const size_t o_ref = put(56 * (size_t)ne), o_oth = put(56 * (size_t)ne), o_cam = put(cam.size() * 8),
                 o_ex = put(56 * (size_t)std::max(1, E->n_cameras)), o_lb = put(4 * (size_t)(ne + 1)),
                 o_lm = put(32 * (size_t)std::max(1, nl)), o_ob = put(4 * (size_t)(nl + 1)),
                 o_oo = put((size_t)std::max(1, no)), o_oc = put(4 * (size_t)std::max(1, no)),
                 o_kp = put(16 * (size_t)std::max(1, no)), o_L = put(32 * (size_t)std::max(1, no)),
                 o_ca = put((size_t)std::max(1, no)), o_out = put(8 * (size_t)kTwoPoseOut * ne);
    char* base = nullptr;
    HIPCHK(hipMalloc(&base, A.size));
    std::unique_ptr<char, void (*)(char*)> guard(base, [](char* p) { (void)hipFree(p); });
    auto up = [&](size_t off, const void* src, size_t bytes) {
      if (bytes && src) HIPCHK(hipMemcpyAsync(base + off, src, bytes, hipMemcpyHostToDevice, c->stream));
    };
    up(o_ref, E->ref_pose, 56 * (size_t)ne);
    up(o_oth, E->other_pose, 56 * (size_t)ne);
    up(o_cam, cam.data(), cam.size() * 8);
    up(o_ex, E->extrinsics, 56 * (size_t)E->n_cameras);
    up(o_lb, E->landmark_begin, 4 * (size_t)(ne + 1));
    if (nl) {
      up(o_lm, E->landmarks, 32 * (size_t)nl);
      up(o_ob, E->obs_begin, 4 * (size_t)(nl + 1));
    }
    if (no) {
      up(o_oo, E->obs_other, (size_t)no);
      up(o_oc, E->obs_camera, 4 * (size_t)no);
      up(o_kp, E->obs_keypoint, 16 * (size_t)no);
      up(o_L, E->obs_sqrt_info, 32 * (size_t)no);
      up(o_ca, cauchy.data(), (size_t)no);
    }
    TwoPoseDev T{};
    T.n_edges = ne;
    T.n_cam = E->n_cameras;
    T.ref_pose = reinterpret_cast<const double*>(base + o_ref);
    T.other_pose = reinterpret_cast<const double*>(base + o_oth);
    T.cam = reinterpret_cast<const double*>(base + o_cam);
    T.extr = reinterpret_cast<const double*>(base + o_ex);
    T.lm_begin = reinterpret_cast<const int32_t*>(base + o_lb);
    T.lm = reinterpret_cast<const double*>(base + o_lm);
    T.obs_begin = reinterpret_cast<const int32_t*>(base + o_ob);
    T.obs_other = reinterpret_cast<const uint8_t*>(base + o_oo);
    T.obs_cam = reinterpret_cast<const int32_t*>(base + o_oc);
    T.obs_kp = reinterpret_cast<const double*>(base + o_kp);
    T.obs_L = reinterpret_cast<const double*>(base + o_L);
    T.obs_cauchy = reinterpret_cast<const uint8_t*>(base + o_ca);
    T.out = reinterpret_cast<double*>(base + o_out);
    if (!nl) HIPCHK(hipMemsetAsync(base + o_ob, 0, 4, c->stream));
    launch_twopose_compute(T, c->stream);
    HIPCHK(hipGetLastError());
    std::vector<double> out((size_t)kTwoPoseOut * ne);
    HIPCHK(hipMemcpyAsync(out.data(), T.out, out.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int e = 0; e < ne; ++e) {
      const double* r = &out[(size_t)kTwoPoseOut * e];
      std::memcpy(&delta_x[6 * (size_t)e], r, 6 * 8);
      std::memcpy(&sqrt_info[36 * (size_t)e], r + 6, 36 * 8);
      std::memcpy(&lin_point[7 * (size_t)e], r + 42, 7 * 8);
      if (H00) std::memcpy(&H00[36 * (size_t)e], r + 49, 36 * 8);
      if (b0) std::memcpy(&b0[6 * (size_t)e], r + 85, 6 * 8);
    }
    return (int)OKVISGPU_OK;
  });
}

}  // extern "C"
