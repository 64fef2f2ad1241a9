// synth.cpp — host-side generator of the synthetic sliding windows the benchmark is quoted on
// (SURVEY.md §8d): EuRoC stereo rig (config/euroc/okvis2.yaml:2-61), smooth sinusoidal 6-DoF motion
// in the style of okvis_ceres/test/TestImuError.cpp:86-185, 200 Hz IMU with the yaml noise
// densities, landmarks in a 2-20 m depth band, pixel noise N(0,1), information 64/8^2 = I
// (ViGraph.hpp:324-327), Cauchy(1) everywhere, first-state priors as ViGraph::addStatesInitialise
// (ViGraph.cpp:347-370). Deterministic: std::mt19937_64(seed). No GPU is touched.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/okvisgpu.h"
#include "okvisgpu_math.hpp"

using okg::Q;

struct okvisgpu_synth_window {
  okvisgpu_problem prob;
  // owned storage
  std::vector<double> poses, sbs, lms, extr;
  std::vector<double> poses0, sbs0, lms0;  // initial estimate (for reset)
  std::vector<double> gt_poses, gt_sbs, gt_lms;
  std::vector<uint8_t> pose_const, sb_const, lm_const;
  std::vector<okvisgpu_camera> cams;
  std::vector<int32_t> obs_pose, obs_lm, obs_cam;
  std::vector<double> obs_kp, obs_L;
  std::vector<uint8_t> obs_cauchy;
  std::vector<int32_t> imu_blocks, imu_begin;
  std::vector<int64_t> imu_t0, imu_t1, imu_ts;
  std::vector<double> imu_ga, imu_state;
  std::vector<int32_t> pp_block, sbp_block;
  std::vector<double> pp_meas, pp_L, sbp_meas, sbp_L;
  std::vector<int32_t> rp_blocks;
  std::vector<double> rp_dx, rp_J, rp_lin;
  std::vector<uint8_t> rp_kind;
  std::vector<double> extr0, gt_extr;     // initial / true T_SC (online calibration windows)
  std::vector<uint8_t> extr_const;
  std::vector<int32_t> ep_cam;
  std::vector<double> ep_meas, ep_L;
};

namespace {

// Rotation matrix -> quaternion (Eigen's Quaternion(Matrix3) algorithm), normalised.
Q quatFromR(const double R[9]) {
  Q q;
  const double t = R[0] + R[4] + R[8];
  if (t > 0) {
    double s = std::sqrt(t + 1.0);
    q.w = 0.5 * s;
    s = 0.5 / s;
    q.x = (R[7] - R[5]) * s;
    q.y = (R[2] - R[6]) * s;
    q.z = (R[3] - R[1]) * s;
  } else {
    int i = 0;
    if (R[4] > R[0]) i = 1;
    if (R[8] > R[i * 3 + i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double s = std::sqrt(R[i * 3 + i] - R[j * 3 + j] - R[k * 3 + k] + 1.0);
    double c[3];
    c[i] = 0.5 * s;
    s = 0.5 / s;
    q.w = (R[k * 3 + j] - R[j * 3 + k]) * s;
    c[j] = (R[j * 3 + i] + R[i * 3 + j]) * s;
    c[k] = (R[k * 3 + i] + R[i * 3 + k]) * s;
    q.x = c[0]; q.y = c[1]; q.z = c[2];
  }
  return okg::qnormalize(q);
}

struct TruthState {
  double r[3], v[3];
  Q q;
};

}  // namespace

extern "C" {

void okvisgpu_synth_default_config(okvisgpu_synth_config* c, int32_t n_kf, int32_t n_lm, int32_t n_obs,
                                   uint64_t seed) {
  c->n_keyframes = n_kf;
  c->n_landmarks = n_lm;
  c->n_observations = n_obs;
  c->max_obs_per_landmark = 20;
  c->kf_dt_s = 0.1;
  c->imu_rate_hz = 200.0;
  c->pixel_noise = 1.0;
  c->init_sigma_pos = 0.05;
  c->init_sigma_rot = 0.01;
  c->init_sigma_lm = 0.05;
  c->init_sigma_vel = 0.02;
  c->seed = seed;
  c->n_relpose = 0;
  c->relpose_stride = 5;
  c->relpose_kind = 0;
  c->do_extrinsics = 0;
  c->extrinsics_sigma_r = 0.001;      // config/hilti22/okvis2.yaml:84-85
  c->extrinsics_sigma_alpha = 0.005;
}

int okvisgpu_synth_create(const okvisgpu_synth_config* cfg, okvisgpu_synth_window** out) {
  if (!cfg || !out || cfg->n_keyframes < 2 || cfg->n_landmarks < 1 || cfg->n_observations < 1)
    return OKVISGPU_ERR_INVALID_ARGUMENT;
  auto* W = new okvisgpu_synth_window();
  std::mt19937_64 rng(cfg->seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::normal_distribution<double> N01(0.0, 1.0);
  auto uni = [&](double a, double b) { return a + (b - a) * U(rng); };

  // ---------------- rig: config/euroc/okvis2.yaml:2-32
  const double Tsc[2][12] = {
      {0.0148655429818, -0.999880929698, 0.00414029679422, -0.0216401454975, 0.999557249008, 0.0149672133247,
       0.025715529948, -0.064676986768, -0.0257744366974, 0.00375618835797, 0.999660727178, 0.00981073058949},
      {0.0125552670891, -0.999755099723, 0.0182237714554, -0.0198435579556, 0.999598781151, 0.0130119051815,
       0.0251588363115, 0.0453689425024, -0.0253898008918, 0.0179005838253, 0.999517347078, 0.00786212447038}};
  const double dist[2][4] = {{-0.28340811217, 0.0739590738929, 0.000193595028569, 1.76187114545e-05},
                             {-0.283683654496, 0.0745128430929, -0.000104738949098, -3.55590700274e-05}};
  const double foc[2][2] = {{458.654880721, 457.296696463}, {457.587426604, 456.13442556}};
  const double pp[2][2] = {{367.215803962, 248.37534061}, {379.99944652, 255.238185386}};
  W->cams.resize(2);
  W->extr.resize(14);
  double C_SC[2][9], t_SC[2][3];
  for (int c = 0; c < 2; ++c) {
    okvisgpu_camera& k = W->cams[c];
    k.distortion = OKVISGPU_DIST_RADTAN;
    k.width = 752;
    k.height = 480;
    k.fu = foc[c][0]; k.fv = foc[c][1]; k.cu = pp[c][0]; k.cv = pp[c][1];
    for (int i = 0; i < 4; ++i) k.dist[i] = dist[c][i];
    double R[9];
    for (int r = 0; r < 3; ++r)
      for (int cc = 0; cc < 3; ++cc) R[r * 3 + cc] = Tsc[c][r * 4 + cc];
    const Q q = quatFromR(R);
    okg::qrot(q, C_SC[c]);
    for (int i = 0; i < 3; ++i) t_SC[c][i] = Tsc[c][i * 4 + 3];
    double* e = &W->extr[7 * c];
    e[0] = t_SC[c][0]; e[1] = t_SC[c][1]; e[2] = t_SC[c][2];
    e[3] = q.x; e[4] = q.y; e[5] = q.z; e[6] = q.w;
  }
  okg::Cam gcam[2];
  for (int c = 0; c < 2; ++c)
    gcam[c] = okg::Cam{1, foc[c][0], foc[c][1], pp[c][0], pp[c][1], dist[c][0], dist[c][1], dist[c][2], dist[c][3],
                       0.0, 0.0, 0.0, 0.0};

  // ---------------- IMU parameters: config/euroc/okvis2.yaml:49-61
  okvisgpu_imu_params ip;
  ip.a_max = 176.0;
  ip.g_max = 7.8;
  ip.sigma_g_c = 20.0e-4;
  ip.sigma_a_c = 20.0e-3;
  ip.sigma_gw_c = 20.0e-5;
  ip.sigma_aw_c = 20.0e-3;
  ip.g = 9.81007;
  const double sigma_bg = 0.01, sigma_ba = 0.1;
  const double a0[3] = {-0.05, 0.09, 0.01};

  // ---------------- ground-truth motion (TestImuError.cpp:86-185 style sinusoids)
  const int nkf = cfg->n_keyframes;
  const double kfdt = cfg->kf_dt_s;
  const double dt_int = 1e-3;                       // truth integration step
  const int64_t imu_dt_ns = (int64_t)std::llround(1e9 / cfg->imu_rate_hz);
  const int64_t t_start_ns = 1000000000LL;          // absolute time origin (1 s)
  const int64_t cam_offset_ns = 1000000;            // KF stamps 1 ms off the IMU grid: exercises
                                                    // the interpolation at t0/t1 (ImuError.cpp:317-335)
  double w_om[3], p_om[3], m_om[3], w_a[3], p_a[3], m_a[3];
  for (int i = 0; i < 3; ++i) {
    w_om[i] = uni(0.5, 3.0);
    p_om[i] = uni(0.0, M_PI);
    m_om[i] = uni(0.05, 0.3);
    w_a[i] = uni(0.5, 3.0);
    p_a[i] = uni(0.1, M_PI);
    m_a[i] = uni(0.2, 1.0);
  }
  double bg_true[3], ba_true[3];
  for (int i = 0; i < 3; ++i) {
    bg_true[i] = 0.002 * N01(rng);
    ba_true[i] = a0[i] + 0.02 * N01(rng);
  }
  // Start orientation: sensor z (~ camera optical axis) looking along world +x, sensor x down.
  const double R0[9] = {0, 0, 1, 0, 1, 0, -1, 0, 0};  // columns: S_x=(0,0,-1), S_y=(0,1,0), S_z=(1,0,0)
  TruthState s;
  s.q = quatFromR(R0);
  s.r[0] = 0; s.r[1] = 0; s.r[2] = 0;
  s.v[0] = 0.1; s.v[1] = 0.8; s.v[2] = 0.0;
  auto omegaS = [&](double t, double o[3]) {
    for (int i = 0; i < 3; ++i) o[i] = m_om[i] * std::sin(w_om[i] * t + p_om[i]);
  };
  auto accW = [&](double t, double o[3]) {
    for (int i = 0; i < 3; ++i) o[i] = m_a[i] * std::sin(w_a[i] * t + p_a[i]);
  };
  const double T_total = (nkf - 1) * kfdt;
  const double t_begin = -0.05, t_end = T_total + 0.06;
  const int64_t first_imu_ns = t_start_ns + (int64_t)std::llround(t_begin * 1e9);
  const int64_t last_imu_ns = t_start_ns + (int64_t)std::llround(t_end * 1e9);
  // integrate truth on the 1 ms grid, record states on the 1 ms grid
  const int nsteps = (int)std::llround((t_end - t_begin) / dt_int) + 1;
  std::vector<TruthState> truth(nsteps);
  for (int k = 0; k < nsteps; ++k) {
    const double t = t_begin + k * dt_int;
    truth[k] = s;
    double om[3], aw[3];
    omegaS(t, om);
    accW(t, aw);
    const double theta_half = std::sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]) * dt_int * 0.5;
    const double sh = okg::sinc(theta_half) * 0.5 * dt_int;
    const Q dq{sh * om[0], sh * om[1], sh * om[2], std::cos(theta_half)};
    s.q = okg::qnormalize(okg::qmul(s.q, dq));
    for (int i = 0; i < 3; ++i) {
      s.v[i] += dt_int * aw[i];
      s.r[i] += dt_int * s.v[i];
    }
  }
  auto truthAt = [&](int64_t t_ns) -> const TruthState& {
    const double t = (double)(t_ns - t_start_ns) * 1e-9;
    int k = (int)std::llround((t - t_begin) / dt_int);
    k = std::max(0, std::min(nsteps - 1, k));
    return truth[k];
  };
  // IMU samples on the imu grid
  std::vector<int64_t> all_ts;
  std::vector<double> all_ga;
  const double sg = ip.sigma_g_c / std::sqrt(1.0 / cfg->imu_rate_hz);
  const double sa = ip.sigma_a_c / std::sqrt(1.0 / cfg->imu_rate_hz);
  for (int64_t t = first_imu_ns; t <= last_imu_ns; t += imu_dt_ns) {
    const TruthState& ts = truthAt(t);
    const double tt = (double)(t - t_start_ns) * 1e-9;
    double om[3], aw[3];
    omegaS(tt, om);
    accW(tt, aw);
    double C[9];
    okg::qrot(ts.q, C);
    const double f_W[3] = {aw[0], aw[1], aw[2] + ip.g};
    double f_S[3];
    okg::mtv3(C, f_W, f_S);
    all_ts.push_back(t);
    for (int i = 0; i < 3; ++i) all_ga.push_back(om[i] + bg_true[i] + sg * N01(rng));
    for (int i = 0; i < 3; ++i) all_ga.push_back(f_S[i] + ba_true[i] + sa * N01(rng));
  }

  // ---------------- keyframes: ground truth poses / speed-biases
  std::vector<int64_t> kf_t(nkf);
  W->gt_poses.resize(7 * nkf);
  W->gt_sbs.resize(9 * nkf);
  for (int k = 0; k < nkf; ++k) {
    kf_t[k] = t_start_ns + cam_offset_ns + (int64_t)std::llround(k * kfdt * 1e9);
    const TruthState& ts = truthAt(kf_t[k]);
    double* p = &W->gt_poses[7 * k];
    p[0] = ts.r[0]; p[1] = ts.r[1]; p[2] = ts.r[2];
    p[3] = ts.q.x; p[4] = ts.q.y; p[5] = ts.q.z; p[6] = ts.q.w;
    double* b = &W->gt_sbs[9 * k];
    for (int i = 0; i < 3; ++i) { b[i] = ts.v[i]; b[3 + i] = bg_true[i]; b[6 + i] = ba_true[i]; }
  }

  // ---------------- landmarks + observations
  const int nlm = cfg->n_landmarks;
  W->gt_lms.resize(4 * nlm);
  // camera-from-world for every KF/camera
  std::vector<double> Tcw(nkf * 2 * 12);
  for (int k = 0; k < nkf; ++k) {
    const double* p = &W->gt_poses[7 * k];
    double C_WS[9];
    okg::qrot(Q{p[3], p[4], p[5], p[6]}, C_WS);
    for (int c = 0; c < 2; ++c) {
      // C_CW = C_SC^T C_WS^T ; t: p_C = C_CW (p_W - r_WS) - C_SC^T t_SC
      double* T = &Tcw[(k * 2 + c) * 12];
      for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) {
          double v = 0;
          for (int m = 0; m < 3; ++m) v += C_SC[c][m * 3 + r] * C_WS[cc * 3 + m];
          T[r * 4 + cc] = v;
        }
      for (int r = 0; r < 3; ++r) {
        double v = 0;
        for (int m = 0; m < 3; ++m) v += T[r * 4 + m] * p[m];
        double w = 0;
        for (int m = 0; m < 3; ++m) w += C_SC[c][m * 3 + r] * t_SC[c][m];
        T[r * 4 + 3] = -v - w;
      }
    }
  }
  auto projectTrue = [&](int k, int c, const double* X, double kp[2]) -> bool {
    const double* T = &Tcw[(k * 2 + c) * 12];
    double pc[3];
    for (int r = 0; r < 3; ++r) pc[r] = T[r * 4 + 0] * X[0] + T[r * 4 + 1] * X[1] + T[r * 4 + 2] * X[2] + T[r * 4 + 3];
    if (pc[2] < 0.5) return false;
    double J[6];
    okg::projectHomogeneous(gcam[c], pc[0], pc[1], pc[2], 1.0, kp, J, false);
    return kp[0] >= 0.0 && kp[0] < 752.0 && kp[1] >= 0.0 && kp[1] < 480.0;
  };
  // visible (kf, cam) list per landmark: contiguous run around an anchor keyframe
  std::vector<std::vector<std::pair<int, int>>> vis(nlm);
  for (int l = 0; l < nlm; ++l) {
    for (int attempt = 0; attempt < 100; ++attempt) {
      const int anchor = (int)(U(rng) * nkf) % nkf;
      const double u = uni(20.0, 732.0), v = uni(20.0, 460.0), depth = uni(2.0, 20.0);
      // back-project through cam0 of the anchor (undistorted ray)
      const double xn = (u - pp[0][0]) / foc[0][0], yn = (v - pp[0][1]) / foc[0][1];
      const double pc[3] = {xn * depth, yn * depth, depth};
      const double* T = &Tcw[(anchor * 2 + 0) * 12];
      double X[3];
      for (int r = 0; r < 3; ++r)
        X[r] = T[0 * 4 + r] * (pc[0] - T[0 * 4 + 3]) + T[1 * 4 + r] * (pc[1] - T[1 * 4 + 3]) +
               T[2 * 4 + r] * (pc[2] - T[2 * 4 + 3]);
      std::vector<std::pair<int, int>> run;
      double kp[2];
      // walk backwards and forwards from the anchor while visible in at least one camera
      int lo = anchor, hi = anchor;
      auto visibleKf = [&](int k) {
        return projectTrue(k, 0, X, kp) || projectTrue(k, 1, X, kp);
      };
      if (!visibleKf(anchor)) continue;
      while (lo - 1 >= 0 && visibleKf(lo - 1) && (hi - lo + 1) < cfg->max_obs_per_landmark / 2) --lo;
      while (hi + 1 < nkf && visibleKf(hi + 1) && (hi - lo + 1) < cfg->max_obs_per_landmark / 2) ++hi;
      for (int k = lo; k <= hi; ++k)
        for (int c = 0; c < 2; ++c)
          if (projectTrue(k, c, X, kp)) run.push_back({k, c});
      if ((int)run.size() < 2) continue;
      vis[l] = run;
      W->gt_lms[4 * l + 0] = X[0]; W->gt_lms[4 * l + 1] = X[1]; W->gt_lms[4 * l + 2] = X[2];
      W->gt_lms[4 * l + 3] = 1.0;
      break;
    }
    if (vis[l].empty()) { delete W; return OKVISGPU_ERR_INVALID_ARGUMENT; }
  }
  // choose per-landmark observation counts summing to the target
  std::vector<int> cnt(nlm);
  const double mean = (double)cfg->n_observations / nlm;
  long total = 0;
  for (int l = 0; l < nlm; ++l) {
    const int cap = std::min((int)vis[l].size(), cfg->max_obs_per_landmark);
    int n = (int)std::lround(mean * std::exp(0.35 * N01(rng)) );
    n = std::max(2, std::min(cap, n));
    cnt[l] = n;
    total += n;
  }
  for (int pass = 0; pass < 64 && total != cfg->n_observations; ++pass) {
    for (int l = 0; l < nlm && total != cfg->n_observations; ++l) {
      const int cap = std::min((int)vis[l].size(), cfg->max_obs_per_landmark);
      if (total < cfg->n_observations && cnt[l] < cap) { ++cnt[l]; ++total; }
      else if (total > cfg->n_observations && cnt[l] > 2) { --cnt[l]; --total; }
    }
  }
  // emit observations: a contiguous sub-run centred in the visible run; sorted by landmark
  for (int l = 0; l < nlm; ++l) {
    const int n = cnt[l];
    const int start = ((int)vis[l].size() - n) / 2;
    for (int i = start; i < start + n; ++i) {
      const int k = vis[l][i].first, c = vis[l][i].second;
      double kp[2];
      projectTrue(k, c, &W->gt_lms[4 * l], kp);
      W->obs_pose.push_back(k);
      W->obs_lm.push_back(l);
      W->obs_cam.push_back(c);
      W->obs_kp.push_back(kp[0] + cfg->pixel_noise * N01(rng));
      W->obs_kp.push_back(kp[1] + cfg->pixel_noise * N01(rng));
      // keypoint size 8 => information = 64/64 I => sqrt information I (ViGraph.hpp:324-327)
      const double size = 8.0, sq = 8.0 / size;
      W->obs_L.push_back(sq); W->obs_L.push_back(0.0); W->obs_L.push_back(0.0); W->obs_L.push_back(sq);
      W->obs_cauchy.push_back(1);
    }
  }

  // ---------------- initial estimates (perturbed) and priors
  W->poses = W->gt_poses;
  W->sbs = W->gt_sbs;
  W->lms = W->gt_lms;
  for (int k = 1; k < nkf; ++k) {  // state 0 is the gauge anchor (prior at truth)
    double* p = &W->poses[7 * k];
    for (int i = 0; i < 3; ++i) p[i] += cfg->init_sigma_pos * N01(rng);
    const Q dq = okg::deltaQ(cfg->init_sigma_rot * N01(rng), cfg->init_sigma_rot * N01(rng),
                             cfg->init_sigma_rot * N01(rng));
    const Q q = okg::qnormalize(okg::qmul(dq, Q{p[3], p[4], p[5], p[6]}));
    p[3] = q.x; p[4] = q.y; p[5] = q.z; p[6] = q.w;
  }
  for (int k = 0; k < nkf; ++k) {
    double* b = &W->sbs[9 * k];
    if (k > 0)
      for (int i = 0; i < 3; ++i) b[i] += cfg->init_sigma_vel * N01(rng);
    for (int i = 0; i < 3; ++i) { b[3 + i] = 0.0; b[6 + i] = a0[i]; }  // yaml g0 / a0
  }
  for (int l = 0; l < nlm; ++l)
    for (int i = 0; i < 3; ++i) W->lms[4 * l + i] += cfg->init_sigma_lm * N01(rng);
  W->poses0 = W->poses;
  W->sbs0 = W->sbs;
  W->lms0 = W->lms;
  W->pose_const.assign(nkf, 0);
  W->sb_const.assign(nkf, 0);
  W->lm_const.assign(nlm, 0);

  // PoseError prior on the first pose, information diag (1e8,1e8,1e8,0,0,1e2) (ViGraph.cpp:347-368)
  W->pp_block.push_back(0);
  W->pp_meas.assign(W->poses.begin(), W->poses.begin() + 7);
  W->pp_L.assign(36, 0.0);
  const double pinfo[6] = {1.0e8, 1.0e8, 1.0e8, 0.0, 0.0, 1.0e2};
  for (int i = 0; i < 6; ++i) W->pp_L[i * 6 + i] = std::sqrt(pinfo[i]);  // PoseError.cpp:34-39
  // SpeedAndBiasError prior: variances 0.1, sigma_bg^2, sigma_ba^2 (ViGraph.cpp:363-370);
  // information diagonal => LLT(info).L^T = diag(sqrt(info))
  W->sbp_block.push_back(0);
  W->sbp_meas.assign(W->sbs.begin(), W->sbs.begin() + 9);
  W->sbp_L.assign(81, 0.0);
  for (int i = 0; i < 3; ++i) {
    W->sbp_L[i * 9 + i] = std::sqrt(1.0 / 0.1);
    W->sbp_L[(3 + i) * 9 + 3 + i] = std::sqrt(1.0 / (sigma_bg * sigma_bg));
    W->sbp_L[(6 + i) * 9 + 6 + i] = std::sqrt(1.0 / (sigma_ba * sigma_ba));
  }

  // ---------------- IMU factors between consecutive keyframes
  W->imu_begin.push_back(0);
  for (int k = 0; k + 1 < nkf; ++k) {
    const int64_t t0 = kf_t[k], t1 = kf_t[k + 1];
    W->imu_blocks.push_back(k); W->imu_blocks.push_back(k);
    W->imu_blocks.push_back(k + 1); W->imu_blocks.push_back(k + 1);
    W->imu_t0.push_back(t0);
    W->imu_t1.push_back(t1);
    // samples spanning [t0, t1]: last sample <= t0 through first sample >= t1 (ImuError.cpp:47-54)
    size_t a = 0;
    while (a + 1 < all_ts.size() && all_ts[a + 1] <= t0) ++a;
    size_t b = a;
    while (b < all_ts.size() && all_ts[b] < t1) ++b;
    for (size_t i = a; i <= b && i < all_ts.size(); ++i) {
      W->imu_ts.push_back(all_ts[i]);
      for (int j = 0; j < 6; ++j) W->imu_ga.push_back(all_ga[6 * i + j]);
    }
    W->imu_begin.push_back((int32_t)W->imu_ts.size());
  }
  W->imu_state.assign((size_t)(nkf - 1) * OKVISGPU_IMU_STATE_DOUBLES, 0.0);

  // ---------------- pose-graph edges (TwoPoseStandardGraphErrorConst), own random stream so the
  // windows without edges are unchanged
  if (cfg->n_relpose > 0) {
    if (cfg->relpose_stride < 1 || cfg->relpose_stride >= nkf) {
      delete W;
      return OKVISGPU_ERR_INVALID_ARGUMENT;
    }
    std::mt19937_64 rng2(cfg->seed ^ 0x9E3779B97F4A7C15ull);
    std::normal_distribution<double> G(0.0, 1.0);
    const double sp = 0.02, sr = 0.005;
    for (int e = 0; e < cfg->n_relpose; ++e) {
      const int a = e % (nkf - cfg->relpose_stride), b = a + cfg->relpose_stride;
      W->rp_blocks.push_back(a);
      W->rp_blocks.push_back(b);
      // kind 1 (RelativePoseError): the perturbed relative pose below is the measurement T_AB and
      // the upper-triangular J_ is LLT(information).L^T of information = J_^T J_
      W->rp_kind.push_back(cfg->relpose_kind == 2 ? (uint8_t)(e & 1) : (uint8_t)(cfg->relpose_kind == 1));
      // linearisation point: ground-truth T_S0S1 perturbed at the edge's noise level
      const double* p0 = &W->gt_poses[7 * a];
      const double* p1 = &W->gt_poses[7 * b];
      const Q q0 = okg::qnormalize(Q{p0[3], p0[4], p0[5], p0[6]}), q1 = okg::qnormalize(Q{p1[3], p1[4], p1[5], p1[6]});
      double C0[9];
      okg::qrot(q0, C0);
      const double d[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
      double r[3];
      okg::mtv3(C0, d, r);
      const Q dq = okg::deltaQ(sr * G(rng2), sr * G(rng2), sr * G(rng2));
      const Q ql = okg::qnormalize(okg::qmul(dq, okg::qmul(okg::qinv(q0), q1)));
      const double lin[7] = {r[0] + sp * G(rng2), r[1] + sp * G(rng2), r[2] + sp * G(rng2), ql.x, ql.y, ql.z, ql.w};
      W->rp_lin.insert(W->rp_lin.end(), lin, lin + 7);
      for (int i = 0; i < 6; ++i) W->rp_dx.push_back(0.5 * (i < 3 ? sp : sr) * G(rng2));
      // J_: upper triangular square-root information, diagonal 1/sigma, 10 % couplings
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
          const double s = 1.0 / (i < 3 ? sp : sr);
          W->rp_J.push_back(j < i ? 0.0 : (j == i ? s : 0.1 * s * G(rng2)));
        }
    }
  }

  // ---------------- online extrinsics calibration (do_extrinsics: true, ViGraph.cpp:372-382): the
  // calibration the window starts from is the true T_SC perturbed at the prior's sigmas, and the
  // prior PoseError(T_SC_init, sigma_r^2, sigma_alpha^2) is centred on it. Own random stream, so
  // windows without online calibration are unchanged.
  W->gt_extr = W->extr;
  W->extr_const.assign(2, 1);
  if (cfg->do_extrinsics) {
    std::mt19937_64 rng3(cfg->seed ^ 0xC2B2AE3D27D4EB4Full);
    std::normal_distribution<double> G(0.0, 1.0);
    const double sr = cfg->extrinsics_sigma_r, sa = cfg->extrinsics_sigma_alpha;
    for (int c = 0; c < 2; ++c) {
      double* e = &W->extr[7 * c];
      for (int i = 0; i < 3; ++i) e[i] += sr * G(rng3);
      const Q q = okg::qnormalize(okg::qmul(okg::deltaQ(sa * G(rng3), sa * G(rng3), sa * G(rng3)), Q{e[3], e[4], e[5], e[6]}));
      e[3] = q.x; e[4] = q.y; e[5] = q.z; e[6] = q.w;
      W->extr_const[c] = 0;
      W->ep_cam.push_back(c);
      W->ep_meas.insert(W->ep_meas.end(), e, e + 7);
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) W->ep_L.push_back(i != j ? 0.0 : 1.0 / (i < 3 ? sr : sa));  // PoseError.cpp:41-66
    }
  }
  W->extr0 = W->extr;

  // ---------------- problem view
  okvisgpu_problem& P = W->prob;
  std::memset(&P, 0, sizeof(P));
  P.n_poses = nkf;
  P.poses = W->poses.data();
  P.pose_constant = W->pose_const.data();
  P.n_speed_biases = nkf;
  P.speed_biases = W->sbs.data();
  P.speed_bias_constant = W->sb_const.data();
  P.n_landmarks = nlm;
  P.landmarks = W->lms.data();
  P.landmark_constant = W->lm_const.data();
  P.n_cameras = 2;
  P.cameras = W->cams.data();
  P.extrinsics = W->extr.data();
  P.n_observations = (int32_t)W->obs_pose.size();
  P.obs_pose = W->obs_pose.data();
  P.obs_landmark = W->obs_lm.data();
  P.obs_camera = W->obs_cam.data();
  P.obs_keypoint = W->obs_kp.data();
  P.obs_sqrt_info = W->obs_L.data();
  P.obs_cauchy = W->obs_cauchy.data();
  P.n_imu = nkf - 1;
  P.imu_blocks = W->imu_blocks.data();
  P.imu_t0_ns = W->imu_t0.data();
  P.imu_t1_ns = W->imu_t1.data();
  P.imu_sample_begin = W->imu_begin.data();
  P.imu_sample_t_ns = W->imu_ts.data();
  P.imu_sample_gyr_acc = W->imu_ga.data();
  P.imu_params = ip;
  P.imu_state = W->imu_state.data();
  P.n_pose_priors = 1;
  P.pose_prior_block = W->pp_block.data();
  P.pose_prior_meas = W->pp_meas.data();
  P.pose_prior_sqrt_info = W->pp_L.data();
  P.n_sb_priors = 1;
  P.sb_prior_block = W->sbp_block.data();
  P.sb_prior_meas = W->sbp_meas.data();
  P.sb_prior_sqrt_info = W->sbp_L.data();
  P.n_relpose = (int32_t)W->rp_blocks.size() / 2;
  P.relpose_blocks = W->rp_blocks.data();
  P.relpose_delta_x = W->rp_dx.data();
  P.relpose_sqrt_info = W->rp_J.data();
  P.relpose_lin_point = W->rp_lin.data();
  P.relpose_kind = W->rp_kind.data();
  P.extrinsics_constant = W->extr_const.data();
  P.n_extrinsics_priors = (int32_t)W->ep_cam.size();
  P.extrinsics_prior_camera = W->ep_cam.data();
  P.extrinsics_prior_meas = W->ep_meas.data();
  P.extrinsics_prior_sqrt_info = W->ep_L.data();
  *out = W;
  return OKVISGPU_OK;
}

const okvisgpu_problem* okvisgpu_synth_problem(okvisgpu_synth_window* w) { return w ? &w->prob : nullptr; }

int okvisgpu_synth_ground_truth(const okvisgpu_synth_window* w, double* poses, double* landmarks,
                                double* sbs) {
  if (!w) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (poses) std::memcpy(poses, w->gt_poses.data(), sizeof(double) * w->gt_poses.size());
  if (landmarks) std::memcpy(landmarks, w->gt_lms.data(), sizeof(double) * w->gt_lms.size());
  if (sbs) std::memcpy(sbs, w->gt_sbs.data(), sizeof(double) * w->gt_sbs.size());
  return OKVISGPU_OK;
}

int okvisgpu_synth_true_extrinsics(const okvisgpu_synth_window* w, double* extrinsics) {
  if (!w || !extrinsics) return OKVISGPU_ERR_INVALID_ARGUMENT;
  std::memcpy(extrinsics, w->gt_extr.data(), sizeof(double) * w->gt_extr.size());
  return OKVISGPU_OK;
}

int okvisgpu_synth_reset(okvisgpu_synth_window* w) {
  if (!w) return OKVISGPU_ERR_INVALID_ARGUMENT;
  w->poses = w->poses0;
  w->sbs = w->sbs0;
  w->lms = w->lms0;
  w->extr = w->extr0;
  w->prob.extrinsics = w->extr.data();
  std::fill(w->imu_state.begin(), w->imu_state.end(), 0.0);
  w->prob.poses = w->poses.data();
  w->prob.speed_biases = w->sbs.data();
  w->prob.landmarks = w->lms.data();
  return OKVISGPU_OK;
}

void okvisgpu_synth_destroy(okvisgpu_synth_window* w) { delete w; }

}  // extern "C"
