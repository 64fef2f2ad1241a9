// graph_io.cpp — the okvis Component text graph (okvis_ceres/src/Component.cpp) as okvisgpu
// problems: Component::load (:50-383) builds the full graph the way ViGraphEstimator does, and
// Component::save (:385-506) writes one. Host code only; no GPU is touched.
//
// Load semantics (restated):
//   VERTEX_SE3:QUAT_TIME id x y z qx qy qz qw t_ns   a state: pose block, time stamp
//   VERTEX_R3:VEL / :ACCBIAS / :GYRBIAS id a b c     speed and biases (sb[0..2] / [6..8] / [3..5])
//   VERTEX_TRACKXYZ id x y z quality                 a landmark, hp = (x, y, z, 1)
//   FRAME id cam extrId x y z qx qy qz qw t_ns       T_SC of camera cam (one extrinsics block per camera:
//                                                    a second extrId for a camera = online calibration,
//                                                    which the GPU path does not support)
//   FRAME:KEYPOINT id cam u v size BRISK2 <hex>      keypoints of that frame, in order (cv::KeyPoint:
//                                                    u, v, size are floats)
//   EDGE_IMU prev id + EDGE_IMU:MEASUREMENTS ax ay az gx gy gz t_ns ...
//                                                    ImuError(measurements, imuParameters, t_prev, t_id)
//   EDGE_OBS id cam kp lmId u v i00 i01 i10 i11      ViGraph::addObservation(multiFrame, lm, kid, true):
//                                                    measurement and information 64/size^2 from the
//                                                    frame's keypoint (ViGraph.hpp:307-352), Cauchy(1)
// The camera intrinsics and the IMU parameters are configuration, not part of the file (Component
// takes them from its NCameraSystem / ImuParameters): the caller passes them.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/okvisgpu.h"

struct okvisgpu_graph {
  okvisgpu_problem prob;
  std::vector<uint64_t> state_ids, landmark_ids;
  std::vector<int64_t> state_t;
  std::vector<double> poses, sbs, lms, extr;
  std::vector<uint8_t> pose_const, sb_const, lm_const, obs_cauchy;
  std::vector<okvisgpu_camera> cams;
  std::vector<int32_t> obs_pose, obs_lm, obs_cam, imu_blocks, imu_begin;
  std::vector<double> obs_kp, obs_L, imu_ga, imu_state;
  std::vector<int64_t> imu_t0, imu_t1, imu_ts;
  std::string error;
};

namespace {

struct Keypoint {
  float u, v, size;
};

struct ParseError {
  std::string msg;
};

void finishProblem(okvisgpu_graph& G, const okvisgpu_imu_params& ip) {
  okvisgpu_problem& P = G.prob;
  std::memset(&P, 0, sizeof(P));
  P.n_poses = (int32_t)G.state_ids.size();
  P.poses = G.poses.data();
  P.pose_constant = G.pose_const.data();
  P.n_speed_biases = P.n_poses;
  P.speed_biases = G.sbs.data();
  P.speed_bias_constant = G.sb_const.data();
  P.n_landmarks = (int32_t)G.landmark_ids.size();
  P.landmarks = G.lms.data();
  P.landmark_constant = G.lm_const.data();
  P.n_cameras = (int32_t)G.cams.size();
  P.cameras = G.cams.data();
  P.extrinsics = G.extr.data();
  P.n_observations = (int32_t)G.obs_pose.size();
  P.obs_pose = G.obs_pose.data();
  P.obs_landmark = G.obs_lm.data();
  P.obs_camera = G.obs_cam.data();
  P.obs_keypoint = G.obs_kp.data();
  P.obs_sqrt_info = G.obs_L.data();
  P.obs_cauchy = G.obs_cauchy.data();
  P.n_imu = (int32_t)G.imu_t0.size();
  P.imu_blocks = G.imu_blocks.data();
  P.imu_t0_ns = G.imu_t0.data();
  P.imu_t1_ns = G.imu_t1.data();
  P.imu_sample_begin = G.imu_begin.data();
  P.imu_sample_t_ns = G.imu_ts.data();
  P.imu_sample_gyr_acc = G.imu_ga.data();
  P.imu_params = ip;
  P.imu_state = G.imu_state.data();
}

}  // namespace

extern "C" {

int okvisgpu_graph_load(const char* path, const okvisgpu_camera* cameras, int32_t n_cameras,
                        const okvisgpu_imu_params* imu, okvisgpu_graph** out) {
  if (!path || !out || !imu || n_cameras < 1 || !cameras) return OKVISGPU_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  std::ifstream file(path);
  if (!file) return OKVISGPU_ERR_INVALID_ARGUMENT;
  auto* G = new okvisgpu_graph();
  try {
    // states_ / landmarks_ are std::maps keyed by id: the problem orders them by id
    std::map<uint64_t, std::vector<double>> pose, sb;
    std::map<uint64_t, int64_t> stamp;
    std::map<uint64_t, std::vector<double>> lm;
    std::map<std::pair<uint64_t, int>, std::vector<Keypoint>> kps;
    std::vector<long long> extrId(n_cameras, -1);
    std::vector<std::vector<double>> extr(n_cameras);
    struct Imu { uint64_t a, b; std::vector<double> ga; std::vector<int64_t> t; };
    std::vector<Imu> imus;
    struct Obs { uint64_t state, lm; int cam, kp; };
    std::vector<Obs> obs;
    std::string line;
    long long lineNo = 0;
    while (std::getline(file, line)) {
      ++lineNo;
      std::istringstream ss(line);
      std::string type;
      if (!(ss >> type)) continue;
      auto bad = [&](const std::string& m) { throw ParseError{"line " + std::to_string(lineNo) + ": " + m}; };
      if (type == "VERTEX_SE3:QUAT_TIME") {
        uint64_t id;
        double v[7];
        long long t;
        if (!(ss >> id >> v[0] >> v[1] >> v[2] >> v[3] >> v[4] >> v[5] >> v[6] >> t)) bad("bad VERTEX_SE3:QUAT_TIME");
        // kinematics::Transformation normalises the quaternion (Transformation.hpp:220-223)
        const double n = std::sqrt(v[3] * v[3] + v[4] * v[4] + v[5] * v[5] + v[6] * v[6]);
        for (int k = 3; k < 7; ++k) v[k] /= n;
        pose[id].assign(v, v + 7);
        stamp[id] = t;
        if (!sb.count(id)) sb[id].assign(9, 0.0);
      } else if (type == "VERTEX_R3:VEL" || type == "VERTEX_R3:ACCBIAS" || type == "VERTEX_R3:GYRBIAS") {
        uint64_t id;
        double a, b, c;
        if (!(ss >> id >> a >> b >> c)) bad("bad " + type);
        if (!sb.count(id)) sb[id].assign(9, 0.0);
        const int off = type == "VERTEX_R3:VEL" ? 0 : (type == "VERTEX_R3:ACCBIAS" ? 6 : 3);
        sb[id][off] = a; sb[id][off + 1] = b; sb[id][off + 2] = c;
      } else if (type == "VERTEX_TRACKXYZ") {
        uint64_t id;
        double x, y, z, q;
        if (!(ss >> id >> x >> y >> z >> q)) bad("bad VERTEX_TRACKXYZ");
        lm[id] = {x, y, z, 1.0};
      } else if (type == "FRAME") {
        uint64_t id;
        int cam;
        long long eid, t;
        double v[7];
        if (!(ss >> id >> cam >> eid >> v[0] >> v[1] >> v[2] >> v[3] >> v[4] >> v[5] >> v[6] >> t)) bad("bad FRAME");
        if (cam < 0 || cam >= n_cameras) bad("FRAME camera index beyond the configured cameras");
        if (extrId[cam] < 0) {
          extrId[cam] = eid;
          const double n = std::sqrt(v[3] * v[3] + v[4] * v[4] + v[5] * v[5] + v[6] * v[6]);
          for (int k = 3; k < 7; ++k) v[k] /= n;
          extr[cam].assign(v, v + 7);
        } else if (extrId[cam] != eid) {
          throw ParseError{"camera " + std::to_string(cam) +
                           " has several extrinsics blocks (online calibration is not supported on the GPU path)"};
        }
        kps[{id, cam}];  // the frame exists even without keypoints
      } else if (type == "FRAME:KEYPOINT") {
        uint64_t id;
        int cam;
        float u, v, size;
        if (!(ss >> id >> cam >> u >> v >> size)) bad("bad FRAME:KEYPOINT");
        kps[{id, cam}].push_back(Keypoint{u, v, size});
      } else if (type == "EDGE_IMU") {
        uint64_t a, b;
        if (!(ss >> a >> b)) bad("bad EDGE_IMU");
        imus.push_back(Imu{a, b, {}, {}});
      } else if (type == "EDGE_IMU:MEASUREMENTS") {
        if (imus.empty()) bad("EDGE_IMU:MEASUREMENTS before EDGE_IMU");
        double acc[3], gyr[3];
        long long t;
        if (!(ss >> acc[0] >> acc[1] >> acc[2] >> gyr[0] >> gyr[1] >> gyr[2] >> t)) bad("bad EDGE_IMU:MEASUREMENTS");
        Imu& f = imus.back();
        f.ga.insert(f.ga.end(), {gyr[0], gyr[1], gyr[2], acc[0], acc[1], acc[2]});
        f.t.push_back(t);
      } else if (type == "EDGE_OBS") {
        uint64_t id, lid;
        int cam, kp;
        if (!(ss >> id >> cam >> kp >> lid)) bad("bad EDGE_OBS");
        obs.push_back(Obs{id, lid, cam, kp});
      } else {
        throw ParseError{"line " + std::to_string(lineNo) + ": unknown type tag " + type};
      }
    }
    // ---- assemble the problem
    std::map<uint64_t, int> stateIdx, lmIdx;
    for (auto& kv : pose) {
      stateIdx[kv.first] = (int)G->state_ids.size();
      G->state_ids.push_back(kv.first);
      G->state_t.push_back(stamp[kv.first]);
      G->poses.insert(G->poses.end(), kv.second.begin(), kv.second.end());
      G->sbs.insert(G->sbs.end(), sb[kv.first].begin(), sb[kv.first].end());
    }
    for (auto& kv : sb)
      if (!pose.count(kv.first)) throw ParseError{"speed/bias vertex without a pose vertex: " + std::to_string(kv.first)};
    for (auto& kv : lm) {
      lmIdx[kv.first] = (int)G->landmark_ids.size();
      G->landmark_ids.push_back(kv.first);
      G->lms.insert(G->lms.end(), kv.second.begin(), kv.second.end());
    }
    for (int c = 0; c < n_cameras; ++c) {
      G->cams.push_back(cameras[c]);
      if (extr[c].empty()) extr[c] = {0, 0, 0, 0, 0, 0, 1};
      G->extr.insert(G->extr.end(), extr[c].begin(), extr[c].end());
    }
    for (const Obs& o : obs) {
      if (!stateIdx.count(o.state)) throw ParseError{"observation of a non-existent state"};
      if (!lmIdx.count(o.lm)) throw ParseError{"observation of a non-existent landmark"};
      auto it = kps.find({o.state, o.cam});
      if (it == kps.end()) throw ParseError{"Observation to non-existant multi-frame"};
      if (o.kp < 0 || o.kp >= (int)it->second.size()) throw ParseError{"observation keypoint index out of range"};
      const Keypoint& k = it->second[o.kp];
      G->obs_pose.push_back(stateIdx[o.state]);
      G->obs_lm.push_back(lmIdx[o.lm]);
      G->obs_cam.push_back(o.cam);
      G->obs_kp.push_back((double)k.u);
      G->obs_kp.push_back((double)k.v);
      // information 64/size^2 I -> squareRootInformation_ = LLT(info).L^T = 8/size I (ViGraph.hpp:324-327)
      const double s = 8.0 / (double)k.size;
      G->obs_L.insert(G->obs_L.end(), {s, 0.0, 0.0, s});
      G->obs_cauchy.push_back(1);
    }
    G->imu_begin.push_back(0);
    for (const Imu& f : imus) {
      if (!stateIdx.count(f.a) || !stateIdx.count(f.b)) throw ParseError{"IMU edge to a non-existent state"};
      const int a = stateIdx[f.a], b = stateIdx[f.b];
      G->imu_blocks.insert(G->imu_blocks.end(), {a, a, b, b});
      G->imu_t0.push_back(G->state_t[a]);
      G->imu_t1.push_back(G->state_t[b]);
      G->imu_ts.insert(G->imu_ts.end(), f.t.begin(), f.t.end());
      G->imu_ga.insert(G->imu_ga.end(), f.ga.begin(), f.ga.end());
      G->imu_begin.push_back((int32_t)G->imu_ts.size());
    }
    G->imu_state.assign(imus.size() * OKVISGPU_IMU_STATE_DOUBLES, 0.0);
    G->pose_const.assign(G->state_ids.size(), 0);
    G->sb_const.assign(G->state_ids.size(), 0);
    G->lm_const.assign(G->landmark_ids.size(), 0);
    finishProblem(*G, *imu);
  } catch (const ParseError& e) {
    std::fprintf(stderr, "okvisgpu_graph_load(%s): %s\n", path, e.msg.c_str());
    delete G;
    return OKVISGPU_ERR_INVALID_ARGUMENT;
  } catch (const std::bad_alloc&) {
    delete G;
    return OKVISGPU_ERR_OUT_OF_MEMORY;
  }
  *out = G;
  return OKVISGPU_OK;
}

const okvisgpu_problem* okvisgpu_graph_problem(okvisgpu_graph* g) { return g ? &g->prob : nullptr; }

int okvisgpu_graph_ids(const okvisgpu_graph* g, uint64_t* state_ids, int64_t* state_t_ns, uint64_t* landmark_ids) {
  if (!g) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (state_ids) std::copy(g->state_ids.begin(), g->state_ids.end(), state_ids);
  if (state_t_ns) std::copy(g->state_t.begin(), g->state_t.end(), state_t_ns);
  if (landmark_ids) std::copy(g->landmark_ids.begin(), g->landmark_ids.end(), landmark_ids);
  return OKVISGPU_OK;
}

void okvisgpu_graph_destroy(okvisgpu_graph* g) { delete g; }

int okvisgpu_graph_save(const okvisgpu_problem* p, const int64_t* state_t_ns, const char* path) {
  if (!p || !path) return OKVISGPU_ERR_INVALID_ARGUMENT;
  if (p->n_speed_biases != p->n_poses) return OKVISGPU_ERR_UNSUPPORTED;  // one speed/bias block per state
  std::ofstream file(path);
  if (!file) return OKVISGPU_ERR_INVALID_ARGUMENT;
  file << std::setprecision(17);
  // state time stamps: given, or the IMU factors' t0 / t1
  std::vector<int64_t> t(p->n_poses, 0);
  if (state_t_ns) {
    std::copy(state_t_ns, state_t_ns + p->n_poses, t.begin());
  } else {
    for (int f = 0; f < p->n_imu; ++f) {
      t[p->imu_blocks[4 * f]] = p->imu_t0_ns[f];
      t[p->imu_blocks[4 * f + 2]] = p->imu_t1_ns[f];
    }
  }
  // per (state, camera) keypoint lists in observation order; per state its observations
  std::vector<std::vector<int>> obsOf(p->n_poses);
  std::vector<int> kpIndex(p->n_observations);
  std::map<std::pair<int, int>, int> kpCount;
  for (int o = 0; o < p->n_observations; ++o) {
    obsOf[p->obs_pose[o]].push_back(o);
    kpIndex[o] = kpCount[{p->obs_pose[o], p->obs_camera[o]}]++;
  }
  std::vector<int> imuInto(p->n_poses, -1);
  for (int f = 0; f < p->n_imu; ++f) imuInto[p->imu_blocks[4 * f + 2]] = f;
  std::vector<uint8_t> written(p->n_landmarks, 0);
  const std::string descriptor(96, '0');
  for (int i = 0; i < p->n_poses; ++i) {
    const double* T = &p->poses[7 * i];
    file << "VERTEX_SE3:QUAT_TIME " << i << " " << T[0] << " " << T[1] << " " << T[2] << " " << T[3] << " " << T[4]
         << " " << T[5] << " " << T[6] << " " << t[i] << "\n";
    const double* s = &p->speed_biases[9 * i];
    file << "VERTEX_R3:VEL " << i << " " << s[0] << " " << s[1] << " " << s[2] << "\n";
    file << "VERTEX_R3:ACCBIAS " << i << " " << s[6] << " " << s[7] << " " << s[8] << "\n";
    file << "VERTEX_R3:GYRBIAS " << i << " " << s[3] << " " << s[4] << " " << s[5] << "\n";
    for (int c = 0; c < p->n_cameras; ++c) {
      const double* E = &p->extrinsics[7 * c];
      file << "FRAME " << i << " " << c << " " << c << " " << E[0] << " " << E[1] << " " << E[2] << " " << E[3] << " "
           << E[4] << " " << E[5] << " " << E[6] << " " << t[i] << "\n";
      for (int o : obsOf[i]) {
        if (p->obs_camera[o] != c) continue;
        // keypoint size from the square-root information 8/size (isotropic information only)
        const double* L = &p->obs_sqrt_info[4 * o];
        file << "FRAME:KEYPOINT " << i << " " << c << " " << (float)p->obs_keypoint[2 * o] << " "
             << (float)p->obs_keypoint[2 * o + 1] << " " << (float)(8.0 / L[0]) << " BRISK2 " << descriptor << "\n";
      }
    }
    const int f = imuInto[i];
    if (f >= 0) {
      file << "EDGE_IMU " << p->imu_blocks[4 * f] << " " << i << "\n";
      for (int k = p->imu_sample_begin[f]; k < p->imu_sample_begin[f + 1]; ++k) {
        const double* ga = &p->imu_sample_gyr_acc[6 * k];
        file << "EDGE_IMU:MEASUREMENTS " << ga[3] << " " << ga[4] << " " << ga[5] << " " << ga[0] << " " << ga[1] << " "
             << ga[2] << " " << p->imu_sample_t_ns[k] << "\n";
      }
    }
    for (int o : obsOf[i]) {
      const int l = p->obs_landmark[o];
      if (!written[l]) {
        const double* h = &p->landmarks[4 * l];
        file << "VERTEX_TRACKXYZ " << l << " " << h[0] / h[3] << " " << h[1] / h[3] << " " << h[2] / h[3] << " " << 1.0
             << "\n";
        written[l] = 1;
      }
      const double* L = &p->obs_sqrt_info[4 * o];
      file << "EDGE_OBS " << i << " " << p->obs_camera[o] << " " << kpIndex[o] << " " << l << " "
           << (float)p->obs_keypoint[2 * o] << " " << (float)p->obs_keypoint[2 * o + 1] << " " << L[0] * L[0] << " "
           << 0.0 << " " << 0.0 << " " << L[3] * L[3] << "\n";
    }
  }
  return file.good() ? OKVISGPU_OK : OKVISGPU_ERR_INVALID_ARGUMENT;
}

}  // extern "C"
