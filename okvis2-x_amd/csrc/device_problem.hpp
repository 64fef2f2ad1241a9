// device_problem.hpp — HBM layout of a batch of sliding windows and the per-window trust-region
// state. One flat, window-concatenated array per quantity so that every kernel covers the whole
// batch in one launch (batch index = window; SURVEY.md §8e "replicas only" sharding).
//
// Index spaces (all global over the batch):
//   pose p in [0, n_pose)   sb s in [0, n_sb)   landmark l in [0, n_lm)   obs o in [0, n_obs)
//   visit v in [0, n_visit) : maximal run of observations of ONE landmark from ONE pose (stereo
//                             pairs of a keyframe aggregate into one visit); obs sorted by
//                             (window, landmark, pose, camera)
//   imu factor f in [0, n_imu)
//   f-vector index: the reduced ("camera") system of window w occupies [foff[w], foff[w]+fdim[w])
//   S of window w: dense row-major fpad[w] x fpad[w] at soff[w] (lower triangle used), padded to a
//   multiple of 64 with identity on the padded diagonal.
#pragma once

#include <cstdint>

namespace okg {

constexpr int kCamDoubles = 13;       // per camera on the device: dist, fu, fv, cu, cv, 8 distortion parameters
constexpr int kTile = 64;             // Cholesky tile (one 64x64 FP64 tile = 32 KiB of LDS)
constexpr int16_t kNoUpdate = 32767;  // tile_fu of a tile no band update writes
constexpr int kImuLin = 15 + 15 * 30; // per-IMU-factor linearisation record: r[15], J[15][30]
constexpr int kImuState = 526;        // == OKVISGPU_IMU_STATE_DOUBLES
// host-evaluated factor records: in = live flag (0 idle, 1 + linearisation buffer) | pad | slot
// values pose0 (7) @8, sb0 (9) @15, pose1 (7) @24, sb1 (9) @31; out = cost | r[15] | J[15][30]
constexpr int kHostIn = 40;
constexpr int kHostOut = 1 + kImuLin;

// Linearisation record per observation (structure of arrays, plane-major):
//   plane 0-1: r (Cauchy-corrected)   plane 2-13: J_pose 2x6   plane 14-19: J_lm 2x3
constexpr int kObsLin = 8;   // r (2) | A = L Jh C_CW (2x3), Cauchy-scaled
constexpr int kSegHG = 28;   // per visit segment: H = sum J_p^T J_p (21, sym packed) | g = sum J_p^T r (6) | pad
constexpr int kSegUz = 8;    // per visit segment: sum U z (6) | pad
constexpr int kLmGroupVisits = 256;  // k_lm_visit: visits of one landmark group (one workgroup)
// A batch of at most a quarter window per CU: the latency regime (per-window reductions at 1,024
// threads, fused launches of the iteration's independent small kernels).
__host__ __device__ constexpr bool fewWindows(int nWin, int cuCount) { return 4 * nWin <= cuCount; }
constexpr int kLmGroupMax = 64;      // landmarks per group
constexpr int kLmPartStage = 2048;   // landmark-pair products per group (staged in LDS)
constexpr int kAsmLightMax = 24;     // contributions of a pose-pose pair assembled by a 16-lane quarter
constexpr int kManyWindows = 64;     // batches from this size use the fewer-workgroup layouts (light
                                     // pairs, several S tiles per workgroup); below it latency rules
constexpr int kLmgInfo = 8;          // ints per landmark-group record (lmg_info)
constexpr int kImuHess = 465 + 30;  // packed upper J^T J (30x30) | J^T r
constexpr int kGrpRed = 8;    // per landmark group: jcc | jgg | jcg | gg | nn | gn | pad
constexpr int kVisitZ = 18;   // per visit: Z = s_p W s_l L^-T (6x3), k_lm_visit LDS only

// contribution record types for the reduced-system assembly
enum ContribType : int32_t {
  C_VISIT = 0,      // a = visit segment: summed Hpp / gp / U z of one pose's visits in a landmark group
  C_PAIR = 1,       // a = partial Schur block: sum over a landmark group of Z_a Z_b^T (= W_a V^-1 W_b^T)
  C_IMU = 2,        // a = factor, b = column offset of row block, c = column offset of col block
  C_PPRIOR = 3,     // a = pose prior
  C_SBPRIOR = 4,    // a = sb prior
  C_RELPOSE = 5,    // a = relative-pose edge, b / c = column offset (0 reference, 6 other) of row / col block
  C_PEXT = 6        // a = pose-extrinsics record: sum J_e^T J_p (row = extrinsics block, col = state pose)
};
constexpr int kRelPoseLin = 6 + 6 * 12;  // per relative-pose edge: r[6] | J minimal 6x12 (reference 6 | other 6)

struct Contrib {
  int32_t type, a, b, c;
};


struct WinState {
  double radius, mu;
  double x_cost, cand_cost, fixed_cost, initial_cost, min_cost;
  double x_norm, step_norm;
  double alpha, dogleg_step_norm, model_cost_change;
  double grad_max_norm, grad_norm;
  double z_mu;                     // mu the stored Z operands were formed with (-1: none)
  double jcc, jgg, jcg;            // |J_s v_c|^2, |J_s v_g|^2, (J_s v_c).(J_s v_g) of the current GN / Cauchy pair
  int32_t xcur, lcur;              // current parameter set / linearisation buffer (0/1)
  int32_t need_gn;                 // !DoglegStrategy::reuse_
  int32_t done, termination;
  int32_t iteration, num_succ, num_unsucc, consecutive_invalid;
  int32_t gn_failed;               // Cholesky / 3x3 inverse failure in this GN attempt
  int32_t eval_cand;               // candidate must be evaluated this iteration
  int32_t step_valid;
  int32_t accepted;
  int32_t dev_error;               // a kernel gave up on this window (pipelined Cholesky wait limit):
                                   // the host reports OKVISGPU_ERR_DEVICE, not a failed GN step
  int32_t pad_[2];
};

// Options mirrored on the device (okvisgpu_options subset used inside kernels).
struct DevOptions {
  int32_t max_num_iterations;
  int32_t jacobi_scaling;
  int32_t max_num_consecutive_invalid_steps;
  int32_t redo_propagation_always;
  double function_tolerance, gradient_tolerance, parameter_tolerance;
  double initial_radius, max_radius, min_radius;
  double min_relative_decrease, min_lm_diagonal, max_lm_diagonal;
};

struct DevProblem {
  const DevProblem* self;          // device-resident copy of this descriptor (what kernels receive)
  int32_t n_win, n_pose, n_sb, n_lm, n_obs, n_visit, n_imu, n_pprior, n_sbprior, n_cam;
  int32_t cu_count;                // compute units of the device (persistent-style grids)
  int32_t lin_prep;                // host only: GN prep inside the linearisation launch (1 / 0),
                                   // fixed per solve (lin_runs_prep); -1 = not yet decided
  int32_t n_fblock, n_pair;
  int32_t max_fpad, max_tiles;     // largest padded reduced dimension / its 64-tile count
  int64_t obs_stride;              // plane stride of the obs linearisation SoA (>= n_obs)

  // --- parameters, two sets (current / candidate), ambient
  double* pose[2];                 // [n_pose][7]
  double* sb[2];                   // [n_sb][9]
  double* lm[2];                   // [n_lm][4]
  const double* extr;              // [n_cam][7] initial T_SC (twopose / reference only; solves read pose-kind blocks)
  const int32_t* cam_pose;         // [n_cam] pose-kind block holding camera c's T_SC (after the window's states)
  const double* cam;               // [n_cam][kCamDoubles]: dist, fu, fv, cu, cv, d0..d7 (dist as double)

  // --- per-block window id and reduced-system offsets (-1: not a free f-block / e-block)
  const int32_t* pose_win;         // [n_pose]
  const int32_t* sb_win;
  const int32_t* lm_win;
  const int32_t* pose_f;           // [n_pose] offset in the window's f-vector, -1 if not free
  const int32_t* sb_f;             // [n_sb]
  const uint8_t* lm_free;          // [n_lm] 1 = e-block
  const uint8_t* pose_active;      // [n_pose] active (free & used) — included in norms / Plus
  const uint8_t* sb_active;

  // --- observations (sorted)
  const int32_t* obs_pose;         // global pose index
  const int32_t* obs_lm;           // global landmark index
  const int32_t* obs_cam;          // global camera index
  const int32_t* obs_win;
  const uint8_t* obs_flags;        // bit0 cauchy, bit1 fixed (all blocks constant)
  const double* obs_kp;            // [n_obs][2]
  const double* obs_L;             // [n_obs][4]
  const double* obs_Ls;            // [n_obs] s of L = diag(s, s) when obs_iso
  int32_t obs_iso;                 // every observation's L is diag(s, s) (runtime.cpp build)
  double* obs_lin[2];              // [kObsLin][obs_stride]; lin[lcur] belongs to params X[xcur]
  double* obs_cost[2];             // [n_obs]
  double* grp_red;                 // [n_lmg][kGrpRed]: per landmark group (k_lm_backsub_jv), fixed-order
                                   // sums jcc | jgg | jcg over its residuals and |grad_l|^2 | |gn_l|^2 |
                                   // grad_l . gn_l over its free landmarks (k_reduce, k_dogleg)

  // --- landmarks / visits
  const int32_t* lm_visit_begin;   // [n_lm+1] visits of landmark l
  const int32_t* visit_pose;       // [n_visit]
  const int32_t* visit_obs_begin;  // [n_visit+1]
  const int32_t* visit_lm;         // [n_visit]
  double* lm_V;                    // [n_lm][6]  sum J_l^T J_l (unscaled, sym packed 00 01 02 11 12 22)
  double* lm_g;                    // [n_lm][3]  J_l^T r
  double* lm_Linv;                 // [n_lm][9]  L^-1, L L^T = s V s + D^2 (lower triangular)
  double* lm_zz;                   // [n_lm][3]  L^-1 (s g)
  const int32_t* lmg_begin;        // [n_lmg+1] landmark groups of k_lm_visit (<= kLmGroupVisits visits each)
  const int32_t* lmg_info;         // [n_lmg+1][kLmgInfo] {first landmark, first visit, window, first segment,
                                   //  first partial block, first landmark-pair product, 0, 0}
  int32_t n_lmg;
  // visit segments: the visits of one free pose inside one landmark group, pre-summed in k_lm_visit
  int32_t n_seg;
  const int32_t* seg_gbegin;       // [n_lmg+1] segments of group g
  const int32_t* seg_pose;         // [n_seg] global pose
  const int32_t* seg_range;        // [n_seg][2] slot range of the segment's visits within its group
  const int32_t* visit_slot;       // [n_visit] slot in the group's (pose, visit) order, -1: pose not free
  double* seg_hg;                  // [n_seg][kSegHG] H (21, sym packed) | g (6), unscaled
  double* seg_uz;                  // [n_seg][kSegUz] U z (6)
  // partial Schur blocks: per landmark group and pose pair, P = sum Z_a Z_b^T (6x6, row-major)
  int32_t n_part;
  const int32_t* part_gbegin;      // [n_lmg+1] partial blocks of group g
  const int32_t* part_cbegin;      // [n_part+1] CSR into part_contrib
  const int32_t* part_contrib;     // (a | b << 16): visit offsets within the group
  double* part_S;                  // [n_part][36]
  // extrinsic visits (variable extrinsics only): per (landmark, variable camera) the landmark's
  // observations through that camera; threads nvg.. of their landmark group (k_lm_visit<.., true>)
  int32_t n_xvisit;
  const int32_t* xvisit_pose;      // [n_xvisit] pose-kind block of the extrinsics
  const int32_t* xvisit_lm;        // [n_xvisit]
  const int32_t* xvisit_obs_begin; // [n_xvisit+1] CSR into xvisit_obs
  const int32_t* xvisit_obs;       // global observation indices
  const int32_t* xvisit_slot;      // [n_xvisit] segment slot within the group
  const int32_t* lmg_xbegin;       // [n_lmg+1] extrinsic visits of group g
  // pose-extrinsics cross blocks (k_pose_extr): per (free state pose, variable camera)
  int32_t n_pe;
  const int32_t* pe_pose;          // [n_pe] state pose
  const int32_t* pe_ext;           // [n_pe] pose-kind block of the extrinsics
  const int32_t* pe_obs_begin;     // [n_pe+1] CSR into pe_obs
  const int32_t* pe_obs;
  double* pe_H;                    // [n_pe][36] sum J_e^T J_p (row-major, rows = extrinsics)

  // --- IMU factors [0, n_imu) and host-evaluated factors [n_imu, n_fac) (okvisgpu_problem host_*,
  // ABI 5): both are <= 15-row factors on <= 2 pose-kind + 2 speed/bias blocks in the same column
  // layout, so the linearisation, J^T J, assembly, J*v and cost kernels treat them alike; only the
  // evaluation differs (k_eval_imu on the device; k_host_gather -> host callback -> k_host_scatter)
  int32_t n_host, n_fac;
  const int32_t* imu_blocks;       // [n_fac][4] global pose0 sb0 pose1 sb1 (host factors: -1 = unused slot)
  const int32_t* imu_win;          // [n_fac]
  const uint8_t* imu_flags;        // [n_fac] bit1 fixed
  const int64_t* imu_t0;
  const int64_t* imu_t1;
  const int32_t* imu_sbegin;       // [n_imu+1]
  const int64_t* imu_ts;
  const double* imu_ga;            // [n_samples][6]
  const double* imu_par;           // [n_win][7]: a_max g_max sigma_g_c sigma_a_c sigma_gw_c sigma_aw_c g
  double* imu_state;               // [n_imu][kImuState]
  double* imu_lin[2];              // [n_fac][kImuLin]
  double* imu_cost[2];             // [n_fac]
  double* imu_H;                   // [n_fac][kImuHess] of the linearisation lin[lcur] (k_imu_hess)
  double* imu_jv;                  // [3][n_fac]
  const int32_t* win_host_range;   // [n_win][2] host factors of the window (global factor indices)
  double* host_in;                 // [n_host][kHostIn] gathered evaluation points (k_host_gather)
  double* host_out;                // [n_host][kHostOut] host results, uploaded (k_host_scatter)

  // --- priors
  const int32_t* pp_block;         // [n_pprior] global pose
  const int32_t* pp_win;
  const double* pp_meas;           // [n][7]
  const double* pp_L;              // [n][36]
  double* pp_lin[2];               // [n][6 + 36]
  double* pp_cost[2];
  double* pp_jv;                   // [3][n]
  const int32_t* sbp_block;
  const int32_t* sbp_win;
  const double* sbp_meas;          // [n][9]
  const double* sbp_L;             // [n][81]
  double* sbp_lin[2];              // [n][9 + 81]
  double* sbp_cost[2];
  double* sbp_jv;

  // --- relative-pose (pose-graph) edges, TwoPoseStandardGraphError(Const)
  int32_t n_relpose;
  const int32_t* rp_blocks;        // [n][2] global reference pose, other pose
  const int32_t* rp_win;
  const uint8_t* rp_flags;         // bit1 fixed (both poses constant)
  const uint8_t* rp_kind;          // 0 TwoPoseStandardGraphError(Const), 1 RelativePoseError
  const double* rp_dx;             // [n][6]  DeltaX_
  const double* rp_J;              // [n][36] J_
  const double* rp_lp;             // [n][7]  linearisationPoint_T_S0S1_
  double* rp_lin[2];               // [n][kRelPoseLin]
  double* rp_cost[2];
  double* rp_jv;                   // [3][n]

  // --- reduced system structure
  const int32_t* win_foff;         // [n_win]
  const int32_t* win_fdim;
  const int32_t* win_fpad;
  const int64_t* win_soff;         // [n_win] offset of S
  const int32_t* win_pose_range;   // [n_win][2]
  const int32_t* win_sb_range;
  const int32_t* win_lm_range;
  const int32_t* win_lmg_range;    // [n_win][2] landmark groups of the window
  const int32_t* win_obs_range;
  const int32_t* win_imu_range;
  const int32_t* win_pp_range;
  const int32_t* win_sbp_range;
  const int32_t* win_rp_range;
  const int32_t* fb_win;           // [n_fblock] window
  const int32_t* fb_kind;          // 0 pose / 1 sb
  const int32_t* fb_index;         // global pose / sb index
  const int32_t* fb_off;           // offset in the window's f-vector
  const int32_t* win_sgap;         // [n_win][2] f offset and length of the gap rows of a nested-
                                   // dissection order (identity rows of S, zero rhs; 0 0: none)
  const int32_t* win_bsplit;       // [n_win][2] tiles tL, tS: left part [0, tL), right part [tL, tS),
                                   // separator [tS, T) of the backward substitution (0 0: no split)
  const int32_t* fb_cbegin;        // [n_fblock+1] gradient / diagonal contributions (C_VISIT, C_IMU, priors)
  const Contrib* fb_contrib;
  const int32_t* asm_pp_items;      // pose-pose pairs, one per wavefront, XCD-grouped order (-1 = pad)
  const int32_t* asm_sb_items;      // pairs with a speed/bias block, one per wavefront
  int32_t n_asm_pp, n_asm_sb;
  const int32_t* asm_ppl_items;     // light pose-pose pairs (off-diagonal, few contributions): 16 lanes each
  int32_t n_asm_ppl;
  const int32_t* pair_win;         // [n_pair]
  const int32_t* pair_fi;          // global f-block index (row, fi >= fj)
  const int32_t* pair_fj;
  const int32_t* pair_cbegin;      // [n_pair+1]
  const int32_t* pair_runs;        // [n_pair][2] start of the landmark-pair run, start of the factor run
  const Contrib* pair_contrib;

  // --- f-vectors (window-concatenated, reduced ordering) and landmark vectors
  double* S;                       // sum over windows fpad^2: the assembled reduced matrix (the
                                   // factorisation never writes it: its entries outside the
                                   // assembled blocks stay zero from the build, no clearing per iteration)
  double* W;                       // same layout: the factorisation's working tiles (updated tiles, L)
  double* Linv;                    // per window (fpad/64) inverses of the 64x64 diagonal factors
  const int64_t* win_linvoff;      // [n_win] offset into Linv
  // tile-level symbolic factorisation (host analysis): the reduced camera matrix of a sliding
  // window is block-banded and LLT creates no fill outside its envelope, so only structurally
  // non-zero 64x64 tiles are zeroed, factored and updated (bitwise identical to the dense LLT).
  const int32_t* tile_items;         // (w, i, j) every structurally non-zero tile (i >= j)
  // tile-parallel schedule (few windows; runtime.cpp cholSchedule): launch 0 factors the root tiles
  // (w, d, first root of the window), launch l >= 1 runs the band-update items (w, i, j,
  // mode | k << 8) scheduled there; begin offsets per launch, host copy for the launch sizes
  const int32_t* chol_root_items;
  int32_t n_chol_roots;
  int32_t n_chol_launches;
  const int32_t* chol_upd_items;
  const int32_t* chol_upd_begin;
  const int32_t* h_upd_begin;
  int32_t chol_schedule;             // 1 persistent per window, 2 tile-parallel (host-resolved)
  const uint8_t* tile_nz;            // per window T x T (row-major) structural non-zero flags of L
  const int16_t* tile_fu;            // per window T x T (same offsets): the first step whose band update
                                     // writes tile (i, j) (kNoUpdate if none): before it the tile is read from S
  const int64_t* win_tnzoff;         // [n_win] offset of the window's flags in tile_nz
  int32_t n_tiles;
  double* chol_defer;              // split persistent schedule: the right part's rhs contributions
  const int64_t* win_defoff;       //   to the separator's rows, [T - tS][tS - tL][64] per window
  double* fwdF;                    // per window fpad: forward-substitution work vector
  const int64_t* win_fwdoff;       // [n_win] offset into fwdF
  double* sF;   double* sL;        // Jacobi scaling (fixed at iteration 0)
  double* diagF; double* diagL;    // dogleg diagonal_
  double* hdF;                     // unscaled diag(H_ff)
  double* gF;   double* gL;        // unscaled gradient J^T r
  double* rhsF;                    // Schur rhs / forward-substitution workspace
  double* yF;   double* yL;        // GN solution (Jacobi-scaled space)
  double* gnF;  double* gnL;       // gauss_newton_step_ (dogleg-scaled)
  double* dgF;  double* dgL;       // gradient_ (dogleg-scaled)
  double* vF;   double* vL;        // J*v operand (Jacobi-scaled space)
  double* stepF; double* stepL;    // trust-region step (Jacobi-scaled space)

  WinState* st;                    // [n_win]
  DevOptions opt;
};

// Batch of TwoPoseStandardGraphError::compute inputs (okvisgpu_twopose_edges on device) and the
// per-edge output record: DeltaX_ [6] | J_ [36] | linearisation point [7] | H00_ [36] | b0_ [6].
constexpr int kTwoPoseOut = 6 + 36 + 7 + 36 + 6;
struct TwoPoseDev {
  int32_t n_edges, n_cam;
  const double* ref_pose;     // [n_edges][7]
  const double* other_pose;   // [n_edges][7]
  const double* cam;          // [n_cam][kCamDoubles] as DevProblem::cam
  const double* extr;         // [n_cam][7]
  const int32_t* lm_begin;    // [n_edges+1]
  const double* lm;           // [n_lm][4]
  const int32_t* obs_begin;   // [n_lm+1]
  const uint8_t* obs_other;   // [n_obs]
  const int32_t* obs_cam;
  const double* obs_kp;       // [n_obs][2]
  const double* obs_L;        // [n_obs][4]
  const uint8_t* obs_cauchy;  // [n_obs]
  double* out;                // [n_edges][kTwoPoseOut]
};

}  // namespace okg
