/*
 * okvisgpu.h — C ABI of the MI355X-native sliding-window bundle-adjustment backend.
 *
 * This is the drop-in boundary that replaces `::ceres::Solve(options_, problem_.get(), &summary_)`
 * inside `okvis::ViGraph::optimise()` (reference: okvis_ceres/src/ViGraph.cpp:1844-1890, the call
 * itself at :1884). Everything the reference hands to Ceres through the `::ceres::Problem` subset
 *  is handed over here as plain structure-of-arrays host buffers; the library copies
 * them to device memory, solves on the GPU, and writes the optimised parameter blocks back into
 * the SAME caller-owned host arrays (the reference's in-place ParameterBlock semantics,
 * okvis_ceres/include/okvis/ceres/PoseParameterBlock.hpp:62-78).
 *
 * Conventions (all FP64, host memory, caller-owned; the library never frees caller memory):
 *   pose / extrinsics block : [t_x t_y t_z q_x q_y q_z q_w]   (PoseParameterBlock, 7 doubles)
 *   speed-and-bias block    : [v(3) b_g(3) b_a(3)]            (SpeedAndBiasParameterBlock, 9)
 *   landmark block          : [x y z w] homogeneous            (HomogeneousPointParameterBlock, 4)
 *   time stamps             : int64 nanoseconds (okvis::Time sec/nsec, okvis_time/.../Time.hpp:124)
 *
 * No C++ exceptions cross this boundary. Every entry point returns an okvisgpu_status; the text
 * of the last error of a context is available from okvisgpu_last_error().
 *
 * Threading (SURVEY.md §8b "Threading"): one okvisgpu_ctx per graph (realtime graph, full graph);
 * each context owns one HIP stream and its device buffers. Entry points are re-entrant across
 * contexts, not within one.
 */
#ifndef OKVISGPU_H_
#define OKVISGPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OKVISGPU_ABI_VERSION 6

/* ---------------------------------------------------------------- status codes */
typedef enum okvisgpu_status {
  OKVISGPU_OK = 0,
  OKVISGPU_ERR_INVALID_ARGUMENT = 1,
  OKVISGPU_ERR_UNSUPPORTED = 2,     /* a problem feature the GPU path does not implement yet */
  OKVISGPU_ERR_DEVICE = 3,          /* HIP runtime error / no device / kernel image missing   */
  OKVISGPU_ERR_OUT_OF_MEMORY = 4,
  OKVISGPU_ERR_NO_PROBLEM = 5,
  OKVISGPU_ERR_NUMERICAL = 6
} okvisgpu_status;

/* ---------------------------------------------------------------- enums mirroring Ceres/okvis */
typedef enum okvisgpu_distortion {
  OKVISGPU_DIST_NONE = 0,           /* okvis_cv/.../NoDistortion.hpp */
  OKVISGPU_DIST_RADTAN = 1,         /* okvis_cv/.../implementation/RadialTangentialDistortion.hpp:70-137 */
  OKVISGPU_DIST_EQUIDISTANT = 2,    /* okvis_cv/.../implementation/EquidistantDistortion.hpp:67-188 */
  OKVISGPU_DIST_RADTAN8 = 3         /* okvis_cv/.../implementation/RadialTangentialDistortion8.hpp:88-170 */
} okvisgpu_distortion;

typedef enum okvisgpu_linear_solver {
  OKVISGPU_DENSE_SCHUR = 0,         /* ViSlamBackend.cpp:877 realtime graph */
  OKVISGPU_SPARSE_NORMAL_CHOLESKY = 1 /* ViGraph.cpp:248 (full graph, ViSlamBackend.cpp:1988-1997):
                                       the Gauss-Newton step solves the same normal equations; it
                                       is computed through the exact tile-sparse Schur complement
                                       (landmarks eliminated, band-envelope LLT of the reduced
                                       matrix), so both options give the same step up to rounding */
} okvisgpu_linear_solver;

typedef enum okvisgpu_tr_strategy {
  OKVISGPU_DOGLEG = 0               /* ViGraph.cpp:249 (traditional dogleg) */
} okvisgpu_tr_strategy;

typedef enum okvisgpu_termination {  /* ::ceres::TerminationType subset */
  OKVISGPU_CONVERGENCE = 0,
  OKVISGPU_NO_CONVERGENCE = 1,
  OKVISGPU_FAILURE = 2,
  OKVISGPU_USER_SUCCESS = 3         /* CeresIterationCallback time limit (CeresIterationCallback.cpp:30-38) */
} okvisgpu_termination;

/* ---------------------------------------------------------------- problem description */
typedef struct okvisgpu_camera {
  int32_t distortion;               /* okvisgpu_distortion */
  int32_t width, height;
  double fu, fv, cu, cv;            /* PinholeCamera intrinsics (PinholeCamera.hpp:288-366) */
  double dist[8];                   /* radtan: k1 k2 p1 p2 ; equidistant: k1 k2 k3 k4 ;
                                       radtan8: k1 k2 p1 p2 k3 k4 k5 k6 (unused entries 0) */
} okvisgpu_camera;

typedef struct okvisgpu_imu_params { /* okvis::ImuParameters subset, okvis_common/.../Parameters.hpp:89-105 */
  double a_max, g_max;
  double sigma_g_c, sigma_a_c, sigma_gw_c, sigma_aw_c;
  double g;
} okvisgpu_imu_params;

/* ---------------------------------------------------------------- robust losses (ABI 6)
 * The ::ceres::LossFunction family (ceres-solver >= 2.1 loss_function.h; un-vendored submodule,
 * SURVEY.md §8c). okvis builds four losses in ViGraph's constructor (ViGraph.cpp:235-238):
 * CauchyLoss(1.0) for reprojections (:338) and Cauchy-robustified submap alignment (:1505),
 * CauchyLoss(3.0) for GPS (:88,:999,:1408), TukeyLoss(2.0) / TukeyLoss(0.1) for LiDAR / depth submap
 * alignment (:1510,:1513). rho(s) of the squared residual norm s, with rho[1] = rho', rho[2] = rho'':
 *   CAUCHY(a)      b = a^2:  b log(1 + s/b)
 *   TUKEY(a)       s <= a^2: a^2/3 (1 - (1 - s/a^2)^3), else a^2/3
 *   HUBER(a)       s <= a^2: s, else 2 a sqrt(s) - a^2
 *   SOFTLONE(a)    2 a^2 (sqrt(1 + s/a^2) - 1)
 *   ARCTAN(a)      a atan2(s, a)
 *   TOLERANT(a, b) b log(1 + exp((s - a)/b)) - b log(1 + exp(-a/b))
 * The backend applies Ceres' Corrector (restated by okvis at TwoPoseGraphError.cpp:292-337): cost
 * 1/2 rho(s); for rho'' <= 0 (or s = 0) r and J scaled by sqrt(rho'); for rho'' > 0 (TOLERANT) the
 * second-order correction alpha = 1 - sqrt(1 + 2 s rho''/rho'), r scaled by sqrt(rho')/(1 - alpha),
 * J <- sqrt(rho') (I - alpha/s r r^T) J. */
typedef enum okvisgpu_loss_kind {
  OKVISGPU_LOSS_NONE = 0,           /* nullptr loss (TrivialLoss)                                */
  OKVISGPU_LOSS_CAUCHY = 1,
  OKVISGPU_LOSS_TUKEY = 2,
  OKVISGPU_LOSS_HUBER = 3,
  OKVISGPU_LOSS_SOFTLONE = 4,
  OKVISGPU_LOSS_ARCTAN = 5,
  OKVISGPU_LOSS_TOLERANT = 6
} okvisgpu_loss_kind;

typedef struct okvisgpu_loss {
  int32_t kind;                     /* okvisgpu_loss_kind                                        */
  int32_t reserved;                 /* 0                                                          */
  double a, b;                      /* scale a (> 0); b: TOLERANT's width (> 0), else unused      */
} okvisgpu_loss;

/* rho[3] = (rho(s), rho'(s), rho''(s)) of a loss, as ::ceres::LossFunction::Evaluate (host only).
 * OKVISGPU_ERR_INVALID_ARGUMENT for an unknown kind or a non-positive scale. */
int okvisgpu_loss_evaluate(const okvisgpu_loss* loss, double s, double* rho);

/* Size (doubles) of one ImuError's persistent preintegration state (in/out, see imu_state). Layout:
 *  [0]       redo counter (0 => never integrated; first Evaluate integrates, ImuError.cpp:837)
 *  [1]       redo_ flag
 *  [2..5]    Delta_q (x y z w)        [6..14]   C_integral (row-major)
 *  [15..23]  C_doubleintegral         [24..26]  acc_integral
 *  [27..29]  acc_doubleintegral       [30..38]  dalpha_db_g
 *  [39..47]  dv_db_g                  [48..56]  dp_db_g
 *  [57..65]  speedAndBiases_ref_ (9)  [66..290] squareRootInformation_ (15x15 row-major)
 *  [291]     steps integrated by the last redo (informational)
 *  [292..300] cross_ (row-major)       [301..525] P_delta_ (15x15, symmetric): what
 *            ImuError::append continues from (ABI 4)                                          */
#define OKVISGPU_IMU_STATE_DOUBLES 526

/* Host-evaluated residual block (ABI 5; SURVEY.md §8b fallback): the contract of
 * ::ceres::CostFunction::Evaluate(parameters, residuals, jacobians) plus the caller's user pointer
 * and the factor's index within its window. parameters[k] holds the ambient values of the factor's
 * k-th parameter block (pose-kind 7, speed/bias 9); residuals[dim]; jacobians[k] the row-major
 * dim x ambient-size Jacobian of block k (always requested: the backend evaluates r and J together
 * at every point it evaluates). The backend applies the pose manifold itself (PoseManifold plus
 * Jacobian, PoseLocalParameterization.cpp:56-68), as Ceres does for a block with a manifold.
 * Return nonzero on success; 0 makes the evaluation fail (a candidate point is then rejected, as
 * Ceres does with candidate_cost = max; a failure at the initial point ends the window's solve with
 * OKVISGPU_FAILURE). Called concurrently from up to options.num_threads host threads.
 * The calls are made from a host node of the context's captured iteration graph (hipLaunchHostFunc):
 * the HIP runtime's callback thread fans them out to the context's persistent worker threads while
 * the context's stream waits. A callback must therefore not call HIP or any okvisgpu_* function (it
 * would wait on the stream it is blocking: deadlock); it may only read its parameters and its own
 * data and write residuals / jacobians. */
typedef int (*okvisgpu_host_evaluate_fn)(void* user, int32_t factor, const double* const* parameters,
                                         double* residuals, double** jacobians);
#define OKVISGPU_HOST_MAX_RESIDUALS 15

typedef struct okvisgpu_problem {
  /* --- parameter blocks (written back in place by okvisgpu_solve / okvisgpu_get_params) */
  int32_t n_poses;
  double* poses;                    /* [n_poses][7] T_WS                                       */
  const uint8_t* pose_constant;     /* [n_poses] 1 = SetParameterBlockConstant (may be NULL)    */
  int32_t n_speed_biases;
  double* speed_biases;             /* [n_speed_biases][9]                                     */
  const uint8_t* speed_bias_constant;
  int32_t n_landmarks;
  double* landmarks;                /* [n_landmarks][4]                                        */
  const uint8_t* landmark_constant;
  int32_t n_cameras;
  const okvisgpu_camera* cameras;   /* [n_cameras]                                             */
  double* extrinsics;               /* [n_cameras][7] T_SC, one block per camera shared by all
                                       states (ViGraph::addStatesPropagate re-uses the block,
                                       ViGraph.cpp:469-473); written back when variable          */

  /* --- ReprojectionError<PinholeCamera<D>> residual blocks (ViGraph.hpp:307-352) */
  int32_t n_observations;
  const int32_t* obs_pose;          /* [n_obs] pose block index                                */
  const int32_t* obs_landmark;      /* [n_obs] landmark block index                            */
  const int32_t* obs_camera;        /* [n_obs] camera / extrinsics index                       */
  const double* obs_keypoint;       /* [n_obs][2] measurement_                                 */
  const double* obs_sqrt_info;      /* [n_obs][4] squareRootInformation_ = LLT(info).L^T, row-major
                                       (ReprojectionError.hpp:49-57; info = 64/size^2 I)         */
  const uint8_t* obs_cauchy;        /* [n_obs] 1 = CauchyLoss(1.0) (ViGraph.cpp:235), NULL = all */

  /* --- ImuError residual blocks (ImuError.cpp:797-1003), parameter order (pose0, sb0, pose1, sb1) */
  int32_t n_imu;
  const int32_t* imu_blocks;        /* [n_imu][4] pose0 sb0 pose1 sb1                           */
  const int64_t* imu_t0_ns;         /* [n_imu]                                                  */
  const int64_t* imu_t1_ns;         /* [n_imu]                                                  */
  const int32_t* imu_sample_begin;  /* [n_imu+1] CSR into the sample arrays                     */
  const int64_t* imu_sample_t_ns;   /* [n_samples]                                              */
  const double* imu_sample_gyr_acc; /* [n_samples][6] gyroscopes(3) accelerometers(3)           */
  okvisgpu_imu_params imu_params;
  double* imu_state;                /* [n_imu][OKVISGPU_IMU_STATE_DOUBLES] in/out, NULL = fresh  */

  /* --- PoseError priors (PoseError.cpp:73-125) */
  int32_t n_pose_priors;
  const int32_t* pose_prior_block;  /* [n] pose index                                           */
  const double* pose_prior_meas;    /* [n][7]                                                   */
  const double* pose_prior_sqrt_info; /* [n][36] row-major                                      */

  /* --- SpeedAndBiasError priors (SpeedAndBiasError.cpp:67-101) */
  int32_t n_sb_priors;
  const int32_t* sb_prior_block;
  const double* sb_prior_meas;      /* [n][9]                                                   */
  const double* sb_prior_sqrt_info; /* [n][81] row-major                                        */

  /* --- TwoPoseStandardGraphError / TwoPoseStandardGraphErrorConst residual blocks: relative-pose
   * (pose-graph) edges that marginalisation leaves between two keyframes of the window
   * (TwoPoseGraphError.cpp:467-606 and :631-767; added without a loss function at
   * ViGraphEstimator.cpp:770). Parameter order (reference pose, other pose). The edge is the output
   * of TwoPoseStandardGraphError::compute (okvisgpu_twopose_compute below). */
  int32_t n_relpose;
  const int32_t* relpose_blocks;    /* [n][2] reference pose, other pose                        */
  const double* relpose_delta_x;    /* [n][6] DeltaX_                                           */
  const double* relpose_sqrt_info;  /* [n][36] J_ row-major (information = J_^T J_)             */
  const double* relpose_lin_point;  /* [n][7] linearisationPoint_T_S0S1_                        */
  /* [n] residual kind (may be NULL = all 0):
   *   0 TwoPoseStandardGraphError(Const): r = J_ (DeltaX_ + [r_S0S1 - r_lin; 2 vec(q_S0S1 q_lin^-1)])
   *   1 RelativePoseError (RelativePoseError.cpp:59-140, added by ViGraph::addRelativePoseConstraint,
   *     ViGraph.cpp:786-808, no loss): relpose_lin_point = the measured T_AB, relpose_sqrt_info =
   *     LLT(information).L^T, relpose_delta_x unused;
   *     r = L [r_AB_meas - r_AB; 2 vec(q_AB_meas q_AB^-1)], T_AB = T_WA^-1 T_WB                 */
  const uint8_t* relpose_kind;

  /* --- ABI 4: variable extrinsics (online calibration, do_extrinsics: true; ViGraph.cpp:330-386)
   * extrinsics_constant [n_cameras]: 0 = the camera's T_SC block is variable (NULL = all constant,
   * do_extrinsics: false). Its PoseError prior, PoseError(T_SC, sigma_r^2, sigma_alpha^2)
   * (ViGraph.cpp:372-382, PoseError.cpp:73-125), comes through the extrinsics_prior_* arrays. */
  const uint8_t* extrinsics_constant;
  int32_t n_extrinsics_priors;
  const int32_t* extrinsics_prior_camera; /* [n] camera index                                   */
  const double* extrinsics_prior_meas;    /* [n][7]                                             */
  const double* extrinsics_prior_sqrt_info; /* [n][36] row-major                                */

  /* --- ABI 5: residual blocks evaluated on the host (SURVEY.md §8b "host-evaluated fallback"):
   * any residual the GPU path has no functor for (GpsErrorSynchronous/Asynchronous,
   * GpsErrorAsynchronous.hpp:42-55; RelativePoseError-like user factors) whose parameter blocks are
   * pose-kind or speed/bias blocks: at most 2 pose-kind and 2 speed/bias blocks, all distinct, at most
   * OKVISGPU_HOST_MAX_RESIDUALS residuals. Each point the solver evaluates (initial point, every
   * candidate) gathers the blocks' values on the device, calls host_evaluate on options.num_threads
   * host threads, and uploads r and the minimal Jacobian, which are accumulated into the reduced
   * system like any device-evaluated factor. Factors on landmarks are not supported
   * (OKVISGPU_ERR_UNSUPPORTED). n_host = 0 (the zero-initialised struct) = none. */
  int32_t n_host;
  const int32_t* host_dim;          /* [n] residual dimension, 1..OKVISGPU_HOST_MAX_RESIDUALS     */
  const int32_t* host_param_kind;   /* [n][4] parameter block k in the functor's order: 0 pose-kind
                                       (index < n_poses: a state's pose; n_poses + c: camera c's
                                       extrinsics), 1 speed/bias, -1 none (trailing)             */
  const int32_t* host_param_index;  /* [n][4]                                                      */
  const uint8_t* host_cauchy;       /* [n] 1 = CauchyLoss(1.0) (may be NULL = no loss); ignored
                                       when host_loss is set                                    */
  okvisgpu_host_evaluate_fn host_evaluate;
  void* host_user;

  /* --- ABI 6: the loss function of each host-evaluated factor (any okvisgpu_loss_kind, e.g.
   * CauchyLoss(3.0) on GPS factors, ViGraph.cpp:999; TukeyLoss(2.0) on LiDAR submap alignment,
   * :1510). NULL = host_cauchy. */
  const okvisgpu_loss* host_loss;   /* [n_host]                                                     */
} okvisgpu_problem;

/* ---------------------------------------------------------------- solver options / summary */
typedef struct okvisgpu_options {   /* ::ceres::Solver::Options fields okvis sets or relies on */
  int32_t max_num_iterations;       /* ViGraph.cpp:1856                                         */
  int32_t linear_solver;            /* okvisgpu_linear_solver                                   */
  int32_t trust_region_strategy;    /* okvisgpu_tr_strategy                                     */
  int32_t jacobi_scaling;           /* Ceres default true                                       */
  double function_tolerance;        /* 1e-6 default; 1e-3 for the first full-graph pass          */
  double gradient_tolerance;        /* 1e-10                                                    */
  double parameter_tolerance;       /* 1e-8                                                     */
  double initial_trust_region_radius; /* 1e4                                                    */
  double max_trust_region_radius;   /* 1e16                                                     */
  double min_trust_region_radius;   /* 1e-32                                                    */
  double min_relative_decrease;     /* 1e-3                                                     */
  double min_lm_diagonal;           /* 1e-6                                                     */
  double max_lm_diagonal;           /* 1e32                                                     */
  int32_t max_num_consecutive_invalid_steps; /* 5                                               */
  double time_limit_s;              /* <0: none (ViGraph::setOptimisationTimeLimit)              */
  int32_t min_iterations;           /* CeresIterationCallback iterationMinimum_                  */
  int32_t redo_propagation_always;  /* ImuError::redoPropagationAlways (ViSlamBackend.cpp:2036)  */
  int32_t num_threads;              /* host threads (reference path / host evaluation)          */
  int32_t verbose;
  int32_t cholesky_schedule;        /* 0 auto, 1 one persistent workgroup per window (batches of */
                                    /* more windows than CUs), 2 tile-parallel launches (fewer    */
                                    /* than half as many), 3 persistent, split over the two parts */
                                    /* of a nested-dissection window (half as many), 4 pipelined  */
                                    /* persistent, two teams per window (up to one per CU), 5 the */
                                    /* split schedule with each part pipelined; all give the same */
                                    /* bits for one batch. Other values: auto.                    */
} okvisgpu_options;

typedef struct okvisgpu_summary {   /* ::ceres::Solver::Summary subset */
  double initial_cost;
  double final_cost;
  int32_t num_iterations;           /* iterations performed, excluding iteration 0              */
  int32_t num_successful_steps;     /* Ceres counts iteration 0 as successful                    */
  int32_t num_unsuccessful_steps;
  int32_t termination_type;         /* okvisgpu_termination                                     */
  double total_time_s;              /* wall time of okvisgpu_solve for this batch               */
  double final_radius;
  double final_mu;
  /* ABI 6: the ::ceres::Solver::Summary timing fields (seconds; one batch, the same in every
   * window's summary). Wall clock of okvisgpu_solve's parts: preprocessor (parameter upload,
   * structure rebuild after freeze / unfreeze, iteration 0, graph instantiation), minimizer (the
   * trust-region iterations), postprocessor (write-back). Device time of the iterations' phases
   * from HIP events on the context's stream, only when options.verbose is set (the iterations then
   * run as eager launches instead of the captured graph: the same kernels in the same order, the
   * same bits), else -1: linear solver (GN prep, Schur assembly, LLT + back substitution, J*v),
   * residual evaluation (candidate evaluation and its cost reduction), Jacobian evaluation
   * (linearisation at the accepted point and the gradient norms), step (the dogleg step, Plus and
   * the accept / reject decision; no Ceres field: part of its minimizer time). */
  double preprocessor_time_s;
  double minimizer_time_s;
  double postprocessor_time_s;
  double linear_solver_time_s;
  double residual_evaluation_time_s;
  double jacobian_evaluation_time_s;
  double step_time_s;
} okvisgpu_summary;

/* ---------------------------------------------------------------- context */
typedef struct okvisgpu_ctx okvisgpu_ctx;

int okvisgpu_abi_version(void);
void okvisgpu_default_options(okvisgpu_options* options);
int okvisgpu_device_count(int32_t* count);
int okvisgpu_ctx_create(int32_t device, okvisgpu_ctx** ctx);
int okvisgpu_ctx_destroy(okvisgpu_ctx* ctx);
const char* okvisgpu_last_error(const okvisgpu_ctx* ctx);

/* Upload a batch of independent windows (one window = one okvis::ViGraph problem). The structure
 * (residual blocks, parameter blocks, constant flags) is analysed once here. The problem structs
 * and the arrays they point to must stay valid until the next okvisgpu_set_problems() call,
 * because okvisgpu_solve() writes results back into them. */
int okvisgpu_set_problems(okvisgpu_ctx* ctx, const okvisgpu_problem* problems, int32_t n_windows);

/* Re-upload only parameter values (and imu_state) from the host arrays (after the caller changed
 * estimates between solves, e.g. ViSlamBackend re-initialising states). */
int okvisgpu_update_params(okvisgpu_ctx* ctx);

/* SetParameterBlockConstant / SetParameterBlockVariable between solves (freeze / unfreeze:
 * ViGraphEstimator.cpp:216-331; extrinsics: ViGraph::setExtrinsicsVariable, ViGraph.cpp:1733-1739,
 * and the tracking solve's freeze, ViSlamBackend.cpp:866-872). kind: 0 pose, 1 speed/bias,
 * 2 landmark, 3 extrinsics (index = camera). Takes effect at the next
 * okvisgpu_solve (the reduced-system structure is rebuilt on the host, values stay on device). */
int okvisgpu_set_block_constant(okvisgpu_ctx* ctx, int32_t window, int32_t kind, int32_t index,
                                int32_t is_constant);

/* ::ceres::Solve equivalent for every window in the batch. summaries: NULL or an array of n_windows
 * entries (n_windows of the last okvisgpu_set_problems: one summary is written for EVERY window).
 * Results are written back into the caller's parameter arrays (and imu_state when provided). */
int okvisgpu_solve(okvisgpu_ctx* ctx, const okvisgpu_options* options, okvisgpu_summary* summaries);

/* Split form of okvisgpu_solve (okvisgpu_solve == begin + iterate(max_num_iterations) + end):
 *   begin   upload the caller's parameter values, iteration 0 (initial evaluation, Jacobi scaling,
 *           gradient norms) and instantiate the captured iteration graph;
 *   iterate enqueue n trust-region iterations on the context's stream (asynchronous; windows that
 *           have terminated skip all work);
 *   end     synchronise, finish windows that spent iterations on LM-regularisation retries, write
 *           results back into the caller's arrays and fill the summaries.
 * okvisgpu_synchronize waits for the context's stream. */
int okvisgpu_solve_begin(okvisgpu_ctx* ctx, const okvisgpu_options* options);
int okvisgpu_solve_iterate(okvisgpu_ctx* ctx, int32_t n);
int okvisgpu_solve_end(okvisgpu_ctx* ctx, okvisgpu_summary* summaries);
int okvisgpu_synchronize(okvisgpu_ctx* ctx);

/* Device time per kernel of ONE trust-region iteration launched eagerly (not from the graph) on
 * the context's stream, bracketed by HIP events; must follow okvisgpu_solve_begin (it advances the
 * solve by one iteration). phase_ms[OKVISGPU_N_PHASES] (ms, summed over the launches of that
 * kernel in the iteration); phase i is named by okvisgpu_phase_name(i). */
#define OKVISGPU_N_PHASES 15
int okvisgpu_profile_iteration(okvisgpu_ctx* ctx, double* phase_ms);
const char* okvisgpu_phase_name(int32_t phase);

/* Measurement hooks (not part of the reference interface; used by bench.py's roofline).
 * okvisgpu_time_kernel re-arms every window of the last finished solve (call after
 * okvisgpu_solve_end / okvisgpu_solve; the device-side solve and IMU state are scratch afterwards:
 * call okvisgpu_update_params before the next solve) and launches one
 * iteration's worth of kernel `kernel` `reps` times on the context's stream between HIP events.
 * avg_ms = device time per repetition; work = algorithmic work of one repetition over the whole
 * batch (compulsory HBM bytes if *bound == 0, FP64 FLOPs if *bound == 1). */
int okvisgpu_kernel_count(void);
const char* okvisgpu_kernel_name(int32_t kernel);
int okvisgpu_time_kernel(okvisgpu_ctx* ctx, int32_t kernel, int32_t reps, double* avg_ms, double* work,
                         int32_t* bound);

/* ---------------------------------------------------------------- pose-graph edges
 * TwoPoseStandardGraphError::compute (TwoPoseGraphError.cpp:162-397) for a batch of edges on the
 * GPU: the reprojection observations of the landmarks shared by a reference keyframe S0 and another
 * keyframe S1 are linearised in S0 coordinates (Cauchy-corrected, |r| > 3 outliers dropped), every
 * landmark is marginalised with the pseudo-inverse square root of its 3x3 block (dropped when
 * rank < 3 and its depth in S0 < 2.99), and the 6x6 relative system H00_, b0_ is decomposed into
 * J_ = D^(1/2) E^T and DeltaX_ = -H^+ b0_ (eigenvalues <= 1e-8*6*max treated as zero, ascending
 * order as Eigen::SelfAdjointEigenSolver). Inputs are the values TwoPoseGraphError::addObservation
 * recorded: landmarks and the other pose as added, the reference pose as its current estimate.
 * The edges of one call share the camera rig (stayConst_ = true, do_extrinsics: false). */
typedef struct okvisgpu_twopose_edges {
  int32_t n_edges;
  const double* ref_pose;           /* [n_edges][7] T_WS0                                        */
  const double* other_pose;         /* [n_edges][7] T_WS1                                        */
  int32_t n_cameras;
  const okvisgpu_camera* cameras;   /* [n_cameras]                                               */
  const double* extrinsics;         /* [n_cameras][7] T_SC                                       */
  const int32_t* landmark_begin;    /* [n_edges+1] CSR: landmarks of edge e (observations_ map order) */
  const double* landmarks;          /* [n_landmarks][4] hp_W                                     */
  const int32_t* obs_begin;         /* [n_landmarks+1] CSR: observations of landmark l           */
  const uint8_t* obs_other;         /* [n_obs] 0 = seen from the reference pose, 1 = from the other */
  const int32_t* obs_camera;        /* [n_obs]                                                   */
  const double* obs_keypoint;       /* [n_obs][2]                                                */
  const double* obs_sqrt_info;      /* [n_obs][4] (ReprojectionError::setInformation; weight applied) */
  const uint8_t* obs_cauchy;        /* [n_obs] 1 = CauchyLoss(1) (may be NULL = all)             */
} okvisgpu_twopose_edges;

/* Outputs per edge (host, caller-owned): delta_x [6], sqrt_info (J_) [36], lin_point [7];
 * H00 [36] and b0 [6] (the marginalised relative system, may be NULL). Uses the context's device and
 * stream; independent of the problem set with okvisgpu_set_problems. */
int okvisgpu_twopose_compute(okvisgpu_ctx* ctx, const okvisgpu_twopose_edges* edges, double* delta_x,
                             double* sqrt_info, double* lin_point, double* H00, double* b0);

/* ---------------------------------------------------------------- IMU-merge elimination
 * ImuError::append (ImuError.cpp:63-255) for a batch of factors on the GPU: the step of
 * ViGraphEstimator::eliminateStateByImuMerge (ViGraphEstimator.cpp:38-171) that extends the IMU
 * link into an eliminated state k with the link out of it. Per factor: `state` is the link's
 * preintegration state (OKVISGPU_IMU_STATE_DOUBLES layout, e.g. written back by a solve), t1_old its
 * t1, t1_new the next link's t1, speed_biases the estimate of state k (the bias the appended part
 * is integrated with), and the samples the next link's imuMeasurements(). On return `state` holds the
 * merged link's state (t0 unchanged, t1 = t1_new; redo counter, redo flag and speedAndBiases_ref_
 * unchanged, as in the reference) and steps[i] the integrated steps (-1: the samples do not reach
 * t1_new, state untouched). The merged factor's samples are the link's followed by the appended ones
 * newer than its last (ImuError.cpp:74-81); the caller rebuilds its problem with them. */
typedef struct okvisgpu_imu_append_batch {
  int32_t n;
  okvisgpu_imu_params imu_params;
  double* state;                    /* [n][OKVISGPU_IMU_STATE_DOUBLES] in/out                     */
  const int64_t* t1_old_ns;         /* [n]                                                         */
  const int64_t* t1_new_ns;         /* [n]                                                         */
  const double* speed_biases;       /* [n][9]                                                      */
  const int32_t* sample_begin;      /* [n+1] CSR of the appended samples                           */
  const int64_t* sample_t_ns;       /* [n_samples]                                                 */
  const double* sample_gyr_acc;     /* [n_samples][6]                                              */
} okvisgpu_imu_append_batch;
int okvisgpu_imu_append(okvisgpu_ctx* ctx, const okvisgpu_imu_append_batch* batch, int32_t* steps);

/* ---------------------------------------------------------------- okvis Component graphs
 * Component::load (okvis_ceres/src/Component.cpp:50-383) as an okvisgpu_problem: states (pose and
 * speed/bias blocks, ordered by state id), landmarks (ordered by id), one extrinsics block per camera,
 * EDGE_IMU factors with their measurements, EDGE_OBS reprojections with the measurement and the
 * information 64/size^2 of the frame's FRAME:KEYPOINT (float, as cv::KeyPoint) and Cauchy(1). The
 * camera intrinsics and IMU parameters are configuration (not in the file) and are passed in. No
 * priors and no constant blocks are added: the caller freezes what its solve needs. Host only. */
typedef struct okvisgpu_graph okvisgpu_graph;
int okvisgpu_graph_load(const char* path, const okvisgpu_camera* cameras, int32_t n_cameras,
                        const okvisgpu_imu_params* imu, okvisgpu_graph** out);
/* The problem view into the graph's arrays (valid until destroy; solves write into them). */
const okvisgpu_problem* okvisgpu_graph_problem(okvisgpu_graph* g);
/* File ids of the states / landmarks in problem order and the state time stamps (may be NULL). */
int okvisgpu_graph_ids(const okvisgpu_graph* g, uint64_t* state_ids, int64_t* state_t_ns, uint64_t* landmark_ids);
void okvisgpu_graph_destroy(okvisgpu_graph* g);
/* Component::save (Component.cpp:385-506) of a problem (one speed/bias block per state, isotropic
 * reprojection information): ids = problem indices, time stamps from state_t_ns or the IMU factors. */
int okvisgpu_graph_save(const okvisgpu_problem* p, const int64_t* state_t_ns, const char* path);

/* Problem statistics of the batch held by a context (the ::ceres::Solver::Summary counters
 * num_parameter_blocks / num_residual_blocks / num_effective_parameters_reduced analogues, plus the
 * layout figures bench.py's roofline work model needs). Sums over all windows. */
typedef struct okvisgpu_problem_stats {
  int32_t n_windows;
  int32_t cholesky_launches;        /* launches of the tile-parallel factorisation (roots + steps) */
  int64_t n_poses, n_speed_biases, n_landmarks, n_landmarks_free, n_extrinsics_free;
  int64_t n_observations, n_visits, n_imu, n_imu_samples, n_pose_priors, n_sb_priors, n_relpose;
  int64_t reduced_dim;              /* sum of the reduced (Schur) dimensions                      */
  int64_t s_tiles_nonzero;          /* 64x64 tiles of S the tile-sparse LLT touches (incl. fill)  */
  int64_t s_tiles_dense;            /* lower-triangle tiles of the dense reduced matrices          */
  int64_t n_block_pairs, n_visit_segments, n_partial_blocks;
  int64_t arena_bytes;              /* device memory held by the context                           */
  int64_t cholesky_split_windows;   /* windows whose nested-dissection parts factor independently */
} okvisgpu_problem_stats;
int okvisgpu_get_stats(okvisgpu_ctx* ctx, okvisgpu_problem_stats* stats);

/* Host-only plan of one window's reduced system (no device, no context; for tests and tools): the
 * state order a batch below one window per CU gives it (nested_dissection = 1) or the natural one
 * (0), its tile pattern and the tile-parallel factorisation schedule. Any output may be NULL.
 *   info[8]:        natural reduced dimension, S dimension (64-padded), tiles T, structurally
 *                   non-zero tiles (after fill), launches (roots + updates), split tL, split tS
 *                   (0 0: none), gap rows
 *   tile_nz[T*T]:   the filled lower-triangular tile pattern (row-major, 1 = non-zero)
 *   step_launch[T]: launch of step k's band updates (0: the step has none)
 *   natural[dim]:   natural index of each row of S (-1: gap or padding row), dim = info[1]
 * Pass tile_nz / step_launch / natural sized from a first call with them NULL. */
int okvisgpu_plan_window(const okvisgpu_problem* problem, int32_t nested_dissection, int64_t* info,
                         uint8_t* tile_nz, int32_t* step_launch, int32_t* natural);

/* Copy device parameter values back into the caller's host arrays without solving. */
int okvisgpu_get_params(okvisgpu_ctx* ctx);

/* ---------------------------------------------------------------- evaluation entry points
 * (::ceres::Problem::Evaluate / EvaluateResidualBlock analogues; also the parity-test hooks)
 *
 * okvisgpu_evaluate: total cost 1/2 sum rho(|r|^2) of window w at the current device parameters.
 */
int okvisgpu_evaluate(okvisgpu_ctx* ctx, int32_t window, double* cost);

/* Linearise window w at the current parameters and eliminate the landmarks (DENSE_SCHUR):
 *   S   = H_ff - H_fl H_ll^-1 H_lf,   rhs = g_f - H_fl H_ll^-1 g_l,   g = J^T r (Cauchy-corrected)
 * with Jacobi scaling (if jacobi_scaling) and the dogleg LM diagonal D = diag(J^T J)^(1/2)*sqrt(mu)
 * exactly as the solver's first Gauss-Newton solve would form them. Outputs (host, may be NULL):
 *   S   [dim*dim] row-major (full symmetric), rhs [dim], cost [1], dim_out [1].
 * The reduced ordering is: for i = 0 .. max(n_poses, n_speed_biases)-1: pose i (6, if variable)
 * then speed/bias i (9, if variable); then the variable extrinsics in camera order (6 each). */
int okvisgpu_linearize_reduce(okvisgpu_ctx* ctx, int32_t window, int32_t jacobi_scaling, double mu,
                              double* S, double* rhs, double* cost, int32_t* dim_out);

/* Raw per-residual evaluation for parity tests (EvaluateWithMinimalJacobians semantics, no loss):
 *   reprojection: r [n_obs][2], J_pose [n_obs][2][6], J_landmark [n_obs][2][3] (minimal, row-major)
 *   imu:          r [n_imu][15], J [n_imu][15][30] minimal columns (pose0 6, sb0 9, pose1 6, sb1 9)
 * Any output pointer may be NULL. The IMU call updates the factor's preintegration state exactly as
 * ImuError::EvaluateWithMinimalJacobians does (ImuError.cpp:833-859). */
int okvisgpu_eval_reprojection(okvisgpu_ctx* ctx, int32_t window, double* r, double* J_pose,
                               double* J_landmark);
int okvisgpu_eval_imu(okvisgpu_ctx* ctx, int32_t window, int32_t redo_always, double* r, double* J);
/*   relative pose: r [n_relpose][6], J [n_relpose][6][12] minimal (reference pose 6, other pose 6) */
int okvisgpu_eval_relpose(okvisgpu_ctx* ctx, int32_t window, double* r, double* J);
/*   host-evaluated blocks, through the device path (gather, host_evaluate, upload; no loss):
 *   r [n_host][15], J [n_host][15][30] minimal in the IMU column layout (first pose-kind block 0..5,
 *   first speed/bias 6..14, second pose-kind 15..20, second speed/bias 21..29), rows >= dim zero. */
int okvisgpu_eval_host(okvisgpu_ctx* ctx, int32_t window, double* r, double* J);

/* ---------------------------------------------------------------- synthetic windows
 * Host-side generator of the synthetic sliding windows the benchmark is quoted on:
 * EuRoC stereo rig (config/euroc/okvis2.yaml:2-32), smooth sinusoidal 6-DoF trajectory
 * (okvis_ceres/test/TestImuError.cpp:86-185 style), 200 Hz IMU, landmarks in a 2-20 m band,
 * observations with N(0,1px^2) noise and information 64/8^2 = I, perturbed initial states, priors as
 * ViGraph::addStatesInitialise (ViGraph.cpp:347-370), Cauchy(1) on every reprojection.
 * std::mt19937_64(seed). No GPU is touched. */
typedef struct okvisgpu_synth_config {
  int32_t n_keyframes;              /* S10: 10, S50: 50 */
  int32_t n_landmarks;              /* S10: 500, S50: 2000 */
  int32_t n_observations;           /* S10: 4000, S50: 16000 */
  int32_t max_obs_per_landmark;     /* 20 */
  double kf_dt_s;                   /* 0.1 */
  double imu_rate_hz;               /* 200 */
  double pixel_noise;               /* 1.0 */
  double init_sigma_pos, init_sigma_rot, init_sigma_lm, init_sigma_vel; /* 0.05 0.01 0.05 0.02 */
  uint64_t seed;
  /* pose-graph edges (TwoPoseStandardGraphErrorConst) from keyframe i to i + relpose_stride,
   * i = 0, 1, ...: information from sigmas 0.02 m / 0.005 rad (random rotation of the frame),
   * linearisation point = the ground-truth relative pose perturbed at that noise, DeltaX_ small.
   * 0 (default) = none, as in the benchmark windows. */
  int32_t n_relpose;
  int32_t relpose_stride;
  int32_t relpose_kind;             /* 0 pose-graph edges, 1 RelativePoseError, 2 alternating */
  /* online extrinsics calibration (ABI 4): both T_SC blocks variable, initialised at the true T_SC
   * perturbed by N(0, sigma_r^2) / N(0, sigma_alpha^2) and held by a PoseError prior centred on that
   * initial value (ViGraph.cpp:372-382). 0 (default) = constant extrinsics. */
  int32_t do_extrinsics;
  double extrinsics_sigma_r, extrinsics_sigma_alpha;  /* 0.001 m, 0.005 rad (config/hilti22) */
} okvisgpu_synth_config;

typedef struct okvisgpu_synth_window okvisgpu_synth_window;  /* owns all arrays of one problem */

void okvisgpu_synth_default_config(okvisgpu_synth_config* cfg, int32_t n_keyframes,
                                   int32_t n_landmarks, int32_t n_observations, uint64_t seed);
int okvisgpu_synth_create(const okvisgpu_synth_config* cfg, okvisgpu_synth_window** out);
/* The problem view into the window's arrays (valid until destroy). */
const okvisgpu_problem* okvisgpu_synth_problem(okvisgpu_synth_window* w);
/* Ground truth: poses [n_kf][7], landmarks [n_lm][4], speed_biases [n_kf][9] (may be NULL); the
 * true extrinsics are okvisgpu_synth_true_extrinsics [n_cameras][7]. */
int okvisgpu_synth_ground_truth(const okvisgpu_synth_window* w, double* poses, double* landmarks,
                                double* speed_biases);
/* Reset the problem's parameter arrays (and imu_state) to the generated initial estimate. */
int okvisgpu_synth_reset(okvisgpu_synth_window* w);
int okvisgpu_synth_true_extrinsics(const okvisgpu_synth_window* w, double* extrinsics);
void okvisgpu_synth_destroy(okvisgpu_synth_window* w);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* OKVISGPU_H_ */
