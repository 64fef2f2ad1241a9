// launch.hpp — host-side launchers of the gfx950 kernels (one stream, graph-capturable: no
// allocation, no synchronisation, no host reads inside any launcher).
#pragma once

#include <hip/hip_runtime.h>

#include "device_problem.hpp"

namespace okg {

// evaluation (kernels_eval.hip); mode 0 current, 1 candidate, 2 initial, 3 initial without loss
void launch_eval(const DevProblem& P, int mode, hipStream_t s);
void launch_eval_obs(const DevProblem& P, int mode, hipStream_t s);
void launch_eval_imu(const DevProblem& P, int mode, hipStream_t s);
void launch_eval_priors(const DevProblem& P, int mode, hipStream_t s);
void launch_eval_imu_as_solved(const DevProblem& P, int mode, hipStream_t s);  // (okvisgpu_time_kernel)
// ImuError::append for a batch (P: n_imu, imu_blocks {0, f, 0, f}, imu_t0 = old t1, imu_t1 = new t1,
// imu_sbegin / imu_ts / imu_ga = appended samples, imu_par (one row), imu_state, sb[0] = biases)
void launch_imu_append(const DevProblem& P, hipStream_t s);
// host-evaluated factors: gather the evaluation points (host_in), scatter the uploaded results
// (host_out) into the linearisation records; the host step between them is the runtime's
void launch_host_gather(const DevProblem& P, int mode, hipStream_t s);
void launch_host_scatter(const DevProblem& P, hipStream_t s);

// landmark / reduced-system kernels (kernels_schur.hip); lin_mode 0 = init, 1 = accepted only
void launch_linearization_blocks(const DevProblem& P, int lin_mode, hipStream_t s);
void launch_gn_reduce(const DevProblem& P, hipStream_t s);    // lm_prep + assemble (S is initialised once per build, ensureS)
void launch_gn_backsub(const DevProblem& P, hipStream_t s);   // landmark back substitution + gn vectors
void launch_lm_blocks(const DevProblem& P, int lin_mode, hipStream_t s);
void launch_imu_hess(const DevProblem& P, int lin_mode, hipStream_t s);
void launch_fgrad(const DevProblem& P, int lin_mode, hipStream_t s);
void launch_lm_prep(const DevProblem& P, hipStream_t s);
// few windows: the GN prep runs inside the linearisation after a step (launch_linearization_blocks),
// so the captured iteration does not start with it and the initial linearisation ends with it
bool lin_runs_prep(const DevProblem& P);
// the non-zero tiles of S: tail = 0 of the windows about to assemble; tail = 1 of every window not
// done (end of the captured iteration, S dead)
void launch_zero_S(const DevProblem& P, hipStream_t s, int tail = 0);
void launch_assemble(const DevProblem& P, hipStream_t s);
void launch_lm_backsub(const DevProblem& P, hipStream_t s);  // kernels_backsub.hip: + landmark dogleg vectors, J*v
void launch_assemble_gradnorm_few(const DevProblem& P, hipStream_t s);  // few windows: + the gradient test
void launch_assemble_pp(const DevProblem& P, hipStream_t s);
void launch_assemble_sb(const DevProblem& P, hipStream_t s);
void launch_lm_visit(const DevProblem& P, int mode, hipStream_t s);  // 0/1: linearisation, 2: GN prep

// dense factorisation + both triangular solves, one persistent workgroup per window
// (kernels_chol.hip)
// persistent Cholesky: does its LDS (static + the window's solve vector) fit a workgroup?
bool cholesky_persistent_fits(int max_fpad, size_t lds_per_block);
bool cholesky_pipe_fits(int max_fpad, size_t lds_per_block);  // (kernels_chol_pipe.hip)
void launch_cholesky(const DevProblem& P, hipStream_t s);
void launch_cholesky_pipe(const DevProblem& P, hipStream_t s, bool split);
void launch_cholesky_split_b(const DevProblem& P, hipStream_t s);  // k_cholesky<2> (kernels_chol.hip)

// trust-region control (kernels_control.hip)
enum ReduceMode { R_COST_INIT = 0, R_COST_CAND = 1, R_JV = 2 };
void launch_reduce(const DevProblem& P, int mode, hipStream_t s);
void launch_jv(const DevProblem& P, hipStream_t s);  // (standalone, for okvisgpu_time_kernel; launch_lm_backsub includes it)
void launch_gradnorm(const DevProblem& P, int lin_mode, hipStream_t s);
void launch_dogleg(const DevProblem& P, hipStream_t s);
void launch_select_current(const DevProblem& P, hipStream_t s);  // set 1 -> set 0 where xcur == 1

// pose-graph edges (kernels_twopose.hip): TwoPoseStandardGraphError::compute, one wavefront per edge
void launch_twopose_compute(const TwoPoseDev& T, hipStream_t s);

}  // namespace okg
