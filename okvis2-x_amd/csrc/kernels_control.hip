// kernels_control.hip — the trust-region loop on the device (no host round trip per iteration).
//
// Restates ceres::internal::TrustRegionMinimizer + DoglegStrategy (TRADITIONAL_DOGLEG) as used by
// okvis (ViGraph.cpp:249, ViSlamBackend.cpp:877) [ext-Ceres, un-vendored; see DESIGN.md]:
//   k_jv        per residual block, once per GN step: J_s v for the Cauchy and GN directions
//               (Jacobi scaling applied on the fly) -> the three quadratic forms every dogleg
//               step of that linearisation needs for its model cost change.
//   k_reduce    one workgroup per window, fixed-order tree reductions (bitwise reproducible):
//               costs, the J*v forms and the Cauchy alpha, and the
//               candidate acceptance test (parameter / function tolerance, relative decrease,
//               radius and mu updates).
//   k_gradnorm  |x - Plus(x, -g)|_inf / _2 and |x| after every accepted step.
//   k_dogleg    one workgroup per window: LM-failure retries of the GN step, the traditional
//               dogleg interpolation, delta = step .* jacobi_scaling, the manifold Plus into
//               the candidate parameter set, model_cost_change and the step-validity bookkeeping.
#include <cfloat>

#include "block_reduce.hpp"
#include "dev_clock.hpp"
#include "device_problem.hpp"
#include "gradnorm.hpp"
#include "jv_groups.hpp"
#include "launch.hpp"
#include "okvisgpu_math.hpp"

namespace okg {

// Per-window workgroup size of k_reduce and k_dogleg (k_gradnorm: always 256): 256 threads for batches, 1,024
// when the batch has at most a quarter window per CU (a single window's reductions are chains of
// dependent loads per thread: four times the threads, a quarter of the chain). A power of two in
// [64, 1024] (the tree reductions); the reduction order follows it, so a window's bits depend on
// the batch size only through this choice (and the Cholesky order, runtime.cpp build).
constexpr int kRBBatch = 256, kRBFew = 1024;

// Bookkeeping common to every iteration end (FinalizeIterationAndCheckIfMinimizerCanContinue):
// iteration cap, then the trust-region radius floor. (The gradient test follows the next
// gradient evaluation: k_gradnorm.)
__device__ void finalizeIteration(const DevProblem& P, WinState& s) {
  if (s.done) return;
  if (s.iteration >= P.opt.max_num_iterations) {
    s.done = 1;
    s.termination = 1;  // NO_CONVERGENCE
    return;
  }
  if (s.radius <= P.opt.min_radius) {
    s.done = 1;
    s.termination = 0;  // CONVERGENCE
  }
}

// J*v reductions of window w (once per GN step): jcc, jgg, jcg and the Cauchy alpha =
// |gradient_|^2 / jcc, stored by thread 0 in the window state; every thread gets alpha.
// Reprojection rows and landmark gradients come as the landmark groups' sums (k_lm_backsub_jv).
// (this thread's partial sums of jcc, jgg, jcg: reduceJv and the merged reduction of k_dogleg)
__device__ __forceinline__ void jvPartials(const DevProblem& P, int w, int t, int RB, double (&a)[3]) {
  const int ib = P.win_imu_range[2 * w], ie = P.win_imu_range[2 * w + 1];
  const int hb = P.win_host_range[2 * w], he = P.win_host_range[2 * w + 1];
  const int pb = P.win_pp_range[2 * w], pe = P.win_pp_range[2 * w + 1];
  const int sbb = P.win_sbp_range[2 * w], sbe = P.win_sbp_range[2 * w + 1];
  const int rpb = P.win_rp_range[2 * w], rpe = P.win_rp_range[2 * w + 1];
  const int gb = P.win_lmg_range[2 * w], ge = P.win_lmg_range[2 * w + 1];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double acc = 0.0;
    for (int g = gb + t; g < ge; g += RB) acc += gmem(P.grp_red)[(size_t)g * kGrpRed + k];
    for (int f = ib + t; f < ie; f += RB) acc += gmem(P.imu_jv)[(size_t)k * P.n_fac + f];
    for (int f = hb + t; f < he; f += RB) acc += gmem(P.imu_jv)[(size_t)k * P.n_fac + f];
    for (int i = pb + t; i < pe; i += RB) acc += gmem(P.pp_jv)[(size_t)k * P.n_pprior + i];
    for (int i = sbb + t; i < sbe; i += RB) acc += gmem(P.sbp_jv)[(size_t)k * P.n_sbprior + i];
    for (int i = rpb + t; i < rpe; i += RB) acc += gmem(P.rp_jv)[(size_t)k * P.n_relpose + i];
    a[k] = acc;
  }
}

template <int RB>
__device__ double reduceJv(const DevProblem& P, int w, WinState& s, double* sh) {
  const int t = threadIdx.x;
  const int gb = P.win_lmg_range[2 * w], ge = P.win_lmg_range[2 * w + 1];
  double a[3];
  jvPartials(P, w, t, RB, a);
  blockSumN<RB, 3>(a, sh);
  // |gradient_|^2 over the window (f-vector + free landmarks)
  double g2 = 0.0;
  const int fo = P.win_foff[w], fd = P.win_fdim[w];
  for (int e = t; e < fd; e += RB) g2 += gmem(P.dgF)[fo + e] * gmem(P.dgF)[fo + e];
  for (int g = gb + t; g < ge; g += RB) g2 += gmem(P.grp_red)[(size_t)g * kGrpRed + 3];
  g2 = blockSum<RB>(g2, sh);
  const double alpha = g2 / a[0];
  if (t == 0) {
    s.jcc = a[0];
    s.jgg = a[1];
    s.jcg = a[2];
    s.alpha = alpha;
  }
  return alpha;
}

template <int RB>
__global__ __launch_bounds__(RB) void k_reduce(const DevProblem* __restrict__ Pp, int mode) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  WinState& s = P.st[w];
  if (s.done) return;
  __shared__ double sh[3 * RB];
  const int t = threadIdx.x;
  const int ob = P.win_obs_range[2 * w], oe = P.win_obs_range[2 * w + 1];
  const int ib = P.win_imu_range[2 * w], ie = P.win_imu_range[2 * w + 1];
  const int pb = P.win_pp_range[2 * w], pe = P.win_pp_range[2 * w + 1];
  const int sbb = P.win_sbp_range[2 * w], sbe = P.win_sbp_range[2 * w + 1];
  const int rpb = P.win_rp_range[2 * w], rpe = P.win_rp_range[2 * w + 1];

  if (mode == R_COST_INIT || mode == R_COST_CAND) {
    if (mode == R_COST_CAND && !s.eval_cand) return;
    const int lb = (mode == R_COST_CAND) ? 1 - s.lcur : s.lcur;
    double c = 0.0, cf = 0.0;
    struct OC { double c; uint8_t f; };
    const auto oc = gmem(P.obs_cost[lb]);
    const auto ofl = gmem(P.obs_flags);
    stridedBatched<RB, 8>(ob, oe, [&](int o) { return OC{oc[o], ofl[o]}; },
                      [&](int, const OC& v) {
                        if (v.f & 2) cf += v.c;
                        else c += v.c;
                      });
    const auto ifl = gmem(P.imu_flags);
    const auto icost = gmem(P.imu_cost[lb]);
    for (int f = ib + t; f < ie; f += RB) {
      if (ifl[f] & 2) cf += icost[f];
      else c += icost[f];
    }
    const int hb = P.win_host_range[2 * w], he = P.win_host_range[2 * w + 1];
    for (int f = hb + t; f < he; f += RB) {
      if (ifl[f] & 2) cf += icost[f];
      else c += icost[f];
    }
    for (int i = pb + t; i < pe; i += RB) {
      if (gmem(P.pose_f)[gmem(P.pp_block)[i]] < 0) cf += gmem(P.pp_cost[lb])[i];
      else c += gmem(P.pp_cost[lb])[i];
    }
    for (int i = sbb + t; i < sbe; i += RB) {
      if (gmem(P.sb_f)[gmem(P.sbp_block)[i]] < 0) cf += gmem(P.sbp_cost[lb])[i];
      else c += gmem(P.sbp_cost[lb])[i];
    }
    for (int i = rpb + t; i < rpe; i += RB) {
      if (gmem(P.rp_flags)[i] & 2) cf += gmem(P.rp_cost[lb])[i];
      else c += gmem(P.rp_cost[lb])[i];
    }
    {
      double r2[2] = {c, cf};
      blockSumN<RB, 2>(r2, sh);
      c = r2[0];
      cf = r2[1];
    }
    if (t != 0) return;
    if (mode == R_COST_CAND) {
      // fixed residuals are not re-evaluated at candidates; their cost is fixed_cost
    }
    if (mode == R_COST_INIT) {
      s.x_cost = c;
      s.fixed_cost = cf;
      s.initial_cost = c + cf;
      s.min_cost = c;
      return;
    }
    // ------------------------------------------------ candidate acceptance (per iteration)
    s.cand_cost = c;
    s.eval_cand = 0;
    s.step_valid = 0;
    // ParameterToleranceReached / FunctionToleranceReached: return without finalising the iteration
    if (s.step_norm <= P.opt.parameter_tolerance * (s.x_norm + P.opt.parameter_tolerance)) {
      s.done = 1;
      s.termination = 0;
      s.iteration -= 1;
      return;
    }
    if (fabs(s.x_cost - c) <= P.opt.function_tolerance * s.x_cost) {
      s.done = 1;
      s.termination = 0;
      s.iteration -= 1;
      return;
    }
    const double rel = isfinite(c) ? (s.x_cost - c) / s.model_cost_change : -DBL_MAX;
    if (rel > P.opt.min_relative_decrease) {
      // HandleSuccessfulStep + DoglegStrategy::StepAccepted
      s.xcur = 1 - s.xcur;
      s.lcur = 1 - s.lcur;
      s.x_cost = c;
      if (c < s.min_cost) s.min_cost = c;
      s.accepted = 1;
      s.num_succ += 1;
      if (rel < 0.25) s.radius *= 0.5;
      if (rel > 0.75) s.radius = fmax(s.radius, 3.0 * s.dogleg_step_norm);
      s.radius = fmin(s.radius, P.opt.max_radius);
      s.mu = fmax(1e-8, 2.0 * s.mu / 10.0);
      s.need_gn = 1;
    } else {
      // HandleUnsuccessfulStep + StepRejected
      s.num_unsucc += 1;
      s.radius *= 0.5;
      s.need_gn = 0;
    }
    finalizeIteration(P, s);
    return;
  }

  // J*v reductions (once per GN step)
  if (!(s.need_gn && !s.gn_failed)) return;
  reduceJv<RB>(P, w, s, sh);
}

// |x - Plus(x, -g)| and |x| over the window's active blocks; gradient tolerance test (gradnorm.hpp).
template <int RB>
__global__ __launch_bounds__(RB) void k_gradnorm(const DevProblem* __restrict__ Pp, int lin_mode) {
  gradnormWindow<RB>(*Pp, (int)blockIdx.x, lin_mode);
}

// One workgroup per window: GN failure handling, traditional dogleg step, Plus into X[1-xcur].
template <int RB>
__global__ __launch_bounds__(RB) void k_dogleg(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  WinState& s = P.st[w];
  if (s.done) return;
  DLCLK_INIT
  __shared__ double sh[6 * RB];
  __shared__ int sflag;
  const int t = threadIdx.x;
  const bool sflagGn = s.need_gn && !s.gn_failed;  // (read before thread 0 updates the state)
  __syncthreads();
  if (t == 0) {
    sflag = 0;
    s.accepted = 0;
    if (s.need_gn) {
      if (s.gn_failed) {
        // ComputeGaussNewtonStep: mu *= 10 and retry within the same iteration while mu < max_mu
        s.gn_failed = 0;
        s.mu *= 10.0;
        if (s.mu < 1.0) {
          sflag = 1;  // retry next pass, iteration not consumed
        } else {
          // LINEAR_SOLVER_FAILURE -> invalid step (HandleInvalidStep, StepIsInvalid). The step that
          // reaches max_num_consecutive_invalid_steps ends the solve before Ceres'
          // FinalizeIteration records it (TrustRegionMinimizer: `if (!HandleInvalidStep()) return;`):
          // neither the iteration nor the unsuccessful step is counted
          if (++s.consecutive_invalid >= P.opt.max_num_consecutive_invalid_steps) {
            s.done = 1;
            s.termination = 2;
          } else {
            s.iteration += 1;
            s.num_unsucc += 1;
            s.mu *= 10.0;
            s.need_gn = 1;
            finalizeIteration(P, s);
          }
          sflag = 1;
        }
      } else {
        s.need_gn = 0;  // reuse_ = true until the step is accepted / invalid
      }
    }
    if (!sflag) s.iteration += 1;
  }
  __syncthreads();
  if (sflag) return;
  DLCLK(0)
  const int foff = P.win_foff[w], fd = P.win_fdim[w];
  const int l0 = P.win_lm_range[2 * w], l1 = P.win_lm_range[2 * w + 1];
  // pass 1: norms (f-blocks here, landmarks as the landmark groups' sums of k_lm_backsub_jv)
  double gg = 0.0, nn = 0.0, gn = 0.0;
  for (int e = t; e < fd; e += RB) {
    const double a = gmem(P.dgF)[foff + e], b = gmem(P.gnF)[foff + e];
    gg += a * a;
    nn += b * b;
    gn += a * b;
  }
  const int gb = P.win_lmg_range[2 * w], ge = P.win_lmg_range[2 * w + 1];
  for (int g = gb + t; g < ge; g += RB) {
    const auto r = gmem(P.grp_red + (size_t)g * kGrpRed);
    gg += r[3];
    nn += r[4];
    gn += r[5];
  }
  // a new GN step also needs its J*v forms (formerly k_reduce R_JV) and alpha = |gradient_|^2 /
  // jcc: reduced in the same tree as the norms (|gradient_|^2 is gg, the same per-thread order as
  // reduceJv's), one tree instead of three, each value with the same additions (same bits)
  double alpha = s.alpha;
  if (sflagGn) {
    double r6[6];
    double a3[3];
    jvPartials(P, w, t, RB, a3);
    DLCLK(1)
    r6[0] = a3[0]; r6[1] = a3[1]; r6[2] = a3[2]; r6[3] = gg; r6[4] = nn; r6[5] = gn;
    blockSumN<RB, 6>(r6, sh);
    DLCLK(2)
    gg = r6[3];
    nn = r6[4];
    gn = r6[5];
    alpha = gg / r6[0];
    if (t == 0) {
      s.jcc = r6[0];
      s.jgg = r6[1];
      s.jcg = r6[2];
      s.alpha = alpha;
    }
  } else {
    double r3[3] = {gg, nn, gn};
    blockSumN<RB, 3>(r3, sh);
    gg = r3[0];
    nn = r3[1];
    gn = r3[2];
  }
  const double gradient_norm = sqrt(gg), gauss_newton_norm = sqrt(nn);
  const double radius = s.radius;
  // step = ca * gradient_ + cb * gauss_newton_step_  (then divided by diagonal_)
  double ca, cb;
  int dcase;
  if (gauss_newton_norm <= radius) {
    ca = 0.0; cb = 1.0; dcase = 1;
  } else if (gradient_norm * alpha >= radius) {
    ca = -(radius / gradient_norm); cb = 0.0; dcase = 2;
  } else {
    const double b_dot_a = -alpha * gn;
    const double a_squared_norm = (alpha * gradient_norm) * (alpha * gradient_norm);
    const double b_minus_a_squared_norm = a_squared_norm - 2 * b_dot_a + gauss_newton_norm * gauss_newton_norm;
    const double c = b_dot_a - a_squared_norm;
    const double d = sqrt(c * c + b_minus_a_squared_norm * (radius * radius - a_squared_norm));
    const double beta = (c <= 0) ? (d - c) / b_minus_a_squared_norm : (radius * radius - a_squared_norm) / (d + c);
    ca = -alpha * (1.0 - beta);
    cb = beta;
    dcase = 3;
  }
  // pass 2: step, delta, Plus, |x - x_cand|
  const int xs = s.xcur, xd = 1 - s.xcur;
  double sn2 = 0.0, dn2 = 0.0, jr = 0.0;
  const int p0 = P.win_pose_range[2 * w], p1 = P.win_pose_range[2 * w + 1];
  // (every operand of a block is loaded before its first store: the stores may alias the
  // f-vectors for the compiler, and a single window is a chain of such rounds)
  for (int p = p0 + t; p < p1; p += RB) {
    const int pf = gmem(P.pose_f)[p];
    if (pf < 0) continue;
    double dg[6], gn[6], dia[6], sc[6], g[6], x[7];
    for (int c = 0; c < 6; ++c) {
      const size_t i = (size_t)foff + pf + c;
      dg[c] = gmem(P.dgF)[i];
      gn[c] = gmem(P.gnF)[i];
      dia[c] = gmem(P.diagF)[i];
      sc[c] = gmem(P.sF)[i];
      g[c] = gmem(P.gF)[i];
    }
    for (int k = 0; k < 7; ++k) x[k] = gmem(P.pose[xs])[7 * (size_t)p + k];
    double delta[6];
    for (int c = 0; c < 6; ++c) {
      const double v = ca * dg[c] + cb * gn[c];
      dn2 += v * v;
      const double st = v / dia[c];
      gmemw(P.stepF)[(size_t)foff + pf + c] = st;
      delta[c] = st * sc[c];
      jr += delta[c] * g[c];
    }
    const auto y = gmemw(P.pose[xd] + 7 * (size_t)p);
    const Q dq = deltaQ(delta[3], delta[4], delta[5]);
    const Q q = qnormalize(qmul(dq, qnormalize(Q{x[3], x[4], x[5], x[6]})));
    double yv[7] = {x[0] + delta[0], x[1] + delta[1], x[2] + delta[2], q.x, q.y, q.z, q.w};
    for (int k = 0; k < 7; ++k) {
      y[k] = yv[k];
      sn2 += (x[k] - yv[k]) * (x[k] - yv[k]);
    }
  }
  const int b0 = P.win_sb_range[2 * w], b1 = P.win_sb_range[2 * w + 1];
  for (int b = b0 + t; b < b1; b += RB) {
    const int sf = gmem(P.sb_f)[b];
    if (sf < 0) continue;
    const auto y = gmemw(P.sb[xd] + 9 * (size_t)b);
    double dg[9], gn[9], dia[9], sc[9], g[9], x[9];
    for (int c = 0; c < 9; ++c) {
      const size_t i = (size_t)foff + sf + c;
      dg[c] = gmem(P.dgF)[i];
      gn[c] = gmem(P.gnF)[i];
      dia[c] = gmem(P.diagF)[i];
      sc[c] = gmem(P.sF)[i];
      g[c] = gmem(P.gF)[i];
      x[c] = gmem(P.sb[xs])[9 * (size_t)b + c];
    }
    for (int c = 0; c < 9; ++c) {
      const double v = ca * dg[c] + cb * gn[c];
      dn2 += v * v;
      const double st = v / dia[c];
      gmemw(P.stepF)[(size_t)foff + sf + c] = st;
      jr += (st * sc[c]) * g[c];
      const double yv = x[c] + st * sc[c];
      y[c] = yv;
      sn2 += (x[c] - yv) * (x[c] - yv);
    }
  }
  DLCLK(3)
  struct LS { double x[4], dg[3], gn[3], dia[3], sl[3], g[3]; uint8_t f; };
  stridedBatched<RB, (RB >= 1024 ? 1 : 4)>(l0, l1,
                    [&](int l) {
                      LS v;
                      v.f = gmem(P.lm_free)[l];
                      for (int k = 0; k < 4; ++k) v.x[k] = gmem(P.lm[xs])[4 * (size_t)l + k];
                      for (int c = 0; c < 3; ++c) {
                        const size_t i = 3 * (size_t)l + c;
                        v.dg[c] = gmem(P.dgL)[i];
                        v.gn[c] = gmem(P.gnL)[i];
                        v.dia[c] = gmem(P.diagL)[i];
                        v.sl[c] = gmem(P.sL)[i];
                        v.g[c] = gmem(P.gL)[i];
                      }
                      return v;
                    },
                    [&](int l, const LS& v) {
                      if (!v.f) return;
                      const auto y = gmemw(P.lm[xd] + 4 * (size_t)l);
                      for (int c = 0; c < 3; ++c) {
                        const double vv = ca * v.dg[c] + cb * v.gn[c];
                        dn2 += vv * vv;
                        const double st = vv / v.dia[c];
                        gmemw(P.stepL)[3 * (size_t)l + c] = st;
                        jr += (st * v.sl[c]) * v.g[c];
                        const double yv = v.x[c] + st * v.sl[c];
                        y[c] = yv;
                        sn2 += (v.x[c] - yv) * (v.x[c] - yv);
                      }
                      y[3] = v.x[3];
                    });
  DLCLK(4)
  {
    double r3[3] = {sn2, dn2, jr};
    blockSumN<RB, 3>(r3, sh);
    sn2 = r3[0];
    dn2 = r3[1];
    jr = r3[2];
  }
  DLCLK(5)
  DLCLK_END
  if (t != 0) return;
  s.dogleg_step_norm = (dcase == 1) ? gauss_newton_norm : (dcase == 2) ? radius : sqrt(dn2);
  s.step_norm = sqrt(sn2);
  // model_cost_change = -(J step).(r + J step / 2), step = ca v_c + cb v_g
  const double jj = (ca * ca) * s.jcc + 2.0 * (ca * cb) * s.jcg + (cb * cb) * s.jgg;
  s.model_cost_change = -(jr + 0.5 * jj);
  if (s.model_cost_change > 0.0) {
    s.step_valid = 1;
    s.consecutive_invalid = 0;
    s.eval_cand = 1;
  } else {
    // HandleInvalidStep + DoglegStrategy::StepIsInvalid; the step that reaches
    // max_num_consecutive_invalid_steps ends the solve unrecorded (iteration and unsuccessful step
    // not counted, as Ceres returns before FinalizeIteration)
    s.step_valid = 0;
    s.eval_cand = 0;
    if (++s.consecutive_invalid >= P.opt.max_num_consecutive_invalid_steps) {
      s.done = 1;
      s.termination = 2;  // FAILURE
      s.iteration -= 1;
      return;
    }
    s.num_unsucc += 1;
    s.mu *= 10.0;
    s.need_gn = 1;
    finalizeIteration(P, s);
  }
}

// The factors' J*v on their own: in the iteration they are the trailing workgroups of
// k_lm_backsub_jv (launch_lm_backsub); this launch serves okvisgpu_time_kernel's table.
__global__ __launch_bounds__(256) void k_jv(const DevProblem* __restrict__ Pp) { jvGroups(*Pp, (int)blockIdx.x); }
void launch_jv(const DevProblem& P, hipStream_t s) {
  if (jvBlocks(P) > 0) hipLaunchKernelGGL(k_jv, dim3(jvBlocks(P)), dim3(256), 0, s, P.self);
}
void launch_reduce(const DevProblem& P, int mode, hipStream_t s) {
  if (fewWindows(P.n_win, P.cu_count)) hipLaunchKernelGGL(k_reduce<kRBFew>, dim3(P.n_win), dim3(kRBFew), 0, s, P.self, mode);
  else hipLaunchKernelGGL(k_reduce<kRBBatch>, dim3(P.n_win), dim3(kRBBatch), 0, s, P.self, mode);
}
// (256 threads for every batch size: the few-window iteration runs the same test inside the
// assembly launch, k_assemble_few, and both forms must give the same bits)
void launch_gradnorm(const DevProblem& P, int lin_mode, hipStream_t s) {
  hipLaunchKernelGGL(k_gradnorm<kRBBatch>, dim3(P.n_win), dim3(kRBBatch), 0, s, P.self, lin_mode);
}
void launch_dogleg(const DevProblem& P, hipStream_t s) {
  if (fewWindows(P.n_win, P.cu_count)) hipLaunchKernelGGL(k_dogleg<kRBFew>, dim3(P.n_win), dim3(kRBFew), 0, s, P.self);
  else hipLaunchKernelGGL(k_dogleg<kRBBatch>, dim3(P.n_win), dim3(kRBBatch), 0, s, P.self);
}

// Write-back staging: a window whose current parameters are set 1 gets them copied into set 0, so
// one device-to-host copy of set 0 holds every window's result (set 0 is then that window's
// candidate buffer, which the next step overwrites before reading). One workgroup per window.
__global__ __launch_bounds__(256) void k_select_current(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  if (P.st[w].xcur != 1) return;
  auto copy = [&](const int32_t* range, int stride, const double* src, double* dst) {
    const int64_t b = (int64_t)range[2 * w] * stride, e = (int64_t)range[2 * w + 1] * stride;
    for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) dst[i] = src[i];
  };
  copy(P.win_pose_range, 7, P.pose[1], P.pose[0]);
  copy(P.win_sb_range, 9, P.sb[1], P.sb[0]);
  copy(P.win_lm_range, 4, P.lm[1], P.lm[0]);
}

void launch_select_current(const DevProblem& P, hipStream_t s) {
  if (P.n_win > 0) hipLaunchKernelGGL(k_select_current, dim3(P.n_win), dim3(256), 0, s, P.self);
}

}  // namespace okg
