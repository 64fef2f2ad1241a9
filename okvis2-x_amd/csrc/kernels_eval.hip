// kernels_eval.hip — batched cost-functor evaluation for gfx950 (FP64).
//
//  k_eval_obs    one thread per ReprojectionError residual block: residual + minimal Jacobians
//                (pose 2x6, landmark 2x3) with the Cauchy(1) corrector applied, written as
//                structure-of-arrays planes (coalesced 8-byte-per-lane stores).
//                Restates implementation/ReprojectionError.hpp:71-220 fused: with
//                A = L * Jh * C_CW,  J_pose = [w A, -A [p]x],  J_lm = -A  (the reference's
//                J0_minimal = Jh_w T_CS J and J1 = -Jh_w T_CW, first three columns).
//  k_eval_imu    one wavefront per ImuError: the data-dependent re-preintegration decision
//                (ImuError.cpp:833-859), the trapezoidal re-preintegration with covariance
//                propagation (ImuError.cpp:258-466; the four dP/dsigma recursions are linear in
//                the noise densities and are carried as their sum P = sum sigma^2 dP/dsigma),
//                the pseudo-inverse square root of P via a parallel (round-robin) Jacobi
//                eigen-solver (PseudoInverse.hpp:132-158), then residual + minimal Jacobians
//                (ImuError.cpp:861-1000).
//  k_eval_priors one thread per PoseError / SpeedAndBiasError (PoseError.cpp:73-125,
//                SpeedAndBiasError.cpp:67-101).
//
// mode: 0 = current point (lin[lcur]); 1 = candidate point (X[1-xcur] -> lin[1-lcur], only windows
// flagged eval_cand); 2 = initial evaluation (also residuals whose blocks are all constant, which
// Ceres evaluates once for fixed_cost); 3 = like 2 without the robust loss (parity hook).
#include <cfloat>

#include "device_problem.hpp"
#include "launch.hpp"
#include "okvisgpu_math.hpp"

namespace okg {

__device__ __forceinline__ bool evalSelect(const DevProblem& P, int w, int mode, int& xs, int& lb) {
  const WinState& s = P.st[w];
  if (s.done) return false;
  if (mode == 1) {  // candidate
    if (!s.eval_cand) return false;
    xs = 1 - s.xcur;
    lb = 1 - s.lcur;
  } else {
    xs = s.xcur;
    lb = s.lcur;
  }
  return true;
}

__global__ __launch_bounds__(256) void k_eval_obs(const DevProblem* __restrict__ Pp, int mode) {
  const DevProblem& P = *Pp;
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= P.n_obs) return;
  const int w = P.obs_win[o];
  int xs, lb;
  if (!evalSelect(P, w, mode, xs, lb)) return;
  uint8_t flags = P.obs_flags[o];
  if ((flags & 2) && mode < 2) return;  // fixed residual: only evaluated once (fixed_cost)
  if (mode == 3) flags &= ~1;           // raw functor output (parity hook): no loss

  const double* pose = P.pose[xs] + 7 * (size_t)P.obs_pose[o];
  const double* hp = P.lm[xs] + 4 * (size_t)P.obs_lm[o];
  const int ci = P.obs_cam[o];
  const double* ex = P.extr + 7 * ci;
  const double* cp = P.cam + 9 * ci;
  const Cam cam{(int)cp[0], cp[1], cp[2], cp[3], cp[4], cp[5], cp[6], cp[7], cp[8]};

  double C_WS[9], C_SC[9];
  qrot(qnormalize(Q{pose[3], pose[4], pose[5], pose[6]}), C_WS);
  qrot(qnormalize(Q{ex[3], ex[4], ex[5], ex[6]}), C_SC);
  const double w4 = hp[3];
  // p = hp_W.xyz - t_WS w ; hp_S = C_SW p ; hp_C = C_CS (hp_S - t_SC w)
  const double p[3] = {hp[0] - pose[0] * w4, hp[1] - pose[1] * w4, hp[2] - pose[2] * w4};
  double hS[3];
  mtv3(C_WS, p, hS);
  const double q3[3] = {hS[0] - ex[0] * w4, hS[1] - ex[1] * w4, hS[2] - ex[2] * w4};
  double hC[3];
  mtv3(C_SC, q3, hC);

  double kp[2], Jh[6];
  projectHomogeneous(cam, hC[0], hC[1], hC[2], w4, kp, Jh, true);
  const double* L = P.obs_L + 4 * (size_t)o;
  const double* m = P.obs_kp + 2 * (size_t)o;
  const double e0 = m[0] - kp[0], e1 = m[1] - kp[1];
  double r0 = L[0] * e0 + L[1] * e1;
  double r1 = L[2] * e0 + L[3] * e1;
  // Jh_w = L Jh (2x3); C_CW = C_SC^T C_WS^T ; A = Jh_w C_CW
  double Jw[6];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    Jw[c] = L[0] * Jh[c] + L[1] * Jh[3 + c];
    Jw[3 + c] = L[2] * Jh[c] + L[3] * Jh[3 + c];
  }
  double B[6];  // Jh_w C_CS = Jh_w C_SC^T : B[r][k] = sum_j Jw[r][j] C_SC[k][j]
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int k = 0; k < 3; ++k)
      B[r * 3 + k] = Jw[r * 3 + 0] * C_SC[k * 3 + 0] + Jw[r * 3 + 1] * C_SC[k * 3 + 1] + Jw[r * 3 + 2] * C_SC[k * 3 + 2];
  double A[6];  // B C_SW = B C_WS^T : A[r][c] = sum_k B[r][k] C_WS[c][k]
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      A[r * 3 + c] = B[r * 3 + 0] * C_WS[c * 3 + 0] + B[r * 3 + 1] * C_WS[c * 3 + 1] + B[r * 3 + 2] * C_WS[c * 3 + 2];

  // Cauchy(1) corrector (rho'' < 0 branch: scale residual and Jacobian by sqrt(rho'))
  const double sq = r0 * r0 + r1 * r1;
  double cost, sc = 1.0;
  if (flags & 1) {
    const double sum = 1.0 + sq;
    cost = 0.5 * log(sum);
    sc = sqrt(fmax(DBL_MIN, 1.0 / sum));
  } else {
    cost = 0.5 * sq;
  }
  double* lin = P.obs_lin[lb];
  const int64_t S = P.obs_stride;
  lin[0 * S + o] = r0 * sc;
  lin[1 * S + o] = r1 * sc;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const double a0 = A[r * 3 + 0], a1 = A[r * 3 + 1], a2 = A[r * 3 + 2];
    // -A [p]x : row a^T [p]x = (a1 p2 - a2 p1, a2 p0 - a0 p2, a0 p1 - a1 p0) ... times -1
    const double c0 = -(a1 * p[2] - a2 * p[1]);
    const double c1 = -(a2 * p[0] - a0 * p[2]);
    const double c2 = -(a0 * p[1] - a1 * p[0]);
    lin[(2 + r * 6 + 0) * S + o] = w4 * a0 * sc;
    lin[(2 + r * 6 + 1) * S + o] = w4 * a1 * sc;
    lin[(2 + r * 6 + 2) * S + o] = w4 * a2 * sc;
    lin[(2 + r * 6 + 3) * S + o] = c0 * sc;
    lin[(2 + r * 6 + 4) * S + o] = c1 * sc;
    lin[(2 + r * 6 + 5) * S + o] = c2 * sc;
    lin[(14 + r * 3 + 0) * S + o] = -a0 * sc;
    lin[(14 + r * 3 + 1) * S + o] = -a1 * sc;
    lin[(14 + r * 3 + 2) * S + o] = -a2 * sc;
  }
  P.obs_cost[lb][o] = cost;
}

// ------------------------------------------------------------------------------------ IMU
namespace {

struct ImuPre {  // preintegrated quantities (ImuError.hpp:273-304), register resident per lane
  Q dq;
  double Ci[9], Cdi[9], ai[3], adi[3], dadbg[9], dvdbg[9], dpdbg[9];
};

__device__ void loadPre(const double* s, ImuPre& p) {
  p.dq = Q{s[2], s[3], s[4], s[5]};
  for (int i = 0; i < 9; ++i) {
    p.Ci[i] = s[6 + i];
    p.Cdi[i] = s[15 + i];
    p.dadbg[i] = s[30 + i];
    p.dvdbg[i] = s[39 + i];
    p.dpdbg[i] = s[48 + i];
  }
  for (int i = 0; i < 3; ++i) {
    p.ai[i] = s[24 + i];
    p.adi[i] = s[27 + i];
  }
}

// F_delta of one integration step (ImuError.cpp:395-410); returns element (i, j).
struct FStep {
  double b03[9], b09[9], b012[9], b39[9], b63[9], b69[9], b612[9], dt;
  __device__ double at(int i, int j) const {
    const int bi = i / 3, bj = j / 3, ii = i % 3, jj = j % 3;
    double v = (i == j) ? 1.0 : 0.0;
    if (bi == 0) {
      if (bj == 1) v = b03[ii * 3 + jj];
      else if (bj == 2) v = (ii == jj) ? dt : 0.0;
      else if (bj == 3) v = b09[ii * 3 + jj];
      else if (bj == 4) v = b012[ii * 3 + jj];
    } else if (bi == 1) {
      if (bj == 3) v = b39[ii * 3 + jj];
    } else if (bi == 2) {
      if (bj == 1) v = b63[ii * 3 + jj];
      else if (bj == 3) v = b69[ii * 3 + jj];
      else if (bj == 4) v = b612[ii * 3 + jj];
    }
    return v;
  }
};

// Parallel cyclic Jacobi (round-robin ordering, 8 disjoint rotations per round) on a 16x16
// symmetric matrix in LDS whose last row/column is a decoupled pad. One wavefront.
__device__ void jacobiEigen16(double* A, double* V, double* rot, int lane) {
  for (int e = lane; e < 256; e += 64) V[e] = ((e >> 4) == (e & 15)) ? 1.0 : 0.0;
  __syncthreads();
  for (int sweep = 0; sweep < 100; ++sweep) {
    // convergence test: off-diagonal vs diagonal energy (same criterion as the oracle)
    double off = 0.0, dg = 0.0;
    for (int e = lane; e < 256; e += 64) {
      const int i = e >> 4, j = e & 15;
      const double a = A[e];
      if (i == j) dg += a * a;
      else if (i < j) off += a * a;
    }
    for (int sh = 32; sh > 0; sh >>= 1) {
      off += __shfl_xor(off, sh, 64);
      dg += __shfl_xor(dg, sh, 64);
    }
    if (off <= 1e-36 * dg || off == 0.0) break;
    for (int round = 0; round < 15; ++round) {
      if (lane < 8) {
        int p, q;
        if (lane == 0) { p = 15; q = round; }
        else { p = (round + lane) % 15; q = (round + 15 - lane) % 15; }
        if (p > q) { const int t = p; p = q; q = t; }
        const double apq = A[p * 16 + q];
        double c = 1.0, s = 0.0;
        if (apq != 0.0) {
          const double app = A[p * 16 + p], aqq = A[q * 16 + q];
          const double theta = (aqq - app) / (2.0 * apq);
          const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          s = t * c;
        }
        rot[lane * 4 + 0] = c;
        rot[lane * 4 + 1] = s;
        rot[lane * 4 + 2] = (double)p;
        rot[lane * 4 + 3] = (double)q;
      }
      __syncthreads();
      // columns: A <- A J, V <- V J   (8 pairs x 16 rows, two matrices)
      for (int t = lane; t < 256; t += 64) {
        const int k = (t >> 4) & 7, row = t & 15;
        double* M = (t < 128) ? A : V;
        const double c = rot[k * 4], s = rot[k * 4 + 1];
        const int p = (int)rot[k * 4 + 2], q = (int)rot[k * 4 + 3];
        const double mp = M[row * 16 + p], mq = M[row * 16 + q];
        M[row * 16 + p] = c * mp - s * mq;
        M[row * 16 + q] = s * mp + c * mq;
      }
      __syncthreads();
      // rows: A <- J^T A
      for (int t = lane; t < 128; t += 64) {
        const int k = t >> 4, col = t & 15;
        const double c = rot[k * 4], s = rot[k * 4 + 1];
        const int p = (int)rot[k * 4 + 2], q = (int)rot[k * 4 + 3];
        const double mp = A[p * 16 + col], mq = A[q * 16 + col];
        A[p * 16 + col] = c * mp - s * mq;
        A[q * 16 + col] = s * mp + c * mq;
      }
      __syncthreads();
      if (lane < 8) {
        const int p = (int)rot[lane * 4 + 2], q = (int)rot[lane * 4 + 3];
        if (rot[lane * 4 + 1] != 0.0) {
          A[p * 16 + q] = 0.0;
          A[q * 16 + p] = 0.0;
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace

__global__ __launch_bounds__(64) void k_eval_imu(const DevProblem* __restrict__ Pp, int mode) {
  const DevProblem& P = *Pp;
  const int f = blockIdx.x;
  if (f >= P.n_imu) return;
  const int w = P.imu_win[f];
  int xs, lb;
  if (!evalSelect(P, w, mode, xs, lb)) return;
  if ((P.imu_flags[f] & 2) && mode < 2) return;
  const int lane = threadIdx.x;

  __shared__ double sP[256], sF[256], sT[256], sV[256], sU[225];
  __shared__ double sRot[32];
  __shared__ double sFF[450];

  const int* blk = P.imu_blocks + 4 * f;
  const double* p0 = P.pose[xs] + 7 * (size_t)blk[0];
  const double* sb0 = P.sb[xs] + 9 * (size_t)blk[1];
  const double* p1 = P.pose[xs] + 7 * (size_t)blk[2];
  const double* sb1 = P.sb[xs] + 9 * (size_t)blk[3];
  double* state = P.imu_state + (size_t)f * kImuState;
  const double* par = P.imu_par + 7 * w;
  const double a_max = par[0], g_max = par[1], sg_c = par[2], sa_c = par[3], sgw_c = par[4], saw_c = par[5],
               gmag = par[6];
  const int64_t t0 = P.imu_t0[f], t1 = P.imu_t1[f];
  const int sbeg = P.imu_sbegin[f], send = P.imu_sbegin[f + 1];

  // ---- re-preintegration decision (ImuError.cpp:833-859)
  int redoCounter = (int)state[0];
  bool redo = state[1] != 0.0;
  double Db[6];
  for (int k = 0; k < 6; ++k) Db[k] = sb0[3 + k] - state[57 + 3 + k];
  redo = redo || (sqrt(Db[0] * Db[0] + Db[1] * Db[1] + Db[2] * Db[2]) > 0.0003);
  const bool doRedo = (redo && ((send - sbeg) < 50 || P.opt.redo_propagation_always)) || redoCounter == 0;
  bool success = true;
  ImuPre pre;

  const bool covered = (send > sbeg) && P.imu_ts[send - 1] >= t1;
  if (doRedo && !covered) {
    // redoPreintegration returns -1 before touching any state (ImuError.cpp:270-273)
    loadPre(state, pre);
    for (int e = lane; e < 225; e += 64) sU[e] = state[66 + e];
    __syncthreads();
    redoCounter++;
    for (int k = 0; k < 6; ++k) Db[k] = 0.0;
    redo = false;
  } else if (doRedo) {
    // ---- redoPreintegration (ImuError.cpp:258-466)
    pre.dq = Q{0, 0, 0, 1};
    for (int i = 0; i < 9; ++i) { pre.Ci[i] = 0; pre.Cdi[i] = 0; pre.dadbg[i] = 0; pre.dvdbg[i] = 0; pre.dpdbg[i] = 0; }
    for (int i = 0; i < 3; ++i) { pre.ai[i] = 0; pre.adi[i] = 0; }
    double cross[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int e = lane; e < 256; e += 64) sP[e] = 0.0;
    const double bg[3] = {sb0[3], sb0[4], sb0[5]}, ba[3] = {sb0[6], sb0[7], sb0[8]};
    int64_t time = t0;
    bool hasStarted = false;
    int steps = 0;
    const int N = send - sbeg;
    {
      for (int it = 0; it < N; ++it) {
        const int s0 = sbeg + it;
        const int s1 = (it + 1 < N) ? s0 + 1 : s0;
        double om0[3], ac0[3], om1[3], ac1[3];
        for (int k = 0; k < 3; ++k) {
          om0[k] = P.imu_ga[6 * (size_t)s0 + k];
          ac0[k] = P.imu_ga[6 * (size_t)s0 + 3 + k];
          om1[k] = P.imu_ga[6 * (size_t)s1 + k];
          ac1[k] = P.imu_ga[6 * (size_t)s1 + 3 + k];
        }
        int64_t nexttime = (it + 1 == N) ? t1 : P.imu_ts[s0 + 1];
        double dt = durToSec(nexttime - time);
        if (t1 < nexttime) {
          const double interval = durToSec(nexttime - P.imu_ts[s0]);
          nexttime = t1;
          dt = durToSec(nexttime - time);
          const double r = dt / interval;
          for (int k = 0; k < 3; ++k) {
            om1[k] = (1.0 - r) * om0[k] + r * om1[k];
            ac1[k] = (1.0 - r) * ac0[k] + r * ac1[k];
          }
        }
        if (dt <= 0.0) continue;
        if (!hasStarted) {
          hasStarted = true;
          const double r = dt / durToSec(nexttime - P.imu_ts[s0]);
          for (int k = 0; k < 3; ++k) {
            om0[k] = r * om0[k] + (1.0 - r) * om1[k];
            ac0[k] = r * ac0[k] + (1.0 - r) * ac1[k];
          }
        }
        double gyr_sat = 1.0, acc_sat = 1.0;
        for (int k = 0; k < 3; ++k) {
          if (fabs(om0[k]) > g_max || fabs(om1[k]) > g_max) gyr_sat = 100.0;
          if (fabs(ac0[k]) > a_max || fabs(ac1[k]) > a_max) acc_sat = 100.0;
        }
        // orientation
        double w_true[3], a_true[3];
        for (int k = 0; k < 3; ++k) {
          w_true[k] = 0.5 * (om0[k] + om1[k]) - bg[k];
          a_true[k] = 0.5 * (ac0[k] + ac1[k]) - ba[k];
        }
        const double theta_half = sqrt(w_true[0] * w_true[0] + w_true[1] * w_true[1] + w_true[2] * w_true[2]) * 0.5 * dt;
        const double sth = sinc(theta_half) * 0.5 * dt;
        const Q dq{sth * w_true[0], sth * w_true[1], sth * w_true[2], cos(theta_half)};
        const Q dq1 = qmul(pre.dq, dq);
        double C[9], C1[9], CC1[9];
        qrot(pre.dq, C);
        qrot(dq1, C1);
        for (int i = 0; i < 9; ++i) CC1[i] = C[i] + C1[i];
        double CCa[3];
        mv3(CC1, a_true, CCa);
        double Ci1[9], ai1[3];
        for (int i = 0; i < 9; ++i) Ci1[i] = pre.Ci[i] + 0.5 * dt * CC1[i];
        for (int i = 0; i < 3; ++i) ai1[i] = pre.ai[i] + 0.5 * dt * CCa[i];
        FStep F;
        F.dt = dt;
        {
          double v[3];
          for (int i = 0; i < 3; ++i) v[i] = pre.ai[i] * dt + 0.25 * dt * dt * CCa[i];
          crossMx(v, F.b03);
          for (int i = 0; i < 9; ++i) F.b03[i] = -F.b03[i];
          for (int i = 0; i < 3; ++i) v[i] = 0.5 * dt * CCa[i];
          crossMx(v, F.b63);
          for (int i = 0; i < 9; ++i) F.b63[i] = -F.b63[i];
        }
        for (int i = 0; i < 9; ++i) {
          pre.Cdi[i] += pre.Ci[i] * dt + 0.25 * dt * dt * CC1[i];
          F.b012[i] = -pre.Ci[i] * dt + 0.25 * dt * dt * CC1[i];
          F.b39[i] = -dt * C1[i];
          F.b612[i] = -0.5 * dt * CC1[i];
        }
        for (int i = 0; i < 3; ++i) pre.adi[i] += pre.ai[i] * dt + 0.25 * dt * dt * CCa[i];
        // Jacobian parts (ImuError.cpp:385-392)
        double wdt[3] = {w_true[0] * dt, w_true[1] * dt, w_true[2] * dt};
        double Jr[9], CJr[9];
        rightJacobian(wdt, Jr);
        mm3(C1, Jr, CJr);
        for (int i = 0; i < 9; ++i) pre.dadbg[i] += CJr[i] * dt;
        double Rdqi[9], tmp[9], cross1[9];
        qrot(qinv(dq), Rdqi);
        mm3(Rdqi, cross, tmp);
        for (int i = 0; i < 9; ++i) cross1[i] = tmp[i] + Jr[i] * dt;
        double ax[9], t1m[9], t2m[9], X[9];
        crossMx(a_true, ax);
        mm3(C, ax, tmp);
        mm3(tmp, cross, t1m);
        mm3(C1, ax, tmp);
        mm3(tmp, cross1, t2m);
        for (int i = 0; i < 9; ++i) X[i] = t1m[i] + t2m[i];
        for (int i = 0; i < 9; ++i) {
          F.b09[i] = dt * pre.dvdbg[i] + 0.25 * dt * dt * X[i];
          F.b69[i] = 0.5 * dt * X[i];
          pre.dpdbg[i] += dt * pre.dvdbg[i] + 0.25 * dt * dt * X[i];
        }
        // covariance propagation P <- F P F^T + sum_j sigma_j^2 K_j (ImuError.cpp:412-426)
        for (int e = lane; e < 225; e += 64) sF[e] = F.at(e / 15, e % 15);
        __syncthreads();
        for (int e = lane; e < 225; e += 64) {
          const int i = e / 15, j = e % 15;
          double acc = 0.0;
          for (int m = 0; m < 15; ++m) acc += sF[i * 15 + m] * sP[m * 15 + j];
          sT[e] = acc;
        }
        __syncthreads();
        for (int e = lane; e < 225; e += 64) {
          const int i = e / 15, j = e % 15;
          double acc = 0.0;
          for (int m = 0; m < 15; ++m) acc += sT[i * 15 + m] * sF[j * 15 + m];
          if (i == j) {
            const int b = i / 3;
            if (b == 0) acc += sa_c * sa_c * (0.5 * dt * dt * dt * acc_sat * acc_sat * acc_sat);
            else if (b == 1) acc += sg_c * sg_c * (gyr_sat * dt);
            else if (b == 2) acc += sa_c * sa_c * (acc_sat * dt);
            else if (b == 3) acc += sgw_c * sgw_c * dt;
            else acc += saw_c * saw_c * dt;
          }
          sP[e] = acc;
        }
        __syncthreads();
        // memory shift
        pre.dq = dq1;
        for (int i = 0; i < 9; ++i) { pre.Ci[i] = Ci1[i]; cross[i] = cross1[i]; }
        for (int i = 0; i < 9; ++i) pre.dvdbg[i] += 0.5 * dt * X[i];
        for (int i = 0; i < 3; ++i) pre.ai[i] = ai1[i];
        time = nexttime;
        ++steps;
        if (nexttime == t1) break;
      }
    }
    // symmetrise, pad to 16x16 and take the pseudo-inverse square root
    for (int e = lane; e < 256; e += 64) {
      const int i = e >> 4, j = e & 15;
      sT[e] = (i < 15 && j < 15) ? 0.5 * sP[i * 15 + j] + 0.5 * sP[j * 15 + i] : 0.0;
    }
    __syncthreads();
    jacobiEigen16(sT, sV, sRot, lane);
    double lmax = -1e300;
    for (int i = 0; i < 15; ++i) lmax = fmax(lmax, sT[i * 16 + i]);
    const double tol = fmax(DBL_EPSILON, DBL_EPSILON * 15.0 * lmax);
    for (int e = lane; e < 225; e += 64) {
      const int i = e / 15, j = e % 15;
      const double li = sT[i * 16 + i];
      sU[e] = sqrt(li > tol ? 1.0 / li : 1.0 / tol) * sV[j * 16 + i];
    }
    __syncthreads();
    if (steps == 0) success = false;
    redoCounter++;
    for (int k = 0; k < 6; ++k) Db[k] = 0.0;
    redo = false;
    // store the new state (lane-parallel)
    if (lane == 0) {
      state[2] = pre.dq.x; state[3] = pre.dq.y; state[4] = pre.dq.z; state[5] = pre.dq.w;
      for (int i = 0; i < 9; ++i) {
        state[6 + i] = pre.Ci[i];
        state[15 + i] = pre.Cdi[i];
        state[30 + i] = pre.dadbg[i];
        state[39 + i] = pre.dvdbg[i];
        state[48 + i] = pre.dpdbg[i];
        state[57 + i] = sb0[i];
      }
      for (int i = 0; i < 3; ++i) { state[24 + i] = pre.ai[i]; state[27 + i] = pre.adi[i]; }
      state[291] = (double)steps;
    }
    for (int e = lane; e < 225; e += 64) state[66 + e] = sU[e];
  } else {
    loadPre(state, pre);
    for (int e = lane; e < 225; e += 64) sU[e] = state[66 + e];
    __syncthreads();
  }
  if (lane == 0) {
    state[0] = (double)redoCounter;
    state[1] = redo ? 1.0 : 0.0;
  }

  // ---- residual and minimal Jacobians (ImuError.cpp:861-1000)
  const Q q0 = qnormalize(Q{p0[3], p0[4], p0[5], p0[6]});
  const Q q1 = qnormalize(Q{p1[3], p1[4], p1[5], p1[6]});
  double C0[9];
  qrot(q0, C0);  // C_WS_0 ; C_S0_W = C0^T
  const double Dt = durToSec(t1 - t0);
  double dp[3], dv[3];
  const double gW[3] = {0.0, 0.0, gmag};
  for (int k = 0; k < 3; ++k) {
    dp[k] = p0[k] - p1[k] + sb0[k] * Dt - 0.5 * gW[k] * Dt * Dt;
    dv[k] = sb0[k] - sb1[k] - gW[k] * Dt;
  }
  double adb[3];
  mv3(pre.dadbg, Db, adb);
  const Q Dq = qmul(deltaQ(-adb[0], -adb[1], -adb[2]), pre.dq);
  const Q q1i = qinv(q1);
  // F0 / F1 blocks needing quaternion algebra
  double M33a[9], M33b[9], M33c[9];
  {
    double Pm[16], Om[16], R[16];
    qplusM(qmul(Dq, q1i), Pm);
    qoplusM(q0, Om);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 4; ++k) s += Pm[r * 4 + k] * Om[k * 4 + c];
        M33a[r * 3 + c] = s;  // F0(3,3)
      }
    qoplusM(qmul(q1i, q0), Pm);
    qoplusM(Dq, Om);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 4; ++k) s += Pm[r * 4 + k] * Om[k * 4 + c];
        R[r * 3 + c] = s;
      }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        M33b[r * 3 + c] = -(R[r * 3 + 0] * pre.dadbg[0 * 3 + c] + R[r * 3 + 1] * pre.dadbg[1 * 3 + c] +
                            R[r * 3 + 2] * pre.dadbg[2 * 3 + c]);  // F0(3,9)
    double Pd[16], O0[16], P1i[16], T4[16];
    qplusM(Dq, Pd);
    qoplusM(q0, O0);
    qplusM(q1i, P1i);
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) {
        double s = 0;
        for (int k = 0; k < 4; ++k) s += Pd[r * 4 + k] * O0[k * 4 + c];
        T4[r * 4 + c] = s;
      }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 4; ++k) s += T4[r * 4 + k] * P1i[k * 4 + c];
        M33c[r * 3 + c] = -s;  // F1(3,3)
      }
  }
  double dpx[9], dvx[9], Cdp[9], Cdv[9];
  crossMx(dp, dpx);
  crossMx(dv, dvx);
  // C_S0_W [dp]x and C_S0_W [dv]x
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      Cdp[r * 3 + c] = C0[0 * 3 + r] * dpx[0 * 3 + c] + C0[1 * 3 + r] * dpx[1 * 3 + c] + C0[2 * 3 + r] * dpx[2 * 3 + c];
      Cdv[r * 3 + c] = C0[0 * 3 + r] * dvx[0 * 3 + c] + C0[1 * 3 + r] * dvx[1 * 3 + c] + C0[2 * 3 + r] * dvx[2 * 3 + c];
    }
  // FF = [F0 | F1] (15 x 30) into LDS
  for (int e = lane; e < 450; e += 64) {
    const int i = e / 30, j = e % 30;
    const bool right = j >= 15;
    const int jj = right ? j - 15 : j;
    const int bi = i / 3, bj = jj / 3, ii = i % 3, kk = jj % 3;
    double v;
    if (!right) {
      v = (i == jj) ? 1.0 : 0.0;
      if (bi == 0) {
        if (bj == 0) v = C0[kk * 3 + ii];
        else if (bj == 1) v = Cdp[ii * 3 + kk];
        else if (bj == 2) v = C0[kk * 3 + ii] * Dt;
        else if (bj == 3) v = pre.dpdbg[ii * 3 + kk];
        else v = -pre.Cdi[ii * 3 + kk];
      } else if (bi == 1) {
        if (bj == 1) v = M33a[ii * 3 + kk];
        else if (bj == 3) v = M33b[ii * 3 + kk];
      } else if (bi == 2) {
        if (bj == 1) v = Cdv[ii * 3 + kk];
        else if (bj == 2) v = C0[kk * 3 + ii];
        else if (bj == 3) v = pre.dvdbg[ii * 3 + kk];
        else if (bj == 4) v = -pre.Ci[ii * 3 + kk];
      }
    } else {
      v = (i == jj) ? -1.0 : 0.0;
      if (bi == 0 && bj == 0) v = -C0[kk * 3 + ii];
      else if (bi == 1 && bj == 1) v = M33c[ii * 3 + kk];
      else if (bi == 2 && bj == 2) v = -C0[kk * 3 + ii];
    }
    sFF[e] = v;
  }
  __syncthreads();
  // error vector (every lane computes it; 15 doubles)
  double err[15];
  {
    double t0v[3], t6v[3];
    mtv3(C0, dp, t0v);
    mtv3(C0, dv, t6v);
    const Q qe = qmul(Dq, qmul(q1i, q0));
    for (int k = 0; k < 3; ++k) {
      // F0.block<3,6>(0,9) * Db = dp_db_g Db_g - C_dint Db_a ; F0.block<3,6>(6,9) * Db = dv_db_g Db_g - C_int Db_a
      const double e0 = pre.dpdbg[k * 3 + 0] * Db[0] + pre.dpdbg[k * 3 + 1] * Db[1] + pre.dpdbg[k * 3 + 2] * Db[2] -
                        (pre.Cdi[k * 3 + 0] * Db[3] + pre.Cdi[k * 3 + 1] * Db[4] + pre.Cdi[k * 3 + 2] * Db[5]);
      const double e6 = pre.dvdbg[k * 3 + 0] * Db[0] + pre.dvdbg[k * 3 + 1] * Db[1] + pre.dvdbg[k * 3 + 2] * Db[2] -
                        (pre.Ci[k * 3 + 0] * Db[3] + pre.Ci[k * 3 + 1] * Db[4] + pre.Ci[k * 3 + 2] * Db[5]);
      err[k] = t0v[k] + pre.adi[k] + e0;
      err[6 + k] = t6v[k] + pre.ai[k] + e6;
    }
    err[3] = 2 * qe.x; err[4] = 2 * qe.y; err[5] = 2 * qe.z;
    for (int k = 0; k < 6; ++k) err[9 + k] = sb0[3 + k] - sb1[3 + k];
    if (!success)
      for (int k = 0; k < 15; ++k) err[k] = 0.0;
  }
  double* lin = P.imu_lin[lb] + (size_t)f * kImuLin;
  double rr = 0.0;
  if (lane < 15) {
    for (int k = 0; k < 15; ++k) rr += sU[lane * 15 + k] * err[k];
    lin[lane] = rr;
  }
  for (int e = lane; e < 450; e += 64) {
    const int i = e / 30, j = e % 30;
    double acc = 0.0;
    if (success)
      for (int k = 0; k < 15; ++k) acc += sU[i * 15 + k] * sFF[k * 30 + j];
    lin[15 + e] = acc;
  }
  double c2 = (lane < 15) ? rr * rr : 0.0;
  for (int sh = 32; sh > 0; sh >>= 1) c2 += __shfl_xor(c2, sh, 64);
  if (lane == 0) P.imu_cost[lb][f] = 0.5 * c2;
}

// ------------------------------------------------------------------------------------ priors
__global__ __launch_bounds__(64) void k_eval_priors(const DevProblem* __restrict__ Pp, int mode) {
  const DevProblem& P = *Pp;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < P.n_pprior) {
    const int i = t;
    const int w = P.pp_win[i];
    int xs, lb;
    if (!evalSelect(P, w, mode, xs, lb)) return;
    if (P.pose_f[P.pp_block[i]] < 0 && mode != 2) return;  // prior on a constant block: fixed_cost
    const double* pose = P.pose[xs] + 7 * (size_t)P.pp_block[i];
    const double* m = P.pp_meas + 7 * (size_t)i;
    const double* L = P.pp_L + 36 * (size_t)i;
    const Q q = qnormalize(Q{pose[3], pose[4], pose[5], pose[6]});
    const Q dq = qmul(Q{m[3], m[4], m[5], m[6]}, qinv(q));
    const double e[6] = {m[0] - pose[0], m[1] - pose[1], m[2] - pose[2], 2 * dq.x, 2 * dq.y, 2 * dq.z};
    double* lin = P.pp_lin[lb] + 42 * (size_t)i;
    double c = 0;
    for (int r = 0; r < 6; ++r) {
      double s = 0;
      for (int k = 0; k < 6; ++k) s += L[r * 6 + k] * e[k];
      lin[r] = s;
      c += s * s;
    }
    // J_min = L [-I 0; 0 -plus(dq)_3x3]
    double Pm[16];
    qplusM(dq, Pm);
    for (int r = 0; r < 6; ++r)
      for (int cc = 0; cc < 6; ++cc) {
        double s = 0;
        if (cc < 3) s = -L[r * 6 + cc];
        else
          for (int k = 0; k < 3; ++k) s += L[r * 6 + 3 + k] * (-Pm[k * 4 + (cc - 3)]);
        lin[6 + r * 6 + cc] = s;
      }
    P.pp_cost[lb][i] = 0.5 * c;
    return;
  }
  const int i = t - P.n_pprior;
  if (i >= P.n_sbprior) return;
  const int w = P.sbp_win[i];
  int xs, lb;
  if (!evalSelect(P, w, mode, xs, lb)) return;
  if (P.sb_f[P.sbp_block[i]] < 0 && mode != 2) return;
  const double* sbv = P.sb[xs] + 9 * (size_t)P.sbp_block[i];
  const double* m = P.sbp_meas + 9 * (size_t)i;
  const double* L = P.sbp_L + 81 * (size_t)i;
  double* lin = P.sbp_lin[lb] + 90 * (size_t)i;
  double e[9];
  for (int k = 0; k < 9; ++k) e[k] = m[k] - sbv[k];
  double c = 0;
  for (int r = 0; r < 9; ++r) {
    double s = 0;
    for (int k = 0; k < 9; ++k) s += L[r * 9 + k] * e[k];
    lin[r] = s;
    c += s * s;
    for (int k = 0; k < 9; ++k) lin[9 + r * 9 + k] = -L[r * 9 + k];
  }
  P.sbp_cost[lb][i] = 0.5 * c;
}

// ------------------------------------------------------------------------------------ launchers
void launch_eval_obs(const DevProblem& P, int mode, hipStream_t s) {
  if (P.n_obs > 0) hipLaunchKernelGGL(k_eval_obs, dim3((P.n_obs + 255) / 256), dim3(256), 0, s, P.self, mode);
}
void launch_eval_imu(const DevProblem& P, int mode, hipStream_t s) {
  if (P.n_imu > 0) hipLaunchKernelGGL(k_eval_imu, dim3(P.n_imu), dim3(64), 0, s, P.self, mode);
}
void launch_eval_priors(const DevProblem& P, int mode, hipStream_t s) {
  const int np = P.n_pprior + P.n_sbprior;
  if (np > 0) hipLaunchKernelGGL(k_eval_priors, dim3((np + 63) / 64), dim3(64), 0, s, P.self, mode);
}
void launch_eval(const DevProblem& P, int mode, hipStream_t s) {
  launch_eval_obs(P, mode, s);
  launch_eval_imu(P, mode, s);
  launch_eval_priors(P, mode, s);
}

}  // namespace okg
