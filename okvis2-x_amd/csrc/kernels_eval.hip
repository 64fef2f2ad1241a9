// kernels_eval.hip — batched cost-functor evaluation for gfx950 (FP64).
//
//  k_eval_obs    one thread per ReprojectionError residual block: residual and the 2x3 factor A
//                of both minimal Jacobians (pose 2x6, landmark 2x3), Cauchy(1) corrector applied,
//                written as structure-of-arrays planes (coalesced 8-byte-per-lane stores).
//                Restates implementation/ReprojectionError.hpp:71-220 fused: with
//                A = L * Jh * C_CW,  J_pose = [w A, -A [p]x],  J_lm = -A  (the reference's
//                J0_minimal = Jh_w T_CS J and J1 = -Jh_w T_CW, first three columns).
//  k_eval_imu    one 16-lane group per ImuError (four per wavefront): the data-dependent
//                re-preintegration decision (ImuError.cpp:833-859), the trapezoidal
//                re-preintegration with covariance propagation (ImuError.cpp:258-466; the four
//                dP/dsigma recursions are linear in the noise densities and are carried as their
//                sum P = sum sigma^2 dP/dsigma), a square-root information factor of P
//                (PseudoInverse.hpp:132-158; see the note above the kernel), then residual +
//                minimal Jacobians (ImuError.cpp:861-1000).
//  k_eval_priors one thread per PoseError / SpeedAndBiasError (PoseError.cpp:73-125,
//                SpeedAndBiasError.cpp:67-101).
//
// mode: 0 = current point (lin[lcur]); 1 = candidate point (X[1-xcur] -> lin[1-lcur], only windows
// flagged eval_cand); 2 = initial evaluation (also residuals whose blocks are all constant, which
// Ceres evaluates once for fixed_cost); 3 = like 2 without the robust loss (parity hook).
#include <cfloat>

#include "dev_clock.hpp"
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

// ISO (DevProblem::obs_iso): L = diag(s, s) read as s alone; the zeros enter the same products
template <bool ISO>
__device__ __forceinline__ void evalObsThread(const DevProblem& P, int o, int mode) {
  if (o >= P.n_obs) return;
  // The observation's record (indices, flags, keypoint, information) is loaded together with no
  // branch in between; the window test (evalSelect) reads the WinState fields at once and consumes
  // the record (o >> 31 is 0), so none of these loads is sunk behind it.
  const int w = gmem(P.obs_win)[o], op = gmem(P.obs_pose)[o], ol = gmem(P.obs_lm)[o], ci = gmem(P.obs_cam)[o];
  uint8_t flags = gmem(P.obs_flags)[o];
  double L[4];
  if (ISO) {
    const double sL = gmem(P.obs_Ls)[o];
    L[0] = sL; L[1] = 0.0; L[2] = 0.0; L[3] = sL;
  } else {
    const auto Lp = gmem(P.obs_L + 4 * (size_t)o);
    L[0] = Lp[0]; L[1] = Lp[1]; L[2] = Lp[2]; L[3] = Lp[3];
  }
  const auto mp = gmem(P.obs_kp + 2 * (size_t)o);
  const double m[2] = {mp[0], mp[1]};
  const auto gst = gmem(P.st + w);
  const int sDone = gst->done, sCand = gst->eval_cand, sX = gst->xcur, sL = gst->lcur;
  const bool sel = (sDone == 0) & (mode != 1 || sCand != 0) & !((flags & 2) && mode < 2);
  const int cpose = gmem(P.cam_pose)[ci];
  const auto cp = gmem(P.cam + kCamDoubles * ci);
  const Cam cam = Cam{(int)cp[0], cp[1], cp[2], cp[3], cp[4], cp[5], cp[6], cp[7], cp[8], cp[9], cp[10], cp[11], cp[12]};
  asm volatile("" ::"v"(L[0]), "v"(L[1]), "v"(L[2]), "v"(L[3]), "v"(m[0]), "v"(m[1]), "v"(sX), "v"(sL), "v"(cam.fu),
               "v"(cam.fv), "v"(cam.cu), "v"(cam.cv));
  if (!sel | (((op ^ ol ^ ci ^ (int)flags ^ cpose ^ cam.dist) & (o >> 31)) != 0)) return;  // (fixed: fixed_cost only)
  const int xs = mode == 1 ? 1 - sX : sX, lb = mode == 1 ? 1 - sL : sL;
  if (mode == 3) flags &= ~1;  // raw functor output (parity hook): no loss

  const double* X = pick2(xs, P.pose[0], P.pose[1]);
  const auto posep = gmem(X + 7 * (size_t)op);
  const auto hpp = gmem(pick2(xs, P.lm[0], P.lm[1]) + 4 * (size_t)ol);
  const auto exp_ = gmem(X + 7 * (size_t)cpose);  // T_SC: a pose-kind block (variable or not)
  double pose[7], hp[4], ex[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    pose[k] = posep[k];
    ex[k] = exp_[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) hp[k] = hpp[k];

  double C_WS[9];
  qrot(qnormalize(Q{pose[3], pose[4], pose[5], pose[6]}), C_WS);
  double r[2], A[6], cost;
  obsCore(cam, L, m, pose, C_WS, hp, ex, (flags & 1) != 0, true, r, A, cost);
  // stored: r and A (both Cauchy-scaled); the pose/landmark Jacobians follow from A and the
  // linearisation point (obsJacobians). (Also at a candidate: measured in round 5, storing only the
  // candidate's cost and forming r and A in k_lm_visit<1> after an accepted step took k_eval_obs
  // 0.98 -> 0.63 ms but k_lm_visit<1> 2.84 -> 3.70 ms at 2,048 S50 windows, 195.7k -> 188.0k
  // window-it/s with the same bits: the eval kernel's thread per residual hides the loads' latency
  // that a landmark group's threads do not.)
  double* lin = pick2(lb, P.obs_lin[0], P.obs_lin[1]);
  const int64_t S = P.obs_stride;
  lin[0 * S + o] = r[0];
  lin[1 * S + o] = r[1];
#pragma unroll
  for (int k = 0; k < 6; ++k) lin[(2 + k) * S + o] = A[k];
  pick2(lb, P.obs_cost[0], P.obs_cost[1])[o] = cost;
}

template <bool ISO>
__global__ __launch_bounds__(256) void k_eval_obs(const DevProblem* __restrict__ Pp, int mode) {
  evalObsThread<ISO>(*Pp, (int)(blockIdx.x * blockDim.x + threadIdx.x), mode);
}

// ------------------------------------------------------------------------------------ IMU
namespace {

struct ImuPre {  // preintegrated quantities (ImuError.hpp:273-304), register resident per lane
  Q dq;
  double Ci[9], Cdi[9], ai[3], adi[3], dadbg[9], dvdbg[9], dpdbg[9];
};

template <typename Ptr>
__device__ __forceinline__ void loadPre(Ptr s, ImuPre& p) {
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

// ---- k_eval_imu: one 16-lane group per ImuError, four factors per wavefront
//
// Lane l of a group owns column l of the preintegration covariance P (l < 15). Per integration
// step every lane evaluates the scalar chain (ImuError.cpp:312-410) redundantly, so the
// block-sparse F_delta (ImuError.cpp:395-410) is register resident and P <- F P F^T + Q needs one
// LDS transpose: M = F P column-locally, then P' = F M^T + Q with row l of M read back.
//
// Square-root information. The solver consumes the IMU block only through U^T U, U^T r (with
// r = U e) and column norms of U J, all invariant under U -> Q U for orthogonal Q. The reference
// forms U = diag(lambda^-1/2) V^T from an eigen-decomposition with eigenvalues <= tol clamped to
// tol (PseudoInverse.hpp:132-158, tol = max(eps, eps*15*lambda_max)). When P is provably far from
// that clamp the pseudo-inverse is the inverse, and the Cholesky factor U = L^-1 (P = L L^T) is an
// admissible square root at a fraction of the cost. The proof used on device:
//   lambda_min(P) >= 1 / ||L^-1||_F^2   and   lambda_max(P) <= trace(P);
// if 1/||U||_F^2 > 4 max(eps, eps*15*trace(P)) no eigenvalue is clamped. Otherwise (e.g. zero
// bias random-walk densities) the group runs the cyclic Jacobi eigen-solver and applies the
// reference's clamp exactly.
constexpr int kImuGroup = 16;
constexpr int kImuPerWG = 4;
constexpr int kStepRec = 26;  // dt | dq (4) | a_true (3) | Jr (9) | R(dq)^T (9)
constexpr int kImuK = 4;      // integration steps per chunk (batches)
constexpr int kImuFewChunkWindows = 2;
#ifndef OKG_IMU_FEW_K
#define OKG_IMU_FEW_K 16  // (build knob for A/B measurements)
#endif
#ifndef OKG_IMU_JAC_ROWS
#define OKG_IMU_JAC_ROWS 1  // (build knob: 0 forms the Jacobian by columns)
#endif
#ifndef OKG_IMU_FREG
#define OKG_IMU_FREG 1  // (build knob: 0 reads F_delta from LDS in both products of a step)
#endif
constexpr int kImuKFew = OKG_IMU_FEW_K;  // one or two windows: a chunk covers a 0.1 s keyframe interval's 20 samples
                              // in two rounds (the step records and products are lane-parallel over a
                              // chunk, so fewer chunks shorten a single factor's latency chain)
constexpr int kFStride = 66;  // F_delta blocks of one step (offsets below) | dt | pad (lanes writing
                              // consecutive steps fall on different LDS banks)
constexpr int kS = 17;        // row stride of the 16x16 LDS matrices: lanes walking a column hit
                              // distinct banks (a stride of 16 doubles put every other lane on one)
// per-group LDS (doubles) during the chain: step records, Delta_q and cross_ after each step (slot
// 0 = before the chunk), C_1 Jr, C + C_1, (C + C_1) a, X, F_delta, noise; the P exchange (15 x kS)
// reuses the first 255. After the chain: P / U (sA, 16 x kS), L / eigenvectors (sB, 16 x kS),
// Jacobi rotations (sR, 32). K = steps per chunk.
template <int K>
struct ImuLds {
  static constexpr int rec = 0, q1 = rec + K * 26 /* kStepRec */, cr = q1 + 4 * (K + 1), cj = cr + 9 * (K + 1),
                       m = 0, cc = (cj + 9 * K > 256 ? cj + 9 * K : 256), ca = cc + 9 * K, xx = ca + 3 * K,
                       f = xx + 9 * K, nz = f + kFStride * K, carry = nz + 5 * K, total = carry + 13;
  static_assert(cj + 9 * K <= cc && 15 * kS <= cc, "chain records / P exchange overlap the sums");
  static_assert(total >= 32 * kS + 32, "the square-root phase needs sA, sB and sR");
};
static_assert(ImuLds<kImuK>::total * 8 * 4 <= 20480, "LDS for eight workgroups (two waves per SIMD) per CU");
static_assert(ImuLds<kImuKFew>::total * 8 * 4 <= 80 * 1024, "two few-window workgroups per CU");

// F_delta (ImuError.cpp:395-410) of one step in LDS: non-identity 3x3 blocks
constexpr int kF03 = 0, kF09 = 9, kF012 = 18, kF39 = 27, kF63 = 36, kF69 = 45, kF612 = 54, kFdt = 63;

// Row r of -[w]x times u, the zero entry of the row skipped: the two remaining products in the
// column order of the full row (F03 and F63 are such blocks; their slots hold w only, 3 LDS reads
// per applyF instead of 9).
__device__ __forceinline__ double negSkewRow(const double* w, int r, double u0, double u1, double u2) {
  return r == 0 ? w[2] * u1 + (-w[1]) * u2 : (r == 1 ? (-w[2]) * u0 + w[0] * u2 : w[1] * u0 + (-w[0]) * u1);
}
// out = F v   (block rows: 0 dp, 1 dalpha, 2 dv, 3 bg, 4 ba); F read from LDS (group broadcast)
__device__ __forceinline__ void applyF(const double* F, const double* v, double* out) {
  const double dt = F[kFdt];
  const double w03[3] = {F[kF03], F[kF03 + 1], F[kF03 + 2]}, w63[3] = {F[kF63], F[kF63 + 1], F[kF63 + 2]};
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    double a = v[r];
    a += negSkewRow(w03, r, v[3], v[4], v[5]);
    a += dt * v[6 + r];
    a += F[kF09 + r * 3 + 0] * v[9] + F[kF09 + r * 3 + 1] * v[10] + F[kF09 + r * 3 + 2] * v[11];
    a += F[kF012 + r * 3 + 0] * v[12] + F[kF012 + r * 3 + 1] * v[13] + F[kF012 + r * 3 + 2] * v[14];
    out[r] = a;
    out[3 + r] = v[3 + r] + F[kF39 + r * 3 + 0] * v[9] + F[kF39 + r * 3 + 1] * v[10] + F[kF39 + r * 3 + 2] * v[11];
    double c = negSkewRow(w63, r, v[3], v[4], v[5]);
    c += v[6 + r];
    c += F[kF69 + r * 3 + 0] * v[9] + F[kF69 + r * 3 + 1] * v[10] + F[kF69 + r * 3 + 2] * v[11];
    c += F[kF612 + r * 3 + 0] * v[12] + F[kF612 + r * 3 + 1] * v[13] + F[kF612 + r * 3 + 2] * v[14];
    out[6 + r] = c;
  }
#pragma unroll
  for (int r = 9; r < 15; ++r) out[r] = v[r];
}

__device__ __forceinline__ double groupSum(double v) {  // sum over the 16 lanes of a group
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}


// Cyclic Jacobi with round-robin ordering on the 16x16 (15 + decoupled pad) symmetric matrix A of
// every group with `need` set; V receives the eigenvectors. Uniform control flow over the wave.
__device__ void groupJacobi(double* A, double* V, double* rot, int l, bool need) {
  for (int e = l; e < 256; e += kImuGroup) V[(e >> 4) * kS + (e & 15)] = ((e >> 4) == (e & 15)) ? 1.0 : 0.0;
  __syncthreads();
  bool run = need;
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0, dg = 0.0;
    for (int j = 0; j < 16; ++j) {
      const double a = A[l * kS + j];
      if (j == l) dg += a * a;
      else if (l < j) off += a * a;
    }
    off = groupSum(off);
    dg = groupSum(dg);
    if (off <= 1e-36 * dg || off == 0.0) run = false;
    if (!__any(run)) break;
    for (int round = 0; round < 15; ++round) {
      if (run && l < 8) {
        int p, q;
        if (l == 0) { p = 15; q = round; }
        else { p = (round + l) % 15; q = (round + 15 - l) % 15; }
        if (p > q) { const int t = p; p = q; q = t; }
        const double apq = A[p * kS + q];
        double c = 1.0, s = 0.0;
        if (apq != 0.0) {
          const double app = A[p * kS + p], aqq = A[q * kS + q];
          const double theta = (aqq - app) / (2.0 * apq);
          const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          s = t * c;
        }
        rot[l * 4 + 0] = c;
        rot[l * 4 + 1] = s;
        rot[l * 4 + 2] = (double)p;
        rot[l * 4 + 3] = (double)q;
      }
      __syncthreads();
      if (run) {
        for (int t = l; t < 256; t += kImuGroup) {  // columns: A <- A J, V <- V J
          const int k = (t >> 4) & 7, row = t & 15;
          double* M = (t < 128) ? A : V;
          const double c = rot[k * 4], s = rot[k * 4 + 1];
          const int p = (int)rot[k * 4 + 2], q = (int)rot[k * 4 + 3];
          const double mp = M[row * kS + p], mq = M[row * kS + q];
          M[row * kS + p] = c * mp - s * mq;
          M[row * kS + q] = s * mp + c * mq;
        }
      }
      __syncthreads();
      if (run) {
        for (int t = l; t < 128; t += kImuGroup) {  // rows: A <- J^T A
          const int k = t >> 4, col = t & 15;
          const double c = rot[k * 4], s = rot[k * 4 + 1];
          const int p = (int)rot[k * 4 + 2], q = (int)rot[k * 4 + 3];
          const double mp = A[p * kS + col], mq = A[q * kS + col];
          A[p * kS + col] = c * mp - s * mq;
          A[q * kS + col] = s * mp + c * mq;
        }
      }
      __syncthreads();
      if (run && l < 8) {
        const int p = (int)rot[l * 4 + 2], q = (int)rot[l * 4 + 3];
        if (rot[l * 4 + 1] != 0.0) {
          A[p * kS + q] = 0.0;
          A[q * kS + p] = 0.0;
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace

#ifndef OKG_IMU_OCC
#define OKG_IMU_OCC 2
#endif
// (development-only phase clock of k_eval_imu: ICLK_INIT / ICLK / ICLK_END, dev_clock.hpp)
// APPEND: ImuError::append (ImuError.cpp:63-255) for a batch of factors (okvisgpu_imu_append): the
// chain starts from the stored state (Delta_q, integrals, cross_, dv_db_g, P) at imu_t0 (= the old
// t1), integrates the appended samples with the eliminated state's bias (sb[0] row blk[1]) up to
// imu_t1, and writes the state and the new square-root information; no residual.
__device__ __noinline__ void evalPriorsThread(const DevProblem& P, int t, int mode);
template <bool APPEND, int K = kImuK>
__device__ __forceinline__ void evalImuBlock(const DevProblem& P, int mode, int bid) {
  using LY = ImuLds<K>;
  if (!APPEND) {  // the trailing workgroups: priors and pose-graph edges (uniform per workgroup)
    const int nImuWG = (P.n_imu + kImuPerWG - 1) / kImuPerWG;
    if (bid >= nImuWG) {
      evalPriorsThread(P, (bid - nImuWG) * 64 + (int)threadIdx.x, mode);
      return;
    }
  }
  const int g = threadIdx.x >> 4, l = threadIdx.x & 15;
  const int f = bid * kImuPerWG + g;
  ICLK_INIT

  // per-group LDS: the chain's records (layout ImuLds<K> above), then symmetric P / Jacobi
  // matrix / U (sA, row-major 16x16); L (column-major) / Jacobi eigenvectors (sB); Jacobi rotations
  // (sR). 19 KB per workgroup: two workgroups (waves) per SIMD.
  __shared__ double sAll[kImuPerWG][LY::total];
  double* sG = sAll[g];
  double* sA = sG;
  double* sB = sG + 16 * kS;
  double* sR = sG + 32 * kS;

  // The factor's record, the head of its stored state and the window state are loaded in two
  // rounds (clamped index) and consumed at one point before any test, so that no load waits behind
  // a branch on another (evalSelect restated branch-free).
  const bool inR = f < P.n_imu;
  const int fc = inR ? f : 0;
  // (the append batch carries no window data: no window, flags or WinState are read there)
  const int wR = APPEND ? 0 : gmem(P.imu_win)[fc];
  const int flR = APPEND ? 0 : gmem(P.imu_flags)[fc];
  const int4 blkR = gmem(reinterpret_cast<const int4*>(P.imu_blocks))[fc];
  const int64_t t0 = gmem(P.imu_t0)[fc], t1 = gmem(P.imu_t1)[fc];
  const int sbeg = gmem(P.imu_sbegin)[fc], send = gmem(P.imu_sbegin)[fc + 1];
  const auto stR = gmem(P.imu_state + (size_t)fc * kImuState);
  const double st0 = stR[0], st1 = stR[1];
  double bref[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) bref[k] = stR[57 + 3 + k];
  int sDone = 0, sCand = 0, sX = 0, sL = 0;
  if (!APPEND) {
    const auto gst = gmem(P.st + wR);
    sDone = gst->done;
    sCand = gst->eval_cand;
    sX = gst->xcur;
    sL = gst->lcur;
  }
  const auto parp = gmem(P.imu_par + 7 * wR);  // (read where needed: nothing held across the chain)
  const int64_t tsLast = gmem(P.imu_ts)[max(send - 1, 0)];
  const int nTot = gmem(P.imu_sbegin)[P.n_imu];  // samples of the batch (bounds of the cache warm-up)
  asm volatile("" ::"v"(flR), "v"(blkR.y), "v"(t0), "v"(t1), "v"(st0), "v"(st1), "v"(bref[0]), "v"(bref[5]),
               "v"(sDone), "v"(sCand), "v"(sX), "v"(sL), "v"(tsLast));
  const bool live = inR && (APPEND || ((sDone == 0) & (mode != 1 || sCand != 0) & !((flR & 2) && mode < 2)));
  const int w = APPEND ? 0 : wR;
  const int xs = APPEND ? 0 : (mode == 1 ? 1 - sX : sX), lb = APPEND ? 0 : (mode == 1 ? 1 - sL : sL);
  const int fs = live ? f : 0;  // safe index for idle groups (writes are all under live)

  const auto blk = gmem(P.imu_blocks + 4 * fs);
  const auto sb0 = gmem(pick2(xs, P.sb[0], P.sb[1]) + 9 * (size_t)blkR.y);
  const auto state = gmemw(P.imu_state + (size_t)fs * kImuState);

  // ---- re-preintegration decision (ImuError.cpp:833-859)
  int redoCounter = (int)st0;
  bool redo = st1 != 0.0;
  {
    const double d0 = sb0[3] - bref[0], d1 = sb0[4] - bref[1], d2 = sb0[5] - bref[2];
    redo = redo || (sqrt(d0 * d0 + d1 * d1 + d2 * d2) > 0.0003);
  }
  const bool doRedo =
      APPEND || (redo && ((send - sbeg) < 50 || P.opt.redo_propagation_always)) || redoCounter == 0;
  // redoPreintegration returns -1 before touching any state when the samples do not cover t1
  // (ImuError.cpp:270-273): the old preintegration is kept.
  const bool covered = (send > sbeg) && tsLast >= t1;
  const bool integrate = live && doRedo && covered;
  const bool resetDb = live && doRedo && !APPEND;  // Delta_b is zero after a redo (ImuError.cpp:855)
  if (resetDb) {
    redoCounter++;
    redo = false;
  }

  // Chain ownership (phase-split integration, below): the quaternion / cross_ chain is carried in
  // every lane's registers (lane 0 stores it); the pure accumulators are distributed: lane e < 9
  // owns component e of C_integral (aCi), C_doubleintegral (aCdi), dalpha_db_g, dv_db_g and
  // dp_db_g, lanes 9..11 own acc_integral (aCi) and acc_doubleintegral (aCdi) component e - 9;
  // lane l < 15 owns column l of P.
  double aCi = 0.0, aCdi = 0.0, adadbg = 0.0, advdbg = 0.0, adpdbg = 0.0;
  double Pc[15];  // column l of P
  for (int i = 0; i < 15; ++i) Pc[i] = 0.0;
  int steps = 0;
  double* const carry = sG + LY::carry;  // Delta_q (4) | cross_ (9) between chunks
  if (l == 0) {
    carry[0] = 0.0; carry[1] = 0.0; carry[2] = 0.0; carry[3] = 1.0;
    for (int i = 0; i < 9; ++i) carry[4 + i] = 0.0;
  }
  if (APPEND && integrate) {  // continue the chain of the stored preintegration
    if (l == 0)
      for (int i = 0; i < 4; ++i) carry[i] = state[2 + i];
    if (l == 0)
      for (int i = 0; i < 9; ++i) carry[4 + i] = state[292 + i];
    if (l < 9) {
      aCi = state[6 + l];
      aCdi = state[15 + l];
      adadbg = state[30 + l];
      advdbg = state[39 + l];
      adpdbg = state[48 + l];
    } else if (l < 12) {
      aCi = state[24 + l - 9];
      aCdi = state[27 + l - 9];
    }
    if (l < 15)
      for (int i = 0; i < 15; ++i) Pc[i] = state[301 + i * 15 + l];
  }

  ICLK(0)
  // ---- redoPreintegration (ImuError.cpp:258-466), uniform trip count over the wavefront, in
  // chunks of K steps and five phases per chunk, so that no phase holds more than its own
  // working set in registers (the single-pass form carried ~140 live doubles per lane and spilled):
  //  R  (lane k, parallel)  step record: dt, interpolated samples, dq = exp(w dt), Jr(w dt),
  //                         R(dq)^T, the noise of the step. The integration time before step `it`
  //                         is t0 for the first sample and max(t0, min(ts[it], t1)) after it: where
  //                         the previous step ended, or unchanged when that step was skipped for
  //                         dt <= 0 (ImuError.cpp:339); steps after the one reaching t1 get dt = 0.
  //  Q  (sequential)        Delta_q <- Delta_q dq and cross_ <- R(dq)^T cross_ + Jr dt, the only
  //                         products on the chain (ImuError.cpp:352-392), stored per step;
  //  I  (lane k, parallel)  C, C_1, C + C_1, (C + C_1) a, C_1 Jr, X (ImuError.cpp:360-392) and the
  //                         F_delta blocks that need no running sum;
  //  S  (lane = component)  the running sums (C_integral, acc_integral, their double integrals,
  //                         dalpha/dv/dp_db_g) and the F_delta blocks that read them (:395-410);
  //  P  (lane = column)     P <- F P F^T + Q (ImuError.cpp:412-426).
  {
    const int N = integrate ? send - sbeg : 0;
    int Nmax = N;
    Nmax = max(Nmax, __shfl_xor(Nmax, 16, 64));
    Nmax = max(Nmax, __shfl_xor(Nmax, 32, 64));
    bool started = false;  // hasStarted: an earlier step was integrated
    double* const rec = sG + LY::rec;
    double* const q1 = sG + LY::q1;
    double* const cr = sG + LY::cr;
    double* const cj = sG + LY::cj;
    double* const cc = sG + LY::cc;
    double* const ca = sG + LY::ca;
    double* const xx = sG + LY::xx;
    double* const Fs = sG + LY::f;
    double* const nz = sG + LY::nz;
    double* const M = sG + LY::m;      // (phase P; aliases the records, q1, cr and cj)
    for (int c0 = 0; c0 < Nmax; c0 += K) {
      const int nk = min(K, Nmax - c0);
      // ---- R
      {
        const double bg[3] = {sb0[3], sb0[4], sb0[5]}, ba[3] = {sb0[6], sb0[7], sb0[8]};
        const double a_max = parp[0], g_max = parp[1], sg_c = parp[2], sa_c = parp[3], sgw_c = parp[4],
                     saw_c = parp[5];
        const int it = c0 + l;
        bool ok = false;
        double dt = 0.0, om0[3] = {0, 0, 0}, ac0[3] = {0, 0, 0}, om1[3] = {0, 0, 0}, ac1[3] = {0, 0, 0};
        int64_t nexttime = 0;
        int s0 = sbeg;
        if (l < K && it < N) {
          s0 = sbeg + it;
          const int s1 = (it + 1 < N) ? s0 + 1 : s0;
          for (int k = 0; k < 3; ++k) {
            om0[k] = gmem(P.imu_ga)[6 * (size_t)s0 + k];
            ac0[k] = gmem(P.imu_ga)[6 * (size_t)s0 + 3 + k];
            om1[k] = gmem(P.imu_ga)[6 * (size_t)s1 + k];
            ac1[k] = gmem(P.imu_ga)[6 * (size_t)s1 + 3 + k];
          }
          nexttime = (it + 1 == N) ? t1 : gmem(P.imu_ts)[s0 + 1];
          const int64_t tb = (it == 0) ? t0 : max(t0, min(gmem(P.imu_ts)[s0], t1));
          dt = durToSec(nexttime - tb);
          if (t1 < nexttime) {
            const double interval = durToSec(nexttime - gmem(P.imu_ts)[s0]);
            nexttime = t1;
            dt = durToSec(nexttime - tb);
            const double r = dt / interval;
            for (int k = 0; k < 3; ++k) {
              om1[k] = (1.0 - r) * om0[k] + r * om1[k];
              ac1[k] = (1.0 - r) * ac0[k] + r * ac1[k];
            }
          }
          ok = dt > 0.0;  // dt <= 0: the sample is skipped (ImuError.cpp:339)
        }
        const unsigned gm = (unsigned)((__ballot(ok) >> (16 * g)) & 0xFFFFull);
        if (ok && !started && l == __ffs(gm) - 1) {  // the first integrated step starts at t0
          const double r = dt / durToSec(nexttime - gmem(P.imu_ts)[s0]);
          for (int k = 0; k < 3; ++k) {
            om0[k] = r * om0[k] + (1.0 - r) * om1[k];
            ac0[k] = r * ac0[k] + (1.0 - r) * ac1[k];
          }
        }
        started = started || gm != 0;
        steps += __popc(gm);
        double* R = rec + min(l, K - 1) * kStepRec;
        if (l < K) {
          R[0] = ok ? dt : 0.0;
          Fs[l * kFStride + kFdt] = ok ? dt : 0.0;
        }
        if (ok) {
          double gyr_sat = 1.0, acc_sat = 1.0;
          for (int k = 0; k < 3; ++k) {
            if (fabs(om0[k]) > g_max || fabs(om1[k]) > g_max) gyr_sat = 100.0;
            if (fabs(ac0[k]) > a_max || fabs(ac1[k]) > a_max) acc_sat = 100.0;
          }
          double w_true[3];
          for (int k = 0; k < 3; ++k) {
            w_true[k] = 0.5 * (om0[k] + om1[k]) - bg[k];
            R[5 + k] = 0.5 * (ac0[k] + ac1[k]) - ba[k];  // a_true
          }
          const double theta_half =
              sqrt(w_true[0] * w_true[0] + w_true[1] * w_true[1] + w_true[2] * w_true[2]) * 0.5 * dt;
          double sh, ch;  // one sincos for dq and the right Jacobian
          sincos(theta_half, &sh, &ch);
          double sincv;  // ode::sinc (ode.hpp:34-46)
          if (fabs(theta_half) > 1.0e-6) {
            sincv = sh / theta_half;
          } else {
            const double x_2 = theta_half * theta_half, x_4 = x_2 * x_2, x_6 = x_2 * x_2 * x_2;
            sincv = 1.0 - (1.0 / 6.0) * x_2 + (1.0 / 120.0) * x_4 - (1.0 / 5040.0) * x_6;
          }
          const double sth = sincv * 0.5 * dt;
          const Q dq{sth * w_true[0], sth * w_true[1], sth * w_true[2], ch};
          R[1] = dq.x; R[2] = dq.y; R[3] = dq.z; R[4] = dq.w;
          const double wdt[3] = {w_true[0] * dt, w_true[1] * dt, w_true[2] * dt};
          double Jr[9], Rdqi[9];
          rightJacobianHalf(wdt, sh, ch, Jr);  // Jacobian parts (ImuError.cpp:385-392)
          qrot(qinv(dq), Rdqi);
          for (int i = 0; i < 9; ++i) {
            R[8 + i] = Jr[i];
            R[17 + i] = Rdqi[i];
          }
          // discrete noise of this step on the diagonal (ImuError.cpp:412-426, summed over sigma)
          double* z = nz + l * 5;
          z[0] = sa_c * sa_c * (0.5 * dt * dt * dt * acc_sat * acc_sat * acc_sat);
          z[1] = sg_c * sg_c * (gyr_sat * dt);
          z[2] = sa_c * sa_c * (acc_sat * dt);
          z[3] = sgw_c * sgw_c * dt;
          z[4] = saw_c * saw_c * dt;
        }
      }
      __syncthreads();
      ICLK(6)
      // Warm the caches with the next chunk's samples (5 samples of 48 B and their time stamps per
      // group): an LDS-DMA touch per 64-byte line, issued now so that its memory latency overlaps
      // this chunk's phases instead of heading the next step-record phase (which read them from
      // HBM with 4 of 16 lanes active). The DMA's data lands in group 0's F_delta block, dead until
      // the I phase writes it (the barrier after the Q phase waits for the DMA); never read.
      if (c0 + K < Nmax) {
        const int nb = min(sbeg + c0 + K, nTot - 1);
        const void* src = l < 4 ? (const void*)(P.imu_ga + min(6 * (int64_t)nb + 8 * l, 6 * (int64_t)nTot - 1))
                                : (const void*)(P.imu_ts + min(nb + 8 * (l & 1), nTot - 1));
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(sAll[0] + LY::f), 4, 0, 0);
      }
      // ---- Q: the two product chains. Delta_q on every lane (lane 0 stores it); cross_ distributed,
      // lane e < 9 owning entry e = (r, c): each step needs column c of the previous cross_ (three
      // shuffles inside the group) instead of the whole 3x3 product on every lane. Same expressions
      // per entry as mm3, so the same bits.
      {
      Q cdq{carry[0], carry[1], carry[2], carry[3]};
      const int er = min(l, 8) / 3, ec = min(l, 8) % 3, gbase = threadIdx.x & ~(kImuGroup - 1);
      double crs = carry[4 + min(l, 8)];
      if (l == 0) {
        q1[0] = cdq.x; q1[1] = cdq.y; q1[2] = cdq.z; q1[3] = cdq.w;
      }
      if (l < 9) cr[l] = crs;
      for (int k = 0; k < nk; ++k) {
        const double* R = rec + k * kStepRec;
        const double dt = R[0];
        if (dt > 0.0) {  // uniform over the group
          cdq = qmul(cdq, Q{R[1], R[2], R[3], R[4]});
          const double b0 = __shfl(crs, gbase + ec, 64), b1 = __shfl(crs, gbase + 3 + ec, 64),
                       b2 = __shfl(crs, gbase + 6 + ec, 64);
          const double* a = R + 17 + 3 * er;
          const double tmp = a[0] * b0 + a[1] * b1 + a[2] * b2;
          crs = tmp + R[8 + 3 * er + ec] * dt;
        }
        if (l == 0) {
          double* qo = q1 + 4 * (k + 1);
          qo[0] = cdq.x; qo[1] = cdq.y; qo[2] = cdq.z; qo[3] = cdq.w;
        }
        if (l < 9) cr[9 * (k + 1) + l] = crs;
      }
      if (l == 0) {
        carry[0] = cdq.x; carry[1] = cdq.y; carry[2] = cdq.z; carry[3] = cdq.w;
      }
      if (l < 9) carry[4 + l] = crs;
      }
      __syncthreads();
      ICLK(7)
      // ---- I: step l's products
      if (l < nk) {
        const double* R = rec + l * kStepRec;
        const double dt = R[0];
        if (dt > 0.0) {
          double C[9], C1[9], CC1[9], CCa[3], tmp[9], t1m[9], X[9], ax[9];
          const double* qa = q1 + 4 * l;
          qrot(Q{qa[0], qa[1], qa[2], qa[3]}, C);
          qrot(Q{qa[4], qa[5], qa[6], qa[7]}, C1);
          for (int i = 0; i < 9; ++i) CC1[i] = C[i] + C1[i];
          const double a_true[3] = {R[5], R[6], R[7]};
          mv3(CC1, a_true, CCa);
          double Jr[9];
          for (int i = 0; i < 9; ++i) Jr[i] = R[8 + i];
          mm3(C1, Jr, tmp);
          for (int i = 0; i < 9; ++i) cj[9 * l + i] = tmp[i];
          crossMx(a_true, ax);
          double crk[9];
          for (int i = 0; i < 9; ++i) crk[i] = cr[9 * l + i];
          mm3(C, ax, tmp);
          mm3(tmp, crk, t1m);
          for (int i = 0; i < 9; ++i) crk[i] = cr[9 * (l + 1) + i];
          mm3(C1, ax, tmp);
          mm3(tmp, crk, X);
          for (int i = 0; i < 9; ++i) X[i] += t1m[i];
          double* F = Fs + l * kFStride;
          for (int i = 0; i < 3; ++i) F[kF63 + i] = 0.5 * dt * CCa[i];  // F63 = -[0.5 dt (C + C_1) a]x
          for (int i = 0; i < 9; ++i) {
            cc[9 * l + i] = CC1[i];
            xx[9 * l + i] = X[i];
            F[kF39 + i] = -dt * C1[i];
            F[kF69 + i] = 0.5 * dt * X[i];
            F[kF612 + i] = -0.5 * dt * CC1[i];
          }
          for (int i = 0; i < 3; ++i) ca[3 * l + i] = CCa[i];
        }
      }
      __syncthreads();
      ICLK(8)
      // ---- S: running sums, component-distributed
      for (int k = 0; k < nk; ++k) {
        double* F = Fs + k * kFStride;
        const double dt = F[kFdt];
        if (dt > 0.0 && l < 12) {
          const double hdt2 = 0.25 * dt * dt;
          if (l < 9) {
            const double c = cc[9 * k + l], x = xx[9 * k + l];
            F[kF012 + l] = -aCi * dt + hdt2 * c;
            aCdi += aCi * dt + hdt2 * c;
            aCi += 0.5 * dt * c;
            adadbg += cj[9 * k + l] * dt;
            const double t = dt * advdbg + hdt2 * x;
            F[kF09 + l] = t;
            adpdbg += t;
            advdbg += 0.5 * dt * x;
          } else {
            const double c = ca[3 * k + l - 9];
            const double v = aCi * dt + hdt2 * c;
            F[kF03 + l - 9] = v;  // F03 = -[acc_integral dt + dt^2/4 (C + C_1) a]x, held as its vector
            aCdi += v;
            aCi += 0.5 * dt * c;
          }
        }
      }
      __syncthreads();
      ICLK(9)
      // ---- P <- F P F^T + Q : M = F P (column l), exchange rows, P' = F M^T (column l)
      for (int k = 0; k < nk; ++k) {
#if OKG_IMU_FREG
        // the step's F_delta blocks read once into registers for both products (the barrier
        // between them would force a second LDS read)
        double F[kFdt + 1];
        {
          const double* Fl = Fs + k * kFStride;
#pragma unroll
          for (int i = 0; i <= kFdt; ++i) F[i] = Fl[i];
        }
#else
        const double* F = Fs + k * kFStride;
#endif
        const bool doStep = F[kFdt] > 0.0;  // uniform over the group
        if (doStep && l < 15) {
          double Mc[15];
          applyF(F, Pc, Mc);
          for (int i = 0; i < 15; ++i) M[l * kS + i] = Mc[i];  // column l of M
        }
        __syncthreads();
        if (doStep && l < 15) {
          double Mr[15];
          for (int j = 0; j < 15; ++j) Mr[j] = M[j * kS + l];  // row l of M
          applyF(F, Mr, Pc);
          const double* z = nz + k * 5;
          const double q = l < 3 ? z[0] : (l < 6 ? z[1] : (l < 9 ? z[2] : (l < 12 ? z[3] : z[4])));
          for (int i = 0; i < 15; ++i) Pc[i] += (i == l) ? q : 0.0;
        }
        __syncthreads();
      }
      ICLK(10)
    }
  }
  ICLK(1)
  // new preintegration state (ImuError.hpp:273-304 members) from the chain registers and the
  // component owners
  double Db[6];  // Delta_b of the residual (ImuError.cpp:841-859), zero after a redo
  for (int k = 0; k < 6; ++k) Db[k] = resetDb ? 0.0 : sb0[3 + k] - stR[60 + k];
  if (integrate) {
    if (l == 0) {
      for (int i = 0; i < 4; ++i) state[2 + i] = carry[i];
      for (int i = 0; i < 9; ++i) {
        state[292 + i] = carry[4 + i];
        if (!APPEND) state[57 + i] = sb0[i];  // append keeps speedAndBiases_ref_
      }
      state[291] = (double)steps;
    }
    if (l < 9) {
      state[6 + l] = aCi;
      state[15 + l] = aCdi;
      state[30 + l] = adadbg;
      state[39 + l] = advdbg;
      state[48 + l] = adpdbg;
    } else if (l < 12) {
      state[24 + l - 9] = aCi;
      state[27 + l - 9] = aCdi;
    }
  }

  ICLK(2)
  // (skipped by a workgroup none of whose factors re-integrated: the common case once the biases
  // have settled; the workgroup is one wavefront, so the test is uniform)
  if (__any(integrate)) {
    // ---- square-root information of P (PseudoInverse.hpp:132-158)
    // symmetrise (ImuError.cpp:441): sB holds P column-major; the symmetric P is kept row-major
    // (16x16 with a decoupled zero pad) in sA for the eigen fallback
    if (integrate && l < 15)
      for (int i = 0; i < 15; ++i) sB[l * kS + i] = Pc[i];
    __syncthreads();
    double trace = 0.0;
    if (integrate) {
      for (int i = 0; i < 15; ++i) Pc[i] = (l < 15) ? 0.5 * Pc[i] + 0.5 * sB[i * kS + l] : 0.0;
      for (int i = 0; i < 16; ++i) sA[l * kS + i] = (i < 15) ? Pc[i] : 0.0;
      if (l < 15)  // P_delta_ (symmetrised), kept for a later append
        for (int i = 0; i < 15; ++i) state[301 + i * 15 + l] = Pc[i];
      for (int i = 0; i < 15; ++i) trace += (i == l) ? Pc[i] : 0.0;
    }
    trace = groupSum(trace);
    __syncthreads();
    ICLK(11)
    // right-looking Cholesky P = L L^T with lane l holding row l (j <= l) in registers: per pivot k
    // the pivot comes by shuffle from lane k, each lane scales its L(l,k) and publishes it into column
    // k of sB (column-major), one barrier, then updates its row with column k. Same products and the
    // same ascending-k order per element as a column-oriented LDS factorisation.
    bool ok = true;
    const int gbase = threadIdx.x & ~(kImuGroup - 1);
    double rw[15];
#pragma unroll
    for (int j = 0; j < 15; ++j) rw[j] = Pc[j];
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const double dk = __shfl(rw[k], gbase + k, 64);
      if (integrate && l >= k && l < 15) {
        if (!(dk > 0.0)) ok = false;
        rw[k] = rw[k] / sqrt(dk);
        sB[k * kS + l] = rw[k];
      }
      __syncthreads();
      if (integrate && l > k && l < 15) {
#pragma unroll
        for (int j = k + 1; j < 15; ++j)
          if (j <= l) rw[j] -= sB[k * kS + j] * rw[k];
      }
    }
    // U = L^-1 per lane (row l of U from L in sB, no barriers):
    //   U(l,l) = 1/L(l,l),  U(l,j) = -(1/L(j,j)) sum_{m=j+1..l} U(l,m) L(m,j)   (j < l)
    double ur[15];
#pragma unroll
    for (int j = 14; j >= 0; --j) {
      ur[j] = 0.0;
      if (integrate && l >= j && l < 15) {
        const double ujj = 1.0 / sB[j * kS + j];
        double acc = 0.0;
#pragma unroll
        for (int m = j + 1; m < 15; ++m)
          if (m <= l) acc += ur[m] * sB[j * kS + m];
        ur[j] = (l == j) ? ujj : -ujj * acc;
      }
    }
    __syncthreads();
    // U column-major into sB (lower triangle) for the norm test, the transpose and the append
    if (integrate && l < 15) {
#pragma unroll
      for (int j = 0; j < 15; ++j)
        if (j <= l) sB[j * kS + l] = ur[j];
    }
    __syncthreads();
    ICLK(12)
    double fro = 0.0;
    if (integrate && l < 15)
      for (int i = l; i < 15; ++i) fro += sB[l * kS + i] * sB[l * kS + i];
    fro = groupSum(fro);
    ok = groupSum(ok ? 0.0 : 1.0) == 0.0;
    const double eps = DBL_EPSILON;
    const bool needEig = integrate && !(ok && fro > 0.0 && 1.0 / fro > 4.0 * fmax(eps, eps * 15.0 * trace));
    __syncthreads();
    ICLK_COUNT(13, needEig && l == 0)
    if (__any(needEig)) {
      // clamped eigenvalues possible: the reference's eigen-decomposition (cyclic Jacobi) of the
      // symmetric P kept in sA; eigenvectors into sB, then U = diag(clamped lambda^-1/2) V^T
      groupJacobi(sA, sB, sR, l, needEig);
      double urow[15];
      if (needEig && l < 15) {
        double lmax = -1e300;
        for (int i = 0; i < 15; ++i) lmax = fmax(lmax, sA[i * kS + i]);
        const double tol = fmax(eps, eps * 15.0 * lmax);
        const double li = sA[l * kS + l];
        const double s = sqrt(li > tol ? 1.0 / li : 1.0 / tol);
        for (int j = 0; j < 15; ++j) urow[j] = s * sB[j * kS + l];
      }
      __syncthreads();
      if (needEig && l < 15)
        for (int j = 0; j < 15; ++j) sA[l * kS + j] = urow[j];
    }
    // Cholesky path: U (column-major in sB, lower triangular) -> row-major sA
    if (integrate && !needEig && l < 15)
      for (int i = 0; i < 15; ++i) sA[i * kS + l] = (i >= l) ? sB[l * kS + i] : 0.0;
    __syncthreads();
  }
  ICLK(3)
  if (integrate) {
    for (int e = l; e < 225; e += kImuGroup) state[66 + e] = sA[(e / 15) * kS + e % 15];
  } else if (live) {
    for (int e = l; e < 225; e += kImuGroup) sA[(e / 15) * kS + e % 15] = state[66 + e];
  }
  ICLK(14)
  __syncthreads();  // state writes of the group visible to all its lanes
  ICLK(15)
  if (APPEND) return;  // uniform over the workgroup
  const auto p0 = gmem(pick2(xs, P.pose[0], P.pose[1]) + 7 * (size_t)blk[0]);
  const auto p1 = gmem(pick2(xs, P.pose[0], P.pose[1]) + 7 * (size_t)blk[2]);
  const auto sb1 = gmem(pick2(xs, P.sb[0], P.sb[1]) + 9 * (size_t)blk[3]);
  ImuPre pre;
  loadPre(state, pre);
  const bool success = live && (!integrate || steps > 0);
  if (live && l == 0) {
    state[0] = (double)redoCounter;
    state[1] = redo ? 1.0 : 0.0;
  }

  // ---- residual and minimal Jacobians (ImuError.cpp:861-1000)
  // The ten distinct 3x3 blocks of [F0 | F1] are staged in LDS (sB, row-major 3x3 each):
  //  0 C_S0_W  1 C_S0_W[dp]x  2 F0(3,3)  3 C_S0_W[dv]x  4 dp_db_g  5 F0(3,9)  6 dv_db_g
  //  7 C_doubleintegral  8 C_integral  9 F1(3,3)
  const Q q0 = qnormalize(Q{p0[3], p0[4], p0[5], p0[6]});
  const Q q1 = qnormalize(Q{p1[3], p1[4], p1[5], p1[6]});
  const Q q1i = qinv(q1);
  const double Dt = durToSec(t1 - t0);
  double err[15];
  Q Dq;
  {
    double C0[9];
    qrot(q0, C0);  // C_WS_0 ; C_S0_W = C0^T
    double dp[3], dv[3];
    const double gW[3] = {0.0, 0.0, parp[6]};
    for (int k = 0; k < 3; ++k) {
      dp[k] = p0[k] - p1[k] + sb0[k] * Dt - 0.5 * gW[k] * Dt * Dt;
      dv[k] = sb0[k] - sb1[k] - gW[k] * Dt;
    }
    double adb[3];
    mv3(pre.dadbg, Db, adb);
    Dq = qmul(deltaQ(-adb[0], -adb[1], -adb[2]), pre.dq);
    double t0v[3], t6v[3];
    mtv3(C0, dp, t0v);
    mtv3(C0, dv, t6v);
    const Q qe = qmul(Dq, qmul(q1i, q0));
    for (int k = 0; k < 3; ++k) {
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
    if (live && l == 0) {
      double dpx[9], dvx[9];
      crossMx(dp, dpx);
      crossMx(dv, dvx);
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          sB[0 * 9 + r * 3 + c] = C0[c * 3 + r];
          sB[1 * 9 + r * 3 + c] = C0[0 * 3 + r] * dpx[0 * 3 + c] + C0[1 * 3 + r] * dpx[1 * 3 + c] + C0[2 * 3 + r] * dpx[2 * 3 + c];
          sB[3 * 9 + r * 3 + c] = C0[0 * 3 + r] * dvx[0 * 3 + c] + C0[1 * 3 + r] * dvx[1 * 3 + c] + C0[2 * 3 + r] * dvx[2 * 3 + c];
        }
      for (int i = 0; i < 9; ++i) {
        sB[4 * 9 + i] = pre.dpdbg[i];
        sB[6 * 9 + i] = pre.dvdbg[i];
        sB[7 * 9 + i] = pre.Cdi[i];
        sB[8 * 9 + i] = pre.Ci[i];
      }
    }
  }
  if (live && l == 1) {
    double Pm[16], Om[16], R[9];
    qplusM(qmul(Dq, q1i), Pm);
    qoplusM(q0, Om);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 4; ++k) s += Pm[r * 4 + k] * Om[k * 4 + c];
        sB[2 * 9 + r * 3 + c] = s;  // F0(3,3)
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
        sB[5 * 9 + r * 3 + c] = -(R[r * 3 + 0] * pre.dadbg[0 * 3 + c] + R[r * 3 + 1] * pre.dadbg[1 * 3 + c] +
                                  R[r * 3 + 2] * pre.dadbg[2 * 3 + c]);  // F0(3,9)
  }
  if (live && l == 2) {
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
        sB[9 * 9 + r * 3 + c] = -s;  // F1(3,3)
      }
  }
  const size_t fl = live ? (size_t)f : 0;
  const auto lin = gmemw(P.imu_lin[lb] + fl * kImuLin);
  double rr = 0.0;
  if (live && l < 15) {
    for (int k = 0; k < 15; ++k) rr += sA[l * kS + k] * err[k];
    lin[l] = rr;
  }
  const double c2 = groupSum(l < 15 ? rr * rr : 0.0);
  if (live && l == 0) gmemw(P.imu_cost[lb])[f] = 0.5 * c2;
  __syncthreads();
  ICLK(4)
  // J = U [F0 | F1]. Column j of [F0 | F1] has at most three non-zero 3-blocks: (block row, staged
  // block, sign, or identity); the table depends on j only.
#if OKG_IMU_JAC_ROWS
  // Lane l < 15 forms row l of J: U's row l in registers, the 30 columns unrolled (the column
  // table a compile-time constant), the staged blocks read as LDS broadcasts; every entry is the
  // same expression as in the column form (same bits), and a lane's 30 stores are contiguous.
  if (live && l < 15) {
    double u[15];
#pragma unroll
    for (int k = 0; k < 15; ++k) u[k] = sA[l * kS + k];
#pragma unroll
    for (int j = 0; j < 30; ++j) {
      const bool right = j >= 15;
      const int jj = right ? j - 15 : j, bj = jj / 3, c = jj % 3;
      int nt = 0, trow[3] = {0, 0, 0}, tblk[3] = {0, 0, 0};
      double tsc[3] = {0.0, 0.0, 0.0};
      auto add = [&](int row, int blk, double sc) { trow[nt] = row; tblk[nt] = blk; tsc[nt] = sc; ++nt; };
      if (!right) {
        if (bj == 0) add(0, 0, 1.0);
        else if (bj == 1) { add(0, 1, 1.0); add(3, 2, 1.0); add(6, 3, 1.0); }
        else if (bj == 2) { add(0, 0, Dt); add(6, 0, 1.0); }
        else if (bj == 3) { add(0, 4, 1.0); add(3, 5, 1.0); add(6, 6, 1.0); }
        else { add(0, 7, -1.0); add(6, 8, -1.0); }
      } else {
        if (bj == 0) add(0, 0, -1.0);
        else if (bj == 1) add(3, 9, 1.0);
        else if (bj == 2) add(6, 0, -1.0);
      }
      const int idrow = (bj >= 3) ? 3 * bj + c : -1;
      const double idv = right ? -1.0 : 1.0;
      double acc = 0.0;
      if (success) {
#pragma unroll
        for (int t = 0; t < 3; ++t)
          if (t < nt) {
            const double* Bk = sB + tblk[t] * 9;
            acc += tsc[t] * (u[trow[t]] * Bk[0 * 3 + c] + u[trow[t] + 1] * Bk[1 * 3 + c] + u[trow[t] + 2] * Bk[2 * 3 + c]);
          }
        if (idrow >= 0) acc += idv * u[idrow];
      }
      lin[15 + l * 30 + j] = acc;
    }
  }
#else
  // (column form: lane l computes columns l and l + 16)
  if (live) {
    for (int pass = 0; pass < 2; ++pass) {
      const int j = l + 16 * pass;
      if (j >= 30) break;
      const bool right = j >= 15;
      const int jj = right ? j - 15 : j, bj = jj / 3, c = jj % 3;
      int nt = 0, trow[3], tblk[3];
      double tsc[3];
      auto add = [&](int row, int blk, double sc) { trow[nt] = row; tblk[nt] = blk; tsc[nt] = sc; ++nt; };
      if (!right) {
        if (bj == 0) add(0, 0, 1.0);
        else if (bj == 1) { add(0, 1, 1.0); add(3, 2, 1.0); add(6, 3, 1.0); }
        else if (bj == 2) { add(0, 0, Dt); add(6, 0, 1.0); }
        else if (bj == 3) { add(0, 4, 1.0); add(3, 5, 1.0); add(6, 6, 1.0); }
        else { add(0, 7, -1.0); add(6, 8, -1.0); }
      } else {
        if (bj == 0) add(0, 0, -1.0);
        else if (bj == 1) add(3, 9, 1.0);
        else if (bj == 2) add(6, 0, -1.0);
      }
      // identity / minus-identity blocks on the bias rows
      const int idrow = (bj >= 3) ? 3 * bj + c : -1;
      const double idv = right ? -1.0 : 1.0;
      for (int i = 0; i < 15; ++i) {
        double acc = 0.0;
        if (success) {
          for (int t = 0; t < nt; ++t) {
            const double* Bk = sB + tblk[t] * 9;
            const double* Ui = sA + i * kS + trow[t];
            acc += tsc[t] * (Ui[0] * Bk[0 * 3 + c] + Ui[1] * Bk[1 * 3 + c] + Ui[2] * Bk[2 * 3 + c]);
          }
          if (idrow >= 0) acc += idv * sA[i * kS + idrow];
        }
        lin[15 + i * 30 + j] = acc;
      }
    }
  }
#endif
  ICLK(5)
  ICLK_END
}

template <bool APPEND>
__global__ __launch_bounds__(64, OKG_IMU_OCC) void k_eval_imu(const DevProblem* __restrict__ Pp, int mode) {
  evalImuBlock<APPEND>(*Pp, mode, (int)blockIdx.x);
}
// Few windows: the observations (64 per workgroup), then the IMU factors, priors and edges, as one
// launch (one graph node fewer on a single window's latency chain). K: steps per IMU chunk
// (kImuKFew for one or two windows, whose IMU factors are a latency chain; its LDS, ~72 KB per
// workgroup, would hold the observation workgroups of larger batches to two per CU).
template <int K>
__global__ __launch_bounds__(64, OKG_IMU_OCC) void k_eval_few(const DevProblem* __restrict__ Pp, int mode, int nObsWG) {
  const DevProblem& P = *Pp;
  if ((int)blockIdx.x < nObsWG) {
    if (P.obs_iso) evalObsThread<true>(P, (int)blockIdx.x * 64 + (int)threadIdx.x, mode);
    else evalObsThread<false>(P, (int)blockIdx.x * 64 + (int)threadIdx.x, mode);
    return;
  }
  evalImuBlock<false, K>(P, mode, (int)blockIdx.x - nObsWG);
}

// ------------------------------------------------------------------------------------ priors
// Pose priors, speed/bias priors and relative-pose edges, one thread each (t = their index in that
// order). Runs as the trailing workgroups of k_eval_imu (evalPriorsThread; one launch fewer).
__device__ __noinline__ void evalPriorsThread(const DevProblem& P, int t, int mode) {
  if (t < P.n_pprior) {
    const int i = t;
    const int w = P.pp_win[i];
    int xs, lb;
    if (!evalSelect(P, w, mode, xs, lb)) return;
    if (P.pose_f[P.pp_block[i]] < 0 && mode != 2) return;  // prior on a constant block: fixed_cost
    // all operands in registers before the first store (a single window is a latency chain)
    double pose[7], m[7], L[36];
    for (int k = 0; k < 7; ++k) {
      pose[k] = P.pose[xs][7 * (size_t)P.pp_block[i] + k];
      m[k] = P.pp_meas[7 * (size_t)i + k];
    }
    for (int k = 0; k < 36; ++k) L[k] = P.pp_L[36 * (size_t)i + k];
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
  if (i < P.n_sbprior) {
    const int w = P.sbp_win[i];
    int xs, lb;
    if (!evalSelect(P, w, mode, xs, lb)) return;
    if (P.sb_f[P.sbp_block[i]] < 0 && mode != 2) return;
    double e[9], L[81];
    for (int k = 0; k < 9; ++k) e[k] = P.sbp_meas[9 * (size_t)i + k] - P.sb[xs][9 * (size_t)P.sbp_block[i] + k];
    for (int k = 0; k < 81; ++k) L[k] = P.sbp_L[81 * (size_t)i + k];
    double* lin = P.sbp_lin[lb] + 90 * (size_t)i;
    double c = 0;
    for (int r = 0; r < 9; ++r) {
      double s = 0;
      for (int k = 0; k < 9; ++k) s += L[r * 9 + k] * e[k];
      lin[r] = s;
      c += s * s;
      for (int k = 0; k < 9; ++k) lin[9 + r * 9 + k] = -L[r * 9 + k];
    }
    P.sbp_cost[lb][i] = 0.5 * c;
    return;
  }
  // ---- relative-pose residual blocks, no loss function:
  //   kind 0 TwoPoseStandardGraphError(Const)::EvaluateWithMinimalJacobians (TwoPoseGraphError.cpp:
  //          467-606 / :631-767; ViGraphEstimator.cpp:770)
  //   kind 1 RelativePoseError::EvaluateWithMinimalJacobians (RelativePoseError.cpp:59-140;
  //          ViGraph.cpp:786-808): T_AB measured in rp_lp, LLT(information).L^T in rp_J
  const int k = i - P.n_sbprior;
  if (k >= P.n_relpose) return;
  const int w = P.rp_win[k];
  int xs, lb;
  if (!evalSelect(P, w, mode, xs, lb)) return;
  if ((P.rp_flags[k] & 2) && mode < 2) return;  // both poses constant: fixed_cost only
  const double* p0 = P.pose[xs] + 7 * (size_t)P.rp_blocks[2 * k];
  const double* p1 = P.pose[xs] + 7 * (size_t)P.rp_blocks[2 * k + 1];
  const double* dx = P.rp_dx + 6 * (size_t)k;
  double Jq[36];
  for (int e = 0; e < 36; ++e) Jq[e] = P.rp_J[36 * (size_t)k + e];
  const double* lp = P.rp_lp + 7 * (size_t)k;
  const bool relErr = P.rp_kind[k] == 1;
  const Q q0 = qnormalize(Q{p0[3], p0[4], p0[5], p0[6]}), q1 = qnormalize(Q{p1[3], p1[4], p1[5], p1[6]});
  const Q ql = qnormalize(Q{lp[3], lp[4], lp[5], lp[6]});
  const Q qlinv = qinv(ql);
  double C0[9];
  qrot(q0, C0);  // C_WS0 (C_WA); C_S0W = C0^T
  const double d01[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
  double rS[3];
  mtv3(C0, d01, rS);  // T_S0Si.r (T_AB.r)
  const Q q0inv = qinv(q0);
  const Q qrel = qnormalize(qmul(q0inv, q1));  // T_S0Si.q (T_AB.q)
  double err[6];
  if (relErr) {  // [r_AB_meas - r_AB; 2 vec(q_AB_meas q_AB^-1)]
    const Q dq = qmul(ql, qinv(qrel));
    err[0] = lp[0] - rS[0]; err[1] = lp[1] - rS[1]; err[2] = lp[2] - rS[2];
    err[3] = 2.0 * dq.x; err[4] = 2.0 * dq.y; err[5] = 2.0 * dq.z;
  } else {  // DeltaX_ + [r_S0Si - r_lin; 2 vec(q_S0Si q_lin^-1)]
    const Q dq = qmul(qrel, qlinv);
    err[0] = dx[0] + rS[0] - lp[0]; err[1] = dx[1] + rS[1] - lp[1]; err[2] = dx[2] + rS[2] - lp[2];
    err[3] = dx[3] + 2.0 * dq.x; err[4] = dx[4] + 2.0 * dq.y; err[5] = dx[5] + 2.0 * dq.z;
  }
  double* lin = P.rp_lin[lb] + kRelPoseLin * (size_t)k;
  double c = 0.0;
  for (int r = 0; r < 6; ++r) {
    double s = 0.0;
    for (int q = 0; q < 6; ++q) s += Jq[r * 6 + q] * err[q];
    lin[r] = s;
    c += s * s;
  }
  // kind 0: Jerr = [C_S0W 0; 0 B], B = (plus(q_WS0^-1) oplus(q_WS q_lin^-1))_3x3,
  //         JerrRef = [-C_S0W, C_S0W [r_WS - r_WS0]x; 0, -B]
  // kind 1: J0 = [C_AW, -C_AW [r_WB - r_WA]x; 0, B], J1 = [-C_AW, 0; 0, -B],
  //         B = (plus(q_AB_meas q_BW) oplus(q_WA))_3x3   (signs folded into sg below)
  double Pm[16], Om[16], B[9];
  if (relErr) {
    qplusM(qmul(ql, qinv(q1)), Pm);
    qoplusM(q0, Om);
  } else {
    qplusM(q0inv, Pm);
    qoplusM(qmul(q1, qlinv), Om);
  }
  for (int r = 0; r < 3; ++r)
    for (int q = 0; q < 3; ++q)
      B[r * 3 + q] = Pm[r * 4 + 0] * Om[0 * 4 + q] + Pm[r * 4 + 1] * Om[1 * 4 + q] + Pm[r * 4 + 2] * Om[2 * 4 + q] +
                     Pm[r * 4 + 3] * Om[3 * 4 + q];
  double X[9], CX[9];
  crossMx(d01, X);
  for (int r = 0; r < 3; ++r)  // C_S0W X = C0^T X
    for (int q = 0; q < 3; ++q) CX[r * 3 + q] = C0[0 * 3 + r] * X[0 * 3 + q] + C0[1 * 3 + r] * X[1 * 3 + q] + C0[2 * 3 + r] * X[2 * 3 + q];
  for (int r = 0; r < 6; ++r) {
    const double* Jr = Jq + r * 6;
    double* Lr = lin + 6 + r * 12;
    for (int q = 0; q < 3; ++q) {
      const double jt = Jr[0] * C0[q * 3 + 0] + Jr[1] * C0[q * 3 + 1] + Jr[2] * C0[q * 3 + 2];  // (J C0^T)_q
      const double jb = Jr[3] * B[0 * 3 + q] + Jr[4] * B[1 * 3 + q] + Jr[5] * B[2 * 3 + q];
      const double jx = Jr[0] * CX[0 * 3 + q] + Jr[1] * CX[1 * 3 + q] + Jr[2] * CX[2 * 3 + q];
      const double sg = relErr ? -1.0 : 1.0;
      Lr[q] = -sg * jt;          // reference pose, translation
      Lr[3 + q] = sg * (jx - jb);  // reference pose, rotation
      Lr[6 + q] = sg * jt;       // other pose, translation
      Lr[9 + q] = sg * jb;       // other pose, rotation
    }
  }
  P.rp_cost[lb][k] = 0.5 * c;
}

// ------------------------------------------------------------------- host-evaluated factors (ABI 5)
// The §8b fallback: k_host_gather packs the evaluation point of every host factor the eval mode
// selects (evalSelect of k_eval_imu: window running, candidate pending for mode 1, fixed factors at
// the initial point only) into host_in; the runtime copies it to pinned memory, evaluates the
// callbacks on host threads (runtime.cpp HostEval) and copies the results back into host_out;
// k_host_scatter then writes r, J and the cost into the factor's IMU-layout linearisation record,
// from where the J^T J, assembly, J*v and cost kernels take it like an IMU factor's.
__global__ __launch_bounds__(64) void k_host_gather(const DevProblem* __restrict__ Pp, int mode) {
  const DevProblem& P = *Pp;
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= P.n_host) return;
  const int f = P.n_imu + h;
  const int w = P.imu_win[f], fl = P.imu_flags[f];
  const WinState& s = P.st[w];
  const bool live = !s.done && (mode != 1 || s.eval_cand) && !((fl & 2) && mode < 2);
  const int xs = mode == 1 ? 1 - s.xcur : s.xcur, lb = mode == 1 ? 1 - s.lcur : s.lcur;
  double* in = P.host_in + (size_t)h * kHostIn;
  in[0] = live ? 1.0 + lb : 0.0;
  in[1] = (double)mode;
  if (!live) return;
  const int4 blk = reinterpret_cast<const int4*>(P.imu_blocks)[f];
  const int slot[4] = {blk.x, blk.y, blk.z, blk.w};
  const int at[4] = {8, 15, 24, 31};
  for (int q = 0; q < 4; ++q) {
    if (slot[q] < 0) continue;
    const int n = (q & 1) ? 9 : 7;
    const double* src = ((q & 1) ? P.sb[xs] : P.pose[xs]) + (size_t)n * slot[q];
    for (int k = 0; k < n; ++k) in[at[q] + k] = src[k];
  }
}

// One wavefront per host factor: the uploaded cost | r | J into lin[lb] / cost[lb].
__global__ __launch_bounds__(256) void k_host_scatter(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int h = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (h >= P.n_host) return;
  const double flag = P.host_in[(size_t)h * kHostIn];
  if (flag == 0.0) return;
  const int lb = (int)flag - 1, f = P.n_imu + h;
  const double* out = P.host_out + (size_t)h * kHostOut;
  double* lin = P.imu_lin[lb] + (size_t)f * kImuLin;
  for (int e = lane; e < kImuLin; e += 64) lin[e] = out[1 + e];
  if (lane == 0) P.imu_cost[lb][f] = out[0];
}

void launch_host_gather(const DevProblem& P, int mode, hipStream_t s) {
  if (P.n_host > 0) hipLaunchKernelGGL(k_host_gather, dim3((P.n_host + 63) / 64), dim3(64), 0, s, P.self, mode);
}
void launch_host_scatter(const DevProblem& P, hipStream_t s) {
  if (P.n_host > 0) hipLaunchKernelGGL(k_host_scatter, dim3((P.n_host + 3) / 4), dim3(256), 0, s, P.self);
}

// ------------------------------------------------------------------------------------ launchers
void launch_eval_obs(const DevProblem& P, int mode, hipStream_t s) {
  if (P.n_obs == 0) return;
  if (P.obs_iso) hipLaunchKernelGGL(k_eval_obs<true>, dim3((P.n_obs + 255) / 256), dim3(256), 0, s, P.self, mode);
  else hipLaunchKernelGGL(k_eval_obs<false>, dim3((P.n_obs + 255) / 256), dim3(256), 0, s, P.self, mode);
}
// k_eval_imu's grid: the IMU factors (4 per workgroup), then the priors and edges (64 per workgroup)
void launch_eval_imu(const DevProblem& P, int mode, hipStream_t s) {
  const int np = P.n_pprior + P.n_sbprior + P.n_relpose;
  const int nb = (P.n_imu + kImuPerWG - 1) / kImuPerWG + (np + 63) / 64;
  if (nb > 0) hipLaunchKernelGGL(k_eval_imu<false>, dim3(nb), dim3(64), 0, s, P.self, mode);
}
void launch_eval_priors(const DevProblem& P, int mode, hipStream_t s) {}  // (in launch_eval_imu)
// The IMU factors (and priors / edges) as the solve's evaluation runs them: one or two windows
// through k_eval_few's IMU chunking (no observation workgroups), else k_eval_imu (okvisgpu_time_kernel).
void launch_eval_imu_as_solved(const DevProblem& P, int mode, hipStream_t s) {
  if (fewWindows(P.n_win, P.cu_count) && P.n_win <= kImuFewChunkWindows) {
    const int np = P.n_pprior + P.n_sbprior + P.n_relpose;
    const int nb = (P.n_imu + kImuPerWG - 1) / kImuPerWG + (np + 63) / 64;
    if (nb > 0) hipLaunchKernelGGL(k_eval_few<kImuKFew>, dim3(nb), dim3(64), 0, s, P.self, mode, 0);
    return;
  }
  launch_eval_imu(P, mode, s);
}
void launch_eval(const DevProblem& P, int mode, hipStream_t s) {
  if (fewWindows(P.n_win, P.cu_count)) {
    const int np = P.n_pprior + P.n_sbprior + P.n_relpose;
    const int nObs = (P.n_obs + 63) / 64, nb = nObs + (P.n_imu + kImuPerWG - 1) / kImuPerWG + (np + 63) / 64;
    if (nb <= 0) return;
    if (P.n_win <= kImuFewChunkWindows) hipLaunchKernelGGL(k_eval_few<kImuKFew>, dim3(nb), dim3(64), 0, s, P.self, mode, nObs);
    else hipLaunchKernelGGL(k_eval_few<kImuK>, dim3(nb), dim3(64), 0, s, P.self, mode, nObs);
    return;
  }
  launch_eval_obs(P, mode, s);
  launch_eval_imu(P, mode, s);
  launch_eval_priors(P, mode, s);
}

void launch_imu_append(const DevProblem& P, hipStream_t s) {
  if (P.n_imu > 0)
    hipLaunchKernelGGL(k_eval_imu<true>, dim3((P.n_imu + kImuPerWG - 1) / kImuPerWG), dim3(64), 0, s, P.self, 0);
}

}  // namespace okg
