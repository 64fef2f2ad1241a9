// kernels_backsub.hip — landmark back substitution, the landmarks' dogleg vectors and the J*v forms
// of the reprojection residuals, in one pass over the landmark groups of k_lm_visit.
//
// After the reduced system is solved (y_f, Jacobi-scaled), DoglegStrategy needs per landmark
//   y_l = V'^-1 (s g_l - s W^T s_p y_p) = L^-T (zz - L^-1 s_l sum_v W_v^T s_p y_p)
//   gauss_newton_step_ = -D y_l,  gradient_ = s g_l / D,  v_c = gradient_ / D
// (SchurEliminator back substitution; DoglegStrategy::ComputeGradient / ComputeGaussNewtonStep)
// and per reprojection residual the rows of J_s v_c and J_s v_g (v_g = -y) whose squares and cross
// product give the model cost of every dogleg step of this linearisation (k_reduce, k_dogleg).
// W_v^T s_p y_p is formed from the stored linearisation (r | A) that the J*v part reads anyway, so
// the per-visit Schur operands Z of k_lm_visit never leave its LDS.
// One workgroup per landmark group (whole landmarks, <= kLmGroupVisits visits), one thread per
// (landmark, pose) visit, three phases separated by barriers:
//   visit    q_v = W_v^T s_p y_p = -sum_obs J_l^T (J_p g_p), g_p = -s_p y_p
//   landmark y_l from the q_v of its visits (visit order), its dogleg vectors, and s v_c, -s y_l
//            to LDS for the visits
//   visit    J_s v_c and J_s v_g of its 1-2 residuals (A re-read from L1/L2)
// The f-blocks' GN vectors come from the Cholesky's back substitution (v_c of the poses); the IMU factors', priors' and
// edges' J*v stay in k_jv. The group's J*v forms and landmark norms leave as one fixed-order sum per
// group (grp_red), so the per-window reductions read ~36 records instead of every visit and landmark.
#include "device_problem.hpp"
#include "jv_groups.hpp"
#include "launch.hpp"
#include "okvisgpu_math.hpp"

namespace okg {

// EXT (batches with variable extrinsics): an observation through a variable camera also carries
// J_e (extrJacobian) in q_v and in its J*v rows; its extrinsics' scaled steps are read per observation.
struct ExtTerm {  // J_e and the extrinsics' s v_c / -s y of one observation
  double Je[12], ce[6], ge[6];
};
__device__ __forceinline__ bool loadExtTerm(const DevProblem& P, int o, int w, int xs, const double C_WS[9],
                                            const double p3[3], double w4, const double A[6], ExtTerm& X) {
  if (!(P.obs_flags[o] & 4)) return false;
  const int e = P.cam_pose[P.obs_cam[o]];
  const size_t b = (size_t)P.win_foff[w] + P.pose_f[e];
  extrJacobian(A, C_WS, p3, w4, P.pose[xs] + 7 * (size_t)e, X.Je);
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    const double sc = P.sF[b + c];
    X.ce[c] = sc * P.vF[b + c];
    X.ge[c] = -sc * P.yF[b + c];
  }
  return true;
}

template <bool EXT>
__global__ __launch_bounds__(kLmGroupVisits) void k_lm_backsub_jv(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  if (!EXT && (int)blockIdx.x >= P.n_lmg) {  // trailing workgroups: the factors' J*v (uniform per workgroup;
                                             // the extrinsics variant launches k_jv beside it instead)
    jvGroups(P, (int)blockIdx.x - P.n_lmg);
    return;
  }
  const int t = threadIdx.x;
  const auto gi = gmem(reinterpret_cast<const int4*>(P.lmg_info + kLmgInfo * blockIdx.x));
  const int4 gi0 = gi[0], gi1 = gi[kLmgInfo / 4];
  const int l0 = gi0.x, l1 = gi1.x;
  const int w = gi0.z;  // a group never spans windows
  const int v0 = gi0.y, v1 = gi1.y;
  const int v = v0 + t;
  const bool hasV = v < v1;
  // The visit record (index clamped, loaded unconditionally) and the WinState fields are loaded
  // together; the window test needs no short-circuit branch and consumes the visit record (vc >> 31
  // is 0), so the compiler cannot sink those loads behind it (as in k_lm_visit).
  const int vc = hasV ? v : v0;
  const int vLm = gmem(P.visit_lm)[vc], vPose = gmem(P.visit_pose)[vc];
  const int obB = gmem(P.visit_obs_begin)[vc], obE = gmem(P.visit_obs_begin)[vc + 1];
  const auto gst = gmem(P.st + w);
  const int sDone = gst->done, sNeed = gst->need_gn, sFail = gst->gn_failed, sLcur = gst->lcur, sXcur = gst->xcur;
  const bool skip = (sDone != 0) | (sNeed == 0) | (sFail != 0) | (((vLm ^ vPose ^ obB ^ obE) & (vc >> 31)) != 0);
  if (skip) return;  // uniform
  __shared__ double sQ[3][kLmGroupVisits];
  __shared__ double sC[6][kLmGroupMax];  // per landmark: s v_c (3) | -s y_l (3)
  const int l = hasV ? vLm : l0;
  const int pose = hasV ? vPose : 0;
  const int ob0 = hasV ? obB : 0, ob1 = hasV ? obE : 0;
  // the landmark flag, the pose's f offset, the parameters and the first observation together
  const auto lin = gmem(pick2(sLcur, P.obs_lin[0], P.obs_lin[1]));
  const int64_t S = P.obs_stride;
  const int lfreeI = gmem(P.lm_free)[l], pfI = gmem(P.pose_f)[pose];
  const auto hpp = gmem(pick2(sXcur, P.lm[0], P.lm[1]) + 4 * (size_t)l);
  const auto twp = gmem(pick2(sXcur, P.pose[0], P.pose[1]) + 7 * (size_t)pose);
  const double hp[4] = {hpp[0], hpp[1], hpp[2], hpp[3]};
  double tw[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) tw[k] = (EXT || k < 3) ? twp[k] : 0.0;
  const int fl0 = gmem(P.obs_flags)[obB];
  double A0[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) A0[k] = lin[(2 + k) * S + obB];
  asm volatile("" ::"v"(lfreeI), "v"(pfI), "v"(hp[0]), "v"(hp[1]), "v"(hp[2]), "v"(hp[3]), "v"(tw[0]), "v"(tw[1]),
               "v"(tw[2]), "v"(fl0), "v"(A0[0]), "v"(A0[1]), "v"(A0[2]), "v"(A0[3]), "v"(A0[4]), "v"(A0[5]));
  const int xs = sXcur;
  const int pf = hasV ? pfI : -1;
  const bool lfree = lfreeI != 0;
  // the pose's scaled step and gradient (a valid dummy address when the pose is not free)
  double cp[6], gp[6];
  {
    const size_t b = pf >= 0 ? (size_t)P.win_foff[w] + pf : 0;
    const auto sFp = gmem(P.sF + b), vFp = gmem(P.vF + b), yFp = gmem(P.yF + b);
    double sc[6], vv[6], yy[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      sc[c] = sFp[c];
      vv[c] = vFp[c];
      yy[c] = yFp[c];
    }
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      cp[c] = pf >= 0 ? sc[c] * vv[c] : 0.0;
      gp[c] = pf >= 0 ? -sc[c] * yy[c] : 0.0;
    }
  }
  const double w4 = hp[3];
  const double p3[3] = {hp[0] - tw[0] * w4, hp[1] - tw[1] * w4, hp[2] - tw[2] * w4};
  double C_WS[9];
  if (EXT) qrot(qnormalize(Q{tw[3], tw[4], tw[5], tw[6]}), C_WS);

  // ---- visit: q_v = W_v^T s_p y_p
  double q[3] = {0.0, 0.0, 0.0};
  if ((pf >= 0 || EXT) && lfree)
    for (int o = ob0; o < ob1; ++o) {
      // (a masked observation contributes exact zeros: selects, so no load sits behind a branch)
      double A[6], Jp[12], Jl[6];
      int fl = fl0;
#pragma unroll
      for (int k = 0; k < 6; ++k) A[k] = A0[k];
      if (o != ob0) {
        fl = gmem(P.obs_flags)[o];
#pragma unroll
        for (int k = 0; k < 6; ++k) A[k] = lin[(2 + k) * S + o];
      }
      const bool use = !(fl & 2);
#pragma unroll
      for (int k = 0; k < 6; ++k) A[k] = use ? A[k] : 0.0;
      obsJacobians(A, p3, w4, Jp, Jl);
      ExtTerm X;
      const bool hasE = EXT && loadExtTerm(P, o, w, xs, C_WS, p3, w4, A, X);
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        double jg = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) jg += Jp[r * 6 + c] * gp[c];
        if (hasE)
#pragma unroll
          for (int c = 0; c < 6; ++c) jg += X.Je[r * 6 + c] * X.ge[c];
#pragma unroll
        for (int a = 0; a < 3; ++a) q[a] -= Jl[r * 3 + a] * jg;
      }
    }
#pragma unroll
  for (int a = 0; a < 3; ++a) sQ[a][t] = q[a];
  ldsBarrier();

  // ---- landmark: y_l = L^-T (zz - L^-1 s_l sum_v q_v), the dogleg vectors
  double lred[3] = {0.0, 0.0, 0.0};
  if (t < l1 - l0) {
    const int L = l0 + t;
    double c6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    // every operand of the landmark is loaded up front, together (stores to the output vectors
    // below would otherwise keep later loads from being hoisted above them)
    const int lf = gmem(P.lm_free)[L];
    const int mb = gmem(P.lm_visit_begin)[L] - v0, me = gmem(P.lm_visit_begin)[L + 1] - v0;
    double li[9], s3[3], zz[3], dgv[3], lg[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) li[i] = gmem(P.lm_Linv)[9 * (size_t)L + i];  // lower triangular
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const size_t i = 3 * (size_t)L + a;
      s3[a] = gmem(P.sL)[i];
      zz[a] = gmem(P.lm_zz)[i];
      dgv[a] = gmem(P.diagL)[i];
      lg[a] = gmem(P.lm_g)[i];
    }
    if (lf) {
      double qs[3] = {0.0, 0.0, 0.0};
      for (int m = mb; m < me; ++m)
#pragma unroll
        for (int a = 0; a < 3; ++a) qs[a] += sQ[a][m];
      double u[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) qs[a] *= s3[a];
#pragma unroll
      for (int a = 0; a < 3; ++a) u[a] = zz[a] - (li[a * 3] * qs[0] + li[a * 3 + 1] * qs[1] + li[a * 3 + 2] * qs[2]);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        double y = 0.0;
#pragma unroll
        for (int c = a; c < 3; ++c) y += li[c * 3 + a] * u[c];
        const size_t i = 3 * (size_t)L + a;
        const double dg = dgv[a];
        gmemw(P.yL)[i] = y;
        const double gn = -dg * y;
        gmemw(P.gnL)[i] = gn;
        const double gr = s3[a] * lg[a] / dg;
        const double vc = gr / dg;
        gmemw(P.dgL)[i] = gr;
        gmemw(P.vL)[i] = vc;
        // this landmark's share of |gradient_|^2, |gauss_newton_step_|^2, gradient_ . gn (k_dogleg,
        // k_reduce), summed per group below
        lred[0] += gr * gr;
        lred[1] += gn * gn;
        lred[2] += gr * gn;
        c6[a] = s3[a] * vc;
        c6[3 + a] = -s3[a] * y;
      }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) sC[i][t] = c6[i];
  }
  ldsBarrier();

  // ---- visit: J_s v_c and J_s v_g of its residuals (fixed residuals excluded)
  const int u = hasV ? l - l0 : 0;
  double cl[3], gl[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    cl[c] = sC[c][u];
    gl[c] = sC[3 + c][u];
  }
  double acc[3] = {0.0, 0.0, 0.0};
  for (int o = ob0; o < ob1; ++o) {
    double A[6], Jp[12], Jl[6];
    const bool use = !(gmem(P.obs_flags)[o] & 2);
#pragma unroll
    for (int k = 0; k < 6; ++k) A[k] = lin[(2 + k) * S + o];
#pragma unroll
    for (int k = 0; k < 6; ++k) A[k] = use ? A[k] : 0.0;
    obsJacobians(A, p3, w4, Jp, Jl);
    ExtTerm X;
    const bool hasE = EXT && loadExtTerm(P, o, w, xs, C_WS, p3, w4, A, X);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      double jc = 0.0, jg = 0.0;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        jc += Jp[r * 6 + c] * cp[c];
        jg += Jp[r * 6 + c] * gp[c];
      }
      if (hasE)
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          jc += X.Je[r * 6 + c] * X.ce[c];
          jg += X.Je[r * 6 + c] * X.ge[c];
        }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        jc += Jl[r * 3 + c] * cl[c];
        jg += Jl[r * 3 + c] * gl[c];
      }
      acc[0] += jc * jc;
      acc[1] += jg * jg;
      acc[2] += jc * jg;
    }
  }
  // ---- the group's sums, fixed order: a shuffle tree per wavefront, then the 4 wavefronts
  double red[6] = {acc[0], acc[1], acc[2], lred[0], lred[1], lred[2]};
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) red[k] += __shfl_xor(red[k], m, 64);
  __shared__ double sW[kLmGroupVisits / 64][6];
  if ((t & 63) == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) sW[t >> 6][k] = red[k];
  ldsBarrier();
  if (t < 6) {
    double a = sW[0][t];
#pragma unroll
    for (int wv = 1; wv < kLmGroupVisits / 64; ++wv) a += sW[wv][t];
    gmemw(P.grp_red)[(size_t)blockIdx.x * kGrpRed + t] = a;
  }
}

// grid: the landmark groups, then the factors' J*v workgroups (jvGroups)
void launch_lm_backsub(const DevProblem& P, hipStream_t s) {
  if (P.n_xvisit > 0) {  // (the J*v path would raise the extrinsics variant's registers: a launch of its own)
    if (P.n_lmg > 0) hipLaunchKernelGGL(k_lm_backsub_jv<true>, dim3(P.n_lmg), dim3(kLmGroupVisits), 0, s, P.self);
    launch_jv(P, s);
    return;
  }
  const int nb = P.n_lmg + jvBlocks(P);
  if (nb > 0) hipLaunchKernelGGL(k_lm_backsub_jv<false>, dim3(nb), dim3(kLmGroupVisits), 0, s, P.self);
}

}  // namespace okg
