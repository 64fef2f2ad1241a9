// jv_groups.hpp — J_s v_c and J_s v_g of the IMU factors, priors and pose-graph edges (formerly
// k_jv in kernels_control.hip), run by the trailing workgroups of k_lm_backsub_jv: the two passes of
// a Gauss-Newton step's J*v share one launch. 256-thread workgroups, 16 groups of 16 lanes each.
#pragma once
#include "device_problem.hpp"
#include "okvisgpu_math.hpp"

namespace okg {

static_assert(kLmGroupVisits == 256, "jvGroups runs as 256-thread workgroups of k_lm_backsub_jv");

__device__ __forceinline__ bool jvSelect(const DevProblem& P, int w) {
  const WinState& s = P.st[w];
  return !s.done && s.need_gn && !s.gn_failed;
}

// Accumulates one residual row's J_s v_c and J_s v_g into (jcc, jgg, jcg).
__device__ __forceinline__ void jvAcc(double jc, double jg, double (&a)[3]) {
  a[0] += jc * jc;
  a[1] += jg * jg;
  a[2] += jc * jg;
}

// Once per Gauss-Newton step, per residual block: J_s v_c and J_s v_g with J_s = J diag(s) (the
// Jacobi-scaled Jacobian the dogleg works in), v_c = gradient_ / diagonal_ (Cauchy direction) and
// v_g = gauss_newton_step_ / diagonal_ = -y. Every dogleg step of this linearisation is
// step = ca v_c + cb v_g, so |J_s step|^2 = ca^2 jcc + 2 ca cb jcg + cb^2 jgg is formed in k_dogleg,
// also for the steps re-tried at a smaller radius without a new GN step (DoglegStrategy reuse_).
// The companion (J_s step).r = step.(s g) uses the gradient g = J^T r already at hand.
// Here the IMU factors, priors and relative-pose edges, one thread each; the reprojection residuals'
// share is formed with the landmark back substitution (k_lm_backsub_jv, kernels_backsub.hip).
// One 16-lane group per factor (IMU factor, pose prior, speed/bias prior, relative-pose edge, in
// that order), lane = residual row: J_s v_c and J_s v_g of its row over the factor's free blocks,
// then (jc^2, jg^2, jc jg) summed over the rows by a fixed shuffle tree.
__device__ __forceinline__ void jvGroups(const DevProblem& P, int block) {
  const int gid = (block * 256 + (int)threadIdx.x) >> 4, r = threadIdx.x & 15;
  const double* __restrict__ cF = P.vF;
  const double* __restrict__ yF = P.yF;
  int u = gid, w = 0, nr = 0, nb = 0, ld = 0;
  const double* J = nullptr;  // row-major rows of stride ld, columns of block q from col[q]
  int off[4] = {-1, -1, -1, -1}, n[4] = {0, 0, 0, 0}, col[4] = {0, 0, 0, 0};
  double* out = nullptr;
  size_t ostride = 0;
  bool live = false;
  // IMU factors (the bulk): every operand in three rounds of loads, no branch on a loaded value
  // before they are issued. Lane r holds row r of the 15x30 Jacobian; lanes r and r + 16 of the
  // group form the scaled direction vectors of columns r and r + 16, exchanged through LDS.
  __shared__ double sVc[256 / 16][32][2];
  if (gid < P.n_fac) {
    const int f = gid, grp = threadIdx.x >> 4;
    const int fw = gmem(P.imu_win)[f], ffl = gmem(P.imu_flags)[f];
    const int4 blk = gmem(reinterpret_cast<const int4*>(P.imu_blocks))[f];
    const auto gst = gmem(P.st + fw);
    const int sDone = gst->done, sNeed = gst->need_gn, sFail = gst->gn_failed, lcur = gst->lcur;
    // (a host-evaluated factor marks unused slots -1: clamped load, offset -1)
    const int o0 = blk.x < 0 ? -1 : gmem(P.pose_f)[max(blk.x, 0)], o1 = blk.y < 0 ? -1 : gmem(P.sb_f)[max(blk.y, 0)],
              o2 = blk.z < 0 ? -1 : gmem(P.pose_f)[max(blk.z, 0)], o3 = blk.w < 0 ? -1 : gmem(P.sb_f)[max(blk.w, 0)];
    const int foff = gmem(P.win_foff)[fw];
    const bool fl = (sDone == 0) & (sNeed != 0) & (sFail == 0), act = fl & !(ffl & 2);
    // this lane's two columns (c = r, r + 16 < 30): block offset and position
    double vcv[2], vgv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = r + 16 * h;
      const int q = c < 6 ? 0 : c < 15 ? 1 : c < 21 ? 2 : 3;
      const int cq = c - (q == 0 ? 0 : q == 1 ? 6 : q == 2 ? 15 : 21);
      const int oq = q == 0 ? o0 : q == 1 ? o1 : q == 2 ? o2 : o3;
      const bool ok = act && c < 30 && oq >= 0;
      const size_t i = ok ? (size_t)foff + oq + cq : 0;
      const double sc = gmem(P.sF)[i], cv = gmem(cF)[i], yv = gmem(yF)[i];
      vcv[h] = ok ? sc * cv : 0.0;
      vgv[h] = ok ? -sc * yv : 0.0;
    }
    const auto Jr = gmem(pick2(lcur, P.imu_lin[0], P.imu_lin[1]) + (size_t)(act ? f : 0) * kImuLin + 15 +
                         30 * (size_t)min(r, 14));
    double jr[30];
#pragma unroll
    for (int c = 0; c < 30; ++c) jr[c] = Jr[c];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      sVc[grp][r + 16 * h][0] = vcv[h];
      sVc[grp][r + 16 * h][1] = vgv[h];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double jc0 = 0.0, jg0 = 0.0;
#pragma unroll
    for (int c = 0; c < 30; ++c) {
      jc0 += jr[c] * sVc[grp][c][0];
      jg0 += jr[c] * sVc[grp][c][1];
    }
    double a3[3] = {r < 15 ? jc0 * jc0 : 0.0, r < 15 ? jg0 * jg0 : 0.0, r < 15 ? jc0 * jg0 : 0.0};
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int m = 8; m > 0; m >>= 1) a3[k] += __shfl_xor(a3[k], m, 64);
    if (fl && r == 0)
      for (int k = 0; k < 3; ++k) P.imu_jv[(size_t)k * P.n_fac + f] = a3[k];
    return;
  }
  if (u < P.n_fac) {
  } else if ((u -= P.n_fac) < P.n_pprior) {
    w = P.pp_win[u];
    if (jvSelect(P, w)) {
      live = true;
      out = P.pp_jv + u;
      ostride = P.n_pprior;
      J = P.pp_lin[P.st[w].lcur] + 42 * (size_t)u + 6;
      nr = 6; ld = 6; nb = 1;
      off[0] = P.pose_f[P.pp_block[u]]; n[0] = 6;
    }
  } else if ((u -= P.n_pprior) < P.n_sbprior) {
    w = P.sbp_win[u];
    if (jvSelect(P, w)) {
      live = true;
      out = P.sbp_jv + u;
      ostride = P.n_sbprior;
      J = P.sbp_lin[P.st[w].lcur] + 90 * (size_t)u + 9;
      nr = 9; ld = 9; nb = 1;
      off[0] = P.sb_f[P.sbp_block[u]]; n[0] = 9;
    }
  } else if ((u -= P.n_sbprior) < P.n_relpose) {
    w = P.rp_win[u];
    if (jvSelect(P, w)) {
      live = true;
      out = P.rp_jv + u;
      ostride = P.n_relpose;
      if (!(P.rp_flags[u] & 2)) {
        J = P.rp_lin[P.st[w].lcur] + kRelPoseLin * (size_t)u + 6;
        nr = 6; ld = 12; nb = 2;
        off[0] = P.pose_f[P.rp_blocks[2 * u]]; off[1] = P.pose_f[P.rp_blocks[2 * u + 1]];
        n[0] = 6; n[1] = 6; col[1] = 6;
      }
    }
  }
  double jc = 0.0, jg = 0.0;
  if (live && r < nr) {
    const size_t foff = P.win_foff[w];
    for (int q = 0; q < nb; ++q) {
      if (off[q] < 0) continue;
      for (int c = 0; c < n[q]; ++c) {
        const size_t i = foff + off[q] + c;
        const double jv = J[r * ld + col[q] + c];
        jc += jv * (P.sF[i] * cF[i]);
        jg += jv * (-P.sF[i] * yF[i]);
      }
    }
  }
  double a[3] = {jc * jc, jg * jg, jc * jg};
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int m = 8; m > 0; m >>= 1) a[k] += __shfl_xor(a[k], m, 64);
  if (live && r == 0)
    for (int k = 0; k < 3; ++k) out[(size_t)k * ostride] = a[k];
}


// 16-lane groups of jvGroups -> workgroups
inline int jvBlocks(const DevProblem& P) { return (P.n_fac + P.n_pprior + P.n_sbprior + P.n_relpose + 15) / 16; }

}  // namespace okg
