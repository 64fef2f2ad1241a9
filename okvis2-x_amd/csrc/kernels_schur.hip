// kernels_schur.hip — landmark elimination (DENSE_SCHUR) for gfx950, FP64.
//
// The reduced ("camera") system of a window is formed exactly as Ceres' SchurEliminator does for
// e-blocks = landmarks, but organised for the GPU:
//   k_lm_visit    one workgroup per landmark group, one thread per (landmark, pose) visit:
//                 J from the stored linearisation, H_pp = J_p^T J_p and g_p = J_p^T r per visit
//                 (unscaled), V = J_l^T J_l and g_l per landmark (iteration 0: Jacobi scaling),
//                 the landmark's 3x3 LLT of s V s + mu D^2 (InvertPSDMatrix) -> L^-1, L^-1 s g,
//                 and per visit Z = s_p W s_l L^-T and U z (Y_a U_b^T = Z_a Z_b^T) — the
//                 per-e-block SchurEliminator work in one pass; W never leaves the registers.
//   k_imu_hess    one wavefront per IMU factor: J^T J (packed) and J^T r of its 15x30 Jacobian.
//   k_fgrad       one wavefront per f-block (pose / speed-bias): unscaled gradient and
//                 diag(H_ff), and at iteration 0 the Jacobi scaling 1/(1+sqrt(diag)).
//   k_zero_S      clears the structurally non-zero tiles of S (padding / gap diagonal = 1), once per build.
//   k_assemble_pp one wavefront per pose-pose block pair (i >= j): 8 groups of 6 lanes (one per
//                 row) sum fixed, interleaved subsets of the pair's contributions — visits,
//                 landmark pairs (the Y_i U_j^T Schur terms), IMU / prior J^T J sub-blocks — and
//                 a fixed tree combines the groups, so the sum is deterministic without atomics;
//                 diagonal pairs also emit the Schur rhs and the dogleg diagonal.
//   k_assemble_sb one wavefront per block pair involving a speed/bias block (one entry per lane).
//   (the f-blocks' Gauss-Newton step / dogleg gradient: the Cholesky's back substitution, gnFinalizeRow)
//                 (the landmarks' back substitution and vectors: k_lm_backsub_jv, kernels_backsub.hip).
#include <algorithm>
#include <cfloat>
#include <cstdlib>

#include "dev_clock.hpp"
#include "device_problem.hpp"
#include "gradnorm.hpp"
#include "launch.hpp"
#include "okvisgpu_math.hpp"

namespace okg {

__device__ __forceinline__ int sym6(int a, int b) {  // packed upper triangle of a 6x6
  if (a > b) { const int t = a; a = b; b = t; }
  return a * 6 - (a * (a - 1)) / 2 + (b - a);
}
__device__ __forceinline__ int sym3(int a, int b) {
  if (a > b) { const int t = a; a = b; b = t; }
  return a * 3 - (a * (a - 1)) / 2 + (b - a);
}

// sum of x[m0..m1) as four interleaved partial sums (four LDS loads in flight, a quarter of the
// dependent adds), combined in a fixed order
__device__ __forceinline__ double rangeSum(const double* x, int m0, int m1) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int m = m0;
  for (; m + 4 <= m1; m += 4) {
    a0 += x[m];
    a1 += x[m + 1];
    a2 += x[m + 2];
    a3 += x[m + 3];
  }
  for (; m < m1; ++m) a0 += x[m];
  return (a0 + a1) + (a2 + a3);
}

__device__ __forceinline__ bool linSelect(const DevProblem& P, int w, int lin_mode) {
  const WinState& s = P.st[w];
  if (s.done) return false;
  if (lin_mode == 1 && !s.accepted) return false;
  return true;
}

// Landmark-major linearisation + landmark elimination prep, one workgroup per landmark group
// (whole landmarks, <= kLmGroupVisits visits; visits of a landmark are contiguous), one thread
// per (landmark, pose) visit. Restates SchurEliminator's per-e-block work:
//   visit    J_p, J_l of its 1-2 residuals from the stored linearisation (r | A) -> W = J_p^T J_l,
//            H = J_p^T J_p and g = J_p^T r (stored for k_fgrad / k_assemble_pp), and its share
//            of V = J_l^T J_l, g_l = J_l^T r (LDS)
//   landmark (one thread each) V, g_l summed over its visits in visit order; iteration 0: the
//            Jacobi scaling 1 / (1 + sqrt(diag V)); then the 3x3 LLT of s V s + mu D^2
//            (InvertPSDMatrix) -> L^-1, zz = L^-1 (s g), the dogleg diagonal D
//   visit    Z = s_p W s_l L^-T and U z = Z zz, the operands of the Schur terms
//            Y_a U_b^T = Z_a Z_b^T (the partial blocks below; Z never leaves the workgroup)
// The barriers order LDS only (ldsBarrier): no thread reads global data another thread of the
// workgroup wrote, and a full __syncthreads() would also wait for the segment / landmark stores.
// mode 0: linearisation at iteration 0 (no Z: the pose scaling comes from k_fgrad afterwards);
// mode 1: linearisation after an accepted step, Z for the new mu (WinState::z_mu);
// mode 2: GN prep of windows whose Z is stale (mu raised by a retry or an invalid step): W is
//         recomputed from the stored linearisation, V / g_l reused.
__device__ __forceinline__ bool lmVisitSelect(const DevProblem& P, int w, int mode) {
  const WinState& s = P.st[w];
  if (s.done) return false;
  if (mode == 0) return true;
  if (mode == 1) return s.accepted;
  return s.need_gn && !s.gn_failed && s.z_mu != s.mu;
}

#ifndef OKG_LMV_OCC
#define OKG_LMV_OCC 3
#endif
#ifndef OKG_PART_ROWS
#define OKG_PART_ROWS 2
#endif
constexpr int kPartRows = OKG_PART_ROWS, kPartThreads = 6 / kPartRows;  // partial-block rows per thread
static_assert(kPartRows == 2 || kPartRows == 3, "OKG_PART_ROWS must be 2 or 3");
// (development-only phase clock of k_lm_visit<1>: LCLK_INIT / LCLK / LCLK_END, dev_clock.hpp)
// (mode is a template parameter: each mode is its own specialised kernel, and rocprof reports them
// apart — k_lm_visit<1> is the per-iteration linearisation, k_lm_visit<2> the GN prep)
// EXT (batches with variable extrinsics): threads nvg.. of a group are its extrinsic visits — per
// (landmark, variable camera) J_e of the landmark's observations through that camera
// (implementation/ReprojectionError.hpp:186-214, extrJacobian), giving W_e, H_ee, g_e, and so Z_e and
// the products with the pose visits' Z exactly like a pose visit; V / g_l come from the pose visits.
// (the body of one landmark group grp; the kernels below run it per workgroup or per window loop)
// LDS of lmVisitGroup at namespace scope: one allocation per kernel whatever modes it runs
// (k_lin_few<.., true> runs modes 1 and 2). gLmvBuf rows 0..8: visit shares of V (6) | g_l (3);
// rows 9..17: visit values being summed into segments; finally rows 0..17: the visits' Z for the
// partial Schur blocks. gLmvLz per landmark: L^-1 (9) | zz (3) | s_l (3). gLmvPC: the group's
// landmark-pair products (a | b << 16).
__shared__ double gLmvBuf[18][kLmGroupVisits];
__shared__ double gLmvLz[15][kLmGroupMax];
__shared__ int gLmvPC[kLmPartStage];
template <int mode, bool EXT>
__device__ __forceinline__ void lmVisitGroup(const DevProblem& P, const int grp) {
  const int t = threadIdx.x;
  const auto gi = gmem(reinterpret_cast<const int4*>(P.lmg_info + kLmgInfo * grp));
  const int4 gi0 = gi[0], gi1 = gi[kLmgInfo / 4];
  const int l0 = gi0.x, l1 = gi1.x, v0 = gi0.y, v1 = gi1.y;
  double (*sBuf)[kLmGroupVisits] = gLmvBuf;
  double (*sLz)[kLmGroupMax] = gLmvLz;
  int* sPC = gLmvPC;
  double (*sVg)[kLmGroupVisits] = sBuf;
  double (*sR)[kLmGroupVisits] = sBuf + 9;
  const int w = gi0.z;                       // a group never spans windows
  const int v = v0 + t;
  const bool hasV = v < v1;
  // window test (lmVisitSelect) from one set of WinState loads, no short-circuit branches
  const auto gst = gmem(P.st + w);
  const int sDone = gst->done, sAcc = gst->accepted, sNeed = gst->need_gn, sFail = gst->gn_failed;
  const int sLcur = gst->lcur, sXcur = gst->xcur;
  const double sZmu = gst->z_mu, sMu = gst->mu;
  const bool selW = mode == 0 ? !sDone : mode == 1 ? (!sDone & (sAcc != 0)) : (!sDone & (sNeed != 0) & !sFail & (sZmu != sMu));
  // GN prep concerns few windows: test first, so that the other groups exit without loading
  if (mode == 2 && !selW) return;  // uniform
  // the visit record (index clamped, loaded unconditionally); in modes 0 / 1 it is issued before
  // the window test so that its latency overlaps the WinState load
  const int vc = hasV ? v : v0;
  const int vLm = gmem(P.visit_lm)[vc], vPose = gmem(P.visit_pose)[vc], vSlot = gmem(P.visit_slot)[vc];
  const int obBeg = gmem(P.visit_obs_begin)[vc], obEnd = gmem(P.visit_obs_begin)[vc + 1];
  // (the visit record is folded into the test, so the compiler issues its loads before the branch
  // instead of after it: vc >> 31 is 0, so the second term is always false)
  const bool skip = !selW | (((vLm ^ vPose ^ vSlot ^ obBeg ^ obEnd) & (vc >> 31)) != 0);
  if (skip) { LCLK_END return; }  // uniform
  LCLK_INIT
  // the group's landmark-pair products go to LDS by DMA now (no registers held; they land with the
  // visit loads below and are read in the last phase)
  const int4 gp0 = gi[1], gp1 = gi[kLmgInfo / 4 + 1];
  const int pg0 = gp0.x, npart = gp1.x - pg0, pc0 = gp0.y, npc = gp1.y - pc0;
  const bool staged = npc <= kLmPartStage;
  if (mode != 0 && staged && npc > 0) {
    const int wv = t >> 6;
    for (int c = 0; c < npc; c += kLmGroupVisits)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(P.part_contrib + pc0 + min(c + t, npc - 1)),
          (__attribute__((address_space(3))) void*)(sPC + c + 64 * wv), 4, 0, 0);
  }
  const int nvg = v1 - v0;
  const int xv = EXT ? P.lmg_xbegin[grp] + t - nvg : 0;
  const bool hasX = EXT && t >= nvg && xv < P.lmg_xbegin[grp + 1];
  const int l = hasV ? vLm : (hasX ? P.xvisit_lm[xv] : l0);
  const bool sel = hasV;
  const bool lfree = gmem(P.lm_free)[l] != 0;
  const int pose = hasV ? vPose : (hasX ? P.xvisit_pose[xv] : 0);
  const int pf = gmem(P.pose_f)[pose];
  // segment bookkeeping (consumed after the landmark phase)
  const int sg0 = gi0.w, nseg = gi1.w - sg0;
  const int slot = hasV ? vSlot : (hasX ? P.xvisit_slot[xv] : -1);
  double W[18], H[21], gp[6], Vv[6], gl[3];
#pragma unroll
  for (int i = 0; i < 18; ++i) W[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 21; ++i) H[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) { gp[i] = 0.0; Vv[i] = 0.0; }
#pragma unroll
  for (int i = 0; i < 3; ++i) gl[i] = 0.0;
  {
    // (buffer pointers picked by select, not by indexing P's arrays with a loaded value: that would
    // be one more dependent load)
    const auto lin = gmem(pick2(sLcur, P.obs_lin[0], P.obs_lin[1]));
    const int64_t S = P.obs_stride;
    // linearisation point of lin[lcur]: params X[xcur]
    const auto hp = gmem(pick2(sXcur, P.lm[0], P.lm[1]) + 4 * (size_t)l);
    const auto tw = gmem(pick2(sXcur, P.pose[0], P.pose[1]) + 7 * (size_t)pose);
    // first observation's flag and linearisation with the parameters, unconditionally (a clamped
    // visit still has one); a masked observation contributes exact zeros (selects, no branch, so
    // the loads are not sunk behind one)
    double r0[2], A0[6];
    const int fl0 = gmem(P.obs_flags)[obBeg];
    r0[0] = lin[0 * S + obBeg];
    r0[1] = lin[1 * S + obBeg];
#pragma unroll
    for (int k = 0; k < 6; ++k) A0[k] = lin[(2 + k) * S + obBeg];
    const double hp4[4] = {hp[0], hp[1], hp[2], hp[3]}, tw3[3] = {tw[0], tw[1], tw[2]};
    // all of the above are in flight together: the empty asm consumes them here, so none is sunk
    // behind a branch on another's value
    asm volatile("" ::"v"(r0[0]), "v"(r0[1]), "v"(A0[0]), "v"(A0[1]), "v"(A0[2]), "v"(A0[3]), "v"(A0[4]),
                 "v"(A0[5]), "v"(hp4[0]), "v"(hp4[1]), "v"(hp4[2]), "v"(hp4[3]), "v"(tw3[0]), "v"(tw3[1]),
                 "v"(tw3[2]), "v"(fl0));
    const bool use0 = sel & !(fl0 & 2);
#pragma unroll
    for (int k = 0; k < 2; ++k) r0[k] = use0 ? r0[k] : 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) A0[k] = use0 ? A0[k] : 0.0;
    const double w4 = hp4[3];
    const double p3[3] = {hp4[0] - tw3[0] * w4, hp4[1] - tw3[1] * w4, hp4[2] - tw3[2] * w4};
    auto accumulate = [&](const double* r, const double* A) {
      double Jp[12], Jl[6];
      obsJacobians(A, p3, w4, Jp, Jl);
      if (lfree) {
#pragma unroll
        for (int a2 = 0; a2 < 3; ++a2) {
          gl[a2] += Jl[a2] * r[0] + Jl[3 + a2] * r[1];
#pragma unroll
          for (int b2 = a2; b2 < 3; ++b2) Vv[sym3(a2, b2)] += Jl[a2] * Jl[b2] + Jl[3 + a2] * Jl[3 + b2];
        }
      }
      if (pf >= 0) {
#pragma unroll
        for (int a2 = 0; a2 < 6; ++a2) {
          gp[a2] += Jp[a2] * r[0] + Jp[6 + a2] * r[1];
#pragma unroll
          for (int b2 = a2; b2 < 6; ++b2) H[sym6(a2, b2)] += Jp[a2] * Jp[b2] + Jp[6 + a2] * Jp[6 + b2];
          if (lfree)
#pragma unroll
            for (int b2 = 0; b2 < 3; ++b2) W[a2 * 3 + b2] += Jp[a2] * Jl[b2] + Jp[6 + a2] * Jl[3 + b2];
        }
      }
    };
    accumulate(r0, A0);
    for (int ob = obBeg + 1; sel && ob < obEnd; ++ob) {
      double r[2], A[6];
      const bool use = !(gmem(P.obs_flags)[ob] & 2);
      r[0] = lin[0 * S + ob];
      r[1] = lin[1 * S + ob];
#pragma unroll
      for (int k = 0; k < 6; ++k) A[k] = lin[(2 + k) * S + ob];
#pragma unroll
      for (int k = 0; k < 2; ++k) r[k] = use ? r[k] : 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) A[k] = use ? A[k] : 0.0;
      accumulate(r, A);
    }
  }
  if (EXT && hasX) {  // extrinsic visit: H_ee, g_e, W_e over the landmark's observations via the camera
    const WinState& st = P.st[w];
    const auto lin = gmem(P.obs_lin[st.lcur]);
    const int64_t S = P.obs_stride;
    const double* hp = P.lm[st.xcur] + 4 * (size_t)l;
    const double* ex = P.pose[st.xcur] + 7 * (size_t)pose;
    const double w4 = hp[3];
    for (int k = P.xvisit_obs_begin[xv]; k < P.xvisit_obs_begin[xv + 1]; ++k) {
      const int ob = P.xvisit_obs[k];
      const double* tw = P.pose[st.xcur] + 7 * (size_t)P.obs_pose[ob];
      const double p3[3] = {hp[0] - tw[0] * w4, hp[1] - tw[1] * w4, hp[2] - tw[2] * w4};
      double C_WS[9];
      qrot(qnormalize(Q{tw[3], tw[4], tw[5], tw[6]}), C_WS);
      double r[2], A[6], Je[12];
      r[0] = lin[0 * S + ob];
      r[1] = lin[1 * S + ob];
#pragma unroll
      for (int kk = 0; kk < 6; ++kk) A[kk] = lin[(2 + kk) * S + ob];
      extrJacobian(A, C_WS, p3, w4, ex, Je);
#pragma unroll
      for (int a2 = 0; a2 < 6; ++a2) {
        gp[a2] += Je[a2] * r[0] + Je[6 + a2] * r[1];
#pragma unroll
        for (int b2 = a2; b2 < 6; ++b2) H[sym6(a2, b2)] += Je[a2] * Je[b2] + Je[6 + a2] * Je[6 + b2];
        if (lfree)  // J_l = -A
#pragma unroll
          for (int b2 = 0; b2 < 3; ++b2) W[a2 * 3 + b2] -= Je[a2] * A[b2] + Je[6 + a2] * A[3 + b2];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) sVg[i][t] = Vv[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) sVg[6 + i][t] = gl[i];
  ldsBarrier();
  LCLK(0)
  // Operands of the later phases, issued now so that they land during the landmark phase: this
  // thread's first segment ranges in the three segment passes (18, 9 and 6 values per segment) and
  // the pose scaling of its visit (a valid dummy address when the pose is not free).
  const auto gsr = gmem(reinterpret_cast<const int2*>(P.seg_range));
  const int sgl = max(nseg - 1, 0);
  const int2 rA = gsr[sg0 + min(t / 18, sgl)], rB = gsr[sg0 + min(t / 9, sgl)], rC = gsr[sg0 + min(t / 6, sgl)];
  // (and this thread's first partial block's product range)
  const int pfi = npart > 0 ? pg0 + min(t / kPartThreads, npart - 1) : 0;  // (index 1 exists: >= 8-byte arrays)
  const int pcA = gmem(P.part_cbegin)[pfi], pcB = gmem(P.part_cbegin)[pfi + 1];
  double spr[6];
  {
    const auto spp = gmem(pf >= 0 ? P.sF + (size_t)P.win_foff[w] + pf : P.pose[0]);
#pragma unroll
    for (int i = 0; i < 6; ++i) spr[i] = mode != 0 ? spp[i] : 0.0;
  }
  // ---- one thread per landmark of the group
  if (t < l1 - l0) {
    const int L = l0 + t;
    // (the window is w and already selected) the landmark's flag, visit range and scaling are
    // loaded together and consumed at one point
    const int lfreeL = gmem(P.lm_free)[L];
    const int ub = gmem(P.lm_visit_begin)[L] - v0, ue = gmem(P.lm_visit_begin)[L + 1] - v0;
    double s[3] = {1.0, 1.0, 1.0};
    if (mode != 0) {
      const auto sLp = gmem(P.sL + 3 * (size_t)L);
      s[0] = sLp[0];
      s[1] = sLp[1];
      s[2] = sLp[2];
    }
    asm volatile("" ::"v"(lfreeL), "v"(ub), "v"(ue), "v"(s[0]), "v"(s[1]), "v"(s[2]));
    WinState& st = P.st[w];
    {
      if (mode == 1 && L == P.win_lm_range[2 * w]) st.z_mu = sMu;  // one writer per window
      if (lfreeL) {
        double V[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
        if (mode == 2) {
#pragma unroll
          for (int i = 0; i < 6; ++i) V[i] = gmem(P.lm_V)[6 * (size_t)L + i];
#pragma unroll
          for (int i = 0; i < 3; ++i) g[i] = gmem(P.lm_g)[3 * (size_t)L + i];
        } else {
          for (int u = ub; u < ue; ++u) {
#pragma unroll
            for (int i = 0; i < 6; ++i) V[i] += sVg[i][u];
#pragma unroll
            for (int i = 0; i < 3; ++i) g[i] += sVg[6 + i][u];
          }
#pragma unroll
          for (int i = 0; i < 6; ++i) gmemw(P.lm_V)[6 * (size_t)L + i] = V[i];
#pragma unroll
          for (int i = 0; i < 3; ++i) gmemw(P.lm_g)[3 * (size_t)L + i] = g[i];
          if (mode == 0)  // Jacobi scaling fixed at iteration 0 (TrustRegionMinimizer)
            for (int a = 0; a < 3; ++a)
              gmemw(P.sL)[3 * (size_t)L + a] = P.opt.jacobi_scaling ? 1.0 / (1.0 + sqrt(V[sym3(a, a)])) : 1.0;
        }
        if (mode != 0) {
          const double mu = sMu;
          double A[9];
          for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) A[a * 3 + b] = s[a] * s[b] * V[sym3(a, b)];
          const double smu = sqrt(mu);
          for (int a = 0; a < 3; ++a) {
            const double dg = sqrt(fmin(fmax(A[a * 3 + a], P.opt.min_lm_diagonal), P.opt.max_lm_diagonal));
            gmemw(P.diagL)[3 * (size_t)L + a] = dg;
            const double d = dg * smu;
            A[a * 3 + a] += d * d;
          }
          // LLT and inverse (InvertPSDMatrix, full rank)
          double Lc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
          bool ok = true;  // (fully unrolled: no dynamically indexed private arrays)
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            double d = A[k * 3 + k];
#pragma unroll
            for (int j = 0; j < k; ++j) d -= Lc[k * 3 + j] * Lc[k * 3 + j];
            ok = ok && (d > 0.0);
            d = ok ? sqrt(d) : 1.0;
            Lc[k * 3 + k] = d;
#pragma unroll
            for (int i = k + 1; i < 3; ++i) {
              double tt = A[i * 3 + k];
#pragma unroll
              for (int j = 0; j < k; ++j) tt -= Lc[i * 3 + j] * Lc[k * 3 + j];
              Lc[i * 3 + k] = tt / d;
            }
          }
          double Li[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, zz[3] = {0, 0, 0};
          if (!ok) {
            st.gn_failed = 1;
          } else {
            // L^-1 (lower) and zz = L^-1 (s g): V'^-1 = L^-T L^-1, so Y_a U_b^T = Z_a Z_b^T, Z = U L^-T
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              Li[c * 3 + c] = 1.0 / Lc[c * 3 + c];
#pragma unroll
              for (int i = c + 1; i < 3; ++i) {
                double tt = 0.0;
#pragma unroll
                for (int j = c; j < i; ++j) tt -= Lc[i * 3 + j] * Li[j * 3 + c];
                Li[i * 3 + c] = tt / Lc[i * 3 + i];
              }
            }
            const double sg[3] = {s[0] * g[0], s[1] * g[1], s[2] * g[2]};
            for (int a = 0; a < 3; ++a) zz[a] = Li[a * 3 + 0] * sg[0] + Li[a * 3 + 1] * sg[1] + Li[a * 3 + 2] * sg[2];
          }
          const auto Lo = gmemw(P.lm_Linv + 9 * (size_t)L);
          for (int i = 0; i < 9; ++i) Lo[i] = Li[i];
          for (int a = 0; a < 3; ++a) gmemw(P.lm_zz)[3 * (size_t)L + a] = zz[a];
#pragma unroll
          for (int i = 0; i < 9; ++i) sLz[i][t] = Li[i];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            sLz[9 + i][t] = zz[i];
            sLz[12 + i][t] = s[i];
          }
        }
      }
    }
  }
  ldsBarrier();
  LCLK(1)
  asm volatile("" ::"v"(rA.x), "v"(rA.y), "v"(rB.x), "v"(rB.y), "v"(rC.x), "v"(rC.y), "v"(pcA),
               "v"(pcB));  // (not sunk into branches)
  // ---- segments: H | g of each (group, free pose) summed over its visits (visits are scattered
  // to their slots so that every segment is a contiguous LDS range). The visit shares of V / g_l
  // are consumed, so all 18 rows of sBuf take values: H[0..17], then H[18..20] | g_p.
  if (mode != 2) {
#pragma unroll
    for (int chunk = 0; chunk < 2; ++chunk) {
      const int nval = chunk == 0 ? 18 : 9;
      if (slot >= 0)
#pragma unroll
        for (int i = 0; i < nval; ++i) {
          const int e = 18 * chunk + i;
          sBuf[i][slot] = e < 21 ? H[e] : gp[e - 21];
        }
      ldsBarrier();
      if (t < nseg * nval) {  // first pass: the prefetched range
        const int sgi = t / nval, i = t - sgi * nval;
        const int2 r = chunk == 0 ? rA : rB;
        gmemw(P.seg_hg)[(size_t)(sg0 + sgi) * kSegHG + 18 * chunk + i] = rangeSum(sBuf[i], r.x, r.y);
      }
      for (int e = t + kLmGroupVisits; e < nseg * nval; e += kLmGroupVisits) {
        const int sgi = e / nval, i = e - sgi * nval;
        const int m0 = gmem(P.seg_range)[2 * (sg0 + sgi)], m1 = gmem(P.seg_range)[2 * (sg0 + sgi) + 1];
        gmemw(P.seg_hg)[(size_t)(sg0 + sgi) * kSegHG + 18 * chunk + i] = rangeSum(sBuf[i], m0, m1);
      }
      ldsBarrier();
    }
  }
  LCLK(2)
  if (mode == 0) return;
  asm volatile("" ::"v"(spr[0]), "v"(spr[1]), "v"(spr[2]), "v"(spr[3]), "v"(spr[4]), "v"(spr[5]));
  // ---- visit: Z = s_p W s_l L^-T (6x3) | U z = Z zz (6, summed into the segments)
  double o[kVisitZ + 6];
#pragma unroll
  for (int i = 0; i < kVisitZ + 6; ++i) o[i] = 0.0;
  if (pf >= 0 && lfree) {
    const int u = l - l0;
    double Li[9], zz[3], s3[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) Li[i] = sLz[i][u];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      zz[i] = sLz[9 + i][u];
      s3[i] = sLz[12 + i][u];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const double u0 = spr[r] * W[r * 3 + 0] * s3[0], u1 = spr[r] * W[r * 3 + 1] * s3[1],
                   u2 = spr[r] * W[r * 3 + 2] * s3[2];
      const double z0 = u0 * Li[0];
      const double z1 = u0 * Li[3] + u1 * Li[4];
      const double z2 = u0 * Li[6] + u1 * Li[7] + u2 * Li[8];
      o[r * 3 + 0] = z0; o[r * 3 + 1] = z1; o[r * 3 + 2] = z2;
      o[18 + r] = z0 * zz[0] + z1 * zz[1] + z2 * zz[2];
    }
  }
  if (slot >= 0)
#pragma unroll
    for (int i = 0; i < 6; ++i) sR[i][slot] = o[kVisitZ + i];
  ldsBarrier();
  if (t < nseg * 6) {  // first pass: the prefetched range
    const int sgi = t / 6, i = t - sgi * 6;
    gmemw(P.seg_uz)[(size_t)(sg0 + sgi) * kSegUz + i] = rangeSum(sR[i], rC.x, rC.y);
  }
  for (int e = t + kLmGroupVisits; e < nseg * 6; e += kLmGroupVisits) {
    const int sgi = e / 6, i = e - sgi * 6;
    const int m0 = gmem(P.seg_range)[2 * (sg0 + sgi)], m1 = gmem(P.seg_range)[2 * (sg0 + sgi) + 1];
    gmemw(P.seg_uz)[(size_t)(sg0 + sgi) * kSegUz + i] = rangeSum(sR[i], m0, m1);
  }
  // ---- partial Schur blocks: for each pose pair of the group, rows 2h, 2h+1 of sum Z_a Z_b^T over
  // the group's landmark-pair products (fixed order), from Z staged visit-major in LDS (144-byte
  // records read with 16-byte LDS loads)
  double* sZ = &sBuf[0][0];
  ldsBarrier();  // sR reads above are done
  LCLK(3)
  {
    double2* zo = reinterpret_cast<double2*>(sZ + kVisitZ * t);
#pragma unroll
    for (int i = 0; i < kVisitZ / 2; ++i) zo[i] = double2{o[2 * i], o[2 * i + 1]};
  }
  // (a group of one landmark with more products than the stage holds streams them from HBM)
  ldsBarrier();
  LCLK(4)
  const auto gPC = gmem(P.part_contrib + pc0);
  // kPartRows rows of the 6x6 block per thread (kPartThreads = 6 / kPartRows threads per block)
  for (int e = t; e < npart * kPartThreads; e += kLmGroupVisits) {
    const int pi = e / kPartThreads, h = e - pi * kPartThreads;
    const int c0 = (e == t ? pcA : gmem(P.part_cbegin)[pg0 + pi]) - pc0, c1 = (e == t ? pcB : gmem(P.part_cbegin)[pg0 + pi + 1]) - pc0;
    double acc[6 * kPartRows];
#pragma unroll
    for (int i = 0; i < 6 * kPartRows; ++i) acc[i] = 0.0;
#ifndef OKG_PART_UNROLL
#define OKG_PART_UNROLL 2
#endif
#define OKG_PRAGMA(x) _Pragma(#x)
#define OKG_UNROLL(n) OKG_PRAGMA(unroll n)
    OKG_UNROLL(OKG_PART_UNROLL)
    for (int c = c0; c < c1; ++c) {
      const int ab = staged ? sPC[c] : gPC[c], a = ab & 0xffff, b = ab >> 16;
      const double* zaP = sZ + kVisitZ * a + 3 * kPartRows * h;
      const double2* zb2 = reinterpret_cast<const double2*>(sZ + kVisitZ * b);
      double za[3 * kPartRows], zb[18];
      if (kPartRows == 2) {  // 16-byte aligned: 3 x 16-byte loads
        const double2* za2 = reinterpret_cast<const double2*>(zaP);
#pragma unroll
        for (int i = 0; i < 3; ++i) { const double2 v = za2[i]; za[2 * i] = v.x; za[2 * i + 1] = v.y; }
      } else {
#pragma unroll
        for (int i = 0; i < 3 * kPartRows; ++i) za[i] = zaP[i];
      }
#pragma unroll
      for (int i = 0; i < 9; ++i) { const double2 v = zb2[i]; zb[2 * i] = v.x; zb[2 * i + 1] = v.y; }
#pragma unroll
      for (int rr = 0; rr < kPartRows; ++rr)
#pragma unroll
        for (int q = 0; q < 6; ++q)
          acc[rr * 6 + q] += za[3 * rr] * zb[3 * q] + za[3 * rr + 1] * zb[3 * q + 1] + za[3 * rr + 2] * zb[3 * q + 2];
    }
    const auto out = gmemw(reinterpret_cast<double2*>(P.part_S + (size_t)(pg0 + pi) * 36 + 6 * kPartRows * h));
#pragma unroll
    for (int q = 0; q < 3 * kPartRows; ++q) out[q] = double2{acc[2 * q], acc[2 * q + 1]};
  }
  LCLK_TAIL(5)
}

template <int mode, bool EXT>
__global__ __launch_bounds__(kLmGroupVisits, OKG_LMV_OCC) void k_lm_visit(const DevProblem* __restrict__ Pp) {
  lmVisitGroup<mode, EXT>(*Pp, blockIdx.x);
}

// GN prep of a large batch: after the first iteration hardly any window needs it (Z is formed for
// the new mu by the linearisation; only retries and invalid steps raise mu), so a workgroup per
// landmark group would dispatch ~30 groups per window that all exit (2,048 S50 windows: 0.43 ms of
// dispatch per iteration). Instead a grid of resident workgroups loops over the windows and runs the
// groups of a selected window one after another (same body, same operations).
template <bool EXT>
__global__ __launch_bounds__(kLmGroupVisits, OKG_LMV_OCC) void k_lm_prep_windows(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  for (int w = blockIdx.x; w < P.n_win; w += gridDim.x) {
    const auto gst = gmem(P.st + w);
    const int sDone = gst->done, sNeed = gst->need_gn, sFail = gst->gn_failed;
    const double sZmu = gst->z_mu, sMu = gst->mu;
    if (sDone | !sNeed | sFail | (sZmu == sMu)) continue;  // lmVisitSelect (uniform)
    const int g0 = P.win_lmg_range[2 * w], g1 = P.win_lmg_range[2 * w + 1];
    for (int g = g0; g < g1; ++g) {
      lmVisitGroup<2, EXT>(P, g);
      __syncthreads();  // the next group's LDS writes wait for this group's readers
    }
  }
}

// Pose-extrinsics cross blocks of F^T F (variable extrinsics only): per (free state pose, variable
// camera) the sum over their observations of J_e^T J_p (6x6, rows = extrinsics), one thread each, in
// observation order. The landmark terms of the same block come from k_lm_visit's partial blocks.
__global__ __launch_bounds__(256) void k_pose_extr(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P.n_pe) return;
  const int w = P.pose_win[P.pe_pose[k]];
  if (!linSelect(P, w, lin_mode)) return;
  const WinState& st = P.st[w];
  const auto lin = gmem(P.obs_lin[st.lcur]);
  const int64_t S = P.obs_stride;
  const double* tw = P.pose[st.xcur] + 7 * (size_t)P.pe_pose[k];
  const double* ex = P.pose[st.xcur] + 7 * (size_t)P.pe_ext[k];
  double C_WS[9];
  qrot(qnormalize(Q{tw[3], tw[4], tw[5], tw[6]}), C_WS);
  double H[36];
#pragma unroll
  for (int i = 0; i < 36; ++i) H[i] = 0.0;
  for (int j = P.pe_obs_begin[k]; j < P.pe_obs_begin[k + 1]; ++j) {
    const int ob = P.pe_obs[j];
    const double* hp = P.lm[st.xcur] + 4 * (size_t)P.obs_lm[ob];
    const double w4 = hp[3];
    const double p3[3] = {hp[0] - tw[0] * w4, hp[1] - tw[1] * w4, hp[2] - tw[2] * w4};
    double A[6], Jp[12], Jl[6], Je[12];
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) A[kk] = lin[(2 + kk) * S + ob];
    obsJacobians(A, p3, w4, Jp, Jl);
    extrJacobian(A, C_WS, p3, w4, ex, Je);
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 6; ++b) H[a * 6 + b] += Je[a] * Jp[b] + Je[6 + a] * Jp[6 + b];
  }
  double* out = P.pe_H + 36 * (size_t)k;
#pragma unroll
  for (int i = 0; i < 36; ++i) out[i] = H[i];
}

// contribution helpers -------------------------------------------------------------------------
__device__ __forceinline__ const double* imuLin(const DevProblem& P, int lb, int f) {
  return P.imu_lin[lb] + (size_t)f * kImuLin;
}

__device__ __forceinline__ int sym30(int a, int b) {  // packed upper triangle of a 30x30
  if (a > b) { const int t = a; a = b; b = t; }
  return a * 30 - (a * (a - 1)) / 2 + (b - a);
}

// J^T J (30x30, packed) and J^T r of every IMU factor of the windows being linearised, one
// wavefront per factor with J staged in LDS; consumed by k_fgrad and both assembly kernels.
__device__ __forceinline__ void imuHessBlock(const DevProblem& P, int bid, int lin_mode) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int f = bid * 4 + wv;
  __shared__ double sJ[4][kImuLin];
  if (f >= P.n_fac) return;
  const int w = P.imu_win[f];
  if (!linSelect(P, w, lin_mode) || (P.imu_flags[f] & 2)) return;
  const auto L = gmem(P.imu_lin[P.st[w].lcur] + (size_t)f * kImuLin);
  double* J = sJ[wv];
  for (int e = lane; e < kImuLin; e += 64) J[e] = L[e];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double* H = P.imu_H + (size_t)f * kImuHess;
  for (int e = lane; e < kImuHess; e += 64) {
    double acc = 0.0;
    if (e < 465) {
      // row a of the packed upper triangle: start(a) = 30 a - a (a - 1) / 2 <= e < start(a + 1),
      // from the root of the quadratic and one exact integer correction each way (no per-lane
      // loop: lanes with different rows diverged over up to 30 iterations)
      int a = (int)((61.0f - sqrtf(3721.0f - 8.0f * (float)e)) * 0.5f);
      a = max(0, min(a, 29));
      if (30 * a - (a * (a - 1)) / 2 > e) --a;
      if (30 * (a + 1) - ((a + 1) * a) / 2 <= e) ++a;
      const int b = a + (e - (30 * a - (a * (a - 1)) / 2));
      for (int k = 0; k < 15; ++k) acc += J[15 + k * 30 + a] * J[15 + k * 30 + b];
    } else {
      const int a = e - 465;
      for (int k = 0; k < 15; ++k) acc += J[15 + k * 30 + a] * J[k];
    }
    H[e] = acc;
  }
}
__global__ __launch_bounds__(256) void k_imu_hess(const DevProblem* __restrict__ Pp, int lin_mode) {
  imuHessBlock(*Pp, (int)blockIdx.x, lin_mode);
}
// Few windows: the landmark groups' linearisation (k_lm_visit<1>) and the IMU factors' J^T J as one
// launch (trailing workgroups), one graph node fewer on a single window's latency chain.
// PREP: a group of a window whose step was not accepted runs the GN prep (k_lm_visit<2>) instead,
// which the next iteration would otherwise start with (one launch fewer per iteration). The prep
// selects exactly such windows (an accepted one gets Z for its new mu here), and nothing between
// this launch and the next assembly changes what it reads: the gradient test (k_gradnorm) passes
// over windows that were not accepted.
template <bool EXT, bool PREP>
__global__ __launch_bounds__(kLmGroupVisits, OKG_LMV_OCC) void k_lin_few(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int b = blockIdx.x;
  if (b >= P.n_lmg) return imuHessBlock(P, b - P.n_lmg, lin_mode);
  if (PREP && !gmem(P.st + gmem(P.lmg_info)[kLmgInfo * b + 2])->accepted) lmVisitGroup<2, EXT>(P, b);
  else lmVisitGroup<1, EXT>(P, b);
}
// Few windows run the GN prep inside the linearisation launch (k_lin_few<.., true>); env override
// OKVISGPU_LIN_PREP=0 (measurements). The runtime decides once per solve (P.lin_prep, set in
// okvisgpu_solve_begin before the initial launches and the graph capture), so the initial
// linearisation and the captured iterations always agree on where the prep runs.
bool lin_runs_prep(const DevProblem& P) {
  if (P.lin_prep >= 0) return P.lin_prep != 0;
  if (!fewWindows(P.n_win, P.cu_count)) return false;
  const char* e = std::getenv("OKVISGPU_LIN_PREP");
  return !(e && e[0] == '0');
}

// A 16-lane group per f-block (16 per 256-thread workgroup; a pose has ~10 contributions): lanes
// stride over the contribution list, then a fixed xor-tree reduction over the group (deterministic).
constexpr int kFgLanes = 16;
template <int PRE>
__global__ __launch_bounds__(256) void k_fgrad(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int fbRaw = blockIdx.x * (256 / kFgLanes) + (threadIdx.x / kFgLanes);
  const int lane = threadIdx.x & (kFgLanes - 1);
  const bool inRange = fbRaw < P.n_fblock;
  const int fb = inRange ? fbRaw : 0;
  // the f-block record, then the window state with this lane's first contribution, consumed (empty
  // asm) before the window test so that no load is sunk behind it
  const int w = gmem(P.fb_win)[fb], kind = gmem(P.fb_kind)[fb];
  const int c0 = gmem(P.fb_cbegin)[fb], c1 = gmem(P.fb_cbegin)[fb + 1];
  const auto gst = gmem(P.st + w);
  const int sDone = gst->done, sAcc = gst->accepted, lb = gst->lcur;
  const Contrib cFirst = gmem(P.fb_contrib)[min(c0 + lane, max(c1 - 1, c0))];
  asm volatile("" ::"v"(cFirst.type), "v"(cFirst.a), "v"(cFirst.b), "v"(lb));
  // (groups of other f-blocks share the wavefront: a group that is not selected contributes nothing
  // and stores nothing, but takes part in the shuffles)
  const bool live = inRange & (sDone == 0) & !(lin_mode == 1 && sAcc == 0);  // linSelect
  if (!__any(live)) return;
  const int n = kind == 0 ? 6 : 9;
  double g[9], hd[9];
#pragma unroll
  for (int c = 0; c < 9; ++c) { g[c] = 0.0; hd[c] = 0.0; }
  // Contributions in rounds of PRE per lane (k = c0 + lane + 16 j): the round's descriptors, then
  // the directly stored values (visit segments, IMU J^T J), then their sums in k order (the same
  // additions in the same order as one at a time, so the same bits). Few windows take two per round
  // (one dependent load round per two contributions on a single window's latency chain), batches
  // one (the registers of a second would halve the occupancy). Priors and edges form their
  // products where they are summed.
  auto loadDirect = [&](const Contrib& cb, double (&vg)[9], double (&vh)[9]) {
    const bool visit = cb.type == C_VISIT, imu = cb.type == C_IMU;
    const double* base = visit ? P.seg_hg + (size_t)cb.a * kSegHG : P.imu_H + (size_t)(imu ? cb.a : 0) * kImuHess;
#pragma unroll
    for (int c = 0; c < 9; ++c) {
      vg[c] = 0.0;
      vh[c] = 0.0;
      if (visit ? c < 6 : (imu && c < n)) {
        vg[c] = visit ? base[21 + c] : base[465 + cb.b + c];
        vh[c] = visit ? base[sym6(c, c)] : base[sym30(cb.b + c, cb.b + c)];
      }
    }
  };
  auto accumulate = [&](const Contrib& cb, const double (&vg)[9], const double (&vh)[9]) {
    if (cb.type == C_VISIT) {
#pragma unroll
      for (int c = 0; c < 6; ++c) { g[c] += vg[c]; hd[c] += vh[c]; }
    } else if (cb.type == C_IMU) {
#pragma unroll
      for (int c = 0; c < 9; ++c)
        if (c < n) {
          g[c] += vg[c];
          hd[c] += vh[c];
        }
    } else if (cb.type == C_PPRIOR) {
      const double* L = P.pp_lin[lb] + 42 * (size_t)cb.a;
      for (int c = 0; c < 6; ++c) {
        double sg = 0, sh = 0;
        for (int k2 = 0; k2 < 6; ++k2) {
          const double j = L[6 + k2 * 6 + c];
          sg += j * L[k2];
          sh += j * j;
        }
        g[c] += sg;
        hd[c] += sh;
      }
    } else if (cb.type == C_RELPOSE) {
      const double* L = P.rp_lin[lb] + kRelPoseLin * (size_t)cb.a;
      for (int c = 0; c < 6; ++c) {
        double sg = 0, sh = 0;
        for (int k2 = 0; k2 < 6; ++k2) {
          const double j = L[6 + k2 * 12 + cb.b + c];
          sg += j * L[k2];
          sh += j * j;
        }
        g[c] += sg;
        hd[c] += sh;
      }
    } else if (cb.type == C_SBPRIOR) {
      const double* L = P.sbp_lin[lb] + 90 * (size_t)cb.a;
      for (int c = 0; c < 9; ++c) {
        double sg = 0, sh = 0;
        for (int k2 = 0; k2 < 9; ++k2) {
          const double j = L[9 + k2 * 9 + c];
          sg += j * L[k2];
          sh += j * j;
        }
        g[c] += sg;
        hd[c] += sh;
      }
    }
  };
  if constexpr (PRE == 1) {
    for (int k = c0 + lane; live && k < c1; k += kFgLanes) {
      const Contrib cb = k == c0 + lane ? cFirst : P.fb_contrib[k];
      if (cb.type == C_VISIT) {
        const double* H = P.seg_hg + (size_t)cb.a * kSegHG;
        const double* gp = H + 21;
#pragma unroll
        for (int c = 0; c < 6; ++c) { g[c] += gp[c]; hd[c] += H[sym6(c, c)]; }
      } else if (cb.type == C_IMU) {
        const double* Hf = P.imu_H + (size_t)cb.a * kImuHess;
        for (int c = 0; c < n; ++c) {
          g[c] += Hf[465 + cb.b + c];
          hd[c] += Hf[sym30(cb.b + c, cb.b + c)];
        }
      } else {
        const double z[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        accumulate(cb, z, z);  // (priors and edges)
      }
    }
  } else
  for (int k = c0 + lane; live && k < c1; k += PRE * kFgLanes) {
    Contrib cb[PRE];
    double vg[PRE][9], vh[PRE][9];
#pragma unroll
    for (int j = 0; j < PRE; ++j) {
      const int kj = k + j * kFgLanes;
      cb[j] = j == 0 && k == c0 + lane ? cFirst : P.fb_contrib[kj < c1 ? kj : k];
      if (kj >= c1) cb[j].type = -1;
    }
#pragma unroll
    for (int j = 0; j < PRE; ++j) loadDirect(cb[j], vg[j], vh[j]);
#pragma unroll
    for (int j = 0; j < PRE; ++j)
      if (k + j * kFgLanes < c1) accumulate(cb[j], vg[j], vh[j]);
  }
#pragma unroll
  for (int c = 0; c < 9; ++c)
#pragma unroll
    for (int sh = kFgLanes / 2; sh > 0; sh >>= 1) {
      g[c] += __shfl_xor(g[c], sh, 64);
      hd[c] += __shfl_xor(hd[c], sh, 64);
    }
  if (lane != 0 || !live) return;
  const size_t base = (size_t)P.win_foff[w] + P.fb_off[fb];
  for (int c = 0; c < n; ++c) {
    P.gF[base + c] = g[c];
    P.hdF[base + c] = hd[c];
    if (lin_mode == 0) P.sF[base + c] = P.opt.jacobi_scaling ? 1.0 / (1.0 + sqrt(hd[c])) : 1.0;
  }
}

__device__ __forceinline__ bool gnSelect(const DevProblem& P, int w) {
  const WinState& s = P.st[w];
  return !s.done && s.need_gn && !s.gn_failed;
}

// Clears the structurally non-zero tiles of S (kZeroTiles consecutive tiles per workgroup; padded
// diagonal = 1). Since round 4 the factorisation works in W and never writes S, and the assembly
// overwrites its blocks every iteration, so S is cleared once per build (mode 2: every window,
// no state test) instead of every iteration. Modes 0 (windows about to assemble) and 1 (every
// window not done) are kept for the eager entry points' semantics.
constexpr int kZeroTiles = 4;  // (one per workgroup below kManyWindows windows: latency)
__global__ __launch_bounds__(256) void k_zero_S(const DevProblem* __restrict__ Pp, int per, int tail) {
  const DevProblem& P = *Pp;
  const auto ti3 = gmem(P.tile_items);
  for (int u = 0; u < per; ++u) {
    const int item = blockIdx.x * per + u;
    if (item >= P.n_tiles) return;
    const int w = ti3[3 * item], ti = ti3[3 * item + 1], tj = ti3[3 * item + 2];
    const auto gst = gmem(P.st + w);
    const int sDone = gst->done, sNeed = gst->need_gn | tail, sFail = gst->gn_failed & (tail ^ 1);
    const int fpad = gmem(P.win_fpad)[w], fdim = gmem(P.win_fdim)[w];
    const int g0 = gmem(P.win_sgap)[2 * w], g1 = g0 + gmem(P.win_sgap)[2 * w + 1];
    const int64_t soff = gmem(P.win_soff)[w];
    asm volatile("" ::"v"(fpad), "v"(fdim), "v"(g0), "v"(g1), "v"(soff));
    if (tail != 2 && ((sDone != 0) | (sNeed == 0) | (sFail != 0))) continue;  // uniform
    double* S = P.S + soff;
    for (int e = threadIdx.x; e < kTile * kTile / 2; e += 256) {
      const int rl = e >> 5, cl = 2 * (e & 31);
      const int r = ti * kTile + rl, c = tj * kTile + cl;
      const bool unit = r >= fdim || (r >= g0 && r < g1);  // padding and gap rows: identity
      const double2 v{(r == c && unit) ? 1.0 : 0.0, (r == c + 1 && unit) ? 1.0 : 0.0};
      *gmemw(reinterpret_cast<double2*>(S + (int64_t)r * fpad + c)) = v;
    }
  }
}

// Assembly of the reduced camera matrix S = s (J_f^T J_f - J_f^T J_l V^-1 J_l^T J_f) s + D^2 and of
// its rhs, one wavefront per block pair (SchurEliminator::Eliminate restated pair-major so that
// every entry is a fixed-order sum; no atomics).
//
// k_assemble_pp: pose-pose pairs. The wavefront is split into 8 groups of 6 lanes; lane
// (g, r) accumulates row r of the 6x6 block over the contributions c with (c - run start) % 8 ==
// g (fixed assignment), then a fixed 3-step tree over the groups sums the rows — deterministic
// without atomics. Each group loads a contribution's U (or H) once for its 6 lanes plus each lane
// its own Y row, and two steps of descriptors/operands are in flight per lane.
constexpr int kGroups = 8;

__device__ __forceinline__ void asmPairsHeavy(const DevProblem& P, int bid) {
  const int lane = threadIdx.x & 63;
  const int item = bid * 4 + (threadIdx.x >> 6);
  if (item >= P.n_asm_pp) return;
  const int k = __builtin_amdgcn_readfirstlane(gmem(P.asm_pp_items)[item]);  // (wave-uniform: scalar loads)
  if (k < 0) return;
  // the pair record in one round of loads; then the window state, the first round of descriptors
  // and the block offsets in the next, all consumed (empty asm) before the window test, so no load
  // is sunk behind it
  const int w = gmem(P.pair_win)[k];
  const int cb = gmem(P.pair_cbegin)[k], ce = gmem(P.pair_cbegin)[k + 1];
  const int2 runs = gmem(reinterpret_cast<const int2*>(P.pair_runs))[k];
  const int pb = runs.x, ob = runs.y;
  const int fi = gmem(P.pair_fi)[k], fj = gmem(P.pair_fj)[k];
  const auto pc = gmem(P.pair_contrib);
  const auto gst = gmem(P.st + w);
  const int sDone = gst->done, sNeed = gst->need_gn, sFail = gst->gn_failed, lb = gst->lcur;
  const double sMu = gst->mu;
  const int myc0 = min(cb + lane, max(pb - 1, cb));
  const int da0 = pc[myc0].a, db0 = pc[myc0].b;
  const int foff = gmem(P.win_foff)[w], offi = gmem(P.fb_off)[fi], offj = gmem(P.fb_off)[fj];
  asm volatile("" ::"v"(da0), "v"(db0), "v"(foff), "v"(offi), "v"(offj), "v"(cb), "v"(ce), "v"(lb), "v"(sMu));
  if ((sDone != 0) | (sNeed == 0) | (sFail != 0)) return;
  const int g = lane / 6, r = lane - 6 * (lane / 6);
  const bool inGroup = g < kGroups;
  const auto vhg = gmem(P.seg_hg);
  const auto suz = gmem(P.seg_uz);
  double H[6], Sc[6], uz = 0.0;
#pragma unroll
  for (int q = 0; q < 6; ++q) { H[q] = 0.0; Sc[q] = 0.0; }
  const int g0 = inGroup ? g : 1 << 29;  // lanes 48..63 idle (factor-block loop)
  // Descriptors: one coalesced load of 64 per round (lane L holds c = base + L), handed to the
  // groups with __shfl, so each step waits on a single round of operand loads.
  // visits (diagonal pairs): row r of H_v, and (U_v z_l)_r
  for (int base = cb; base < pb; base += 64) {
    const int myc = min(base + lane, pb - 1);
    const int da = base == cb ? da0 : pc[myc].a, db = base == cb ? db0 : pc[myc].b;
    const int nstep = min(64, pb - base);
    for (int st = 0; st < nstep; st += kGroups) {
      const int k0 = st + g;
      const int a0 = __shfl(da, k0 & 63, 64), b0 = __shfl(db, k0 & 63, 64);
      const bool v0 = inGroup && k0 < nstep;
      const auto H0 = vhg + (size_t)a0 * kSegHG;
      double h0[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) h0[q] = H0[sym6(r, q)];
      const double z0 = suz[(size_t)a0 * kSegUz + r];
#pragma unroll
      for (int q = 0; q < 6; ++q) H[q] += v0 ? h0[q] : 0.0;
      uz += v0 ? z0 : 0.0;
    }
  }
  // partial Schur blocks of the landmark groups: row r of sum Z_a Z_b^T (= Y_a U_b^T)
  // (two of the lane's contributions per round (80 VGPRs): descriptors, then rows, each round in flight
  // together; clamped indices, masked sums, same order as one by one)
  const auto ps = gmem(P.part_S);
  for (int c = pb + g0; c < ob; c += 2 * kGroups) {
    int ai[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) ai[u] = pc[min(c + u * kGroups, ob - 1)].a;
    double2 v[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const auto R2 = reinterpret_cast<gptr<double2>>(ps + (size_t)ai[u] * 36 + 6 * r);
#pragma unroll
      for (int q = 0; q < 3; ++q) v[u][q] = R2[q];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool ok = c + u * kGroups < ob;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        Sc[2 * q] += ok ? v[u][q].x : 0.0;
        Sc[2 * q + 1] += ok ? v[u][q].y : 0.0;
      }
    }
  }
  // factor blocks (IMU, relative pose, pose prior): row r of J_i^T J_j
  for (int c = ob + g0; c < ce; c += kGroups) {
    const Contrib C = pc[c];
    if (C.type == C_IMU) {
      const auto Hf = gmem(P.imu_H + (size_t)C.a * kImuHess);
#pragma unroll
      for (int q = 0; q < 6; ++q) H[q] += Hf[sym30(C.b + r, C.c + q)];
    } else if (C.type == C_RELPOSE) {
      const double* L = P.rp_lin[lb] + kRelPoseLin * (size_t)C.a + 6;
      for (int k2 = 0; k2 < 6; ++k2) {
        const double jr = L[k2 * 12 + C.b + r];
#pragma unroll
        for (int q = 0; q < 6; ++q) H[q] += jr * L[k2 * 12 + C.c + q];
      }
    } else if (C.type == C_PEXT) {  // row r of sum J_e^T J_p (extrinsics row block, pose column block)
      const auto Hx = gmem(P.pe_H + 36 * (size_t)C.a + 6 * r);
#pragma unroll
      for (int q = 0; q < 6; ++q) H[q] += Hx[q];
    } else {  // C_PPRIOR
      const double* L = P.pp_lin[lb] + 42 * (size_t)C.a + 6;
      for (int k2 = 0; k2 < 6; ++k2) {
        const double jr = L[k2 * 6 + r];
#pragma unroll
        for (int q = 0; q < 6; ++q) H[q] += jr * L[k2 * 6 + q];
      }
    }
  }
  // fixed tree over the groups: g += g + 4, g += g + 2, g += g + 1
#pragma unroll
  for (int d = 4; d >= 1; d >>= 1) {
    const int src = min(lane + 6 * d, 63);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      H[q] += __shfl(H[q], src, 64);
      Sc[q] += __shfl(Sc[q], src, 64);
    }
    uz += __shfl(uz, src, 64);
  }
  if (lane >= 6) return;
  const bool diag = fi == fj;
  const double si = gmem(P.sF)[(size_t)foff + offi + r];
  const auto Srow = gmemw(P.S + gmem(P.win_soff)[w] + (int64_t)(offi + r) * gmem(P.win_fpad)[w] + offj);
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const double sj = gmem(P.sF)[(size_t)foff + offj + q];
    double val = si * sj * H[q] - Sc[q];
    if (diag && r == q) {
      const size_t idx = (size_t)foff + offi + r;
      const double dg = sqrt(fmin(fmax(si * si * gmem(P.hdF)[idx], P.opt.min_lm_diagonal), P.opt.max_lm_diagonal));
      gmemw(P.diagF)[idx] = dg;
      const double d = dg * sqrt(sMu);
      val += d * d;
    }
    Srow[q] = val;
  }
  if (diag) {
    // Schur rhs: s_i g_i - sum_visits U_v z_l
    const size_t idx = (size_t)foff + offi + r;
    gmemw(P.rhsF)[idx] = gmem(P.sF)[idx] * gmem(P.gF)[idx] - uz;
  }
}
__global__ __launch_bounds__(256, 6) void k_assemble_pp(const DevProblem* __restrict__ Pp) { asmPairsHeavy(*Pp, (int)blockIdx.x); }

// k_assemble_pp_light: off-diagonal pose-pose pairs with few contributions (no visits; partial
// blocks, then factor blocks; <= kAsmLightMax). A 16-lane quarter of a wavefront per pair: 2 groups
// of 6 lanes (one per row) take alternate contributions, one fixed combining step. Same sums as
// k_assemble_pp with kGroups = 2.
constexpr int kPplLanes = 16, kPplGroups = 2;
__device__ __forceinline__ void asmPairsLight(const DevProblem& P, int bid) {
  const int lane = threadIdx.x & 63, sub = threadIdx.x & (kPplLanes - 1);
  const int item = (bid * 256 + threadIdx.x) / kPplLanes;
  const int kRaw = item < P.n_asm_ppl ? gmem(P.asm_ppl_items)[item] : -1;
  const bool has = kRaw >= 0;
  const int k = has ? kRaw : 0;
  // the pair record, then the window state and offsets, consumed before any test (no loads sunk)
  const int w = gmem(P.pair_win)[k];
  const int ce = gmem(P.pair_cbegin)[k + 1];
  const int2 runs = gmem(reinterpret_cast<const int2*>(P.pair_runs))[k];
  const int pb = runs.x, ob = runs.y;
  const int fi = gmem(P.pair_fi)[k], fj = gmem(P.pair_fj)[k];
  const auto pc = gmem(P.pair_contrib);
  const auto gst = gmem(P.st + w);
  const int sDone = gst->done, sNeed = gst->need_gn, sFail = gst->gn_failed, lb = gst->lcur;
  const int g = sub / 6, r = sub - 6 * (sub / 6);
  // the group's first factor-block descriptor and its first round of partial-block descriptors,
  // loaded with the window state (before the test: one level of dependent loads fewer per pair)
  const int cFirst = min(ob + g, max(ce - 1, pb));
  const Contrib C0 = pc[cFirst];
  int ai0[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) ai0[u] = pc[max(min(pb + g + u * kPplGroups, ob - 1), 0)].a;
  const int foff = gmem(P.win_foff)[w], offi = gmem(P.fb_off)[fi], offj = gmem(P.fb_off)[fj];
  asm volatile("" ::"v"(C0.type), "v"(C0.a), "v"(C0.b), "v"(C0.c), "v"(foff), "v"(offi), "v"(offj), "v"(lb),
               "v"(ai0[0]), "v"(ai0[1]), "v"(ai0[2]), "v"(ai0[3]));
  const bool live = has & (sDone == 0) & (sNeed != 0) & (sFail == 0);  // gnSelect
  if (!__any(live)) return;
  const int g0 = (live && g < kPplGroups) ? g : 1 << 29;  // lanes 12..15 of a quarter idle
  double H[6], Sc[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) { H[q] = 0.0; Sc[q] = 0.0; }
  // partial blocks, four of the lane's contributions per round: their descriptors, then their rows,
  // each round of loads in flight together (clamped indices, masked sums; same order as one by one)
  const auto ps = gmem(P.part_S);
  for (int c = pb + g0; c < ob; c += 4 * kPplGroups) {
    int ai[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) ai[u] = c == pb + g ? ai0[u] : pc[min(c + u * kPplGroups, ob - 1)].a;
    double2 v[4][3];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const auto R2 = reinterpret_cast<gptr<double2>>(ps + (size_t)ai[u] * 36 + 6 * r);
#pragma unroll
      for (int q = 0; q < 3; ++q) v[u][q] = R2[q];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = c + u * kPplGroups < ob;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        Sc[2 * q] += ok ? v[u][q].x : 0.0;
        Sc[2 * q + 1] += ok ? v[u][q].y : 0.0;
      }
    }
  }
  for (int c = ob + g0; c < ce; c += kPplGroups) {
    const Contrib C = c == cFirst ? C0 : pc[c];
    if (C.type == C_IMU) {
      const auto Hf = gmem(P.imu_H + (size_t)C.a * kImuHess);
#pragma unroll
      for (int q = 0; q < 6; ++q) H[q] += Hf[sym30(C.b + r, C.c + q)];
    } else if (C.type == C_RELPOSE) {
      const double* L = P.rp_lin[lb] + kRelPoseLin * (size_t)C.a + 6;
      for (int k2 = 0; k2 < 6; ++k2) {
        const double jr = L[k2 * 12 + C.b + r];
#pragma unroll
        for (int q = 0; q < 6; ++q) H[q] += jr * L[k2 * 12 + C.c + q];
      }
    } else if (C.type == C_PEXT) {
      const auto Hx = gmem(P.pe_H + 36 * (size_t)C.a + 6 * r);
#pragma unroll
      for (int q = 0; q < 6; ++q) H[q] += Hx[q];
    } else {  // C_PPRIOR
      const double* L = P.pp_lin[lb] + 42 * (size_t)C.a + 6;
      for (int k2 = 0; k2 < 6; ++k2) {
        const double jr = L[k2 * 6 + r];
#pragma unroll
        for (int q = 0; q < 6; ++q) H[q] += jr * L[k2 * 6 + q];
      }
    }
  }
  // group 0 += group 1
  const int src = min(lane + 6, 63);
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    H[q] += __shfl(H[q], src, 64);
    Sc[q] += __shfl(Sc[q], src, 64);
  }
  if (sub >= 6 || !live) return;
  const double si = gmem(P.sF)[(size_t)foff + offi + r];
  const auto Srow = gmemw(P.S + gmem(P.win_soff)[w] + (int64_t)(offi + r) * gmem(P.win_fpad)[w] + offj);
#pragma unroll
  for (int q = 0; q < 6; ++q) Srow[q] = si * gmem(P.sF)[(size_t)foff + offj + q] * H[q] - Sc[q];
}
__global__ __launch_bounds__(256) void k_assemble_pp_light(const DevProblem* __restrict__ Pp) { asmPairsLight(*Pp, (int)blockIdx.x); }

// k_assemble_sb: pairs with a speed/bias block (6x9, 9x9): few contributions (IMU factors,
// speed/bias priors), one entry per lane. The first kSbPre contribution descriptors are loaded with
// the pair record (before the window test), and the IMU entries of a pair's contributions are
// loaded together before they are summed in contribution order (the same sums): a pair costs one
// dependent global load per level instead of two per contribution.
constexpr int kSbPre = 4;
__device__ __forceinline__ double sbPriorTerm(const DevProblem& P, const Contrib& C, int lb, int r, int q) {
  if (C.type == C_SBPRIOR) {
    const double* L = P.sbp_lin[lb] + 90 * (size_t)C.a + 9;
    double s2 = 0;
    for (int k2 = 0; k2 < 9; ++k2) s2 += L[k2 * 9 + r] * L[k2 * 9 + q];
    return s2;
  }
  const double* L = P.pp_lin[lb] + 42 * (size_t)C.a + 6;  // C_PPRIOR
  double s2 = 0;
  for (int k2 = 0; k2 < 6; ++k2) s2 += L[k2 * 6 + r] * L[k2 * 6 + q];
  return s2;
}
__device__ __forceinline__ void asmPairsSb(const DevProblem& P, int bid) {
  const int lane = threadIdx.x & 63;
  const int item = bid * 4 + (threadIdx.x >> 6);
  if (item >= P.n_asm_sb) return;
  // (wave-uniform from here: the pair record and its descriptors go to scalar registers)
  const int k = __builtin_amdgcn_readfirstlane(gmem(P.asm_sb_items)[item]);
  // the pair record, then the window state, the block offsets and the first contribution
  // descriptors, consumed (empty asm) before the window test so that no load is sunk behind it
  const int w = gmem(P.pair_win)[k], fi = gmem(P.pair_fi)[k], fj = gmem(P.pair_fj)[k];
  const int cb = gmem(P.pair_cbegin)[k], ce = gmem(P.pair_cbegin)[k + 1];
  const auto gst = gmem(P.st + w);
  const int sDone = gst->done, sNeed = gst->need_gn, sFail = gst->gn_failed, lb = gst->lcur;
  const double sMu = gst->mu;
  const int ki = gmem(P.fb_kind)[fi], kj = gmem(P.fb_kind)[fj];
  const int offi = gmem(P.fb_off)[fi], offj = gmem(P.fb_off)[fj];
  const int foff = gmem(P.win_foff)[w], ld = gmem(P.win_fpad)[w];
  const int64_t soff = gmem(P.win_soff)[w];
  const int nc = ce - cb;
  Contrib Cs[kSbPre];
#pragma unroll
  for (int u = 0; u < kSbPre; ++u) Cs[u] = gmem(P.pair_contrib)[cb + min(u, max(nc - 1, 0))];
  asm volatile("" ::"v"(ki), "v"(kj), "v"(offi), "v"(offj), "v"(foff), "v"(ld), "v"(soff), "v"(cb), "v"(ce),
               "v"(lb), "v"(sMu), "v"(Cs[0].a), "v"(Cs[kSbPre - 1].a));
  if ((sDone != 0) | (sNeed == 0) | (sFail != 0)) return;  // gnSelect
  const int ni = ki == 0 ? 6 : 9, nj = kj == 0 ? 6 : 9;
  const bool diag = fi == fj;
  const auto S = gmemw(P.S + soff);
  const double smu = sqrt(sMu);
  const auto imuH = gmem(P.imu_H);
  for (int e = lane; e < ni * nj; e += 64) {
    const int r = e / nj, q = e - r * nj;
    const double si = gmem(P.sF)[(size_t)foff + offi + r], sj = gmem(P.sF)[(size_t)foff + offj + q];
    double H = 0.0;
    if (nc <= kSbPre) {
      double v[kSbPre];
#pragma unroll
      for (int u = 0; u < kSbPre; ++u) {
        const Contrib& C = Cs[u];
        v[u] = C.type == C_IMU ? imuH[(size_t)C.a * kImuHess + sym30(C.b + r, C.c + q)] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kSbPre; ++u)
        if (u < nc) H += Cs[u].type == C_IMU ? v[u] : sbPriorTerm(P, Cs[u], lb, r, q);
    } else {
      for (int c = cb; c < ce; ++c) {
        const Contrib C = P.pair_contrib[c];
        H += C.type == C_IMU ? P.imu_H[(size_t)C.a * kImuHess + sym30(C.b + r, C.c + q)] : sbPriorTerm(P, C, lb, r, q);
      }
    }
    double val = si * sj * H;
    if (diag && r == q) {
      const size_t idx = (size_t)foff + offi + r;
      const double dg = sqrt(fmin(fmax(si * si * gmem(P.hdF)[idx], P.opt.min_lm_diagonal), P.opt.max_lm_diagonal));
      gmemw(P.diagF)[idx] = dg;
      const double d = dg * smu;
      val += d * d;
    }
    S[(int64_t)(offi + r) * ld + offj + q] = val;
  }
  if (diag && lane < ni) {
    const size_t idx = (size_t)foff + offi + lane;
    gmemw(P.rhsF)[idx] = gmem(P.sF)[idx] * gmem(P.gF)[idx];
  }
}
__global__ __launch_bounds__(256) void k_assemble_sb(const DevProblem* __restrict__ Pp) { asmPairsSb(*Pp, (int)blockIdx.x); }

// ------------------------------------------------------------------------------------ launchers
void launch_lm_visit(const DevProblem& P, int mode, hipStream_t s) {
  if (P.n_lmg <= 0) return;
  const dim3 g(P.n_lmg), b(kLmGroupVisits);
  if (mode == 2 && P.n_win >= kManyWindows) {  // window loop over resident workgroups
    const dim3 gw(std::min(P.n_win, P.cu_count * OKG_LMV_OCC));
    if (P.n_xvisit > 0) hipLaunchKernelGGL((k_lm_prep_windows<true>), gw, b, 0, s, P.self);
    else hipLaunchKernelGGL((k_lm_prep_windows<false>), gw, b, 0, s, P.self);
    return;
  }
  if (P.n_xvisit > 0) {
    if (mode == 0) hipLaunchKernelGGL((k_lm_visit<0, true>), g, b, 0, s, P.self);
    else if (mode == 1) hipLaunchKernelGGL((k_lm_visit<1, true>), g, b, 0, s, P.self);
    else hipLaunchKernelGGL((k_lm_visit<2, true>), g, b, 0, s, P.self);
  } else {
    if (mode == 0) hipLaunchKernelGGL((k_lm_visit<0, false>), g, b, 0, s, P.self);
    else if (mode == 1) hipLaunchKernelGGL((k_lm_visit<1, false>), g, b, 0, s, P.self);
    else hipLaunchKernelGGL((k_lm_visit<2, false>), g, b, 0, s, P.self);
  }
}
void launch_assemble_pp(const DevProblem& P, hipStream_t s) {
  if (P.n_asm_pp > 0) hipLaunchKernelGGL(k_assemble_pp, dim3((P.n_asm_pp + 3) / 4), dim3(256), 0, s, P.self);
  if (P.n_asm_ppl > 0)
    hipLaunchKernelGGL(k_assemble_pp_light, dim3((P.n_asm_ppl + 256 / kPplLanes - 1) / (256 / kPplLanes)), dim3(256), 0,
                       s, P.self);
}
void launch_assemble_sb(const DevProblem& P, hipStream_t s) {
  if (P.n_asm_sb > 0) hipLaunchKernelGGL(k_assemble_sb, dim3((P.n_asm_sb + 3) / 4), dim3(256), 0, s, P.self);
}
void launch_lm_blocks(const DevProblem& P, int lin_mode, hipStream_t s) {
  launch_lm_visit(P, lin_mode, s);
  if (P.n_pe > 0) hipLaunchKernelGGL(k_pose_extr, dim3((P.n_pe + 255) / 256), dim3(256), 0, s, P.self, lin_mode);
}
void launch_fgrad(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (P.n_fblock <= 0) return;
  const dim3 g((P.n_fblock + 256 / kFgLanes - 1) / (256 / kFgLanes));
  if (fewWindows(P.n_win, P.cu_count)) hipLaunchKernelGGL(k_fgrad<2>, g, dim3(256), 0, s, P.self, lin_mode);
  else hipLaunchKernelGGL(k_fgrad<1>, g, dim3(256), 0, s, P.self, lin_mode);
}
void launch_imu_hess(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (P.n_fac > 0) hipLaunchKernelGGL(k_imu_hess, dim3((P.n_fac + 3) / 4), dim3(256), 0, s, P.self, lin_mode);
}
void launch_linearization_blocks(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (lin_mode == 1 && fewWindows(P.n_win, P.cu_count)) {
    const int nb = P.n_lmg + (P.n_fac + 3) / 4;
    if (nb > 0) {
      const bool prep = lin_runs_prep(P);
      if (P.n_xvisit > 0) {
        if (prep) hipLaunchKernelGGL((k_lin_few<true, true>), dim3(nb), dim3(kLmGroupVisits), 0, s, P.self, lin_mode);
        else hipLaunchKernelGGL((k_lin_few<true, false>), dim3(nb), dim3(kLmGroupVisits), 0, s, P.self, lin_mode);
      } else {
        if (prep) hipLaunchKernelGGL((k_lin_few<false, true>), dim3(nb), dim3(kLmGroupVisits), 0, s, P.self, lin_mode);
        else hipLaunchKernelGGL((k_lin_few<false, false>), dim3(nb), dim3(kLmGroupVisits), 0, s, P.self, lin_mode);
      }
    }
    if (P.n_pe > 0) hipLaunchKernelGGL(k_pose_extr, dim3((P.n_pe + 255) / 256), dim3(256), 0, s, P.self, lin_mode);
  } else {
    launch_lm_blocks(P, lin_mode, s);
    launch_imu_hess(P, lin_mode, s);
  }
  launch_fgrad(P, lin_mode, s);
}
void launch_lm_prep(const DevProblem& P, hipStream_t s) { launch_lm_visit(P, 2, s); }
void launch_zero_S(const DevProblem& P, hipStream_t s, int tail) {
  const int per = P.n_win >= kManyWindows ? kZeroTiles : 1;
  if (P.n_tiles > 0) hipLaunchKernelGGL(k_zero_S, dim3((P.n_tiles + per - 1) / per), dim3(256), 0, s, P.self, per, tail);
}
// Few windows: the three assembly kernels as one launch (block ranges; the kernels are independent:
// disjoint pairs of S), two graph nodes fewer on a single window's latency chain.
// With grad (the captured few-window iteration, runtime.cpp launchIteration): one more block per
// window runs the gradient tolerance test of the previous iteration's linearisation (gradnorm.hpp,
// 256 threads as everywhere): it reads the parameters, the gradient and the window state, which
// the assembly does not write, and the assembly needs no result of it (a window it ends is
// skipped from the Cholesky on), so the two share a launch instead of following each other.
__global__ __launch_bounds__(256) void k_assemble_few(const DevProblem* __restrict__ Pp, int nHeavy, int nLight, int nAsm) {
  const DevProblem& P = *Pp;
  const int b = blockIdx.x;
  if (b < nHeavy) asmPairsHeavy(P, b);
  else if (b < nHeavy + nLight) asmPairsLight(P, b - nHeavy);
  else if (b < nAsm) asmPairsSb(P, b - nHeavy - nLight);
  else gradnormWindow<256>(P, b - nAsm, 1);
}
static void launchAssembleFew(const DevProblem& P, hipStream_t s, bool grad) {
  const int nH = (P.n_asm_pp + 3) / 4, nL = (P.n_asm_ppl + 256 / kPplLanes - 1) / (256 / kPplLanes),
            nS = (P.n_asm_sb + 3) / 4, nA = nH + nL + nS, nG = grad ? P.n_win : 0;
  if (nA + nG > 0) hipLaunchKernelGGL(k_assemble_few, dim3(nA + nG), dim3(256), 0, s, P.self, nH, nL, nA);
}
void launch_assemble(const DevProblem& P, hipStream_t s) {
  if (fewWindows(P.n_win, P.cu_count)) {
    launchAssembleFew(P, s, false);
    return;
  }
  launch_assemble_pp(P, s);
  launch_assemble_sb(P, s);
}
void launch_assemble_gradnorm_few(const DevProblem& P, hipStream_t s) { launchAssembleFew(P, s, true); }
void launch_gn_reduce(const DevProblem& P, hipStream_t s) {
  launch_lm_prep(P, s);
  launch_assemble(P, s);
}
void launch_gn_backsub(const DevProblem& P, hipStream_t s) {
  launch_lm_backsub(P, s);  // (the f-blocks' GN vectors are written by the Cholesky's back substitution)
}

}  // namespace okg
