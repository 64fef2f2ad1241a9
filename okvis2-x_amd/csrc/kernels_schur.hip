// kernels_schur.hip — landmark elimination (DENSE_SCHUR) for gfx950, FP64.
//
// The reduced ("camera") system of a window is formed exactly as Ceres' SchurEliminator does for
// e-blocks = landmarks, but organised for the GPU:
//   k_visit_lin   one thread per (landmark, pose) visit: W = J_p^T J_l, H_pp = J_p^T J_p,
//                 g_p = J_p^T r and the visit's share of V = J_l^T J_l, g_l = J_l^T r from the
//                 stored linearisation (unscaled; the Jacobi scaling is applied by consumers).
//   k_lm_lin      one thread per landmark: V, g_l over its visits; iteration 0: Jacobi scaling.
//   k_imu_hess    one wavefront per IMU factor: J^T J (packed) and J^T r of its 15x30 Jacobian.
//   k_fgrad       one wavefront per f-block (pose / speed-bias): unscaled gradient and
//                 diag(H_ff), and at iteration 0 the Jacobi scaling 1/(1+sqrt(diag)).
//   k_lm_prep     one thread per landmark: 3x3 LLT of s V s + D^2 (InvertPSDMatrix), L^-1, L^-1 s g.
//   k_visit_prep  one thread per visit: Z = s_p W s_l L^-T and U z (Y_a U_b^T = Z_a Z_b^T).
//   k_zero_S      clears the structurally non-zero tiles of S (padded diagonal = 1).
//   k_assemble_pp one wavefront per pose-pose block pair (i >= j): 8 groups of 6 lanes (one per
//                 row) sum fixed, interleaved subsets of the pair's contributions — visits,
//                 landmark pairs (the Y_i U_j^T Schur terms), IMU / prior J^T J sub-blocks — and
//                 a fixed tree combines the groups, so the sum is deterministic without atomics;
//                 diagonal pairs also emit the Schur rhs and the dogleg diagonal.
//   k_assemble_sb one wavefront per block pair involving a speed/bias block (one entry per lane).
//   k_lm_backsub  one thread per landmark: y_l = V^-1 (g_l - W^T y_f).
//   k_gn_finalize Gauss-Newton step / dogleg gradient in the dogleg-scaled space.
#include <cfloat>

#include "device_problem.hpp"
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

__device__ __forceinline__ bool linSelect(const DevProblem& P, int w, int lin_mode) {
  const WinState& s = P.st[w];
  if (s.done) return false;
  if (lin_mode == 1 && !s.accepted) return false;
  return true;
}

// One thread per (landmark, pose) visit: the 1-2 reprojection residuals of the visit give the
// pose-landmark blocks W = J_p^T J_l, H = J_p^T J_p, g = J_p^T r and the visit's share of the
// landmark block (V, J_l^T r): one 54-double AoS record per visit (16-byte stores, merged in L2).
__global__ __launch_bounds__(256) void k_visit_lin(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= P.n_visit) return;
  const int l = P.visit_lm[v];
  const int w = P.lm_win[l];
  if (!linSelect(P, w, lin_mode)) return;
  double o[kVisitLin];  // W 0..17 | H 18..38 | g 39..44 | V 45..50 | g_l 51..53
#pragma unroll
  for (int i = 0; i < kVisitLin; ++i) o[i] = 0.0;
  const bool lfree = P.lm_free[l] != 0;
  const bool pf = P.pose_f[P.visit_pose[v]] >= 0;
  const WinState& st = P.st[w];
  const auto lin = gmem(P.obs_lin[st.lcur]);
  const int64_t S = P.obs_stride;
  // linearisation point of lin[lcur]: params X[xcur]
  const double* hp = P.lm[st.xcur] + 4 * (size_t)l;
  const double* tw = P.pose[st.xcur] + 7 * (size_t)P.visit_pose[v];
  const double w4 = hp[3];
  const double p3[3] = {hp[0] - tw[0] * w4, hp[1] - tw[1] * w4, hp[2] - tw[2] * w4};
  for (int ob = P.visit_obs_begin[v]; ob < P.visit_obs_begin[v + 1]; ++ob) {
    if (P.obs_flags[ob] & 2) continue;
    double r[2], A[6], Jp[12], Jl[6];
    r[0] = lin[0 * S + ob];
    r[1] = lin[1 * S + ob];
#pragma unroll
    for (int k = 0; k < 6; ++k) A[k] = lin[(2 + k) * S + ob];
    obsJacobians(A, p3, w4, Jp, Jl);
    if (lfree) {
#pragma unroll
      for (int a2 = 0; a2 < 3; ++a2) {
        o[51 + a2] += Jl[a2] * r[0] + Jl[3 + a2] * r[1];
#pragma unroll
        for (int b2 = a2; b2 < 3; ++b2) o[45 + sym3(a2, b2)] += Jl[a2] * Jl[b2] + Jl[3 + a2] * Jl[3 + b2];
      }
    }
    if (pf) {
#pragma unroll
      for (int a2 = 0; a2 < 6; ++a2) {
        o[39 + a2] += Jp[a2] * r[0] + Jp[6 + a2] * r[1];
#pragma unroll
        for (int b2 = a2; b2 < 6; ++b2) o[18 + sym6(a2, b2)] += Jp[a2] * Jp[b2] + Jp[6 + a2] * Jp[6 + b2];
        if (lfree)
#pragma unroll
          for (int b2 = 0; b2 < 3; ++b2) o[a2 * 3 + b2] += Jp[a2] * Jl[b2] + Jp[6 + a2] * Jl[3 + b2];
      }
    }
  }
  double2* out = reinterpret_cast<double2*>(P.visit_lin + (size_t)v * kVisitLin);
#pragma unroll
  for (int i = 0; i < kVisitLin / 2; ++i) out[i] = double2{o[2 * i], o[2 * i + 1]};
}

// One thread per landmark: V = sum over visits, J_l^T r, and (iteration 0) the landmark's Jacobi
// scaling 1 / (1 + sqrt(diag(V)))  (TrustRegionMinimizer / ScaledJacobian).
__global__ __launch_bounds__(256) void k_lm_lin(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= P.n_lm || !P.lm_free[l]) return;
  const int w = P.lm_win[l];
  if (!linSelect(P, w, lin_mode)) return;
  double V[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
  for (int v = P.lm_visit_begin[l]; v < P.lm_visit_begin[l + 1]; ++v) {
    const double* src = P.visit_lin + (size_t)v * kVisitLin + 45;
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] += src[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) g[i] += src[6 + i];
  }
  for (int i = 0; i < 6; ++i) P.lm_V[6 * (size_t)l + i] = V[i];
  for (int i = 0; i < 3; ++i) P.lm_g[3 * (size_t)l + i] = g[i];
  if (lin_mode == 0)  // Jacobi scaling fixed at iteration 0 (TrustRegionMinimizer)
    for (int a = 0; a < 3; ++a)
      P.sL[3 * (size_t)l + a] = P.opt.jacobi_scaling ? 1.0 / (1.0 + sqrt(V[sym3(a, a)])) : 1.0;
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
__global__ __launch_bounds__(256) void k_imu_hess(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int f = blockIdx.x * 4 + wv;
  __shared__ double sJ[4][kImuLin];
  if (f >= P.n_imu) return;
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
      int a = 0, rem = e;
      while (rem >= 30 - a) { rem -= 30 - a; ++a; }
      const int b = a + rem;
      for (int k = 0; k < 15; ++k) acc += J[15 + k * 30 + a] * J[15 + k * 30 + b];
    } else {
      const int a = e - 465;
      for (int k = 0; k < 15; ++k) acc += J[15 + k * 30 + a] * J[k];
    }
    H[e] = acc;
  }
}

// One wavefront per f-block: lanes stride over the contribution list, then a fixed xor-tree
// reduction (deterministic).
__global__ __launch_bounds__(64) void k_fgrad(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int fb = blockIdx.x;
  if (fb >= P.n_fblock) return;
  const int w = P.fb_win[fb];
  if (!linSelect(P, w, lin_mode)) return;
  const int lane = threadIdx.x;
  const int lb = P.st[w].lcur;
  const int n = P.fb_kind[fb] == 0 ? 6 : 9;
  double g[9], hd[9];
#pragma unroll
  for (int c = 0; c < 9; ++c) { g[c] = 0.0; hd[c] = 0.0; }
  for (int k = P.fb_cbegin[fb] + lane; k < P.fb_cbegin[fb + 1]; k += 64) {
    const Contrib cb = P.fb_contrib[k];
    if (cb.type == C_VISIT) {
      const double* H = P.visit_lin + (size_t)cb.a * kVisitLin + 18;
      const double* gp = H + 21;
#pragma unroll
      for (int c = 0; c < 6; ++c) { g[c] += gp[c]; hd[c] += H[sym6(c, c)]; }
    } else if (cb.type == C_IMU) {
      const double* Hf = P.imu_H + (size_t)cb.a * kImuHess;
      for (int c = 0; c < n; ++c) {
        g[c] += Hf[465 + cb.b + c];
        hd[c] += Hf[sym30(cb.b + c, cb.b + c)];
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
  }
#pragma unroll
  for (int c = 0; c < 9; ++c)
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
      g[c] += __shfl_xor(g[c], sh, 64);
      hd[c] += __shfl_xor(hd[c], sh, 64);
    }
  if (lane != 0) return;
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

__global__ __launch_bounds__(256) void k_lm_prep(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= P.n_lm) return;
  if (!P.lm_free[l]) return;
  const int w = P.lm_win[l];
  if (!gnSelect(P, w)) return;
  const double mu = P.st[w].mu;
  const double* V = P.lm_V + 6 * (size_t)l;
  const double* s = P.sL + 3 * (size_t)l;
  const double* g = P.lm_g + 3 * (size_t)l;
  double A[9];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) A[a * 3 + b] = s[a] * s[b] * V[sym3(a, b)];
  const double smu = sqrt(mu);
  for (int a = 0; a < 3; ++a) {
    const double dg = sqrt(fmin(fmax(A[a * 3 + a], P.opt.min_lm_diagonal), P.opt.max_lm_diagonal));
    P.diagL[3 * (size_t)l + a] = dg;
    const double d = dg * smu;
    A[a * 3 + a] += d * d;
  }
  // LLT and inverse (InvertPSDMatrix, full rank)
  double L[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  bool ok = true;
  for (int k = 0; k < 3 && ok; ++k) {
    double d = A[k * 3 + k];
    for (int j = 0; j < k; ++j) d -= L[k * 3 + j] * L[k * 3 + j];
    if (!(d > 0.0)) { ok = false; break; }
    d = sqrt(d);
    L[k * 3 + k] = d;
    for (int i = k + 1; i < 3; ++i) {
      double t = A[i * 3 + k];
      for (int j = 0; j < k; ++j) t -= L[i * 3 + j] * L[k * 3 + j];
      L[i * 3 + k] = t / d;
    }
  }
  if (!ok) {
    P.st[w].gn_failed = 1;
    return;
  }
  // L^-1 (lower triangular) and zz = L^-1 (s g): V'^-1 = L^-T L^-1, so the Schur terms factor as
  // Y_a U_b^T = U_a V'^-1 U_b^T = Z_a Z_b^T with Z = U L^-T (k_visit_prep)
  double Li[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int c = 0; c < 3; ++c) {
    Li[c * 3 + c] = 1.0 / L[c * 3 + c];
    for (int i = c + 1; i < 3; ++i) {
      double t = 0.0;
      for (int j = c; j < i; ++j) t -= L[i * 3 + j] * Li[j * 3 + c];
      Li[i * 3 + c] = t / L[i * 3 + i];
    }
  }
  const double sg[3] = {s[0] * g[0], s[1] * g[1], s[2] * g[2]};
  double* Lo = P.lm_Linv + 9 * (size_t)l;
  for (int i = 0; i < 9; ++i) Lo[i] = Li[i];
  for (int a = 0; a < 3; ++a)
    P.lm_zz[3 * (size_t)l + a] = Li[a * 3 + 0] * sg[0] + Li[a * 3 + 1] * sg[1] + Li[a * 3 + 2] * sg[2];
}

// One thread per visit with a free pose and landmark: Z = U L^-T with U = s_p W s_l, and U z = Z zz
// — the operands of the Schur terms Y_a U_b^T = Z_a Z_b^T (24-double AoS records; 16-byte stores,
// merged in L2).
__global__ __launch_bounds__(256) void k_visit_prep(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= P.n_visit) return;
  const int l = P.visit_lm[v];
  const int w = P.lm_win[l];
  if (!gnSelect(P, w)) return;
  const int pf = P.pose_f[P.visit_pose[v]];
  double2* out = reinterpret_cast<double2*>(P.visit_UY + (size_t)v * kVisitUY);
  if (pf < 0 || !P.lm_free[l]) {
#pragma unroll
    for (int i = 0; i < kVisitUY / 2; ++i) out[i] = double2{0.0, 0.0};
    return;
  }
  const auto W = gmem(P.visit_lin + (size_t)v * kVisitLin);
  const auto sl = gmem(P.sL + 3 * (size_t)l);
  const auto Lig = gmem(P.lm_Linv + 9 * (size_t)l);
  const auto zg = gmem(P.lm_zz + 3 * (size_t)l);
  const auto sp = gmem(P.sF + (size_t)P.win_foff[w] + pf);
  double w18[18], Li[9], zz[3], s3[3], spr[6];
#pragma unroll
  for (int i = 0; i < 18; ++i) w18[i] = W[i];
#pragma unroll
  for (int i = 0; i < 9; ++i) Li[i] = Lig[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) { zz[i] = zg[i]; s3[i] = sl[i]; }
#pragma unroll
  for (int i = 0; i < 6; ++i) spr[i] = sp[i];
  double o[kVisitUY];  // Z = s_p W s_l L^-T (6x3) | U z = Z zz (6)
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const double u0 = spr[r] * w18[r * 3 + 0] * s3[0], u1 = spr[r] * w18[r * 3 + 1] * s3[1],
                 u2 = spr[r] * w18[r * 3 + 2] * s3[2];
    const double z0 = u0 * Li[0];
    const double z1 = u0 * Li[3] + u1 * Li[4];
    const double z2 = u0 * Li[6] + u1 * Li[7] + u2 * Li[8];
    o[r * 3 + 0] = z0; o[r * 3 + 1] = z1; o[r * 3 + 2] = z2;
    o[18 + r] = z0 * zz[0] + z1 * zz[1] + z2 * zz[2];
  }
#pragma unroll
  for (int i = 0; i < kVisitUY / 2; ++i) out[i] = double2{o[2 * i], o[2 * i + 1]};
}

// Clears the structurally non-zero tiles of S (one workgroup per tile; padded diagonal = 1). Zero
// tiles are never written by the factorisation and stay zero from the initial arena clear.
__global__ __launch_bounds__(256) void k_zero_S(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int item = blockIdx.x;
  const int w = P.tile_items[3 * item], ti = P.tile_items[3 * item + 1], tj = P.tile_items[3 * item + 2];
  if (!gnSelect(P, w)) return;
  const int fpad = P.win_fpad[w], fdim = P.win_fdim[w];
  double* S = P.S + P.win_soff[w];
  for (int e = threadIdx.x; e < kTile * kTile; e += 256) {
    const int r = ti * kTile + (e >> 6), c = tj * kTile + (e & 63);
    S[(int64_t)r * fpad + c] = (r == c && r >= fdim) ? 1.0 : 0.0;
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

__global__ __launch_bounds__(256, 6) void k_assemble_pp(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= P.n_asm_pp) return;
  const int k = P.asm_pp_items[item];
  if (k < 0) return;
  const int w = P.pair_win[k];
  if (!gnSelect(P, w)) return;
  const int g = lane / 6, r = lane - 6 * (lane / 6);
  const bool inGroup = g < kGroups;
  const int cb = P.pair_cbegin[k], pb = P.pair_runs[2 * k], ob = P.pair_runs[2 * k + 1], ce = P.pair_cbegin[k + 1];
  const auto pc = gmem(P.pair_contrib);
  const auto vlin = gmem(P.visit_lin);
  const auto vuy = gmem(P.visit_UY);
  double H[6], Sc[6], uz = 0.0;
#pragma unroll
  for (int q = 0; q < 6; ++q) { H[q] = 0.0; Sc[q] = 0.0; }
  const int g0 = inGroup ? g : 1 << 29;  // lanes 48..63 idle (factor-block loop)
  // Descriptors: one coalesced load of 64 per round (lane L holds c = base + L), handed to the
  // groups with __shfl, so each step waits on a single round of operand loads.
  // visits (diagonal pairs): row r of H_v, and (U_v z_l)_r
  for (int base = cb; base < pb; base += 64) {
    const int myc = min(base + lane, pb - 1);
    const int da = pc[myc].a, db = pc[myc].b;
    const int nstep = min(64, pb - base);
    for (int st = 0; st < nstep; st += kGroups) {
      const int k0 = st + g;
      const int a0 = __shfl(da, k0 & 63, 64), b0 = __shfl(db, k0 & 63, 64);
      const bool v0 = inGroup && k0 < nstep;
      const auto H0 = vlin + (size_t)a0 * kVisitLin + 18;
      double h0[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) h0[q] = H0[sym6(r, q)];
      const double z0 = vuy[(size_t)a0 * kVisitUY + 18 + r];
#pragma unroll
      for (int q = 0; q < 6; ++q) H[q] += v0 ? h0[q] : 0.0;
      uz += (v0 && b0) ? z0 : 0.0;
    }
  }
  // landmark pairs: row r of Z_a Z_b^T (= Y_a U_b^T); one contribution per group and step keeps
  // the operand registers low enough for 6 wavefronts per SIMD
  for (int base = pb; base < ob; base += 64) {
    const int myc = min(base + lane, ob - 1);
    const int da = pc[myc].a, db = pc[myc].b;
    const int nstep = min(64, ob - base);
    for (int st = 0; st < nstep; st += kGroups) {
      const int k0 = st + g;
      const int a0 = __shfl(da, k0 & 63, 64), b0 = __shfl(db, k0 & 63, 64);
      const bool v0 = inGroup && k0 < nstep;
      const auto Y0 = vuy + (size_t)a0 * kVisitUY + 3 * r;
      const auto U0 = vuy + (size_t)b0 * kVisitUY;
      double y0[3], u0[18];
#pragma unroll
      for (int i = 0; i < 3; ++i) y0[i] = Y0[i];
#pragma unroll
      for (int i = 0; i < 18; ++i) u0[i] = U0[i];
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const double t0 = y0[0] * u0[3 * q] + y0[1] * u0[3 * q + 1] + y0[2] * u0[3 * q + 2];
        Sc[q] += v0 ? t0 : 0.0;
      }
    }
  }
  // factor blocks (IMU, pose prior): row r of J_i^T J_j
  const int lb = P.st[w].lcur;
  for (int c = ob + g0; c < ce; c += kGroups) {
    const Contrib C = pc[c];
    if (C.type == C_IMU) {
      const auto Hf = gmem(P.imu_H + (size_t)C.a * kImuHess);
#pragma unroll
      for (int q = 0; q < 6; ++q) H[q] += Hf[sym30(C.b + r, C.c + q)];
    } else {
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
  const int fi = P.pair_fi[k], fj = P.pair_fj[k];
  const int foff = P.win_foff[w];
  const int offi = P.fb_off[fi], offj = P.fb_off[fj];
  const bool diag = fi == fj;
  const double si = P.sF[(size_t)foff + offi + r];
  double* Srow = P.S + P.win_soff[w] + (int64_t)(offi + r) * P.win_fpad[w] + offj;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const double sj = P.sF[(size_t)foff + offj + q];
    double val = si * sj * H[q] - Sc[q];
    if (diag && r == q) {
      const size_t idx = (size_t)foff + offi + r;
      const double dg = sqrt(fmin(fmax(si * si * P.hdF[idx], P.opt.min_lm_diagonal), P.opt.max_lm_diagonal));
      P.diagF[idx] = dg;
      const double d = dg * sqrt(P.st[w].mu);
      val += d * d;
    }
    Srow[q] = val;
  }
  if (diag) {
    // Schur rhs: s_i g_i - sum_visits U_v z_l
    const size_t idx = (size_t)foff + offi + r;
    P.rhsF[idx] = P.sF[idx] * P.gF[idx] - uz;
  }
}

// k_assemble_sb: pairs with a speed/bias block (6x9, 9x9): few contributions (IMU factors,
// speed/bias priors), one entry per lane.
__global__ __launch_bounds__(256) void k_assemble_sb(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= P.n_asm_sb) return;
  const int k = P.asm_sb_items[item];
  const int w = P.pair_win[k];
  if (!gnSelect(P, w)) return;
  const int lb = P.st[w].lcur;
  const int fi = P.pair_fi[k], fj = P.pair_fj[k];
  const int ni = P.fb_kind[fi] == 0 ? 6 : 9, nj = P.fb_kind[fj] == 0 ? 6 : 9;
  const int foff = P.win_foff[w];
  const int offi = P.fb_off[fi], offj = P.fb_off[fj];
  const bool diag = fi == fj;
  const int cb = P.pair_cbegin[k], ce = P.pair_cbegin[k + 1];
  double* S = P.S + P.win_soff[w];
  const int ld = P.win_fpad[w];
  const double smu = sqrt(P.st[w].mu);
  for (int e = lane; e < ni * nj; e += 64) {
    const int r = e / nj, q = e - r * nj;
    double H = 0.0;
    for (int c = cb; c < ce; ++c) {
      const Contrib C = P.pair_contrib[c];
      if (C.type == C_IMU) {
        H += P.imu_H[(size_t)C.a * kImuHess + sym30(C.b + r, C.c + q)];
      } else if (C.type == C_SBPRIOR) {
        const double* L = P.sbp_lin[lb] + 90 * (size_t)C.a + 9;
        double s2 = 0;
        for (int k2 = 0; k2 < 9; ++k2) s2 += L[k2 * 9 + r] * L[k2 * 9 + q];
        H += s2;
      } else if (C.type == C_PPRIOR) {
        const double* L = P.pp_lin[lb] + 42 * (size_t)C.a + 6;
        double s2 = 0;
        for (int k2 = 0; k2 < 6; ++k2) s2 += L[k2 * 6 + r] * L[k2 * 6 + q];
        H += s2;
      }
    }
    const double si = P.sF[(size_t)foff + offi + r], sj = P.sF[(size_t)foff + offj + q];
    double val = si * sj * H;
    if (diag && r == q) {
      const size_t idx = (size_t)foff + offi + r;
      const double dg = sqrt(fmin(fmax(si * si * P.hdF[idx], P.opt.min_lm_diagonal), P.opt.max_lm_diagonal));
      P.diagF[idx] = dg;
      const double d = dg * smu;
      val += d * d;
    }
    S[(int64_t)(offi + r) * ld + offj + q] = val;
  }
  if (diag && lane < ni) {
    const size_t idx = (size_t)foff + offi + lane;
    P.rhsF[idx] = P.sF[idx] * P.gF[idx];
  }
}

__global__ __launch_bounds__(256) void k_lm_backsub(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= P.n_lm) return;
  if (!P.lm_free[l]) return;
  const int w = P.lm_win[l];
  if (!gnSelect(P, w)) return;
  const int foff = P.win_foff[w];
  // y_l = V'^-1 (s g - sum_v U_v^T y_p) = L^-T (zz - sum_v Z_v^T y_p)
  const double* zz = P.lm_zz + 3 * (size_t)l;
  double t3[3] = {zz[0], zz[1], zz[2]};
  for (int v = P.lm_visit_begin[l]; v < P.lm_visit_begin[l + 1]; ++v) {
    const int pf = P.pose_f[P.visit_pose[v]];
    if (pf < 0) continue;
    const double* Z = P.visit_UY + (size_t)v * kVisitUY;
    for (int rr = 0; rr < 6; ++rr) {
      const double y = P.yF[(size_t)foff + pf + rr];
      for (int a = 0; a < 3; ++a) t3[a] -= Z[rr * 3 + a] * y;
    }
  }
  const double* Li = P.lm_Linv + 9 * (size_t)l;
  for (int a = 0; a < 3; ++a) {
    double y = 0.0;
    for (int c = a; c < 3; ++c) y += Li[c * 3 + a] * t3[c];
    P.yL[3 * (size_t)l + a] = y;
  }
}

// gauss_newton_step_ = -diagonal_ .* y ; gradient_ = s .* g / diagonal_ ; v = gradient_ / diagonal_
// (DoglegStrategy::ComputeGradient / ComputeCauchyPoint / ComputeGaussNewtonStep)
__global__ __launch_bounds__(256) void k_gn_finalize(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < P.n_fblock) {
    const int w = P.fb_win[t];
    if (!gnSelect(P, w)) return;
    const int n = P.fb_kind[t] == 0 ? 6 : 9;
    const size_t base = (size_t)P.win_foff[w] + P.fb_off[t];
    for (int c = 0; c < n; ++c) {
      const size_t i = base + c;
      const double dg = P.diagF[i];
      P.gnF[i] = -dg * P.yF[i];
      const double gr = P.sF[i] * P.gF[i] / dg;
      P.dgF[i] = gr;
      P.vF[i] = gr / dg;
    }
    return;
  }
  const int l = t - P.n_fblock;
  if (l >= P.n_lm || !P.lm_free[l]) return;
  const int w = P.lm_win[l];
  if (!gnSelect(P, w)) return;
  for (int a = 0; a < 3; ++a) {
    const size_t i = 3 * (size_t)l + a;
    const double dg = P.diagL[i];
    P.gnL[i] = -dg * P.yL[i];
    const double gr = P.sL[i] * P.lm_g[i] / dg;
    P.dgL[i] = gr;
    P.vL[i] = gr / dg;
  }
}

// ------------------------------------------------------------------------------------ launchers
void launch_visit_lin(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (P.n_visit > 0)
    hipLaunchKernelGGL(k_visit_lin, dim3((P.n_visit + 255) / 256), dim3(256), 0, s, P.self, lin_mode);
}
void launch_visit_prep(const DevProblem& P, hipStream_t s) {
  if (P.n_visit > 0) hipLaunchKernelGGL(k_visit_prep, dim3((P.n_visit + 255) / 256), dim3(256), 0, s, P.self);
}
void launch_assemble_pp(const DevProblem& P, hipStream_t s) {
  if (P.n_asm_pp > 0) hipLaunchKernelGGL(k_assemble_pp, dim3((P.n_asm_pp + 3) / 4), dim3(256), 0, s, P.self);
}
void launch_assemble_sb(const DevProblem& P, hipStream_t s) {
  if (P.n_asm_sb > 0) hipLaunchKernelGGL(k_assemble_sb, dim3((P.n_asm_sb + 3) / 4), dim3(256), 0, s, P.self);
}
void launch_lm_blocks(const DevProblem& P, int lin_mode, hipStream_t s) {
  launch_visit_lin(P, lin_mode, s);
  if (P.n_lm > 0) hipLaunchKernelGGL(k_lm_lin, dim3((P.n_lm + 255) / 256), dim3(256), 0, s, P.self, lin_mode);
}
void launch_fgrad(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (P.n_fblock > 0) hipLaunchKernelGGL(k_fgrad, dim3(P.n_fblock), dim3(64), 0, s, P.self, lin_mode);
}
void launch_imu_hess(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (P.n_imu > 0) hipLaunchKernelGGL(k_imu_hess, dim3((P.n_imu + 3) / 4), dim3(256), 0, s, P.self, lin_mode);
}
void launch_linearization_blocks(const DevProblem& P, int lin_mode, hipStream_t s) {
  launch_lm_blocks(P, lin_mode, s);
  launch_imu_hess(P, lin_mode, s);
  launch_fgrad(P, lin_mode, s);
}
void launch_lm_prep(const DevProblem& P, hipStream_t s) {
  if (P.n_lm > 0) hipLaunchKernelGGL(k_lm_prep, dim3((P.n_lm + 255) / 256), dim3(256), 0, s, P.self);
  launch_visit_prep(P, s);
}
void launch_zero_S(const DevProblem& P, hipStream_t s) {
  if (P.n_tiles > 0) hipLaunchKernelGGL(k_zero_S, dim3(P.n_tiles), dim3(256), 0, s, P.self);
}
void launch_assemble(const DevProblem& P, hipStream_t s) {
  launch_assemble_pp(P, s);
  launch_assemble_sb(P, s);
}
void launch_gn_reduce(const DevProblem& P, hipStream_t s) {
  launch_lm_prep(P, s);
  launch_zero_S(P, s);
  launch_assemble(P, s);
}
void launch_lm_backsub(const DevProblem& P, hipStream_t s) {
  if (P.n_lm > 0) hipLaunchKernelGGL(k_lm_backsub, dim3((P.n_lm + 255) / 256), dim3(256), 0, s, P.self);
}
void launch_gn_finalize(const DevProblem& P, hipStream_t s) {
  const int n = P.n_fblock + P.n_lm;
  if (n > 0) hipLaunchKernelGGL(k_gn_finalize, dim3((n + 255) / 256), dim3(256), 0, s, P.self);
}
void launch_gn_backsub(const DevProblem& P, hipStream_t s) {
  launch_lm_backsub(P, s);
  launch_gn_finalize(P, s);
}

}  // namespace okg
