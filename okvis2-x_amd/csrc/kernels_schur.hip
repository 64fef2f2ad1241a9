// kernels_schur.hip — landmark elimination (DENSE_SCHUR) for gfx950, FP64.
//
// The reduced ("camera") system of a window is formed exactly as Ceres' SchurEliminator does for
// e-blocks = landmarks, but organised for the GPU:
//   k_lm_blocks   one thread per landmark: per-visit blocks W = J_p^T J_l, H_pp = J_p^T J_p,
//                 g_p = J_p^T r and per-landmark V = J_l^T J_l, g_l = J_l^T r from the stored
//                 linearisation (unscaled; the Jacobi scaling is applied by the consumers).
//   k_fgrad       one thread per f-block (pose / speed-bias): unscaled gradient and diag(H_ff),
//                 and at iteration 0 the Jacobi scaling 1/(1+sqrt(diag)).
//   k_lm_prep     one thread per landmark: (s V s + D^2)^-1 via 3x3 LLT (InvertPSDMatrix), z.
//   k_zero_S      clears the dense lower triangle (padded diagonal = 1).
//   k_assemble    one workgroup per non-zero f-block pair (i >= j): every entry is a fixed-order
//                 sum over that pair's contribution list — visits, landmark pairs (the
//                 W_i V^-1 W_j^T Schur terms), IMU / prior J^T J sub-blocks — so the reduction is
//                 deterministic without atomics; diagonal pairs also emit the Schur rhs and the
//                 dogleg diagonal.
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

__global__ __launch_bounds__(256) void k_lm_blocks(const DevProblem* __restrict__ Pp, int lin_mode) {
  const DevProblem& P = *Pp;
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= P.n_lm) return;
  const int w = P.lm_win[l];
  if (!linSelect(P, w, lin_mode)) return;
  const int vb = P.lm_visit_begin[l], ve = P.lm_visit_begin[l + 1];
  if (vb == ve) return;
  const int lb = P.st[w].lcur;
  const bool lfree = P.lm_free[l] != 0;
  const double* lin = P.obs_lin[lb];
  const int64_t S = P.obs_stride;
  double V[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
  for (int v = vb; v < ve; ++v) {
    const bool pf = P.pose_f[P.visit_pose[v]] >= 0;
    double W[18], H[21], gp[6];
    for (int i = 0; i < 18; ++i) W[i] = 0.0;
    for (int i = 0; i < 21; ++i) H[i] = 0.0;
    for (int i = 0; i < 6; ++i) gp[i] = 0.0;
    for (int o = P.visit_obs_begin[v]; o < P.visit_obs_begin[v + 1]; ++o) {
      if (P.obs_flags[o] & 2) continue;
      double r[2], Jp[12], Jl[6];
      r[0] = lin[0 * S + o];
      r[1] = lin[1 * S + o];
#pragma unroll
      for (int k = 0; k < 12; ++k) Jp[k] = lin[(2 + k) * S + o];
#pragma unroll
      for (int k = 0; k < 6; ++k) Jl[k] = lin[(14 + k) * S + o];
      if (lfree) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          g[a] += Jl[a] * r[0] + Jl[3 + a] * r[1];
#pragma unroll
          for (int b = a; b < 3; ++b) V[sym3(a, b)] += Jl[a] * Jl[b] + Jl[3 + a] * Jl[3 + b];
        }
      }
      if (pf) {
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          gp[a] += Jp[a] * r[0] + Jp[6 + a] * r[1];
#pragma unroll
          for (int b = a; b < 6; ++b) H[sym6(a, b)] += Jp[a] * Jp[b] + Jp[6 + a] * Jp[6 + b];
          if (lfree)
#pragma unroll
            for (int b = 0; b < 3; ++b) W[a * 3 + b] += Jp[a] * Jl[b] + Jp[6 + a] * Jl[3 + b];
        }
      }
    }
    if (pf) {
      double* Wd = P.visit_W + 18 * (size_t)v;
      double* Hd = P.visit_H + 21 * (size_t)v;
      double* gd = P.visit_g + 6 * (size_t)v;
      for (int i = 0; i < 18; ++i) Wd[i] = W[i];
      for (int i = 0; i < 21; ++i) Hd[i] = H[i];
      for (int i = 0; i < 6; ++i) gd[i] = gp[i];
    }
  }
  if (lfree) {
    for (int i = 0; i < 6; ++i) P.lm_V[6 * (size_t)l + i] = V[i];
    for (int i = 0; i < 3; ++i) P.lm_g[3 * (size_t)l + i] = g[i];
    if (lin_mode == 0)  // Jacobi scaling fixed at iteration 0 (TrustRegionMinimizer)
      for (int a = 0; a < 3; ++a)
        P.sL[3 * (size_t)l + a] = P.opt.jacobi_scaling ? 1.0 / (1.0 + sqrt(V[sym3(a, a)])) : 1.0;
  }
}

// contribution helpers -------------------------------------------------------------------------
__device__ __forceinline__ const double* imuLin(const DevProblem& P, int lb, int f) {
  return P.imu_lin[lb] + (size_t)f * kImuLin;
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
      const double* H = P.visit_H + 21 * (size_t)cb.a;
      const double* gp = P.visit_g + 6 * (size_t)cb.a;
#pragma unroll
      for (int c = 0; c < 6; ++c) { g[c] += gp[c]; hd[c] += H[sym6(c, c)]; }
    } else if (cb.type == C_IMU) {
      const double* L = imuLin(P, lb, cb.a);
      for (int c = 0; c < n; ++c) {
        double sg = 0, sh = 0;
        for (int k2 = 0; k2 < 15; ++k2) {
          const double j = L[15 + k2 * 30 + cb.b + c];
          sg += j * L[k2];
          sh += j * j;
        }
        g[c] += sg;
        hd[c] += sh;
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
  double inv[9];
  for (int c = 0; c < 3; ++c) {
    double e[3] = {0, 0, 0};
    e[c] = 1.0;
    for (int i = 0; i < 3; ++i) {
      double t = e[i];
      for (int j = 0; j < i; ++j) t -= L[i * 3 + j] * e[j];
      e[i] = t / L[i * 3 + i];
    }
    for (int i = 2; i >= 0; --i) {
      double t = e[i];
      for (int j = i + 1; j < 3; ++j) t -= L[j * 3 + i] * e[j];
      e[i] = t / L[i * 3 + i];
    }
    for (int r = 0; r < 3; ++r) inv[r * 3 + c] = e[r];
  }
  double sg[3] = {s[0] * g[0], s[1] * g[1], s[2] * g[2]};
  double* Vi = P.lm_Vinv + 9 * (size_t)l;
  for (int i = 0; i < 9; ++i) Vi[i] = inv[i];
  double z[3];
  for (int a = 0; a < 3; ++a) {
    z[a] = inv[a * 3 + 0] * sg[0] + inv[a * 3 + 1] * sg[1] + inv[a * 3 + 2] * sg[2];
    P.lm_z[3 * (size_t)l + a] = z[a];
  }
  // per visit (free pose): U = s_p W s_l, Y = U Vinv, uz = U z — the operands of the Schur terms
  const int foff = P.win_foff[w];
  for (int v = P.lm_visit_begin[l]; v < P.lm_visit_begin[l + 1]; ++v) {
    const int pf = P.pose_f[P.visit_pose[v]];
    if (pf < 0) continue;
    const double* W = P.visit_W + 18 * (size_t)v;
    double* UY = P.visit_UY + 36 * (size_t)v;
    double* uz = P.visit_uz + 6 * (size_t)v;
    for (int r = 0; r < 6; ++r) {
      const double sp = P.sF[(size_t)foff + pf + r];
      const double u0 = sp * W[r * 3 + 0] * s[0], u1 = sp * W[r * 3 + 1] * s[1], u2 = sp * W[r * 3 + 2] * s[2];
      UY[r * 3 + 0] = u0; UY[r * 3 + 1] = u1; UY[r * 3 + 2] = u2;
      for (int b = 0; b < 3; ++b) UY[18 + r * 3 + b] = u0 * inv[0 * 3 + b] + u1 * inv[1 * 3 + b] + u2 * inv[2 * 3 + b];
      uz[r] = u0 * z[0] + u1 * z[1] + u2 * z[2];
    }
  }
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

// One workgroup per non-zero f-block pair; contributions are processed in chunks of 64 whose
// operands (visit H / uz, or the Y_i, U_j pair of a landmark) are first staged into LDS with
// coalesced loads, so the per-entry accumulation reads only LDS (no dependent global chains).
constexpr int kChunk = 64;
constexpr int kStage = 36;

__global__ __launch_bounds__(128) void k_assemble(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int k = blockIdx.x;
  if (k >= P.n_pair) return;
  const int w = P.pair_win[k];
  if (!gnSelect(P, w)) return;
  __shared__ double stage[kChunk * kStage];
  __shared__ Contrib sc[kChunk];
  const int lb = P.st[w].lcur;
  const double mu = P.st[w].mu;
  const int fi = P.pair_fi[k], fj = P.pair_fj[k];
  const int ni = P.fb_kind[fi] == 0 ? 6 : 9, nj = P.fb_kind[fj] == 0 ? 6 : 9;
  const int foff = P.win_foff[w];
  const int offi = P.fb_off[fi], offj = P.fb_off[fj];
  const int t = threadIdx.x;
  const int cb = P.pair_cbegin[k], ce = P.pair_cbegin[k + 1];
  const bool entry = t < ni * nj;
  const int r = entry ? t / nj : 0, c = entry ? t % nj : 0;
  const bool diag = (fi == fj);
  double H = 0.0, schur = 0.0, uzacc = 0.0;
  for (int c0 = cb; c0 < ce; c0 += kChunk) {
    const int nc = min(kChunk, ce - c0);
    __syncthreads();
    if (t < nc) sc[t] = P.pair_contrib[c0 + t];
    __syncthreads();
    for (int e = t; e < nc * kStage; e += 128) {
      const int q = e / kStage, x = e - q * kStage;
      const Contrib C = sc[q];
      double v = 0.0;
      if (C.type == C_PAIR) v = (x < 18) ? P.visit_UY[36 * (size_t)C.a + 18 + x] : P.visit_UY[36 * (size_t)C.b + x - 18];
      else if (C.type == C_VISIT) v = (x < 21) ? P.visit_H[21 * (size_t)C.a + x]
                                    : (x < 27 && C.b) ? P.visit_uz[6 * (size_t)C.a + x - 21] : 0.0;
      stage[e] = v;
    }
    __syncthreads();
    for (int q = 0; q < nc; ++q) {
      const Contrib C = sc[q];  // uniform across the workgroup
      const double* st = stage + q * kStage;
      if (C.type == C_PAIR) {
        if (entry) schur += st[r * 3 + 0] * st[18 + c * 3 + 0] + st[r * 3 + 1] * st[18 + c * 3 + 1] +
                            st[r * 3 + 2] * st[18 + c * 3 + 2];
      } else if (C.type == C_VISIT) {
        if (entry) H += st[sym6(r, c)];
        if (diag && t < ni) uzacc += st[21 + t];
      } else if (C.type == C_IMU) {
        if (entry) {
          const double* L = imuLin(P, lb, C.a) + 15;
          double s2 = 0;
          for (int k2 = 0; k2 < 15; ++k2) s2 += L[k2 * 30 + C.b + r] * L[k2 * 30 + C.c + c];
          H += s2;
        }
      } else if (C.type == C_PPRIOR) {
        if (entry) {
          const double* L = P.pp_lin[lb] + 42 * (size_t)C.a + 6;
          double s2 = 0;
          for (int k2 = 0; k2 < 6; ++k2) s2 += L[k2 * 6 + r] * L[k2 * 6 + c];
          H += s2;
        }
      } else if (C.type == C_SBPRIOR) {
        if (entry) {
          const double* L = P.sbp_lin[lb] + 90 * (size_t)C.a + 9;
          double s2 = 0;
          for (int k2 = 0; k2 < 9; ++k2) s2 += L[k2 * 9 + r] * L[k2 * 9 + c];
          H += s2;
        }
      }
    }
  }
  if (entry) {
    const double si = P.sF[(size_t)foff + offi + r], sj = P.sF[(size_t)foff + offj + c];
    double val = si * sj * H - schur;
    if (diag && r == c) {
      const double dg = sqrt(fmin(fmax(si * si * P.hdF[(size_t)foff + offi + r], P.opt.min_lm_diagonal),
                                  P.opt.max_lm_diagonal));
      P.diagF[(size_t)foff + offi + r] = dg;
      const double d = dg * sqrt(mu);
      val += d * d;
    }
    P.S[P.win_soff[w] + (int64_t)(offi + r) * P.win_fpad[w] + offj + c] = val;
  }
  if (diag && t < ni) {
    // Schur rhs: s_i g_i - sum_visits U_v z_l
    const size_t idx = (size_t)foff + offi + t;
    P.rhsF[idx] = P.sF[idx] * P.gF[idx] - uzacc;
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
  const double* s = P.sL + 3 * (size_t)l;
  const double* g = P.lm_g + 3 * (size_t)l;
  double rhs[3] = {s[0] * g[0], s[1] * g[1], s[2] * g[2]};
  for (int v = P.lm_visit_begin[l]; v < P.lm_visit_begin[l + 1]; ++v) {
    const int pf = P.pose_f[P.visit_pose[v]];
    if (pf < 0) continue;
    const double* U = P.visit_UY + 36 * (size_t)v;  // U = s_p W s_l
    for (int rr = 0; rr < 6; ++rr) {
      const double y = P.yF[(size_t)foff + pf + rr];
      for (int a = 0; a < 3; ++a) rhs[a] -= U[rr * 3 + a] * y;
    }
  }
  const double* Vi = P.lm_Vinv + 9 * (size_t)l;
  for (int a = 0; a < 3; ++a)
    P.yL[3 * (size_t)l + a] = Vi[a * 3 + 0] * rhs[0] + Vi[a * 3 + 1] * rhs[1] + Vi[a * 3 + 2] * rhs[2];
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
void launch_lm_blocks(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (P.n_lm > 0) hipLaunchKernelGGL(k_lm_blocks, dim3((P.n_lm + 255) / 256), dim3(256), 0, s, P.self, lin_mode);
}
void launch_fgrad(const DevProblem& P, int lin_mode, hipStream_t s) {
  if (P.n_fblock > 0) hipLaunchKernelGGL(k_fgrad, dim3(P.n_fblock), dim3(64), 0, s, P.self, lin_mode);
}
void launch_linearization_blocks(const DevProblem& P, int lin_mode, hipStream_t s) {
  launch_lm_blocks(P, lin_mode, s);
  launch_fgrad(P, lin_mode, s);
}
void launch_lm_prep(const DevProblem& P, hipStream_t s) {
  if (P.n_lm > 0) hipLaunchKernelGGL(k_lm_prep, dim3((P.n_lm + 255) / 256), dim3(256), 0, s, P.self);
}
void launch_zero_S(const DevProblem& P, hipStream_t s) {
  if (P.n_tiles > 0) hipLaunchKernelGGL(k_zero_S, dim3(P.n_tiles), dim3(256), 0, s, P.self);
}
void launch_assemble(const DevProblem& P, hipStream_t s) {
  if (P.n_pair > 0) hipLaunchKernelGGL(k_assemble, dim3(P.n_pair), dim3(128), 0, s, P.self);
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
