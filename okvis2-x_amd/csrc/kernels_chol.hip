// kernels_chol.hip — dense LLT of the reduced camera matrix S (Eigen::LLT semantics: fail at the
// first non-positive pivot) and the two triangular solves, batched over windows (blockIdx.y).
//
// Right-looking blocked Cholesky with 64x64 FP64 tiles. Per panel k:
//   k_potrf_inv(k)   one workgroup per window: factor the diagonal tile with register-owned
//                    elements and one barrier per column, fused with the inverse of the factor
//                    and with the forward substitution y_k = L_kk^-1 rhs_k.
//   (only structurally non-zero tiles: the work lists come from the host's tile-level symbolic
//    factorisation, DevProblem::chol_*_items)
//   k_panel(k)       one workgroup per tile row i > k: L_ik = A_ik (L_kk^-1)^T — a 64x64x64 GEMM on
//                    the FP64 matrix cores — and rhs_i -= L_ik y_k.
//   k_chol_update(k) one workgroup per trailing tile (i, j), k < j <= i: A_ij -= L_ik L_jk^T — the
//                    dense reduced-camera block multiply (v_mfma_f64_16x16x4_f64).
//   k_trsv           one workgroup per window: block backward substitution, every diagonal solve a
//                    mat-vec with the stored L_kk^-1 (no serial inner loop).
//
// MFMA tile: each of the 4 wavefronts owns a 32x32 quarter of the 64x64 output (2x2 16x16 MFMA
// tiles), K = 64 in steps of 4. v_mfma_f64_16x16x4_f64 operand map: lane l supplies A[l&15][l>>4]
// and B[l>>4][l&15]; result reg r of lane l is C[(l>>4) + 4r][l&15] (cdna_hip_programming.md §3).
#include "device_problem.hpp"
#include "launch.hpp"

namespace okg {

constexpr int kLd = kTile + 1;  // padded LDS row (65 doubles)

typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool cholSelect(const DevProblem& P, int w) {
  const WinState& s = P.st[w];
  return !s.done && s.need_gn && !s.gn_failed;
}

__device__ __forceinline__ void loadTile(const double* A, int64_t ld, int r0, int c0, double* s, int t) {
  for (int e = t; e < kTile * kTile; e += 256) {
    const int r = e >> 6, c = e & 63;
    s[r * kLd + c] = A[(int64_t)(r0 + r) * ld + c0 + c];
  }
}

// acc = sA * sB^T over the 64-deep inner dimension (both tiles row-major [64][kLd] in LDS).
__device__ __forceinline__ void mfmaTileNT(const double* sA, const double* sB, dbl4 acc[2][2], int t) {
  const int wave = t >> 6, lane = t & 63;
  const int r0 = 32 * (wave >> 1), c0 = 32 * (wave & 1);
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int kk = 0; kk < kTile; kk += 4) {
    double av[2], bv[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) av[a] = sA[(r0 + 16 * a + lr) * kLd + kk + lk];
#pragma unroll
    for (int b = 0; b < 2; ++b) bv[b] = sB[(c0 + 16 * b + lr) * kLd + kk + lk];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
  }
}

template <bool SUB>
__device__ __forceinline__ void storeTile(double* A, int64_t ld, int r0g, int c0g, const dbl4 acc[2][2], int t) {
  const int wave = t >> 6, lane = t & 63;
  const int r0 = 32 * (wave >> 1), c0 = 32 * (wave & 1);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int rr = r0 + 16 * a + (lane >> 4) + 4 * reg;
        const int cc = c0 + 16 * b + (lane & 15);
        double* dst = A + (int64_t)(r0g + rr) * ld + c0g + cc;
        if (SUB) *dst -= acc[a][b][reg];
        else *dst = acc[a][b][reg];
      }
}

// Factor + invert the diagonal tile k with register-owned elements: thread (tr, tc) owns rows
// tr + 16a and columns tc + 16b (a, b < 4) of both A (being factored) and X = L^-1. One barrier
// per column c: owners publish column c of A (right-looking with deferred scaling,
// A_ij -= A_ic A_jc / A_cc) and, lagging one column, the finalised row c-1 of X (right-looking
// inverse: X_c /= L_cc; X_i -= L_ic X_c); multi-buffered LDS rows avoid write-after-read hazards.
// The forward substitution of the Schur rhs is fused: y_k = L_kk^-1 rhs_k.
__global__ __launch_bounds__(256) void k_potrf_inv(const DevProblem* __restrict__ Pp, int k) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  if (!cholSelect(P, w)) return;
  const int ld = P.win_fpad[w];
  const int T = ld / kTile;
  if (k >= T) return;
  double* Sg = P.S + P.win_soff[w];
  double* work = P.fwdF + P.win_fwdoff[w];
  // colbuf[s][i]: column c of A for rows i > c, ZERO for i <= c (so the updates need no masks);
  // triple-buffered because the lagging inverse still reads column c-1 during step c.
  __shared__ double colbuf[3][kTile];
  __shared__ double rowbuf[2][kTile];
  __shared__ double dgs[3];
  __shared__ double rsq[kTile];  // 1 / sqrt(pivot)
  __shared__ double sy[kTile];
  const int t = threadIdx.x;
  const int tr = t >> 4, tc = t & 15;
  if (k == 0)  // start of the factorisation: work = rhs (zero-padded)
    for (int e = t; e < ld; e += 256) work[e] = (e < P.win_fdim[w]) ? P.rhsF[(size_t)P.win_foff[w] + e] : 0.0;
  double A[4][4], X[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int i = tr + 16 * a, j = tc + 16 * b;
      A[a][b] = Sg[(int64_t)(k * kTile + i) * ld + k * kTile + j];
      X[a][b] = (i == j) ? 1.0 : 0.0;
    }
  bool failed = false;
  double rl_prev = 0.0;  // 1/sqrt(pivot c-1)
  for (int c = 0; c <= kTile; ++c) {
    const int cb = c % 3, pb = (c + 2) % 3, rb = (c - 1) & 1;
    // ---- publish: column c of A (owners tc == c%16, block column c/16) and row c-1 of X
    if (c < kTile && tc == (c & 15)) {
      const int bc = c >> 4;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        double v = 0.0;
#pragma unroll
        for (int b = 0; b < 4; ++b) v = (b == bc) ? A[a][b] : v;
        const int i = tr + 16 * a;
        colbuf[cb][i] = (i > c) ? v : 0.0;
        if (i == c) dgs[cb] = v;
      }
    }
    if (c >= 1 && tr == ((c - 1) & 15)) {
      const int ac = (c - 1) >> 4;
#pragma unroll
      for (int a = 0; a < 4; ++a)
        if (a == ac)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            X[a][b] *= rl_prev;
            rowbuf[rb][tc + 16 * b] = X[a][b];
          }
    }
    __syncthreads();
    // ---- X update with column c-1 of L and row c-1 of X (rows <= c-1 see zeros)
    if (c >= 1) {
      double li[4], xr[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) li[a] = colbuf[pb][tr + 16 * a] * rl_prev;
#pragma unroll
      for (int b = 0; b < 4; ++b) xr[b] = rowbuf[rb][tc + 16 * b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) X[a][b] -= li[a] * xr[b];
    }
    if (c == kTile) break;
    // ---- A update with column c: A_ij -= A_ic A_jc / A_cc (zeros outside the trailing block)
    const double dcc = dgs[cb];
    if (!(dcc > 0.0)) { failed = true; break; }  // uniform across the workgroup
    const double rinv = 1.0 / dcc;
    rl_prev = 1.0 / sqrt(dcc);
    if (t == 0) rsq[c] = rl_prev;
    double ci[4], cj[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) ci[a] = colbuf[cb][tr + 16 * a] * rinv;
#pragma unroll
    for (int b = 0; b < 4; ++b) cj[b] = colbuf[cb][tc + 16 * b];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) A[a][b] -= ci[a] * cj[b];
  }
  if (failed) {
    if (t == 0) P.st[w].gn_failed = 1;
    return;
  }
  __syncthreads();
  // ---- L_kk back into S, X into the inverse store, forward substitution y_k
  double* Li = P.Linv + P.win_linvoff[w] + (int64_t)k * kTile * kTile;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int i = tr + 16 * a, j = tc + 16 * b;
      if (j <= i) {
        const double rj = rsq[j];
        Sg[(int64_t)(k * kTile + i) * ld + k * kTile + j] = (i == j) ? 1.0 / rj : A[a][b] * rj;
      }
      Li[i * kTile + j] = (j <= i) ? X[a][b] : 0.0;
    }
  if (t < kTile) sy[t] = work[k * kTile + t];
  __syncthreads();
  double part[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    part[a] = 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int i = tr + 16 * a, j = tc + 16 * b;
      part[a] += (j <= i) ? X[a][b] * sy[j] : 0.0;
    }
#pragma unroll
    for (int sh = 8; sh > 0; sh >>= 1) part[a] += __shfl_xor(part[a], sh, 16);
  }
  if (tc == 0)
#pragma unroll
    for (int a = 0; a < 4; ++a) work[k * kTile + tr + 16 * a] = part[a];
}

// L_ik = A_ik (L_kk^-1)^T on the matrix cores, then the fused forward-substitution update
// rhs_i -= L_ik y_k.
__global__ __launch_bounds__(256) void k_panel(const DevProblem* __restrict__ Pp, int k) {
  const DevProblem& P = *Pp;
  const int item = P.chol_panel_begin[k] + blockIdx.x;
  const int w = P.chol_panel_items[2 * item], i = P.chol_panel_items[2 * item + 1];
  if (!cholSelect(P, w)) return;
  const int ld = P.win_fpad[w];
  double* A = P.S + P.win_soff[w];
  double* work = P.fwdF + P.win_fwdoff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sB[kTile * kLd];
  __shared__ double sy[kTile];
  const int t = threadIdx.x;
  loadTile(A, ld, i * kTile, k * kTile, sA, t);
  const double* Li = P.Linv + P.win_linvoff[w] + (int64_t)k * kTile * kTile;
  for (int e = t; e < kTile * kTile; e += 256) sB[(e >> 6) * kLd + (e & 63)] = Li[e];
  if (t < kTile) sy[t] = work[k * kTile + t];
  __syncthreads();
  dbl4 acc[2][2];
  mfmaTileNT(sA, sB, acc, t);  // A_ik (L_kk^-1)^T
  storeTile<false>(A, ld, i * kTile, k * kTile, acc, t);
  __syncthreads();
  // stage L_ik into LDS (reuse sA) for the rhs update
  {
    const int wave = t >> 6, lane = t & 63;
    const int r0 = 32 * (wave >> 1), c0 = 32 * (wave & 1);
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b)
        for (int reg = 0; reg < 4; ++reg)
          sA[(r0 + 16 * a + (lane >> 4) + 4 * reg) * kLd + c0 + 16 * b + (lane & 15)] = acc[a][b][reg];
  }
  __syncthreads();
  const int row = t >> 2, q = t & 3;
  double s = 0.0;
  for (int c = q; c < kTile; c += 4) s += sA[row * kLd + c] * sy[c];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  if (q == 0) work[i * kTile + row] -= s;
}

__global__ __launch_bounds__(256) void k_chol_update(const DevProblem* __restrict__ Pp, int k) {
  const DevProblem& P = *Pp;
  const int item = P.chol_upd_begin[k] + blockIdx.x;
  const int w = P.chol_upd_items[3 * item], i = P.chol_upd_items[3 * item + 1], j = P.chol_upd_items[3 * item + 2];
  if (!cholSelect(P, w)) return;
  const int ld = P.win_fpad[w];
  double* A = P.S + P.win_soff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sB[kTile * kLd];
  const int t = threadIdx.x;
  loadTile(A, ld, i * kTile, k * kTile, sA, t);
  loadTile(A, ld, j * kTile, k * kTile, sB, t);
  __syncthreads();
  dbl4 acc[2][2];
  mfmaTileNT(sA, sB, acc, t);
  storeTile<true>(A, ld, i * kTile, j * kTile, acc, t);
}

// Backward substitution L^T y = u (u = the forward-substituted rhs left by k_potrf_inv / k_panel),
// y in LDS (dynamic shared memory: fpad doubles); diagonal blocks through the stored inverses.
__global__ __launch_bounds__(256) void k_trsv(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  if (!cholSelect(P, w)) return;
  extern __shared__ double y[];
  __shared__ double part[4 * kTile];
  __shared__ double v[kTile];
  const int ld = P.win_fpad[w], fdim = P.win_fdim[w], foff = P.win_foff[w];
  const int T = ld / kTile;
  const double* A = P.S + P.win_soff[w];
  const double* Linv = P.Linv + P.win_linvoff[w];
  const double* work = P.fwdF + P.win_fwdoff[w];
  const int t = threadIdx.x;
  for (int e = t; e < ld; e += 256) y[e] = work[e];
  __syncthreads();
  for (int I = T - 1; I >= 0; --I) {
    {
      const int col = t & 63, q = t >> 6;
      double acc = 0.0;
      for (int r = (I + 1) * kTile + q; r < ld; r += 4) acc += A[(int64_t)r * ld + I * kTile + col] * y[r];
      part[q * kTile + col] = acc;
    }
    __syncthreads();
    if (t < kTile) v[t] = y[I * kTile + t] - (part[t] + part[kTile + t] + part[2 * kTile + t] + part[3 * kTile + t]);
    __syncthreads();
    {
      const int col = t & 63, q = t >> 6;
      const double* Li = Linv + (int64_t)I * kTile * kTile;
      double acc = 0.0;
      for (int r = col + q; r < kTile; r += 4) acc += Li[r * kTile + col] * v[r];
      part[q * kTile + col] = acc;
    }
    __syncthreads();
    if (t < kTile) y[I * kTile + t] = part[t] + part[kTile + t] + part[2 * kTile + t] + part[3 * kTile + t];
    __syncthreads();
  }
  for (int e = t; e < fdim; e += 256) P.yF[(size_t)foff + e] = y[e];
}

void launch_potrf(const DevProblem& P, int k, hipStream_t s) {
  hipLaunchKernelGGL(k_potrf_inv, dim3(P.n_win), dim3(256), 0, s, P.self, k);
}
void launch_panel(const DevProblem& P, int k, hipStream_t s) {
  const int n = P.h_panel_begin[k + 1] - P.h_panel_begin[k];
  if (n > 0) hipLaunchKernelGGL(k_panel, dim3(n), dim3(256), 0, s, P.self, k);
}
void launch_chol_panel(const DevProblem& P, int k, hipStream_t s) {
  launch_potrf(P, k, s);
  launch_panel(P, k, s);
}
void launch_chol_update(const DevProblem& P, int k, hipStream_t s) {
  const int n = P.h_upd_begin[k + 1] - P.h_upd_begin[k];
  if (n > 0) hipLaunchKernelGGL(k_chol_update, dim3(n), dim3(256), 0, s, P.self, k);
}
void launch_cholesky(const DevProblem& P, int max_tiles, hipStream_t s) {
  for (int k = 0; k < max_tiles; ++k) {
    launch_chol_panel(P, k, s);
    launch_chol_update(P, k, s);
  }
}

void launch_trsv(const DevProblem& P, hipStream_t s) {
  if (P.max_fpad > 0) hipLaunchKernelGGL(k_trsv, dim3(P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P.self);
}

}  // namespace okg
