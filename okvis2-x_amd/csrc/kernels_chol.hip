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

__device__ __forceinline__ double readlaneD(double v, int lane) {  // v of `lane`, wave-uniform
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 16x16 block product on one wavefront: acc += sign * A(16 x 16K) B(16K x 16) with
// A[m][k] = a[m * lda + k], B[k][n] = b[k * ldbk + n * ldbn] (LDS), result in the MFMA C layout.
template <int KB>
__device__ __forceinline__ void mfma16(const double* a, int lda, const double* b, int ldbk, int ldbn, double sign,
                                       dbl4& acc, int lane) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int q = 0; q < 4 * KB; ++q) {
    const double av = sign * a[lr * lda + 4 * q + lk];
    const double bv = b[(4 * q + lk) * ldbk + lr * ldbn];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
}
__device__ __forceinline__ dbl4 loadC16(const double* c, int ldc, int lane) {
  dbl4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = c[((lane >> 4) + 4 * r) * ldc + (lane & 15)];
  return v;
}
__device__ __forceinline__ void storeC16(double* c, int ldc, const dbl4& v, int lane) {
#pragma unroll
  for (int r = 0; r < 4; ++r) c[((lane >> 4) + 4 * r) * ldc + (lane & 15)] = v[r];
}

// Diagonal tile k of every active window: L_kk (into S), X = L_kk^-1 (into Linv) and the forward
// substitution y_k = X work_k. One workgroup (4 wavefronts) per window, tile staged in LDS.
// Blocked right-looking LLT with 16-column panels (Eigen::LLT semantics: fail at the first
// non-positive pivot):
//   panel p   wavefront 0, lane = row i >= 16p holding its 16 panel entries in registers; the 16
//             column steps broadcast pivots and column entries with v_readlane (no barriers)
//   update p  A22 -= L21 L21^T on the matrix cores (v_mfma_f64_16x16x4_f64), 16x16 output blocks
//             spread over the 4 wavefronts
// then X = L^-1 blockwise: the 4 diagonal 16x16 inverses in parallel (one per wavefront), and
// X_ij = -X_ii (sum_{m=j}^{i-1} L_im X_mj) by sub-diagonal on the matrix cores.
__global__ __launch_bounds__(256) void k_potrf_inv(const DevProblem* __restrict__ Pp, int k) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  if (!cholSelect(P, w)) return;
  const int ld = P.win_fpad[w];
  const int T = ld / kTile;
  if (k >= T) return;
  double* Sg = P.S + P.win_soff[w] + (int64_t)k * kTile * ld + k * kTile;  // tile origin
  double* work = P.fwdF + P.win_fwdoff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sy[kTile];
  __shared__ int sFail;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  if (k == 0)  // start of the factorisation: work = rhs (zero-padded)
    for (int e = t; e < ld; e += 256) work[e] = (e < P.win_fdim[w]) ? P.rhsF[(size_t)P.win_foff[w] + e] : 0.0;
  for (int e = t; e < kTile * kTile; e += 256) {
    const int r = e >> 6, c = e & 63;
    sA[r * kLd + c] = Sg[(int64_t)r * ld + c];
    sX[r * kLd + c] = 0.0;
  }
  if (t == 0) sFail = 0;
  __syncthreads();
  if (t < kTile) sy[t] = work[k * kTile + t];
  for (int p = 0; p < 4; ++p) {
    // ---- panel p: columns [16p, 16p + 16), rows >= 16p, wavefront 0
    if (wave == 0) {
      const int i = lane;
      double a[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) a[c] = sA[i * kLd + 16 * p + c];
      bool bad = false;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int col = 16 * p + c;
        const double dcc = readlaneD(a[c], col);
        if (!(dcc > 0.0)) bad = true;  // wave-uniform
        const double rl = 1.0 / sqrt(dcc);
        const double l = (i == col) ? dcc * rl : a[c] * rl;
        a[c] = l;
#pragma unroll
        for (int j = c + 1; j < 16; ++j) a[j] -= l * readlaneD(l, 16 * p + j);
      }
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (i >= 16 * p + c) sA[i * kLd + 16 * p + c] = a[c];
      if (bad && lane == 0) sFail = 1;
    }
    __syncthreads();
    if (sFail) break;
    // ---- trailing update of the blocks (rb, cb), p < cb <= rb < 4
    {
      int idx = 0;
      for (int rb = p + 1; rb < 4; ++rb)
        for (int cb = p + 1; cb <= rb; ++cb, ++idx) {
          if ((idx & 3) != wave) continue;
          double* C = sA + 16 * rb * kLd + 16 * cb;
          dbl4 acc = loadC16(C, kLd, lane);
          // acc -= L[rb, p] L[cb, p]^T : B[k][n] = L[16cb + n][16p + k]
          mfma16<1>(sA + 16 * rb * kLd + 16 * p, kLd, sA + 16 * cb * kLd + 16 * p, 1, kLd, -1.0, acc, lane);
          storeC16(C, kLd, acc, lane);
        }
    }
    __syncthreads();
  }
  if (sFail) {
    if (t == 0) P.st[w].gn_failed = 1;
    return;
  }
  // ---- X = L^-1: diagonal 16x16 blocks, one per wavefront (lanes 0..15 = columns)
  {
    const int q = wave, j = lane;
    if (j < 16) {
      double x[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        double v = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int m = 0; m < i; ++m) v -= sA[(16 * q + i) * kLd + 16 * q + m] * x[m];
        x[i] = (i >= j) ? v / sA[(16 * q + i) * kLd + 16 * q + i] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) sX[(16 * q + i) * kLd + 16 * q + j] = x[i];
    }
  }
  __syncthreads();
  // ---- off-diagonal blocks by sub-diagonal d: X_ij = -X_ii (sum_{m=j}^{i-1} L_im X_mj), i = j + d
  for (int d = 1; d < 4; ++d) {
    const int j = wave, i = wave + d;
    if (i < 4) {
      dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
      for (int m = j; m < i; ++m)  // T = sum L_im X_mj   (B[k][n] = X[16m + k][16j + n])
        mfma16<1>(sA + 16 * i * kLd + 16 * m, kLd, sX + 16 * m * kLd + 16 * j, kLd, 1, 1.0, acc, lane);
      double* Xij = sX + 16 * i * kLd + 16 * j;
      storeC16(Xij, kLd, acc, lane);  // T staged in the (i, j) block (this wavefront only)
      dbl4 x = dbl4{0.0, 0.0, 0.0, 0.0};
      mfma16<1>(sX + 16 * i * kLd + 16 * i, kLd, Xij, kLd, 1, -1.0, x, lane);
      storeC16(Xij, kLd, x, lane);
    }
    __syncthreads();
  }
  // ---- L_kk back into S (lower), X into the inverse store, forward substitution y_k = X work_k
  double* Li = P.Linv + P.win_linvoff[w] + (int64_t)k * kTile * kTile;
  for (int e = t; e < kTile * kTile; e += 256) {
    const int r = e >> 6, c = e & 63;
    if (c <= r) Sg[(int64_t)r * ld + c] = sA[r * kLd + c];
    Li[e] = (c <= r) ? sX[r * kLd + c] : 0.0;
  }
  if (t < kTile) {
    double y = 0.0;
    for (int j = 0; j <= t; ++j) y += sX[t * kLd + j] * sy[j];
    work[k * kTile + t] = y;
  }
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
