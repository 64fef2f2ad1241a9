// kernels_chol.hip — dense LLT of the reduced camera matrix S (Eigen::LLT semantics: fail at the
// first non-positive pivot) and the two triangular solves. Two schedules of the same tile
// routines: one persistent workgroup per window (large batches: fills the chip with whole
// windows) or per-step launches over all windows' panel / band-update tiles (few windows:
// spreads each window over many CUs); launch_cholesky picks the host-resolved one.
//
// k_cholesky: right-looking blocked Cholesky over 64x64 FP64 tiles, only structurally non-zero
// tiles (the host's tile-level symbolic factorisation, DevProblem::tile_nz: the reduced camera
// matrix of a sliding window is block-banded and LLT creates no fill outside its envelope, so
// skipping zero tiles is exact). Per step k, inside one workgroup:
//   diagonal  L_kk and X = L_kk^-1 (16-column register panels with v_readlane broadcasts, MFMA
//             trailing updates, blockwise inverse), fused forward substitution y_k = X rhs_k
//   panel     L_ik = A_ik X^T for every non-zero tile below (64x64x64 on the FP64 matrix cores)
//             and rhs_i -= L_ik y_k
//   update    A_ij -= L_ik L_jk^T for the non-zero tiles of the trailing band (matrix cores;
//             operands staged in LDS, freshly written tiles come back from L2)
// then the backward substitution x = L^-T y with the stored diagonal inverses.
//
// MFMA tile: each of the 4 wavefronts owns a 32x32 quarter of the 64x64 output (2x2 16x16 MFMA
// tiles), K = 64 in steps of 4. v_mfma_f64_16x16x4_f64 operand map: lane l supplies A[l&15][l>>4]
// and B[l>>4][l&15]; result reg r of lane l is C[(l>>4) + 4r][l&15] (cdna_hip_programming.md §3).
#include "device_problem.hpp"
#include "launch.hpp"

namespace okg {

constexpr int kLd = kTile + 1;  // padded LDS row (65 doubles)

// Development-only phase clock (make OPT="-O3 -DOKG_CHOL_CLOCK"): workgroup 0 of k_cholesky
// accumulates s_memrealtime ticks (100 MHz) per phase and prints them.
#ifdef OKG_CHOL_CLOCK
__device__ unsigned long long g_cholClk[16];
#define CLK_INIT unsigned long long clkLast = __builtin_amdgcn_s_memrealtime();
#define CLK(i)                                                                  \
  if (blockIdx.x == 0 && threadIdx.x == 0) {                                    \
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();            \
    g_cholClk[i] += now - clkLast;                                              \
    clkLast = now;                                                              \
  }
#else
#define CLK_INIT
#define CLK(i)
#endif

typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool cholSelect(const DevProblem& P, int w) {
  const WinState& s = P.st[w];
  return !s.done && s.need_gn && !s.gn_failed;
}

// 64x64 global tile (row stride ld) -> LDS [64][kLd]: all 8 16-byte loads of a thread are issued
// before the LDS stores.
__device__ __forceinline__ void loadTile(const double* A, int64_t ld, int r0, int c0, double* s, int t) {
  double2 v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = t + 256 * u, r = e >> 5, c = 2 * (e & 31);
    v[u] = *reinterpret_cast<const double2*>(A + (int64_t)(r0 + r) * ld + c0 + c);
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = t + 256 * u, r = e >> 5, c = 2 * (e & 31);
    s[r * kLd + c] = v[u].x;
    s[r * kLd + c + 1] = v[u].y;
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

// 1/sqrt(d) to ~1 ulp: v_rsq_f64 (~5e-8 relative) refined by two Newton steps (measured on
// gfx950: 2.3e-16 max relative error over d in [e^-40, e^40]).
__device__ __forceinline__ double rsqrtRefined(double d) {
  double r = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  r = r * (1.5 - h * r * r);
  r = r * (1.5 - h * r * r);
  return r;
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

// Diagonal tile: L_kk (into S, lower), X = L_kk^-1 (into sX and the Linv store) and y_k = X rhs_k
// (sy holds rhs_k on entry, y_k on exit; also written to work). Blocked right-looking LLT with
// 16-column panels:
//   panel p   wavefront 0, lane = row i >= 16p holding its 16 panel entries in registers; the 16
//             column steps broadcast pivots and column entries with v_readlane (no barriers)
//   update p  A22 -= L21 L21^T on the matrix cores, 16x16 output blocks over the 4 wavefronts
// then X blockwise: the 4 diagonal 16x16 inverses in parallel (one per wavefront), and
// X_ij = -X_ii (sum_{m=j}^{i-1} L_im X_mj) by sub-diagonal on the matrix cores.
// Returns false (uniformly) at a non-positive pivot.
// (one non-inlined instantiation per calling kernel: a shared callee gets a generic register
// budget that halves the persistent kernel's occupancy)
template <int kCaller>
__device__ __noinline__ bool potrfTile(double* Sg, int64_t ld, double* Li, double* workk, double* sA, double* sX, double* sy,
                                      double* sRl, int* sFail, int t) {
  const int wave = t >> 6, lane = t & 63;
  CLK_INIT
  loadTile(Sg, ld, 0, 0, sA, t);
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = t + 256 * u;
    sX[(e >> 6) * kLd + (e & 63)] = 0.0;
  }
  if (t == 0) *sFail = 0;
  __syncthreads();
  CLK(4)
  for (int p = 0; p < 4; ++p) {
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
        const double rl = rsqrtRefined(dcc);
        if (lane == 0) sRl[col] = rl;  // 1 / L_cc for the inverse
        const double l = (i == col) ? dcc * rl : a[c] * rl;
        a[c] = l;
#pragma unroll
        for (int j = c + 1; j < 16; ++j) a[j] -= l * readlaneD(l, 16 * p + j);
      }
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (i >= 16 * p + c) sA[i * kLd + 16 * p + c] = a[c];
      if (bad && lane == 0) *sFail = 1;
    }
    __syncthreads();
    CLK(5)
    if (*sFail) return false;
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
    __syncthreads();
    CLK(6)
  }
  if (lane < 16) {  // diagonal 16x16 inverses, wavefront q, lane = column
    const int q = wave, j = lane;
    double x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      double v = (i == j) ? 1.0 : 0.0;
#pragma unroll
      for (int m = 0; m < i; ++m) v -= sA[(16 * q + i) * kLd + 16 * q + m] * x[m];
      x[i] = (i >= j) ? v * sRl[16 * q + i] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) sX[(16 * q + i) * kLd + 16 * q + j] = x[i];
  }
  __syncthreads();
  CLK(7)
  for (int d = 1; d < 4; ++d) {  // sub-diagonal d: X_ij, i = j + d, wavefront j
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
  CLK(8)
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = t + 256 * u, r = e >> 5, c = 2 * (e & 31);
    if (c <= r) Sg[(int64_t)r * ld + c] = sA[r * kLd + c];
    if (c + 1 <= r) Sg[(int64_t)r * ld + c + 1] = sA[r * kLd + c + 1];
    *reinterpret_cast<double2*>(Li + r * kTile + c) =
        double2{(c <= r) ? sX[r * kLd + c] : 0.0, (c + 1 <= r) ? sX[r * kLd + c + 1] : 0.0};
  }
  __syncthreads();
  CLK(9)
  {  // y_k = X rhs_k: row t & 63, quarter t >> 6 of the columns, partials through LDS
    const int row = t & 63, qq = t >> 6;
    double y = 0.0;
#pragma unroll
    for (int j = 16 * qq; j < 16 * qq + 16; ++j) y += (j <= row) ? sX[row * kLd + j] * sy[j] : 0.0;
    sA[qq * kTile + row] = y;  // sA is free once L_kk has been stored
  }
  __syncthreads();
  if (t < kTile) {
    const double y = (sA[t] + sA[kTile + t]) + (sA[2 * kTile + t] + sA[3 * kTile + t]);
    sy[t] = y;
    workk[t] = y;
  }
  __syncthreads();
  CLK(10)
  return true;
}

// L_ik = A_ik X^T (X = L_kk^-1 in sX, y_k in sy) stored over A_ik, and rhs_i -= L_ik y_k.
__device__ void panelTile(double* Aik, int64_t ld, double* worki, double* sA, const double* sX, const double* sy,
                          int t) {
  loadTile(Aik, ld, 0, 0, sA, t);
  __syncthreads();
  dbl4 acc[2][2];
  mfmaTileNT(sA, sX, acc, t);
  __syncthreads();
  storeTile<false>(Aik, ld, 0, 0, acc, t);
  storeTile<false>(sA, kLd, 0, 0, acc, t);  // L_ik staged for the rhs update
  __syncthreads();
  if (t < kTile) {
    double a = 0.0;
    for (int c = 0; c < kTile; ++c) a += sA[t * kLd + c] * sy[c];
    worki[t] -= a;
  }
  __syncthreads();
}

// Backward substitution x = L^-T y (work holds y), x := y_F. x lives in LDS (sx, ld doubles);
// per block row I the 16 row loads of every non-zero tile below are issued together, then
// x_I = X_II^T (y_I - sum_i L_iI^T x_i) with the stored diagonal inverse.
__device__ void backSubstitute(const DevProblem& P, int w, const double* S, int64_t ld, int T, const double* work,
                               const double* Linv, const uint8_t* nz, double* sx, double* sA, double* sy, int t) {
  for (int e = t; e < ld; e += 256) sx[e] = work[e];
  __syncthreads();
  const int col = t & 63, q = t >> 6;
  for (int I = T - 1; I >= 0; --I) {
    double acc = 0.0;
    for (int i = I + 1; i < T; ++i) {
      if (!nz[i * T + I]) continue;
      const double* Lt = S + i * kTile * ld + I * kTile + col;
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = Lt[(int64_t)(q + 4 * u) * ld];
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u] * sx[i * kTile + q + 4 * u];
    }
    const double* Li = Linv + (int64_t)I * kTile * kTile + col;
    double li[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) li[u] = Li[(q + 4 * u) * kTile];
    sA[q * kTile + col] = acc;
    __syncthreads();
    if (t < kTile) sy[t] = sx[I * kTile + t] - ((sA[t] + sA[kTile + t]) + (sA[2 * kTile + t] + sA[3 * kTile + t]));
    __syncthreads();
    double a = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) a += (q + 4 * u >= col) ? li[u] * sy[q + 4 * u] : 0.0;
    sA[256 + q * kTile + col] = a;
    __syncthreads();
    if (t < kTile)
      sx[I * kTile + t] = (sA[256 + t] + sA[256 + kTile + t]) + (sA[256 + 2 * kTile + t] + sA[256 + 3 * kTile + t]);
    __syncthreads();
  }
  const int fdim = P.win_fdim[w];
  for (int e = t; e < fdim; e += 256) P.yF[(size_t)P.win_foff[w] + e] = sx[e];
}

__global__ __launch_bounds__(256) void k_cholesky(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  const int T = (int)(ld / kTile);
  double* S = P.S + P.win_soff[w];
  double* work = P.fwdF + P.win_fwdoff[w];
  double* Linv = P.Linv + P.win_linvoff[w];
  const uint8_t* nz = P.tile_nz + P.win_tnzoff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sy[2 * kTile];  // y_k | panel column scratch
  __shared__ double sRl[kTile];
  __shared__ int sFail;
  const int t = threadIdx.x;
  const int fdim = P.win_fdim[w];
  CLK_INIT
  for (int e = t; e < ld; e += 256) work[e] = (e < fdim) ? P.rhsF[(size_t)P.win_foff[w] + e] : 0.0;
  __syncthreads();
  for (int k = 0; k < T; ++k) {
    CLK(11)
    if (t < kTile) sy[t] = work[k * kTile + t];
    __syncthreads();
    if (!potrfTile<0>(S + k * kTile * ld + k * kTile, ld, Linv + (int64_t)k * kTile * kTile, work + k * kTile, sA, sX,
                   sy, sRl, &sFail, t)) {
      if (t == 0) P.st[w].gn_failed = 1;
      return;
    }
    CLK(0)
    // ---- panel: L_ik = A_ik X^T, rhs_i -= L_ik y_k
    for (int i = k + 1; i < T; ++i)
      if (nz[i * T + k]) panelTile(S + i * kTile * ld + k * kTile, ld, work + i * kTile, sA, sX, sy, t);
    CLK(1)
    // ---- trailing band update: A_ij -= L_ik L_jk^T, k < j <= i, both tiles non-zero
    for (int i = k + 1; i < T; ++i) {
      if (!nz[i * T + k]) continue;
      loadTile(S + i * kTile * ld + k * kTile, ld, 0, 0, sA, t);
      for (int j = k + 1; j <= i; ++j) {
        if (!nz[j * T + k]) continue;
        if (j != i) loadTile(S + j * kTile * ld + k * kTile, ld, 0, 0, sX, t);
        __syncthreads();
        dbl4 acc[2][2];
        mfmaTileNT(sA, j == i ? sA : sX, acc, t);
        storeTile<true>(S + i * kTile * ld + j * kTile, ld, 0, 0, acc, t);
        __syncthreads();
      }
    }
  }
  CLK(2)
  extern __shared__ double sxDyn[];
  backSubstitute(P, w, S, ld, T, work, Linv, nz, sxDyn, sA, sy, t);
  CLK(3)
#ifdef OKG_CHOL_CLOCK
  if (blockIdx.x == 0 && t == 0)
    printf("CHOLCLK T=%d potrf %llu panel %llu update %llu bsub %llu | load %llu pfac %llu ptrail %llu dinv %llu subd %llu store %llu y %llu (x10ns)\n",
           T, g_cholClk[0], g_cholClk[1], g_cholClk[2] + g_cholClk[11], g_cholClk[3], g_cholClk[4], g_cholClk[5], g_cholClk[6],
           g_cholClk[7], g_cholClk[8], g_cholClk[9], g_cholClk[10]);
#endif
}

// ---- tile-parallel schedule: per step k one launch each for the diagonal tiles, the panel tiles
// and the band updates of all windows (many workgroups per window), then the backward solves.
__global__ __launch_bounds__(256) void k_chol_diag(const DevProblem* __restrict__ Pp, int k) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  const int T = (int)(ld / kTile);
  if (k >= T) return;
  double* S = P.S + P.win_soff[w];
  double* work = P.fwdF + P.win_fwdoff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sy[2 * kTile];
  __shared__ double sRl[kTile];
  __shared__ int sFail;
  const int t = threadIdx.x;
  if (k == 0) {
    const int fdim = P.win_fdim[w];
    for (int e = t; e < ld; e += 256) work[e] = (e < fdim) ? P.rhsF[(size_t)P.win_foff[w] + e] : 0.0;
    __syncthreads();
  }
  if (t < kTile) sy[t] = work[k * kTile + t];
  __syncthreads();
  if (!potrfTile<1>(S + k * kTile * ld + k * kTile, ld, P.Linv + P.win_linvoff[w] + (int64_t)k * kTile * kTile,
                 work + k * kTile, sA, sX, sy, sRl, &sFail, t))
    if (t == 0) P.st[w].gn_failed = 1;
}

__global__ __launch_bounds__(256) void k_chol_panel(const DevProblem* __restrict__ Pp, int k) {
  const DevProblem& P = *Pp;
  const int item = P.chol_panel_begin[k] + blockIdx.x;
  const int w = P.chol_panel_items[2 * item], i = P.chol_panel_items[2 * item + 1];
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  double* work = P.fwdF + P.win_fwdoff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sy[kTile];
  const int t = threadIdx.x;
  const double* X = P.Linv + P.win_linvoff[w] + (int64_t)k * kTile * kTile;
  loadTile(X, kTile, 0, 0, sX, t);
  if (t < kTile) sy[t] = work[k * kTile + t];
  panelTile(P.S + P.win_soff[w] + i * kTile * ld + k * kTile, ld, work + i * kTile, sA, sX, sy, t);
}

// band updates of step k; the workgroup owning tile (k+1,k+1) factors it right after its update
// (mode bit 1), so the next diagonal overlaps the remaining updates of this step
__global__ __launch_bounds__(256) void k_chol_update(const DevProblem* __restrict__ Pp, int k) {
  const DevProblem& P = *Pp;
  const int item = P.chol_upd_begin[k] + blockIdx.x;
  const int4 it = reinterpret_cast<const int4*>(P.chol_upd_items)[item];
  const int w = it.x, i = it.y, j = it.z, mode = it.w;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  double* S = P.S + P.win_soff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sy[2 * kTile];
  __shared__ double sRl[kTile];
  __shared__ int sFail;
  const int t = threadIdx.x;
  if (mode & 1) {
    loadTile(S + i * kTile * ld + k * kTile, ld, 0, 0, sA, t);
    if (j != i) loadTile(S + j * kTile * ld + k * kTile, ld, 0, 0, sX, t);
    __syncthreads();
    dbl4 acc[2][2];
    mfmaTileNT(sA, j == i ? sA : sX, acc, t);
    storeTile<true>(S + i * kTile * ld + j * kTile, ld, 0, 0, acc, t);
  }
  if (!(mode & 2)) return;
  double* work = P.fwdF + P.win_fwdoff[w];
  const int d = k + 1;
  __syncthreads();
  if (t < kTile) sy[t] = work[d * kTile + t];
  __syncthreads();
  if (!potrfTile<2>(S + d * kTile * ld + d * kTile, ld, P.Linv + P.win_linvoff[w] + (int64_t)d * kTile * kTile,
                    work + d * kTile, sA, sX, sy, sRl, &sFail, t))
    if (t == 0) P.st[w].gn_failed = 1;
}

__global__ __launch_bounds__(256) void k_chol_bsub(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = blockIdx.x;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  __shared__ double sA[8 * kTile];
  __shared__ double sy[kTile];
  extern __shared__ double sxDyn[];
  backSubstitute(P, w, P.S + P.win_soff[w], ld, (int)(ld / kTile), P.fwdF + P.win_fwdoff[w],
                 P.Linv + P.win_linvoff[w], P.tile_nz + P.win_tnzoff[w], sxDyn, sA, sy, threadIdx.x);
}

void launch_cholesky(const DevProblem& P, hipStream_t s) {
  if (P.n_win == 0) return;
  if (P.chol_schedule == 1) {
    hipLaunchKernelGGL(k_cholesky, dim3(P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P.self);
    return;
  }
  hipLaunchKernelGGL(k_chol_diag, dim3(P.n_win), dim3(256), 0, s, P.self, 0);
  for (int k = 0; k < P.max_tiles; ++k) {
    const int np = P.h_panel_begin[k + 1] - P.h_panel_begin[k];
    if (np > 0) hipLaunchKernelGGL(k_chol_panel, dim3(np), dim3(256), 0, s, P.self, k);
    const int nu = P.h_upd_begin[k + 1] - P.h_upd_begin[k];
    if (nu > 0) hipLaunchKernelGGL(k_chol_update, dim3(nu), dim3(256), 0, s, P.self, k);
  }
  hipLaunchKernelGGL(k_chol_bsub, dim3(P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P.self);
}

}  // namespace okg
