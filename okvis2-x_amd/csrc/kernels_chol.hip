// kernels_chol.hip — dense LLT of the reduced camera matrix S (Eigen::LLT semantics: fail at the
// first non-positive pivot) and the two triangular solves, batched over windows (blockIdx.y).
//
// Right-looking blocked Cholesky with 64x64 FP64 tiles:
//   k_chol_panel(k)   one workgroup per tile row i >= k of panel k: factor the diagonal tile in LDS
//                     (every workgroup redundantly, so the panel needs no extra launch) and solve
//                     L_ik = A_ik L_kk^-T.
//   k_chol_update(k)  one workgroup per trailing tile (i, j), k < j <= i:
//                     A_ij -= L_ik L_jk^T — the dense reduced-camera block multiply, on the FP64
//                     matrix cores (v_mfma_f64_16x16x4_f64): each of the 4 wavefronts owns a 32x32
//                     quarter of the output tile (2x2 MFMA tiles), K = 64 in steps of 4.
//   k_trsv            one workgroup per window: L u = rhs, L^T y = u with the vector in LDS.
#include "device_problem.hpp"
#include "launch.hpp"

namespace okg {

constexpr int kLd = kTile + 1;  // padded LDS row (65 doubles): conflict-free column walks

__device__ __forceinline__ bool cholSelect(const DevProblem& P, int w) {
  const WinState& s = P.st[w];
  return !s.done && s.need_gn && !s.gn_failed;
}

// In-LDS factorisation of a 64x64 SPD tile (lower). Returns false on a non-positive pivot.
__device__ bool factorTile(double* L, int t, int nthreads, int* sflag) {
  if (t == 0) *sflag = 0;
  __syncthreads();
  for (int c = 0; c < kTile; ++c) {
    if (t == 0) {
      const double d = L[c * kLd + c];
      if (!(d > 0.0)) *sflag = 1;
      else L[c * kLd + c] = sqrt(d);
    }
    __syncthreads();
    if (*sflag) return false;
    const double dc = L[c * kLd + c];
    for (int r = c + 1 + t; r < kTile; r += nthreads) L[r * kLd + c] /= dc;
    __syncthreads();
    const int m = kTile - 1 - c;
    for (int e = t; e < m * m; e += nthreads) {
      const int i = c + 1 + e / m, j = c + 1 + e % m;
      if (j <= i) L[i * kLd + j] -= L[i * kLd + c] * L[j * kLd + c];
    }
    __syncthreads();
  }
  return true;
}

__global__ __launch_bounds__(256) void k_chol_panel(DevProblem P, int k) {
  const int w = blockIdx.y;
  if (!cholSelect(P, w)) return;
  const int T = P.win_fpad[w] / kTile;
  const int i = k + blockIdx.x;
  if (k >= T || i >= T) return;
  const int ld = P.win_fpad[w];
  double* A = P.S + P.win_soff[w];
  __shared__ double Lkk[kTile * kLd];
  __shared__ double X[kTile * kLd];
  __shared__ int flag;
  const int t = threadIdx.x;
  for (int e = t; e < kTile * kTile; e += 256) {
    const int r = e / kTile, c = e % kTile;
    Lkk[r * kLd + c] = A[(int64_t)(k * kTile + r) * ld + k * kTile + c];
  }
  __syncthreads();
  if (!factorTile(Lkk, t, 256, &flag)) {
    if (t == 0) P.st[w].gn_failed = 1;
    return;
  }
  if (i == k) {
    for (int e = t; e < kTile * kTile; e += 256) {
      const int r = e / kTile, c = e % kTile;
      if (c <= r) A[(int64_t)(k * kTile + r) * ld + k * kTile + c] = Lkk[r * kLd + c];
    }
    return;
  }
  for (int e = t; e < kTile * kTile; e += 256) {
    const int r = e / kTile, c = e % kTile;
    X[r * kLd + c] = A[(int64_t)(i * kTile + r) * ld + k * kTile + c];
  }
  __syncthreads();
  // X L^T = A  (right-looking over columns)
  for (int c = 0; c < kTile; ++c) {
    const double dc = Lkk[c * kLd + c];
    if (t < kTile) X[t * kLd + c] /= dc;
    __syncthreads();
    const int m = kTile - 1 - c;
    for (int e = t; e < kTile * m; e += 256) {
      const int r = e / m, j = c + 1 + e % m;
      X[r * kLd + j] -= X[r * kLd + c] * Lkk[j * kLd + c];
    }
    __syncthreads();
  }
  for (int e = t; e < kTile * kTile; e += 256) {
    const int r = e / kTile, c = e % kTile;
    A[(int64_t)(i * kTile + r) * ld + k * kTile + c] = X[r * kLd + c];
  }
}

typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_chol_update(DevProblem P, int k) {
  const int w = blockIdx.y;
  if (!cholSelect(P, w)) return;
  const int T = P.win_fpad[w] / kTile;
  const int m = T - k - 1;
  if (m <= 0) return;
  const int b = blockIdx.x;
  if (b >= m * (m + 1) / 2) return;
  int ii = (int)((sqrt(8.0 * b + 1.0) - 1.0) * 0.5);
  while (ii * (ii + 1) / 2 > b) --ii;
  while ((ii + 1) * (ii + 2) / 2 <= b) ++ii;
  const int jj = b - ii * (ii + 1) / 2;
  const int i = k + 1 + ii, j = k + 1 + jj;
  const int ld = P.win_fpad[w];
  double* A = P.S + P.win_soff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sB[kTile * kLd];
  const int t = threadIdx.x;
  for (int e = t; e < kTile * kTile; e += 256) {
    const int r = e / kTile, c = e % kTile;
    sA[r * kLd + c] = A[(int64_t)(i * kTile + r) * ld + k * kTile + c];
    sB[r * kLd + c] = A[(int64_t)(j * kTile + r) * ld + k * kTile + c];
  }
  __syncthreads();
  // wave q owns rows 32*(q>>1).., cols 32*(q&1)..; 2x2 MFMA 16x16 tiles.
  const int wave = t >> 6, lane = t & 63;
  const int r0 = 32 * (wave >> 1), c0 = 32 * (wave & 1);
  dbl4 acc[2][2];
  for (int a = 0; a < 2; ++a)
    for (int bb = 0; bb < 2; ++bb) acc[a][bb] = dbl4{0.0, 0.0, 0.0, 0.0};
  // v_mfma_f64_16x16x4_f64: A operand lane l -> A[row l&15][k l>>4], B operand -> B[k l>>4][col l&15]
  const int lr = lane & 15, lk = lane >> 4;
  for (int kk = 0; kk < kTile; kk += 4) {
    double av[2], bv[2];
    for (int a = 0; a < 2; ++a) av[a] = sA[(r0 + 16 * a + lr) * kLd + kk + lk];
    for (int bb = 0; bb < 2; ++bb) bv[bb] = sB[(c0 + 16 * bb + lr) * kLd + kk + lk];  // (L_jk^T)[k][col]
    for (int a = 0; a < 2; ++a)
      for (int bb = 0; bb < 2; ++bb) acc[a][bb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[bb], acc[a][bb], 0, 0, 0);
  }
  // C/D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * reg
  for (int a = 0; a < 2; ++a)
    for (int bb = 0; bb < 2; ++bb)
      for (int reg = 0; reg < 4; ++reg) {
        const int rr = r0 + 16 * a + (lane >> 4) + 4 * reg;
        const int cc = c0 + 16 * bb + (lane & 15);
        A[(int64_t)(i * kTile + rr) * ld + j * kTile + cc] -= acc[a][bb][reg];
      }
}

// L u = rhs ; L^T y = u   (y kept in LDS; dynamic shared memory = fpad doubles)
__global__ __launch_bounds__(256) void k_trsv(DevProblem P) {
  const int w = blockIdx.x;
  if (!cholSelect(P, w)) return;
  extern __shared__ double y[];
  __shared__ double part[4 * kTile];
  const int ld = P.win_fpad[w], fdim = P.win_fdim[w], foff = P.win_foff[w];
  const int T = ld / kTile;
  const double* A = P.S + P.win_soff[w];
  const int t = threadIdx.x;
  for (int e = t; e < ld; e += 256) y[e] = (e < fdim) ? P.rhsF[(size_t)foff + e] : 0.0;
  __syncthreads();
  // forward
  for (int I = 0; I < T; ++I) {
    const int row = t >> 2, q = t & 3;
    double acc = 0.0;
    const double* Ar = A + (int64_t)(I * kTile + row) * ld;
    for (int j = q; j < I * kTile; j += 4) acc += Ar[j] * y[j];
    part[q * kTile + row] = acc;
    __syncthreads();
    if (t < kTile) y[I * kTile + t] -= part[t] + part[kTile + t] + part[2 * kTile + t] + part[3 * kTile + t];
    __syncthreads();
    for (int c = 0; c < kTile; ++c) {
      const int gc = I * kTile + c;
      if (t == 0) y[gc] /= A[(int64_t)gc * ld + gc];
      __syncthreads();
      const double yc = y[gc];
      if (t > c && t < kTile) y[I * kTile + t] -= A[(int64_t)(I * kTile + t) * ld + gc] * yc;
      __syncthreads();
    }
  }
  // backward
  for (int I = T - 1; I >= 0; --I) {
    const int col = t & 63, q = t >> 6;
    double acc = 0.0;
    for (int r = (I + 1) * kTile + q; r < ld; r += 4) acc += A[(int64_t)r * ld + I * kTile + col] * y[r];
    part[q * kTile + col] = acc;
    __syncthreads();
    if (t < kTile) y[I * kTile + t] -= part[t] + part[kTile + t] + part[2 * kTile + t] + part[3 * kTile + t];
    __syncthreads();
    for (int c = kTile - 1; c >= 0; --c) {
      const int gc = I * kTile + c;
      if (t == 0) y[gc] /= A[(int64_t)gc * ld + gc];
      __syncthreads();
      const double yc = y[gc];
      if (t < c) y[I * kTile + t] -= A[(int64_t)gc * ld + I * kTile + t] * yc;
      __syncthreads();
    }
  }
  for (int e = t; e < fdim; e += 256) P.yF[(size_t)foff + e] = y[e];
}

void launch_chol_panel(const DevProblem& P, int k, hipStream_t s) {
  hipLaunchKernelGGL(k_chol_panel, dim3(P.max_tiles - k, P.n_win), dim3(256), 0, s, P, k);
}
void launch_chol_update(const DevProblem& P, int k, hipStream_t s) {
  const int m = P.max_tiles - k - 1;
  if (m > 0) hipLaunchKernelGGL(k_chol_update, dim3(m * (m + 1) / 2, P.n_win), dim3(256), 0, s, P, k);
}
void launch_cholesky(const DevProblem& P, int max_tiles, hipStream_t s) {
  for (int k = 0; k < max_tiles; ++k) {
    launch_chol_panel(P, k, s);
    launch_chol_update(P, k, s);
  }
}

void launch_trsv(const DevProblem& P, hipStream_t s) {
  if (P.max_fpad > 0) hipLaunchKernelGGL(k_trsv, dim3(P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P);
}

}  // namespace okg
