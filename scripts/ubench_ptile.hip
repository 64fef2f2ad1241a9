// Development micro-benchmark: okg::potrfTile<1> (the diagonal tile of the Cholesky: LLT, X = L^-1,
// y = X rhs) on one 256-thread workgroup, isolated (1 workgroup) and under load (2 per CU).
// Phase cuts: build with -DOKG_POTRF_STOP=n (1 sweep, 2 + X21, 3 + sub-diagonals, 4 + X store).
// hipcc --offload-arch=gfx950 -O3 -I include scripts/ubench_ptile.hip -o scripts/ubench_ptile
#include "../okvis2-x_amd/csrc/kernels_chol.hip"

#include <cstdio>
#include <cmath>
#include <vector>

__global__ __launch_bounds__(256, 2) void kptile(const double* A, double* Li, double* work, int reps,
                                                 unsigned long long* ticks) {
  __shared__ double sA[okg::kTile * okg::kLd];
  __shared__ double sX[okg::kTile * okg::kLd];
  __shared__ double sy[2 * okg::kTile];
  __shared__ double sRl[okg::kTile];
  __shared__ int sFl[4];
  const int t = threadIdx.x;
  unsigned long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    if (t < 64) sy[t] = 1.0 + t;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    okg::potrfTile<1>(const_cast<double*>(A), 64, Li + (size_t)blockIdx.x * 4096, work + (size_t)blockIdx.x * 64, sA, sX,
                      sy, sRl, sFl, t, false);
    __syncthreads();
    tot += __builtin_amdgcn_s_memrealtime() - t0;
  }
  if (t == 0) ticks[blockIdx.x] = tot;
}

int main() {
  std::vector<double> A(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) A[i * 64 + j] = 1.0 / (1.0 + i + j) + ((i == j) ? 4.0 + 0.1 * i : 0.0);
  const int nb = 512, reps = 200;
  double *dA, *dL, *dW;
  unsigned long long* dT;
  (void)hipMalloc(&dA, 8 * 4096);
  (void)hipMalloc(&dL, 8 * 4096 * (size_t)nb);
  (void)hipMalloc(&dW, 8 * 64 * (size_t)nb);
  (void)hipMalloc(&dT, 8 * nb);
  (void)hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  for (int cfg = 0; cfg < 2; ++cfg) {
    const int blocks = cfg == 0 ? 1 : nb;
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(kptile, blocks, 256, 0, 0, dA, dL, dW, reps, dT);
      (void)hipDeviceSynchronize();
    }
    std::vector<unsigned long long> t(blocks);
    (void)hipMemcpy(t.data(), dT, 8 * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (int b = 0; b < blocks; ++b) s += (double)t[b];
    printf("%s blocks %4d: %.3f us per tile\n", OKG_TAG, blocks, s / blocks * 10.0 / 1000.0 / reps);
  }
  // check: X L = I on the first block's X (L from a host LLT)
  std::vector<double> X(4096), L(4096, 0.0);
  (void)hipMemcpy(X.data(), dL, 8 * 4096, hipMemcpyDeviceToHost);
  for (int j = 0; j < 64; ++j) {
    double d = A[j * 64 + j];
    for (int k = 0; k < j; ++k) d -= L[j * 64 + k] * L[j * 64 + k];
    L[j * 64 + j] = std::sqrt(d);
    for (int i = j + 1; i < 64; ++i) {
      double v = A[i * 64 + j];
      for (int k = 0; k < j; ++k) v -= L[i * 64 + k] * L[j * 64 + k];
      L[i * 64 + j] = v / L[j * 64 + j];
    }
  }
  double err = 0;
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      double v = 0;
      for (int k = 0; k < 64; ++k) v += X[i * 64 + k] * L[k * 64 + j];
      err = std::fmax(err, std::fabs(v - (i == j ? 1.0 : 0.0)));
    }
  printf("%s max |X L - I| = %.2e\n", OKG_TAG, err);
#ifdef OKG_SWEEP_TRACE
  hipLaunchKernelGGL(kptile, 1, 256, 0, 0, dA, dL, dW, 1, dT);
  (void)hipDeviceSynchronize();
  unsigned long long T[2][8][8];
  (void)hipMemcpyFromSymbol(T, HIP_SYMBOL(okg::g_sweepT), sizeof(T));
  const unsigned long long b = T[0][0][0];
  printf("sweep timeline (s_memtime ticks from sub-panel 0 start)\n"
         "  s | w0: start  waited  lookahd  chol8  stored | w1: got  inv8  trail  wbar  xdiag  xoff  ystore\n");
  for (int s = 0; s < 8; ++s) {
    printf("  %d |", s);
    for (int i = 0; i < 5; ++i) printf(" %7lld", (long long)(T[0][s][i] - b));
    printf(" |");
    for (int i = 0; i < 7; ++i) printf(" %7lld", (s & 1) || i < 4 ? (long long)(T[1][s][i] - b) : 0LL);
    printf("\n");
  }
#endif
  return 0;
}
