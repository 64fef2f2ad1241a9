// Development micro-benchmark for a two-team persistent Cholesky: how much does the diagonal tile
// factor (okg::potrfTile in team mode, waves 0-3) slow down while the other four wavefronts of the
// workgroup (waves 4-7) run 64x64x64 FP64 MFMA tile products (band updates / panels) on the same
// CU? Modes: 0 team B idle, 1 team B busy, 2 team B busy and team F at s_setprio 3, 3 the product's
// 256-thread potrfTile alone (reference). One workgroup per CU (LDS ~134 KB) and one workgroup.
// hipcc --offload-arch=gfx950 -O3 -I include scripts/ubench_team.hip -o scripts/ubench_team
#include "../okvis2-x_amd/csrc/kernels_chol.hip"

#include <cmath>
#include <cstdio>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(512, 1) void kteam(const double* A, double* Li, double* work, const double* Bsrc,
                                                double* Bdst, int reps, unsigned long long* ticks,
                                                unsigned long long* bcount) {
  __shared__ double sA[okg::kTile * okg::kLd];
  __shared__ double sX[okg::kTile * okg::kLd];
  __shared__ double sB1[okg::kTile * okg::kLd];
  __shared__ double sB2[okg::kTile * okg::kLd];
  __shared__ double sy[2 * okg::kTile];
  __shared__ double sRl[okg::kTile];
  __shared__ int sFl[8];
  __shared__ int sDone;
  const int t = threadIdx.x, team = t >> 8, tt = t & 255, lane = t & 63;
  if (t < 8) sFl[t] = 0;
  if (t == 0) sDone = 0;
  __syncthreads();
  if (team == 0) {
    if (MODE == 2) __builtin_amdgcn_s_setprio(3);
    int gen = 0;
    unsigned long long tot = 0;
    for (int r = 0; r < reps; ++r) {
      if (tt < 64) sy[tt] = 1.0 + tt;
      okg::waveBarrier<true>(&sFl[4], gen, 4, lane);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      okg::potrfTile<21>(A, 64, Li + (size_t)blockIdx.x * 4096, nullptr, sA, sX, sy, sRl, sFl, tt, false, gen);
      gen += okg::kPotrfBarriers;
      tot += __builtin_amdgcn_s_memrealtime() - t0;
    }
    if (tt == 0) {
      ticks[blockIdx.x] = tot;
      __hip_atomic_store(&sDone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else if (MODE != 0) {
    // team B: stage two tiles once, then C = A B^T tile products stored to global until team F ends
    okg::loadTile(Bsrc, 64, 0, 0, sB1, tt);
    okg::loadTile(Bsrc + 4096, 64, 0, 0, sB2, tt);
    int gen = 0;
    okg::waveBarrier<false>(&sFl[5], gen, 4, lane);
    unsigned long long n = 0;
    while (__hip_atomic_load(&sDone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
      okg::dbl4 acc[2][2];
      okg::mfmaTileNT(sB1, sB2, acc, tt);
      okg::storeTile<false>(Bdst + (size_t)blockIdx.x * 4096, 64, 0, 0, acc, tt);
      ++n;
    }
    if (tt == 0) bcount[blockIdx.x] = n;
  }
}

__global__ __launch_bounds__(256, 2) void ksolo(const double* A, double* Li, double* work, int reps,
                                               unsigned long long* ticks) {
  __shared__ double sA[okg::kTile * okg::kLd];
  __shared__ double sX[okg::kTile * okg::kLd];
  __shared__ double sy[2 * okg::kTile];
  __shared__ double sRl[okg::kTile];
  __shared__ int sFl[8];
  const int t = threadIdx.x;
  unsigned long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    if (t < 64) sy[t] = 1.0 + t;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    okg::potrfTile<19>(A, 64, Li + (size_t)blockIdx.x * 4096, nullptr, sA, sX, sy, sRl, sFl, t, false);
    __syncthreads();
    tot += __builtin_amdgcn_s_memrealtime() - t0;
  }
  if (t == 0) ticks[blockIdx.x] = tot;
}

static double check(const double* dL, const std::vector<double>& A) {
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
    for (int j = 0; j <= i; ++j) {  // (lower triangle stored by the persistent callers)
      double v = 0;
      for (int k = 0; k < 64; ++k) v += X[i * 64 + k] * L[k * 64 + j];
      err = std::fmax(err, std::fabs(v - (i == j ? 1.0 : 0.0)));
    }
  return err;
}

int main() {
  std::vector<double> A(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) A[i * 64 + j] = 1.0 / (1.0 + i + j) + ((i == j) ? 4.0 + 0.1 * i : 0.0);
  const int nb = 512, reps = 100;
  double *dA, *dL, *dW, *dB, *dBo;
  unsigned long long *dT, *dC;
  (void)hipMalloc(&dA, 8 * 4096);
  (void)hipMalloc(&dL, 8 * 4096 * (size_t)nb);
  (void)hipMalloc(&dW, 8 * 64 * (size_t)nb);
  (void)hipMalloc(&dB, 8 * 8192);
  (void)hipMalloc(&dBo, 8 * 4096 * (size_t)nb);
  (void)hipMalloc(&dT, 8 * nb);
  (void)hipMalloc(&dC, 8 * nb);
  (void)hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB + 4096, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  for (int blocks : {1, cus}) {
    for (int mode = 0; mode < 4; ++mode) {
      std::vector<unsigned long long> t(blocks), c(blocks, 0);
      for (int pass = 0; pass < 2; ++pass) {
        (void)hipMemset(dC, 0, 8 * nb);
        if (mode == 0) hipLaunchKernelGGL(kteam<0>, blocks, 512, 0, 0, dA, dL, dW, dB, dBo, reps, dT, dC);
        if (mode == 1) hipLaunchKernelGGL(kteam<1>, blocks, 512, 0, 0, dA, dL, dW, dB, dBo, reps, dT, dC);
        if (mode == 2) hipLaunchKernelGGL(kteam<2>, blocks, 512, 0, 0, dA, dL, dW, dB, dBo, reps, dT, dC);
        if (mode == 3) hipLaunchKernelGGL(ksolo, blocks, 256, 0, 0, dA, dL, dW, reps, dT);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      }
      (void)hipMemcpy(t.data(), dT, 8 * blocks, hipMemcpyDeviceToHost);
      (void)hipMemcpy(c.data(), dC, 8 * blocks, hipMemcpyDeviceToHost);
      double s = 0, n = 0;
      for (int b = 0; b < blocks; ++b) { s += (double)t[b]; n += (double)c[b]; }
      const double us = s / blocks * 10.0 / 1000.0 / reps;
      printf("mode %d blocks %3d: factor %.3f us per tile; team B %.1f tile products per factor (%.2f us each); "
             "max |X L - I| %.1e\n", mode, blocks, us, n / blocks / reps, n > 0 ? us * reps * blocks / n : 0.0,
             check(dL, A));
    }
  }
  return 0;
}
