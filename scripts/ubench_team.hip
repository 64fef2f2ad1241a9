// Development micro-benchmark for a two-team persistent Cholesky: how much does the diagonal tile
// factor (okg::potrfTile in team mode, team F) slow down while the other team of the 512-thread
// workgroup (team B) works on the same CU? Team B's load: MODE 0 none, 1 64x64x64 FP64 MFMA tile
// products from LDS (band updates / panels), 2 the same MFMAs on register operands (no LDS reads),
// 3 the LDS operand reads alone (no MFMA), 4 FP64 VALU FMAs; MAP 0: team F = waves 0-3, MAP 1: team F
// = the even waves. Also: the product's 256-thread potrfTile alone, and the SIMD each wave of a
// 512-thread workgroup lands on (HW_ID). One workgroup per CU (LDS ~134 KB) and one workgroup.
// hipcc --offload-arch=gfx950 -O3 -I include scripts/ubench_team.hip -o scripts/ubench_team
#include "../okvis2-x_amd/csrc/chol_tiles.hpp"

#include <cmath>
#include <cstdio>
#include <vector>

template <int MODE, int MAP>
__global__ __launch_bounds__(512, 1) void kteam(const double* A, double* Li, double* work, const double* Bsrc,
                                                double* Bdst, int reps, unsigned long long* ticks,
                                                unsigned long long* bcount, int* simd) {
  __shared__ double sA[okg::kTile * okg::kLd];
  __shared__ double sX[okg::kTile * okg::kLd];
  __shared__ double sB1[okg::kTile * okg::kLd];
  __shared__ double sB2[okg::kTile * okg::kLd];
  __shared__ double sy[2 * okg::kTile];
  __shared__ double sRl[okg::kTile];
  __shared__ int sFl[8];
  __shared__ int sDone;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int team = MAP == 0 ? wave >> 2 : wave & 1;
  const int tt = (MAP == 0 ? (wave & 3) : (wave >> 1)) * 64 + lane, t = threadIdx.x;
  if (blockIdx.x == 0 && lane == 0) simd[wave] = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3;
  if (t < 8) sFl[t] = 0;
  if (t == 0) sDone = 0;
  __syncthreads();
  if (team == 0) {
    int gen = 0;
    unsigned long long tot = 0;
    for (int r = 0; r < reps; ++r) {
      if (tt < 64) sy[tt] = 1.0 + tt;
      okg::waveBarrier<true>(&sFl[4], gen, 4, lane);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      okg::potrfTileBody<21>(A, 64, Li + (size_t)blockIdx.x * 4096, nullptr, sA, sX, sy, sRl, sFl, tt, false, gen, 4);
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
    double rv[4];
    for (int i = 0; i < 4; ++i) rv[i] = sB1[tt + 64 * i];
    while (__hip_atomic_load(&sDone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
      okg::dbl4 acc[2][2];
      if (MODE == 1) {
        okg::mfmaTileNT(sB1, sB2, acc, tt);
      } else if (MODE == 2) {  // the same 64 MFMAs per wavefront on register operands
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 2; ++b) acc[a][b] = okg::dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
        for (int kk = 0; kk < 16; ++kk)
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(rv[a] + kk, rv[2 + b], acc[a][b], 0, 0, 0);
      } else if (MODE == 3) {  // the operand reads of a tile product alone
        const int wv = tt >> 6, lr = lane & 15, lk = lane >> 4, r0 = 32 * (wv >> 1), c0 = 32 * (wv & 1);
        double s4[4] = {0, 0, 0, 0};
#pragma unroll 4
        for (int kk = 0; kk < 64; kk += 4)
          for (int a = 0; a < 2; ++a) {
            s4[a] += sB1[(r0 + 16 * a + lr) * okg::kLd + kk + lk];
            s4[2 + a] += sB2[(c0 + 16 * a + lr) * okg::kLd + kk + lk];
          }
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 2; ++b) acc[a][b] = okg::dbl4{s4[a], s4[b], s4[2 + a], s4[2 + b]};
      } else {  // FP64 VALU: 4 independent FMA chains of 64 steps
        double f[4] = {rv[0], rv[1], rv[2], rv[3]};
        for (int i = 0; i < 64; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) f[j] = fma(f[j], 0.999, 1e-3);
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 2; ++b) acc[a][b] = okg::dbl4{f[a], f[b], f[2 + a], f[2 + b]};
      }
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
  int* dS;
  (void)hipMalloc(&dS, 4 * 8);
  auto run = [&](auto kern, int blocks, int threads, const char* tag) {
    std::vector<unsigned long long> t(blocks), c(blocks, 0);
    for (int pass = 0; pass < 2; ++pass) {
      (void)hipMemset(dC, 0, 8 * nb);
      if (threads == 512) hipLaunchKernelGGL(kern, blocks, 512, 0, 0, dA, dL, dW, dB, dBo, reps, dT, dC, dS);
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); exit(1); }
    }
    (void)hipMemcpy(t.data(), dT, 8 * blocks, hipMemcpyDeviceToHost);
    (void)hipMemcpy(c.data(), dC, 8 * blocks, hipMemcpyDeviceToHost);
    double s = 0, n = 0;
    for (int b = 0; b < blocks; ++b) { s += (double)t[b]; n += (double)c[b]; }
    const double us = s / blocks * 10.0 / 1000.0 / reps;
    printf("%-28s blocks %3d: factor %.3f us per tile; team B %.1f units per factor (%.2f us each); max |X L - I| %.1e\n",
           tag, blocks, us, n / blocks / reps, n > 0 ? us * reps * blocks / n : 0.0, check(dL, A));
  };
  for (int blocks : {1, cus}) {
    run(kteam<0, 0>, blocks, 512, "B idle, F = waves 0-3");
    run(kteam<0, 1>, blocks, 512, "B idle, F = even waves");
    run(kteam<1, 0>, blocks, 512, "B MFMA+LDS, F = waves 0-3");
    run(kteam<1, 1>, blocks, 512, "B MFMA+LDS, F = even waves");
    run(kteam<2, 0>, blocks, 512, "B MFMA regs, F = waves 0-3");
    run(kteam<2, 1>, blocks, 512, "B MFMA regs, F = even waves");
    run(kteam<3, 0>, blocks, 512, "B LDS reads, F = waves 0-3");
    run(kteam<4, 0>, blocks, 512, "B FP64 VALU, F = waves 0-3");
    {
      std::vector<unsigned long long> t(blocks);
      hipLaunchKernelGGL(ksolo, blocks, 256, 0, 0, dA, dL, dW, reps, dT);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(t.data(), dT, 8 * blocks, hipMemcpyDeviceToHost);
      double s = 0;
      for (int b = 0; b < blocks; ++b) s += (double)t[b];
      printf("%-28s blocks %3d: factor %.3f us per tile\n", "256-thread potrfTile alone", blocks, s / blocks * 10.0 / 1000.0 / reps);
    }
  }
  int simd[8];
  (void)hipMemcpy(simd, dS, 4 * 8, hipMemcpyDeviceToHost);
  printf("SIMD of waves 0..7 of a 512-thread workgroup:");
  for (int i = 0; i < 8; ++i) printf(" %d", simd[i]);
  printf("\n");
  return 0;
}
