// Development micro-benchmark of the Cholesky's diagonal tile (okg::potrfTile: LLT, X = L^-1,
// y = X rhs) on one 256-thread workgroup, isolated (1 workgroup) and under load (2 per CU), plus a
// stamped copy of the sweep's chain wavefront (variant V, -DOKG_V=n) whose per-sub-panel phase
// times (s_memtime, shader clock) show where the chain spends its cycles.
// hipcc --offload-arch=gfx950 -O3 -I include scripts/ubench_ptile.hip -o scripts/ubench_ptile
#include "../okvis2-x_amd/csrc/chol_tiles.hpp"

#include <cmath>
#include <cstdio>
#include <vector>


namespace okg {
__device__ unsigned long long g_tr[8][8];

// The chain wavefront's loop of potrfTile with stamps (lane 0 of wavefront 0, workgroup 0):
// [0] start [1] waited [2] r loaded [3] look-ahead FMAs [4] r stored [5] chol8 [6] stored
// Variants: 0 stamps + scheduling fences (lgkmcnt wait after the r loads, r / x consumed before the
// stores), 2 fences without stamps, 3 the consumption fences only (the product's form since round
// 4), 4 stamps only. Round-4 result: every variant ~16 us per tile, the product without any of
// them 22.6 us (the compiler then interleaves the row stores / loads with the FP64 chain).
#define STAMP(s, k) if (V == 0 || V == 4) st[s][k] = __builtin_amdgcn_s_memtime();
template <int V>
__device__ __noinline__ bool potrfExp(const double* Sg, int64_t ld, double* Li, double* workk, double* sA, double* sX,
                                      double* sy, double* sRl, int* sFl, int t) {
  const int wave = t >> 6, lane = t & 63;
  loadTile(Sg, ld, 0, 0, sA, t);
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = t + 256 * u;
    sX[(e >> 6) * kLd + (e & 63)] = 0.0;
  }
  if (t < 4) sFl[t] = 0;
  ldsBarrier();
  const bool tr = blockIdx.x == 0 && t == 0;
  unsigned long long st[8][8];
  if (wave == 0) {
    const int i = lane;
    double xp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) xp[k] = 0.0;
#pragma unroll 1
    for (int s = 0; s < 8; ++s) {
      const int c0 = 8 * s;
      STAMP(s, 0)
      if (s >= 2 && !waitFlag<true>(&sFl[1], s - 1, &sFl[2])) break;
      STAMP(s, 1)
      double r[8], x[8], rl[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = sA[i * kLd + c0 + k];
      if (V == 0 || V == 2) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      STAMP(s, 2)
      if (s >= 1) {
#pragma unroll
        for (int c = 0; c < 8; ++c)
#pragma unroll
          for (int m = 0; m < 8; ++m) r[m] -= xp[c] * sA[(c0 + m) * kLd + c0 - 8 + c];
        if (V != 4) asm volatile("" ::"v"(r[0]), "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7]));
        STAMP(s, 3)
        if (V == 1 ? (i >= c0 && i < c0 + 8) : i >= c0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) sA[i * kLd + c0 + k] = r[k];
        }
        __builtin_amdgcn_wave_barrier();
      } else {
        if (V == 0 || V == 4) st[s][3] = st[s][2];
      }
      STAMP(s, 4)
      if (!chol8Row(sA, c0, r, x, rl)) {
        if (lane == 0) ldsReleaseL(&sFl[2], 1);
        break;
      }
      if (V != 4) asm volatile("" ::"v"(x[7]));
      STAMP(s, 5)
      storeRow8(sA, c0, x, i);
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) sRl[c0 + k] = rl[k];
        ldsReleaseL(&sFl[0], s + 1);
      }
      STAMP(s, 6)
#pragma unroll
      for (int k = 0; k < 8; ++k) xp[k] = x[k];
    }
    if ((V == 0 || V == 4) && tr)
      for (int s = 0; s < 8; ++s)
        for (int k = 0; k < 7; ++k) g_tr[s][k] = st[s][k];
  } else {
    const int g = wave - 1;
    int gen = 0;
#pragma unroll 1
    for (int s = 0; s < 8; ++s) {
      if (!waitFlag<true>(&sFl[0], s + 1, &sFl[2])) break;
      if (g == 0) inv8(sA, sRl, sX + 8 * s * kLd + 8 * s, 8 * s, lane);
      if (s < 6) trailingFrom(sA, 8 * s, 8 * s + 16, g, 3, lane);
      waveBarrier<true>(&sFl[3], gen, 3, lane);
      if (g == 0 && lane == 0) ldsReleaseL(&sFl[1], s + 1);
      if (s & 1) {
        const int q = s >> 1;
        if (g == 0) xDiag16(sA, sX, q, lane);
        waveBarrier<true>(&sFl[3], gen, 3, lane);
        if (g < q) xOffDiag16(sA, sX, q, g, lane);
        waveBarrier<true>(&sFl[3], gen, 3, lane);
        if (g == 0) yBlock16(sX, sy, q, lane);
        xStoreRows16<1>(sX, Li, q, g, lane);
      }
    }
  }
  ldsBarrier();
  if (sFl[2]) return false;
  if (t < kTile) {
    const double y = sy[kTile + t];
    sy[t] = y;
    workk[t] = y;
  }
  ldsBarrier();
  return true;
}
}  // namespace okg

// -1: the product's potrfTile as the tile-parallel kernels instantiate it, -2: as the persistent
// kernel does; each through an instantiation of its own (3, 19: one caller, like the product's, so
// that the register budget and the code match the product build), else potrfExp<EXP>
template <int EXP>
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
    if (EXP >= 0)
      okg::potrfExp<(EXP < 0 ? 0 : EXP)>(A, 64, Li + (size_t)blockIdx.x * 4096, work + (size_t)blockIdx.x * 64, sA, sX, sy, sRl, sFl, t);
    else if (EXP == -1)
      okg::potrfTile<3>(A, 64, Li + (size_t)blockIdx.x * 4096, work + (size_t)blockIdx.x * 64, sA, sX, sy, sRl, sFl, t,
                        false);
    else
      okg::potrfTile<19>(A, 64, Li + (size_t)blockIdx.x * 4096, nullptr, sA, sX, sy, sRl, sFl, t, false);
    __syncthreads();
    tot += __builtin_amdgcn_s_memrealtime() - t0;
  }
  if (t == 0) ticks[blockIdx.x] = tot;
}

template <int EXP>
static void run(const char* tag, const double* dA, double* dL, double* dW, unsigned long long* dT, const std::vector<double>& A) {
  const int nb = 512, reps = 200;
  for (int cfg = 0; cfg < 2; ++cfg) {
    const int blocks = cfg == 0 ? 1 : nb;
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(kptile<EXP>, blocks, 256, 0, 0, dA, dL, dW, reps, dT);
      (void)hipDeviceSynchronize();
    }
    std::vector<unsigned long long> t(blocks);
    (void)hipMemcpy(t.data(), dT, 8 * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (int b = 0; b < blocks; ++b) s += (double)t[b];
    printf("%s blocks %4d: %.3f us per tile\n", tag, blocks, s / blocks * 10.0 / 1000.0 / reps);
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
  printf("%s max |X L - I| = %.2e\n", tag, err);
}

int main() {
  std::vector<double> A(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) A[i * 64 + j] = 1.0 / (1.0 + i + j) + ((i == j) ? 4.0 + 0.1 * i : 0.0);
  const int nb = 512;
  double *dA, *dL, *dW;
  unsigned long long* dT;
  (void)hipMalloc(&dA, 8 * 4096);
  (void)hipMalloc(&dL, 8 * 4096 * (size_t)nb);
  (void)hipMalloc(&dW, 8 * 64 * (size_t)nb);
  (void)hipMalloc(&dT, 8 * nb);
  (void)hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  run<-1>("product (tile-parallel)", dA, dL, dW, dT, A);
  run<-2>("product (persistent)", dA, dL, dW, dT, A);
  run<2>("fences", dA, dL, dW, dT, A);
  run<3>("consume-only", dA, dL, dW, dT, A);
  run<4>("stamps-only", dA, dL, dW, dT, A);
  run<0>("stamped", dA, dL, dW, dT, A);
  hipLaunchKernelGGL(kptile<0>, 1, 256, 0, 0, dA, dL, dW, 1, dT);
  (void)hipDeviceSynchronize();
  unsigned long long T[8][8];
  (void)hipMemcpyFromSymbol(T, HIP_SYMBOL(okg::g_tr), sizeof(T));
  printf("chain wavefront per sub-panel (shader clocks): wait  rload  lookahead  rstore  chol8  store  -> next\n");
  for (int s = 0; s < 8; ++s) {
    printf("  %d |", s);
    for (int k = 1; k < 7; ++k) printf(" %7lld", (long long)(T[s][k] - T[s][k - 1]));
    printf(" %7lld\n", s < 7 ? (long long)(T[s + 1][0] - T[s][6]) : 0LL);
  }
  printf("sweep total %lld clocks\n", (long long)(T[7][6] - T[0][0]));
  return 0;
}
