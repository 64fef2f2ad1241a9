// Development micro-benchmark: okg::potrfWave (the wave-specialised schedule's diagonal tile) on
// one wavefront, isolated, with the in-kernel phase clock (build with -DOKG_CHOL_CLOCK).
// hipcc --offload-arch=gfx950 -O3 -DOKG_CHOL_CLOCK -I include scripts/ubench_potrf.hip -o scripts/ubench_potrf
#include "../okvis2-x_amd/csrc/kernels_chol.hip"

#include <cstdio>
#include <vector>

__global__ void kpotrf(const double* A, int reps, unsigned long long* ticks, double* out) {
  __shared__ double sF[okg::kTile * okg::kLd];
  __shared__ double sX[okg::kTile * okg::kLd];
  __shared__ double sRl[64], sY[64], sZ[64];
  __shared__ int xFree, fail;
  const int lane = threadIdx.x;
  if (lane == 0) { xFree = 0; fail = 0; }
  unsigned long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    for (int e = lane; e < 4096; e += 64) sF[(e >> 6) * okg::kLd + (e & 63)] = A[e];
    __builtin_amdgcn_wave_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    okg::potrfWave(sF, sX, sRl, sY, sZ, 1.0 + lane, &xFree, 0, &fail, lane);
    tot += __builtin_amdgcn_s_memrealtime() - t0;
  }
  out[lane] = sZ[lane];
  if (lane == 0) *ticks = tot;
}

int main() {
  std::vector<double> A(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) A[i * 64 + j] = (i == j) ? 64.0 + i : 1.0 / (1.0 + i + j);
  double *dA, *dO;
  unsigned long long* dT;
  (void)hipMalloc(&dA, 8 * 4096);
  (void)hipMalloc(&dO, 8 * 64);
  (void)hipMalloc(&dT, 8);
  (void)hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  const int reps = 100;
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(kpotrf, 1, 64, 0, 0, dA, reps, dT, dO);
    (void)hipDeviceSynchronize();
  }
  unsigned long long t;
  (void)hipMemcpy(&t, dT, 8, hipMemcpyDeviceToHost);
  printf("potrfWave %.3f us per tile (isolated, 1 wavefront)\n", t * 10.0 / 1000.0 / reps);
  unsigned long long clk[32];
  (void)hipMemcpyFromSymbol(clk, HIP_SYMBOL(okg::g_cholClk), sizeof(clk));
  const char* nm[7] = {"pfac", "ptrail", "waitXFree", "zeroX", "dinv", "subd", "yz"};
  for (int i = 0; i < 7; ++i) printf("  %-10s %.3f us\n", nm[i], clk[4 + i] * 10.0 / 1000.0 / (2 * reps));
  return 0;
}
