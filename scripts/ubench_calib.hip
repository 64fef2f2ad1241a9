// Development micro-benchmark: s_memtime tick rate vs s_memrealtime (100 MHz), and FP64 VALU
// dependent-chain latency / independent issue rate on one wavefront, plus LDS broadcast read
// latency. hipcc --offload-arch=gfx950 -O3 scripts/ubench_calib.hip -o scripts/ubench_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void kcal(double* out, unsigned long long* t, int n, double a, double b) {
  __shared__ double sh[256];
  const int l = threadIdx.x;
  sh[l] = a + l;
  __syncthreads();
  double x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = a + k + l;
  // dependent chain
  unsigned long long m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double y = x[0];
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) y = __builtin_fma(y, b, a);
  }
  unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  // 8 independent chains
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = __builtin_fma(x[k], b, a);
  }
  unsigned long long m2 = __builtin_amdgcn_s_memtime();
  // dependent LDS reads (pointer chase through the value)
  int idx = l & 1;
  double z = 0;
  for (int i = 0; i < n; ++i) {
    const double v = sh[idx];
    z += v;
    idx = ((int)v) & 7;
  }
  unsigned long long m3 = __builtin_amdgcn_s_memtime();
  // rsqrt dependent chain
  double q = a + 2.0;
  for (int i = 0; i < n; ++i) q = __builtin_amdgcn_rsq(q) + 1.0;
  unsigned long long m4 = __builtin_amdgcn_s_memtime();
  double s = y + z + q;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  out[l] = s;
  if (l == 0) {
    t[0] = m1 - m0; t[1] = r1 - r0; t[2] = m2 - m1; t[3] = m3 - m2; t[4] = m4 - m3;
  }
}

int main() {
  double* o;
  unsigned long long* t;
  (void)hipMalloc(&o, 8 * 64);
  (void)hipMalloc(&t, 64);
  const int n = 2000;
  for (int p = 0; p < 3; ++p) {
    hipLaunchKernelGGL(kcal, 1, 64, 0, 0, o, t, n, 1.0, 0.999);
    (void)hipDeviceSynchronize();
  }
  unsigned long long h[5];
  (void)hipMemcpy(h, t, 40, hipMemcpyDeviceToHost);
  const double ns = h[1] * 10.0;
  printf("s_memtime ticks %llu over %.1f us -> %.3f ticks/ns\n", h[0], ns / 1000, h[0] / ns);
  printf("dependent FP64 FMA: %.2f ticks each\n", (double)h[0] / (8.0 * n));
  printf("independent FP64 FMA (8 chains): %.2f ticks per instruction\n", (double)h[2] / (8.0 * n));
  printf("dependent LDS read + add + cvt: %.2f ticks each\n", (double)h[3] / n);
  printf("dependent rsq + add: %.2f ticks each\n", (double)h[4] / n);
  return 0;
}
