// Development check (not part of the library): DPP row_newbcast:n on gfx950 gives every lane of a
// 16-lane row the value of lane n of that row (the semantics kernels_eval.hip relies on).
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/dpp_bcast_check scripts/dpp_bcast_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
template <int K>
__device__ __forceinline__ double rowBcast(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)__double2loint(v), 0x150 + K, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)__double2hiint(v), 0x150 + K, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
template <int K>
__device__ void all(double v, double* o) {
  o[K * 64 + threadIdx.x] = rowBcast<K>(v);
  if constexpr (K < 15) all<K + 1>(v, o);
}
__global__ void k(const double* in, double* o) { all<0>(in[threadIdx.x], o); }
int main() {
  double h[64], r[16 * 64];
  for (int i = 0; i < 64; ++i) h[i] = 1000.0 + i * 1.25;
  double *din, *dout;
  if (hipMalloc(&din, sizeof h) != hipSuccess || hipMalloc(&dout, sizeof r) != hipSuccess) return 2;
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
  hipMemcpy(r, dout, sizeof r, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int n = 0; n < 16; ++n)
    for (int t = 0; t < 64; ++t)
      if (r[n * 64 + t] != h[(t & ~15) + n]) ++bad;
  printf("row_newbcast check: %d mismatches of %d\n", bad, 16 * 64);
  hipFree(din);
  hipFree(dout);
  return bad ? 1 : 0;
}
