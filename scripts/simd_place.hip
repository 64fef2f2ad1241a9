// Development probe: which SIMD does each wavefront of two co-resident 256-thread workgroups land
// on (the persistent Cholesky's shape: 74 KB of LDS, so two workgroups per CU)? Every wavefront
// records HW_ID (SIMD id [5:4], CU [11:8], SH [12], SE [15:13]) and XCC_ID; the host groups the
// workgroups by CU and prints the SIMDs of wavefronts 0-3 of each pair.
// hipcc --offload-arch=gfx950 -O3 scripts/simd_place.hip -o scripts/simd_place
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256, 2) void kplace(unsigned* out, int spin) {
  __shared__ double pad[74 * 1024 / 8];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  pad[threadIdx.x] = 1.0;
  __syncthreads();
  if (lane == 0) {
    out[(blockIdx.x * 4 + wave) * 2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    out[(blockIdx.x * 4 + wave) * 2 + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
  // keep the workgroup resident for a while so that the co-resident pairs overlap
  const long long t0 = clock64();
  while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(2);
  if (pad[(threadIdx.x + 1) & 255] < 0) out[0] = 0;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int blocks = 2 * prop.multiProcessorCount;
  unsigned* d;
  (void)hipMalloc(&d, sizeof(unsigned) * 8 * blocks);
  hipLaunchKernelGGL(kplace, blocks, 256, 0, 0, d, 2000000);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<unsigned> h(8 * blocks);
  (void)hipMemcpy(h.data(), d, sizeof(unsigned) * 8 * blocks, hipMemcpyDeviceToHost);
  std::map<std::tuple<unsigned, unsigned, unsigned, unsigned>, std::vector<int>> byCu;
  for (int b = 0; b < blocks; ++b) {
    const unsigned hw = h[b * 8], xcc = h[b * 8 + 1] & 0xf;
    byCu[{xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15}].push_back(b);
  }
  std::map<std::string, int> patterns;
  for (auto& kv : byCu) {
    std::string p;
    for (int b : kv.second) {
      p += "[";
      for (int w = 0; w < 4; ++w) p += char('0' + ((h[(b * 4 + w) * 2] >> 4) & 3));
      p += "]";
    }
    ++patterns[p];
  }
  printf("%zu CUs seen for %d workgroups; SIMD of wavefronts 0-3 of the workgroups sharing a CU:\n", byCu.size(), blocks);
  for (auto& kv : patterns) printf("  %s x %d\n", kv.first.c_str(), kv.second);
  return 0;
}
