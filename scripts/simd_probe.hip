// Wave placement probe (development): which SIMD / wave slot each wavefront of a 256-thread
// workgroup lands on when two such workgroups share a CU (the persistent Cholesky's shape: ~74 KB
// of LDS, launch_bounds(256, 2)). Prints, per co-resident pair of workgroups, the SIMD of each
// workgroup's wavefront 0. hipcc --offload-arch=gfx950 -O3 simd_probe.hip -o simd_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256, 2) void probe(unsigned* out, int spin) {
  __shared__ double big[74 * 1024 / 8];
  const int t = threadIdx.x;
  big[t] = t;
  __syncthreads();
  // HW_REG_HW_ID (4): wave slot [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]; XCC_ID (20)
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);
  long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(10);
  if ((t & 63) == 0) {
    out[4 * (blockIdx.x * 4 + (t >> 6)) + 0] = hw;
    out[4 * (blockIdx.x * 4 + (t >> 6)) + 1] = xcc;
    out[4 * (blockIdx.x * 4 + (t >> 6)) + 2] = (unsigned)t0;
    out[4 * (blockIdx.x * 4 + (t >> 6)) + 3] = (unsigned)big[t + 1];
  }
}

int main() {
  const int nb = 2048;
  unsigned* d;
  hipMalloc(&d, nb * 4 * 4 * sizeof(unsigned));
  hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 0, 0, d, 20000);  // ~200 us per workgroup
  hipDeviceSynchronize();
  std::vector<unsigned> h(nb * 16);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  // group workgroups by (xcc, se, sh, cu) and start time window
  std::map<std::tuple<int, int, int, int>, std::vector<int>> cu;
  int sameSimd0 = 0, pairs = 0;
  std::map<int, int> hist;
  for (int b = 0; b < nb; ++b) {
    const unsigned hw = h[16 * b], xcc = h[16 * b + 1] & 15;
    const int cuid = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    cu[{(int)xcc, se, sh, cuid}].push_back(b);
    int simds = 0;
    for (int w = 0; w < 4; ++w) simds |= 1 << ((h[16 * b + 4 * w] >> 4) & 3);
    hist[((h[16 * b] >> 4) & 3) * 16 + (h[16 * b] & 15)]++;
    if (simds != 15) std::printf("block %d: waves not on 4 distinct SIMDs (mask %x)\n", b, simds);
  }
  for (auto& kv : cu) {
    auto& v = kv.second;
    for (size_t i = 0; i + 1 < v.size(); i += 2) {
      const int a = v[i], b = v[i + 1];
      const long long ta = h[16 * a + 2], tb = h[16 * b + 2];
      if (std::llabs(ta - tb) > 5000) continue;  // not co-resident
      ++pairs;
      if (((h[16 * a] >> 4) & 3) == ((h[16 * b] >> 4) & 3)) ++sameSimd0;
    }
  }
  std::printf("CUs seen %zu, co-resident pairs %d, pairs whose wavefront 0 share a SIMD: %d\n", cu.size(), pairs,
              sameSimd0);
  std::printf("wavefront 0 (simd, slot) histogram:");
  for (auto& kv : hist) std::printf(" (%d,%d):%d", kv.first / 16, kv.first % 16, kv.second);
  std::printf("\n");
  for (int b = 0; b < 8; ++b) {
    std::printf("block %d:", b);
    for (int w = 0; w < 4; ++w) {
      const unsigned hw = h[16 * b + 4 * w];
      std::printf(" w%d simd %u slot %u cu %u se %u xcc %u |", w, (hw >> 4) & 3, hw & 15, (hw >> 8) & 15, (hw >> 13) & 7,
                  h[16 * b + 4 * w + 1] & 15);
    }
    std::printf("\n");
  }
  hipFree(d);
  return 0;
}
