// pmc_calib.hip — calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access shapes of
// okvisgpu's kernels (MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a 16 B/lane
// streaming read; other widths are uncalibrated there). Each kernel touches a known number of bytes of
// a 1 GiB buffer (4x the Infinity Cache, so every byte comes from HBM once); the profile of this
// program divided by these counts gives the per-shape factors scripts/pmc_traffic.py applies.
//   read16   16 B per lane, consecutive lanes consecutive (loadTile of the Cholesky, LDS staging)
//   read8    8 B per lane, consecutive (SoA planes: k_eval_obs, k_lm_visit, k_lm_backsub_jv)
//   readrow  the Cholesky's loadC shape: 8 B per lane, 16 lanes along a 64-double tile row, 4 rows of
//            a 768-double row stride per wave instruction (64x64 tiles of a 768x768 matrix)
//   write16, write8, writerow   the same shapes as stores
// Usage: pmc_calib [shape] (all shapes by default); prints the bytes each dispatch touches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr size_t kBytes = 1ull << 30;
constexpr size_t kD = kBytes / 8;  // doubles

__global__ void read16(const double2* a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  out[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = s;
}
__global__ void read8(const double* a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  out[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = s;
}
// one 64x64 tile per workgroup of 256 threads, loadC's lane map: element (r0 + 16a + (lane>>4) + 4reg,
// c0 + 16b + (lane&15)) of a row-major matrix with 768-double rows (12 x 12 tiles per matrix)
__global__ void readrow(const double* a, size_t ntiles, double* out) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int r0 = 32 * (wave >> 1), c0 = 32 * (wave & 1);
  double s = 0.0;
  for (size_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const size_t m = tile / 144, ti = (tile % 144) / 12, tj = tile % 12;
    const double* A = a + m * 768 * 768 + ti * 64 * 768 + tj * 64;
    for (int aa = 0; aa < 2; ++aa)
      for (int b = 0; b < 2; ++b)
        for (int reg = 0; reg < 4; ++reg) s += A[(size_t)(r0 + 16 * aa + (lane >> 4) + 4 * reg) * 768 + c0 + 16 * b + (lane & 15)];
  }
  out[blockIdx.x * (size_t)blockDim.x + t] = s;
}
__global__ void write16(double2* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = double2{(double)i, 1.0};
}
__global__ void write8(double* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}
__global__ void writerow(double* a, size_t ntiles) {
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int r0 = 32 * (wave >> 1), c0 = 32 * (wave & 1);
  for (size_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const size_t m = tile / 144, ti = (tile % 144) / 12, tj = tile % 12;
    double* A = a + m * 768 * 768 + ti * 64 * 768 + tj * 64;
    for (int aa = 0; aa < 2; ++aa)
      for (int b = 0; b < 2; ++b)
        for (int reg = 0; reg < 4; ++reg)
          A[(size_t)(r0 + 16 * aa + (lane >> 4) + 4 * reg) * 768 + c0 + 16 * b + (lane & 15)] = (double)tile;
  }
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;
  double *a = nullptr, *out = nullptr;
  CK(hipMalloc(&a, kBytes));
  const int grid = 4096, block = 256;
  CK(hipMalloc(&out, sizeof(double) * grid * block));
  CK(hipMemset(a, 0, kBytes));
  CK(hipDeviceSynchronize());
  const size_t tiles = (kD / (768 * 768)) * 144;  // whole 768x768 matrices in the buffer
  auto want = [&](const char* s) { return !only || std::strcmp(only, s) == 0; };
  // bytes each dispatch touches (the out[] write of the read kernels is 8 MiB, listed apart)
  if (want("read16")) { hipLaunchKernelGGL(read16, grid, block, 0, 0, (const double2*)a, kD / 2, out); std::printf("read16 %zu\n", kBytes); }
  if (want("read8")) { hipLaunchKernelGGL(read8, grid, block, 0, 0, a, kD, out); std::printf("read8 %zu\n", kBytes); }
  if (want("readrow")) { hipLaunchKernelGGL(readrow, grid, block, 0, 0, a, tiles, out); std::printf("readrow %zu\n", tiles * 64 * 64 * 8); }
  if (want("write16")) { hipLaunchKernelGGL(write16, grid, block, 0, 0, (double2*)a, kD / 2); std::printf("write16 %zu\n", kBytes); }
  if (want("write8")) { hipLaunchKernelGGL(write8, grid, block, 0, 0, a, kD); std::printf("write8 %zu\n", kBytes); }
  if (want("writerow")) { hipLaunchKernelGGL(writerow, grid, block, 0, 0, a, tiles); std::printf("writerow %zu\n", tiles * 64 * 64 * 8); }
  CK(hipDeviceSynchronize());
  std::printf("out_bytes %zu\n", sizeof(double) * grid * block);
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
