// Development micro-benchmark: FP64 dependent-chain latency and the 8-column sub-panel step of the
// diagonal-tile LLT (kernels_chol.hip subPanel8 / trailing8), one workgroup, many repetitions.
// hipcc --offload-arch=gfx950 -O3 -I okvis2-x_amd/csrc scripts/ubench_sub8.hip -o /tmp/ubench_sub8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "device_problem.hpp"

namespace okg {
constexpr int kLd = kTile + 1;
typedef double dbl4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double rsqrtRefined(double d) {
  double r = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  r = r * (1.5 - h * r * r);
  r = r * (1.5 - h * r * r);
  return r;
}
__device__ __forceinline__ dbl4 loadC16(const double* c, int ldc, int lane) {
  dbl4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = c[((lane >> 4) + 4 * r) * ldc + (lane & 15)];
  return v;
}
__device__ __forceinline__ void storeC16(double* c, int ldc, const dbl4& v, int lane) {
#pragma unroll
  for (int r = 0; r < 4; ++r) c[((lane >> 4) + 4 * r) * ldc + (lane & 15)] = v[r];
}
#include "ubench_sub8_body.inc"
}  // namespace okg
using namespace okg;

__global__ void k_chain(double* out, long long* cyc, int n) {
  double a = out[threadIdx.x], b = 1.0000001;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) a = fma(a, b, 1e-9);
  }
  long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_rsq(double* out, long long* cyc, int n) {
  double a = out[threadIdx.x] + 2.0;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) a = rsqrtRefined(a) + 1.5;
  long long t1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_mfma(double* out, long long* cyc, int n) {
  dbl4 acc = {0, 0, 0, 0};
  double a = out[threadIdx.x], b = 0.5;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_sweep(const double* A, double* out, long long* cyc, int reps, int mode) {
  __shared__ double sA[kTile * kLd], sX[kTile * kLd], sRl[kTile];
  __shared__ int fail;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  long long tsub = 0, ttr = 0;
  for (int r = 0; r < reps; ++r) {
    for (int e = t; e < kTile * kTile; e += blockDim.x) sA[(e >> 6) * kLd + (e & 63)] = A[e];
    __syncthreads();
    for (int s = 0; s < 8; ++s) {
      long long t0 = clock64();
      if (wave == 0) subPanel8(sA, sX + 8 * s * kLd + 8 * s, sRl, 8 * s, lane);
      __syncthreads();
      long long t1 = clock64();
      if (s < 7 && mode == 0) trailing8(sA, 8 * s, wave, blockDim.x / 64, lane);
      __syncthreads();
      long long t2 = clock64();
      tsub += t1 - t0;
      ttr += t2 - t1;
    }
  }
  for (int e = t; e < kTile * kTile; e += blockDim.x) out[e] = sA[(e >> 6) * kLd + (e & 63)];
  if (t == 0) { cyc[0] = tsub; cyc[1] = ttr; }
}

__global__ void k_clock(double* out, long long* cyc, int n) {
  double a = out[threadIdx.x], b = 1.0000001;
  long long t0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) a = fma(a, b, 1e-9);
  }
  long long t1 = clock64(), w1 = wall_clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = w1 - w0; }
}

__device__ __forceinline__ void ldsBarrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ double sum32(const double* p) {
  double a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = (p[64 * k] + p[64 * (k + 8)]) + (p[64 * (k + 16)] + p[64 * (k + 24)]);
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}
// mode 0: full step (partials, 4 barriers, 2 sum32); 1: barriers only; 2: __syncthreads barriers only
__global__ void k_bstep(double* out, long long* cyc, int n, int mode) {
  __shared__ double sA[32 * 64], sx[768], sy[64];
  const int t = threadIdx.x;
  for (int e = t; e < 768; e += blockDim.x) sx[e] = e;
  __syncthreads();
  long long t0 = clock64();
  for (int I = n - 1; I >= 0; --I) {
    if (mode == 0) {
      for (int k = 0; k < 2; ++k) {
        const int vt = t + 512 * k, c2 = 2 * (vt & 31), rg = vt >> 5;
        double ax = 0, ay = 0;
        for (int m = 0; m < 3; ++m) { ax += sx[(m + 1) * 64 + rg] * 0.5; ay += sx[(m + 1) * 64 + rg + 32] * 0.25; }
        sA[rg * 64 + c2] = ax; sA[rg * 64 + c2 + 1] = ay;
      }
      ldsBarrier();
      if (t < 64) sy[t] = sx[(I % 12) * 64 + t] - sum32(sA + t);
      ldsBarrier();
      for (int k = 0; k < 2; ++k) {
        const int vt = t + 512 * k, c2 = 2 * (vt & 31), rg = vt >> 5;
        sA[rg * 64 + c2] = sy[rg] * 0.5; sA[rg * 64 + c2 + 1] = sy[rg + 32] * 0.5;
      }
      ldsBarrier();
      if (t < 64) sx[(I % 12) * 64 + t] = sum32(sA + t) * 1e-3;
      ldsBarrier();
    } else if (mode == 1) {
      ldsBarrier(); ldsBarrier(); ldsBarrier(); ldsBarrier();
    } else {
      __syncthreads(); __syncthreads(); __syncthreads(); __syncthreads();
    }
  }
  long long t1 = clock64();
  if (t == 0) { cyc[0] = t1 - t0; out[0] = sx[5]; }
}

// LDS latency: dependent chain of ds_read_b32 (index chasing), one wave; and a store->load round trip
__global__ void k_ldslat(int* out, long long* cyc, int n) {
  __shared__ int s[1024];
  __shared__ double d[1024];
  for (int e = threadIdx.x; e < 1024; e += blockDim.x) { s[e] = (e * 7 + 3) & 1023; d[e] = e; }
  __syncthreads();
  int j = threadIdx.x;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) j = s[j];
  long long t1 = clock64();
  double a = 1.0;
  long long t2 = clock64();
  for (int i = 0; i < n; ++i) {
    d[threadIdx.x] = a;
    __builtin_amdgcn_wave_barrier();
    a = d[(threadIdx.x + 1) & 63] + 1.0;
  }
  long long t3 = clock64();
  out[threadIdx.x] = j + (int)a;
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t3 - t2; }
}

// global memory latency: dependent pointer chase over a buffer (hot: small, repeated; cold: large stride)
__global__ void k_glat(const int* __restrict__ nxt, int* out, long long* cyc, int n) {
  int j = 0;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) j = __builtin_nontemporal_load(nxt + j) + 0;
  long long t1 = clock64();
  out[0] = j;
  cyc[0] = t1 - t0;
}

__global__ void k_empty(int* o) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && o[0] == 12345) o[1] = 1;
}

int main() {
  double *d, *o;
  long long* c;
  hipMalloc(&d, 64 * 64 * 8);
  hipMalloc(&o, 64 * 64 * 8);
  hipMalloc(&c, 64);
  std::vector<double> A(64 * 64);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) A[i * 64 + j] = (i == j ? 64.0 : 0.0) + 1.0 / (1 + i + j);
  hipMemcpy(d, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(o, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  long long h[2];
  const int n = 1000;
  k_chain<<<1, 64>>>(o, c, n);
  hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
  printf("fp64 fma dependent chain: %.2f cycles per op\n", (double)h[0] / (16.0 * n));
  for (int rep = 0; rep < 3; ++rep) {
    k_clock<<<1, 64>>>(o, c, 20000);
    hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    printf("clock64 %lld ticks over %lld wall ticks (%.0f MHz wall): shader clock %.0f MHz\n", h[0], h[1], 100.0,
           100.0 * h[0] / h[1]);
  }
  k_rsq<<<1, 64>>>(o, c, n);
  hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
  printf("rsqrtRefined + add chain: %.2f cycles per step\n", (double)h[0] / n);
  k_mfma<<<1, 64>>>(o, c, n);
  hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
  printf("mfma_f64_16x16x4 dependent chain: %.2f cycles per op\n", (double)h[0] / (16.0 * n));
  for (int mode = 0; mode < 2; ++mode) {
    k_sweep<<<1, 256>>>(d, o, c, 100, mode);
    hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    printf("sweep mode %d: subPanel8+bar %.0f cycles per sub-panel, trailing8+bar %.0f per sub-panel\n", mode,
           h[0] / 800.0, h[1] / 800.0);
  }
  {
    int* oi;
    hipMalloc(&oi, 4096);
    k_ldslat<<<1, 64>>>(oi, c, 1000);
    hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
    printf("LDS dependent read chain: %.1f cycles; store->load round trip: %.1f cycles\n", h[0] / 1000.0, h[1] / 1000.0);
  }
  {
    const size_t N = 64u << 20;  // 256 MiB of ints
    int* nx;
    hipMalloc(&nx, N * 4);
    std::vector<int> hn(N);
    for (int mode = 0; mode < 2; ++mode) {
      const size_t span = mode == 0 ? 4096 : N;      // hot (16 KiB) / cold (256 MiB)
      const size_t stride = mode == 0 ? 33 : 1000003; // ints
      for (size_t i = 0; i < N; ++i) hn[i] = 0;
      size_t j = 0;
      for (int k = 0; k < 4096; ++k) { size_t nj = (j + stride) % span; hn[j] = (int)nj; j = nj; }
      hipMemcpy(nx, hn.data(), N * 4, hipMemcpyHostToDevice);
      int* oo; hipMalloc(&oo, 64);
      k_glat<<<1, 1>>>(nx, oo, c, 2000);
      hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
      printf("global dependent load (%s): %.0f cycles\n", mode == 0 ? "hot 16KiB" : "cold 256MiB", h[0] / 2000.0);
    }
  }
  for (int nt = 256; nt <= 1024; nt *= 2)
    for (int mode = 0; mode < 3; ++mode) {
      k_bstep<<<1, nt>>>(o, c, 120, mode);
      hipMemcpy(h, c, 8, hipMemcpyDeviceToHost);
      printf("bsub step threads %d mode %d: %.0f cycles per step\n", nt, mode, h[0] / 120.0);
    }
  {  // per-launch cost of a chain of small kernels in a captured graph
    int* oo; hipMalloc(&oo, 64); hipMemset(oo, 0, 64);
    hipStream_t st; hipStreamCreate(&st);
    for (int nb : {1, 64}) {
      hipGraph_t g; hipGraphExec_t ge;
      hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
      for (int i = 0; i < 100; ++i) k_empty<<<nb, 256, 0, st>>>(oo);
      hipStreamEndCapture(st, &g);
      hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      hipGraphLaunch(ge, st); hipStreamSynchronize(st);
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a, st);
      for (int r = 0; r < 20; ++r) hipGraphLaunch(ge, st);
      hipEventRecord(b, st); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("graph of 100 empty kernels (%d blocks): %.2f us per kernel\n", nb, ms * 1e3 / 2000.0);
    }
  }
  hipError_t e = hipDeviceSynchronize();
  printf("%s\n", hipGetErrorString(e));
  return 0;
}
