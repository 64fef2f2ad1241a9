// Development micro-benchmark: the 16-column panel factorisation of the 64x64 diagonal tile
// (potrfTile's wave-0 chain) in several formulations, one wavefront, timed over many repetitions.
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_pfac.hip -o /tmp/ubench_pfac
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

constexpr int kLd = 65;

__device__ __forceinline__ double readlaneD(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double rsqrt2(double d) {
  double r = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  r = r * (1.5 - h * r * r);
  r = r * (1.5 - h * r * r);
  return r;
}
__device__ __forceinline__ double rsqrt1(double d) {
  double r = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  const double e = fma(-h * r, r, 0.5);
  return fma(r, e, r);
}

// V0: current: readlane pivot + readlane column broadcasts
template <int RS>
__device__ void pfacV0(double* sA, double* sRl, int lane, int p) {
  const int i = lane;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = sA[i * kLd + 16 * p + c];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int col = 16 * p + c;
    const double dcc = readlaneD(a[c], col);
    const double rl = RS == 2 ? rsqrt2(dcc) : rsqrt1(dcc);
    if (lane == 0) sRl[col] = rl;
    const double l = (i == col) ? dcc * rl : a[c] * rl;
    a[c] = l;
#pragma unroll
    for (int j = c + 1; j < 16; ++j) a[j] -= l * readlaneD(l, 16 * p + j);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c)
    if (i >= 16 * p + c) sA[i * kLd + 16 * p + c] = a[c];
}

// V1: pivot by readlane; the column (lanes 16p..16p+15) staged through LDS, broadcast reads
__device__ void pfacV1(double* sA, double* sRl, double* sCol, int lane, int p) {
  const int i = lane;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = sA[i * kLd + 16 * p + c];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int col = 16 * p + c;
    const double dcc = readlaneD(a[c], col);
    const double rl = rsqrt2(dcc);
    if (lane == 0) sRl[col] = rl;
    const double l = (i == col) ? dcc * rl : a[c] * rl;
    a[c] = l;
    if (i >= 16 * p && i < 16 * p + 16) sCol[c * 16 + (i - 16 * p)] = l;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = c + 1; j < 16; ++j) a[j] -= l * sCol[c * 16 + j];
  }
#pragma unroll
  for (int c = 0; c < 16; ++c)
    if (i >= 16 * p + c) sA[i * kLd + 16 * p + c] = a[c];
}

// V2: look-ahead order: update column c+1 first, start its pivot, then the rest of column c
template <int RS>
__device__ void pfacV2(double* sA, double* sRl, int lane, int p) {
  const int i = lane;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = sA[i * kLd + 16 * p + c];
  double dcc = readlaneD(a[0], 16 * p);
  double rl = RS == 2 ? rsqrt2(dcc) : rsqrt1(dcc);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int col = 16 * p + c;
    if (lane == 0) sRl[col] = rl;
    const double l = (i == col) ? dcc * rl : a[c] * rl;
    a[c] = l;
    double ndcc = 0.0, nrl = 0.0;
    if (c + 1 < 16) {
      a[c + 1] -= l * readlaneD(l, col + 1);
      ndcc = readlaneD(a[c + 1], col + 1);
      nrl = RS == 2 ? rsqrt2(ndcc) : rsqrt1(ndcc);
    }
#pragma unroll
    for (int j = c + 2; j < 16; ++j) a[j] -= l * readlaneD(l, 16 * p + j);
    dcc = ndcc;
    rl = nrl;
  }
#pragma unroll
  for (int c = 0; c < 16; ++c)
    if (i >= 16 * p + c) sA[i * kLd + 16 * p + c] = a[c];
}

// V0 on wave 4 while waves 0..3 poll an LDS flag (the wave-specialised kernel's idle MFMA waves)
__global__ void kbenchSpin(const double* A, double* out, int reps, unsigned long long* ticks, int mode, int fw) {
  __shared__ double sA[64 * kLd];
  __shared__ double sRl[64];
  __shared__ int flag;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) flag = 0;
  for (int e = t; e < 64 * 64; e += blockDim.x) sA[(e >> 6) * kLd + (e & 63)] = A[e];
  __syncthreads();
  if (wave != fw) {
    if (mode == 1)
      while (__hip_atomic_load(&flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
    if (mode >= 2) {  // MFMA stream
      typedef double dbl4 __attribute__((ext_vector_type(4)));
      dbl4 acc = {0, 0, 0, 0};
      double av = 1.0 + lane, bv = 0.5;
      while (__hip_atomic_load(&flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        for (int q = 0; q < 16; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      if (acc[0] == 12345.0) out[0] = acc[1];
    }
    return;
  }
  unsigned long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < 4; ++p) {
      pfacV0<2>(sA, sRl, lane, p);
      __builtin_amdgcn_wave_barrier();
    }
    tot += __builtin_amdgcn_s_memrealtime() - t0;
    for (int e = lane; e < 64 * 64; e += 64) sA[(e >> 6) * kLd + (e & 63)] = A[e];
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0) {
    *ticks = tot;
    __hip_atomic_store(&flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// grid-wide: every block = wave 0 pfac + waves 1..3 MFMA, padded LDS so that 2 blocks share a CU
__global__ void kbenchGrid(const double* A, double* out, int reps, unsigned long long* ticks, int fw) {
  // fw < 0: waves 0 and 4 both run the panel chain (two windows per workgroup)
  extern __shared__ double dyn[];
  double* sA = dyn;
  double* sRl = dyn + 64 * kLd;
  __shared__ int flag;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) flag = 0;
  for (int e = t; e < 64 * 64; e += blockDim.x) sA[(e >> 6) * kLd + (e & 63)] = A[e];
  __syncthreads();
  const bool isF = fw >= 0 ? wave == fw : (wave & 3) == 0;
  if (fw < 0) { sA += (wave >> 2) * 64 * kLd; sRl = dyn + 2 * 64 * kLd + 64 * (wave >> 2); }
  if (fw < 0 && isF) {
    for (int e = lane; e < 64 * 64; e += 64) sA[(e >> 6) * kLd + (e & 63)] = A[e];
    __builtin_amdgcn_wave_barrier();
  }
  if (!isF) {
    typedef double dbl4 __attribute__((ext_vector_type(4)));
    dbl4 acc = {0, 0, 0, 0};
    double av = 1.0 + lane, bv = 0.5;
    while (__hip_atomic_load(&flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < (fw < 0 ? 2 : 1))
      for (int q = 0; q < 16; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    if (acc[0] == 12345.0) out[0] = acc[1];
    return;
  }
  unsigned long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < 4; ++p) {
      pfacV0<2>(sA, sRl, lane, p);
      __builtin_amdgcn_wave_barrier();
    }
    tot += __builtin_amdgcn_s_memrealtime() - t0;
    for (int e = lane; e < 64 * 64; e += 64) sA[(e >> 6) * kLd + (e & 63)] = A[e];
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0) {
    ticks[fw < 0 ? 2 * blockIdx.x + (wave >> 2) : blockIdx.x] = tot;
    if (fw >= 0) __hip_atomic_store(&flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_fetch_add(&flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

template <int V>
__global__ void kbench(const double* A, double* out, int reps, unsigned long long* ticks) {
  __shared__ double sA[64 * kLd];
  __shared__ double sRl[64];
  __shared__ double sCol[256];
  const int lane = threadIdx.x;
  unsigned long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    for (int e = lane; e < 64 * 64; e += 64) sA[(e >> 6) * kLd + (e & 63)] = A[e];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < 4; ++p) {
      if (V == 0) pfacV0<2>(sA, sRl, lane, p);
      if (V == 1) pfacV1(sA, sRl, sCol, lane, p);
      if (V == 2) pfacV2<2>(sA, sRl, lane, p);
      if (V == 3) pfacV0<1>(sA, sRl, lane, p);
      if (V == 4) pfacV2<1>(sA, sRl, lane, p);
      __syncthreads();
    }
    tot += __builtin_amdgcn_s_memrealtime() - t0;
  }
  for (int e = lane; e < 64 * 64; e += 64) out[e] = sA[(e >> 6) * kLd + (e & 63)];
  if (lane == 0) *ticks = tot;
}

int main() {
  std::vector<double> A(64 * 64);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) A[i * 64 + j] = (i == j) ? 64.0 + i : 1.0 / (1.0 + i + j);
  double *dA, *dO;
  unsigned long long* dT;
  hipMalloc(&dA, 8 * 4096);
  hipMalloc(&dO, 8 * 4096);
  hipMalloc(&dT, 8);
  hipMemcpy(dA, A.data(), 8 * 4096, hipMemcpyHostToDevice);
  const int reps = 200;
  std::vector<double> ref(4096), o(4096);
  const char* names[5] = {"V0 readlane rsqrt2", "V1 lds-broadcast", "V2 lookahead rsqrt2", "V3 readlane rsqrt1",
                          "V4 lookahead rsqrt1"};
  for (int v = 0; v < 5; ++v) {
    for (int pass = 0; pass < 2; ++pass) {
      switch (v) {
        case 0: hipLaunchKernelGGL(kbench<0>, 1, 64, 0, 0, dA, dO, reps, dT); break;
        case 1: hipLaunchKernelGGL(kbench<1>, 1, 64, 0, 0, dA, dO, reps, dT); break;
        case 2: hipLaunchKernelGGL(kbench<2>, 1, 64, 0, 0, dA, dO, reps, dT); break;
        case 3: hipLaunchKernelGGL(kbench<3>, 1, 64, 0, 0, dA, dO, reps, dT); break;
        case 4: hipLaunchKernelGGL(kbench<4>, 1, 64, 0, 0, dA, dO, reps, dT); break;
      }
      hipDeviceSynchronize();
    }
    unsigned long long t;
    hipMemcpy(&t, dT, 8, hipMemcpyDeviceToHost);
    hipMemcpy(o.data(), dO, 8 * 4096, hipMemcpyDeviceToHost);
    if (v == 0) ref = o;
    double md = 0;
    for (int e = 0; e < 4096; ++e) md = fmax(md, fabs(o[e] - ref[e]) / (fabs(ref[e]) + 1e-300));
    printf("%-22s %8.3f us per 64x64 pfac   max rel diff vs V0 %.2e\n", names[v], t * 10.0 / 1000.0 / reps, md);
  }
  const char* sn[6] = {"w4 pfac + 4 idle waves", "w4 pfac + 4 polling waves", "w4 pfac + 4 MFMA waves",
                       "w0 pfac + 1 MFMA wave", "w0 pfac + 3 MFMA waves", "w0 pfac + 7 MFMA waves"};
  const int thr[6] = {320, 320, 320, 128, 256, 512}, fws[6] = {4, 4, 4, 0, 0, 0}, md[6] = {0, 1, 2, 2, 2, 2};
  for (int mode = 0; mode < 6; ++mode) {
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(kbenchSpin, 1, thr[mode], 0, 0, dA, dO, reps, dT, md[mode], fws[mode]);
      hipDeviceSynchronize();
    }
    unsigned long long t;
    hipMemcpy(&t, dT, 8, hipMemcpyDeviceToHost);
    printf("%-26s %8.3f us per 64x64 pfac\n", sn[mode], t * 10.0 / 1000.0 / reps);
  }
  {
    unsigned long long* dTg;
    hipMalloc(&dTg, 8 * 2048);
    hipFuncSetAttribute((const void*)kbenchGrid, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    for (int cfg = 0; cfg < 3; ++cfg) {
      const int nb = cfg == 0 ? 256 : (cfg == 1 ? 512 : 256);
      const int nt = cfg == 2 ? 512 : 256, fw = cfg == 2 ? -1 : 0;
      const int lds = cfg == 2 ? 140 * 1024 : 72 * 1024;
      for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL(kbenchGrid, nb, nt, lds, 0, dA, dO, 20, dTg, fw);
        hipDeviceSynchronize();
      }
      const int nr = cfg == 2 ? 2 * nb : nb;
      std::vector<unsigned long long> tg(nr);
      hipMemcpy(tg.data(), dTg, 8 * nr, hipMemcpyDeviceToHost);
      double mx = 0, mean = 0;
      int slow = 0;
      for (int b = 0; b < nr; ++b) {
        const double us = tg[b] * 10.0 / 1000.0 / 20;
        mx = fmax(mx, us);
        mean += us / nr;
        slow += us > 20.0;
      }
      printf("cfg %d: grid %d x %d threads: mean %.2f max %.2f us, %d chains > 20 us\n", cfg, nb, nt, mean, mx, slow);
    }
  }
  return 0;
}
