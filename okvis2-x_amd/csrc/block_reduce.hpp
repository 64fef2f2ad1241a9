// block_reduce.hpp — fixed-order per-workgroup reductions and the batched strided loop of the
// per-window kernels (k_reduce, k_gradnorm, k_dogleg; the gradient norms also run inside the
// few-window assembly launch, kernels_schur.hip).
#pragma once
#include "okvisgpu_math.hpp"

namespace okg {

// Fixed-order tree reductions over the workgroup. The barriers order LDS only (ldsBarrier): a
// __syncthreads() also waited for every global store still in flight (k_dogleg's Plus pass leaves
// thousands), and N values reduced together share one tree's barriers: per value the same
// additions in the same order as a separate tree, so the same bits.
// The levels that pair entries of different wavefronts (s >= 128) go through LDS with a barrier
// each; the last seven (s = 64 .. 1) run in wavefront 0, lane t holding entry t, each level adding
// lane t + s to lane t as the LDS level did (same pairs, same operand order, so the same bits):
// 6 barriers per tree instead of 12 at 1,024 threads (a single window's reductions), 4 instead of
// 10 at 256.
template <int RB, class Op>
__device__ __forceinline__ double treeTail(const double* sh, int t, Op op) {  // (t < 64; entry 0's total in lane 0)
  double a = RB >= 128 ? op(sh[t], sh[t + 64]) : sh[t];
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) a = op(a, __shfl_down(a, s, 64));
  return a;
}
template <int RB, int N>
__device__ __forceinline__ void blockSumN(double (&v)[N], double* sh) {  // sh: N * RB doubles
  static_assert(RB >= 64 && (RB & (RB - 1)) == 0, "a power of two from 64");
  const int t = threadIdx.x;
#pragma unroll
  for (int n = 0; n < N; ++n) sh[n * RB + t] = v[n];
  ldsBarrier();
  for (int s = RB / 2; s >= 128; s >>= 1) {
    if (t < s) {
#pragma unroll
      for (int n = 0; n < N; ++n) sh[n * RB + t] += sh[n * RB + t + s];
    }
    ldsBarrier();
  }
  if (t < 64) {
    double r[N];
#pragma unroll
    for (int n = 0; n < N; ++n) r[n] = treeTail<RB>(sh + n * RB, t, [](double x, double y) { return x + y; });
    __builtin_amdgcn_wave_barrier();  // (every lane's reads of sh before lane 0's writes)
    if (t == 0) {
#pragma unroll
      for (int n = 0; n < N; ++n) sh[n * RB] = r[n];
    }
  }
  ldsBarrier();
#pragma unroll
  for (int n = 0; n < N; ++n) v[n] = sh[n * RB];
  ldsBarrier();
}
template <int RB>
__device__ __forceinline__ double blockSum(double v, double* sh) {
  double a[1] = {v};
  blockSumN<RB, 1>(a, sh);
  return a[0];
}
// Strided per-thread loop over i = b + t, b + t + RB, ... < e with the loads of U consecutive
// iterations issued before any of them is consumed. A window's reductions run in one workgroup, so a
// single window is a chain of dependent loads per thread; batching shortens it U-fold. use() sees the
// elements in the order of the plain loop, so every sum is bitwise the same.
template <int RB, int U, class Load, class Use>
__device__ __forceinline__ void stridedBatched(int b, int e, Load load, Use use) {
  int i = b + (int)threadIdx.x;
  for (; i + (U - 1) * RB < e; i += U * RB) {
    decltype(load(i)) v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = load(i + u * RB);
#pragma unroll
    for (int u = 0; u < U; ++u) use(i + u * RB, v[u]);
  }
  for (; i < e; i += RB) use(i, load(i));
}

template <int RB>
__device__ __forceinline__ double blockMax(double v, double* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  ldsBarrier();
  for (int s = RB / 2; s >= 128; s >>= 1) {
    if (t < s) sh[t] = fmax(sh[t], sh[t + s]);
    ldsBarrier();
  }
  if (t < 64) {
    const double m = treeTail<RB>(sh, t, [](double x, double y) { return fmax(x, y); });
    __builtin_amdgcn_wave_barrier();
    if (t == 0) sh[0] = m;
  }
  ldsBarrier();
  const double r = sh[0];
  ldsBarrier();
  return r;
}

}  // namespace okg
