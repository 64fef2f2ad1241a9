// dev_clock.hpp — development-only phase clocks of the kernels whose phases were profiled
// from the inside (k_cholesky / k_chol_bsub, k_eval_imu, k_lm_visit<1>, k_dogleg). Off in every product build:
// each macro below expands to nothing unless its OKG_*_CLOCK switch is given on the compiler line
// (make OPT="-O3 -DOKG_CHOL_CLOCK" etc.). The kernels only name the macros; the clock state and the
// printf reports live here.
#pragma once

// ---- k_cholesky / k_chol_bsub (-DOKG_CHOL_CLOCK): workgroup 0 accumulates s_memrealtime ticks
// (100 MHz) per phase and prints them at its end.
#ifdef OKG_CHOL_CLOCK
static __device__ unsigned long long g_cholClk[32];
#define CLK_INIT unsigned long long clkLast = __builtin_amdgcn_s_memrealtime();
#define CLK(i)                                                                  \
  if (blockIdx.x == 0 && threadIdx.x == 0) {                                    \
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();            \
    g_cholClk[i] += now - clkLast;                                              \
    clkLast = now;                                                              \
  }
#define CLKW(i, cond)                                                           \
  if (blockIdx.x == 0 && (cond)) {                                              \
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();            \
    g_cholClk[i] += now - clkLast;                                              \
    clkLast = now;                                                              \
  }
#define CHOL_CLK_REPORT(T)                                                                               \
  if (blockIdx.x == 0 && threadIdx.x == 0)                                                               \
    printf("CHOLCLK T=%d potrf %llu panel %llu update %llu bsub %llu | load %llu pfac %llu ptrail %llu " \
           "dinv %llu subd %llu store %llu y %llu | sweep: wait %llu lookahead %llu chol8 %llu "         \
           "publish %llu loop %llu (x10ns)\n",                                                            \
           (T), g_cholClk[0], g_cholClk[1], g_cholClk[2] + g_cholClk[11], g_cholClk[3], g_cholClk[4],    \
           g_cholClk[5], g_cholClk[6], g_cholClk[7], g_cholClk[8], g_cholClk[9], g_cholClk[10],          \
           g_cholClk[21], g_cholClk[22], g_cholClk[23], g_cholClk[24], g_cholClk[25]);
#define BSUB_CLK_REPORT(T)                                                                               \
  if (blockIdx.x == 0 && threadIdx.x == 0)                                                               \
    printf("BSUBCLK T=%d init %llu steps %llu (x10ns)\n", (T), g_cholClk[12], g_cholClk[13]);
#else
#define CLK_INIT
#define CLK(i)
#define CLKW(i, cond)
#define CHOL_CLK_REPORT(T)
#define BSUB_CLK_REPORT(T)
#endif

// ---- k_eval_imu (-DOKG_IMU_CLOCK): every wavefront accumulates its s_memrealtime ticks per phase in
// wave-uniform (scalar) registers and adds them to the totals once, at its end (per-phase atomics
// contended and inflated the phases they fell into); the last workgroup prints the totals. Uses the
// kernel's APPEND template parameter.
#ifdef OKG_IMU_CLOCK
static __device__ unsigned long long g_imuClk[16];
static __device__ unsigned int g_imuDone;
#define ICLK_INIT                                                                       \
  unsigned long long iclk = __builtin_amdgcn_s_memrealtime(), iacc[16];                 \
  for (int i_ = 0; i_ < 16; ++i_) iacc[i_] = 0;
#define ICLK(i)                                                                         \
  {                                                                                     \
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();                    \
    iacc[i] += now - iclk;                                                              \
    iclk = now;                                                                         \
  }
#define ICLK_END                                                                        \
  if (!APPEND && threadIdx.x == 0) {                                                    \
    for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&g_imuClk[i_], iacc[i_]);                 \
    __threadfence();                                                                    \
    if (atomicAdd(&g_imuDone, 1u) == (unsigned)((P.n_imu + kImuPerWG - 1) / kImuPerWG) - 1) { \
      printf("IMUCLK pro %llu chain %llu state %llu sqrt %llu resid %llu jac %llu | R %llu Q %llu I %llu S %llu " \
             "P %llu | sqrt: sym %llu chol %llu (x10ns) | eigen groups %llu | tail: stores %llu wait %llu\n", g_imuClk[0], g_imuClk[1], g_imuClk[2], g_imuClk[3], g_imuClk[4], g_imuClk[5], \
             g_imuClk[6], g_imuClk[7], g_imuClk[8], g_imuClk[9], g_imuClk[10], g_imuClk[11], g_imuClk[12], g_imuClk[13], g_imuClk[14], g_imuClk[15]);                               \
      for (int i_ = 0; i_ < 16; ++i_) g_imuClk[i_] = 0;                                 \
      g_imuDone = 0;                                                                    \
    }                                                                                   \
  }
#define ICLK_COUNT(i, cond) \
  if (cond) atomicAdd(&g_imuClk[i], 1ull);
#else
#define ICLK_INIT
#define ICLK(i)
#define ICLK_COUNT(i, cond)
#define ICLK_END
#endif

// ---- k_lm_visit<1> (-DOKG_LMV_CLOCK): thread 0 of every workgroup adds its s_memrealtime ticks per
// phase with vector atomics; the last landmark group prints the totals (also inside k_lin_few, whose
// grid has further blocks). Uses the kernel's `mode` and `P`.
#ifdef OKG_LMV_CLOCK
static __device__ unsigned long long g_lmvClk[8];
static __device__ unsigned int g_lmvDone;
#define LCLK_INIT unsigned long long lclk = __builtin_amdgcn_s_memrealtime();
#define LCLK(i)                                                                         \
  if (mode == 1 && threadIdx.x == 0) {                                                  \
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();                    \
    atomicAdd(&g_lmvClk[i], now - lclk);                                                \
    lclk = now;                                                                         \
  }
#define LCLK_END                                                                        \
  if (mode == 1 && threadIdx.x == 0) {                                                  \
    __threadfence();                                                                    \
    if (atomicAdd(&g_lmvDone, 1u) == (unsigned)P.n_lmg - 1) {                          \
      printf("LMVCLK visit %llu lm %llu seg %llu z %llu stage %llu part %llu (x10ns, summed)\n", \
             g_lmvClk[0], g_lmvClk[1], g_lmvClk[2], g_lmvClk[3], g_lmvClk[4], g_lmvClk[5]);       \
      for (int i = 0; i < 8; ++i) g_lmvClk[i] = 0;                                      \
      g_lmvDone = 0;                                                                    \
    }                                                                                   \
  }
#define LCLK_TAIL(i) \
  __syncthreads();   \
  LCLK(i)            \
  LCLK_END
#else
#define LCLK_INIT
#define LCLK(i)
#define LCLK_END
#define LCLK_TAIL(i)
#endif

// ---- k_cholesky_pipe (-DOKG_PIPE_CLOCK): workgroup 0, one thread per team (t 0: team F, t 256:
// team B) accumulates s_memrealtime ticks (100 MHz) per phase; printed at the kernel's end.
#ifdef OKG_PIPE_CLOCK
static __device__ unsigned long long g_pipeClk[16];
#define PCLK_INIT unsigned long long pclk = __builtin_amdgcn_s_memrealtime();
#define PCLK(i, tid)                                                            \
  if (blockIdx.x == 0 && threadIdx.x == (tid)) {                                \
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();            \
    g_pipeClk[i] += now - pclk;                                                 \
    pclk = now;                                                                 \
  }
#define PCLK_REPORT(T)                                                                                   \
  if (blockIdx.x == 0 && threadIdx.x == 0)                                                               \
    printf("PIPECLK T=%d F: wait %llu potrf %llu | B: waitX %llu prep %llu crit %llu panels %llu "       \
           "updates %llu prefetch %llu | F tail %llu bsub %llu (x10ns)\n",                              \
           (T), g_pipeClk[0], g_pipeClk[1], g_pipeClk[2], g_pipeClk[3], g_pipeClk[4], g_pipeClk[5],       \
           g_pipeClk[6], g_pipeClk[7], g_pipeClk[9], g_pipeClk[8]);
#else
#define PCLK_INIT
#define PCLK(i, tid)
#define PCLK_REPORT(T)
#endif

// ---- k_dogleg (-DOKG_DOGLEG_CLOCK): workgroup 0, thread 0 after an added workgroup barrier per
// phase (the barriers are part of the clock build only); prints the per-call averages every 200 calls.
#ifdef OKG_DOGLEG_CLOCK
static __device__ unsigned long long g_dlClk[8], g_dlCalls;
#define DLCLK_INIT unsigned long long dlclk = __builtin_amdgcn_s_memrealtime();
#define DLCLK(i)                                                                \
  __syncthreads();                                                              \
  if (blockIdx.x == 0 && threadIdx.x == 0) {                                    \
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();            \
    g_dlClk[i] += now - dlclk;                                                  \
    dlclk = now;                                                                \
  }
#define DLCLK_END                                                                                        \
  if (blockIdx.x == 0 && threadIdx.x == 0 && ++g_dlCalls == 200) {                                       \
    printf("DLCLK per call (x10ns): state %.1f pass1 loads %.1f tree1 %.1f pass2 f %.1f pass2 lm %.1f " \
           "tree2 %.1f\n", g_dlClk[0] / 200.0, g_dlClk[1] / 200.0, g_dlClk[2] / 200.0, g_dlClk[3] / 200.0, \
           g_dlClk[4] / 200.0, g_dlClk[5] / 200.0);                                                      \
    for (int i_ = 0; i_ < 8; ++i_) g_dlClk[i_] = 0;                                                      \
    g_dlCalls = 0;                                                                                       \
  }
#else
#define DLCLK_INIT
#define DLCLK(i)
#define DLCLK_END
#endif
