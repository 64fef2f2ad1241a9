// kernels_chol_pipe.hip — the pipelined persistent schedule of the reduced camera matrix's LLT
// (Cholesky schedule 4, runtime.cpp setOptions): one 512-thread workgroup per window, split into two
// teams of four wavefronts that work on consecutive steps of the right-looking factorisation.
//
//   team F (wavefronts 0-3): the diagonal tiles, potrfTile (L_kk, X_k = L_kk^-1, y_k = X_k rhs_k),
//            one after the other, each followed by the step's critical pair: the panel L_(k+1)k
//            (X_k still in LDS) and its update of tile (k+1, k+1), which stays in LDS for the next
//            factor;
//   team B (wavefronts 4-7): step k's other panels L_ik = A_ik X_k^T with rhs_i -= A_ik X_k^T y_k
//            and band updates A_ij -= L_ik L_jk^T, on the FP64 matrix cores.
//
// The persistent kernel (k_cholesky<0>) runs the three phases of a step one after the other with
// the whole workgroup, so while wavefront 0 walks the diagonal tile's latency chain the matrix cores
// wait. Here team B takes X_k (into registers, in MFMA fragment order) as soon as team F has it and
// runs the step's other panels and updates (row k+2 first: the next critical pair reads it) while
// team F forms the critical pair and factors tile k+1. The step time becomes factor + one panel +
// one update instead of factor + every panel and update of the step. (Until round 5 team B formed
// the critical pair and handed the tile over; the team-F form is 3 % faster at one window per CU,
// gpurun_out r05ag: team B no longer waits with its own step's work queued behind the pair.)
//
// The tile operations are those of the other schedules (chol_tiles.hpp: the same routines, the same
// operands, each tile's updates in step order), so the factorisation gives their bits. The teams
// synchronise through LDS flags (workgroup-scope release / acquire, which also order the global W
// tiles one team writes and the other reads) and barriers of their own four wavefronts; the
// backward substitution runs on all 512 threads once both teams are done.
#include "chol_tiles.hpp"
#include "launch.hpp"

namespace okg {

// Barrier of one team's four wavefronts on an LDS arrival counter (LOCAL: orders LDS only; else
// also the global stores of the team, e.g. W tiles another wavefront of the team reads next).
template <bool LOCAL>
struct TeamSync {
  int* ctr;
  int* gen;
  int lane;
  __device__ __forceinline__ void operator()() const { waveBarrier<LOCAL>(ctr, *gen, 4, lane); }
};

// X^T's B-operand fragments of mfmaTileNT(sA, sX) for this wavefront (columns c0 + 16 b + lr,
// k = 4 q + lk), so that the panels of a step no longer need X in LDS.
__device__ __forceinline__ void loadXFrag(const double* sX, double (&xf)[16][2], int t) {
  const int wave = t >> 6, lane = t & 63;
  const int c0 = 32 * (wave & 1), lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int q = 0; q < 16; ++q)
#pragma unroll
    for (int b = 0; b < 2; ++b) xf[q][b] = sX[(c0 + 16 * b + lr) * kLd + 4 * q + lk];
}
// acc = sA X^T with X^T's fragments in registers: the MFMA sequence of mfmaTileNT(sA, sX), cut
// where X's upper triangle (exact zeros) would only add zeros (block column cb needs k < 16 (cb + 1):
// mfmaPanelRows in chol_tiles.hpp), so the same bits: 24 MFMAs on the wavefronts of block columns
// 0-1, 56 on those of 2-3, instead of 64.
template <int HALF>
__device__ __forceinline__ void mfmaTileNTXHalf(const double* sA, const double (&xf)[16][2], dbl4 acc[2][2], int r0,
                                                int lr, int lk) {
#pragma unroll
  for (int q = 0; q < 8 + 8 * HALF; ++q) {
    double av[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) av[a] = sA[(r0 + 16 * a + lr) * kLd + 4 * q + lk];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        if (q < 4 * (2 * HALF + b + 1))  // (block column 2 HALF + b)
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], xf[q][b], acc[a][b], 0, 0, 0);
  }
}
__device__ __forceinline__ void mfmaTileNTX(const double* sA, const double (&xf)[16][2], dbl4 acc[2][2], int t) {
  const int wave = t >> 6, lane = t & 63;
  const int r0 = 32 * (wave >> 1);
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  if (wave & 1) mfmaTileNTXHalf<1>(sA, xf, acc, r0, lr, lk);
  else mfmaTileNTXHalf<0>(sA, xf, acc, r0, lr, lk);
}

// Panel of team B: L_ik = A_ik X^T (A_ik staged in sBuf), rhs_i -= A_ik z (panelTile's
// operations), L_ik stored to W and left in sBuf for the step's band updates.
// (defer: the split schedule's right part stores the rhs term of a separator row instead, for the
// separator's launch to subtract in step order)
template <class Sync>
__device__ __forceinline__ void pipePanel(const double* Aik, double* Lik, int64_t ld, double* worki, double* sBuf,
                                          const double (&xf)[16][2], const double* sz, int t, Sync sync,
                                          double* defer = nullptr) {
  loadTile(Aik, ld, 0, 0, sBuf, t);
  sync();
  dbl4 acc[2][2];
  mfmaTileNTX(sBuf, xf, acc, t);
  const double a = panelRhsRow(sBuf, sz, t);
  if ((t & 3) == 0) {
    if (defer) defer[t >> 2] = a;
    else worki[t >> 2] -= a;  // rhs_i in LDS
  }
  sync();  // every wavefront has read A_ik
  accToLds(sBuf, acc, t);
  storeTile<false>(Lik, ld, 0, 0, acc, t);
  sync();  // L_ik in sBuf for every wavefront of the team
}

// Wavefront -> team. On gfx950 wavefront w of a 512-thread workgroup runs on SIMD (3, 0, 2, 1)[w % 4]
// (HW_ID, scripts/ubench_team.hip), and FP64 MFMAs on a SIMD stall the FP64 VALU chain of another
// wavefront there: with team B's products beside it the diagonal factor took 46-70 us per tile
// against 18 alone. MAP 1: team F = the even wavefronts (SIMDs 3, 2), team B = the odd ones (SIMDs
// 0, 1), so the chain never shares a SIMD with team B, but team B's products then take ~4.1 us
// instead of ~2.9 on half the matrix cores; MAP 0 (default): F = wavefronts 0-3, B = 4-7, one of
// each team per SIMD. One window per CU (256 S50 windows): MAP 0 168.0k against MAP 1 161.6k
// window-it/s (gpurun_out r05f): team B's step work outweighs the chain's slowdown.
// A third mapping from the SIMD each wavefront landed on (HW_ID), team F = the chain, its SIMD's
// other wavefront and one wavefront on each of two further SIMDs, team B = the rest (three SIMDs,
// none shared with the chain), ran 163.0k against 169.5k window-it/s (k_cholesky 0.578 against
// 0.515 ms, gpurun_out r05m) and was removed.
#ifndef OKG_PIPE_MAP
#define OKG_PIPE_MAP 0
#endif
// The teams' waits on each other. fail (pipe[3]) = 1: team F met a non-positive pivot and stopped;
// it set no flag after that, so once fail is seen the flag has its final value and is re-read:
// every wavefront of a team returns the same outcome (a wavefront that saw the flag earlier saw a
// value the re-read also sees), and the team barriers that follow stay matched. A spin limit no
// correct run reaches (~1 s) ends a wait that never completes with fail = 2 (atomic max, so a pivot
// failure is not overwritten): the window is reported as a device error (WinState::dev_error ->
// OKVISGPU_ERR_DEVICE), not as a failed GN step, instead of hanging the device.
__device__ __forceinline__ bool pipeWait(int* p, int v, int* fail) {
  for (int it = 0; it < (1 << 24); ++it) {
    if (ldsAcquire(p) >= v) return true;
    if (ldsAcquire(fail)) return ldsAcquire(p) >= v;
    __builtin_amdgcn_s_sleep(OKG_WAIT_SLEEP);
  }
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_max(fail, 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  return ldsAcquire(p) >= v;
}

// LDS of the pipelined kernel besides the window's rhs / y (dynamic, ld doubles)
struct PipeLds {
  double sA[kTile * kLd];     // F: the diagonal tile being factored, then the critical pair's operands
  double sX[kTile * kLd];     // F: X_k
  double sB[2][kTile * kLd];  // B: A_ik staging / the step's L tiles
  double sy[2 * kTile];       // F: rhs_k -> y_k | scratch (backward substitution: y_I)
  double sz[2 * kTile];       // B: y_k | z_k = X_k^T y_k
  double sRl[kTile];          // F: 1 / L_cc
  int sFl[8];                 // potrfTile's flags [0..3], team F's barrier [4], team B's barrier [5]
  int pipe[8];                // [0] steps factored (F), [1] X_k taken (B), [3] failed pivot, [4]
                              // critical panels stored (F), [5] rows whose earlier updates are
                              // applied (B)
};

// MODE 0: the whole window (schedule 4). MODE 1: launch A of the split schedule over a nested-
// dissection window's two independent parts (schedule 5; k_cholesky<1>'s roles, pipelined):
// workgroup 2w + part runs the part's steps [k0, k1); the right part (part 1) updates only targets
// left of the separator and, for the separator's rows, stores L and each panel's rhs term
// (chol_defer); both leave their y / rhs rows in fwdF for launch B (k_cholesky<2>: the separator's
// contributions in step order, its factorisation and the backward substitution). A window without
// a split runs MODE 0's work in part 0.
template <int MODE>
__global__ __launch_bounds__(512, 1) void k_cholesky_pipe(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = MODE == 1 ? (int)(blockIdx.x >> 1) : (int)blockIdx.x, part = MODE == 1 ? (int)(blockIdx.x & 1) : 0;
  if (!cholSelect(P, w)) return;  // (uniform over the workgroup)
  const int64_t ld = P.win_fpad[w];
  const int T = (int)(ld / kTile);
  const int tL = MODE == 0 ? 0 : P.win_bsplit[2 * w], tS = MODE == 0 ? 0 : P.win_bsplit[2 * w + 1];
  const bool split = MODE != 0 && tS > 0;
  if (MODE == 1 && part == 1 && !split) return;
  const int k0 = !split ? 0 : (part == 0 ? 0 : tL), k1 = !split ? T : (part == 0 ? tL : tS);
  const int jEnd = split && part == 1 ? tS : T;  // targets (i, j) with j < jEnd
  double* defer = split && part == 1 ? P.chol_defer + P.win_defoff[w] : nullptr;
  auto deferAt = [&](int i, int k) { return defer + ((size_t)(i - tS) * (tS - tL) + (k - tL)) * kTile; };
  const TileSrc cur = tileSrc(P, w, ld);
  double* W = P.W + P.win_soff[w];
  double* Linv = P.Linv + P.win_linvoff[w];
  const uint8_t* nz = P.tile_nz + P.win_tnzoff[w];
  __shared__ PipeLds L;
  extern __shared__ double sxDyn[];  // rhs / y of the whole window
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int team = OKG_PIPE_MAP == 0 ? wave >> 2 : wave & 1;
  const int tt = (OKG_PIPE_MAP == 0 ? (wave & 3) : (wave >> 1)) * 64 + lane;
  const int fdim = P.win_fdim[w];
  for (int e = t; e < ld; e += 512) sxDyn[e] = (e < fdim) ? P.rhsF[(size_t)P.win_foff[w] + e] : 0.0;
  if (t < 8) L.sFl[t] = 0;
  if (t < 8) L.pipe[t] = t == 5 ? k0 + 1 : 0;  // (row k0+1 has no updates of earlier steps in this part)
  __syncthreads();
  PCLK_INIT
  if (team == 0) {
    // ---- team F: the diagonal tiles in order, and after each the critical pair of the step: panel
    // L_(k+1)k = A_(k+1)k X_k^T (X_k still in sX) and its update of tile (k+1, k+1), which stays in
    // sA for the next factor. Team B takes the rest of the step.
    int fgen = 0;
    const TeamSync<false> fsync{&L.sFl[4], &fgen, lane};
    const TeamSync<true> fsyncL{&L.sFl[4], &fgen, lane};
    bool inLds = false;  // tile k already in sA (the previous step's critical update)
    for (int k = k0; k < k1; ++k) {
      if (k > k0) {
        // X_(k-1) taken by team B (sX is overwritten next); without the critical update in sA the
        // tile comes from W once team B has applied its updates
        if (!pipeWait(&L.pipe[1], k, &L.pipe[3])) break;
        if (!inLds && !pipeWait(&L.pipe[5], k, &L.pipe[3])) break;
      }
      PCLK(0, 0)
      if (tt < kTile) L.sy[tt] = sxDyn[k * kTile + tt];
      if (!potrfTileBody<20>(cur.at(k, k, k), ld, Linv + (int64_t)k * kTile * kTile, nullptr, L.sA, L.sX, L.sy, L.sRl,
                             L.sFl, tt, inLds, fgen, tileBlocks(P, w, k))) {
        if (tt == 0) ldsRelease(&L.pipe[3], 1);
        break;
      }
      fgen += kPotrfBarriers;
      if (tt < kTile) sxDyn[k * kTile + tt] = L.sy[tt];  // y_k
      if (tt == 0) ldsRelease(&L.pipe[0], k + 1);         // X_k in sX, y_k in sxDyn
      PCLK(1, 0)
      inLds = false;
      if (k + 1 < k1 && nz[(k + 1) * T + k]) {
        // tiles (k+1, k) and (k+1, k+1) have team B's updates of the earlier steps
        int tc = tt;  // (opaque: the section's addresses are formed here, not held across the loop)
        asm volatile("" : "+v"(tc));
        if (!pipeWait(&L.pipe[5], k + 1, &L.pipe[3])) break;
        panelRhsVector(L.sX, L.sy, L.sy + kTile, L.sA, tc, fsyncL);  // z_k (sA: scratch, L_kk is not needed)
        loadTile(cur.at(k + 1, k, k), ld, 0, 0, L.sA, tc);
        dbl4 c[3];
        loadCDiag(cur.at(k + 1, k + 1, k), ld, c, tc);  // (in flight during the panel)
        fsyncL();
        dbl4 acc[4];
        mfmaPanelRows(L.sA, L.sX, acc, tc);
        {
          const double a = panelRhsRow(L.sA, L.sy + kTile, tc);
          if ((tc & 3) == 0) sxDyn[(k + 1) * kTile + (tc >> 2)] -= a;  // rhs_(k+1) in LDS
        }
        fsyncL();  // every wavefront has read A_(k+1)k
        panelRowsToLds(L.sA, acc, tc);
        storePanelRows(W + (int64_t)(k + 1) * kTile * ld + k * kTile, ld, acc, tc);
        fsyncL();
        dbl4 acc3[3];
        mfmaDiagNT(L.sA, acc3, tc);
        fsyncL();  // every wavefront has read L_(k+1)k
        diagSubToLds(L.sA, c, acc3, tc);
        fsync();  // (orders the L_(k+1)k stores before the flag)
        if (tc == 0) ldsRelease(&L.pipe[4], k + 1);  // L_(k+1)k in W
        inLds = true;
        PCLK(2, 0)
      }
    }
  } else {
    // ---- team B: the step's other panels and band updates once X_k is there
    const int tt0 = tt;
    int bgen = 0;
    const TeamSync<false> bsync{&L.sFl[5], &bgen, lane};
    const TeamSync<true> bsyncL{&L.sFl[5], &bgen, lane};
    double xf[16][2];
    for (int k = k0; k < k1; ++k) {
      if (!pipeWait(&L.pipe[0], k + 1, &L.pipe[3])) break;
      PCLK(3, 256)
      bool below = false;  // (a step without tiles below has nothing for team B)
      for (int i = k + 1; i < T; ++i) below = below || nz[i * T + k];
      if (!below) {
        if (tt0 == 0) {
          ldsRelease(&L.pipe[1], k + 1);
          ldsRelease(&L.pipe[5], k + 2);
        }
        continue;
      }
      // the thread index, opaque per step: the step's LDS / global addresses are formed in the step
      // instead of being hoisted out of the loop (and spilled: the kernel is at 256 VGPRs)
      int tt = tt0;
      asm volatile("" : "+v"(tt));
      // z_k = X_k^T y_k and X_k into registers from team F's sX, then sX is released
      if (tt < kTile) L.sz[tt] = sxDyn[k * kTile + tt];
      bsyncL();
      panelRhsVector(L.sX, L.sz, L.sz + kTile, L.sB[1], tt, bsyncL);
      loadXFrag(L.sX, xf, tt);
      bsyncL();
      if (tt == 0) ldsRelease(&L.pipe[1], k + 1);
      const bool crit = k + 1 < k1 && nz[(k + 1) * T + k] != 0;
      int held[2] = {-1, -1};  // block row i of the L_ik in sB[0] / sB[1]
      int hb = 0;
      // the step's other panels (the last two stay in LDS for the updates); without the critical
      // pair this includes row k+1: at the end of a part of a split window, where tile k+1 is the
      // separator's
      for (int i = crit ? k + 2 : k + 1; i < T; ++i) {
        if (!nz[i * T + k]) continue;
        pipePanel(cur.at(i, k, k), W + (int64_t)i * kTile * ld + k * kTile, ld, sxDyn + i * kTile, L.sB[hb], xf,
                  L.sz + kTile, tt, bsyncL, i >= jEnd ? deferAt(i, k) : nullptr);
        held[hb] = i;
        hb ^= 1;
      }
      bsync();  // the L tiles in W for reloads by other wavefronts of the team
      if (crit && !pipeWait(&L.pipe[4], k + 1, &L.pipe[3])) break;  // L_(k+1)k from team F
      PCLK(4, 256)
      // band updates A_ij -= L_ik L_jk^T of step k but (k+1, k+1) (team F's): row k+2 first (team
      // F's next critical pair reads it), then the rest bottom-up; each tile once per step, so the
      // order across tiles does not change the bits
      for (int r = 0; r < T; ++r) {
        const int i = r == 0 ? k + 2 : (r == 1 ? k + 1 : T + 1 - r);  // k+2, k+1, T-1, ..., k+3
        if (i <= k || i >= T || (r >= 2 && i <= k + 2) || !nz[i * T + k]) {
          if (r == 0) {
            bsync();
            if (tt == 0) ldsRelease(&L.pipe[5], k + 2);
          }
          continue;
        }
        for (int j = k + 1; j <= i; ++j) {
          if (!nz[j * T + k] || (i == k + 1 && crit) || j >= jEnd) continue;
          int bi = held[0] == i ? 0 : (held[1] == i ? 1 : -1);
          int bj = j == i ? bi : (held[0] == j ? 0 : (held[1] == j ? 1 : -1));
          bool loaded = false;
          if (bi < 0) {
            bi = bj >= 0 ? bj ^ 1 : 0;
            loadTile(W + (int64_t)i * kTile * ld + k * kTile, ld, 0, 0, L.sB[bi], tt);
            held[bi] = i;
            if (j == i) bj = bi;
            loaded = true;
          }
          if (bj < 0) {
            bj = bi ^ 1;
            loadTile(W + (int64_t)j * kTile * ld + k * kTile, ld, 0, 0, L.sB[bj], tt);
            held[bj] = j;
            loaded = true;
          }
          if (loaded) bsyncL();
          if (j == i) {
            dbl4 c[3], acc[3];
            loadCDiag(cur.at(i, j, k), ld, c, tt);
            mfmaDiagNT(L.sB[bi], acc, tt);
            storeDiagSub(W + (int64_t)i * kTile * ld + j * kTile, ld, c, acc, tt);
          } else {
            dbl4 c[2][2], acc[2][2];
            loadC(cur.at(i, j, k), ld, c, tt);
            mfmaTileNT(L.sB[bi], L.sB[bj], acc, tt);
            storeTileSub(W + (int64_t)i * kTile * ld + j * kTile, ld, c, acc, tt);
          }
          bsyncL();  // the operands may be replaced next
        }
        if (r == 0) {  // row k+2 done: team F's next critical pair may read its tiles
          bsync();
          if (tt == 0) ldsRelease(&L.pipe[5], k + 2);
        }
      }
      bsync();  // the updated tiles in W for the next step's panels
      PCLK(7, 256)
    }
  }
  __syncthreads();
  if (L.pipe[3]) {
    if (t == 0) {
      if (L.pipe[3] == 1) P.st[w].gn_failed = 1;  // non-positive pivot: the GN step is retried
      else P.st[w].dev_error = 1;                 // wait limit
    }
    return;
  }
  if (split) {  // launch A: this part's rows of y (part 0 also the separator's rhs) for launch B
    double* work = P.fwdF + P.win_fwdoff[w];
    const int e0 = part == 0 ? 0 : tL * kTile, e1 = part == 0 ? tL * kTile : tS * kTile;
    for (int e = t; e < ld; e += 512)
      if ((e >= e0 && e < e1) || (part == 0 && e >= tS * kTile)) work[e] = sxDyn[e];
    return;
  }
  PCLK(9, 0)
  backSubstitute<512>(P, w, W, ld, T, Linv, nz, sxDyn, L.sB[0], L.sy, t);
  PCLK(8, 0)
  PCLK_REPORT(T)
}

bool cholesky_pipe_fits(int max_fpad, size_t lds_per_block) {
  hipFuncAttributes attr;
  if (hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(k_cholesky_pipe<1>)) != hipSuccess) return false;
  return attr.sharedSizeBytes + sizeof(double) * (size_t)max_fpad <= lds_per_block;
}

// split: schedule 5 (launch A pipelined per nested-dissection part, launch B = k_cholesky<2>)
void launch_cholesky_pipe(const DevProblem& P, hipStream_t s, bool split) {
  if (P.n_win == 0) return;
  if (!split) {
    hipLaunchKernelGGL(k_cholesky_pipe<0>, dim3(P.n_win), dim3(512), sizeof(double) * P.max_fpad, s, P.self);
    return;
  }
  hipLaunchKernelGGL(k_cholesky_pipe<1>, dim3(2 * P.n_win), dim3(512), sizeof(double) * P.max_fpad, s, P.self);
  launch_cholesky_split_b(P, s);
}

}  // namespace okg
