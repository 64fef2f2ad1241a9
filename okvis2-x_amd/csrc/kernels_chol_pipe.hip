// kernels_chol_pipe.hip — the pipelined persistent schedule of the reduced camera matrix's LLT
// (Cholesky schedule 4, runtime.cpp setOptions): one 512-thread workgroup per window, split into two
// teams of four wavefronts that work on consecutive steps of the right-looking factorisation.
//
//   team F (wavefronts 0-3): the diagonal tiles, potrfTile (L_kk, X_k = L_kk^-1, y_k = X_k rhs_k),
//            one after the other;
//   team B (wavefronts 4-7): step k's panels L_ik = A_ik X_k^T with rhs_i -= A_ik X_k^T y_k and band
//            updates A_ij -= L_ik L_jk^T, on the FP64 matrix cores.
//
// The persistent kernel (k_cholesky<0>) runs the three phases of a step one after the other with
// the whole workgroup, so while wavefront 0 walks the diagonal tile's latency chain the matrix cores
// wait. Here team B takes X_k (into registers, in MFMA fragment order) as soon as team F has it and
// first runs the two products on the critical path — the panel L_(k+1)k and its update of the next
// diagonal tile, which it writes straight into team F's LDS tile — then hands tile k+1 to team F
// and runs the step's other panels and updates while team F factors it. The step time becomes
// factor + one panel + one update instead of factor + every panel and update of the step.
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
// (staged: A_ik is in sBuf already, prefetched by the previous step)
template <class Sync>
__device__ __forceinline__ void pipePanel(const double* Aik, double* Lik, int64_t ld, double* worki, double* sBuf,
                                          const double (&xf)[16][2], const double* sz, int t, Sync sync,
                                          double* defer = nullptr, bool staged = false) {
  if (!staged) loadTile(Aik, ld, 0, 0, sBuf, t);
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

// LDS of the pipelined kernel besides the window's rhs / y (dynamic, ld doubles)
struct PipeLds {
  double sA[kTile * kLd];     // F: the diagonal tile being factored (team B writes the next one here)
  double sX[kTile * kLd];     // F: X_k
  double sB[2][kTile * kLd];  // B: A_ik staging / the step's L tiles
  double sy[2 * kTile];       // F: rhs_k -> y_k | scratch (backward substitution: y_I)
  double sz[2 * kTile];       // B: y_k | z_k = X_k^T y_k
  double sRl[kTile];          // F: 1 / L_cc
  int sFl[8];                 // potrfTile's flags [0..3], team F's barrier [4], team B's barrier [5]
  int pipe[4];                // [0] steps factored (F), [1] diagonal tiles handed over (B),
                              // [2] the handed-over tile is in sA, [3] failed pivot
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
  if (t < 4) L.pipe[t] = 0;
  __syncthreads();
  PCLK_INIT
  if (team == 0) {
    // ---- team F: the diagonal tiles in order
    int fgen = 0;
    for (int k = k0; k < k1; ++k) {
      bool inLds = false;
      if (k > k0) {  // tile k has all its updates (and rhs_k its panel terms); X_(k-1) was taken
        if (!waitFlag<false>(&L.pipe[1], k, &L.pipe[3])) break;
        inLds = L.pipe[2] != 0;
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
    }
  } else {
    // ---- team B: the panels and band updates of step k once X_k is there
    const int tt0 = tt;
    int bgen = 0;
    const TeamSync<false> bsync{&L.sFl[5], &bgen, lane};
    const TeamSync<true> bsyncL{&L.sFl[5], &bgen, lane};
    double xf[16][2];
    int staged = -1;  // the step whose critical A_(k+1)k is in sB[0] (prefetched at the previous step's end)
    for (int k = k0; k < k1; ++k) {
      PCLK(6, 256)
      if (!waitFlag<false>(&L.pipe[0], k + 1, &L.pipe[3])) break;
      PCLK(2, 256)
      bool below = false;  // (a step without tiles below only hands the next tile over)
      for (int i = k + 1; i < T; ++i) below = below || nz[i * T + k];
      if (!below) {
        if (tt0 == 0) {
          L.pipe[2] = 0;
          ldsRelease(&L.pipe[1], k + 1);
        }
        continue;
      }
      // the thread index, opaque per step: the step's LDS / global addresses are formed in the step
      // instead of being hoisted out of the loop (and spilled: the kernel is at 256 VGPRs)
      int tt = tt0;
      asm volatile("" : "+v"(tt));
      // z_k = X_k^T y_k and X_k into registers from team F's sX (untouched until tile k+1 is
      // handed over below)
      if (tt < kTile) L.sz[tt] = sxDyn[k * kTile + tt];
      bsyncL();
      panelRhsVector(L.sX, L.sz, L.sz + kTile, L.sB[1], tt, bsyncL);  // (scratch: sB[0] may hold A staged)
      loadXFrag(L.sX, xf, tt);
      PCLK(3, 256)
      int held[2] = {-1, -1};  // block row i of the L_ik in sB[0] / sB[1]
      const bool crit = k + 1 < k1 && nz[(k + 1) * T + k] != 0;
      if (crit) {
        // the critical path: panel (k+1, k), then its update of tile (k+1, k+1) into team F's sA
        pipePanel(cur.at(k + 1, k, k), W + (int64_t)(k + 1) * kTile * ld + k * kTile, ld, sxDyn + (k + 1) * kTile,
                  L.sB[0], xf, L.sz + kTile, tt, bsyncL, nullptr, staged == k);
        held[0] = k + 1;
        dbl4 c[3], acc[3];  // (a diagonal tile: its lower block triangle, chol_tiles.hpp)
        loadCDiag(cur.at(k + 1, k + 1, k), ld, c, tt);
        mfmaDiagNT(L.sB[0], acc, tt);
        diagSubToLds(L.sA, c, acc, tt);
        bsyncL();
      }
      if (tt == 0) {
        L.pipe[2] = crit ? 1 : 0;
        ldsRelease(&L.pipe[1], k + 1);
      }
      PCLK(4, 256)
      // the step's other panels (the last ones stay in LDS for the updates)
      int hb = crit ? 1 : 0;
      // (without the critical pair this includes row k+1: at the end of a part of a split window,
      // where tile k+1 is the separator's)
      for (int i = crit ? k + 2 : k + 1; i < T; ++i) {
        if (!nz[i * T + k]) continue;
        pipePanel(cur.at(i, k, k), W + (int64_t)i * kTile * ld + k * kTile, ld, sxDyn + i * kTile, L.sB[hb], xf,
                  L.sz + kTile, tt, bsyncL, i >= jEnd ? deferAt(i, k) : nullptr);
        held[hb] = i;
        if (!crit) hb ^= 1;
      }
      bsync();  // the L tiles in W for reloads by other wavefronts of the team
      PCLK(5, 256)
      // band updates A_ij -= L_ik L_jk^T of step k but (k+1, k+1), bottom-up
      for (int i = T - 1; i > k; --i) {
        if (!nz[i * T + k]) continue;
        for (int j = k + 1; j <= i; ++j) {
          // (row k+1: only (k+1, k+1), done above when critical; the right part of a split
          // window leaves the separator's tiles to launch B)
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
      }
      bsync();  // the updated tiles in W for the next step's panels
      // the next step's critical A_(k+2)(k+1) has all its updates now: into sB[0] while team F
      // factors tile k+1 (one global round trip off the next step's critical path; the panel's
      // first team barrier orders these LDS writes before its reads)
      if (k + 2 < k1 && nz[(k + 2) * T + k + 1]) {
        loadTile(cur.at(k + 2, k + 1, k + 1), ld, 0, 0, L.sB[0], tt);
        staged = k + 1;
      }
      PCLK(7, 256)
    }
  }
  __syncthreads();
  if (L.pipe[3]) {
    if (t == 0) P.st[w].gn_failed = 1;
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
