// kernels_chol.hip — dense LLT of the reduced camera matrix S (Eigen::LLT semantics: fail at the
// first non-positive pivot) and the two triangular solves. Two schedules of the same tile
// routines: one persistent workgroup per window (large batches: fills the chip with whole
// windows) or per-step launches over all windows' panel / band-update tiles (few windows:
// spreads each window over many CUs); launch_cholesky picks the host-resolved one.
//
// k_cholesky: right-looking blocked Cholesky over 64x64 FP64 tiles, only structurally non-zero
// tiles (the host's tile-level symbolic factorisation, DevProblem::tile_nz: the reduced camera
// matrix of a sliding window is block-banded and LLT creates no fill outside its envelope, so
// skipping zero tiles is exact). Per step k, inside one workgroup:
//   diagonal  L_kk and X = L_kk^-1 (8-column sub-panels on one wavefront with a look-ahead, MFMA
//             trailing updates and X by 16-row block rows on the other three; potrfTile), fused
//             forward substitution y_k = X rhs_k
//   panel     L_ik = A_ik X^T for every non-zero tile below (64x64x64 on the FP64 matrix cores)
//             and rhs_i -= L_ik y_k
//   update    A_ij -= L_ik L_jk^T for the non-zero tiles of the trailing band (matrix cores;
//             operands staged in LDS, freshly written tiles come back from L2)
// then the backward substitution x = L^-T y with the stored diagonal inverses.
// (the tile routines: chol_tiles.hpp; the pipelined two-team persistent schedule:
// kernels_chol_pipe.hip)
#include "chol_tiles.hpp"
#include "launch.hpp"

namespace okg {

#ifndef OKG_CHOL_OCC
#define OKG_CHOL_OCC 2
#endif
// Persistent schedule, one workgroup per window (MODE 0), or split over a nested-dissection
// window's two independent parts (win_bsplit; schedule 3, runtime.cpp setOptions):
//   MODE 1 (launch A, workgroups 2w and 2w+1): part 0 runs the left part's steps [0, tL) with all
//          their updates; part 1 the right part's steps [tL, tS) with the updates of targets left
//          of the separator, and for the separator's tiles it stores only L (the panels) and each
//          panel's rhs contribution (chol_defer); both write their y / rhs rows to fwdF.
//   MODE 2 (launch B, one workgroup per window): the right steps' updates of the separator's
//          tiles and their rhs contributions, step by step, then the separator's steps [tS, T)
//          and the backward substitution.
// Every tile receives its updates in step order in all modes (the left part's steps precede the
// right part's), each with the same operations, so the split gives the bits of MODE 0 on the same
// order. A window without a split runs MODE 0 in part 0 of launch A (MODE 2 skips it).

template <int MODE>
__global__ __launch_bounds__(256, OKG_CHOL_OCC) void k_cholesky(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = MODE == 1 ? (int)(blockIdx.x >> 1) : (int)blockIdx.x, part = MODE == 1 ? (int)(blockIdx.x & 1) : 0;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  const int T = (int)(ld / kTile);
  const int tL = MODE == 0 ? 0 : P.win_bsplit[2 * w], tS = MODE == 0 ? 0 : P.win_bsplit[2 * w + 1];
  const bool split = MODE != 0 && tS > 0;
  if ((MODE == 1 && part == 1 && !split) || (MODE == 2 && !split)) return;
  // this workgroup's steps [k0, k1), targets (i, j) with j < jEnd, and whether it ends the window
  const int k0 = !split ? 0 : (MODE == 2 ? tS : (part == 0 ? 0 : tL));
  const int k1 = !split ? T : (MODE == 2 ? T : (part == 0 ? tL : tS));
  const int jEnd = split && MODE == 1 && part == 1 ? tS : T;
  const bool finish = !split || MODE == 2;
  const TileSrc cur = tileSrc(P, w, ld);
  double* W = P.W + P.win_soff[w];
  double* Linv = P.Linv + P.win_linvoff[w];
  const uint8_t* nz = P.tile_nz + P.win_tnzoff[w];
  double* work = P.fwdF + P.win_fwdoff[w];
  double* defer = split ? P.chol_defer + P.win_defoff[w] : nullptr;
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sy[2 * kTile];  // y_k | panel column scratch
  __shared__ double sRl[kTile];
  __shared__ int sFl[4];
  const int t = threadIdx.x;
  const int fdim = P.win_fdim[w];
  CLK_INIT
  // rhs / y of the whole window in LDS (sxDyn, ld doubles) for the forward substitution, the
  // panels' rhs updates and the backward substitution (no global round trip per step)
  extern __shared__ double sxDyn[];
  if (MODE == 2) {
    for (int e = t; e < ld; e += 256) sxDyn[e] = work[e];
  } else {
    for (int e = t; e < ld; e += 256) sxDyn[e] = (e < fdim) ? P.rhsF[(size_t)P.win_foff[w] + e] : 0.0;
  }
  __syncthreads();
  // ---- trailing band update of step k: A_ij -= L_ik L_jk^T, k < j <= i, jLo <= j < jEnd, both
  // tiles non-zero. The A_ij read of the read-modify-write is issued before the MFMAs, so its
  // latency overlaps them. Block rows from the bottom: the L_jk staged in sX for a lower row is
  // reused as the row operand when its own row comes (one staging per L tile on a 2-tile band
  // instead of 3), and the last update, S_(k+1)(k+1), goes to sA for the next factor instead of
  // through global memory (toLds). Independent tiles, the same operations: the same bits in any
  // order. Returns whether S_(k+1)(k+1) was left in sA.
  // the thread index, opaque per step (set in the step loop): the step's LDS / global addresses
  // are formed in the step instead of being hoisted out of the loop and spilled
  int tStep = t;
  auto bandUpdate = [&](int k, int jLo, bool toLds) {
    const int t = tStep;
    int xHeld = -1;  // block row of the L tile in sX
    bool inLds = false;
    for (int i = T - 1; i > k && i >= jLo; --i) {
      if (!nz[i * T + k]) continue;
      const bool aInX = xHeld == i;
      const double* aBuf = aInX ? sX : sA;
      bool aLoaded = aInX;
      for (int j = max(k + 1, jLo); j <= i && j < jEnd; ++j) {
        if (!nz[j * T + k]) continue;
        if (!aLoaded) {
          loadTile(W + i * kTile * ld + k * kTile, ld, 0, 0, sA, t);
          aLoaded = true;
        }
        const double* bBuf = aBuf;
        if (j != i) {
          if (aInX) {
            loadTile(W + j * kTile * ld + k * kTile, ld, 0, 0, sA, t);
            bBuf = sA;
          } else {
            if (xHeld != j) loadTile(W + j * kTile * ld + k * kTile, ld, 0, 0, sX, t);
            xHeld = j;
            bBuf = sX;
          }
        }
        ldsBarrier();
        double* Cij = W + i * kTile * ld + j * kTile;
        if (j == i) {  // diagonal tile: its lower block triangle only (chol_tiles.hpp)
          dbl4 c[3], acc[3];
          loadCDiag(cur.at(i, j, k), ld, c, t);
          mfmaDiagNT(aBuf, acc, t);
          if (toLds && i == k + 1) {  // the next diagonal tile: c - acc straight into sA
            ldsBarrier();             // every wavefront has read its operands
            diagSubToLds(sA, c, acc, t);
            inLds = true;  // its global copy is stale from here on and never read
          } else {
            storeDiagSub(Cij, ld, c, acc, t);
          }
        } else {
          dbl4 c[2][2], acc[2][2];
          loadC(cur.at(i, j, k), ld, c, t);
          mfmaTileNT(aBuf, bBuf, acc, t);
          storeTileSub(Cij, ld, c, acc, t);
        }
        ldsBarrier();  // LDS-only: the updated tiles are read from the next step on, after full barriers
      }
    }
    return inLds;
  };
  if (MODE == 2) {
    // the right part's contributions to the separator, in step order: each step's panel rhs terms,
    // then its updates of the separator's tiles (L from W, written by launch A)
    for (int k = tL; k < tS; ++k) {
      for (int i = tS; i < T; ++i)
        if (nz[i * T + k] && t < kTile)
          sxDyn[i * kTile + t] -= defer[((size_t)(i - tS) * (tS - tL) + (k - tL)) * kTile + t];
      __syncthreads();
      bandUpdate(k, tS, false);
      __syncthreads();
    }
  }
  bool haveDiag = false;  // S_kk (updated by the previous step) already in sA
  for (int k = k0; k < k1; ++k) {
    CLK(11)
    if (t < kTile) sy[t] = sxDyn[k * kTile + t];
    __syncthreads();  // full: the factor and the panels read the tiles the last band update stored
    if (!potrfTile<10 + MODE>(cur.at(k, k, k), ld, Linv + (int64_t)k * kTile * kTile, nullptr, sA, sX,
                   sy, sRl, sFl, t, haveDiag, 0, tileBlocks(P, w, k))) {
      if (t == 0) P.st[w].gn_failed = 1;
      return;
    }
    if (t < kTile) sxDyn[k * kTile + t] = sy[t];  // y_k (ordered before its readers by the barriers below)
    CLK(0)
    tStep = t;
    asm volatile("" : "+v"(tStep));
    // ---- panel: L_ik = A_ik X^T, rhs_i -= L_ik y_k = A_ik X^T y_k (the separator's rows deferred
    // by part 1 of the split)
    panelRhsVector(sX, sy, sy + kTile, sA, t);
    for (int i = k + 1; i < T; ++i)
      if (nz[i * T + k])
        panelTile(cur.at(i, k, k), W + i * kTile * ld + k * kTile, ld, sxDyn + i * kTile, sA, sX, sy + kTile, tStep,
                  i >= jEnd ? defer + ((size_t)(i - tS) * (tS - tL) + (k - tL)) * kTile : nullptr);
    __syncthreads();  // full barrier: the band update reads the L_ik just stored
    CLK(1)
    haveDiag = bandUpdate(k, 0, true);
  }
  CLK(2)
  if (!finish) {  // launch A: this part's rows of y (part 0 also the separator's rhs) for launch B
    const int e0 = part == 0 ? 0 : tL * kTile, e1 = part == 0 ? tL * kTile : tS * kTile;
    for (int e = t; e < ld; e += 256)
      if ((e >= e0 && e < e1) || (part == 0 && e >= tS * kTile)) work[e] = sxDyn[e];
    return;
  }
  backSubstitute(P, w, W, ld, T, Linv, nz, sxDyn, sA, sy, t);
  CLK(3)
  CHOL_CLK_REPORT(T)
}

// ---- tile-parallel schedule (few windows: spreads each window over many CUs; runtime.cpp
// cholSchedule). Launch 0 factors the root tiles (no band update writes them: the first tile of
// each independent part of a nested-dissection order); launch l >= 1 runs the band updates of the
// steps scheduled there over all windows. Every workgroup forms the panels it needs itself
// (L_ik = A_ik X_k^T from the final A_ik and the stored X_k), so no launch sits between a diagonal
// factor and its updates. A_ik stays in place during the step (other workgroups of the same launch
// still read it): the workgroup of the diagonal update (i,i) writes L_ik to the unused upper slot
// (k,i) of W and applies rhs_i -= L_ik y_k; the backward substitution of this schedule reads L
// there. The workgroup of a diagonal tile's last update factors it right after.
// (launch bounds of two workgroups per CU: without them the compiler gives potrfTile<1> the
// one-wave-per-SIMD register budget and emits a longer chain, 22.3 against 16.3 us per tile in
// scripts/ubench_ptile.hip)
__global__ __launch_bounds__(256, 2) void k_chol_roots(const DevProblem* __restrict__ Pp) {
  const DevProblem& P = *Pp;
  const int w = P.chol_root_items[3 * blockIdx.x], d = P.chol_root_items[3 * blockIdx.x + 1];
  const bool first = P.chol_root_items[3 * blockIdx.x + 2] != 0;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  const int T = (int)(ld / kTile);
  const TileSrc cur = tileSrc(P, w, ld);
  double* work = P.fwdF + P.win_fwdoff[w];
  const uint8_t* nz = P.tile_nz + P.win_tnzoff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sy[2 * kTile];
  __shared__ double sRl[kTile];
  __shared__ int sFl[4];
  const int t = threadIdx.x;
  // the window's rhs into its work vector: each root item its own block row, the first one also
  // every block row that is not a root (read from launch 1 on)
  const int fdim = P.win_fdim[w];
  const double* rhs = P.rhsF + P.win_foff[w];
  for (int e = t; e < ld; e += 256) {
    const int b = e / kTile;
    bool mine = b == d;
    if (first && b != d) {
      bool root = true;  // (a root is a diagonal tile with no non-zero tile left of it)
      for (int q = 0; q < b && root; ++q) root = !nz[b * T + q];
      mine = !root;
    }
    if (mine) work[e] = e < fdim ? rhs[e] : 0.0;
  }
  __syncthreads();
  if (t < kTile) sy[t] = work[d * kTile + t];
  __syncthreads();
  if (!potrfTile<1>(cur.at(d, d, d), ld, P.Linv + P.win_linvoff[w] + (int64_t)d * kTile * kTile,
                    work + d * kTile, sA, sX, sy, sRl, sFl, t, false, 0, tileBlocks(P, w, d)))
    if (t == 0) P.st[w].gn_failed = 1;
}


__global__ __launch_bounds__(256, 2) void k_chol_update(const DevProblem* __restrict__ Pp, int launch) {
  const DevProblem& P = *Pp;
  const int item = P.chol_upd_begin[launch] + blockIdx.x;
  const int4 it = reinterpret_cast<const int4*>(P.chol_upd_items)[item];
  const int w = it.x, i = it.y, j = it.z, mode = it.w & 0xff, k = it.w >> 8;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  const TileSrc cur = tileSrc(P, w, ld);
  double* W = P.W + P.win_soff[w];
  double* work = P.fwdF + P.win_fwdoff[w];
  __shared__ double sA[kTile * kLd];
  __shared__ double sX[kTile * kLd];
  __shared__ double sB[kTile * kLd];
  __shared__ double sy[2 * kTile];
  __shared__ double sRl[kTile];
  __shared__ int sFl[4];
  const int t = threadIdx.x;
  // (every item updates; bit 1: tile (i,i)'s last update, which factors it afterwards)
  {
    // panels of step k: L_ik (and L_jk) = A (X_k)^T, operands staged in LDS
    loadTile(P.Linv + P.win_linvoff[w] + (int64_t)k * kTile * kTile, kTile, 0, 0, sX, t);
    loadTile(cur.at(i, k, k), ld, 0, 0, sA, t);
    if (j != i) loadTile(cur.at(j, k, k), ld, 0, 0, sB, t);
    if (i == j && t < kTile) sy[t] = work[k * kTile + t];
    const int row = t >> 2, q = t & 3;
    const double rhsOld = (i == j && q == 0) ? work[i * kTile + row] : 0.0;
    __syncthreads();
    // rhs_i -= L_ik y_k, formed as A_ik z with z = X_k^T y_k from the A_ik tile in LDS (the same
    // operations as panelTile, so all schedules give the same bits)
    if (i == j) panelRhsVector(sX, sy, sy + kTile, sB, t);
    dbl4 li[4], lj[4];
    mfmaPanelRows(sA, sX, li, t);
    if (j != i) mfmaPanelRows(sB, sX, lj, t);
    if (i == j) {
      const double a = panelRhsRow(sA, sy + kTile, t);
      if (q == 0) {
        const double nr = rhsOld - a;
        gmemw(work)[i * kTile + row] = nr;
        if (mode & 2) sRl[row] = nr;  // rhs_{k+1} for the factor below (sRl is free until then)
      }
    }
    ldsBarrier();  // every wavefront has read A_ik / A_jk (LDS-only: the rhs store stays in flight)
    panelRowsToLds(sA, li, t);
    if (j != i) panelRowsToLds(sB, lj, t);
    double* Cij = W + i * kTile * ld + j * kTile;
    if (i == j) {  // diagonal tile: its lower block triangle only (chol_tiles.hpp)
      dbl4 c[3];
      loadCDiag(cur.at(i, j, k), ld, c, t);  // read of the read-modify-write overlaps the barrier and the MFMAs
      storePanelRows(W + k * kTile * ld + i * kTile, ld, li, t);  // L_ik -> upper slot (k,i)
      ldsBarrier();  // no reader of the upper slot in this launch
      dbl4 acc[3];
      mfmaDiagNT(sA, acc, t);
      if (mode & 2) {
        // tile (i,i) after its last update: straight to LDS for the factor (its global copy is stale
        // from here on and never read), and so is rhs_i
        ldsBarrier();  // every wavefront has read L_ik from sA
        diagSubToLds(sA, c, acc, t);
        __syncthreads();
        if (t < kTile) sy[t] = sRl[t];
      } else {
        storeDiagSub(Cij, ld, c, acc, t);
      }
    } else {
      dbl4 c[2][2];
      loadC(cur.at(i, j, k), ld, c, t);
      ldsBarrier();
      dbl4 acc[2][2];
      mfmaTileNT(sA, sB, acc, t);
      storeTileSub(Cij, ld, c, acc, t);
    }
  }
  if (!(mode & 2)) return;
  const int d = i;
  __syncthreads();
  if (!potrfTile<2>(cur.at(d, d, d), ld, P.Linv + P.win_linvoff[w] + (int64_t)d * kTile * kTile,
                    work + d * kTile, sA, sX, sy, sRl, sFl, t, true, 0, tileBlocks(P, w, d)))
    if (t == 0) P.st[w].gn_failed = 1;
}

// Tile-parallel schedule's backward substitution: 512 threads (2 virtual threads each), software
// pipelined. Step I-1's operands do not depend on x, so their loads are issued before step I's
// reductions (a single window is a chain of T steps that would otherwise each wait a full memory
// latency); two register sets, no copies; barriers order LDS only, so the loads stay in flight
// across them. Same operations in the same order as backSubstitute. A nested-dissection window
// (win_bsplit) is solved by two workgroups: both solve the separator's block rows, then workgroup
// 0 the left part and workgroup 1 the right part (independent: no non-zero tile between them);
// each step's operations are those of the one-workgroup order, so the bits are the same.
constexpr int kBsReal = 512;
__global__ __launch_bounds__(kBsReal) void k_chol_bsub(const DevProblem* __restrict__ Pp) {
  constexpr int kV = kBsThreads / kBsReal;
  const DevProblem& P = *Pp;
  const int w = blockIdx.x, h = blockIdx.y;
  if (!cholSelect(P, w)) return;
  const int64_t ld = P.win_fpad[w];
  const int T = (int)(ld / kTile);
  const int tL = P.win_bsplit[2 * w], tS = P.win_bsplit[2 * w + 1];
  const bool split = tS > 0;
  if (h == 1 && !split) return;
  // step n -> block row: the separator [tS, T) (whole window without a split), then this
  // workgroup's part, descending
  const int nSep = split ? T - tS : T;
  const int nSteps = nSep + (split ? (h == 0 ? tL : tS - tL) : 0);
  const int partTop = h == 0 ? tL - 1 : tS - 1;
  auto rowAt = [&](int n) { return n < nSep ? T - 1 - n : partTop - (n - nSep); };
  const double* S = P.W + P.win_soff[w];  // L in the upper slots of the working copy
  const double* work = P.fwdF + P.win_fwdoff[w];
  const double* Linv = P.Linv + P.win_linvoff[w];
  __shared__ double sA[32 * kTile];
  __shared__ double sy[kTile];
  // x (ld doubles), then per block row its tile list ((1 + kBsPre) ints), then the bitmap (T * T bytes)
  extern __shared__ double sx[];
  int* lists = reinterpret_cast<int*>(sx + ld);
  uint8_t* nz = reinterpret_cast<uint8_t*>(lists + (1 + kBsPre) * T);
  const int t = threadIdx.x;
  CLK_INIT
  for (int e = t; e < T * T; e += kBsReal) nz[e] = P.tile_nz[P.win_tnzoff[w] + e];
  for (int e = t; e < ld; e += kBsReal) sx[e] = work[e];
  if (t < T) bsList(P.tile_nz + P.win_tnzoff[w], T, t, lists + (1 + kBsPre) * t);
  __syncthreads();
  BsOps ping[kV], pong[kV];
  auto load = [&](int I, BsOps* o) {
#pragma unroll
    for (int k = 0; k < kV; ++k) bsLoad<true>(S, ld, Linv, lists + (1 + kBsPre) * I, I, t + kBsReal * k, o[k]);
  };
  auto step = [&](int I, const BsOps* c) {
    const int* lst = lists + (1 + kBsPre) * I;
#pragma unroll
    for (int k = 0; k < kV; ++k) bsPartial<true>(S, ld, T, nz, lst, I, c[k], sx, sA, t + kBsReal * k);
    ldsBarrier();
    if (t < kTile) sy[t] = sx[I * kTile + t] - sum32(sA + t);
    ldsBarrier();
#pragma unroll
    for (int k = 0; k < kV; ++k) bsDiag(c[k], sy, sA, t + kBsReal * k);
    ldsBarrier();
    if (t < kTile) sx[I * kTile + t] = sum32(sA + t);
    ldsBarrier();
  };
  load(rowAt(0), ping);
  CLK(12)
  for (int n = 0; n < nSteps; n += 2) {  // (loads clamped, not skipped: no loads under a branch)
    load(rowAt(min(n + 1, nSteps - 1)), pong);
    step(rowAt(n), ping);
    if (n + 1 == nSteps) break;
    load(rowAt(min(n + 2, nSteps - 1)), ping);
    step(rowAt(n + 1), pong);
  }
  CLK(13)
  // x of the rows this workgroup owns (the separator's by workgroup 0)
  const int fdim = P.win_fdim[w];
  const int e0 = !split ? 0 : (h == 0 ? 0 : tL * kTile), e1 = !split ? fdim : (h == 0 ? fdim : tS * kTile);
  for (int e = e0 + t; e < e1; e += kBsReal)
    if ((!split || h == 1 || e < tL * kTile || e >= tS * kTile) && !gapRow(P, w, e))
      gnFinalizeRow(P, (size_t)P.win_foff[w] + e, sx[e]);
  BSUB_CLK_REPORT(T)
}

void launch_cholesky_split_b(const DevProblem& P, hipStream_t s) {
  hipLaunchKernelGGL(k_cholesky<2>, dim3(P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P.self);
}

bool cholesky_persistent_fits(int max_fpad, size_t lds_per_block) {
  hipFuncAttributes attr;
  if (hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(k_cholesky<0>)) != hipSuccess) return false;
  return attr.sharedSizeBytes + sizeof(double) * (size_t)max_fpad <= lds_per_block;
}

void launch_cholesky(const DevProblem& P, hipStream_t s) {
  if (P.n_win == 0) return;
  if (P.chol_schedule == 4 || P.chol_schedule == 5) {
    launch_cholesky_pipe(P, s, P.chol_schedule == 5);
    return;
  }
  if (P.chol_schedule == 1) {
    hipLaunchKernelGGL(k_cholesky<0>, dim3(P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P.self);
    return;
  }
  if (P.chol_schedule == 3) {
    hipLaunchKernelGGL(k_cholesky<1>, dim3(2 * P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P.self);
    hipLaunchKernelGGL(k_cholesky<2>, dim3(P.n_win), dim3(256), sizeof(double) * P.max_fpad, s, P.self);
    return;
  }
  hipLaunchKernelGGL(k_chol_roots, dim3(P.n_chol_roots), dim3(256), 0, s, P.self);
  for (int l = 1; l < P.n_chol_launches; ++l) {
    const int nu = P.h_upd_begin[l + 1] - P.h_upd_begin[l];
    if (nu > 0) hipLaunchKernelGGL(k_chol_update, dim3(nu), dim3(256), 0, s, P.self, l);
  }
  hipLaunchKernelGGL(k_chol_bsub, dim3(P.n_win, 2), dim3(kBsReal),
                     sizeof(double) * P.max_fpad + sizeof(int) * (1 + kBsPre) * P.max_tiles + P.max_tiles * P.max_tiles, s,
                     P.self);
}

}  // namespace okg
