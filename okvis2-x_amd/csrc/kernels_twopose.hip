// kernels_twopose.hip — TwoPoseStandardGraphError::compute (okvis_ceres/src/TwoPoseGraphError.cpp:
// 162-397) for a batch of pose-graph edges: one wavefront per edge.
//
// The landmarks of the edge are dealt to the 64 lanes (lane L takes landmarks L, L+64, ...). A lane
// linearises every observation of its landmark in S0 coordinates (the reference keyframe is the
// origin, the other keyframe sits at T_S0S1), drops |r| > 3 outliers, applies the Cauchy corrector,
// forms the landmark's 6x6 / 6x3 / 3x3 blocks in registers and marginalises the landmark with the
// pseudo-inverse of its 3x3 block (3x3 Jacobi eigen-solve; PseudoInverse::symmSqrt,
// PseudoInverse.hpp:101-129, tolerance 1e-7), skipping it when rank < 3 and its S0 depth < 2.99.
// The 54 accumulated values (H00 21 packed, b0 6, W V^+ W^T 21, W V^+ b1 6) are summed over the
// lanes by a fixed xor tree (deterministic), and lane 0 decomposes the 6x6 relative system into
// J_ = D^(1/2) E^T and DeltaX_ = -H^+ b0 (6x6 Jacobi eigen-solve, tolerance 1e-8 * 6 * max).
//
// This runs when keyframes are marginalised into pose-graph edges (ViGraphEstimator.cpp:425-575),
// not inside the trust-region loop; it is latency-bound and sized for batches of edges.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "device_problem.hpp"
#include "launch.hpp"
#include "okvisgpu_math.hpp"

namespace okg {

namespace {

OKG_HD int sym6i(int a, int b) {  // packed upper 6x6 index
  if (a > b) { const int t = a; a = b; b = t; }
  return a * 6 - a * (a - 1) / 2 + (b - a);
}

}  // namespace

__global__ __launch_bounds__(64) void k_twopose_compute(TwoPoseDev T) {
  const int e = blockIdx.x;
  if (e >= T.n_edges) return;
  const int lane = threadIdx.x;
  const double* P0 = T.ref_pose + 7 * (size_t)e;
  const double* P1 = T.other_pose + 7 * (size_t)e;
  const Q q0 = qnormalize(Q{P0[3], P0[4], P0[5], P0[6]}), q1 = qnormalize(Q{P1[3], P1[4], P1[5], P1[6]});
  double C0[9];
  qrot(q0, C0);  // C_WS0 (C_S0W = C0^T)
  const double d01[3] = {P1[0] - P0[0], P1[1] - P0[1], P1[2] - P0[2]};
  double rel[7];  // T_S0S1 = T_WS0^-1 T_WS1
  mtv3(C0, d01, rel);
  const Q qr = qnormalize(qmul(qinv(q0), q1));
  rel[3] = qr.x; rel[4] = qr.y; rel[5] = qr.z; rel[6] = qr.w;
  const double ident[7] = {0, 0, 0, 0, 0, 0, 1};

  double acc[54];
#pragma unroll
  for (int i = 0; i < 54; ++i) acc[i] = 0.0;
  bool sawOther = false;
  const int lb = T.lm_begin[e], le = T.lm_begin[e + 1];
  for (int l = lb + lane; l < le; l += 64) {
    const double* hw = T.lm + 4 * (size_t)l;
    const double dw[3] = {hw[0] - P0[0] * hw[3], hw[1] - P0[1] * hw[3], hw[2] - P0[2] * hw[3]};
    double hp[4];
    mtv3(C0, dw, hp);  // hp_S0 = T_S0W hp_W
    hp[3] = hw[3];
    const double minDist = hp[2] / hp[3];
    double H00[21], b0[6], H01[18], H11[6], b1[3];
#pragma unroll
    for (int i = 0; i < 21; ++i) H00[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 18; ++i) H01[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) { b0[i] = 0.0; H11[i] = 0.0; }
    b1[0] = b1[1] = b1[2] = 0.0;
    for (int o = T.obs_begin[l]; o < T.obs_begin[l + 1]; ++o) {
      const bool other = T.obs_other[o] != 0;
      sawOther = sawOther || other;
      const int ci = T.obs_cam[o];
      const Cam cam = loadCam(T.cam + kCamDoubles * ci);
      double r[2], A[6], p[3];
      reprojectA(cam, other ? rel : ident, hp, T.extr + 7 * ci, T.obs_L + 4 * (size_t)o, T.obs_kp + 2 * (size_t)o, r,
                 A, p);
      if (sqrt(r[0] * r[0] + r[1] * r[1]) > 3.0) continue;  // obvious outliers (:285-288)
      if (T.obs_cauchy[o]) {  // Corrector, CauchyLoss (rho'' < 0): scale by sqrt(rho')
        const double s = sqrt(fmax(DBL_MIN, 1.0 / (1.0 + r[0] * r[0] + r[1] * r[1])));
        r[0] *= s; r[1] *= s;
#pragma unroll
        for (int i = 0; i < 6; ++i) A[i] *= s;
      }
      // J1 = -A (2x3); J0 = [w A, -A [p]x] (2x6)
      double J0[12];
      for (int rr = 0; rr < 2; ++rr) {
        const double a0 = A[rr * 3], a1 = A[rr * 3 + 1], a2 = A[rr * 3 + 2];
        J0[rr * 6 + 0] = hp[3] * a0;
        J0[rr * 6 + 1] = hp[3] * a1;
        J0[rr * 6 + 2] = hp[3] * a2;
        J0[rr * 6 + 3] = -(a1 * p[2] - a2 * p[1]);
        J0[rr * 6 + 4] = -(a2 * p[0] - a0 * p[2]);
        J0[rr * 6 + 5] = -(a0 * p[1] - a1 * p[0]);
      }
      if (other) {
        for (int a = 0; a < 6; ++a) {
          for (int b = a; b < 6; ++b) H00[sym6i(a, b)] += J0[a] * J0[b] + J0[6 + a] * J0[6 + b];
          b0[a] -= J0[a] * r[0] + J0[6 + a] * r[1];
          for (int b = 0; b < 3; ++b) H01[a * 3 + b] -= J0[a] * A[b] + J0[6 + a] * A[3 + b];
        }
      }
      int k = 0;
      for (int a = 0; a < 3; ++a) {
        for (int b = a; b < 3; ++b) H11[k++] += A[a] * A[b] + A[3 + a] * A[3 + b];
        b1[a] += A[a] * r[0] + A[3 + a] * r[1];  // -J1^T r
      }
    }
    // V^+ with the symmSqrt clamp: eigenvalues <= tol map to 1/tol
    double V[9] = {H11[0], H11[1], H11[2], H11[1], H11[3], H11[4], H11[2], H11[4], H11[5]};
    double lam[3], Ev[9];
    jacobiEigenSym<3>(V, lam, Ev);
    const double tol = fmax(1.0e-7, 1.0e-7 * 3.0 * lam[2]);
    const int rank = (lam[0] > tol) + (lam[1] > tol) + (lam[2] > tol);
    if (rank < 3 && minDist < 2.99) continue;
    double f[3];
    for (int i = 0; i < 3; ++i) {
      const double s = sqrt(lam[i] > tol ? 1.0 / lam[i] : 1.0 / tol);
      f[i] = s * s;
    }
    double Vp[9];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b)
        Vp[a * 3 + b] = Ev[a * 3 + 0] * f[0] * Ev[b * 3 + 0] + Ev[a * 3 + 1] * f[1] * Ev[b * 3 + 1] +
                        Ev[a * 3 + 2] * f[2] * Ev[b * 3 + 2];
    double WV[18];
    for (int a = 0; a < 6; ++a)
      for (int b = 0; b < 3; ++b)
        WV[a * 3 + b] = H01[a * 3 + 0] * Vp[0 * 3 + b] + H01[a * 3 + 1] * Vp[1 * 3 + b] + H01[a * 3 + 2] * Vp[2 * 3 + b];
#pragma unroll
    for (int i = 0; i < 21; ++i) acc[i] += H00[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) acc[21 + i] += b0[i];
    for (int a = 0; a < 6; ++a) {
      for (int b = a; b < 6; ++b)
        acc[27 + sym6i(a, b)] += WV[a * 3] * H01[b * 3] + WV[a * 3 + 1] * H01[b * 3 + 1] + WV[a * 3 + 2] * H01[b * 3 + 2];
      acc[48 + a] += WV[a * 3] * b1[0] + WV[a * 3 + 1] * b1[1] + WV[a * 3 + 2] * b1[2];
    }
  }
#pragma unroll
  for (int i = 0; i < 54; ++i)
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) acc[i] += __shfl_xor(acc[i], sh, 64);
  const bool relPoseSet = __ballot(sawOther) != 0;
  if (lane != 0) return;
  double H[36], bb[6];
  for (int a = 0; a < 6; ++a) {
    for (int b = 0; b < 6; ++b) H[a * 6 + b] = acc[sym6i(a, b)] - acc[27 + sym6i(a, b)];
    bb[a] = acc[21 + a] - acc[48 + a];
  }
  double* out = T.out + (size_t)kTwoPoseOut * e;
  for (int i = 0; i < 36; ++i) out[49 + i] = H[i];
  for (int i = 0; i < 6; ++i) out[85 + i] = bb[i];
  double lam[6], Ev[36];
  jacobiEigenSym<6>(H, lam, Ev);
  const double tol = 1.0e-8 * 6.0 * lam[5];
  double Etb[6];
  for (int i = 0; i < 6; ++i) {
    const bool keep = lam[i] > tol;
    const double ds = keep ? sqrt(lam[i]) : 0.0;
    double s = 0.0;
    for (int k = 0; k < 6; ++k) {
      out[6 + i * 6 + k] = ds * Ev[k * 6 + i];  // J_ row i = sqrt(lambda_i) e_i^T
      s += Ev[k * 6 + i] * bb[k];
    }
    Etb[i] = keep ? s / lam[i] : 0.0;
  }
  for (int k = 0; k < 6; ++k) {
    double s = 0.0;
    for (int i = 0; i < 6; ++i) s += Ev[k * 6 + i] * Etb[i];
    out[k] = -s;  // DeltaX_ = -H^+ b0_
  }
  for (int i = 0; i < 7; ++i) out[42 + i] = relPoseSet ? rel[i] : ident[i];
}

void launch_twopose_compute(const TwoPoseDev& T, hipStream_t s) {
  if (T.n_edges > 0) hipLaunchKernelGGL(k_twopose_compute, dim3(T.n_edges), dim3(64), 0, s, T);
}

}  // namespace okg
