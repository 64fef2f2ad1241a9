// gradnorm.hpp — the gradient tolerance test of one window (TrustRegionMinimizer: |x - Plus(x, -g)|
// max and 2-norms and |x| after every accepted step, termination by gradient tolerance), one
// RB-thread workgroup per window: k_gradnorm (kernels_control.hip) and the gradient-norm blocks
// of the few-window assembly launch (kernels_schur.hip k_assemble_few).
#pragma once
#include "block_reduce.hpp"
#include "device_problem.hpp"
#include "okvisgpu_math.hpp"

namespace okg {

template <int RB>
__device__ __forceinline__ void gradnormWindow(const DevProblem& P, const int w, int lin_mode) {
  WinState& s = P.st[w];
  if (s.done) return;
  if (lin_mode == 1 && !s.accepted) return;
  __shared__ double sh[3 * RB];
  const int t = threadIdx.x;
  const int xs = s.xcur;
  const int foff = P.win_foff[w];
  double mx = 0.0, g2 = 0.0, x2 = 0.0;
  const int p0 = P.win_pose_range[2 * w], p1 = P.win_pose_range[2 * w + 1];
  for (int p = p0 + t; p < p1; p += RB) {
    if (!gmem(P.pose_active)[p]) continue;
    const auto x = gmem(P.pose[xs] + 7 * (size_t)p);
    for (int k = 0; k < 7; ++k) x2 += x[k] * x[k];
    const int pf = gmem(P.pose_f)[p];
    const auto g = gmem(P.gF + foff + pf);
    double xp[7];
    for (int k = 0; k < 3; ++k) xp[k] = x[k] + (-g[k]);
    const Q dq = deltaQ(-g[3], -g[4], -g[5]);
    const Q q = qnormalize(qmul(dq, qnormalize(Q{x[3], x[4], x[5], x[6]})));
    xp[3] = q.x; xp[4] = q.y; xp[5] = q.z; xp[6] = q.w;
    for (int k = 0; k < 7; ++k) {
      const double d = x[k] - xp[k];
      mx = fmax(mx, fabs(d));
      g2 += d * d;
    }
  }
  const int s0 = P.win_sb_range[2 * w], s1 = P.win_sb_range[2 * w + 1];
  for (int b = s0 + t; b < s1; b += RB) {
    if (!gmem(P.sb_active)[b]) continue;
    const auto x = gmem(P.sb[xs] + 9 * (size_t)b);
    const auto g = gmem(P.gF + foff + gmem(P.sb_f)[b]);
    for (int k = 0; k < 9; ++k) {
      x2 += x[k] * x[k];
      const double d = x[k] - (x[k] + (-g[k]));
      mx = fmax(mx, fabs(d));
      g2 += d * d;
    }
  }
  const int l0 = P.win_lm_range[2 * w], l1 = P.win_lm_range[2 * w + 1];
  struct LX { double x[4], g[3]; uint8_t f; };
  stridedBatched<RB, 4>(l0, l1,
                    [&](int l) {
                      LX v;
                      v.f = gmem(P.lm_free)[l];
                      for (int k = 0; k < 4; ++k) v.x[k] = gmem(P.lm[xs])[4 * (size_t)l + k];
                      for (int k = 0; k < 3; ++k) v.g[k] = gmem(P.lm_g)[3 * (size_t)l + k];
                      return v;
                    },
                    [&](int, const LX& v) {
                      if (!v.f) return;
                      for (int k = 0; k < 4; ++k) x2 += v.x[k] * v.x[k];
                      for (int k = 0; k < 3; ++k) {
                        const double d = v.x[k] - (v.x[k] + (-v.g[k]));
                        mx = fmax(mx, fabs(d));
                        g2 += d * d;
                      }
                    });
  mx = blockMax<RB>(mx, sh);
  {
    double r2[2] = {g2, x2};
    blockSumN<RB, 2>(r2, sh);
    g2 = r2[0];
    x2 = r2[1];
  }
  if (t != 0) return;
  s.grad_max_norm = mx;
  s.grad_norm = sqrt(g2);
  s.x_norm = sqrt(x2);
  if (lin_mode == 0 && s.iteration >= P.opt.max_num_iterations) {
    s.done = 1;
    s.termination = 1;
    return;
  }
  if (mx <= P.opt.gradient_tolerance) {
    s.done = 1;
    s.termination = 0;
    return;
  }
  if (lin_mode == 0 && s.radius <= P.opt.min_radius) {
    s.done = 1;
    s.termination = 0;
  }
}


}  // namespace okg
