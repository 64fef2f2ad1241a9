"""A submap-alignment-shaped host-evaluated factor for the loss tests (TEST INFRASTRUCTURE).

Shape of okvis' SubmapIcpError as ViGraph adds it (okvis_ceres/src/ViGraph.cpp:1498-1520): ONE
residual on two poses (state_A's pose, state_B's pose), robustified with CauchyLoss(1.0) or
TukeyLoss(2.0) (LiDAR) / TukeyLoss(0.1) (depth). The reference functor queries a supereight2
occupancy field (un-vendored); this factor uses a point-to-plane distance of the same
block structure instead:

    r = n . (T_WB p_B - T_WA q_A) / sigma

with a point p_B in B's frame, its match q_A in A's frame and the plane normal n (world frame).
Minimal Jacobians in okvis' pose perturbation (r <- r + dr, R <- exp(da) R) are turned into the
ambient ones Ceres expects through the PoseManifold lift Jacobian, as tests/_gps.py does."""
import numpy as np

import okvisgpu as og
from _gps import gps_window, lift, quat_R, skew


class SubmapFactors:
    """Per factor: blocks (a, b), p_B [3], q_A [3], n [3] (unit), sigma (the sensor error)."""

    def __init__(self, pairs, p_B, q_A, n, sigma):
        self.pairs = np.asarray(pairs, dtype=np.int32).reshape(-1, 2)
        self.p_B = np.asarray(p_B, dtype=np.float64).reshape(-1, 3)
        self.q_A = np.asarray(q_A, dtype=np.float64).reshape(-1, 3)
        self.n = np.asarray(n, dtype=np.float64).reshape(-1, 3)
        self.sigma = np.broadcast_to(np.asarray(sigma, dtype=np.float64), (len(self.pairs),)).copy()

    def residual(self, h, TA, TB):
        pW = quat_R(TB[3:7]) @ self.p_B[h] + TB[:3]
        qW = quat_R(TA[3:7]) @ self.q_A[h] + TA[:3]
        return float(self.n[h] @ (pW - qW)) / self.sigma[h]

    def evaluate(self, h, params):
        TA, TB = params
        r = self.residual(h, TA, TB)
        nrm = self.n[h] / self.sigma[h]
        a = quat_R(TA[3:7]) @ self.q_A[h]
        b = quat_R(TB[3:7]) @ self.p_B[h]
        JA = -np.concatenate([nrm, -nrm @ skew(a)])[None, :]
        JB = np.concatenate([nrm, -nrm @ skew(b)])[None, :]
        return np.array([r]), [JA @ lift(TA), JB @ lift(TB)]


def loss_window(seed=41, n_kf=10, per_pair=3, sigma=0.02, gps_loss=("cauchy", 3.0),
                submap_losses=(("tukey", 2.0), ("tukey", 0.1)), tolerant_every=4):
    """S10 + GPS factors (loss gps_loss, ViGraph.cpp:999; every `tolerant_every`-th one under
    TolerantLoss(4, 1) instead, whose rho'' > 0 exercises the Corrector's second-order branch) and
    `per_pair` submap-shaped factors between consecutive keyframes, alternating over
    submap_losses (TukeyLoss(2.0) LiDAR / TukeyLoss(0.1) depth, ViGraph.cpp:1510,1513). A factor's
    sensor error is `sigma` scaled so that its loss scale is ~2.5 noise standard deviations (the
    initial pose errors put some factors in Tukey's outlier region, the solve moves them in). Three GPS
    measurements carry gross errors and every fifth submap factor a 20-sigma outlier, so the losses
    shape the solve. The callbacks of both factor kinds go through one host_evaluate. Returns (problem,
    gps factors, submap factors)."""
    rng = np.random.default_rng(seed)
    P, gps, T_GW = gps_window(seed=seed, n_kf=n_kf)
    sw = og.SynthWindow(n_kf, 500, 4000, seed=seed)
    gt, _, _ = sw.ground_truth()
    del sw
    gps.meas[[1, 4, 7]] += np.array([2.0, -2.0, 1.5])
    pairs, pB, qA, nn, sg = [], [], [], [], []
    for k in range(n_kf - 1):
        for j in range(per_pair):
            pairs.append((k, k + 1))
            a = submap_losses[(len(pairs) - 1) % len(submap_losses)][1]
            sg.append(sigma * 2.5 / a)  # r = distance / sigma: the loss scale a ~ 2.5 noise sigmas
            p = rng.uniform(-3.0, 3.0, 3) + np.array([0.0, 0.0, 6.0])
            RA, RB = quat_R(gt[k][3:7]), quat_R(gt[k + 1][3:7])
            pW = RB @ p + gt[k + 1][:3]
            n = rng.normal(size=3)
            n /= np.linalg.norm(n)
            noise = rng.normal(0.0, sigma)
            if len(pairs) % 5 == 0:
                noise += 20.0 * sigma
            q = RA.T @ (pW - n * noise - gt[k][:3])
            pB.append(p)
            qA.append(q)
            nn.append(n)
    sub = SubmapFactors(pairs, pB, qA, nn, sg)
    n_gps, n_sub = n_kf, len(pairs)
    P.host_dim = np.concatenate([np.full(n_gps, 3), np.full(n_sub, 1)]).astype(np.int32)
    P.host_param_kind = np.vstack([np.tile([0, 1, 0, -1], (n_gps, 1)), np.tile([0, 0, -1, -1], (n_sub, 1))]).astype(np.int32)
    P.host_param_index = np.vstack([np.array([[k, k, n_kf, -1] for k in range(n_gps)]),
                                    np.array([[a, b, -1, -1] for a, b in pairs])]).astype(np.int32)
    P.host_cauchy = np.zeros(n_gps + n_sub, np.uint8)
    specs = [(("tolerant", 4.0, 1.0) if (tolerant_every and k % tolerant_every == tolerant_every - 1) else gps_loss)
             for k in range(n_gps)]
    specs += [submap_losses[i % len(submap_losses)] for i in range(n_sub)]
    P.host_loss = og.loss_array(specs)

    def evaluate(h, params):
        if h < n_gps:
            return gps.evaluate(h, params)
        return sub.evaluate(h - n_gps, params)

    P.submap = sub
    P.host_fn = og.host_evaluate(evaluate, [[7, 9, 7]] * n_gps + [[7, 7]] * n_sub)
    P.bind()
    return P, gps, sub
