"""A GPS-shaped host-evaluated factor for the §8b fallback tests (TEST INFRASTRUCTURE).

Shape of okvis' GpsErrorAsynchronous (okvis_ceres/include/okvis/ceres/GpsErrorAsynchronous.hpp:42-55):
3 residuals on the state's pose T_WS (7), its speed/bias (9) and the GPS-world alignment T_GW (7).
The antenna position at the measurement time t_k + dt, propagated with the state's velocity,

    r = L (p_GA_meas - (R_GW (r_WS + v_W dt + R_WS r_SA) + r_GW)),

with minimal Jacobians in okvis' pose perturbation (r <- r + dr, R <- exp(da) R) turned into the
ambient ones Ceres expects through the PoseManifold lift Jacobian (okvis' functors do the same:
ambient = minimal * liftJacobian, PoseLocalParameterization.cpp:89-103). This is NOT the reference's
functor (whose GNSS frame handling needs GeographicLib, absent here): it is a factor of the same
block structure, to exercise the host-evaluated path end to end."""
import numpy as np

import okvisgpu as og
from _problem import OwnedProblem


def quat_R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def oplus(q):
    x, y, z, w = q
    return np.array([[w, z, -y, x], [-z, w, x, y], [y, -x, w, z], [-x, -y, -z, w]])


def lift(T):
    """PoseManifold lift Jacobian (6x7) at T = [r, q] (PoseLocalParameterization.cpp:89-103)."""
    q = T[3:7]
    L = np.zeros((6, 7))
    L[:3, :3] = np.eye(3)
    L[3:, 3:] = 2.0 * oplus(np.array([-q[0], -q[1], -q[2], q[3]]))[:3, :]
    return L


def pose_plus(T, d):
    """okvis pose Plus: r + dr, q <- deltaQ(da) * q (PoseLocalParameterization.cpp:29-50)."""
    a = np.asarray(d[3:6], dtype=np.float64)
    n = np.linalg.norm(a)
    half = 0.5 * n
    s = np.sin(half) / n if n > 1e-12 else 0.5
    dq = np.array([a[0] * s, a[1] * s, a[2] * s, np.cos(half)])
    q = T[3:7] / np.linalg.norm(T[3:7])
    x1, y1, z1, w1 = dq
    x2, y2, z2, w2 = q
    qn = np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                   w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])
    return np.concatenate([T[:3] + d[:3], qn / np.linalg.norm(qn)])


class GpsFactors:
    """Per factor: measured antenna position [3], dt [s], 3x3 square-root information; one lever
    arm r_SA for all. evaluate(h, params) has the og.host_evaluate signature."""

    def __init__(self, meas, dt, sqrt_info, r_SA, fail=None):
        self.meas = np.asarray(meas, dtype=np.float64).reshape(-1, 3)
        self.dt = np.asarray(dt, dtype=np.float64)
        self.L = np.asarray(sqrt_info, dtype=np.float64).reshape(-1, 3, 3)
        self.r_SA = np.asarray(r_SA, dtype=np.float64)
        self.fail = fail  # fail(h, params) -> True: report an evaluation failure
        self.calls = 0

    def predict(self, h, T, sb, G):
        R_WS, R_GW = quat_R(T[3:7]), quat_R(G[3:7])
        a = R_WS @ self.r_SA
        pW = T[:3] + sb[:3] * self.dt[h] + a
        return R_GW @ pW + G[:3], a, pW, R_GW

    def evaluate(self, h, params):
        self.calls += 1
        if self.fail is not None and self.fail(h, params):
            return None
        T, sb, G = params
        pG, a, pW, R_GW = self.predict(h, T, sb, G)
        L = self.L[h]
        r = L @ (self.meas[h] - pG)
        JT = np.hstack([-L @ R_GW, L @ R_GW @ skew(a)])
        Jsb = np.zeros((3, 9))
        Jsb[:, :3] = -L @ R_GW * self.dt[h]
        JG = np.hstack([-L, L @ skew(R_GW @ pW)])
        return r, [JT @ lift(T), Jsb, JG @ lift(G)]


def random_quat(rng, sigma):
    a = rng.normal(0.0, sigma, 3)
    return pose_plus(np.array([0, 0, 0, 0, 0, 0, 1.0]), np.concatenate([[0, 0, 0], a]))[3:]


def gps_window(seed=7, n_kf=10, n_lm=500, n_obs=4000, sigma=0.05, t_gw_variable=True, fail=None):
    """A synthetic S10-shaped window (SynthWindow) with one GPS factor per keyframe on (pose k,
    speed/bias k, T_GW); T_GW is an extra pose-kind block (index n_kf) with a PoseError prior.
    Returns (problem, factors, truth T_GW)."""
    rng = np.random.default_rng(seed)
    sw = og.SynthWindow(n_kf, n_lm, n_obs, seed=seed)
    gt_poses, _, gt_sb = sw.ground_truth()
    P = OwnedProblem.copy_of(sw.problem)
    del sw
    T_GW = np.concatenate([rng.normal(0.0, 2.0, 3), random_quat(rng, 0.3)])
    r_SA = np.array([0.05, -0.02, 0.1])
    dt = rng.uniform(0.0, 0.05, n_kf)
    fac = GpsFactors(np.zeros((n_kf, 3)), dt, np.tile(np.eye(3) / sigma, (n_kf, 1, 1)), r_SA, fail=fail)
    meas = np.array([fac.predict(k, gt_poses[k], gt_sb[k], T_GW)[0] for k in range(n_kf)])
    fac.meas = meas + rng.normal(0.0, sigma, meas.shape)
    # T_GW block: initial guess perturbed from the truth, prior centred on that guess
    G0 = pose_plus(T_GW, np.concatenate([rng.normal(0.0, 0.3, 3), rng.normal(0.0, 0.05, 3)]))
    P.poses = np.vstack([P.poses, G0])
    P.pose_constant = np.concatenate([P.pose_constant, [0 if t_gw_variable else 1]]).astype(np.uint8)
    P.pose_prior_block = np.concatenate([P.pose_prior_block, [n_kf]]).astype(np.int32)
    P.pose_prior_meas = np.vstack([P.pose_prior_meas.reshape(-1, 7), G0])
    Lg = np.diag([1.0 / 1.0] * 3 + [1.0 / 0.3] * 3).reshape(-1)
    P.pose_prior_sqrt_info = np.vstack([P.pose_prior_sqrt_info.reshape(-1, 36), Lg])
    P.host_dim = np.full(n_kf, 3, np.int32)
    P.host_param_kind = np.tile(np.array([0, 1, 0, -1], np.int32), (n_kf, 1))
    P.host_param_index = np.array([[k, k, n_kf, -1] for k in range(n_kf)], np.int32)
    P.host_cauchy = np.zeros(n_kf, np.uint8)
    P.gps = fac  # keep the functor and its C callback alive with the problem
    P.host_fn = og.host_evaluate(fac.evaluate, [[7, 9, 7]] * n_kf)
    P.bind()
    return P, fac, T_GW
