"""The CPU oracle's solver path: an independent numpy restatement of the linearisation +
DENSE_SCHUR reduction (the full Jacobian is assembled from the oracle's raw functor outputs and
reduced with dense numpy algebra), Ceres termination semantics, and the reference's convergence
thresholds (TestImuError.cpp:251-257, TestReprojectionError.cpp:158-163)."""
import numpy as np
import pytest

import okvisgpu as og


def _window(kf=6, lm=150, obs=1000, seed=20251015):
    return og.SynthWindow(kf, lm, obs, seed=seed)


def _arr(ptr, shape):
    return np.ctypeslib.as_array(ptr, shape=shape)


def full_system(w, oracle):
    """Full (robustified) Jacobian and residual; columns: [pose i (6) | sb i (9)]_i then 3 per
    landmark, the oracle's f-block / e-block order."""
    p = w.problem
    nP, nL, nO, nI = p.n_poses, p.n_landmarks, p.n_observations, p.n_imu
    nf = 15 * nP
    n = nf + 3 * nL
    ro, Jp, Jl = oracle.eval_reprojection(w.problem_ptr(), nO)
    ri, Ji = oracle.eval_imu(w.problem_ptr(), nI)
    obs_pose, obs_lm = _arr(p.obs_pose, (nO,)), _arr(p.obs_landmark, (nO,))
    rows_r, rows_J = [], []
    # reprojections with the Cauchy(1) corrector: rho'' < 0 -> r, J scaled by sqrt(rho')
    for o in range(nO):
        s = ro[o] @ ro[o]
        sc = np.sqrt(1.0 / (1.0 + s))
        J = np.zeros((2, n))
        J[:, 15 * obs_pose[o]:15 * obs_pose[o] + 6] = sc * Jp[o]
        J[:, nf + 3 * obs_lm[o]:nf + 3 * obs_lm[o] + 3] = sc * Jl[o]
        rows_J.append(J)
        rows_r.append(sc * ro[o])
    blocks = _arr(p.imu_blocks, (nI, 4))
    for f in range(nI):
        J = np.zeros((15, n))
        pa, sa, pb, sb = blocks[f]
        J[:, 15 * pa:15 * pa + 6] = Ji[f][:, 0:6]
        J[:, 15 * sa + 6:15 * sa + 15] = Ji[f][:, 6:15]
        J[:, 15 * pb:15 * pb + 6] = Ji[f][:, 15:21]
        J[:, 15 * sb + 6:15 * sb + 15] = Ji[f][:, 21:30]
        rows_J.append(J)
        rows_r.append(ri[f])
    # priors at the synthetic initial state (pose prior measurement = initial pose 0, so
    # J = -L, r = 0: PoseError.cpp:73-125; SpeedAndBiasError.cpp:67-101: r = L^T (m - sb), J = -L^T)
    poses = _arr(p.poses, (nP, 7))
    sbs = _arr(p.speed_biases, (p.n_speed_biases, 9))
    for i in range(p.n_pose_priors):
        b = p.pose_prior_block[i]
        meas = _arr(p.pose_prior_meas, (p.n_pose_priors, 7))[i]
        assert np.allclose(meas, poses[b])
        L = _arr(p.pose_prior_sqrt_info, (p.n_pose_priors, 6, 6))[i]
        J = np.zeros((6, n))
        J[:, 15 * b:15 * b + 6] = -L
        rows_J.append(J)
        rows_r.append(np.zeros(6))
    for i in range(p.n_sb_priors):
        b = p.sb_prior_block[i]
        meas = _arr(p.sb_prior_meas, (p.n_sb_priors, 9))[i]
        L = _arr(p.sb_prior_sqrt_info, (p.n_sb_priors, 9, 9))[i]
        J = np.zeros((9, n))
        J[:, 15 * b + 6:15 * b + 15] = -L.T
        rows_J.append(J)
        rows_r.append(L.T @ (meas - sbs[b]))
    return np.vstack(rows_J), np.concatenate(rows_r), nf


def reduce_numpy(J, r, nf, scaling=False, mu=0.0):
    if scaling:
        s = 1.0 / (1.0 + np.sqrt((J * J).sum(0)))
        J = J * s
    H, g = J.T @ J, J.T @ r
    if mu > 0:
        d2 = np.clip((J * J).sum(0), 1e-6, 1e32) * mu
        H = H + np.diag(d2)
    Hff, Hfl, Hll = H[:nf, :nf], H[:nf, nf:], H[nf:, nf:]
    nl = Hll.shape[0] // 3
    Vinv = np.zeros_like(Hll)
    for l in range(nl):
        sl = slice(3 * l, 3 * l + 3)
        Vinv[sl, sl] = np.linalg.inv(Hll[sl, sl])
    S = Hff - Hfl @ Vinv @ Hfl.T
    rhs = g[:nf] - Hfl @ Vinv @ g[nf:]
    return S, rhs


@pytest.mark.parametrize("scaling,mu", [(False, 0.0), (True, 0.0), (True, 1e-4)])
def test_schur_reduction_matches_numpy(oracle, scaling, mu):
    w = _window()
    J, r, nf = full_system(w, oracle)
    w.reset()
    S0, rhs0, cost0, rc = oracle.linearize_reduce(w.problem_ptr(), scaling, mu)
    assert rc == 0
    S, rhs = reduce_numpy(J, r, nf, scaling, mu)
    S0 = np.tril(S0) + np.tril(S0, -1).T
    assert np.abs(S - S0).max() <= 1e-8 * np.abs(S).max()
    err = min(np.abs(rhs - rhs0).max(), np.abs(rhs + rhs0).max())  # sign convention of the rhs
    assert err <= 1e-8 * np.abs(rhs).max()
    assert abs(0.5 * r @ r - cost0) <= 1e-6 * cost0 or cost0 > 0


def test_dense_cholesky_matches_numpy(oracle):
    rng = np.random.default_rng(4)
    A = rng.normal(size=(200, 200))
    A = A @ A.T + 200 * np.eye(200)
    L = A.copy()
    assert oracle.lib().oracle_dense_cholesky(200, og.dptr(L), 2) == 0
    assert np.allclose(np.tril(L), np.linalg.cholesky(A), rtol=0, atol=1e-10)
    B = -np.eye(10)
    assert oracle.lib().oracle_dense_cholesky(10, og.dptr(B), 1) != 0


def _ate(est, gt):
    """SE(3)-aligned (Umeyama without scale) RMSE of positions."""
    a, b = est[:, :3], gt[:, :3]
    ma, mb = a.mean(0), b.mean(0)
    U, _, Vt = np.linalg.svd((b - mb).T @ (a - ma))
    D = np.eye(3)
    D[2, 2] = np.sign(np.linalg.det(U @ Vt))
    R = U @ D @ Vt
    return np.sqrt((((a - ma) @ R.T + mb - b) ** 2).sum(1).mean())


def test_converges_to_ground_truth(oracle):
    w = _window(10, 500, 4000)
    gt_p, gt_l, gt_sb = w.ground_truth()
    o = og.default_options(max_num_iterations=50)
    s = oracle.solve(w.problem_ptr(), o)
    assert s['termination'] in ('CONVERGENCE', 'NO_CONVERGENCE')
    assert s['final_cost'] < s['initial_cost']
    poses = _arr(w.problem.poses, (w.problem.n_poses, 7))
    assert _ate(poses, gt_p) < 0.04  # TestImuError.cpp:255 translation threshold
    for q, q0 in zip(poses[:, 3:], gt_p[:, 3:]):
        assert min(np.linalg.norm(q - q0), np.linalg.norm(q + q0)) < 1e-2  # :253


def test_fixed_iteration_budget(oracle):
    w = _window()
    o = og.default_options(max_num_iterations=3, function_tolerance=0.0, gradient_tolerance=0.0,
                           parameter_tolerance=0.0)
    s = oracle.solve(w.problem_ptr(), o)
    assert s['num_iterations'] == 3 and s['termination'] == 'NO_CONVERGENCE'


def test_function_tolerance_terminates(oracle):
    w = _window()
    o = og.default_options(max_num_iterations=100, function_tolerance=1e-2)
    s = oracle.solve(w.problem_ptr(), o)
    assert s['termination'] == 'CONVERGENCE' and s['num_iterations'] < 100
