"""GPU parity of the two-pose residual blocks through the C ABI against the CPU oracle
(tests/test_oracle_twopose.py pins the oracle): the pose-graph edge (TwoPoseStandardGraphError,
TwoPoseGraphError.cpp:162-767) and RelativePoseError (RelativePoseError.cpp:59-140); the synthetic
windows mix both kinds unless a test says otherwise.

Tolerances (FP64 both sides, different operation orders):
  * edge residuals / minimal Jacobians: 1e-12 relative to the block norm;
  * compute(): the marginalised H00_ / b0_ 1e-9 relative (lane-tree vs sequential landmark sums),
    J_^T J_ 1e-9, DeltaX_ through J_^T J_ DeltaX_ = -b0_ and 1e-7 relative directly (H00_ has a
    condition number ~1e4-1e6), the linearisation point 1e-14;
  * reduced system and full solves with edges in the window: as test_gpu_parity.py.
"""
import numpy as np
import pytest

import _twopose as tp

pytestmark = pytest.mark.gpu


def _relpose_window(og, kf=10, lm=500, obs=4000, n_relpose=6, stride=3, seed=20251015, kind=2):
    """kind 0 pose-graph edges, 1 RelativePoseError, 2 alternating."""
    return og.SynthWindow(kf, lm, obs, seed=seed, n_relpose=n_relpose, relpose_stride=stride, relpose_kind=kind)


def _opts(og, iters, **kw):
    return og.default_options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0, **kw)


@pytest.mark.parametrize("kind", [0, 1])
def test_relpose_functor_parity(og, oracle, gpu_ctx, kind):
    w = _relpose_window(og, kind=kind)
    P = w.poses()
    rng = np.random.default_rng(5)
    P[:, :3] += rng.normal(0, 0.05, P[:, :3].shape)  # away from the linearisation points
    n = w.problem.n_relpose
    gpu_ctx.set_problems([w.problem])
    r, J = gpu_ctx.eval_relpose(n)
    r0, J0 = oracle.eval_relpose(w.problem_ptr(), n)
    assert np.abs(r - r0).max() <= 1e-12 * np.abs(r0).max()
    err = np.linalg.norm((J - J0).reshape(n, -1), axis=1)
    assert np.all(err <= 1e-12 * np.linalg.norm(J0.reshape(n, -1), axis=1))


def test_twopose_compute_parity(og, oracle, gpu_ctx):
    edges = []
    for seed in range(6):
        e, cams, ex = tp.scene(oracle, 100 + seed, n_lm=30 + 25 * seed, outliers=2 * (seed % 3),
                               mono_far=seed % 2, mono_near=(seed + 1) % 2)
        edges.append(e)
    e, cams, ex = tp.scene(oracle, 200, n_lm=12, no_other=True)
    edges.append(e)
    # a moved reference keyframe (T_WS0 != I)
    e, cams, ex = tp.scene(oracle, 201, n_lm=80, ref_pose=np.r_[[1.0, -2.0, 0.3], tp.quat_from_axis_angle(
        np.array([0.1, 0.3, -0.7]))])
    edges.append(e)
    batch = og.TwoPoseBatch(edges, cams, ex)
    g = gpu_ctx.twopose_compute(batch)
    c = oracle.twopose_compute(batch)
    for k in range(len(edges)):
        H0 = c["H00"][k]
        s = max(np.abs(H0).max(), 1e-300)
        assert np.abs(g["H00"][k] - H0).max() <= 1e-9 * s, k
        assert np.abs(g["b0"][k] - c["b0"][k]).max() <= 1e-9 * max(np.abs(c["b0"][k]).max(), 1e-300), k
        JtJ, JtJ0 = g["sqrt_info"][k].T @ g["sqrt_info"][k], c["sqrt_info"][k].T @ c["sqrt_info"][k]
        assert np.abs(JtJ - JtJ0).max() <= 1e-9 * max(np.abs(JtJ0).max(), 1e-300), k
        assert np.abs(JtJ @ g["delta_x"][k] + g["b0"][k]).max() <= 1e-7 * max(np.abs(c["b0"][k]).max(), 1e-300), k
        dx0 = c["delta_x"][k]
        assert np.abs(g["delta_x"][k] - dx0).max() <= 1e-7 * max(np.abs(dx0).max(), 1e-300), k
        assert np.abs(g["lin_point"][k] - c["lin_point"][k]).max() <= 1e-14, k
    assert np.array_equal(g["lin_point"][6], [0, 0, 0, 0, 0, 0, 1])


@pytest.mark.parametrize("mu", [0.0, 1e-4])
def test_linearize_reduce_with_relpose(og, oracle, gpu_ctx, mu):
    w = _relpose_window(og, n_relpose=8, stride=4)
    gpu_ctx.set_problems([w.problem])
    S, rhs, cost = gpu_ctx.linearize_reduce(0, True, mu)
    w.reset()
    S0, rhs0, cost0, rc = oracle.linearize_reduce(w.problem_ptr(), True, mu)
    assert rc == 0 and S.shape == S0.shape
    assert abs(cost - cost0) <= 1e-10 * cost0
    assert np.abs(S - S0).max() <= 1e-8 * np.abs(S0).max()
    assert np.abs(rhs - rhs0).max() <= 1e-8 * np.abs(rhs0).max()


def _close(sg, so, rel=1e-7):
    assert sg["num_iterations"] == so["num_iterations"], (sg, so)
    assert sg["termination"] == so["termination"], (sg, so)
    assert abs(sg["final_cost"] - so["final_cost"]) <= rel * so["final_cost"], (sg, so)


@pytest.mark.parametrize("iters", [3, 10])
def test_solve_parity_with_relpose(og, oracle, gpu_ctx, iters):
    w = _relpose_window(og, n_relpose=8, stride=4)
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(_opts(og, iters), 1)[0]
    P = w.poses().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), _opts(og, iters))
    _close(sg, so)
    assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6


def test_ragged_batch_with_relpose(og, oracle, gpu_ctx):
    """Windows with and without pose-graph edges (and a constant reference pose) in one batch."""
    ws = [_relpose_window(og, 6, 150, 1000, n_relpose=3, stride=2, seed=41),
          og.SynthWindow(10, 500, 4000, seed=42),
          _relpose_window(og, 12, 500, 4000, n_relpose=10, stride=5, seed=43)]
    ws[2].problem.pose_constant[1] = 1  # an edge whose reference pose is frozen
    gpu_ctx.set_problems([w.problem for w in ws])
    sgs = gpu_ctx.solve(_opts(og, 4), len(ws))
    for w, sg in zip(ws, sgs):
        P = w.poses().copy()
        w.reset()
        so = oracle.solve(w.problem_ptr(), _opts(og, 4))
        _close(sg, so, rel=2e-6)
        assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6


def test_relpose_cholesky_schedules(og, oracle, gpu_ctx):
    """Non-adjacent keyframe pairs widen the band of S: every schedule must follow the fill."""
    w = _relpose_window(og, 20, 800, 6000, n_relpose=6, stride=9, seed=44)
    so = None
    for sched in (1, 2, 3, 4, 5):
        w.reset()
        gpu_ctx.set_problems([w.problem])
        sg = gpu_ctx.solve(_opts(og, 4, cholesky_schedule=sched), 1)[0]
        P = w.poses().copy()
        if so is None:
            w.reset()
            so = oracle.solve(w.problem_ptr(), _opts(og, 4))
            P0 = w.poses().copy()
        _close(sg, so)
        assert np.abs(P[:, :3] - P0[:, :3]).max() <= 1e-6


def test_wide_band_schedules_bitwise(og, oracle, gpu_ctx):
    """Edges 30 keyframes apart give columns of S with more non-zero tiles below the diagonal than
    the back substitution keeps in its prefetch list (kBsPre = 3): the persistent and tile-parallel
    schedules must still agree bitwise, and both with the oracle."""
    w = _relpose_window(og, 40, 1600, 12000, n_relpose=4, stride=30, seed=45)
    res = []
    for sched in (1, 2, 3, 4, 5):
        w.reset()
        gpu_ctx.set_problems([w.problem])
        sg = gpu_ctx.solve(_opts(og, 4, cholesky_schedule=sched), 1)[0]
        res.append((sg, w.poses().copy()))
    for r in res[1:]:
        assert r[0]["final_cost"] == res[0][0]["final_cost"]
        assert np.array_equal(r[1], res[0][1])
    w.reset()
    so = oracle.solve(w.problem_ptr(), _opts(og, 4))
    _close(res[0][0], so)
    assert np.abs(res[0][1][:, :3] - w.poses()[:, :3]).max() <= 1e-6
