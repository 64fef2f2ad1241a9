"""Variable extrinsics (online calibration, do_extrinsics: true):
one T_SC block per camera shared by all states of the window (ViGraph.cpp:330-336,469-473), the
reprojection Jacobian J2 w.r.t. it (implementation/ReprojectionError.hpp:186-214) and its
PoseError prior (ViGraph.cpp:372-382), on the CPU oracle and on the GPU against it.

The GPU keeps the extrinsics as pose-kind blocks after the states: their f-blocks close the reduced
ordering (S = the states' band + a dense border), extrinsic visits (landmark, camera) join the
landmark groups of the Schur elimination and k_pose_extr forms the pose-extrinsics cross blocks.
Tolerances as tests/test_gpu_parity.py."""
import numpy as np
import pytest

from _ref_scenarios import qinv, qmul


def _window(og, kf=10, lm=500, obs=4000, seed=51, **kw):
    return og.SynthWindow(kf, lm, obs, seed=seed, do_extrinsics=1, **kw)


def _zero_tol(og, iters, **kw):
    return og.default_options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0, **kw)


def _rot(a, b):
    return 2 * np.linalg.norm(qmul(a, qinv(b))[:3])


def test_synth_online_calibration_window(og):
    w = _window(og)
    p = w.problem
    assert p.n_extrinsics_priors == 2 and list(p.extrinsics_constant[:2]) == [0, 0]
    init, true = w.extrinsics().copy(), w.true_extrinsics()
    assert 0 < np.abs(init[:, :3] - true[:, :3]).max() < 0.01
    w2 = og.SynthWindow(10, 500, 4000, seed=51)  # the same window without online calibration
    assert np.array_equal(w2.poses(), w.poses()) and np.array_equal(w2.true_extrinsics(), true)
    assert list(w2.problem.extrinsics_constant[:2]) == [1, 1]


@pytest.mark.parametrize("obs", [0, 1, 2, 3, 4000 - 1])
def test_oracle_extrinsics_jacobian_numdiff(og, oracle, obs):
    """jacobiansCorrect semantics (ErrorInterface.cpp:44-163) on all three blocks of the
    reprojection error, including J2 w.r.t. T_SC."""
    w = _window(og)
    assert oracle.check_jacobians(w.problem_ptr(), 0, obs) < 1e-6


def test_oracle_calibrates_extrinsics(og, oracle):
    """With the prior at the perturbed calibration, the window's observations pull T_SC towards the
    truth (rotation, the well-observed part)."""
    for seed in (52, 53):
        w = _window(og, kf=20, lm=1000, obs=8000, seed=seed)
        true = w.true_extrinsics()
        before = [_rot(true[c, 3:], w.extrinsics()[c, 3:]) for c in range(2)]
        s = oracle.solve(w.problem_ptr(), og.default_options(max_num_iterations=30))
        after = [_rot(true[c, 3:], w.extrinsics()[c, 3:]) for c in range(2)]
        assert s["termination"] in ("CONVERGENCE", "NO_CONVERGENCE") and s["final_cost"] < 1e-3 * s["initial_cost"]
        assert sum(after) < 0.75 * sum(before) and all(a < b for a, b in zip(after, before)), (before, after)


@pytest.mark.gpu
@pytest.mark.parametrize("mu", [0.0, 1e-8, 1e-2])
def test_gpu_linearize_reduce_extrinsics(og, oracle, gpu_ctx, mu):
    w = _window(og)
    gpu_ctx.set_problems([w.problem])
    assert gpu_ctx.stats()["n_extrinsics_free"] == 2
    S, rhs, cost = gpu_ctx.linearize_reduce(0, True, mu)
    w.reset()
    S0, rhs0, cost0, rc = oracle.linearize_reduce(w.problem_ptr(), True, mu)
    assert rc == 0 and S.shape == S0.shape == (162, 162)
    assert abs(cost - cost0) <= 1e-10 * cost0
    assert np.abs(S - S0).max() <= 1e-8 * np.abs(S0).max(), np.abs(S - S0).max() / np.abs(S0).max()
    assert np.abs(rhs - rhs0).max() <= 1e-8 * np.abs(rhs0).max()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["s10", "s50", "s50_equidistant"])
def test_gpu_solve_extrinsics(og, oracle, gpu_ctx, shape):
    """Full solves with both extrinsics variable (the Hilti-shaped case: equidistant camera at S50)."""
    if shape == "s10":
        w = _window(og, seed=53)
    else:
        w = _window(og, 50, 2000, 16000, seed=54)
        if shape == "s50_equidistant":
            from test_gpu_parity import CAMERA_MODELS, _switch_camera_model
            _switch_camera_model(oracle, w, *CAMERA_MODELS["equidistant"])
    opts = _zero_tol(og, 5)
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(opts)[0]
    P, E = w.poses().copy(), w.extrinsics().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    assert sg["num_iterations"] == so["num_iterations"] and sg["termination"] == so["termination"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-7 * so["final_cost"], (sg, so)
    assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6
    assert np.abs(E[:, :3] - w.extrinsics()[:, :3]).max() <= 1e-7
    assert max(_rot(E[c, 3:], w.extrinsics()[c, 3:]) for c in range(2)) <= 1e-7


@pytest.mark.gpu
def test_gpu_extrinsics_batch_and_freeze(og, oracle, gpu_ctx):
    """A batch mixing windows with and without online calibration, then freezing one camera's
    extrinsics between solves (okvisgpu_set_block_constant kind 3)."""
    ws = [_window(og, seed=55), og.SynthWindow(10, 500, 4000, seed=56), _window(og, 6, 150, 1000, seed=57)]
    opts = _zero_tol(og, 4)
    gpu_ctx.set_problems([w.problem for w in ws])
    sgs = gpu_ctx.solve(opts)
    for w, sg in zip(ws, sgs):
        P, E = w.poses().copy(), w.extrinsics().copy()
        w.reset()
        so = oracle.solve(w.problem_ptr(), opts)
        assert sg["num_iterations"] == so["num_iterations"]
        assert abs(sg["final_cost"] - so["final_cost"]) <= 2e-6 * so["final_cost"], (sg, so)
        assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6
        assert np.abs(E[:, :3] - w.extrinsics()[:, :3]).max() <= 1e-7
    # freeze camera 1 of window 0 (the tracking solve's extrinsics freeze, ViSlamBackend.cpp:866-872)
    for w in ws:
        w.reset()
    gpu_ctx.update_params()
    gpu_ctx.set_block_constant(0, 3, 1, True)
    sg = gpu_ctx.solve(opts)[0]
    E = ws[0].extrinsics().copy()
    ws[0].reset()
    e1 = ws[0].extrinsics()[1].copy()
    ws[0].problem.extrinsics_constant[1] = 1
    so = oracle.solve(ws[0].problem_ptr(), opts)
    assert np.array_equal(E[1], e1)
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-7 * so["final_cost"]
    assert np.abs(E[0, :3] - ws[0].extrinsics()[0, :3]).max() <= 1e-7
