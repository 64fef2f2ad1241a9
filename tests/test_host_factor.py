"""§8b host-evaluated fallback (ABI 5): residual blocks the GPU path has no functor for are evaluated
by the caller's CostFunction::Evaluate on host threads at every point the solver evaluates, and
their r / J (manifold and loss applied by the backend) join the reduced system like any
device-evaluated factor. Tested with a GPS-shaped factor (GpsErrorAsynchronous.hpp:42-55 block
shape: pose 7 / speed-bias 9 / alignment pose 7; tests/_gps.py) on S10 synthetic windows.

CPU: the oracle's restatement (Ceres ResidualBlock with manifolds) gets the minimal Jacobian right
(numeric differentiation on the manifold), solves the window, and handles evaluation failure
(initial point: FAILURE; candidate: rejected step, Ceres' candidate_cost = max).
GPU: okvisgpu's gather -> host callback -> upload path reproduces the oracle (r bit for bit, J to
1e-14) at the
functor level and the solve's iterations / termination / estimates across single windows, batches
(threaded host evaluation, forked iteration graph), fixed factors and failures."""
import ctypes as C

import numpy as np
import pytest

import okvisgpu as og
import _oracle
from _gps import gps_window, pose_plus

N_KF = 10


def _numeric_minimal_jacobian(fac, h, T, sb, G, eps=1e-7):
    def res(T, sb, G):
        return fac.evaluate(h, [T, sb, G])[0]
    Jn = np.zeros((3, 30))
    for c in range(6):
        d = np.zeros(6)
        d[c] = eps
        Jn[:, c] = (res(pose_plus(T, d), sb, G) - res(pose_plus(T, -d), sb, G)) / (2 * eps)
        Jn[:, 15 + c] = (res(T, sb, pose_plus(G, d)) - res(T, sb, pose_plus(G, -d))) / (2 * eps)
    for c in range(9):
        d = np.zeros(9)
        d[c] = eps
        Jn[:, 6 + c] = (res(T, sb + d, G) - res(T, sb - d, G)) / (2 * eps)
    return Jn


def test_oracle_host_factor_minimal_jacobian(og):
    """Ambient Jacobians x PoseManifold plus Jacobian = the numeric minimal Jacobian on the manifold
    (jacobiansCorrect semantics, ErrorInterface.cpp:44-163), and the residual rows past dim are 0."""
    P, fac, _ = gps_window()
    r, J, rc = _oracle.eval_host(P.ptr(), N_KF)
    assert rc == 0
    assert np.all(r[:, 3:] == 0.0) and np.all(J[:, 3:, :] == 0.0)
    worst = 0.0
    for h in range(N_KF):
        Jn = _numeric_minimal_jacobian(fac, h, P.poses[h], P.speed_biases[h], P.poses[N_KF])
        worst = max(worst, np.abs(Jn - J[h, :3]).max() / np.abs(J[h, :3]).max())
        assert np.allclose(r[h, :3], fac.evaluate(h, [P.poses[h], P.speed_biases[h], P.poses[N_KF]])[0], rtol=0, atol=0)
    print(f"host factor minimal Jacobian vs numeric: max rel {worst:.2e}")
    assert worst < 1e-6


def test_oracle_gps_window_solve(og):
    """The window with GPS factors solves and the alignment T_GW moves toward the truth."""
    P, fac, T_GW = gps_window()
    before = np.abs(P.poses[N_KF, :3] - T_GW[:3]).max()
    s = _oracle.solve(P.ptr(), og.default_options(max_num_iterations=10, num_threads=2))
    assert s["final_cost"] < 1e-2 * s["initial_cost"]
    after = np.abs(P.poses[N_KF, :3] - T_GW[:3]).max()
    assert after < 0.3 * before, (before, after)
    assert fac.calls > N_KF * (s["num_iterations"] + 1) // 2


def test_oracle_host_failure_semantics(og):
    """Failure at the initial point ends the solve with FAILURE (no step taken); failures at
    candidates only reject those steps (candidate_cost = max)."""
    P, fac, _ = gps_window(fail=lambda h, prm: h == 3)
    x0 = P.poses.copy()
    s = _oracle.solve(P.ptr(), og.default_options(max_num_iterations=10))
    assert s["termination"] == "FAILURE" and s["num_iterations"] == 0
    assert np.array_equal(P.poses, x0)

    P, fac, _ = gps_window()
    G0 = P.poses[N_KF].copy()
    # fail whenever the alignment's translation moved more than 0.1 m from its initial guess: the
    # first Gauss-Newton step (~0.25 m) is rejected and the trust region shrinks until it passes
    fac.fail = lambda h, prm: np.abs(prm[2][:3] - G0[:3]).max() > 0.1
    s = _oracle.solve(P.ptr(), og.default_options(max_num_iterations=10))
    assert s["num_unsuccessful_steps"] >= 1 and s["num_successful_steps"] >= 2
    assert s["termination"] != "FAILURE"


# ------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_host_factor_validation(og):
    """set_problems rejects malformed host factors: a landmark block (UNSUPPORTED: the fallback
    covers pose-kind / speed-bias blocks), a repeated block, a bad dimension, a missing callback."""
    ctx = og.Context(0)
    try:
        cases = [("param_kind", (0, 2), 2, "UNSUPPORTED"), ("param_index", (0, 2), 0, "repeated"),
                 ("dim", (0,), 16, "dimension"), ("fn", None, None, "missing")]
        for field, at, val, what in cases:
            P, _, _ = gps_window()
            if field == "fn":
                P.host_fn = None
            else:
                getattr(P, "host_" + field)[at] = val
            P.bind()
            with pytest.raises(og.OkvisGpuError) as e:
                ctx.set_problems([P.struct])
            code = 2 if what == "UNSUPPORTED" else 1
            assert f"({code})" in str(e.value), (field, str(e.value))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_eval_host_matches_oracle(og, parity):
    """Functor level: gathered parameters and the callback give r identical to the oracle's (0 ulp);
    the ambient -> minimal conversion J = J_amb * PlusJacobian agrees to 1e-14 relative (same
    operation order; the two host compilers contract the products into FMAs differently)."""
    P, fac, _ = gps_window()
    rc_ref, Jc_ref, rc = _oracle.eval_host(P.ptr(), N_KF)
    assert rc == 0
    ctx = og.Context(0)
    try:
        ctx.set_problems([P.struct])
        r, J = ctx.eval_host(N_KF)
    finally:
        ctx.close()
    parity("host factor r (max abs diff)", np.abs(r - rc_ref).max(), 0.0)
    parity("host factor minimal J (max abs / max |J|)", np.abs(J - Jc_ref).max() / np.abs(Jc_ref).max(), 1e-14)


def _solve_both(probs, options, **ctx_opts):
    """okvisgpu on copies of `probs` (one batch) and the oracle on each; returns both results."""
    snaps = [P.snapshot() for P in probs]
    ctx = og.Context(0)
    try:
        ctx.set_problems([P.struct for P in probs])
        gsum = ctx.solve(options)
    finally:
        ctx.close()
    gpu = [(P.poses.copy(), P.speed_biases.copy(), P.landmarks.copy()) for P in probs]
    csum = []
    for P, snap in zip(probs, snaps):
        P.restore(snap)
        csum.append(_oracle.solve(P.ptr(), options))
    cpu = [(P.poses.copy(), P.speed_biases.copy(), P.landmarks.copy()) for P in probs]
    return gsum, csum, gpu, cpu


def _assert_parity(parity, gsum, csum, gpu, cpu, tag):
    worst_p = worst_c = 0.0
    for w, (g, c) in enumerate(zip(gsum, csum)):
        assert (g["num_iterations"], g["termination"], g["num_successful_steps"], g["num_unsuccessful_steps"]) == \
            (c["num_iterations"], c["termination"], c["num_successful_steps"], c["num_unsuccessful_steps"]), (tag, w, g, c)
        if np.isfinite(c["final_cost"]):
            worst_c = max(worst_c, abs(g["final_cost"] - c["final_cost"]) / c["final_cost"])
        worst_p = max(worst_p, float(np.abs(gpu[w][0][:, :3] - cpu[w][0][:, :3]).max()))
    parity(f"host factors, {tag}: positions (m)", worst_p, 1e-6)
    parity(f"host factors, {tag}: final cost (rel)", worst_c, 1e-7)


@pytest.mark.gpu
def test_gpu_gps_window_solve_parity(og, parity):
    P, _, _ = gps_window()
    o = og.default_options(max_num_iterations=10, num_threads=2)
    _assert_parity(parity, *_solve_both([P], o), "S10 + GPS")


@pytest.mark.gpu
def test_gpu_gps_batch_forked_graph_parity(og, monkeypatch, parity):
    """24 windows, 240 host factors evaluated on 4 host threads, inside the forked iteration graph
    (forced with OKVISGPU_SERIAL_GRAPH=0); every fifth window with a constant alignment block."""
    monkeypatch.setenv("OKVISGPU_SERIAL_GRAPH", "0")
    probs = [gps_window(seed=100 + i, t_gw_variable=(i % 5 != 0))[0] for i in range(24)]
    o = og.default_options(max_num_iterations=10, num_threads=4)
    _assert_parity(parity, *_solve_both(probs, o), "24 x (S10 + GPS), forked graph")


@pytest.mark.gpu
def test_gpu_host_fixed_factors_parity(og, parity):
    """Host factors whose blocks are all constant (frozen states 0-1, constant alignment) contribute
    fixed cost only (evaluated at the initial point, excluded from the reduced system), as Ceres
    removes fully-constant residual blocks; the other GPS factors stay in the solve."""
    P, _, _ = gps_window(t_gw_variable=False)
    P.pose_constant[:2] = 1
    P.speed_bias_constant[:2] = 1
    P.bind()
    o = og.default_options(max_num_iterations=8)
    _assert_parity(parity, *_solve_both([P], o), "fixed host factors")


@pytest.mark.gpu
@pytest.mark.parametrize("serial", ["1", "0"])
def test_gpu_host_failure_parity(og, parity, monkeypatch, serial):
    """Failure at the initial point (window ends with FAILURE, parameters untouched) and at
    candidates (rejected steps) give the oracle's summaries; the other windows of the batch are
    unaffected. Both captured graphs: the forked one clears S at the end of every iteration for the
    next (k_zero_S tail mode), which the rejected steps of window 1 exercise."""
    monkeypatch.setenv("OKVISGPU_SERIAL_GRAPH", serial)
    P0, _, _ = gps_window(seed=11, fail=lambda h, prm: h == 3)
    P1, f1, _ = gps_window(seed=12)
    G0 = P1.poses[N_KF].copy()
    f1.fail = lambda h, prm: np.abs(prm[2][:3] - G0[:3]).max() > 0.1
    P2, _, _ = gps_window(seed=13)
    x0 = P0.poses.copy()
    o = og.default_options(max_num_iterations=10)
    gsum, csum, gpu, cpu = _solve_both([P0, P1, P2], o)
    assert gsum[0]["termination"] == "FAILURE" and np.array_equal(gpu[0][0], x0)
    assert gsum[1]["num_unsuccessful_steps"] >= 1
    _assert_parity(parity, gsum, csum, gpu, cpu, f"host evaluation failures, serial graph {serial}")


def _cauchy_window(seed=21):
    """S10 + GPS with CauchyLoss(1) on every other factor and three gross GPS outliers (2 m on
    keyframes 1, 4, 7, against sigma 0.05 m), so the loss changes both the cost and the step."""
    P, fac, T_GW = gps_window(seed=seed)
    P.host_cauchy[::2] = 1
    P.host_cauchy[[1, 7]] = 1
    fac.meas[[1, 4, 7]] += np.array([2.0, -2.0, 1.5])
    P.bind()
    return P, fac


def test_oracle_host_cauchy_semantics(og):
    """The oracle's Corrector on host factors: cost 0.5 log(1 + |r|^2) and r, J scaled by
    sqrt(rho') = 1 / sqrt(1 + |r|^2) (Ceres' Corrector with rho'' < 0: TwoPoseGraphError.cpp:292-337
    restates it), against the raw evaluation of the same factors."""
    P, fac = _cauchy_window()
    cost = _oracle.evaluate(P.ptr())
    P.host_cauchy[:] = 0
    P.bind()
    raw = _oracle.evaluate(P.ptr())
    expect = 0.0
    for h in range(N_KF):
        r, _ = fac.evaluate(h, [P.poses[h], P.speed_biases[h], P.poses[N_KF]])
        s = float(r @ r)
        expect += (0.5 * np.log1p(s) if h in (0, 1, 2, 4, 6, 7, 8) else 0.5 * s) - 0.5 * s
    assert abs((cost - raw) - expect) <= 1e-9 * abs(raw)


@pytest.mark.gpu
def test_gpu_host_cauchy_parity(og, parity):
    """Host factors with CauchyLoss(1) (host_cauchy = 1): the runtime's Corrector scaling and
    0.5 log(1 + s) cost against the oracle, at the initial point (okvisgpu_evaluate) and in a solve."""
    P, _ = _cauchy_window()
    c_ref = _oracle.evaluate(P.ptr())
    ctx = og.Context(0)
    try:
        ctx.set_problems([P.struct])
        c_gpu = ctx.evaluate(0)
    finally:
        ctx.close()
    parity("host factors, Cauchy: initial cost (rel)", abs(c_gpu - c_ref) / c_ref, 1e-12)
    o = og.default_options(max_num_iterations=10, num_threads=2)
    _assert_parity(parity, *_solve_both([P], o), "S10 + GPS with Cauchy")


@pytest.mark.gpu
def test_gpu_evaluate_reports_host_failure(og):
    """okvisgpu_evaluate (ceres::Problem::Evaluate) with a failing host factor returns
    OKVISGPU_ERR_NUMERICAL, as okvisgpu_eval_host does, instead of OK with an infinite cost."""
    P, _, _ = gps_window(seed=11, fail=lambda h, prm: h == 3)
    ctx = og.Context(0)
    try:
        ctx.set_problems([P.struct])
        with pytest.raises(og.OkvisGpuError) as e:
            ctx.evaluate(0)
        assert "host_evaluate failed" in str(e.value)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_profile_iteration_with_host_factors(og):
    """okvisgpu_profile_iteration runs a real iteration of the live solve: with host factors its
    candidate evaluation includes them, so the solve it advanced matches a solve without profiling."""
    opts = og.default_options(max_num_iterations=6, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    res = []
    for profile in (False, True):
        P, _, _ = gps_window(seed=31)
        ctx = og.Context(0)
        try:
            ctx.set_problems([P.struct])
            ctx.solve_begin(opts)
            for it in range(6):
                if profile and it in (1, 3):
                    ctx.profile_iteration()
                else:
                    ctx.solve_iterate(1)
            s = ctx.solve_end()[0]
        finally:
            ctx.close()
        res.append((s, P.poses.copy()))
    (s0, x0), (s1, x1) = res
    assert s0["num_iterations"] == s1["num_iterations"] and s0["final_cost"] == s1["final_cost"], (s0, s1)
    assert np.array_equal(x0, x1)
