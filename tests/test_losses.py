"""Robust losses at the boundary (ABI 6): the ::ceres::LossFunction family okvis attaches
(ViGraph.cpp:235-238: CauchyLoss(1.0), CauchyLoss(3.0) for GPS, TukeyLoss(0.1) / TukeyLoss(2.0) for
depth / LiDAR submap alignment) plus Huber, SoftLOne, Arctan and Tolerant, and Ceres' Corrector with
both of its branches (rho'' <= 0: sqrt(rho') scaling; rho'' > 0: the second-order alpha correction;
okvis restates it at TwoPoseGraphError.cpp:292-337).

Parity of the loss functions themselves is unpinned by reference vectors (Ceres is an un-vendored
submodule): they are pinned here by their closed forms (an independent numpy
restatement of the published definitions), by numeric differentiation (rho' and rho''), and the
Corrector by its defining identities J_c^T r_c = rho' J^T r and J_c^T J_c = J^T (rho' I + 2 rho''
r r^T) J (alpha branch) / rho' J^T J (first-order branch).

CPU: the library's okvisgpu_loss_evaluate (what the runtime's host-factor path applies) against the
oracle's restatement and the closed forms; the oracle's Corrector identities; the oracle's solve
cost against the raw factors. GPU: S10 + Cauchy(3) / Tolerant GPS factors + Tukey(2.0) / Tukey(0.1)
submap-shaped two-pose factors, initial cost and full solves against the oracle."""
import numpy as np
import pytest

import okvisgpu as og
import _oracle
from _gps import gps_window
from _submap import loss_window

N_KF = 10

# (kind, a, b), closed form rho(s) of the published definition
LOSSES = [
    ("cauchy", 1.0, 0.0, lambda s, a, b: a * a * np.log1p(s / (a * a))),
    ("cauchy", 3.0, 0.0, lambda s, a, b: a * a * np.log1p(s / (a * a))),
    ("tukey", 0.1, 0.0, lambda s, a, b: a * a / 3 * (1 - (1 - s / (a * a)) ** 3) if s <= a * a else a * a / 3),
    ("tukey", 2.0, 0.0, lambda s, a, b: a * a / 3 * (1 - (1 - s / (a * a)) ** 3) if s <= a * a else a * a / 3),
    ("huber", 1.5, 0.0, lambda s, a, b: s if s <= a * a else 2 * a * np.sqrt(s) - a * a),
    ("softlone", 0.7, 0.0, lambda s, a, b: 2 * a * a * (np.sqrt(1 + s / (a * a)) - 1)),
    ("arctan", 2.0, 0.0, lambda s, a, b: a * np.arctan2(s, a)),
    ("tolerant", 4.0, 1.0, lambda s, a, b: b * np.log1p(np.exp((s - a) / b)) - b * np.log1p(np.exp(-a / b))),
]
S_GRID = [0.0, 1e-4, 0.003, 0.2, 0.9, 2.0, 3.9, 4.0, 4.1, 8.5, 30.0, 200.0]


@pytest.mark.parametrize("kind,a,b,rho_ref", LOSSES, ids=[f"{k}{a}" for k, a, _, _ in LOSSES])
def test_loss_closed_form_and_derivatives(og, kind, a, b, rho_ref):
    """rho from the library and from the oracle agree (1e-14 relative, 1e-15 a^2 absolute: the two
    compilers contract products into FMAs differently, and Tukey's 1 - v^3 cancels), match the
    published closed form, and rho', rho'' match central differences of rho (away from kinks)."""
    for s in S_GRID:
        lib = np.array(og.loss_evaluate(kind, a, b, s))
        orc = np.array(_oracle.loss_evaluate(kind, a, b, s))
        assert np.allclose(lib, orc, rtol=1e-14, atol=1e-15 * max(1.0, a * a)), (kind, a, s, lib, orc)
        assert abs(lib[0] - rho_ref(s, a, b)) <= 1e-13 * max(1.0, abs(lib[0])), (kind, a, s, lib[0])
        kink = kind in ("tukey", "huber") and abs(s - a * a) < 1e-3
        if s < 1e-3 or kink:
            continue
        h = 1e-6 * max(1.0, s)
        up, dn = og.loss_evaluate(kind, a, b, s + h), og.loss_evaluate(kind, a, b, s - h)
        assert abs((up[0] - dn[0]) / (2 * h) - lib[1]) <= 1e-6 * max(1.0, abs(lib[1])), (kind, a, s)
        assert abs((up[1] - dn[1]) / (2 * h) - lib[2]) <= 1e-5 * max(1.0, abs(lib[2])), (kind, a, s)
    assert og.loss_evaluate("none", 1.0, 0.0, 2.5) == (2.5, 1.0, 0.0)


def test_loss_invalid_scale_rejected(og):
    for kind, a, b in (("cauchy", 0.0, 0.0), ("tukey", -2.0, 0.0), ("tolerant", 1.0, 0.0), (42, 1.0, 0.0)):
        with pytest.raises(og.OkvisGpuError):
            og.loss_evaluate(kind, a, b, 1.0)


@pytest.mark.parametrize("kind,a,b", [("cauchy", 3.0, 0.0), ("tukey", 2.0, 0.0), ("tolerant", 4.0, 1.0),
                                      ("tolerant", 0.5, 2.0), ("huber", 0.5, 0.0)])
def test_oracle_corrector_identities(og, kind, a, b):
    """The oracle's Corrector reproduces the robustified gradient rho' J^T r and Gauss-Newton Hessian
    J^T (rho' I + 2 rho'' r r^T) J for the second-order branch (rho'' > 0: Tolerant), rho' J^T J
    for the first-order one, and cost rho(s)/2."""
    import ctypes as C
    rng = np.random.default_rng(3)
    L = og.Loss(og.LOSS_KINDS[kind], 0, a, b)
    for nres, scale in ((1, 0.6), (3, 1.1), (6, 0.4), (15, 0.35)):
        r = rng.normal(0.0, scale, nres)
        J = rng.normal(size=(nres, 12))
        rc, Jc, cost = r.copy(), J.copy(), C.c_double()
        assert _oracle.lib().oracle_loss_correct(C.byref(L), nres, 12, og.dptr(rc), og.dptr(Jc), C.byref(cost)) == 0
        s = float(r @ r)
        rho = og.loss_evaluate(kind, a, b, s)
        assert abs(cost.value - 0.5 * rho[0]) <= 1e-15 * max(1.0, abs(rho[0]))
        if rho[1] == 0.0:  # Tukey outlier region: no gradient, no curvature
            assert np.all(Jc == 0.0) and np.all(rc == 0.0)
            continue
        g = Jc.T @ rc
        assert np.allclose(g, rho[1] * (J.T @ r), rtol=1e-12, atol=1e-13)
        H = Jc.T @ Jc
        Href = rho[1] * (J.T @ J) + (2.0 * rho[2] * np.outer(J.T @ r, J.T @ r) if rho[2] > 0 else 0.0)
        assert np.allclose(H, Href, rtol=1e-11, atol=1e-11 * np.abs(Href).max()), (kind, nres)


def test_oracle_host_losses_cost(og):
    """The oracle's cost of a window with per-factor losses = the raw window's cost with each host
    factor's 1/2 |r|^2 replaced by 1/2 rho(|r|^2) of its own loss."""
    P, gps, sub = loss_window()
    cost = _oracle.evaluate(P.ptr())
    losses = P.host_loss.copy()
    P.host_loss = og.loss_array([("none",)] * len(losses))
    P.bind()
    raw = _oracle.evaluate(P.ptr())
    expect = 0.0
    n_gps = N_KF
    for h, Lh in enumerate(losses):
        if h < n_gps:
            r, _ = gps.evaluate(h, [P.poses[h], P.speed_biases[h], P.poses[N_KF]])
        else:
            i = h - n_gps
            a, b = sub.pairs[i]
            r = np.array([sub.residual(i, P.poses[a], P.poses[b])])
        s = float(r @ r)
        rho = og.loss_evaluate(int(Lh["kind"]), float(Lh["a"]), float(Lh["b"]), s)
        expect += 0.5 * rho[0] - 0.5 * s
    assert abs((cost - raw) - expect) <= 1e-9 * abs(raw)


def test_oracle_loss_window_solve(og):
    """The window with Cauchy(3) / Tolerant GPS factors and Tukey submap factors solves: the cost
    drops and the gross GPS outliers do not drag the alignment (its translation error shrinks)."""
    P, gps, _ = loss_window()
    s = _oracle.solve(P.ptr(), og.default_options(max_num_iterations=15, num_threads=2))
    assert s["termination"] != "FAILURE" and s["final_cost"] < 0.5 * s["initial_cost"], s


def test_host_loss_overrides_host_cauchy(og):
    """host_loss (ABI 6) takes precedence over host_cauchy; NULL keeps the ABI-5 meaning."""
    P, _, _ = gps_window()
    P.host_cauchy[:] = 1
    P.bind()
    c_cauchy = _oracle.evaluate(P.ptr())
    P.host_loss = og.loss_array([("cauchy", 1.0)] * N_KF)
    P.bind()
    assert _oracle.evaluate(P.ptr()) == c_cauchy
    P.host_loss = og.loss_array([("none",)] * N_KF)
    P.bind()
    assert _oracle.evaluate(P.ptr()) != c_cauchy


# ------------------------------------------------------------------------------------------ GPU
def _solve_both(P, options):
    snap = P.snapshot()
    ctx = og.Context(0)
    try:
        ctx.set_problems([P.struct])
        g = ctx.solve(options)[0]
    finally:
        ctx.close()
    gpu = P.poses.copy()
    P.restore(snap)
    c = _oracle.solve(P.ptr(), options)
    return g, c, gpu, P.poses.copy()


@pytest.mark.gpu
def test_gpu_host_losses_initial_cost(og, parity):
    """okvisgpu_evaluate of a window whose host factors carry every loss of the family equals the
    oracle's (host path: gather -> callback -> Corrector -> upload)."""
    specs = [("cauchy", 3.0), ("tukey", 2.0), ("tukey", 0.1), ("huber", 0.5), ("softlone", 0.7),
             ("arctan", 2.0), ("tolerant", 4.0, 1.0)]
    P, _, sub = loss_window()
    P.host_loss = og.loss_array([specs[h % len(specs)] for h in range(len(P.host_dim))])
    P.bind()
    c_ref = _oracle.evaluate(P.ptr())
    ctx = og.Context(0)
    try:
        ctx.set_problems([P.struct])
        c_gpu = ctx.evaluate(0)
    finally:
        ctx.close()
    parity("host losses (7 kinds): initial cost (rel)", abs(c_gpu - c_ref) / c_ref, 1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("tolerant_every", [0, 4], ids=["cauchy3_tukey", "with_tolerant"])
def test_gpu_loss_window_solve_parity(og, parity, tolerant_every):
    """S10 + GPS factors under CauchyLoss(3.0) (ViGraph.cpp:999; with every 4th under TolerantLoss,
    the Corrector's alpha branch) + submap-shaped two-pose factors under TukeyLoss(2.0) / (0.1)
    (ViGraph.cpp:1510,1513): iterations, termination and steps exact, cost 1e-7, poses 1e-6 m."""
    P, _, _ = loss_window(tolerant_every=tolerant_every)
    o = og.default_options(max_num_iterations=12, num_threads=2)
    g, c, xg, xc = _solve_both(P, o)
    assert (g["num_iterations"], g["termination"], g["num_successful_steps"], g["num_unsuccessful_steps"]) == \
        (c["num_iterations"], c["termination"], c["num_successful_steps"], c["num_unsuccessful_steps"]), (g, c)
    tag = "Cauchy(3) GPS + Tukey submap" + (" + Tolerant GPS" if tolerant_every else "")
    parity(f"losses, {tag}: final cost (rel)", abs(g["final_cost"] - c["final_cost"]) / c["final_cost"], 1e-7)
    parity(f"losses, {tag}: positions (m)", float(np.abs(xg[:, :3] - xc[:, :3]).max()), 1e-6)
    assert g["final_cost"] < 0.5 * g["initial_cost"]
