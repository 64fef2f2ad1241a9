"""The CPU oracle's pose-graph edge (TwoPoseStandardGraphError, TwoPoseGraphError.cpp:162-767)
against properties the reference's math implies (the reference ships no fixtures for it and has no
unit test of TwoPoseStandardGraphError itself; TestPoseGraphError.cpp covers the older
PoseGraphError class):
  * analytic-vs-numeric Jacobians with jacobiansCorrect semantics (ErrorInterface.cpp:44-163);
  * compute() marginalises exactly the landmarks of the edge: with the reference keyframe at the
    origin and every landmark block full rank, H00_ equals the Schur complement of the full
    reprojection problem (reference pose constant) and -b0_ its reduced gradient, both taken from
    the oracle's own DENSE_SCHUR reduction (itself cross-checked by an independent numpy
    restatement in test_oracle_solver.py);
  * J_^T J_ = H00_ and J_^T J_ DeltaX_ = -b0_ (the eigen-decomposition of :376-385);
  * the |r| > 3 outlier rule and the rank < 3 / depth < 2.99 landmark rule.
"""
import numpy as np
import pytest

import okvisgpu as og
import _twopose as tp


def _relpose_window(n_relpose=6, stride=3, seed=20251015, kind=0):
    return og.SynthWindow(8, 200, 1600, seed=seed, n_relpose=n_relpose, relpose_stride=stride, relpose_kind=kind)


@pytest.mark.parametrize("kind", [0, 1])
def test_relpose_jacobians(oracle, kind):
    """kind 0: TwoPoseStandardGraphError(Const); kind 1: RelativePoseError (RelativePoseError.cpp)."""
    w = _relpose_window(kind=kind)
    for i in range(w.problem.n_relpose):
        assert oracle.check_jacobians(w.problem_ptr(), 4, i) < 1e-6


def test_relative_pose_error_at_measurement(oracle):
    """RelativePoseError is zero with the measured T_AB, and its residual is L times the
    [translation; 2 vec(dq)] error (RelativePoseError.cpp:70-86)."""
    w = _relpose_window(kind=1, n_relpose=4)
    p = w.problem
    P = w.poses()
    blocks = np.ctypeslib.as_array(p.relpose_blocks, (p.n_relpose, 2))
    lin = np.ctypeslib.as_array(p.relpose_lin_point, (p.n_relpose, 7))
    for i in range(p.n_relpose):
        a, b = blocks[i]
        # place pose b exactly at T_WA * T_AB_meas
        Ra = tp.rot(P[a, 3:])
        P[b, :3] = P[a, :3] + Ra @ lin[i, :3]
        x0, y0, z0, w0 = P[a, 3:] / np.linalg.norm(P[a, 3:])
        x1, y1, z1, w1 = lin[i, 3:]
        P[b, 3:] = [w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1, w0 * y1 + y0 * w1 + z0 * x1 - x0 * z1,
                    w0 * z1 + z0 * w1 + x0 * y1 - y0 * x1, w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1]
        r, _ = oracle.eval_relpose(w.problem_ptr(), p.n_relpose)
        assert np.abs(r[i]).max() < 1e-9


def test_relpose_jacobians_rotated_reference(oracle):
    """Jacobians at a point away from the linearisation point (perturbed poses)."""
    w = _relpose_window(seed=7)
    P = w.poses()
    rng = np.random.default_rng(3)
    for k in range(P.shape[0]):
        P[k, :3] += rng.normal(0, 0.2, 3)
        q = tp.quat_from_axis_angle(rng.normal(0, 0.1, 3))
        x0, y0, z0, w0 = q
        x1, y1, z1, w1 = P[k, 3:]
        P[k, 3:] = [w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1, w0 * y1 + y0 * w1 + z0 * x1 - x0 * z1,
                    w0 * z1 + z0 * w1 + x0 * y1 - y0 * x1, w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1]
    for i in range(w.problem.n_relpose):
        assert oracle.check_jacobians(w.problem_ptr(), 4, i) < 1e-6


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_compute_is_schur_complement(oracle, seed):
    edge, cams, ex = tp.scene(oracle, seed, n_lm=40)
    out = oracle.twopose_compute(og.TwoPoseBatch([edge], cams, ex))
    sp = tp.SceneProblem(edge, cams, ex)
    r, _, _ = oracle.eval_reprojection(sp.ptr(), sp.problem.n_observations)
    assert np.linalg.norm(r, axis=1).max() < 3.0  # no |r| > 3 outlier: compute() keeps every observation
    S, rhs, _, rc = oracle.linearize_reduce(sp.ptr(), jacobi_scaling=False, mu=0.0)
    assert rc == 0 and S.shape == (6, 6)
    H00, b0 = out["H00"][0], out["b0"][0]
    assert np.abs(H00 - S).max() <= 1e-9 * np.abs(S).max()
    assert np.abs(-b0 - rhs).max() <= 1e-9 * np.abs(rhs).max()
    J, dx = out["sqrt_info"][0], out["delta_x"][0]
    assert np.abs(J.T @ J - H00).max() <= 1e-9 * np.abs(H00).max()
    assert np.abs(J.T @ J @ dx + b0).max() <= 1e-8 * np.abs(b0).max()
    # linearisation point = T_S0S1 (reference at the origin: the other pose itself)
    assert np.allclose(out["lin_point"][0], edge["other_pose"], atol=1e-15)


def test_compute_reference_frame_invariance(oracle):
    """Moving the whole scene by a rigid transform leaves the relative system unchanged."""
    e0, cams, ex = tp.scene(oracle, 5, n_lm=30)
    T = np.r_[[3.0, -2.0, 0.5], tp.quat_from_axis_angle(np.array([0.2, -0.4, 1.1]))]
    R = tp.rot(T[3:])

    def move(P):
        x0, y0, z0, w0 = T[3:]
        x1, y1, z1, w1 = P[3:]
        q = [w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1, w0 * y1 + y0 * w1 + z0 * x1 - x0 * z1,
             w0 * z1 + z0 * w1 + x0 * y1 - y0 * x1, w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1]
        return np.r_[R @ P[:3] + T[:3], q]

    e1 = dict(e0)
    e1["ref_pose"], e1["other_pose"] = move(e0["ref_pose"]), move(e0["other_pose"])
    e1["landmarks"] = np.array([np.r_[R @ l[:3] + T[:3] * l[3], l[3]] for l in e0["landmarks"]])
    a = oracle.twopose_compute(og.TwoPoseBatch([e0], cams, ex))
    b = oracle.twopose_compute(og.TwoPoseBatch([e1], cams, ex))
    for k in ("H00", "b0", "delta_x", "lin_point"):
        assert np.abs(a[k] - b[k]).max() <= 1e-8 * max(1.0, np.abs(a[k]).max()), k


def test_compute_outliers_and_rank_rules(oracle):
    base, cams, ex = tp.scene(oracle, 11, n_lm=25)
    out_base = oracle.twopose_compute(og.TwoPoseBatch([base], cams, ex))
    # near single-camera landmarks (rank 2, depth < 2.99) are skipped entirely
    near, _, _ = tp.scene(oracle, 11, n_lm=25, mono_near=3)
    out_near = oracle.twopose_compute(og.TwoPoseBatch([near], cams, ex))
    assert np.abs(out_near["H00"] - out_base["H00"]).max() == 0.0
    assert np.abs(out_near["b0"] - out_base["b0"]).max() == 0.0
    # far single-camera landmarks are kept: reference-only observations add nothing to H00 but the
    # clamped pseudo-inverse (1/tol) is used for the null direction, and nothing breaks
    far, _, _ = tp.scene(oracle, 11, n_lm=25, mono_far=3)
    out_far = oracle.twopose_compute(og.TwoPoseBatch([far], cams, ex))
    assert np.all(np.isfinite(out_far["H00"])) and np.all(np.isfinite(out_far["delta_x"]))
    assert np.abs(out_far["H00"] - out_base["H00"]).max() <= 1e-9 * np.abs(out_base["H00"]).max()
    # |r| > 3 outliers are dropped: the same scene without them matches the Schur complement of the
    # problem with those observations removed
    outl, _, _ = tp.scene(oracle, 13, n_lm=25, outliers=4)
    o = oracle.twopose_compute(og.TwoPoseBatch([outl], cams, ex))
    clean = dict(outl)
    clean["observations"] = [[ob for ob in obs if not (ob[0] and ob[1] == 0 and li < 4)]
                             for li, obs in enumerate(outl["observations"])]
    c = oracle.twopose_compute(og.TwoPoseBatch([clean], cams, ex))
    assert np.abs(o["H00"] - c["H00"]).max() <= 1e-12 * np.abs(c["H00"]).max()


def test_compute_without_other_observations(oracle):
    """No observation from the other keyframe: H00_ = 0, J_ = 0, DeltaX_ = 0 and the
    linearisation point stays the identity (relPoseSet false, :267-270)."""
    edge, cams, ex = tp.scene(oracle, 17, n_lm=10, no_other=True)
    out = oracle.twopose_compute(og.TwoPoseBatch([edge], cams, ex))
    assert np.abs(out["H00"]).max() == 0.0
    assert np.abs(out["sqrt_info"]).max() == 0.0 and np.abs(out["delta_x"]).max() == 0.0
    assert np.array_equal(out["lin_point"][0], [0, 0, 0, 0, 0, 0, 1])


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_oracle_solve_with_relpose_edges(oracle, kind):
    w = _relpose_window(n_relpose=5, stride=4, kind=kind)
    opts = og.default_options(max_num_iterations=10)
    c0 = oracle.evaluate(w.problem_ptr())
    s = oracle.solve(w.problem_ptr(), opts)
    assert s["final_cost"] < c0
    assert s["termination"] in ("CONVERGENCE", "NO_CONVERGENCE")
