"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Tolerances (FP64 on both sides; different but equivalent operation orders). Every test records
the deviation it measured (conftest `parity`; OKVISGPU_PARITY_REPORT writes them, the round's copy
is profiles/r03_parity.json):
  * reprojection residuals / minimal Jacobians: 1e-12 relative to the block norm (fused GPU
    formula vs the reference's 4x4-matrix chain; measured 1e-15);
  * IMU factor: only basis-invariant quantities (J^T J, J^T r, cost) are compared, because the
    pseudo-inverse square root's eigenvector basis is arbitrary; 1e-12 relative
    (measured 3e-15);
  * reduced camera system S / rhs: 1e-11 relative to max|S| (landmark elimination sums in another
    order, Jacobi scaling applied to blocks instead of to J columns; measured 1.2e-13);
  * full solves: final cost 1e-7 relative, poses within 1e-6 m / 1e-6 rad (the parity contract of
    SURVEY.md §8c).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _window(og, kf=10, lm=500, obs=4000, seed=20251015):
    return og.SynthWindow(kf, lm, obs, seed=seed)


def _block_rel(a, b, n):
    """max over observations of |a - b| / |b| (Frobenius norms of the per-observation blocks)."""
    err = np.linalg.norm((a - b).reshape(n, -1), axis=1)
    ref = np.linalg.norm(b.reshape(n, -1), axis=1)
    return float(np.max(err / np.maximum(ref, 1e-300)))


def _reprojection_parity(gpu_ctx, oracle, w, parity, tag):
    n = w.problem.n_observations
    gpu_ctx.set_problems([w.problem])
    r, Jp, Jl = gpu_ctx.eval_reprojection(n)
    r0, Jp0, Jl0 = oracle.eval_reprojection(w.problem_ptr(), n)
    parity(f"{tag} reprojection r (max abs / max |r|)", np.abs(r - r0).max() / np.abs(r0).max(), R_TOL)
    parity(f"{tag} reprojection J_pose (block rel)", _block_rel(Jp, Jp0, n), J_TOL)
    parity(f"{tag} reprojection J_landmark (block rel)", _block_rel(Jl, Jl0, n), J_TOL)


# reprojection functor bounds: the GPU forms r and J from a fused chain (C_CW, L Jh, no 4x4
# matrices) where the reference multiplies the 4x4 transformation chain; both FP64. Measured on
# MI355X (profiles/r03_parity.json): r 8e-15, J 1e-15 relative -- the bound keeps ~100x headroom.
R_TOL = 1e-12
J_TOL = 1e-12


def test_reprojection_functor_parity(og, oracle, gpu_ctx, parity):
    _reprojection_parity(gpu_ctx, oracle, _window(og), parity, "radtan")


EQUIDISTANT_TEST = (-0.0041, 0.0063, -0.0067, 0.0023)
# RadialTangentialDistortion8::testObject (RadialTangentialDistortion8.hpp:94-95): k1 k2 p1 p2 k3 k4 k5 k6
RADTAN8_TEST = (0.6261, 0.001, -0.0002, 0.0001, 0.0001, 0.9541, 0.1151, -0.0075)
CAMERA_MODELS = {"none": (0, ()), "equidistant": (2, EQUIDISTANT_TEST), "radtan8": (3, RADTAN8_TEST)}


def _switch_camera_model(oracle, w, kind, params):
    """Gives every camera of a synthetic (radtan) window another distortion model and moves each
    measured keypoint so that its weighted residual at the initial estimate is unchanged: the same
    noise and initial error, now consistent with the new model."""
    p = w.problem
    n = p.n_observations
    r_old, _, _ = oracle.eval_reprojection(w.problem_ptr(), n)
    for c in range(p.n_cameras):
        cam = p.cameras[c]
        cam.distortion = kind
        for i in range(8):
            cam.dist[i] = params[i] if i < len(params) else 0.0
    r_new, _, _ = oracle.eval_reprojection(w.problem_ptr(), n)
    kp = np.ctypeslib.as_array(p.obs_keypoint, shape=(n, 2))
    L = np.ctypeslib.as_array(p.obs_sqrt_info, shape=(n, 2, 2))
    kp -= np.linalg.solve(L, (r_new - r_old)[..., None])[..., 0]


@pytest.mark.parametrize("distortion", sorted(CAMERA_MODELS))
def test_distortion_models_parity(og, oracle, gpu_ctx, distortion, parity):
    """The other camera models of PinholeCamera<D> (NoDistortion, EquidistantDistortion.hpp:87-188,
    RadialTangentialDistortion8.hpp:88-170): functor outputs and a short full solve against the
    oracle."""
    w = _window(og, seed=27)
    assert og.DIST_EQUIDISTANT == 2 and og.DIST_RADTAN8 == 3
    _switch_camera_model(oracle, w, *CAMERA_MODELS[distortion])
    p = w.problem
    _reprojection_parity(gpu_ctx, oracle, w, parity, distortion)
    opts = og.default_options(max_num_iterations=4, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    sg = gpu_ctx.solve(opts, 1)[0]
    P = w.poses().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    assert sg["num_iterations"] == so["num_iterations"]
    parity(f"{distortion} 4-iteration solve final cost (rel)", abs(sg["final_cost"] - so["final_cost"]) / so["final_cost"], 1e-6)
    parity(f"{distortion} 4-iteration solve poses (m)", np.abs(P[:, :3] - w.poses()[:, :3]).max(), 1e-6)


def test_anisotropic_information_parity(og, oracle, gpu_ctx, parity):
    """Reprojection square-root information other than diag(s, s): the general 2x2 read of
    k_eval_obs (okvis' keypoint-size information is isotropic, and such batches read s alone,
    runtime.cpp obs_iso). Functor outputs and a short solve against the oracle."""
    w = _window(og, seed=31)
    p = w.problem
    n = p.n_observations
    L = np.ctypeslib.as_array(p.obs_sqrt_info, shape=(n, 2, 2))
    rng = np.random.default_rng(5)
    L[:, 1, 0] = 0.1 * L[:, 0, 0] * rng.standard_normal(n)  # sheared, lower triangular
    L[:, 1, 1] *= 1.0 + 0.2 * rng.random(n)
    _reprojection_parity(gpu_ctx, oracle, w, parity, "anisotropic")
    opts = og.default_options(max_num_iterations=4, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    sg = gpu_ctx.solve(opts, 1)[0]
    P = w.poses().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    assert sg["num_iterations"] == so["num_iterations"]
    parity("anisotropic 4-iteration solve final cost (rel)", abs(sg["final_cost"] - so["final_cost"]) / so["final_cost"], 1e-7)
    parity("anisotropic 4-iteration solve poses (m)", np.abs(P[:, :3] - w.poses()[:, :3]).max(), 1e-6)


def test_imu_functor_invariants(og, oracle, gpu_ctx, parity):
    w = _window(og)
    p = w.problem
    gpu_ctx.set_problems([w.problem])
    r, J = gpu_ctx.eval_imu(p.n_imu)
    w.reset()
    r0, J0 = oracle.eval_imu(w.problem_ptr(), p.n_imu)
    eH = eg = ec = 0.0
    for f in range(p.n_imu):
        H, H0 = J[f].T @ J[f], J0[f].T @ J0[f]
        g, g0 = J[f].T @ r[f], J0[f].T @ r0[f]
        eH = max(eH, np.linalg.norm(H - H0) / np.linalg.norm(H0))
        eg = max(eg, np.linalg.norm(g - g0) / (np.linalg.norm(g0) + 1e-300))
        ec = max(ec, abs(r[f] @ r[f] - r0[f] @ r0[f]) / (r0[f] @ r0[f]))
    tag = "imu"
    parity(f"{tag} J^T J (Frobenius rel)", eH, 1e-12)
    parity(f"{tag} J^T r (rel)", eg, 1e-12)
    parity(f"{tag} |r|^2 (rel)", ec, 1e-12)


def test_imu_functor_pseudo_inverse(og, oracle, gpu_ctx, parity):
    """Zero bias random-walk densities make the preintegrated covariance singular, so the
    square-root information takes the clamped eigen-decomposition branch of
    PseudoInverse::symmSqrtU (PseudoInverse.hpp:132-158) instead of the Cholesky shortcut."""
    w = _window(og)
    p = w.problem
    p.imu_params.sigma_gw_c = 0.0
    p.imu_params.sigma_aw_c = 0.0
    gpu_ctx.set_problems([p])
    r, J = gpu_ctx.eval_imu(p.n_imu)
    w.reset()
    r0, J0 = oracle.eval_imu(w.problem_ptr(), p.n_imu)
    eH = eg = ec = 0.0
    for f in range(p.n_imu):
        H, H0 = J[f].T @ J[f], J0[f].T @ J0[f]
        g, g0 = J[f].T @ r[f], J0[f].T @ r0[f]
        eH = max(eH, np.linalg.norm(H - H0) / np.linalg.norm(H0))
        eg = max(eg, np.linalg.norm(g - g0) / (np.linalg.norm(g0) + 1e-300))
        ec = max(ec, abs(r[f] @ r[f] - r0[f] @ r0[f]) / (r0[f] @ r0[f]))
    tag = "imu pseudo-inverse branch"
    parity(f"{tag} J^T J (Frobenius rel)", eH, 1e-12)
    parity(f"{tag} J^T r (rel)", eg, 1e-12)
    parity(f"{tag} |r|^2 (rel)", ec, 1e-12)


@pytest.mark.parametrize("mu", [0.0, 1e-8, 1e-2])
def test_linearize_reduce_parity(og, oracle, gpu_ctx, mu, parity):
    w = _window(og)
    gpu_ctx.set_problems([w.problem])
    S, rhs, cost = gpu_ctx.linearize_reduce(0, True, mu)
    w.reset()
    S0, rhs0, cost0, rc = oracle.linearize_reduce(w.problem_ptr(), True, mu)
    assert rc == 0
    assert S.shape == S0.shape
    parity("S10 initial cost (rel)", abs(cost - cost0) / cost0, 1e-12)
    parity(f"S10 reduced system S, mu={mu} (max abs / max |S|)", np.abs(S - S0).max() / np.abs(S0).max(), 1e-11)
    parity(f"S10 reduced rhs, mu={mu} (max abs / max |rhs|)", np.abs(rhs - rhs0).max() / np.abs(rhs0).max(), 1e-11)


def _rot_err(q, q0):
    # 2 |vec(q * q0^-1)|
    x1, y1, z1, w1 = q
    x0, y0, z0, w0 = -q0[0], -q0[1], -q0[2], q0[3]
    v = np.array([w1 * x0 + x1 * w0 + y1 * z0 - z1 * y0,
                  w1 * y0 + y1 * w0 + z1 * x0 - x1 * z0,
                  w1 * z0 + z1 * w0 + x1 * y0 - y1 * x0])
    return 2 * np.linalg.norm(v)


@pytest.mark.parametrize("iters", [1, 3, 10])
def test_solve_parity_s10(og, oracle, gpu_ctx, iters, parity):
    w = _window(og)
    opts = og.default_options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(opts, 1)[0]
    P, L = w.poses().copy(), w.landmarks().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    P0, L0 = w.poses().copy(), w.landmarks().copy()
    assert sg["num_iterations"] == so["num_iterations"]
    assert sg["num_successful_steps"] == so["num_successful_steps"]
    assert abs(sg["initial_cost"] - so["initial_cost"]) <= 1e-10 * so["initial_cost"]
    # One GN step from a far initial point amplifies rounding by the reduced system's condition
    # number (~1e8): 1e-7 relative after the first step; later iterations contract towards the same
    # optimum and the 3- and 10-iteration cases also hold this bound.
    parity(f"S10 {iters}-iteration solve final cost (rel)", abs(sg["final_cost"] - so["final_cost"]) / so["final_cost"], 1e-7)
    parity(f"S10 {iters}-iteration solve positions (m)", np.abs(P[:, :3] - P0[:, :3]).max(), 1e-6)
    parity(f"S10 {iters}-iteration solve rotations (rad)", max(_rot_err(P[i, 3:], P0[i, 3:]) for i in range(len(P))), 1e-6)
    parity(f"S10 {iters}-iteration solve landmarks (m)", np.abs(L[:, :3] / L[:, 3:] - L0[:, :3] / L0[:, 3:]).max(), 1e-3)


def test_batched_windows_match_single(og, gpu_ctx):
    ws = [_window(og, seed=s) for s in (1, 2, 3)]
    opts = og.default_options(max_num_iterations=5)
    gpu_ctx.set_problems([w.problem for w in ws])
    sb = gpu_ctx.solve(opts, 3)
    Pb = [w.poses().copy() for w in ws]
    for k, w in enumerate(ws):
        w.reset()
        gpu_ctx.set_problems([w.problem])
        s1 = gpu_ctx.solve(opts, 1)[0]
        assert s1["final_cost"] == sb[k]["final_cost"]
        assert np.array_equal(w.poses(), Pb[k])


@pytest.mark.parametrize("n_batch", [100, 300])
def test_window_alone_vs_large_batch(og, gpu_ctx, parity, n_batch):
    """A window's operation order depends on the batch only through the batch size against the
    device's CU count (runtime.cpp: the nested-dissection state order below one window per CU;
    device_problem.hpp fewWindows: 1,024-thread per-window reductions and fused launches at or
    below a quarter window per CU). On MI355X (256 CUs) a window alone runs with both, in a batch of
    100 with the order but not the reductions, in a batch of 300 with neither. Bitwise equality
    holds inside one regime (test_batched_windows_match_single); across regimes the solves agree to
    rounding: same iterations, termination and successful steps, cost and poses to the solve
    tolerances."""
    seeds = [900 + k for k in range(n_batch)]
    ws = [_window(og, seed=s) for s in seeds]
    opts = og.default_options(max_num_iterations=5)
    gpu_ctx.set_problems([w.problem for w in ws])
    sb = gpu_ctx.solve(opts, n_batch)
    picks = (0, n_batch // 2, n_batch - 1)
    Pb = {k: ws[k].poses().copy() for k in picks}
    for k in picks:
        w = ws[k]
        w.reset()
        gpu_ctx.set_problems([w.problem])
        s1 = gpu_ctx.solve(opts, 1)[0]
        for f in ("num_iterations", "termination_type", "num_successful_steps"):
            assert s1[f] == sb[k][f], (f, k)
        parity(f"window alone vs in a batch of {n_batch}: cost (rel)",
               abs(s1["final_cost"] - sb[k]["final_cost"]) / sb[k]["final_cost"], 1e-9)
        parity(f"window alone vs in a batch of {n_batch}: positions (m)",
               float(np.abs(w.poses()[:, :3] - Pb[k][:, :3]).max()), 1e-8)


@pytest.mark.parametrize("n_batch", [1, 8, 80, 300], ids=["alone", "batch8", "batch80", "batch300"])
def test_gradient_tolerance_termination(og, oracle, gpu_ctx, parity, n_batch):
    """The gradient test ends the solve at the oracle's iteration (TrustRegionMinimizer: max-norm of
    x - Plus(x, -g) <= gradient_tolerance after an accepted step). Alone and in a batch of 8 (a
    quarter window per CU or less) the test runs inside the next iteration's assembly launch with one
    standalone test closing each captured graph; in a batch of 80 (one-stream graph) it is its own
    launch after the
    linearisation; in a batch of 300 (the forked graph: more windows than CUs on MI355X) likewise,
    after k_fgrad on the main stream. The tolerance is picked so that the
    oracle converges by it after 5 to 20 iterations (three tolerances, so that the last iteration
    falls at different places of the four-iteration graphs); iterations, termination, steps exact,
    cost 1e-7."""
    w = _window(og, seed=61)
    base = dict(max_num_iterations=25, function_tolerance=0.0, parameter_tolerance=0.0)
    picks = []
    for g in (3e3, 1e3, 3e2, 1e2, 3e1, 1e1, 3.0, 1.0, 0.3, 0.1, 3e-2, 1e-2, 3e-3, 1e-3, 1e-4, 1e-5, 1e-6):
        w.reset()
        so = oracle.solve(w.problem_ptr(), og.default_options(gradient_tolerance=g, **base))
        if so["termination"] == "CONVERGENCE" and 5 <= so["num_iterations"] <= 20:
            picks.append((g, so))
        if len(picks) == 3:
            break
    assert picks, "no gradient tolerance ends the oracle's solve by its gradient test"
    others = [_window(og, seed=700 + k) for k in range(n_batch - 1)]
    for g, so in picks:
        w.reset()
        for o in others:
            o.reset()
        gpu_ctx.set_problems([w.problem] + [o.problem for o in others])
        sg = gpu_ctx.solve(og.default_options(gradient_tolerance=g, **base), n_batch)[0]
        for f in ("num_iterations", "termination", "num_successful_steps", "num_unsuccessful_steps"):
            assert sg[f] == so[f], (f, g, sg, so)
        parity(f"gradient-tolerance {g:g} termination ({'alone' if n_batch == 1 else f'batch of {n_batch}'}): final cost (rel)",
               abs(sg["final_cost"] - so["final_cost"]) / so["final_cost"], 1e-7)


def test_solve_is_deterministic(og, gpu_ctx):
    w = _window(og)
    opts = og.default_options(max_num_iterations=5)
    gpu_ctx.set_problems([w.problem])
    a = gpu_ctx.solve(opts, 1)[0]
    Pa = w.poses().copy()
    w.reset()
    gpu_ctx.update_params()
    b = gpu_ctx.solve(opts, 1)[0]
    assert a["final_cost"] == b["final_cost"]
    assert np.array_equal(Pa, w.poses())


def test_forked_and_serial_graphs_agree(og, gpu_ctx, monkeypatch):
    """The captured iteration with fork streams (batches of at least one window per CU) and the
    single-stream one (fewer windows; runtime.cpp ensureGraph) run the same kernels on disjoint
    data in a fixed order per buffer: bitwise-equal solves, also with mu retries (GN prep)."""
    ws = [_window(og, seed=s) for s in (41, 42, 43)]
    opts = og.default_options(max_num_iterations=6, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    res = []
    for ser in ("0", "1"):
        monkeypatch.setenv("OKVISGPU_SERIAL_GRAPH", ser)
        for w in ws:
            w.reset()
        gpu_ctx.set_problems([w.problem for w in ws])  # drops the captured graph
        s = gpu_ctx.solve(opts, len(ws))
        res.append((s, [w.poses().copy() for w in ws], [w.landmarks().copy() for w in ws]))
    for k in range(len(ws)):
        assert res[0][0][k]["final_cost"] == res[1][0][k]["final_cost"]
        assert res[0][0][k]["num_iterations"] == res[1][0][k]["num_iterations"] == 6
        assert np.array_equal(res[0][1][k], res[1][1][k])
        assert np.array_equal(res[0][2][k], res[1][2][k])


def test_graph_iterations_and_prep_placement_agree(og, gpu_ctx, monkeypatch):
    """Iterations per captured graph (runtime.cpp iterGraphK: solve_iterate runs n / K launches of
    the K-iteration graph and n mod K of the single one) and the few-window GN prep inside the
    linearisation launch (k_lin_few<.., true>) change the launch structure only: bitwise-equal
    solves, with the prep as its own launch and one iteration per graph as the reference."""
    ws = [_window(og, seed=s) for s in (51, 52)]
    opts = og.default_options(max_num_iterations=7, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    res = []
    for iters, prep in (("1", "0"), ("4", "1"), ("3", "1"), ("8", "0")):
        monkeypatch.setenv("OKVISGPU_GRAPH_ITERS", iters)
        monkeypatch.setenv("OKVISGPU_LIN_PREP", prep)
        for w in ws:
            w.reset()
        gpu_ctx.set_problems([w.problem for w in ws])  # drops the captured graphs
        s = gpu_ctx.solve(opts, len(ws))
        res.append((s, [w.poses().copy() for w in ws], [w.landmarks().copy() for w in ws]))
    for r in res[1:]:
        for k in range(len(ws)):
            assert r[0][k]["final_cost"] == res[0][0][k]["final_cost"]
            assert r[0][k]["num_iterations"] == res[0][0][k]["num_iterations"] == 7
            assert np.array_equal(r[1][k], res[0][1][k])
            assert np.array_equal(r[2][k], res[0][2][k])


def _close(sg, so, rel=1e-7):
    assert sg["num_iterations"] == so["num_iterations"], (sg, so)
    assert sg["termination"] == so["termination"], (sg, so)
    assert abs(sg["final_cost"] - so["final_cost"]) <= rel * so["final_cost"], (sg, so)


def test_solve_default_tolerances(og, oracle, gpu_ctx):
    """Ceres default tolerances (function_tolerance 1e-6 etc.): same termination and count."""
    w = _window(og)
    opts = og.default_options(max_num_iterations=50)
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(opts, 1)[0]
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    _close(sg, so)


def test_ragged_batch(og, oracle, gpu_ctx):
    """Windows of different sizes in one batch, each against its own oracle solve."""
    ws = [og.SynthWindow(6, 150, 1000, seed=11), og.SynthWindow(10, 500, 4000, seed=12),
          og.SynthWindow(3, 40, 200, seed=13), og.SynthWindow(20, 800, 6000, seed=14)]
    opts = og.default_options(max_num_iterations=4, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    gpu_ctx.set_problems([w.problem for w in ws])
    sgs = gpu_ctx.solve(opts, len(ws))
    for w, sg in zip(ws, sgs):
        P = w.poses().copy()
        w.reset()
        so = oracle.solve(w.problem_ptr(), opts)
        # the 3-keyframe window is far from converged after 4 steps: positions agree to ~1e-8 m but
        # the cost gradient there (~1e6) turns that into ~1e-6 relative cost differences
        _close(sg, so, rel=2e-6)
        assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6


def test_constant_blocks(og, oracle, gpu_ctx):
    """Frozen pose / speed-bias / landmark blocks (SetParameterBlockConstant, ViGraph.cpp:597-637)."""
    w = _window(og, seed=21)
    p = w.problem
    p.pose_constant[0] = 1
    p.speed_bias_constant[0] = 1
    p.pose_constant[3] = 1
    for l in range(0, p.n_landmarks, 7):
        p.landmark_constant[l] = 1
    opts = og.default_options(max_num_iterations=5, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    gpu_ctx.set_problems([p])
    sg = gpu_ctx.solve(opts, 1)[0]
    P = w.poses().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    _close(sg, so)
    assert np.array_equal(P[0], w.poses()[0]) and np.array_equal(P[3], w.poses()[3])
    assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6


def test_set_block_constant_between_solves(og, oracle, gpu_ctx):
    """Freeze a state after set_problems (the realtime graph's freeze/unfreeze pattern)."""
    w = _window(og, seed=22)
    opts = og.default_options(max_num_iterations=4, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    gpu_ctx.set_problems([w.problem])
    gpu_ctx.set_block_constant(0, 0, 2, True)
    gpu_ctx.set_block_constant(0, 1, 2, True)
    sg = gpu_ctx.solve(opts, 1)[0]
    w.reset()
    w.problem.pose_constant[2] = 1
    w.problem.speed_bias_constant[2] = 1
    so = oracle.solve(w.problem_ptr(), opts)
    _close(sg, so)


def test_s50_window_parity(og, oracle, gpu_ctx):
    """The north-star window after the bench's 10 iterations: SURVEY.md §8c contract (poses within
    1e-6 m, landmarks within 1e-5 m of the oracle)."""
    w = og.SynthWindow(50, 2000, 16000, seed=20251015)
    opts = og.default_options(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(opts, 1)[0]
    P, L = w.poses().copy(), w.landmarks().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    _close(sg, so)
    assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6
    # Landmarks: a few synthetic points have (numerically) unobservable depth (smallest eigenvalue
    # of their robustified J_l^T J_l ~1e-16) and drift to tens of km in both solvers; compare all
    # landmarks in the information metric and the well-determined ones in metres.
    p = w.problem
    L0 = w.landmarks()
    r, _, Jl = oracle.eval_reprojection(w.problem_ptr(), p.n_observations)
    obs_lm = np.ctypeslib.as_array(p.obs_landmark, (p.n_observations,))
    wgt = 1.0 / (1.0 + (r * r).sum(1))  # Cauchy corrector weight rho'
    V = np.zeros((p.n_landmarks, 3, 3))
    np.add.at(V, obs_lm, wgt[:, None, None] * np.einsum("oki,okj->oij", Jl, Jl))
    d = L[:, :3] - L0[:, :3]
    maha = np.sqrt(np.einsum("li,lij,lj->l", d, V, d))
    assert maha.max() <= 1e-4, maha.max()
    well_determined = np.linalg.eigvalsh(V)[:, 0] > 1e-1  # every direction's sigma below ~3 px-equivalents
    assert well_determined.mean() > 0.5, well_determined.mean()
    assert np.abs(d[well_determined]).max() <= 1e-5


def test_pseudo_inverse_solve(og, oracle, gpu_ctx):
    """A full solve whose IMU square roots all take the clamped-eigenvalue branch."""
    w = _window(og, seed=23)
    w.problem.imu_params.sigma_gw_c = 0.0
    w.problem.imu_params.sigma_aw_c = 0.0
    opts = og.default_options(max_num_iterations=3, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(opts, 1)[0]
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    assert sg["num_iterations"] == so["num_iterations"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"], (sg, so)


def test_kernel_timing_hook(og, gpu_ctx):
    w = _window(og, seed=24)
    gpu_ctx.set_problems([w.problem])
    gpu_ctx.solve(og.default_options(max_num_iterations=2), 1)
    for name in og.kernel_names():
        ms, work, bound = gpu_ctx.time_kernel(name, 2)
        assert ms > 0 and work > 0 and bound in ("hbm", "mfma"), name


def test_cholesky_schedules_agree(og, oracle, gpu_ctx):
    """The persistent per-window and the tile-parallel Cholesky schedules run the same tile
    operations in the same order: bitwise-equal solves, both matching the oracle."""
    ws = [og.SynthWindow(10, 500, 4000, seed=s) for s in (31, 32)]
    res = []
    for sched in (1, 2, 4):
        for w in ws:
            w.reset()
        opts = og.default_options(max_num_iterations=5, function_tolerance=0.0, gradient_tolerance=0.0,
                                  parameter_tolerance=0.0, cholesky_schedule=sched)
        gpu_ctx.set_problems([w.problem for w in ws])
        s = gpu_ctx.solve(opts, len(ws))
        res.append((s, [w.poses().copy() for w in ws]))
    for k in range(len(ws)):
        assert res[0][0][k]["final_cost"] == res[1][0][k]["final_cost"]
        assert np.array_equal(res[0][1][k], res[1][1][k])
    ws[0].reset()
    so = oracle.solve(ws[0].problem_ptr(), og.default_options(max_num_iterations=5, function_tolerance=0.0,
                                                              gradient_tolerance=0.0, parameter_tolerance=0.0))
    _close(res[1][0][0], so)


def test_cholesky_schedules_agree_nested_dissection(og, oracle, gpu_ctx):
    """S50 windows in a small batch are held in a nested-dissection order (runtime.cpp chooseNd):
    the tile-parallel launches, the persistent kernel and the persistent kernel split over the two
    parts (launch A per part, launch B for the separator) give bitwise-equal solves; the oracle
    (natural order) agrees to the usual tolerance."""
    ws = [og.SynthWindow(50, 2000, 16000, seed=s) for s in (33, 34)]
    res = []
    for sched in (1, 2, 3, 4, 5):
        for w in ws:
            w.reset()
        opts = og.default_options(max_num_iterations=4, function_tolerance=0.0, gradient_tolerance=0.0,
                                  parameter_tolerance=0.0, cholesky_schedule=sched)
        gpu_ctx.set_problems([w.problem for w in ws])
        st = gpu_ctx.stats()
        assert st["cholesky_split_windows"] == len(ws) and st["cholesky_launches"] < 12, st
        s = gpu_ctx.solve(opts, len(ws))
        res.append((s, [w.poses().copy() for w in ws], [w.landmarks().copy() for w in ws]))
    for r in res[1:]:
        for k in range(len(ws)):
            assert r[0][k]["final_cost"] == res[0][0][k]["final_cost"]
            assert np.array_equal(r[1][k], res[0][1][k]) and np.array_equal(r[2][k], res[0][2][k])
    ws[0].reset()
    so = oracle.solve(ws[0].problem_ptr(), og.default_options(max_num_iterations=4, function_tolerance=0.0,
                                                              gradient_tolerance=0.0, parameter_tolerance=0.0))
    _close(res[0][0][0], so)
    assert np.abs(res[0][1][0][:, :3] - ws[0].poses()[:, :3]).max() <= 1e-6


def test_cholesky_schedules_ragged_batch(og, gpu_ctx):
    """Windows of different sizes, some terminating early (done windows skip the factorisation):
    the persistent, tile-parallel and pipelined schedules give the same bits."""
    shapes = [(10, 500, 4000), (30, 1200, 9000), (12, 600, 5000), (50, 2000, 16000), (20, 900, 7000)]
    ws = [og.SynthWindow(kf, lm, obs, seed=60 + k) for k, (kf, lm, obs) in enumerate(shapes)]
    res = []
    for sched in (1, 2, 4, 5):
        for w in ws:
            w.reset()
        opts = og.default_options(max_num_iterations=5, cholesky_schedule=sched)
        gpu_ctx.set_problems([w.problem for w in ws])
        s = gpu_ctx.solve(opts, len(ws))
        res.append((s, [w.poses().copy() for w in ws]))
    for r in res[1:]:
        for k in range(len(ws)):
            assert r[0][k]["num_iterations"] == res[0][0][k]["num_iterations"]
            assert r[0][k]["final_cost"] == res[0][0][k]["final_cost"], k
            assert np.array_equal(r[1][k], res[0][1][k]), k


def test_graph_file_solve_parity(og, oracle, gpu_ctx, tmp_path):
    """A window written as an okvis Component graph and loaded back (okvisgpu_graph_save / _load)
    solves on the GPU like the oracle on the same loaded arrays."""
    import ctypes as C
    w = _window(og, seed=25)
    path = tmp_path / "w.graph"
    og.save_graph(w.problem_ptr(), path)
    p = w.problem
    cams = [og.Camera() for _ in range(p.n_cameras)]
    for i in range(p.n_cameras):
        C.pointer(cams[i])[0] = p.cameras[i]
    opts = og.default_options(max_num_iterations=5, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    g = og.Graph(path, cams, p.imu_params)
    g.problem.pose_constant[0] = 1  # gauge: the loaded full graph carries no priors
    gpu_ctx.set_problems([g.problem])
    sg = gpu_ctx.solve(opts, 1)[0]
    P = g.poses().copy()
    g2 = og.Graph(path, cams, p.imu_params)
    g2.problem.pose_constant[0] = 1
    so = oracle.solve(g2.problem_ptr(), opts)
    _close(sg, so)
    assert np.abs(P[:, :3] - g2.poses()[:, :3]).max() <= 1e-6


def test_large_window_parity(og, oracle, gpu_ctx):
    """A 200-keyframe window (reduced dimension 3,000, 47 tiles: the full-graph / final-BA size
    class) against the oracle: two iterations."""
    w = og.SynthWindow(200, 8000, 64000, seed=26)
    opts = og.default_options(max_num_iterations=2, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0, num_threads=8)
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(opts, 1)[0]
    P = w.poses().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    _close(sg, so, rel=1e-6)
    assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= 1e-6


def _window_with_degenerate_state(og, seed, j=25):
    """An S50 window with an extra state (pose + speed/bias, index j) whose only residual is a
    host-evaluated constant factor: its 15 columns of J are exactly zero. With min_lm_diagonal = 0
    the LM diagonal adds nothing there, so the diagonal tile holding them has a zero pivot and every
    Gauss-Newton attempt of this window fails (mu retries, then invalid steps, then FAILURE after
    max_num_consecutive_invalid_steps), in the middle of the factorisation's chain."""
    from _problem import OwnedProblem
    sw = og.SynthWindow(50, 2000, 16000, seed=seed)
    P = OwnedProblem.copy_of(sw.problem)
    del sw
    P.poses = np.insert(P.poses, j, P.poses[j], axis=0)
    P.speed_biases = np.insert(P.speed_biases, j, P.speed_biases[j], axis=0)
    P.pose_constant = np.insert(P.pose_constant, j, 0)
    P.speed_bias_constant = np.insert(P.speed_bias_constant, j, 0)
    P.obs_pose = np.where(P.obs_pose >= j, P.obs_pose + 1, P.obs_pose)
    P.imu_blocks = np.where(P.imu_blocks >= j, P.imu_blocks + 1, P.imu_blocks)
    P.pose_prior_block = np.where(P.pose_prior_block >= j, P.pose_prior_block + 1, P.pose_prior_block)
    P.sb_prior_block = np.where(P.sb_prior_block >= j, P.sb_prior_block + 1, P.sb_prior_block)
    P.host_dim = np.array([1], np.int32)
    P.host_param_kind = np.array([[0, 1, -1, -1]], np.int32)
    P.host_param_index = np.array([[j, j, -1, -1]], np.int32)
    P.host_cauchy = np.zeros(1, np.uint8)
    P.host_fn = og.host_evaluate(lambda h, prm: (np.array([0.1]), [np.zeros((1, 7)), np.zeros((1, 9))]), [[7, 9]])
    P.bind()
    return P


def test_cholesky_failure_path_all_schedules(og, oracle, gpu_ctx):
    """A failed factorisation (zero pivot in the middle of one window's chain) in a batch of three
    S50 windows: the persistent (1), pipelined (4: team F stops, team B sees the failure through
    pipe[3]) and split pipelined (5) schedules give the same iterations, unsuccessful steps,
    termination and bits; the failing window's summary is the oracle's; the two healthy windows
    get the bits they get in a batch without the failing one (same size regime)."""
    from _problem import OwnedProblem
    bad = _window_with_degenerate_state(og, seed=71)
    good = [OwnedProblem.copy_of(og.SynthWindow(50, 2000, 16000, seed=s).problem) for s in (72, 73)]
    probs = [good[0], bad, good[1]]
    snaps = [p.snapshot() for p in probs]
    opts = dict(max_num_iterations=8, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0,
                min_lm_diagonal=0.0)
    res = []
    for sched in (1, 4, 5):
        for p, s in zip(probs, snaps):
            p.restore(s)
        gpu_ctx.set_problems([p.struct for p in probs])
        if sched == 5:
            assert gpu_ctx.stats()["cholesky_split_windows"] >= 2
        s = gpu_ctx.solve(og.default_options(cholesky_schedule=sched, **opts), len(probs))
        res.append((s, [p.poses.copy() for p in probs]))
    key = lambda s: (s["num_iterations"], s["num_successful_steps"], s["num_unsuccessful_steps"], s["termination"])  # noqa: E731
    for r in res[1:]:
        for k in range(len(probs)):
            assert key(r[0][k]) == key(res[0][0][k]), (k, r[0][k], res[0][0][k])
            assert r[0][k]["final_cost"] == res[0][0][k]["final_cost"], k
            assert np.array_equal(r[1][k], res[0][1][k]), k
    sb = res[0][0][1]
    assert sb["termination"] == "FAILURE" and sb["num_successful_steps"] == 1, sb
    bad.restore(snaps[1])
    so = oracle.solve(bad.ptr(), og.default_options(**opts))
    assert key(so) == key(sb), (so, sb)
    assert abs(so["final_cost"] - sb["final_cost"]) <= 1e-9 * so["final_cost"]
    # the healthy windows: as in a batch of their own
    for p, s in zip(good, (snaps[0], snaps[2])):
        p.restore(s)
    gpu_ctx.set_problems([p.struct for p in good])
    sg = gpu_ctx.solve(og.default_options(cholesky_schedule=1, **opts), len(good))
    for k, i in ((0, 0), (1, 2)):
        assert key(sg[k]) == key(res[0][0][i]) and sg[k]["final_cost"] == res[0][0][i]["final_cost"], (k, sg[k])
        assert np.array_equal(good[k].poses, res[0][1][i])
