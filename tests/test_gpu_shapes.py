"""GPU parity on the realistic window shapes and solver branches the synthetic S10/S50 benchmark
windows do not reach (VERDICT r01 "Next round" 1): long IMU factors with and without
redoPropagationAlways, the frontend's tracking solve, the final-BA size, the Hilti camera model at
S50, the CeresIterationCallback time limit, landmarks observed from many keyframes, and a failed
set_problems. Every case runs through the C ABI against the CPU oracle on identical inputs.

Tolerances as tests/test_gpu_parity.py: iteration count and termination exact, final cost 1e-7
relative (looser where a case states why), positions 1e-6 m."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _zero_tol(og, iters, **kw):
    return og.default_options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0, **kw)


def _close(sg, so, rel=1e-7):
    assert sg["num_iterations"] == so["num_iterations"], (sg, so)
    assert sg["termination"] == so["termination"], (sg, so)
    assert abs(sg["final_cost"] - so["final_cost"]) <= rel * so["final_cost"], (sg, so)


def _solve_both(og, oracle, gpu_ctx, w, opts, rel=1e-7, pos_tol=1e-6):
    gpu_ctx.set_problems([w.problem])
    sg = gpu_ctx.solve(opts)[0]
    P = w.poses().copy()
    imu_g = w.imu_state().copy() if w.problem.n_imu else None
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    _close(sg, so, rel)
    assert np.abs(P[:, :3] - w.poses()[:, :3]).max() <= pos_tol
    return sg, so, P, imu_g


@pytest.mark.parametrize("redo_always", [0, 1])
def test_long_imu_factors_s50(og, oracle, gpu_ctx, redo_always):
    """S50 with 0.5 s keyframe spacing: ~100 IMU samples per factor, so ImuError.cpp:837 only
    re-integrates on first use (>= 50 samples) unless redoPropagationAlways is set (the final-BA mode,
    ViSlamBackend.cpp:2036), and the bias correction is first order otherwise."""
    w = og.SynthWindow(50, 2000, 16000, seed=41, kf_dt_s=0.5)
    sb = np.ctypeslib.as_array(w.problem.imu_sample_begin, shape=(w.problem.n_imu + 1,))
    assert np.diff(sb).min() >= 100
    sg, so, _, imu_g = _solve_both(og, oracle, gpu_ctx, w, _zero_tol(og, 5, redo_propagation_always=redo_always))
    # the ImuError state written back: >= 50 samples integrate once (first use) unless redo_always.
    # (Ceres evaluates an accepted point twice — candidate cost, then Jacobians — so the
    # informational redo counter of the oracle runs ahead of the device's one-evaluation-per-
    # iteration count under redo_always; the state itself is that of the same point.)
    imu_o = w.imu_state()
    if redo_always:
        assert imu_g[:, 0].min() > 1 and imu_o[:, 0].min() > 1
    else:
        assert np.all(imu_g[:, 0] == 1) and np.all(imu_o[:, 0] == 1)


def test_tracking_solve(og, oracle, gpu_ctx):
    """The frontend's tracking solve (Frontend.cpp:1591-1601 -> ViSlamBackend::optimiseRealtimeGraph
    with freezePosesUntil / freezeSpeedAndBiasesUntil the second-newest state and every landmark
    constant, ViSlamBackend.cpp:854-863): only the newest pose and speed/bias are free, so the
    reduced system has no e-blocks and dimension 15."""
    w = og.SynthWindow(50, 2000, 16000, seed=42)
    p = w.problem
    for i in range(p.n_poses - 1):
        p.pose_constant[i] = 1
        p.speed_bias_constant[i] = 1
    for l in range(p.n_landmarks):
        p.landmark_constant[l] = 1
    opts = og.default_options(max_num_iterations=8)
    gpu_ctx.set_problems([p])
    st = gpu_ctx.stats()
    assert st["reduced_dim"] == 15 and st["n_landmarks_free"] == 0
    sg = gpu_ctx.solve(opts)[0]
    P = w.poses().copy()
    w.reset()
    so = oracle.solve(w.problem_ptr(), opts)
    _close(sg, so)
    assert np.array_equal(P[:-1], w.poses()[:-1])  # frozen states untouched
    assert np.abs(P[-1, :3] - w.poses()[-1, :3]).max() <= 1e-9


def test_final_ba_size_500kf(og, oracle, gpu_ctx):
    """BASELINE config 4 size class: 500 keyframes / 20,000 landmarks / 160,000 reprojections /
    499 IMU factors (reduced dimension 7,500), two iterations."""
    w = og.SynthWindow(500, 20000, 160000, seed=43)
    _solve_both(og, oracle, gpu_ctx, w, _zero_tol(og, 2, num_threads=8), rel=1e-6)


def test_final_ba_hilti_500kf(og, oracle, gpu_ctx):
    """BASELINE config 4 as okvis runs it (ViSlamBackend::doFinalBa, ViSlamBackend.cpp:2005-2164) on a
    Hilti-shaped 500-keyframe graph: equidistant cameras (config/hilti22), both extrinsics variable
    with their PoseError priors (do_extrinsics: true, config/hilti22/okvis2.yaml:82-83), everything
    unfrozen (:2026-2033), redoPropagationAlways (:2036), SPARSE_NORMAL_CHOLESKY (ViGraph.cpp:248),
    and the pass sequence of optimiseFullGraph twice (:2041,2059; :1971-2003):
      1a  loop-closure RelativePoseErrors (keyframes 460.. back to 0..; 100 x information,
          :1985-1986) with function_tolerance 1e-3 for numIter/3 iterations (:1988-1989);
      1b  constraints removed, function_tolerance 1e-6 (:1990-1997);
      2   speed/bias prior removed (:2044), extrinsics soft-constrained at their estimate (:2050-2052),
          optimiseFullGraph again (:2059).
    Iteration counts are cut (3 / 3 / 3 instead of 33 / 100 / 100) so the oracle finishes in
    seconds; GPU and oracle each carry their own estimates (and IMU states) from pass to pass."""
    from _problem import OwnedProblem
    from test_gpu_parity import CAMERA_MODELS, _switch_camera_model
    w = og.SynthWindow(500, 20000, 160000, seed=48, n_relpose=30, relpose_stride=460, relpose_kind=1,
                       do_extrinsics=1)
    _switch_camera_model(oracle, w, *CAMERA_MODELS["equidistant"])
    q = OwnedProblem.copy_of(w.problem)
    assert q.relpose_blocks[:, 1].min() - q.relpose_blocks[:, 0].max() >= 400 and np.all(q.extrinsics_constant == 0)
    q.relpose_sqrt_info *= 10.0                        # 100 x information
    q.bind()
    gpu, cpu = q, OwnedProblem.copy_of(q.struct)
    base = dict(linear_solver=og.SPARSE_NORMAL_CHOLESKY, redo_propagation_always=1, num_threads=16,
                gradient_tolerance=1e-10, parameter_tolerance=1e-8)
    passes = [("1a", dict(max_num_iterations=3, function_tolerance=1e-3)),
              ("1b", dict(max_num_iterations=3, function_tolerance=1e-6)),
              ("2", dict(max_num_iterations=3, function_tolerance=1e-6))]
    for name, kw in passes:
        if name == "1b":
            for p in (gpu, cpu):                       # removeRelativePoseConstraint
                p.relpose_blocks, p.relpose_delta_x = p.relpose_blocks[:0], p.relpose_delta_x[:0]
                p.relpose_sqrt_info, p.relpose_lin_point = p.relpose_sqrt_info[:0], p.relpose_lin_point[:0]
                p.relpose_kind = p.relpose_kind[:0]
                p.bind()
        if name == "2":
            for p in (gpu, cpu):                       # removeSpeedAndBiasPrior + softConstrainExtrinsics
                p.sb_prior_block, p.sb_prior_meas, p.sb_prior_sqrt_info = (
                    p.sb_prior_block[:0], p.sb_prior_meas[:0], p.sb_prior_sqrt_info[:0])
                p.extrinsics_prior_meas = p.extrinsics.copy()
                p.extrinsics_prior_sqrt_info = np.tile(np.diag([100.0] * 6).reshape(-1), (len(p.extrinsics), 1))
                p.bind()
        opts = og.default_options(**base, **kw)
        gpu_ctx.set_problems([gpu.struct])
        sg = gpu_ctx.solve(opts)[0]
        so = oracle.solve(cpu.ptr(), opts)
        _close(sg, so, rel=1e-7)
        assert sg["num_successful_steps"] == so["num_successful_steps"], (name, sg, so)
        dp = np.abs(gpu.poses[:, :3] - cpu.poses[:, :3]).max()
        de = np.abs(gpu.extrinsics[:, :3] - cpu.extrinsics[:, :3]).max()
        print(f"final BA pass {name}: {sg['num_iterations']} it, {sg['termination']}, cost {sg['final_cost']:.10g} "
              f"(rel {abs(sg['final_cost'] - so['final_cost']) / so['final_cost']:.2e}), max pose dev {dp:.2e} m, "
              f"extrinsics dev {de:.2e} m")
        assert dp <= 1e-6 and de <= 1e-6, (name, dp, de)


def test_equidistant_s50(og, oracle, gpu_ctx):
    """S50 with the Hilti camera model (EquidistantDistortion, config/hilti22)."""
    from test_gpu_parity import CAMERA_MODELS, _switch_camera_model
    w = og.SynthWindow(50, 2000, 16000, seed=44)
    _switch_camera_model(oracle, w, *CAMERA_MODELS["equidistant"])
    _solve_both(og, oracle, gpu_ctx, w, _zero_tol(og, 5), rel=1e-7)


def test_time_limit_user_success(og, oracle, gpu_ctx):
    """CeresIterationCallback (CeresIterationCallback.cpp:30-38): stop once iteration >=
    iterationMinimum and cumulative + iteration time exceed the limit. A zero limit stops exactly at
    the minimum (USER_SUCCESS, result = that iterate); a generous one never triggers."""
    w = og.SynthWindow(10, 500, 4000, seed=45)
    gpu_ctx.set_problems([w.problem])
    ref = gpu_ctx.solve(_zero_tol(og, 3))[0]
    P3 = w.poses().copy()
    for min_it in (3, 0):
        w.reset()
        gpu_ctx.update_params()
        sg = gpu_ctx.solve(_zero_tol(og, 10, time_limit_s=0.0, min_iterations=min_it))[0]
        assert sg["termination"] == "USER_SUCCESS" and sg["num_iterations"] == min_it, sg
        Pg = w.poses().copy()
        w.reset()
        so = oracle.solve(w.problem_ptr(), _zero_tol(og, 10, time_limit_s=0.0, min_iterations=min_it))
        _close(sg, so)
        if min_it == 3:
            assert sg["final_cost"] == ref["final_cost"] and np.array_equal(Pg, P3)
        else:
            assert sg["final_cost"] == sg["initial_cost"]
    w.reset()
    gpu_ctx.update_params()
    sg = gpu_ctx.solve(_zero_tol(og, 4, time_limit_s=1e6, min_iterations=1))[0]
    assert sg["termination"] == "NO_CONVERGENCE" and sg["num_iterations"] == 4


def test_landmarks_seen_from_many_keyframes(og, oracle, gpu_ctx):
    """Landmarks observed from up to 100 free keyframes (> 2,048 visit-pair products, more than a
    landmark group stages in LDS): k_lm_visit streams their products from HBM."""
    w = og.SynthWindow(100, 200, 30000, seed=7, kf_dt_s=0.02, max_obs_per_landmark=240)
    p = w.problem
    ol = np.ctypeslib.as_array(p.obs_landmark, shape=(p.n_observations,))
    op = np.ctypeslib.as_array(p.obs_pose, shape=(p.n_observations,))
    assert max(len(set(op[ol == l])) for l in range(p.n_landmarks)) >= 90
    _solve_both(og, oracle, gpu_ctx, w, _zero_tol(og, 3, num_threads=8), rel=1e-6)


def test_failed_set_problems_leaves_no_problem(og, gpu_ctx):
    """A set_problems that fails validation after a valid one leaves the context without a problem
    (no stale batch is used): get_params / solve return OKVISGPU_ERR_NO_PROBLEM."""
    import ctypes as C
    w = og.SynthWindow(6, 150, 1000, seed=46)
    gpu_ctx.set_problems([w.problem])
    bad = og.SynthWindow(6, 150, 1000, seed=47)
    bad.problem.obs_pose[0] = 99  # out of range
    with pytest.raises(og.OkvisGpuError):
        gpu_ctx.set_problems([w.problem, bad.problem])
    assert og.lib().okvisgpu_get_params(gpu_ctx.h) == 5          # OKVISGPU_ERR_NO_PROBLEM
    o = og.default_options()
    sums = (og.Summary * 2)()
    assert og.lib().okvisgpu_solve(gpu_ctx.h, C.byref(o), sums) == 5
    # and the context is usable again
    gpu_ctx.set_problems([w.problem])
    assert gpu_ctx.solve(og.default_options(max_num_iterations=2))[0]["num_iterations"] == 2
