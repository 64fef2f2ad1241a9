"""ImuError::append (ImuError.cpp:63-255) and the IMU-merge elimination it serves
(ViGraphEstimator::eliminateStateByImuMerge, ViGraphEstimator.cpp:38-171).

The merge of the links k-1 -> k and k -> k+1 continues the first link's preintegration (Delta_q,
the (double) integrals, the bias Jacobians, cross_ and the covariance) from its t1 over the second
link's samples up to the second link's t1, integrating the appended part with the eliminated
state's bias; t0, the redo counter / flag and speedAndBiases_ref_ stay as they were.

CPU: the oracle's restatement against properties of the reference (appending at the reference bias
= integrating across the merged interval, up to the split step at the old t1; bookkeeping fields
untouched). GPU (okvisgpu_imu_append, batched): the merged states against the oracle, then a solve
of the window with the state eliminated, GPU against the oracle."""
import numpy as np
import pytest

from _problem import OwnedProblem

CHAIN = list(range(2, 66)) + list(range(292, 301))  # Delta_q .. dp_db_g, sb_ref, cross_
P_DELTA = slice(301, 526)
SQRT = slice(66, 291)


def _window(og, seed=61, kf=10, **kw):
    return og.SynthWindow(kf, 500, 4000, seed=seed, **kw)


def _merged_samples(p, f):
    """The merged link's samples: link f's, then link f+1's newer than its last (ImuError.cpp:74-81)."""
    sb = np.ctypeslib.as_array(p.imu_sample_begin, shape=(p.n_imu + 1,))
    ts = np.ctypeslib.as_array(p.imu_sample_t_ns, shape=(sb[-1],))
    ga = np.ctypeslib.as_array(p.imu_sample_gyr_acc, shape=(sb[-1], 6))
    a = np.arange(sb[f], sb[f + 1])
    b = np.arange(sb[f + 1], sb[f + 2])
    b = b[ts[b] > ts[a[-1]]]
    idx = np.concatenate([a, b])
    return ts[idx].copy(), ga[idx].copy(), (ts[sb[f + 1]:sb[f + 2]].copy(), ga[sb[f + 1]:sb[f + 2]].copy())


def _info(state):
    U = state[SQRT].reshape(15, 15)
    return U.T @ U


def test_oracle_append_equals_integration_across(og, oracle):
    """With the eliminated state's bias equal to the reference bias, appending link k -> k+1 to link
    k-1 -> k reproduces one integration over [t0(k-1), t1(k+1)] of the merged samples, except for the
    trapezoid step split at the old t1 (keyframes sit 1 ms off the 200 Hz grid)."""
    w = _window(og)
    p = w.problem
    f = 3
    sb_ref = w.speed_biases()[p.imu_blocks[4 * f + 1]].copy()
    merged, steps = oracle.imu_merge(w.problem_ptr(), f, sb_ref)
    assert steps > 0
    # one link over the merged interval, integrated from scratch at the same bias
    q = OwnedProblem.copy_of(p)
    ts, ga, _ = _merged_samples(p, f)
    q.imu_blocks = q.imu_blocks[f:f + 1].copy()
    q.imu_t0_ns = q.imu_t0_ns[f:f + 1].copy()
    q.imu_t1_ns = q.imu_t1_ns[f + 1:f + 2].copy()
    q.imu_blocks[0, 2:] = p.imu_blocks[4 * (f + 1) + 2], p.imu_blocks[4 * (f + 1) + 3]
    q.imu_sample_begin = np.array([0, len(ts)], np.int32)
    q.imu_sample_t_ns, q.imu_sample_gyr_acc = ts, ga
    q.imu_state = np.zeros((1, og.IMU_STATE_DOUBLES))
    q.bind()
    oracle.eval_imu(q.ptr(), 1)
    direct = q.imu_state[0]
    for lo, hi, tol in ((2, 6, 1e-6), (6, 30, 1e-5), (30, 57, 1e-4), (292, 301, 1e-4)):
        d, m = direct[lo:hi], merged[lo:hi]
        assert np.abs(d - m).max() <= tol * max(1.0, np.abs(d).max()), (lo, np.abs(d - m).max())
    Pd, Pm = direct[P_DELTA], merged[P_DELTA]
    assert np.abs(Pd - Pm).max() <= 1e-3 * np.abs(Pd).max()
    np.testing.assert_allclose(_info(merged), _info(direct), rtol=0, atol=2e-3 * np.abs(_info(direct)).max())


def test_oracle_append_bookkeeping(og, oracle):
    """append leaves the redo counter, the redo flag and speedAndBiases_ref_ alone (the reference
    sets only t1 and the integration members), and integrates with the given bias."""
    w = _window(og)
    p = w.problem
    f = 2
    sb = w.speed_biases()[p.imu_blocks[4 * f + 3]].copy()
    sb[3:6] += 1e-3
    merged, steps = oracle.imu_merge(w.problem_ptr(), f, sb)
    single = np.zeros(og.IMU_STATE_DOUBLES)
    oracle.eval_imu(w.problem_ptr(), p.n_imu)
    single = w.imu_state()[f].copy()
    assert merged[0] == single[0] == 1 and merged[1] == single[1]
    assert np.array_equal(merged[57:66], single[57:66])
    assert steps > 0 and merged[291] == steps
    assert not np.allclose(merged[2:6], single[2:6])


@pytest.mark.gpu
def test_gpu_imu_append_batch(og, oracle, gpu_ctx):
    """okvisgpu_imu_append on every other link of a window (batched), starting from the states the
    GPU wrote back, against the oracle's merge from its own integration."""
    w = _window(og, seed=62)
    p = w.problem
    gpu_ctx.set_problems([p])
    gpu_ctx.eval_imu(p.n_imu)  # integrates every link (first use) and writes the states back
    st = w.imu_state().copy()
    fs = list(range(0, p.n_imu - 1, 2))
    sbs = np.array([w.speed_biases()[p.imu_blocks[4 * f + 3]] for f in fs])
    sbs[:, 3:6] += 5e-4  # the eliminated states' biases differ from the reference bias
    begin, ts, ga = [0], [], []
    for f in fs:
        _, _, (t_next, g_next) = _merged_samples(p, f)
        ts.append(t_next)
        ga.append(g_next)
        begin.append(begin[-1] + len(t_next))
    t1 = np.ctypeslib.as_array(p.imu_t1_ns, shape=(p.n_imu,))
    state = np.ascontiguousarray(st[fs])
    steps = gpu_ctx.imu_append(p.imu_params, state, t1[fs], t1[[f + 1 for f in fs]], sbs, begin,
                               np.concatenate(ts), np.concatenate(ga))
    w.reset()
    for i, f in enumerate(fs):
        ref, rsteps = oracle.imu_merge(w.problem_ptr(), f, sbs[i])
        assert steps[i] == rsteps > 0
        g = state[i]
        for k in CHAIN:
            assert abs(g[k] - ref[k]) <= 1e-9 * max(1.0, abs(ref[k])), (f, k, g[k], ref[k])
        assert np.abs(g[P_DELTA] - ref[P_DELTA]).max() <= 1e-9 * np.abs(ref[P_DELTA]).max()
        Ig, Ir = _info(g), _info(ref)
        assert np.abs(Ig - Ir).max() <= 1e-7 * np.abs(Ir).max()
        assert g[0] == ref[0] and g[1] == ref[1]


@pytest.mark.gpu
def test_gpu_merged_window_solve(og, oracle, gpu_ctx):
    """eliminateStateByImuMerge of state k in a window, then a solve: the merged link (state from
    okvisgpu_imu_append) between k-1 and k+1, state k and its observations gone. GPU vs oracle."""
    w = _window(og, seed=63)
    p = w.problem
    k = 5
    gpu_ctx.set_problems([p])
    gpu_ctx.eval_imu(p.n_imu)
    st = w.imu_state().copy()
    f = k - 1
    ts_m, ga_m, (t_next, g_next) = _merged_samples(p, f)
    t1 = np.ctypeslib.as_array(p.imu_t1_ns, shape=(p.n_imu,))
    sb_k = w.speed_biases()[k].copy()
    state = np.ascontiguousarray(st[[f]])
    steps = gpu_ctx.imu_append(p.imu_params, state, t1[[f]], t1[[f + 1]], sb_k[None], [0, len(t_next)], t_next, g_next)
    assert steps[0] > 0
    w.reset()
    q = OwnedProblem.copy_of(p)
    keep_obs = q.obs_pose != k
    for name in ("obs_pose", "obs_landmark", "obs_camera", "obs_keypoint", "obs_sqrt_info", "obs_cauchy"):
        setattr(q, name, getattr(q, name)[keep_obs].copy())
    q.obs_pose[q.obs_pose > k] -= 1
    q.poses = np.delete(q.poses, k, axis=0)
    q.pose_constant = np.delete(q.pose_constant, k)
    q.speed_biases = np.delete(q.speed_biases, k, axis=0)
    q.speed_bias_constant = np.delete(q.speed_bias_constant, k)
    sb = np.ctypeslib.as_array(p.imu_sample_begin, shape=(p.n_imu + 1,))
    ts_all = np.ctypeslib.as_array(p.imu_sample_t_ns, shape=(sb[-1],))
    ga_all = np.ctypeslib.as_array(p.imu_sample_gyr_acc, shape=(sb[-1], 6))
    blocks, t0s, t1s, begin, ts, ga, states = [], [], [], [0], [], [], []
    for g in range(p.n_imu):
        if g == f + 1:
            continue
        b = list(p.imu_blocks[4 * g:4 * g + 4])
        if g == f:
            b[2:] = [k + 1, k + 1]
            t_s, g_s, stt, t_end = ts_m, ga_m, state[0], t1[f + 1]
        else:
            t_s, g_s, stt, t_end = ts_all[sb[g]:sb[g + 1]], ga_all[sb[g]:sb[g + 1]], np.zeros(og.IMU_STATE_DOUBLES), t1[g]
        blocks.append([x - (x > k) for x in b])
        t0s.append(p.imu_t0_ns[g])
        t1s.append(t_end)
        ts.append(t_s)
        ga.append(g_s)
        begin.append(begin[-1] + len(t_s))
        states.append(stt)
    q.imu_blocks = np.array(blocks, np.int32)
    q.imu_t0_ns, q.imu_t1_ns = np.array(t0s, np.int64), np.array(t1s, np.int64)
    q.imu_sample_begin = np.array(begin, np.int32)
    q.imu_sample_t_ns, q.imu_sample_gyr_acc = np.concatenate(ts), np.concatenate(ga)
    q.imu_state = np.array(states)
    q.bind()
    snap = q.snapshot()
    opts = og.default_options(max_num_iterations=5, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    gpu_ctx.set_problems([q.struct])
    sg = gpu_ctx.solve(opts)[0]
    P = q.poses.copy()
    q.restore(snap)
    so = oracle.solve(q.ptr(), opts)
    assert sg["num_iterations"] == so["num_iterations"] and sg["termination"] == so["termination"]
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-7 * so["final_cost"], (sg, so)
    assert np.abs(P[:, :3] - q.poses[:, :3]).max() <= 1e-6
