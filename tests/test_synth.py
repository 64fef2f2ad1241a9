"""Synthetic window generator: deterministic per seed, consistent with its own
ground truth, and reset() restores the initial state."""
import numpy as np

import okvisgpu as og


def _arrays(w):
    p = w.problem
    return {
        "poses": np.ctypeslib.as_array(p.poses, (p.n_poses * 7,)).copy(),
        "lms": np.ctypeslib.as_array(p.landmarks, (p.n_landmarks * 4,)).copy(),
        "kp": np.ctypeslib.as_array(p.obs_keypoint, (p.n_observations * 2,)).copy(),
        "obs_lm": np.ctypeslib.as_array(p.obs_landmark, (p.n_observations,)).copy(),
        "imu": np.ctypeslib.as_array(p.imu_sample_gyr_acc, (p.imu_sample_begin[p.n_imu] * 6,)).copy(),
    }


def test_deterministic_per_seed():
    a, b = og.SynthWindow(10, 500, 4000, seed=7), og.SynthWindow(10, 500, 4000, seed=7)
    c = og.SynthWindow(10, 500, 4000, seed=8)
    A, B, Cc = _arrays(a), _arrays(b), _arrays(c)
    for k in A:
        assert np.array_equal(A[k], B[k]), k
    assert not np.array_equal(A["poses"], Cc["poses"])


def test_shapes_and_counts():
    w = og.SynthWindow(50, 2000, 16000, seed=20251015)
    p = w.problem
    assert (p.n_poses, p.n_speed_biases, p.n_landmarks, p.n_observations) == (50, 50, 2000, 16000)
    assert p.n_imu == 49 and p.n_cameras == 2
    obs_lm = np.ctypeslib.as_array(p.obs_landmark, (p.n_observations,))
    counts = np.bincount(obs_lm, minlength=p.n_landmarks)
    assert counts.min() >= 2 and counts.max() <= 20
    blocks = np.ctypeslib.as_array(p.imu_blocks, (p.n_imu, 4))
    assert np.array_equal(blocks[:, 0] + 1, blocks[:, 2])


def test_ground_truth_is_consistent(oracle):
    w = og.SynthWindow(10, 500, 4000, seed=3)
    p = w.problem
    gp, gl, gsb = w.ground_truth()
    np.ctypeslib.as_array(p.poses, (p.n_poses, 7))[:] = gp
    np.ctypeslib.as_array(p.landmarks, (p.n_landmarks, 4))[:] = gl
    np.ctypeslib.as_array(p.speed_biases, (p.n_speed_biases, 9))[:] = gsb
    r, _, _ = oracle.eval_reprojection(w.problem_ptr(), p.n_observations)
    rms = np.sqrt((r ** 2).sum(1).mean())
    assert 0.8 < rms < 2.0  # 1 px isotropic noise per coordinate (information = I)
    ri, _ = oracle.eval_imu(w.problem_ptr(), p.n_imu)
    assert np.sqrt((ri ** 2).sum(1).mean()) < 20.0  # whitened preintegration residual at the truth


def test_reset_restores_initial_state():
    w = og.SynthWindow(10, 500, 4000, seed=5)
    before = _arrays(w)
    p = w.problem
    np.ctypeslib.as_array(p.poses, (p.n_poses * 7,))[:] += 1.0
    w.reset()
    after = _arrays(w)
    assert np.array_equal(before["poses"], after["poses"])
