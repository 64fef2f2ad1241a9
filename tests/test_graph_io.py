"""okvis Component text graphs (okvis_ceres/src/Component.cpp) <-> okvisgpu problems (host code,
no GPU). The reference ships no graph files, so the load semantics are checked by round trips of the
synthetic windows through okvisgpu_graph_save / okvisgpu_graph_load, hand-written files for the
format's rules (ids ordered as std::map keys, information 64/size^2 from the FRAME:KEYPOINT,
float keypoints as cv::KeyPoint, one extrinsics block per camera) and the loader's error paths."""
import numpy as np
import pytest

import okvisgpu as og


def _cams_imu(w):
    p = w.problem
    cams = [og.Camera() for _ in range(p.n_cameras)]
    import ctypes as C
    for i in range(p.n_cameras):
        C.pointer(cams[i])[0] = p.cameras[i]
    return cams, p.imu_params


def _arr(ptr, shape, dtype=np.float64):
    return np.ctypeslib.as_array(ptr, shape=shape).astype(dtype, copy=True)


def test_round_trip_synthetic_window(tmp_path, oracle):
    w = og.SynthWindow(10, 500, 4000, seed=20251015)
    path = tmp_path / "window.graph"
    og.save_graph(w.problem_ptr(), path)
    cams, imu = _cams_imu(w)
    g = og.Graph(path, cams, imu)
    p, q = w.problem, g.problem
    assert (q.n_poses, q.n_landmarks, q.n_observations, q.n_imu) == (p.n_poses, p.n_landmarks, p.n_observations,
                                                                      p.n_imu)
    np.testing.assert_array_equal(_arr(q.poses, (q.n_poses, 7)), _arr(p.poses, (p.n_poses, 7)))
    np.testing.assert_array_equal(_arr(q.speed_biases, (q.n_poses, 9)), _arr(p.speed_biases, (p.n_poses, 9)))
    np.testing.assert_array_equal(_arr(q.landmarks, (q.n_landmarks, 4)), _arr(p.landmarks, (p.n_landmarks, 4)))
    # observations come back grouped per state and camera (Component::save order); keypoints are
    # cv::KeyPoint floats, information 64/size^2 with a float size
    key = lambda P, n: np.lexsort((_arr(P.obs_landmark, (n,), np.int64), _arr(P.obs_camera, (n,), np.int64),
                                   _arr(P.obs_pose, (n,), np.int64)))
    n = p.n_observations
    a, b = key(p, n), key(q, n)
    for f in ("obs_pose", "obs_landmark", "obs_camera"):
        np.testing.assert_array_equal(_arr(getattr(q, f), (n,), np.int64)[b], _arr(getattr(p, f), (n,), np.int64)[a])
    kp_p = _arr(p.obs_keypoint, (n, 2))[a]
    np.testing.assert_array_equal(_arr(q.obs_keypoint, (n, 2))[b], kp_p.astype(np.float32).astype(np.float64))
    np.testing.assert_allclose(_arr(q.obs_sqrt_info, (n, 4))[b], _arr(p.obs_sqrt_info, (n, 4))[a], rtol=1e-7)
    assert np.all(_arr(q.obs_cauchy, (n,), np.int64) == 1)
    # IMU factors and their measurements exactly
    ni = p.n_imu
    np.testing.assert_array_equal(_arr(q.imu_blocks, (ni, 4), np.int64), _arr(p.imu_blocks, (ni, 4), np.int64))
    np.testing.assert_array_equal(_arr(q.imu_t0_ns, (ni,), np.int64), _arr(p.imu_t0_ns, (ni,), np.int64))
    np.testing.assert_array_equal(_arr(q.imu_t1_ns, (ni,), np.int64), _arr(p.imu_t1_ns, (ni,), np.int64))
    sb_p = _arr(p.imu_sample_begin, (ni + 1,), np.int64)
    sb_q = _arr(q.imu_sample_begin, (ni + 1,), np.int64)
    np.testing.assert_array_equal(np.diff(sb_q), np.diff(sb_p))
    ns = sb_p[-1] - sb_p[0]
    np.testing.assert_array_equal(_arr(q.imu_sample_gyr_acc, (ns, 6)), _arr(p.imu_sample_gyr_acc, (ns, 6)))
    np.testing.assert_array_equal(_arr(q.imu_sample_t_ns, (ns,), np.int64), _arr(p.imu_sample_t_ns, (ns,), np.int64))
    # and it saves back to the same text
    path2 = tmp_path / "again.graph"
    og.save_graph(g.problem_ptr(), path2)
    assert path.read_text() == path2.read_text()
    # the loaded graph is a valid problem (fix the gauge like the window's prior would)
    q.pose_constant[0] = 1
    s = oracle.solve(g.problem_ptr(), og.default_options(max_num_iterations=3))
    assert s["final_cost"] < s["initial_cost"]


def test_load_rules(tmp_path):
    """Ids ordered as map keys, 64/size^2 information, normalised quaternions, speed/bias layout."""
    txt = """VERTEX_SE3:QUAT_TIME 20 1 2 3 0 0 0 2 2000
VERTEX_R3:VEL 20 0.1 0.2 0.3
VERTEX_R3:ACCBIAS 20 0.01 0.02 0.03
VERTEX_R3:GYRBIAS 20 0.001 0.002 0.003
FRAME 20 0 7 0 0 0 0 0 0 1 2000
FRAME:KEYPOINT 20 0 100.25 200.5 16 BRISK2 00
VERTEX_SE3:QUAT_TIME 10 0 0 0 0 0 0 1 1000
FRAME 10 0 7 0 0 0 0 0 0 1 1000
FRAME:KEYPOINT 10 0 50.5 60.5 8 BRISK2 00
EDGE_IMU 10 20
EDGE_IMU:MEASUREMENTS 0 0 9.81 0.1 0.2 0.3 900
EDGE_IMU:MEASUREMENTS 0 0 9.81 0.1 0.2 0.3 2100
VERTEX_TRACKXYZ 5 1 1 5 0.9
EDGE_OBS 20 0 0 5 100.25 200.5 0.25 0 0 0.25
EDGE_OBS 10 0 0 5 50.5 60.5 1 0 0 1
"""
    path = tmp_path / "g.graph"
    path.write_text(txt)
    w = og.SynthWindow(3, 20, 60, seed=1)
    cams, imu = _cams_imu(w)
    g = og.Graph(path, cams[:1], imu)
    p = g.problem
    sid, t, lid = g.ids()
    assert list(sid) == [10, 20] and list(t) == [1000, 2000] and list(lid) == [5]
    P = g.poses()
    np.testing.assert_array_equal(P[1], [1, 2, 3, 0, 0, 0, 1])           # quaternion normalised
    sb = _arr(p.speed_biases, (2, 9))
    np.testing.assert_array_equal(sb[1], [0.1, 0.2, 0.3, 0.001, 0.002, 0.003, 0.01, 0.02, 0.03])
    np.testing.assert_array_equal(sb[0], np.zeros(9))
    assert p.n_observations == 2
    np.testing.assert_array_equal(_arr(p.obs_pose, (2,), np.int64), [1, 0])
    np.testing.assert_array_equal(_arr(p.obs_sqrt_info, (2, 4)), [[0.5, 0, 0, 0.5], [1, 0, 0, 1]])  # 8 / size
    assert p.n_imu == 1
    np.testing.assert_array_equal(_arr(p.imu_blocks, (1, 4), np.int64), [[0, 0, 1, 1]])
    assert (p.imu_t0_ns[0], p.imu_t1_ns[0]) == (1000, 2000)
    np.testing.assert_array_equal(_arr(p.imu_sample_gyr_acc, (2, 6))[0], [0.1, 0.2, 0.3, 0, 0, 9.81])
    np.testing.assert_array_equal(g.landmarks()[0], [1, 1, 5, 1])


@pytest.mark.parametrize("text", [
    "VERTEX_SE3:QUAT_TIME 1 0 0 0 0 0 0 1 0\nBOGUS 1\n",                                   # unknown tag
    "VERTEX_SE3:QUAT_TIME 1 0 0 0 0 0 0 1 0\nVERTEX_TRACKXYZ 2 0 0 1 1\nEDGE_OBS 1 0 0 2 0 0 1 0 0 1\n",  # no frame
    "VERTEX_SE3:QUAT_TIME 1 0 0 0 0 0 0 1 0\nFRAME 1 0 5 0 0 0 0 0 0 1 0\n"
    "VERTEX_SE3:QUAT_TIME 2 0 0 0 0 0 0 1 0\nFRAME 2 0 6 0 0 0 0 0 0 1 0\n",               # online calibration
    "VERTEX_SE3:QUAT_TIME 1 0 0 0 0 0 0 1 0\nEDGE_IMU 1 3\n",                               # missing state
])
def test_load_errors(tmp_path, text):
    path = tmp_path / "bad.graph"
    path.write_text(text)
    w = og.SynthWindow(3, 20, 60, seed=1)
    cams, imu = _cams_imu(w)
    with pytest.raises(og.OkvisGpuError):
        og.Graph(path, cams[:1], imu)
