"""The CPU oracle's functors against the reference's own test properties:
analytic-vs-numeric Jacobians with jacobiansCorrect semantics (ErrorInterface.cpp:44-163,
delta 1e-7, tolerance 1e-6), the PoseManifold numeric-diff check (PoseLocalParameterization.cpp:
109-137, delta 1e-9, tolerance 1e-6) and the camera Jacobian check (TestPinholeCamera.cpp:94-116,
< 1e-4). The reference ships no golden vectors for these functors."""
import ctypes as C

import numpy as np
import pytest

import okvisgpu as og


def _window(kf=6, lm=120, obs=900, seed=20251015):
    return og.SynthWindow(kf, lm, obs, seed=seed)


EQUIDISTANT_TEST = (-0.0041, 0.0063, -0.0067, 0.0023)
# RadialTangentialDistortion8::testObject (RadialTangentialDistortion8.hpp:94-95): k1 k2 p1 p2 k3 k4 k5 k6
RADTAN8_TEST = (0.6261, 0.001, -0.0002, 0.0001, 0.0001, 0.9541, 0.1151, -0.0075)
DISTORTIONS = [og.DIST_NONE, og.DIST_RADTAN, og.DIST_EQUIDISTANT, og.DIST_RADTAN8]


@pytest.mark.parametrize("distortion", DISTORTIONS)
def test_reprojection_jacobians(oracle, distortion):
    w = _window()
    p = w.problem
    for c in range(p.n_cameras):
        cam = p.cameras[c]
        cam.distortion = distortion
        params = {og.DIST_EQUIDISTANT: EQUIDISTANT_TEST, og.DIST_RADTAN8: RADTAN8_TEST}.get(distortion)
        if params is not None:
            for i in range(8):
                cam.dist[i] = params[i] if i < len(params) else 0.0
    rng = np.random.default_rng(0)
    for o in rng.choice(p.n_observations, 40, replace=False):
        assert oracle.check_jacobians(w.problem_ptr(), 0, int(o)) < 1e-6


def test_imu_jacobians(oracle):
    w = _window()
    for f in range(w.problem.n_imu):
        assert oracle.check_jacobians(w.problem_ptr(), 1, f) < 1e-6


def test_prior_jacobians(oracle):
    w = _window()
    # perturb the prior-carrying first state away from its measurement
    p = w.problem
    p.poses[0] += 0.01
    p.poses[4] += 0.02
    p.speed_biases[1] += 0.05
    assert oracle.check_jacobians(w.problem_ptr(), 2, 0) < 1e-6
    assert oracle.check_jacobians(w.problem_ptr(), 3, 0) < 1e-6


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _rand_pose(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    return np.concatenate([rng.normal(size=3), q])


def test_pose_manifold_plus_jacobian_numdiff(oracle):
    rng = np.random.default_rng(1)
    L = oracle.lib()
    for _ in range(20):
        x = _rand_pose(rng)
        J = np.zeros((7, 6))
        L.oracle_pose_plus_jacobian(_dp(x), _dp(J))
        Jn = np.zeros((7, 6))
        d = 1e-9
        for k in range(6):
            dp, dm = np.zeros(6), np.zeros(6)
            dp[k], dm[k] = d, -d
            xp, xm = np.zeros(7), np.zeros(7)
            L.oracle_pose_plus(_dp(x), _dp(dp), _dp(xp))
            L.oracle_pose_plus(_dp(x), _dp(dm), _dp(xm))
            Jn[:, k] = (xp - xm) / (2 * d)
        assert np.abs(J - Jn).max() < 1e-6


def test_pose_manifold_lift_times_plus_is_identity(oracle):
    rng = np.random.default_rng(2)
    L = oracle.lib()
    for _ in range(20):
        x = _rand_pose(rng)
        Jp, Jm = np.zeros((7, 6)), np.zeros((6, 7))
        L.oracle_pose_plus_jacobian(_dp(x), _dp(Jp))
        L.oracle_pose_minus_jacobian(_dp(x), _dp(Jm))
        assert np.abs(Jm @ Jp - np.eye(6)).max() < 1e-12


def _camera(distortion):
    cam = og.Camera()
    cam.distortion, cam.width, cam.height = distortion, 752, 480
    cam.fu, cam.fv, cam.cu, cam.cv = 350.0, 360.0, 378.0, 238.0  # PinholeCamera::testObject
    d = {og.DIST_NONE: (0, 0, 0, 0), og.DIST_RADTAN: (-0.16, 0.15, 3e-4, 2e-4),
         og.DIST_EQUIDISTANT: EQUIDISTANT_TEST, og.DIST_RADTAN8: RADTAN8_TEST}[distortion]
    for i, v in enumerate(d):
        cam.dist[i] = v
    return cam


@pytest.mark.parametrize("distortion", DISTORTIONS)
def test_camera_point_jacobian(oracle, distortion):
    cam = _camera(distortion)
    rng = np.random.default_rng(3)
    L = oracle.lib()
    for _ in range(50):
        hp = np.array([rng.uniform(-1, 1), rng.uniform(-0.7, 0.7), 1.0, 1.0]) * np.array([1, 1, 1, 1])
        hp[:3] *= rng.uniform(1, 10)
        kp, J = np.zeros(2), np.zeros((2, 4))
        L.oracle_project(C.byref(cam), _dp(hp), _dp(kp), _dp(J))
        Jn = np.zeros((2, 4))
        d = 1e-6
        for k in range(4):
            e = np.zeros(4)
            e[k] = d
            kpp, kpm, tmp = np.zeros(2), np.zeros(2), np.zeros((2, 4))
            L.oracle_project(C.byref(cam), _dp(hp + e), _dp(kpp), _dp(tmp))
            L.oracle_project(C.byref(cam), _dp(hp - e), _dp(kpm), _dp(tmp))
            Jn[:, k] = (kpp - kpm) / (2 * d)
        assert np.abs(J - Jn).max() < 1e-4 * max(1.0, np.abs(J).max())


def test_project_homogeneous_negative_w_quirk(oracle):
    """PinholeCamera::projectHomogeneous (PinholeCamera.hpp:503-517): for w < 0 the head is
    negated for the projection but the Jacobian is not."""
    cam = _camera(og.DIST_RADTAN)
    L = oracle.lib()
    hp = np.array([0.3, -0.2, 2.0, 0.5])
    kp1, J1, kp2, J2 = np.zeros(2), np.zeros((2, 4)), np.zeros(2), np.zeros((2, 4))
    L.oracle_project(C.byref(cam), _dp(hp), _dp(kp1), _dp(J1))
    L.oracle_project(C.byref(cam), _dp(-hp), _dp(kp2), _dp(J2))
    assert np.allclose(kp1, kp2, rtol=0, atol=1e-12)
    assert np.allclose(J1, J2, rtol=0, atol=1e-12)
