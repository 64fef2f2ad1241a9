"""The reference's own solver unit-test problems, rebuilt as okvisgpu problems (test data only).

The reference ships no golden vectors for this path; the tests that run a solve are
its only result-level pins, and they assert convergence thresholds:

  * okvis_ceres/test/TestReprojectionError.cpp:48-164 — one free pose T_WS_init = T_WS * T_disturb
    (T_WS.setRandom(10, pi), T_disturb.setRandom(1, 0.01)), constant extrinsics
    T_SC.setRandom(0.2, pi), a PinholeCamera<NoDistortion> test object (752x480, f 350/360,
    c 378/238), 99 constant landmarks createRandomVisibleHomogeneousPoint((i % 10) * 3 + 2) seen
    through T_WS * T_SC, keypoints = projection + Random() (uniform in [-1, 1]^2), information I,
    no loss. Thresholds: 2|vec(q q_est^-1)| < 1e-2, |r - r_est| < 1e-1.
  * okvis_ceres/test/TestImuError.cpp:63-258 — 1 s of 1 kHz IMU (sinusoidal omega_S and a_W with
    random frequencies / phases / magnitudes, uniform noise sigma_c / sqrt(dt) * Random()), pose
    and speed/bias at samples 10 and 990, T_WS_1 disturbed by setRandom(1, 0.02), one ImuError over
    all samples, PoseError(T_WS_0, 1e-12, 1e-4) and SpeedAndBiasError(sb_0, 1e-12, 1e-12, 1e-12)
    priors, no loss. Thresholds: final_cost < 1e-2, rotation < 1e-2, |r_1 - r_1,est| < 0.04.

Eigen's Random() is std::rand()-based, so the exact draws cannot be reproduced; the scenes are
drawn from numpy generators of the same distributions and checked over several seeds."""
import numpy as np

import okvisgpu as og
from _problem import OwnedProblem, pose_error_sqrt_info, speed_bias_error_sqrt_info


# ---------------------------------------------------------------- quaternion helpers (x y z w)
def qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz])


def qinv(q):
    return np.array([-q[0], -q[1], -q[2], q[3]])


def qrot(q):
    x, y, z, w = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def angle_axis(v):
    a = np.linalg.norm(v)
    if a == 0:
        return np.array([0.0, 0.0, 0.0, 1.0])
    return np.concatenate([np.sin(a / 2) * v / a, [np.cos(a / 2)]])


def set_random(rng, trans_max, rot_max):
    """Transformation::setRandom (Transformation.hpp:199-208): axis = rot_max * Random(), angle =
    |axis|, r = trans_max * Random(); Random() uniform in [-1, 1]."""
    axis = rot_max * rng.uniform(-1, 1, 3)
    r = trans_max * rng.uniform(-1, 1, 3)
    return np.concatenate([r, angle_axis(axis)])


def compose(A, B):
    """T_A * T_B for [r, q] poses."""
    return np.concatenate([A[:3] + qrot(A[3:]) @ B[:3], qmul(A[3:], B[3:])])


def rot_err(q, q_est):
    """2 |vec(q * q_est^-1)| (the tests' rotation criterion)."""
    return 2 * np.linalg.norm(qmul(q, qinv(q_est))[:3])


# ---------------------------------------------------------------- TestReprojectionError scene
TEST_CAMERA = (752, 480, 350.0, 360.0, 378.0, 238.0)   # PinholeCamera::createTestObject


def reprojection_scene(seed):
    rng = np.random.default_rng(seed)
    T_WS = set_random(rng, 10.0, np.pi)
    T_disturb = set_random(rng, 1.0, 0.01)
    T_WS_init = compose(T_WS, T_disturb)
    T_SC = set_random(rng, 0.2, np.pi)
    W, H, fu, fv, cu, cv = TEST_CAMERA
    T_WC = compose(T_WS, T_SC)
    lms, kps = [], []
    for i in range(1, 100):
        min_d, max_d = (i % 10) * 3 + 2.0, 10.0
        img = (rng.uniform(-1, 1, 2) + 1.0) * 0.5 * np.array([W - 0.022, H - 0.022]) + 0.011
        depth = rng.uniform(-1, 1)
        ray = np.array([(img[0] - cu) / fu, (img[1] - cv) / fv, 1.0])
        ray = ray / np.linalg.norm(ray) * (0.5 * (max_d - min_d) * (depth + 1.0) + min_d)
        p_W = T_WC[:3] + qrot(T_WC[3:]) @ ray
        lms.append(np.concatenate([p_W, [1.0]]))
        kp = np.array([fu * ray[0] / ray[2] + cu, fv * ray[1] / ray[2] + cv]) + rng.uniform(-1, 1, 2)
        kps.append(kp)
    p = OwnedProblem()
    p.poses = T_WS_init[None].copy()
    p.pose_constant = np.zeros(1, np.uint8)
    p.landmarks = np.array(lms)
    p.landmark_constant = np.ones(len(lms), np.uint8)
    cam = og.Camera()
    cam.distortion = og.DIST_NONE
    cam.width, cam.height = W, H
    cam.fu, cam.fv, cam.cu, cam.cv = fu, fv, cu, cv
    p.cameras = [cam]
    p.extrinsics = T_SC[None].copy()
    n = len(lms)
    p.obs_pose = np.zeros(n, np.int32)
    p.obs_landmark = np.arange(n, dtype=np.int32)
    p.obs_camera = np.zeros(n, np.int32)
    p.obs_keypoint = np.array(kps)
    p.obs_sqrt_info = np.tile([1.0, 0.0, 0.0, 1.0], (n, 1))
    p.obs_cauchy = np.zeros(n, np.uint8)                 # AddResidualBlock(cost, nullptr, ...)
    p.bind()
    return p, T_WS


# ---------------------------------------------------------------- TestImuError scene
def imu_scene(seed):
    rng = np.random.default_rng(seed)
    ip = og.ImuParams()
    ip.g, ip.a_max, ip.g_max = 9.81, 1000.0, 1000.0
    ip.sigma_g_c, ip.sigma_a_c, ip.sigma_gw_c, ip.sigma_aw_c = 6.0e-4, 2.0e-3, 3.0e-6, 2.0e-5
    rate, duration = 1000, 1.0
    w_om = rng.uniform(0.1, 10.0, 3)
    p_om = rng.uniform(0.0, np.pi, 3)
    m_om = rng.uniform(0.1, 1.0, 3)
    w_a = rng.uniform(0.1, 10.0, 3)
    p_a = rng.uniform(0.1, np.pi, 3)
    m_a = rng.uniform(0.1, 10.0, 3)
    dt = 1.0 / rate
    q = np.array([0.0, 0.0, 0.0, 1.0])
    r = np.zeros(3)
    v = np.zeros(3)
    n = int(duration * rate)
    ts, ga = [], []
    T0 = T1 = sb0 = sb1 = None
    for i in range(n):
        t = i / rate
        if i == 10:
            T0, sb0 = np.concatenate([r, q]), np.concatenate([v, np.zeros(6)])
        if i == n - 10:
            T1, sb1 = np.concatenate([r, q]), np.concatenate([v, np.zeros(6)])
        om = m_om * np.sin(w_om * t + p_om)
        aW = m_a * np.sin(w_a * t + p_a)
        th = np.linalg.norm(om) * dt * 0.5
        sinc = np.sinc(th / np.pi)
        dq = np.concatenate([sinc * 0.5 * dt * om, [np.cos(th)]])
        q = qmul(q, dq)
        v = v + dt * aW
        r = r + dt * v
        gyr = om + ip.sigma_g_c / np.sqrt(dt) * rng.uniform(-1, 1, 3)
        acc = qrot(q).T @ (aW + np.array([0, 0, ip.g])) + ip.sigma_a_c / np.sqrt(dt) * rng.uniform(-1, 1, 3)
        ts.append(i * 1_000_000)                            # okvis::Time(i / 1 kHz) in ns
        ga.append(np.concatenate([gyr, acc]))
    T_disturb = set_random(rng, 1.0, 0.02)
    T1_dist = compose(T1, T_disturb)
    p = OwnedProblem()
    p.poses = np.stack([T0, T1_dist])
    p.pose_constant = np.zeros(2, np.uint8)
    p.speed_biases = np.stack([sb0, sb1])
    p.speed_bias_constant = np.zeros(2, np.uint8)
    p.imu_blocks = np.array([[0, 0, 1, 1]], np.int32)
    p.imu_t0_ns = np.array([10 * 1_000_000], np.int64)
    p.imu_t1_ns = np.array([(n - 10) * 1_000_000], np.int64)
    p.imu_sample_begin = np.array([0, n], np.int32)
    p.imu_sample_t_ns = np.array(ts, np.int64)
    p.imu_sample_gyr_acc = np.array(ga)
    p.imu_state = np.zeros((1, og.IMU_STATE_DOUBLES))
    p.imu_params = ip
    p.pose_prior_block = np.zeros(1, np.int32)
    p.pose_prior_meas = T0[None].copy()
    p.pose_prior_sqrt_info = pose_error_sqrt_info(1e-12, 1e-4)[None]
    p.sb_prior_block = np.zeros(1, np.int32)
    p.sb_prior_meas = sb0[None].copy()
    p.sb_prior_sqrt_info = speed_bias_error_sqrt_info(1e-12, 1e-12, 1e-12)[None]
    p.bind()
    return p, T1
