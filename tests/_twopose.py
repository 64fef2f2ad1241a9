"""Two-keyframe scenes for TwoPoseStandardGraphError::compute tests (test infrastructure).

A scene is the reference keyframe S0, another keyframe S1 and landmarks seen from both through the
EuRoC stereo rig of the synthetic windows (config/euroc/okvis2.yaml). It is returned both as an
okvisgpu.TwoPoseBatch edge (the compute() input) and as an okvisgpu_problem with the same
reprojection residuals (reference pose constant), so that the marginalised relative system can be
checked against the Schur complement of the full problem.
"""
import ctypes as C

import numpy as np

import okvisgpu as og


def rot(q):
    """Eigen toRotationMatrix of (x, y, z, w)."""
    x, y, z, w = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def quat_from_axis_angle(a):
    th = np.linalg.norm(a)
    if th < 1e-15:
        return np.array([0.0, 0.0, 0.0, 1.0])
    s = np.sin(th / 2) / th
    return np.array([a[0] * s, a[1] * s, a[2] * s, np.cos(th / 2)])


def rig():
    """Cameras and extrinsics of the synthetic windows (EuRoC stereo, radtan)."""
    w = og.SynthWindow(3, 20, 60, seed=1)
    p = w.problem
    cams = [og.Camera() for _ in range(p.n_cameras)]
    for i in range(p.n_cameras):
        C.pointer(cams[i])[0] = p.cameras[i]
    ex = np.ctypeslib.as_array(p.extrinsics, shape=(p.n_cameras, 7)).copy()
    return cams, ex


def project(oracle, cam, T_WS, T_SC, hp_W):
    R_WS, R_SC = rot(T_WS[3:]), rot(T_SC[3:])
    hp_S = np.r_[R_WS.T @ (hp_W[:3] - T_WS[:3] * hp_W[3]), hp_W[3]]
    hp_C = np.r_[R_SC.T @ (hp_S[:3] - T_SC[:3] * hp_S[3]), hp_S[3]]
    kp = np.zeros(2)
    J = np.zeros(8)
    ok = oracle.lib().oracle_project(C.byref(cam), og.dptr(hp_C), og.dptr(kp), og.dptr(J))
    return kp, ok == 0 and hp_C[2] > 0


def scene(oracle, seed, n_lm=40, ref_pose=None, noise=0.3, baseline=(0.3, 0.1, 0.05), outliers=0,
          mono_far=0, mono_near=0, no_other=False):
    """One edge. mono_far / mono_near: extra landmarks seen by ONE camera of the reference only
    (rank-2 3x3 block) at S0 depth >= 3 (kept, clamped pseudo-inverse) or < 2.99 (skipped)."""
    rng = np.random.default_rng(seed)
    cams, ex = rig()
    T0 = np.array([0, 0, 0, 0, 0, 0, 1.0]) if ref_pose is None else np.asarray(ref_pose, dtype=np.float64)
    q1 = quat_from_axis_angle(rng.normal(0, 0.05, 3))
    R0 = rot(T0[3:])
    # T_WS1 = T_WS0 * (baseline, q1): q_WS1 = q_WS0 q1
    x0, y0, z0, w0 = T0[3:]
    x1, y1, z1, w1 = q1
    qW1 = np.array([w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1, w0 * y1 + y0 * w1 + z0 * x1 - x0 * z1,
                    w0 * z1 + z0 * w1 + x0 * y1 - y0 * x1, w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1])
    T1 = np.r_[T0[:3] + R0 @ np.asarray(baseline), qW1]
    landmarks, observations = [], []

    def point_in_front(depth_lo, depth_hi):
        # a point in camera 0's frame of the reference keyframe, mapped to world
        d = rng.uniform(depth_lo, depth_hi)
        pc = np.array([rng.uniform(-0.4, 0.4) * d, rng.uniform(-0.3, 0.3) * d, d])
        ps = rot(ex[0, 3:]) @ pc + ex[0, :3]
        return np.r_[R0 @ ps + T0[:3], 1.0]

    def s0_depth(hp):
        return (R0.T @ (hp[:3] - T0[:3]))[2]

    k = 0
    tries = 0
    while len(landmarks) < n_lm:
        tries += 1
        assert tries < 100 * n_lm, "scene(): cannot place landmarks"
        hp = point_in_front(3.0, 12.0)
        obs = []
        for other, T in ((False, T0), (True, T1)):
            if other and no_other:
                continue
            for c in range(len(cams)):
                kp, ok = project(oracle, cams[c], T, ex[c], hp)
                if not ok:
                    continue
                meas = kp + rng.normal(0, noise, 2)
                if k < outliers and other and c == 0:
                    meas = kp + np.array([6.0, -5.0])  # |r| > 3: dropped by compute()
                obs.append((other, c, meas, [1.0, 0.0, 0.0, 1.0], True))
        if len(obs) < (2 if no_other else 3):
            continue
        k += 1
        landmarks.append(hp + np.r_[rng.normal(0, 0.002, 3), 0.0])  # the estimate, not the truth
        observations.append(obs)
    for want_far, count in ((True, mono_far), (False, mono_near)):
        made = 0
        for _ in range(1000 * count):
            if made == count:
                break
            hp = point_in_front(4.0, 8.0) if want_far else point_in_front(0.8, 1.6)
            if want_far != (s0_depth(hp) >= 2.99):
                continue
            kp, ok = project(oracle, cams[0], T0, ex[0], hp)
            if not ok:
                continue
            landmarks.append(hp)
            observations.append([(False, 0, kp + rng.normal(0, noise, 2), [1.0, 0.0, 0.0, 1.0], True)])
            made += 1
    edge = {"ref_pose": T0, "other_pose": T1, "landmarks": np.array(landmarks), "observations": observations}
    return edge, cams, ex


class SceneProblem:
    """The edge's reprojection residuals as an okvisgpu_problem: pose 0 constant, pose 1 free,
    landmarks free, Cauchy(1), no IMU / priors."""

    def __init__(self, edge, cams, ex):
        self.poses = np.ascontiguousarray(np.stack([edge["ref_pose"], edge["other_pose"]]))
        self.pc = np.array([1, 0], dtype=np.uint8)
        self.lms = np.ascontiguousarray(edge["landmarks"], dtype=np.float64)
        op, ol, oc, kp, L = [], [], [], [], []
        for l, obs in enumerate(edge["observations"]):
            for other, c, m, s, _ in obs:
                op.append(1 if other else 0)
                ol.append(l)
                oc.append(c)
                kp.append(m)
                L.append(s)
        self.op = np.asarray(op, dtype=np.int32)
        self.ol = np.asarray(ol, dtype=np.int32)
        self.oc = np.asarray(oc, dtype=np.int32)
        self.kp = np.ascontiguousarray(kp, dtype=np.float64)
        self.L = np.ascontiguousarray(L, dtype=np.float64)
        self.cams = (og.Camera * len(cams))(*cams)
        self.ex = np.ascontiguousarray(ex)
        p = og.Problem()
        p.n_poses = 2
        p.poses = og.dptr(self.poses)
        p.pose_constant = self.pc.ctypes.data_as(C.POINTER(C.c_uint8))
        p.n_landmarks = len(self.lms)
        p.landmarks = og.dptr(self.lms)
        p.n_cameras = len(cams)
        p.cameras = self.cams
        p.extrinsics = og.dptr(self.ex)
        p.n_observations = len(self.op)
        p.obs_pose = self.op.ctypes.data_as(C.POINTER(C.c_int32))
        p.obs_landmark = self.ol.ctypes.data_as(C.POINTER(C.c_int32))
        p.obs_camera = self.oc.ctypes.data_as(C.POINTER(C.c_int32))
        p.obs_keypoint = og.dptr(self.kp)
        p.obs_sqrt_info = og.dptr(self.L)
        self.problem = p

    def ptr(self):
        return C.pointer(self.problem)
