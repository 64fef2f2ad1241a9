"""Numpy-owned okvisgpu_problem for tests (the C generator's windows are owned by the library; these
are built or copied in Python so tests can reshape a problem: extra observations, other blocks,
the reference's own unit-test scenes). Plain data only — no solver logic."""
import ctypes as C

import numpy as np

import okvisgpu as og

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_lp = C.POINTER(C.c_int64)
_up = C.POINTER(C.c_uint8)

# field -> (dtype, per-item shape, count attribute); count None = n+1 CSR
_ARRAYS = {
    "poses": (np.float64, (7,), "n_poses"), "pose_constant": (np.uint8, (), "n_poses"),
    "speed_biases": (np.float64, (9,), "n_speed_biases"), "speed_bias_constant": (np.uint8, (), "n_speed_biases"),
    "landmarks": (np.float64, (4,), "n_landmarks"), "landmark_constant": (np.uint8, (), "n_landmarks"),
    "extrinsics": (np.float64, (7,), "n_cameras"),
    "obs_pose": (np.int32, (), "n_observations"), "obs_landmark": (np.int32, (), "n_observations"),
    "obs_camera": (np.int32, (), "n_observations"), "obs_keypoint": (np.float64, (2,), "n_observations"),
    "obs_sqrt_info": (np.float64, (4,), "n_observations"), "obs_cauchy": (np.uint8, (), "n_observations"),
    "imu_blocks": (np.int32, (4,), "n_imu"), "imu_t0_ns": (np.int64, (), "n_imu"), "imu_t1_ns": (np.int64, (), "n_imu"),
    "imu_state": (np.float64, (og.IMU_STATE_DOUBLES,), "n_imu"),
    "pose_prior_block": (np.int32, (), "n_pose_priors"), "pose_prior_meas": (np.float64, (7,), "n_pose_priors"),
    "pose_prior_sqrt_info": (np.float64, (36,), "n_pose_priors"),
    "sb_prior_block": (np.int32, (), "n_sb_priors"), "sb_prior_meas": (np.float64, (9,), "n_sb_priors"),
    "sb_prior_sqrt_info": (np.float64, (81,), "n_sb_priors"),
    "relpose_blocks": (np.int32, (2,), "n_relpose"), "relpose_delta_x": (np.float64, (6,), "n_relpose"),
    "relpose_sqrt_info": (np.float64, (36,), "n_relpose"), "relpose_lin_point": (np.float64, (7,), "n_relpose"),
    "relpose_kind": (np.uint8, (), "n_relpose"),
    "extrinsics_constant": (np.uint8, (), "n_cameras"),
    "extrinsics_prior_camera": (np.int32, (), "n_extrinsics_priors"),
    "extrinsics_prior_meas": (np.float64, (7,), "n_extrinsics_priors"),
    "extrinsics_prior_sqrt_info": (np.float64, (36,), "n_extrinsics_priors"),
    "host_dim": (np.int32, (), "n_host"), "host_param_kind": (np.int32, (4,), "n_host"),
    "host_param_index": (np.int32, (4,), "n_host"), "host_cauchy": (np.uint8, (), "n_host"),
}
_PTR = {np.float64: _dp, np.int32: _ip, np.int64: _lp, np.uint8: _up}
_COUNTS = ("n_poses", "n_speed_biases", "n_landmarks", "n_cameras", "n_observations", "n_imu", "n_pose_priors",
           "n_sb_priors", "n_relpose", "n_extrinsics_priors", "n_host")


class OwnedProblem:
    """Arrays in numpy (attribute per okvisgpu_problem field) + `struct` (an og.Problem view).
    Call `bind()` after replacing arrays. Cameras: list of og.Camera; imu sample arrays:
    imu_sample_begin [n_imu+1], imu_sample_t_ns [n_s], imu_sample_gyr_acc [n_s, 6]."""

    def __init__(self):
        for k, (dt, shp, _) in _ARRAYS.items():
            setattr(self, k, np.zeros((0,) + shp, dtype=dt))
        self.cameras = []
        self.imu_sample_begin = np.zeros(1, dtype=np.int32)
        self.imu_sample_t_ns = np.zeros(0, dtype=np.int64)
        self.imu_sample_gyr_acc = np.zeros((0, 6))
        self.imu_params = og.ImuParams()
        self.host_fn = None  # og.host_evaluate(...) callback of the host factors (ABI 5)
        self.host_loss = None  # og.loss_array(...) per host factor (ABI 6), None = host_cauchy
        self.struct = og.Problem()
        self.bind()

    @classmethod
    def copy_of(cls, prob):
        """Deep copy of an og.Problem (e.g. a SynthWindow's)."""
        self = cls()
        n = {c: getattr(prob, c) for c in _COUNTS}
        for k, (dt, shp, cnt) in _ARRAYS.items():
            ptr = getattr(prob, k)
            m = n[cnt]
            if not ptr or m == 0:
                arr = np.zeros((m,) + shp, dtype=dt)
                if k in ("obs_cauchy", "extrinsics_constant"):  # NULL = Cauchy everywhere / constant T_SC
                    arr[:] = 1
                setattr(self, k, arr)
                continue
            setattr(self, k, np.ctypeslib.as_array(ptr, shape=(m,) + shp).copy())
        self.cameras = [og.Camera() for _ in range(n["n_cameras"])]
        for i in range(n["n_cameras"]):
            C.pointer(self.cameras[i])[0] = prob.cameras[i]
        ni = n["n_imu"]
        if ni:
            self.imu_sample_begin = np.ctypeslib.as_array(prob.imu_sample_begin, shape=(ni + 1,)).copy()
            ns = int(self.imu_sample_begin[-1])
            self.imu_sample_t_ns = np.ctypeslib.as_array(prob.imu_sample_t_ns, shape=(ns,)).copy()
            self.imu_sample_gyr_acc = np.ctypeslib.as_array(prob.imu_sample_gyr_acc, shape=(ns, 6)).copy()
        C.pointer(self.imu_params)[0] = prob.imu_params
        self.bind()
        return self

    def bind(self):
        s = self.struct
        for k, (dt, shp, cnt) in _ARRAYS.items():
            a = np.ascontiguousarray(getattr(self, k), dtype=dt)
            setattr(self, k, a)
            setattr(s, k, a.ctypes.data_as(_PTR[dt]) if a.size else None)
        s.n_poses = len(self.poses)
        s.n_speed_biases = len(self.speed_biases)
        s.n_landmarks = len(self.landmarks)
        s.n_cameras = len(self.cameras)
        s.n_observations = len(self.obs_pose)
        s.n_imu = len(self.imu_blocks)
        s.n_pose_priors = len(self.pose_prior_block)
        s.n_sb_priors = len(self.sb_prior_block)
        s.n_relpose = len(self.relpose_blocks)
        s.n_extrinsics_priors = len(self.extrinsics_prior_camera)
        s.n_host = len(self.host_dim)
        s.host_evaluate = self.host_fn if self.host_fn is not None else og.HOST_EVALUATE_FN()
        if self.host_loss is not None:
            self.host_loss = np.ascontiguousarray(self.host_loss, dtype=og.LOSS_DTYPE)
            assert len(self.host_loss) == s.n_host
            s.host_loss = self.host_loss.ctypes.data
        else:
            s.host_loss = None
        if len(self.extrinsics_constant) != len(self.cameras):  # default: constant extrinsics
            self.extrinsics_constant = np.ones(len(self.cameras), np.uint8)
            s.extrinsics_constant = self.extrinsics_constant.ctypes.data_as(_up) if len(self.cameras) else None
        self._cams = (og.Camera * max(1, len(self.cameras)))(*self.cameras)
        s.cameras = self._cams if self.cameras else None
        self.imu_sample_begin = np.ascontiguousarray(self.imu_sample_begin, dtype=np.int32)
        self.imu_sample_t_ns = np.ascontiguousarray(self.imu_sample_t_ns, dtype=np.int64)
        self.imu_sample_gyr_acc = np.ascontiguousarray(self.imu_sample_gyr_acc, dtype=np.float64).reshape(-1, 6)
        s.imu_sample_begin = self.imu_sample_begin.ctypes.data_as(_ip) if s.n_imu else None
        s.imu_sample_t_ns = self.imu_sample_t_ns.ctypes.data_as(_lp) if s.n_imu else None
        s.imu_sample_gyr_acc = self.imu_sample_gyr_acc.ctypes.data_as(_dp) if s.n_imu else None
        s.imu_params = self.imu_params
        return self

    def ptr(self):
        return C.pointer(self.struct)

    def snapshot(self):
        """Copies of the mutable parameter arrays (to restore an initial estimate)."""
        return {k: getattr(self, k).copy() for k in ("poses", "speed_biases", "landmarks", "imu_state")}

    def restore(self, snap):
        for k, v in snap.items():
            getattr(self, k)[...] = v


def pose_error_sqrt_info(translation_variance, rotation_variance):
    """PoseError(measurement, translationVariance, rotationVariance) (PoseError.cpp:34-39):
    information diag(1/tv x3, 1/rv x3), square root = its LLT factor (diagonal)."""
    L = np.zeros((6, 6))
    for i in range(3):
        L[i, i] = np.sqrt(1.0 / translation_variance)
        L[3 + i, 3 + i] = np.sqrt(1.0 / rotation_variance)
    return L.reshape(-1)


def speed_bias_error_sqrt_info(speed_variance, gyr_bias_variance, acc_bias_variance):
    """SpeedAndBiasError(measurement, speedVariance, gyrBiasVariance, accBiasVariance)
    (SpeedAndBiasError.cpp:26-61)."""
    d = np.array([speed_variance] * 3 + [gyr_bias_variance] * 3 + [acc_bias_variance] * 3)
    return np.diag(np.sqrt(1.0 / d)).reshape(-1)
