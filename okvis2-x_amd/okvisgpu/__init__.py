"""ctypes binding of the okvisgpu C ABI (include/okvisgpu.h).

The product is the C-ABI shared library ``okvis2-x_amd/libokvisgpu.so`` (HIP kernels for gfx950 +
C++ host runtime). This module only marshals structs for tests, the benchmark and Python callers;
it contains no solver logic and no CPU fallback: if the library (or its GPU code object) is
missing, every call fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("OKVISGPU_LIB") or os.path.join(PKG_ROOT, "libokvisgpu.so")  # env: A/B builds

IMU_STATE_DOUBLES = 526

DIST_NONE, DIST_RADTAN, DIST_EQUIDISTANT, DIST_RADTAN8 = 0, 1, 2, 3
DENSE_SCHUR, SPARSE_NORMAL_CHOLESKY = 0, 1
TERMINATION = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE", 3: "USER_SUCCESS"}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_lp = C.POINTER(C.c_int64)
_up = C.POINTER(C.c_uint8)


class Camera(C.Structure):
    _fields_ = [("distortion", C.c_int32), ("width", C.c_int32), ("height", C.c_int32),
                ("fu", C.c_double), ("fv", C.c_double), ("cu", C.c_double), ("cv", C.c_double),
                ("dist", C.c_double * 8)]


class ImuParams(C.Structure):
    _fields_ = [("a_max", C.c_double), ("g_max", C.c_double), ("sigma_g_c", C.c_double),
                ("sigma_a_c", C.c_double), ("sigma_gw_c", C.c_double), ("sigma_aw_c", C.c_double),
                ("g", C.c_double)]


# robust losses (ABI 6; okvisgpu_loss_kind): ::ceres::LossFunction family
LOSS_NONE, LOSS_CAUCHY, LOSS_TUKEY, LOSS_HUBER, LOSS_SOFTLONE, LOSS_ARCTAN, LOSS_TOLERANT = range(7)
LOSS_KINDS = {"none": LOSS_NONE, "cauchy": LOSS_CAUCHY, "tukey": LOSS_TUKEY, "huber": LOSS_HUBER,
              "softlone": LOSS_SOFTLONE, "arctan": LOSS_ARCTAN, "tolerant": LOSS_TOLERANT}


class Loss(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("a", C.c_double), ("b", C.c_double)]


# numpy record layout of okvisgpu_loss (arrays of per-factor losses: host_loss)
LOSS_DTYPE = np.dtype([("kind", "<i4"), ("reserved", "<i4"), ("a", "<f8"), ("b", "<f8")])


def loss_array(specs):
    """[(kind name or id, a[, b]), ...] -> LOSS_DTYPE array for okvisgpu_problem.host_loss."""
    out = np.zeros(len(specs), dtype=LOSS_DTYPE)
    for i, sp in enumerate(specs):
        k = LOSS_KINDS[sp[0]] if isinstance(sp[0], str) else int(sp[0])
        out[i] = (k, 0, float(sp[1]) if len(sp) > 1 else 1.0, float(sp[2]) if len(sp) > 2 else 0.0)
    return out


def loss_evaluate(kind, a=1.0, b=0.0, s=0.0):
    """okvisgpu_loss_evaluate: (rho, rho', rho'') of a loss at the squared norm s (host only)."""
    L = Loss(LOSS_KINDS[kind] if isinstance(kind, str) else int(kind), 0, a, b)
    rho = (C.c_double * 3)()
    rc = lib().okvisgpu_loss_evaluate(C.byref(L), float(s), rho)
    if rc != 0:
        raise OkvisGpuError(f"okvisgpu_loss_evaluate failed ({rc})")
    return tuple(rho)


# okvisgpu_host_evaluate_fn (ABI 5): (user, factor, parameters, residuals, jacobians) -> nonzero = ok
HOST_EVALUATE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.POINTER(_dp), _dp, C.POINTER(_dp))
HOST_MAX_RESIDUALS = 15


class Problem(C.Structure):
    _fields_ = [
        ("n_poses", C.c_int32), ("poses", _dp), ("pose_constant", _up),
        ("n_speed_biases", C.c_int32), ("speed_biases", _dp), ("speed_bias_constant", _up),
        ("n_landmarks", C.c_int32), ("landmarks", _dp), ("landmark_constant", _up),
        ("n_cameras", C.c_int32), ("cameras", C.POINTER(Camera)), ("extrinsics", _dp),
        ("n_observations", C.c_int32), ("obs_pose", _ip), ("obs_landmark", _ip), ("obs_camera", _ip),
        ("obs_keypoint", _dp), ("obs_sqrt_info", _dp), ("obs_cauchy", _up),
        ("n_imu", C.c_int32), ("imu_blocks", _ip), ("imu_t0_ns", _lp), ("imu_t1_ns", _lp),
        ("imu_sample_begin", _ip), ("imu_sample_t_ns", _lp), ("imu_sample_gyr_acc", _dp),
        ("imu_params", ImuParams), ("imu_state", _dp),
        ("n_pose_priors", C.c_int32), ("pose_prior_block", _ip), ("pose_prior_meas", _dp),
        ("pose_prior_sqrt_info", _dp),
        ("n_sb_priors", C.c_int32), ("sb_prior_block", _ip), ("sb_prior_meas", _dp),
        ("sb_prior_sqrt_info", _dp),
        ("n_relpose", C.c_int32), ("relpose_blocks", _ip), ("relpose_delta_x", _dp),
        ("relpose_sqrt_info", _dp), ("relpose_lin_point", _dp), ("relpose_kind", _up),
        ("extrinsics_constant", _up), ("n_extrinsics_priors", C.c_int32), ("extrinsics_prior_camera", _ip),
        ("extrinsics_prior_meas", _dp), ("extrinsics_prior_sqrt_info", _dp),
        ("n_host", C.c_int32), ("host_dim", _ip), ("host_param_kind", _ip), ("host_param_index", _ip),
        ("host_cauchy", _up), ("host_evaluate", HOST_EVALUATE_FN), ("host_user", C.c_void_p),
        ("host_loss", C.c_void_p),
    ]


def host_evaluate(fn, block_sizes):
    """Wrap a Python cost function as an okvisgpu_host_evaluate_fn (the §8b host fallback).

    fn(factor, params) -> (r, jacobians) or None (evaluation failure): params is the list of the
    factor's parameter blocks (numpy copies, ambient: 7 pose-kind / 9 speed-bias), r the residual
    vector, jacobians one ambient [dim, size] array per block (ceres::CostFunction::Evaluate
    semantics). block_sizes[factor] = the blocks' ambient sizes. Keep the returned object alive as
    long as a problem points at it."""
    def cb(_user, factor, params, residuals, jacobians):
        try:
            sizes = block_sizes[factor]
            out = fn(factor, [np.ctypeslib.as_array(params[k], shape=(n,)).copy() for k, n in enumerate(sizes)])
            if out is None:
                return 0
            r, J = out
            r = np.asarray(r, dtype=np.float64)
            np.ctypeslib.as_array(residuals, shape=(len(r),))[:] = r
            if jacobians:
                for k, n in enumerate(sizes):
                    if jacobians[k]:
                        np.ctypeslib.as_array(jacobians[k], shape=(len(r) * n,))[:] = np.asarray(J[k]).reshape(-1)
            return 1
        except Exception:  # a Python error is an evaluation failure, never an unwinding through C
            return 0
    return HOST_EVALUATE_FN(cb)


class Options(C.Structure):
    _fields_ = [
        ("max_num_iterations", C.c_int32), ("linear_solver", C.c_int32),
        ("trust_region_strategy", C.c_int32), ("jacobi_scaling", C.c_int32),
        ("function_tolerance", C.c_double), ("gradient_tolerance", C.c_double),
        ("parameter_tolerance", C.c_double), ("initial_trust_region_radius", C.c_double),
        ("max_trust_region_radius", C.c_double), ("min_trust_region_radius", C.c_double),
        ("min_relative_decrease", C.c_double), ("min_lm_diagonal", C.c_double),
        ("max_lm_diagonal", C.c_double), ("max_num_consecutive_invalid_steps", C.c_int32),
        ("time_limit_s", C.c_double), ("min_iterations", C.c_int32),
        ("redo_propagation_always", C.c_int32), ("num_threads", C.c_int32), ("verbose", C.c_int32),
        ("cholesky_schedule", C.c_int32),
    ]


class Summary(C.Structure):
    _fields_ = [("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("num_iterations", C.c_int32), ("num_successful_steps", C.c_int32),
                ("num_unsuccessful_steps", C.c_int32), ("termination_type", C.c_int32),
                ("total_time_s", C.c_double), ("final_radius", C.c_double), ("final_mu", C.c_double),
                ("preprocessor_time_s", C.c_double), ("minimizer_time_s", C.c_double),
                ("postprocessor_time_s", C.c_double), ("linear_solver_time_s", C.c_double),
                ("residual_evaluation_time_s", C.c_double), ("jacobian_evaluation_time_s", C.c_double),
                ("step_time_s", C.c_double)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["termination"] = TERMINATION.get(self.termination_type, "?")
        return d


class SynthConfig(C.Structure):
    _fields_ = [("n_keyframes", C.c_int32), ("n_landmarks", C.c_int32), ("n_observations", C.c_int32),
                ("max_obs_per_landmark", C.c_int32), ("kf_dt_s", C.c_double), ("imu_rate_hz", C.c_double),
                ("pixel_noise", C.c_double), ("init_sigma_pos", C.c_double), ("init_sigma_rot", C.c_double),
                ("init_sigma_lm", C.c_double), ("init_sigma_vel", C.c_double), ("seed", C.c_uint64),
                ("n_relpose", C.c_int32), ("relpose_stride", C.c_int32), ("relpose_kind", C.c_int32),
                ("do_extrinsics", C.c_int32), ("extrinsics_sigma_r", C.c_double), ("extrinsics_sigma_alpha", C.c_double)]


class ProblemStats(C.Structure):
    _fields_ = [("n_windows", C.c_int32), ("cholesky_launches", C.c_int32)] + [(k, C.c_int64) for k in (
        "n_poses", "n_speed_biases", "n_landmarks", "n_landmarks_free", "n_extrinsics_free", "n_observations",
        "n_visits", "n_imu", "n_imu_samples", "n_pose_priors", "n_sb_priors", "n_relpose", "reduced_dim",
        "s_tiles_nonzero", "s_tiles_dense", "n_block_pairs", "n_visit_segments", "n_partial_blocks",
        "arena_bytes", "cholesky_split_windows")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class ImuAppendBatch(C.Structure):
    _fields_ = [("n", C.c_int32), ("imu_params", ImuParams), ("state", _dp), ("t1_old_ns", _lp), ("t1_new_ns", _lp),
                ("speed_biases", _dp), ("sample_begin", _ip), ("sample_t_ns", _lp), ("sample_gyr_acc", _dp)]


class TwoPoseEdges(C.Structure):
    _fields_ = [("n_edges", C.c_int32), ("ref_pose", _dp), ("other_pose", _dp),
                ("n_cameras", C.c_int32), ("cameras", C.POINTER(Camera)), ("extrinsics", _dp),
                ("landmark_begin", _ip), ("landmarks", _dp), ("obs_begin", _ip), ("obs_other", _up),
                ("obs_camera", _ip), ("obs_keypoint", _dp), ("obs_sqrt_info", _dp), ("obs_cauchy", _up)]


# Exported symbols of include/okvisgpu.h (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = [
    "okvisgpu_abi_version", "okvisgpu_default_options", "okvisgpu_device_count", "okvisgpu_ctx_create",
    "okvisgpu_ctx_destroy", "okvisgpu_last_error", "okvisgpu_set_problems", "okvisgpu_update_params",
    "okvisgpu_set_block_constant", "okvisgpu_solve", "okvisgpu_get_params", "okvisgpu_evaluate",
    "okvisgpu_linearize_reduce", "okvisgpu_eval_reprojection", "okvisgpu_eval_imu",
    "okvisgpu_synth_default_config", "okvisgpu_synth_create", "okvisgpu_synth_problem",
    "okvisgpu_synth_ground_truth", "okvisgpu_synth_reset", "okvisgpu_synth_destroy",
    "okvisgpu_solve_begin", "okvisgpu_solve_iterate", "okvisgpu_solve_end", "okvisgpu_synchronize",
    "okvisgpu_profile_iteration", "okvisgpu_phase_name", "okvisgpu_kernel_count", "okvisgpu_kernel_name",
    "okvisgpu_time_kernel", "okvisgpu_eval_relpose", "okvisgpu_twopose_compute",
    "okvisgpu_graph_load", "okvisgpu_graph_problem", "okvisgpu_graph_ids", "okvisgpu_graph_destroy",
    "okvisgpu_graph_save", "okvisgpu_get_stats", "okvisgpu_synth_true_extrinsics", "okvisgpu_imu_append",
    "okvisgpu_eval_host", "okvisgpu_plan_window", "okvisgpu_loss_evaluate",
]
N_PHASES = 15

_lib = None


def lib():
    """Load libokvisgpu.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"okvisgpu: {LIB_PATH} missing — build it with `make -C okvis2-x_amd`")
        L = C.CDLL(LIB_PATH)
        L.okvisgpu_abi_version.restype = C.c_int
        L.okvisgpu_default_options.argtypes = [C.POINTER(Options)]
        L.okvisgpu_device_count.argtypes = [_ip]
        L.okvisgpu_ctx_create.argtypes = [C.c_int32, C.POINTER(C.c_void_p)]
        L.okvisgpu_ctx_destroy.argtypes = [C.c_void_p]
        L.okvisgpu_last_error.argtypes = [C.c_void_p]
        L.okvisgpu_last_error.restype = C.c_char_p
        L.okvisgpu_set_problems.argtypes = [C.c_void_p, C.POINTER(Problem), C.c_int32]
        L.okvisgpu_update_params.argtypes = [C.c_void_p]
        L.okvisgpu_set_block_constant.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32]
        L.okvisgpu_solve.argtypes = [C.c_void_p, C.POINTER(Options), C.POINTER(Summary)]
        L.okvisgpu_get_params.argtypes = [C.c_void_p]
        L.okvisgpu_evaluate.argtypes = [C.c_void_p, C.c_int32, _dp]
        L.okvisgpu_linearize_reduce.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_double, _dp, _dp, _dp, _ip]
        L.okvisgpu_eval_reprojection.argtypes = [C.c_void_p, C.c_int32, _dp, _dp, _dp]
        L.okvisgpu_eval_imu.argtypes = [C.c_void_p, C.c_int32, C.c_int32, _dp, _dp]
        L.okvisgpu_synth_default_config.argtypes = [C.POINTER(SynthConfig), C.c_int32, C.c_int32, C.c_int32, C.c_uint64]
        L.okvisgpu_synth_create.argtypes = [C.POINTER(SynthConfig), C.POINTER(C.c_void_p)]
        L.okvisgpu_synth_problem.argtypes = [C.c_void_p]
        L.okvisgpu_synth_problem.restype = C.POINTER(Problem)
        L.okvisgpu_synth_ground_truth.argtypes = [C.c_void_p, _dp, _dp, _dp]
        L.okvisgpu_synth_reset.argtypes = [C.c_void_p]
        L.okvisgpu_synth_true_extrinsics.argtypes = [C.c_void_p, _dp]
        L.okvisgpu_synth_destroy.argtypes = [C.c_void_p]
        L.okvisgpu_solve_begin.argtypes = [C.c_void_p, C.POINTER(Options)]
        L.okvisgpu_solve_iterate.argtypes = [C.c_void_p, C.c_int32]
        L.okvisgpu_solve_end.argtypes = [C.c_void_p, C.POINTER(Summary)]
        L.okvisgpu_synchronize.argtypes = [C.c_void_p]
        L.okvisgpu_profile_iteration.argtypes = [C.c_void_p, _dp]
        L.okvisgpu_phase_name.argtypes = [C.c_int32]
        L.okvisgpu_phase_name.restype = C.c_char_p
        L.okvisgpu_kernel_count.restype = C.c_int
        L.okvisgpu_kernel_name.argtypes = [C.c_int32]
        L.okvisgpu_kernel_name.restype = C.c_char_p
        L.okvisgpu_time_kernel.argtypes = [C.c_void_p, C.c_int32, C.c_int32, _dp, _dp, C.POINTER(C.c_int32)]
        L.okvisgpu_eval_relpose.argtypes = [C.c_void_p, C.c_int32, _dp, _dp]
        L.okvisgpu_eval_host.argtypes = [C.c_void_p, C.c_int32, _dp, _dp]
        L.okvisgpu_graph_load.argtypes = [C.c_char_p, C.POINTER(Camera), C.c_int32, C.POINTER(ImuParams),
                                          C.POINTER(C.c_void_p)]
        L.okvisgpu_graph_problem.argtypes = [C.c_void_p]
        L.okvisgpu_graph_problem.restype = C.POINTER(Problem)
        L.okvisgpu_graph_ids.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), _lp, C.POINTER(C.c_uint64)]
        L.okvisgpu_graph_destroy.argtypes = [C.c_void_p]
        L.okvisgpu_graph_save.argtypes = [C.POINTER(Problem), _lp, C.c_char_p]
        L.okvisgpu_get_stats.argtypes = [C.c_void_p, C.POINTER(ProblemStats)]
        L.okvisgpu_plan_window.argtypes = [C.POINTER(Problem), C.c_int32, _lp, C.POINTER(C.c_uint8), _ip, _ip]
        L.okvisgpu_imu_append.argtypes = [C.c_void_p, C.POINTER(ImuAppendBatch), _ip]
        L.okvisgpu_twopose_compute.argtypes = [C.c_void_p, C.POINTER(TwoPoseEdges), _dp, _dp, _dp, _dp, _dp]
        L.okvisgpu_loss_evaluate.argtypes = [C.POINTER(Loss), C.c_double, _dp]
        _lib = L
    return _lib


def plan_window(problem, nested_dissection):
    """okvisgpu_plan_window (host only): the window's state order, filled tile pattern and
    tile-parallel factorisation schedule."""
    L = lib()
    info = (C.c_int64 * 8)()
    pp = C.byref(problem) if isinstance(problem, Problem) else problem
    rc = L.okvisgpu_plan_window(pp, int(nested_dissection), info, None, None, None)
    if rc != 0:
        raise RuntimeError(f"okvisgpu_plan_window failed ({rc})")
    keys = ("reduced_dim", "s_dim", "tiles", "nonzero_tiles", "launches", "split_tL", "split_tS", "gap_rows")
    out = {k: int(v) for k, v in zip(keys, info)}
    T, D = out["tiles"], out["s_dim"]
    nz = np.zeros(T * T, dtype=np.uint8)
    launch = np.zeros(T, dtype=np.int32)
    nat = np.zeros(D, dtype=np.int32)
    rc = L.okvisgpu_plan_window(pp, int(nested_dissection), info, nz.ctypes.data_as(C.POINTER(C.c_uint8)),
                                launch.ctypes.data_as(_ip), nat.ctypes.data_as(_ip))
    if rc != 0:
        raise RuntimeError(f"okvisgpu_plan_window failed ({rc})")
    out["tile_nz"] = nz.reshape(T, T)
    out["step_launch"] = launch
    out["natural"] = nat
    return out


def default_options(**kw) -> Options:
    o = Options()
    lib().okvisgpu_default_options(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dp)


class OkvisGpuError(RuntimeError):
    pass


class _OwnedBuffer:
    """numpy base object of a view into library-owned memory: holds a reference to the Python
    object that owns the memory, so the view keeps it (and its C allocation) alive."""

    def __init__(self, ptr, shape, owner):
        addr = C.cast(ptr, C.c_void_p).value
        if not addr and int(np.prod(shape)) > 0:
            raise OkvisGpuError("null array in problem")
        self.__array_interface__ = {"data": (addr or 0, False), "shape": tuple(int(n) for n in shape),
                                    "typestr": "<f8", "version": 3}
        self._owner = owner


def _owned_view(ptr, shape, owner) -> np.ndarray:
    return np.asarray(_OwnedBuffer(ptr, shape, owner))


def _owned_problem(ptr, owner):
    """POINTER(Problem) / Problem from the library, each holding a reference to its owner (the
    SynthWindow / Graph whose allocation the arrays point into)."""
    ptr._owner = owner
    return ptr


class SynthWindow:
    """A synthetic sliding window (owned by the C library)."""

    def __init__(self, n_kf=10, n_lm=500, n_obs=4000, seed=20251015, **overrides):
        cfg = SynthConfig()
        lib().okvisgpu_synth_default_config(C.byref(cfg), n_kf, n_lm, n_obs, seed)
        for k, v in overrides.items():
            setattr(cfg, k, v)
        h = C.c_void_p()
        rc = lib().okvisgpu_synth_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise OkvisGpuError(f"okvisgpu_synth_create failed ({rc})")
        self.handle = h
        self.cfg = cfg

    @property
    def problem(self) -> Problem:
        pr = self.problem_ptr().contents
        pr._owner = self  # the struct's arrays live in this window's allocation
        return pr

    def problem_ptr(self):
        return _owned_problem(lib().okvisgpu_synth_problem(self.handle), self)

    def reset(self):
        lib().okvisgpu_synth_reset(self.handle)

    def ground_truth(self):
        p = self.problem
        poses = np.zeros((p.n_poses, 7))
        lms = np.zeros((p.n_landmarks, 4))
        sbs = np.zeros((p.n_speed_biases, 9))
        lib().okvisgpu_synth_ground_truth(self.handle, dptr(poses), dptr(lms), dptr(sbs))
        return poses, lms, sbs

    def true_extrinsics(self):
        e = np.zeros((self.problem.n_cameras, 7))
        lib().okvisgpu_synth_true_extrinsics(self.handle, dptr(e))
        return e

    def extrinsics(self):
        p = self.problem
        return _owned_view(p.extrinsics, (p.n_cameras, 7), self)

    # views into the (mutable) parameter arrays; each view keeps this window alive
    def poses(self):
        p = self.problem
        return _owned_view(p.poses, (p.n_poses, 7), self)

    def speed_biases(self):
        p = self.problem
        return _owned_view(p.speed_biases, (p.n_speed_biases, 9), self)

    def landmarks(self):
        p = self.problem
        return _owned_view(p.landmarks, (p.n_landmarks, 4), self)

    def imu_state(self):
        p = self.problem
        return _owned_view(p.imu_state, (p.n_imu, IMU_STATE_DOUBLES), self)

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().okvisgpu_synth_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def imu_append_batch(imu_params, state, t1_old, t1_new, speed_biases, sample_begin, sample_t, sample_ga):
    """An okvisgpu_imu_append_batch over numpy arrays: (struct, arrays it points into). `state`
    [n, IMU_STATE_DOUBLES] float64 C-contiguous is referenced, not copied (updated in place)."""
    n = len(t1_old)
    keep = [np.ascontiguousarray(t1_old, dtype=np.int64), np.ascontiguousarray(t1_new, dtype=np.int64),
            np.ascontiguousarray(speed_biases, dtype=np.float64).reshape(n, 9),
            np.ascontiguousarray(sample_begin, dtype=np.int32), np.ascontiguousarray(sample_t, dtype=np.int64),
            np.ascontiguousarray(sample_ga, dtype=np.float64).reshape(-1, 6)]
    assert state.dtype == np.float64 and state.flags["C_CONTIGUOUS"] and state.shape == (n, IMU_STATE_DOUBLES)
    b = ImuAppendBatch()
    b.n = n
    b.imu_params = imu_params
    b.state = dptr(state)
    b.t1_old_ns, b.t1_new_ns = keep[0].ctypes.data_as(_lp), keep[1].ctypes.data_as(_lp)
    b.speed_biases = dptr(keep[2])
    b.sample_begin = keep[3].ctypes.data_as(_ip)
    b.sample_t_ns = keep[4].ctypes.data_as(_lp)
    b.sample_gyr_acc = dptr(keep[5])
    return b, keep


class TwoPoseBatch:
    """Owns the arrays of an okvisgpu_twopose_edges batch (TwoPoseStandardGraphError::compute inputs).

    edges: list of dicts with keys ref_pose [7], other_pose [7], landmarks [n_l,4] and
    observations: list (one per landmark) of lists of (other: bool, camera: int, keypoint [2],
    sqrt_info [4], cauchy: bool). cameras: list of Camera; extrinsics [n_cam,7]."""

    def __init__(self, edges, cameras, extrinsics):
        self.ref = np.ascontiguousarray([e["ref_pose"] for e in edges], dtype=np.float64).reshape(-1, 7)
        self.other = np.ascontiguousarray([e["other_pose"] for e in edges], dtype=np.float64).reshape(-1, 7)
        lb, lms, ob, oo, oc, kp, L, ca = [0], [], [0], [], [], [], [], []
        for e in edges:
            for l, obs in zip(e["landmarks"], e["observations"]):
                lms.append(l)
                for (other, cam, k, s, cauchy) in obs:
                    oo.append(1 if other else 0)
                    oc.append(cam)
                    kp.append(k)
                    L.append(s)
                    ca.append(1 if cauchy else 0)
                ob.append(len(oo))
            lb.append(len(lms))
        self.lb = np.asarray(lb, dtype=np.int32)
        self.lms = np.ascontiguousarray(np.asarray(lms, dtype=np.float64).reshape(-1, 4))
        self.ob = np.asarray(ob, dtype=np.int32)
        self.oo = np.asarray(oo, dtype=np.uint8)
        self.oc = np.asarray(oc, dtype=np.int32)
        self.kp = np.ascontiguousarray(np.asarray(kp, dtype=np.float64).reshape(-1, 2))
        self.L = np.ascontiguousarray(np.asarray(L, dtype=np.float64).reshape(-1, 4))
        self.ca = np.asarray(ca, dtype=np.uint8)
        self.cams = (Camera * len(cameras))(*cameras)
        self.ex = np.ascontiguousarray(extrinsics, dtype=np.float64).reshape(-1, 7)
        s = TwoPoseEdges()
        s.n_edges = len(edges)
        s.ref_pose, s.other_pose = dptr(self.ref), dptr(self.other)
        s.n_cameras = len(cameras)
        s.cameras = self.cams
        s.extrinsics = dptr(self.ex)
        s.landmark_begin = self.lb.ctypes.data_as(_ip)
        s.landmarks = dptr(self.lms)
        s.obs_begin = self.ob.ctypes.data_as(_ip)
        s.obs_other = self.oo.ctypes.data_as(_up)
        s.obs_camera = self.oc.ctypes.data_as(_ip)
        s.obs_keypoint = dptr(self.kp)
        s.obs_sqrt_info = dptr(self.L)
        s.obs_cauchy = self.ca.ctypes.data_as(_up)
        self.struct = s


class Graph:
    """An okvis Component text graph loaded into an okvisgpu problem (okvisgpu_graph_load)."""

    def __init__(self, path, cameras, imu_params):
        cams = (Camera * len(cameras))(*cameras)
        h = C.c_void_p()
        rc = lib().okvisgpu_graph_load(str(path).encode(), cams, len(cameras), C.byref(imu_params), C.byref(h))
        if rc != 0:
            raise OkvisGpuError(f"okvisgpu_graph_load({path}) failed ({rc})")
        self.handle = h

    @property
    def problem(self) -> Problem:
        pr = self.problem_ptr().contents
        pr._owner = self
        return pr

    def problem_ptr(self):
        return _owned_problem(lib().okvisgpu_graph_problem(self.handle), self)

    def ids(self):
        p = self.problem
        sid = (C.c_uint64 * p.n_poses)()
        lid = (C.c_uint64 * max(1, p.n_landmarks))()
        t = np.zeros(p.n_poses, dtype=np.int64)
        lib().okvisgpu_graph_ids(self.handle, sid, t.ctypes.data_as(_lp), lid)
        return np.array(sid[:], dtype=np.uint64), t, np.array(lid[:p.n_landmarks], dtype=np.uint64)

    def poses(self):
        p = self.problem
        return _owned_view(p.poses, (p.n_poses, 7), self)

    def landmarks(self):
        p = self.problem
        return _owned_view(p.landmarks, (p.n_landmarks, 4), self)

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().okvisgpu_graph_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def save_graph(problem_ptr, path, state_t_ns=None):
    """okvisgpu_graph_save: write a problem as an okvis Component text graph."""
    t = None if state_t_ns is None else np.ascontiguousarray(state_t_ns, dtype=np.int64).ctypes.data_as(_lp)
    rc = lib().okvisgpu_graph_save(problem_ptr, t, str(path).encode())
    if rc != 0:
        raise OkvisGpuError(f"okvisgpu_graph_save({path}) failed ({rc})")


class Context:
    """One okvisgpu_ctx (one HIP stream + device buffers) holding a batch of windows."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        rc = lib().okvisgpu_ctx_create(device, C.byref(h))
        if rc != 0:
            raise OkvisGpuError(f"okvisgpu_ctx_create({device}) failed with status {rc}")
        self.h = h
        self._keep = None

    def _check(self, rc, what):
        if rc != 0:
            msg = lib().okvisgpu_last_error(self.h)
            raise OkvisGpuError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def set_problems(self, problems):
        arr = (Problem * len(problems))(*problems)
        self._keep = None
        self._check(lib().okvisgpu_set_problems(self.h, arr, len(problems)), "okvisgpu_set_problems")
        self._keep = (arr, list(problems))

    def update_params(self):
        self._check(lib().okvisgpu_update_params(self.h), "okvisgpu_update_params")

    def set_block_constant(self, window, kind, index, is_constant):
        self._check(lib().okvisgpu_set_block_constant(self.h, window, kind, index, int(is_constant)),
                    "okvisgpu_set_block_constant")

    def _n_windows(self, n_windows):
        """Summaries are written for every window of the context (okvisgpu_solve / _solve_end fill
        [n_windows] entries), so the buffer is sized from the problems held, never smaller."""
        if self._keep is None:
            raise OkvisGpuError("no problem set")
        n = len(self._keep[1])
        if n_windows is not None and n_windows != n:
            raise ValueError(f"n_windows={n_windows} but the context holds {n} windows")
        return n

    def solve(self, options: Optional[Options] = None, n_windows: Optional[int] = None):
        o = options or default_options()
        sums = (Summary * self._n_windows(n_windows))()
        self._check(lib().okvisgpu_solve(self.h, C.byref(o), sums), "okvisgpu_solve")
        return [s.as_dict() for s in sums]

    def solve_begin(self, options: Options):
        self._opts = options
        self._check(lib().okvisgpu_solve_begin(self.h, C.byref(options)), "okvisgpu_solve_begin")

    def solve_iterate(self, n: int):
        self._check(lib().okvisgpu_solve_iterate(self.h, n), "okvisgpu_solve_iterate")

    def synchronize(self):
        self._check(lib().okvisgpu_synchronize(self.h), "okvisgpu_synchronize")

    def solve_end(self, n_windows: Optional[int] = None):
        sums = (Summary * self._n_windows(n_windows))()
        self._check(lib().okvisgpu_solve_end(self.h, sums), "okvisgpu_solve_end")
        return [s.as_dict() for s in sums]

    def profile_iteration(self):
        ms = np.zeros(N_PHASES)
        self._check(lib().okvisgpu_profile_iteration(self.h, dptr(ms)), "okvisgpu_profile_iteration")
        return {lib().okvisgpu_phase_name(i).decode(): float(ms[i]) for i in range(N_PHASES)}

    def time_kernel(self, name, reps=5):
        """(avg_ms, work, bound) of one iteration's launches of kernel `name` (see include/okvisgpu.h)."""
        names = kernel_names()
        k = names.index(name)
        ms, work, bound = C.c_double(), C.c_double(), C.c_int32()
        self._check(lib().okvisgpu_time_kernel(self.h, k, reps, C.byref(ms), C.byref(work), C.byref(bound)),
                    "okvisgpu_time_kernel")
        return ms.value, work.value, ("hbm", "mfma")[bound.value]

    def stats(self):
        st = ProblemStats()
        self._check(lib().okvisgpu_get_stats(self.h, C.byref(st)), "okvisgpu_get_stats")
        return st.as_dict()

    def get_params(self):
        self._check(lib().okvisgpu_get_params(self.h), "okvisgpu_get_params")

    def evaluate(self, window=0):
        c = C.c_double()
        self._check(lib().okvisgpu_evaluate(self.h, window, C.byref(c)), "okvisgpu_evaluate")
        return c.value

    def linearize_reduce(self, window=0, jacobi_scaling=True, mu=0.0, dim_hint=None):
        dim = C.c_int32()
        cost = C.c_double()
        self._check(lib().okvisgpu_linearize_reduce(self.h, window, int(jacobi_scaling), mu, None, None,
                                                     C.byref(cost), C.byref(dim)), "linearize_reduce(dim)")
        n = dim.value
        S = np.zeros((n, n))
        rhs = np.zeros(n)
        self._check(lib().okvisgpu_linearize_reduce(self.h, window, int(jacobi_scaling), mu, dptr(S), dptr(rhs),
                                                     C.byref(cost), C.byref(dim)), "linearize_reduce")
        return S, rhs, cost.value

    def eval_reprojection(self, n_obs, window=0):
        r = np.zeros((n_obs, 2))
        Jp = np.zeros((n_obs, 2, 6))
        Jl = np.zeros((n_obs, 2, 3))
        self._check(lib().okvisgpu_eval_reprojection(self.h, window, dptr(r), dptr(Jp), dptr(Jl)),
                    "eval_reprojection")
        return r, Jp, Jl

    def eval_imu(self, n_imu, window=0, redo_always=False):
        r = np.zeros((n_imu, 15))
        J = np.zeros((n_imu, 15, 30))
        self._check(lib().okvisgpu_eval_imu(self.h, window, int(redo_always), dptr(r), dptr(J)), "eval_imu")
        return r, J

    def eval_relpose(self, n_relpose, window=0):
        r = np.zeros((n_relpose, 6))
        J = np.zeros((n_relpose, 6, 12))
        self._check(lib().okvisgpu_eval_relpose(self.h, window, dptr(r), dptr(J)), "eval_relpose")
        return r, J

    def eval_host(self, n_host, window=0):
        """Host-evaluated factors through the device path (gather, callback, upload), no loss:
        r [n, 15], minimal J [n, 15, 30] in the IMU column layout."""
        r = np.zeros((n_host, 15))
        J = np.zeros((n_host, 15, 30))
        self._check(lib().okvisgpu_eval_host(self.h, window, dptr(r), dptr(J)), "eval_host")
        return r, J

    def imu_append(self, imu_params, state, t1_old, t1_new, speed_biases, sample_begin, sample_t, sample_ga):
        """okvisgpu_imu_append (ImuError::append for a batch): `state` [n, IMU_STATE_DOUBLES] is updated
        in place; returns the integrated steps per factor (-1: samples do not reach t1_new)."""
        b, keep = imu_append_batch(imu_params, state, t1_old, t1_new, speed_biases, sample_begin, sample_t,
                                   sample_ga)
        steps = np.zeros(b.n, dtype=np.int32)
        self._check(lib().okvisgpu_imu_append(self.h, C.byref(b), steps.ctypes.data_as(_ip)), "okvisgpu_imu_append")
        return steps

    def twopose_compute(self, edges: "TwoPoseBatch"):
        """TwoPoseStandardGraphError::compute for every edge of the batch: dict of DeltaX_ [n,6],
        J_ [n,6,6], linearisation point [n,7], H00_ [n,6,6], b0_ [n,6]."""
        n = edges.struct.n_edges
        out = {"delta_x": np.zeros((n, 6)), "sqrt_info": np.zeros((n, 6, 6)), "lin_point": np.zeros((n, 7)),
               "H00": np.zeros((n, 6, 6)), "b0": np.zeros((n, 6))}
        self._check(lib().okvisgpu_twopose_compute(self.h, C.byref(edges.struct), dptr(out["delta_x"]),
                                                   dptr(out["sqrt_info"]), dptr(out["lin_point"]), dptr(out["H00"]),
                                                   dptr(out["b0"])), "okvisgpu_twopose_compute")
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().okvisgpu_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def kernel_names():
    return [lib().okvisgpu_kernel_name(i).decode() for i in range(lib().okvisgpu_kernel_count())]


def device_count() -> int:
    n = C.c_int32(0)
    rc = lib().okvisgpu_device_count(C.byref(n))
    return n.value if rc == 0 else 0
