"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the okvis_ceres hot path used as the parity checker and as
the CPU baseline. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
"""
import ctypes as C
import os

import numpy as np

from _paths import REPO  # noqa: F401
import okvisgpu as og

ORACLE_PATH = os.path.join(REPO, "oracle", "liboracle.so")
_lib = None
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_PATH):
            raise RuntimeError("oracle/liboracle.so missing — run `make -C oracle`")
        L = C.CDLL(ORACLE_PATH)
        P = C.POINTER(og.Problem)
        L.oracle_solve.argtypes = [P, C.POINTER(og.Options), C.POINTER(og.Summary)]
        L.oracle_evaluate.argtypes = [P, _dp]
        L.oracle_linearize_reduce.argtypes = [P, C.c_int32, C.c_double, _dp, _dp, _dp, _ip]
        L.oracle_eval_reprojection.argtypes = [P, _dp, _dp, _dp]
        L.oracle_eval_imu.argtypes = [P, C.c_int32, _dp, _dp]
        L.oracle_check_jacobians.argtypes = [P, C.c_int32, C.c_int32, C.c_double, _dp]
        L.oracle_project.argtypes = [C.POINTER(og.Camera), _dp, _dp, _dp]
        L.oracle_pose_plus.argtypes = [_dp, _dp, _dp]
        L.oracle_pose_plus_jacobian.argtypes = [_dp, _dp]
        L.oracle_pose_minus_jacobian.argtypes = [_dp, _dp]
        L.oracle_dense_cholesky.argtypes = [C.c_int32, _dp, C.c_int32]
        L.oracle_eval_relpose.argtypes = [P, _dp, _dp]
        L.oracle_eval_host.argtypes = [P, _dp, _dp]
        L.oracle_imu_merge.argtypes = [P, C.c_int32, _dp, _dp]
        L.oracle_twopose_compute.argtypes = [C.POINTER(og.TwoPoseEdges), _dp, _dp, _dp, _dp, _dp]
        L.oracle_imu_append.argtypes = [C.POINTER(og.ImuAppendBatch), _ip]
        L.oracle_loss_evaluate.argtypes = [C.POINTER(og.Loss), C.c_double, _dp]
        L.oracle_loss_correct.argtypes = [C.POINTER(og.Loss), C.c_int32, C.c_int32, _dp, _dp, _dp]
        _lib = L
    return _lib


def solve(problem_ptr, options):
    s = og.Summary()
    rc = lib().oracle_solve(problem_ptr, C.byref(options), C.byref(s))
    assert rc == 0
    return s.as_dict()


def loss_evaluate(kind, a=1.0, b=0.0, s=0.0):
    """The oracle's ::ceres::LossFunction::Evaluate restatement: (rho, rho', rho'')."""
    L = og.Loss(og.LOSS_KINDS[kind] if isinstance(kind, str) else int(kind), 0, a, b)
    rho = (C.c_double * 3)()
    assert lib().oracle_loss_evaluate(C.byref(L), float(s), rho) == 0
    return tuple(rho)


def evaluate(problem_ptr):
    c = C.c_double()
    lib().oracle_evaluate(problem_ptr, C.byref(c))
    return c.value


def linearize_reduce(problem_ptr, jacobi_scaling=True, mu=0.0):
    dim = C.c_int32()
    cost = C.c_double()
    lib().oracle_linearize_reduce(problem_ptr, int(jacobi_scaling), mu, None, None, C.byref(cost), C.byref(dim))
    n = dim.value
    S = np.zeros((n, n))
    rhs = np.zeros(n)
    rc = lib().oracle_linearize_reduce(problem_ptr, int(jacobi_scaling), mu, og.dptr(S), og.dptr(rhs),
                                       C.byref(cost), C.byref(dim))
    return S, rhs, cost.value, rc


def eval_reprojection(problem_ptr, n_obs):
    r = np.zeros((n_obs, 2))
    Jp = np.zeros((n_obs, 2, 6))
    Jl = np.zeros((n_obs, 2, 3))
    lib().oracle_eval_reprojection(problem_ptr, og.dptr(r), og.dptr(Jp), og.dptr(Jl))
    return r, Jp, Jl


def eval_imu(problem_ptr, n_imu, redo_always=False):
    r = np.zeros((n_imu, 15))
    J = np.zeros((n_imu, 15, 30))
    lib().oracle_eval_imu(problem_ptr, int(redo_always), og.dptr(r), og.dptr(J))
    return r, J


def check_jacobians(problem_ptr, kind, index, delta=1e-7):
    m = C.c_double()
    lib().oracle_check_jacobians(problem_ptr, kind, index, delta, C.byref(m))
    return m.value


def eval_relpose(problem_ptr, n):
    r = np.zeros((n, 6))
    J = np.zeros((n, 6, 12))
    lib().oracle_eval_relpose(problem_ptr, og.dptr(r), og.dptr(J))
    return r, J


def eval_host(problem_ptr, n):
    """Host-evaluated factors (ABI 5), no loss: r [n, 15], minimal J [n, 15, 30] (IMU column layout)."""
    r = np.zeros((n, 15))
    J = np.zeros((n, 15, 30))
    rc = lib().oracle_eval_host(problem_ptr, og.dptr(r), og.dptr(J))
    return r, J, rc


def twopose_compute(batch):
    n = batch.struct.n_edges
    out = {"delta_x": np.zeros((n, 6)), "sqrt_info": np.zeros((n, 6, 6)), "lin_point": np.zeros((n, 7)),
           "H00": np.zeros((n, 6, 6)), "b0": np.zeros((n, 6))}
    rc = lib().oracle_twopose_compute(C.byref(batch.struct), og.dptr(out["delta_x"]), og.dptr(out["sqrt_info"]),
                                      og.dptr(out["lin_point"]), og.dptr(out["H00"]), og.dptr(out["b0"]))
    assert rc == 0
    return out


def imu_append(imu_params, state, t1_old, t1_new, speed_biases, sample_begin, sample_t, sample_ga):
    """okvisgpu_imu_append semantics on the CPU (state updated in place; steps, -1 = untouched)."""
    b, keep = og.imu_append_batch(imu_params, state, t1_old, t1_new, speed_biases, sample_begin, sample_t, sample_ga)
    steps = np.zeros(b.n, dtype=np.int32)
    rc = lib().oracle_imu_append(C.byref(b), steps.ctypes.data_as(_ip))
    assert rc == 0
    return steps


def imu_merge(problem_ptr, f, sb):
    state = np.zeros(og.IMU_STATE_DOUBLES)
    steps = lib().oracle_imu_merge(problem_ptr, f, og.dptr(np.ascontiguousarray(sb, dtype=np.float64)), og.dptr(state))
    return state, steps
