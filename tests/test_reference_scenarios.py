"""The reference's own solver unit tests (TestReprojectionError.cpp:48-164, TestImuError.cpp:63-258),
rebuilt as problems (tests/_ref_scenarios.py) and held to the reference's thresholds: on the CPU
oracle (pins the restatement on the reference's result-level tests) and on the GPU through the C ABI
(also against the oracle on the same problem).

The reference runs them with default ::ceres::Solver::Options (Levenberg-Marquardt); the okvis
solve path, and therefore this backend, is DOGLEG + DENSE_SCHUR (ViGraph.cpp:248-249), so the
thresholds are asserted for that solver."""
import numpy as np
import pytest

from _ref_scenarios import imu_scene, reprojection_scene, rot_err

SEEDS = [1, 2, 3, 4, 5]


def _opts(og, **kw):
    return og.default_options(**kw)


@pytest.mark.parametrize("seed", SEEDS)
def test_oracle_reprojection_scene_thresholds(og, oracle, seed):
    p, T_WS = reprojection_scene(seed)
    s = oracle.solve(p.ptr(), _opts(og))
    est = p.poses[0]
    assert s["termination"] == "CONVERGENCE", s
    assert rot_err(T_WS[3:], est[3:]) < 1e-2          # TestReprojectionError.cpp:158-160
    assert np.linalg.norm(T_WS[:3] - est[:3]) < 1e-1   # :161-163


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("redo_always", [0, 1])
def test_oracle_imu_scene_thresholds(og, oracle, seed, redo_always):
    p, T1 = imu_scene(seed)
    s = oracle.solve(p.ptr(), _opts(og, redo_propagation_always=redo_always))
    est = p.poses[1]
    assert s["final_cost"] < 1e-2, s                   # TestImuError.cpp:251
    assert rot_err(T1[3:], est[3:]) < 1e-2             # :252-254
    assert np.linalg.norm(T1[:3] - est[:3]) < 0.04     # :255-257


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_gpu_reprojection_scene(og, oracle, gpu_ctx, seed):
    p, T_WS = reprojection_scene(seed)
    snap = p.snapshot()
    gpu_ctx.set_problems([p.struct])
    sg = gpu_ctx.solve(_opts(og))[0]
    est = p.poses[0].copy()
    assert sg["termination"] == "CONVERGENCE", sg
    assert rot_err(T_WS[3:], est[3:]) < 1e-2
    assert np.linalg.norm(T_WS[:3] - est[:3]) < 1e-1
    p.restore(snap)
    so = oracle.solve(p.ptr(), _opts(og))
    assert sg["num_iterations"] == so["num_iterations"], (sg, so)
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-9 * so["final_cost"] + 1e-12, (sg, so)
    assert np.abs(est[:3] - p.poses[0][:3]).max() <= 1e-8
    assert rot_err(est[3:], p.poses[0][3:]) <= 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("redo_always", [0, 1])
def test_gpu_imu_scene(og, oracle, gpu_ctx, seed, redo_always):
    """One 980-sample ImuError (the >= 50-sample branch of ImuError.cpp:837 unless redo_always:
    first-order bias correction after the first integration) with its two priors."""
    p, T1 = imu_scene(seed)
    snap = p.snapshot()
    gpu_ctx.set_problems([p.struct])
    sg = gpu_ctx.solve(_opts(og, redo_propagation_always=redo_always))[0]
    est = p.poses[1].copy()
    assert sg["final_cost"] < 1e-2, sg
    assert rot_err(T1[3:], est[3:]) < 1e-2
    assert np.linalg.norm(T1[:3] - est[:3]) < 0.04
    p.restore(snap)
    so = oracle.solve(p.ptr(), _opts(og, redo_propagation_always=redo_always))
    assert sg["num_iterations"] == so["num_iterations"], (sg, so)
    assert sg["termination"] == so["termination"], (sg, so)
    assert abs(sg["final_cost"] - so["final_cost"]) <= 1e-6 * so["final_cost"] + 1e-9, (sg, so)
    assert np.abs(est[:3] - p.poses[1][:3]).max() <= 1e-6
