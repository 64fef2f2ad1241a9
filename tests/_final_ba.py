"""The final-BA protocol of BASELINE config 4 (test infrastructure, shared by the fixture generator
tests/golden/make_final_ba.py and the GPU test tests/test_final_ba_golden.py).

okvis runs it as ViSlamBackend::doFinalBa (okvis_ceres/src/ViSlamBackend.cpp:2005-2164) on the whole
graph: everything unfrozen (:2026-2033), redoPropagationAlways (:2036), SPARSE_NORMAL_CHOLESKY
(ViGraph.cpp:248) and optimiseFullGraph twice (:2041, :2059), each being (:1971-2003)
  1a  loop-closure RelativePoseErrors at 100 x information (:1985-1986), function_tolerance 1e-3,
      numIter / 3 iterations (:1988-1989);
  1b  the constraints removed, function_tolerance 1e-6, numIter iterations (:1990-1997);
and between the two calls the speed/bias prior is removed (:2044) and the extrinsics are
soft-constrained at their estimate (:2050-2052), then
  2   optimiseFullGraph again (:2059): its own 1a / 1b with the (already removed) constraints, i.e.
      a numIter-iteration solve at function_tolerance 1e-6.
numIter = 100 (okvis_multisensor_processing/src/ThreadedSlam.cpp:1539), so 33 / 100 / 100.

The window is Hilti-shaped: equidistant cameras (config/hilti22), both extrinsics variable with
their PoseError priors (do_extrinsics: true, config/hilti22/okvis2.yaml:82-83), loop-closure edges
from the last keyframes back to the first."""
import numpy as np

from _problem import OwnedProblem

ITERATIONS = {"1a": 33, "1b": 100, "2": 100}
FUNCTION_TOL = {"1a": 1e-3, "1b": 1e-6, "2": 1e-6}


def window(og, oracle, kf, lm, obs, seed):
    """The seeded Hilti-shaped window (a SynthWindow, equidistant keypoints placed by the oracle's
    projection so the synthetic noise is unchanged; see test_gpu_parity._switch_camera_model)."""
    from test_gpu_parity import CAMERA_MODELS, _switch_camera_model
    stride = kf - 40
    w = og.SynthWindow(kf, lm, obs, seed=seed, n_relpose=30, relpose_stride=stride, relpose_kind=1, do_extrinsics=1)
    _switch_camera_model(oracle, w, *CAMERA_MODELS["equidistant"])
    return w


def problem(w):
    """The protocol's own copy of the window with the loop closures at 100 x information."""
    q = OwnedProblem.copy_of(w.problem)
    assert np.all(q.extrinsics_constant == 0) and len(q.relpose_blocks) > 0
    q.relpose_sqrt_info = q.relpose_sqrt_info * 10.0
    q.bind()
    return q


def options(og, name, num_threads=16):
    return og.default_options(linear_solver=og.SPARSE_NORMAL_CHOLESKY, redo_propagation_always=1,
                              num_threads=num_threads, gradient_tolerance=1e-10, parameter_tolerance=1e-8,
                              max_num_iterations=ITERATIONS[name], function_tolerance=FUNCTION_TOL[name])


def before_pass(p, name):
    """The graph edits okvis makes before each pass (in place on the OwnedProblem)."""
    if name == "1b":  # removeRelativePoseConstraint
        p.relpose_blocks, p.relpose_delta_x = p.relpose_blocks[:0], p.relpose_delta_x[:0]
        p.relpose_sqrt_info, p.relpose_lin_point = p.relpose_sqrt_info[:0], p.relpose_lin_point[:0]
        p.relpose_kind = p.relpose_kind[:0]
        p.bind()
    if name == "2":  # removeSpeedAndBiasPrior + softConstrainExtrinsics
        p.sb_prior_block, p.sb_prior_meas, p.sb_prior_sqrt_info = (
            p.sb_prior_block[:0], p.sb_prior_meas[:0], p.sb_prior_sqrt_info[:0])
        p.extrinsics_prior_meas = p.extrinsics.copy()
        p.extrinsics_prior_sqrt_info = np.tile(np.diag([100.0] * 6).reshape(-1), (len(p.extrinsics), 1))
        p.bind()


PASSES = ("1a", "1b", "2")
