#!/usr/bin/env python3
"""Generates the frozen parity fixtures of tests/test_golden.py (test infrastructure).

For each fixture: the seeded synthetic window (okvisgpu_synth_create) is built, a
SHA-256 of every input array is recorded (so a generator change is detected instead of silently
moving the target), and the CPU oracle (oracle/liboracle.so, the restatement of the reference's
functors + the Ceres DOGLEG / DENSE_SCHUR minimizer) solves it with all tolerances 0. The fixture
holds the summary, the final poses / speed-biases / landmarks and the initial cost.

Usage: python tests/golden/make_golden.py   (writes tests/golden/*.npz)"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _paths  # noqa: E402,F401
import okvisgpu as og  # noqa: E402
import _oracle  # noqa: E402
from _problem import OwnedProblem  # noqa: E402

FIXTURES = {
    "s10_seed20251015_it10": dict(kf=10, lm=500, obs=4000, seed=20251015, iters=10),
    "s50_seed20251015_it10": dict(kf=50, lm=2000, obs=16000, seed=20251015, iters=10),
}


# the inputs that define a window (fixed list, so that appending ABI fields or growing the IMU
# state layout does not move the digest; the IMU state of a fresh window is all zeros)
DIGEST_FIELDS = ("poses", "pose_constant", "speed_biases", "speed_bias_constant", "landmarks", "landmark_constant",
                 "extrinsics", "obs_pose", "obs_landmark", "obs_camera", "obs_keypoint", "obs_sqrt_info", "obs_cauchy",
                 "imu_blocks", "imu_t0_ns", "imu_t1_ns", "pose_prior_block", "pose_prior_meas", "pose_prior_sqrt_info",
                 "sb_prior_block", "sb_prior_meas", "sb_prior_sqrt_info", "relpose_blocks", "relpose_delta_x",
                 "relpose_sqrt_info", "relpose_lin_point", "relpose_kind")


def input_digest(problem, variable_extrinsics=False):
    """SHA-256 over the input arrays of a problem (DIGEST_FIELDS, then samples, cameras, IMU params;
    with variable_extrinsics also the extrinsics flags and priors)."""
    p = OwnedProblem.copy_of(problem)
    assert not np.any(p.imu_state), "a golden window starts from fresh IMU states"
    fields = DIGEST_FIELDS
    if variable_extrinsics:
        fields = fields + ("extrinsics_constant", "extrinsics_prior_camera", "extrinsics_prior_meas",
                           "extrinsics_prior_sqrt_info")
    else:
        assert np.all(p.extrinsics_constant == 1), "golden windows have constant extrinsics"
    h = hashlib.sha256()
    for k in fields:
        h.update(k.encode())
        h.update(np.ascontiguousarray(getattr(p, k)).tobytes())
    for a in (p.imu_sample_begin, p.imu_sample_t_ns, p.imu_sample_gyr_acc):
        h.update(np.ascontiguousarray(a).tobytes())
    for c in p.cameras:  # field values (not struct bytes: padding)
        h.update(np.array([c.distortion, c.width, c.height], np.int64).tobytes())
        h.update(np.array([c.fu, c.fv, c.cu, c.cv] + list(c.dist), np.float64).tobytes())
    ip = p.imu_params
    h.update(np.array([getattr(ip, k) for k, _ in ip._fields_], np.float64).tobytes())
    return h.hexdigest()


def options(iters):
    return og.default_options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0, num_threads=1)


def window(cfg):
    return og.SynthWindow(cfg["kf"], cfg["lm"], cfg["obs"], seed=cfg["seed"])


def main():
    for name, cfg in FIXTURES.items():
        w = window(cfg)
        digest = input_digest(w.problem)
        s = _oracle.solve(w.problem_ptr(), options(cfg["iters"]))
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(
            path, input_sha256=np.array(digest), kf=cfg["kf"], lm=cfg["lm"], obs=cfg["obs"], seed=cfg["seed"],
            iters=cfg["iters"], initial_cost=s["initial_cost"], final_cost=s["final_cost"],
            num_iterations=s["num_iterations"], num_successful_steps=s["num_successful_steps"],
            termination_type=s["termination_type"], poses=w.poses().copy(), speed_biases=w.speed_biases().copy(),
            landmarks=w.landmarks().copy())
        print(name, digest[:16], s["final_cost"], os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
