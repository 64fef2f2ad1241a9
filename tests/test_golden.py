"""Frozen parity fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py): oracle
solves of one S10 and one S50 synthetic window, 10 iterations, all tolerances 0.

* CPU: the generator still produces the recorded inputs (SHA-256 of every input array), and the
  oracle still reproduces the recorded solve — a change to either shows up here instead of moving
  the parity target silently.
* GPU: the HIP path through the C ABI against the frozen solve (SURVEY.md §8c contract:
  iterations / termination exact, final cost 1e-7 relative, positions 1e-6 m)."""
import glob
import os

import numpy as np
import pytest

from _paths import REPO

GOLDEN = sorted(p for p in glob.glob(os.path.join(REPO, "tests", "golden", "*.npz"))
                if not os.path.basename(p).startswith("final_ba_"))  # (those: test_final_ba_golden.py)


def _load(path):
    return dict(np.load(path, allow_pickle=False))


def _window(og, g):
    return og.SynthWindow(int(g["kf"]), int(g["lm"]), int(g["obs"]), seed=int(g["seed"]))


def _opts(og, g, threads=1):
    return og.default_options(max_num_iterations=int(g["iters"]), function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0, num_threads=threads)


def _check(s, P, L, g, rel=1e-7):
    assert s["num_iterations"] == int(g["num_iterations"])
    assert s["termination_type"] == int(g["termination_type"])
    assert s["num_successful_steps"] == int(g["num_successful_steps"])
    assert abs(s["initial_cost"] - float(g["initial_cost"])) <= 1e-10 * float(g["initial_cost"])
    assert abs(s["final_cost"] - float(g["final_cost"])) <= rel * float(g["final_cost"]), (s, float(g["final_cost"]))
    assert np.abs(P[:, :3] - g["poses"][:, :3]).max() <= 1e-6


def test_golden_fixtures_present():
    assert len(GOLDEN) >= 2


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_generator_reproduces_golden_inputs(og, path):
    sys_path = os.path.join(REPO, "tests", "golden")
    import sys
    sys.path.insert(0, sys_path)
    from make_golden import input_digest
    g = _load(path)
    w = _window(og, g)
    assert input_digest(w.problem) == str(g["input_sha256"])


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
@pytest.mark.parametrize("threads", [1, 4])
def test_oracle_reproduces_golden(og, oracle, path, threads):
    g = _load(path)
    w = _window(og, g)
    s = oracle.solve(w.problem_ptr(), _opts(og, g, threads))
    _check(s, w.poses(), w.landmarks(), g)


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_gpu_matches_golden(og, gpu_ctx, path):
    g = _load(path)
    w = _window(og, g)
    gpu_ctx.set_problems([w.problem])
    s = gpu_ctx.solve(_opts(og, g))[0]
    _check(s, w.poses(), w.landmarks(), g)
