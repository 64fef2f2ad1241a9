"""The final-BA protocol at the reference's iteration counts (BASELINE config 4), against frozen
oracle fixtures (tests/golden/final_ba_*.npz, written by tests/golden/make_final_ba.py).

tests/_final_ba.py restates ViSlamBackend::doFinalBa (ViSlamBackend.cpp:1971-2059; numIter = 100,
ThreadedSlam.cpp:1539): passes 1a / 1b / 2 at 33 / 100 / 100 iterations with redoPropagationAlways
on a Hilti-shaped window (equidistant cameras, variable extrinsics, loop-closure edges at 100 x
information). The GPU carries its own estimates and IMU preintegration states from pass to pass,
like okvis does, and every pass is compared with the oracle's pass of the fixture: iterations,
termination and successful steps exact, cost 1e-7 relative, positions and extrinsics 1e-6 m.

* CPU: the generator still produces the fixture's inputs (SHA-256 of every input array).
* GPU (-m gpu): the protocol through the C ABI against both fixtures (200 and 500 keyframes)."""
import glob
import os

import numpy as np
import pytest

import _final_ba as fba
from _paths import REPO

GOLDEN = sorted(glob.glob(os.path.join(REPO, "tests", "golden", "final_ba_*.npz")))


def _load(path):
    return dict(np.load(path, allow_pickle=False))


def _window(og, oracle, g):
    return fba.window(og, oracle, int(g["kf"]), int(g["lm"]), int(g["obs"]), int(g["seed"]))


def test_final_ba_fixtures_present():
    assert {os.path.basename(p) for p in GOLDEN} >= {"final_ba_s200_seed48.npz", "final_ba_s500_seed48.npz"}


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_generator_reproduces_final_ba_inputs(og, oracle, path):
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from make_golden import input_digest
    g = _load(path)
    w = _window(og, oracle, g)
    assert input_digest(w.problem, variable_extrinsics=True) == str(g["input_sha256"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_final_ba_protocol_matches_fixture(og, oracle, gpu_ctx, parity, path):
    g = _load(path)
    kf = int(g["kf"])
    q = fba.problem(_window(og, oracle, g))
    for name in fba.PASSES:
        fba.before_pass(q, name)
        gpu_ctx.set_problems([q.struct])
        s = gpu_ctx.solve(fba.options(og, name))[0]
        pre = f"p{name}_"
        for k in ("num_iterations", "termination_type", "num_successful_steps"):
            assert s[k] == int(g[pre + k]), (name, k, s[k], int(g[pre + k]))
        print(f"S{kf} final BA pass {name}: {s['num_iterations']} it, {s['termination']}, "
              f"cost {s['final_cost']:.10g} (fixture {float(g[pre + 'final_cost']):.10g})")
        parity(f"final BA S{kf} pass {name}: initial cost (rel)",
               abs(s["initial_cost"] - float(g[pre + "initial_cost"])) / float(g[pre + "initial_cost"]), 1e-7)
        parity(f"final BA S{kf} pass {name}: final cost (rel)",
               abs(s["final_cost"] - float(g[pre + "final_cost"])) / float(g[pre + "final_cost"]), 1e-7)
        parity(f"final BA S{kf} pass {name}: positions (m)",
               float(np.abs(q.poses[:, :3] - g[pre + "poses"][:, :3]).max()), 1e-6)
        parity(f"final BA S{kf} pass {name}: extrinsics translation (m)",
               float(np.abs(q.extrinsics[:, :3] - g[pre + "extrinsics"][:, :3]).max()), 1e-6)
        parity(f"final BA S{kf} pass {name}: speed/biases (abs)",
               float(np.abs(q.speed_biases - g[pre + "speed_biases"]).max()), 1e-5)
