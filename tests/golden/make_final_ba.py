#!/usr/bin/env python3
"""Generates the final-BA protocol fixture of tests/test_final_ba_golden.py (test infrastructure).

BASELINE config 4 as okvis runs it (tests/_final_ba.py: ViSlamBackend::doFinalBa,
ViSlamBackend.cpp:1971-2059, numIter = 100 from ThreadedSlam.cpp:1539): a Hilti-shaped seeded window
solved by the CPU oracle (oracle/liboracle.so) through the passes 1a / 1b / 2 at the reference's
iteration counts 33 / 100 / 100 with redoPropagationAlways. The fixture holds the SHA-256 of the
window's inputs and, after every pass, the summary (initial / final cost, iterations, successful
steps, termination), the poses, speed/biases and extrinsics. The oracle is deterministic for any
thread count (fixed-order reductions), which the CPU test re-checks on a cut protocol.

Usage: python tests/golden/make_final_ba.py [--kf 200]   (writes tests/golden/final_ba_*.npz)"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import _paths  # noqa: E402,F401
import okvisgpu as og  # noqa: E402
import _oracle  # noqa: E402
import _final_ba as fba  # noqa: E402
from make_golden import input_digest  # noqa: E402

SHAPES = {200: dict(kf=200, lm=8000, obs=64000, seed=48), 500: dict(kf=500, lm=20000, obs=160000, seed=48)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kf", type=int, default=200, choices=sorted(SHAPES))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    cfg = SHAPES[a.kf]
    w = fba.window(og, _oracle, cfg["kf"], cfg["lm"], cfg["obs"], cfg["seed"])
    digest = input_digest(w.problem, variable_extrinsics=True)
    q = fba.problem(w)
    out = dict(input_sha256=np.array(digest), **{k: v for k, v in cfg.items()})
    for name in fba.PASSES:
        fba.before_pass(q, name)
        t0 = time.perf_counter()
        s = _oracle.solve(q.ptr(), fba.options(og, name, a.threads))
        dt = time.perf_counter() - t0
        for k in ("initial_cost", "final_cost", "num_iterations", "num_successful_steps", "termination_type"):
            out[f"p{name}_{k}"] = s[k]
        out[f"p{name}_poses"] = q.poses.copy()
        out[f"p{name}_speed_biases"] = q.speed_biases.copy()
        out[f"p{name}_extrinsics"] = q.extrinsics.copy()
        print(f"pass {name}: {s['num_iterations']} it ({s['num_successful_steps']} successful), "
              f"{s['termination']}, cost {s['initial_cost']:.10g} -> {s['final_cost']:.10g}, {dt:.1f} s", flush=True)
    path = os.path.join(HERE, f"final_ba_s{a.kf}_seed{cfg['seed']}.npz")
    np.savez_compressed(path, **out)
    print(path, digest[:16], os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
