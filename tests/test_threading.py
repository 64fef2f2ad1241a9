"""The §8b threading contract: one okvisgpu_ctx per graph, entry points re-entrant across contexts
(VERDICT r03 item 2). okvis runs the realtime solve and the full-graph solve concurrently on two
graphs from two threads (ThreadedSlam.cpp:945 optimiseRealtimeGraph, :955 optimiseFullGraph):

  realtime   an S50 window, DENSE_SCHUR (ViSlamBackend.cpp:877), 10 iterations;
  full graph a 200-keyframe graph with a GPS-shaped host-evaluated factor per keyframe (the §8b
             fallback, callbacks on 3 host threads), SPARSE_NORMAL_CHOLESKY (ViGraph.cpp:248).

Each graph is solved alone first, then both at once from two Python threads (ctypes releases the
GIL inside okvisgpu_set_problems / okvisgpu_solve; the GPS callbacks take it) — three rounds, each
result bitwise equal to the solo run — and each is matched to the oracle."""
import threading

import numpy as np
import pytest

from _gps import gps_window
from _problem import OwnedProblem


def _opts(og, iters, **kw):
    return og.default_options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0, **kw)


class Graph:
    def __init__(self, og, problem, opts):
        self.og, self.problem, self.opts = og, problem, opts
        self.snap = problem.snapshot()
        self.ctx = og.Context(0)

    def run(self):
        """ViGraph::optimise: (re)upload the graph, solve, read the result back."""
        self.problem.restore(self.snap)
        self.ctx.set_problems([self.problem.struct])
        s = self.ctx.solve(self.opts)[0]
        return s, {k: getattr(self.problem, k).copy() for k in ("poses", "speed_biases", "landmarks", "imu_state")}

    def close(self):
        self.ctx.close()


def _bitwise(a, b, what):
    sa, xa = a
    sb, xb = b
    for k in ("num_iterations", "termination", "num_successful_steps", "initial_cost", "final_cost"):
        assert sa[k] == sb[k], (what, k, sa[k], sb[k])
    for k in xa:
        assert np.array_equal(xa[k], xb[k]), (what, k)


@pytest.mark.gpu
def test_two_graphs_concurrently(og, oracle, parity):
    sw = og.SynthWindow(50, 2000, 16000, seed=20251015)  # (kept alive while its arrays are copied)
    rt = OwnedProblem.copy_of(sw.problem)
    del sw
    fg, gps, _ = gps_window(seed=9, n_kf=200, n_lm=8000, n_obs=64000)
    graphs = {"realtime": Graph(og, rt, _opts(og, 10, num_threads=3)),
              "full": Graph(og, fg, _opts(og, 3, num_threads=3, linear_solver=og.SPARSE_NORMAL_CHOLESKY))}
    try:
        solo = {name: g.run() for name, g in graphs.items()}
        calls_solo = gps.calls
        assert calls_solo > 0
        for rnd in range(3):
            out, errs = {}, []

            def work(name):
                try:
                    out[name] = graphs[name].run()
                except Exception as e:  # noqa: BLE001 (reported below)
                    errs.append((name, repr(e)))

            ts = [threading.Thread(target=work, args=(n,)) for n in graphs]
            for t in ts:
                t.start()
            for t in ts:
                t.join(timeout=300)
            assert not errs and not any(t.is_alive() for t in ts), errs
            for name in graphs:
                _bitwise(out[name], solo[name], (rnd, name))
        # and each graph against the oracle
        for name, g in graphs.items():
            s, x = solo[name]
            g.problem.restore(g.snap)
            so = oracle.solve(g.problem.ptr(), g.opts)
            assert s["num_iterations"] == so["num_iterations"] and s["termination"] == so["termination"], (name, s, so)
            dc = abs(s["final_cost"] - so["final_cost"]) / so["final_cost"]
            dp = float(np.abs(x["poses"][:, :3] - g.problem.poses[:, :3]).max())
            parity(f"threading_{name}_cost_rel", dc, 1e-7 if name == "realtime" else 1e-6)
            parity(f"threading_{name}_pose_m", dp, 1e-6)
    finally:
        for g in graphs.values():
            g.close()
