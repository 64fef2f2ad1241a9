"""Final-BA size class (BASELINE config 4, ~500 keyframes) on one GPU: per-iteration time of one large
window for each Cholesky schedule, and the final-BA protocol end to end (two solves of up to 100
iterations, ViSlamBackend.cpp:2041,2059; tolerances 0 so every iteration runs; set_problems included).
Usage: python scripts/large_window.py [KF] [LM] [OBS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

kf, lm, obs = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (500, 20000, 160000)))
w = og.SynthWindow(kf, lm, obs, seed=20251015)
ctx = og.Context(0)
ctx.set_problems([w.problem])
res = {"keyframes": kf, "landmarks": lm, "observations": obs}
for sched in (2, 1, 3):
    w.reset()
    ctx.update_params()
    o = og.default_options(max_num_iterations=13, function_tolerance=0.0, gradient_tolerance=0.0,
                           parameter_tolerance=0.0, cholesky_schedule=sched)
    ctx.solve_begin(o)
    ctx.solve_iterate(3)
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.solve_iterate(10)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / 10
    s = ctx.solve_end(1)[0]
    w.reset()
    ctx.update_params()
    ctx.solve_begin(o)
    ctx.solve_iterate(3)
    ph = ctx.profile_iteration()
    ctx.solve_end(1)
    res[f"schedule_{sched}"] = {"ms_per_iteration": dt * 1e3, "final_cost": s["final_cost"],
                                "phases_ms": {k: round(v, 3) for k, v in ph.items() if v > 0.01}}
st = ctx.stats()
res["cholesky_launches"] = st["cholesky_launches"]
res["cholesky_split_windows"] = st["cholesky_split_windows"]
res["reduced_dim"] = st["reduced_dim"]
w.reset()
o = og.default_options(max_num_iterations=100, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
t0 = time.perf_counter()
for _ in range(2):
    ctx.set_problems([w.problem])
    s = ctx.solve(o)[0]
wall = time.perf_counter() - t0
res["final_ba_2x100"] = {"wall_s": wall, "iterations": 2 * 100, "ms_per_iteration": wall / 200 * 1e3,
                         "final_cost": s["final_cost"], "termination": s["termination"]}
print(json.dumps(res))
