"""Single-window end-to-end latency split: okvisgpu_set_problems (host analysis + upload + graph
capture on the first solve) vs okvisgpu_solve, for one S50 window, repeated."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

w = og.SynthWindow(50, 2000, 16000, seed=20251015)
ctx = og.Context(0)
o = og.default_options(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
for rep in range(6):
    w.reset()
    t0 = time.perf_counter()
    ctx.set_problems([w.problem])
    t1 = time.perf_counter()
    s = ctx.solve(o)[0]
    t2 = time.perf_counter()
    s2 = ctx.solve(o)[0]  # same problem again: no analysis, graph reused
    t3 = time.perf_counter()
    print(f"rep {rep}: set_problems {1e3 * (t1 - t0):.2f} ms, first solve {1e3 * (t2 - t1):.2f} ms "
          f"({s['num_iterations']} it), repeat solve {1e3 * (t3 - t2):.2f} ms")
ctx.close()
