"""Single-window latency probe: one S50 window (the reference's own use: one window per solve),
K resident iterations timed between two synchronisations; for rocprofv3 --kernel-trace."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sched = int(sys.argv[2]) if len(sys.argv) > 2 else 0
kf, lm, obs = (int(x) for x in (sys.argv[3:6] if len(sys.argv) > 5 else (50, 2000, 16000)))
w = og.SynthWindow(kf, lm, obs, seed=20251015)
ctx = og.Context(0)
ctx.set_problems([w.problem])
o = og.default_options(max_num_iterations=n + 3, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0,
                       cholesky_schedule=sched)
ctx.solve_begin(o)
ctx.solve_iterate(3)
ctx.synchronize()
t0 = time.perf_counter()
ctx.solve_iterate(n)
ctx.synchronize()
dt = time.perf_counter() - t0
s = ctx.solve_end()[0]
st = ctx.stats()
print(f"sched {sched}: {n / dt:.1f} it/s, {dt / n * 1e3:.3f} ms/it, final cost {s['final_cost']!r}, "
      f"{st['cholesky_launches']} cholesky launches, {st['s_tiles_nonzero']} tiles, dim {st['reduced_dim']}")
ctx.close()
