"""Single-window IMU latency probe (A/B of the few-window IMU chunking; OKVISGPU_LIB selects the
library): forced re-integration of every factor of one window (okvisgpu_time_kernel k_eval_imu, as
the solve evaluates it), the graph-launched time of the leading re-integrating iterations, the
steady-state rate, and the final cost (bits). Usage: imu_probe.py KF LM OBS"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

kf, lm, obs = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (50, 2000, 16000)))
w = og.SynthWindow(kf, lm, obs, seed=20251015)
ctx = og.Context(0)
ctx.set_problems([w.problem])
o = og.default_options(max_num_iterations=40, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)


def graph_ms(start, n):
    w.reset()
    ctx.update_params()
    ctx.solve_begin(o)
    ctx.solve_iterate(start)
    ctx.synchronize()
    a = time.perf_counter()
    ctx.solve_iterate(n)
    ctx.synchronize()
    dt = (time.perf_counter() - a) / n * 1e3
    s = ctx.solve_end()[0]
    return dt, s


first = min(graph_ms(0, 2)[0] for _ in range(5))
steady = min(graph_ms(8, 30)[0] for _ in range(3))
_, s = graph_ms(0, 40)
w.reset()
ctx.update_params()
forced = ctx.time_kernel("k_eval_imu", 20)[0]
print(f"S{kf}: forced re-integration {forced * 1e3:.1f} us, iterations 1-2 {first:.4f} ms/it, steady {steady:.4f} ms/it, "
      f"final cost {s['final_cost']!r}")
ctx.close()
