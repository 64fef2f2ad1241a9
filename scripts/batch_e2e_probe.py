"""Batched per-solve split (what bench.py's per_solve_incl_pcie sums): update_params, solve_begin
(options, graph capture, parameter upload, iteration 0), the 13 iterations, solve_end (state read,
write-back) for N S50 windows. Usage: python scripts/batch_e2e_probe.py [N]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
ws = [og.SynthWindow(50, 2000, 16000, seed=20251015 + i) for i in range(n)]
ctx = og.Context(0)
L = og.lib()
t = time.perf_counter()
ctx.set_problems([w.problem for w in ws])
print(f"set_problems {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
o = og.default_options(max_num_iterations=13, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
sums = (og.Summary * n)()
for rep in range(4):
    for w in ws:
        w.reset()
    t0 = time.perf_counter()
    assert L.okvisgpu_update_params(ctx.h) == 0
    t1 = time.perf_counter()
    assert L.okvisgpu_solve_begin(ctx.h, C.byref(o)) == 0
    assert L.okvisgpu_synchronize(ctx.h) == 0
    t2 = time.perf_counter()
    assert L.okvisgpu_solve_iterate(ctx.h, 13) == 0
    assert L.okvisgpu_synchronize(ctx.h) == 0
    t3 = time.perf_counter()
    assert L.okvisgpu_solve_end(ctx.h, sums) == 0
    t4 = time.perf_counter()
    print(f"rep {rep}: update_params {1e3 * (t1 - t0):.1f} ms, solve_begin {1e3 * (t2 - t1):.1f} ms, "
          f"13 iterations {1e3 * (t3 - t2):.1f} ms, solve_end {1e3 * (t4 - t3):.1f} ms", flush=True)
ctx.close()
