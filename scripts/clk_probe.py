"""Development: per-phase clocks of a Cholesky schedule (library built with -DOKG_CHOL_CLOCK,
selected by OKVISGPU_LIB). Usage: clk_probe.py N_WINDOWS SCHED"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

n, sched = int(sys.argv[1]), int(sys.argv[2])
ws = [og.SynthWindow(50, 2000, 16000, seed=20251015 + i) for i in range(n)]
c = og.Context(0)
c.set_problems([w.problem for w in ws])
o = og.default_options(max_num_iterations=int(sys.argv[3]) if len(sys.argv) > 3 else 1, function_tolerance=0, gradient_tolerance=0, parameter_tolerance=0)
o.cholesky_schedule = sched
c.solve(o, n)
c.close()
print("windows", n, "sched", sched)
