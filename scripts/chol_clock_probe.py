"""Development: per-phase clock of the Cholesky (workgroup 0's window) in a batch of N S50 windows.
Run with OKVISGPU_LIB=okvis2-x_amd/lib_cclk.so (scripts/build_variant.sh cclk -DOKG_CHOL_CLOCK).
Usage: python scripts/chol_clock_probe.py N SCHED"""
import sys
sys.path.insert(0, 'okvis2-x_amd')
import okvisgpu as og
n, sched = int(sys.argv[1]), int(sys.argv[2])
ws = [og.SynthWindow(50, 2000, 16000, seed=20251015 + i % 64) for i in range(n)]
c = og.Context(0)
c.set_problems([w.problem for w in ws])
o = og.default_options(max_num_iterations=1, function_tolerance=0, gradient_tolerance=0, parameter_tolerance=0)
o.cholesky_schedule = sched
c.solve(o, n)
c.close()
print("windows", n, "schedule", sched, flush=True)
