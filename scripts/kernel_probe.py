"""Development: okvisgpu_time_kernel of the named kernels on N S50 windows of the bench's workload
after one solver iteration (library chosen with OKVISGPU_LIB, e.g. a phase-skipping timing build).
Usage: kernel_probe.py N name [name ...]"""
import os
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

n = int(sys.argv[1])
og = bench.og_module()
ws = bench.make_windows(bench.CONFIGS["s50"], range(n))
c = og.Context(0)
c.set_problems([w.problem for w in ws])
c.solve(og.default_options(max_num_iterations=1, function_tolerance=0, gradient_tolerance=0, parameter_tolerance=0,
                           cholesky_schedule=int(os.environ.get("OKG_PROBE_SCHED", "0"))), n)
print(" ".join(f"{k} {c.time_kernel(k, 5)[0]:.3f}" for k in sys.argv[2:]), flush=True)
c.close()
