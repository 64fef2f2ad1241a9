"""Development: per-phase clocks of k_eval_imu (library built with -DOKG_IMU_CLOCK, selected by
OKVISGPU_LIB): one forced re-integration launch over N S50 windows. Usage: imu_clk_probe.py N"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

n = int(sys.argv[1])
ws = [og.SynthWindow(50, 2000, 16000, seed=20251015 + i) for i in range(n)]
c = og.Context(0)
c.set_problems([w.problem for w in ws])
o = og.default_options(max_num_iterations=1, function_tolerance=0, gradient_tolerance=0, parameter_tolerance=0)
c.solve(o, n)
print("time_kernel k_eval_imu", c.time_kernel("k_eval_imu", 1), flush=True)
c.close()
