"""IMU phase clock (lib_iclk.so, -DOKG_IMU_CLOCK): forced re-integration of one window's factors as the
solve evaluates them; the kernel prints the per-phase tick sums of its wavefronts (x10 ns)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

kf, lm, obs, nwin = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (50, 2000, 16000, 1)))
ws = [og.SynthWindow(kf, lm, obs, seed=20251015 + i) for i in range(nwin)]
ctx = og.Context(0)
ctx.set_problems([w.problem for w in ws])
ctx.solve(og.default_options(max_num_iterations=1))
print("waves", (ws[0].problem.n_imu * nwin + 3) // 4, flush=True)
ctx.time_kernel("k_eval_imu", 3)
ctx.close()
