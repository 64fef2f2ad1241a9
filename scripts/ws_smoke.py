"""Development: one small and one S50 solve with the wave-specialised Cholesky schedule vs schedule 1."""
import sys
import time
sys.path.insert(0, 'okvis2-x_amd')
import numpy as np
import okvisgpu as og

for args in ((10, 500, 4000), (50, 2000, 16000)):
    res = []
    for sched in (1, 3):
        w = og.SynthWindow(*args, seed=7)
        c = og.Context(0)
        c.set_problems([w.problem])
        o = og.default_options(max_num_iterations=5, function_tolerance=0, gradient_tolerance=0, parameter_tolerance=0)
        o.cholesky_schedule = sched
        t = time.time()
        s = c.solve(o, 1)[0]
        res.append((s["final_cost"], w.poses().copy()))
        print(args, sched, s["final_cost"], s["termination"], f"{time.time() - t:.3f}s", flush=True)
        c.close()
    print("pose max diff", np.abs(res[0][1] - res[1][1]).max(), flush=True)
