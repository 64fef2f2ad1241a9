import sys, os
sys.path.insert(0, 'okvis2-x_amd'); sys.path.insert(0, 'tests')
import numpy as np, okvisgpu as og, _oracle as oracle
ctx = og.Context(0)
for cfg in [(6, 150, 1000, 11), (3, 40, 200, 13)]:
    for it in range(1, 7):
        w = og.SynthWindow(cfg[0], cfg[1], cfg[2], seed=cfg[3])
        opts = og.default_options(max_num_iterations=it, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
        ctx.set_problems([w.problem]); sg = ctx.solve(opts, 1)[0]; P = w.poses().copy()
        w.reset(); so = oracle.solve(w.problem_ptr(), opts)
        print(cfg[0], it, sg['num_successful_steps'], so['num_successful_steps'], f"{sg['final_cost']:.12g} {so['final_cost']:.12g} rel {abs(sg['final_cost']-so['final_cost'])/so['final_cost']:.2e} dpos {np.abs(P[:,:3]-w.poses()[:,:3]).max():.2e} radius {sg['final_radius']:.3g} {so['final_radius']:.3g}")
