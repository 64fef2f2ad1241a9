import sys
sys.path.insert(0, 'okvis2-x_amd'); sys.path.insert(0, 'tests')
import numpy as np, okvisgpu as og, _oracle as oracle
ctx = og.Context(0)
w = og.SynthWindow(50, 2000, 16000, seed=20251015)
opts = og.default_options(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
ctx.set_problems([w.problem]); sg = ctx.solve(opts, 1)[0]; L = w.landmarks().copy(); P = w.poses().copy()
w.reset(); so = oracle.solve(w.problem_ptr(), opts); L0 = w.landmarks().copy()
print(sg['final_cost'], so['final_cost'], sg['num_successful_steps'], so['num_successful_steps'])
p = w.problem
r, Jp, Jl = oracle.eval_reprojection(w.problem_ptr(), p.n_observations)
obs_lm = np.ctypeslib.as_array(p.obs_landmark, (p.n_observations,))
dev = np.abs(L[:, :3] - L0[:, :3]).max(1)
gt_p, gt_l, _ = w.ground_truth()
for l in np.argsort(-dev)[:6]:
    m = obs_lm == l
    V = np.zeros((3, 3))
    for o in np.where(m)[0]:
        s = r[o] @ r[o]; sc = 1 / (1 + s)
        V += sc * Jl[o].T @ Jl[o]
    ev = np.linalg.eigvalsh(V)
    d = L[l, :3] - L0[l, :3]
    print(l, f"dev {dev[l]:.3e} nobs {m.sum()} eig {ev} maha {np.sqrt(d @ V @ d):.3e} err_gt {np.linalg.norm(L0[l,:3]-gt_l[l,:3]):.3f} resid {np.sqrt((r[m]**2).sum(1)).max():.2f}")
