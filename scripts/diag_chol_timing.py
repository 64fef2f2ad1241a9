import sys; sys.path.insert(0,'okvis2-x_amd')
import okvisgpu as og
w=og.SynthWindow(50,2000,16000,seed=20251015)
c=og.Context(0); c.set_problems([w.problem])
c.solve(og.default_options(max_num_iterations=1,function_tolerance=0,gradient_tolerance=0,parameter_tolerance=0), 1); c.close()
