set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for s in 1 3; do
OKVISGPU_LIB=okvis2-x_amd/lib_clk.so timeout -k 10 120 python - $s <<'PY'
import sys; sys.path.insert(0, 'okvis2-x_amd')
import okvisgpu as og
w = og.SynthWindow(50, 2000, 16000, seed=20251015)
c = og.Context(0); c.set_problems([w.problem])
o = og.default_options(max_num_iterations=1, function_tolerance=0, gradient_tolerance=0, parameter_tolerance=0)
o.cholesky_schedule = int(sys.argv[1])
c.solve(o); c.close()
PY
done
