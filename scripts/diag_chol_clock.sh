#!/bin/bash
# Development: per-phase clock of the persistent Cholesky (workgroup 0), 1 and N windows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
make -s -C okvis2-x_amd clean && make -s -C okvis2-x_amd -j16 OPT="-O3 -DOKG_CHOL_CLOCK" || exit 1
for n in ${CLKWINDOWS:-1 64 512}; do
timeout -k 10 300 python - $n ${SCHED:-3} <<'PY' || exit 1
import sys; sys.path.insert(0, 'okvis2-x_amd')
import okvisgpu as og
n = int(sys.argv[1])
ws = [og.SynthWindow(50, 2000, 16000, seed=20251015 + i) for i in range(n)]
c = og.Context(0); c.set_problems([w.problem for w in ws])
o = og.default_options(max_num_iterations=1, function_tolerance=0, gradient_tolerance=0, parameter_tolerance=0)
o.cholesky_schedule = int(sys.argv[2]) if len(sys.argv) > 2 else 1
c.solve(o, n); c.close()
print("windows", n)
PY
done
