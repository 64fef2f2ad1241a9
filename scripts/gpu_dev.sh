#!/bin/bash
# Development round trip: -m gpu suite, single-window rates per Cholesky schedule, optional
# phase clocks (lib_clk.so) and a short default bench. Usage: bash scripts/gpu_dev.sh TAG [clk] [bench]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for s in 0 1 2 3; do timeout -k 10 120 python scripts/single_window.py 50 $s >> $OUT/single.txt 2>&1 || { cat $OUT/single.txt; exit 1; }; done
cat $OUT/single.txt
if [[ " $* " == *" clk "* ]]; then
  for s in 1 2; do OKVISGPU_LIB=$PWD/okvis2-x_amd/lib_clk.so timeout -k 10 120 python scripts/clk_probe.py 1 $s || exit 1; done
fi
if [[ " $* " == *" bench "* ]]; then
  timeout -k 10 600 python bench.py --no-cpu --no-profile > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'single',d['single_window']['iters_per_s'],d['single_window']['e2e_set_problems_plus_solve_ms'])"
fi
