#!/bin/bash
# GPU suite + single-window rate + short default bench (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 120 python scripts/single_window.py 50 0 > $OUT/single.txt 2>&1 || { cat $OUT/single.txt; exit 1; }
cat $OUT/single.txt
timeout -k 10 600 python bench.py --no-cpu --no-profile > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'single',d['single_window']['iters_per_s'],d['single_window']['e2e_set_problems_plus_solve_ms'])"
