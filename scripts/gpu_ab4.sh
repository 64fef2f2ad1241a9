#!/bin/bash
# GPU: -m gpu suite, then 256-window bench lines with Cholesky schedules 4 and 1 (A/B, twice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | head -30; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2; do for s in 4 1; do
  timeout -k 10 300 python3 bench.py --windows 256 --steps 20 --no-cpu --no-latency --cholesky-schedule $s > $OUT/b256_$s.json 2>$OUT/b256_$s.err || { tail -5 $OUT/b256_$s.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/b256_$s.json').read().strip().splitlines()[-1]);print('w256 sched $s', round(d['value']), round(d['ms_per_step'],3), d['kernels']['k_cholesky']['ms'])"
done; done
