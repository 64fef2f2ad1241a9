#!/bin/bash
# GPU parity tests (optional) + a short default-workload bench with the per-kernel table.
# Usage (via gpurun): bash scripts/quick_bench.sh TAG [test]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" = "test" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
timeout -k 10 600 python bench.py --no-cpu --no-latency --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', round(d['value']), 'ms/it', round(d['ms_per_step'],3))
for k,v in d['kernels'].items(): print(f'{k:18s} {v[\"ms\"]:8.3f} ms  {v[\"frac\"]*100:5.1f}%')
"
