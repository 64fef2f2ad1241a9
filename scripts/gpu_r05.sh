#!/bin/bash
# Round-5 GPU round trip (via gpurun, from the repo root): the -m gpu suite (optionally a -k
# selection) with the parity report, then optionally a bench line.
# Usage: bash scripts/gpu_r05.sh TAG [pytest -k expr | all | none] [bench args | nobench]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
SEL=${2:-all}
if [ "$SEL" != "none" ]; then
  K=(); [ "$SEL" != "all" ] && K=(-k "$SEL")
  OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
if [ -n "$3" ] && [ "$3" != "nobench" ]; then
  timeout -k 10 500 python -u bench.py $3 > $OUT/bench.txt 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.txt; exit 1; }
  python3 -c "
import json,sys
l=[x for x in open('$OUT/bench.txt') if x.startswith('{')][-1]; d=json.loads(l)
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'chol', d['roofline'].get('ms_per_iteration'), 'frac', round(d['roofline']['frac'],4))
sw=d.get('single_window',{}); print('single', sw.get('iters_per_s'), {k:v for k,v in sw.items() if k.startswith('speedup')})
print('cpu', d.get('cpu_baseline',{}).get('value'), d.get('speedup_vs_cpu_baseline'))"
fi
