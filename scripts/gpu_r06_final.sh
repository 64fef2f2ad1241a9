#!/bin/bash
# Round-6 closing run (via gpurun): the -m gpu suite with the parity report, the profile set
# (scripts/gpu_r06_prof.sh: MFMA counters, PMC traffic, default bench + rocprofv3 trace, windows
# per GPU) and the S10 bench line. Usage: bash scripts/gpu_r06_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r06z}
OUT=gpurun_out/$TAG; mkdir -p $OUT
OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
bash scripts/gpu_r06_prof.sh $TAG || exit 1
timeout -k 10 600 python bench.py --config s10 > $OUT/bench_s10.json 2> $OUT/bench_s10.err || { echo "s10 rc=$?"; tail -20 $OUT/bench_s10.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench_s10.json').read().strip().splitlines()[-1])
sw=d['single_window']
print('s10 value', round(d['value']), 'single', round(sw['iters_per_s']), 'x3', round(sw.get('speedup_vs_cpu_3_threads', 0), 2))"
