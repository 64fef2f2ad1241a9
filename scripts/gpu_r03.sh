#!/bin/bash
# Round-3 GPU round trip (via gpurun, from the repo root): the -m gpu suite with the parity report,
# the default bench line, and a rocprofv3 kernel trace + stats of the same bench command.
# Usage: bash scripts/gpu_r03.sh TAG [notest]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "notest" ]; then
  OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "roofline", d.get("roofline", {}).get("kernel"), round(d.get("roofline", {}).get("frac", 0), 3))
print("single window", round(d.get("single_window", {}).get("iters_per_s", 0)), d.get("single_window", {}).get("kernel_ms_per_iteration"))
print("kernels", {k: v["ms"] for k, v in d.get("kernels", {}).items()})
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench_prof.err; exit 1; }
python3 scripts/kstats_grouped.py $OUT/prof/run_kernel_trace.csv 40 > $OUT/kernel_trace_grouped.txt
echo prof-ok
