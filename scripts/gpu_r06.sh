#!/bin/bash
# Round-6 GPU run (via gpurun): the -m gpu suite with the parity report, then the default bench line.
# Usage: bash scripts/gpu_r06.sh TAG [pytest selection]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r06}
SEL=${2:-tests}
OUT=gpurun_out/$TAG; mkdir -p $OUT
OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$OUT/bench.json").read().strip().splitlines()[-1])
r = d.get("roofline", {})
sw = d.get("single_window", {})
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "roofline", r.get("kernel"), round(r.get("frac", 0), 4),
      "issued", r.get("frac_issued"), "ms", r.get("ms_per_iteration"), "single", round(sw.get("iters_per_s", 0)))
PY
