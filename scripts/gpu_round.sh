#!/bin/bash
# GPU round trip: the -m gpu suite, then the default bench line (strong scaling, 1 GPU) and the
# per-kernel table. Usage (from the repo root, via gpurun): bash scripts/gpu_round.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-dev}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "roofline", d.get("roofline", {}).get("kernel"), round(d.get("roofline", {}).get("frac", 0), 3))
print("single window", round(d.get("single_window", {}).get("iters_per_s", 0)), d.get("single_window", {}).get("kernel_ms_per_iteration"))
print("kernels", {k: v["ms"] for k, v in d.get("kernels", {}).items()})
print("cpu", d.get("cpu_baseline", {}).get("variants"))
PY
