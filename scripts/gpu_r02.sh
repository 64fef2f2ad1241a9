#!/bin/bash
# Round-2 GPU round trip: the -m gpu suite, then the default bench.py line (driver command).
# Usage (via gpurun, from the repo root): bash scripts/gpu_r02.sh TAG [bench]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -40 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
if [ "$2" = "bench" ]; then
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
