#!/bin/bash
# Round-4 GPU round trip (via gpurun, from the repo root): optional probe, the -m gpu suite with the
# parity report, then an A/B of library variants (scripts/lib_ab.sh).
# Usage: bash scripts/gpu_r04.sh TAG [tests|notest] ["base variant ..."]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -x scripts/simd_probe ]; then timeout -k 10 60 ./scripts/simd_probe > $OUT/simd_probe.txt 2>&1 || echo "probe rc=$?"; fi
if [ "$2" != "notest" ]; then
  OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
if [ -n "$3" ]; then bash scripts/lib_ab.sh $TAG "$3" || exit 1; fi
