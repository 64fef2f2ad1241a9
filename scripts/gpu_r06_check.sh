#!/bin/bash
# Check run on the current library: the whole -m gpu suite with the parity report, then the
# single-window probes (S50 / S10).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06chk}; mkdir -p $OUT
OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2; do for shape in "50 2000 16000" "10 500 4000"; do
  timeout -k 10 120 python scripts/imu_probe.py $shape | tee -a $OUT/probe.txt || exit 1
done; done
