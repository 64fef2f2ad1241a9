#!/bin/bash
# Single-window latency by Cholesky schedule (S10 and S50, 50 timed iterations after 3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05s}; mkdir -p $OUT
for shape in "10 500 4000" "50 2000 16000"; do for s in 0 1 2 4; do
  timeout -k 10 120 python scripts/single_window.py 50 $s $shape >> $OUT/single.txt 2>&1 || { echo "single $shape $s rc=$?"; tail -5 $OUT/single.txt; exit 1; }
done; done
cat $OUT/single.txt
