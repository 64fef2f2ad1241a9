#!/bin/bash
# Single-window latency: it/s per Cholesky schedule, then a kernel trace of the default schedule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-single}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in 0 1 2 3; do timeout -k 10 120 python scripts/single_window.py 50 $s >> $OUT/rates.txt 2>&1 || exit 1; done
cat $OUT/rates.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python scripts/single_window.py 20 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo prof-ok
