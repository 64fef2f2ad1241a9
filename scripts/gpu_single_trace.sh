#!/bin/bash
# Single-window kernel trace (default schedule): rocprofv3 kernel trace of 20 resident iterations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-single}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python scripts/single_window.py 20 ${2:-0} > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cat $OUT/prof.log | tail -2
