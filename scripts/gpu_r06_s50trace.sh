#!/bin/bash
# Kernel trace of one S50 window (50 resident iterations after 3): per-kernel averages and the
# timeline of the last launches (busy vs idle, the largest gaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06s50tr}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python scripts/single_window.py 50 0 > $OUT/out.txt 2>&1 || exit 1
tail -1 $OUT/out.txt
python3 scripts/ktimeline.py $(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | head -1) 300 > $OUT/timeline.txt || exit 1
head -30 $OUT/timeline.txt
