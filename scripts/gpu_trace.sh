#!/bin/bash
# rocprofv3 kernel trace of the timed bench loop only (no roofline/latency/CPU legs).
# Usage (via gpurun): bash scripts/gpu_trace.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-trace}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-latency --no-profile ${*:---steps 10 --warmup 3} > $OUT/bench.json 2> $OUT/bench.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python3 scripts/kstats.py $OUT/prof/run_kernel_stats.csv 30
