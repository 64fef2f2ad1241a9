#!/bin/bash
# Default bench.py run (the driver's command) plus a rocprofv3 kernel-trace of the same command.
# Usage (via gpurun, from the repo root): bash scripts/gpu_bench.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench_prof.err; exit 1; }
echo prof-ok
