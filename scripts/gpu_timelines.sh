#!/bin/bash
# Batched-iteration timelines (rocprofv3 kernel trace of short bench runs) at several window counts.
# Usage: bash scripts/gpu_timelines.sh TAG N1 [N2 ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; shift
for N in "$@"; do
  OUT=gpurun_out/$TAG/w$N
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-latency --no-profile --steps 5 --warmup 2 --windows $N > $OUT/bench.json 2> $OUT/bench.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench.err; exit 1; }
  echo "== $N windows: $(python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'], 3))")"
  python3 scripts/batch_iter_timeline.py $OUT/prof/run_kernel_trace.csv > $OUT/timeline.txt && cat $OUT/timeline.txt
done
