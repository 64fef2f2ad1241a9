#!/bin/bash
# Cholesky schedules against window counts (bench value, no profiling).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for N in ${WINDOWS:-256 512}; do
  for S in ${SCHEDS:-1 2 3}; do
    v=$(timeout -k 10 200 python bench.py --no-cpu --no-latency --no-profile --steps 10 --warmup 3 --windows $N --cholesky-schedule $S 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3))") || exit 1
    echo "windows $N sched $S: $v"
  done
done
