#!/bin/bash
# Throughput vs batch size for both Cholesky schedules (strong-scaling shares of one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for n in ${WINDOWS:-8 32 64 128 256 512}; do for sch in ${SCHEDULES:-1 2}; do
  timeout -k 10 300 python bench.py --windows $n --cholesky-schedule $sch --no-cpu --no-latency --no-profile --steps 10 --warmup 3 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print($n, $sch, round(d['value']), round(d['ms_per_step'],3))" || exit 1
done; done
