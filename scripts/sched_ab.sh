#!/bin/bash
# Cholesky schedule A/B on the default workload. Usage (via gpurun): bash scripts/sched_ab.sh TAG "1 2 3"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for s in $2; do
  timeout -k 10 300 python bench.py --no-cpu --no-latency --steps 10 --warmup 3 --cholesky-schedule $s ${3:-} > $OUT/bench_$s.json 2> $OUT/bench_$s.err || { echo "bench $s rc=$?"; tail -20 $OUT/bench_$s.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$s.json').read().strip().splitlines()[-1])
print('schedule $s value', round(d['value']), 'ms/it', round(d['ms_per_step'],3), 'cholesky', d['kernels']['k_cholesky']['ms'])
"
done
