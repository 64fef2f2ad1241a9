#!/bin/bash
# A/B of an environment knob on the default workload (bench per-kernel table).
# Usage (via gpurun): bash scripts/env_ab.sh TAG VAR "v1 v2 ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=$1; VAR=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in $3; do
  n=$(basename "$v" | tr -c 'A-Za-z0-9_.\n' '_')
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu --no-latency --steps 10 --warmup 3 > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "bench $v rc=$?"; tail -20 $OUT/bench_$n.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$n.json').read().strip().splitlines()[-1])
ks=d['kernels']
print('$VAR=$v value', round(d['value']), 'ms/it', round(d['ms_per_step'],3), ' '.join(f'{k[2:]}={v[\"ms\"]:.3f}' for k,v in ks.items()))
"
done
