#!/bin/bash
# A/B of the pose-pose assembly variants (OKVISGPU_ASM) on the default workload: parity tests for
# each variant, then the bench's per-kernel table. Usage (via gpurun): bash scripts/asm_ab.sh TAG "0 1 2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-asm}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in ${2:-0 1 2}; do
  OKVISGPU_ASM=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_relpose.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.txt 2>&1 || { echo "pytest v$v rc=$?"; tail -30 $OUT/pytest_$v.txt; exit 1; }
  echo "v$v: $(tail -1 $OUT/pytest_$v.txt)"
  OKVISGPU_ASM=$v timeout -k 10 300 python bench.py --no-cpu --no-latency --steps 10 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench v$v rc=$?"; tail -20 $OUT/bench_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1])
k=d['kernels']['k_assemble_pp']
print('v$v value', round(d['value']), 'ms/it', round(d['ms_per_step'],3), 'assemble_pp', k['ms'], 'ms', round(k['frac']*100,1), '%')
"
done
