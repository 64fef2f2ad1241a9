#!/bin/bash
# Pipelined Cholesky (schedule 4) round trip: team micro-benchmark, schedule-equality tests, then
# batch rates of schedule 1 vs 4 at a few windows-per-GPU points. Usage: bash scripts/gpu_r05_pipe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05d}; mkdir -p $OUT
if [ -x scripts/ubench_team ]; then timeout -k 10 120 ./scripts/ubench_team > $OUT/ubench_team.txt 2>&1 || { echo "ubench rc=$?"; exit 1; }; cat $OUT/ubench_team.txt; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "schedules" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for n in 256 2048; do for s in 1 4; do
  timeout -k 10 300 python -u bench.py --windows $n --cholesky-schedule $s --no-cpu --no-latency --steps 10 --warmup 3 > $OUT/bench_${n}_$s.txt 2>&1 || { echo "bench $n $s rc=$?"; tail -5 $OUT/bench_${n}_$s.txt; exit 1; }
  python3 -c "
import json
l=[x for x in open('$OUT/bench_${n}_$s.txt') if x.startswith('{')][-1]; d=json.loads(l)
print('windows $n sched $s value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'chol ms', round(d['kernels']['k_cholesky']['ms'],4))"
done; done
