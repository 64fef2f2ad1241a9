#!/bin/bash
# Schedule tests, then single-window latency by Cholesky schedule (S10 and S50, 50 timed iterations
# after 3) and the batch rate of the pipelined split schedule at a few batch sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05s}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "schedules" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for shape in "10 500 4000" "50 2000 16000"; do for s in 0 1 2 3 4 5; do
  timeout -k 10 120 python scripts/single_window.py 50 $s $shape >> $OUT/single.txt 2>&1 || { echo "single $shape $s rc=$?"; tail -5 $OUT/single.txt; exit 1; }
done; done
cat $OUT/single.txt
for n in 64 128 192; do for s in 0 3 5; do
  timeout -k 10 300 python bench.py --windows $n --cholesky-schedule $s --no-cpu --no-latency --no-profile --steps 10 --warmup 3 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('windows $n sched $s', round(d['value']), round(d['ms_per_step'],3))" || exit 1
done; done
