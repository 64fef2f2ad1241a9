#!/bin/bash
# A/B of the GN prep inside the few-window linearisation launch (OKVISGPU_LIN_PREP=0/1) via gpurun:
# the -m gpu suite, single-window rates (100 iterations) with final costs, and 16 / 64-window batch
# lines with their final cost sums (same bits expected).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05lp}; mkdir -p $OUT
OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2; do for shape in "10 500 4000" "50 2000 16000"; do for lp in 0 1; do
  OKVISGPU_LIN_PREP=$lp timeout -k 10 120 python scripts/single_window.py 100 0 $shape > $OUT/single.tmp 2>&1 || { echo "single $lp rc=$?"; tail -5 $OUT/single.tmp; exit 1; }
  echo "linprep $lp ${shape%% *} $(tail -1 $OUT/single.tmp)" | tee -a $OUT/single.txt
done; done; done
for n in 16 64; do for lp in 0 1; do
  OKVISGPU_LIN_PREP=$lp timeout -k 10 300 python bench.py --windows $n --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('linprep $lp windows $n', round(d['value']), round(d['ms_per_step'],4), repr(d['gather']['final_cost_sum']))" | tee -a $OUT/batch.txt || exit 1
done; done
timeout -k 10 300 python bench.py --config s10 --steps 10 --warmup 3 --no-cpu --no-profile > $OUT/s10.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.loads(open('$OUT/s10.json').read().strip().splitlines()[-1]); sw=d['single_window']; print('s10 bench single', sw.get('iters_per_s'), sw.get('e2e_set_problems_plus_solve_ms'), sw.get('final_cost'))"
