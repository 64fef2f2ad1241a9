#!/bin/bash
# A/B of a few-window change against lib_base1.so = the previous commit (via gpurun; k_fgrad rounds, r05fg; batched strided tails, r05sb): the -m gpu suite, then
# single-window rates (100 iterations) with final costs and batch lines with final cost sums for
# lib_base1.so (before) and the current library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05fg}; mkdir -p $OUT
OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
B0=$PWD/okvis2-x_amd/lib_base1.so; B=$PWD/okvis2-x_amd/libokvisgpu.so
for rep in 1 2; do for shape in "10 500 4000" "50 2000 16000"; do for v in "base1:$B0" "new:$B"; do
  IFS=: read name L <<< "$v"
  OKVISGPU_LIB=$L timeout -k 10 120 python scripts/single_window.py 100 0 $shape > $OUT/single.tmp 2>&1 || { echo "single $v rc=$?"; tail -5 $OUT/single.tmp; exit 1; }
  echo "$name ${shape%% *} $(tail -1 $OUT/single.tmp)" | tee -a $OUT/single.txt
done; done; done
for n in 64 2048; do for v in "base1:$B0" "new:$B"; do
  IFS=: read name L <<< "$v"
  OKVISGPU_LIB=$L timeout -k 10 300 python bench.py --windows $n --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name windows $n', round(d['value']), round(d['ms_per_step'],4), repr(d['gather']['final_cost_sum']))" | tee -a $OUT/batch.txt || exit 1
done; done
