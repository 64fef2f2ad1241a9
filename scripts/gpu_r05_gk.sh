#!/bin/bash
# Round-5 A/B of the per-window reduction trees and the multi-iteration graph (via gpurun): the -m gpu
# suite, then single-window rates (100 iterations) and batch lines with their final costs for
# lib_base0.so (before) and the tree's library with OKVISGPU_GRAPH_ITERS = default / 1 / 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05gk}; mkdir -p $OUT
OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
B0=$PWD/okvis2-x_amd/lib_base0.so; B=$PWD/okvis2-x_amd/libokvisgpu.so
for rep in 1 2; do for shape in "10 500 4000" "50 2000 16000"; do
  for v in "base0:$B0:" "new:$B:" "new-g1:$B:1" "new-g8:$B:8"; do
    IFS=: read name L g <<< "$v"
    OKVISGPU_GRAPH_ITERS=$g OKVISGPU_LIB=$L timeout -k 10 120 python scripts/single_window.py 100 0 $shape > $OUT/single.tmp 2>&1 || { echo "single $v rc=$?"; tail -5 $OUT/single.tmp; exit 1; }
    echo "$name ${shape%% *} $(tail -1 $OUT/single.tmp)" | tee -a $OUT/single.txt
  done
done; done
for n in 256 2048; do for v in "base0:$B0" "new:$B"; do
  IFS=: read name L <<< "$v"
  OKVISGPU_LIB=$L timeout -k 10 300 python bench.py --windows $n --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$name windows $n', round(d['value']), round(d['ms_per_step'],4), repr(d['gather']['final_cost_sum']))" | tee -a $OUT/batch.txt || exit 1
done; done
OKVISGPU_LIB=$B0 timeout -k 10 300 python bench.py --config s10 --steps 10 --warmup 3 --no-cpu --no-profile > $OUT/s10_base0.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --config s10 --steps 10 --warmup 3 --no-cpu --no-profile > $OUT/s10_new.json 2>/dev/null || exit 1
for f in base0 new; do python3 -c "
import json; d=json.loads(open('$OUT/s10_$f.json').read().strip().splitlines()[-1]); sw=d['single_window']; print('$f s10 bench single', sw.get('iters_per_s'), {k: v for k, v in sw.items() if 'e2e' in k or 'solve' in k})"; done
