#!/bin/bash
# Launch-structure A/B (OKVISGPU_FUSE bits of a measured-and-dropped build, profiles/r05_fuse_ab.txt;
# the variants are not in the tree): GPU suite with the default structure, then
# the batch rate and the final cost sum (same bits expected) per mask and batch size.
# Usage (via gpurun): bash scripts/gpu_r05_fuse.sh TAG "MASKS" "WINDOWS"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05fu}; mkdir -p $OUT
MASKS=${2:-"0 1 2 4 8"}
WINS=${3:-"256"}
if [ -z "$SKIPTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
  tail -1 $OUT/pytest.txt
fi
for n in $WINS; do for m in $MASKS; do
  OKVISGPU_FUSE=$m timeout -k 10 300 python bench.py --windows $n --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('windows $n mask $m', round(d['value']), round(d['ms_per_step'],4), repr(d['gather']['final_cost_sum']))" | tee -a $OUT/fuse.txt || exit 1
done; done
