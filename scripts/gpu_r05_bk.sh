#!/bin/bash
# Batch A/B of iterations per captured graph (OKVISGPU_GRAPH_ITERS) via gpurun: rate and final cost
# sum (same bits expected) per batch size. Usage: bash scripts/gpu_r05_bk.sh TAG "K ..." "WINDOWS ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05bk}; mkdir -p $OUT
for n in ${3:-256 2048}; do for k in ${2:-1 4 1 4}; do
  OKVISGPU_GRAPH_ITERS=$k timeout -k 10 300 python bench.py --windows $n --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('windows $n K $k', round(d['value']), round(d['ms_per_step'],4), repr(d['gather']['final_cost_sum']))" | tee -a $OUT/bk.txt || exit 1
done; done
