#!/bin/bash
# Diagonal-tile sweep variants (OKG_POTRF_V): the tile micro-benchmark per variant, then the batch,
# one S50 and one S10 window with the library variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05v}; mkdir -p $OUT
for v in 0 1 2 3; do
  timeout -k 10 120 ./scripts/ubench_ptile_v$v > $OUT/ubench_v$v.txt 2>&1 || { echo "ubench v$v rc=$?"; exit 1; }
  echo "v$v: $(grep 'product (persistent)' $OUT/ubench_v$v.txt | head -2 | tr '\n' ' ')"
done
for lib in base pv1 pv2 pv3; do
  if [ "$lib" = base ]; then L=$PWD/okvis2-x_amd/libokvisgpu.so; else L=$PWD/okvis2-x_amd/lib_$lib.so; fi
  a=$(OKVISGPU_LIB=$L timeout -k 10 120 python scripts/single_window.py 50 0 2>&1 | cut -d, -f1)
  b=$(OKVISGPU_LIB=$L timeout -k 10 120 python scripts/single_window.py 50 0 10 500 4000 2>&1 | cut -d, -f1)
  c=$(OKVISGPU_LIB=$L timeout -k 10 300 python bench.py --no-cpu --no-latency --no-profile --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],3), repr(d['gather']['final_cost_sum']))")
  echo "$lib | S50 single $a | S10 single $b | batch $c"
done
