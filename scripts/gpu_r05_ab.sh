#!/bin/bash
# Round-5 A/B round trip (via gpurun): micro-benchmarks, the -m gpu suite, then bench lines for
# "LIB:WINDOWS:SCHEDULE" specs (WINDOWS s10 / s50: one window of that shape; LIB = base or a lib_NAME.so variant from scripts/build_variant.sh).
# Usage: bash scripts/gpu_r05_ab.sh TAG [tests|notest] "spec ..." [ubench]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05ab}; mkdir -p $OUT
if [ "$4" = ubench ]; then
  for u in ubench_team ubench_ptile_la1 ubench_ptile_la0; do
    [ -x scripts/$u ] || continue
    timeout -k 10 150 ./scripts/$u > $OUT/$u.txt 2>&1 || { echo "$u rc=$?"; exit 1; }
    echo "== $u"; grep -v "^  [0-9] |" $OUT/$u.txt | head -30
  done
fi
if [ "$2" = tests ]; then
  # (TESTLIB=NAME: the suite on lib_NAME.so)
  [ -n "$TESTLIB" ] && export OKVISGPU_LIB=$PWD/okvis2-x_amd/lib_$TESTLIB.so
  OKVISGPU_PARITY_REPORT=$OUT/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; tail -5 $OUT/pytest.txt; exit 1; }
  tail -1 $OUT/pytest.txt
  unset OKVISGPU_LIB
fi
for spec in $3; do
  IFS=: read lib n s <<< "$spec"
  if [ "$lib" = base ]; then L=$PWD/okvis2-x_amd/libokvisgpu.so; else L=$PWD/okvis2-x_amd/lib_$lib.so; fi
  if [ "$n" = s10 ] || [ "$n" = s50 ]; then  # single window: 100 timed iterations after 3
    shape="10 500 4000"; [ "$n" = s50 ] && shape="50 2000 16000"
    OKVISGPU_LIB=$L timeout -k 10 120 python scripts/single_window.py 100 $s $shape > $OUT/single_${lib}_${n}_$s.txt 2>&1 || { echo "single $spec rc=$?"; tail -5 $OUT/single_${lib}_${n}_$s.txt; exit 1; }
    echo "$spec $(tail -1 $OUT/single_${lib}_${n}_$s.txt)"
    continue
  fi
  OKVISGPU_LIB=$L timeout -k 10 300 python -u bench.py --windows $n --cholesky-schedule $s --no-cpu --no-latency --steps 10 --warmup 3 > $OUT/bench_${lib}_${n}_$s.txt 2>&1 || { echo "bench $spec rc=$?"; tail -5 $OUT/bench_${lib}_${n}_$s.txt; exit 1; }
  python3 -c "
import json
l=[x for x in open('$OUT/bench_${lib}_${n}_$s.txt') if x.startswith('{')][-1]; d=json.loads(l)
print('$spec value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'chol ms', round(d['kernels']['k_cholesky']['ms'],4), 'cost', repr(d['gather']['final_cost_sum']))"
done
