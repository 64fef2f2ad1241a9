#!/bin/bash
# (OKVISGPU_ND is read only by a library built with -DOKG_ND_OVERRIDE: make OPT="-O3 -DOKG_ND_OVERRIDE")
# Kernel-trace stats of the Cholesky launches per schedule at a batch size (via gpurun): TAG WINDOWS "SCHEDULES"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for sch in $3; do
  OKVISGPU_ND=$([ $sch = 1 ] && echo 0 || echo 1) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_$2_$sch -o run -- \
    python bench.py --windows $2 --cholesky-schedule $sch --no-cpu --no-latency --no-profile --steps 5 --warmup 2 > $OUT/tr_$2_$sch.json 2> $OUT/tr_$2_$sch.err || { echo "trace $sch rc=$?"; tail -5 $OUT/tr_$2_$sch.err; exit 1; }
  python3 - "$OUT/tr_$2_$sch/run_kernel_stats.csv" "$2 sched $sch" <<'PY' | tee -a $OUT/chol_trace.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'  {r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:8.1f} us total {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
done
