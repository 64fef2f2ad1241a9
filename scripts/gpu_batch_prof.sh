#!/bin/bash
# Kernel statistics of the default batched workload (rocprofv3 kernel trace of a short bench run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-batch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-latency --no-profile --steps 5 --warmup 2 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench_prof.err; exit 1; }
python scripts/kstats_grouped.py $OUT/prof/run_kernel_trace.csv > $OUT/grouped.txt 2>&1 || true
cat $OUT/grouped.txt | head -40
