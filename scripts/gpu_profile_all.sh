#!/bin/bash
# Round profile set (via gpurun): PMC passes -> pmc_traffic.json (also used by this run's bench),
# then the default bench and a rocprofv3 kernel trace of the same command, all under gpurun_out/TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/gpu_pmc.sh ${TAG}_pmc || exit 1
python3 scripts/pmc_traffic.py $OUT/pmc_traffic.json 2048 gpurun_out/${TAG}_pmc/p1/run_counter_collection.csv \
  gpurun_out/${TAG}_pmc/p2/run_counter_collection.csv > /dev/null || exit 1
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench_prof.err; exit 1; }
python3 scripts/kstats_grouped.py $OUT/prof/run_kernel_trace.csv 40 > $OUT/kernel_trace_grouped.txt
cat $OUT/bench.json
