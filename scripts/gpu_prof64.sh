#!/bin/bash
# rocprofv3 kernel trace of the bench at a given window count (strong-scaling share of one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
N=${1:-64}
OUT=gpurun_out/prof_w$N
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python bench.py --windows $N --no-cpu --no-latency --no-profile --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/err.txt || { echo "rc=$?"; tail $OUT/err.txt; exit 1; }
cat $OUT/bench.json
