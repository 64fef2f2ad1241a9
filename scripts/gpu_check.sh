#!/bin/bash
# GPU round-trip used during development: parity tests, then a rocprof kernel-trace of the
# default bench workload. Usage (from the repo root, via gpurun): bash scripts/gpu_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu --no-latency --no-profile --steps 5 --warmup 2 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench_prof.err; exit 1; }
cat $OUT/bench_prof.json
