#!/bin/bash
# Single-window rate per Cholesky schedule for the S10 and S50 shapes (via gpurun): TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$1
mkdir -p $OUT
for shape in "10 500 4000" "50 2000 16000"; do for sch in 0 1 2 3; do
  timeout -k 10 120 python scripts/single_window.py 50 $sch $shape | sed "s/^/S${shape%% *} /" | tee -a $OUT/single_probe.txt || exit 1
done; done
