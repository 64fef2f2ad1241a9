#!/bin/bash
# Landmark-group phase clock (lib_lmvclk.so, -DOKG_LMV_CLOCK) on one S50 window: per-phase tick sums
# over the window's groups for each linearisation (x10 ns).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r06lmv}; mkdir -p $OUT
OKVISGPU_LIB=$PWD/okvis2-x_amd/lib_lmvclk.so timeout -k 10 120 python scripts/single_window.py 8 0 > $OUT/clk.txt 2>&1 || exit 1
grep LMVCLK $OUT/clk.txt | tail -4; tail -1 $OUT/clk.txt
