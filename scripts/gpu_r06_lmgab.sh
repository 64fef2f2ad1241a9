#!/bin/bash
# Landmark-group bounds for few windows (lib_lmg.so, -DOKG_LMG_OVERRIDE, OKVISGPU_LMG=visits,landmarks):
# single-window S50 / S10 steady and re-integrating iteration times and final costs, then the
# landmark-group phase clock (lib_lmvclk.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r06lmg}; mkdir -p $OUT
for rep in 1 2; do for g in 256,64 128,32 96,24 64,16; do
  for shape in "50 2000 16000" "10 500 4000"; do
    OKVISGPU_LMG=$g OKVISGPU_LIB=okvis2-x_amd/lib_lmg.so timeout -k 10 120 python scripts/imu_probe.py $shape | sed "s/^/lmg $g /" | tee -a $OUT/probe.txt || exit 1
  done
done; done
bash scripts/gpu_r06_lmvclk.sh $(basename $OUT)_clk
