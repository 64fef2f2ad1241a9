#!/bin/bash
# IMU phase clock (lib_iclk.so): one S50 window and 256 windows, forced re-integration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r06iclk}; mkdir -p $OUT
for n in 1 256; do
  OKVISGPU_LIB=okvis2-x_amd/lib_iclk.so timeout -k 10 300 python scripts/imu_clock.py 50 2000 16000 $n >> $OUT/iclk.txt 2>&1 || exit 1
done
cat $OUT/iclk.txt
