#!/bin/bash
# Round-6 probes: the IMU phase clock of one S50 window's forced re-integration (few-window chunking),
# then the backward-substitution dummy-load A/B (scripts/gpu_r06_bsab.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r06b}; mkdir -p $OUT
OKVISGPU_LIB=$PWD/okvis2-x_amd/lib_iclk.so timeout -k 10 120 python scripts/imu_clock.py 50 2000 16000 1 > $OUT/imu_clock.txt 2>&1 || { cat $OUT/imu_clock.txt; exit 1; }
cat $OUT/imu_clock.txt
bash scripts/gpu_r06_bsab.sh ${1:-r06b}_bs
