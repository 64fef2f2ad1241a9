#!/bin/bash
# Timing probe (development): batched forced IMU re-integration with the square-root-information
# (U) and / or covariance (P_delta) state stores compiled out (lib_nou / lib_nop / lib_noup; results
# of those builds are not valid solves, only the kernel's time is read). The two compile switches
# (OKG_IMU_NO_USTORE / OKG_IMU_NO_PSTORE around the two store loops of evalImuBlock) lived in the
# working tree for this probe only; result: profiles/r06_imu_store_probe.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r06stp}; mkdir -p $OUT
for rep in 1 2; do for lib in libokvisgpu.so lib_nou.so lib_nop.so lib_noup.so; do
  OKVISGPU_LIB=okvis2-x_amd/$lib timeout -k 10 200 python scripts/kernel_probe.py 2048 k_eval_imu | sed "s/^/$lib 2048: /" | tee -a $OUT/probe.txt || exit 1
done; done
