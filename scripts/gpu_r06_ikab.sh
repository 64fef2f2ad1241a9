#!/bin/bash
# Batch IMU chunk size (steps per chunk, OKG_IMU_BATCH_K): 4 (libokvisgpu.so) vs 6 / 8 (lib_ik6 /
# lib_ik8.so; more LDS per workgroup, fewer co-resident waves): forced re-integration at 2,048
# (the OKG_IMU_BATCH_K switch lived in kernels_eval.hip for this A/B only; result: profiles/r06_imu_batch_chunk_ab.txt)
# windows and the batched bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06ik}; mkdir -p $OUT
for rep in 1 2; do for lib in libokvisgpu.so lib_ik6.so lib_ik8.so; do
  OKVISGPU_LIB=okvis2-x_amd/$lib timeout -k 10 200 python scripts/kernel_probe.py 2048 k_eval_imu | sed "s/^/$lib 2048: /" | tee -a $OUT/probe.txt || exit 1
done; done
AB_STEPS=20 AB_WARMUP=5 bash scripts/lib_ab.sh $(basename $OUT)_ab "base ik6 ik8" | tee $OUT/ab.txt
