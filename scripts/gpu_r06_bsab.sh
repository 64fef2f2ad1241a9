#!/bin/bash
# A/B of the backward substitution's dummy loads (lib_bsdiag.so = round-5 form): k_cholesky event time
# at 2,048 / 512 windows and the batch / single-window rates (scripts/lib_ab.sh), two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r06bs}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do for lib in libokvisgpu.so lib_bsdiag.so; do for n in 2048 512; do
  echo "$lib $n $(OKVISGPU_LIB=$PWD/okvis2-x_amd/$lib timeout -k 10 300 python scripts/kernel_probe.py $n k_cholesky)" | tee -a $OUT/kprobe.txt || exit 1
done; done; done
AB_STEPS=20 AB_WARMUP=5 bash scripts/lib_ab.sh $TAG "base bsdiag base bsdiag" | tee $OUT/ab.txt
