#!/bin/bash
# A/B of non-temporal S-tile reads in the persistent Cholesky (libokvisgpu.so) against ordinary
# loads (lib_nont.so): k_cholesky at 2,048 and 512 windows, the batched bench line, twice.
# (the OKG_CHOL_NT switch lived in kernels_chol.hip for this A/B only; result: profiles/r06_chol_nt_ab.txt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06nt}; mkdir -p $OUT
for rep in 1 2; do for lib in libokvisgpu.so lib_nont.so; do for n in 2048 512; do
  echo "$lib $n $(OKVISGPU_LIB=$PWD/okvis2-x_amd/$lib timeout -k 10 300 python scripts/kernel_probe.py $n k_cholesky)" | tee -a $OUT/kprobe.txt || exit 1
done; done; done
AB_STEPS=20 AB_WARMUP=5 bash scripts/lib_ab.sh $(basename $OUT)_ab "base nont base nont" | tee $OUT/ab.txt
