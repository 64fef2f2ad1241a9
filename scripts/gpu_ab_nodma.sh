#!/bin/bash
# A/B at 256 windows: Cholesky schedule 1 vs 4 (panel tiles by DMA during the factor) vs 4 without
# the DMA (lib_nodma: tiles loaded at panel time, L kept in LDS for the updates).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
for rep in 1 2; do for v in "base 1" "base 4" "nodma 4"; do
  set -- $v; lib=$PWD/okvis2-x_amd/libokvisgpu.so; [ $1 = nodma ] && lib=$PWD/okvis2-x_amd/lib_nodma.so
  r=$(OKG_PROBE_SCHED=$2 OKVISGPU_LIB=$lib timeout -k 10 120 python3 scripts/kernel_probe.py 256 k_cholesky) || exit 1
  echo "$1 sched$2: $r"
done; done
