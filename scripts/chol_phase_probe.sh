#!/bin/bash
# Cholesky phase decomposition by phase-cut builds (scripts/build_variant.sh) at several batch
# sizes: okvisgpu_time_kernel("cholesky"). Usage (via gpurun): bash scripts/chol_phase_probe.sh "256 2048" "base occ1 nopanel noupd nopu"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
for n in $1; do
  for v in $2; do
    if [ "$v" = base ]; then lib=$PWD/okvis2-x_amd/libokvisgpu.so; else lib=$PWD/okvis2-x_amd/lib_$v.so; fi
    r=$(OKVISGPU_LIB=$lib timeout -k 10 120 python3 scripts/kernel_probe.py $n k_cholesky) || exit 1
    echo "windows $n $v: $r"
  done
done
