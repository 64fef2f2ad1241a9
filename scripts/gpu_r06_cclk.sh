#!/bin/bash
# Persistent-Cholesky phase clock (lib_cclk.so, -DOKG_CHOL_CLOCK): workgroup 0's phases, including
# the diagonal factor's wavefront-0 sweep (wait for the trailing update, look-ahead, 8-column
# factor, publish), for one S50 window and for 512 windows (schedule 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r06cclk}; mkdir -p $OUT
OKVISGPU_LIB=$PWD/okvis2-x_amd/lib_cclk.so timeout -k 10 120 python scripts/single_window.py 2 1 > $OUT/one.txt 2>&1 || exit 1
grep CHOLCLK $OUT/one.txt | tail -2
OKVISGPU_LIB=$PWD/okvis2-x_amd/lib_cclk.so OKG_PROBE_SCHED=1 timeout -k 10 300 python scripts/kernel_probe.py 512 k_cholesky > $OUT/b512.txt 2>&1 || exit 1
grep CHOLCLK $OUT/b512.txt | tail -2
