#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (scripts/pmc_calib.hip, built on the host) and the MFMA
# counters of k_cholesky on the default bench workload. One rocprofv3 --pmc pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_calib}
mkdir -p $OUT
./scripts/pmc_calib > $OUT/calib_bytes.txt || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/calib_$C -o run -- ./scripts/pmc_calib > $OUT/calib_$C.log 2>&1 || { echo "calib $C failed"; tail $OUT/calib_$C.log; exit 1; }
done
ARGS="--no-cpu --no-latency --no-profile --steps 2 --warmup 1"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_WAVES SQ_WAVE_CYCLES --kernel-include-regex k_cholesky --output-format csv -d $OUT/mfma -o run -- python3 bench.py $ARGS > $OUT/mfma.log 2>&1 || { echo "mfma pass failed"; tail $OUT/mfma.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex k_cholesky --output-format csv -d $OUT/grbm -o run -- python3 bench.py $ARGS > $OUT/grbm.log 2>&1 || { echo "grbm pass failed"; tail $OUT/grbm.log; exit 1; }
echo ok
