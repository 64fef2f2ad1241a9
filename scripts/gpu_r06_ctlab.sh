#!/bin/bash
# A/B of libokvisgpu.so against okvis2-x_amd/lib_prev.so (the previous commit): single-window rates
# (S50 / S10, steady state and re-integrating iterations, final-cost bits) and the batched bench
# line, twice; then the whole -m gpu suite on libokvisgpu.so (SKIP_PYTEST=1 skips it).
# Usage: gpu_r06_ctlab.sh OUTNAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06ctl}; mkdir -p $OUT
for rep in 1 2; do for lib in libokvisgpu.so lib_prev.so; do
  for shape in "50 2000 16000" "10 500 4000"; do
    OKVISGPU_LIB=okvis2-x_amd/$lib timeout -k 10 120 python scripts/imu_probe.py $shape | sed "s/^/$lib /" | tee -a $OUT/probe.txt || exit 1
  done
done; done
AB_STEPS=20 AB_WARMUP=5 bash scripts/lib_ab.sh $(basename $OUT)_ab "base prev base prev" | tee $OUT/ab.txt || exit 1
[ -n "$SKIP_PYTEST" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | tail -20; exit 1; }
tail -1 $OUT/pytest.txt
