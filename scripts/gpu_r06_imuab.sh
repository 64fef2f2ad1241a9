#!/bin/bash
# IMU A/B: libokvisgpu.so against okvis2-x_amd/$1 (single-window probe S50 / S10 and batched
# k_eval_imu at 2,048 windows, twice), then the IMU-touching GPU tests on libokvisgpu.so.
# Usage: gpu_r06_imuab.sh LIB_B OUTNAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${2:-r06imuab}; mkdir -p $OUT
for rep in 1 2; do for lib in libokvisgpu.so $1; do
  for shape in "50 2000 16000" "10 500 4000"; do
    OKVISGPU_LIB=okvis2-x_amd/$lib timeout -k 10 120 python scripts/imu_probe.py $shape | sed "s/^/$lib /" | tee -a $OUT/imu_probe.txt || exit 1
  done
  OKVISGPU_LIB=okvis2-x_amd/$lib timeout -k 10 200 python scripts/kernel_probe.py 2048 k_eval_imu | sed "s/^/$lib 2048: /" | tee -a $OUT/imu_probe.txt || exit 1
done; done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_imu_append.py tests/test_reference_scenarios.py tests/test_losses.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -20 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
