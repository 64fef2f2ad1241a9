#!/bin/bash
# Development: SQ / SQC counters of k_eval_imu on the forced re-integration launch
# (scripts/imu_clk_probe.py), one rocprofv3 --pmc pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-imu_pmc}; N=${2:-512}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --kernel-include-regex k_eval_imu -d $OUT/p1 -o p1 --output-format csv -- python3 scripts/imu_clk_probe.py $N > $OUT/p1.log 2>&1 || { echo p1 failed; tail $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH --kernel-include-regex k_eval_imu -d $OUT/p2 -o p2 --output-format csv -- python3 scripts/imu_clk_probe.py $N > $OUT/p2.log 2>&1 || { echo p2 failed; tail $OUT/p2.log; }
find $OUT -name "*counter_collection.csv" | head
