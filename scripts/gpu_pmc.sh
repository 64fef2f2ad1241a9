#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains besides kernel dispatch)
# over a short bench run. Usage (via gpurun, from the repo root): bash scripts/gpu_pmc.sh TAG [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
ARGS=${*:---no-cpu --no-latency --no-profile --steps 2 --warmup 1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- python bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($CTRS) rc=$?"; tail -20 $OUT/p$i.log; exit 1; }
done
echo done
