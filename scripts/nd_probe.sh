#!/bin/bash
# (OKVISGPU_ND is read only by a library built with -DOKG_ND_OVERRIDE: make OPT="-O3 -DOKG_ND_OVERRIDE")
# Batch rate vs windows per GPU for the Cholesky schedule x state order (nested dissection on/off):
# which one the automatic choice should take at each batch size. Usage (via gpurun): nd_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$1
mkdir -p $OUT
for n in ${WINDOWS:-64 128 256 512}; do for v in ${VARIANTS:-1:0 2:1 1:1 2:0}; do
  sch=${v%:*}; nd=${v#*:}
  OKVISGPU_ND=$nd timeout -k 10 300 python bench.py --windows $n --cholesky-schedule $sch --no-cpu --no-latency --no-profile --steps 10 --warmup 3 2>>$OUT/nd_probe.err \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('windows $n sched $sch nd $nd', round(d['value']), round(d['ms_per_step'],3), d['problem_stats_per_gpu'].get('cholesky_launches'))" | tee -a $OUT/nd_probe.txt || exit 1
done; done
