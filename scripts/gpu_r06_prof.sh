#!/bin/bash
# Round-6 profile set (via gpurun): MFMA counters of k_cholesky + FETCH/WRITE calibration, the PMC
# traffic passes, the default bench line, its rocprofv3 kernel trace, and the windows-per-GPU probe
# at the driver's iteration counts. Usage: bash scripts/gpu_r06_prof.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r06p}
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash scripts/gpu_pmc_calib.sh ${TAG}_calib > $OUT/calib.txt 2>&1 || { echo "calib failed"; cat $OUT/calib.txt; exit 1; }
python3 scripts/pmc_calib_summary.py gpurun_out/${TAG}_calib $OUT/pmc_calib.json > /dev/null || exit 1
cp $OUT/pmc_calib.json profiles/r06_pmc_calib.json  # (the bench runs below report frac_issued from it)
bash scripts/gpu_profile_all.sh ${TAG}_all > $OUT/profile_all.txt 2>&1 || { echo "profile_all failed"; tail -20 $OUT/profile_all.txt; exit 1; }
for n in 256 512 1024 2048; do
  timeout -k 10 300 python bench.py --windows $n --no-cpu --no-latency --no-profile --steps 20 --warmup 5 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print($n, round(d['value']), round(d['ms_per_step'],3))" >> $OUT/scaling_probe.txt || exit 1
done
cat $OUT/scaling_probe.txt
python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_all/bench.json').read().strip().splitlines()[-1])
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'roofline', d['roofline']['kernel'], d['roofline']['ms_per_iteration'], round(d['roofline']['frac'],4))
print('single', round(d['single_window']['iters_per_s']), d['single_window'].get('imu_reintegrated_factors_per_iteration'))
print('cpu', d['cpu_baseline']['value'], 'speedup', d['speedup_vs_cpu_baseline'])"
