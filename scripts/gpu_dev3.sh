#!/bin/bash
# Dev round trip (via gpurun): potrfTile micro-benchmark, the -m gpu suite, a bench line without
# the CPU baseline, and optionally the 256-window strong-scaling point. Usage: bash scripts/gpu_dev3.sh TAG [w256]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
bash scripts/ubench_ptile.sh run > $OUT/ptile.txt 2>&1 || { cat $OUT/ptile.txt; exit 1; }
grep "us per tile\|X L" $OUT/ptile.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest.txt | head -30; tail -5 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "chol", d["kernels"]["k_cholesky"]["ms"], "imu", d["kernels"]["k_eval_imu"]["ms"])
sw = d.get("single_window", {})
print("single window", round(sw.get("iters_per_s", 0)), "chol", sw.get("kernel_ms_per_iteration", {}).get("cholesky"), "imu", sw.get("kernel_ms_per_iteration", {}).get("eval_imu"))
PY
if [ "$2" = w256 ]; then
  timeout -k 10 300 python3 bench.py --windows 256 --steps 20 --no-cpu --no-latency > $OUT/b256.json 2>$OUT/b256.err || exit 1
  python3 -c "import json;d=json.loads(open('$OUT/b256.json').read().strip().splitlines()[-1]);print('w256', round(d['value']), round(d['ms_per_step'],3))"
fi
