#!/bin/bash
# Development: Cholesky phase clocks (lib_cclk.so variant) at 2048 / 256 / 1 windows, then the bench
# at 2,048 (with the single-window mode) and at 256 windows. Output under gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-chol_ab}
mkdir -p gpurun_out/$TAG
for a in "2048 1" "256 1" "1 1"; do
  OKVISGPU_LIB=okvis2-x_amd/lib_cclk.so timeout -k 10 200 python scripts/chol_clock_probe.py $a >> gpurun_out/$TAG/cclk.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu --no-profile > gpurun_out/$TAG/b2048.json 2> gpurun_out/$TAG/b2048.err || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-latency --no-profile --windows 256 > gpurun_out/$TAG/b256.json 2>&1 || exit 1
grep -v "^$" gpurun_out/$TAG/cclk.log
python3 - $TAG <<'PY'
import json, sys
t = sys.argv[1]
for n in ("2048", "256"):
    d = json.loads(open(f"gpurun_out/{t}/b{n}.json").read().strip().splitlines()[-1])
    sw = d.get("single_window", {})
    print(n, round(d["value"]), round(d["ms_per_step"], 3), "single", round(sw.get("iters_per_s", 0)),
          "chol_ms", sw.get("kernel_ms_per_iteration", {}).get("cholesky"))
PY
