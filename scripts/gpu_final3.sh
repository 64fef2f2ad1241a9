#!/bin/bash
# Round-3 final GPU set (via gpurun): schedule-4 occupancy A/B at 256 windows, the default bench line,
# a rocprofv3 kernel trace + stats of the same command, and the windows-per-GPU (strong-scaling share)
# probe. Usage: bash scripts/gpu_final3.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
L2=$PWD/okvis2-x_amd/lib_wide2.so
OKVISGPU_LIB=$L2 timeout -k 10 300 python3 bench.py --windows 256 --steps 20 --no-cpu --no-latency --cholesky-schedule 4 > $OUT/b256_w2.json 2>$OUT/b256_w2.err || { tail -5 $OUT/b256_w2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/b256_w2.json').read().strip().splitlines()[-1]);print('w256 sched4 occ2', round(d['value']), round(d['ms_per_step'],3), d['kernels']['k_cholesky']['ms'])"
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "roofline", d["roofline"]["kernel"], round(d["roofline"]["frac"], 3))
sw = d["single_window"]; print("single window", round(sw["iters_per_s"]), sw["kernel_ms_per_iteration"])
print("kernels", {k: v["ms"] for k, v in d["kernels"].items()})
print("cpu", d["cpu_baseline"]["variants"])
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench_prof.err; exit 1; }
python3 scripts/kstats_grouped.py $OUT/prof/run_kernel_trace.csv 40 > $OUT/kernel_trace_grouped.txt
for w in 256 512 1024; do
  timeout -k 10 300 python3 bench.py --windows $w --steps 20 --no-cpu --no-latency --no-profile > $OUT/s$w.json 2>$OUT/s$w.err || exit 1
  python3 -c "import json;d=json.loads(open('$OUT/s$w.json').read().strip().splitlines()[-1]);print('windows $w', round(d['value']), round(d['ms_per_step'],3))"
done
echo final-ok
