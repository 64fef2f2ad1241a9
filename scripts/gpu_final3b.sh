#!/bin/bash
# Round-3 closing GPU set (via gpurun): the default bench line and a rocprofv3 kernel trace + stats
# of the same command. Usage: bash scripts/gpu_final3b.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "roofline", d["roofline"]["kernel"], round(d["roofline"]["frac"], 3), "traffic", d["roofline"]["traffic"])
sw = d["single_window"]; print("single window", round(sw["iters_per_s"]), "x cpu3", round(sw.get("speedup_vs_cpu_3_threads", 0), 1))
print("cpu", {k: round(v["value"], 1) for k, v in d["cpu_baseline"]["variants"].items()})
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "rocprof rc=$?"; tail -20 $OUT/bench_prof.err; exit 1; }
python3 scripts/kstats_grouped.py $OUT/prof/run_kernel_trace.csv 40 > $OUT/kernel_trace_grouped.txt
echo final-ok
