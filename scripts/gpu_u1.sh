set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out/u1
bash scripts/ubench_ptile.sh run > gpurun_out/u1/ptile.txt 2>&1 || { cat gpurun_out/u1/ptile.txt; exit 1; }
cat gpurun_out/u1/ptile.txt
for w in 256 512; do
  timeout -k 10 300 python3 bench.py --windows $w --steps 20 --no-cpu --no-latency > gpurun_out/u1/b$w.json 2>gpurun_out/u1/b$w.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u1/p$w -o run -- python3 bench.py --windows $w --steps 20 --no-cpu --no-latency > /dev/null 2>gpurun_out/u1/p$w.err || exit 1
  python3 scripts/kstats_grouped.py gpurun_out/u1/p$w/run_kernel_trace.csv 30 > gpurun_out/u1/k$w.txt
  python3 -c "import json;d=json.loads(open('gpurun_out/u1/b$w.json').read().strip().splitlines()[-1]);print($w, round(d['value']), round(d['ms_per_step'],3))"
done
