set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q > gpurun_out/t2.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t2.log
timeout -k 10 300 python bench.py --windows 8 --steps 5 --warmup 2 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo "bench rc=$?"
