set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r05a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.txt 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench.txt; exit 1; }
tail -c 3000 $OUT/bench.txt
