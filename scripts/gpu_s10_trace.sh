cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/s10tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s10tr/prof -o run -- python scripts/single_window.py 50 0 10 500 4000 > gpurun_out/s10tr/out.txt 2>&1 && tail -2 gpurun_out/s10tr/out.txt
